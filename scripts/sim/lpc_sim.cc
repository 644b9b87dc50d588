// Host emulation of the decode tables (k_hf_tables) and the lane-per-chunk decoder
// (k_hf_decode_lane) in cusz_amd/csrc/huffman.hip, lane by lane, with bounds assertions.
// Development tool: g++ -O2 -o lpc_sim lpc_sim.cc ; ./lpc_sim <dir>  (files written by lpc_sim.py)
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include <string>

#ifndef L2CAP
#define L2CAP 2048
#endif
constexpr int kLmax = 27, kLutBits = 12, kL1 = 4096, kL2Cap = L2CAP, kLongLens = kLmax - kLutBits;
static std::vector<uint8_t> rd(const char* dir, const char* name)
{
  char p[512];
  snprintf(p, sizeof p, "%s/%s", dir, name);
  FILE* f = fopen(p, "rb");
  if (!f) { fprintf(stderr, "missing %s\n", p); exit(2); }
  std::vector<uint8_t> v;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}
static uint32_t pack(uint32_t ns, uint32_t bits, uint32_t l0, uint32_t s0, uint32_t s1)
{
  return (ns << 30) | (bits << 25) | (l0 << 20) | (s1 << 10) | s0;
}
int main(int argc, char** argv)
{
  const char* dir = argv[1];
  auto rv = rd(dir, "revbook.bin");
  auto nb = rd(dir, "nbit.bin");
  auto en = rd(dir, "entry.bin");
  auto bs = rd(dir, "bitstream.bin");  // with `pre` leading pad bytes
  auto meta = rd(dir, "meta.bin");     // n, sublen, bklen, pre (u64 each)
  uint64_t mv[4];
  memcpy(mv, meta.data(), 32);
  const uint64_t n = mv[0];
  const uint32_t sublen = (uint32_t)mv[1], bklen = (uint32_t)mv[2], pre = (uint32_t)mv[3];
  const int pardeg = (int)(nb.size() / 4);
  const int32_t* r32 = (const int32_t*)rv.data();
  uint32_t first[32], entry[32];
  for (int i = 0; i < 32; i++) first[i] = (uint32_t)r32[i], entry[i] = (uint32_t)r32[32 + i];
  const uint16_t* keys = (const uint16_t*)(rv.data() + 256);
  int maxl = 1;
  for (int l = 1; l < 31; l++)
    if (entry[l + 1] > entry[l]) maxl = l;
  uint32_t thr[32], base[32];
  for (int l = 0; l < 32; l++) {
    thr[l] = (l >= 1 && l <= maxl) ? (first[l] << (32 - l)) : 0u;
    base[l] = entry[l] - first[l];
  }
  for (int l = 1; l < maxl; l++) assert(((uint64_t)first[l] << (32 - l)) >= ((uint64_t)first[l + 1] << (31 - l)));
  auto dec1 = [&](uint32_t v, uint32_t& sym) {
    uint32_t l = 1;
    for (int k = 1; k <= kLmax; k++) l += (k <= maxl && (v >> (32 - k)) < first[k]) ? 1u : 0u;
    if (l > (uint32_t)maxl) l = maxl;
    uint32_t k = std::min(base[l] + (v >> (32 - l)), bklen - 1);
    assert(k < bklen);
    sym = keys[k];
    return l;
  };
  std::vector<uint32_t> L1(kL1), L2(kL2Cap, 0);
  const uint32_t P = maxl > kLutBits ? std::min(first[kLutBits], (uint32_t)kL1) : 0u;
  for (uint32_t i = 0; i < kL1; i++) {
    uint32_t v = i << 20, s0, s1;
    uint32_t l0 = dec1(v, s0);
    L1[i] = 0;
    if (i >= P && l0 <= 12) {
      uint32_t rest = 12 - l0;
      uint32_t l1 = rest ? dec1(v << l0, s1) : 99;
      L1[i] = l1 <= rest ? pack(2, l0 + l1, l0, s0, s1) : pack(1, l0, l0, s0, 0);
    }
    else if (i < P) assert(l0 > 12 && l0 <= 27);
  }
  const uint32_t n2 = std::min(P << 4, (uint32_t)kL2Cap - 1);
  for (uint32_t q = 0; q < n2; q++) {
    uint32_t s0, l = dec1(q << 16, s0);
    if (l <= 16) L2[q] = pack(1, l, l, s0, 0);
  }
  printf("maxl=%d P=%u L2 entries=%u (wanted %u)\n", maxl, P, n2, P << 4);
  auto entry_of = [&](uint32_t win) {
    uint32_t e1 = L1[win >> 20];
    uint32_t e2 = L2[std::min(win >> 16, (uint32_t)kL2Cap - 1)];
    uint32_t e = (e1 >> 30) ? e1 : e2;
    if (!(e >> 30)) {
      uint32_t l = kLutBits + 1;
      for (int q = 0; q < kLongLens; q++) {
        const int k = kLutBits + 1 + q;
        l += (k <= maxl && (win >> (32 - k)) < first[k]) ? 1u : 0u;
      }
      if (l > (uint32_t)kLmax) l = kLmax;
      uint32_t s = keys[std::min(base[l] + (win >> (32 - l)), bklen - 1)];
      e = pack(1, l, l, s, 0);
    }
    return e;
  };
  const uint32_t* par_nbit = (const uint32_t*)nb.data();
  const uint32_t* par_entry = (const uint32_t*)en.data();
  const uint8_t* bsb = bs.data() + pre;  // bitstream start (byte address as in the kernel)
  const size_t bs_bytes = bs.size() - pre;
  std::vector<uint16_t> out(n, 0xFFFF);
  long long max_lag = 0;
  for (int c = 0; c < pardeg; c++) {
    const uint64_t obase = (uint64_t)c * sublen;
    const uint32_t nsym = (uint32_t)std::min<uint64_t>(sublen, n - obase);
    const uint32_t nbit = par_nbit[c], ent = par_entry[c], ncell = (nbit + 31) >> 5;
    const uintptr_t addr = (uintptr_t)(pre + 4ull * ent);  // byte offset inside bs (16-B alignment of bs[0] assumed)
    const uint32_t mis = addr & 15, skip = mis >> 2;
    const int64_t gb = (int64_t)addr - mis - pre;  // byte offset of block 0 relative to bitstream start
    const uint32_t nblk = (skip + ncell + 3) >> 2;
    const bool tail = c + 1 == pardeg;
    auto load_block = [&](uint32_t b, uint32_t v[4]) {
      uint32_t bb = std::min(b, nblk ? nblk - 1 : 0u);
      bool partial = tail && (bb + 1) * 4 > skip + ncell;
      int64_t o = gb + 16ll * bb;
      if (!partial) {
        assert(o + (int64_t)pre >= 0 && o + 16 <= (int64_t)bs_bytes + 64);
        for (int k = 0; k < 4; k++) {
          int64_t q = o + 4 * k;
          v[k] = (q >= 0 && q + 4 <= (int64_t)bs_bytes) ? *(const uint32_t*)(bsb + q) : 0xDEADBEEF;
        }
      }
      else {
        uint32_t lim = skip + ncell - bb * 4;
        assert(lim >= 1 && lim <= 3);
        for (int k = 0; k < 4; k++) {
          int64_t q = o + 4 * k;
          if ((uint32_t)k < lim) {
            assert(q >= 0 && q + 4 <= (int64_t)bs_bytes);
            v[k] = *(const uint32_t*)(bsb + q);
          }
          else
            v[k] = 0;
        }
      }
    };
    uint32_t ring[20], oring[16];
    memset(ring, 0, sizeof ring);
    memset(oring, 0, sizeof oring);
    uint16_t* o16 = (uint16_t*)oring;
    auto ring_put = [&](uint32_t b, const uint32_t v[4]) {
      memcpy(ring + 4 * (b & 3), v, 16);
    };
    uint32_t ld = std::min(nblk, 4u);
    for (uint32_t b = 0; b < ld; b++) {
      uint32_t v[4];
      load_block(b, v);
      ring_put(b, v);
    }
    uint32_t bA = ld, bB = ld + 1, pA[4], pB[4];
    load_block(bA, pA);
    load_block(bB, pB);
    uint32_t cnt = 0, flushed = 0;
    uint64_t buf = ((uint64_t)ring[skip & 15] << 32) | ring[(skip + 1) & 15];
    uint32_t avail = 64, nw = skip + 2, nxt = ring[nw & 15];
    uint64_t consumed = 0;
    auto steps = [&]() {
      for (int s = 0; s < 4; s++) {
        if (cnt < nsym) {
          if (!(nw + 1 < ld * 4 || ld >= nblk)) {
            fprintf(stderr, "chunk %d: ring underrun nw=%u ld=%u\n", c, nw, ld);
            exit(3);
          }
          uint32_t e = entry_of((uint32_t)(buf >> 32));
          uint32_t l0 = (e >> 20) & 31u;
          bool both = (e >> 30) == 2u && cnt + 1 < nsym;
          uint32_t i0 = cnt & 31u, i1 = both ? ((cnt + 1) & 31u) : i0;
          o16[i0] = (uint16_t)(e & 1023u);
          o16[i1] = (uint16_t)(both ? ((e >> 10) & 1023u) : (e & 1023u));
          cnt += both ? 2u : 1u;
          uint32_t l = both ? ((e >> 25) & 31u) : l0;
          buf <<= l;
          avail -= l;
          consumed += l;
          if (avail < 32) {
            buf |= (uint64_t)nxt << (32 - avail);
            avail += 32;
            nw++;
            nxt = ring[nw & 15];
          }
        }
      }
    };
    auto cadence = [&](uint32_t p[4], uint32_t& b) {
      if (b == ld && ld < nblk && ld - (nw >> 2) < 4u) {
        ring_put(ld, p);
        ld++;
      }
      if (b < ld) b += 2;
      load_block(b, p);
      if (cnt - flushed >= 16u) {
        assert(cnt - flushed < 32);
        memcpy(&out[obase + flushed], o16 + (flushed & 16u), 32);
        assert(obase + flushed + 16 <= n);
        flushed += 16;
      }
    };
    while (cnt < nsym) {
      steps();
      cadence(pA, bA);
      steps();
      cadence(pB, bB);
    }
    for (uint32_t i = flushed; i < cnt; i++) out[obase + i] = o16[i & 31u];
    if ((long long)consumed != (long long)nbit) max_lag = std::max(max_lag, std::llabs((long long)consumed - (long long)nbit));
  }
  FILE* f = fopen((std::string(dir) + "/out.bin").c_str(), "wb");
  fwrite(out.data(), 2, n, f);
  fclose(f);
  printf("done: %d chunks, max |end-nbit| = %lld\n", pardeg, max_lag);
  return 0;
}
