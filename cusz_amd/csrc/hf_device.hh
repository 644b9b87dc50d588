// cusz_amd/csrc/hf_device.hh -- device helpers shared by the Huffman kernels (huffman.hip)
// and the fused brick kernels (brick.hip): wave64 scans, MSB-first codeword packing into LDS
// cells, and the canonical-code decode table.
//
// Canonical decoding follows the reference rule (codec/hf/src/hf_kernels.cuhip.inl:351-365):
// the code length is the first l with prefix_l >= first[l]; symbol = keys[entry[l] + prefix_l -
// first[l]].  revbook layout (hf_bk.seq.cc:135-142): first i32[32] | entry i32[32] | keys[bklen].
#pragma once

#include <cstddef>

#include "common.hh"

namespace cusz_amd {
namespace hfd {

// inclusive wave64 prefix sum with DPP (row_shr inside 16-lane rows, then row_bcast15/31)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

__device__ __forceinline__ void wave_sync()
{
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Pack this lane's codewords (book words: code | len << 27) MSB-first starting at bit `pos`
// of the LDS cell buffer.  Words only this lane touches are plain stores; the first word (when
// `pos` is not word aligned) and the trailing partial word may be shared with neighbouring
// lanes and are merged with LDS atomic OR (the buffer is zero beforehand).
template <int N>
__device__ __forceinline__ void pack_words(uint32_t* cells, uint32_t pos, const uint32_t (&w)[N], int mine)
{
  uint32_t q = pos >> 5;
  uint64_t acc = 0;
  uint32_t fill = pos & 31;
  bool first = fill != 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    if (i >= mine) break;
    const uint32_t l = w[i] >> 27, v = w[i] & 0x07FFFFFFu;
    acc |= (uint64_t)v << (64 - fill - l);
    fill += l;
    if (fill >= 32) {
      const uint32_t word = (uint32_t)(acc >> 32);
      if (first)
        atomicOr(&cells[q], word);
      else
        cells[q] = word;
      first = false;
      acc <<= 32;
      fill -= 32;
      q++;
    }
  }
  if (fill) atomicOr(&cells[q], (uint32_t)(acc >> 32));
}

// Same result as pack_words<4> for a lane whose 4 codewords total L <= 64 bits: Horner-pack them
// right-aligned into 64 bits (shift by the length, OR the code into the low word), align the
// stream end to a word boundary and OR the (up to) three words ending at word (pos+L-1)/32 into
// the zeroed LDS cells.  Words of the lane's range not covered by its bits receive 0.
__device__ __forceinline__ void pack4_or(uint32_t* cells, uint32_t pos, const uint32_t (&w)[4], uint32_t L)
{
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    acc <<= (w[k] >> 27);
    acc |= w[k] & 0x07FFFFFFu;
  }
  const uint32_t e = pos + L, E = (e - 1) >> 5, t = (32u - (e & 31u)) & 31u;
  const uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
  const uint32_t w2 = lo << t;
  const uint32_t w1 = t ? __builtin_amdgcn_alignbit(hi, lo, 32u - t) : hi;
  const uint32_t w0 = t ? hi >> (32u - t) : 0u;
  atomicOr(&cells[E], w2);
  if (E >= 1) atomicOr(&cells[E - 1], w1);
  if (E >= 2) atomicOr(&cells[E - 2], w0);
}

// Same bits as pack4_or, addressed from the START of the lane's range: the <= 64 bits are
// left-justified in hi:lo and OR-ed as the three words from word pos/32 on (bits past the lane's
// range are 0, so the third word may be pure padding -- the caller keeps two words of zeroed
// slack after the last row).  No exec masking: the shifts and alignbit take pos mod 32 from the
// low bits of pos itself.  cells must be a compile-time LDS address (the word offsets fold into
// the ds immediates).
__device__ __forceinline__ void pack4_or_lj(uint32_t* cells, uint32_t pos, const uint32_t (&w)[4], uint32_t L)
{
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    acc <<= (w[k] >> 27);
    acc |= w[k] & 0x07FFFFFFu;
  }
  acc <<= (64u - L) & 63u;  // left-justify (L = 0: acc is 0 either way)
  const uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
  uint32_t* c = cells + (pos >> 5);
  atomicOr(&c[0], hi >> (pos & 31u));
  atomicOr(&c[1], __builtin_amdgcn_alignbit(hi, lo, pos & 31u));
  atomicOr(&c[2], __builtin_amdgcn_alignbit(lo, 0u, pos & 31u));
}

// ---- decode tables --------------------------------------------------------------------------
// Entry (u32) for the codeword(s) at the top of a window: [9:0] first symbol, [15:14] symbols
// (1 or 2), [25:16] second symbol, [30:26] bits consumed, [31] two symbols.  0 = not in this
// table -- and, read as an entry, "0 symbols, 0 bits": a decoder may step on it without moving.
// The symbols sit where one 32-bit LDS store writes them as two consecutive u16 codes
// (value & 0x03FF03FF).
__device__ __forceinline__ uint32_t ent_pack(uint32_t two, uint32_t bits, uint32_t s0, uint32_t s1)
{
  return (two << 31) | (bits << 26) | (s1 << 16) | ((1u + two) << 14) | s0;
}
__device__ __forceinline__ uint32_t ent_bits(uint32_t e) { return (e >> 26) & 31u; }
__device__ __forceinline__ uint32_t ent_nsym(uint32_t e) { return (e >> 14) & 3u; }
constexpr uint32_t kEntSymMask = 0x03FF03FFu;

// longest code length present (last l with entry[l+1] > entry[l])
__device__ __forceinline__ int longest_code(const uint32_t* entry)
{
  int m = 1;
  for (int l = 1; l < 31; l++)
    if (entry[l + 1] > entry[l]) m = l;
  return m;
}

// One symbol from a left-justified 32-bit window by the reference rule.  The thresholds
// first[l] * 2^(32-l) never increase with l (canonical construction), so the failing lengths
// form a prefix 1..m and the code length is 1 + the number of failing lengths.
__device__ __forceinline__ uint32_t tab_decode1(uint32_t v, const uint32_t* first, int maxl, const uint32_t* base,
                                                const uint16_t* keys, uint32_t bklen, uint32_t& sym)
{
  uint32_t l = 1;
#pragma unroll
  for (int k = 1; k <= kLmax; k++) l += (k <= maxl && (v >> (32 - k)) < first[k]) ? 1u : 0u;
  if (l > (uint32_t)maxl) l = (uint32_t)maxl;
  sym = keys[min(base[l] + (v >> (32 - l)), bklen - 1)];
  return l;
}

// Decode tables resident in LDS.
//  L1: 2^B entries indexed by the next B bits, one or two whole codewords of <= B bits; 0 for
//      a prefix of a longer code.
//  L2: single-symbol entries indexed DIRECTLY by the next 16 bits.  Canonical codes put every
//      code longer than B bits below first[B] (longer codes are numerically smaller), so only
//      windows whose B-bit prefix is < first[B] have an entry: first[B] << (16 - B) entries
//      (capped; its last entry and every entry past them stay 0).  Exactly one of the two
//      lookups is nonzero for a code of <= 16 bits, so entry = L1 | L2 (read together).
//  Codes longer than 16 bits (or past the cap) count failing lengths against thresholds the
//  caller keeps in registers (DecRegs).
constexpr int kL2Bits = 16;
#ifndef CUSZ_AMD_SLOW_UNROLL
#define CUSZ_AMD_SLOW_UNROLL 16  // unroll of the rare >16-bit code search (1: keep it small)
#endif
#ifndef CUSZ_AMD_DEC_L2CAP
#define CUSZ_AMD_DEC_L2CAP 4096
#endif
constexpr int kL2Cap = CUSZ_AMD_DEC_L2CAP;

template <int B>
struct LdsTables {
  uint32_t l1[1 << B];
  uint32_t l2[kL2Cap];
  uint32_t first[32];
  uint32_t base[32];
  uint32_t entry[32];
  uint32_t maxl;
  uint32_t pad[3];
  uint16_t keys[kMaxBklen];
};

// wave-uniform thresholds for the rare untabulated codes (first[l], l = 12..27)
constexpr int kSlowFrom = 12;
struct DecRegs {
  uint32_t first[kLmax - kSlowFrom + 1];
  uint32_t maxl;
  uint32_t thr;  // windows below thr start with a code longer than B bits (lookup1)
};

// Cooperative build by the whole workgroup (ends with a barrier).
template <int B>
__device__ __forceinline__ void build_tables(LdsTables<B>& t, const uint8_t* revbook, int bklen)
{
  const int tid = threadIdx.x, nt = blockDim.x;
  const int32_t* rv = reinterpret_cast<const int32_t*>(revbook);
  if (tid < 32) t.first[tid] = (uint32_t)rv[tid], t.entry[tid] = (uint32_t)rv[32 + tid];
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(revbook + 256);
  for (int i = tid; i < bklen; i += nt) t.keys[i] = keys[i];
  __syncthreads();
  const int maxl = longest_code(t.entry);
  if (tid < 32) {
    t.base[tid] = t.entry[tid] - t.first[tid];
    if (tid == 0) t.maxl = (uint32_t)maxl;
  }
  __syncthreads();
  uint32_t first[32];  // registers: the unrolled threshold loop reads no LDS
#pragma unroll
  for (int k = 0; k < 32; k++) first[k] = t.first[k];
  const uint32_t* base = t.base;
  const uint32_t ub = (uint32_t)bklen;
  for (uint32_t i = tid; i < (1u << B); i += nt) {
    const uint32_t v = i << (32 - B);
    uint32_t s0, s1, e = 0;
    const uint32_t l0 = tab_decode1(v, first, maxl, base, t.keys, ub, s0);
    if (l0 <= (uint32_t)B) {
      const uint32_t rest = B - l0;
      const uint32_t l1 = rest ? tab_decode1(v << l0, first, maxl, base, t.keys, ub, s1) : 99u;
      e = l1 <= rest ? ent_pack(1, l0 + l1, s0, s1) : ent_pack(0, l0, s0, 0);
    }
    t.l1[i] = e;
  }
  const uint32_t P = maxl > B ? min(first[B], 1u << B) : 0u;
  const uint32_t n2 = min(P << (kL2Bits - B), (uint32_t)kL2Cap - 1);
  for (uint32_t q = tid; q < (uint32_t)kL2Cap; q += nt) {
    uint32_t e = 0;
    if (q < n2) {
      uint32_t s0;
      const uint32_t l = tab_decode1(q << (32 - kL2Bits), first, maxl, base, t.keys, ub, s0);
      if (l <= (uint32_t)kL2Bits) e = ent_pack(0, l, s0, 0);
    }
    t.l2[q] = e;
  }
  __syncthreads();
}

template <int B>
__device__ __forceinline__ DecRegs load_dec_regs(const LdsTables<B>& t)
{
  static_assert(B + 1 >= kSlowFrom, "slow path thresholds start at B + 1");
  DecRegs r;
#pragma unroll
  for (int q = 0; q < kLmax - kSlowFrom + 1; q++) r.first[q] = __builtin_amdgcn_readfirstlane(t.first[kSlowFrom + q]);
  r.maxl = __builtin_amdgcn_readfirstlane(t.maxl);
  // canonical codes: a code is longer than B bits iff the window's top B bits are < first[B]
  const uint32_t fb = __builtin_amdgcn_readfirstlane(t.first[B]);
  r.thr = r.maxl <= (uint32_t)B ? 0u : (fb >= (1u << B) ? 0xFFFFFFFFu : fb << (32 - B));
  return r;
}

// Entry for the codeword(s) at the top of `win`.
template <int B>
__device__ __forceinline__ uint32_t lookup(const LdsTables<B>& t, const DecRegs& rg, uint32_t win, uint32_t bklen)
{
  const uint32_t e1 = t.l1[win >> (32 - B)];
  const uint32_t e2 = t.l2[min(win >> (32 - kL2Bits), (uint32_t)kL2Cap - 1)];
  uint32_t e = e1 | e2;
  if (__builtin_expect(e == 0, 0)) {  // all lengths <= 16 failed: count the rest
    uint32_t l = B + 1;
#pragma unroll CUSZ_AMD_SLOW_UNROLL
    for (int q = B + 1 - kSlowFrom; q < kLmax - kSlowFrom + 1; q++)
      l += (kSlowFrom + q < (int)rg.maxl && (win >> (32 - (kSlowFrom + q))) < rg.first[q]) ? 1u : 0u;
    if (l > rg.maxl) l = rg.maxl;
    const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), bklen - 1)];
    e = ent_pack(0, l, s, 0);
  }
  return e;
}

// The rare codes longer than 16 bits (no table entry): count the failing lengths against the
// thresholds in registers.
template <int B>
__device__ __forceinline__ uint32_t lookup_long(const LdsTables<B>& t, const DecRegs& rg, uint32_t win, uint32_t bklen)
{
  uint32_t l = B + 1;
#pragma unroll
  for (int q = B + 1 - kSlowFrom; q < kLmax - kSlowFrom + 1; q++)
    l += (kSlowFrom + q < (int)rg.maxl && (win >> (32 - (kSlowFrom + q))) < rg.first[q]) ? 1u : 0u;
  if (l > rg.maxl) l = rg.maxl;
  const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), bklen - 1)];
  return ent_pack(0, l, s, 0);
}

// One table read, no branch: the entry, or 0 for a code longer than 16 bits (lookup_long).
template <int B>
__device__ __forceinline__ uint32_t lookup_short(const LdsTables<B>& t, const DecRegs& rg, uint32_t win)
{
  const uint32_t a = win < rg.thr ? (1u << B) + min(win >> (32 - kL2Bits), (uint32_t)kL2Cap - 1) : win >> (32 - B);
  return t.l1[a];
}

// Same entry as lookup() with ONE table read: L1 and L2 are exclusive (L2 holds exactly the
// windows below rg.thr), so the window picks its table before the read.  L2 follows L1 in
// LdsTables, so both are one array.
template <int B>
__device__ __forceinline__ uint32_t lookup1(const LdsTables<B>& t, const DecRegs& rg, uint32_t win, uint32_t bklen)
{
  static_assert(offsetof(LdsTables<B>, l2) == sizeof(uint32_t) << B, "l2 follows l1");
  const uint32_t a = win < rg.thr ? (1u << B) + min(win >> (32 - kL2Bits), (uint32_t)kL2Cap - 1) : win >> (32 - B);
  uint32_t e = t.l1[a];
  if (__builtin_expect(e == 0, 0)) {  // all lengths <= 16 failed: count the rest
    uint32_t l = B + 1;
#pragma unroll
    for (int q = B + 1 - kSlowFrom; q < kLmax - kSlowFrom + 1; q++)
      l += (kSlowFrom + q < (int)rg.maxl && (win >> (32 - (kSlowFrom + q))) < rg.first[q]) ? 1u : 0u;
    if (l > rg.maxl) l = rg.maxl;
    const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), bklen - 1)];
    e = ent_pack(0, l, s, 0);
  }
  return e;
}

// Same entry as lookup(), reading the L2 table only for the lanes whose L1 entry is 0 (a second,
// dependent LDS round trip for them instead of an L2 read by every lane on every step).
template <int B>
__device__ __forceinline__ uint32_t lookup_l1_first(const LdsTables<B>& t, const DecRegs& rg, uint32_t win,
                                                    uint32_t bklen)
{
  uint32_t e = t.l1[win >> (32 - B)];
  if (e == 0) {
    e = t.l2[min(win >> (32 - kL2Bits), (uint32_t)kL2Cap - 1)];
    if (__builtin_expect(e == 0, 0)) {
      uint32_t l = B + 1;
#pragma unroll CUSZ_AMD_SLOW_UNROLL
      for (int q = B + 1 - kSlowFrom; q < kLmax - kSlowFrom + 1; q++)
        l += (kSlowFrom + q < (int)rg.maxl && (win >> (32 - (kSlowFrom + q))) < rg.first[q]) ? 1u : 0u;
      if (l > rg.maxl) l = rg.maxl;
      const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), bklen - 1)];
      e = ent_pack(0, l, s, 0);
    }
  }
  return e;
}

// ---- compact decode tables (the 3-D fused decoder) ---------------------------------------------
// One u32 entry per window, laid out for few instructions per decode step:
//   [9:0] first symbol, [12:10] 2 x symbols (0, 2 or 4: the tile pointer's advance in bytes),
//   [25:16] second symbol, [31:27] bits consumed; 0 = "no symbol, no bits" (a code longer than
//   16 bits, or a window past the L2 cap: decoded by lookup_long).
// L1 (2^12 entries) by the top 12 bits, one or two whole codewords; L2 (kL2Cap4 entries) right
// after it, by the top 16 bits, for the windows below the canonical threshold first[12] << 20.
// Stored symbols are (e & kEnt4SymMask): two u16 halves.
constexpr int kL2Cap4 = 2048;
constexpr uint32_t kEnt4SymMask = 0x03FF03FFu;
__device__ __forceinline__ uint32_t ent4_pack(uint32_t nsym, uint32_t bits, uint32_t s0, uint32_t s1)
{
  return (bits << 27) | (s1 << 16) | ((2u * nsym) << 10) | s0;
}
__device__ __forceinline__ uint32_t ent4_bits(uint32_t e) { return e >> 27; }
__device__ __forceinline__ uint32_t ent4_adv(uint32_t e) { return (e >> 10) & 7u; }

struct Tab4 {
  uint32_t e[(1 << 12) + kL2Cap4];
  uint32_t T[16];  // lookup_long4's thresholds, lengths 13..27 (load_dec_regs4)
  uint32_t first[32];
  uint32_t base[32];
  uint32_t entry[32];
  uint32_t maxl;
  uint16_t keys[kMaxBklen];
};

// Cooperative build by the whole workgroup (ends with a barrier); same decoding rule as
// build_tables (hf_kernels.cuhip.inl:351-365), entries in the compact format.  Every decoder
// workgroup builds it before its first step, so it is kept cheap (≈ 2x fewer VALU than one
// counting decode per symbol slot):
//  * the failing-length count compares (win >> 1) with uniform thresholds first[k] << (31 - k)
//    (SGPRs; 0 past the longest code), one compare + one add per length;
//  * one decode per 12-bit window: the first codes go to a u16 scratch table (length << 10 |
//    symbol, 0 = longer than 12 bits) in the L2 area; an L1 entry's second code is that table's
//    entry for the window shifted past the first code (the zero-filled low bits never decide a
//    code that fits the remaining bits: prefix-free), so the second decode is one LDS read;
//  * then the L2 entries overwrite the scratch.
__device__ __forceinline__ void build_tab4(Tab4& t, const uint8_t* revbook, int bklen)
{
  constexpr int B = 12;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int32_t* rv = reinterpret_cast<const int32_t*>(revbook);
  if (tid < 32) t.first[tid] = (uint32_t)rv[tid], t.entry[tid] = (uint32_t)rv[32 + tid];
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(revbook + 256);
  for (int i = tid; i < bklen; i += nt) t.keys[i] = keys[i];
  __syncthreads();
  const int maxl = longest_code(t.entry);
  if (tid < 32) {
    t.base[tid] = t.entry[tid] - t.first[tid];
    if (tid == 0) t.maxl = (uint32_t)maxl;
  }
  __syncthreads();
  // (win >> (32 - k)) < first[k]  <=>  (win >> 1) < first[k] << (31 - k)   (first[k] <= 2^k)
  uint32_t T[kLmax + 1];
#pragma unroll
  for (int k = 1; k <= kLmax; k++) {
    const uint32_t f = t.first[k];
    T[k] = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(k > maxl ? 0u : (f >= (1u << k) ? 0xFFFFFFFFu : f << (31 - k))));
  }
  const uint32_t ub = (uint32_t)bklen, ml = (uint32_t)maxl;
  auto decode1 = [&](uint32_t v, uint32_t& sym) -> uint32_t {
    const uint32_t h = v >> 1;
    uint32_t l = 1;
#pragma unroll
    for (int k = 1; k <= kLmax; k++) l += h < T[k] ? 1u : 0u;
    l = min(l, ml);
    sym = t.keys[min(t.base[l] + (v >> (32 - l)), ub - 1)];
    return l;
  };
  uint16_t* s1 = reinterpret_cast<uint16_t*>(t.e + (1 << B));  // 4096 u16 = the L2 area
  static_assert(kL2Cap4 * 2 >= (1 << B), "scratch fits the L2 area");
  for (uint32_t i = tid; i < (1u << B); i += nt) {
    uint32_t s;
    const uint32_t l = decode1(i << (32 - B), s);
    s1[i] = (uint16_t)(l <= (uint32_t)B ? (l << 10) | s : 0u);
  }
  __syncthreads();
  for (uint32_t i = tid; i < (1u << B); i += nt) {
    const uint32_t a = s1[i];
    const uint32_t l0 = a >> 10, rest = B - l0;
    const uint32_t b = a && rest ? s1[(i << l0) & ((1u << B) - 1)] : 0u;
    const uint32_t l1 = b >> 10;
    t.e[i] = !a ? 0u : (b && l1 <= rest ? ent4_pack(2, l0 + l1, a & 1023u, b & 1023u) : ent4_pack(1, l0, a & 1023u, 0));
  }
  __syncthreads();
  const uint32_t P = maxl > B ? min(t.first[B], 1u << B) : 0u;
  const uint32_t n2 = min(P << (kL2Bits - B), (uint32_t)kL2Cap4 - 1);
  for (uint32_t q = tid; q < (uint32_t)kL2Cap4; q += nt) {
    uint32_t e = 0;
    if (q < n2) {
      uint32_t s0;
      const uint32_t l = decode1(q << (32 - kL2Bits), s0);
      if (l <= (uint32_t)kL2Bits) e = ent4_pack(1, l, s0, 0);
    }
    t.e[(1 << B) + q] = e;
  }
  __syncthreads();
}

// Wave-uniform values for the compact decoder: the L1/L2 threshold and the longest code; and in
// Tab4::T, for the rare codes no table entry holds, the canonical thresholds of lengths 13..27
// pre-shifted so that one compare of (win >> 1) decides each:
//   (win >> (32 - L)) < first[L]  <=>  (win >> 1) < first[L] << (31 - L)
// (first[L] <= 2^L keeps the right side in 32 bits; lengths past the longest code never count).
struct DecRegs4 {
  uint32_t maxl;
  uint32_t thr;
};

// Called by every thread after build_tab4 (ends with a barrier: thread q < 15 writes T[q]).
__device__ __forceinline__ DecRegs4 load_dec_regs4(Tab4& t)
{
  constexpr int B = 12;
  DecRegs4 r;
  r.maxl = __builtin_amdgcn_readfirstlane(t.maxl);
  if (threadIdx.x < 16) {
    const int L = 13 + (int)threadIdx.x;
    const uint32_t f = L <= kLmax ? t.first[L] : 0u;
    t.T[threadIdx.x] = L > kLmax || L >= (int)r.maxl ? 0u : (f >= (1u << L) ? 0xFFFFFFFFu : f << (31 - L));
  }
  const uint32_t fb = __builtin_amdgcn_readfirstlane(t.first[B]);
  r.thr = r.maxl <= (uint32_t)B ? 0u : (fb >= (1u << B) ? 0xFFFFFFFFu : fb << (32 - B));
  __syncthreads();
  return r;
}

// Index in Tab4::e of the entry for the codeword(s) at the top of `win` (L1 or L2 by the
// canonical threshold: exclusive, one table read).
__device__ __forceinline__ uint32_t tab4_index(const DecRegs4& rg, uint32_t win)
{
  return win < rg.thr ? (1u << 12) + min(win >> (32 - kL2Bits), (uint32_t)kL2Cap4 - 1) : win >> 20;
}

// Codes longer than 16 bits (and windows past the L2 cap): the length by counting the failing
// lengths 13..27 (the reference rule, hf_kernels.cuhip.inl:351-365), one compare each; the
// entry in the compact format (one symbol).
__device__ __forceinline__ uint32_t lookup_long4(const Tab4& t, const DecRegs4& rg, uint32_t win, uint32_t bklen)
{
  const uint32_t h = win >> 1;
  uint32_t l = 13;
  uint32_t T[16];
  __builtin_memcpy(T, t.T, sizeof(T));  // wave-uniform: broadcast LDS reads (keeps SGPRs free)
#pragma unroll
  for (int q = 0; q < kLmax - 12; q++) l += h < T[q] ? 1u : 0u;
  if (l > rg.maxl) l = rg.maxl;
  const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), bklen - 1)];
  return ent4_pack(1, l, s, 0);
}

}  // namespace hfd
}  // namespace cusz_amd
