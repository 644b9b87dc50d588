// cusz_amd/csrc/huffman.hip -- coarse-grained canonical Huffman encode/decode for gfx950.
//
// Output format = the reference phf segment (codec/hf/src/hf_kernels.cuhip.inl:76-170,
// hf_buf.cc:111-139,191-211): chunk c covers codes [c*sublen, (c+1)*sublen); its codewords
// are packed MSB-first into u32 cells starting on a fresh cell; par_nbit[c] bits,
// par_entry[c] = exclusive scan of per-chunk cell counts; bitstream = concatenated cells.
//
// MI355X design (not the reference's 4-phase encode with a host scan round trip):
//  * one kernel: a 256-thread workgroup owns a group of G consecutive chunks, computes each
//    chunk's bit offsets with a workgroup scan, ORs the codewords into LDS cells, then gets
//    the group's global cell offset by decoupled look-back over per-group status words
//    ({flag, value} packed in one 8-byte agent-scope atomic, so the value IS the flag) and
//    writes the cells straight into the archive, coalesced.  Codes are read once from HBM.
//  * decode: one lane per chunk (reference semantics, hf_kernels.cuhip.inl:331-396) but
//    table-driven: a 2^K-entry LDS lookup table resolves codes of <= K bits per step
//    instead of one bit per step; longer codes fall back to the canonical first[]/entry[]
//    search.  Four symbols are buffered per 8-byte store.
#include "common.hh"
#include "kernels.hh"

namespace cusz_amd {

namespace {

constexpr int kEncThreads = 256;
constexpr int kMaxGroup = 8;
constexpr unsigned long long kFlagAgg = 1ull << 32;
constexpr unsigned long long kFlagIncl = 2ull << 32;
constexpr unsigned int kSpinLimit = 1u << 20;

__device__ __forceinline__ unsigned long long ld_status(unsigned long long* p)
{
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(unsigned long long* p, unsigned long long v)
{
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane)
{
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// exclusive scan over the 256-thread workgroup; returns the prefix, writes the total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_wave, uint32_t& total)
{
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan(v, lane);
  if (lane == 63) s_wave[wid] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kEncThreads / 64; w++) {
    const uint32_t t = s_wave[w];
    off += (w < wid) ? t : 0u;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

// read this thread's PER codes of a chunk (PER = sublen / 256) and apply f(word)
template <typename F>
__device__ __forceinline__ void for_my_codes(const uint16_t* __restrict__ codes, size_t start, int per,
                                             int cnt, const uint32_t* s_book, F&& f)
{
  const int mine = threadIdx.x * per;
  const uint16_t* p = codes + start + mine;
  if ((per & 7) == 0 && mine + per <= cnt) {
    for (int i = 0; i < per; i += 8) {
      uint4 w = *reinterpret_cast<const uint4*>(p + i);
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int h = 0; h < 4; h++) {
        f(s_book[ws[h] & 0xFFFFu]);
        f(s_book[ws[h] >> 16]);
      }
    }
  }
  else {
    for (int i = 0; i < per; i++)
      if (mine + i < cnt) f(s_book[p[i]]);
  }
}

__global__ void __launch_bounds__(kEncThreads) k_hf_encode(HfEncodeArgs a, int G, int cellcap)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_book = smem;                    // bklen words
  uint32_t* s_cells = smem + a.bklen;         // G * cellcap words
  __shared__ uint32_t s_wave[kEncThreads / 64];
  __shared__ uint32_t s_nbit[kMaxGroup];
  __shared__ uint32_t s_base;

  for (int i = threadIdx.x; i < a.bklen; i += kEncThreads) s_book[i] = a.book[i];
  for (int i = threadIdx.x; i < G * cellcap; i += kEncThreads) s_cells[i] = 0;
  __syncthreads();

  const int g = blockIdx.x;
  const int per = a.sublen / kEncThreads;
  const int c0 = g * G;

  for (int j = 0; j < G; j++) {
    const int c = c0 + j;
    if (c >= a.pardeg) {
      if (threadIdx.x == 0) s_nbit[j] = 0;
      continue;
    }
    const size_t start = (size_t)c * a.sublen;
    const int cnt = (int)((a.n - start) < (size_t)a.sublen ? (a.n - start) : (size_t)a.sublen);
    uint32_t bits = 0;
    for_my_codes(a.codes, start, per, cnt, s_book, [&](uint32_t w) { bits += w >> 27; });
    uint32_t total;
    uint32_t pos = block_excl_scan(bits, s_wave, total);
    uint32_t* cells = s_cells + j * cellcap;
    // MSB-first pack (hf_kernels.cuhip.inl:114-151) into LDS cells
    for_my_codes(a.codes, start, per, cnt, s_book, [&](uint32_t w) {
      const uint32_t l = w >> 27, v = w & 0x07FFFFFFu;
      const uint32_t q = pos >> 5, o = pos & 31;
      if (o + l <= 32)
        atomicOr(&cells[q], v << (32 - o - l));
      else {
        const uint32_t sp = o + l - 32;
        atomicOr(&cells[q], v >> sp);
        atomicOr(&cells[q + 1], v << (32 - sp));
      }
      pos += l;
    });
    if (threadIdx.x == 0) s_nbit[j] = total;
  }
  __syncthreads();

  uint32_t gcells = 0;
  for (int j = 0; j < G; j++) gcells += (s_nbit[j] + 31) >> 5;

  // decoupled look-back over group status words
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint32_t base = 0;
    if (g == 0) {
      if (lane == 0) st_status(&a.status[0], kFlagIncl | gcells);
    }
    else {
      if (lane == 0) st_status(&a.status[g], kFlagAgg | gcells);
      int j = g - 1;
      unsigned int spins = 0;
      while (true) {
        const int idx = j - lane;
        const unsigned long long st = idx >= 0 ? ld_status(&a.status[idx]) : kFlagIncl;
        const uint32_t flag = (uint32_t)(st >> 32);
        if (__ballot(flag == 0)) {
          if (++spins > kSpinLimit) {
            if (lane == 0) atomicOr(a.timeout, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        const unsigned long long incl = __ballot(flag == 2);
        const int first = incl ? (__ffsll((long long)incl) - 1) : 64;
        base += wave_sum(lane <= first ? (uint32_t)st : 0u);
        if (incl) break;
        j -= 64;
      }
      if (lane == 0) st_status(&a.status[g], kFlagIncl | (unsigned long long)(base + gcells));
    }
    if (lane == 0) s_base = base;
  }
  __syncthreads();

  uint32_t off = s_base;
  for (int j = 0; j < G; j++) {
    const int c = c0 + j;
    if (c >= a.pardeg) break;
    const uint32_t nb = s_nbit[j], nc = (nb + 31) >> 5;
    if (threadIdx.x == 0) a.par_nbit[c] = nb, a.par_entry[c] = off;
    const uint32_t* cells = s_cells + j * cellcap;
    for (uint32_t i = threadIdx.x; i < nc; i += kEncThreads) a.bitstream[off + i] = cells[i];
    off += nc;
  }
}

constexpr int kLutBits = 10;

__global__ void __launch_bounds__(256) k_hf_decode(HfDecodeArgs a)
{
  __shared__ uint32_t lut[1 << kLutBits];
  __shared__ uint32_t s_first[32], s_entry[32];
  __shared__ uint16_t s_keys[kMaxBklen];

  const int32_t* rv = reinterpret_cast<const int32_t*>(a.revbook);
  if (threadIdx.x < 32) s_first[threadIdx.x] = (uint32_t)rv[threadIdx.x], s_entry[threadIdx.x] = (uint32_t)rv[32 + threadIdx.x];
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(a.revbook + 256);
  for (int i = threadIdx.x; i < a.bklen; i += blockDim.x) s_keys[i] = keys[i];
  __syncthreads();
  // LUT: same rule as the reference decoder (first l with prefix >= first[l])
  for (int i = threadIdx.x; i < (1 << kLutBits); i += blockDim.x) {
    uint32_t e = 0;
    for (int l = 1; l <= kLutBits; l++) {
      const uint32_t v = (uint32_t)i >> (kLutBits - l);
      if (v >= s_first[l]) {
        uint32_t k = s_entry[l] + v - s_first[l];
        if (k >= (uint32_t)a.bklen) k = a.bklen - 1;
        e = ((uint32_t)s_keys[k] << 16) | (uint32_t)l;
        break;
      }
    }
    lut[i] = e;
  }
  __syncthreads();

  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.pardeg) return;
  const uint32_t* src = a.bitstream + a.par_entry[c];
  const uint32_t nbit = a.par_nbit[c];
  const uint32_t ncell = (nbit + 31) >> 5;
  const size_t obase = (size_t)c * a.sublen;
  if (obase >= a.n) return;
  const uint32_t nsym = (uint32_t)((a.n - obase) < (size_t)a.sublen ? (a.n - obase) : (size_t)a.sublen);
  uint16_t* dst = a.out + obase;

  auto cell = [&](uint32_t i) -> uint64_t { return i < ncell ? (uint64_t)src[i] : 0ull; };
  uint64_t buf = (cell(0) << 32) | cell(1);
  int avail = 64;
  uint32_t ci = 2;
  uint64_t pack = 0;
  uint32_t j = 0;
  for (; j < nsym; j++) {
    if (avail <= 32) {
      buf |= cell(ci++) << (32 - avail);
      avail += 32;
    }
    const uint32_t e = lut[buf >> (64 - kLutBits)];
    uint32_t l = e & 0xFFu, sym = e >> 16;
    if (l == 0) {  // long code: canonical search (hf_kernels.cuhip.inl:351-365)
      for (l = kLutBits + 1; l <= (uint32_t)kLmax; l++) {
        const uint32_t v = (uint32_t)(buf >> (64 - l));
        if (v >= s_first[l]) {
          uint32_t k = s_entry[l] + v - s_first[l];
          if (k >= (uint32_t)a.bklen) k = a.bklen - 1;
          sym = s_keys[k];
          break;
        }
      }
    }
    buf <<= l;
    avail -= (int)l;
    pack |= (uint64_t)sym << (16 * (j & 3));
    if ((j & 3) == 3) {
      *reinterpret_cast<uint2*>(dst + j - 3) = make_uint2((uint32_t)pack, (uint32_t)(pack >> 32));
      pack = 0;
    }
  }
  for (uint32_t t = j & ~3u; t < j; t++) dst[t] = (uint16_t)(pack >> (16 * (t & 3)));
}

}  // namespace

static int enc_group(int sublen, int& cellcap)
{
  cellcap = sublen * kLmax / 32 + 2;
  int G = 32768 / (cellcap * 4);
  if (G < 1) G = 1;
  if (G > kMaxGroup) G = kMaxGroup;
  return G;
}

int hf_encode_groups(int sublen, int pardeg)
{
  int cellcap;
  const int G = enc_group(sublen, cellcap);
  return (pardeg + G - 1) / G;
}

int launch_hf_encode(const HfEncodeArgs& a, hipStream_t st)
{
  int cellcap;
  const int G = enc_group(a.sublen, cellcap);
  const int ngroups = (a.pardeg + G - 1) / G;
  const size_t lds = (size_t)(a.bklen + G * cellcap) * 4;
  k_hf_encode<<<ngroups, kEncThreads, lds, st>>>(a, G, cellcap);
  return (int)hipGetLastError();
}

int launch_hf_decode(const HfDecodeArgs& a, hipStream_t st)
{
  const int grid = (a.pardeg + 255) / 256;
  k_hf_decode<<<grid, 256, 0, st>>>(a);
  return (int)hipGetLastError();
}

}  // namespace cusz_amd
