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
//    table-driven: a 4096-entry LDS table resolves up to TWO codewords per lookup from the
//    next 12 bits (the reference walks one bit per step); longer codes fall back to the
//    canonical first[]/entry[] search.  The bitstream is fetched in 4-cell groups with the
//    next group in flight, and symbols are staged per lane in LDS and written 32 B at a time
//    (full write granules instead of 2-8 B partial writes).
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

constexpr int kMaxPer = 32;  // sublen <= 8192

// Pack this thread's codewords (MSB-first, starting at bit `pos` of the chunk) into the LDS
// cell buffer.  Words that only this thread touches are plain stores; the first word (when
// `pos` is not word aligned) and the trailing partial word may be shared with neighbouring
// threads and are merged with LDS atomic OR (the buffer is zeroed beforehand).
__device__ __forceinline__ void pack_words(uint32_t* cells, uint32_t pos, const uint32_t (&w)[kMaxPer], int mine)
{
  uint32_t q = pos >> 5;
  uint64_t acc = 0;
  uint32_t fill = pos & 31;  // bits already owned by earlier threads in word q
  bool first = fill != 0;
#pragma unroll
  for (int i = 0; i < kMaxPer; i++) {
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
    // this thread's codes [tid*per, tid*per + per) -> codewords in registers
    const int lo = threadIdx.x * per;
    const int mine = cnt - lo < 0 ? 0 : (cnt - lo < per ? cnt - lo : per);
    const uint16_t* p = a.codes + start + lo;
    uint32_t w[kMaxPer];
    uint32_t bits = 0;
    if ((per & 7) == 0 && mine == per) {
#pragma unroll
      for (int i = 0; i < kMaxPer; i += 8) {
        if (i >= per) break;
        const uint4 v = *reinterpret_cast<const uint4*>(p + i);
        const uint32_t vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 4; h++) w[i + 2 * h] = s_book[vs[h] & 0xFFFFu], w[i + 2 * h + 1] = s_book[vs[h] >> 16];
      }
    }
    else {
#pragma unroll
      for (int i = 0; i < kMaxPer; i++)
        if (i < mine) w[i] = s_book[p[i]];
    }
#pragma unroll
    for (int i = 0; i < kMaxPer; i++)
      if (i < mine) bits += w[i] >> 27;
    uint32_t total;
    const uint32_t pos = block_excl_scan(bits, s_wave, total);
    if (mine) pack_words(s_cells + j * cellcap, pos, w, mine);
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

constexpr int kLutBits = 12;           // 4096-entry LDS table
constexpr int kDecThreads = 256;
constexpr int kRing = 32;               // per-lane output ring (symbols)
constexpr int kRingStride = 36;         // u32 words per lane (16-B aligned, spreads banks)

// LUT entry: [31:30] nsym (0 = long code), [29:25] consumed bits, [24:15] sym1, [14:5] sym0.
__device__ __forceinline__ uint32_t lut_pack(uint32_t nsym, uint32_t bits, uint32_t s0, uint32_t s1)
{
  return (nsym << 30) | (bits << 25) | (s1 << 15) | (s0 << 5);
}

// canonical decode of one symbol from the top `have` bits of v (reference rule,
// hf_kernels.cuhip.inl:351-365: the first l with prefix_l >= first[l]); returns length or 0
__device__ __forceinline__ uint32_t canon_one(uint32_t v, int have, const uint32_t* first, const uint32_t* entry,
                                              const uint16_t* keys, int bklen, int maxl, uint32_t& sym)
{
  for (int l = 1; l <= have && l <= maxl; l++) {
    const uint32_t p = v >> (have - l);
    if (p >= first[l]) {
      uint32_t k = entry[l] + p - first[l];
      sym = keys[k < (uint32_t)bklen ? k : (uint32_t)bklen - 1];
      return (uint32_t)l;
    }
  }
  return 0;
}

__global__ void __launch_bounds__(kDecThreads) k_hf_decode(HfDecodeArgs a)
{
  __shared__ uint32_t lut[1 << kLutBits];
  __shared__ uint32_t s_first[32], s_entry[32];
  __shared__ uint16_t s_keys[kMaxBklen];
  __shared__ __attribute__((aligned(16))) uint32_t ring[kDecThreads * kRingStride];
  __shared__ int s_maxl;

  const int32_t* rv = reinterpret_cast<const int32_t*>(a.revbook);
  if (threadIdx.x < 32) s_first[threadIdx.x] = (uint32_t)rv[threadIdx.x], s_entry[threadIdx.x] = (uint32_t)rv[32 + threadIdx.x];
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(a.revbook + 256);
  for (int i = threadIdx.x; i < a.bklen; i += blockDim.x) s_keys[i] = keys[i];
  __syncthreads();
  if (threadIdx.x == 0) {  // longest length: last l with a code (entry[l+1] > entry[l])
    int m = 1;
    for (int l = 1; l < 31; l++)
      if (s_entry[l + 1] > s_entry[l]) m = l;
    s_maxl = m;
  }
  __syncthreads();
  const int maxl = s_maxl;
  // two-symbol table (same rule as the reference decoder, applied twice)
  for (int i = threadIdx.x; i < (1 << kLutBits); i += blockDim.x) {
    uint32_t s0 = 0, s1 = 0;
    const uint32_t l0 = canon_one((uint32_t)i, kLutBits, s_first, s_entry, s_keys, a.bklen, maxl, s0);
    uint32_t e = 0;
    if (l0) {
      const int rest = kLutBits - (int)l0;
      const uint32_t l1 = rest > 0 ? canon_one((uint32_t)i & ((1u << rest) - 1), rest, s_first, s_entry, s_keys,
                                               a.bklen, maxl, s1)
                                   : 0u;
      e = l1 ? lut_pack(2, l0 + l1, s0, s1) : lut_pack(1, l0, s0, 0);
    }
    lut[i] = e;
  }
  __syncthreads();

  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.pardeg) return;
  const size_t obase = (size_t)c * a.sublen;
  if (obase >= a.n) return;
  const uint32_t nsym = (uint32_t)((a.n - obase) < (size_t)a.sublen ? (a.n - obase) : (size_t)a.sublen);
  const uint32_t* src = a.bitstream + a.par_entry[c];
  const uint32_t ncell = (a.par_nbit[c] + 31) >> 5;
  uint16_t* dst = a.out + obase;
  uint16_t* my_ring = reinterpret_cast<uint16_t*>(ring + threadIdx.x * kRingStride);

  // bit supply: 4-cell groups, the next group's loads in flight while this one is consumed
  auto ld = [&](uint32_t i) -> uint32_t { return i < ncell ? src[i] : 0u; };
  uint32_t g0 = ld(0), g1 = ld(1), g2 = ld(2), g3 = ld(3);
  uint32_t h0 = ld(4), h1 = ld(5), h2 = ld(6), h3 = ld(7);
  uint32_t next = 8;
  uint64_t buf = 0;
  int avail = 0;
  uint32_t j = 0;

  auto emit = [&](uint32_t sym) {
    my_ring[j & (kRing - 1)] = (uint16_t)sym;
    j++;
    if ((j & 15) == 0) {  // a half ring is complete: 32 B to HBM
      const uint4* q = reinterpret_cast<const uint4*>(my_ring + ((j - 16) & (kRing - 1)));
      uint4* d = reinterpret_cast<uint4*>(dst + j - 16);
      d[0] = q[0];
      d[1] = q[1];
    }
  };

  auto decode_some = [&]() {
    while (avail > 32 && j < nsym) {
      const uint32_t e = lut[buf >> (64 - kLutBits)];
      const uint32_t ns = e >> 30;
      if (ns) {
        const uint32_t bits = (e >> 25) & 31u;
        emit((e >> 5) & 1023u);
        if (ns == 2 && j < nsym) emit((e >> 15) & 1023u);  // (a 2nd symbol past the chunk end is dropped)
        buf <<= bits;
        avail -= (int)bits;
      }
      else {  // code longer than the table: canonical search on up to 27 bits
        uint32_t sym = 0;
        const uint32_t l = canon_one((uint32_t)(buf >> (64 - kLmax)), kLmax, s_first, s_entry, s_keys, a.bklen,
                                     maxl, sym);
        const uint32_t ll = l ? l : 1u;
        emit(sym);
        buf <<= ll;
        avail -= (int)ll;
      }
    }
  };

  while (j < nsym) {
    buf |= (uint64_t)g0 << (32 - avail), avail += 32;
    decode_some();
    buf |= (uint64_t)g1 << (32 - avail), avail += 32;
    decode_some();
    buf |= (uint64_t)g2 << (32 - avail), avail += 32;
    decode_some();
    buf |= (uint64_t)g3 << (32 - avail), avail += 32;
    decode_some();
    g0 = h0, g1 = h1, g2 = h2, g3 = h3;
    h0 = ld(next), h1 = ld(next + 1), h2 = ld(next + 2), h3 = ld(next + 3);
    next += 4;
  }
  // tail: symbols not yet flushed
  for (uint32_t t = j & ~15u; t < j; t++) dst[t] = my_ring[t & (kRing - 1)];
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
