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
//  * decode: the reference decodes one chunk per thread, bit by bit (hf_kernels.cuhip.inl:
//    331-396) -- 65,536 serial threads at 512^3.  Here one WAVE decodes a chunk: its bits are
//    split into 64 segments decoded in parallel from guessed starts, corrected by Huffman
//    self-synchronisation; a 4096-entry LDS table resolves up to two codewords per lookup;
//    cells and output are staged in LDS so HBM sees coalesced reads and 16-B writes.
#include "common.hh"
#include "hf_device.hh"
#include "kernels.hh"
#include "pub_device.hh"

namespace cusz_amd {

namespace {


// inclusive wave64 prefix sum with DPP (row_shr inside 16-lane rows, then row_bcast15/31 across
// rows): six VALU ops instead of six LDS-routed ds_bpermute round trips
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int /*lane*/)
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



// Pack this thread's codewords (MSB-first, starting at bit `pos` of the chunk) into the LDS
// cell buffer.  Words that only this thread touches are plain stores; the first word (when
// `pos` is not word aligned) and the trailing partial word may be shared with neighbouring
// threads and are merged with LDS atomic OR (the buffer is zeroed beforehand).
template <int N>
__device__ __forceinline__ void pack_words(uint32_t* cells, uint32_t pos, const uint32_t (&w)[N], int mine)
{
  uint32_t q = pos >> 5;
  uint64_t acc = 0;
  uint32_t fill = pos & 31;  // bits already owned by earlier threads in word q
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

// codes are read 16 per lane per round (two 16-B loads, issued for the next round before the
// current one is packed)
constexpr int kEncW = 4;    // chunks (waves) per workgroup
constexpr int kRound = 16;  // codes per lane per round

__device__ __forceinline__ void load_codes16(const uint16_t* p, int mine, uint32_t (&v)[8], bool vec)
{
  if (vec) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
  }
  else {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t lo = 2 * i < mine ? p[2 * i] : 0u, hi = 2 * i + 1 < mine ? p[2 * i + 1] : 0u;
      v[i] = lo | (hi << 16);
    }
  }
}


// ---- three-phase encoder (reference layout) ----------------------------------------------------
// A decoupled look-back serialises workgroups on their predecessors' prefixes; on MI355X that
// latency, not bandwidth, bounds it (measured in round 1).  Here:
//  (1) k_hf_pack: persistent waves, one chunk per wave at a time, codes prefetched a round
//      ahead; the chunk's cells go to a scratch slot at a fixed worst-case stride;
//  (2) k_hf_tile_sums: cells and bits per tile of 64 chunks; its last workgroup scans the tile
//      totals into tile offsets (k_hf_tile_scan, a launch of its own, past kFusedTiles tiles);
//  (3) k_hf_gather: per tile, par_entry from the tile offset + an in-tile scan, then the
//      chunks' cells copied to their final place (coalesced).
// The extra 2 x (compressed bytes) of traffic is far cheaper than the look-back chain.
static int enc_wave_cellcap(int sublen) { return ((sublen * kLmax / 32 + 2) + 3) / 4 * 4; }
static size_t hf_encode_tile_words(int pardeg) { return 2 * (((size_t)pardeg + 63) / 64) + 4; }
constexpr int kPackWaves = 4;
// per-tile cell totals (tile = kGatherTile consecutive chunks)
constexpr int kGatherTile = 64;
// k_hf_tile_sums' last workgroup scans up to kFusedTiles tile totals in one pass (256 threads)
constexpr int kScanPer = 8;
constexpr int kFusedTiles = 256 * kScanPer;

__global__ void __launch_bounds__(64 * kPackWaves) k_hf_pack(HfEncodeArgs a, int cellcap)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_book = smem;                          // bklen words (rounded to 4)
  uint32_t* s_cells = smem + ((a.bklen + 3) & ~3);  // kPackWaves * cellcap words
  for (int i = threadIdx.x; i < a.bklen; i += blockDim.x) s_book[i] = a.book[i];
  for (int i = threadIdx.x; i < kPackWaves * cellcap / 4; i += blockDim.x)
    reinterpret_cast<uint4*>(s_cells)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int stride = gridDim.x * kPackWaves;
  const int per = a.sublen / 64 < kRound ? a.sublen / 64 : kRound;  // codes per lane per round
  const int span = per * 64;
  const bool vec_ok = per == kRound;
  uint32_t* cells = s_cells + wid * cellcap;
  auto chunk_len = [&](int c) -> int {
    const size_t start = (size_t)c * a.sublen;
    return (int)((a.n - start) < (size_t)a.sublen ? (a.n - start) : (size_t)a.sublen);
  };
  auto load_round = [&](int c, int r0, int cnt, uint32_t(&v)[8]) {
    const int lo = r0 + lane * per, mine = min(max(cnt - lo, 0), per);
    load_codes16(a.codes + (size_t)c * a.sublen + lo, mine, v, vec_ok && mine == per);
  };

  int c = blockIdx.x * kPackWaves + wid;
  uint32_t nxt[8];
  if (c < a.pardeg) load_round(c, 0, chunk_len(c), nxt);
  for (; c < a.pardeg; c += stride) {
    const int cnt = chunk_len(c);
    uint32_t nbits = 0;
    for (int r0 = 0; r0 < cnt; r0 += span) {
      const int lo = r0 + lane * per, mine = min(max(cnt - lo, 0), per);
      uint32_t cur[8];
#pragma unroll
      for (int i = 0; i < 8; i++) cur[i] = nxt[i];
      if (r0 + span < cnt)  // prefetch: next round of this chunk, or the first of the next chunk
        load_round(c, r0 + span, cnt, nxt);
      else if (c + stride < a.pardeg)
        load_round(c + stride, 0, chunk_len(c + stride), nxt);
      uint32_t w[kRound], bits = 0;
#pragma unroll
      for (int i = 0; i < kRound; i++) {
        const uint32_t code = (cur[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
        w[i] = i < mine ? s_book[code] : 0u;
        bits += w[i] >> 27;
      }
      const uint32_t inc = wave_incl_scan(bits, lane);
      // full rounds whose 4-code groups each fit 64 bits (every lane): Horner-pack each group and
      // OR it in (hf_device.hh pack4_or); otherwise the general word-by-word packer
      uint32_t lg[kRound / 4];
      bool fast = mine == kRound;
#pragma unroll
      for (int g = 0; g < kRound / 4; g++) {
        lg[g] = (w[4 * g] >> 27) + (w[4 * g + 1] >> 27) + (w[4 * g + 2] >> 27) + (w[4 * g + 3] >> 27);
        fast = fast && lg[g] <= 64u;
      }
      if (__builtin_expect(__ballot(!fast) == 0, 1)) {
        uint32_t p = nbits + inc - bits;
#pragma unroll
        for (int g = 0; g < kRound / 4; g++) {
          const uint32_t wg[4] = {w[4 * g], w[4 * g + 1], w[4 * g + 2], w[4 * g + 3]};
          hfd::pack4_or(cells, p, wg, lg[g]);
          p += lg[g];
        }
      }
      else if (mine)
        pack_words<kRound>(cells, nbits + inc - bits, w, mine);
      nbits += __shfl(inc, 63);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint32_t nc = (nbits + 31) >> 5;
    uint32_t* dst = a.temp + (size_t)c * cellcap;
    for (uint32_t i = lane; i < nc; i += 64) {
      dst[i] = cells[i];
      cells[i] = 0u;  // ready for the next chunk
    }
    if (lane == 0) a.par_nbit[c] = nbits;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// per-tile cell totals, one wave per tile.  With a ticket (kPubTicketWords words zeroed per call)
// and at most kFusedTiles tiles the last workgroup also does k_hf_tile_scan's work: the exclusive
// scan of the totals, kScanPer consecutive tiles per thread in one pass (one launch fewer).
// (Per-tile bit totals, not one atomic per tile on the single total_nbit word: those queued
// 2,048 waves at the L2 -- 27 us for config 5's 131,072 chunks.)
__global__ void __launch_bounds__(256) k_hf_tile_sums(const uint32_t* __restrict__ par_nbit, int pardeg,
                                                      uint32_t* __restrict__ tile_sum, uint32_t* __restrict__ tile_bits,
                                                      int ntiles, uint32_t* ticket, unsigned long long* total_nbit)
{
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int t = blockIdx.x * 4 + wid;
  if (t < ntiles) {
    uint32_t acc = 0, bits = 0;
    for (int i = t * kGatherTile + lane; i < min((t + 1) * kGatherTile, pardeg); i += 64) {
      const uint32_t nb = par_nbit[i];
      acc += (nb + 31) >> 5;
      bits += nb;  // a tile of 64 chunks of <= 8192 codes of <= 27 bits: < 2^32
    }
    acc = wave_sum(acc);
    bits = wave_sum(bits);
    if (lane == 0) {  // (agent scope: the last workgroup may read them from another XCD)
      __hip_atomic_store(tile_sum + t, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(tile_bits + t, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (!ticket || !last_block(ticket)) return;
  __shared__ uint32_t s_wc[4];
  __shared__ unsigned long long s_wb[4];
  unsigned long long tb = 0;  // this thread's share of the bit total
  uint32_t carry = 0;
  for (int base = 0; base < ntiles; base += 256 * kScanPer) {
    uint32_t v[kScanPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      const int i = base + (int)threadIdx.x * kScanPer + k;
      v[k] = i < ntiles ? __hip_atomic_load(tile_sum + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      tb += i < ntiles ? __hip_atomic_load(tile_bits + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      sum += v[k];
    }
    const uint32_t inc = wave_incl_scan(sum, lane);
    if (lane == 63) s_wc[wid] = inc;
    __syncthreads();
    uint32_t run = carry, tot = carry;
    for (int w = 0; w < 4; w++) tot += s_wc[w], run += w < wid ? s_wc[w] : 0u;
    run += inc - sum;
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      const int i = base + (int)threadIdx.x * kScanPer + k;
      if (i < ntiles) tile_sum[i] = run;
      run += v[k];
    }
    carry = tot;
    __syncthreads();
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) tb += __shfl_xor(tb, d);
  if (lane == 0) s_wb[wid] = tb;
  __syncthreads();
  if (threadIdx.x == 0 && total_nbit) {
    unsigned long long tot = 0;
    for (int w = 0; w < 4; w++) tot += s_wb[w];
    *total_nbit = tot;
  }
}

// exclusive scan of the tile totals in place (one workgroup; ntiles <= 1024 * 8)
__global__ void __launch_bounds__(1024) k_hf_tile_scan(uint32_t* __restrict__ tile_sum,
                                                      const uint32_t* __restrict__ tile_bits, int ntiles,
                                                      unsigned long long* total_nbit)
{
  __shared__ uint32_t s_wave[16];
  __shared__ uint32_t s_carry;
  __shared__ unsigned long long s_bits[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  unsigned long long bits = 0;  // this thread's share of the total bit count
  for (int base = 0; base < ntiles; base += 1024 * 8) {
    uint32_t v[8], sum = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int i = base + tid * 8 + k;
      v[k] = i < ntiles ? tile_sum[i] : 0u;
      bits += i < ntiles ? tile_bits[i] : 0u;
      sum += v[k];
    }
    const uint32_t inc = wave_incl_scan(sum, lane);
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint32_t run = s_carry;
    for (int w = 0; w < wid; w++) run += s_wave[w];
    const uint32_t tot = s_carry + [&] { uint32_t t2 = 0; for (int w = 0; w < 16; w++) t2 += s_wave[w]; return t2; }();
    run += inc - sum;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int i = base + tid * 8 + k;
      if (i < ntiles) tile_sum[i] = run;
      run += v[k];
    }
    __syncthreads();
    if (tid == 0) s_carry = tot;
    __syncthreads();
  }
  if (!total_nbit) return;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) bits += __shfl_xor(bits, d);
  if (lane == 0) s_bits[wid] = bits;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < 16; w++) t += s_bits[w];
    *total_nbit = t;
  }
}

// one workgroup per tile: wave 0 turns the tile offset + in-tile exclusive scan into
// par_entry; then the 4 waves copy the tile's chunks scratch -> bitstream, two chunks per wave
// per iteration with all their loads issued before the stores.
__global__ void __launch_bounds__(256) k_hf_gather(HfEncodeArgs a, int cellcap, const uint32_t* __restrict__ tile_off)
{
  __shared__ uint32_t s_ent[kGatherTile], s_nc[kGatherTile];
  const int t = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c0 = t * kGatherTile;
  if (wid == 0) {
    const int c = c0 + lane;
    const uint32_t nc = c < a.pardeg ? (a.par_nbit[c] + 31) >> 5 : 0u;
    const uint32_t inc = wave_incl_scan(nc, lane);
    const uint32_t off = tile_off[t] + inc - nc;
    s_ent[lane] = off, s_nc[lane] = nc;
    if (c < a.pardeg) a.par_entry[c] = off;
  }
  __syncthreads();
  const int nch = min(kGatherTile, a.pardeg - c0);
  for (int j = 2 * wid; j < nch; j += 8) {  // chunk pairs (j, j + 1)
    const int j2 = j + 1;
    const uint32_t n1 = s_nc[j], e1 = s_ent[j];
    const uint32_t n2 = j2 < nch ? s_nc[j2] : 0u, e2 = j2 < nch ? s_ent[j2] : 0u;
    const uint32_t* src1 = a.temp + (size_t)(c0 + j) * cellcap;
    const uint32_t* src2 = a.temp + (size_t)(c0 + j2) * cellcap;
    for (uint32_t i = lane; i < max(n1, n2); i += 256) {
      uint32_t v1[4], v2[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t ii = i + 64 * k;
        v1[k] = ii < n1 ? src1[ii] : 0u;
        v2[k] = ii < n2 ? src2[ii] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t ii = i + 64 * k;
        if (ii < n1) a.bitstream[e1 + ii] = v1[k];
        if (ii < n2) a.bitstream[e2 + ii] = v2[k];
      }
    }
  }
}

// ============================== decode ======================================================
// Tables (built once per decompress by k_hf_tables into a device scratch, copied to LDS):
//  L1: 4096 entries indexed by the next 12 stream bits.  An entry resolves one or two whole
//      codewords: [31:30] nsym (1|2), [29:25] bits of the nsym codes, [24:20] length of the
//      first code, [19:10] second symbol, [9:0] first symbol; 0 if the code is longer.
//  L2: single-symbol entries indexed DIRECTLY by the next 16 bits.  Canonical codes put every
//      code longer than 12 bits below first[12] (hf_canon.seq.cc: longer codes are numerically
//      smaller), so only windows with a 12-bit prefix < first[12] reach it: the table is
//      first[12] * 16 entries, and both lookups can be issued together (no pointer chase).
//  Codes longer than 16 bits (or past the table) take the slow path (threshold counting).
constexpr int kLutBits = 12;
constexpr int kL1 = 1 << kLutBits;
constexpr int kTabMaxl = kL1;       // longest code length
constexpr int kTabFirst = kL1 + 1;  // [32] first[l] (0 beyond the longest code)
constexpr int kTabBase = kL1 + 33;  // [32] entry[l] - first[l]
constexpr int kTabL2 = kL1 + 128;   // second level
constexpr int kL2Cap = 2048;        // second-level entries (the last one stays 0)
constexpr int kL2Bits = 16;         // second level: codes of up to 16 bits
static_assert(kTabL2 + kL2Cap <= kHfDecTableWords, "decode table scratch too small");
constexpr int kLongLens = kLmax - kLutBits;  // lengths only the slow path resolves

__device__ __forceinline__ uint32_t lut_pack(uint32_t nsym, uint32_t bits, uint32_t l0, uint32_t s0, uint32_t s1)
{
  return (nsym << 30) | (bits << 25) | (l0 << 20) | (s1 << 10) | s0;
}

__device__ __forceinline__ int longest_code(const uint32_t* entry)
{
  int m = 1;  // last l with a code (entry[l+1] > entry[l])
  for (int l = 1; l < 31; l++)
    if (entry[l + 1] > entry[l]) m = l;
  return m;
}

// One symbol from a left-justified window, reference rule (hf_kernels.cuhip.inl:351-365: the
// first length l with prefix_l >= first[l]).  The thresholds first[l] * 2^(32-l) never increase
// with l (canonical construction: first[l] >= (first[l+1] + count[l+1]) / 2), so the lengths
// that fail form a prefix 1..m and the code length is 1 + the number of failing lengths.
// (The prefix form prefix_l < first[l] is exact even when first[l] = 2^l.)
__device__ __forceinline__ uint32_t tab_decode1(uint32_t v, const uint32_t (&first)[kLmax + 1], int maxl,
                                                const uint32_t* base, const uint16_t* keys, uint32_t bklen,
                                                uint32_t& sym)
{
  uint32_t l = 1;
#pragma unroll
  for (int k = 1; k <= kLmax; k++) l += (k <= maxl && (v >> (32 - k)) < first[k]) ? 1u : 0u;
  if (l > (uint32_t)maxl) l = (uint32_t)maxl;
  sym = keys[min(base[l] + (v >> (32 - l)), bklen - 1)];
  return l;
}

__global__ void __launch_bounds__(1024) k_hf_tables(const uint8_t* revbook, int bklen, uint32_t* tab)
{
  __shared__ uint32_t s_first[32], s_entry[32], s_base[32];
  __shared__ uint16_t s_keys[kMaxBklen];
  const int tid = threadIdx.x;
  const int32_t* rv = reinterpret_cast<const int32_t*>(revbook);
  if (tid < 32) s_first[tid] = (uint32_t)rv[tid], s_entry[tid] = (uint32_t)rv[32 + tid];
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(revbook + 256);
  for (int i = tid; i < bklen; i += blockDim.x) s_keys[i] = keys[i];
  __syncthreads();
  const int maxl = longest_code(s_entry);
  if (tid < 32) {
    tab[kTabFirst + tid] = (tid >= 1 && tid <= maxl) ? s_first[tid] : 0u;  // slow path
    s_base[tid] = s_entry[tid] - s_first[tid];
    tab[kTabBase + tid] = s_entry[tid] - s_first[tid];
  }
  if (tid == 0) tab[kTabMaxl] = (uint32_t)maxl;
  __syncthreads();
  uint32_t thr[kLmax + 1];  // first[l]
#pragma unroll
  for (int k = 0; k <= kLmax; k++) thr[k] = s_first[k];
  const uint32_t ub = (uint32_t)bklen;
  const uint32_t P = maxl > kLutBits ? min(s_first[kLutBits], (uint32_t)kL1) : 0u;

  // L1: one or two whole codewords of <= 12 bits; 0 for the long-code prefixes [0, P)
  for (uint32_t i = tid; i < (uint32_t)kL1; i += blockDim.x) {
    const uint32_t v = i << (32 - kLutBits);
    uint32_t s0, s1, e = 0;
    const uint32_t l0 = tab_decode1(v, thr, maxl, s_base, s_keys, ub, s0);
    if (i >= P && l0 <= (uint32_t)kLutBits) {
      const uint32_t rest = kLutBits - l0;
      const uint32_t l1 = rest ? tab_decode1(v << l0, thr, maxl, s_base, s_keys, ub, s1) : 99u;
      e = l1 <= rest ? lut_pack(2, l0 + l1, l0, s0, s1) : lut_pack(1, l0, l0, s0, 0);
    }
    tab[i] = e;
  }
  // L2 (direct): indexed by the top 16 bits of windows whose 12-bit prefix is < P; codes of
  // 13..16 bits; 0 (slow path) beyond 16 bits or past the table (its last slot stays 0)
  const uint32_t n2 = min(P << (kL2Bits - kLutBits), (uint32_t)kL2Cap - 1);
  for (uint32_t q = tid; q < (uint32_t)kL2Cap; q += blockDim.x) {
    uint32_t e = 0;
    if (q < n2) {
      uint32_t s0;
      const uint32_t l = tab_decode1(q << (32 - kL2Bits), thr, maxl, s_base, s_keys, ub, s0);
      if (l <= (uint32_t)kL2Bits) e = lut_pack(1, l, l, s0, 0);
    }
    tab[kTabL2 + q] = e;
  }
}

__device__ __forceinline__ void wave_sync()
{
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

struct HfTables {
  const uint32_t* l1;
  const uint32_t* l2;
  const uint32_t* base;  // entry[l] - first[l]
  const uint16_t* keys;
  uint32_t bklen;
  uint32_t first[kLongLens];  // first[l], l = 13..27 (wave-uniform, SGPRs)
};

// entry for the codeword(s) at the top of `win`: L1 and L2 read together, then the rare
// untabulated case
__device__ __forceinline__ uint32_t hf_entry(const HfTables& t, uint32_t win)
{
  const uint32_t e1 = t.l1[win >> (32 - kLutBits)];
  const uint32_t e2 = t.l2[min(win >> (32 - kL2Bits), (uint32_t)kL2Cap - 1)];
  uint32_t e = (e1 >> 30) ? e1 : e2;
  if (__builtin_expect(!(e >> 30), 0)) {  // count failed lengths (all <= 12 failed)
    uint32_t l = kLutBits + 1;
#pragma unroll
    for (int q = 0; q < kLongLens; q++) l += (win >> (32 - (kLutBits + 1 + q))) < t.first[q] ? 1u : 0u;
    if (l > kLmax) l = kLmax;
    const uint32_t s = t.keys[min(t.base[l] + (win >> (32 - l)), t.bklen - 1)];
    e = lut_pack(1, l, l, s, 0);
  }
  return e;
}

template <typename Tab>
__device__ __forceinline__ void load_tables(const HfDecodeArgs& a, uint32_t* s_l1, uint32_t* s_l2, uint32_t* s_base,
                                            uint16_t* s_keys, Tab& tb)
{
  const uint16_t* keys = reinterpret_cast<const uint16_t*>(a.revbook + 256);
  for (int i = threadIdx.x; i < a.bklen; i += blockDim.x) s_keys[i] = keys[i];
  for (int i = threadIdx.x; i < kL1 / 4; i += blockDim.x)
    reinterpret_cast<uint4*>(s_l1)[i] = reinterpret_cast<const uint4*>(a.lut)[i];
  for (int i = threadIdx.x; i < kL2Cap / 4; i += blockDim.x)
    reinterpret_cast<uint4*>(s_l2)[i] = reinterpret_cast<const uint4*>(a.lut + kTabL2)[i];
  if (threadIdx.x < 32) s_base[threadIdx.x] = a.lut[kTabBase + threadIdx.x];
  tb.l1 = s_l1;
  tb.l2 = s_l2;
  tb.base = s_base;
  tb.keys = s_keys;
  tb.bklen = (uint32_t)a.bklen;
#pragma unroll
  for (int q = 0; q < kLongLens; q++) tb.first[q] = __builtin_amdgcn_readfirstlane(a.lut[kTabFirst + kLutBits + 1 + q]);
}

#ifdef CUSZ_AMD_DEC_PROFILE
// per-wave phase clocks and step counts (diagnostic build only; read by psz_amd_debug_decode_profile)
__device__ unsigned long long g_dec_prof[4096 * 16];
#define DP_STEP(x) (x)++
#else
#define DP_STEP(x) (void)0
#endif

struct DecProf {
#ifdef CUSZ_AMD_DEC_PROFILE
  unsigned long long v[16] = {0};
  unsigned long long t = 0;
  __device__ void start() { t = __builtin_readcyclecounter(); }
  __device__ void mark(int k)
  {
    const unsigned long long n = __builtin_readcyclecounter();
    v[k] += n - t;
    t = n;
  }
  __device__ void add(int k, uint32_t x) { v[k] += x; }
  __device__ void add_max(int k, uint32_t x)
  {
    for (int d = 32; d > 0; d >>= 1) x = max(x, (uint32_t)__shfl_xor(x, d));
    v[k] += x;
  }
#else
  __device__ void start() {}
  __device__ void mark(int) {}
  __device__ void add(int, uint32_t) {}
  __device__ void add_max(int, uint32_t) {}
#endif
};

constexpr int kCad = 4;         // <= 4 * 27 bits consumed per cadence < one 128-bit block

// ---- windowed lane-per-chunk decoder ------------------------------------------------------------
// Each lane decodes one whole chunk (every codeword decoded once).  The workgroup's 512 chunks
// are staged through LDS in windows of 16 cells per chunk, double-buffered with LDS-DMA
// (global_load_lds_dwordx4, four lanes per 64-B window piece, so one DMA instruction fetches
// 16 chunks' windows as 64-B segments) while the current window is decoded; a barrier separates
// windows.  Decoding touches only LDS and registers: the bit buffer lives in registers and is
// refilled from the window one cell ahead; the two table lookups are issued together.  Output
// goes through a 32-symbol LDS ring per lane and is flushed cooperatively: ready lanes post a
// request, two helper lanes per request store its 32 B, so stores leave as 32-B segments.
constexpr int kWinLanes = 512;  // chunks per workgroup (8 waves)
constexpr int kWin = 16;        // cells per window per chunk
constexpr int kWinOut = 32;     // output ring symbols per lane

__global__ void __launch_bounds__(kWinLanes) k_hf_decode_win(HfDecodeArgs a)
{
  __shared__ __attribute__((aligned(16))) uint32_t s_l1[kL1];
  __shared__ __attribute__((aligned(16))) uint32_t s_l2[kL2Cap];
  __shared__ uint32_t s_base[32];
  __shared__ uint16_t s_keys[kMaxBklen];
  __shared__ __attribute__((aligned(16))) uint32_t s_in[2 * kWinLanes * kWin];        // [half][lane][16]
  __shared__ __attribute__((aligned(16))) uint32_t s_out[kWinOut / 2 * kWinLanes];    // [sym pair][lane]
  __shared__ uint32_t s_gb[kWinLanes];                                                // chunk base, 16-B units
  __shared__ uint32_t s_lim[kWinLanes];                                               // cells from s_gb (0: none)
  __shared__ uint32_t s_req[kWinLanes / 64][64];                                      // flush requests per wave
  __shared__ uint32_t s_nwin;
  HfTables tb;
  load_tables(a, s_l1, s_l2, s_base, s_keys, tb);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t c0 = blockIdx.x * kWinLanes;
  const uint32_t c = c0 + tid;
  const size_t obase = (size_t)c * a.sublen;
  const bool live = c < (uint32_t)a.pardeg && obase < a.n;
  const uint32_t nsym = live ? (uint32_t)min((size_t)a.sublen, a.n - obase) : 0u;
  const uint32_t nbit = live ? a.par_nbit[c] : 0u;
  const uint32_t entry = live ? a.par_entry[c] : 0u;
  const uint32_t ncell = (nbit + 31) >> 5;
  const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(a.bitstream + entry) & 15);
  const uint4* gb = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.bitstream + entry) - mis);
  const uint32_t skip = mis >> 2;
  const uint32_t lim = live ? skip + ncell : 0u;  // cells of this chunk, counted from gb
  if (tid == 0) s_nwin = 0;
  // chunk bases as 16-B offsets from an aligned base (pointers kept in LDS would load as flat)
  const uint4* gbase = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.bitstream) -
                                                      (reinterpret_cast<uintptr_t>(a.bitstream) & 15));
  s_gb[tid] = (uint32_t)(gb - gbase);
  s_lim[tid] = lim;
  // the last chunk's final partial 16-B piece is read by cells (never past the stream's end)
  const bool tail = live && c + 1 == (uint32_t)a.pardeg && (lim & 3);
  const uint32_t tq = tail ? (lim - 1) & ~3u : 0u;  // first cell of that piece
  uint32_t t0 = 0, t1 = 0, t2 = 0;
  if (tail) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(gb) + tq;
    t0 = q[0];
    if (lim - tq > 1) t1 = q[1];
    if (lim - tq > 2) t2 = q[2];
  }
  __syncthreads();
  atomicMax(&s_nwin, (lim + kWin - 1) / kWin);

  const uint4* gsafe = reinterpret_cast<const uint4*>(a.lut);
  // Window w of every chunk is fetched as 32 x (16 chunks x 64 B) segments, four per wave:
  // lane t covers chunk 16 g + t/4, piece t%4.  Loads go to registers at the start of a
  // phase and are written to LDS at its end (an LDS-DMA would make every LDS read of the
  // phase wait for it: the compiler cannot tell the two halves apart).
  uint4 sv0, sv1, sv2, sv3;
#define CUSZ_STAGE_LOAD(W)                                                                   \
  do {                                                                                        \
    uint4* svp[4] = {&sv0, &sv1, &sv2, &sv3};                                                 \
    _Pragma("unroll") for (int k = 0; k < 4; k++)                                             \
    {                                                                                         \
      const int g = wid * 4 + k;                                                              \
      const int L = g * 16 + (lane >> 2), j = lane & 3;                                       \
      const uint32_t q = (W) * kWin + 4 * j;                                                  \
      const uint32_t ll = s_lim[L];                                                           \
      const bool tl = (L + c0 + 1 == (uint32_t)a.pardeg) && (ll & 3);                         \
      const bool ok = q < ll && !(tl && q + 4 > ll);                                          \
      *svp[k] = *(ok ? gbase + s_gb[L] + (q >> 2) : gsafe);                                   \
    }                                                                                         \
  } while (0)
#define CUSZ_STAGE_STORE(W)                                                                  \
  do {                                                                                        \
    uint4* base = reinterpret_cast<uint4*>(s_in + ((W) & 1) * (kWinLanes * kWin) + wid * 64 * kWin); \
    base[lane] = sv0;                                                                         \
    base[64 + lane] = sv1;                                                                    \
    base[128 + lane] = sv2;                                                                   \
    base[192 + lane] = sv3;                                                                   \
  } while (0)
  auto patch_tail = [&](uint32_t w) {  // the owner lane writes its partial piece after the DMA landed
    if (tail && (tq >> 4) == w) {
      uint32_t* r = s_in + (w & 1) * (kWinLanes * kWin) + tid * kWin + (tq & 15);
      r[0] = t0, r[1] = t1, r[2] = t2, r[3] = 0u;
    }
  };
  auto cell = [&](uint32_t n) -> uint32_t { return s_in[((n >> 4) & 1) * (kWinLanes * kWin) + tid * kWin + (n & 15)]; };

  __syncthreads();
  const uint32_t nwin = s_nwin;
  CUSZ_STAGE_LOAD(0u);
  CUSZ_STAGE_STORE(0u);
  __syncthreads();
  patch_tail(0);

  uint64_t buf = ((uint64_t)cell(skip) << 32) | cell(skip + 1);
  uint32_t avail = 64, nw = skip + 2;
  uint32_t nxt = cell(nw);
  uint32_t cnt = 0, flushed = 0;
  // output ring, slot-major ([symbol pair][lane]): a wave's 64 ring writes hit 64 banks
  uint16_t* oring = reinterpret_cast<uint16_t*>(s_out);
  auto oslot = [&](uint32_t i) -> uint32_t { return (((i & (kWinOut - 1)) >> 1) * kWinLanes + tid) * 2 + (i & 1); };

  // cooperative flush: ready lanes post (lane << 16 | flushed); helpers store 2 x 16 B each
  auto flush = [&]() {
    const bool ready = cnt - flushed >= 16u;
    const uint64_t m = __ballot(ready);
    if (!m) return;
    const uint32_t n = (uint32_t)__popcll(m);
    if (ready) {
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
      s_req[wid][rank] = ((uint32_t)lane << 16) | flushed;
      flushed += 16;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i0 = 0; i0 < n; i0 += 32) {
      const uint32_t i = i0 + (lane >> 1), j = lane & 1;
      if (i < n) {
        const uint32_t r = s_req[wid][i];
        const uint32_t lf = r >> 16, fl = r & 0xFFFFu;
        const uint32_t L = wid * 64 + lf;
        const uint32_t* srcw = s_out + (((fl & 16u) >> 1) + 4 * j) * kWinLanes + L;  // 4 symbol pairs
        const uint4 v = make_uint4(srcw[0], srcw[kWinLanes], srcw[2 * kWinLanes], srcw[3 * kWinLanes]);
        uint16_t* dst = a.out + (size_t)(c0 + L) * a.sublen + fl + 8 * j;
        *reinterpret_cast<uint4*>(dst) = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };

  DecProf pf;
  pf.start();
  uint32_t iters = 0;
  for (uint32_t w = 0; w < nwin; w++) {
    if (w + 1 < nwin) CUSZ_STAGE_LOAD(w + 1);
    pf.mark(0);
    const uint32_t wend = (w + 1) * kWin;
    const bool last_here = lim <= wend;  // all of this chunk's cells are resident
    while (true) {
      const bool any = cnt < nsym && (nw + 1 < wend || last_here);
      if (!__any(any)) break;
#pragma unroll
      for (int st = 0; st < kCad; st++) {
        if (cnt < nsym && (nw + 1 < wend || last_here)) {
          const uint32_t e = hf_entry(tb, (uint32_t)(buf >> 32));
          const uint32_t l0 = (e >> 20) & 31u;
          const bool both = (e >> 30) == 2u && cnt + 1 < nsym;
          const uint32_t i0 = oslot(cnt), i1 = both ? oslot(cnt + 1) : i0;
          oring[i0] = (uint16_t)(e & 1023u);
          oring[i1] = (uint16_t)(both ? ((e >> 10) & 1023u) : (e & 1023u));
          cnt += both ? 2u : 1u;
          const uint32_t l = both ? ((e >> 25) & 31u) : l0;
          buf <<= l;
          avail -= l;
          if (avail < 32) {
            buf |= (uint64_t)nxt << (32 - avail);
            avail += 32;
            nw++;
            nxt = cell(nw);
          }
        }
      }
      pf.mark(1);
      if (iters & 1) flush();
      pf.mark(2);
      iters++;
    }
    if (w + 1 < nwin) CUSZ_STAGE_STORE(w + 1);
    pf.mark(3);
    __syncthreads();
    pf.mark(4);
    patch_tail(w + 1);
  }
  pf.add(8, iters);
  pf.add(9, nwin);
  pf.add(13, 1u);
#ifdef CUSZ_AMD_DEC_PROFILE
  if (lane == 0 && blockIdx.x * 8 + wid < 4096)
    for (int q = 0; q < 16; q++) g_dec_prof[(blockIdx.x * 8 + wid) * 16 + q] = pf.v[q];
#endif
  // drain: full halves first (cooperatively), then the remainder lane by lane
  flush();
  flush();
  for (uint32_t i = flushed; i < cnt; i++) a.out[obase + i] = oring[oslot(i)];
#undef CUSZ_STAGE_LOAD
#undef CUSZ_STAGE_STORE
}


// ---- wave-per-chunk decoder (for few, long chunks) ------------------------------------------
constexpr int kDecWaves = 4;   // waves per decode workgroup
constexpr int kSyncWin = 64;   // bits of a segment whose codeword starts are remembered


// the 32 stream bits starting at bit `pos` (MSB-first cells)
template <bool GLOBAL>
__device__ __forceinline__ uint32_t window(const uint32_t* cells, uint32_t ncell, uint32_t pos)
{
  const uint32_t w = pos >> 5;
  const uint32_t c0 = cells[w];
  const uint32_t c1 = GLOBAL ? (w + 1 < ncell ? cells[w + 1] : 0u) : cells[w + 1];
  return (uint32_t)((((uint64_t)c0 << 32) | c1) >> (32 - (pos & 31)));
}

// One table step at `pos`: returns the bits consumed and the codewords counted (1 or 2; the
// second only if it starts before `hi`).  `l0` = length of the first codeword, syms in s0/s1.
template <bool GLOBAL>
__device__ __forceinline__ uint32_t dec_step(const uint32_t* cells, uint32_t ncell, uint32_t pos, uint32_t hi,
                                             const HfTables& t, uint32_t& n, uint32_t& l0, uint32_t& s0,
                                             uint32_t& s1)
{
  const uint32_t e = hf_entry(t, window<GLOBAL>(cells, ncell, pos));
  l0 = (e >> 20) & 31u;
  s0 = e & 1023u;
  s1 = (e >> 10) & 1023u;
  const bool both = (e >> 30) == 2 && pos + l0 < hi;
  n = both ? 2u : 1u;
  return both ? ((e >> 25) & 31u) : l0;
}

// Pass A: count codewords starting in [lo, hi) from the guess lo; remember which of the first
// kSyncWin bits are codeword starts on this path (bm).  Returns the count; end = first start >= hi.
template <bool GLOBAL>
__device__ __forceinline__ uint32_t pass_count(const uint32_t* cells, uint32_t ncell, uint32_t lo, uint32_t hi,
                                               const HfTables& t, uint32_t& end, uint64_t& bm, uint32_t& steps)
{
  uint32_t cnt = 0, pos = lo;
  bm = 0;
  while (pos < hi) {
    DP_STEP(steps);
    uint32_t n, l0, s0, s1;
    const uint32_t adv = dec_step<GLOBAL>(cells, ncell, pos, hi, t, n, l0, s0, s1);
    const uint32_t d = pos - lo;
    if (d < kSyncWin) {
      bm |= 1ull << d;
      if (n == 2 && d + l0 < kSyncWin) bm |= 1ull << (d + l0);
    }
    cnt += n;
    pos += adv;
  }
  end = pos;
  return cnt;
}

// Re-count from the corrected start s (>= lo).  Huffman codes self-synchronise: once this path
// lands on a codeword start of pass A's path (bm), the rest of the segment is pass A's.
template <bool GLOBAL>
__device__ __forceinline__ uint32_t pass_resync(const uint32_t* cells, uint32_t ncell, uint32_t lo, uint32_t hi,
                                                uint32_t s, const HfTables& t, uint64_t bm, uint32_t cnt_a,
                                                uint32_t end_a, uint32_t& end, uint32_t& steps)
{
  uint32_t cnt = 0, pos = s;
  while (pos < hi) {
    DP_STEP(steps);
    const uint32_t d = pos - lo;
    if (d < kSyncWin && ((bm >> d) & 1ull)) {
      end = end_a;
      return cnt + cnt_a - (uint32_t)__builtin_popcountll(bm & ((1ull << d) - 1ull));
    }
    uint32_t n, l0, s0, s1;
    pos += dec_step<GLOBAL>(cells, ncell, pos, hi, t, n, l0, s0, s1);
    cnt += n;
  }
  end = pos;
  return cnt;
}

template <bool GLOBAL>
__device__ __forceinline__ void pass_emit(const uint32_t* cells, uint32_t ncell, uint32_t pos, uint32_t hi,
                                          const HfTables& t, uint16_t* out, uint32_t& steps)
{
  while (pos < hi) {
    DP_STEP(steps);
    uint32_t n, l0, s0, s1;
    pos += dec_step<GLOBAL>(cells, ncell, pos, hi, t, n, l0, s0, s1);
    out[0] = (uint16_t)s0;
    if (n == 2) out[1] = (uint16_t)s1;
    out += n;
  }
}


template <bool GLOBAL>
__device__ __forceinline__ void decode_chunk(const uint32_t* cells, uint32_t ncell, uint32_t nbit, uint32_t nsym,
                                             const HfTables& t, uint16_t* outs, int lane, DecProf& pf)
{
  const uint32_t seg = (nbit + 63) / 64;
  const uint32_t lo = min(lane * seg, nbit), hi = min(lo + seg, nbit);
  uint32_t end_a, st_a = 0, st_r = 0, st_e = 0;
  uint64_t bm;
  const uint32_t cnt_a = pass_count<GLOBAL>(cells, ncell, lo, hi, t, end_a, bm, st_a);
  pf.mark(1);
  uint32_t start = lo, cnt = cnt_a, end = end_a;
  int it = 0;
  for (; it < 64; it++) {
    uint32_t s_new = __shfl_up(end, 1);
    if (lane == 0) s_new = 0;
    const bool changed = s_new != start;
    if (!__ballot(changed)) break;
    if (changed) {
      start = s_new;
      cnt = pass_resync<GLOBAL>(cells, ncell, lo, hi, start, t, bm, cnt_a, end_a, end, st_r);
    }
  }
  pf.mark(2);
  uint32_t inc = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(inc, d);
    if (lane >= d) inc += v;
  }
  const uint32_t off = inc - cnt;
  if (cnt && off + cnt <= nsym) pass_emit<GLOBAL>(cells, ncell, start, hi, t, outs + off, st_e);
  pf.mark(3);
  pf.add_max(8, st_a);
  pf.add_max(9, st_r);
  pf.add_max(10, st_e);
  pf.add(11, (uint32_t)it);
  pf.add(12, GLOBAL ? 1u : 0u);
  pf.add(13, 1u);
}

__global__ void __launch_bounds__(64 * kDecWaves) k_hf_decode(HfDecodeArgs a, int cellcap)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];
  __shared__ __attribute__((aligned(16))) uint32_t s_l1[kL1];
  __shared__ __attribute__((aligned(16))) uint32_t s_l2[kL2Cap];
  __shared__ uint32_t s_base[32];
  __shared__ uint16_t s_keys[kMaxBklen];
  HfTables tb;
  load_tables(a, s_l1, s_l2, s_base, s_keys, tb);
  __syncthreads();

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* cells = dsm + wid * (cellcap + (((a.sublen + 1) >> 1) + 3) / 4 * 4);
  uint16_t* outs = reinterpret_cast<uint16_t*>(cells + cellcap);

  DecProf pf;
  pf.start();
  for (int c = blockIdx.x * kDecWaves + wid; c < a.pardeg; c += gridDim.x * kDecWaves) {
    const size_t obase = (size_t)c * a.sublen;
    if (obase >= a.n) break;
    const uint32_t nsym = (uint32_t)((a.n - obase) < (size_t)a.sublen ? (a.n - obase) : (size_t)a.sublen);
    const uint32_t nbit = a.par_nbit[c];
    const uint32_t ncell = (nbit + 31) >> 5;
    const uint32_t* src = a.bitstream + a.par_entry[c];
    if (ncell + 2 <= (uint32_t)cellcap) {
      for (uint32_t i = lane; i < ncell; i += 64) cells[i] = src[i];
      if (lane < 2) cells[ncell + lane] = 0;
      wave_sync();
      pf.mark(0);
      decode_chunk<false>(cells, ncell, nbit, nsym, tb, outs, lane, pf);
    }
    else {  // a chunk too big for the staging area: read its cells from global memory
      pf.mark(0);
      decode_chunk<true>(src, ncell, nbit, nsym, tb, outs, lane, pf);
    }
    wave_sync();
    uint16_t* dst = a.out + obase;
    const uint32_t n8 = (obase & 7) ? 0u : nsym >> 3;  // 16-B stores only when aligned
    for (uint32_t i = lane; i < n8; i += 64) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(outs)[i];
    for (uint32_t i = (n8 << 3) + lane; i < nsym; i += 64) dst[i] = outs[i];
    wave_sync();
    pf.mark(4);
  }
#ifdef CUSZ_AMD_DEC_PROFILE
  const unsigned gw = blockIdx.x * kDecWaves + wid;
  if (lane == 0 && gw < 4096)
    for (int k = 0; k < 16; k++) g_dec_prof[gw * 16 + k] = pf.v[k];
#endif
}

}  // namespace


int hf_encode_groups(int sublen, int pardeg)
{
  (void)sublen;
  return (pardeg + kEncW - 1) / kEncW;
}

static_assert(kGatherTile == 64, "hf_encode_tile_words");
size_t hf_encode_temp_words(int sublen, int pardeg)
{  // chunk slots at a worst-case stride, then the per-tile cell and bit totals
  return (size_t)enc_wave_cellcap(sublen) * (size_t)pardeg + hf_encode_tile_words(pardeg);
}
static size_t hf_encode_tile_offset(int sublen, int pardeg)
{
  return hf_encode_temp_words(sublen, pardeg) - hf_encode_tile_words(pardeg);
}

// sublen: a multiple of 256 (the pipeline rounds it), so every chunk is a whole number of
// 16-code lane rounds of its wave
int launch_hf_encode(const HfEncodeArgs& a, hipStream_t st)
{
  if (!a.temp || a.sublen % 64 != 0 || a.sublen > 8192) return (int)hipErrorInvalidValue;
  const int cellcap = enc_wave_cellcap(a.sublen);
  const size_t lds = (size_t)(((a.bklen + 3) & ~3) + kPackWaves * cellcap) * 4;
  int dev = 0, ncu = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_hf_pack, 64 * kPackWaves, lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int need = (a.pardeg + kPackWaves - 1) / kPackWaves;
  const int grid = need < per_cu * ncu ? need : per_cu * ncu;
  k_hf_pack<<<grid, 64 * kPackWaves, lds, st>>>(a, cellcap);
  const int ntiles = (a.pardeg + kGatherTile - 1) / kGatherTile;
  uint32_t* tile_sum = a.temp + hf_encode_tile_offset(a.sublen, a.pardeg);
  uint32_t* tile_bits = tile_sum + ntiles;
  uint32_t* const ticket = ntiles <= kFusedTiles ? a.ticket : nullptr;
  k_hf_tile_sums<<<(ntiles + 3) / 4, 256, 0, st>>>(a.par_nbit, a.pardeg, tile_sum, tile_bits, ntiles, ticket,
                                                   a.total_nbit);
  if (!ticket) k_hf_tile_scan<<<1, 1024, 0, st>>>(tile_sum, tile_bits, ntiles, a.total_nbit);
  k_hf_gather<<<ntiles, 256, 0, st>>>(a, cellcap, tile_sum);
  return (int)hipGetLastError();
}

int launch_hf_decode(const HfDecodeArgs& a, hipStream_t st)
{
  if (a.bklen < 1 || a.bklen > kMaxBklen || a.sublen < 1) return (int)hipErrorInvalidValue;
  k_hf_tables<<<1, 1024, 0, st>>>(a.revbook, a.bklen, a.lut);
  if (a.pardeg <= 0) return (int)hipGetLastError();
  // the current device's CU count (queried per launch: one process may drive several GPUs)
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  // Many chunks: one lane per chunk (every codeword decoded once).  Few long chunks: one wave
  // per chunk (three passes, but 64-way parallel inside a chunk).
  const bool lane = a.sublen % 16 == 0 && (a.decoder == 1 || (a.decoder == 0 && a.pardeg >= 64 * ncu));
  if (lane) {
    k_hf_decode_win<<<(a.pardeg + kWinLanes - 1) / kWinLanes, kWinLanes, 0, st>>>(a);
    return (int)hipGetLastError();
  }
  // per wave: staged cells + the chunk's output tile.  The staging area covers the average
  // chunk with margin; larger chunks read straight from global memory.
  const int worst = (a.sublen * kLmax / 32 + 4 + 3) / 4 * 4;
  int cellcap = worst;
  if (a.avg_cells > 0) {
    const size_t want = a.avg_cells + a.avg_cells / 2 + 64;
    cellcap = (int)((want + 15) / 16 * 16);
    if (cellcap > worst) cellcap = worst;
  }
  // the staging area never needs to cover a whole chunk (longer chunks decode from global
  // memory): clamp it to the LDS left after the output tiles
  const size_t tile_words = (((size_t)a.sublen + 1) / 2 + 3) / 4 * 4;
  const size_t budget = 120 * 1024 / 4 / kDecWaves;
  if (tile_words + 16 > budget) return (int)hipErrorInvalidValue;  // sublen > ~15k: never produced
  if ((size_t)cellcap + tile_words > budget) cellcap = (int)((budget - tile_words) / 16 * 16);
  const size_t lds = ((size_t)cellcap + tile_words) * 4 * kDecWaves;
  int per_cu = 0;  // occupancy for this LDS size on the current device (no process-global cache)
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_hf_decode, 64 * kDecWaves, lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int nblk = (a.pardeg + kDecWaves - 1) / kDecWaves;
  const int full = per_cu * ncu;
  const int grid = nblk < full ? nblk : full;
  k_hf_decode<<<grid, 64 * kDecWaves, lds, st>>>(a, cellcap);
  return (int)hipGetLastError();
}

#ifdef CUSZ_AMD_DEC_PROFILE
// copies the per-wave decoder profile of the last decode (u64[4096*16]) to host memory
extern "C" int psz_amd_debug_decode_profile(unsigned long long* host, int nwords)
{
  if (nwords > 4096 * 16) nwords = 4096 * 16;
  (void)hipDeviceSynchronize();
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dec_prof), (size_t)nwords * 8, 0, hipMemcpyDeviceToHost);
}
#endif

}  // namespace cusz_amd
