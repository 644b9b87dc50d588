// cusz_amd/csrc/brick.hip -- fused brick pipeline for gfx950: the Lorenzo predictor feeds the
// Huffman packer directly (compress) and the Huffman decoder feeds the Lorenzo reconstructor
// directly (decompress), so quant codes never touch HBM.
//
// Reference semantics (unchanged, bit-exact): predictor lrz_c.cuhip.inl:275-372 (3D 8^3 tiles),
// reconstruct lrz_x.cuhip.inl:271-360, histogram hist.cuhip.inl:55-89, chunked MSB-first
// Huffman cells hf_kernels.cuhip.inl:97-157, canonical decode hf_kernels.cuhip.inl:331-396.
//
// MI355X layout.  A wave owns a brick of W x 8 x 8 elements (W = 64 V: lane l holds x in
// [l V, l V + V)).  The Huffman chunk length is W, so every brick ROW (fixed y, z) is exactly one
// reference chunk: chunk c covers codes [c W, c W + W) of the linear (x-fastest) order.
//   pass 1 (k_brick3_scan):  predict -> per-brick histogram (u16, kept for the reservation),
//                            global histogram, outlier cells.  Reads the input once.
//   host:                    canonical codebook from the global histogram (exact reference heap).
//   reserve (k_brick_reserve + k_brick_offsets): a brick's bits = sum(hist_b[s] * len[s]); its
//                            region in the bitstream is that many bits plus one partial cell per
//                            row -- an upper bound, known BEFORE encoding, so every brick writes
//                            at a fixed offset: no look-back, no scratch, no gather.
//   pass 2 (k_brick3_pack):  predict again -> codewords -> pack each row (= chunk) into LDS
//                            cells -> store at region + running offset; par_nbit / par_entry.
//   decompress (k_brick3_decode): stage the brick's 64 chunks into LDS with one coalesced
//                            copy, decode one chunk per lane in x-blocks of 64 symbols into an
//                            LDS code tile, reconstruct the block (reference scan order), store.
// The archive is the reference phf format: par_entry[c] points at chunk c (the reference decoder
// reads chunk c from there, hf_kernels.cuhip.inl:386-391); chunks are laid out brick by brick,
// and the few cells between a brick's last chunk and the next region are zero.
#include "common.hh"
#include "hf_device.hh"
#include "kernels.hh"
#include "lrz_device.hh"

namespace cusz_amd {

using namespace lrzd;

namespace {

constexpr int kBrickWaves = 4;  // waves per workgroup in the encode passes
constexpr int kDecB = 11;       // decode table index bits
constexpr int kXB = 32;         // decode x-block (symbols per chunk per step = columns reconstructed)
constexpr int kPitch = 40;      // LDS code tile row pitch (u16): rows 4 apart are 16 banks apart
constexpr int kTileWords = 64 * kPitch / 2;
constexpr int kWorkShards = 8;
constexpr uint32_t kRingRows = 32;  // decoder input ring rows (power of two): 8 KB per wave
constexpr int kMaxRefill = 12;      // ring rows refilled per 32-symbol block (registers)  // decoder work counters, 64 B apart (kBrickWorkWords words)

__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// ---- 3D brick prediction ----------------------------------------------------------------
// One y-step of a brick: d[z][k] = Lorenzo residual at (x0 + k, y0 + y, z0 + z) in the
// reference's order (z-diff, x-diff inside 8-wide tiles, y-diff), lrz_c.cuhip.inl:341-352.
// the 8 z-rows of one y-step (issued one step ahead of their use: software prefetch)
template <typename T, int V>
__device__ __forceinline__ void load_ystep(const T* __restrict__ in, size_t plane, uint32_t lx, uint32_t ly,
                                           uint32_t lz, uint32_t x0, uint32_t gy, uint32_t z0, T (&raw)[8][V])
{
#pragma unroll
  for (int z = 0; z < 8; z++) {
    const bool ok = (z0 + z) < lz && gy < ly;
    load_row<T, V>(in, (size_t)(z0 + z) * plane + (size_t)gy * lx, x0, lx, ok, raw[z]);
  }
}

template <typename T, int V>
__device__ __forceinline__ void predict_ystep(const T (&raw)[8][V], uint32_t x0, int y, T ebx2_r, T (&bprev)[8][V],
                                              T (&p)[8][V])
{
#pragma unroll
  for (int z = 0; z < 8; z++)
#pragma unroll
    for (int k = 0; k < V; k++) p[z][k] = dround(raw[z][k] * ebx2_r);
#pragma unroll
  for (int z = 7; z > 0; z--)
#pragma unroll
    for (int k = 0; k < V; k++) p[z][k] = p[z][k] - p[z - 1][k];
#pragma unroll
  for (int z = 0; z < 8; z++) {
    const T west = shr_in_tile<T, 1, 8 / V>(p[z][V - 1]);
#pragma unroll
    for (int k = V - 1; k > 0; k--) p[z][k] = p[z][k] - p[z][k - 1];
    if (x0 % 8 != 0) p[z][0] = p[z][0] - west;
  }
#pragma unroll
  for (int z = 0; z < 8; z++)
#pragma unroll
    for (int k = 0; k < V; k++) {
      const T a = p[z][k];
      p[z][k] = (y > 0) ? a - bprev[z][k] : a;
      bprev[z][k] = a;
    }
}

// =========================================================================================
// pass 1: predict -> histograms + outliers
// =========================================================================================
template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(64 * kBrickWaves)
k_brick3_scan(const T* __restrict__ in, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2_r, T r, OutlierSink ol,
              uint32_t* __restrict__ g_hist, uint16_t* __restrict__ bhist, int bklen, uint32_t nbx, uint32_t nby,
              uint32_t nbricks)
{
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* s_wg = smem;                                // workgroup histogram (-> global, once)
  uint32_t* s_hist = smem + (1 + wid) * kMaxBklen;      // this wave's brick histogram
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_wg[i] = 0;
  for (int i = lane; i < bklen; i += 64) s_hist[i] = 0;
  __syncthreads();
  const size_t plane = (size_t)lx * ly;
  const uint32_t nw = gridDim.x * kBrickWaves;
  for (uint32_t brick = blockIdx.x * kBrickWaves + wid; brick < nbricks; brick += nw) {
    const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 8, z0 = bz * 8;
    uint32_t cnt = 0;
    T bprev[8][V], nxt[8][V];
    load_ystep<T, V>(in, plane, lx, ly, lz, x0, y0, z0, nxt);
    for (int y = 0; y < 8; y++) {
      const uint32_t gy = y0 + y;
      if (gy >= ly) break;
      T raw[8][V], d[8][V];
#pragma unroll
      for (int z = 0; z < 8; z++)
#pragma unroll
        for (int k = 0; k < V; k++) raw[z][k] = nxt[z][k];
      if (y < 7) load_ystep<T, V>(in, plane, lx, ly, lz, x0, gy + 1, z0, nxt);
      predict_ystep<T, V>(raw, x0, y, ebx2_r, bprev, d);
#pragma unroll
      for (int z = 0; z < 8; z++) {
        if (z0 + z >= lz) break;
        float olv[V];
        size_t idx[V];
        uint32_t mask = 0;
        const size_t base = (size_t)(z0 + z) * plane + (size_t)gy * lx;
#pragma unroll
        for (int k = 0; k < V; k++) {
          bool is_ol;
          const uint16_t q = quantize<T, ZZ>(d[z][k], r, is_ol, olv[k]);
          idx[k] = base + x0 + k;
          atomicAdd(&s_hist[q], 1u);
          mask |= (uint32_t)is_ol << k;
        }
        if (__ballot(mask != 0)) emit_outliers<V>(ol, brick, cnt, mask, olv, idx);
      }
    }
    if (lane == 0) ol.brick_cnt[brick] = cnt;
    hfd::wave_sync();
    uint16_t* bh = bhist + (size_t)brick * bklen;
    for (int i = lane; i < bklen; i += 64) {
      const uint32_t c = s_hist[i];
      bh[i] = (uint16_t)c;
      if (c) atomicAdd(&s_wg[i], c);
      s_hist[i] = 0;
    }
    hfd::wave_sync();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) {
    const uint32_t c = s_wg[i];
    if (c) atomicAdd(&g_hist[i], c);
  }
}

// =========================================================================================
// reservation: per-brick bit count and region size, then the exclusive scan
// =========================================================================================
__device__ __forceinline__ uint32_t brick_rows3(uint32_t brick, uint32_t nbx, uint32_t nby, uint32_t ly, uint32_t lz)
{
  const uint32_t t = brick / nbx, by = t % nby, bz = t / nby;
  return min(8u, ly - by * 8) * min(8u, lz - bz * 8);
}

__global__ void __launch_bounds__(256)
k_brick_reserve(const uint16_t* __restrict__ bhist, int bklen, const uint32_t* __restrict__ book, uint32_t nbricks,
                uint32_t nbx, uint32_t nby, uint32_t ly, uint32_t lz, uint32_t* __restrict__ ub,
                unsigned long long* total_nbit)
{
  __shared__ uint32_t s_len[kMaxBklen];
  __shared__ unsigned long long s_bits[4];
  for (int i = threadIdx.x; i < bklen; i += 256) s_len[i] = book[i] >> 27;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t brick = blockIdx.x * 4 + wid;
  uint32_t bits = 0;
  if (brick < nbricks) {
    const uint16_t* h = bhist + (size_t)brick * bklen;
    for (int i = lane; i < bklen; i += 64) bits += (uint32_t)h[i] * s_len[i];
    bits = hfd::wave_sum(bits);
    if (lane == 0) ub[brick] = (bits + 31u * brick_rows3(brick, nbx, nby, ly, lz)) >> 5;
  }
  if (lane == 0) s_bits[wid] = bits;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(total_nbit, s_bits[0] + s_bits[1] + s_bits[2] + s_bits[3]);
}

// exclusive scan of ub[0..n) into base[0..n]; base[n] = total cells (one workgroup)
__global__ void __launch_bounds__(1024) k_brick_offsets(const uint32_t* __restrict__ ub, uint32_t n,
                                                        uint32_t* __restrict__ base, CompressInfo* info)
{
  __shared__ uint32_t s_scan[16];
  __shared__ uint32_t s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  constexpr int PER = 8;
  for (uint32_t b0 = 0; b0 < n; b0 += 1024 * PER) {
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t b = b0 + tid * PER + k;
      v[k] = b < n ? ub[b] : 0u;
      sum += v[k];
    }
    const uint32_t inc = hfd::wave_incl_scan(sum);
    if (lane == 63) s_scan[wid] = inc;
    __syncthreads();
    uint32_t off = s_carry;
    for (int w = 0; w < wid; w++) off += s_scan[w];
    uint32_t run = off + inc - sum;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const uint32_t b = b0 + tid * PER + k;
      if (b < n) base[b] = run;
      run += v[k];
    }
    __syncthreads();
    if (tid == 1023) s_carry = off + inc;
    __syncthreads();
  }
  if (tid == 0) {
    base[n] = s_carry;
    info->total_ncell = s_carry;
  }
}

// =========================================================================================
// pass 2: predict -> codewords -> one chunk per brick row, written at the brick's region
// =========================================================================================
template <int V>
constexpr int pack_cells_words()
{  // worst case cells of one row (27-bit codes) + slack, multiple of 4
  return ((64 * V * kLmax + 31) / 32 + 4 + 3) / 4 * 4;
}

template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(64 * kBrickWaves)
k_brick3_pack(const T* __restrict__ in, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2_r, T r,
              const uint32_t* __restrict__ book, int bklen, const uint32_t* __restrict__ bbase,
              uint32_t* __restrict__ par_nbit, uint32_t* __restrict__ par_entry, uint32_t* __restrict__ bitstream,
              uint32_t nbx, uint32_t nby, uint32_t nbricks, int reverse, unsigned int* overflow)
{
  constexpr int CW = pack_cells_words<V>();
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_book = smem;  // kMaxBklen words
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* cells = smem + kMaxBklen + wid * CW;
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_book[i] = book[i];
  for (int i = lane; i < CW; i += 64) cells[i] = 0;
  __syncthreads();
  const size_t plane = (size_t)lx * ly;
  const uint32_t nw = gridDim.x * kBrickWaves;
  for (uint32_t it = blockIdx.x * kBrickWaves + wid; it < nbricks; it += nw) {
    const uint32_t brick = reverse ? nbricks - 1 - it : it;
    const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 8, z0 = bz * 8;
    const uint32_t base = bbase[brick], lim = bbase[brick + 1] - base;
    uint32_t* dst = bitstream + base;
    uint32_t off = 0, my_nbit = 0, my_entry = 0;
    T bprev[8][V], nxt[8][V];
    load_ystep<T, V>(in, plane, lx, ly, lz, x0, y0, z0, nxt);
    for (int y = 0; y < 8; y++) {
      const uint32_t gy = y0 + y;
      if (gy >= ly) break;
      T raw[8][V], d[8][V];
#pragma unroll
      for (int z = 0; z < 8; z++)
#pragma unroll
        for (int k = 0; k < V; k++) raw[z][k] = nxt[z][k];
      if (y < 7) load_ystep<T, V>(in, plane, lx, ly, lz, x0, gy + 1, z0, nxt);
      predict_ystep<T, V>(raw, x0, y, ebx2_r, bprev, d);
#pragma unroll
      for (int z = 0; z < 8; z++) {
        if (z0 + z >= lz) break;
        uint32_t w[V], bits = 0;
#pragma unroll
        for (int k = 0; k < V; k++) {
          bool is_ol;
          float olv;
          const uint16_t q = quantize<T, ZZ>(d[z][k], r, is_ol, olv);
          w[k] = s_book[q];
          bits += w[k] >> 27;
        }
        const uint32_t inc = hfd::wave_incl_scan(bits);
        const uint32_t tot = readlane(inc, 63);
        hfd::pack_words<V>(cells, inc - bits, w, V);
        hfd::wave_sync();
        const uint32_t nc = (tot + 31) >> 5;
        for (uint32_t i = lane; i < nc; i += 64) {
          if (off + i < lim) dst[off + i] = cells[i];
          cells[i] = 0;
        }
        if (lane == y * 8 + z) my_nbit = tot, my_entry = base + off;
        off += nc;
        hfd::wave_sync();
      }
    }
    if (off > lim && lane == 0) atomicOr(overflow, 1u);  // cannot happen (region is an upper bound)
    for (uint32_t i = off + lane; i < lim; i += 64) dst[i] = 0u;
    const uint32_t ry = lane >> 3, rz = lane & 7;
    if (y0 + ry < ly && z0 + rz < lz) {
      const size_t c = ((size_t)(z0 + rz) * ly + (y0 + ry)) * nbx + bx;
      par_nbit[c] = my_nbit;
      par_entry[c] = my_entry;
    }
  }
}

// =========================================================================================
// decompress: chunk decode + reconstruct, one wave per brick
// =========================================================================================
// Input staging.  Lane l decodes chunk l (brick row (y, z) = (l / 8, l % 8)).  The words of all
// 64 chunks are staged in an LDS ring laid out [word k][lane]: row k holds word k of every chunk,
// filled by one LDS-DMA instruction with per-lane source addresses (lane-linear destination),
// so a lane's reads ring[(k % R) * 64 + lane] never conflict.  Rows are issued a block ahead and
// land while the current block decodes; a lane that outruns the resident rows reads HBM.
struct BitReader {
  uint64_t buf;    // next bits of the chunk, left-justified
  uint32_t avail;  // valid bits in buf (>= 32 between steps)
  uint32_t nw;     // index of the next chunk word to append
};

// LDS pointer type: keeps ring reads ds_read_* (a generic pointer that may alias global memory
// would become a flat load, which waits on every outstanding DMA and store)
using lds_u32 = __attribute__((address_space(3))) const uint32_t;

struct Ring {
  lds_u32* ring;         // this wave's kRingRows x 64 words, row k % kRingRows holds chunk word k
  uint32_t valid_top;    // rows [.., valid_top) have landed
  const uint32_t* gsrc;  // this lane's chunk in HBM (fallback past the resident rows)
  uint32_t nc;           // words in this lane's chunk
};

// A chunk word the ring does not hold yet, read from HBM.  The load and its wait are inline asm
// so the compiler's wait insertion does not place a vmcnt(0) -- which would also wait for every
// in-flight ring DMA and output store -- at the join after this rare branch on the common path.
__device__ __forceinline__ uint32_t fallback_word(const Ring& rs, uint32_t k)
{
  if (k >= rs.nc) return 0u;
  uint32_t v;
  asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(rs.gsrc + k) : "memory");
  return v;
}

// decode kXB symbols of this lane's chunk into its tile row (plus a carried symbol when a
// two-symbol step crossed the previous block's end; the row has slack for the overrun).
// Branch-free step: the L1/L2 entries and the next input word are read together; a finished
// lane keeps stepping with a zero length (no state change) until the whole wave is done.
__device__ __forceinline__ void decode_block(const hfd::LdsTables<kDecB>& tb, const hfd::DecRegs& rg, uint32_t bklen,
                                             bool live, BitReader& br, int& carry, uint16_t* row, const Ring& rs,
                                             int lane)
{
  uint32_t cnt = 0;
  if (carry >= 0) row[0] = (uint16_t)carry, cnt = 1;
  carry = -1;
  if (!live) cnt = kXB + 1;
  while (__builtin_amdgcn_ballot_w64(cnt < kXB)) {
#pragma unroll
    for (int st = 0; st < 4; st++) {
      const uint32_t win = (uint32_t)(br.buf >> 32);
      uint32_t nxt = rs.ring[(br.nw & (kRingRows - 1)) * 64 + lane];
      if (__builtin_expect(br.nw >= rs.valid_top, 0)) nxt = fallback_word(rs, br.nw);
      const uint32_t e = hfd::lookup<kDecB>(tb, rg, win, bklen);
      const bool act = cnt < kXB;
      const uint32_t c = min(cnt, (uint32_t)kXB + 1);
      row[c] = (uint16_t)(e & 1023u);
      row[c + 1] = (uint16_t)((e >> 10) & 1023u);  // overwritten next step unless two symbols
      const uint32_t l = act ? ((e >> 25) & 31u) : 0u;  // bits consumed (1 or 2 codes)
      cnt += act ? (e >> 30) : 0u;
      br.buf <<= l;
      br.avail -= l;
      const bool rf = br.avail < 32;
      br.buf |= rf ? ((uint64_t)nxt << (32 - br.avail)) : 0ull;
      br.avail += rf ? 32u : 0u;
      br.nw += rf ? 1u : 0u;
    }
  }
  if (cnt == kXB + 1 && live) carry = row[kXB];
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d));
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
  return v;
}

constexpr int kDecMaxWaves = 12;  // 3 waves per SIMD: up to 168 VGPRs without spills

template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(64 * kDecMaxWaves)
k_brick3_decode(const uint32_t* __restrict__ bitstream, const uint8_t* __restrict__ revbook, int bklen,
                const uint32_t* __restrict__ par_nbit, const uint32_t* __restrict__ par_entry, T* out, uint32_t lx,
                uint32_t ly, uint32_t lz, T ebx2, T r, uint32_t nbx, uint32_t nby, uint32_t nbricks,
                uint32_t ahead, unsigned int* work, int dbg)
{
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  auto& tb = *reinterpret_cast<hfd::LdsTables<kDecB>*>(dsm);
  constexpr size_t kTabBytes = (sizeof(hfd::LdsTables<kDecB>) + 15) / 16 * 16;
  hfd::build_tables<kDecB>(tb, revbook, bklen);
  const hfd::DecRegs rg = hfd::load_dec_regs(tb);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr uint32_t R = kRingRows;
  uint32_t* ring = reinterpret_cast<uint32_t*>(dsm + kTabBytes) + (size_t)wid * (R * 64 + kTileWords);
  uint16_t* tile = reinterpret_cast<uint16_t*>(ring + R * 64);
  uint16_t* myrow = tile + lane * kPitch;
  const size_t plane = (size_t)lx * ly;
  const uint32_t ubk = (uint32_t)bklen;
  constexpr uint32_t W = 64 * V;
  // reconstruct layout: lane = (z half, column) of a 32-column block
  const uint32_t col = lane & 31, zh = lane >> 5;

  // bricks are handed out by kWorkShards counters (one word saturates near ~90 dequeues/us);
  // shard q owns bricks [q per, (q + 1) per); a wave drains its home shard, then the others
  const uint32_t per = (nbricks + kWorkShards - 1) / kWorkShards;
  const uint32_t q0 = blockIdx.x % kWorkShards;
  for (uint32_t qi = 0; qi < (uint32_t)kWorkShards;) {
    const uint32_t q = (q0 + qi) % kWorkShards;
    uint32_t got = 0;
    if (lane == 0) got = atomicAdd(work + q * 16, 1u);
    got = readlane(got, 0);
    const uint32_t brick = q * per + got;
    if (got >= per || brick >= nbricks) {
      qi++;
      continue;
    }
    const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
    const uint32_t y0 = by * 8, z0 = bz * 8;
    const uint32_t ry = lane >> 3, rz = lane & 7;  // this lane's chunk = brick row (ry, rz)
    const bool live = y0 + ry < ly && z0 + rz < lz;
    const size_t c = ((size_t)(z0 + rz) * ly + (y0 + ry)) * nbx + bx;
    const uint32_t nbit = live ? par_nbit[c] : 0u;
    const uint32_t ent = live ? par_entry[c] : 0u;
    const uint32_t nc = (nbit + 31) >> 5;
    const uint32_t* gsrc = bitstream + ent;
    const uint32_t top_all = wave_max(nc) + 3;  // no row is needed past every chunk's end
    // issue rows [from, to) of the ring (LDS-DMA, lane-linear destination, per-lane source)
    auto issue = [&](uint32_t from, uint32_t to) {
      for (uint32_t k = from; k < to; k++) {
        const uint32_t* g = gsrc + (k < nc ? k : 0u);
        __builtin_amdgcn_global_load_lds(g, ring + (k & (R - 1)) * 64, 4, 0, 0);
      }
    };
    uint32_t issued = min(R, min(top_all, 2 * ahead + 3));
    issue(0, issued);
    // compiler-visible vmcnt(0) (an asm wait would leave the waitcnt pass assuming the DMA is
    // still in flight and make it wait inside the decode loop)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    Ring rs{(lds_u32*)ring, issued, gsrc, nc};
    BitReader br;
    br.buf = ((uint64_t)ring[lane] << 32) | ring[64 + lane];
    br.avail = 64, br.nw = 2;
    int carry = -1;
    // later rows: loaded into registers one block ahead, written to the ring the block after
    uint32_t pend[kMaxRefill];
    uint32_t pend_from = issued, pend_cnt = 0;

    for (int xb = 0; xb < (int)(W / kXB); xb++) {
      if (xb > 0) {
#pragma unroll
        for (int j = 0; j < kMaxRefill; j++)
          if (j < (int)pend_cnt) ring[((pend_from + j) & (R - 1)) * 64 + lane] = pend[j];
        rs.valid_top = pend_from + pend_cnt;
        const uint32_t lo = wave_min(live ? br.nw : 0xFFFFFFFFu);
        const uint32_t hi = wave_max(live ? br.nw : 0u);
        const uint32_t want = min(issued + kMaxRefill, min(top_all, min(lo + R - 1, hi + ahead)));
        pend_from = issued;
        pend_cnt = want > issued ? want - issued : 0u;
#pragma unroll
        for (int j = 0; j < kMaxRefill; j++)
          if (j < (int)pend_cnt) {
            const uint32_t k = issued + j;
            pend[j] = gsrc[k < nc ? k : 0u];
          }
        issued += pend_cnt;
      }
      if (!(dbg & 1)) decode_block(tb, rg, ubk, live, br, carry, myrow, rs, lane);
      hfd::wave_sync();
      if (dbg & 2) continue;  // diagnostic: no reconstruction
      // reconstruct 32 columns (lrz_x.cuhip.inl:311-353 order): lane = (z half zh, column);
      // z in [4 zh, 4 zh + 4) in registers, the z scan crosses halves with lane shuffles
      const uint32_t xg = bx * W + xb * kXB + col;
      uint16_t code[8][4];
      T ov[8][4];
#pragma unroll
      for (int y = 0; y < 8; y++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t z = 4 * zh + k;
          const bool ok = z0 + z < lz && y0 + y < ly;
          code[y][k] = ok ? tile[(y * 8 + z) * kPitch + col] : uint16_t(1);
          ov[y][k] = 0;
        }
#pragma unroll
      for (int y = 0; y < 8; y++)
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (code[y][k] == 0) ov[y][k] = out[(size_t)(z0 + 4 * zh + k) * plane + (size_t)(y0 + y) * lx + xg];
      T s[4];
#pragma unroll
      for (int y = 0; y < 8; y++) {
        const uint32_t gy = y0 + y;
        if (gy >= ly) break;
        T tz[4][1];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const bool ok = z0 + 4 * zh + k < lz;
          T v;
          if constexpr (ZZ)
            v = ok ? ov[y][k] + (T)zz_dec(code[y][k]) : T(0);
          else
            v = ok ? (ov[y][k] + (T)code[y][k]) - r : T(0);
          s[k] = (y > 0) ? v + s[k] : v;
          tz[k][0] = s[k];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
          hs_step<T, 1, 8, 1>(tz[k], xg);
          hs_step<T, 1, 8, 2>(tz[k], xg);
          hs_step<T, 1, 8, 4>(tz[k], xg);
        }
        // z Hillis-Steele, d = 1, 2, 4 (descending z keeps each round's sources unmodified);
        // the upper half reads the lower half's pre-round values
        {
          const T l3 = __shfl(tz[3][0], (int)col);  // lower half's t[3] (lane col)
          tz[3][0] = tz[3][0] + tz[2][0];
          tz[2][0] = tz[2][0] + tz[1][0];
          tz[1][0] = tz[1][0] + tz[0][0];
          if (zh) tz[0][0] = tz[0][0] + l3;
        }
        {
          const T l2 = __shfl(tz[2][0], (int)col), l3 = __shfl(tz[3][0], (int)col);
          tz[3][0] = tz[3][0] + tz[1][0];
          tz[2][0] = tz[2][0] + tz[0][0];
          if (zh) tz[1][0] = tz[1][0] + l3, tz[0][0] = tz[0][0] + l2;
        }
        {
          T lo4[4];
#pragma unroll
          for (int k = 0; k < 4; k++) lo4[k] = __shfl(tz[k][0], (int)col);
          if (zh)
#pragma unroll
            for (int k = 0; k < 4; k++) tz[k][0] = tz[k][0] + lo4[k];
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (z0 + 4 * zh + k < lz) out[(size_t)(z0 + 4 * zh + k) * plane + (size_t)gy * lx + xg] = tz[k][0] * ebx2;
      }
      hfd::wave_sync();
    }
  }
}

}  // namespace

// =========================================================================================
// host launchers
// =========================================================================================

BrickGeom brick_geom(int ndim, size_t lx, size_t ly, size_t lz, int elem_bytes)
{
  BrickGeom g{};
  g.V = 4;  // W = 256: f32 16-B loads, f64 32-B loads per lane
  g.W = 64 * g.V;
  g.ok = ndim == 3 && lx % (size_t)g.W == 0 && lx * ly * lz < (1ull << 32) && (elem_bytes == 4 || elem_bytes == 8);
  if (!g.ok) return g;
  g.nbx = (uint32_t)(lx / g.W);
  g.nby = (uint32_t)((ly + 7) / 8);
  g.nbz = (uint32_t)((lz + 7) / 8);
  g.nbricks = g.nbx * g.nby * g.nbz;
  g.brick_elems = (uint32_t)g.W * 64;
  g.nchunks = (uint32_t)(lx / g.W * ly * lz);
  return g;
}

size_t brick_decode_lds(int waves)
{
  const size_t tab = (sizeof(hfd::LdsTables<kDecB>) + 15) / 16 * 16;
  return tab + (size_t)waves * ((size_t)kRingRows * 64 + kTileWords) * 4;
}

uint32_t brick_decode_max_ahead() { return kRingRows - 6; }

int brick_configure(BrickLaunch& L, int elem_bytes, int device)
{
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
  L.ncu = ncu;
  int per_scan = 0, per_pack = 0;
  const size_t lds_scan = (size_t)(1 + kBrickWaves) * kMaxBklen * 4;
  const size_t lds_pack = ((size_t)kMaxBklen + (size_t)kBrickWaves * pack_cells_words<4>()) * 4;
  hipError_t e1, e2;
  if (elem_bytes == 8) {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_scan, k_brick3_scan<double, 4, false>, 64 * kBrickWaves, lds_scan);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pack, k_brick3_pack<double, 4, false>, 64 * kBrickWaves, lds_pack);
  }
  else {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_scan, k_brick3_scan<float, 4, false>, 64 * kBrickWaves, lds_scan);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pack, k_brick3_pack<float, 4, false>, 64 * kBrickWaves, lds_pack);
  }
  if (e1 != hipSuccess || per_scan < 1) per_scan = 1;
  if (e2 != hipSuccess || per_pack < 1) per_pack = 1;
  const int need = (int)((L.g.nbricks + kBrickWaves - 1) / kBrickWaves);
  L.grid_scan = need < per_scan * ncu ? need : per_scan * ncu;
  L.grid_pack = need < per_pack * ncu ? need : per_pack * ncu;
  if (L.grid_scan < 1) L.grid_scan = 1;
  if (L.grid_pack < 1) L.grid_pack = 1;
  return (int)hipSuccess;
}

template <typename T>
int launch_brick_scan(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const OutlierSink& ol,
                      uint32_t* hist, uint16_t* bhist, int bklen, hipStream_t st)
{
  const T ebx2_r = (T)(1.0 / (eb * 2));  // lrz_c.cuhip.inl:489
  const T r = (T)radius;
  const BrickGeom& g = L.g;
  const size_t lds = (size_t)(1 + kBrickWaves) * kMaxBklen * 4;
  const int grid = L.grid_scan;
  if (zz)
    k_brick3_scan<T, 4, true><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, ol, hist, bhist,
                                                                   bklen, g.nbx, g.nby, g.nbricks);
  else
    k_brick3_scan<T, 4, false><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, ol, hist, bhist,
                                                                    bklen, g.nbx, g.nby, g.nbricks);
  return (int)hipGetLastError();
}

int launch_brick_reserve(const BrickLaunch& L, const uint16_t* bhist, int bklen, const uint32_t* book, uint32_t* ub,
                         uint32_t* bbase, CompressInfo* info, hipStream_t st)
{
  const BrickGeom& g = L.g;
  k_brick_reserve<<<(g.nbricks + 3) / 4, 256, 0, st>>>(bhist, bklen, book, g.nbricks, g.nbx, g.nby, L.ly, L.lz, ub,
                                                       &info->total_nbit);
  k_brick_offsets<<<1, 1024, 0, st>>>(ub, g.nbricks, bbase, info);
  return (int)hipGetLastError();
}

template <typename T>
int launch_brick_pack(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const uint32_t* book,
                      int bklen, const uint32_t* bbase, uint32_t* par_nbit, uint32_t* par_entry, uint32_t* bitstream,
                      int reverse, unsigned int* overflow, hipStream_t st)
{
  const T ebx2_r = (T)(1.0 / (eb * 2));
  const T r = (T)radius;
  const BrickGeom& g = L.g;
  const size_t lds = ((size_t)kMaxBklen + (size_t)kBrickWaves * pack_cells_words<4>()) * 4;
  const int grid = L.grid_pack;
  if (zz)
    k_brick3_pack<T, 4, true><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, book, bklen, bbase,
                                                                   par_nbit, par_entry, bitstream, g.nbx, g.nby,
                                                                   g.nbricks, reverse, overflow);
  else
    k_brick3_pack<T, 4, false><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, book, bklen,
                                                                    bbase, par_nbit, par_entry, bitstream, g.nbx,
                                                                    g.nby, g.nbricks, reverse, overflow);
  return (int)hipGetLastError();
}

template <typename T>
int launch_brick_decode(const BrickLaunch& L, const uint32_t* bitstream, const uint8_t* revbook, int bklen,
                        const uint32_t* par_nbit, const uint32_t* par_entry, T* out, double eb, int radius, bool zz,
                        uint32_t ahead, int waves, unsigned int* work, hipStream_t st)
{
  const T ebx2 = (T)(eb * 2);  // lrz_x.cuhip.inl:432
  const T r = (T)radius;
  const BrickGeom& g = L.g;
  const size_t lds = brick_decode_lds(waves);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  const int grid = L.ncu;
  // diagnostic switch (profiling only): 1 = skip the decode loop, 2 = skip the reconstruction
  const char* dbs = getenv("CUSZ_AMD_DEC_DEBUG");
  const int dbg = dbs ? atoi(dbs) : 0;
  if (zz)
    k_brick3_decode<T, 4, true><<<grid, 64 * waves, lds, st>>>(bitstream, revbook, bklen, par_nbit, par_entry, out,
                                                                L.lx, L.ly, L.lz, ebx2, r, g.nbx, g.nby, g.nbricks,
                                                                ahead, work, dbg);
  else
    k_brick3_decode<T, 4, false><<<grid, 64 * waves, lds, st>>>(bitstream, revbook, bklen, par_nbit, par_entry, out,
                                                                 L.lx, L.ly, L.lz, ebx2, r, g.nbx, g.nby, g.nbricks,
                                                                 ahead, work, dbg);
  return (int)hipGetLastError();
}

#define INST(T)                                                                                                   \
  template int launch_brick_scan<T>(const BrickLaunch&, const T*, double, int, bool, const OutlierSink&, uint32_t*, \
                                    uint16_t*, int, hipStream_t);                                                  \
  template int launch_brick_pack<T>(const BrickLaunch&, const T*, double, int, bool, const uint32_t*, int,          \
                                    const uint32_t*, uint32_t*, uint32_t*, uint32_t*, int, unsigned int*,           \
                                    hipStream_t);                                                                  \
  template int launch_brick_decode<T>(const BrickLaunch&, const uint32_t*, const uint8_t*, int, const uint32_t*,    \
                                      const uint32_t*, T*, double, int, bool, uint32_t, int, unsigned int*,        \
                                      hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace cusz_amd
