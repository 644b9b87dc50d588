// cusz_amd/csrc/brick.hip -- fused brick pipeline for gfx950: the Lorenzo predictor feeds the
// Huffman packer (compress) and the Huffman decoder feeds the Lorenzo reconstructor directly
// (decompress).
//
// Reference semantics (unchanged, bit-exact): predictor lrz_c.cuhip.inl:275-372 (3D 8^3 tiles),
// reconstruct lrz_x.cuhip.inl:271-360, histogram hist.cuhip.inl:55-89, chunked MSB-first
// Huffman cells hf_kernels.cuhip.inl:97-157, canonical decode hf_kernels.cuhip.inl:331-396.
//
// MI355X layout.  A wave owns a brick of W x 8 x 8 elements (W = 64 V: lane l holds x in
// [l V, l V + V)).  The Huffman chunk length is W, so every brick ROW (fixed y, z) is exactly one
// reference chunk: chunk c covers codes [c W, c W + W) of the linear (x-fastest) order.
//   pass 1 (k_brick3_scan):  predict -> codes in brick order (byte rows; u16 rows when a code
//                            leaves the byte window, one mask bit per row), per-unit histogram
//                            (u16, kept for the plan), global histogram, outlier slots.  Reads
//                            the input once.
//   host:                    canonical codebook from the global histogram (exact reference heap).
//   plan (k_brick_plan):     a unit's bits = sum(hist_u[s] * len[s]); its region in the bitstream
//                            is that many bits plus one partial cell per row -- an upper bound,
//                            known BEFORE encoding, so every unit writes at a fixed offset: no
//                            look-back, no scratch, no gather.  The last block writes the headers.
//   pass 2 (k_brick3_pack):  codes (read back, not re-predicted) -> codewords -> pack each row
//                            (= chunk) into LDS cells -> store at region + running offset;
//                            par_nbit / par_entry; the unit's outlier slot is copied out.
//   decompress (k_brick3_decode): one wave per brick, one chunk per lane decoded in x-blocks of
//                            32 symbols (f32; 64 for f64) into an LDS code tile; the block is
//                            reconstructed (reference scan order) and stored as whole rows.
// Single-pass mode (k_brick3_sample, k_brick3_stream, k_brick3_stream_finish): the book comes
// from a 1/16 sample of 32 x 8 x 8 units before the field is predicted, and one pass -- a
// workgroup per brick, a wave per y-step -- predicts, sizes (look-back over the bricks) and packs
// each brick; see the section before the launchers.
// The archive is the reference phf format: par_entry[c] points at chunk c (the reference decoder
// reads chunk c from there, hf_kernels.cuhip.inl:386-391); chunks are laid out brick by brick,
// and the few cells between a brick's last chunk and the next region are zero.
#include <algorithm>
#include <type_traits>

#include "archive_device.hh"
#include "common.hh"
#include "hf_device.hh"
#include "kernels.hh"
#include "lrz_device.hh"
#include "pub_device.hh"

namespace cusz_amd {

using namespace lrzd;

namespace {

constexpr int kBrickWaves = 4;  // waves per workgroup in the encode passes
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// A unit = kUnitBricks consecutive bricks, processed by one wave in both encode passes: one
// histogram record (u16 counts: a unit has at most 32768 elements), one outlier slot and one
// reserved bitstream region per unit.
constexpr int kUnitBricks = 1;
#ifndef CUSZ_AMD_HIST_COPIES
#define CUSZ_AMD_HIST_COPIES 1
#endif
constexpr int kHistCopies = CUSZ_AMD_HIST_COPIES;  // lane-interleaved copies of a wave's brick histogram
// per-brick u16 histograms are stored at a stride of whole 16-B groups (the plan kernel's loads)
__host__ __device__ constexpr int bhist_stride(int bklen) { return (bklen + 7) & ~7; }

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

// Prequant of one y-step: p = round(x * ebx2_r) (lrz_c.cuhip.inl:305-309).
template <typename T, int V>
__device__ __forceinline__ void prequant_ystep(const T (&raw)[8][V], T ebx2_r, T (&p)[8][V])
{
#pragma unroll
  for (int z = 0; z < 8; z++)
#pragma unroll
    for (int k = 0; k < V; k++) p[z][k] = dround(raw[z][k] * ebx2_r);
}

// Residuals of one y-step in place: z-diff, x-diff inside 8-wide tiles (DPP row_shr), y-diff
// against the previous y-step's z/x residuals (lrz_c.cuhip.inl:341-352 order).
template <typename T, int V>
__device__ __forceinline__ void residual_ystep(uint32_t x0, int y, T (&bprev)[8][V], T (&p)[8][V])
{
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

// The encode passes walk a stream of y-steps: (brick it, y = 0..7), it += waves in the grid.
// The rows of step s + NB are loaded while step s is computed, across brick boundaries, into the
// buffer step s has just consumed (NB divides 8, so the fully unrolled y loop needs no copies).
// NB = 2 for f32 (16 KiB in flight per wave at 2 waves/SIMD); f64 rows are twice as wide: 1.
template <typename T>
constexpr int kStepBuffers = sizeof(T) == 4 ? 2 : 1;
#ifndef CUSZ_AMD_SCAN_LOAD_AUX
#define CUSZ_AMD_SCAN_LOAD_AUX 2  // cache-policy bits of pass 1's field loads: 2 = nontemporal
// (config 2 pass 1 189 -> 163 us: the streamed field no longer evicts the code rows pass 2 reads)
#endif
template <typename T, int V>
struct StepLoader {
  const T* in;
  size_t plane;
  uint32_t lx, ly, lz, nbx, nby, nbricks;
  int reverse;
  uint32_t lane;
  __device__ __forceinline__ uint32_t brick_of(uint32_t it) const { return reverse ? nbricks - 1 - it : it; }
  // Rows (y, z = 0..7) of brick `it` by raw buffer loads from the brick's origin: one 16-B (f64:
  // two) load per lane and row, rows outside the field get an offset past the range and read 0.
  // Straight-line code: no per-row branches, so the waitcnt pass can count the loads exactly.
  // row `row` = 8 y + z of brick `it` (rows outside the field read 0)
  __device__ __forceinline__ void issue_row(uint32_t it, int row, T (&dst)[V]) const
  {
    // past the last brick the load still issues (at brick 0's origin, past the range: reads 0,
    // touches no memory): every path issues the same loads, so the compiler counts the waits
    // (vmcnt(7) for the row loaded 8 rows ago, not vmcnt(0): compress -3 us, 1-D -9 us)
    const bool live = it < nbricks;
    const uint32_t b = live ? brick_of(it) : 0u, bx = b % nbx, t = b / nbx, by = t % nby, bz = t / nby;
    const T* origin = in + (size_t)bz * 8 * plane + (size_t)by * 8 * lx + (size_t)bx * (64 * V);
    const uint32_t span = (uint32_t)(8 * plane * sizeof(T));  // < 2^31 (brick_geom)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(origin), 0, (int)span, 0x00020000);
    const uint32_t y = (uint32_t)row >> 3, z = (uint32_t)row & 7u;
    const bool ok = live && by * 8 + y < ly && bz * 8 + z < lz;
    const uint32_t off =
        ok ? (uint32_t)(((size_t)z * plane + (size_t)y * lx) * sizeof(T)) + lane * (V * sizeof(T)) : span;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < (int)(V * sizeof(T) / 16); h++) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16 * h), 0, CUSZ_AMD_SCAN_LOAD_AUX);
      __builtin_memcpy(reinterpret_cast<char*>(&dst[0]) + 16 * h, &v, 16);
    }
  }
  // The same loads with the brick's address work done once per brick (BrickRows): per row only
  // the in-brick offset and two compares, instead of the brick coordinates, the 64-bit origin and
  // the descriptor again for every row (pass 1: ~50 scalar instructions and the SGPR spills they
  // cause, per row).
  struct BrickRows {
    __amdgpu_buffer_rsrc_t rs;  // at the brick's origin, 8 planes long
    uint32_t nyv, nzv;          // rows y < nyv, z < nzv lie in the field (0: past the last brick)
  };
  __device__ __forceinline__ BrickRows rows_of(uint32_t it) const
  {
    const bool live = it < nbricks;
    const uint32_t b = live ? brick_of(it) : 0u, bx = b % nbx, t = b / nbx, by = t % nby, bz = t / nby;
    const T* origin = in + (size_t)bz * 8 * plane + (size_t)by * 8 * lx + (size_t)bx * (64 * V);
    const uint32_t span = (uint32_t)(8 * plane * sizeof(T));  // < 2^31 (brick_geom)
    return {__builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(origin), 0, (int)span, 0x00020000),
            live ? min(8u, ly - by * 8) : 0u, live ? min(8u, lz - bz * 8) : 0u};
  }
  __device__ __forceinline__ void issue_row(const BrickRows& br, uint32_t y, uint32_t z, T (&dst)[V]) const
  {
    const uint32_t span = (uint32_t)(8 * plane * sizeof(T));
    const bool ok = y < br.nyv && z < br.nzv;
    const uint32_t off = ok ? (z * (uint32_t)plane + y * lx) * (uint32_t)sizeof(T) + lane * (V * sizeof(T)) : span;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < (int)(V * sizeof(T) / 16); h++) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(br.rs, (int)(off + 16 * h), 0, CUSZ_AMD_SCAN_LOAD_AUX);
      __builtin_memcpy(reinterpret_cast<char*>(&dst[0]) + 16 * h, &v, 16);
    }
  }
  __device__ __forceinline__ void issue(uint32_t it, int y, T (&dst)[8][V]) const
  {
    if (it >= nbricks) return;
    const uint32_t b = brick_of(it), bx = b % nbx, t = b / nbx, by = t % nby, bz = t / nby;
    const T* origin = in + (size_t)bz * 8 * plane + (size_t)by * 8 * lx + (size_t)bx * (64 * V);
    const uint32_t span = (uint32_t)(8 * plane * sizeof(T));  // < 2^31 (brick_geom)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(origin), 0, (int)span, 0x00020000);
    const bool yok = by * 8 + (uint32_t)y < ly;
    const uint32_t nzv = min(8u, lz - bz * 8);
#pragma unroll
    for (int z = 0; z < 8; z++) {
      const uint32_t off = (yok && (uint32_t)z < nzv)
                               ? (uint32_t)(((size_t)z * plane + (size_t)y * lx) * sizeof(T)) + lane * (V * sizeof(T))
                               : span;
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int h = 0; h < (int)(V * sizeof(T) / 16); h++) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16 * h), 0, CUSZ_AMD_SCAN_LOAD_AUX);
        __builtin_memcpy(reinterpret_cast<char*>(&dst[z][0]) + 16 * h, &v, 16);
      }
    }
  }
};

template <int V>
__device__ __forceinline__ void store_codes_row(uint16_t* p, const uint16_t (&q)[V])
{
  static_assert(V == 4, "one 8-B store per lane and row");
  uint2 w;
  w.x = (uint32_t)q[0] | ((uint32_t)q[1] << 16);
  w.y = (uint32_t)q[2] | ((uint32_t)q[3] << 16);
  *reinterpret_cast<uint2*>(p) = w;
}

// One brick row of codes between the encode passes: bytes (code - c0, and 255 for the outlier
// code 0) when every code of the row fits [c0, c0 + 254] or is 0, else u16 with the row's bit set
// in the brick's row mask (BrickCodes).  Code 0 is always stored as 255 (never code - c0).
template <int V>
__device__ __forceinline__ void store_brick_row(const BrickCodes& bcs, uint16_t* cbrick, uint8_t* cbrick8, int row,
                                                const uint16_t (&qc)[V], uint64_t& rowmask)
{
  static_assert(V == 4, "one 4-B byte-code store per lane and row");
  bool wide = false;
#pragma unroll
  for (int k = 0; k < V; k++) wide |= (uint32_t)qc[k] - bcs.c0 > 254u && qc[k] != 0;
  if (__builtin_amdgcn_ballot_w64(wide)) {
    store_codes_row<V>(cbrick + (size_t)row * (64 * V), qc);
    rowmask |= 1ull << row;
  }
  else {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < V; k++) w |= (qc[k] == 0 ? 255u : (uint32_t)qc[k] - bcs.c0) << (8 * k);
    *reinterpret_cast<uint32_t*>(cbrick8 + (size_t)row * (64 * V)) = w;
  }
}

// Pass-1 visiting order (BrickSample): iteration j < count takes sample brick j stride + stride / 2,
// then the other bricks in index order (the k-th of them: group k / (stride - 1), skipping the
// group's sample position; stride - 1 is a power of two).  stride 1: index order.
__device__ __forceinline__ uint32_t pass1_brick(uint32_t j, const BrickSample& sp)
{
  if (sp.stride <= 1) return j;
  const uint32_t o = sp.stride / 2;
  if (j < sp.count) return j * sp.stride + o;
  const uint32_t k = j - sp.count, m = sp.stride - 2, g = k >> (31 - __builtin_clz(sp.stride - 1)), p = k & m;
  return g * sp.stride + (p < o ? p : p + 1);
}

// End of a pass-1 unit: outlier count, row mask, the unit's histogram as a u16 record (16-B
// stores, 8 bins per lane; the wave's LDS copy is cleared) and into the workgroup histogram; a
// sample brick also adds it to the codebook sample (global atomics) and then counts itself done.
__device__ __forceinline__ void finish_unit(const OutlierSink& ol, const BrickCodes& bcs, uint32_t u, uint32_t cnt,
                                            uint64_t rowmask, uint32_t* s_hist, uint32_t* s_wg, uint16_t* bhist,
                                            int hs, int lane, const BrickSample& sp, bool sample)
{
  if (lane == 0) ol.brick_cnt[u] = cnt;
  if (lane == 0) bcs.rowmask[u] = rowmask;  // kUnitBricks == 1: unit = brick
  hfd::wave_sync();
  uint16_t* bh = bhist + (size_t)u * hs;
  for (int i0 = lane * 8; i0 < hs; i0 += 512) {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      c[k] = 0;
#pragma unroll
      for (int j = 0; j < kHistCopies; j++) c[k] += s_hist[(i0 + k) * kHistCopies + j];
    }
#pragma unroll
    for (int k = 0; k < 8 * kHistCopies; k++) s_hist[i0 * kHistCopies + k] = 0;
    *reinterpret_cast<uint4*>(bh + i0) =
        make_uint4(c[0] | c[1] << 16, c[2] | c[3] << 16, c[4] | c[5] << 16, c[6] | c[7] << 16);
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (c[k]) atomicAdd(&s_wg[i0 + k], c[k]);
    if (sample)
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (c[k]) atomicAdd(&sp.hist[(i0 + k) * kSampleBinStride], c[k]);
  }
  hfd::wave_sync();
  if (sample) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's sample atomics have completed
    uint32_t prev = 0;
    // release / acquire at agent scope: the wave completing the sample sees every sample brick's
    // atomics by the memory model, not only by the hardware's ordering (once per sample brick)
    if (lane == 0) prev = __hip_atomic_fetch_add(sp.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)prev) == sp.count - 1 && sp.pub_flag) {
      // the sample is complete: this wave hands it to the host (agent-scope reads: every
      // sample brick's atomics have completed before its count)
      for (int i = lane; i < sp.bklen; i += 64)
        sp.pub_dst[i] = __hip_atomic_load(sp.hist + i * kSampleBinStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      hfd::wave_sync();
      if (lane == 0) __hip_atomic_store(sp.pub_flag, sp.pub_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// =========================================================================================
// pass 1: predict -> histograms + outliers
// =========================================================================================
// Rows are streamed: one brick row (y, z) at a time, in (y, z) order, with the z-diff against
// the previous row of the same y-step and the y-diff against row (y - 1, z) kept in registers
// (bprev).  kScanAhead rows (two y-steps) are in flight per wave, loaded into a register queue
// whose slot is the row's position modulo kScanAhead (the row loop is unrolled by kScanAhead, so
// the queue needs no copies); the loads run across brick boundaries.  f32: capped at 128 VGPRs
// (4 waves per SIMD: a 512^3 field's 8192 bricks are exactly two rounds of the 4096 waves).
template <typename T>
#ifndef CUSZ_AMD_SCAN_AHEAD
#define CUSZ_AMD_SCAN_AHEAD 8
#endif
constexpr int kScanAhead = sizeof(T) == 4 ? CUSZ_AMD_SCAN_AHEAD : 8;

template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(64 * kBrickWaves)
__attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 3 : 1)))  // f32: <= 168 VGPRs, 3 waves per SIMD
k_brick3_scan(const T* __restrict__ in, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2_r, T r, OutlierSink ol,
              uint32_t* __restrict__ g_hist, uint16_t* __restrict__ bhist, BrickCodes bcs, int bklen,
              uint32_t nbx, uint32_t nby, uint32_t nbricks, HostPub pub, BrickSample sp)
{
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wid: uniform (SGPR)
  uint32_t* s_wg = smem;                                // workgroup histogram (-> global, once)
  uint32_t* s_hist = smem + (1 + wid * kHistCopies) * kMaxBklen;  // this wave's brick histogram
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_wg[i] = 0;
  for (int i = lane; i < bhist_stride(bklen) * kHistCopies; i += 64) s_hist[i] = 0;
  const uint32_t hc = (uint32_t)lane & (kHistCopies - 1);
  __syncthreads();
  const uint32_t nw = gridDim.x * kBrickWaves;
  const StepLoader<T, V> ld{in, (size_t)lx * ly, lx, ly, lz, nbx, nby, nbricks, 0, (uint32_t)lane};
  const size_t plane = ld.plane;
  const uint32_t nunits = (nbricks + kUnitBricks - 1) / kUnitBricks;
  const int hs = bhist_stride(bklen);
  constexpr int D = kScanAhead<T>;
  static_assert(64 % D == 0 && D % 8 == 0, "the queue holds whole y-steps");
  uint32_t it = blockIdx.x * kBrickWaves + wid;  // iteration; its brick in the pass-1 order (BrickSample)
  const T bias = r - (T)bcs.c0;  // the byte-first path (below)
  T q[D][V];
  {
    const auto b0 = ld.rows_of(it < nunits ? pass1_brick(it, sp) : nbricks);
#pragma unroll
    for (int j = 0; j < D; j++) ld.issue_row(b0, (uint32_t)j >> 3, (uint32_t)j & 7u, q[j]);
  }
  static_assert(kUnitBricks == 1, "one row mask per unit");
  uint64_t rowmask = 0;  // rows of the brick stored as u16 (uniform)
  for (; it < nunits; it += nw) {
    uint32_t cnt = 0;
    const uint32_t u = pass1_brick(it, sp);
    const uint32_t bend = u + 1;
    for (uint32_t brick = u; brick < bend; brick++) {
      const uint32_t bnext = it + nw < nunits ? pass1_brick(it + nw, sp) : nbricks;  // next brick of the stream
      const auto rc = ld.rows_of(brick), rn = ld.rows_of(bnext);
      const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
      const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 8, z0 = bz * 8;
      uint16_t* cbrick = bcs.c16 + (size_t)brick * 64 * (64 * V) + (size_t)lane * V;
      uint8_t* cbrick8 = bcs.c8 + (size_t)brick * 64 * (64 * V) + (size_t)lane * V;
      rowmask = 0;
      T bprev[8][V], pprev[V];
#pragma unroll
      for (int z = 0; z < 8; z++)
#pragma unroll
        for (int k = 0; k < V; k++) bprev[z][k] = (T)0;
      static_assert(D == 8, "one y-step in flight: the rows ahead are one y-step of one brick");
#pragma unroll 1
      for (int r0 = 0; r0 < 64; r0 += D) {  // not unrolled: instruction cache
        const bool last = r0 + D >= 64;  // the rows ahead are the next brick's first y-step
        const auto ahead = last ? rn : rc;
        const uint32_t ya = last ? 0u : (uint32_t)(r0 + D) >> 3;
#pragma unroll
        for (int j = 0; j < D; j++) {
          const int row = r0 + j, z = j & 7, y = row >> 3;
          T p[V];
#pragma unroll
          for (int k = 0; k < V; k++) p[k] = dround(q[j][k] * ebx2_r);
          ld.issue_row(ahead, ya, (uint32_t)j & 7u, q[j]);  // row + D: y-step ya of `ahead`, z = j
          const uint32_t gy = y0 + (uint32_t)y;
          // z-diff (lrz_c.cuhip.inl:341-352 order: z, then x inside the 8-wide tile, then y)
          T a[V];
#pragma unroll
          for (int k = 0; k < V; k++) {
            a[k] = z > 0 ? p[k] - pprev[k] : p[k];
            pprev[k] = p[k];
          }
          const T west = shr_in_tile<T, 1, 8 / V>(a[V - 1]);
#pragma unroll
          for (int k = V - 1; k > 0; k--) a[k] = a[k] - a[k - 1];
          if (x0 % 8 != 0) a[0] = a[0] - west;
          T d[V];
#pragma unroll
          for (int k = 0; k < V; k++) {
            d[k] = a[k] - bprev[z][k];  // bprev = 0 on the brick's first y-step: a - 0 == a
            bprev[z][k] = a[k];
          }
          if (gy >= ly || z0 + (uint32_t)z >= lz) continue;  // outside the field (wave-uniform)
          float olv[V];
          uint16_t qc[V];
          uint64_t anyol = 0;  // SALU: OR of the per-element outlier lane masks
          if constexpr (!ZZ && sizeof(T) == 4 && kHistCopies == 1) {
            // Byte-first quantization.  d is integer-valued, so for |d| < r the reference code
            // (int)(d + r) equals (int)(d + bias) + c0 (bias = r - c0, i.e. 127 unless r < 127) and
            // the byte is (int)(d + bias).
            // A row is clean when every element has |d| < r and a byte in [0, 254]: then the
            // bytes pack by shifts, the histogram bin is byte + c0, and nothing else is computed.
            // Any other row (an outlier, a NaN, a code outside the byte window) takes the exact path.
            int cib[V];
            bool q[V];
            uint64_t suspect = 0;
#pragma unroll
            for (int k = 0; k < V; k++) {
              cib[k] = (int)(d[k] + bias);
              q[k] = dabs(d[k]) < r;
              anyol |= __ballot(!q[k]);
              suspect |= __ballot((uint32_t)cib[k] > 254u);
            }
            if ((suspect | anyol) == 0) {
              uint32_t* s_hc0 = s_hist + bcs.c0;
#pragma unroll
              for (int k = 0; k < V; k++) atomicAdd(&s_hc0[cib[k]], 1u);
              static_assert(V == 4, "one 4-B byte store per lane and row");
              *reinterpret_cast<uint32_t*>(cbrick8 + (size_t)row * (64 * V)) =
                  (uint32_t)cib[0] | (uint32_t)cib[1] << 8 | (uint32_t)cib[2] << 16 | (uint32_t)cib[3] << 24;
              continue;
            }
#pragma unroll
            for (int k = 0; k < V; k++) {
              qc[k] = q[k] ? (uint16_t)(cib[k] + (int)bcs.c0) : uint16_t(0);
              olv[k] = (float)(d[k] + r);  // quantize(): the outlier value is d + r
              atomicAdd(&s_hist[qc[k]], 1u);
            }
          }
          else {
#pragma unroll
            for (int k = 0; k < V; k++) {
              bool is_ol;
              qc[k] = quantize<T, ZZ>(d[k], r, is_ol, olv[k]);
              anyol |= __ballot(is_ol);
              atomicAdd(&s_hist[qc[k] * kHistCopies + hc], 1u);
            }
          }
          store_brick_row<V>(bcs, cbrick, cbrick8, row, qc, rowmask);
          if (anyol) {
            uint32_t mask = 0;
            size_t idx[V];
            const size_t base = (size_t)(z0 + z) * plane + (size_t)gy * lx;
#pragma unroll
            for (int k = 0; k < V; k++) {
              mask |= (uint32_t)(qc[k] == 0 && (ZZ ? !(dabs(d[k]) < r) : true)) << k;
              idx[k] = base + x0 + k;
            }
            emit_outliers<V>(ol, u, cnt, mask, olv, idx);  // one slot per unit
          }
        }
      }
    }
    finish_unit(ol, bcs, u, cnt, rowmask, s_hist, s_wg, bhist, hs, lane, sp, sp.hist && it < sp.count);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) {
    const uint32_t c = s_wg[i];
    if (c) atomicAdd(&g_hist[i], c);
  }
  publish_last(pub);
}

// 1-D pass 1 (lrz_c.cuhip.inl:23-109): a brick is 64 consecutive chunks of W = 256 (16 tiles
// of 1024), brick row r = chunk 64 b + r, so brick order is index order.  Lane l holds x in
// [4 l, 4 l + 4) of each row; the prequant of the element before the row's first comes from lane
// 63 of the previous row, 0 at a tile start.  Rows are loaded kScanAhead ahead (register queue,
// raw buffer loads from the brick's origin, past the field's end they read 0); codes, histograms,
// outlier slots and row masks as in the 3-D pass.
//
// 2-D fields use the same linear bricks (ND = 2, lx % 4 == 0, lx >= 256): the predictor is the
// reference's 2-D one (lrz_c.cuhip.inl:187-273, 32 x 32 tiles: a = p - p(north) unless y % 32 == 0,
// then d = a - a(west) unless x % 32 == 0), the north row coming from a second load queue.
template <typename T, int V, bool ZZ, int ND>
__global__ void __launch_bounds__(64 * kBrickWaves)
k_brick1_scan(const T* __restrict__ in, size_t n, T ebx2_r, T r, OutlierSink ol, uint32_t* __restrict__ g_hist,
              uint16_t* __restrict__ bhist, BrickCodes bcs, int bklen, uint32_t nbricks, HostPub pub, uint32_t lx,
              BrickSample sp)
{
  static_assert(V == 4, "W = 256");
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* s_wg = smem;
  uint32_t* s_hist = smem + (1 + wid * kHistCopies) * kMaxBklen;
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_wg[i] = 0;
  for (int i = lane; i < bhist_stride(bklen) * kHistCopies; i += 64) s_hist[i] = 0;
  const uint32_t hc = (uint32_t)lane & (kHistCopies - 1);
  __syncthreads();
  const uint32_t nw = gridDim.x * kBrickWaves;
  const int hs = bhist_stride(bklen);
  constexpr int D = kScanAhead<T>;
  constexpr uint32_t kBE = 64 * 64 * V;  // elements per brick
  const uint32_t x0 = (uint32_t)lane * V;
  // a brick's descriptor, made once per brick (past the last brick: brick 0 with an empty range,
  // which reads 0 and touches no memory, so every path issues the same loads and the waits can
  // be counted, StepLoader::issue_row)
  auto rows_of = [&](uint32_t b) {
    const bool live = b < nbricks;
    const size_t o = live ? (size_t)b * kBE : 0;
    const uint32_t span = live ? (uint32_t)(min((size_t)kBE, n - o) * sizeof(T)) : 0u;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(in + o), 0, (int)span, 0x00020000);
  };
  auto issue_row = [&](__amdgpu_buffer_rsrc_t rs, int row, T (&dst)[V]) {
    const uint32_t off = ((uint32_t)row * (64 * V) + x0) * (uint32_t)sizeof(T);
#pragma unroll
    for (int h = 0; h < (int)(V * sizeof(T) / 16); h++) {
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16 * h), 0, CUSZ_AMD_SCAN_LOAD_AUX);
      __builtin_memcpy(reinterpret_cast<char*>(&dst[0]) + 16 * h, &v, 16);
    }
  };
  // 2-D: the north row (element i - lx) of the row issued, by a whole-field resource (the field is
  // < 2^31 bytes, brick_geom); rows on a tile's first line (y % 32 == 0) read 0 past its range.
  // (xi, yi) is the issue cursor of this lane's first element, (xl, yl) the compute cursor.
  const __amdgpu_buffer_rsrc_t rsall =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(in), 0, (int)(ND == 2 ? n * sizeof(T) : 0), 0x00020000);
  uint32_t xi = 0, yi = 0;
  auto cursor_at = [&](uint32_t b, uint32_t& x, uint32_t& y) {
    const size_t i = (size_t)b * kBE + x0;
    x = (uint32_t)(i % lx), y = (uint32_t)(i / lx);
  };
  auto advance = [&](uint32_t& x, uint32_t& y) {  // next row: + 64 V elements (lx >= 64 V)
    x += 64 * V;
    if (x >= lx) x -= lx, y++;
  };
  auto issue_north = [&](uint32_t b, uint32_t x, uint32_t y, T (&dst)[V]) {
    const size_t i = (size_t)y * lx + x;
    const uint32_t off = (b < nbricks && y % 32u != 0u) ? (uint32_t)((i - lx) * sizeof(T)) : 0x80000000u;
#pragma unroll
    for (int h = 0; h < (int)(V * sizeof(T) / 16); h++) {
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rsall, (int)(off + 16 * h), 0, 0);
      __builtin_memcpy(reinterpret_cast<char*>(&dst[0]) + 16 * h, &v, 16);
    }
  };
  uint32_t it = blockIdx.x * kBrickWaves + wid;  // iteration; its brick in the pass-1 order (BrickSample)
  T q[D][V];
  T qn[ND == 2 ? D : 1][V];
  {
    const uint32_t u0 = it < nbricks ? pass1_brick(it, sp) : nbricks;
    if constexpr (ND == 2) cursor_at(u0, xi, yi);
    const __amdgpu_buffer_rsrc_t r0s = rows_of(u0);
#pragma unroll
    for (int j = 0; j < D; j++) {
      issue_row(r0s, j, q[j]);
      if constexpr (ND == 2) {
        issue_north(u0, xi, yi, qn[j]);
        advance(xi, yi);
      }
    }
  }
  for (; it < nbricks; it += nw) {
    const uint32_t u = pass1_brick(it, sp), un = it + nw < nbricks ? pass1_brick(it + nw, sp) : nbricks;
    uint32_t cnt = 0;
    uint64_t rowmask = 0;
    const size_t bbase = (size_t)u * kBE;
    const bool full = n - bbase >= kBE;  // no element past the field's end (uniform)
    uint16_t* cbrick = bcs.c16 + bbase + x0;
    uint8_t* cbrick8 = bcs.c8 + bbase + x0;
    T carry = 0;  // 1-D: prequant, 2-D: y-difference, of the previous row's last element
    uint32_t xl = 0, yl = 0;
    if constexpr (ND == 2) {
      cursor_at(u, xl, yl);
      // a brick starts on a 1-D tile boundary, not on a 2-D one: the element before it belongs
      // to the previous brick (a is needed when it lies in the same 32-wide tile row)
      if (bbase > 0) {
        const size_t i = bbase - 1;
        const uint32_t y = (uint32_t)(i / lx);
        T a = dround(in[i] * ebx2_r);
        if (y % 32u != 0u) a = a - dround(in[i - lx] * ebx2_r);
        carry = a;
      }
    }
    const __amdgpu_buffer_rsrc_t rc = rows_of(u), rn = rows_of(un);
    static_assert(64 % D == 0, "the rows ahead of a D-row block lie in one brick");
#pragma unroll 1
    for (int r0 = 0; r0 < 64; r0 += D) {
      const bool tail = r0 + D >= 64;  // the rows ahead are the next brick's first rows
      const __amdgpu_buffer_rsrc_t ahead = tail ? rn : rc;
      const int ra = tail ? r0 + D - 64 : r0 + D;
#pragma unroll
      for (int j = 0; j < D; j++) {
        const int row = r0 + j;
        T p[V];
#pragma unroll
        for (int k = 0; k < V; k++) p[k] = dround(q[j][k] * ebx2_r);
        if constexpr (ND == 2) {  // a = p - p(north): 0 past the field / on a tile's first line
#pragma unroll
          for (int k = 0; k < V; k++) p[k] = p[k] - dround(qn[j][k] * ebx2_r);
        }
        const uint32_t bnext = row + D < 64 ? u : un;
        issue_row(ahead, ra + j, q[j]);
        if constexpr (ND == 2) {
          if (row + D == 64) cursor_at(un, xi, yi);  // the queue moves on to the next brick
          issue_north(bnext, xi, yi, qn[j]);
          advance(xi, yi);
        }
        const size_t base = bbase + (size_t)row * (64 * V);
        T west = __shfl_up(p[V - 1], 1);
        const T last = __shfl(p[V - 1], 63);
        if (lane == 0) west = (ND == 2 || (row & 3)) ? carry : T(0);
        carry = last;
        const uint32_t xcur = xl;
        if constexpr (ND == 2) advance(xl, yl);
        if (!full && base >= n) continue;  // past the field's end (uniform)
        T d[V];
#pragma unroll
        for (int k = V - 1; k > 0; k--) d[k] = p[k] - p[k - 1];
        if constexpr (ND == 2)
          d[0] = (xcur % 32u != 0u) ? p[0] - west : p[0];  // x % 32 == 0: a tile's first column
        else
          d[0] = p[0] - west;
        float olv[V];
        uint16_t qc[V];
        uint32_t mask = 0;
#pragma unroll
        for (int k = 0; k < V; k++) {
          bool is_ol;
          qc[k] = quantize<T, ZZ>(d[k], r, is_ol, olv[k]);
          const bool inr = full || base + x0 + k < n;
          if (inr) atomicAdd(&s_hist[qc[k] * kHistCopies + hc], 1u);
          mask |= (uint32_t)(inr && is_ol) << k;
        }
        store_brick_row<V>(bcs, cbrick, cbrick8, row, qc, rowmask);
        if (__builtin_amdgcn_ballot_w64(mask != 0)) {
          size_t idx[V];
#pragma unroll
          for (int k = 0; k < V; k++) idx[k] = base + x0 + k;
          emit_outliers<V>(ol, u, cnt, mask, olv, idx);
        }
      }
    }
    finish_unit(ol, bcs, u, cnt, rowmask, s_hist, s_wg, bhist, hs, lane, sp, sp.hist && it < sp.count);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) {
    const uint32_t c = s_wg[i];
    if (c) atomicAdd(&g_hist[i], c);
  }
  publish_last(pub);
}

// =========================================================================================
// plan: per-brick region sizes and outlier offsets, archive totals and headers
// =========================================================================================
// One launch after the codebook upload plans the whole archive (per unit of kUnitBricks bricks;
// "brick" below indexes units):
//  * per unit: region upper bound ub = (sum_s hist_u[s] len[s] + 31 rows) / 32 cells and its
//    outlier count; block-local exclusive prefixes of both (kPlanBricks units per block);
//  * block totals by agent-scope atomics; the block that finishes last scans them (every brick's
//    base = local prefix + block prefix), fills the size fields and writes both headers.
// Replaces the reference's host-side scans (hf_kernels.cuhip.inl:449-473, compressor.inl:398-418).
constexpr int kPlanBricks = 64;  // units per plan block: 4 per wave (one per wave, 512 blocks: 15 -> 20 us)
constexpr int kPlanThreads = 1024;
constexpr int kPlanWaves = kPlanThreads / 64;
static_assert(kPlanBricks % kPlanWaves == 0 && kPlanBricks <= 64, "wave 0 scans the block's units");

__device__ __forceinline__ uint32_t brick_rows3(uint32_t brick, uint32_t nbx, uint32_t nby, uint32_t ly, uint32_t lz)
{
  const uint32_t t = brick / nbx, by = t % nby, bz = t / nby;
  return min(8u, ly - by * 8) * min(8u, lz - bz * 8);
}

__global__ void __launch_bounds__(kPlanThreads) k_brick_plan(BrickPlanArgs a, HeaderTpl tpl)
{
  __shared__ uint32_t s_len[kMaxBklen];
  __shared__ uint32_t s_ub[kPlanBricks], s_oc[kPlanBricks];
  __shared__ unsigned long long s_bits[kPlanWaves];
  __shared__ uint32_t s_last;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < a.bhs; i += kPlanThreads) s_len[i] = i < a.bklen ? a.book[i] >> 27 : 0u;
  __syncthreads();
  const uint32_t nblk = gridDim.x, b0 = blockIdx.x * kPlanBricks;
  unsigned long long wbits = 0;
  // every histogram of the wave's units is requested before the first is used: bhs <= 1024, two
  // 16-B loads (8 bins each) per lane and unit, bins past bhs (and units past the end) read 0
  constexpr int kPer = kPlanBricks / kPlanWaves;
  const int i0 = lane * 8, i1 = lane * 8 + 512;
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(a.bhist), 0, (int)min((size_t)a.nunits * a.bhs * 2u, (size_t)0x7FFFFFFF), 0x00020000);
  u32x4_t hv[kPer][2];
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const uint32_t brick = b0 + wid * kPer + j;
    const uint32_t hb = brick * (uint32_t)a.bhs * 2u;
    hv[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rh, (int)(brick < a.nunits && i0 < a.bhs ? hb + i0 * 2u : 0x80000000u), 0, 0);
    hv[j][1] = __builtin_amdgcn_raw_buffer_load_b128(rh, (int)(brick < a.nunits && i1 < a.bhs ? hb + i1 * 2u : 0x80000000u), 0, 0);
  }
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const uint32_t slot = wid * kPer + j, brick = b0 + slot;
    uint32_t ub = 0, oc = 0;
    if (brick < a.nunits) {
      uint32_t bits = 0;
      const uint32_t w[8] = {hv[j][0].x, hv[j][0].y, hv[j][0].z, hv[j][0].w, hv[j][1].x, hv[j][1].y, hv[j][1].z, hv[j][1].w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = (k < 4 ? i0 : i1) + 2 * (k & 3);
        if (i < a.bhs) bits += (w[k] & 0xFFFFu) * s_len[i] + (w[k] >> 16) * s_len[i + 1];
      }
      bits = readlane(hfd::wave_incl_scan(bits), 63);  // DPP, no LDS round trips
      wbits += bits;
      uint32_t rows = 0;  // chunks of the unit: each may end with a partial cell
      for (uint32_t b = brick * kUnitBricks; b < min((brick + 1) * kUnitBricks, a.nbricks); b++)
        rows += a.nd == 1 ? min(64u, a.nchunks - 64u * b) : brick_rows3(b, a.nbx, a.nby, a.ly, a.lz);
      ub = (bits + 31u * rows) >> 5;
      const uint32_t bc = a.brick_cnt[brick];
      oc = min(bc, a.cap_per_brick);
      if (bc > a.cap_per_brick && lane == 0) atomicMax(&a.info->max_brick_cnt, bc);  // slot growth
    }
    if (lane == 0) s_ub[slot] = ub, s_oc[slot] = oc;
  }
  if (lane == 0) s_bits[wid] = wbits;
  __syncthreads();
  if (wid == 0) {  // one unit per lane (lanes < kPlanBricks)
    const bool in = lane < kPlanBricks;
    const uint32_t ub = in ? s_ub[lane] : 0u, oc = in ? s_oc[lane] : 0u;
    const uint32_t iu = hfd::wave_incl_scan(ub), io = hfd::wave_incl_scan(oc);
    const uint32_t brick = b0 + lane;
    if (in && brick < a.nunits) a.ub[brick] = ub, a.cell_local[brick] = iu - ub, a.ol_local[brick] = io - oc;
    if (lane == 63) {
      atomicExch(a.cell_pre + blockIdx.x, iu);
      atomicExch(a.ol_pre + blockIdx.x, io);
      unsigned long long tb = 0;
      for (int w = 0; w < kPlanWaves; w++) tb += s_bits[w];
      atomicAdd(&a.info->total_nbit, tb);
      // two-level ticket (pub_device.hh): blocks by blockIdx % 8, then the groups' last ones
      const uint32_t g = blockIdx.x % kPubGroups;
      const uint32_t in_group = nblk / kPubGroups + (g < nblk % kPubGroups ? 1u : 0u);
      const uint32_t groups = nblk < kPubGroups ? nblk : kPubGroups;
      bool last = false;
      if (__hip_atomic_fetch_add(a.ticket + g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1)
        last = __hip_atomic_fetch_add(a.ticket + kPubGroups, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
      s_last = last;
    }
  }
  __syncthreads();
  if (!s_last) return;
  // last block: exclusive scans of the block totals (read back by atomics: other XCDs' L2s)
  __shared__ uint32_t s_wsum[2][kPlanWaves];
  __shared__ uint32_t s_carry[2];
  if (tid < 2) s_carry[tid] = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nblk; c0 += kPlanThreads) {
    const uint32_t i = c0 + tid;
    const uint32_t vc = i < nblk ? atomicAdd(a.cell_pre + i, 0u) : 0u;
    const uint32_t vo = i < nblk ? atomicAdd(a.ol_pre + i, 0u) : 0u;
    const uint32_t ic = hfd::wave_incl_scan(vc), io = hfd::wave_incl_scan(vo);
    if (lane == 63) s_wsum[0][wid] = ic, s_wsum[1][wid] = io;
    __syncthreads();
    uint32_t oc = s_carry[0], oo = s_carry[1];
    for (int w = 0; w < wid; w++) oc += s_wsum[0][w], oo += s_wsum[1][w];
    if (i < nblk) a.cell_pre[i] = oc + ic - vc, a.ol_pre[i] = oo + io - vo;
    __syncthreads();
    if (tid == kPlanThreads - 1) s_carry[0] = oc + ic, s_carry[1] = oo + io;
    __syncthreads();
  }
  if (tid == 0) {
    const unsigned long long ncell = s_carry[0], slot_total = s_carry[1];
    a.cell_pre[nblk] = (uint32_t)ncell;
    a.ol_pre[nblk] = (uint32_t)slot_total;
    const uint32_t sp = *a.spill_cnt;
    const uint32_t sp_kept = sp < a.spill_cap ? sp : a.spill_cap;
    const unsigned long long nbit = __hip_atomic_load(&a.info->total_nbit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.info->total_ncell = ncell;
    a.info->splen = slot_total + sp_kept;
    a.info->outlier_lost = sp > a.spill_cap ? sp - a.spill_cap : 0u;
    a.info->spilled = sp;
    write_headers_dev(a.archive, tpl, nbit, ncell, slot_total + sp_kept, a.phf_offset, a.bitstream_rel);
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
constexpr int kPackRowMax = (64 * 4 * kLmax + 31) / 32 + 2;  // words one row's packing may touch
constexpr int kPackCells = 768;  // per-wave LDS cell buffer (words): rows accumulate until a flush
static_assert(kPackCells >= 2 * kPackRowMax, "a flush every row or two at worst");

// Pass 2 packs the brick's rows from the codes pass 1 left in brick order (row r of brick b at
// (b * 64 + r) * W): per row, codewords (byte rows through a 256-entry table of the byte window)
// -> wave scan of their lengths -> MSB-first packing into the wave's LDS cell buffer (each row
// starts a new cell, hf_kernels.cuhip.inl:97-157).  Rows accumulate back to back in the buffer;
// it is copied to the brick's region in coalesced 256-B stores when the next row might not fit
// and at the brick's end.  Each row's load is issued when the same z of the previous y-step is
// consumed (8 rows in flight).  The loop is VALU-issue-bound (SQ counters: VALU busy ~75 % of
// the kernel), so a row is kept to ~40 VALU: LDS tables at static addresses (their offsets fold
// into the ds immediates), bricks inside the field take a path with no row checks, lanes pack
// left-justified words with no exec masking, one lane records the row's size and entry in LDS.  ~60 VGPRs:
// 8 waves per SIMD.
template <int V, int ND>
__global__ void __launch_bounds__(64 * kBrickWaves) __attribute__((amdgpu_waves_per_eu(8)))
k_brick3_pack(BrickCodes bcs, uint32_t ly, uint32_t lz, const uint32_t* __restrict__ book,
              int bklen, BrickPlanArgs pl, uint32_t* __restrict__ par_nbit, uint32_t* __restrict__ par_entry,
              uint32_t* __restrict__ bitstream, uint32_t nbx, uint32_t nby, uint32_t nbricks, int reverse,
              unsigned int* overflow, HostPub pub)
{
  static_assert(V == 4, "8-B code loads");
  __shared__ uint32_t s_book[kMaxBklen];  // book word by code
  __shared__ uint32_t s_b8[256];          // book word by byte code (255: code 0)
  __shared__ uint32_t s_cells[kBrickWaves][kPackCells];
  __shared__ uint2 s_rowinfo[kBrickWaves][64];  // per row of the wave's brick: bits, first cell
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wid: uniform (SGPR)
  uint32_t* const cells = s_cells[wid];
  const uint32_t nw = gridDim.x * kBrickWaves;  // (read before the divergent fill loops)
  for (int i = threadIdx.x; i < bklen; i += 64 * kBrickWaves) s_book[i] = book[i];
  for (int i = threadIdx.x; i < 256; i += 64 * kBrickWaves) {
    const uint32_t c = i == 255 ? 0u : (uint32_t)i + bcs.c0;
    s_b8[i] = c < (uint32_t)bklen ? book[c] : 0u;
  }
  for (int i = lane; i < kPackCells; i += 64) cells[i] = 0;
  __syncthreads();
  const uint32_t ncell = pl.cell_pre[pl.nblk];
  uint2* ol_dst = reinterpret_cast<uint2*>(bitstream + ncell);  // outlier cells follow the bitstream
  {  // spill list (bricks past their slot; not expected below 10 % outliers) after every slot
    const uint32_t slot_total = pl.ol_pre[pl.nblk], sp = min(*pl.spill_cnt, pl.spill_cap);
    for (uint32_t i = (blockIdx.x * kBrickWaves + wid) * 64 + lane; i < sp; i += nw * 64) {
      const uint64_t c = pl.spill[i];
      ol_dst[slot_total + i] = make_uint2((uint32_t)c, (uint32_t)(c >> 32));
    }
  }
  const uint32_t nunits = pl.nunits;
  const uint32_t lo8 = (uint32_t)lane * 8u, lo4 = (uint32_t)lane * 4u;
  for (uint32_t it = blockIdx.x * kBrickWaves + wid; it < nunits; it += nw) {
    const uint32_t unit = reverse ? nunits - 1 - it : it;
    const uint32_t pb = unit / kPlanBricks;
    // (uniform values loaded per lane: read back as scalars)
    const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)(pl.cell_local[unit] + pl.cell_pre[pb]));
    const uint32_t lim = (uint32_t)__builtin_amdgcn_readfirstlane((int)pl.ub[unit]);
    {  // this unit's outlier slot -> the archive's outlier segment (unit = brick order)
      const uint32_t cnt = min(pl.brick_cnt[unit], pl.cap_per_brick);
      const uint64_t* slot = pl.slots + (size_t)unit * pl.cap_per_brick;
      uint2* d = ol_dst + pl.ol_local[unit] + pl.ol_pre[pb];
      for (uint32_t i = lane; i < cnt; i += 64) {
        const uint64_t c = slot[i];
        d[i] = make_uint2((uint32_t)c, (uint32_t)(c >> 32));
      }
    }
    uint32_t* dst = bitstream + base;
    uint32_t off = 0;    // region words packed (buffered or copied)
    uint32_t fbase = 0;  // region word at the buffer's start
    // buffered words [fbase, off) -> the region (never past lim: the region is an upper bound, so
    // the clamp only guards a corrupt plan), buffer cleared
    auto flush = [&]() {
      hfd::wave_sync();
      const uint32_t n = off - fbase, nst = fbase >= lim ? 0u : min(n, lim - fbase);
      for (uint32_t i0 = 0; i0 < n; i0 += 64) {  // uniform trip count
        const uint32_t i = i0 + (uint32_t)lane;
        if (i < n) {
          const uint32_t v = cells[i];
          cells[i] = 0;
          if (i < nst) dst[fbase + i] = v;
        }
      }
      fbase = off;
      hfd::wave_sync();
    };
    const uint32_t bend = min((unit + 1) * kUnitBricks, nbricks);
    for (uint32_t brick = unit * kUnitBricks; brick < bend; brick++) {
      const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
      const uint32_t y0 = by * 8, z0 = bz * 8;
      // 1-D: rows [0, nrow) of the brick are chunks 64 brick + row (row = 8 y + z)
      const uint32_t nrow = ND == 1 ? min(64u, pl.nchunks - 64u * brick) : 64u;
      const uint32_t nyv = ND == 1 ? (nrow + 7u) / 8u : min(8u, ly - y0), nzv = ND == 1 ? 8u : min(8u, lz - z0);
      const uint8_t* src16 = reinterpret_cast<const uint8_t*>(bcs.c16 + (size_t)brick * 64 * (64 * V));
      const uint8_t* src8 = bcs.c8 + (size_t)brick * 64 * (64 * V);
      const uint64_t rm = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bcs.rowmask[brick]) & 0xFFFFFFFFull) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(bcs.rowmask[brick] >> 32)) << 32);
      // row r: 8 u16 bytes per lane when bit r of rm is set, else 4 code bytes (.x); one 8-B load
      // either way (a byte row's lane reads its neighbour's 4 bytes too: no branch around loads);
      // the row's base is uniform, the lane's offset one of two registers
      auto load_row = [&](uint32_t row) -> uint2 {
        const bool wide = (rm >> row) & 1ull;
        const uint8_t* a = (wide ? src16 + (size_t)row * 512 : src8 + (size_t)row * 256) + (wide ? lo8 : lo4);
        uint2 v;
        __builtin_memcpy(&v, a, 8);
        return v;
      };
      // full: every row of the brick lies in the field (no row checks, no short chunk)
      const bool full = ND == 1 ? nrow == 64u && pl.n - (size_t)brick * 64u * (64u * V) >= 64u * 64u * V
                                : nyv == 8u && nzv == 8u;
      // Packing order: 3-D, the rows in order.  1-D, position k holds row 4 (k mod 16) + k / 16:
      // the brick's 16 tiles' chunks of one phase are adjacent, as the 1-D decoder's lanes read
      // them (lane = tile, phase p = the tile's chunk p: k_brick1_decode), so neighbouring lanes
      // share cache lines instead of reading chunks 4 apart.  par_entry records the placement.
      auto prow = [](uint32_t k) -> uint32_t { return ND == 1 ? 4u * (k & 15u) + (k >> 4) : k; };
      auto row_ok = [&](uint32_t row) { return ND == 1 ? row < nrow : (row & 7u) < nzv; };
      // Straight-line row loop (no branch around a load: the compiler then waits for each row's
      // own load, not for all of them): every row's load is issued, rows outside the field read
      // a row of the brick's own code block and pack nothing.
      uint2 qv[8];
#pragma unroll
      for (int z = 0; z < 8; z++) qv[z] = load_row(prow(z));
      for (uint32_t y = 0; y < (ND == 1 ? 8u : nyv); y++) {
#pragma unroll
        for (int z = 0; z < 8; z++) {
          const uint32_t k = y * 8 + z, row = prow(k);
          if (off - fbase + kPackRowMax > kPackCells) flush();
          uint32_t w[V];
          if ((rm >> row) & 1ull) {
            w[0] = s_book[qv[z].x & 0xFFFFu], w[1] = s_book[qv[z].x >> 16];
            w[2] = s_book[qv[z].y & 0xFFFFu], w[3] = s_book[qv[z].y >> 16];
          }
          else {
#pragma unroll
            for (int k = 0; k < 4; k++) w[k] = s_b8[(qv[z].x >> (8 * k)) & 255u];
          }
          qv[z] = load_row(prow((k + 8) & 63u));
          if (__builtin_expect(!full, 0)) {
            asm volatile("" ::: "memory");  // a real branch: full bricks run no selects here
            if (!row_ok(row)) {
#pragma unroll
              for (int k = 0; k < V; k++) w[k] = 0;
            }
            // 1-D: the field's last chunk may be short; codes past its end get no codeword
            if (ND == 1) {
              const size_t cfirst = ((size_t)brick * 64u + row) * (64u * V);
              if (pl.n - cfirst < 64u * V)
#pragma unroll
                for (int k = 0; k < V; k++)
                  if (cfirst + (uint32_t)lane * V + k >= pl.n) w[k] = 0;
            }
          }
          uint32_t bits = 0;
#pragma unroll
          for (int k = 0; k < V; k++) bits += w[k] >> 27;
          const uint32_t inc = hfd::wave_incl_scan(bits);
          const uint32_t tot = readlane(inc, 63);
          const uint32_t pos = ((off - fbase) << 5) + inc - bits;
          if (__builtin_expect(__builtin_amdgcn_ballot_w64(bits > 64u) == 0, 1))
            hfd::pack4_or_lj(cells, pos, w, bits);
          else
            hfd::pack_words<V>(cells, pos, w, V);
          if (lane == 0) s_rowinfo[wid][row] = make_uint2(tot, base + off);  // the row's bits and first cell
          off += (tot + 31) >> 5;
        }
      }
      flush();  // (ends with a wave sync: every row's info is in)
      const uint32_t ry = lane >> 3, rz = lane & 7;
      const bool lane_ok = ND == 1 ? (uint32_t)lane < nrow : ry < nyv && rz < nzv;
      if (lane_ok) {
        const uint2 ri = s_rowinfo[wid][lane];
        const size_t c = ND == 1 ? (size_t)brick * 64u + (uint32_t)lane : ((size_t)(z0 + rz) * ly + (y0 + ry)) * nbx + bx;
        par_nbit[c] = ri.x;
        par_entry[c] = ri.y;
      }
    }
    if (off > lim && lane == 0) atomicOr(overflow, 1u);  // cannot happen (region is an upper bound)
    for (uint32_t i = off + lane; i < lim; i += 64) dst[i] = 0u;
  }
  // the workgroup that finishes last publishes the compress summary (header, totals, status)
  publish_last(pub);
}

// =========================================================================================
// decompress: chunk decode + reconstruct, one wave per brick
// =========================================================================================
// Lane l decodes chunk l of the brick (brick row (y, z) = (l / 8, l % 8)) in blocks of 64
// symbols into an LDS code tile [row][column]; after each block the wave reconstructs it with
// lane = column (y running sums and z Hillis-Steele in registers, x Hillis-Steele across lanes by
// DPP) and stores whole 256-B rows.
//
// Decode step.  The lane keeps its bits in registers: w0:w1 is a 64-bit window (`sh` = 32 - bits
// of w0 consumed, so the next 32 chunk bits are alignbit(w0, w1, sh)), w2 and nx are the next two
// words.  A step is one table lookup (L1: one or two codes of <= 12 bits; L2: one code of <= 16
// bits, read together; longer codes by threshold counting, hf_device.hh), the symbols' store to
// the tile, and, when the step crosses a word boundary, a shift of the window with nx refilled
// from the lane's LDS ring (word k in slot k % kRing, [slot][lane]: conflict-free).
//
// Ring refills are wave-uniform, every kF steps: each lane issues one 16-B load of its next four
// words (or an out-of-range load that returns nothing, when its ring is full or its chunk read)
// and writes the group it loaded two refills earlier, so a load has 2 kF steps to land and the
// wait for it is a counted vmcnt(1) -- never behind the reconstruction's stores, which are only
// issued after the ring has been drained at the block's end.
//
// Steps are grouped in quarters of kF: a lane takes part in a whole quarter or sits it out,
// decided once from its column count and ring fill (one word crossed per step at most), so the
// steps carry no predicates.  A step reads one table (L1 or L2, chosen by the window: they are
// exclusive) and has no branch: a code longer than 16 bits reads entry 0, "no symbol, no bits",
// so the lane stands still, and one extra step after the quarter decodes it by threshold counting
// (hf_device.hh lookup_long) for the lanes that need it.  A lane may thus run up to 2 kF + 1
// symbols past the block end, into tile columns [64, 74), which move to the block's front after
// the reconstruction.  Tile stores: each step writes both symbol slots of its entry as two
// naturally aligned u16 stores (ds_write_b16 / _d16_hi of one register; a compiler barrier keeps
// them from merging into a 2-B aligned b32 store, which stalls the LDS pipeline); a slot past
// the entry's symbols is overwritten by the next step.
//
// Outliers.  When the archive's cells are grouped by brick and sorted by (row, x) -- this
// compressor writes them so, k_brick_cell_bounds checks -- the k-th zero code of a row takes the
// row's k-th cell (values staged in LDS per brick), and no scatter pass runs; otherwise the
// scatter pass has written the values into `out`, where the reconstruction reads them.
#ifndef CUSZ_AMD_DEC_B  // tuning knobs (overridable at build time for experiments)
#define CUSZ_AMD_DEC_B 12
#endif
#ifndef CUSZ_AMD_DEC_F
#define CUSZ_AMD_DEC_F 4
#endif
#ifndef CUSZ_AMD_DEC_WAVES
#define CUSZ_AMD_DEC_WAVES 8
#endif
#ifndef CUSZ_AMD_DEC_G
#define CUSZ_AMD_DEC_G 2  // ring refill groups in flight (2 or 4)
#endif
constexpr int kDecB = CUSZ_AMD_DEC_B;        // L1 decode table index bits
constexpr int kF = CUSZ_AMD_DEC_F;           // decode steps between ring refills
constexpr int kDecWaves = CUSZ_AMD_DEC_WAVES;  // waves per workgroup (one workgroup per CU)
constexpr int kBlk = 64;                     // columns reconstructed per block (= lanes)
constexpr uint32_t kRing = 16;               // ring words per lane (power of two)
constexpr int kTP = kBlk + 6 + 2 * kF;       // tile row pitch (u16), an odd number of dwords
static_assert(((kTP / 2) & 1) == 1, "odd dword pitch: row r starts at bank (kTP / 2) r");
constexpr uint32_t kCellCap = 128;           // outlier values of a brick kept in LDS
// per wave: ring + junk slot | tile | cell values | row starts (65) | row carries (64)
constexpr size_t kDecTile = (size_t)(kRing + 1) * 64 * 4;
constexpr size_t kDecCells = kDecTile + (size_t)64 * kTP * 2;
constexpr size_t kDecRows = kDecCells + (size_t)kCellCap * 4;
constexpr size_t kDecWaveBytes = kDecRows + (size_t)(65 + 64) * 4;
constexpr uint32_t kBufRsrcW3 = 0x00020000;  // raw buffer resource word 3 (gfx9)
constexpr uint32_t kOOB = 0x80000000u;       // buffer offset past any bitstream: the load returns 0
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);  // uniform: keep it in an SGPR
}
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// x Hillis-Steele inside 8-wide tiles across lanes (lrz_x.cuhip.inl:311-353 order: d = 1, 2, 4;
// t += t[lane - d] when lane % 8 >= d).  d = 1, 2: the source is zeroed on the lanes whose
// value would cross into the next tile, so the DPP add is unconditional (t + 0 == t: no -0
// arises in the reconstruction); d = 4: the bank mask keeps lanes 4-7 and 12-15 of each row.
template <int CTRL, int BANK>
__device__ __forceinline__ float dppf(float v)
{
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, BANK, false));
}
template <int CTRL, int BANK>
__device__ __forceinline__ double dppf(double v)
{
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, BANK, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, BANK, false);
  return __builtin_bit_cast(double, (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32));
}
template <typename T>
__device__ __forceinline__ T x_scan8(T t, uint32_t l7)
{
  t = t + dppf<0x111, 0xf>(l7 == 7 ? T(0) : t);
  t = t + dppf<0x112, 0xf>(l7 >= 6 ? T(0) : t);
  t = t + dppf<0x114, 0xa>(t);
  return t;
}

template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const T* base)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(base), 0, (int)0xFFFFFFFF, (int)kBufRsrcW3);
}
#ifndef CUSZ_AMD_OUT_STORE_AUX
#define CUSZ_AMD_OUT_STORE_AUX 2  // cache-policy bits of the decoders' output stores: 2 = nontemporal
// (config 2 858 -> 893 GB/s: the written field no longer evicts what the next step reads)
#endif
template <typename T>
__device__ __forceinline__ void buf_store(T v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff);
template <>
__device__ __forceinline__ void buf_store<float>(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)voff, (int)soff, CUSZ_AMD_OUT_STORE_AUX);
}
template <>
__device__ __forceinline__ void buf_store<double>(double v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, (int)voff, (int)soff, CUSZ_AMD_OUT_STORE_AUX);
}

// four consecutive elements (16 B for f32, 32 B for f64) at byte offset voff
template <typename T>
__device__ __forceinline__ void buf_store4(const T* v, __amdgpu_buffer_rsrc_t r, uint32_t voff)
{
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
  u32x4v w[sizeof(T) / 4];
  __builtin_memcpy(&w[0], v, 4 * sizeof(T));
#pragma unroll
  for (int i = 0; i < (int)sizeof(T) / 4; i++) __builtin_amdgcn_raw_buffer_store_b128(w[i], r, (int)(voff + 16 * i), 0, CUSZ_AMD_OUT_STORE_AUX);
}

template <typename T>
__device__ __forceinline__ void lds_store4(T* p, const T (&v)[4])
{
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < (int)sizeof(T) / 4; i++) {
    u32x4v w;
    __builtin_memcpy(&w, reinterpret_cast<const char*>(&v[0]) + 16 * i, 16);
    reinterpret_cast<u32x4v*>(p)[i] = w;
  }
}
template <typename T>
__device__ __forceinline__ void lds_load4(const T* p, T (&v)[4])
{
  typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < (int)sizeof(T) / 4; i++) {
    const u32x4v w = reinterpret_cast<const u32x4v*>(p)[i];
    __builtin_memcpy(reinterpret_cast<char*>(&v[0]) + 16 * i, &w, 16);
  }
}

// Outlier values of one brick for the reconstruction, without the scatter pass: the archive's
// cells of the brick are contiguous and sorted by (row, x) (this compressor writes them so; a
// bounds pass checks it), so the k-th zero code of a row, in x order, takes the row's k-th cell.
// `val` holds the brick's values in LDS (or points at the archive's cells, stride 2 words, when
// the brick has more than fit), row_start[64 + 1] the first cell of each row, carry[64] the cells
// of each row consumed by earlier blocks.
struct BrickCells {
  const uint32_t* val;   // value bits of cell j at val[j * vstride]
  uint32_t vstride;
  uint32_t* row_start;   // LDS, 65 entries
  uint32_t* carry;       // LDS, 64 entries
};

// Column of the block a lane reconstructs.  Each 16-lane DPP row holds two 8-wide x tiles
// interleaved -- even lanes the first, odd lanes the second -- so the x Hillis-Steele step d reads
// lane - 2 d (row_shr 2 d) and the lanes whose source lies in the previous tile read past the DPP
// row, which returns 0: no selects (lrz_x.cuhip.inl:311-353 order d = 1, 2, 4; t + 0 == t).
__device__ __forceinline__ uint32_t rcol(uint32_t l) { return (l & 48u) | ((l & 1u) << 3) | ((l & 15u) >> 1); }

template <int CTRL>
__device__ __forceinline__ float dpp0(float v)
{
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp0(double v)
{
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32));
}
// Each step must stay one v_add_*_dpp: left alone, the SLP vectorizer pairs two z rows' steps
// into v_mov_b32_dpp x 2 (plus two movs of the 0 `old`) + v_pk_add_f32, 5 instructions for 2;
// the empty asm makes every step's result opaque to it.
template <typename T>
__device__ __forceinline__ void no_slp(T& t)
{
  if constexpr (sizeof(T) == 4) asm("" : "+v"(t));  // (not volatile: free to schedule)
}
template <typename T>
__device__ __forceinline__ T x_scan8i(T t)
{
  t = t + dpp0<0x112>(t);  // row_shr:2 = column x - 1
  no_slp(t);
  t = t + dpp0<0x114>(t);  // row_shr:4 = column x - 2
  no_slp(t);
  t = t + dpp0<0x118>(t);  // row_shr:8 = column x - 4
  no_slp(t);
  return t;
}

// Rank, in column order, of this lane's zero code among the row's zero codes (m: ballot of the
// row's zero codes over lanes; rcol's order: DPP rows in turn, even lanes before odd lanes).
__device__ __forceinline__ uint32_t col_rank(uint64_t m, uint32_t l)
{
  const uint32_t r0 = l & 48u;
  const uint32_t below = (uint32_t)__builtin_popcountll(m & ((1ull << r0) - 1ull));
  const uint32_t row = (uint32_t)(m >> r0) & 0xFFFFu, li = l & 15u;
  const uint32_t before = (1u << li) - 1u;
  return below + ((l & 1u) ? (uint32_t)__builtin_popcount(row & 0x5555u) + (uint32_t)__builtin_popcount(row & 0xAAAAu & before)
                           : (uint32_t)__builtin_popcount(row & 0x5555u & before));
}

// Reconstruct columns [x0, x0 + 64) of the brick from the code tile (lane l = column rcol(l),
// row pitch TP).  lrz_x.cuhip.inl:271-360 order: v = (outlier + code) - r; y running sum
// (sequential); x then z Hillis-Steele; times 2 eb.  Outlier values (code 0) come from the ranked
// cells (CELLS) or from `out`, where the scatter pass has put them.  Stores address the block's
// row (y, z) as a buffer at base + y lx with z plane as the scalar offset.
template <typename T, bool ZZ, bool BUF, int TP, bool CELLS>
__device__ __forceinline__ void recon_block(const uint16_t* tile, T* out, size_t plane, uint32_t lx, uint32_t nyv,
                                            uint32_t nzv, size_t base_elem, T r, T ebx2, int lane,
                                            const BrickCells* bc = nullptr)
{
  T* base = out + base_elem;  // element (x0, y0, z0) of this block
  const uint32_t col = rcol((uint32_t)lane);
  const uint32_t voff = col * (uint32_t)sizeof(T);
  const bool full = nyv == 8u && nzv == 8u;  // wave-uniform
  T s[8];
#pragma unroll
  for (int y = 0; y < 8; y++) {
    if ((uint32_t)y >= nyv) break;
    uint32_t cd[8];
#pragma unroll
    for (int z = 0; z < 8; z++) cd[z] = tile[(y * 8 + z) * TP + col];
    T v[8];
#pragma unroll
    for (int z = 0; z < 8; z++) {
      if constexpr (ZZ)
        v[z] = (T)zz_dec((uint16_t)cd[z]);
      else
        v[z] = (T)cd[z] - r;
    }
    const uint32_t mn = min(min(min(cd[0], cd[1]), min(cd[2], cd[3])), min(min(cd[4], cd[5]), min(cd[6], cd[7])));
    if (__builtin_amdgcn_ballot_w64(mn == 0u)) {  // a zero code in this y step (rare)
      if constexpr (CELLS) {  // outliers: ranked cells of the brick
#pragma unroll
        for (int z = 0; z < 8; z++) {
          const uint64_t m = __builtin_amdgcn_ballot_w64(cd[z] == 0u);
          if (m && (uint32_t)z < nzv) {
            const uint32_t row = (uint32_t)y * 8u + (uint32_t)z;
            const uint32_t c0 = bc->row_start[row] + bc->carry[row], ce = bc->row_start[row + 1];
            const uint32_t j = c0 + col_rank(m, (uint32_t)lane);
            if (cd[z] == 0u) v[z] = (j < ce ? (T)__builtin_bit_cast(float, bc->val[j * bc->vstride]) : T(0)) - r;
            hfd::wave_sync();
            if (lane == 0) bc->carry[row] += (uint32_t)__builtin_popcountll(m);
          }
        }
      }
      else {  // outliers: their values were scattered into out
        T ov[8];
#pragma unroll
        for (int z = 0; z < 8; z++) {
          ov[z] = T(0);
          if (__builtin_amdgcn_ballot_w64(cd[z] == 0u) && (uint32_t)z < nzv) ov[z] = base[(size_t)z * plane + (size_t)y * lx + col];
        }
#pragma unroll
        for (int z = 0; z < 8; z++)
          if (cd[z] == 0u) v[z] = ZZ ? ov[z] + T(0) : ov[z] - r;
      }
    }
    T t[8];
    if constexpr (sizeof(T) == 4) {
      // the same IEEE operations, two z rows per packed instruction where the operands pair up
      // (v_pk_add_f32 / v_pk_mul_f32): the y sums, the z Hillis-Steele steps d = 2, 4, the scale
      typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < 4; j++) {
        f2 sv = {s[2 * j], s[2 * j + 1]};
        const f2 vv = {v[2 * j], v[2 * j + 1]};
        sv = y > 0 ? sv + vv : vv;
        s[2 * j] = sv.x, s[2 * j + 1] = sv.y;
        t[2 * j] = x_scan8i<T>(sv.x), t[2 * j + 1] = x_scan8i<T>(sv.y);
      }
#pragma unroll
      for (int z = 7; z >= 1; z--) t[z] = t[z] + t[z - 1];
      f2 tp[4];
#pragma unroll
      for (int j = 0; j < 4; j++) tp[j] = f2{t[2 * j], t[2 * j + 1]};
      tp[3] = tp[3] + tp[2], tp[2] = tp[2] + tp[1], tp[1] = tp[1] + tp[0];  // d = 2 (descending)
      tp[3] = tp[3] + tp[1], tp[2] = tp[2] + tp[0];                          // d = 4
#pragma unroll
      for (int j = 0; j < 4; j++) tp[j] = tp[j] * f2{(float)ebx2, (float)ebx2};
#pragma unroll
      for (int j = 0; j < 4; j++) t[2 * j] = tp[j].x, t[2 * j + 1] = tp[j].y;
    }
    else {
#pragma unroll
      for (int z = 0; z < 8; z++) {
        s[z] = y > 0 ? s[z] + v[z] : v[z];
        t[z] = x_scan8i<T>(s[z]);
      }
#pragma unroll
      for (int d = 1; d < 8; d *= 2)
#pragma unroll
        for (int z = 7; z >= d; z--) t[z] = t[z] + t[z - d];
#pragma unroll
      for (int z = 0; z < 8; z++) t[z] = t[z] * ebx2;
    }
    T* rowb = base + (size_t)y * lx;
    if constexpr (BUF) {
      const __amdgpu_buffer_rsrc_t ro = rsrc(rowb);
      if (full) {
#pragma unroll
        for (int z = 0; z < 8; z++) buf_store<T>(t[z], ro, voff, (uint32_t)((size_t)z * plane * sizeof(T)));
      }
      else {
#pragma unroll
        for (int z = 0; z < 8; z++)
          if ((uint32_t)z < nzv) buf_store<T>(t[z], ro, voff, (uint32_t)((size_t)z * plane * sizeof(T)));
      }
    }
    else {
#pragma unroll
      for (int z = 0; z < 8; z++)
        if ((uint32_t)z < nzv) rowb[(size_t)z * plane + col] = t[z];
    }
  }
}

// lanes 32-63: lane - 32's x; lanes 0-31: -0.0 (v_permlane32_swap: lanes 32-63 of the first
// operand trade with lanes 0-31 of the second)
template <typename T>
__device__ __forceinline__ T from_lower_half(T x)
{
  if constexpr (sizeof(T) == 4) {
    const auto s = __builtin_amdgcn_permlane32_swap(0x80000000u, __builtin_bit_cast(uint32_t, x), false, false);
    return __builtin_bit_cast(T, (uint32_t)s[0]);
  }
  else {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const auto lo = __builtin_amdgcn_permlane32_swap(0u, (uint32_t)u, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(0x80000000u, (uint32_t)(u >> 32), false, false);
    return __builtin_bit_cast(T, (uint64_t)(uint32_t)lo[0] | ((uint64_t)(uint32_t)hi[0] << 32));
  }
}

// 32-column blocks (the 12-wave decoder, k_brick3_decode32): lane l reconstructs column
// rcol(l mod 32) of y-steps 4 h .. 4 h + 3, h = l / 32, so both halves' x and z scans run
// together.  The y running sum keeps the reference's order: every lane sums its four values
// from a start value, -0.0 in the lower half (-0.0 + v == v for every v, so s_0 = v_0 exactly)
// and, in the upper half, the lower half's s_3 of the same column (v_permlane32_swap).
// Outliers: as recon_block, each row's zero codes ranked among the 32 lanes of its half.
template <typename T, bool ZZ, bool BUF, int TP, bool CELLS>
__device__ __forceinline__ void recon_block32(const uint16_t* tile, T* out, size_t plane, uint32_t lx, uint32_t nyv,
                                              uint32_t nzv, size_t base_elem, T r, T ebx2, int lane,
                                              const BrickCells* bc = nullptr)
{
  T* base = out + base_elem;  // element (x0, y0, z0) of this block
  const uint32_t hl = (uint32_t)lane >> 5, l32 = (uint32_t)lane & 31u;
  const uint32_t col = rcol(l32);
  const uint32_t ybase = 4u * hl;
  T v[4][8];
#pragma unroll
  for (int yy = 0; yy < 4; yy++) {
    const uint32_t y = ybase + (uint32_t)yy;
    const bool yok = y < nyv;
    uint32_t cd[8];
#pragma unroll
    for (int z = 0; z < 8; z++) cd[z] = tile[(y * 8 + (uint32_t)z) * TP + col];
#pragma unroll
    for (int z = 0; z < 8; z++) {
      if constexpr (ZZ)
        v[yy][z] = (T)zz_dec((uint16_t)cd[z]);
      else
        v[yy][z] = (T)cd[z] - r;
    }
    const uint32_t mn = min(min(min(cd[0], cd[1]), min(cd[2], cd[3])), min(min(cd[4], cd[5]), min(cd[6], cd[7])));
    if (__builtin_amdgcn_ballot_w64(yok && mn == 0u)) {  // a zero code in this y step (rare)
      if constexpr (CELLS) {  // outliers: ranked cells of the brick
#pragma unroll
        for (int z = 0; z < 8; z++) {
          const uint64_t m = __builtin_amdgcn_ballot_w64(yok && cd[z] == 0u);
          if (m && (uint32_t)z < nzv) {
            const uint32_t mh = (uint32_t)(m >> (32u * hl));  // this half's row
            const uint32_t row = y * 8u + (uint32_t)z;
            if (mh) {
              const uint32_t c0 = bc->row_start[row] + bc->carry[row], ce = bc->row_start[row + 1];
              const uint32_t j = c0 + col_rank((uint64_t)mh, l32);
              if (cd[z] == 0u) v[yy][z] = (j < ce ? (T)__builtin_bit_cast(float, bc->val[j * bc->vstride]) : T(0)) - r;
            }
            hfd::wave_sync();
            if (l32 == 0 && mh) bc->carry[row] += (uint32_t)__builtin_popcount(mh);
          }
        }
      }
      else {  // outliers: their values were scattered into out
#pragma unroll
        for (int z = 0; z < 8; z++) {
          if (yok && cd[z] == 0u && (uint32_t)z < nzv) {
            const T o = base[(size_t)z * plane + (size_t)y * lx + col];
            v[yy][z] = ZZ ? o + T(0) : o - r;
          }
        }
      }
    }
  }
  // y running sums: the lower half's s_3 (computed by every lane, used by the upper half)
  T c[8];
#pragma unroll
  for (int z = 0; z < 8; z++) {
    T u = v[0][z];
#pragma unroll
    for (int yy = 1; yy < 4; yy++) u = u + v[yy][z];
    c[z] = from_lower_half<T>(u);
  }
#pragma unroll
  for (int yy = 0; yy < 4; yy++) {
    const uint32_t y = ybase + (uint32_t)yy;
    T t[8];
#pragma unroll
    for (int z = 0; z < 8; z++) {
      c[z] = c[z] + v[yy][z];
      t[z] = x_scan8i<T>(c[z]);
    }
#pragma unroll
    for (int d = 1; d < 8; d *= 2)
#pragma unroll
      for (int z = 7; z >= d; z--) t[z] = t[z] + t[z - d];
#pragma unroll
    for (int z = 0; z < 8; z++) t[z] = t[z] * ebx2;
    if (y < nyv) {
      if constexpr (BUF) {
        const __amdgpu_buffer_rsrc_t ro = rsrc(base + (size_t)yy * lx);
        const uint32_t voff = (col + hl * 4u * lx) * (uint32_t)sizeof(T);
#pragma unroll
        for (int z = 0; z < 8; z++)
          if ((uint32_t)z < nzv) buf_store<T>(t[z], ro, voff, (uint32_t)((size_t)z * plane * sizeof(T)));
      }
      else {
        T* rowb = base + (size_t)y * lx;
#pragma unroll
        for (int z = 0; z < 8; z++)
          if ((uint32_t)z < nzv) rowb[(size_t)z * plane + col] = t[z];
      }
    }
  }
}

#ifdef CUSZ_AMD_DEC_PROFILE
// diagnostic build (psz_amd_debug_brick_profile): per-phase clocks and counts summed over waves:
// 0 bricks, 1 brick-start cycles (cells, loads and their wait), 2 decode-loop cycles, 3 drain
// cycles, 4 reconstruct cycles, 5 loop iterations, 6 lane-quarters sat out for want of data,
// 7 lane-steps done
__device__ unsigned long long g_brick_prof[16];
#define BPROF(...) __VA_ARGS__
#else
#define BPROF(...)
#endif

// Cells of a brick-layout archive: bstart[b] = first cell of brick b (nbricks + 1 entries) and
// *unsorted != 0 unless the cells are grouped by brick and sorted by (row, x) inside each brick
// -- key (brick, row = (y % 8) * 8 + z % 8, x % 256) strictly increasing: then every bstart
// entry is written; otherwise *unsorted = epoch (the word is never reset: no memset launch).
__global__ void __launch_bounds__(256) k_brick_cell_bounds(const uint32_t* __restrict__ cells, size_t ncell,
                                                           uint32_t lx, uint32_t ly, uint32_t lz, uint32_t nbx,
                                                           uint32_t nby, uint32_t nbricks, uint32_t* bstart,
                                                           uint32_t* unsorted, uint32_t epoch)
{
  auto key = [&](uint32_t idx, uint32_t& brick) -> uint64_t {
    const uint32_t x = idx % lx, yz = idx / lx, y = yz % ly, z = yz / ly;
    brick = (z < lz) ? ((z / 8) * nby + y / 8) * nbx + x / 256 : nbricks;
    return ((uint64_t)brick << 14) | (((y & 7u) * 8u + (z & 7u)) << 8) | (x & 255u);
  };
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < ncell; i += (size_t)gridDim.x * 256) {
    uint32_t b, bp = 0;
    const uint64_t k = key(cells[2 * i + 1], b);
    int64_t prev = -1;
    if (i > 0) {
      const uint64_t kp = key(cells[2 * i - 1], bp);
      if (kp >= k) *unsorted = epoch;
      prev = bp;
    }
    if (b >= nbricks) *unsorted = epoch;
    for (int64_t u = prev + 1; u <= (int64_t)b && u <= (int64_t)nbricks; u++) bstart[u] = (uint32_t)i;
    if (i + 1 == ncell)
      for (int64_t u = (int64_t)b + 1; u <= (int64_t)nbricks; u++) bstart[u] = (uint32_t)ncell;
  }
}

#ifdef CUSZ_AMD_DEC_PROFILE
#define BPROF_P , unsigned long long(&pc)[16], unsigned long long &tk, unsigned long long &tp
#define BPROF_A , pc, tk, tp
#define BPROF_A4 , pc, tk, tp
#define BPROF_P4 , unsigned long long(&pc)[16], unsigned long long &tk, unsigned long long &tp0
#else
#define BPROF_P4
#define BPROF_P
#define BPROF_A
#define BPROF_A4
#endif

// One wave's decoder state that outlives a chunk: bitstream resource, the lane's ring column, the
// code tile.
struct DecWave {
  __amdgpu_buffer_rsrc_t rbits;
  uint32_t* ring_lane;
  uint16_t* tile;
  uint32_t ubk;
  int lane;
};

// Decode one chunk per lane (chunk bits at word vbase / 4, nbit bits, vlen <= W symbols; a dead
// lane decodes nothing) in W / kBlk blocks of kBlk columns into the tile; after each block the
// wave calls recon(blk).  pro() runs while the first words are in flight; blk_start(blk) before
// each block's decode.  W: the chunk length (a multiple of kBlk; 256 in the fused decoders).
template <class Pro, class BlkStart, class Recon>
__device__ __forceinline__ void decode_chunks(const hfd::LdsTables<kDecB>& tb, const hfd::DecRegs& rg,
                                              const DecWave& dw, bool live, uint32_t vbase, uint32_t nbit,
                                              uint32_t vlen, Pro&& pro, BlkStart&& blk_start,
                                              Recon&& recon BPROF_P, uint32_t W = 256,
                                              const u32x4* first = nullptr)
{
  const int lane = dw.lane;
  uint32_t* ring_lane = dw.ring_lane;
  const uint32_t nwords = (nbit + 31u) >> 5;
  // words 0..7 (0..2 into registers, 2..7 into the ring): loaded by the caller ahead of time
  // (first[0..1]), or now, before pro()
  u32x4 a0, a1;
  if (first)
    a0 = first[0], a1 = first[1];
  else {
    a0 = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(live ? vbase : kOOB), 0, 0);
    a1 = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(live ? vbase + 16u : kOOB), 0, 0);
  }
  pro();
  uint32_t w0 = 0, w1 = a0.x, w2 = a0.y, nx = a0.z;
  ring_lane[2 * 64] = a0.z;  // nx is re-read every step, also by a first step that does not move
  ring_lane[3 * 64] = a0.w;
  ring_lane[4 * 64] = a1.x, ring_lane[5 * 64] = a1.y, ring_lane[6 * 64] = a1.z, ring_lane[7 * 64] = a1.w;
  uint32_t kk = 2;    // word index held by nx
  uint32_t ctop = 8;  // words [0, ctop) have been written (ring or registers)
  uint32_t ltop = 8;  // words [0, ltop) have been requested
  uint32_t sh = 0;    // 32 - bits of w0 consumed
  uint32_t cnt = live ? 0u : 0x40000000u;  // symbols decoded; a dead lane never steps
  uint32_t rdy = ctop >= nwords ? 0xFFFFFFFFu : ctop;  // words [0, rdy) are readable
  u32x4 pa, pb;       // groups in flight
  bool fa = false, fb = false;
  BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[1] += tk - tp; tp = tk;)

  auto issue = [&](u32x4& p, bool& f) {
    const bool ok = ltop < nwords && ltop + 4u <= kk + kRing;  // never over a word still needed
    p = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(ok ? vbase + ltop * 4u : kOOB), 0, 0);
    f = ok;
    ltop += ok ? 4u : 0u;
  };
  // Write a landed group into the ring.  The stores are unconditional (a lane without a group
  // writes the junk slot kRing), so the compiler's wait for the load sits here on every path and
  // no load is left pending past the block's end.
  auto consume = [&](const u32x4& p, bool& f) {
#pragma unroll
    for (int i = 0; i < 4; i++) ring_lane[(f ? ((ctop + (uint32_t)i) & (kRing - 1u)) : kRing) * 64] = p[i];
    ctop += f ? 4u : 0u;
    f = false;
    rdy = ctop >= nwords ? 0xFFFFFFFFu : ctop;
  };

  for (int blk = 0; blk < (int)(W / kBlk); blk++) {
    blk_start(blk);
    uint16_t* rowp = dw.tile + lane * kTP - blk * kBlk;  // rowp[cnt] = tile column cnt - 64 blk
    const uint32_t target = min((uint32_t)(blk + 1) * kBlk, vlen);
    auto quarter = [&]() {
      BPROF(pc[6] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(cnt < target && !(kk + (uint32_t)kF + 1u < rdy)));
            pc[7] += kF * __builtin_popcountll(__builtin_amdgcn_ballot_w64(cnt < target && kk + (uint32_t)kF + 1u < rdy));)
      if (cnt < target && kk + (uint32_t)kF + 1u < rdy) {  // at most one word crossed per step
        uint32_t e = 0;
        auto step = [&](bool lng) {
          const uint32_t win = __builtin_amdgcn_alignbit(w0, w1, sh);  // chunk bits [pos, pos + 32)
          // a code longer than 16 bits has no table entry: e = 0 consumes nothing, and the lane
          // decodes it after the quarter (rare: no branch in the steps)
          e = lng ? hfd::lookup_long<kDecB>(tb, rg, win, dw.ubk) : hfd::lookup_short<kDecB>(tb, rg, win);
          // both symbol slots written as naturally aligned u16 stores (the low and high halves
          // of one register); a slot past the entry's symbols is overwritten by the next step
          const uint32_t sy = e & hfd::kEntSymMask;
          rowp[cnt] = (uint16_t)sy;
          asm volatile("" ::: "memory");  // two u16 stores: merged they would be an unaligned b32
          rowp[cnt + 1] = (uint16_t)(sy >> 16);
          cnt += hfd::ent_nsym(e);
          const int32_t s2 = (int32_t)sh - (int32_t)hfd::ent_bits(e);
          const bool shf = s2 < 0;  // crossed into the next word
          sh = (uint32_t)s2 & 31u;
          w0 = shf ? w1 : w0;
          w1 = shf ? w2 : w1;
          w2 = shf ? nx : w2;
          kk += shf ? 1u : 0u;
          nx = ring_lane[(kk & (kRing - 1u)) * 64];
        };
#pragma unroll
        for (int st = 0; st < kF; st++) step(false);
        if (__builtin_amdgcn_ballot_w64(e == 0)) {  // a lane met a long code: one slow step
          if (e == 0) step(true);
        }
      }
    };
#if CUSZ_AMD_DEC_G == 4
    // four groups in flight: a group is written into the ring four refills after its load
    u32x4 pc4, pd4;
    bool fc = false, fd = false;
    issue(pa, fa);
    quarter();
    issue(pb, fb);
    quarter();
    issue(pc4, fc);
    quarter();
    issue(pd4, fd);
    quarter();
    bool odd = false;
    for (;;) {
      consume(pa, fa);
      issue(pa, fa);
      quarter();
      consume(pb, fb);
      issue(pb, fb);
      quarter();
      BPROF(pc[5]++;)
      if (!__builtin_amdgcn_ballot_w64(cnt < target)) { odd = true; break; }
      consume(pc4, fc);
      issue(pc4, fc);
      quarter();
      consume(pd4, fd);
      issue(pd4, fd);
      quarter();
      BPROF(pc[5]++;)
      if (!__builtin_amdgcn_ballot_w64(cnt < target)) break;
    }
    BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[2] += tk - tp; tp = tk;)
    if (odd) {  // in flight, oldest first: c, d, a, b
      consume(pc4, fc);
      consume(pd4, fd);
    }
    consume(pa, fa);
    consume(pb, fb);
    if (!odd) {
      consume(pc4, fc);
      consume(pd4, fd);
    }
#else
    // a group is written into the ring two refills after its load; the first wait of a block
    // comes 2 kF steps after the previous block's stores
    issue(pa, fa);
    quarter();
    issue(pb, fb);
    quarter();
    do {
      BPROF(unsigned long long tc0 = __builtin_readcyclecounter();)
      consume(pa, fa);
      BPROF(hfd::wave_sync(); pc[10] += __builtin_readcyclecounter() - tc0;)
      issue(pa, fa);
      quarter();
      BPROF(tc0 = __builtin_readcyclecounter();)
      consume(pb, fb);
      BPROF(hfd::wave_sync(); pc[10] += __builtin_readcyclecounter() - tc0;)
      issue(pb, fb);
      quarter();
      BPROF(pc[5]++;)
    } while (__builtin_amdgcn_ballot_w64(cnt < target));
    BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[2] += tk - tp; tp = tk;)
    consume(pa, fa);  // drain: nothing stays in flight across the stores below
    consume(pb, fb);
#endif
    hfd::wave_sync();
    BPROF(tk = __builtin_readcyclecounter(); pc[3] += tk - tp; tp = tk;)
    // symbols decoded past the block end move to its front; they
    // are held in registers across the reconstruction, which may use the tile as scratch
    uint32_t* rw = reinterpret_cast<uint32_t*>(dw.tile + lane * kTP);
    uint32_t ovs[kF + 1];
#pragma unroll
    for (int i = 0; i <= kF; i++) ovs[i] = rw[kBlk / 2 + i];
    recon(blk);
    hfd::wave_sync();
#pragma unroll
    for (int i = 0; i <= kF; i++) rw[i] = ovs[i];
    hfd::wave_sync();
    BPROF(tk = __builtin_readcyclecounter(); pc[4] += tk - tp; tp = tk;)
  }
}

// ---- compact decoder (3-D fused path) ---------------------------------------------------------
// The same chunk decode as decode_chunks with fewer instructions per step (the loop is bound by
// how fast one wave issues its dependent chain, not by LDS or HBM bandwidth; round-4 counters:
// 40 VALU + 6 LDS + 6 SALU per step before, ~15 + 4 after):
//  * the window is read from the LDS ring each step: words J and J+1 by one ds_read2st64 (slot
//    16 mirrors slot 0, so the pair never wraps), shifted by alignbit -- no window registers to
//    rotate, no word-crossing test; 8 x (the lane's bit position + 511) masked by 0xF00 is the
//    slot's byte offset, `npos` (= -position) the shift;
//  * compact table entries (hfd::Tab4): the tile pointer advance, the bits and the symbols come
//    out of the entry with one or two instructions each;
//  * the state is the position and the tile pointer: a lane takes part in a quarter while its
//    pointer is below the block's limit and the ring holds every word the quarter can reach.
// Smaller tables and tile (74 columns: 64 + the 9 overshoot) let up to 9 waves share a CU.
constexpr int kTP4 = kBlk + 10;
static_assert(((kTP4 / 2) & 1) == 1, "odd dword pitch");
static_assert(kBlk + 2 * kF + 1 <= kTP4, "overshoot columns");
constexpr uint32_t kRing4 = 16;                                // ring words per lane (+ mirror, junk)
constexpr size_t kD4Tile = (size_t)(kRing4 + 2) * 256;          // slots 0..15, mirror 16, junk 17
constexpr size_t kD4Cells = kD4Tile + (size_t)64 * kTP4 * 2;
constexpr size_t kD4Rows = kD4Cells + (size_t)kCellCap * 4;
constexpr size_t kD4WaveBytes = kD4Rows + (size_t)(65 + 64) * 4;
// 8 waves per CU: a 512^3 field's 8192 bricks are 4 full rounds of the 2048 waves (9 waves left
// a partial fourth round: decode 285 -> 259 us)
#ifndef CUSZ_AMD_DEC4_WAVES
#define CUSZ_AMD_DEC4_WAVES 8
#endif
#ifndef CUSZ_AMD_DEC4_REGWIN
#define CUSZ_AMD_DEC4_REGWIN 0
#endif
constexpr int kDec4Waves = CUSZ_AMD_DEC4_WAVES;
static_assert(sizeof(hfd::Tab4) + kDec4Waves * kD4WaveBytes <= 160 * 1024, "LDS");

// pos8 limit for entering a quarter: every word the quarter reads (<= 4 x 16 + 27 bits on) is in
// the ring (window pair: p + 122 < 32 ctop; register window, which reads word J + 3: p + 186)
constexpr uint32_t kRdy4 = CUSZ_AMD_DEC4_REGWIN ? 8u * (511u - 186u) : 8u * (511u - 123u);

struct DecWave4 {
  __amdgpu_buffer_rsrc_t rbits;
  uint32_t* ring_lane;  // slot s of this lane at ring_lane[64 s]
  uint16_t* tile;
  uint32_t ubk;
  int lane;
};

// One chunk per lane (bits at byte vbase, nbit bits, vlen <= W symbols; a dead lane decodes
// nothing; its first 8 words in first[0..1]) in W / kBlk blocks into the tile; recon(blk) after
// each block, blk_start(blk) before it, pro() while the first words are written.
template <int BLK = kBlk, int TP = kTP4, class Pro, class BlkStart, class Recon>
__device__ __forceinline__ void decode_chunks4(const hfd::Tab4& tb, const hfd::DecRegs4& rg, const DecWave4& dw,
                                               bool live, uint32_t vbase, uint32_t nbit, uint32_t vlen, Pro&& pro,
                                               BlkStart&& blk_start, Recon&& recon BPROF_P4, uint32_t W,
                                               const u32x4* first)
{
  const int lane = dw.lane;
  uint32_t* const ring = dw.ring_lane;
  const uint32_t nwords = live ? (nbit + 31u) >> 5 : 0u;
  u32x4 a0, a1;  // words 0..7: loaded by the caller ahead of time (first[0..1]), or now
  if (first)
    a0 = first[0], a1 = first[1];
  else {
    a0 = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(live ? vbase : kOOB), 0, 0);
    a1 = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(live ? vbase + 16u : kOOB), 0, 0);
  }
  pro();
  ring[0] = a0.x, ring[64] = a0.y, ring[2 * 64] = a0.z, ring[3 * 64] = a0.w;
  ring[4 * 64] = a1.x, ring[5 * 64] = a1.y, ring[6 * 64] = a1.z, ring[7 * 64] = a1.w;
  ring[16 * 64] = a0.x;  // mirror of slot 0
#if CUSZ_AMD_DEC4_REGWIN
  // (variant) window in registers: w0:w1 the 64-bit window, w2 and nx the next words (nx = word
  // kk, re-read from the ring every step), sh = 32 - bits of w0 consumed
  uint32_t w0 = 0, w1 = a0.x, w2 = a0.y, nx = a0.z, sh = 0, kk = 2;
#else
  uint32_t A = 0, Bw = a0.x;  // words J, J + 1 of the window (J = -1 at bit 0: junk, shift 0)
#endif
  uint32_t pos8 = 8u * 511u, npos = 0;  // 8 x (chunk bit position + 511); -position (the shift)
  uint32_t ltop = 8, ctop = 8;   // words requested / written to the ring
  // a quarter reaches at most 4 x 16 + 27 bits: the lane steps only if their words are in
  // (pos8 < 8 (32 ctop + 388))
  uint32_t rdy = ctop >= nwords ? 0xFFFFFFFFu : 256u * ctop + kRdy4;
  uint16_t* tp = dw.tile + lane * TP;
  u32x4 pa, pb;  // groups in flight
  bool fa = false, fb = false;
  BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[1] += tk - tp0; tp0 = tk;)

  // next four words of the chunk, once their slots are free (words before J are)
  auto issue = [&](u32x4& p, bool& f) {
    const bool ok = ltop < nwords && ltop + 4u <= (pos8 >> 8);
    p = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(ok ? vbase + ltop * 4u : kOOB), 0, 0);
    f = ok;
    ltop += ok ? 4u : 0u;
  };
  // a landed group into its slots (and the mirror)
  auto consume = [&](const u32x4& p, bool& f) {
    if (f) {
      uint32_t* sl = ring + (ctop & (kRing4 - 1u)) * 64;
      sl[0] = p.x, sl[64] = p.y, sl[128] = p.z, sl[192] = p.w;
      if ((ctop & (kRing4 - 1u)) == 0u) ring[16 * 64] = p.x;
      ctop += 4u;
      rdy = ctop >= nwords ? 0xFFFFFFFFu : 256u * ctop + kRdy4;
    }
    f = false;
  };
  // the entry's symbols into the tile, the position forward, the next window read
  auto advance = [&](uint32_t e) {
    const uint32_t sy = e & hfd::kEnt4SymMask;
    tp[0] = (uint16_t)sy;
    asm volatile("" ::: "memory");  // two u16 stores: merged they would be an unaligned b32
    tp[1] = (uint16_t)(sy >> 16);
    tp = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(tp) + hfd::ent4_adv(e));
    const uint32_t b = hfd::ent4_bits(e);
#if CUSZ_AMD_DEC4_REGWIN
    const int32_t s2 = (int32_t)sh - (int32_t)b;
    const bool shf = s2 < 0;  // crossed into the next word
    sh = (uint32_t)s2 & 31u;
    w0 = shf ? w1 : w0;
    w1 = shf ? w2 : w1;
    w2 = shf ? nx : w2;
    kk += shf ? 1u : 0u;
    nx = ring[(kk & (kRing4 - 1u)) * 64];
    pos8 += b << 3;
#else
    pos8 += b << 3;
    npos -= b;
    const uint32_t* rr = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ring) + (pos8 & 0xF00u));
    A = rr[0];
    Bw = rr[64];
#endif
  };
#if CUSZ_AMD_DEC4_REGWIN
  auto window = [&]() { return __builtin_amdgcn_alignbit(w0, w1, sh); };
#else
  auto window = [&]() { return __builtin_amdgcn_alignbit(A, Bw, npos); };
#endif

  for (int blk = 0; blk < (int)(W / BLK); blk++) {
    blk_start(blk);
    const uint32_t done = (uint32_t)blk * BLK;
    const uint32_t target = live && vlen > done ? min((uint32_t)BLK, vlen - done) : 0u;
    uint16_t* const tlim = dw.tile + lane * TP + target;
    auto quarter = [&]() {
      BPROF(pc[8] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tp < tlim && !(pos8 < rdy)));
            pc[9] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tp < tlim));)
      if (tp < tlim && pos8 < rdy) {
        uint32_t e = 0;
#pragma unroll
        for (int st = 0; st < kF; st++) {
          e = tb.e[hfd::tab4_index(rg, window())];
          advance(e);
        }
        BPROF(pc[7] += __builtin_amdgcn_ballot_w64(e == 0) ? 1 : 0;)
        if (__builtin_amdgcn_ballot_w64(e == 0)) {  // a code longer than 16 bits stopped the lane
          if (e == 0) advance(hfd::lookup_long4(tb, rg, window(), dw.ubk));
        }
      }
      BPROF(pc[6]++;)
    };
    // one group per two quarters (a lane reads at most 2 x 91 bits in them, 6 words: the ring
    // buffers the difference), each in flight for four quarters
    issue(pa, fa);
    quarter();
    quarter();
    issue(pb, fb);
    quarter();
    quarter();
    bool odd = false;
    // the block ends after the first quarter that leaves no lane short of it
    for (;;) {
      consume(pa, fa);
      issue(pa, fa);
      quarter();
      BPROF(pc[5]++;)
      if (!__builtin_amdgcn_ballot_w64(tp < tlim)) {
        odd = true;
        break;
      }
      quarter();
      if (!__builtin_amdgcn_ballot_w64(tp < tlim)) {
        odd = true;
        break;
      }
      consume(pb, fb);
      issue(pb, fb);
      quarter();
      BPROF(pc[5]++;)
      if (!__builtin_amdgcn_ballot_w64(tp < tlim)) break;
      quarter();
      if (!__builtin_amdgcn_ballot_w64(tp < tlim)) break;
    }
    BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[2] += tk - tp0; tp0 = tk;)
    if (odd) consume(pb, fb);  // drain in issue order: nothing stays in flight across the stores
    consume(pa, fa);
    consume(pb, fb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // a group no lane consumed may be in flight
    hfd::wave_sync();
    BPROF(tk = __builtin_readcyclecounter(); pc[3] += tk - tp0; tp0 = tk;)
    // symbols decoded past the block end move to its front; they are held in registers across
    // the reconstruction, which may use the tile as scratch
    uint32_t* rw = reinterpret_cast<uint32_t*>(dw.tile + lane * TP);
    uint32_t ovs[kF + 1];
#pragma unroll
    for (int i = 0; i <= kF; i++) ovs[i] = rw[BLK / 2 + i];
    recon(blk);
    hfd::wave_sync();
#pragma unroll
    for (int i = 0; i <= kF; i++) rw[i] = ovs[i];
    hfd::wave_sync();
    // next block's columns; a lane that stopped short of the block (a dead or short chunk)
    // restarts at column 0, where its (zero) target keeps it out of the quarters
    uint16_t* const row = dw.tile + lane * TP;
    tp = tp >= row + BLK ? tp - BLK : row;
    BPROF(tk = __builtin_readcyclecounter(); pc[4] += tk - tp0; tp0 = tk;)
  }
}

// Per block width: 64 columns (8 waves per CU, a 15 KB ring + tile per wave) or 32 columns (12
// waves per CU in 11 KB each: 3 waves per SIMD on the same LDS, recon_block32).  The step's chain
// of two LDS round trips bounds the loop, so a third wave per SIMD pays although a 512^3 field's
// 8192 bricks then make 2.67 rounds: f32 decompress 255 -> 229 us (config 2).  f64 keeps 64
// columns (at 32 its reconstruction spills 29-37 VGPRs).
#ifndef CUSZ_AMD_DEC3_BLK
#define CUSZ_AMD_DEC3_BLK 0  // 0: 32 for f32 fields of >= 12 bricks per CU, else 64
#endif
template <int BLK>
struct Dec3Cfg {
  static constexpr int TP = BLK + 10;  // 9 overshoot columns, odd dword pitch
  static constexpr size_t kCells = kD4Tile + (size_t)64 * TP * 2;
  static constexpr size_t kRows = kCells + (size_t)kCellCap * 4;
  static constexpr size_t kWaveBytes = kRows + (size_t)(65 + 64) * 4;
  static constexpr int kWaves = BLK == 64 ? kDec4Waves : 12;
  static_assert(((TP / 2) & 1) == 1 && BLK + 2 * kF + 1 <= TP, "tile pitch");
  static_assert(sizeof(hfd::Tab4) + kWaves * kWaveBytes <= 160 * 1024, "LDS");
};

template <typename T, bool ZZ, bool BUF, int BLK>
__global__ void __launch_bounds__(64 * Dec3Cfg<BLK>::kWaves)
k_brick3_decode(const uint32_t* __restrict__ bitstream, uint32_t bs_words, const uint8_t* __restrict__ revbook,
                int bklen, const uint32_t* __restrict__ par_nbit, const uint32_t* __restrict__ par_entry, T* out,
                uint32_t lx, uint32_t ly, uint32_t lz, T ebx2, T r, uint32_t nbx, uint32_t nby, uint32_t nbricks,
                BrickOutliers ol)
{
  __shared__ hfd::Tab4 tb;  // static: table addresses fold into the ds offsets
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  typedef Dec3Cfg<BLK> C;
  uint8_t* wbase = dsm + (size_t)wid * C::kWaveBytes;
  uint16_t* tile = reinterpret_cast<uint16_t*>(wbase + kD4Tile);
  uint32_t* cval = reinterpret_cast<uint32_t*>(wbase + C::kCells);
  BrickCells bc{cval, 1, reinterpret_cast<uint32_t*>(wbase + C::kRows), reinterpret_cast<uint32_t*>(wbase + C::kRows) + 65};
  const bool ranked = !ZZ && (ol.ncell == 0 || *ol.unsorted != ol.epoch);
  const DecWave4 dw{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bitstream), 0, (int)(bs_words * 4u), (int)kBufRsrcW3),
                    reinterpret_cast<uint32_t*>(wbase) + lane, tile, (uint32_t)bklen, lane};
  const size_t plane = (size_t)lx * ly;
  constexpr uint32_t W = 256;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const uint32_t ry = (uint32_t)lane >> 3, rz = (uint32_t)lane & 7u;

  BPROF(unsigned long long pc[16] = {}; unsigned long long tk = __builtin_readcyclecounter(), tp = tk;)
  // A brick's chunk sizes / offsets and cell range are loaded during the previous brick's last
  // block (they land while it decodes), so a brick starts with the bitstream loads only.
  // Its first bitstream words and first two outlier cells per lane are loaded at the start of
  // the previous brick's last reconstruction (they land under its stores).
  struct Next {
    uint32_t nbit, entry, cb, ce;
    bool live;
  };
  auto fetch = [&](uint32_t b) {
    Next x{0, 0, 0, 0, false};
    if (b >= nbricks) return x;
    const uint32_t bx = b % nbx, t = b / nbx, by = t % nby, bz = t / nby;
    x.live = by * 8 + ry < ly && bz * 8 + rz < lz;
    if (x.live) {
      const size_t c = ((size_t)(bz * 8 + rz) * ly + (by * 8 + ry)) * nbx + bx;
      x.nbit = par_nbit[c], x.entry = par_entry[c];
    }
    if (ranked && ol.ncell) x.cb = ol.bstart[b], x.ce = ol.bstart[b + 1];
    return x;
  };
  u32x4 first[2];
  uint2 pcell[2];  // cells cb + lane and cb + 64 + lane of the next brick: {value, index}
  auto prefetch = [&](const Next& x) {
    first[0] = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(x.live ? x.entry * 4u : kOOB), 0, 0);
    first[1] = __builtin_amdgcn_raw_buffer_load_b128(dw.rbits, (int)(x.live ? x.entry * 4u + 16u : kOOB), 0, 0);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint32_t j = x.cb + (uint32_t)lane + 64u * k;
      pcell[k] = ranked && j < x.ce ? make_uint2(ol.cells[2 * (size_t)j], ol.cells[2 * (size_t)j + 1]) : make_uint2(0, 0);
    }
  };
  // a wave's first brick: 8 consecutive bricks per workgroup (they share par_nbit / par_entry /
  // bitstream lines in one L2), unless the field has fewer bricks than waves (a small slab): then
  // wave w of every workgroup takes brick w * grid + block, spreading them over every CU (one per
  // SIMD for 1024 bricks) instead of filling half the CUs two waves per SIMD
  // (32-column blocks: always wave-major, so that the bricks' last, partial round is spread over
  // every CU instead of ending on the first 170)
  const uint32_t b0 = BLK == 32 || nbricks <= nw ? (uint32_t)wid * gridDim.x + blockIdx.x : blockIdx.x * (blockDim.x >> 6) + wid;
  Next nx = fetch(b0);  // (lands while the tables are built)
  hfd::build_tab4(tb, revbook, bklen);
  const hfd::DecRegs4 rg = hfd::load_dec_regs4(tb);
  prefetch(nx);
  for (uint32_t brick = b0; brick < nbricks; brick += nw) {
    BPROF(pc[0]++; tp = __builtin_readcyclecounter();)
    const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
    const uint32_t y0 = by * 8, z0 = bz * 8;
    const bool live = y0 + ry < ly && z0 + rz < lz;
    const Next cur = nx;
    const uint32_t nbit = live ? cur.nbit : 0u;
    const uint32_t vbase = (live ? cur.entry : 0u) * 4u;
    const u32x4 f2[2] = {first[0], first[1]};
    const uint2 cp[2] = {pcell[0], pcell[1]};
    // the brick's outlier cells [cb, ce): per-row counts -> row starts; values into LDS
    auto pro = [&]() {
      if (!ranked) return;
      const uint32_t cb = cur.cb, ce = cur.ce;
      const uint32_t nc = ce - cb;
      bc.row_start[lane] = 0;
      hfd::wave_sync();
      for (uint32_t j = (uint32_t)lane; j < nc; j += 64) {
        const uint2 cell = j < 64u    ? cp[0]
                           : j < 128u ? cp[1]
                                      : make_uint2(ol.cells[2 * (size_t)(cb + j)], ol.cells[2 * (size_t)(cb + j) + 1]);
        const uint32_t idx = cell.y;
        const uint32_t yz = idx / lx;  // y + ly z
        atomicAdd(&bc.row_start[((yz % ly) & 7u) * 8u + ((yz / ly) & 7u)], 1u);
        if (nc <= kCellCap) cval[j] = cell.x;
      }
      hfd::wave_sync();
      const uint32_t cr = bc.row_start[lane];
      const uint32_t incl = hfd::wave_incl_scan(cr);
      bc.row_start[lane] = incl - cr;
      if (lane == 63) bc.row_start[64] = incl;
      bc.carry[lane] = 0;
      bc.val = nc <= kCellCap ? cval : ol.cells + 2 * (size_t)cb;
      bc.vstride = nc <= kCellCap ? 1u : 2u;
    };
    auto recon = [&](int blk) {
      if (blk == (int)(W / BLK) - 1) prefetch(nx);  // the next brick (fetched during this block)
      const uint32_t nyv = min(8u, ly - y0), nzv = min(8u, lz - z0);
      const size_t base_elem = (size_t)z0 * plane + (size_t)y0 * lx + (size_t)bx * W + (size_t)blk * BLK;
      if constexpr (BLK == 64) {
        if (ranked)
          recon_block<T, ZZ, BUF, C::TP, true>(tile, out, plane, lx, nyv, nzv, base_elem, r, ebx2, lane, &bc);
        else
          recon_block<T, ZZ, BUF, C::TP, false>(tile, out, plane, lx, nyv, nzv, base_elem, r, ebx2, lane);
      }
      else {
        if (ranked)
          recon_block32<T, ZZ, BUF, C::TP, true>(tile, out, plane, lx, nyv, nzv, base_elem, r, ebx2, lane, &bc);
        else
          recon_block32<T, ZZ, BUF, C::TP, false>(tile, out, plane, lx, nyv, nzv, base_elem, r, ebx2, lane);
      }
    };
    auto blk_start = [&](int blk) {
      if (blk == (int)(W / BLK) - 1) nx = fetch(brick + nw);
    };
    decode_chunks4<BLK, C::TP>(tb, rg, dw, live, vbase, nbit, W, pro, blk_start, recon BPROF_A4, W, f2);
  }
#ifdef CUSZ_AMD_DEC_PROFILE
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_brick_prof[i], pc[i]);
#endif
}
// ---- 1-D: fused decode + reconstruct -------------------------------------------------------
// A wave owns a unit of 64 tiles of 1024 (4 chunks of 256 each); lane l owns tile 64 u + l and
// decodes its four chunks in four phases (phase p: chunk 4 t + p).  After each block of 64
// columns the lane reconstructs its own row -- 16 reference threads of 4 elements -- in
// registers, in the reference's 1-D order (lrz_x.cuhip.inl:11-78, wave32.cuhip.inl:7-66): per
// thread 4 sequential sums; Hillis-Steele over the 32 thread totals of each 128-element segment
// (a block is half a segment: the first half's raw totals stay in registers for the second
// half, which runs the 32-wide scan); a serial sum of the segment totals, carried per tile
// across the phases.  No cross-lane traffic; the lane stores its 256-B row piece.
//
// Outliers (archive cells in index order, k_x1d_bounds with chunk granularity): each lane
// prefetches the next kCellPf cell values of its chunk at a block's start (they land while the
// block decodes, and go to LDS for the reconstruction); zero codes take them by rank, ranks past
// the prefetch read the cell directly.
constexpr uint32_t kCellPf = 8;
constexpr uint32_t kCvPitch = kCellPf + 1;  // odd word pitch: lane rows on distinct banks
constexpr size_t kD1Cv = kD4Tile + (size_t)64 * kTP4 * 2;  // values[64][kCvPitch]
constexpr size_t kD1WaveBytes = kD1Cv + (size_t)64 * kCvPitch * 4;
constexpr int kD1MaxWaves = (int)((160 * 1024 - sizeof(hfd::Tab4) - 512) / kD1WaveBytes);
static_assert(kD1MaxWaves >= 4, "LDS");
static_assert(64 * 144 <= 64 * kTP4 * 2, "store staging fits the code tile");

template <typename T, bool ZZ>
__global__ void __launch_bounds__(64 * kDecWaves)
k_brick1_decode(const uint32_t* __restrict__ bitstream, uint32_t bs_words, const uint8_t* __restrict__ revbook,
                int bklen, const uint32_t* __restrict__ par_nbit, const uint32_t* __restrict__ par_entry, T* out,
                size_t n, T ebx2, T r, uint32_t nchunks, uint32_t nunits, BrickOutliers ol)
{
  __shared__ hfd::Tab4 tb;
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  hfd::build_tab4(tb, revbook, bklen);
  const hfd::DecRegs4 rg = hfd::load_dec_regs4(tb);
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* wbase = dsm + (size_t)wid * kD1WaveBytes;
  uint16_t* tile = reinterpret_cast<uint16_t*>(wbase + kD4Tile);
  uint32_t* cv = reinterpret_cast<uint32_t*>(wbase + kD1Cv) + lane * kCvPitch;  // this lane's values
  const bool ranked = !ZZ && (ol.ncell == 0 || *ol.unsorted != ol.epoch);  // else: values in `out` (scatter)
  const uint32_t npf = ol.ncell < (1u << 28) ? kCellPf : 0u;  // prefetched ranks (32-bit buffer offsets)
  const DecWave4 dw{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bitstream), 0, (int)(bs_words * 4u), (int)kBufRsrcW3),
                    reinterpret_cast<uint32_t*>(wbase) + lane, tile, (uint32_t)bklen, lane};
  const __amdgpu_buffer_rsrc_t rcells = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(ol.cells), 0, (int)min(ol.ncell * 8, (size_t)0x7FFFFFFF), (int)kBufRsrcW3);
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  BPROF(unsigned long long pc[16] = {}; unsigned long long tk = __builtin_readcyclecounter(), tp = tk;)
  // chunk size / offset and cell range of each phase's chunk, loaded during the previous phase's
  // last block (they land while it decodes)
  struct Next {
    uint32_t nbit, entry, cb, ce;
  };
  auto fetch = [&](uint32_t u, uint32_t p) {
    Next x{0, 0, 0, 0};
    const size_t c = ((size_t)u * 64u + (uint32_t)lane) * 4u + p;
    if (u < nunits && c < nchunks) {
      x.nbit = par_nbit[c], x.entry = par_entry[c];
      if (ranked && ol.ncell) x.cb = ol.bstart[c], x.ce = ol.bstart[c + 1];
    }
    return x;
  };
  Next nxt = fetch(blockIdx.x * (blockDim.x >> 6) + wid, 0);
  for (uint32_t u = blockIdx.x * (blockDim.x >> 6) + wid; u < nunits; u += nw) {
    T carry = T(0);  // serial sum of this tile's segment totals (exclusive)
    T fh[16];        // raw thread totals of the current segment's first half
    const size_t ubase = (size_t)u * 65536u;
    const bool full = ubase + 65536u <= n;  // every element of the unit is in the field (uniform)
    // unit-relative stores: 32-bit offsets; past the field's end they are dropped
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        out + ubase, 0, (int)(min((size_t)65536u, n - ubase) * sizeof(T)), (int)kBufRsrcW3);
    for (uint32_t p = 0; p < 4; p++) {
      BPROF(pc[0]++; tp = __builtin_readcyclecounter();)
      const size_t c = ((size_t)u * 64u + (uint32_t)lane) * 4u + p;
      const bool live = c < nchunks;
      const Next me = nxt;
      const uint32_t nbit = live ? me.nbit : 0u;
      const uint32_t vbase = (live ? me.entry : 0u) * 4u;
      const uint32_t vlen = live ? (uint32_t)min((size_t)256, n - c * 256u) : 0u;
      uint32_t cur = 0, cend = 0;  // this chunk's cells [cur, cend), cur advancing
      u32x4 pf[kCellPf / 2];
      auto pro = [&]() {
        if (ranked && live && ol.ncell) cur = me.cb, cend = me.ce;
      };
      auto blk_start = [&](int blk) {
        if (blk == (int)(256 / kBlk) - 1) nxt = p < 3 ? fetch(u, p + 1) : fetch(u + nw, 0);
        if (!ranked) return;
        // only pairs that start inside the chunk's cells: a chunk's cells are re-read by every
        // block, and a phase's blocks lie too far apart for the lines to stay in L2
#pragma unroll
        for (int h = 0; h < (int)kCellPf / 2; h++)
          pf[h] = __builtin_amdgcn_raw_buffer_load_b128(
              rcells, (int)(live && npf && cur + 2u * h < cend ? cur * 8u + 16u * h : kOOB), 0, 0);
      };
      auto recon = [&](int blk) {
        const uint32_t roff = ((uint32_t)lane * 1024u + p * 256u + (uint32_t)blk * kBlk) * (uint32_t)sizeof(T);
        const uint32_t* trow = reinterpret_cast<const uint32_t*>(tile + lane * kTP4);
        if (ranked) {  // the prefetched values; ranks at or past the chunk's last cell read 0
#pragma unroll
          for (int h = 0; h < (int)kCellPf / 2; h++) {
            cv[2 * h] = cur + 2u * h < cend ? pf[h].x : 0u;
            cv[2 * h + 1] = cur + 2u * h + 1u < cend ? pf[h].z : 0u;
          }
        }
        T v[64];
        uint32_t tw[32];  // the row's 64 codes, all read before use (one LDS wait)
#pragma unroll
        for (int q = 0; q < 32; q++) tw[q] = trow[q];
        uint32_t rk = 0;  // zero codes so far in this block
        // values of the codes: (o + c) - r, where a zero code's o is its cell by rank and any other
        // code's o is 0 -- one of the two is zero, so the sum is the other exactly and the value is
        // (z ? o : c) - r.  The rank's value is read for every code and selected bitwise, so no
        // code branches.
        // The value reads are issued 16 at a time (ranks first, then the reads, then the selects):
        // under the decode's LDS traffic their latency is long, and a wait per code would serialise.
        auto values = [&](auto rtag) {
          constexpr bool RK = decltype(rtag)::value;
#pragma unroll
          for (int s = 0; s < 4; s++) {
            uint32_t val[16];
            if constexpr (RK && !ZZ) {
              uint32_t rr = rk;
#pragma unroll
              for (int e = 0; e < 16; e++) {
                const uint32_t cd = (e & 1) ? tw[8 * s + e / 2] >> 16 : tw[8 * s + e / 2] & 0xFFFFu;
                val[e] = cv[rr];  // ranks past the prefetch: fixed below (reads stay in LDS)
                rr += cd == 0u ? 1u : 0u;
              }
            }
#pragma unroll
            for (int e = 0; e < 16; e++) {
              const int q = 8 * s + e / 2, h = e & 1;
              const uint32_t cd = h ? tw[q] >> 16 : tw[q] & 0xFFFFu;
              T x;
              if constexpr (ZZ)
                x = (T)zz_dec((uint16_t)cd);
              else if constexpr (RK) {
                const uint32_t zm = 0u - (uint32_t)(cd == 0u);  // all ones for a zero code
                const float cf = (float)cd;                      // exact (codes < 2^16)
                const uint32_t b = (val[e] & zm) | (__builtin_bit_cast(uint32_t, cf) & ~zm);
                x = (T)__builtin_bit_cast(float, b) - r;
                rk -= zm;  // + 1 for a zero code
              }
              else
                x = (T)cd - r;
              v[2 * q + h] = x;
            }
          }
        };
        if (ranked)
          values(std::true_type{});
        else
          values(std::false_type{});
        if (ranked && __builtin_amdgcn_ballot_w64(rk > npf)) {  // ranks past the prefetch (rare)
          uint32_t j = 0;
#pragma unroll
          for (int q = 0; q < 32; q++) {
            const uint32_t w = tw[q];
#pragma unroll
            for (int h = 0; h < 2; h++) {
              const bool z = (h ? w >> 16 : w & 0xFFFFu) == 0u;
              if (z && j >= npf)
                v[2 * q + h] = (cur + j < cend ? (T)__builtin_bit_cast(float, ol.cells[2 * (size_t)(cur + j)]) : T(0)) - r;
              j += z ? 1u : 0u;
            }
          }
        }
        if (ranked) cur += rk;
        BPROF(const unsigned long long tv = __builtin_readcyclecounter(); pc[8] += tv - tk;)
        if (!ranked) {  // values scattered into `out`: plane + zz_dec(0), or (plane + 0) - r
#pragma unroll
          for (int q = 0; q < 32; q++) {
            const uint32_t w = tw[q];
#pragma unroll
            for (int h = 0; h < 2; h++) {
              if ((h ? w >> 16 : w & 0xFFFFu) == 0u) {
                const uint32_t off = roff + (uint32_t)(2 * q + h) * (uint32_t)sizeof(T);
                T o;
                if constexpr (sizeof(T) == 4)
                  o = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(ro, (int)off, 0, 0));
                else
                  o = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(ro, (int)off, 0, 0));
                v[2 * q + h] = ZZ ? o + v[2 * q + h] : o - r;
              }
            }
          }
        }
        // per thread: 4 sequential elements (wave32.cuhip.inl:10); then the thread totals'
        // Hillis-Steele over the segment's 32 (wave32.cuhip.inl:14-17), descending in place (each
        // stage reads the previous stage's values): a[t] holds thread t's inclusive total and
        // thread t adds a[t - 1]; then the segment carry and the scale.  f32: the same IEEE
        // operations two at a time where the operands pair up (v_pk_add_f32 / v_pk_mul_f32).
        T tot = T(0);
        auto scan = [&](auto otag) {
          constexpr bool ODD = decltype(otag)::value;
          constexpr int t0 = ODD ? 16 : 0, nt = t0 + 16;  // this block's threads: t0 .. t0 + 15
          T a[32];
          if constexpr (sizeof(T) == 4) {
            typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int k = 1; k < 4; k++)
#pragma unroll
              for (int t = 0; t < 16; t += 2) {
                f2 x = {v[4 * t + k], v[4 * t + 4 + k]};
                x = x + f2{v[4 * t + k - 1], v[4 * t + 3 + k]};
                v[4 * t + k] = x.x, v[4 * t + 4 + k] = x.y;
              }
#pragma unroll
            for (int t = 0; t < 16; t++) {
              if constexpr (ODD) a[t] = fh[t];
              a[t0 + t] = v[4 * t + 3];
              if constexpr (!ODD) fh[t] = v[4 * t + 3];
            }
#pragma unroll
            for (int d = 1; d < 32; d *= 2) {
              if (d >= nt) break;
#pragma unroll
              for (int t = nt - 1; t >= d; t -= 2) {
                if (t - 1 >= d) {  // pair (t, t - 1): both sources still hold the previous stage
                  f2 x = {a[t], a[t - 1]};
                  x = x + f2{a[t - d], a[t - 1 - d]};
                  a[t] = x.x, a[t - 1] = x.y;
                }
                else
                  a[t] = a[t] + a[t - d];
              }
            }
          }
          else {
#pragma unroll
            for (int t = 0; t < 16; t++) {
              v[4 * t + 1] = v[4 * t + 1] + v[4 * t];
              v[4 * t + 2] = v[4 * t + 2] + v[4 * t + 1];
              v[4 * t + 3] = v[4 * t + 3] + v[4 * t + 2];
            }
#pragma unroll
            for (int t = 0; t < 16; t++) {
              if constexpr (ODD) a[t] = fh[t];
              a[t0 + t] = v[4 * t + 3];
              if constexpr (!ODD) fh[t] = v[4 * t + 3];
            }
#pragma unroll
            for (int d = 1; d < 32; d *= 2)
#pragma unroll
              for (int t = nt - 1; t >= d; t--) a[t] = a[t] + a[t - d];
          }
#pragma unroll
          for (int t = 0; t < 16; t++) {
            T o[4];
            if (t0 + t > 0) {
#pragma unroll
              for (int k = 0; k < 4; k++) v[4 * t + k] = v[4 * t + k] + a[t0 + t - 1];
            }
            if constexpr (sizeof(T) == 4) {
              typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
              for (int k = 0; k < 4; k += 2) {
                f2 x = {v[4 * t + k], v[4 * t + k + 1]};
                x = (x + f2{carry, carry}) * f2{ebx2, ebx2};
                o[k] = x.x, o[k + 1] = x.y;
              }
            }
            else {
#pragma unroll
              for (int k = 0; k < 4; k++) o[k] = (v[4 * t + k] + carry) * ebx2;
            }
            if (full) {
              // through the tile's space (the codes are in registers): RE elements of every row
              // per round (128 B), then each store instruction writes whole 128-B pieces of
              // 64 / (RE / 4) rows instead of 16-B pieces of 64 rows
              T* st = reinterpret_cast<T*>(tile);
              constexpr uint32_t RE = 128 / sizeof(T), RT = RE / 4, LPR = RE / 4;  // elements, threads, lanes per row
              constexpr uint32_t SP = RE + 16 / sizeof(T);  // row pitch (elements): 144 B
              lds_store4<T>(st + lane * SP + 4u * (t % RT), o);
              if (t % RT == RT - 1) {
#pragma unroll
                for (int m = 0; m < (int)(64 / (64 / LPR)); m++) {
                  const uint32_t row = (64u / LPR) * m + (uint32_t)lane / LPR, sub = (uint32_t)lane % LPR;
                  T w[4];
                  lds_load4<T>(st + row * SP + 4u * sub, w);
                  buf_store4<T>(w, ro, (row * 1024u + p * 256u + (uint32_t)blk * kBlk + RE * (t / RT) + 4u * sub) *
                                           (uint32_t)sizeof(T));
                }
              }
            }
            else {
              const uint32_t off = roff + (uint32_t)(4 * t) * (uint32_t)sizeof(T);
#pragma unroll
              for (int k = 0; k < 4; k++) buf_store<T>(o[k], ro, off + (uint32_t)k * (uint32_t)sizeof(T), 0);
            }
          }
          if constexpr (ODD) tot = v[63];  // the segment's total
        };
        if (blk & 1)
          scan(std::true_type{});
        else
          scan(std::false_type{});
        if (blk & 1) carry = carry + tot;
        BPROF(pc[9] += __builtin_readcyclecounter() - tv;)
      };
      decode_chunks4(tb, rg, dw, live, vbase, nbit, vlen, pro, blk_start, recon BPROF_A4, 256, nullptr);
    }
  }
#ifdef CUSZ_AMD_DEC_PROFILE
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_brick_prof[i], pc[i]);
#endif
}

// ---- decode only: any layout -> codes in index order ------------------------------------------
// The fused decoders' chunk loop with the tile copied out instead of reconstructed: wave u
// decodes chunks [64 u, 64 u + 64) (lane = chunk), and after each block of 64 columns stores the
// tile as codes (two rows of 128 B per store instruction).  Used for every archive (chunk length
// a multiple of 64) the fused decoders do not take: 2-D, spline, the reference layout, a
// standalone decode of the codes.
template <int DUMMY>
__global__ void __launch_bounds__(64 * kDecWaves)
k_chunk_decode(const uint32_t* __restrict__ bitstream, uint32_t bs_words, const uint8_t* __restrict__ revbook,
               int bklen, const uint32_t* __restrict__ par_nbit, const uint32_t* __restrict__ par_entry,
               uint16_t* __restrict__ codes, size_t n, uint32_t nchunks, uint32_t sublen, uint32_t wpb)
{
  __shared__ hfd::Tab4 tb;
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  BPROF(const unsigned long long tb0 = __builtin_readcyclecounter();)
  hfd::build_tab4(tb, revbook, bklen);
  const hfd::DecRegs4 rg = hfd::load_dec_regs4(tb);
  BPROF(const unsigned long long tb1 = __builtin_readcyclecounter();)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* wbase = dsm + (size_t)wid * kD4Cells;  // ring + tile (no cell staging)
  uint16_t* tile = reinterpret_cast<uint16_t*>(wbase + kD4Tile);
  const DecWave4 dw{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bitstream), 0, (int)(bs_words * 4u), (int)kBufRsrcW3),
                    reinterpret_cast<uint32_t*>(wbase) + lane, tile, (uint32_t)bklen, lane};
  // waves [wpb, 8) only help build the tables (launch_chunk_decode)
  const uint32_t nw = gridDim.x * wpb;
  const uint32_t nunits = (nchunks + 63) / 64;
  BPROF(unsigned long long pc[16] = {}; unsigned long long tk = __builtin_readcyclecounter(), tp = tk;)
  for (uint32_t u = blockIdx.x * wpb + wid; (uint32_t)wid < wpb && u < nunits; u += nw) {
    const size_t c = (size_t)u * 64u + (uint32_t)lane;
    const bool live = c < nchunks;
    const uint32_t nbit = live ? par_nbit[c] : 0u;
    const uint32_t vbase = (live ? par_entry[c] : 0u) * 4u;
    const uint32_t vlen = live ? (uint32_t)min((size_t)sublen, n - c * sublen) : 0u;
    auto recon = [&](int blk) {
      const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tile);
      const uint32_t cp = (uint32_t)lane & 31u;  // column pair
#pragma unroll 4
      for (uint32_t it = 0; it < 32; it++) {
        const uint32_t row = 2u * it + ((uint32_t)lane >> 5);
        const uint32_t w = t32[row * (kTP4 / 2) + cp];
        const size_t e = ((size_t)u * 64u + row) * sublen + (uint32_t)blk * kBlk + 2u * cp;
        if ((uint32_t)blk * kBlk + 2u * cp >= sublen) continue;  // (sublen is a multiple of kBlk)
        if (e + 1 < n)
          *reinterpret_cast<uint32_t*>(codes + e) = w;
        else if (e < n)
          codes[e] = (uint16_t)w;
      }
    };
    BPROF(pc[0]++;)
    decode_chunks4(tb, rg, dw, live, vbase, nbit, vlen, [] {}, [](int) {}, recon BPROF_A4, sublen, nullptr);
  }
#ifdef CUSZ_AMD_DEC_PROFILE
  pc[11] += tb1 - tb0;  // table build (per wave)
  pc[12] += __builtin_readcyclecounter() - tb0;  // whole wave
  pc[13] += 1;
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_brick_prof[i], pc[i]);
#endif
}


// =========================================================================================
// single-pass mode (PSZ_AMD_CODEBOOK_STREAM): sample -> host codebook -> one streaming pass
// =========================================================================================
// North-star pins the quant codes, the outliers and the reconstruction, not the bitstream, so
// the codebook may come from a sample and the field need be read only once:
//  * k_brick3_sample: the exact codes of a systematic 1/16 sample of 32 x 8 x 8 units (four 8^3
//    tiles: the units cycle through every x position and visit every (y, z) tile row), one unit
//    per wave step with all 8 z-rows in flight; its last workgroup hands the histogram to the
//    host (host-mapped), which builds the two-queue book of sample + 1 (every code encodable).
//  * k_brick3_stream: ONE WORKGROUP PER BRICK, wave y owning the brick's y-step y (rows (y, z),
//    z = 0..7): the wave predicts its 8 rows (z-diff and the x-diff inside the 8-wide tiles in
//    registers; the y-diff against wave y - 1's z/x residuals, exchanged through LDS), looks the
//    codewords up and sums each row's bits.  The workgroup's total is the brick's size: wave 0
//    publishes it for the decoupled look-back over the bricks before it while every wave packs
//    its rows into its own LDS area, and once the offset is known each wave writes its rows
//    straight to the archive.  Codes never touch HBM, nothing is staged per brick beyond a
//    y-step's cells, there is no plan pass and no gap between bricks.  Workgroup 0 takes the
//    host's book (a device-polled gate) while every workgroup predicts its first brick.
//  * k_brick3_stream_finish: outlier segment (the per-(brick, y-step) slots in brick order, then
//    the spill list), totals, both headers; the last workgroup publishes the compress summary.
// Deadlock-free: bricks are claimed in ticket order by resident workgroups, a workgroup claims
// its next brick only while working on an earlier one, and a look-back waits only on aggregates
// of smaller tickets -- the smallest unfinished brick always has every predecessor's.
constexpr uint32_t kSampleStride = 16;
constexpr unsigned long long kStAgg = 1ull << 62, kStInc = 2ull << 62;  // look-back status flags

// sample units of 32 x 8 x 8 elements; stride 16 from 4096 units up (>= 256 samples), else all
__host__ __device__ inline uint32_t sample_units(uint32_t lx, uint32_t ly, uint32_t lz)
{
  return (lx / 32u) * ((ly + 7u) / 8u) * ((lz + 7u) / 8u);
}
__host__ __device__ inline uint32_t sample_stride(uint32_t units) { return units >= 256u * kSampleStride ? kSampleStride : 1u; }

template <typename T>
__device__ __forceinline__ T shfl_up8(T v)
{
  if constexpr (sizeof(T) == 4)
    return __builtin_bit_cast(T, __shfl_up(__builtin_bit_cast(int, v), 8));
  else {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __shfl_up((int)(uint32_t)u, 8), hi = __shfl_up((int)(uint32_t)(u >> 32), 8);
    return __builtin_bit_cast(T, (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32));
  }
}

constexpr int kSampleThreads = 256;
template <typename T, bool ZZ>
__global__ void __launch_bounds__(kSampleThreads)
k_brick3_sample(const T* __restrict__ in, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2_r, T r,
                uint32_t* __restrict__ g_hist, int bklen, uint32_t* ticket, uint32_t* h_hist, uint32_t* flag,
                uint32_t epoch)
{
  __shared__ uint32_t s_h[kMaxBklen];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_h[i] = 0;
  __syncthreads();
  const uint32_t nux = lx / 32u, nuy = (ly + 7u) / 8u, units = sample_units(lx, ly, lz);
  const uint32_t stride = sample_stride(units), nsamp = (units + stride - 1) / stride;
  const size_t plane = (size_t)lx * ly;
  const uint32_t ly_l = (uint32_t)lane >> 3, xq = (uint32_t)lane & 7u;
  constexpr int kW = kSampleThreads / 64;
  for (uint32_t i = blockIdx.x * kW + wid; i < nsamp; i += gridDim.x * kW) {
    const uint32_t u = i * stride + i % stride;
    if (u >= units) continue;  // (uniform)
    const uint32_t ux = u % nux, t = u / nux, uy = t % nuy, uz = t / nuy;
    const uint32_t y = uy * 8u + ly_l, x0 = ux * 32u + xq * 4u, z0 = uz * 8u;
    T v[8][4];
#pragma unroll
    for (int z = 0; z < 8; z++) {
      const bool ok = y < ly && z0 + (uint32_t)z < lz;
      load_row<T, 4>(in, (size_t)(z0 + z) * plane + (size_t)y * lx, x0, lx, ok, v[z]);
    }
    // prequant, z-diff, x-diff inside the 8-wide tile (two lanes), y-diff across lanes (the
    // reference's order, lrz_c.cuhip.inl:341-352)
    T a[8][4], pp[4];
#pragma unroll
    for (int z = 0; z < 8; z++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const T p = dround(v[z][k] * ebx2_r);
        a[z][k] = z > 0 ? p - pp[k] : p;
        pp[k] = p;
      }
#pragma unroll
    for (int z = 0; z < 8; z++) {
      const T west = shr_in_tile<T, 1, 2>(a[z][3]);
#pragma unroll
      for (int k = 3; k > 0; k--) a[z][k] = a[z][k] - a[z][k - 1];
      if (lane & 1) a[z][0] = a[z][0] - west;
    }
#pragma unroll
    for (int z = 0; z < 8; z++) {
      const bool ok = y < ly && z0 + (uint32_t)z < lz;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const T north = shfl_up8(a[z][k]);
        const T d = lane >= 8 ? a[z][k] - north : a[z][k];
        bool ol;
        float ov;
        const uint16_t c = quantize<T, ZZ>(d, r, ol, ov);
        if (ok) atomicAdd(&s_h[c], 1u);
      }
    }
  }
  // bins one 64-B line apart (kSampleBinStride): the workgroups finish together, and their
  // atomics would queue on the few lines of a dense array
  __syncthreads();
  for (int i = threadIdx.x; i < bklen; i += blockDim.x)
    if (s_h[i]) atomicAdd(&g_hist[i * kSampleBinStride], s_h[i]);
  if (!last_block(ticket)) return;  // the last workgroup: the sample histogram -> the host, flag raised
  for (int i = threadIdx.x; i < bklen; i += blockDim.x)
    h_hist[i] = __hip_atomic_load(g_hist + i * kSampleBinStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned long long st_word(unsigned long long flag, uint32_t cells, uint32_t oc)
{
  return flag | (unsigned long long)cells | ((unsigned long long)oc << 32);
}

// Exclusive prefix (cells, slot outliers) of `brick` from its predecessors' status words: 256 per
// step (4 per lane, distance 4 lane + q), back to the nearest one holding an inclusive prefix.
// Bounded spins: a word still empty after them counts as 0 and raises *timeout (never expected).
__device__ __forceinline__ void lookback(const unsigned long long* status, uint32_t brick, int lane, uint32_t& xc,
                                         uint32_t& xo, unsigned int* timeout)
{
  uint32_t sc = 0, so = 0;
  for (int64_t j = (int64_t)brick - 1;; j -= 256) {
    unsigned long long v[4];
    uint32_t qinc = 4;  // this lane's nearest inclusive word (4: none)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int64_t me = j - 4 * lane - q;
      v[q] = kStInc;  // before brick 0: an inclusive prefix of 0
      if (me >= 0) {
        uint32_t spins = 0;
        do
          v[q] = __hip_atomic_load(status + me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((v[q] >> 62) == 0 && ++spins < (1u << 22));
        if ((v[q] >> 62) == 0) atomicOr(timeout, 1u);
      }
    }
#pragma unroll
    for (int q = 3; q >= 0; q--)
      if ((v[q] >> 62) == 2) qinc = (uint32_t)q;
    const uint64_t inc = __builtin_amdgcn_ballot_w64(qinc < 4);
    const int k = inc ? __builtin_ctzll(inc) : 64;  // the lane holding the nearest inclusive word
    uint32_t c = 0, o = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool take = lane < k || (lane == k && (uint32_t)q <= qinc);
      c += take ? (uint32_t)v[q] : 0u;
      o += take ? (uint32_t)(v[q] >> 32) & 0x3FFFFFFFu : 0u;
    }
    sc += readlane(hfd::wave_incl_scan(c), 63);
    so += readlane(hfd::wave_incl_scan(o), 63);
    if (inc) break;
  }
  xc = sc, xo = so;
}

struct StreamArgs {
  uint32_t lx, ly, lz, nbx, nby, nbricks;
  OutlierSink ol;              // one slot per (brick, y-step): slot 8 brick + y, cap_per_brick = its cap
  uint32_t* book;              // device book: written by workgroup 0 from the host's
  int bklen;
  uint32_t* par_nbit;
  uint32_t* par_entry;
  uint32_t* bitstream;
  uint32_t bs_cap;             // bitstream capacity (cells)
  unsigned long long* status;  // per brick, zeroed per call
  uint32_t* ticket;            // zeroed per call
  uint32_t* ol_dst;            // per slot: its first cell in the archive's outlier segment
  CompressInfo* info;
  unsigned int* timeout;
  // the codebook gate: the host writes the book and reverse book to host-mapped memory and sets
  // *gate = gate_epoch; workgroup 0 copies them to `book` and the archive, then sets *book_flag
  const uint32_t* gate;
  uint32_t gate_epoch;
  const uint32_t* h_book;
  const uint32_t* h_revbook;
  uint32_t* revbook;  // the archive's reverse book
  int rv_words;
  uint32_t* book_flag;  // device word, never reset (epoch-compared)
};

constexpr int kStreamWaves = 8;  // one wave per y-step of the brick
#ifndef CUSZ_AMD_STREAM_PF_LATE
#define CUSZ_AMD_STREAM_PF_LATE 0  // 1: the next brick's rows are issued after barrier B, not A
#endif
// LDS per workgroup: waves 0..6 hand their y-step's z/x residuals to the next wave (the y-diff)
// through an exchange area; every wave stages its y-step's packed cells in a staging area until
// the brick's offset is known (one brick later: the look-back is deferred)
template <typename T>
constexpr int kStreamXsWords = 8 * 64 * 4 * (int)sizeof(T) / 4;
constexpr int kStageW = 512;  // staging words per wave
static_assert(kStageW >= 2 * kPackRowMax + 2, "the flush path holds two rows");
template <typename T>
constexpr size_t stream_lds_bytes()
{
  return ((size_t)(kStreamWaves - 1) * kStreamXsWords<T> + (size_t)kStreamWaves * kStageW) * 4;
}
constexpr uint32_t kNoBrick = 0xFFFFFFFFu;

// Single-pass encoder, one workgroup per brick, wave y = the brick's y-step y.  Per brick:
//   phase 1   prequant, z-diff, x-diff of the wave's 8 rows (loaded one brick ahead), residuals
//             -> the exchange area; (A) the next brick's rows are issued, y-diff from the area
//   phase 2   codes, outliers (the y-step's slot), row bits (LDS book), row scans; (B) sizes
//   wave 0    publishes the brick's aggregate, then looks back for the PREVIOUS brick (its
//             predecessors published a brick ago: the walk rarely waits) and publishes its
//             inclusive prefix; (C)
//   all       copy the previous brick's staged cells out, then pack this brick's into staging.
// A brick with a y-step too large for the staging (noisy fields) takes its own offset at once
// and packs through the staging area with flushes.
template <typename T, bool ZZ>
__global__ void __launch_bounds__(64 * kStreamWaves)
__attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 4 : 2)))  // f32: 2 workgroups per CU (LDS, 128 VGPRs)
k_brick3_stream(const T* __restrict__ in, StreamArgs a, T ebx2_r, T r)
{
  constexpr int V = 4;
  constexpr int XW = kStreamXsWords<T>;
  extern __shared__ uint32_t smem[];  // exchange areas (waves 0..6), then staging areas
  __shared__ uint32_t s_book[kMaxBklen];
  __shared__ uint32_t s_wc[kStreamWaves], s_wo[kStreamWaves];
  __shared__ uint32_t s_next[2], s_x[4];
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  T* const xsT = reinterpret_cast<T*>(smem + (wid < kStreamWaves - 1 ? wid : 0) * XW);
  const T* const xprev = reinterpret_cast<const T*>(smem + (wid > 0 ? wid - 1 : 0) * XW);
  uint32_t* const stg = smem + (kStreamWaves - 1) * XW + wid * kStageW;
  const StepLoader<T, V> ld{in, (size_t)a.lx * a.ly, a.lx, a.ly, a.lz, a.nbx, a.nby, a.nbricks, 0, (uint32_t)lane};
  const uint32_t subcap = a.ol.cap_per_brick;

  // workgroup 0, wave 0: the host's codebook -> device memory and the archive, then the flag
  if (blockIdx.x == 0 && wid == 0) {
    uint32_t ok = 1;
    if (lane == 0) {
      for (uint32_t spin = 0;; spin++) {
        const uint32_t v = __hip_atomic_load(a.gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int32_t)(v - a.gate_epoch) >= 0) break;
        if (spin > (1u << 22)) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    ok = (uint32_t)__builtin_amdgcn_readfirstlane((int)ok);
    if (!ok && lane == 0) atomicOr(a.timeout, 2u);
    for (int i = lane; i < a.bklen; i += 64) a.book[i] = a.h_book[i];
    for (int i = lane; i < a.rv_words; i += 64) a.revbook[i] = a.h_revbook[i];
    __builtin_amdgcn_s_waitcnt(0);
    hfd::wave_sync();
    if (lane == 0) __hip_atomic_store(a.book_flag, a.gate_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }

  if (threadIdx.x == 0) s_next[0] = atomicAdd(a.ticket, 1u);
  __syncthreads();
  uint32_t brick = s_next[0];
  T q[8][V];  // this wave's rows of the brick (loaded one brick ahead)
#pragma unroll
  for (int z = 0; z < 8; z++) ld.issue_row(brick, 8 * wid + z, q[z]);
  bool have_book = false;
  unsigned long long wbits = 0;  // bits this wave packed (the header's total)
  uint32_t par = 0;
  // the deferred brick (uniform): its index, totals, this wave's cells / slot outliers before it
  // and its own; lane z: its row z's bits and first cell
  uint32_t dbrick = kNoBrick, d_ct = 0, d_ot = 0, d_cb = 0, d_ob = 0, d_cells = 0, d_cnt = 0;
  uint32_t d_nbit = 0, d_loc = 0;
  // diagnostic build: per-phase clocks summed over waves (0 wave-bricks, 1 phase 1 incl. the
  // loads' wait, 2 barrier A + y-diff + book, 3 phase 2, 4 barrier B, 5 look-back (wave 0),
  // 6 barrier C, 7 copy-out of the deferred brick, 8 pack)
  BPROF(unsigned long long pc[16] = {}; unsigned long long tk = 0, tp = __builtin_readcyclecounter();)
#define SPROF(i) BPROF(hfd::wave_sync(); tk = __builtin_readcyclecounter(); pc[i] += tk - tp; tp = tk;)
  for (;;) {
    const bool live = brick < a.nbricks;  // (uniform over the workgroup)
    if (!live && dbrick == kNoBrick) break;
    BPROF(pc[0] += live;)
    const uint32_t bx = brick % a.nbx, t = brick / a.nbx, by = t % a.nby, bz = t / a.nby;
    const uint32_t x0 = bx * (64 * V) + lane * V, z0 = bz * 8, gy = by * 8 + (uint32_t)wid;
    const bool yok = live && gy < a.ly;  // (uniform per wave)
    const uint32_t nzv = live ? min(8u, a.lz - z0) : 0u;
    const uint32_t slot = brick * kStreamWaves + (uint32_t)wid;
    uint32_t cnt = 0, cells = 0;
    uint32_t cp[8][2], inc[8];  // codes as u16 pairs, row scans of the bits (lane 63: the row's bits)
    bool wide = false;                  // a lane's four codewords of some row exceed 64 bits
    uint32_t bnext = kNoBrick;
    if (live) {
      // phase 1: prequant, z-diff, x-diff inside the 8-wide tile (lrz_c.cuhip.inl:341-352 order)
      T av[8][V];
      {
        T pprev[V];
#pragma unroll
        for (int z = 0; z < 8; z++) {
#pragma unroll
          for (int k = 0; k < V; k++) {
            const T p = dround(q[z][k] * ebx2_r);
            av[z][k] = z > 0 ? p - pprev[k] : p;
            pprev[k] = p;
          }
          const T west = shr_in_tile<T, 1, 8 / V>(av[z][V - 1]);
#pragma unroll
          for (int k = V - 1; k > 0; k--) av[z][k] = av[z][k] - av[z][k - 1];
          if (x0 % 8 != 0) av[z][0] = av[z][0] - west;
        }
      }
      if (wid < kStreamWaves - 1)
#pragma unroll
        for (int z = 0; z < 8; z++) lds_store4(xsT + ((size_t)z * 64 + lane) * V, av[z]);
      if (threadIdx.x == 0) s_next[par ^ 1] = atomicAdd(a.ticket, 1u);
      SPROF(1)
      __syncthreads();  // (A) residuals exchanged, next brick known
      bnext = s_next[par ^ 1];
      par ^= 1;
#if !CUSZ_AMD_STREAM_PF_LATE
#pragma unroll
      for (int z = 0; z < 8; z++) ld.issue_row(bnext, 8 * wid + z, q[z]);
#endif
      if (!have_book) {  // first brick: the codebook (workgroup 0 raises the flag)
        if (threadIdx.x == 0) {
          for (uint32_t spin = 0;; spin++) {
            const uint32_t v = __hip_atomic_load(a.book_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (v == a.gate_epoch) break;
            if (spin > (1u << 22)) {
              atomicOr(a.timeout, 2u);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < a.bklen; i += 64 * kStreamWaves)
          s_book[i] = __hip_atomic_load(a.book + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        have_book = true;
      }
      SPROF(2)
      // phase 2: y-diff against the previous y-step (the brick's first y-step has none), codes
      // (kept as u16 pairs), outliers (into this y-step's slot), row bits
#pragma unroll
      for (int z = 0; z < 8; z++) {
        const bool rok = yok && (uint32_t)z < nzv;
        if (wid > 0) {
          T bp[V];
          lds_load4(xprev + ((size_t)z * 64 + lane) * V, bp);
#pragma unroll
          for (int k = 0; k < V; k++) av[z][k] = av[z][k] - bp[k];
        }
        uint16_t c[V];
        float olv[V];
        uint32_t mask = 0;
#pragma unroll
        for (int k = 0; k < V; k++) {
          bool is_ol;
          c[k] = quantize<T, ZZ>(av[z][k], r, is_ol, olv[k]);
          mask |= (uint32_t)(is_ol && rok) << k;
        }
        if (__builtin_amdgcn_ballot_w64(mask != 0)) {  // (rare; the field has < 2^32 elements)
          const uint32_t base = (uint32_t)((z0 + z) * ld.plane + (size_t)gy * a.lx) + x0;
          emit_outliers32<V>(a.ol, slot, cnt, mask, olv, base);
        }
        uint32_t bits = 0;  // (rows outside the field: no codewords)
#pragma unroll
        for (int k = 0; k < V; k++) bits += rok ? s_book[c[k]] >> 27 : 0u;
        cp[z][0] = (uint32_t)c[0] | (uint32_t)c[1] << 16;
        cp[z][1] = (uint32_t)c[2] | (uint32_t)c[3] << 16;
        wide |= bits > 64u;
        inc[z] = hfd::wave_incl_scan(bits);
        cells += (readlane(inc[z], 63) + 31) >> 5;
      }
      if (lane == 0) s_wc[wid] = cells, s_wo[wid] = min(cnt, subcap);
      SPROF(3)
    }
    __syncthreads();  // (B) every y-step's size; the exchange areas are free
#if CUSZ_AMD_STREAM_PF_LATE
    if (live)
#pragma unroll
      for (int z = 0; z < 8; z++) ld.issue_row(bnext, 8 * wid + z, q[z]);
#endif
    SPROF(4)
    uint32_t cb = 0, ob = 0, ct = 0, ot = 0, cmax = 0;  // before this wave, brick totals, largest y-step
    if (live) {
#pragma unroll
      for (int v = 0; v < kStreamWaves; v++) {
        const uint32_t c = s_wc[v], o = s_wo[v];
        if (v < wid) cb += c, ob += o;
        ct += c, ot += o;
        cmax = max(cmax, c);
      }
    }
    const bool direct = live && cmax + 2 > (uint32_t)kStageW;  // (uniform) too large to stage: offsets now
    if (wid == 0) {
      if (live && lane == 0)  // the brick's aggregate (brick 0: its inclusive prefix)
        __hip_atomic_store(a.status + brick, st_word(brick == 0 ? kStInc : kStAgg, ct, ot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (dbrick != kNoBrick) {  // the deferred brick's offsets
        uint32_t xc = 0, xo = 0;
        if (dbrick != 0) {
          lookback(a.status, dbrick, lane, xc, xo, a.timeout);
          if (lane == 0)
            __hip_atomic_store(a.status + dbrick, st_word(kStInc, xc + d_ct, xo + d_ot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_x[0] = xc, s_x[1] = xo;
      }
      if (direct) {  // this brick's offsets at once
        uint32_t xc = 0, xo = 0;
        if (brick != 0) {
          lookback(a.status, brick, lane, xc, xo, a.timeout);
          if (lane == 0)
            __hip_atomic_store(a.status + brick, st_word(kStInc, xc + ct, xo + ot), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_x[2] = xc, s_x[3] = xo;
      }
    }
    SPROF(5)
    __syncthreads();  // (C) the offsets
    SPROF(6)
    // cells -> the archive, with the brick's chunk tables and slot destination
    auto emit = [&](uint32_t b, uint32_t woff, uint32_t oo, uint32_t ncells, uint32_t nbit, uint32_t loc,
                    uint32_t scnt) {
      const uint32_t bxx = b % a.nbx, tt = b / a.nbx, byy = tt % a.nby, bzz = tt / a.nby;
      const uint32_t gyy = byy * 8 + (uint32_t)wid, nz = min(8u, a.lz - bzz * 8);
      if (woff + ncells <= a.bs_cap) {
        for (uint32_t i = (uint32_t)lane; i < ncells; i += 64) a.bitstream[woff + i] = stg[i];
      }
      else if (lane == 0)
        atomicOr(a.timeout, 4u);
      if (lane < 8 && gyy < a.ly && (uint32_t)lane < nz) {
        const size_t c = ((size_t)(bzz * 8 + (uint32_t)lane) * a.ly + gyy) * a.nbx + bxx;
        a.par_nbit[c] = nbit;
        a.par_entry[c] = woff + loc;
      }
      if (lane == 0) {
        const uint32_t s = b * kStreamWaves + (uint32_t)wid;
        a.ol.brick_cnt[s] = scnt;
        a.ol_dst[s] = oo;
        if (scnt > subcap) atomicMax(&a.info->max_brick_cnt, scnt * kStreamWaves);  // slot growth
      }
    };
    if (dbrick != kNoBrick) {
      hfd::wave_sync();
      emit(dbrick, s_x[0] + d_cb, s_x[1] + d_ob, d_cells, d_nbit, d_loc, d_cnt);
      dbrick = kNoBrick;
    }
    SPROF(7)
    if (live) {
      // pack the y-step's rows into the staging area (zeroed first; two words of slack); the
      // codewords are looked up again (fewer registers live across the barriers than holding them)
      const bool any_wide = __builtin_amdgcn_ballot_w64(wide) != 0;
      uint32_t off = 0, fbase = 0, my_nbit = 0, my_loc = 0;  // lane z: row z's bits and first cell
      const uint32_t woff = direct ? s_x[2] + cb : 0u;
      auto flush = [&]() {  // (direct) staged words [fbase, off) -> the archive, staging cleared
        hfd::wave_sync();
        const uint32_t m = off - fbase;
        const bool fits = woff + off <= a.bs_cap;
        if (!fits && lane == 0) atomicOr(a.timeout, 4u);
        for (uint32_t i = (uint32_t)lane; i < m; i += 64) {
          const uint32_t v = stg[i];
          stg[i] = 0u;
          if (fits) a.bitstream[woff + fbase + i] = v;
        }
        fbase = off;
        hfd::wave_sync();
      };
      for (uint32_t i = (uint32_t)lane; i < (direct ? (uint32_t)kStageW : cells + 2); i += 64) stg[i] = 0u;
#pragma unroll
      for (int z = 0; z < 8; z++) {
        if (direct && off - fbase + kPackRowMax > (uint32_t)kStageW) flush();
        uint32_t w[V];
        w[0] = s_book[cp[z][0] & 0xFFFFu], w[1] = s_book[cp[z][0] >> 16];
        w[2] = s_book[cp[z][1] & 0xFFFFu], w[3] = s_book[cp[z][1] >> 16];
        if (!(yok && (uint32_t)z < nzv)) w[0] = w[1] = w[2] = w[3] = 0u;  // a row outside the field (uniform)
        const uint32_t bits = (w[0] >> 27) + (w[1] >> 27) + (w[2] >> 27) + (w[3] >> 27);
        const uint32_t pos = ((off - fbase) << 5) + inc[z] - bits;
        if (!any_wide)
          hfd::pack4_or_lj(stg, pos, w, bits);
        else
          hfd::pack_words<V>(stg, pos, w, V);
        const uint32_t tot = readlane(inc[z], 63);
        if (lane == z) my_nbit = tot, my_loc = off;
        off += (tot + 31) >> 5;
        wbits += tot;
      }
      if (direct) {
        flush();
        emit(brick, woff, s_x[3] + ob, 0u, my_nbit, my_loc, cnt);  // (the cells are out)
      }
      else {
        dbrick = brick, d_ct = ct, d_ot = ot, d_cb = cb, d_ob = ob, d_cells = cells, d_cnt = cnt;
        d_nbit = my_nbit, d_loc = my_loc;
      }
      brick = bnext;
    }
    SPROF(8)
  }
#undef SPROF
  if (lane == 0 && wbits) atomicAdd(&a.info->total_nbit, wbits);
#ifdef CUSZ_AMD_DEC_PROFILE
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&g_brick_prof[i], pc[i]);
#endif
}

// after the streaming pass: the outlier segment (the slots in (brick, y-step) order -- brick
// order, row order inside a brick -- then the spill list), the totals and both headers; the last
// workgroup publishes the compress summary.  Each wave copies 64 consecutive slots: their
// destinations are one contiguous range, a cell finds its slot by a binary search over the
// slots' prefix counts.
constexpr int kFinishThreads = 256;
__global__ void __launch_bounds__(kFinishThreads) k_brick3_stream_finish(StreamArgs a, HeaderTpl tpl, uint8_t* archive,
                                                                         size_t phf_offset, size_t bits_rel, HostPub pub)
{
  __shared__ uint32_t s_ex[kFinishThreads / 64][65];
  const unsigned long long last =
      __hip_atomic_load(a.status + a.nbricks - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t ncell = (uint32_t)last, slot_total = (uint32_t)(last >> 32) & 0x3FFFFFFFu;
  uint2* ol_dst = reinterpret_cast<uint2*>(a.bitstream + ncell);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* ex = s_ex[wid];
  const uint32_t nslot = a.nbricks * kStreamWaves, cap = a.ol.cap_per_brick;
  const uint32_t nwv = gridDim.x * (kFinishThreads / 64);
  for (uint32_t g = blockIdx.x * (kFinishThreads / 64) + wid; g * 64 < nslot; g += nwv) {
    const uint32_t s = g * 64 + (uint32_t)lane;
    const uint32_t c = s < nslot ? min(a.ol.brick_cnt[s], cap) : 0u;
    const uint32_t d = s < nslot ? a.ol_dst[s] : 0u;
    const uint32_t incl = hfd::wave_incl_scan(c), total = readlane(incl, 63), d0 = readlane(d, 0);
    ex[lane] = incl - c;
    hfd::wave_sync();
    for (uint32_t j = (uint32_t)lane; j < total; j += 64) {
      uint32_t lo = 0;  // the last slot whose first cell is <= j
#pragma unroll
      for (uint32_t step = 32; step > 0; step >>= 1)
        if (lo + step < 64 && ex[lo + step] <= j) lo += step;
      const uint64_t cell = a.ol.slots[(size_t)(g * 64 + lo) * cap + (j - ex[lo])];
      ol_dst[d0 + j] = make_uint2((uint32_t)cell, (uint32_t)(cell >> 32));
    }
    hfd::wave_sync();
  }
  const uint32_t sp = *a.ol.spill_cnt, sp_kept = min(sp, a.ol.spill_cap);
  for (uint32_t i = blockIdx.x * kFinishThreads + threadIdx.x; i < sp_kept; i += gridDim.x * kFinishThreads) {
    const uint64_t c = a.ol.spill[i];
    ol_dst[slot_total + i] = make_uint2((uint32_t)c, (uint32_t)(c >> 32));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long nbit = __hip_atomic_load(&a.info->total_nbit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.info->total_ncell = ncell;
    a.info->splen = slot_total + sp_kept;
    a.info->outlier_lost = sp > a.ol.spill_cap ? sp - a.ol.spill_cap : 0u;
    a.info->spilled = sp;
    write_headers_dev(archive, tpl, nbit, ncell, slot_total + sp_kept, phf_offset, bits_rel);
    __threadfence();  // the header and totals reach memory before the ticket (the publisher may be another XCD)
  }
  publish_last(pub);
}

}  // namespace

BrickSample brick_sample_plan(uint32_t nbricks, uint32_t* hist, uint32_t* done)
{
  BrickSample s;
  s.hist = hist, s.done = done;
  // stride - 1 a power of two (the order's arithmetic); ~256 sample bricks where possible (a
  // 512^3 field: every 33rd brick, 4 M codes -- the book's bits +0.001 % against every 17th, and
  // pass 1 adds half the sample atomics: -6 us)
  s.stride = nbricks >= 8192 ? 33u : nbricks >= 4352 ? 17u : nbricks >= 2304 ? 9u : nbricks >= 1280 ? 5u : nbricks >= 768 ? 3u : 1u;
  const uint32_t o = s.stride / 2;
  s.count = s.stride == 1 ? nbricks : (nbricks > o ? (nbricks - o + s.stride - 1) / s.stride : 0u);
  return s;
}

// =========================================================================================
// host launchers
// =========================================================================================

BrickGeom brick_geom(int ndim, size_t lx, size_t ly, size_t lz, int elem_bytes)
{
  BrickGeom g{};
  g.V = 4;  // W = 256: f32 16-B loads, f64 32-B loads per lane
  g.W = 64 * g.V;
  g.ndim = ndim;
  g.n = lx * ly * lz;
  if (ndim == 1 || ndim == 2) {  // linear bricks (2-D: x extent a multiple of 4, >= 256; < 2 GiB)
    g.ok = g.n < (1ull << 32) && (elem_bytes == 4 || elem_bytes == 8) &&
           (ndim == 1 || (lx % 4 == 0 && lx >= (size_t)g.W && g.n * elem_bytes < (1ull << 31)));
    if (!g.ok) return g;
    g.brick_elems = (uint32_t)g.W * 64;
    g.nbricks = (uint32_t)((g.n + g.brick_elems - 1) / g.brick_elems);
    g.nbx = g.nbricks, g.nby = 1, g.nbz = 1;
    g.nchunks = (uint32_t)((g.n + g.W - 1) / g.W);
    return g;
  }
  g.ok = ndim == 3 && lx % (size_t)g.W == 0 && lx * ly * lz < (1ull << 32) && (elem_bytes == 4 || elem_bytes == 8) &&
         8 * lx * ly * (size_t)elem_bytes < (1ull << 31);  // 32-bit buffer offsets within 8 planes
  if (!g.ok) return g;
  g.nbx = (uint32_t)(lx / g.W);
  g.nby = (uint32_t)((ly + 7) / 8);
  g.nbz = (uint32_t)((lz + 7) / 8);
  g.nbricks = g.nbx * g.nby * g.nbz;
  g.brick_elems = (uint32_t)g.W * 64;
  g.nchunks = (uint32_t)(lx / g.W * ly * lz);
  return g;
}

int brick_configure(BrickLaunch& L, int elem_bytes, int device)
{
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
  L.ncu = ncu;
  int per_scan = 0, per_pack = 0;
  const size_t lds_scan = (size_t)(1 + kBrickWaves * kHistCopies) * kMaxBklen * 4;
  const size_t lds_pack = 0;  // static LDS only
  hipError_t e1, e2;
  if (elem_bytes == 8) {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_scan, k_brick3_scan<double, 4, false>, 64 * kBrickWaves, lds_scan);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pack, k_brick3_pack<4, 3>, 64 * kBrickWaves, lds_pack);
  }
  else {
    e1 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_scan, k_brick3_scan<float, 4, false>, 64 * kBrickWaves, lds_scan);
    e2 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pack, k_brick3_pack<4, 3>, 64 * kBrickWaves, lds_pack);
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
int launch_brick_scan(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const BrickSample& sample,
                      const OutlierSink& ol, uint32_t* hist, uint16_t* bhist, const BrickCodes& bcodes, int bklen,
                      hipStream_t st, const HostPub& pub)
{
  const T ebx2_r = (T)(1.0 / (eb * 2));  // lrz_c.cuhip.inl:489
  const T r = (T)radius;
  const BrickGeom& g = L.g;
  const size_t lds = (size_t)(1 + kBrickWaves * kHistCopies) * kMaxBklen * 4;
  const int grid = L.grid_scan;
  if (g.ndim == 1 || g.ndim == 2) {
#define SCAN1(ZZ, ND)                                                                                           \
  k_brick1_scan<T, 4, ZZ, ND><<<grid, 64 * kBrickWaves, lds, st>>>(in, g.n, ebx2_r, r, ol, hist, bhist, bcodes, \
                                                                   bklen, g.nbricks, pub, L.lx, sample)
    if (g.ndim == 1) {
      if (zz) SCAN1(true, 1); else SCAN1(false, 1);
    }
    else {
      if (zz) SCAN1(true, 2); else SCAN1(false, 2);
    }
#undef SCAN1
    return (int)hipGetLastError();
  }
  if (zz)
    k_brick3_scan<T, 4, true><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, ol, hist, bhist,
                                                                   bcodes, bklen, g.nbx, g.nby, g.nbricks, pub, sample);
  else
    k_brick3_scan<T, 4, false><<<grid, 64 * kBrickWaves, lds, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, ol, hist, bhist,
                                                                    bcodes, bklen, g.nbx, g.nby, g.nbricks, pub, sample);
  return (int)hipGetLastError();
}

int launch_brick_plan(const BrickLaunch& L, const BrickPlanArgs& a, const void* psz_tpl, const void* phf_tpl,
                      hipStream_t st)
{
  HeaderTpl t;
  __builtin_memcpy(t.psz, psz_tpl, 176);
  __builtin_memcpy(t.phf, phf_tpl, 64);
  k_brick_plan<<<a.nblk, kPlanThreads, 0, st>>>(a, t);
  return (int)hipGetLastError();
}

uint32_t brick_units(uint32_t nbricks) { return (nbricks + kUnitBricks - 1) / kUnitBricks; }
uint32_t brick_plan_blocks(uint32_t nbricks) { return (brick_units(nbricks) + kPlanBricks - 1) / kPlanBricks; }
int brick_hist_stride(int bklen) { return bhist_stride(bklen); }

int launch_brick_pack(const BrickLaunch& L, const BrickCodes& bcodes, const uint32_t* book, int bklen,
                      const BrickPlanArgs& plan, uint32_t* par_nbit, uint32_t* par_entry, uint32_t* bitstream,
                      int reverse, unsigned int* overflow, hipStream_t st, const HostPub& pub)
{
  const BrickGeom& g = L.g;
  const size_t lds = 0;  // static LDS only
  if (g.ndim != 3)
    k_brick3_pack<4, 1><<<L.grid_pack, 64 * kBrickWaves, lds, st>>>(bcodes, L.ly, L.lz, book, bklen, plan, par_nbit,
                                                                    par_entry, bitstream, g.nbx, g.nby, g.nbricks,
                                                                    reverse, overflow, pub);
  else
    k_brick3_pack<4, 3><<<L.grid_pack, 64 * kBrickWaves, lds, st>>>(bcodes, L.ly, L.lz, book, bklen, plan, par_nbit,
                                                                    par_entry, bitstream, g.nbx, g.nby, g.nbricks,
                                                                    reverse, overflow, pub);
  return (int)hipGetLastError();
}

template <typename T>
int launch_brick_sample(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, uint32_t* hist, int bklen,
                        uint32_t* ticket, uint32_t* h_hist, uint32_t* flag, uint32_t epoch, hipStream_t st)
{
  const BrickGeom& g = L.g;
  if (g.ndim != 3 || bklen > kMaxBklen) return (int)hipErrorInvalidValue;
  const T ebx2_r = (T)(1.0 / (eb * 2)), r = (T)radius;
  const uint32_t units = sample_units(L.lx, L.ly, L.lz), stride = sample_stride(units);
  const uint32_t nsamp = (units + stride - 1) / stride;
  constexpr uint32_t kW = kSampleThreads / 64;
  // two sample units per wave on a 512^3 field: half the workgroups' histogram flushes
  const uint32_t grid = std::max(1u, std::min((nsamp + kW - 1) / kW, 2u * (uint32_t)L.ncu));
  if (zz)
    k_brick3_sample<T, true><<<grid, kSampleThreads, 0, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, hist, bklen, ticket,
                                                               h_hist, flag, epoch);
  else
    k_brick3_sample<T, false><<<grid, kSampleThreads, 0, st>>>(in, L.lx, L.ly, L.lz, ebx2_r, r, hist, bklen, ticket,
                                                                h_hist, flag, epoch);
  return (int)hipGetLastError();
}

template <typename T>
int launch_brick_stream(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const BrickSingle& s,
                        const void* psz_tpl, const void* phf_tpl, hipStream_t st, const HostPub& pub)
{
  const BrickGeom& g = L.g;
  if (g.ndim != 3 || s.bklen > kMaxBklen) return (int)hipErrorInvalidValue;
  const T ebx2_r = (T)(1.0 / (eb * 2)), r = (T)radius;
  StreamArgs a{L.lx,        L.ly,   L.lz,         g.nbx,        g.nby,      g.nbricks, s.ol,       s.book,
               s.bklen,     s.par_nbit, s.par_entry, s.bitstream, s.bs_cap, s.status,  s.ticket,   s.ol_dst,
               s.info,      s.timeout, s.gate,     s.gate_epoch, s.h_book,   s.h_revbook, s.revbook, s.rv_words,
               s.book_flag};
  const size_t lds = stream_lds_bytes<T>();  // dynamic: the exchange and staging areas
  static int per_cu[2] = {0, 0};
  int& pc = per_cu[sizeof(T) == 8];
  if (!pc) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, k_brick3_stream<T, false>, 64 * kStreamWaves, lds) !=
            hipSuccess ||
        pc < 1)
      pc = 1;
  }
  // persistent workgroups claim bricks from the ticket; every one must be resident (a look-back
  // waits only on claimed bricks, and workgroup 0 hands every other one the codebook)
  const uint32_t grid = std::max(1u, std::min(g.nbricks, (uint32_t)(pc * L.ncu)));
  if (zz)
    k_brick3_stream<T, true><<<grid, 64 * kStreamWaves, lds, st>>>(in, a, ebx2_r, r);
  else
    k_brick3_stream<T, false><<<grid, 64 * kStreamWaves, lds, st>>>(in, a, ebx2_r, r);
  if (hipError_t e = hipGetLastError()) return (int)e;
  HeaderTpl t;
  __builtin_memcpy(t.psz, psz_tpl, 176);
  __builtin_memcpy(t.phf, phf_tpl, 64);
  const uint32_t nslot_groups = (g.nbricks * kStreamWaves + 63) / 64;
  const uint32_t fgrid = std::max(1u, std::min((nslot_groups + 3) / 4, 1024u));
  k_brick3_stream_finish<<<fgrid, kFinishThreads, 0, st>>>(a, t, s.archive, s.phf_offset, s.bits_rel, pub);
  return (int)hipGetLastError();
}

template int launch_brick_sample<float>(const BrickLaunch&, const float*, double, int, bool, uint32_t*, int,
                                        uint32_t*, uint32_t*, uint32_t*, uint32_t, hipStream_t);
template int launch_brick_sample<double>(const BrickLaunch&, const double*, double, int, bool, uint32_t*, int,
                                         uint32_t*, uint32_t*, uint32_t*, uint32_t, hipStream_t);
template int launch_brick_stream<float>(const BrickLaunch&, const float*, double, int, bool, const BrickSingle&,
                                        const void*, const void*, hipStream_t, const HostPub&);
template int launch_brick_stream<double>(const BrickLaunch&, const double*, double, int, bool, const BrickSingle&,
                                         const void*, const void*, hipStream_t, const HostPub&);

int launch_brick_cell_bounds(const BrickLaunch& L, const uint32_t* cells, size_t ncell, uint32_t* bstart,
                             uint32_t* unsorted, uint32_t epoch, hipStream_t st)
{
  if (!ncell) return (int)hipSuccess;
  const uint32_t grid = (uint32_t)std::min<size_t>((ncell + 255) / 256, 2048);
  k_brick_cell_bounds<<<grid, 256, 0, st>>>(cells, ncell, L.lx, L.ly, L.lz, L.g.nbx, L.g.nby, L.g.nbricks, bstart,
                                            unsorted, epoch);
  return (int)hipGetLastError();
}

template <typename T>
int launch_brick_decode(const BrickLaunch& L, const uint32_t* bitstream, size_t bs_words, const uint8_t* revbook,
                        int bklen, const uint32_t* par_nbit, const uint32_t* par_entry, T* out, double eb, int radius,
                        bool zz, const BrickOutliers& ol, hipStream_t st)
{
  const T ebx2 = (T)(eb * 2);  // lrz_x.cuhip.inl:432
  const T r = (T)radius;
  const BrickGeom& g = L.g;
  static_assert(sizeof(hfd::LdsTables<kDecB>) + kDecWaves * kDecWaveBytes <= 160 * 1024, "LDS");
  if (bs_words >= (1ull << 30)) return (int)hipErrorInvalidValue;
  if (g.ndim == 1) {
    const uint32_t ntiles = (uint32_t)((g.n + 1023) / 1024), nunits = (ntiles + 63) / 64;
    // waves per CU: the static unit assignment ends when the busiest wave's units are done, and
    // the CU is throughput-bound, so minimise rounds x waves (ties: more waves)
    int wpb = 4;
    size_t best = ~(size_t)0;
    for (int w = 4; w <= kD1MaxWaves && w <= kDecWaves; w++) {
      const size_t rounds = (nunits + (size_t)L.ncu * w - 1) / ((size_t)L.ncu * w);
      if (rounds * w <= best) best = rounds * w, wpb = w;
    }
#ifdef CUSZ_AMD_D1_WAVES  // (experiment: fixed waves per CU)
    wpb = CUSZ_AMD_D1_WAVES;
#endif
    const uint32_t grid = (uint32_t)std::max<size_t>(1, std::min<size_t>(L.ncu, (nunits + wpb - 1) / wpb));
    const size_t lds1 = (size_t)wpb * kD1WaveBytes;
    if (zz)
      k_brick1_decode<T, true><<<grid, 64 * wpb, lds1, st>>>(bitstream, (uint32_t)bs_words, revbook, bklen, par_nbit,
                                                             par_entry, out, g.n, ebx2, r, g.nchunks, nunits, ol);
    else
      k_brick1_decode<T, false><<<grid, 64 * wpb, lds1, st>>>(bitstream, (uint32_t)bs_words, revbook, bklen, par_nbit,
                                                              par_entry, out, g.n, ebx2, r, g.nchunks, nunits, ol);
    return (int)hipGetLastError();
  }
  // buffer stores address a brick block with 32-bit offsets from its first element
  const size_t plane = (size_t)L.lx * L.ly;
  const bool buf = (7 * plane + 7 * (size_t)L.lx + (size_t)kBlk) * sizeof(T) < (1ull << 31);
  const uint32_t bw = (uint32_t)bs_words;
  // 32-column blocks pay once the bricks fill the 12-wave slots (a 512^3 field); a small slab,
  // one brick per wave, is bound by one brick's latency, which the 64-column blocks keep shorter
  // (512 x 512 x 64: 88 against 94 us)
  const bool b32 = CUSZ_AMD_DEC3_BLK ? CUSZ_AMD_DEC3_BLK == 32
                                     : sizeof(T) == 4 && g.nbricks >= (uint32_t)Dec3Cfg<32>::kWaves * (uint32_t)L.ncu;
  auto launch = [&](auto blk) {
    constexpr int B3 = decltype(blk)::value;
    const size_t lds = (size_t)Dec3Cfg<B3>::kWaves * Dec3Cfg<B3>::kWaveBytes;  // dynamic part
#define DEC_LAUNCH(ZZ, BUF)                                                                                     \
    k_brick3_decode<T, ZZ, BUF, B3><<<L.ncu, 64 * Dec3Cfg<B3>::kWaves, lds, st>>>(bitstream, bw, revbook, bklen, par_nbit, \
                                                                              par_entry, out, L.lx, L.ly, L.lz, ebx2, r, \
                                                                              g.nbx, g.nby, g.nbricks, ol)
    if (zz) {
      if (buf) DEC_LAUNCH(true, true); else DEC_LAUNCH(true, false);
    }
    else {
      if (buf) DEC_LAUNCH(false, true); else DEC_LAUNCH(false, false);
    }
#undef DEC_LAUNCH
  };
  if constexpr (sizeof(T) == 4) {
    if (b32) launch(std::integral_constant<int, 32>{});
    else launch(std::integral_constant<int, 64>{});
  }
  else
    launch(std::integral_constant<int, 64>{});
  return (int)hipGetLastError();
}


int launch_chunk_decode(const BrickLaunch& L, const uint32_t* bitstream, size_t bs_words, const uint8_t* revbook,
                        int bklen, const uint32_t* par_nbit, const uint32_t* par_entry, uint16_t* codes, size_t n,
                        uint32_t nchunks, uint32_t sublen, hipStream_t st)
{
  if (bs_words >= (1ull << 30) || bklen < 1 || bklen > kMaxBklen || sublen % kBlk != 0 || sublen == 0)
    return (int)hipErrorInvalidValue;
  if (!nchunks) return (int)hipSuccess;
  // Fewer units than 8 per CU (a 2-D field of a few million values): spread them over every CU,
  // ceil(units / nCU) decoding waves per workgroup, instead of 8 on a fifth of the chip; the
  // workgroup keeps 8 waves so the tables take no longer to build.
  const uint32_t units = (nchunks + 63) / 64;
  const uint32_t ncu = L.ncu > 0 ? (uint32_t)L.ncu : 256u;
  const uint32_t wpb = std::min<uint32_t>(kDecWaves, (units + ncu - 1) / ncu);
  const size_t lds = (size_t)wpb * kD4Cells;
  const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(ncu, (units + wpb - 1) / wpb));
  k_chunk_decode<0><<<grid, 64 * kDecWaves, lds, st>>>(bitstream, (uint32_t)bs_words, revbook, bklen, par_nbit,
                                                       par_entry, codes, n, nchunks, sublen, wpb);
  return (int)hipGetLastError();
}

#ifdef CUSZ_AMD_DEC_PROFILE
extern "C" int psz_amd_debug_brick_profile(unsigned long long* host, int reset)
{
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_brick_prof), sizeof(unsigned long long) * 16);
  if (reset) {
    unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_brick_prof), z, sizeof(z));
  }
  return (int)e;
}
#endif

#define INST(T)                                                                                                   \
  template int launch_brick_scan<T>(const BrickLaunch&, const T*, double, int, bool, const BrickSample&,            \
                                    const OutlierSink&, uint32_t*, uint16_t*, const BrickCodes&, int, hipStream_t,   \
                                    const HostPub&);                                                                \
  template int launch_brick_decode<T>(const BrickLaunch&, const uint32_t*, size_t, const uint8_t*, int,            \
                                      const uint32_t*, const uint32_t*, T*, double, int, bool, const BrickOutliers&, \
                                      hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace cusz_amd
