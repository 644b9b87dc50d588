// cusz_amd/csrc/spline.hip -- cuSZ-i spline3 predictor-quantizer and reconstruction for gfx950.
//
// Semantics: psz/src/kernel/detail/spline3.inl (compress kernel :916-973, reconstruct :975-1016,
// interpolation schedule :678-900, per-point rule :391-618), launched per 32x8x8 tile on a 33x9x9
// scratch that includes the +1 faces of the next tiles (spline3.cu:22-63).  The CPU restatement
// is oracle/spline_oracle.c; results are bit-identical to it (parity with the reference itself is
// unpinned: the reference has no test and no wired pipeline for this path).
//
// MI355X design (not the reference's 384-thread block with 10..1296 busy threads per stage and an
// atomicAdd outlier race):
//  * persistent workgroups of 256 threads (4 waves) walk the tiles; the histogram lives in LDS for
//    the workgroup's whole life and is merged once, so 65,536 tiles cost ~1k global merges;
//  * the tile's 33x9x9 region is read with x-contiguous rows (the +1 face rows come from L2:
//    the neighbouring tile reads the same lines);
//  * the nine stages run back to back in LDS with one barrier each; codes stay in LDS as int32
//    and leave as coalesced u16 rows together with the histogram and the outliers;
//  * outliers get deterministic slots: (z, y, x) order inside the tile, wave ballots + a
//    4-wave scan, into the tile's fixed slot range (spill list past 10 % + 16), the same
//    OutlierSink the Lorenzo kernels use;
//  * decompression reads each tile's outliers (and its seven upper neighbours', for the faces)
//    from per-tile buckets built by three small kernels, instead of the reference's scatter into
//    the output buffer that other tiles are already writing.
#include <algorithm>

#include "common.hh"
#include "hf_device.hh"
#include "kernels.hh"

namespace cusz_amd {

namespace {

constexpr int kSX = 33, kSY = 9, kSZ = 9, kSN = kSX * kSY * kSZ;  // 2673
constexpr int kSplThreads = 256;
constexpr int kPer = (kSN + kSplThreads - 1) / kSplThreads;  // scratch points per thread (11)

__device__ __forceinline__ int sidx(int x, int y, int z) { return x + kSX * (y + kSY * z); }

// a value the compiler cannot treat as loop-invariant: the prefetch's per-point coordinates are
// then recomputed at each fetch instead of living in ~40 extra VGPRs across the whole tile loop
__device__ __forceinline__ int opaque(int v)
{
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

struct TileInfo {
  uint32_t bx, by, bz;
  bool lastx, lasty, lastz;
  uint32_t X, Y, Z;
};

// per-point prediction (spline3.inl:457-585); DIR 0 along z (BLUE), 1 along y (YELLOW), 2 along x
// (HOLLOW).  Expressions keep the reference's operation order; -ffp-contract=off keeps them unfused.
template <typename T, int DIR>
__device__ __forceinline__ T spl_pred(const T* s, const TileInfo& t, int x, int y, int z, int u)
{
  const int c = DIR == 0 ? z : DIR == 1 ? y : x;
  const int blk = DIR == 2 ? 32 : 8;
  const int stride = DIR == 0 ? kSX * kSY : DIR == 1 ? kSX : 1;
  const uint32_t g = DIR == 0 ? t.bz * 8 + z : DIR == 1 ? t.by * 8 + y : t.bx * 32 + x;
  const uint32_t dsz = DIR == 0 ? t.Z : DIR == 1 ? t.Y : t.X;
  const bool last = DIR == 0 ? t.lastz : DIR == 1 ? t.lasty : t.lastx;
  const T* p = s + sidx(x, y, z);
  const int m3 = -3 * u * stride, m1 = -u * stride, p1 = u * stride, p3 = 3 * u * stride;
  if (!last) {
    if (c >= 3 * u && c + 3 * u <= blk) return (-p[m3] + 9 * p[m1] + 9 * p[p1] - p[p3]) / 16;
    if (c + 3 * u <= blk) return (3 * p[m1] + 6 * p[p1] - p[p3]) / 8;
    if (c >= 3 * u) return (-p[m3] + 6 * p[m1] + 3 * p[p1]) / 8;
    return (p[m1] + p[p1]) / 2;
  }
  if (c >= 3 * u) {
    if (c + 3 * u <= blk && g + 3 * u < dsz) return (-p[m3] + 9 * p[m1] + 9 * p[p1] - p[p3]) / 16;
    if (g + u < dsz) return (-p[m3] + 6 * p[m1] + 3 * p[p1]) / 8;
    return p[m1];
  }
  if (c + 3 * u <= blk && g + 3 * u < dsz) return (3 * p[m1] + 6 * p[p1] - p[p3]) / 8;
  if (g + u < dsz) return (p[m1] + p[p1]) / 2;
  return p[m1];
}

// one stage (spline3.inl:620-660): points (x, y, z) of the DX x DY x DZ lattice of this direction
template <typename T, int DIR, int U, int DX, int DY, int DZ, bool INCL, bool COMP>
__device__ __forceinline__ void spl_stage(T* s, int* e, const TileInfo& t, float eb_r, float ebx2, int radius)
{
  constexpr int N = DX * DY * DZ;
#pragma unroll 1
  for (int q = threadIdx.x; q < N; q += kSplThreads) {
    const int ix = q % DX, iy = (q / DX) % DY, iz = q / (DX * DY);
    const int x = DIR == 2 ? U * (2 * ix + 1) : U * 2 * ix;
    const int y = DIR == 1 ? U * (2 * iy + 1) : DIR == 0 ? U * 2 * iy : U * iy;
    const int z = DIR == 0 ? U * (2 * iz + 1) : U * iz;
    const uint32_t gx = t.bx * 32 + x, gy = t.by * 8 + y, gz = t.bz * 8 + z;
    if (!(gx < t.X && gy < t.Y && gz < t.Z)) continue;
    if (!INCL && !(x < 32 + (int)t.lastx && y < 8 + (int)t.lasty && z < 8 + (int)t.lastz)) continue;
    const T pred = spl_pred<T, DIR>(s, t, x, y, z, U);
    const int i = sidx(x, y, z);
    if (COMP) {
      const T err = s[i] - pred;
      T code = (sizeof(T) == 4 ? (T)__builtin_fabsf((float)err) : (T)__builtin_fabs((double)err)) * (T)eb_r + 1;
      code = err < 0 ? -code : code;
      const int ci = (int)(code / 2) + radius;
      e[i] = ci;
      s[i] = pred + ((T)ci - radius) * (T)ebx2;
    }
    else {
      s[i] = pred + ((T)e[i] - radius) * (T)ebx2;
    }
  }
}

// calc_eb (spline3.inl:730-745): level error bounds, float arithmetic through double like the
// reference's FP=float members multiplied by the double alpha
__device__ __forceinline__ void spl_level_eb(int unit, float eb_r0, float ebx20, float& eb_r, float& ebx2)
{
  eb_r = eb_r0, ebx2 = ebx20;
  for (int tmp = 1; tmp < unit; tmp *= 2) {
    eb_r = (float)((double)eb_r * 1.25);
    ebx2 = (float)((double)ebx2 / 1.25);
  }
  if ((double)ebx2 < (double)ebx20 / 2.0) {
    ebx2 = (float)((double)ebx20 / 2.0);
    eb_r = (float)((double)eb_r0 * 2.0);
  }
}

// spline3d_layout2_interpolate with reverse = {false,false,false} and cubic interpolation
template <typename T, bool COMP>
__device__ void spl_interpolate(T* s, int* e, const TileInfo& t, float eb_r0, float ebx20, int radius)
{
  float r, x2;
  spl_level_eb(4, eb_r0, ebx20, r, x2);
  spl_stage<T, 0, 4, 5, 2, 1, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 1, 4, 5, 1, 3, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 2, 4, 4, 3, 3, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_level_eb(2, eb_r0, ebx20, r, x2);
  spl_stage<T, 0, 2, 9, 3, 2, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 1, 2, 9, 2, 5, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 2, 2, 8, 5, 5, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_level_eb(1, eb_r0, ebx20, r, x2);
  spl_stage<T, 0, 1, 17, 5, 4, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 1, 1, 17, 4, 9, true, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
  spl_stage<T, 2, 1, 16, 9, 9, false, COMP>(s, e, t, r, x2, radius);
  __syncthreads();
}

// The tiles a persistent workgroup walks: blocks b and b + 8 share an XCD (dispatch is
// round-robin; used for speed only), so block b takes the it-th tile of XCD range b % 8 -- each
// XCD works through one contiguous eighth of the tiles, and tiles that share +1 faces are read
// through the same L2.  Any grid that is not a multiple of 8 walks tile = b + it * grid.
struct TileOrder {
  uint32_t hi, first, step;
  __device__ TileOrder(uint32_t n)
  {
    if (gridDim.x % 8u == 0u && gridDim.x >= 8u) {
      const uint32_t per = (n + 7u) / 8u, lo = min((blockIdx.x & 7u) * per, n);
      hi = min(lo + per, n), first = lo + (blockIdx.x >> 3), step = gridDim.x >> 3;
    }
    else
      hi = n, first = blockIdx.x, step = gridDim.x;
  }
  // tile of iteration it, or ~0u past the last
  __device__ uint32_t at(uint32_t it) const
  {
    const uint64_t t = (uint64_t)first + (uint64_t)it * step;
    return t < hi ? (uint32_t)t : ~0u;
  }
};

__device__ __forceinline__ TileInfo tile_of(uint32_t tile, uint32_t gdx, uint32_t gdy, uint32_t gdz, uint32_t X,
                                            uint32_t Y, uint32_t Z)
{
  TileInfo t;
  t.bx = tile % gdx;
  t.by = (tile / gdx) % gdy;
  t.bz = tile / (gdx * gdy);
  t.lastx = t.bx == gdx - 1, t.lasty = t.by == gdy - 1, t.lastz = t.bz == gdz - 1;
  t.X = X, t.Y = Y, t.Z = Z;
  return t;
}

template <typename T>
__global__ void __launch_bounds__(kSplThreads, 4) k_spline3_c(SplineArgs<T> a)
{
  __shared__ T s_data[kSN];
  __shared__ int s_code[kSN];
  __shared__ uint32_t s_hist[kMaxBklen];
  __shared__ uint32_t s_pc[8][4];  // outliers per (plane, wave), then their exclusive offsets
  __shared__ uint32_t s_sp;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < a.bklen; i += kSplThreads) s_hist[i] = 0;
  const uint32_t X = a.X, Y = a.Y, Z = a.Z;
  const uint32_t ax = (X + 7) / 8, ay = (Y + 7) / 8;
  const int radius = a.radius;
  // the next tile's 33x9x9 region is fetched into registers (kPer values per thread) while the
  // current tile interpolates, so the load latency is not paid once per tile and row
  T pv[kPer];
  auto fetch = [&](uint32_t tile) {
    const TileInfo t = tile_of(tile, a.gdx, a.gdy, a.gdz, X, Y, Z);
    const int ot = opaque(tid);  // recomputed per fetch, not hoisted into live registers
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int i = ot + k * kSplThreads;
      const int x = i % kSX, y = (i / kSX) % kSY, z = i / (kSX * kSY);
      const uint32_t gx = t.bx * 32 + x, gy = t.by * 8 + y, gz = t.bz * 8 + z;
      T v = 0;
      if (i < kSN && gx < X && gy < Y && gz < Z) v = a.in[gx + (size_t)X * (gy + (size_t)Y * gz)];
      pv[k] = v;
    }
  };
  const TileOrder order(a.ntiles);
  if (order.at(0) != ~0u) fetch(order.at(0));
  for (uint32_t it = 0, tile = order.at(0); tile != ~0u; tile = order.at(++it)) {
    const TileInfo t = tile_of(tile, a.gdx, a.gdy, a.gdz, X, Y, Z);
    // scratch: data of the 33x9x9 region (0 outside the field), anchor codes = radius
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int i = tid + k * kSplThreads;
      if (i < kSN) {
        const int x = i % kSX, y = (i / kSX) % kSY, z = i / (kSX * kSY);
        s_data[i] = pv[k];
        s_code[i] = (x % 8 == 0 && y % 8 == 0 && z % 8 == 0) ? radius : 0;
      }
    }
    __syncthreads();
    // anchors: the tile's interior points on the 8-lattice (c_gather_anchor, spline3.inl:205-220);
    // no stage writes them, so they are read back from the scratch
    if (tid < 4) {
      const uint32_t gx = t.bx * 32 + 8 * tid, gy = t.by * 8, gz = t.bz * 8;
      if (gx < X && gy < Y && gz < Z) a.anchor[gx / 8 + ax * (gy / 8 + (size_t)ay * (gz / 8))] = s_data[sidx(8 * tid, 0, 0)];
    }
    if (order.at(it + 1) != ~0u) fetch(order.at(it + 1));
    spl_interpolate<T, true>(s_data, s_code, t, a.eb_r, a.ebx2, radius);
    // interior codes out (shmem2global_32x8x8data_with_compaction, spline3.inl:370-398): plane z
    // of the tile per pass, thread -> (x, y).  Outliers get their (z, y, x) rank from a count
    // pass first, so a tile over its slot reserves one spill range and the order stays fixed.
    const int px = tid & 31, py = tid >> 5;
    const uint32_t gx = t.bx * 32 + px, gy = t.by * 8 + py;
    uint32_t mine = 0;  // bit z: this thread's point of plane z is an outlier
    const size_t gid0 = gx + (size_t)X * (gy + (size_t)Y * (t.bz * 8));
    const size_t plane = (size_t)X * Y;
    for (int z = 0; z < 8; z++) {  // codes and histogram; outliers counted per (plane, wave)
      const int cand = s_code[sidx(px, py, z)];
      const bool in = gx < X && gy < Y && t.bz * 8 + z < Z;
      const bool q = cand >= 0 && cand < 2 * radius;
      if (in) {
        a.codes[gid0 + z * plane] = q ? (uint16_t)cand : (uint16_t)0;
        atomicAdd(&s_hist[q ? cand : 0], 1u);
      }
      const bool ol = in && !q;
      const uint64_t m = __ballot(ol);
      if (lane == 0) s_pc[z][wid] = (uint32_t)__popcll(m);
      mine |= (uint32_t)ol << z;
    }
    __syncthreads();
    if (wid == 0) {  // exclusive offsets in (z, wave) order: one DPP scan over the 32 counts
      uint32_t* pc = &s_pc[0][0];
      const uint32_t c = lane < 32 ? pc[lane] : 0u;
      const uint32_t inc = hfd::wave_incl_scan(c);
      if (lane < 32) pc[lane] = inc - c;
      const uint32_t run = (uint32_t)__builtin_amdgcn_readlane((int)inc, 31);
      if (lane == 0) {
        s_sp = run > a.ol.cap_per_brick ? atomicAdd(a.ol.spill_cnt, run - a.ol.cap_per_brick) : 0u;
        a.ol.brick_cnt[tile] = run;
        if (run > a.ol.cap_per_brick) a.ol.spill_start[tile] = s_sp;
      }
    }
    __syncthreads();
    uint64_t* slot = a.ol.slots + (size_t)tile * a.ol.cap_per_brick;
    for (int z = 0; z < 8; z++) {  // outlier cells at their (z, y, x) rank
      const uint64_t m = __ballot((mine >> z) & 1u);
      if (!m) continue;
      if ((mine >> z) & 1u) {
        const int cand = s_code[sidx(px, py, z)];
        const size_t gid = gid0 + z * plane;
        const uint32_t pos = s_pc[z][wid] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        const uint64_t cell = make_cell((float)cand, (uint32_t)gid);
        if (pos < a.ol.cap_per_brick) slot[pos] = cell;
        else if (s_sp + (pos - a.ol.cap_per_brick) < a.ol.spill_cap) a.ol.spill[s_sp + (pos - a.ol.cap_per_brick)] = cell;
      }
    }
    __syncthreads();
  }
  __syncthreads();
  for (int i = tid; i < a.bklen; i += kSplThreads)
    if (s_hist[i]) atomicAdd(&a.hist[i], s_hist[i]);
}

// ---- decompression ------------------------------------------------------------------------------
// Outlier cells -> per-tile buckets: count, scan, fill (order inside a bucket is irrelevant).
__device__ __forceinline__ uint32_t tile_of_index(uint32_t gid, uint32_t X, uint32_t Y, uint32_t gdx, uint32_t gdy)
{
  const uint32_t gx = gid % X, gy = (gid / X) % Y, gz = gid / (X * Y);
  return gx / 32 + gdx * (gy / 8 + gdy * (gz / 8));
}

// Archives written by this compressor list outlier cells tile by tile (ranged spill, see
// OutlierSink::spill_start), so the cells already ARE the buckets: one pass finds each tile's
// first cell (no atomics).  Any descent in tile order sets *unsorted and the count / scan / fill
// kernels below build the buckets instead (they return at once when the cells are sorted).
__global__ void __launch_bounds__(256) k_spl_bucket_bounds(const uint32_t* cells, size_t ncell, size_t n, uint32_t X,
                                                           uint32_t Y, uint32_t gdx, uint32_t gdy, uint32_t ntiles,
                                                           uint32_t* off, uint32_t* unsorted)
{
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < ncell; i += (size_t)gridDim.x * 256) {
    const uint32_t gid = cells[2 * i + 1];
    if (gid >= n) {
      atomicOr(unsorted, 1u);
      continue;
    }
    const int64_t t = tile_of_index(gid, X, Y, gdx, gdy);
    int64_t tp = -1;
    if (i > 0) {
      const uint32_t gp = cells[2 * i - 1];
      tp = gp < n ? (int64_t)tile_of_index(gp, X, Y, gdx, gdy) : (int64_t)ntiles;
    }
    if (t < tp) atomicOr(unsorted, 1u);
    for (int64_t u = tp + 1; u <= t; u++) off[u] = (uint32_t)i;
    if (i + 1 == ncell)
      for (int64_t u = t + 1; u <= (int64_t)ntiles; u++) off[u] = (uint32_t)ncell;
  }
}

__global__ void __launch_bounds__(256) k_spl_bucket_count(const uint32_t* cells, size_t ncell, size_t n,
                                                          uint32_t X, uint32_t Y, uint32_t gdx, uint32_t gdy,
                                                          uint32_t* cnt, const uint32_t* unsorted)
{
  if (!*unsorted) return;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < ncell; i += (size_t)gridDim.x * 256) {
    const uint32_t gid = cells[2 * i + 1];
    if (gid < n) atomicAdd(&cnt[tile_of_index(gid, X, Y, gdx, gdy)], 1u);
  }
}

// exclusive scan of cnt[0..m) into off[0..m], one workgroup of 1024 threads, sequential chunks
__global__ void __launch_bounds__(1024) k_spl_bucket_scan(const uint32_t* cnt, uint32_t m, uint32_t* off,
                                                          const uint32_t* unsorted)
{
  if (!*unsorted) return;
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t b = 0; b < m; b += 1024) {
    const uint32_t i = b + tid;
    const uint32_t v = i < m ? cnt[i] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d);
      if (lane >= d) inc += o;
    }
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    uint32_t wo = s_carry;
    for (int w = 0; w < wid; w++) wo += s_w[w];
    if (i < m) off[i] = wo + inc - v;
    __syncthreads();
    if (tid == 1023) s_carry = wo + inc;
    __syncthreads();
  }
  if (tid == 0) off[m] = s_carry;
}

__global__ void __launch_bounds__(256) k_spl_bucket_fill(const uint32_t* cells, size_t ncell, size_t n, uint32_t X,
                                                         uint32_t Y, uint32_t gdx, uint32_t gdy, const uint32_t* off,
                                                         uint32_t* fill, uint32_t* bucket, const uint32_t* unsorted)
{
  if (!*unsorted) return;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < ncell; i += (size_t)gridDim.x * 256) {
    const uint32_t v = cells[2 * i], gid = cells[2 * i + 1];
    if (gid >= n) continue;
    const uint32_t tl = tile_of_index(gid, X, Y, gdx, gdy);
    const uint32_t p = off[tl] + atomicAdd(&fill[tl], 1u);
    bucket[2 * p] = v;
    bucket[2 * p + 1] = gid;
  }
}

template <typename T>
__global__ void __launch_bounds__(kSplThreads, 4) k_spline3_x(SplineXArgs<T> a)
{
  __shared__ T s_data[kSN];
  __shared__ int s_code[kSN];
  const int tid = threadIdx.x;
  const uint32_t X = a.X, Y = a.Y, Z = a.Z;
  const uint32_t ax = (X + 7) / 8, ay = (Y + 7) / 8, az = (Z + 7) / 8;
  const int radius = a.radius;
  const uint32_t* bk = a.nbucket ? (*a.unsorted ? a.bucket : a.cells) : nullptr;
  // bucket ranges [b0, b1) of a tile and its seven upper neighbours, double-buffered by tile parity
  __shared__ uint32_t s_rng[2][8][2];
  // The next tile's codes and anchors (threads 0..19, one 8-lattice point each), the bucket ranges
  // of the tile after it (threads 0..7) and the next tile's first kEnt * 256 bucket entries are
  // fetched into registers while the current tile interpolates.
  constexpr int kEnt = 3;
  int pc[kPer];
  T pa = 0;
  uint32_t pr0 = 0, pr1 = 0;
  uint32_t pcv[kEnt], pgid[kEnt], pm = 0;
  auto ranges_of = [&](uint32_t tile, uint32_t& r0, uint32_t& r1) {
    r0 = r1 = 0;
    if (!bk || tid >= 8 || tile == ~0u) return;
    const TileInfo t = tile_of(tile, a.gdx, a.gdy, a.gdz, X, Y, Z);
    const uint32_t nbx = t.bx + (tid & 1), nby = t.by + ((tid >> 1) & 1), nbz = t.bz + (tid >> 2);
    if (nbx < a.gdx && nby < a.gdy && nbz < a.gdz) {
      const uint32_t nt = nbx + a.gdx * (nby + a.gdy * nbz);
      r0 = a.boff[nt], r1 = a.boff[nt + 1];
    }
  };
  auto fetch = [&](uint32_t tile, uint32_t after) {
    const TileInfo t = tile_of(tile, a.gdx, a.gdy, a.gdz, X, Y, Z);
    const int ot = opaque(tid);  // recomputed per fetch, not hoisted into live registers
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int i = ot + k * kSplThreads;
      const int x = i % kSX, y = (i / kSX) % kSY, z = i / (kSX * kSY);
      const uint32_t gx = t.bx * 32 + x, gy = t.by * 8 + y, gz = t.bz * 8 + z;
      int c = 0;
      if (i < kSN && gx < X && gy < Y && gz < Z) c = a.codes[gx + (size_t)X * (gy + (size_t)Y * gz)];
      pc[k] = c;
    }
    pa = 0;
    if (tid < 20) {  // x_reset_scratch_33x9x9data + global2shmem_fuse (spline3.inl:241-278, :309-328)
      const uint32_t Ax = tid % 5 + t.bx * 4, Ay = (tid / 5) % 2 + t.by, Az = tid / 10 + t.bz;
      if (Ax < ax && Ay < ay && Az < az) pa = a.anchor[Ax + ax * (Ay + (size_t)ay * Az)];
    }
    ranges_of(after, pr0, pr1);
  };
  // entry e of the concatenated ranges of buffer `buf` -> its cell index (false past the end)
  auto locate = [&](int buf, uint32_t e, uint32_t& j) {
    uint32_t pre = 0;
    bool found = false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t b0 = s_rng[buf][k][0], len = s_rng[buf][k][1] - b0;
      if (!found && e < pre + len) j = b0 + (e - pre), found = true;
      pre += len;
    }
    return found;
  };
  auto entries = [&](int buf) {  // registers <- the first kEnt * 256 entries
    pm = 0;
#pragma unroll
    for (int m = 0; m < kEnt; m++) {
      uint32_t j;
      if (locate(buf, (uint32_t)tid + kSplThreads * m, j)) {
        pcv[m] = bk[2 * j], pgid[m] = bk[2 * j + 1];
        pm |= 1u << m;
      }
    }
  };
  auto put = [&](const TileInfo& t, uint32_t cv, uint32_t gid) {
    uint32_t gx, gy, gz;
    if (a.ndiv) gx = gid % X, gy = (gid / X) % Y, gz = gid / (X * Y);
    else {
      const uint32_t r = __umulhi(gid, a.mX) >> a.sX;  // gid / X
      gz = __umulhi(r, a.mY) >> a.sY;                 // r / Y
      gx = gid - r * X, gy = r - gz * Y;
    }
    const int lx = (int)gx - (int)(t.bx * 32), ly = (int)gy - (int)(t.by * 8), lz = (int)gz - (int)(t.bz * 8);
    if (lx >= 0 && lx < kSX && ly >= 0 && ly < kSY && lz >= 0 && lz < kSZ)
      s_code[sidx(lx, ly, lz)] = (int)__builtin_bit_cast(float, cv);
  };
  int par = 0;
  const TileOrder order(a.ntiles);
  if (order.at(0) != ~0u) {
    ranges_of(order.at(0), pr0, pr1);
    if (tid < 8) s_rng[0][tid][0] = pr0, s_rng[0][tid][1] = pr1;
    fetch(order.at(0), order.at(1));
    __syncthreads();
    if (bk) entries(0);
  }
  for (uint32_t it = 0, tile = order.at(0); tile != ~0u; tile = order.at(++it), par ^= 1) {
    const TileInfo t = tile_of(tile, a.gdx, a.gdy, a.gdz, X, Y, Z);
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const int i = tid + k * kSplThreads;
      if (i < kSN) {
        const int x = i % kSX, y = (i / kSX) % kSY, z = i / (kSX * kSY);
        if (!(x % 8 == 0 && y % 8 == 0 && z % 8 == 0)) s_data[i] = 0;
        s_code[i] = pc[k];
      }
    }
    if (tid < 20) s_data[sidx(8 * (tid % 5), 8 * ((tid / 5) % 2), 8 * (tid / 10))] = pa;
    if (tid < 8) s_rng[par ^ 1][tid][0] = pr0, s_rng[par ^ 1][tid][1] = pr1;  // the next tile's
    __syncthreads();
    // outlier codes of this tile and of the faces it shares with its upper neighbours: the
    // prefetched entries, then (rarely) the ones past kEnt * 256 straight from the buckets
    if (bk) {
      uint32_t total = 0;
      for (int k = 0; k < 8; k++) total += s_rng[par][k][1] - s_rng[par][k][0];
#pragma unroll
      for (int m = 0; m < kEnt; m++)
        if ((pm >> m) & 1u) put(t, pcv[m], pgid[m]);
      for (uint32_t e = (uint32_t)tid + kSplThreads * kEnt; e < total; e += kSplThreads) {
        uint32_t j;
        if (locate(par, e, j)) put(t, bk[2 * j], bk[2 * j + 1]);
      }
      if (total) __syncthreads();
    }
    if (order.at(it + 1) != ~0u) {
      fetch(order.at(it + 1), order.at(it + 2));
      if (bk) entries(par ^ 1);
    }
    spl_interpolate<T, false>(s_data, s_code, t, a.eb_r, a.ebx2, radius);
    {
      const int x = tid & 31, y = tid >> 5;
      const uint32_t gx = t.bx * 32 + x, gy = t.by * 8 + y;
      T* o = a.out + (gx + (size_t)X * (gy + (size_t)Y * (t.bz * 8)));
      const size_t plane = (size_t)X * Y;
      const uint32_t nz = min(8u, Z - t.bz * 8);
      if (gx < X && gy < Y)
#pragma unroll
        for (int z = 0; z < 8; z++)
          if ((uint32_t)z < nz) o[z * plane] = s_data[sidx(x, y, z)];
    }
    __syncthreads();
  }
}

int spl_grid(const void* fn, size_t lds, uint32_t ntiles)
{
  int dev = 0, ncu = 0;  // the current device (no process-global cache: several GPUs per process)
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kSplThreads, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const uint32_t full = (uint32_t)(per_cu * ncu);
  return (int)(ntiles < full ? ntiles : full);
}

}  // namespace

SplineGeom spline_geom(size_t x, size_t y, size_t z)
{
  SplineGeom g;
  g.gdx = (uint32_t)((x + 31) / 32), g.gdy = (uint32_t)((y + 7) / 8), g.gdz = (uint32_t)((z + 7) / 8);
  g.ntiles = g.gdx * g.gdy * g.gdz;
  g.anchor_len = ((x + 7) / 8) * ((y + 7) / 8) * ((z + 7) / 8);
  return g;
}

template <typename T>
int launch_spline3_c(const SplineArgs<T>& a, hipStream_t st)
{
  if (a.ntiles == 0) return 0;
  const int grid = spl_grid((const void*)k_spline3_c<T>, 0, a.ntiles);
  k_spline3_c<T><<<grid, kSplThreads, 0, st>>>(a);
  return (int)hipGetLastError();
}

template <typename T>
int launch_spline3_x(SplineXArgs<T> a, const uint32_t* cells, size_t ncell, uint32_t* scratch, hipStream_t st)
{
  if (a.ntiles == 0) return 0;
  // scratch: cnt[ntiles] | fill[ntiles] | off[ntiles+1] | unsorted | bucket[2 ncell]
  a.nbucket = ncell;
  if (ncell) {
    uint32_t* cnt = scratch;
    uint32_t* fill = scratch + a.ntiles;
    uint32_t* off = scratch + 2 * (size_t)a.ntiles;
    uint32_t* unsorted = off + a.ntiles + 1;
    uint32_t* bucket = unsorted + 1;
    const size_t n = (size_t)a.X * a.Y * a.Z;
    if (hipMemsetAsync(scratch, 0, (3 * (size_t)a.ntiles + 2) * 4, st) != hipSuccess) return (int)hipGetLastError();
    const int gb = (int)std::min<size_t>((ncell + 255) / 256, 4096);
    k_spl_bucket_bounds<<<gb, 256, 0, st>>>(cells, ncell, n, a.X, a.Y, a.gdx, a.gdy, a.ntiles, off, unsorted);
    k_spl_bucket_count<<<gb, 256, 0, st>>>(cells, ncell, n, a.X, a.Y, a.gdx, a.gdy, cnt, unsorted);
    k_spl_bucket_scan<<<1, 1024, 0, st>>>(cnt, a.ntiles, off, unsorted);
    k_spl_bucket_fill<<<gb, 256, 0, st>>>(cells, ncell, n, a.X, a.Y, a.gdx, a.gdy, off, fill, bucket, unsorted);
    a.boff = off;
    a.bucket = bucket;
    a.cells = cells;
    a.unsorted = unsorted;
  }
  if ((size_t)a.X * a.Y * a.Z < (1ull << 31)) {
    // d >= 2, l = ceil(log2 d): m = ceil(2^(31 + l) / d) < 2^32, i / d = (i * m) >> (31 + l)
    auto magic = [](uint32_t d, uint32_t& m, uint32_t& sh) {
      uint32_t l = 1;
      while ((1ull << l) < d) l++;
      m = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
      sh = l - 1;
    };
    a.ndiv = a.X < 2 || a.Y < 2;
    if (!a.ndiv) magic(a.X, a.mX, a.sX), magic(a.Y, a.mY, a.sY);
  }
  const int grid = spl_grid((const void*)k_spline3_x<T>, 0, a.ntiles);
  k_spline3_x<T><<<grid, kSplThreads, 0, st>>>(a);
  return (int)hipGetLastError();
}

size_t spline_x_scratch_words(uint32_t ntiles, size_t ncell) { return 3 * (size_t)ntiles + 4 + 2 * ncell; }  // + unsorted flag fits the +4

template int launch_spline3_c<float>(const SplineArgs<float>&, hipStream_t);
template int launch_spline3_c<double>(const SplineArgs<double>&, hipStream_t);
template int launch_spline3_x<float>(SplineXArgs<float>, const uint32_t*, size_t, uint32_t*, hipStream_t);
template int launch_spline3_x<double>(SplineXArgs<double>, const uint32_t*, size_t, uint32_t*, hipStream_t);

}  // namespace cusz_amd
