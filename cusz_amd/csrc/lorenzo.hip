// cusz_amd/csrc/lorenzo.hip -- Lorenzo predictor-quantizer and reconstructor for gfx950.
//
// Semantics restate the reference GPU kernels exactly (integer codes and outlier set
// bit-exact, reconstruction in the reference's floating-point operation order):
//   compress   psz/src/kernel/detail/lrz_c.cuhip.inl:23-109 (1D), 187-273 (2D), 275-372 (3D)
//   decompress psz/src/kernel/detail/lrz_x.cuhip.inl:11-78 (1D), 178-269 (2D), 271-360 (3D)
//              + scan order of psz/src/kernel/detail/wave32.cuhip.inl:7-66
// Tiles (launch.hh:47-121): 1D 1024, 2D 32x32, 3D 8x8x8; values outside the data are 0.
//
// MI355X layout (not the reference's): one wave64 owns a "brick" and walks it serially,
// each lane holding V consecutive x-elements (V=4 f32 -> 16-B loads, 1 KiB per wave
// instruction).  3D brick = (64V) x 8 x 8: the lane keeps its 8 z-values of a row column
// in registers, so the z-difference is in-register, the x-difference is a one-lane shuffle
// and the y-difference uses the previous row's registers.  The code histogram is fused
// (per-workgroup LDS bins, merged once), and outliers go to a per-brick slot, so the
// predictor reads the input exactly once and writes only codes (+ sparse outliers).
#include "common.hh"
#include "kernels.hh"
#include "lrz_device.hh"
#include "pub_device.hh"

namespace cusz_amd {

using namespace lrzd;

// Row loads by raw buffer instructions (2-D kernels): a row outside the field, or a lane past
// its end, gets an offset past the row's range and reads 0, so the loads need no branch and the
// waitcnt pass can count them (a load in a branch costs a wait for everything in flight).
// The row's range is lx * sizeof(E) bytes: < 2^31 (launch_lorenzo_c / _x check).
constexpr uint32_t kRowOOB = 0x80000000u;
template <typename E>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const E* p, size_t row_start, uint32_t lx)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<E*>(p + row_start), 0, (int)(lx * sizeof(E)), 0x00020000);
}
template <typename T, int V>
__device__ __forceinline__ void bload_row(__amdgpu_buffer_rsrc_t rs, uint32_t off, T (&v)[V])
{
  constexpr int B = (int)sizeof(T) * V;
  if constexpr (B >= 16) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int h = 0; h < B / 16; h++) {
      const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u * h), 0, 0);
      __builtin_memcpy(reinterpret_cast<char*>(&v[0]) + 16 * h, &w, 16);
    }
  }
  else if constexpr (B == 8) {
    const auto w = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 0);
    __builtin_memcpy(&v[0], &w, 8);
  }
  else {
    static_assert(B == 4, "row piece of 4, 8, 16 or 32 bytes");
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0);
    __builtin_memcpy(&v[0], &w, 4);
  }
}
// V codes packed two per u32
template <int V>
__device__ __forceinline__ void bload_codes(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t (&w)[(V + 1) / 2])
{
  if constexpr (V == 4) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 0);
    __builtin_memcpy(&w[0], &q, 8);
  }
  else if constexpr (V == 2)
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 0);
  else
    w[0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)off, 0, 0);
}


// =========================================================================================
// predictor-quantizer kernels
// =========================================================================================

// 1D: brick = 16 tiles of 1024; wave step = 256 elements (V=4 per lane).
template <typename T, bool ZZ>
__global__ void __launch_bounds__(256)
k_lorenzo_c1d(const T* __restrict__ in, size_t n, T ebx2_r, T r, uint16_t* __restrict__ codes,
              OutlierSink ol, uint32_t* __restrict__ g_hist, int bklen, uint32_t nbricks, HostPub pub)
{
  constexpr int V = 4;
  __shared__ uint32_t s_hist[kMaxBklen];
  hist_init(s_hist, bklen);
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    uint32_t cnt = 0;
    T carry = 0;
    const size_t bbase = (size_t)brick * 16384;
    const uint32_t x0 = lane * V;
    // row s + 1 is loaded while row s is processed (software pipelining of the row loop)
    T nxt[V];
    load_row<T, V>(in, bbase, x0, (uint32_t)(n - bbase < 256 ? n - bbase : 256), true, nxt);
    for (int s = 0; s < 64; s++) {
      const size_t base = bbase + (size_t)s * 256;
      // treat [base, n) as one long row of length n - base
      const uint32_t rowlen = (uint32_t)(n - base < 256 ? n - base : 256);
      if (base >= n) break;
      T p[V];
#pragma unroll
      for (int k = 0; k < V; k++) p[k] = nxt[k];
      const size_t nbase = base + 256;
      if (s < 63 && nbase < n) load_row<T, V>(in, nbase, x0, (uint32_t)(n - nbase < 256 ? n - nbase : 256), true, nxt);
#pragma unroll
      for (int k = 0; k < V; k++) p[k] = dround(p[k] * ebx2_r);
      T west = __shfl_up(p[V - 1], 1);
      const T last = __shfl(p[V - 1], 63);
      if (lane == 0) west = (s & 3) ? carry : T(0);
      carry = last;
      T d[V];
#pragma unroll
      for (int k = V - 1; k > 0; k--) d[k] = p[k] - p[k - 1];
      d[0] = p[0] - west;
      quantize_row<T, V, ZZ>(d, r, codes, base, x0, rowlen, true, s_hist, ol, brick, cnt);
    }
    if (lane == 0) ol.brick_cnt[brick] = cnt;
  }
  hist_flush(s_hist, g_hist, bklen);
  publish_last(pub);  // the histogram to the host (pipeline.cc compress_scan)
}

// 2D: brick = (64V) x 32 rows (one tile row); tiles 32 wide.
template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(256)
k_lorenzo_c2d(const T* __restrict__ in, uint32_t lx, uint32_t ly, T ebx2_r, T r,
              uint16_t* __restrict__ codes, OutlierSink ol, uint32_t* __restrict__ g_hist, int bklen,
              uint32_t nbx, uint32_t nbricks, HostPub pub)
{
  __shared__ uint32_t s_hist[kMaxBklen];
  hist_init(s_hist, bklen);
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    const uint32_t bx = brick % nbx, by = brick / nbx;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 32;
    uint32_t cnt = 0;
    T pprev[V];
#pragma unroll
    for (int k = 0; k < V; k++) pprev[k] = 0;
    // rows are loaded in groups of 8, a group ahead: a field of a few million values gives about
    // one wave per SIMD, so a load per row would put 32 memory latencies in a row on every brick
    constexpr int G = 8;
    T raw[2][G][V];
    auto issue = [&](int g) {
#pragma unroll
      for (int j = 0; j < G; j++) {
        const uint32_t gy = y0 + g * G + j;
        bload_row<T, V>(row_rsrc(in, (size_t)gy * lx, lx), gy < ly && x0 < lx ? x0 * (uint32_t)sizeof(T) : kRowOOB,
                        raw[g & 1][j]);
      }
    };
    issue(0);
#pragma unroll
    for (int y = 0; y < 32; y++) {
      const uint32_t gy = y0 + y;
      const bool ok = gy < ly;
      const size_t base = (size_t)gy * lx;
      if (y % G == 0 && y + G < 32) issue(y / G + 1);
      T p[V];
#pragma unroll
      for (int k = 0; k < V; k++) p[k] = dround(raw[(y / G) & 1][y % G][k] * ebx2_r);
      T a[V];
#pragma unroll
      for (int k = 0; k < V; k++) a[k] = p[k] - pprev[k], pprev[k] = p[k];
      const T west = shr_in_tile<T, 1, 32 / V>(a[V - 1]);
      T d[V];
#pragma unroll
      for (int k = V - 1; k > 0; k--) d[k] = a[k] - a[k - 1];
      d[0] = (x0 % 32 != 0) ? a[0] - west : a[0];
      quantize_row<T, V, ZZ>(d, r, codes, base, x0, lx, ok, s_hist, ol, brick, cnt);
    }
    if (lane == 0) ol.brick_cnt[brick] = cnt;
  }
  hist_flush(s_hist, g_hist, bklen);
  publish_last(pub);  // the histogram to the host (pipeline.cc compress_scan)
}

// 3D: brick = (64V) x 8 x 8 (8V tiles of 8^3 along x).
template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(256)
k_lorenzo_c3d(const T* __restrict__ in, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2_r, T r,
              uint16_t* __restrict__ codes, OutlierSink ol, uint32_t* __restrict__ g_hist, int bklen,
              uint32_t nbx, uint32_t nby, uint32_t nbricks, HostPub pub)
{
  __shared__ uint32_t s_hist[kMaxBklen];
  hist_init(s_hist, bklen);
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const size_t plane = (size_t)lx * ly;
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    const uint32_t bx = brick % nbx, t = brick / nbx, by = t % nby, bz = t / nby;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 8, z0 = bz * 8;
    uint32_t cnt = 0;
    T bprev[8][V];
    for (int y = 0; y < 8; y++) {
      const uint32_t gy = y0 + y;
      if (gy >= ly) break;
      T p[8][V];
#pragma unroll
      for (int z = 0; z < 8; z++) {
        const bool ok = (z0 + z) < lz;
        load_row<T, V>(in, (size_t)(z0 + z) * plane + (size_t)gy * lx, x0, lx, ok, p[z]);
#pragma unroll
        for (int k = 0; k < V; k++) p[z][k] = dround(p[z][k] * ebx2_r);
      }
      // z-difference (descending keeps p[z-1] original); a[0] = p[0] - 0
#pragma unroll
      for (int z = 7; z > 0; z--)
#pragma unroll
        for (int k = 0; k < V; k++) p[z][k] = p[z][k] - p[z - 1][k];
      // x-difference inside 8-wide tiles
#pragma unroll
      for (int z = 0; z < 8; z++) {
        const T west = shr_in_tile<T, 1, 8 / V>(p[z][V - 1]);
#pragma unroll
        for (int k = V - 1; k > 0; k--) p[z][k] = p[z][k] - p[z][k - 1];
        if (x0 % 8 != 0) p[z][0] = p[z][0] - west;
      }
      // y-difference against the previous row of the brick
#pragma unroll
      for (int z = 0; z < 8; z++) {
        T d[V];
#pragma unroll
        for (int k = 0; k < V; k++) {
          d[k] = (y > 0) ? p[z][k] - bprev[z][k] : p[z][k];
          bprev[z][k] = p[z][k];
        }
        const bool ok = (z0 + z) < lz;
        quantize_row<T, V, ZZ>(d, r, codes, (size_t)(z0 + z) * plane + (size_t)gy * lx, x0, lx, ok,
                               s_hist, ol, brick, cnt);
      }
    }
    if (lane == 0) ol.brick_cnt[brick] = cnt;
  }
  hist_flush(s_hist, g_hist, bklen);
  publish_last(pub);  // the histogram to the host (pipeline.cc compress_scan)
}

// =========================================================================================
// reconstruct kernels.  `out` doubles as the outlier plane: the scatter kernel wrote the
// outlier values there; it is read only where code == 0, so non-outlier positions need not
// be pre-zeroed (Lorenzo).  ZigZag additionally needs a zeroed plane (code 0 = delta 0).
// =========================================================================================

// V codes packed two per u32 (prefetch registers)
template <int V>
__device__ __forceinline__ void load_codes_packed(const uint16_t* __restrict__ c, size_t base, uint32_t x0,
                                                  uint32_t lx, bool row_ok, uint32_t (&w)[(V + 1) / 2])
{
  if (row_ok && x0 + V <= lx) {
    const uint16_t* q = c + base + x0;
    if constexpr (V == 4) {
      const uint2 u = *reinterpret_cast<const uint2*>(q);
      w[0] = u.x, w[1] = u.y;
    }
    else if constexpr (V == 2) {
      w[0] = *reinterpret_cast<const uint32_t*>(q);
    }
    else {
#pragma unroll
      for (int k = 0; k < (V + 1) / 2; k++) w[k] = 0;
#pragma unroll
      for (int k = 0; k < V; k++) w[k >> 1] |= (uint32_t)q[k] << ((k & 1) * 16);
    }
  }
  else {
#pragma unroll
    for (int k = 0; k < (V + 1) / 2; k++) w[k] = 0;
#pragma unroll
    for (int k = 0; k < V; k++)
      w[k >> 1] |= (uint32_t)((row_ok && x0 + k < lx) ? c[base + x0 + k] : uint16_t(0)) << ((k & 1) * 16);
  }
}

// codes already in registers (loaded a step ahead); the outlier plane is read only where
// code == 0
template <typename T, int V, bool ZZ>
__device__ __forceinline__ void fuse_codes(const uint32_t (&w)[(V + 1) / 2], const T* plane, size_t base,
                                           uint32_t x0, uint32_t lx, bool ok, T r, T (&v)[V])
{
  uint16_t c[V];
#pragma unroll
  for (int k = 0; k < V; k++) c[k] = (uint16_t)(w[k >> 1] >> ((k & 1) * 16));
#pragma unroll
  for (int k = 0; k < V; k++) {
    const bool in = ok && (x0 + k < lx);
    T o = 0;
    if (in && c[k] == 0) o = plane[base + x0 + k];
    if constexpr (ZZ)
      v[k] = in ? o + (T)zz_dec(c[k]) : T(0);
    else
      v[k] = in ? (o + (T)c[k]) - r : T(0);
  }
}

template <typename T, int V, bool ZZ>
__device__ __forceinline__ void fuse_row(const uint16_t* __restrict__ codes, const T* plane, size_t base,
                                         uint32_t x0, uint32_t lx, bool ok, T r, T (&v)[V])
{
  uint16_t c[V];
  load_codes<V>(codes, base, x0, lx, ok, c);
#pragma unroll
  for (int k = 0; k < V; k++) {
    const bool in = ok && (x0 + k < lx);
    T o = 0;
    if (in && c[k] == 0) o = plane[base + x0 + k];
    if constexpr (ZZ)
      v[k] = in ? o + (T)zz_dec(c[k]) : T(0);
    else
      v[k] = in ? (o + (T)c[k]) - r : T(0);
  }
}

template <typename T, bool ZZ>
__global__ void __launch_bounds__(256)
k_lorenzo_x1d(const uint16_t* __restrict__ codes, T* out, size_t n, T ebx2, T r, uint32_t nbricks, X1dOutliers ox)
{
  constexpr int V = 4;  // the reference thread owns 4 consecutive elements (launch.hh:124-132)
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  // outlier values from the sorted cells (see X1dOutliers) instead of the scattered `out`
  const bool fused = !ZZ && ox.cells && *ox.unsorted != ox.epoch;
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    const size_t bbase = (size_t)brick * 16384;
    T carry = 0;
    const uint32_t x0 = lane * V;
    // pipelined row loop: codes arrive two rows ahead, the outlier values (read from `out`
    // where the code is 0, or from the cells) one row ahead, so no row waits on a load it has
    // just issued
    auto rlen = [&](size_t b0) { return (uint32_t)(n - b0 < 256 ? n - b0 : 256); };
    size_t cp = fused ? ox.bstart[brick] : 0;  // next cell of this brick
    // one past the brick's last cell: a brick with fewer cells than zero codes (outliers dropped
    // at the cap, always an index-order suffix) reads 0 for the missing ones, as the scatter
    // path does, and never reaches into the next brick's cells
    const size_t cend = fused ? ox.bstart[brick + 1] : 0;
    auto outliers = [&](const uint16_t (&c)[V], size_t b0, T (&o)[V]) {
      const uint32_t len = rlen(b0);
      if (!fused) {
#pragma unroll
        for (int k = 0; k < V; k++) o[k] = (x0 + k < len && c[k] == 0) ? out[b0 + x0 + k] : T(0);
        return;
      }
      // rank of each zero code in (lane, k) = index order: zeros of lower lanes, then of lower k
      bool z[V];
      uint32_t below = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < V; k++) {
        z[k] = x0 + k < len && c[k] == 0;
        const uint64_t m = __ballot(z[k]);
        below += __popcll(m & lt), tot += __popcll(m);
      }
      uint32_t rank = below;
#pragma unroll
      for (int k = 0; k < V; k++) {
        T v = 0;
        if (z[k]) {
          const size_t j = cp + rank;
          if (j < cend) v = (T)__builtin_bit_cast(float, ox.cells[2 * j]);
          rank++;
        }
        o[k] = v;
      }
      cp += tot;
    };
    uint16_t c1[V], c2[V];
    T o1[V];
    load_codes<V>(codes, bbase, x0, rlen(bbase), true, c1);
    if (bbase + 256 < n) load_codes<V>(codes, bbase + 256, x0, rlen(bbase + 256), true, c2);
    outliers(c1, bbase, o1);
    for (int s = 0; s < 64; s++) {
      const size_t base = bbase + (size_t)s * 256;
      if (base >= n) break;
      const uint32_t rowlen = rlen(base);
      uint16_t c[V];
      T o[V];
#pragma unroll
      for (int k = 0; k < V; k++) c[k] = c1[k], o[k] = o1[k];
      const size_t b1 = base + 256, b2 = base + 512;
      if (s < 63 && b1 < n) {
#pragma unroll
        for (int k = 0; k < V; k++) c1[k] = c2[k];
        outliers(c1, b1, o1);
        if (s < 62 && b2 < n) load_codes<V>(codes, b2, x0, rlen(b2), true, c2);
      }
      T b[V];
#pragma unroll
      for (int k = 0; k < V; k++) {
        const bool in = x0 + k < rowlen;
        if constexpr (ZZ)
          b[k] = in ? o[k] + (T)zz_dec(c[k]) : T(0);
        else
          b[k] = in ? (o[k] + (T)c[k]) - r : T(0);
      }
      // per-thread sequential scan (wave32.cuhip.inl:10)
#pragma unroll
      for (int k = 1; k < V; k++) b[k] = b[k] + b[k - 1];
      // 32-lane Hillis-Steele over thread totals (wave32.cuhip.inl:14-17)
      T addend = b[V - 1];
#pragma unroll
      for (int d = 1; d < 32; d *= 2) {
        T nb = __shfl_up(addend, d, 32);
        if ((lane & 31) >= d) addend = addend + nb;
      }
      const T prev = __shfl_up(addend, 1, 32);
      if ((lane & 31) > 0)
#pragma unroll
        for (int k = 0; k < V; k++) b[k] = b[k] + prev;
      // cross-warp serial exclusive scan over the tile's 8 warps (wave32.cuhip.inl:38-42)
      const T tot0 = __shfl(b[V - 1], 31), tot1 = __shfl(b[V - 1], 63);
      if ((s & 3) == 0) carry = 0;
      const T c0 = carry, c1 = c0 + tot0;
      const T add = lane < 32 ? c0 : c1;
#pragma unroll
      for (int k = 0; k < V; k++) b[k] = (b[k] + add) * ebx2;
      carry = c1 + tot1;
      store_row<T, V>(out, base, x0, rowlen, true, b);
    }
  }
}

template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(256)
k_lorenzo_x2d(const uint16_t* __restrict__ codes, T* out, uint32_t lx, uint32_t ly, T ebx2, T r,
              uint32_t nbx, uint32_t nbricks)
{
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    const uint32_t bx = brick % nbx, by = brick / nbx;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 32;
    T s[V], S0[V], acc1[V], acc2[V];
    // codes are loaded in groups of 8 rows, a group ahead (see k_lorenzo_c2d); a group with a
    // zero code (an outlier) reads those values from the plane, in a branch that waits for them
    constexpr int G = 8, W = (V + 1) / 2;
    uint32_t cw[2][G][W];
    auto issue = [&](int g) {
#pragma unroll
      for (int j = 0; j < G; j++) {
        const uint32_t gy = y0 + g * G + j;
        bload_codes<V>(row_rsrc(codes, (size_t)gy * lx, lx), gy < ly && x0 < lx ? x0 * 2u : kRowOOB, cw[g & 1][j]);
      }
    };
    issue(0);
    T val[G][V];  // the current group's values (o + c) - r
#pragma unroll
    for (int y = 0; y < 32; y++) {
      const uint32_t gy = y0 + y;
      const bool ok = gy < ly;
      const size_t base = (size_t)gy * lx;
      if (y % G == 0) {
        if (y + G < 32) issue(y / G + 1);
        const int g = y / G;
        bool anyz = false;
#pragma unroll
        for (int j = 0; j < G; j++)
#pragma unroll
          for (int k = 0; k < V; k++) {
            const uint32_t c = (cw[g & 1][j][k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
            const bool in = y0 + g * G + j < ly && x0 + k < lx;
            if constexpr (ZZ)
              val[j][k] = in ? T(0) + (T)zz_dec((uint16_t)c) : T(0);
            else
              val[j][k] = in ? (T(0) + (T)c) - r : T(0);
            anyz |= in && c == 0;
          }
        if (__ballot(anyz)) {
#pragma unroll
          for (int j = 0; j < G; j++)
            fuse_codes<T, V, ZZ>(cw[g & 1][j], out, (size_t)(y0 + g * G + j) * lx, x0, lx, y0 + g * G + j < ly, r,
                                 val[j]);
        }
      }
      T v[V];
#pragma unroll
      for (int k = 0; k < V; k++) v[k] = val[y % G][k];
      const int strip = y >> 3;
      T t[V];
#pragma unroll
      for (int k = 0; k < V; k++) {
        s[k] = (y & 7) ? v[k] + s[k] : v[k];  // per-strip sequential scan (lrz_x:214)
        if (strip == 0)
          t[k] = s[k];
        else if (strip == 1)
          t[k] = s[k] + S0[k];
        else if (strip == 2)
          t[k] = s[k] + acc1[k];
        else
          t[k] = s[k] + acc2[k];
        if ((y & 7) == 7) {  // strip totals -> cross-strip addends (lrz_x:217-236)
          if (strip == 0) S0[k] = s[k];
          if (strip == 1) acc1[k] = s[k] + S0[k];
          if (strip == 2) acc2[k] = s[k] + acc1[k];
        }
      }
      // 32-wide Hillis-Steele along x (lrz_x:247-253)
      hs_step<T, V, 32, 1>(t, x0);
      hs_step<T, V, 32, 2>(t, x0);
      hs_step<T, V, 32, 4>(t, x0);
      hs_step<T, V, 32, 8>(t, x0);
      hs_step<T, V, 32, 16>(t, x0);
#pragma unroll
      for (int k = 0; k < V; k++) t[k] = t[k] * ebx2;
      store_row<T, V>(out, base, x0, lx, ok, t);
    }
  }
}

template <typename T, int V, bool ZZ>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_lorenzo_x3d(const uint16_t* __restrict__ codes, T* out, uint32_t lx, uint32_t ly, uint32_t lz, T ebx2,
              T r, uint32_t nbx, uint32_t nby, uint32_t nbricks)
{
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const size_t plane = (size_t)lx * ly;
  for (uint32_t brick = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); brick < nbricks; brick += nw) {
    const uint32_t bx = brick % nbx, tt = brick / nbx, by = tt % nby, bz = tt / nby;
    const uint32_t x0 = bx * (64 * V) + lane * V, y0 = by * 8, z0 = bz * 8;
    T s[8][V];
    // codes are loaded one y-step ahead so a step waits at most for its (rare) outlier reads
    constexpr int W = (V + 1) / 2;
    uint32_t cn[8][W];
#pragma unroll
    for (int z = 0; z < 8; z++)
      load_codes_packed<V>(codes, (size_t)(z0 + z) * plane + (size_t)y0 * lx, x0, lx, (z0 + z) < lz && y0 < ly,
                           cn[z]);
    for (int y = 0; y < 8; y++) {
      const uint32_t gy = y0 + y;
      if (gy >= ly) break;
      uint32_t cc[8][W];
#pragma unroll
      for (int z = 0; z < 8; z++)
#pragma unroll
        for (int k = 0; k < W; k++) cc[z][k] = cn[z][k];
      if (y + 1 < 8) {
        const bool nok = gy + 1 < ly;
#pragma unroll
        for (int z = 0; z < 8; z++)
          load_codes_packed<V>(codes, (size_t)(z0 + z) * plane + (size_t)(gy + 1) * lx, x0, lx,
                               nok && (z0 + z) < lz, cn[z]);
      }
      T t[8][V];
#pragma unroll
      for (int z = 0; z < 8; z++) {
        const bool ok = (z0 + z) < lz;
        T v[V];
        fuse_codes<T, V, ZZ>(cc[z], out, (size_t)(z0 + z) * plane + (size_t)gy * lx, x0, lx, ok, r, v);
#pragma unroll
        for (int k = 0; k < V; k++) {
          s[z][k] = (y > 0) ? v[k] + s[z][k] : v[k];  // y sequential (lrz_x:315)
          t[z][k] = s[z][k];
        }
      }
      // x Hillis-Steele within 8-wide tiles (lrz_x:324-327)
#pragma unroll
      for (int z = 0; z < 8; z++) {
        hs_step<T, V, 8, 1>(t[z], x0);
        hs_step<T, V, 8, 2>(t[z], x0);
        hs_step<T, V, 8, 4>(t[z], x0);
      }
      // z Hillis-Steele (lrz_x:335-338), in-lane; descending z keeps sources unmodified
#pragma unroll
      for (int d = 1; d < 8; d *= 2)
#pragma unroll
        for (int z = 7; z >= d; z--)
#pragma unroll
          for (int k = 0; k < V; k++) t[z][k] = t[z][k] + t[z - d][k];
#pragma unroll
      for (int z = 0; z < 8; z++) {
#pragma unroll
        for (int k = 0; k < V; k++) t[z][k] = t[z][k] * ebx2;
        store_row<T, V>(out, (size_t)(z0 + z) * plane + (size_t)gy * lx, x0, lx, (z0 + z) < lz, t[z]);
      }
    }
  }
}

// outlier scatter (spvn.cuhip.inl:41-50): cells are {f32 val, u32 idx}, 4-byte aligned in
// the archive (read as two u32).
template <typename T>
__global__ void __launch_bounds__(256)
k_scatter(const uint32_t* __restrict__ cells, size_t nnz, T* out, size_t n, const uint32_t* only_if, uint32_t epoch)
{
  if (only_if && *only_if != epoch) return;  // the 1-D reconstruction reads the sorted cells itself
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nnz; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t vb = cells[2 * i], idx = cells[2 * i + 1];
    if (idx < n) out[idx] = (T)__builtin_bit_cast(float, vb);
  }
}

// first cell of every 1-D brick (16384 elements) and whether the cells are strictly increasing
// (every bstart entry is written when the cells are sorted; *unsorted = epoch otherwise)
__global__ void __launch_bounds__(256) k_x1d_bounds(const uint32_t* __restrict__ cells, size_t ncell, size_t n,
                                                    uint32_t nbricks, uint32_t* bstart, uint32_t* unsorted,
                                                    uint32_t epoch, uint32_t ushift)
{
  // cell i's index against its predecessor's (ip, read only when i > 0)
  auto cell = [&](size_t i, uint32_t idx, uint32_t ip) {
    const int64_t b = idx < n ? (int64_t)(idx >> ushift) : (int64_t)nbricks;
    int64_t bp = -1;
    if (i > 0) {
      if (ip >= idx) *unsorted = epoch;
      bp = ip < n ? (int64_t)(ip >> ushift) : (int64_t)nbricks;
    }
    if (idx >= n) *unsorted = epoch;
    for (int64_t u = bp + 1; u <= b && u <= (int64_t)nbricks; u++) bstart[u] = (uint32_t)i;
    if (i + 1 == ncell)
      for (int64_t u = b + 1; u <= (int64_t)nbricks; u++) bstart[u] = (uint32_t)ncell;
  };
  // four cells per thread and step (two 16-B loads; the predecessor's index from the cache), up
  // to 2^28 cells (32-bit buffer offsets); the rest one by one
  const size_t nq = ncell < (1u << 28) ? ncell / 4 : 0;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(cells), 0, (int)(nq * 32u), 0x00020000);
  for (size_t q = blockIdx.x * (size_t)256 + threadIdx.x; q < nq; q += (size_t)gridDim.x * 256) {
    typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
    const u32x4v v0 = __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(q * 32u), 0, 0);
    const u32x4v v1 = __builtin_amdgcn_raw_buffer_load_b128(rc, (int)(q * 32u + 16u), 0, 0);
    const uint32_t ip = q > 0 ? __builtin_amdgcn_raw_buffer_load_b32(rc, (int)(q * 32u - 4u), 0, 0) : 0u;
    const size_t i = 4 * q;
    cell(i, v0.y, ip);
    cell(i + 1, v0.w, v0.y);
    cell(i + 2, v1.y, v0.w);
    cell(i + 3, v1.w, v1.y);
  }
  for (size_t i = 4 * nq + blockIdx.x * (size_t)256 + threadIdx.x; i < ncell; i += (size_t)gridDim.x * 256)
    cell(i, cells[2 * i + 1], i > 0 ? cells[2 * i - 1] : 0u);
}

// =========================================================================================
// host launchers
// =========================================================================================

static inline uint32_t cdiv(size_t a, size_t b) { return (uint32_t)((a + b - 1) / b); }

static int grid_for(uint32_t nbricks)
{
  const uint32_t waves = nbricks;
  uint32_t g = (waves + 3) / 4;
  return (int)(g < 4096 ? (g ? g : 1) : 4096);
}

LorenzoGeom lorenzo_geom(int ndim, size_t lx, size_t ly, size_t lz, int elem_bytes)
{
  LorenzoGeom g{};
  g.ndim = ndim;
  if (ndim == 1) {
    g.V = 4;
    g.nbx = cdiv(lx * ly * lz, 16384), g.nby = 1, g.nbz = 1;
    g.brick_elems = 16384;
  }
  else {
    int V = 1;
    if (elem_bytes == 4 && lx % 4 == 0) V = 4;
    else if (elem_bytes == 8 && lx % 2 == 0) V = 2;
    else if (elem_bytes == 4 && lx % 2 == 0) V = 2;
    g.V = V;
    g.nbx = cdiv(lx, 64 * V);
    if (ndim == 2) g.nby = cdiv(ly, 32), g.nbz = 1, g.brick_elems = 64 * V * 32;
    else g.nby = cdiv(ly, 8), g.nbz = cdiv(lz, 8), g.brick_elems = 64 * V * 64;
  }
  g.nbricks = g.nbx * g.nby * g.nbz;
  return g;
}

#define DISPATCH_V(V, ...)                       \
  switch (V) {                                   \
    case 4: { constexpr int VV = 4; __VA_ARGS__; } break; \
    case 2: { constexpr int VV = 2; __VA_ARGS__; } break; \
    default: { constexpr int VV = 1; __VA_ARGS__; } break; \
  }

template <typename T>
int launch_lorenzo_c(const T* in, size_t lx, size_t ly, size_t lz, double eb, int radius, bool zigzag,
                     const LorenzoGeom& g, uint16_t* codes, const OutlierSink& ol, uint32_t* hist,
                     int bklen, hipStream_t st, const HostPub& pub)
{
  const T ebx2_r = (T)(1.0 / (eb * 2));  // lrz_c.cuhip.inl:489
  const T r = (T)radius;
  const int grid = grid_for(g.nbricks);
  if (g.ndim == 1) {
    if (zigzag)
      k_lorenzo_c1d<T, true><<<grid, 256, 0, st>>>(in, lx, ebx2_r, r, codes, ol, hist, bklen, g.nbricks, pub);
    else
      k_lorenzo_c1d<T, false><<<grid, 256, 0, st>>>(in, lx, ebx2_r, r, codes, ol, hist, bklen, g.nbricks, pub);
  }
  else if (g.ndim == 2) {
    if (lx * sizeof(T) >= 0x80000000ull) return (int)hipErrorInvalidValue;  // row_rsrc range
    DISPATCH_V(g.V, if (zigzag) k_lorenzo_c2d<T, VV, true><<<grid, 256, 0, st>>>(
                        in, lx, ly, ebx2_r, r, codes, ol, hist, bklen, g.nbx, g.nbricks, pub);
               else k_lorenzo_c2d<T, VV, false><<<grid, 256, 0, st>>>(
                   in, lx, ly, ebx2_r, r, codes, ol, hist, bklen, g.nbx, g.nbricks, pub));
  }
  else {
    DISPATCH_V(g.V, if (zigzag) k_lorenzo_c3d<T, VV, true><<<grid, 256, 0, st>>>(
                        in, lx, ly, lz, ebx2_r, r, codes, ol, hist, bklen, g.nbx, g.nby, g.nbricks, pub);
               else k_lorenzo_c3d<T, VV, false><<<grid, 256, 0, st>>>(
                   in, lx, ly, lz, ebx2_r, r, codes, ol, hist, bklen, g.nbx, g.nby, g.nbricks, pub));
  }
  return (int)hipGetLastError();
}

template <typename T>
int launch_lorenzo_x(const uint16_t* codes, T* out, size_t lx, size_t ly, size_t lz, double eb, int radius,
                     bool zigzag, const LorenzoGeom& g, hipStream_t st, const X1dOutliers* ox)
{
  const T ebx2 = (T)(eb * 2);  // lrz_x.cuhip.inl:432
  const T r = (T)radius;
  const int grid = grid_for(g.nbricks);
  if (g.ndim == 1) {
    const X1dOutliers o = ox ? *ox : X1dOutliers{};
    if (zigzag)
      k_lorenzo_x1d<T, true><<<grid, 256, 0, st>>>(codes, out, lx, ebx2, r, g.nbricks, o);
    else
      k_lorenzo_x1d<T, false><<<grid, 256, 0, st>>>(codes, out, lx, ebx2, r, g.nbricks, o);
  }
  else if (g.ndim == 2) {
    if (lx * sizeof(T) >= 0x80000000ull) return (int)hipErrorInvalidValue;  // row_rsrc range
    DISPATCH_V(g.V, if (zigzag) k_lorenzo_x2d<T, VV, true><<<grid, 256, 0, st>>>(
                        codes, out, lx, ly, ebx2, r, g.nbx, g.nbricks);
               else k_lorenzo_x2d<T, VV, false><<<grid, 256, 0, st>>>(codes, out, lx, ly, ebx2, r,
                                                                        g.nbx, g.nbricks));
  }
  else {
    DISPATCH_V(g.V, if (zigzag) k_lorenzo_x3d<T, VV, true><<<grid, 256, 0, st>>>(
                        codes, out, lx, ly, lz, ebx2, r, g.nbx, g.nby, g.nbricks);
               else k_lorenzo_x3d<T, VV, false><<<grid, 256, 0, st>>>(
                   codes, out, lx, ly, lz, ebx2, r, g.nbx, g.nby, g.nbricks));
  }
  return (int)hipGetLastError();
}

template <typename T>
int launch_scatter(const uint32_t* cells, size_t nnz, T* out, size_t n, hipStream_t st, const uint32_t* only_if,
                   uint32_t epoch)
{
  if (nnz == 0) return 0;
  uint32_t grid = cdiv(nnz, 256);
  if (grid > 4096) grid = 4096;
  k_scatter<T><<<grid, 256, 0, st>>>(cells, nnz, out, n, only_if, epoch);
  return (int)hipGetLastError();
}

int launch_x1d_bounds(const uint32_t* cells, size_t ncell, size_t n, uint32_t nbricks, uint32_t* bstart,
                      uint32_t* unsorted, uint32_t epoch, hipStream_t st, uint32_t ushift)
{
  if (ncell == 0) return 0;
  uint32_t grid = cdiv((ncell + 3) / 4, 256);
  if (grid > 4096) grid = 4096;
  k_x1d_bounds<<<grid, 256, 0, st>>>(cells, ncell, n, nbricks, bstart, unsorted, epoch, ushift);
  return (int)hipGetLastError();
}

template int launch_lorenzo_c<float>(const float*, size_t, size_t, size_t, double, int, bool,
                                     const LorenzoGeom&, uint16_t*, const OutlierSink&, uint32_t*, int,
                                     hipStream_t, const HostPub&);
template int launch_lorenzo_c<double>(const double*, size_t, size_t, size_t, double, int, bool,
                                      const LorenzoGeom&, uint16_t*, const OutlierSink&, uint32_t*, int,
                                      hipStream_t, const HostPub&);
template int launch_lorenzo_x<float>(const uint16_t*, float*, size_t, size_t, size_t, double, int, bool,
                                     const LorenzoGeom&, hipStream_t, const X1dOutliers*);
template int launch_lorenzo_x<double>(const uint16_t*, double*, size_t, size_t, size_t, double, int, bool,
                                      const LorenzoGeom&, hipStream_t, const X1dOutliers*);
template int launch_scatter<float>(const uint32_t*, size_t, float*, size_t, hipStream_t, const uint32_t*, uint32_t);
template int launch_scatter<double>(const uint32_t*, size_t, double*, size_t, hipStream_t, const uint32_t*, uint32_t);

}  // namespace cusz_amd
