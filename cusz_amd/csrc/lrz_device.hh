// cusz_amd/csrc/lrz_device.hh -- Lorenzo device helpers shared by lorenzo.hip (brick-wise
// kernels over a code buffer) and brick.hip (fused predict+encode / decode+reconstruct).
//
// Semantics restate the reference GPU kernels: prequant/quantize lrz_c.cuhip.inl:50-89,
// 216-260, 305-331; ZigZag composite.hh:61-84; reconstruct scans lrz_x.cuhip.inl +
// wave32.cuhip.inl:7-66.
#pragma once

#include "common.hh"
#include "kernels.hh"

namespace cusz_amd {
namespace lrzd {

template <typename T>
__device__ __forceinline__ T dround(T v);
template <>
__device__ __forceinline__ float dround<float>(float v)
{
  // roundf (half away from zero) as trunc(v + copysign(pred(0.5), v)): 3 VALU instead of 6;
  // identical for every f32 (checked exhaustively on the host), including -0, ties and |v| >= 2^23
  return __builtin_truncf(v + __builtin_copysignf(0.49999997f, v));
}
template <>
__device__ __forceinline__ double dround<double>(double v) { return round(v); }

template <typename T>
__device__ __forceinline__ T dabs(T v);
template <>
__device__ __forceinline__ float dabs<float>(float v) { return fabsf(v); }
template <>
__device__ __forceinline__ double dabs<double>(double v) { return fabs(v); }

__device__ __forceinline__ uint16_t zz_enc(int16_t v)
{  // composite.hh:61-70
  return (uint16_t)(((uint16_t)v << 1) ^ (uint16_t)(v >> 15));
}
__device__ __forceinline__ int16_t zz_dec(uint16_t u)
{  // composite.hh:72-83
  return (int16_t)((u >> 1) ^ (uint16_t)(-(int16_t)(u & 1)));
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// value of lane (l - L) when both lanes lie in the same TILE_LANES-aligned group.  Groups of
// <= 16 lanes never cross a DPP row, so a row_shr:L DPP move does it in one VALU op (no LDS
// permute); wider groups fall back to ds_bpermute (__shfl_up).
template <int L>
__device__ __forceinline__ int dpp_shr(int v)
{
  static_assert(L >= 1 && L <= 15, "row_shr range");
  return __builtin_amdgcn_update_dpp(0, v, 0x110 + L, 0xf, 0xf, false);
}

template <typename T, int L, int TILE_LANES>
__device__ __forceinline__ T shr_in_tile(T v)
{
  if constexpr (TILE_LANES <= 16) {
    if constexpr (sizeof(T) == 4)
      return __builtin_bit_cast(T, dpp_shr<L>(__builtin_bit_cast(int, v)));
    else {
      const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
      const int lo = dpp_shr<L>((int)(uint32_t)u), hi = dpp_shr<L>((int)(uint32_t)(u >> 32));
      return __builtin_bit_cast(T, (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32));
    }
  }
  else
    return __shfl_up(v, L);
}

__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// ---- vector row I/O -------------------------------------------------------------------
template <typename T, int V>
__device__ __forceinline__ void load_row(const T* __restrict__ p, size_t base, uint32_t x0, uint32_t lx,
                                         bool row_ok, T (&v)[V])
{
  if (row_ok && x0 + V <= lx) {
    const T* q = p + base + x0;
    if constexpr (sizeof(T) * V == 16) {
      auto w = *reinterpret_cast<const uint4*>(q);
      __builtin_memcpy(&v[0], &w, 16);
    }
    else if constexpr (sizeof(T) * V == 8) {
      auto w = *reinterpret_cast<const uint2*>(q);
      __builtin_memcpy(&v[0], &w, 8);
    }
    else if constexpr (sizeof(T) * V == 32) {
      auto w0 = reinterpret_cast<const uint4*>(q)[0];
      auto w1 = reinterpret_cast<const uint4*>(q)[1];
      __builtin_memcpy(&v[0], &w0, 16);
      __builtin_memcpy(reinterpret_cast<char*>(&v[0]) + 16, &w1, 16);
    }
    else {
#pragma unroll
      for (int k = 0; k < V; k++) v[k] = q[k];
    }
  }
  else {
#pragma unroll
    for (int k = 0; k < V; k++) v[k] = (row_ok && x0 + k < lx) ? p[base + x0 + k] : T(0);
  }
}

template <int V>
__device__ __forceinline__ void load_codes(const uint16_t* __restrict__ c, size_t base, uint32_t x0,
                                           uint32_t lx, bool row_ok, uint16_t (&v)[V])
{
  if (row_ok && x0 + V <= lx) {
    const uint16_t* q = c + base + x0;
    if constexpr (V == 4) {
      auto w = *reinterpret_cast<const uint2*>(q);
      __builtin_memcpy(&v[0], &w, 8);
    }
    else if constexpr (V == 2) {
      auto w = *reinterpret_cast<const uint32_t*>(q);
      __builtin_memcpy(&v[0], &w, 4);
    }
    else {
#pragma unroll
      for (int k = 0; k < V; k++) v[k] = q[k];
    }
  }
  else {
#pragma unroll
    for (int k = 0; k < V; k++) v[k] = (row_ok && x0 + k < lx) ? c[base + x0 + k] : uint16_t(0);
  }
}

template <int V>
__device__ __forceinline__ void store_codes(uint16_t* __restrict__ c, size_t base, uint32_t x0,
                                            uint32_t lx, bool row_ok, const uint16_t (&v)[V])
{
  if (!row_ok) return;
  if (x0 + V <= lx) {
    uint16_t* q = c + base + x0;
    if constexpr (V == 4) {
      uint2 w;
      __builtin_memcpy(&w, &v[0], 8);
      *reinterpret_cast<uint2*>(q) = w;
    }
    else if constexpr (V == 2) {
      uint32_t w;
      __builtin_memcpy(&w, &v[0], 4);
      *reinterpret_cast<uint32_t*>(q) = w;
    }
    else {
#pragma unroll
      for (int k = 0; k < V; k++) q[k] = v[k];
    }
  }
  else {
#pragma unroll
    for (int k = 0; k < V; k++)
      if (x0 + k < lx) c[base + x0 + k] = v[k];
  }
}

template <typename T, int V>
__device__ __forceinline__ void store_row(T* __restrict__ p, size_t base, uint32_t x0, uint32_t lx,
                                          bool row_ok, const T (&v)[V])
{
  if (!row_ok) return;
  if (x0 + V <= lx) {
    T* q = p + base + x0;
    if constexpr (sizeof(T) * V == 16) {
      uint4 w;
      __builtin_memcpy(&w, &v[0], 16);
      *reinterpret_cast<uint4*>(q) = w;
    }
    else if constexpr (sizeof(T) * V == 8) {
      uint2 w;
      __builtin_memcpy(&w, &v[0], 8);
      *reinterpret_cast<uint2*>(q) = w;
    }
    else if constexpr (sizeof(T) * V == 32) {
      uint4 w0, w1;
      __builtin_memcpy(&w0, &v[0], 16);
      __builtin_memcpy(&w1, reinterpret_cast<const char*>(&v[0]) + 16, 16);
      reinterpret_cast<uint4*>(q)[0] = w0;
      reinterpret_cast<uint4*>(q)[1] = w1;
    }
    else {
#pragma unroll
      for (int k = 0; k < V; k++) q[k] = v[k];
    }
  }
  else {
#pragma unroll
    for (int k = 0; k < V; k++)
      if (x0 + k < lx) p[base + x0 + k] = v[k];
  }
}

// ---- quantization + outlier/histogram side effects -------------------------------------
// lrz_c.cuhip.inl:310-331: code = (|d| < r) ? (u2)(d + r) : 0; outlier cell {(f4)(d + r), idx}
// (ZigZag: code = zz((i16)(q*d)), cell val (f4)d).
template <typename T, bool ZZ>
__device__ __forceinline__ uint16_t quantize(T d, T r, bool& ol, float& olval)
{
  bool q = dabs(d) < r;
  ol = !q;
  if constexpr (ZZ) {
    olval = (float)d;
    return q ? zz_enc((int16_t)(int)d) : uint16_t(0);
  }
  else {
    T c = d + r;
    olval = (float)c;
    return q ? (uint16_t)(int)c : uint16_t(0);
  }
}

// Rare path of emit_outliers: some cells of this row go past the brick's slot.  The row's cells
// past the slot take ONE reservation on the spill counter per wave (a ballot prefix gives each
// lane its place): an outlier-dominated field (Nyx velocities at abs 1e-4) would otherwise issue
// one returning atomic per element on a single word.  Called with the wave's active lanes of
// emit_outliers (the whole row).
template <int V>
__device__ __forceinline__ void emit_outliers_spill(const OutlierSink& ol, uint32_t brick, uint32_t pos,
                                                              uint32_t mask, const float (&val)[V],
                                                              const size_t (&idx)[V])
{
  static_assert(V <= 15, "4 ballots count a lane's spilled cells");
  uint64_t* slot = ol.slots + (size_t)brick * ol.cap_per_brick;
  const uint32_t cap = ol.cap_per_brick, c = (uint32_t)__popc(mask);
  const uint32_t nsp = pos >= cap ? c : (pos + c > cap ? pos + c - cap : 0u);  // this lane's spilled cells
  const uint64_t b0 = __ballot(nsp & 1u), b1 = __ballot(nsp & 2u), b2 = __ballot(nsp & 4u), b3 = __ballot(nsp & 8u);
  const uint64_t lt = lanemask_lt();
  const uint32_t excl = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt) + 8 * __popcll(b3 & lt);
  const uint32_t tot = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2) + 8 * __popcll(b3);
  const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
  uint32_t s0 = 0;
  if (lane_id() == leader) s0 = atomicAdd(ol.spill_cnt, tot);
  uint32_t s = (uint32_t)__shfl((int)s0, leader) + excl;
#pragma unroll
  for (int k = 0; k < V; k++) {
    if ((mask >> k) & 1u) {
      const uint64_t cell = make_cell(val[k], (uint32_t)idx[k]);
      if (pos < cap)
        slot[pos] = cell;
      else {
        if (s < ol.spill_cap) ol.spill[s] = cell;
        s++;
      }
      pos++;
    }
  }
}

// Emit the outliers of one wave row in (lane, k) order into the brick's slot.
template <int V>
__device__ __forceinline__ void emit_outliers(const OutlierSink& ol, uint32_t brick, uint32_t& cnt,
                                              uint32_t mask, const float (&val)[V],
                                              const size_t (&idx)[V])
{
  const int c = __popc(mask);
  const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
  const uint64_t lt = lanemask_lt();
  uint32_t pos = cnt + __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
  const uint32_t tot = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  if (__builtin_expect(cnt + tot <= ol.cap_per_brick, 1)) {  // uniform: the whole row fits the slot
    uint64_t* slot = ol.slots + (size_t)brick * ol.cap_per_brick;
#pragma unroll
    for (int k = 0; k < V; k++)
      if ((mask >> k) & 1u) slot[pos++] = make_cell(val[k], (uint32_t)idx[k]);
  }
  else
    emit_outliers_spill<V>(ol, brick, pos, mask, val, idx);
  cnt += tot;
}

// emit_outliers for a lane's V consecutive elements base .. base + V - 1 (32-bit indices)
template <int V>
__device__ __forceinline__ void emit_outliers32(const OutlierSink& ol, uint32_t brick, uint32_t& cnt, uint32_t mask,
                                                const float (&val)[V], uint32_t base)
{
  size_t idx[V];
#pragma unroll
  for (int k = 0; k < V; k++) idx[k] = base + (uint32_t)k;
  emit_outliers<V>(ol, brick, cnt, mask, val, idx);
}

// Quantize one row of V elements (in-range mask), store codes, histogram, outliers.
template <typename T, int V, bool ZZ>
__device__ __forceinline__ void quantize_row(const T (&d)[V], T r, uint16_t* __restrict__ codes,
                                             size_t base, uint32_t x0, uint32_t lx, bool row_ok,
                                             uint32_t* s_hist, const OutlierSink& ol, uint32_t brick,
                                             uint32_t& cnt)
{
  uint16_t q[V];
  float olv[V];
  size_t idx[V];
  uint32_t mask = 0;
#pragma unroll
  for (int k = 0; k < V; k++) {
    bool is_ol;
    q[k] = quantize<T, ZZ>(d[k], r, is_ol, olv[k]);
    idx[k] = base + x0 + k;
    const bool in = row_ok && (x0 + k < lx);
    if (in) atomicAdd(&s_hist[q[k]], 1u);
    mask |= (uint32_t)(in && is_ol) << k;
  }
  store_codes<V>(codes, base, x0, lx, row_ok, q);
  if (__ballot(mask != 0)) emit_outliers<V>(ol, brick, cnt, mask, olv, idx);
}

__device__ __forceinline__ void hist_init(uint32_t* s_hist, int bklen)
{
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) s_hist[i] = 0;
  __syncthreads();
}

__device__ __forceinline__ void hist_flush(uint32_t* s_hist, uint32_t* g_hist, int bklen)
{
  __syncthreads();
  for (int i = threadIdx.x; i < bklen; i += blockDim.x) {
    uint32_t v = s_hist[i];
    if (v) atomicAdd(&g_hist[i], v);
  }
}

// Hillis-Steele step of the reference's shuffle scans (val += shfl_up(val, D) when the
// in-tile position >= D), for a lane holding V consecutive positions of a TW-wide tile.
template <typename T, int V, int TW, int D>
__device__ __forceinline__ void hs_step(T (&t)[V], uint32_t x0)
{
  T old[V];
#pragma unroll
  for (int k = 0; k < V; k++) old[k] = t[k];
#pragma unroll
  for (int k = 0; k < V; k++) {
    const int kk = k - D;
    T src;
    if (kk >= 0)
      src = old[kk >= 0 ? kk : 0];
    else {
      constexpr int TL = TW / V;  // lanes per tile
      const int L = (-kk + V - 1) / V;
      const int k2 = kk + L * V;
      if (L == 1) src = shr_in_tile<T, 1, TL>(old[k2]);
      else if (L == 2) src = shr_in_tile<T, 2, TL>(old[k2]);
      else if (L == 3) src = shr_in_tile<T, 3, TL>(old[k2]);
      else if (L == 4) src = shr_in_tile<T, 4, TL>(old[k2]);
      else if (L == 8) src = shr_in_tile<T, 8, TL>(old[k2]);
      else src = __shfl_up(old[k2], L);
    }
    const uint32_t px = (x0 + k) % TW;
    if (px >= (uint32_t)D) t[k] = old[k] + src;
  }
}

}  // namespace lrzd
}  // namespace cusz_amd
