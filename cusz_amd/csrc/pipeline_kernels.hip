// cusz_amd/csrc/pipeline_kernels.hip -- small device-side glue of the compress pipeline:
// archive finalisation (segment sizes, outlier compaction, headers) and the Rel-mode
// extrema probe.  Everything stays on the device; the host reads back one header at the end.
//
// Reference counterparts: compress wrap-up psz/src/compressor.inl:398-418 (D2D concat),
// phf header/offsets codec/hf/src/hf_buf.cc:191-211, GPU_extrema
// psz/src/stat/detail/extrema.cuhip.inl:86-208.
#include <algorithm>

#include "archive_device.hh"
#include "common.hh"
#include "hf_device.hh"
#include "kernels.hh"
#include "pub_device.hh"

namespace cusz_amd {

namespace {

__device__ __forceinline__ unsigned long long wsum64(unsigned long long v)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// sum of per-chunk bit counts: many blocks, one 64-bit atomic each (total_nbit zeroed before)
__global__ void __launch_bounds__(256) k_sum_nbit(const uint32_t* __restrict__ par_nbit, int pardeg,
                                                  unsigned long long* total)
{
  __shared__ unsigned long long s_red[4];
  unsigned long long acc = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < pardeg; i += gridDim.x * 256) acc += par_nbit[i];
  acc = wsum64(acc);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(total, s_red[0] + s_red[1] + s_red[2] + s_red[3]);
}

// one workgroup of 1024 threads: exclusive scan of per-brick outlier counts and the archive
// totals.  Each of the 16 waves owns a contiguous segment (a multiple of 256 counts): pass 1
// sums it with coalesced 16-byte loads, one barrier exchanges the segment sums, pass 2 scans
// it 256 counts (4 per lane) at a time with a carry, the next group's load issued before the
// current group's scan (65,536 spline tiles: the former 8-k-per-pass block scan took 63 us).
__global__ void __launch_bounds__(1024) k_finalize_scan(FinalizeArgs a, HeaderTpl hdr, uint8_t* archive,
                                                       size_t phf_offset, size_t bitstream_rel, int write_hdr)
{
  __shared__ uint32_t s_scan[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t seg = ((a.nbricks + 4095) / 4096) * 256;
  const uint32_t w0 = min((uint32_t)wid * seg, a.nbricks), w1 = min(w0 + seg, a.nbricks);
  const bool vec = (reinterpret_cast<uintptr_t>(a.brick_cnt) & 15) == 0;
  auto clamp = [&](uint32_t c) { return a.spill_start ? c : min(c, a.cap_per_brick); };
  auto load4raw = [&](uint32_t b) {  // counts b..b+3 of this segment (0 past its end)
    uint4 v{0, 0, 0, 0};
    if (vec && b + 3 < w1) v = *reinterpret_cast<const uint4*>(a.brick_cnt + b);
    else {
      if (b < w1) v.x = a.brick_cnt[b];
      if (b + 1 < w1) v.y = a.brick_cnt[b + 1];
      if (b + 2 < w1) v.z = a.brick_cnt[b + 2];
      if (b + 3 < w1) v.w = a.brick_cnt[b + 3];
    }
    return v;
  };
  auto load4 = [&](uint32_t b) {
    const uint4 v = load4raw(b);
    return uint4{clamp(v.x), clamp(v.y), clamp(v.z), clamp(v.w)};
  };
  uint32_t sum = 0, mx = 0;  // mx: the largest count (the slot capacity a repeat needs)
#pragma unroll 8
  for (uint32_t b = w0 + 4 * lane; b < w1; b += 256) {
    const uint4 v = load4raw(b);
    mx = max(mx, max(max(v.x, v.y), max(v.z, v.w)));
    sum += clamp(v.x) + clamp(v.y) + clamp(v.z) + clamp(v.w);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) sum += __shfl_xor(sum, d), mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
  if (lane == 0 && mx) atomicMax(&a.info->max_brick_cnt, mx);
  if (lane == 0) s_scan[wid] = sum;
  __syncthreads();
  uint32_t carry = 0, total = 0;
  for (int w = 0; w < 16; w++) {
    carry += w < wid ? s_scan[w] : 0u;
    total += s_scan[w];
  }
  uint4 nxt = load4(w0 + 4 * lane);
  for (uint32_t base = w0; base < w1; base += 256) {
    const uint4 v = nxt;
    nxt = load4(base + 256 + 4 * lane);
    const uint32_t own = v.x + v.y + v.z + v.w;
    const uint32_t inc = hfd::wave_incl_scan(own);  // DPP: no LDS round trips in the loop
    const uint32_t b = base + 4 * lane;
    uint32_t r = carry + inc - own;
    if (b < w1) a.brick_off[b] = r;
    r += v.x;
    if (b + 1 < w1) a.brick_off[b + 1] = r;
    r += v.y;
    if (b + 2 < w1) a.brick_off[b + 2] = r;
    r += v.z;
    if (b + 3 < w1) a.brick_off[b + 3] = r;
    carry += __shfl(inc, 63);
  }
  const uint32_t s_carry = total;
  if (tid == 0) {
    const int last = a.pardeg - 1;
    const unsigned long long ncell =
        a.sizes_known ? a.info->total_ncell
                      : (last >= 0 ? (unsigned long long)a.par_entry[last] + ((a.par_nbit[last] + 31u) >> 5) : 0ull);
    const uint32_t slot_total = s_carry;
    const uint32_t sp = *a.spill_cnt;
    const uint32_t sp_kept = sp < a.spill_cap ? sp : a.spill_cap;
    a.brick_off[a.nbricks] = slot_total;
    a.info->total_ncell = ncell;
    a.info->splen = (unsigned long long)slot_total + (a.spill_start ? 0u : sp_kept);
    a.info->outlier_lost = sp > a.spill_cap ? sp - a.spill_cap : 0u;
    a.info->spilled = sp;
    if (write_hdr)
      write_headers_dev(archive, hdr, a.info->total_nbit, ncell, a.info->splen, phf_offset, bitstream_rel);
  }
}

// one wave per brick copies its slot to the archive; trailing blocks copy the spill list.  The
// last workgroup publishes the compress summary when pub.flag is set: that costs every block a
// barrier on its stores and a ticket round trip, so the caller sets it only for small grids
// (config 5's 16,448 blocks: 35 -> 196 us with it).
__global__ void __launch_bounds__(256) k_outlier_copy(OutlierCopyArgs a, uint32_t spill_blocks, HostPub pub)
{
  const unsigned long long ncell = a.info->total_ncell;
  uint32_t* dst = reinterpret_cast<uint32_t*>(a.archive + a.bitstream_offset + ncell * 4);
  const uint32_t slot_total = a.brick_off[a.nbricks];
  const uint32_t brick_blocks = gridDim.x - spill_blocks;
  if (blockIdx.x < brick_blocks) {
    for (uint32_t brick = blockIdx.x * 4 + (threadIdx.x >> 6); brick < a.nbricks; brick += brick_blocks * 4) {
      const uint32_t all = a.brick_cnt[brick];
      const uint32_t cnt = min(all, a.cap_per_brick);
      const uint64_t* src = a.slots + (size_t)brick * a.cap_per_brick;
      uint32_t* d = dst + 2ull * a.brick_off[brick];
      if ((reinterpret_cast<uintptr_t>(d) & 7) == 0) {  // the archive offset decides (wave-uniform)
        uint64_t* d8 = reinterpret_cast<uint64_t*>(d);
#pragma unroll 4
        for (uint32_t i = threadIdx.x & 63; i < cnt; i += 64) d8[i] = src[i];
      }
      else
#pragma unroll 4
        for (uint32_t i = threadIdx.x & 63; i < cnt; i += 64) {
          const uint64_t c = src[i];
          d[2 * i] = (uint32_t)c;
          d[2 * i + 1] = (uint32_t)(c >> 32);
        }
      if (a.spill_start && all > cnt) {  // this brick's contiguous spill range follows its slot
        const uint32_t s0 = a.spill_start[brick];
        for (uint32_t i = threadIdx.x & 63; i < all - cnt; i += 64) {
          const uint64_t c = s0 + i < a.spill_cap ? a.spill[s0 + i] : 0ull;
          d[2 * (cnt + i)] = (uint32_t)c;
          d[2 * (cnt + i) + 1] = (uint32_t)(c >> 32);
        }
      }
    }
  }
  else if (!a.spill_start) {
    const uint32_t sp = min(*a.spill_cnt, a.spill_cap);
    uint32_t* d = dst + 2ull * slot_total;
    for (uint32_t i = (blockIdx.x - brick_blocks) * 256 + threadIdx.x; i < sp; i += spill_blocks * 256) {
      const uint64_t c = a.spill[i];
      d[2 * i] = (uint32_t)c;
      d[2 * i + 1] = (uint32_t)(c >> 32);
    }
  }
  publish_last(pub);
}

template <typename T>
__global__ void __launch_bounds__(256) k_extrema_partial(const T* __restrict__ in, size_t n, double* part)
{
  __shared__ T s_mn[4], s_mx[4];
  T mn = INFINITY, mx = -INFINITY;
  // 16-B loads, two in flight per lane per iteration; the scalar tail covers n % per-iteration
  constexpr int E = 16 / sizeof(T);
  const bool aligned = ((uintptr_t)in & 15) == 0;  // a caller may pass any element-aligned pointer
  const size_t nv = aligned ? n / (2 * E) : 0, stride = (size_t)gridDim.x * blockDim.x;
  const uint4* in4 = reinterpret_cast<const uint4*>(in);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    const uint4 a = in4[2 * i], b = in4[2 * i + 1];
    T v[2 * E];
    __builtin_memcpy(&v[0], &a, 16);
    __builtin_memcpy(&v[E], &b, 16);
#pragma unroll
    for (int k = 0; k < 2 * E; k++) {
      mn = v[k] < mn ? v[k] : mn;
      mx = v[k] > mx ? v[k] : mx;
    }
  }
  for (size_t i = nv * 2 * E + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const T v = in[i];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    T a = __shfl_xor(mn, d), b = __shfl_xor(mx, d);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) s_mn[wid] = mn, s_mx[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++) mn = s_mn[w] < mn ? s_mn[w] : mn, mx = s_mx[w] > mx ? s_mx[w] : mx;
    part[2 * blockIdx.x] = (double)s_mn[0] < (double)mn ? (double)s_mn[0] : (double)mn;
    part[2 * blockIdx.x + 1] = (double)s_mx[0] > (double)mx ? (double)s_mx[0] : (double)mx;
  }
}

// one 256-thread block reduces the per-block partials (extrema.cuhip.inl:150-208 does the same
// final step with a second kernel launch)
__global__ void __launch_bounds__(256) k_extrema_final(const double* part, int nparts, double* out)
{
  __shared__ double s_mn[4], s_mx[4];
  double mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    const double a = part[2 * i], b = part[2 * i + 1];
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const double a = __shfl_xor(mn, d), b = __shfl_xor(mx, d);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) s_mn[wid] = mn, s_mx[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++) mn = s_mn[w] < mn ? s_mn[w] : mn, mx = s_mx[w] > mx ? s_mx[w] : mx;
    out[0] = mn, out[1] = mx;
  }
}

// Copy device words into host-mapped (coherent, pinned) memory, then raise a flag the host
// polls.  Replaces hipMemcpyAsync(D2H) + hipStreamSynchronize on the compress critical path.
__global__ void __launch_bounds__(256) k_publish(XferRegions r, uint32_t* flag, uint32_t epoch)
{
  for (int k = 0; k < r.count; k++)
    for (int i = threadIdx.x; i < r.nwords[k]; i += 256) r.dst[k][i] = r.src[k][i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Zero up to 4 small device regions in one launch (per-call state reset: cheaper than one
// hipMemsetAsync per region on the compress critical path).
__global__ void __launch_bounds__(256) k_zero(XferRegions r)
{
  for (int k = 0; k < r.count; k++)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < r.nwords[k]; i += gridDim.x * 256) r.dst[k][i] = 0u;
}

// Copy host-mapped words (written by the host before this launch) into device memory.
__global__ void __launch_bounds__(256) k_upload(XferRegions r)
{
  for (int k = 0; k < r.count; k++)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < r.nwords[k]; i += gridDim.x * 256) r.dst[k][i] = r.src[k][i];
}

// Copy host-mapped words into device memory once the host has opened the gate (*gate reaches
// epoch: the codebook is built).  One thread per workgroup polls the host word with system-scope
// acquire loads; then every thread copies at most a word or two (each read crosses PCIe, so the
// copy is spread over kGateBlocks workgroups).  A poller gives up after a few seconds and flags
// the timeout word (the host always opens the gate, also on its error paths).
__global__ void __launch_bounds__(256) k_gate_upload(XferRegions r, const uint32_t* gate, uint32_t epoch,
                                                     unsigned int* timeout)
{
  __shared__ uint32_t s_ok;
  if (threadIdx.x == 0) {
    uint32_t ok = 1;
    for (uint32_t spin = 0;; spin++) {
      const uint32_t v = __hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - epoch) >= 0) break;
      if (spin > (1u << 22)) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok) {
    if (threadIdx.x == 0) atomicOr(timeout, 2u);
    return;
  }
  for (int k = 0; k < r.count; k++)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < r.nwords[k]; i += gridDim.x * 256) r.dst[k][i] = r.src[k][i];
}

}  // namespace

int launch_gate_upload(const XferRegions& r, const uint32_t* gate, uint32_t epoch, unsigned int* timeout,
                       hipStream_t st)
{
  constexpr int kGateBlocks = 8;
  k_gate_upload<<<kGateBlocks, 256, 0, st>>>(r, gate, epoch, timeout);
  return (int)hipGetLastError();
}

int launch_publish(const XferRegions& r, uint32_t* flag, uint32_t epoch, hipStream_t st)
{
  k_publish<<<1, 256, 0, st>>>(r, flag, epoch);
  return (int)hipGetLastError();
}

int launch_zero(const XferRegions& r, hipStream_t st)
{
  int words = 0;
  for (int k = 0; k < r.count; k++) words = r.nwords[k] > words ? r.nwords[k] : words;
  int grid = (words + 255) / 256;
  grid = grid < 1 ? 1 : (grid > 256 ? 256 : grid);
  k_zero<<<grid, 256, 0, st>>>(r);
  return (int)hipGetLastError();
}

// the sharded compress's overflow word: outlier cells of the last pass 1 beyond the spill list
__global__ void k_excess(const uint32_t* spill_cnt, uint32_t cap, uint32_t* dst)
{
  if (threadIdx.x == 0) {
    const uint32_t c = *spill_cnt;
    *dst = c > cap ? c - cap : 0u;
  }
}

int launch_excess(const uint32_t* spill_cnt, uint32_t cap, uint32_t* dst, hipStream_t st)
{
  k_excess<<<1, 64, 0, st>>>(spill_cnt, cap, dst);
  return (int)hipGetLastError();
}

int launch_upload(const XferRegions& r, hipStream_t st)
{
  k_upload<<<4, 256, 0, st>>>(r);
  return (int)hipGetLastError();
}

int launch_finalize_scan(const FinalizeArgs& a, hipStream_t st, const void* psz_tpl, const void* phf_tpl,
                         uint8_t* archive, size_t phf_offset, size_t bitstream_rel)
{
  int grid = (a.pardeg + 255) / 256;
  grid = grid < 1 ? 1 : (grid > 128 ? 128 : grid);
  if (!a.sizes_known && !a.nbit_known) k_sum_nbit<<<grid, 256, 0, st>>>(a.par_nbit, a.pardeg, &a.info->total_nbit);
  HeaderTpl t;
  const int wh = psz_tpl && phf_tpl && archive;
  if (wh) {
    __builtin_memcpy(t.psz, psz_tpl, 176);
    __builtin_memcpy(t.phf, phf_tpl, 64);
  }
  else
    __builtin_memset(&t, 0, sizeof(t));
  k_finalize_scan<<<1, 1024, 0, st>>>(a, t, archive, phf_offset, bitstream_rel, wh);
  return (int)hipGetLastError();
}

int launch_outlier_copy(const OutlierCopyArgs& a, hipStream_t st, const HostPub& pub)
{
  const uint32_t brick_blocks = std::max(1u, (a.nbricks + 3) / 4);
  const uint32_t spill_blocks = 64;
  k_outlier_copy<<<brick_blocks + spill_blocks, 256, 0, st>>>(a, spill_blocks, pub);
  return (int)hipGetLastError();
}

template <typename T>
int launch_extrema(const T* in, size_t n, double* d_minmax, unsigned int* d_scratch, hipStream_t st)
{
  // d_scratch must hold 2 * 1024 doubles of partials
  double* part = reinterpret_cast<double*>(d_scratch);
  int grid = (int)((n + 255) / 256);
  if (grid > 1024) grid = 1024;
  if (grid < 1) grid = 1;
  k_extrema_partial<T><<<grid, 256, 0, st>>>(in, n, part);
  k_extrema_final<<<1, 256, 0, st>>>(part, grid, d_minmax);
  return (int)hipGetLastError();
}

template int launch_extrema<float>(const float*, size_t, double*, unsigned int*, hipStream_t);
template int launch_extrema<double>(const double*, size_t, double*, unsigned int*, hipStream_t);

}  // namespace cusz_amd
