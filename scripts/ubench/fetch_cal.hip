// FETCH_SIZE calibration for the decoders' read pattern (diagnostic, not product code).
// Reads exactly N bytes twice: (A) coalesced, 16 B per lane, consecutive lanes adjacent;
// (B) per-lane streams as the chunk decoders read them: lane l of a wave walks its own 288-B
// piece of the wave's 18 KB block, 16 B per load.  rocprofv3 --pmc FETCH_SIZE gives each
// kernel's counted bytes; their ratio to N calibrates the counter for the pattern.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_coalesced(const uint4* __restrict__ in, size_t n16, unsigned* out)
{
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

constexpr int kPiece = 288;  // bytes per lane (a decoder chunk at CR ~3.5)
__global__ void k_streams(const uint8_t* __restrict__ in, size_t nblocks, unsigned* out)
{
  const int lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6, nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t b = wave; b < nblocks; b += nw) {
    const uint8_t* p = in + b * (64 * kPiece) + (size_t)lane * kPiece;
#pragma unroll
    for (int k = 0; k < kPiece / 16; k++) {
      const uint4 v = *reinterpret_cast<const uint4*>(p + 16 * k);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
  const size_t nblocks = 65536, N = nblocks * 64 * kPiece;  // 1.2 GB: past the 256 MiB L3
  uint8_t* d = nullptr;
  unsigned* o = nullptr;
  if (hipMalloc(&d, N) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
  (void)hipMemset(d, 1, N);
  k_coalesced<<<4096, 256>>>(reinterpret_cast<const uint4*>(d), N / 16, o);
  k_streams<<<4096, 256>>>(d, nblocks, o);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("bytes read per kernel: %zu (%.1f MB)\n", N, N / 1e6);
  (void)hipFree(d);
  (void)hipFree(o);
  return 0;
}
