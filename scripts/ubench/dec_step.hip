// Micro-benchmark (diagnostic, not product code): the fused decoder's step chain on synthetic
// tables, with W waves per CU and C independent chains per lane, no ring refills (the ring is
// pre-filled and wraps).  Reports cycles per step per wave.  Build: see Makefile next to it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int B = 12;
constexpr uint32_t kRing = 16;
constexpr int kTP = 78;

__device__ __forceinline__ uint32_t hsh(uint32_t x)
{
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int C, int MODE>
__global__ void __launch_bounds__(1024) k_step(uint32_t* out, int nsteps, uint32_t thr, int tile_bytes, int pitch)
{
  __shared__ uint32_t tab[(1 << B) + 4096];
  __shared__ uint2 tab8[MODE == 9 || MODE == 10 ? (1 << B) + 2048 : 1];
  if constexpr (MODE == 9 || MODE == 10) {
    for (int i = threadIdx.x; i < (1 << B) + 2048; i += blockDim.x) {
      const uint32_t h = hsh(i * 2654435761u + 17);
      const uint32_t bits = 4 + h % 7;
      const uint32_t two = (h >> 8) & 1;
      const uint32_t b = bits + two * 3;
      tab8[i] = make_uint2((((h >> 9) & 1023) << 16) | ((h >> 19) & 1023), b | (b << 8) | ((2 + 2 * two) << 16));
    }
  }
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  for (int i = threadIdx.x; i < (1 << B) + 4096; i += blockDim.x) {
    const uint32_t h = hsh(i * 2654435761u + 17);
    const uint32_t bits = 4 + h % 7;  // 4..10 bits
    const uint32_t two = (h >> 8) & 1;
    tab[i] = (two << 31) | ((bits + two * 3) << 26) | (((h >> 9) & 1023) << 16) | ((1 + two) << 14) | ((h >> 19) & 1023);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t wbytes = (size_t)C * ((kRing + 1) * 256 + tile_bytes);
  uint8_t* wb = dsm + wid * wbytes;
  uint32_t w0[C], w1[C], w2[C], nx[C], sh[C], kk[C], cnt[C], acc[C];
  uint32_t* ring[C];
  uint16_t* rowp[C];
#pragma unroll
  for (int c = 0; c < C; c++) {
    ring[c] = reinterpret_cast<uint32_t*>(wb + c * ((kRing + 1) * 256 + tile_bytes)) + lane;
    rowp[c] = reinterpret_cast<uint16_t*>(wb + c * ((kRing + 1) * 256 + tile_bytes) + (kRing + 1) * 256) + lane * pitch;
    for (uint32_t s = 0; s <= kRing; s++) ring[c][s * 64] = hsh(lane * 977 + s * 131 + c * 7 + blockIdx.x);
    w0[c] = 0; w1[c] = hsh(lane + c); w2[c] = hsh(lane + 3 + c); nx[c] = ring[c][2 * 64];
    sh[c] = 0; kk[c] = 2; cnt[c] = 0; acc[c] = 0;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < nsteps; it++) {
#pragma unroll
    for (int c = 0; c < C; c++) {
      if constexpr (MODE == 9) {
        // u64 entries, register window
        const uint32_t win = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
        const uint32_t a = win < thr ? (1u << B) + min(win >> 16, 2047u) : win >> (32 - B);
        const uint2 E = tab8[a];
        uint16_t* rp = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rowp[c]) + (cnt[c] & (pitch >= 74 ? 126u : 62u)));
        rp[0] = (uint16_t)E.x;
        asm volatile("" ::: "memory");
        rp[1] = (uint16_t)(E.x >> 16);
        cnt[c] += (E.y >> 16) & 255u;
        const int32_t s2 = (int32_t)sh[c] - (int32_t)(E.y & 255u);
        const bool shf = s2 < 0;
        sh[c] = (uint32_t)s2 & 31u;
        w0[c] = shf ? w1[c] : w0[c];
        w1[c] = shf ? w2[c] : w1[c];
        w2[c] = shf ? nx[c] : w2[c];
        kk[c] += shf ? 256u : 0u;
        nx[c] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ring[c]) + (kk[c] & 0xF00u));
        continue;
      }
      if constexpr (MODE == 11) {
        // u32 entries: [9:0] sym0 [15:13] 2 nsym [25:16] sym1 [31:27] bits; read2 window
        const uint32_t win = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
        const uint32_t a = win < thr ? (1u << B) + min(win >> 16, 2047u) : win >> (32 - B);
        const uint32_t e = tab[a];
        uint16_t* rp = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rowp[c]) + (cnt[c] & (pitch >= 74 ? 126u : 62u)));
        rp[0] = (uint16_t)e;
        asm volatile("" ::: "memory");
        rp[1] = (uint16_t)(e >> 16);
        cnt[c] += (e >> 13) & 7u;
        const uint32_t bits = e >> 27;
        kk[c] += bits << 3;
        sh[c] -= bits;
        const uint32_t* rr = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ring[c]) + (kk[c] & 0xF00u));
        w0[c] = rr[0];
        w1[c] = rr[64];
        continue;
      }
      if constexpr (MODE == 10) {
        // u64 entries, window from ds_read2 of slots J, J+1 (w0/w1); sh = -pos; kk = 8 (pos + 511)
        const uint32_t win = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
        const uint32_t a = win < thr ? (1u << B) + min(win >> 16, 2047u) : win >> (32 - B);
        const uint2 E = tab8[a];
        uint16_t* rp = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(rowp[c]) + (cnt[c] & (pitch >= 74 ? 126u : 62u)));
        rp[0] = (uint16_t)E.x;
        asm volatile("" ::: "memory");
        rp[1] = (uint16_t)(E.x >> 16);
        cnt[c] += (E.y >> 16) & 255u;
        kk[c] += (E.y >> 8) & 255u;
        sh[c] -= E.y & 255u;
        const uint32_t* rr = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ring[c]) + (kk[c] & 0xF00u));
        w0[c] = rr[0];
        w1[c] = rr[64];
        continue;
      }
      if constexpr (MODE >= 5) {
        // w0/w1 hold words J, J+1 (read last step); sh = -pos; kk = pos + 511
        const uint32_t win = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
        const uint32_t a = win < thr ? (1u << B) + min(win >> 16, 4095u) : win >> (32 - B);
        const uint32_t e = tab[a];
        const uint32_t sy = e & 0x03FF03FFu;
        uint16_t* rp = rowp[c] + (cnt[c] & (pitch >= 74 ? 63u : 31u));
        rp[0] = (uint16_t)sy;
        asm volatile("" ::: "memory");
        rp[1] = (uint16_t)(sy >> 16);
        cnt[c] += (e >> 14) & 3u;
        const uint32_t bits = e >> 26 & 31u;
        kk[c] += bits;
        sh[c] -= bits;
        const uint32_t* rr = ring[c] + ((kk[c] >> 5) & 15u) * 64;
        w0[c] = rr[0];
        w1[c] = rr[64];
        continue;
      }
      const uint32_t win = __builtin_amdgcn_alignbit(w0[c], w1[c], sh[c]);
      const uint32_t a = win < thr ? (1u << B) + min(win >> 16, 4095u) : win >> (32 - B);
      const uint32_t e = tab[a];
      const uint32_t sy = e & 0x03FF03FFu;
      uint16_t* rp = rowp[c] + (cnt[c] & (pitch >= 74 ? 63u : 31u));
      if constexpr (MODE == 6) {
        uint16_t* q = rowp[c] + (it & 31);
        q[0] = (uint16_t)sy;
        asm volatile("" ::: "memory");
        q[1] = (uint16_t)(sy >> 16);
      }
      else if constexpr (MODE == 7) {
        *reinterpret_cast<uint32_t*>(rowp[c] + (cnt[c] & 30u)) = sy;
      }
      else if constexpr (MODE == 8) {
        uint16_t* q = rowp[c] - lane * pitch + lane + (cnt[c] & 31u) * 66;
        q[0] = (uint16_t)sy;
        asm volatile("" ::: "memory");
        q[66] = (uint16_t)(sy >> 16);
      }
      else if constexpr (MODE == 0 || MODE == 2) {
        rp[0] = (uint16_t)sy;
        asm volatile("" ::: "memory");
        rp[1] = (uint16_t)(sy >> 16);
      }
      else if constexpr (MODE == 4) {
        acc[c] = acc[c] * 33u + sy;
        if ((it & 3) == 3) *reinterpret_cast<uint2*>(rowp[c] + ((cnt[c] >> 2) & 7u) * 4) = make_uint2(acc[c], sy);
      }
      else
        acc[c] = acc[c] * 33u + sy;
      cnt[c] += (e >> 14) & 3u;
      const int32_t s2 = (int32_t)sh[c] - (int32_t)((e >> 26) & 31u);
      const bool shf = s2 < 0;
      sh[c] = (uint32_t)s2 & 31u;
      w0[c] = shf ? w1[c] : w0[c];
      w1[c] = shf ? w2[c] : w1[c];
      w2[c] = shf ? nx[c] : w2[c];
      kk[c] += shf ? 1u : 0u;
      if constexpr (MODE == 2 || MODE == 3)
        nx[c] = kk[c] * 0x9E3779B9u;
      else
        nx[c] = ring[c][(kk[c] & (kRing - 1u)) * 64];
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t1 = __builtin_readcyclecounter();
  uint32_t accs = 0;
#pragma unroll
  for (int c = 0; c < C; c++) accs += w0[c] ^ cnt[c] ^ sh[c] ^ acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = accs;
  if (lane == 0) reinterpret_cast<unsigned long long*>(out + gridDim.x * blockDim.x)[blockIdx.x * 32 + wid] = t1 - t0;
}

template <int C, int MODE>
void run(int waves, int pitch, uint32_t thr, int nsteps)
{
  const int tile_bytes = 64 * pitch * 2;
  const int grid = 256;
  const size_t wbytes = (size_t)C * ((kRing + 1) * 256 + tile_bytes);
  const size_t lds = wbytes * waves;
  uint32_t* d;
  if (lds + (MODE == 9 || MODE == 10 ? 49152 + 49152 : 32768) > 163840 + 16384 || waves > 16) { printf("skip C=%d waves %d lds %zu\n", C, waves, lds); return; }
  hipMalloc(&d, (size_t)grid * 1024 * 4 + grid * 32 * 8);
  auto kern = k_step<C, MODE>;
  if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
    printf("attr fail\n");
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, 0, d, nsteps, thr, tile_bytes, pitch);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), lds, 0, d, nsteps, thr, tile_bytes, pitch);
  hipEventRecord(e1);
  hipError_t err = hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> cyc(grid * 32);
  hipMemcpy(cyc.data(), reinterpret_cast<char*>(d) + (size_t)grid * 1024 * 4, grid * 32 * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int b = 0; b < grid; b++)
    for (int w = 0; w < waves; w++) avg += cyc[b * 32 + w];
  avg /= grid * waves;
  const double steps = (double)nsteps * C;
  printf("pitch=%d C=%d mode=%d waves/CU=%2d lds=%6zu: %s %.3f ms, %.1f cyc/wave-step (chain-steps), %.2f ns per chain-step per CU, clock %.2f GHz\n",
         pitch, C, MODE, waves, lds, err == hipSuccess ? "ok" : "ERR", ms, avg / steps, ms * 1e6 / (steps * waves),
         avg / (ms * 1e6));
  hipFree(d);
}

int main(int argc, char** argv)
{
  const int nsteps = 4000;
  const uint32_t thr = 0x08000000u;  // ~3 % of windows go to L2
  run<1, 0>(8, 74, thr, nsteps);
  run<1, 10>(7, 74, thr, nsteps);
  run<1, 10>(8, 74, thr, nsteps);
  run<1, 11>(8, 74, thr, nsteps);
  run<1, 11>(9, 74, thr, nsteps);
  run<1, 11>(10, 42, thr, nsteps);
  return 0;
}
