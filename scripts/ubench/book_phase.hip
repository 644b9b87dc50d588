// Micro-benchmark (diagnostic, not product code): phase clocks of the device codebook
// (book_device.hh) on a few histograms.  Build + run: hipcc -O3 --offload-arch=gfx950
// -I cusz_amd/csrc -I include -o scripts/ubench/book_phase scripts/ubench/book_phase.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#include "book_device.hh"

using namespace cusz_amd;

__global__ void __launch_bounds__(1024) k_phase(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book,
                                                uint8_t* rev, unsigned long long* clk)
{
  __shared__ hbook::Smem sm;
  const int t = threadIdx.x;
  auto stamp = [&](int i) {
    __syncthreads();
    if (t == 0) clk[i] = wall_clock64();
  };
  stamp(0);
  const unsigned long long c0 = clock64();
  unsigned long long w = t < bklen ? (unsigned long long)hist[t] + smooth : 0ull;
  const unsigned long long key = w ? (w << 11 | (unsigned long long)t) : hbook::kInf;
  const uint32_t n = hbook::block_sum(w ? 1u : 0u, sm, t);
  stamp(1);
  const unsigned long long v = hbook::sort_keys(key, sm, t);
  __syncthreads();
  sm.key[t] = v;
  stamp(2);
  uint32_t maxl = n >= 2 ? hbook::tree_lengths(sm, n, t) : 1;
  stamp(3);
  hbook::build(hist, bklen, smooth, book, rev, sm);
  stamp(4);
  if (t == 0) clk[5] = maxl, clk[6] = clock64() - c0;
}

int main()
{
  const int bklen = 1024;
  std::vector<std::vector<uint32_t>> hs;
  std::vector<uint32_t> h(bklen);
  for (int i = 0; i < bklen; i++) h[i] = (uint32_t)(1e6 * std::exp(-std::fabs(i - 512.0) / 8.0));
  hs.push_back(h);
  for (int i = 0; i < bklen; i++) h[i] = (uint32_t)(2.5e5 * std::exp(-std::fabs(i - 512.0) / 60.0));
  hs.push_back(h);
  for (int i = 0; i < bklen; i++) h[i] = 7;
  hs.push_back(h);
  uint32_t *dh, *db;
  uint8_t* dr;
  unsigned long long* dc;
  hipMalloc(&dh, 4 * bklen);
  hipMalloc(&db, 4 * bklen);
  hipMalloc(&dr, 4096);
  hipMalloc(&dc, 64);
  for (auto& x : hs)
    for (int smooth = 0; smooth < 2; smooth++) {
      hipMemcpy(dh, x.data(), 4 * bklen, hipMemcpyHostToDevice);
      unsigned long long c[8];
      for (int rep = 0; rep < 200; rep++) {
        k_phase<<<1, 1024>>>(dh, bklen, smooth, db, dr, dc);
        hipMemcpy(c, dc, 64, hipMemcpyDeviceToHost);
      }
      // wall_clock64: 100 MHz
      printf("smooth %d maxl %llu: count %.2f us  sort %.2f us  tree %.2f us  build(all) %.2f us  (core clock %.0f MHz)\n",
             smooth, c[5], (c[1] - c[0]) / 100.0, (c[2] - c[1]) / 100.0, (c[3] - c[2]) / 100.0, (c[4] - c[3]) / 100.0,
             c[6] * 100.0 / (double)(c[4] - c[0]));
    }
  return 0;
}
