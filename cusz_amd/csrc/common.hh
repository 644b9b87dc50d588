// cusz_amd/csrc/common.hh -- shared device/host definitions for the MI355X (gfx950) path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace cusz_amd {

constexpr int kWave = 64;       // CDNA wavefront
constexpr int kLmax = 27;       // max Huffman code length in a u32 book word (hf_impl.hh:40-59)
constexpr int kMaxBklen = 1024; // 2 * max radius (buf_comp.hh:53-54)

// Outlier cell as stored in the archive: packed {f32 val, u32 idx} (sp_interface.h:20-26),
// little-endian, so as a u64 the value bits are the low word.
__host__ __device__ inline uint64_t make_cell(float v, uint32_t idx)
{
  return (uint64_t)__builtin_bit_cast(uint32_t, v) | ((uint64_t)idx << 32);
}

// Where the predictor writes outliers: a fixed slot per brick (deterministic order:
// brick order, then the brick's own scan order), plus a shared spill list for bricks that
// exceed their slot (order of spilled cells is not deterministic; never hit below 10 %).
struct OutlierSink {
  uint64_t* slots;       // nbricks * cap_per_brick cells
  uint32_t* brick_cnt;   // cells produced per brick (may exceed cap; excess went to spill)
  uint64_t* spill;       // spill_cap cells
  uint32_t* spill_cnt;   // atomic counter
  uint32_t cap_per_brick;
  uint32_t spill_cap;
  // nullptr: cells past a brick's slot go to the spill list one by one (order not deterministic).
  // Otherwise a brick over its slot reserves one contiguous spill range for all of its excess
  // (spill_start[brick]); the archive then lists every brick's cells in brick order.
  uint32_t* spill_start = nullptr;
};

// Device-side summary produced by the finalize kernel and read back by the host once.
struct CompressInfo {
  unsigned long long total_nbit;
  unsigned long long total_ncell;
  unsigned long long splen;        // outlier cells written to the archive
  unsigned long long outlier_lost; // cells that did not fit (=> PSZ_WARN_OUTLIER_TOO_MANY)
  unsigned int lookback_timeout;   // nonzero if a bounded spin gave up (should never happen)
  unsigned int spilled;            // outlier cells past their brick's slot (the spill list)
  unsigned int ticket;             // single-pass brick tickets
  unsigned int max_brick_cnt;      // largest outlier count of one brick (slot growth)
};

}  // namespace cusz_amd

#define CUSZ_AMD_HIP_CHECK(expr)                                        \
  do {                                                                  \
    hipError_t _e = (expr);                                             \
    if (_e != hipSuccess) return cusz_amd::report_hip_error(_e, #expr, __FILE__, __LINE__); \
  } while (0)

namespace cusz_amd {
int report_hip_error(hipError_t e, const char* expr, const char* file, int line);
}
