// cusz_amd/csrc/book.hip -- the device codebook (book_device.hh) as a launch: one workgroup of
// 1024 threads reads a device histogram and writes the book and the reverse book.  The sampled
// codebook path builds it inside its sample kernel instead (k_brick3_sample's last workgroup);
// this launch serves the exported psz_amd_build_book_device (tests, timing).
#include "book_device.hh"
#include "kernels.hh"

namespace cusz_amd {

namespace {

__global__ void __launch_bounds__(hbook::kThreads) k_book(const uint32_t* hist, int bklen, uint32_t smooth,
                                                           uint32_t* book, uint8_t* revbook)
{
  __shared__ hbook::Smem sm;
  hbook::build<hbook::kThreads>(hist, bklen, smooth, book, revbook, sm);
}

}  // namespace

int launch_book_device(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook,
                       hipStream_t st)
{
  if (bklen < 1 || bklen > hbook::kThreads) return (int)hipErrorInvalidValue;
  k_book<<<1, hbook::kThreads, 0, st>>>(hist, bklen, smooth, book, revbook);
  return (int)hipGetLastError();
}

}  // namespace cusz_amd
