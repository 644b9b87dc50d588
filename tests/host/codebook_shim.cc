// tests/host/codebook_shim.cc -- C entry point over the library's host codebook builder
// (cusz_amd/csrc/codebook.cc), compiled by tests/test_codebook_host.py for a CPU-only check
// against the oracle's independent builder.
#include <cstdint>

namespace cusz_amd {
int build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook);
int build_codebook_twoqueue(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook);
}

extern "C" int shim_build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook)
{
  return cusz_amd::build_codebook(hist, bklen, book, revbook);
}

extern "C" int shim_build_codebook_twoqueue(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book,
                                            uint8_t* revbook)
{
  return cusz_amd::build_codebook_twoqueue(hist, bklen, smooth, book, revbook);
}
