// cusz_amd/csrc/archive_device.hh -- device-side archive header fill, shared by the finalize
// kernel (pipeline_kernels.hip) and the brick reservation kernel (brick.hip).
//
// Layouts: psz_header psz/include/cusz/header.h:19-48 (entry[6] @56, splen @104), phf_header
// codec/hf/include/hf.h:40-46 (total_nbit @24, total_ncell @32, entry[6] @40).
#pragma once

#include "common.hh"

namespace cusz_amd {

// static header fields from the host; the size-dependent ones are filled on the device
struct HeaderTpl {
  uint32_t psz[176 / 4];
  uint32_t phf[64 / 4];
};

// one thread: writes the psz header (176 B) and the phf header (64 B + zeroed pad to 128 B)
__device__ inline void write_headers_dev(uint8_t* archive, HeaderTpl t, unsigned long long nb, unsigned long long nc,
                                         unsigned long long sp, size_t phf_offset, size_t bitstream_rel)
{
  uint32_t* phf = t.phf;
  phf[6] = (uint32_t)nb, phf[7] = (uint32_t)(nb >> 32);
  phf[8] = (uint32_t)nc, phf[9] = (uint32_t)(nc >> 32);
  const uint32_t phf_end = (uint32_t)(bitstream_rel + nc * 4);
  phf[10 + 5] = phf_end;  // entry[END]; entries 0..4 are static, set by the host
  uint32_t* psz = t.psz;
  const uint32_t e_spfmt = (uint32_t)(phf_offset + phf_end);
  psz[14 + 3] = e_spfmt;
  psz[14 + 4] = (uint32_t)(e_spfmt + sp * 8);
  psz[14 + 5] = (uint32_t)(e_spfmt + sp * 8);
  psz[26] = (uint32_t)sp, psz[27] = (uint32_t)(sp >> 32);
  uint32_t* a32 = reinterpret_cast<uint32_t*>(archive);
  for (int i = 0; i < 176 / 4; i++) a32[i] = psz[i];
  uint32_t* p32 = reinterpret_cast<uint32_t*>(archive + phf_offset);
  for (int i = 0; i < 64 / 4; i++) p32[i] = phf[i];
  for (int i = 64 / 4; i < 128 / 4; i++) p32[i] = 0;  // defined padding (reference: stale)
}

}  // namespace cusz_amd
