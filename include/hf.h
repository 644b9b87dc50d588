/* include/hf.h -- Huffman ("phf") segment format and codec-level C entry points.
 *
 * phf_header layout is byte-identical to the reference codec/hf/include/hf.h:40-46
 * (64 B; padded to PHFHEADER_FORCED_ALIGN=128 in the archive, hf_buf.cc:199-211):
 *   bklen:16 @0 | sublen @4 | pardeg @8 | original_len @16 | total_nbit @24 |
 *   total_ncell @32 | entry[6] @40  (segment byte offsets, relative to the phf segment)
 * segments: [header 128][revbook: first i32[32] entry i32[32] keys u16[bklen]]
 *           [par_nbit u32[pardeg]][par_entry u32[pardeg]][bitstream u32[total_ncell]]
 *
 * The reference declares phf_create/phf_encode/phf_decode (hf.h:65-72) but never defines
 * them; this library defines the helpers it does define (phf_coarse_tune*, phf_encoded_bytes,
 * phf_reverse_book_bytes) with the same semantics, tuned for the caller's current device.
 */
#ifndef CUSZ_AMD_HF_H
#define CUSZ_AMD_HF_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stddef.h>
#include <stdint.h>

#include "c_type.h"

#define PHF_SUCCESS 0
#define PHF_WRONG_DTYPE 1
#define PHF_FAIL_GPU_MALLOC 2
#define PHF_FAIL_GPU_MEMCPY 3
#define PHF_FAIL_GPU_ILLEGAL_ACCESS 4
#define PHF_FAIL_GPU_OUT_OF_MEMORY 5
#define PHF_NOT_IMPLEMENTED 99

#define PHFHEADER_FORCED_ALIGN 128
#define PHFHEADER_HEADER 0
#define PHFHEADER_RVBK 1
#define PHFHEADER_PAR_NBIT 2
#define PHFHEADER_PAR_ENTRY 3
#define PHFHEADER_BITSTREAM 4
#define PHFHEADER_END 5

typedef void* phf_stream_t;
typedef uint32_t PHF_METADATA;
typedef uint8_t PHF_BIN;
typedef uint8_t PHF_BYTE;

typedef enum { HF_U1, HF_U2, HF_U4, HF_U8, HF_ULL, HF_INVALID } phf_dtype;

typedef struct {
  int bklen : 16;
  int sublen, pardeg;
  size_t original_len;
  size_t total_nbit, total_ncell;
  uint32_t entry[PHFHEADER_END + 1];
} phf_header;

uint32_t phf_encoded_bytes(phf_header* h);
size_t phf_coarse_tune_sublen(size_t len);
void phf_coarse_tune(size_t len, int* sublen, int* pardeg);
size_t phf_reverse_book_bytes(u2 bklen, size_t BK_UNIT_BYTES, size_t SYM_BYTES);
void phf_version(void);
void phf_versioninfo(void);

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_HF_H */
