/* include/cusz.h -- the older compressor-object C API (secondary boundary).
 *
 * Replaces the reference psz/include/cusz.h:32-111 (implemented psz/src/libcusz.cc:29-214):
 *   psz_create            libcusz.cc:29-50     psz_create_default     libcusz.cc:52-69
 *   psz_create_from_context libcusz.cc:71-87   psz_create_from_header libcusz.cc:89-103
 *   psz_release           libcusz.cc:105-117   psz_compress           libcusz.cc:119-166
 *   psz_decompress        libcusz.cc:168-194   psz_clear_buffer       libcusz.cc:196-214
 * Same device-pointer conventions as cusz_rev1.h; `stream` is a hipStream_t.
 */
#ifndef CUSZ_AMD_CUSZ_H
#define CUSZ_AMD_CUSZ_H

#ifdef __cplusplus
extern "C" {
#endif

#include "cusz/context.h"
#include "cusz/header.h"
#include "cusz/type.h"

psz_compressor* psz_create(psz_dtype const dtype, psz_len3 const uncomp_len,
                           psz_predictor const predictor, int const quantizer_radius,
                           psz_codec const codec);
psz_compressor* psz_create_default(psz_dtype const dtype, psz_len3 const uncomp_len);
psz_compressor* psz_create_from_context(psz_ctx* const ctx, psz_len3 const uncomp_len);
psz_compressor* psz_create_from_header(psz_header* const header);
pszerror psz_release(psz_compressor* comp);

pszerror psz_compress(psz_compressor* comp, void* d_in, psz_len3 const in_len3, double const eb,
                      psz_mode const mode, uint8_t** d_compressed, size_t* comp_bytes,
                      psz_header* header, void* record, void* stream);
pszerror psz_decompress(psz_compressor* comp, uint8_t* d_compressed, size_t const comp_len,
                        void* d_decompressed, psz_len3 const decomp_len, void* record,
                        void* stream);
pszerror psz_clear_buffer(psz_compressor* comp);

void psz_version(void);
void psz_versioninfo(void);

void* psz_make_timerecord(void);
void psz_review_comp_time_breakdown(void* r, psz_header* h);
void psz_review_comp_time_from_header(psz_header* h);
void psz_review_decomp_time_from_header(psz_header* h);
void psz_review_compression(void* r, psz_header* h);
void psz_review_decompression(void* r, size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_CUSZ_H */
