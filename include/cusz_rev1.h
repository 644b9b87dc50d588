/* include/cusz_rev1.h -- the resource-manager C API (primary drop-in boundary).
 *
 * Each entry point replaces the reference symbol of the same name
 * (declared psz/include/cusz_rev1.h:13-22, implemented psz/src/libcusz.cc:219-366):
 *
 *   psz_create_resource_manager            libcusz.cc:219-232
 *   psz_create_resource_manager_from_CLI   (declared only in the reference)
 *   psz_create_resource_manager_from_header libcusz.cc:234-248
 *   psz_modify_resource_manager_from_header libcusz.cc:250-255
 *   psz_release_resource                   libcusz.cc:257-274
 *   psz_compress_float / _double           libcusz.cc:295-329
 *   psz_compress_analyize_float            libcusz.cc:331-346
 *   psz_decompress_float / _double         libcusz.cc:348-366
 *
 * Conventions kept: input/output are caller-owned DEVICE pointers on the caller's current
 * HIP device; `stream` is a hipStream_t (NULL = default stream) fixed at creation;
 * *OUT_d_compressed points into the manager's device buffer and stays valid until the
 * next compress or release; compress is synchronous w.r.t. the host, decompress returns
 * with work queued on `stream`.  Return values are psz_error_status codes.
 * Deliberate fixes: the decompress output need NOT be pre-zeroed; per-call
 * state (outlier counter, histogram) is reset on every call; the caller's current device
 * is honoured (no hipSetDevice(0)); nothing throws across this boundary.
 */
#ifndef CUSZ_AMD_REV1_H
#define CUSZ_AMD_REV1_H

#ifdef __cplusplus
extern "C" {
#endif

#include "cusz/context.h"

#define DEFAULT_RADIUS 512

psz_resource* psz_create_resource_manager(psz_dtype dtype, psz_len len, psz_pipeline pipeline,
                                          void* stream);
psz_resource* psz_create_resource_manager_from_CLI(int argc, char** argv, void* stream);
psz_resource* psz_create_resource_manager_from_header(psz_header* header, void* stream);
void psz_modify_resource_manager_from_header(psz_resource* manager, psz_header* header);
int psz_release_resource(psz_resource* manager);

int psz_compress_float(psz_resource* manager, psz_rc2 rc, float* IN_d_data, psz_header* OUT_header,
                       uint8_t** OUT_d_compressed, size_t* OUT_compressed_bytes);
int psz_compress_double(psz_resource* manager, psz_rc2 rc, double* IN_d_data,
                        psz_header* OUT_header, uint8_t** OUT_d_compressed,
                        size_t* OUT_compressed_bytes);
int psz_compress_analyize_float(psz_resource* manager, psz_rc2 rc, float* IN_d_data,
                                u4* exported_h_hist);

int psz_decompress_float(psz_resource* manager, uint8_t* IN_d_compressed,
                         size_t const IN_compressed_len, float* OUT_d_decompressed);
int psz_decompress_double(psz_resource* manager, uint8_t* IN_d_compressed,
                          size_t const IN_compressed_len, double* OUT_d_decompressed);

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_REV1_H */
