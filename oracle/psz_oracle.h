/* oracle/psz_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of cuSZ's GPU hot path (Lorenzo predictor-quantizer,
 * histogram, canonical Huffman codebook, coarse-grained Huffman encode/decode).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so, and only as the checker.  The product (cusz_amd/) never calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference tree, szcompressor/cuSZ @ 2026-03-13).
 */
#ifndef PSZ_ORACLE_H
#define PSZ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* number of dimensions, psz/include/kernel/launch.hh:19-38 */
int orc_ndim(size_t x, size_t y, size_t z);

/* Lorenzo predict-quantize, GPU semantics (psz/src/kernel/detail/lrz_c.cuhip.inl:23-372).
 * codes[N] receives u16 quant codes; outliers (val,idx) are written in increasing idx
 * order, at most ol_cap of them.  Returns the total number of outliers (may exceed
 * ol_cap, in which case only the first ol_cap were written). */
size_t orc_lorenzo_c_f32(const float* in, size_t x, size_t y, size_t z, double eb,
                         uint16_t radius, int zigzag, uint16_t* codes, float* ol_val,
                         uint32_t* ol_idx, size_t ol_cap);
size_t orc_lorenzo_c_f64(const double* in, size_t x, size_t y, size_t z, double eb,
                         uint16_t radius, int zigzag, uint16_t* codes, float* ol_val,
                         uint32_t* ol_idx, size_t ol_cap);

/* Lorenzo reconstruct, GPU semantics (psz/src/kernel/detail/lrz_x.cuhip.inl:11-360,
 * scan order of wave32.cuhip.inl:7-66).  Outliers are scattered first (reference
 * GPU_scatter::kernel_v2, spvn.cuhip.inl:41-76) onto a zero plane. */
void orc_lorenzo_x_f32(const uint16_t* codes, const float* ol_val, const uint32_t* ol_idx,
                       size_t nol, size_t x, size_t y, size_t z, double eb, uint16_t radius,
                       int zigzag, float* out);
void orc_lorenzo_x_f64(const uint16_t* codes, const float* ol_val, const uint32_t* ol_idx,
                       size_t nol, size_t x, size_t y, size_t z, double eb, uint16_t radius,
                       int zigzag, double* out);

/* histogram, psz/src/kernel/detail/hist.cuhip.inl:55-89 (result equals the serial one,
 * psz/src/kernel/hist_generic.seq.cc:17-30) */
void orc_histogram_u2(const uint16_t* codes, size_t n, uint32_t* hist, int bklen);

/* Canonical Huffman codebook (codec/hf/src/hf_bk.seq.cc:72-145, hf_bk_impl1.seq.cc:103-199,
 * hf_bk_internal.seq.cc:64-107, hf_canon.seq.cc:105-161).
 * book: u32[bklen] (code | len<<27, unused = 0xFFFFFFFF); revbook: first i32[32] | entry i32[32]
 * | keys u16[bklen].  Deviations (documented in DESIGN.md): a single used symbol gets a
 * 1-bit code; lengths above 27 are limited to 27.  Returns revbook bytes, or -1. */
int orc_build_codebook_u2(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook);

/* code lengths only (before canonisation); returns max length */
int orc_huffman_lengths(const uint32_t* hist, int bklen, uint8_t* lens);

/* The device codebook's algorithm (cusz_amd/csrc/book_device.hh), serially: two-queue Huffman
 * over (weight, symbol)-sorted leaves of hist + smooth, leaf first on equal weights, depth > 27
 * halves the weights and rebuilds; reference canonisation.  Returns revbook bytes. */
int orc_book_twoqueue_u2(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook);

/* chunking (codec/hf/src/libphf.cc:26-70); n_cu = #CUs, max_threads = max threads/block */
void orc_coarse_tune(size_t len, int n_cu, int max_threads, int* sublen, int* pardeg);

/* Coarse-grained encode (codec/hf/src/hf_kernels.cuhip.inl:76-170,449-501).
 * Writes par_nbit[pardeg], par_entry[pardeg] and the concatenated bitstream (u32 cells).
 * Returns total cells, or (size_t)-1 if bitstream_cap would be exceeded. */
size_t orc_hf_encode_u2(const uint16_t* codes, size_t n, const uint32_t* book, int sublen,
                        uint32_t* par_nbit, uint32_t* par_entry, uint32_t* bitstream,
                        size_t bitstream_cap, uint64_t* total_nbit);

/* canonical decode (codec/hf/src/hf_kernels.cuhip.inl:331-396) */
void orc_hf_decode_u2(const uint32_t* bitstream, const uint8_t* revbook, int bklen,
                      const uint32_t* par_nbit, const uint32_t* par_entry, int sublen,
                      int pardeg, size_t n, uint16_t* out);

/* cuSZ-i spline3 predictor-quantizer (psz/src/kernel/detail/spline3.inl:916-973, launched by
 * spline3.cu:22-44) and reconstruction (spline3.inl:975-1016).  PARITY UNPINNED (no reference
 * test or pipeline exists for this path).  anchors: T[ceil(x/8)*ceil(y/8)*ceil(z/8)];
 * outliers: (float)code and index, tile order then (z,y,x) inside the tile; returns the count. */
size_t orc_spline3_c_f32(const float* in, size_t x, size_t y, size_t z, double eb, int radius,
                         uint16_t* codes, float* anchors, float* ol_val, uint32_t* ol_idx, size_t ol_cap);
size_t orc_spline3_c_f64(const double* in, size_t x, size_t y, size_t z, double eb, int radius,
                         uint16_t* codes, double* anchors, float* ol_val, uint32_t* ol_idx, size_t ol_cap);
void orc_spline3_x_f32(const uint16_t* codes, const float* anchors, const float* ol_val, const uint32_t* ol_idx,
                       size_t nol, size_t x, size_t y, size_t z, double eb, int radius, float* out);
void orc_spline3_x_f64(const uint16_t* codes, const double* anchors, const float* ol_val, const uint32_t* ol_idx,
                       size_t nol, size_t x, size_t y, size_t z, double eb, int radius, double* out);

#ifdef __cplusplus
}
#endif
#endif
