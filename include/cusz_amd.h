/* include/cusz_amd.h -- extensions of this implementation beyond the cuSZ C API.
 *
 * None of these exist in the reference; they expose what the MI355X build measures and
 * what the parity tests need (stage timings, intermediate device buffers, tuning knobs,
 * slab sharding helpers for multi-GPU runs).  All functions return the status codes below.
 */
#ifndef CUSZ_AMD_EXT_H
#define CUSZ_AMD_EXT_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stddef.h>
#include <stdint.h>

#include "cusz/context.h"

/* Status codes.  Every entry point returns a psz_error_status value (cusz/type.h: the reference's
 * values, used where one applies: PSZ_ABORT_UNSUPPORTED_TYPE for a dtype mismatch,
 * PSZ_ABORT_UNSUPPORTED_DIMENSION for an archive of another shape, ...) or one of these, for
 * failures the reference enum has no value for (it reports them as crashes or exceptions): */
#define PSZ_AMD_ERR_INVALID_ARG 100 /* null handle or pointer, a size or knob value out of range   */
#define PSZ_AMD_ERR_BAD_ARCHIVE 101 /* archive or header malformed, truncated or inconsistent      */
#define PSZ_AMD_ERR_DEVICE 102      /* a HIP runtime call, allocation or kernel launch failed       */
#define PSZ_AMD_ERR_STATE 103       /* call out of order (compress_finish without a pending scan)   */
#define PSZ_AMD_ERR_ENCODER 104     /* the encoder's own overflow / look-back check failed (a bug)  */

/* Stage indices for psz_amd_stage_times (milliseconds of the last call, HIP events on the
 * manager's stream; only filled after psz_amd_enable_timing(m, 1)). */
enum {
  PSZ_AMD_T_EXTREMA = 0,   /* Rel mode range probe                         */
  PSZ_AMD_T_PREDICT = 1,   /* Lorenzo predict-quantize + histogram + outliers */
  PSZ_AMD_T_BOOK = 2,      /* histogram D2H + host codebook + H2D          */
  PSZ_AMD_T_ENCODE = 3,    /* Huffman encode (bit packing + look-back)      */
  PSZ_AMD_T_FINALIZE = 4,  /* outlier compaction + headers + readback       */
  PSZ_AMD_T_COMPRESS = 5,  /* whole compress call                           */
  PSZ_AMD_T_SCATTER = 6,   /* decompress: outlier scatter (+ zeroing)       */
  PSZ_AMD_T_DECODE = 7,    /* decompress: Huffman decode                    */
  PSZ_AMD_T_RECON = 8,     /* decompress: Lorenzo reconstruct               */
  PSZ_AMD_T_DECOMPRESS = 9,/* whole decompress call                         */
  PSZ_AMD_T_COUNT = 10
};

typedef struct psz_amd_internals {
  uint16_t* d_quant_codes; /* quant codes of the last compress (or decoded codes) */
  uint32_t* d_hist;        /* histogram u32[bklen] of the last compress          */
  uint32_t* d_book;        /* codebook u32[bklen]                                 */
  size_t len;              /* number of elements                                  */
  int bklen;
  int sublen;
  int pardeg;
  int ndim;
  size_t splen;            /* outlier cells of the last compress                  */
  size_t archive_capacity; /* bytes reserved for the device archive               */
  int layout;              /* archive layout of the last compress: PSZ_AMD_LAYOUT_* */
  int brick_width;         /* chunk length of the brick layout (0: not eligible)  */
} psz_amd_internals;

int psz_amd_get_internals(psz_resource* m, psz_amd_internals* out);
int psz_amd_enable_timing(psz_resource* m, int on);
int psz_amd_stage_times(psz_resource* m, float* ms, int n);

/* Override the Huffman chunk length (symbols per chunk, rounded up to a multiple of 256,
 * at most 8192) used by the next compress; 0 restores the default (nCU * 512 chunks, see
 * DESIGN.md; the reference's libphf.cc:26-70 rule targets one encode thread per chunk). */
int psz_amd_set_sublen(psz_resource* m, int sublen);

/* Decode-only entry point used by the multi-GPU gather path and tests: decodes the Huffman
 * segment of a device archive into the manager's code buffer. */
int psz_amd_decode_codes(psz_resource* m, uint8_t* IN_d_compressed);

/* Huffman decoder selection: 0 auto (default: the fused brick decoder when the archive's chunk
 * length is the brick width, else lane/wave by chunk count), 1 one lane per chunk
 * (LDS-windowed), 2 one wave per chunk.  1 and 2 decode into the code buffer and reconstruct
 * separately.  All decode the same archives bit-exactly; tests exercise each.  Other values
 * are rejected. */
#define PSZ_AMD_DECODER_AUTO 0
#define PSZ_AMD_DECODER_LANE 1
#define PSZ_AMD_DECODER_WAVE 2
int psz_amd_set_decoder(psz_resource* m, int kind);

/* Archive layout.  Both are the reference phf format (chunk c of sublen codes at par_entry[c]).
 *  BRICK (default when eligible: 3-D, x extent a multiple of the brick width): chunk = one brick
 *    row, predictor fused with the encoder and decoder with the reconstructor; chunks are laid
 *    out brick by brick with zero cells between brick regions.
 *  REFERENCE: chunks in index order, no gaps (byte-identical to the reference encoder). */
#define PSZ_AMD_LAYOUT_BRICK 0
#define PSZ_AMD_LAYOUT_REFERENCE 1
/* BRICK_FORCE: the brick layout also for small 2-D fields (BRICK keeps the reference layout for
 * 2-D fields with fewer than 4 bricks per CU, where it is faster). */
#define PSZ_AMD_LAYOUT_BRICK_FORCE 2
int psz_amd_set_layout(psz_resource* m, int layout);

/* Codebook source.  Quant codes, outliers, the error bound and the decompressed field are the
 * same in every mode; the codebook (hence the bitstream and, marginally, the CR) differs.  Every
 * archive is an ordinary phf archive: the reference decoder reads it.
 *  EXACT: the reference's codebook (its binary heap, hf_bk_impl1.seq.cc) of the full histogram,
 *    built on the host (compressor.inl:339-458): the archive is byte-identical to the reference
 *    encoder's output for the same codes and chunking.
 *  SAMPLED (default): no host round trip on the critical path.  3-D and 1-D brick fields: pass 1
 *    visits every 33rd brick first (17th / 9th / 5th / 3rd / all for fewer bricks) and hands that
 *    sample's histogram to the host mid-pass, which builds the two-queue Huffman codebook of
 *    sample + 1 per bin while pass 1 goes on (the device builder's algorithm, run on the host).
 *    Reference layout and 2-D bricks: the EXACT book of the full histogram (published by the
 *    predictor's last workgroup).  Spline fields and a sharded finish (reduced histogram): the
 *    two-queue codebook of the full histogram built on the DEVICE (book_device.hh; the same
 *    total bits as the heap's on the same histogram).
 *  STREAM (3-D brick fields): the sampled codebook, then ONE pass predicts and packs (k_brick3_
 *    stream: no code buffer, no gaps between bricks); experimental. */
#define PSZ_AMD_CODEBOOK_EXACT 0
#define PSZ_AMD_CODEBOOK_SAMPLED 1
#define PSZ_AMD_CODEBOOK_STREAM 2
int psz_amd_set_codebook(psz_resource* m, int mode);

/* ---- sharded compress (multi-GPU; the reference has no multi-GPU path) ----
 * A field split into tile-aligned slabs (z: multiples of 8 planes) is compressed one slab per
 * GPU with ONE codebook:
 *   1. psz_amd_compress_scan_*: pass 1 only (predict, histogram, outliers); the slab's
 *      histogram u32[2 * radius] is copied to OUT_d_hist (device, on the manager's stream),
 *      followed by one more word: the slab's outlier cells beyond its current capacity.
 *   2. the caller sums these u32[2 * radius + 1] of all slabs (e.g. an RCCL all-reduce).
 *   3. psz_amd_compress_finish: codebook from IN_d_hist (device u32[2 * radius + 1]; NULL: the
 *      slab's own histogram), encode, archive -- outputs as psz_compress_float.  When the last
 *      word is nonzero (some slab had more outliers than its capacity: past the reference's
 *      10 %), every slab's finish returns PSZ_WARN_OUTLIER_TOO_MANY, the slabs that overflowed
 *      have grown their capacity, and repeating steps 1-3 succeeds on every rank together.
 * psz_compress_analyize_float (cusz_rev1.h) is step 1 with the histogram exported to the host
 * (compressor.inl:305-337). */
int psz_amd_compress_scan_float(psz_resource* m, psz_rc2 rc, float* IN_d_data, uint32_t* OUT_d_hist);
int psz_amd_compress_scan_double(psz_resource* m, psz_rc2 rc, double* IN_d_data, uint32_t* OUT_d_hist);
int psz_amd_compress_finish(psz_resource* m, const uint32_t* IN_d_hist, psz_header* OUT_header,
                            uint8_t** OUT_d_compressed, size_t* OUT_compressed_bytes);

/* Value range of a device field of the manager's dtype and length: writes {min, max} as two
 * doubles to OUT_d_minmax (device memory), queued on the manager's stream (no host sync).  The
 * Rel (r2r) mode probe of libcusz.cc:287-293 / extrema.cuhip.inl:150-208, exported so that a
 * sharded compress can all-reduce the slabs' ranges before pass 1.  IN_len = 0 means the
 * manager's length. */
int psz_amd_value_range(psz_resource* m, const void* IN_d_data, size_t IN_len, double* OUT_d_minmax);

/* Merge per-slab archives (HOST memory, in field order) compressed with one shared codebook
 * into the archive of the whole field: the archive one process would have written for it
 * (chunks concatenated, par_entry rebased by the cells before each slab, outlier indices by
 * the slab's element offset).  elem_offsets (may be NULL) are checked against the running
 * sum.  *out_bytes receives the merged size; with out == NULL that is all (a size query,
 * PSZ_SUCCESS); with out_cap too small nothing is written and PSZ_AMD_ERR_INVALID_ARG is
 * returned.  Malformed parts: PSZ_AMD_ERR_BAD_ARCHIVE; parts that are not tile-aligned slabs of
 * the field: PSZ_ABORT_UNSUPPORTED_DIMENSION; parts of different runs (codebook, eb, dtype):
 * PSZ_AMD_ERR_INVALID_ARG / PSZ_ABORT_UNSUPPORTED_TYPE. */
int psz_amd_merge_archives(const uint8_t* const* parts, const size_t* part_bytes, int nparts,
                           const size_t* elem_offsets, psz_len full_len, uint8_t* out, size_t out_cap,
                           size_t* out_bytes);

const char* psz_amd_version(void);

/* The device codebook (no host round trip; NOT the reference's heap order, the same total bit
 * count): canonical Huffman book (u32[bklen]) and reverse book (4 * 64 + 2 * bklen bytes) of the
 * device histogram IN_d_hist (+ smooth per bin: 1 makes every symbol encodable), all device
 * pointers, on `stream`.  bklen <= 1024.  Spline fields, sharded finishes and the stream mode build
 * their book this way. */
int psz_amd_build_book_device(const uint32_t* IN_d_hist, int bklen, uint32_t smooth, uint32_t* OUT_d_book,
                              uint8_t* OUT_d_revbook, void* stream);

/* Status of this thread's last psz_create_resource_manager* call (PSZ_SUCCESS when it returned a
 * manager): the resource-manager API returns NULL on failure, as the reference does, and this
 * says why -- e.g. PSZ_ABORT_UNSUPPORTED_DIMENSION for a shape the build does not take. */
int psz_amd_last_create_status(void);

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_EXT_H */
