/* include/cusz/type.h -- enums and plain structs of the cuSZ C API.
 *
 * Layout/value-compatible with the reference psz/include/cusz/type.h:15-135:
 * psz_error_status, psz_mode, psz_predictor, psz_codec, psz_hist, psz_pipeline,
 * psz_rc2 (runtime config: mode, eb, radius), psz_compressor, psz_interp_params.
 */
#ifndef CUSZ_AMD_TYPE_H
#define CUSZ_AMD_TYPE_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "c_type.h"

typedef _portable_dtype psz_dtype;
typedef _portable_len3 psz_len3;
typedef _portable_len3 psz_len; /* up to 3-D */
typedef _portable_size3 psz_size3;
typedef _portable_device psz_device;
typedef _portable_runtime psz_runtime;
typedef _portable_runtime psz_backend;
typedef _portable_toolkit psz_toolkit;
typedef _portable_stream_t psz_stream_t;
typedef _portable_mem_control psz_mem_control;
typedef _portable_data_summary psz_data_summary;

/* return codes (type.h:42-53); the API returns these as int and never throws */
typedef enum {
  PSZ_SUCCESS,
  PSZ_WARN_RADIUS_TOO_LARGE,
  PSZ_WARN_OUTLIER_TOO_MANY,
  PSZ_ABORT_UNSUPPORTED_TYPE,
  PSZ_ABORT_UNSUPPORTED_DIMENSION,
  PSZ_ABORT_NOT_IMPLEMENTED,
  PSZ_ABORT_NO_SUCH_PREDICTOR,
  PSZ_ABORT_NO_SUCH_CODEC,
  PSZ_ABORT_TOO_MANY_UNPREDICTABLE,
  PSZ_ABORT_TOO_MANY_ENC_BREAK,
} psz_error_status;
typedef psz_error_status pszerror;
#define CUSZ_SUCCESS PSZ_SUCCESS

typedef uint8_t byte_t;

typedef enum { Abs, Rel } psz_mode;
typedef enum { Lorenzo, LorenzoZigZag, LorenzoProto, Spline } psz_predictor;
typedef enum { FP64toFP32, LogTransform, ShiftedLogTransform, Binning2x2, Binning2x1, Binning1x2 } _future_psz_preprocess;
typedef enum { Huffman, HuffmanRevisit, LC, FZCodec, RunLength, NullCodec } psz_codec;
typedef enum { HistogramGeneric, HistogramSparse, NullHistogram } psz_hist;

#define DEFAULT_PREDICTOR Lorenzo
#define DEFAULT_HISTOGRAM HistogramGeneric
#define DEFAULT_CODEC Huffman
#define NULL_HISTOGRAM NullHistogram
#define NULL_CODEC NullCodec

typedef struct psz_pipeline {
  psz_predictor predictor;
  psz_hist hist;
  psz_codec codec1;
  psz_codec codec2;
} psz_pipeline;

typedef struct psz_runtime_config2 {
  psz_mode mode;
  double eb;
  uint16_t radius;
} psz_rc2;

struct psz_context;
typedef struct psz_context psz_ctx;
struct psz_header;
typedef struct psz_header psz_header;

typedef struct psz_compressor {
  void* compressor;
  psz_ctx* ctx;
  psz_error_status last_error;
  void* mem;
} psz_compressor;

typedef struct psz_statistics {
  psz_data_summary odata, xdata;
  f8 score_PSNR, score_MSE, score_NRMSE, score_coeff;
  f8 max_err_abs, max_err_rel, max_err_pwrrel;
  size_t max_err_idx;
  f8 autocor_lag_one, autocor_lag_two;
  f8 user_eb;
  size_t len;
} psz_statistics;

/* cuSZ-i interpolation parameters (type.h:112-135); 40 B */
typedef struct psz_interp_params {
  double alpha, beta;
  bool use_md[6];
  bool use_natural[6];
  bool reverse[6];
  uint8_t auto_tuning;
} psz_interp_params;
typedef struct psz_interp_params INTERPOLATION_PARAMS;

static inline psz_interp_params make_default_params(void)
{
  psz_interp_params p;
  p.alpha = 1.75;
  p.beta = 4.0;
  for (int i = 0; i < 6; i++) p.use_md[i] = i < 2, p.use_natural[i] = 0, p.reverse[i] = 0;
  p.auto_tuning = 3;
  return p;
}

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_TYPE_H */
