/* include/c_type.h -- portable scalar and shape types shared by the C API.
 *
 * ABI-identical to the reference's portable/include/c_type.h:42-74 (enum values and
 * struct layouts), so callers compiled against cuSZ's headers link unchanged.
 */
#ifndef CUSZ_AMD_C_TYPE_H
#define CUSZ_AMD_C_TYPE_H

#ifdef __cplusplus
extern "C" {
#endif

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

/* fixed-width aliases used throughout the API */
typedef uint8_t u1;
typedef uint16_t u2;
typedef uint32_t u4;
typedef uint64_t u8;
typedef unsigned long long ull;
typedef int8_t i1;
typedef int16_t i2;
typedef int32_t i4;
typedef int64_t i8;
typedef float f4;
typedef double f8;
typedef size_t szt;

/* element-type tags: F4 = float, F8 = double, ... (c_type.h:51) */
typedef enum { F4, F8, U1, U2, U4, U8, I1, I2, I4, I8, ULL } _portable_dtype;

/* platform tags (kept for ABI; this build is always AMDGPU / ROCM / HIP) */
typedef enum { CPU, NVGPU, AMDGPU, INTELGPU } _portable_device;
typedef enum { SEQ, SIMD, OPENMP, CUDA, ROCM, SYCL, THRUST_DPL } _portable_runtime;
typedef enum { VENDOR_NATIVE, KOKKOS, ONEAPI, HIP } _portable_toolkit;

typedef enum _portable_mem_control {
  Malloc, MallocHost, MallocManaged, MallocShared,
  Free, FreeHost, FreeManaged, FreeShared,
  ClearHost, ClearDevice,
  H2D, H2H, D2H, D2D,
  Async_H2D, Async_H2H, Async_D2H, Async_D2D,
  ToFile, FromFile,
  ExtremaScan,
  DBG,
} _portable_mem_control;

typedef enum { _SUCCESS, _FAIL_GENERAL, _FAIL_UNSUPPORTED_DTYPE, _NOT_IMPLIMENTED } _portable_error_status;

typedef void* _portable_stream_t;

/* x is the fastest-varying extent (CUDA dim3 order) */
typedef struct _portable_len3 {
  size_t x, y, z;
} _portable_len3;
typedef _portable_len3 _portable_dim3;

/* z-y-x "math" order */
typedef struct _portable_size3 {
  size_t z, y, x;
} _portable_size3;

typedef struct _portable_data_summary {
  f8 min, max, rng, std, avg;
} _portable_data_summary;

#ifdef __cplusplus
}
#endif

#endif /* CUSZ_AMD_C_TYPE_H */
