// common.h — shared helpers for the ainp HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ainp.h"

namespace ainp {

// Record the failing hip error for ainp_last_error(); returns AINP_ELAUNCH.
int record_error(hipError_t e, const char* where);
int record_msg(const char* msg);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int check_launch(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return record_error(e, where);
  return AINP_OK;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Upper bound of the persistent-grid multiplier of the bf16 (NP = 1) 3x3 conv
// kernels (conv_x6.hip conv_x6_occ16): BatchNorm partial rows and weight-
// gradient slabs are sized for it.
constexpr int X6_OCC_MAX = 4;
int conv_x6_occ16();

// Wave-level (64-lane) reductions.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
// D[row=(l>>4)*4+r][col=l&15] in register r.  Exact f32 fma chain.
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

}  // namespace ainp
