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

// The BatchNorm-backward reduce a 3x3 data gradient can fuse into its
// epilogue (conv_x6.hip Bnr helpers; ainp_conv3x3_dgrad_bnr): the consuming
// layer's pre-BatchNorm output y (channel-last, fp32 or bf16 storage), its
// BatchNorm+ReLU affine and saved (mean, rstd).  y == nullptr: none.
struct Bnr {
  const void* y;
  const float* sc;
  const float* sh;
  const float* save;   // mean [C], rstd [C]
  int y16;             // y in bf16 storage
};
// The fused reduce is latency-sensitive (it sits in the epilogue of
// latency-bound kernels), so the pieces are split: y is loaded early
// (bnr_ld4: raw words, branch-free -- a masked pixel loads element 0), the
// per-channel constants are staged once into LDS (bnr_stage: rows scale,
// shift, mean, rstd of stride CS), and the epilogue only forms the terms.
__device__ __forceinline__ uint4 bnr_ld4(const Bnr& b, int64_t e) {
  if (b.y16) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(b.y) + e);
    return make_uint4(u.x, u.y, 0u, 0u);
  }
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(b.y) + e);
}
__device__ __forceinline__ void bnr_dec4(int y16, uint4 r, float (&yv)[4]) {
  if (y16) {
    yv[0] = __uint_as_float(r.x << 16);
    yv[1] = __uint_as_float(r.x & 0xffff0000u);
    yv[2] = __uint_as_float(r.y << 16);
    yv[3] = __uint_as_float(r.y & 0xffff0000u);
  } else {
    yv[0] = __uint_as_float(r.x);
    yv[1] = __uint_as_float(r.y);
    yv[2] = __uint_as_float(r.z);
    yv[3] = __uint_as_float(r.w);
  }
}
__device__ __forceinline__ void bnr_stage(const Bnr& b, float* sbn, int C, int CS, int tid,
                                          int nt) {
  for (int i = tid; i < 4 * C; i += nt) {
    const int k = i / C, c = i % C;
    sbn[k * CS + c] = k == 0 ? b.sc[c] : k == 1 ? b.sh[c] : b.save[(k - 2) * C + c];
  }
}
// channels c0 .. c0+3: y values yv, dx values v -> s = gz, q = gz * xhat as
// bn_relu_bwd_reduce_cl forms them (zeros where !ok)
template <int CS>
__device__ __forceinline__ void bnr_terms4(const float* sbn, int c0, const float (&yv)[4],
                                           const float (&v)[4], bool ok, float* s, float* q) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + k;
    const float gz = fmaf(yv[k], sbn[c], sbn[CS + c]) > 0.f ? v[k] : 0.f;
    s[k] = ok ? gz : 0.f;
    q[k] = ok ? gz * ((yv[k] - sbn[2 * CS + c]) * sbn[3 * CS + c]) : 0.f;
  }
}

// sums[o] = fixed-order sum of partial[0 .. nblk)[o], o < C2 (bn.hip)
int bn_cl_sum_partials(const double* partial, int nblk, int C2, double* sums, hipStream_t s);

// Two fp32 -> packed bf16 (round-to-nearest-even, lo in the low half): the
// gfx950 conversion instruction (a software rounding sequence otherwise)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

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
