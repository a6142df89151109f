// gemm3_lab.hip — lab for an fp32-accurate GEMM on bf16 MFMA (tools only).
//
// Each fp32 operand element x is split exactly into three bf16 pieces
// x = x0 + x1 + x2 (round-to-nearest each step: |x1| <= 2^-8|x|, |x2| <= 2^-16|x|)
// while it is staged into LDS, and the product is the six terms of order
// >= 2^-16: x2y0 + x1y1 + x0y2 + x1y0 + x0y1 + x0y0 (smallest first) on
// v_mfma_f32_32x32x16_bf16 with f32 accumulation.  Dropped terms are
// <= ~2^-23 |xy|, i.e. at the level of f32 rounding.  The lab times the three
// CNNBLSTM layer-0 GEMM shapes against the shipped f32-MFMA kernel and reports
// the error of both against an fp64 host reference on sampled outputs.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 gemm3_lab.hip -o gemm3_lab \
//     -L../ml-audio-inpainting_amd/ainp -lainp -Wl,-rpath,...
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../include/ainp.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int THREADS = 256;

__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// exact 3-way split of (a, b) -> packed bf16 pairs p0, p1, p2
__device__ __forceinline__ void split2(float a, float b, uint32_t& p0, uint32_t& p1,
                                       uint32_t& p2) {
  p0 = cvt_pk_bf16(a, b);
#ifdef LAB_NOSPLIT  // ceiling probe: same MFMA/LDS work, no split arithmetic (wrong results)
  p1 = p0;
  p2 = p0;
  return;
#endif
  const float ra = a - bf_lo(p0), rb = b - bf_hi(p0);
  p1 = cvt_pk_bf16(ra, rb);
  const float sa = ra - bf_lo(p1), sb = rb - bf_hi(p1);
  p2 = cvt_pk_bf16(sa, sb);
}

// LDS image of one operand: 3 planes of [128 rows][BK k] bf16, row stride
// RS bytes (BK=32: 80 B, BK=16: 48 B; conflict-free ds_read_b128 fragments).
template <int BK>
struct Img3 {
  static constexpr int RS = BK == 32 ? 80 : 48;
  static constexpr int PLANE = 128 * RS;
  static constexpr int BYTES = 3 * PLANE;
};

// 128 x BK fp32 operand tile -> registers -> split -> LDS.
//  KC: memory contiguous along k (element (r,k) at p[r*ld + k])
//  MC: memory contiguous along rows (element (r,k) at p[k*ld + r])
template <bool KC, int BK>
struct Stage {
  static constexpr int NV = 128 * BK / 4 / THREADS;  // float4 per thread
  float4 v[NV];

  __device__ __forceinline__ void load(const float* __restrict__ p, int64_t ld, int64_t r0,
                                       int64_t k0, int64_t R, int64_t K) {
    const int tid = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = tid + i * THREADS;
        const int rr = idx / (BK / 4), kk = (idx % (BK / 4)) * 4;
        const int64_t gr = r0 + rr, gk = k0 + kk;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < R && gk < K) x = *reinterpret_cast<const float4*>(p + gr * ld + gk);
        v[i] = x;
      }
    } else {
      // thread: 4 consecutive rows (rq) x NV consecutive k
      constexpr int KQ = BK / NV;           // k groups per tile
      const int kq = tid % KQ, rq = tid / KQ;
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        const int64_t gk = k0 + kq * NV + e, gr = r0 + 4 * rq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < K && gr < R) x = *reinterpret_cast<const float4*>(p + gk * ld + gr);
        v[e] = x;
      }
    }
  }

  __device__ __forceinline__ void store(unsigned char* img) const {
    using I = Img3<BK>;
    const int tid = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = tid + i * THREADS;
        const int rr = idx / (BK / 4), kk = (idx % (BK / 4)) * 4;
        uint32_t a0, a1, a2, b0, b1, b2;
        split2(v[i].x, v[i].y, a0, a1, a2);
        split2(v[i].z, v[i].w, b0, b1, b2);
        unsigned char* q = img + rr * I::RS + kk * 2;
        *reinterpret_cast<uint2*>(q) = make_uint2(a0, b0);
        *reinterpret_cast<uint2*>(q + I::PLANE) = make_uint2(a1, b1);
        *reinterpret_cast<uint2*>(q + 2 * I::PLANE) = make_uint2(a2, b2);
      }
    } else {
      constexpr int KQ = BK / NV;
      const int kq = tid % KQ, rq = tid / KQ;
      const float* f = reinterpret_cast<const float*>(v);  // f[e*4 + j] = (row 4rq+j, k e)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        unsigned char* q = img + (4 * rq + j) * I::RS + kq * NV * 2;
        if (NV == 4) {
          uint32_t a0, a1, a2, b0, b1, b2;
          split2(f[0 * 4 + j], f[1 * 4 + j], a0, a1, a2);
          split2(f[2 * 4 + j], f[3 * 4 + j], b0, b1, b2);
          *reinterpret_cast<uint2*>(q) = make_uint2(a0, b0);
          *reinterpret_cast<uint2*>(q + I::PLANE) = make_uint2(a1, b1);
          *reinterpret_cast<uint2*>(q + 2 * I::PLANE) = make_uint2(a2, b2);
        } else {  // NV == 2
          uint32_t a0, a1, a2;
          split2(f[0 * 4 + j], f[1 * 4 + j], a0, a1, a2);
          *reinterpret_cast<uint32_t*>(q) = a0;
          *reinterpret_cast<uint32_t*>(q + I::PLANE) = a1;
          *reinterpret_cast<uint32_t*>(q + 2 * I::PLANE) = a2;
        }
      }
    }
  }
};

template <int BK>
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int plane, int row, int s,
                                       int h) {
  using I = Img3<BK>;
  const uint4 u =
      *reinterpret_cast<const uint4*>(img + plane * I::PLANE + row * I::RS + (16 * s + 8 * h) * 2);
  return __builtin_bit_cast(bf16x8, u);
}

struct Ptrs {
  const float* A[2];
  const float* B[2];
  float* C[2];
  int ksum;  // 1: grid.y segments are summed into C[0] (one pointer batch per K segment)
};

template <bool AKC, bool BKC, int BK, int WGS, bool DB = false>
__global__ __launch_bounds__(THREADS, WGS) void gemm3_kernel(int64_t M, int64_t N, int64_t K,
                                                              Ptrs P, int64_t lda, int64_t ldb,
                                                              int64_t ldc, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[(DB ? 4 : 2) * Img3<BK>::BYTES];
  unsigned char* As = smem;
  unsigned char* Bs = smem + Img3<BK>::BYTES;

  const int64_t nwg = gridDim.x;
  const int64_t bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8;
  const int64_t q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + 127) / 128;
  const int64_t group = 8;
  const int64_t per_group = group * tiles_m;
  const int64_t g = bid / per_group;
  const int64_t first_n = g * group;
  const int64_t gsize = (tiles_n - first_n) < group ? (tiles_n - first_n) : group;
  const int64_t in_g = bid % per_group;
  const int64_t tn = first_n + (in_g % gsize);
  const int64_t tm = in_g / gsize;
  const int64_t m0 = tm * 128, n0 = tn * 128;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nseg = P.ksum ? 2 : 1;
  const int b = P.ksum ? 0 : blockIdx.y;
  const int64_t nk = (K + BK - 1) / BK;
  const int64_t total = nk * nseg;
  Stage<AKC, BK> la;
  Stage<BKC, BK> lb;
  auto src = [&](int64_t it, const float*& a, const float*& bb, int64_t& k0) {
    const int seg = P.ksum ? (int)(it / nk) : b;
    a = P.A[seg];
    bb = P.B[seg];
    k0 = (it % nk) * BK;
  };
  {
    const float *a, *bb;
    int64_t k0;
    src(0, a, bb, k0);
    la.load(a, lda, m0, k0, M, K);
    lb.load(bb, ldb, n0, k0, N, K);
  }
  auto mma = [&](const unsigned char* Ai, const unsigned char* Bi) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 a[3][2], bq[3][2];
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          a[p][i] = frag<BK>(Ai, p, wm + i * 32 + li, s, lh);
          bq[p][i] = frag<BK>(Bi, p, wn + i * 32 + li, s, lh);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], bq[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], bq[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[2][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], bq[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[0][j], c, 0, 0, 0);
          acc[i][j] = c;
        }
    }
  };
  if (!DB) {
    for (int64_t it = 0; it < total; ++it) {
      if (it > 0) __syncthreads();
      la.store(As);
      lb.store(Bs);
      __syncthreads();
      if (it + 1 < total) {
        const float *a, *bb;
        int64_t k0;
        src(it + 1, a, bb, k0);
        la.load(a, lda, m0, k0, M, K);
        lb.load(bb, ldb, n0, k0, N, K);
      }
      mma(As, Bs);
    }
  } else {
    // double-buffered: one barrier per K-tile; tile it+1 is split/stored into
    // the other buffer while tile it's MFMAs run
    constexpr int IB = Img3<BK>::BYTES;
    la.store(smem);
    lb.store(smem + IB);
    if (total > 1) {
      const float *a, *bb;
      int64_t k0;
      src(1, a, bb, k0);
      la.load(a, lda, m0, k0, M, K);
      lb.load(bb, ldb, n0, k0, N, K);
    }
    __syncthreads();
    for (int64_t it = 0; it < total; ++it) {
      unsigned char* cur = smem + (it & 1) * 2 * IB;
      unsigned char* nxt = smem + ((it + 1) & 1) * 2 * IB;
      mma(cur, cur + IB);
      if (it + 1 < total) {
        la.store(nxt);
        lb.store(nxt + IB);
        if (it + 2 < total) {
          const float *a, *bb;
          int64_t k0;
          src(it + 2, a, bb, k0);
          la.load(a, lda, m0, k0, M, K);
          lb.load(bb, ldb, n0, k0, N, K);
        }
      }
      __syncthreads();
    }
  }
  float* C = P.C[b];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) C[m * ldc + n] = acc[i][j][r];
      }
    }
}

// ---- 16x16x32 variant: K-tile 32 ([row][32 k] planes, 80-byte rows), wave
// tile 64x64 as 4x4 MFMA tiles of 16x16 (lane (r = l&15, g = l>>4) holds
// k = 8g..8g+7 of row r: one ds_read_b128 per fragment)
typedef float f32x4l __attribute__((ext_vector_type(4)));
template <bool AKC, bool BKC, int WGS>
__global__ __launch_bounds__(THREADS, WGS) void gemm16_kernel(int64_t M, int64_t N, int64_t K,
                                                               Ptrs P, int64_t lda, int64_t ldb,
                                                               int64_t ldc, int tiles_n) {
  constexpr int BK = 32;
  using I = Img3<BK>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * I::BYTES];
  unsigned char* As = smem;
  unsigned char* Bs = smem + I::BYTES;
  const int64_t nwg = gridDim.x;
  const int64_t bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8;
  const int64_t q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + 127) / 128;
  const int64_t per_group = 8 * tiles_m;
  const int64_t g8 = bid / per_group;
  const int64_t first_n = g8 * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t tn = first_n + (in_g % gsize), tm = in_g / gsize;
  const int64_t m0 = tm * 128, n0 = tn * 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int l16 = lane & 15, lg = lane >> 4;
  f32x4l acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4l{0.f, 0.f, 0.f, 0.f};
  const int b = P.ksum ? 0 : blockIdx.y;
  const int nseg = P.ksum ? 2 : 1;
  const int64_t nk = (K + BK - 1) / BK, total = nk * nseg;
  Stage<AKC, BK> la;
  Stage<BKC, BK> lb;
  auto src = [&](int64_t it, const float*& a, const float*& bb, int64_t& k0) {
    const int seg = P.ksum ? (int)(it / nk) : b;
    a = P.A[seg];
    bb = P.B[seg];
    k0 = (it % nk) * BK;
  };
  {
    const float *a, *bb;
    int64_t k0;
    src(0, a, bb, k0);
    la.load(a, lda, m0, k0, M, K);
    lb.load(bb, ldb, n0, k0, N, K);
  }
  for (int64_t it = 0; it < total; ++it) {
    if (it > 0) __syncthreads();
    la.store(As);
    lb.store(Bs);
    __syncthreads();
    if (it + 1 < total) {
      const float *a, *bb;
      int64_t k0;
      src(it + 1, a, bb, k0);
      la.load(a, lda, m0, k0, M, K);
      lb.load(bb, ldb, n0, k0, N, K);
    }
    bf16x8 bq[3][4];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) bq[p][j] = frag<BK>(Bs, p, wn + 16 * j + l16, lg >> 1, lg & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 a[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = frag<BK>(As, p, wm + 16 * i + l16, lg >> 1, lg & 1);
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const int pa = t == 0 ? 2 : (t == 1 || t == 3) ? 1 : 0;
        const int pb = t == 2 ? 2 : (t == 1 || t == 4) ? 1 : 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[pa], bq[pb][j], acc[i][j], 0, 0, 0);
      }
    }
  }
  float* C = P.C[b];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn + 16 * j + l16;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm + 16 * i + 4 * lg + r;
        if (m < M) C[m * ldc + n] = acc[i][j][r];
      }
    }
}

// ---- 8-wave variant (KC/KC only): 512 threads per 128x128 tile, wave = 64x32
template <int WGS>
__global__ __launch_bounds__(512, WGS) void gemm3w8_kernel(int64_t M, int64_t N, int64_t K,
                                                            Ptrs P, int64_t lda, int64_t ldb,
                                                            int64_t ldc, int tiles_n) {
  constexpr int BK = 16;
  using I = Img3<BK>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * I::BYTES];
  unsigned char* As = smem;
  unsigned char* Bs = smem + I::BYTES;
  const int64_t nwg = gridDim.x;
  const int64_t bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8;
  const int64_t q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + 127) / 128;
  const int64_t per_group = 8 * tiles_m;
  const int64_t g = bid / per_group;
  const int64_t first_n = g * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t tn = first_n + (in_g % gsize), tm = in_g / gsize;
  const int64_t m0 = tm * 128, n0 = tn * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 2) * 64, wn = (wave & 3) * 32;
  const int li = lane & 31, lh = lane >> 5;
  const int b = blockIdx.y;
  const float* A = P.A[b];
  const float* B = P.B[b];
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int rr = tid >> 2, kk = (tid & 3) * 4;
  float4 va, vb;
  auto load = [&](int64_t k0) {
    va = (m0 + rr < M) ? *reinterpret_cast<const float4*>(A + (m0 + rr) * lda + k0 + kk)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    vb = (n0 + rr < N) ? *reinterpret_cast<const float4*>(B + (n0 + rr) * ldb + k0 + kk)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto store = [&]() {
    uint32_t a0, a1, a2, b0, b1, b2;
    unsigned char* q = As + rr * I::RS + kk * 2;
    split2(va.x, va.y, a0, a1, a2);
    split2(va.z, va.w, b0, b1, b2);
    *reinterpret_cast<uint2*>(q) = make_uint2(a0, b0);
    *reinterpret_cast<uint2*>(q + I::PLANE) = make_uint2(a1, b1);
    *reinterpret_cast<uint2*>(q + 2 * I::PLANE) = make_uint2(a2, b2);
    q = Bs + rr * I::RS + kk * 2;
    split2(vb.x, vb.y, a0, a1, a2);
    split2(vb.z, vb.w, b0, b1, b2);
    *reinterpret_cast<uint2*>(q) = make_uint2(a0, b0);
    *reinterpret_cast<uint2*>(q + I::PLANE) = make_uint2(a1, b1);
    *reinterpret_cast<uint2*>(q + 2 * I::PLANE) = make_uint2(a2, b2);
  };
  const int64_t nk = K / BK;
  load(0);
  for (int64_t it = 0; it < nk; ++it) {
    if (it > 0) __syncthreads();
    store();
    __syncthreads();
    if (it + 1 < nk) load((it + 1) * BK);
    bf16x8 a[3][2], bq[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < 2; ++i) a[p][i] = frag<BK>(As, p, wm + i * 32 + li, 0, lh);
      bq[p] = frag<BK>(Bs, p, wn + li, 0, lh);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x16 c = acc[i];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], bq[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], bq[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[2], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], bq[0], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[1], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], bq[0], c, 0, 0, 0);
      acc[i] = c;
    }
  }
  float* C = P.C[b];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t n = n0 + wn + li;
    if (n >= N) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (m < M) C[m * ldc + n] = acc[i][r];
    }
  }
}

// ------------------------------------------------------------------ harness
struct Shape {
  const char* name;
  int64_t M, N, K;
  bool akc, bkc;
  int64_t lda, ldb;
  int ksum;  // 2 K segments summed (dgrad over both directions)
  int64_t a_rows, a_cols, b_rows, b_cols;  // allocation of one A / B buffer
};

static void fill(std::vector<float>& v, uint64_t seed, float scale) {
  uint64_t s = seed * 6364136223846793005ull + 1442695040888963407ull;
  for (auto& x : v) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    x = scale * ((float)((s >> 40) & 0xffffff) / 16777216.0f - 0.5f);
  }
}

template <bool AKC, bool BKC, int BK, int WGS, bool DB>
static void launch3(const Shape& s, const Ptrs& P, hipStream_t st) {
  const int tiles_n = (int)((s.N + 127) / 128);
  const int tiles_m = (int)((s.M + 127) / 128);
  dim3 grid(tiles_m * tiles_n, s.ksum ? 1 : 2);
  hipLaunchKernelGGL((gemm3_kernel<AKC, BKC, BK, WGS, DB>), grid, dim3(THREADS), 0, st, s.M, s.N, s.K,
                     P, s.lda, s.ldb, s.N, tiles_n);
}

template <int BK, int WGS, bool DB = false>
static void run3(const Shape& s, const Ptrs& P, hipStream_t st) {
  if (s.akc && s.bkc) launch3<true, true, BK, WGS, DB>(s, P, st);
  else if (s.akc) launch3<true, false, BK, WGS, DB>(s, P, st);
  else if (s.bkc) launch3<false, true, BK, WGS, DB>(s, P, st);
  else launch3<false, false, BK, WGS, DB>(s, P, st);
}

int main() {
  const int64_t NT = 10688, I = 16448, G = 512;
  Shape shapes[] = {
      // fwd: zx[:, d] = X W_d^T   (A = X [NT][I] k-contig, B = W_d [G][I] k-contig)
      {"fwd  M=10688 N=512x2 K=16448", NT, G, I, true, true, I, I, 0, NT, I, G, I},
      // dgrad: dX = sum_d dg_d W_d (A = dg [NT][2G] k-contig, B = W_d [G][I] n-contig)
      {"dgrad M=10688 N=16448 K=512x2", NT, I, G, true, false, 2 * G, I, 1, NT, 2 * G, G, I},
      // wgrad: dW_d = dg_d^T X (A = dg_d^T: (m,k)=dg[k][m] m-contig, B = X n-contig)
      {"wgrad M=512 N=16448 K=10688 x2", G, I, NT, false, false, 2 * G, I, 0, NT, 2 * G, NT, I},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    std::vector<float> hA(s.a_rows * s.a_cols), hB0(s.b_rows * s.b_cols), hB1(s.b_rows * s.b_cols);
    fill(hA, 1, 2.0f);
    fill(hB0, 2, 0.02f);
    fill(hB1, 3, 0.02f);
    float *dA, *dB0, *dB1, *dC0, *dC1, *dR0, *dR1;
    const int64_t csz = s.M * s.N;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB0, hB0.size() * 4));
    CK(hipMalloc(&dB1, hB1.size() * 4));
    CK(hipMalloc(&dC0, csz * 4));
    CK(hipMalloc(&dC1, csz * 4));
    CK(hipMalloc(&dR0, csz * 4));
    CK(hipMalloc(&dR1, csz * 4));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB0, hB0.data(), hB0.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB1, hB1.data(), hB1.size() * 4, hipMemcpyHostToDevice));
    // per-direction A pointers: fwd shares X; dgrad/wgrad take column halves of dg
    const float* A0 = dA;
    const float* A1 = (s.akc && s.ksum) || !s.akc ? dA + G : dA;
    if (s.akc && !s.ksum) A1 = dA;
    Ptrs P{{A0, A1}, {dB0, dB1}, {dC0, dC1}, s.ksum};
    // shipped f32 kernel (with stream-K workspace when it wants one)
    const float* Ar[2] = {A0, A1};
    const float* Br[2] = {dB0, dB1};
    float* Cr[2] = {dR0, s.ksum ? dR0 : dR1};
    const int64_t sam = s.akc ? s.lda : 1, sak = s.akc ? 1 : s.lda;
    const int64_t sbk = s.bkc ? 1 : s.ldb, sbn = s.bkc ? s.ldb : 1;
    const size_t wsb = ainp_gemm_f32_workspace(s.M, s.N, s.K, 2, 1, s.ksum);
    void* ws = nullptr;
    if (wsb) CK(hipMalloc(&ws, wsb));
    auto ref = [&]() {
      int rc = ainp_gemm_f32_ws(s.M, s.N, s.K, 1.f, Ar, sam, sak, 0, Br, sbk, sbn, 0, 0.f, Cr, s.N,
                                1, 0, nullptr, nullptr, 2, 1, s.ksum, ws, wsb, st);
      if (rc) {
        fprintf(stderr, "ref rc %d %s\n", rc, ainp_last_error());
        exit(1);
      }
    };
    const double flop = 2.0 * s.M * s.N * s.K * 2;
    auto timeit = [&](auto fn) {
      for (int w = 0; w < 3; ++w) fn();
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      const int reps = 10;
      for (int r = 0; r < reps; ++r) fn();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms / reps;
    };
    // host fp64 reference on sampled outputs of batch 0 (dgrad: the summed output)
    std::vector<float> hB0c = hB0, hB1c = hB1;
    auto aval = [&](int d, int64_t m, int64_t k) -> double {
      const int64_t off = (d == 1 && (s.ksum || !s.akc)) ? G : 0;
      return s.akc ? hA[m * s.lda + k + off] : hA[k * s.lda + m + off];
    };
    auto bval = [&](int d, int64_t n, int64_t k) -> double {
      const std::vector<float>& B = d ? hB1c : hB0c;
      return s.bkc ? B[n * s.ldb + k] : B[k * s.ldb + n];
    };
    const int NS = 400;
    std::vector<int64_t> sm(NS), sn(NS);
    std::vector<double> want(NS), amag(NS);
    for (int q = 0; q < NS; ++q) {
      sm[q] = (q * 7919LL + 13) % s.M;
      sn[q] = (q * 104729LL + 7) % s.N;
      double acc = 0, mag = 0;
      for (int d = 0; d < (s.ksum ? 2 : 1); ++d)
        for (int64_t k = 0; k < s.K; ++k) {
          const double p = aval(d, sm[q], k) * bval(d, sn[q], k);
          acc += p;
          mag += fabs(p);
        }
      want[q] = acc;
      amag[q] = mag;
    }
    auto check = [&](float* dC, const char* nm, float ms) {
      std::vector<float> h(csz);
      CK(hipMemcpy(h.data(), dC, csz * 4, hipMemcpyDeviceToHost));
      double worst = 0, worst_rel_mag = 0, num = 0, den = 0;
      for (int q = 0; q < NS; ++q) {
        const double d = fabs((double)h[sm[q] * s.N + sn[q]] - want[q]);
        num += d * d;
        den += want[q] * want[q];
        worst = fmax(worst, d);
        worst_rel_mag = fmax(worst_rel_mag, d / amag[q]);
      }
      printf("  %-34s %8.3f ms %7.1f TF   relL2 %.2e  max|err|/sum|ab| %.2e\n", nm, ms,
             flop / ms / 1e9, sqrt(num / den), worst_rel_mag);
    };
    printf("%s\n", s.name);
    float mr = timeit(ref);
    check(dR0, "shipped f32 MFMA", mr);
    auto prod = [&](int flags, bool use_ws) {
      int rc = ainp_gemm_f32_ex(s.M, s.N, s.K, 1.f, Ar, sam, sak, 0, Br, sbk, sbn, 0, 0.f, Cr, s.N,
                                1, 0, nullptr, nullptr, 2, 1, s.ksum, flags, use_ws ? ws : nullptr,
                                use_ws ? wsb : 0, st);
      if (rc) {
        fprintf(stderr, "prod rc %d %s\n", rc, ainp_last_error());
        exit(1);
      }
    };
    float mp = timeit([&] { prod(0, true); });
    check(dR0, "product x6 (stream-K if chosen)", mp);
    float mq = timeit([&] { prod(0, false); });
    check(dR0, "product x6 plain grid", mq);
    if (s.akc && s.bkc) {
      const int tn = (int)((s.N + 127) / 128), tmm = (int)((s.M + 127) / 128);
      float w2 = timeit([&] {
        hipLaunchKernelGGL((gemm3w8_kernel<2>), dim3(tmm * tn, 2), dim3(512), 0, st, s.M, s.N,
                           s.K, P, s.lda, s.ldb, s.N, tn);
      });
      check(dC0, "8-wave 64x32/wave, 2 WG/CU", w2);
      float w3 = timeit([&] {
        hipLaunchKernelGGL((gemm3w8_kernel<3>), dim3(tmm * tn, 2), dim3(512), 0, st, s.M, s.N,
                           s.K, P, s.lda, s.ldb, s.N, tn);
      });
      check(dC0, "8-wave 64x32/wave, 3 WG/CU", w3);
    }
    {
      const int tn = (int)((s.N + 127) / 128), tmm = (int)((s.M + 127) / 128);
      const dim3 grid(tmm * tn, P.ksum ? 1 : 2);
#define AINP_G16(AK, BK_)                                                                      \
  if (s.akc == AK && s.bkc == BK_) {                                                           \
    float t16 = timeit([&] {                                                                   \
      hipLaunchKernelGGL((gemm16_kernel<AK, BK_, 2>), grid, dim3(THREADS), 0, st, s.M, s.N,    \
                         s.K, P, s.lda, s.ldb, s.N, tn);                                       \
    });                                                                                        \
    check(dC0, "16x16x32 x6 BK32 2WG", t16);                                                   \
  }
      AINP_G16(true, true) AINP_G16(true, false) AINP_G16(false, true) AINP_G16(false, false)
#undef AINP_G16
    }
    float m1 = timeit([&] { run3<16, 2, true>(s, P, st); });
    CK(hipGetLastError());
    check(dC0, "bf16x6 BK16 2WG double-buffered", m1);
    float m4 = timeit([&] { run3<32, 2, true>(s, P, st); });
    CK(hipGetLastError());
    check(dC0, "bf16x6 BK32 1WG double-buffered", m4);
    float m2 = timeit([&] { run3<16, 3>(s, P, st); });
    CK(hipGetLastError());
    check(dC0, "bf16x6 BK16 3WG", m2);
    float m3 = timeit([&] { run3<16, 2>(s, P, st); });
    check(dC0, "bf16x6 BK16 2WG", m3);
    CK(hipFree(dA)); CK(hipFree(dB0)); CK(hipFree(dB1)); CK(hipFree(dC0)); CK(hipFree(dC1));
    CK(hipFree(dR0)); CK(hipFree(dR1));
    if (ws) CK(hipFree(ws));
  }
  printf("done\n");
  return 0;
}
