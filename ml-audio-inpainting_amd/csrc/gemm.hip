// gemm.hip — strided / batched fp32 GEMM on gfx950 MFMA.
//
// Replaces the ATen GEMMs behind nn.LSTM input projections and nn.Linear of
// models/CNNBLSTM/model.py:46-50,77,80 (forward and backward).  Two main loops
// share the tiling, batching, stream-K and epilogue code:
//
//  * x6 (default): each fp32 operand element is split EXACTLY into three bf16
//    pieces x = x0 + x1 + x2 (round-to-nearest at each step, |x1| <= 2^-8|x|,
//    |x2| <= 2^-16|x|) while it is staged into LDS, and a*b is accumulated as
//    the six cross terms of order >= 2^-16 (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 +
//    a0b0, smallest first) on v_mfma_f32_32x32x16_bf16 with f32 accumulation.
//    The dropped terms are <= ~2^-23|ab|, the level of f32 rounding, so results
//    are fp32-accurate (tests/test_gpu_kernels.py checks both paths against
//    fp64); the bf16 MFMA rate (16x f32) leaves 2.7x of f32 headroom.
//  * exact (AINP_GEMM_EXACT_F32): v_mfma_f32_32x32x2_f32, an exact k-ordered
//    fmaf chain (MI355X_MICROARCH "Matrix cores").
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves as 2x2, each
// wave 64x64 = 2x2 MFMA 32x32 tiles, 64 accumulator VGPRs), one LDS image per
// operand with the next K-tile prefetched in registers.
//  exact: K-tile 32; k-contiguous operands keep a [row][k] f32 image (16-byte
//    stores, one ds_read_b128 = 4 MFMA k-steps per lane), row-contiguous
//    operands a [k][row] image.  The k order inside an 8-k group is lane-half
//    h -> k = 4h+e, identical for A and B, so the sum over k is unchanged.
//  x6: K-tile 16; three bf16 planes [row][16 k] per operand with 48-byte rows
//    (conflict-free ds_read_b128 fragments: lane (r, h) reads k = 8h..8h+7 of
//    row r, the 32x32x16 operand map, identical for A and B).
#include <stdlib.h>

#include "common.h"

namespace ainp {

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int GEMM_THREADS = 256;

struct GemmPtrs {
  const float* A[8];
  const float* B[8];
  float* C[8];
  const float* bias1[8];
  const float* bias2[8];
  int64_t sA, sB, sC;  // strides between strided batches
  int nptr;            // pointer batches; batch b -> (b % nptr, b / nptr)
  int ksplit_mode;     // 0 none, 1 sum all batches into C[0], 2 per pointer batch
};

typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16v mfma32(float a, float b, f32x16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16v mfma32bf(bf16x8v a, bf16x8v b, f32x16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Load a 128xBK operand tile (128 rows along m or n, BK along k) into
// registers.  KC: source contiguous along k (element (r,k) at p[r*ld + k]);
// otherwise contiguous along rows (element (r,k) at p[k*ld + r]).
// VEC: 16-byte vector loads are legal (ld%4==0, extent%4==0, base aligned).
template <bool KC, bool VEC>
struct TileLoader {
  static constexpr int NV = (128 * BK) / (4 * GEMM_THREADS);  // float4 per thread = 4
  float4 v[NV];

  __device__ __forceinline__ void load(const float* __restrict__ p, int64_t ld,
                                       int64_t r0, int64_t k0, int64_t R,
                                       int64_t K) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + i * GEMM_THREADS;  // 0..1023
      int rr, kk;
      if (KC) {  // 8 float4 per row of 32 k
        rr = idx >> 3;
        kk = (idx & 7) * 4;
      } else {  // 32 float4 per k-row of 128 rows
        kk = idx >> 5;
        rr = (idx & 31) * 4;
      }
      const int64_t gr = r0 + rr, gk = k0 + kk;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KC) {
        if (gr < R) {
          const float* q = p + gr * ld + gk;
          if (VEC) {
            if (gk < K) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gk + 0 < K) x.x = q[0];
            if (gk + 1 < K) x.y = q[1];
            if (gk + 2 < K) x.z = q[2];
            if (gk + 3 < K) x.w = q[3];
          }
        }
      } else {
        if (gk < K) {
          const float* q = p + gk * ld + gr;
          if (VEC) {
            if (gr < R) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gr + 0 < R) x.x = q[0];
            if (gr + 1 < R) x.y = q[1];
            if (gr + 2 < R) x.z = q[2];
            if (gr + 3 < R) x.w = q[3];
          }
        }
      }
      v[i] = x;
    }
  }

  // KC: image s[r][k] (row length 36: 16-byte rows, conflict-free b128 reads
  // and writes).  MC: image s[k][r] (row length 132).  Both 16-byte stores.
  __device__ __forceinline__ void store(float* s) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + i * GEMM_THREADS;
      if (KC) {
        const int rr = idx >> 3, kk = (idx & 7) * 4;
        *reinterpret_cast<float4*>(&s[rr * 36 + kk]) = v[i];
      } else {
        const int kk = idx >> 5, rr = (idx & 31) * 4;
        *reinterpret_cast<float4*>(&s[kk * 132 + rr]) = v[i];
      }
    }
  }
};

template <bool KC>
struct Img {
  static constexpr int SIZE = KC ? 128 * 36 : BK * 132;  // floats
  // fragment of k-group kg (8 k): lane (row r, half h) gets k = 8kg+4h+e
  __device__ __forceinline__ static float4 frag(const float* s, int r, int kg, int h) {
    if (KC) return *reinterpret_cast<const float4*>(&s[r * 36 + kg * 8 + 4 * h]);
    const int k = kg * 8 + 4 * h;
    return make_float4(s[(k + 0) * 132 + r], s[(k + 1) * 132 + r], s[(k + 2) * 132 + r],
                       s[(k + 3) * 132 + r]);
  }
};

// ======================================================= x6 (split bf16) path
namespace x6 {
constexpr int KT = 16;            // K-tile
constexpr int RS = 48;            // bytes per image row: 16 bf16 + 16 B pad
constexpr int PLANE = 128 * RS;   // one bf16 plane of a 128-row operand tile
constexpr int IMG = 3 * PLANE;    // three planes

__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// exact three-way split of (a, b) into packed bf16 pairs p0 + p1 + p2
__device__ __forceinline__ void split2(float a, float b, uint32_t& p0, uint32_t& p1,
                                       uint32_t& p2) {
  p0 = cvt_pk_bf16(a, b);
  const float ra = a - bf_lo(p0), rb = b - bf_hi(p0);
  p1 = cvt_pk_bf16(ra, rb);
  const float sa = ra - bf_lo(p1), sb = rb - bf_hi(p1);
  p2 = cvt_pk_bf16(sa, sb);
}

// 128 x 16 fp32 operand tile -> registers -> split -> three LDS planes.
//  KC: thread = one row x 4 consecutive k (two float4 per thread);
//  MC: thread = 4 consecutive rows x 2 consecutive k (one float4 per k), so the
//      4-row vector is transposed in registers into per-row k pairs.
template <bool KC, bool VEC>
struct Loader {
  float4 v[2];

  __device__ __forceinline__ void load(const float* __restrict__ p, int64_t ld, int64_t r0,
                                       int64_t k0, int64_t R, int64_t K) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KC) {
        const int idx = tid + i * GEMM_THREADS;
        const int64_t gr = r0 + (idx >> 2), gk = k0 + (idx & 3) * 4;
        if (gr < R) {
          const float* q = p + gr * ld + gk;
          if (VEC) {
            if (gk < K) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gk + 0 < K) x.x = q[0];
            if (gk + 1 < K) x.y = q[1];
            if (gk + 2 < K) x.z = q[2];
            if (gk + 3 < K) x.w = q[3];
          }
        }
      } else {
        const int64_t gk = k0 + 2 * (tid & 7) + i, gr = r0 + 4 * (tid >> 3);
        if (gk < K) {
          const float* q = p + gk * ld + gr;
          if (VEC) {
            if (gr < R) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gr + 0 < R) x.x = q[0];
            if (gr + 1 < R) x.y = q[1];
            if (gr + 2 < R) x.z = q[2];
            if (gr + 3 < R) x.w = q[3];
          }
        }
      }
      v[i] = x;
    }
  }

  __device__ __forceinline__ void store(unsigned char* img) const {
    const int tid = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = tid + i * GEMM_THREADS;
        uint32_t a0, a1, a2, b0, b1, b2;
        split2(v[i].x, v[i].y, a0, a1, a2);
        split2(v[i].z, v[i].w, b0, b1, b2);
        unsigned char* q = img + (idx >> 2) * RS + (idx & 3) * 8;
        *reinterpret_cast<uint2*>(q) = make_uint2(a0, b0);
        *reinterpret_cast<uint2*>(q + PLANE) = make_uint2(a1, b1);
        *reinterpret_cast<uint2*>(q + 2 * PLANE) = make_uint2(a2, b2);
      }
    } else {
      const float* f0 = reinterpret_cast<const float*>(&v[0]);
      const float* f1 = reinterpret_cast<const float*>(&v[1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t a0, a1, a2;
        split2(f0[j], f1[j], a0, a1, a2);
        unsigned char* q = img + (4 * (tid >> 3) + j) * RS + (tid & 7) * 4;
        *reinterpret_cast<uint32_t*>(q) = a0;
        *reinterpret_cast<uint32_t*>(q + PLANE) = a1;
        *reinterpret_cast<uint32_t*>(q + 2 * PLANE) = a2;
      }
    }
  }
};

__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int plane, int row, int h) {
  const uint4 u = *reinterpret_cast<const uint4*>(img + plane * PLANE + row * RS + 16 * h);
  return __builtin_bit_cast(bf16x8v, u);
}
}  // namespace x6

// ======================================================= bf16 operand path
// AINP_GEMM_BF16 (the bf16 configurations C3-C5): each fp32 operand element is
// rounded once to bf16 (round-to-nearest-even, v_cvt_pk_bf16_f32) while it is
// staged, and a*b accumulates in f32 on v_mfma_f32_32x32x16_bf16 -- torch's
// bf16-operand / fp32-accumulate autocast arithmetic.  K-tile 32, one plane per
// operand, 80-byte image rows (conflict-free ds_read_b128 fragments).
namespace b16 {
template <int KT> constexpr int rs() { return KT * 2 + 16; }   // image row: KT bf16 + 16 B pad
template <int KT> constexpr int img() { return 128 * rs<KT>(); }

// 128 x KT fp32 operand tile -> registers -> bf16 -> one LDS plane.
//  KC: thread = one row x 4 consecutive k (KT/8 float4 per thread);
//  MC: thread = 4 consecutive rows x k pairs {2p, 2p+1} + 16 g, g < KT/16.
template <bool KC, bool VEC, int KT = 32>
struct Loader {
  static constexpr int NV = KT / 8;
  static constexpr int RS = rs<KT>();
  float4 v[NV];

  __device__ __forceinline__ void load(const float* __restrict__ p, int64_t ld, int64_t r0,
                                       int64_t k0, int64_t R, int64_t K) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KC) {
        const int idx = tid + i * GEMM_THREADS;
        const int64_t gr = r0 + idx / (KT / 4), gk = k0 + (idx % (KT / 4)) * 4;
        if (gr < R) {
          const float* q = p + gr * ld + gk;
          if (VEC) {
            if (gk < K) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gk + 0 < K) x.x = q[0];
            if (gk + 1 < K) x.y = q[1];
            if (gk + 2 < K) x.z = q[2];
            if (gk + 3 < K) x.w = q[3];
          }
        }
      } else {
        const int64_t gk = k0 + 2 * (tid & 7) + (i & 1) + 16 * (i >> 1);
        const int64_t gr = r0 + 4 * (tid >> 3);
        if (gk < K) {
          const float* q = p + gk * ld + gr;
          if (VEC) {
            if (gr < R) x = *reinterpret_cast<const float4*>(q);
          } else {
            if (gr + 0 < R) x.x = q[0];
            if (gr + 1 < R) x.y = q[1];
            if (gr + 2 < R) x.z = q[2];
            if (gr + 3 < R) x.w = q[3];
          }
        }
      }
      v[i] = x;
    }
  }

  __device__ __forceinline__ void store(unsigned char* img) const {
    const int tid = threadIdx.x;
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int idx = tid + i * GEMM_THREADS;
        unsigned char* q = img + (idx / (KT / 4)) * RS + (idx % (KT / 4)) * 8;
        *reinterpret_cast<uint2*>(q) =
            make_uint2(x6::cvt_pk_bf16(v[i].x, v[i].y), x6::cvt_pk_bf16(v[i].z, v[i].w));
      }
    } else {
#pragma unroll
      for (int h = 0; h < KT / 16; ++h) {
        const float* f0 = reinterpret_cast<const float*>(&v[2 * h]);
        const float* f1 = reinterpret_cast<const float*>(&v[2 * h + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned char* q = img + (4 * (tid >> 3) + j) * RS + (tid & 7) * 4 + 32 * h;
          *reinterpret_cast<uint32_t*>(q) = x6::cvt_pk_bf16(f0[j], f1[j]);
        }
      }
    }
  }
};

// fragment of k-step ks (16 k): lane (row, half h) gets k = 16 ks + 8h .. +7
template <int KT>
__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int row, int ks, int h) {
  const uint4 u = *reinterpret_cast<const uint4*>(img + row * rs<KT>() + 32 * ks + 16 * h);
  return __builtin_bit_cast(bf16x8v, u);
}
}  // namespace b16

// ===================================================== main-loop policies
// Exact f32 path: K-tile 32, f32 images, 32x32x2 f32 MFMA.
template <bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolF32 {
  static constexpr int KT = BK;
  static constexpr int A_BYTES = Img<AKC>::SIZE * 4, B_BYTES = Img<BKC>::SIZE * 4;
  static constexpr int SMEM = A_BYTES + B_BYTES;
  using LA = TileLoader<AKC, AVEC>;
  using LB = TileLoader<BKC, BVEC>;
  __device__ static __forceinline__ void store(const LA& la, const LB& lb, unsigned char* sm) {
    la.store(reinterpret_cast<float*>(sm));
    lb.store(reinterpret_cast<float*>(sm + A_BYTES));
  }
  __device__ static __forceinline__ void compute(const unsigned char* sm, f32x16v (&acc)[2][2],
                                                 int wm, int wn, int li, int lh) {
    const float* As = reinterpret_cast<const float*>(sm);
    const float* Bs = reinterpret_cast<const float*>(sm + A_BYTES);
#pragma unroll
    for (int kg = 0; kg < BK / 8; ++kg) {
      float4 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = Img<AKC>::frag(As, wm + i * 32 + li, kg, lh);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Img<BKC>::frag(Bs, wn + j * 32 + li, kg, lh);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma32(af[i].x, bf[j].x, acc[i][j]);
          acc[i][j] = mfma32(af[i].y, bf[j].y, acc[i][j]);
          acc[i][j] = mfma32(af[i].z, bf[j].z, acc[i][j]);
          acc[i][j] = mfma32(af[i].w, bf[j].w, acc[i][j]);
        }
    }
  }
};

// x6 path: K-tile 16, three bf16 planes per operand, six 32x32x16 bf16 MFMAs.
template <bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolX6 {
  static constexpr int KT = x6::KT;
  static constexpr int SMEM = 2 * x6::IMG;
  using LA = x6::Loader<AKC, AVEC>;
  using LB = x6::Loader<BKC, BVEC>;
  __device__ static __forceinline__ void store(const LA& la, const LB& lb, unsigned char* sm) {
    la.store(sm);
    lb.store(sm + x6::IMG);
  }
  __device__ static __forceinline__ void compute(const unsigned char* sm, f32x16v (&acc)[2][2],
                                                 int wm, int wn, int li, int lh) {
    bf16x8v a[3][2], b[3][2];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[p][i] = x6::frag(sm, p, wm + i * 32 + li, lh);
        b[p][i] = x6::frag(sm + x6::IMG, p, wn + i * 32 + li, lh);
      }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16v c = acc[i][j];
        c = mfma32bf(a[2][i], b[0][j], c);
        c = mfma32bf(a[1][i], b[1][j], c);
        c = mfma32bf(a[0][i], b[2][j], c);
        c = mfma32bf(a[1][i], b[0][j], c);
        c = mfma32bf(a[0][i], b[1][j], c);
        c = mfma32bf(a[0][i], b[0][j], c);
        acc[i][j] = c;
      }
  }
};

// bf16 path: K-tile KT (32, or 64 with AINP_GEMM_B16_KT=64), one bf16 plane
// per operand, KT/16 rounds of four 32x32x16 MFMAs per tile.
template <bool AKC, bool BKC, bool AVEC, bool BVEC, int KTB = 32>
struct PolB16 {
  static constexpr int KT = KTB;
  static constexpr int IMG = b16::img<KT>();
  static constexpr int SMEM = 2 * IMG;
  using LA = b16::Loader<AKC, AVEC, KT>;
  using LB = b16::Loader<BKC, BVEC, KT>;
  __device__ static __forceinline__ void store(const LA& la, const LB& lb, unsigned char* sm) {
    la.store(sm);
    lb.store(sm + IMG);
  }
  __device__ static __forceinline__ void compute(const unsigned char* sm, f32x16v (&acc)[2][2],
                                                 int wm, int wn, int li, int lh) {
#pragma unroll
    for (int ks = 0; ks < KT / 16; ++ks) {
      bf16x8v a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = b16::frag<KT>(sm, wm + i * 32 + li, ks, lh);
        b[i] = b16::frag<KT>(sm + IMG, wn + i * 32 + li, ks, lh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32bf(a[i], b[j], acc[i][j]);
    }
  }
};

// main loop: PM_F32 exact f32, PM_X6 fp32-accurate split bf16, PM_B16 bf16 operands
constexpr int PM_F32 = 0, PM_X6 = 1, PM_B16 = 2, PM_B16K64 = 3;
template <int PM, bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolSel {
  using type = PolF32<AKC, BKC, AVEC, BVEC>;
};
template <bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolSel<PM_X6, AKC, BKC, AVEC, BVEC> {
  using type = PolX6<AKC, BKC, AVEC, BVEC>;
};
template <bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolSel<PM_B16, AKC, BKC, AVEC, BVEC> {
  using type = PolB16<AKC, BKC, AVEC, BVEC, 32>;
};
template <bool AKC, bool BKC, bool AVEC, bool BVEC>
struct PolSel<PM_B16K64, AKC, BKC, AVEC, BVEC> {
  using type = PolB16<AKC, BKC, AVEC, BVEC, 64>;
};

// ================================================================ tile grid
// Single-buffered LDS + one K-tile of register prefetch: <= 37 KB of LDS and
// <= 168 VGPRs -> 3 workgroups per CU (768 resident tiles on the chip).
template <int PM, bool AKC, bool BKC, bool AVEC, bool BVEC>
__global__ __launch_bounds__(GEMM_THREADS, PM == PM_B16K64 ? 2 : 3) void gemm_f32_kernel(
    int64_t M, int64_t N, int64_t K, float alpha, GemmPtrs ptrs, int64_t lda,
    int64_t ldb, float beta, int64_t scm, int64_t scn, int nseg, int tiles_n) {
  using Pol = typename PolSel<PM, AKC, BKC, AVEC, BVEC>::type;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Pol::SMEM];

  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs,
  // so remap bid -> linear tile L giving each XCD a contiguous range of L
  // (bijective for any grid size).  Within L, groups of 8 n-tiles walk down
  // m, so the 8 blocks sharing an A panel run together on one XCD's L2.
  const int64_t nwg = gridDim.x;
  const int64_t bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8;
  const int64_t q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t group = 8;
  const int64_t per_group = group * tiles_m;
  const int64_t g = bid / per_group;
  const int64_t first_n = g * group;
  const int64_t gsize = (tiles_n - first_n) < group ? (tiles_n - first_n) : group;
  const int64_t in_g = bid % per_group;
  const int64_t tn = first_n + (in_g % gsize);
  const int64_t tm = in_g / gsize;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  const int batch = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;

  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  typename Pol::LA la;
  typename Pol::LB lb;
  const int64_t nk = (K + Pol::KT - 1) / Pol::KT;
  const int64_t total = nk * nseg;

  // ksplit mode 1 (nseg = all batches): batch index = segment; mode 2
  // (nseg = nstrided, grid.y = pointer batch): segment walks the strided
  // batches of this block's pointer batch.  The (segment, k) position is kept
  // as counters so the main loop has no integer division.
  const bool per_ptr = ptrs.ksplit_mode == 2;
  auto seg_base = [&](int seg, const float*& a, const float*& b) {
    int pb, sb;
    if (per_ptr) {
      pb = batch;
      sb = seg;
    } else {
      const int bi = (nseg > 1) ? seg : batch;
      pb = bi % ptrs.nptr;
      sb = bi / ptrs.nptr;
    }
    a = ptrs.A[pb] + sb * ptrs.sA;
    b = ptrs.B[pb] + sb * ptrs.sB;
  };

  const float *pa, *pb;
  seg_base(0, pa, pb);
  int seg = 0;
  int64_t k0 = 0;  // k offset of the tile in registers (prefetched next)
  la.load(pa, lda, m0, 0, M, K);
  lb.load(pb, ldb, n0, 0, N, K);

  for (int64_t it = 0; it < total; ++it) {
    if (it > 0) __syncthreads();  // every wave is done reading the LDS images
    Pol::store(la, lb, smem);
    __syncthreads();
    if (it + 1 < total) {  // next K-tile's loads fly during this tile's MFMAs
      k0 += Pol::KT;
      if (k0 >= K) {
        k0 = 0;
        seg_base(++seg, pa, pb);
      }
      la.load(pa, lda, m0, k0, M, K);
      lb.load(pb, ldb, n0, k0, N, K);
    }
    Pol::compute(smem, acc, wm, wn, li, lh);
  }

  // epilogue: D[row=(r&3)+8*(r>>2)+4*lh][col=li] of each 32x32 tile
  const int cb = per_ptr ? batch : (nseg > 1 ? 0 : batch);
  float* C = per_ptr ? ptrs.C[cb] : ptrs.C[cb % ptrs.nptr] + (cb / ptrs.nptr) * ptrs.sC;
  const float* bias1 = ptrs.bias1[per_ptr ? cb : cb % ptrs.nptr];
  const float* bias2 = ptrs.bias2[per_ptr ? cb : cb % ptrs.nptr];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn + j * 32 + li;
      if (n >= N) continue;
      const float bv = (bias1 ? bias1[n] : 0.f) + (bias2 ? bias2[n] : 0.f);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) {
          float* q = C + m * scm + n * scn;
          float v = alpha * acc[i][j][r] + bv;
          if (beta != 0.f) v += beta * *q;
          *q = v;
        }
      }
    }
}

// ------------------------------------------------------------- stream-K
// When the tile count does not fill the resident workgroup slots evenly (the
// BLSTM layer-0 projections: 672 / 1032 tiles of 128x128 on 768 slots), a
// persistent grid of exactly the resident slots splits the (batch, tile,
// k-iteration) space into equal contiguous ranges.  Tiles whose whole K range
// falls in one workgroup are written directly; a split tile's pieces go to a
// workspace slot (first or last piece of the workgroup's range) and are summed
// in workgroup (= k) order by gemm_streamk_fixup, so results are deterministic.
// Logical workgroup ids are XCD-major (each XCD owns a contiguous range), and
// tiles are ordered so that consecutive tiles share the larger operand panel.
constexpr int SK_SLOTS = 768;   // 256 CUs x 3 resident workgroups

struct SkGeom {
  int64_t units, nk, tiles_m, tiles_n;
  int nbatch, order, P;  // order 0: (tm, batch, tn); 1: (tn, batch, tm)
};

__device__ __forceinline__ void sk_decode(const SkGeom& g, int64_t t, int& b, int64_t& tm,
                                          int64_t& tn) {
  if (g.order == 0) {
    tn = t % g.tiles_n;
    b = (int)((t / g.tiles_n) % g.nbatch);
    tm = t / (g.tiles_n * g.nbatch);
  } else {
    tm = t % g.tiles_m;
    b = (int)((t / g.tiles_m) % g.nbatch);
    tn = t / (g.tiles_m * g.nbatch);
  }
}
__device__ __forceinline__ int64_t sk_u0(const SkGeom& g, int64_t L) { return g.units * L / g.P; }

// full-tile epilogue (shared by the stream-K kernel and its fixup); get(idx)
// returns accumulator idx = (i*2+j)*16 + r
template <typename Get>
__device__ __forceinline__ void sk_store(const GemmPtrs& ptrs, int b, int64_t m0, int64_t n0,
                                         int64_t M, int64_t N, float alpha, float beta,
                                         int64_t scm, int64_t scn, Get get) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;
  float* C = ptrs.C[b % ptrs.nptr] + (int64_t)(b / ptrs.nptr) * ptrs.sC;
  const float* bias1 = ptrs.bias1[b % ptrs.nptr];
  const float* bias2 = ptrs.bias2[b % ptrs.nptr];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn + j * 32 + li;
      if (n >= N) continue;
      const float bv = (bias1 ? bias1[n] : 0.f) + (bias2 ? bias2[n] : 0.f);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) {
          float* q = C + m * scm + n * scn;
          float x = alpha * get((i * 2 + j) * 16 + r) + bv;
          if (beta != 0.f) x += beta * *q;
          *q = x;
        }
      }
    }
}

template <int PM, bool AKC, bool BKC, bool AVEC, bool BVEC>
__global__ __launch_bounds__(GEMM_THREADS, 3) void gemm_f32_streamk(
    int64_t M, int64_t N, int64_t K, float alpha, GemmPtrs ptrs, int64_t lda, int64_t ldb,
    float beta, int64_t scm, int64_t scn, SkGeom g, float* __restrict__ ws) {
  using Pol = typename PolSel<PM, AKC, BKC, AVEC, BVEC>::type;
  __shared__ __attribute__((aligned(16))) unsigned char smem[Pol::SMEM];
  const int w = blockIdx.x;
  const int64_t L = (int64_t)(w % 8) * (g.P / 8) + w / 8;
  const int64_t u0 = sk_u0(g, L), u1 = sk_u0(g, L + 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;
  typename Pol::LA la;
  typename Pol::LB lb;

  for (int64_t u = u0; u < u1;) {
    const int64_t t = u / g.nk, kb = u % g.nk;
    const int64_t ke = (g.nk - kb) < (u1 - u) ? g.nk : kb + (u1 - u);
    int b;
    int64_t tm, tn;
    sk_decode(g, t, b, tm, tn);
    const int64_t m0 = tm * BM, n0 = tn * BN;
    const float* A = ptrs.A[b % ptrs.nptr] + (int64_t)(b / ptrs.nptr) * ptrs.sA;
    const float* B = ptrs.B[b % ptrs.nptr] + (int64_t)(b / ptrs.nptr) * ptrs.sB;

    f32x16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    __syncthreads();  // the previous segment's LDS reads are done
    la.load(A, lda, m0, kb * Pol::KT, M, K);
    lb.load(B, ldb, n0, kb * Pol::KT, N, K);
    for (int64_t it = kb; it < ke; ++it) {
      if (it > kb) __syncthreads();
      Pol::store(la, lb, smem);
      __syncthreads();
      if (it + 1 < ke) {
        la.load(A, lda, m0, (it + 1) * Pol::KT, M, K);
        lb.load(B, ldb, n0, (it + 1) * Pol::KT, N, K);
      }
      Pol::compute(smem, acc, wm, wn, li, lh);
    }
    if (kb == 0 && ke == g.nk) {
      sk_store(ptrs, b, m0, n0, M, N, alpha, beta, scm, scn,
               [&](int idx) { return acc[idx >> 5][(idx >> 4) & 1][idx & 15]; });
    } else {
      const int slot = (u == u0) ? 0 : 1;
      float* q = ws + ((L * 2 + slot) * 64) * GEMM_THREADS + threadIdx.x;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) q[((i * 2 + j) * 16 + r) * GEMM_THREADS] = acc[i][j][r];
    }
    u += ke - kb;
  }
}

// Sum the pieces of every split tile in workgroup order and apply the epilogue.
__global__ __launch_bounds__(GEMM_THREADS) void gemm_streamk_fixup(
    int64_t M, int64_t N, float alpha, GemmPtrs ptrs, float beta, int64_t scm, int64_t scn,
    SkGeom g, const float* __restrict__ ws) {
  const int64_t t = blockIdx.x;
  const int64_t x0 = t * g.nk, x1 = x0 + g.nk - 1;  // first/last unit of the tile
  auto owner = [&](int64_t x) {
    int64_t L = x * g.P / g.units;
    while (L > 0 && sk_u0(g, L) > x) --L;
    while (sk_u0(g, L + 1) <= x) ++L;
    return L;
  };
  const int64_t Lf = owner(x0), Ll = owner(x1);
  if (Lf == Ll) return;  // written whole by its workgroup
  float v[64];
#pragma unroll
  for (int r = 0; r < 64; ++r) v[r] = 0.f;
  for (int64_t L = Lf; L <= Ll; ++L) {
    const int slot = sk_u0(g, L) >= x0 ? 0 : 1;
    const float* q = ws + ((L * 2 + slot) * 64) * GEMM_THREADS + threadIdx.x;
#pragma unroll
    for (int r = 0; r < 64; ++r) v[r] += q[r * GEMM_THREADS];
  }
  int b;
  int64_t tm, tn;
  sk_decode(g, t, b, tm, tn);
  sk_store(ptrs, b, tm * BM, tn * BN, M, N, alpha, beta, scm, scn,
           [&](int idx) { return v[idx]; });
}

// Stream-K geometry for a non-split-K call, or P == 0 when the plain grid is
// already balanced (>= 90 % of its last wave of resident slots filled) or K is
// too short (< 2048) to amortise the fixup.  kt: the main loop's K-tile.
static SkGeom streamk_geom(int64_t M, int64_t N, int64_t K, int64_t nb, int ksplit, int kt) {
  SkGeom g{};
  g.P = 0;
  if (ksplit != 0 || nb > 65535) return g;
  g.tiles_m = cdiv(M, BM);
  g.tiles_n = cdiv(N, BN);
  g.nk = cdiv(K, kt);
  const int64_t tiles = g.tiles_m * g.tiles_n * nb;
  if (K < 64 * BK || tiles < SK_SLOTS / 4) return g;
  const int64_t waves = cdiv(tiles, SK_SLOTS);
  if (tiles * 10 >= waves * SK_SLOTS * 9) return g;
  g.units = tiles * g.nk;
  g.nbatch = (int)nb;
  g.order = g.tiles_n <= g.tiles_m ? 0 : 1;
  g.P = SK_SLOTS;
  return g;
}

template <int PM, bool AKC, bool BKC>
static void launch_gemm(bool avec, bool bvec, dim3 grid, hipStream_t s,
                        int64_t M, int64_t N, int64_t K, float alpha,
                        const GemmPtrs& p, int64_t lda, int64_t ldb,
                        float beta, int64_t scm, int64_t scn, int nseg,
                        int tiles_n) {
#define AINP_GEMM_LAUNCH(AV, BV)                                             \
  hipLaunchKernelGGL((gemm_f32_kernel<PM, AKC, BKC, AV, BV>), grid,         \
                     dim3(GEMM_THREADS), 0, s, M, N, K, alpha, p, lda, ldb, \
                     beta, scm, scn, nseg, tiles_n)
  if (avec && bvec) AINP_GEMM_LAUNCH(true, true);
  else if (avec) AINP_GEMM_LAUNCH(true, false);
  else if (bvec) AINP_GEMM_LAUNCH(false, true);
  else AINP_GEMM_LAUNCH(false, false);
#undef AINP_GEMM_LAUNCH
}

template <int PM, bool AKC, bool BKC>
static void launch_streamk(bool avec, bool bvec, hipStream_t s, int64_t M, int64_t N, int64_t K,
                           float alpha, const GemmPtrs& p, int64_t lda, int64_t ldb, float beta,
                           int64_t scm, int64_t scn, const SkGeom& g, float* ws) {
#define AINP_SK(AV, BV)                                                                       \
  hipLaunchKernelGGL((gemm_f32_streamk<PM, AKC, BKC, AV, BV>), dim3(g.P), dim3(GEMM_THREADS), \
                     0, s, M, N, K, alpha, p, lda, ldb, beta, scm, scn, g, ws)
  if (avec && bvec) AINP_SK(true, true);
  else if (avec) AINP_SK(true, false);
  else if (bvec) AINP_SK(false, true);
  else AINP_SK(false, false);
#undef AINP_SK
}

// layout dispatch for both main loops: streamk selects the persistent kernel
template <int PM>
static void dispatch_gemm(bool streamk, bool akc, bool bkc, bool avec, bool bvec, dim3 grid,
                          hipStream_t s, int64_t M, int64_t N, int64_t K, float alpha,
                          const GemmPtrs& p, int64_t lda, int64_t ldb, float beta, int64_t scm,
                          int64_t scn, int nseg, int tiles_n, const SkGeom& g, float* ws) {
#define AINP_DISPATCH(AK, BK_)                                                                 \
  do {                                                                                         \
    if (streamk)                                                                               \
      launch_streamk<PM, AK, BK_>(avec, bvec, s, M, N, K, alpha, p, lda, ldb, beta, scm, scn, \
                                  g, ws);                                                      \
    else                                                                                       \
      launch_gemm<PM, AK, BK_>(avec, bvec, grid, s, M, N, K, alpha, p, lda, ldb, beta, scm,   \
                               scn, nseg, tiles_n);                                           \
  } while (0)
  if (akc && bkc) AINP_DISPATCH(true, true);
  else if (akc) AINP_DISPATCH(true, false);
  else if (bkc) AINP_DISPATCH(false, true);
  else AINP_DISPATCH(false, false);
#undef AINP_DISPATCH
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace ainp

using namespace ainp;


extern "C" size_t ainp_gemm_f32_workspace(int64_t M, int64_t N, int64_t K, int nptr,
                                          int64_t nstrided, int ksplit) {
  // the same decision for both main loops (it depends on K, not on the K-tile)
  const SkGeom g = streamk_geom(M, N, K, (int64_t)nptr * nstrided, ksplit, BK);
  return g.P ? (size_t)g.P * 2 * 64 * GEMM_THREADS * sizeof(float) : 0;
}

extern "C" int ainp_gemm_f32(int64_t M, int64_t N, int64_t K, float alpha,
                             const float* const* A, int64_t sam, int64_t sak,
                             int64_t strideA, const float* const* B,
                             int64_t sbk, int64_t sbn, int64_t strideB,
                             float beta, float* const* C, int64_t scm,
                             int64_t scn, int64_t strideC,
                             const float* const* bias1,
                             const float* const* bias2, int nptr,
                             int64_t nstrided, int ksplit, void* stream) {
  return ainp_gemm_f32_ex(M, N, K, alpha, A, sam, sak, strideA, B, sbk, sbn, strideB, beta, C,
                          scm, scn, strideC, bias1, bias2, nptr, nstrided, ksplit, 0, nullptr, 0,
                          stream);
}

extern "C" int ainp_gemm_f32_ws(int64_t M, int64_t N, int64_t K, float alpha,
                                const float* const* A, int64_t sam, int64_t sak,
                                int64_t strideA, const float* const* B,
                                int64_t sbk, int64_t sbn, int64_t strideB,
                                float beta, float* const* C, int64_t scm,
                                int64_t scn, int64_t strideC,
                                const float* const* bias1,
                                const float* const* bias2, int nptr,
                                int64_t nstrided, int ksplit, void* workspace,
                                size_t ws_bytes, void* stream) {
  return ainp_gemm_f32_ex(M, N, K, alpha, A, sam, sak, strideA, B, sbk, sbn, strideB, beta, C,
                          scm, scn, strideC, bias1, bias2, nptr, nstrided, ksplit, 0, workspace,
                          ws_bytes, stream);
}

extern "C" int ainp_gemm_f32_ex(int64_t M, int64_t N, int64_t K, float alpha,
                                const float* const* A, int64_t sam, int64_t sak,
                                int64_t strideA, const float* const* B,
                                int64_t sbk, int64_t sbn, int64_t strideB,
                                float beta, float* const* C, int64_t scm,
                                int64_t scn, int64_t strideC,
                                const float* const* bias1,
                                const float* const* bias2, int nptr,
                                int64_t nstrided, int ksplit, int flags, void* workspace,
                                size_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0 || nptr < 1 || nptr > 8 || nstrided < 1 ||
      !A || !B || !C)
    return record_msg("ainp_gemm_f32: bad argument");
  if (flags & ~(AINP_GEMM_EXACT_F32 | AINP_GEMM_BF16))
    return record_msg("ainp_gemm_f32: unknown flags");
  if ((flags & AINP_GEMM_EXACT_F32) && (flags & AINP_GEMM_BF16))
    return record_msg("ainp_gemm_f32: EXACT_F32 and BF16 are exclusive");
  if (sam != 1 && sak != 1) return record_msg("ainp_gemm_f32: A needs a unit stride");
  if (sbk != 1 && sbn != 1) return record_msg("ainp_gemm_f32: B needs a unit stride");
  if (scm != 1 && scn != 1) return record_msg("ainp_gemm_f32: C needs a unit stride");
  const int64_t nb = nptr * nstrided;
  if (!ksplit && nb > 65535) return record_msg("ainp_gemm_f32: too many batches");
  if (M == 0 || N == 0) return AINP_OK;
  GemmPtrs p;
  for (int i = 0; i < 8; ++i) {
    p.A[i] = i < nptr ? A[i] : nullptr;
    p.B[i] = i < nptr ? B[i] : nullptr;
    p.C[i] = i < nptr ? C[i] : nullptr;
    p.bias1[i] = (bias1 && i < nptr) ? bias1[i] : nullptr;
    p.bias2[i] = (bias2 && i < nptr) ? bias2[i] : nullptr;
  }
  p.sA = strideA;
  p.sB = strideB;
  p.sC = strideC;
  p.nptr = nptr;
  p.ksplit_mode = ksplit;
  const int pm = (flags & AINP_GEMM_BF16) ? PM_B16 : (flags & AINP_GEMM_EXACT_F32) ? PM_F32 : PM_X6;
  const bool use_x6 = pm != PM_F32;   // the split-bf16 and bf16 loops: plain grid
  // contiguous dimension of each operand (prefer k when both strides are 1)
  const bool akc = (sak == 1);
  const bool bkc = (sbk == 1);
  const int64_t lda = akc ? sam : sak;
  const int64_t ldb = bkc ? sbn : sbk;
  // vector loads need 16-byte aligned rows and a contiguous extent % 4 == 0
  bool avec = (lda % 4 == 0) && ((akc ? K : M) % 4 == 0) && (strideA % 4 == 0);
  bool bvec = (ldb % 4 == 0) && ((bkc ? K : N) % 4 == 0) && (strideB % 4 == 0);
  for (int i = 0; i < nptr; ++i) {
    avec = avec && aligned16(A[i]);
    bvec = bvec && aligned16(B[i]);
  }
  if (ksplit < 0 || ksplit > 2) return record_msg("ainp_gemm_f32: ksplit must be 0, 1 or 2");
  if (ksplit && nb > (1 << 20)) return record_msg("ainp_gemm_f32: too many segments");
  const int nseg = ksplit == 1 ? (int)nb : (ksplit == 2 ? (int)nstrided : 1);
  const int64_t tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  hipStream_t s = as_stream(stream);
  // stream-K pays off for the exact f32 loop only: the x6 loop's plain grid
  // (3 resident tiles per CU) measured 13 % faster on the layer-0 shapes
  // (tools/gemm3_lab.hip), so it always takes the plain grid.
  const SkGeom g = streamk_geom(M, N, K, nb, ksplit, BK);
  const bool sk = !use_x6 && g.P && workspace &&
                  ws_bytes >= (size_t)g.P * 2 * 64 * GEMM_THREADS * sizeof(float);
  const unsigned gy = ksplit == 1 ? 1u : (ksplit == 2 ? (unsigned)nptr : (unsigned)nb);
  const dim3 grid((unsigned)(tiles_m * tiles_n), gy);
  float* ws = reinterpret_cast<float*>(workspace);
  static const bool k64 = [] {
    const char* e = getenv("AINP_GEMM_B16_KT");
    return e && e[0] == '6';
  }();
  if (pm == PM_B16 && k64)
    dispatch_gemm<PM_B16K64>(sk, akc, bkc, avec, bvec, grid, s, M, N, K, alpha, p, lda, ldb,
                             beta, scm, scn, nseg, (int)tiles_n, g, ws);
  else if (pm == PM_B16)
    dispatch_gemm<PM_B16>(sk, akc, bkc, avec, bvec, grid, s, M, N, K, alpha, p, lda, ldb, beta,
                          scm, scn, nseg, (int)tiles_n, g, ws);
  else if (pm == PM_X6)
    dispatch_gemm<PM_X6>(sk, akc, bkc, avec, bvec, grid, s, M, N, K, alpha, p, lda, ldb, beta,
                         scm, scn, nseg, (int)tiles_n, g, ws);
  else
    dispatch_gemm<PM_F32>(sk, akc, bkc, avec, bvec, grid, s, M, N, K, alpha, p, lda, ldb, beta,
                          scm, scn, nseg, (int)tiles_n, g, ws);
  int rc = check_launch(sk ? "gemm_f32_streamk" : "ainp_gemm_f32");
  if (rc || !sk) return rc;
  hipLaunchKernelGGL(gemm_streamk_fixup, dim3((unsigned)(g.units / g.nk)), dim3(GEMM_THREADS), 0,
                     s, M, N, alpha, p, beta, scm, scn, g, ws);
  return check_launch("gemm_streamk_fixup");
}
