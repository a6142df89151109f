// gemm16.hip — bf16-operand GEMM for the bf16 configurations (BASELINE C3).
//
// C[m][n] = sum_k A[m][k] B[n][k] (+ bias) with A, B stored as bf16 in HBM,
// both k-contiguous ("NT"), fp32 accumulation on v_mfma_f32_32x32x16_bf16.
// Replaces, in the bf16 configuration, the three layer-0 GEMMs of nn.LSTM
// (models/CNNBLSTM/model.py:46-47,77) -- the input projection and its data /
// weight gradients -- whose producers write the bf16 operands directly in the
// layouts this kernel wants (the encoder's last BN+ReLU writes X and X^T, the
// BPTT gradient is cast to dg and dg^T, the weights to W and W^T once per
// optimizer step), so every operand arrives k-contiguous at 2 bytes/element:
// half the HBM/L2 bytes of the fp32-staged bf16 loop (gemm.hip PM_B16) and one
// 16-byte load per 8 elements, no conversion in the main loop.
//
// Tile 128 x 128 x 64 per 256-thread workgroup (4 waves as 2 x 2, each wave
// 64 x 64 = 2 x 2 MFMA 32x32 tiles); A and B images [row][64 k] with 144-byte
// rows in LDS (conflict-free ds_read_b128 fragments), the next K-tile
// prefetched in registers (4 x 16 B per operand per thread); <= 168 VGPRs so
// three workgroups fit per CU.  XCD-aware block order as gemm.hip.  Split-K:
// blockIdx.y = split s covers k in [s*kc, min(K, (s+1)*kc)) and writes slab
// C + s*strideC (summed by ainp_sum_slabs in fixed order).  Unsplit GEMMs
// with M, N >= 512 and at most 1536 tiles of 128 x 128 run on g256 below
// instead (256 x 256 tiles, LDS-DMA ring; routing rule at the launcher).
#include "common.h"

#include <stdlib.h>

namespace ainp {
namespace g16 {

constexpr int BM = 128, BN = 128, BK = 64, THREADS = 256;
constexpr int RS = BK * 2 + 16;      // image row bytes: 64 bf16 + 16 B pad
constexpr int IMG = 128 * RS;        // one operand image

typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

// 128 rows x 64 k of a k-contiguous bf16 operand: chunk c = tid + 256 i
// (i < 4) is row c / 8, 16-byte column c % 8 (8 threads read one 128-B row).
struct Loader {
  uint4 v[4];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ p, int64_t ld, int64_t r0,
                                       int64_t k0, int64_t R, int64_t kend) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * THREADS;
      const int64_t r = r0 + (c >> 3), k = k0 + (c & 7) * 8;
      uint4 x = make_uint4(0u, 0u, 0u, 0u);
      if (r < R && k < kend) x = *reinterpret_cast<const uint4*>(p + r * ld + k);
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * THREADS;
      *reinterpret_cast<uint4*>(img + (c >> 3) * RS + (c & 7) * 16) = v[i];
    }
  }
};

__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int row, int ks, int h) {
  return __builtin_bit_cast(bf16x8v,
                            *reinterpret_cast<const uint4*>(img + row * RS + 32 * ks + 16 * h));
}

struct Bias {
  const float* a1;   // n in [0, nsplit): a1[n] + a2[n]
  const float* a2;
  const float* b1;   // n in [nsplit, N): b1[n - nsplit] + b2[n - nsplit]
  const float* b2;
  int64_t nsplit;
};

__global__ __launch_bounds__(THREADS, 3) void gemm_bf16nt_kernel(
    int64_t M, int64_t N, int64_t K, const uint16_t* __restrict__ A, int64_t lda,
    const uint16_t* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
    int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * IMG];
  // XCD-aware order (gemm.hip): each XCD owns a contiguous range of linear
  // tiles; within it groups of 8 n-tiles walk down m (A panels shared in L2).
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;

  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  float* Cs = C + split * strideC;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Loader la, lb;
  if (kbeg < kend) {
    la.load(A, lda, m0, kbeg, M, kend);
    lb.load(B, ldb, n0, kbeg, N, kend);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    if (k0 > kbeg) __syncthreads();     // every wave is done with the images
    la.store(smem);
    lb.store(smem + IMG);
    __syncthreads();
    if (k0 + BK < kend) {               // next K-tile's loads fly during the MFMAs
      la.load(A, lda, m0, k0 + BK, M, kend);
      lb.load(B, ldb, n0, k0 + BK, N, kend);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8v a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = frag(smem, wm + i * 32 + li, ks, lh);
        b[i] = frag(smem + IMG, wn + i * 32 + li, ks, lh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: D[row=(r&3)+8*(r>>2)+4*lh][col=li] of each 32x32 tile
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split != 0) {   // split-K: the bias goes into slab 0 only
    } else if (n < bias.nsplit) {
      if (bias.a1) bv += bias.a1[n];
      if (bias.a2) bv += bias.a2[n];
    } else {
      if (bias.b1) bv += bias.b1[n - bias.nsplit];
      if (bias.b2) bv += bias.b2[n - bias.nsplit];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}

// fp32 [R][ld_in] -> bf16 out [R][ld_out] (optional) and its transpose
// outT [C][ld_t] (optional); 64 x 64 tiles through LDS, round-to-nearest-even.
__global__ __launch_bounds__(256) void cast_bf16_t_kernel(const float* __restrict__ x, int64_t R,
                                                          int64_t Cc, int64_t ld_in,
                                                          uint16_t* __restrict__ out,
                                                          int64_t ld_out,
                                                          uint16_t* __restrict__ outT,
                                                          int64_t ld_t) {
  __shared__ uint16_t tile[64][66];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    uint16_t b = 0;
    if (r < R && c < Cc) {
      const __bf16 h = (__bf16)x[r * ld_in + c];
      b = __builtin_bit_cast(uint16_t, h);
      if (out) out[r * ld_out + c] = b;
    }
    tile[i][tx] = b;
  }
  if (!outT) return;
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < Cc && r < R) outT[c * ld_t + r] = tile[tx][i];
  }
}


// fp32 [R][ld_in] -> its transpose outT [C][ld_t]; 64 x 64 tiles through LDS
// (the layer-0 data gradient's k-contiguous W_ih^T operand)
__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* __restrict__ x, int64_t R,
                                                            int64_t Cc, int64_t ld_in,
                                                            float* __restrict__ outT,
                                                            int64_t ld_t) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < Cc) ? x[r * ld_in + c] : 0.f;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < Cc && r < R) outT[c * ld_t + r] = tile[tx][i];
  }
}

// ------------------------------------------------- implicit-GEMM weight gradient
// Weight gradient of a k x k / stride s conv with the layer input x in
// channel-last bf16 (x16 [N][H][W][Cin], the copy the forward conv read):
//   G[m][ci*KK + tap] = sum_q A[m][q] * x16[n][oy*s+ky-pad][ox*s+kx-pad][ci],
//   G[m][Cin*KK]      = sum_q A[m][q]          (the bias: a ones row),
// q = n*Ho*Wo + oy*Wo + ox, A = the bf16 output gradient [M][lda] (d_prep16's
// gA).  gemm_bf16nt_kernel's tiles, MFMA loop, K order and split-K, with the
// B operand built from x16 instead of materialised im2col16 columns: GEMM
// column n = tap*Cin + ci (a 16-byte chunk of 8 channels of one tap per load),
// the tile's rows gathered for four consecutive q per thread and transposed in
// registers to the k-contiguous LDS image; the epilogue stores column n at
// ci*KK + tap.  Same products, same order: bit-identical to im2col16 + GEMM.
struct WgGeom {
  const uint16_t* x16;
  int N, Cin, H, W, KW, KK, stride, pad, Ho, Wo;
  int64_t NP;
};

__global__ __launch_bounds__(THREADS, 3) void wgrad16_nhwc_kernel(
    int64_t M, int64_t Ncol, int64_t K, const uint16_t* __restrict__ A, int64_t lda, WgGeom g,
    float* __restrict__ C, int64_t ldc, int64_t kc, int64_t strideC, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * IMG];
  // one linear grid of tiles x splits, numbered XCD-major: each XCD owns a
  // contiguous run of splits with all their tiles, so the tiles that gather
  // the same input pixels (same K range, other taps / channels) share its L2
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t tiles = tiles_m * tiles_n;
  const int64_t split = bid / tiles, t = bid - split * tiles;
  const int64_t m0 = (t % tiles_m) * BM, n0 = (t / tiles_m) * BN;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  float* Cs = C + split * strideC;

  // this thread's B chunk: rows n0 + 8c .. +7 (one tap, 8 channels), q group qg
  const int tid = threadIdx.x;
  const int c = tid & 15, qg = tid >> 4;
  const int64_t nb = n0 + 8 * c;
  const int64_t KC = (int64_t)g.KK * g.Cin;
  const int kind = nb < KC ? 0 : (nb == KC ? 1 : 2);   // channels / ones row / past N
  const int tap = kind == 0 ? (int)(nb / g.Cin) : 0;
  const int ci0 = kind == 0 ? (int)(nb - (int64_t)tap * g.Cin) : 0;
  const int ky = tap / g.KW, kx = tap - ky * g.KW;
  const int64_t HWo = (int64_t)g.Ho * g.Wo;

  uint4 vb[4];
  auto load_b = [&](int64_t k0) {
    int64_t q = k0 + 4 * qg;
    int img = 0, oy = 0, ox = 0;
    if (q < g.NP) {
      img = (int)(q / HWo);
      const int r = (int)(q - (int64_t)img * HWo);
      oy = r / g.Wo;
      ox = r - oy * g.Wo;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m, ++q) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (q < kend && q < g.NP) {
        if (kind == 0) {
          const int iy = oy * g.stride - g.pad + ky, ix = ox * g.stride - g.pad + kx;
          if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
            v = *reinterpret_cast<const uint4*>(
                g.x16 + (((int64_t)img * g.H + iy) * g.W + ix) * g.Cin + ci0);
        } else if (kind == 1) {
          v.x = 0x3F80u;   // 1.0 in row n0 + 8c, zero in the rows after it
        }
      }
      vb[m] = v;
      if (++ox == g.Wo) {
        ox = 0;
        if (++oy == g.Ho) {
          oy = 0;
          ++img;
        }
      }
    }
  };
  // 4 q x 8 channels -> 8 rows of 4 q (8 bytes each) in the B image
  auto store_b = [&](unsigned char* img) {
    const uint32_t w[4][4] = {{vb[0].x, vb[0].y, vb[0].z, vb[0].w},
                              {vb[1].x, vb[1].y, vb[1].z, vb[1].w},
                              {vb[2].x, vb[2].y, vb[2].z, vb[2].w},
                              {vb[3].x, vb[3].y, vb[3].z, vb[3].w}};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint2 lo = make_uint2((w[0][p] & 0xffffu) | (w[1][p] << 16),
                                  (w[2][p] & 0xffffu) | (w[3][p] << 16));
      const uint2 hi = make_uint2((w[0][p] >> 16) | (w[1][p] & 0xffff0000u),
                                  (w[2][p] >> 16) | (w[3][p] & 0xffff0000u));
      *reinterpret_cast<uint2*>(img + (8 * c + 2 * p) * RS + 8 * qg) = lo;
      *reinterpret_cast<uint2*>(img + (8 * c + 2 * p + 1) * RS + 8 * qg) = hi;
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Loader la;
  if (kbeg < kend) {
    la.load(A, lda, m0, kbeg, M, kend);
    load_b(kbeg);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    if (k0 > kbeg) __syncthreads();
    la.store(smem);
    store_b(smem + IMG);
    __syncthreads();
    if (k0 + BK < kend) {
      la.load(A, lda, m0, k0 + BK, M, kend);
      load_b(k0 + BK);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8v a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = frag(smem, wm + i * 32 + li, ks, lh);
        b[i] = frag(smem + IMG, wn + i * 32 + li, ks, lh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= Ncol) continue;
    int64_t col = n;   // the ones row stays last
    if (n < KC) {
      const int t = (int)(n / g.Cin);
      col = (n - (int64_t)t * g.Cin) * g.KK + t;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + col] = acc[i][j][r];
      }
  }
}

}  // namespace g16

// Large GEMMs (M, N >= 512): 256 x 256 x 32 tiles with LDS-DMA staging.
//
// 512 threads = 8 waves as 2 (m) x 4 (n); each wave owns 128 x 64 outputs =
// 4 x 2 tiles of v_mfma_f32_32x32x16_bf16 (128 accumulator VGPRs).  Operand
// tiles (256 rows x 32 k, 64-byte rows) arrive by global_load_lds_dwordx4
// (16 B per lane, one 1-KB contiguous LDS block per wave instruction: 16 rows)
// into a ring of 4 LDS stages (4 x 32 KB), two K-tiles kept in flight across
// each barrier by a counted vmcnt; one raw s_barrier per K-tile.  The LDS
// image is row-linear with the four 16-byte chunks of a row XOR-swizzled by
// bits 2..3 of the row (applied on the global source address, since the DMA
// destination is lane-linear), so the 16 lanes of a ds_read_b128 quarter
// (16 consecutive rows, one k-chunk) hit 16 distinct 16-byte bank slots.
namespace g256 {
constexpr int BM = 256, BN = 256, BK = 32, THREADS = 512, NSTAGE = 4;
constexpr int ROWB = BK * 2;             // 64 bytes per image row
constexpr int IMG = BM * ROWB;           // 16 KB per operand per stage
constexpr int STAGE = 2 * IMG;           // A + B
constexpr int LDS_BYTES = NSTAGE * STAGE;  // 128 KB
constexpr int GLDS_PER_TILE = 4;         // per wave: 2 for A, 2 for B

using g16::bf16x8v;
using g16::f32x16v;
using g16::Bias;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

// Stage one operand's 256 x 32 K-tile: wave w, instruction i covers image
// rows 16 (2w + i) .. +16; lane L -> row + L/4, physical chunk L % 4.
__device__ __forceinline__ void stage(const uint16_t* __restrict__ P, int64_t ld, int64_t r0,
                                      int64_t R, int64_t k0, unsigned char* img, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = 2 * wave + i;
    const int row = 16 * blk + (lane >> 2);
    const int c = swz(row, lane & 3);
    int64_t gr = r0 + row;
    gr = gr < R ? gr : R - 1;  // rows past the end: any valid row (never stored)
    const uint16_t* src = P + gr * ld + k0 + 8 * c;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8v,
                            *reinterpret_cast<const uint4*>(img + row * ROWB + 16 * swz(row, chunk)));
}

// k-major ("T") operand: element (r, k) at P[k*ld + r] -- the layer-0 weight
// gradient's dg [NT, 8H] and X [NT, I] as they lie, no transposed copies.
// Image: 32 k-rows of 256 elements (512 B), 16-byte chunk c of k-row kr at
// physical chunk c ^ 4(kr & 3), so the transposed fragment reads below hit 64
// distinct banks per half-wave.  Stage: wave w, instruction i covers k-rows
// 2(2w+i), +1 (1 KB); lane L: k-row + L/32, physical chunk L % 32, fetching
// the logical chunk it holds (columns past R clamp to R - 8: R % 8 == 0,
// never stored).
__device__ __forceinline__ int kswz(int kr, int c) { return c ^ (4 * (kr & 3)); }

__device__ __forceinline__ void stage_km(const uint16_t* __restrict__ P, int64_t ld, int64_t r0,
                                         int64_t R, int64_t k0, unsigned char* img, int wave,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = 2 * wave + i;
    const int kr = 2 * blk + (lane >> 5);
    const int c = kswz(kr, lane & 31);
    int64_t col = r0 + 8 * c;
    col = col + 8 <= R ? col : R - 8;
    const uint16_t* src = P + (k0 + kr) * ld + col;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

// The 32x32x16 operand of rows row0 .. row0+31, k = 16 ks + 8 (lane / 32) + 0..7,
// from a k-major image by two ds_read_b64_tr_b16 (cdna_hip_programming.md
// T10): lane 4q+p of each 16-lane group supplies k-row kb + q, columns
// 4p .. 4p+3 of its group's 16; lane i of the group receives column i, rows
// kb .. kb+3 -- the same (row, k) values frag() gives from a k-contiguous image.
typedef short v4s16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8v frag_km(const unsigned char* img, int row0, int ks, int lane) {
  const int g = (lane & 31) >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int col = row0 + 16 * g + 4 * p;
  v4s16 h[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kr = 16 * ks + 8 * (lane >> 5) + 4 * t + q;
    const unsigned char* a = img + kr * 512 + 16 * kswz(kr, col >> 3) + 2 * (col & 7);
    h[t] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s16*)(const_cast<unsigned char*>(a)));
  }
  typedef short v8s16 __attribute__((ext_vector_type(8)));
  const v8s16 r = __builtin_shufflevector(h[0], h[1], 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8v, r);
}

template <int N_INFLIGHT>
__device__ __forceinline__ void wait_vm() {
  if (N_INFLIGHT == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (N_INFLIGHT == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Tile (m0, n0) of Cs over k in [kbeg, kbeg + nk*BK): the 4-stage LDS-DMA ring
// main loop and the store epilogue shared by the single- and multi-problem
// kernels (bias only in split 0).
template <bool AKM, bool BKM>
__device__ __forceinline__ void tile256(int64_t M, int64_t N, const uint16_t* __restrict__ A,
                                        int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
                                        float* __restrict__ Cs, int64_t ldc, int64_t m0,
                                        int64_t n0, int64_t kbeg, int nk, int64_t split,
                                        const Bias& bias, unsigned char* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NSTAGE) * STAGE;
    if (AKM) stage_km(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    else stage(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    if (BKM) stage_km(B, ldb, n0, N, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
    else stage(B, ldb, n0, N, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
  };
  // prologue: tiles 0, 1, 2 in flight
#pragma unroll
  for (int q = 0; q < NSTAGE - 1; ++q)
    if (q < nk) issue(q);

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt must have landed; tiles kt+1, kt+2 (if issued) may stay in flight
    const int ahead = nk - 1 - kt;
    if (ahead >= 2) wait_vm<2>();
    else if (ahead == 1) wait_vm<1>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all waves' DMAs for tile kt visible; stage kt-1 free
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1);  // into the stage of tile kt-1
    const unsigned char* sa = smem + (kt % NSTAGE) * STAGE;
    const unsigned char* sb = sa + IMG;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8v a[4], b[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = BKM ? frag_km(sb, wn + j * 32, ks, lane) : frag(sb, wn + j * 32 + li, 2 * ks + lh);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = AKM ? frag_km(sa, wm + i * 32, ks, lane) : frag(sa, wm + i * 32 + li, 2 * ks + lh);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: D[row=(r&3)+8*(r>>2)+4*lh][col=li] of each 32x32 tile
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split != 0) {   // split-K: the bias goes into slab 0 only
    } else if (n < bias.nsplit) {
      if (bias.a1) bv += bias.a1[n];
      if (bias.a2) bv += bias.a2[n];
    } else {
      if (bias.b1) bv += bias.b1[n - bias.nsplit];
      if (bias.b2) bv += bias.b2[n - bias.nsplit];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}

// Round 6: the same tile on 64-deep K-tiles (tools/g256b_lab.hip: 3-10 %
// faster on the layer-0 shapes, bit-identical -- the same MFMAs in the same k
// order).  Two 64 KB LDS stages (A + B): k-contiguous images of 256 rows x
// 128 B, 16-byte chunk c of row r at physical chunk c ^ (r & 7) (a ds_read_b128
// quarter: 16 rows of one chunk, 16 distinct bank groups); k-major images of
// 64 k-rows x 512 B read by frag_km as above.  32 MFMAs per wave between
// barriers (twice the 32-deep ring's), one K-tile in flight across each
// barrier, the next k-step's fragments read while the current one's MFMAs run.
namespace b64 {
constexpr int BK = 64, NST = 2, ROWB = 2 * BK, IMG = BM * ROWB, STAGE = 2 * IMG;
static_assert(NST * STAGE == LDS_BYTES, "the 32-deep ring's 128 KB");

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

// k-contiguous operand: wave w, instruction i covers image rows 8 (4w + i) .. +8;
// lane L -> row + L/8, physical chunk L % 8
__device__ __forceinline__ void stage(const uint16_t* __restrict__ P, int64_t ld, int64_t r0,
                                      int64_t R, int64_t k0, unsigned char* img, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = 4 * wave + i;
    const int row = 8 * blk + (lane >> 3);
    const int c = swz(row, lane & 7);
    int64_t gr = r0 + row;
    gr = gr < R ? gr : R - 1;  // rows past the end: any valid row (never stored)
    const uint16_t* src = P + gr * ld + k0 + 8 * c;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

// k-major operand: wave w, instruction i covers k-rows 2 (4w + i), +1 (stage_km's map)
__device__ __forceinline__ void stage_km(const uint16_t* __restrict__ P, int64_t ld, int64_t r0,
                                         int64_t R, int64_t k0, unsigned char* img, int wave,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = 4 * wave + i;
    const int kr = 2 * blk + (lane >> 5);
    const int c = kswz(kr, lane & 31);
    int64_t col = r0 + 8 * c;
    col = col + 8 <= R ? col : R - 8;
    const uint16_t* src = P + (k0 + kr) * ld + col;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8v,
                            *reinterpret_cast<const uint4*>(img + row * ROWB + 16 * swz(row, chunk)));
}
}  // namespace b64

template <bool AKM, bool BKM>
__device__ __forceinline__ void tile256b(int64_t M, int64_t N, const uint16_t* __restrict__ A,
                                         int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
                                         float* __restrict__ Cs, int64_t ldc, int64_t m0,
                                         int64_t n0, int64_t kbeg, int nk, int64_t split,
                                         const Bias& bias, unsigned char* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % b64::NST) * b64::STAGE;
    const int64_t k0 = kbeg + (int64_t)kt * b64::BK;
    if (AKM) b64::stage_km(A, lda, m0, M, k0, st, wave, lane);
    else b64::stage(A, lda, m0, M, k0, st, wave, lane);
    if (BKM) b64::stage_km(B, ldb, n0, N, k0, st + b64::IMG, wave, lane);
    else b64::stage(B, ldb, n0, N, k0, st + b64::IMG, wave, lane);
  };
  auto fa_ = [&](const unsigned char* sa, int i, int ks) {
    return AKM ? frag_km(sa, wm + i * 32, ks, lane) : b64::frag(sa, wm + i * 32 + li, 2 * ks + lh);
  };
  auto fb_ = [&](const unsigned char* sb, int j, int ks) {
    return BKM ? frag_km(sb, wn + j * 32, ks, lane) : b64::frag(sb, wn + j * 32 + li, 2 * ks + lh);
  };
  if (nk > 0) issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile kt: the only DMA in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's DMAs of tile kt; stage of kt-1 free
    asm volatile("" ::: "memory");
    if (kt + 1 < nk) issue(kt + 1);
    const unsigned char* sa = smem + (kt % b64::NST) * b64::STAGE;
    const unsigned char* sb = sa + b64::IMG;
    bf16x8v fa[2][4], fb[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[0][j] = fb_(sb, j, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[0][i] = fa_(sa, i, 0);
#pragma unroll
    for (int ks = 0; ks < b64::BK / 16; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < b64::BK / 16) {
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[cur ^ 1][j] = fb_(sb, j, ks + 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[cur ^ 1][i] = fa_(sa, i, ks + 1);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the MFMAs
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][i], fb[cur][j], acc[i][j], 0,
                                                              0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split != 0) {   // split-K: the bias goes into slab 0 only
    } else if (n < bias.nsplit) {
      if (bias.a1) bv += bias.a1[n];
      if (bias.a2) bv += bias.a2[n];
    } else {
      if (bias.b1) bv += bias.b1[n - bias.nsplit];
      if (bias.b2) bv += bias.b2[n - bias.nsplit];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}

__global__ __launch_bounds__(THREADS, 1) void gemm_bf16nt_256_kernel(
    int64_t M, int64_t N, int64_t K, const uint16_t* __restrict__ A, int64_t lda,
    const uint16_t* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
    int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  // XCD-aware order: each XCD owns a contiguous range of linear tiles; within
  // it groups of (up to) 8 n-tiles walk down m, sharing A panels in its L2
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;

  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  const int nk = (int)((kend - kbeg) / BK);  // the launcher guarantees BK | kc, BK | K
  tile256<false, false>(M, N, A, lda, B, ldb, C + split * strideC, ldc, m0, n0, kbeg, nk, split,
                        bias, smem);
}

// the same grid on 64-deep K-tiles (BK = 64 divides K and kc)
__global__ __launch_bounds__(THREADS, 1) void gemm_bf16nt_256b_kernel(
    int64_t M, int64_t N, int64_t K, const uint16_t* __restrict__ A, int64_t lda,
    const uint16_t* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc,
    int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  const int nk = (int)((kend - kbeg) / b64::BK);
  tile256b<false, false>(M, N, A, lda, B, ldb, C + split * strideC, ldc, m0, n0, kbeg, nk, split,
                         bias, smem);
}

// Several bf16 GEMMs in ONE grid (ainp_gemm_bf16nt_multi): problem q's work
// items (tiles x splits) follow problem q-1's, each problem starting on a
// multiple of 8 blocks.  Per problem the items are spread over the XCDs in
// contiguous ranges (the single-problem kernel's order), so the long-K weight
// gradient's items issue first and the short data-gradient items fill in
// behind them -- the bf16 layer-0 backward pair without a second stream.
constexpr int MAXP = 3;
struct MProb {
  const uint16_t* A; const uint16_t* B; float* C;
  int64_t lda, ldb, ldc, M, N, K, kc, strideC;
  int tiles_m, tiles_n, nsplit, a_km, b_km;
  int64_t items, first;
};
struct MJob {
  MProb p[MAXP];
  int np;
  int bk64;   // every problem's K and kc multiples of 64: tile256b
};

__global__ __launch_bounds__(THREADS, 1) void gemm_bf16nt_256_multi_kernel(MJob job) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int64_t bid0 = blockIdx.x;
  int pi = 0;
#pragma unroll
  for (int q = 1; q < MAXP; ++q)
    if (q < job.np && bid0 >= job.p[q].first) pi = q;
  const MProb& P = job.p[pi];
  const int64_t n8 = (P.items + 7) / 8 * 8;
  const int64_t loc0 = bid0 - P.first;
  const int64_t loc = (loc0 % 8) * (n8 / 8) + loc0 / 8;   // contiguous range per XCD
  if (loc >= P.items) return;
  const int64_t tiles = (int64_t)P.tiles_m * P.tiles_n;
  const int64_t split = loc / tiles, t = loc - split * tiles;
  const int64_t per_group = 8 * (int64_t)P.tiles_m;
  const int64_t first_n = (t / per_group) * 8;
  const int64_t gsize = (P.tiles_n - first_n) < 8 ? (P.tiles_n - first_n) : 8;
  const int64_t in_g = t % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  const int64_t kbeg = split * P.kc;
  const int64_t kend = (kbeg + P.kc) < P.K ? (kbeg + P.kc) : P.K;
  const Bias nob{nullptr, nullptr, nullptr, nullptr, 0};
  float* Cs = P.C + split * P.strideC;
  if (job.bk64) {
    const int nk = (int)((kend - kbeg) / b64::BK);
    if (P.a_km && P.b_km)
      tile256b<true, true>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split,
                           nob, smem);
    else if (P.a_km)
      tile256b<true, false>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split,
                            nob, smem);
    else if (P.b_km)
      tile256b<false, true>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split,
                            nob, smem);
    else
      tile256b<false, false>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split,
                             nob, smem);
    return;
  }
  const int nk = (int)((kend - kbeg) / BK);
  if (P.a_km && P.b_km)
    tile256<true, true>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split, nob,
                        smem);
  else if (P.a_km)
    tile256<true, false>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split, nob,
                         smem);
  else if (P.b_km)
    tile256<false, true>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split, nob,
                         smem);
  else
    tile256<false, false>(P.M, P.N, P.A, P.lda, P.B, P.ldb, Cs, P.ldc, m0, n0, kbeg, nk, split,
                          nob, smem);
}
}  // namespace g256

// ---------------------------------------------------------------------------
// fp32-accurate ("x6") layer-0 projection on the same 256 x 256 LDS-DMA ring:
// C[m][n] = sum_k A[m][k] B[n][k] + bias, A and B fp32 and k-contiguous, B
// given as two halves (the two LSTM directions' W_ih: rows n < bsplit from B1,
// the rest from B2).  K-tile 16 fp32 = the same 64-byte image rows as the
// bf16 kernel; each lane reads its fragment's 8 fp32 (two ds_read_b128) and
// splits them exactly into three bf16 pieces (x = x0 + x1 + x2, gemm.hip x6),
// then accumulates the six cross products a2b0 + a1b1 + a0b2 + a1b0 + a0b1 +
// a0b0 per 16-k step -- the same split, products and order as gemm.hip's x6
// main loop, so the result is bit-identical to it.  The split is repeated by
// the waves sharing a fragment (4 for A, 2 for B); the VALU work hides under
// the 48 MFMAs per wave per K-tile.
namespace x6_256 {
using g256::BM;
using g256::BN;
using g256::NSTAGE;
using g256::THREADS;
constexpr int BK = 16;                   // fp32 k per tile: 64-byte rows
constexpr int ROWB = BK * 4;
constexpr int IMG = BM * ROWB;
constexpr int STAGE = 2 * IMG;
constexpr int LDS_BYTES = NSTAGE * STAGE;
static_assert(ROWB == g256::ROWB && LDS_BYTES == g256::LDS_BYTES, "same image geometry");
using g16::bf16x8v;
using g16::f32x16v;
using g16::Bias;

__device__ __forceinline__ void stage(const float* __restrict__ P, int64_t ld, int64_t r0,
                                      int64_t R, int64_t k0, unsigned char* img, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = 2 * wave + i;
    const int row = 16 * blk + (lane >> 2);
    const int c = g256::swz(row, lane & 3);
    int64_t gr = r0 + row;
    gr = gr < R ? gr : R - 1;
    const float* src = P + gr * ld + k0 + 4 * c;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// the fragment (row, k = 8h .. 8h+7) as three bf16x8 pieces
__device__ __forceinline__ void frag3(const unsigned char* img, int row, int h, bf16x8v& p0,
                                      bf16x8v& p1, bf16x8v& p2) {
  const float4 u = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h));
  const float4 v = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h + 1));
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  uint32_t q0[4], q1[4], q2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    q0[e] = cvt_pk(a, b);
    const float ra = a - __uint_as_float(q0[e] << 16), rb = b - __uint_as_float(q0[e] & 0xffff0000u);
    q1[e] = cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(q1[e] << 16), sb = rb - __uint_as_float(q1[e] & 0xffff0000u);
    q2[e] = cvt_pk(sa, sb);
  }
  p0 = __builtin_bit_cast(bf16x8v, make_uint4(q0[0], q0[1], q0[2], q0[3]));
  p1 = __builtin_bit_cast(bf16x8v, make_uint4(q1[0], q1[1], q1[2], q1[3]));
  p2 = __builtin_bit_cast(bf16x8v, make_uint4(q2[0], q2[1], q2[2], q2[3]));
}

__global__ __launch_bounds__(THREADS, 1) void gemm_x6nt_256_kernel(
    int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
    const float* __restrict__ B1, const float* __restrict__ B2, int64_t ldb, int64_t bsplit,
    float* __restrict__ C, int64_t ldc, int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  // this n-tile's B half (the launcher guarantees bsplit % 256 == 0)
  const bool hi = n0 >= bsplit;
  const float* Bp = hi ? B2 : B1;
  const int64_t nb0 = hi ? n0 - bsplit : n0, NB = hi ? N - bsplit : bsplit;
  // split-K: blockIdx.y = split s sums k in [s*kc, min(K, (s+1)*kc)) into
  // slab C + s*strideC; the bias goes into slab 0 only
  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  float* Cs = C + split * strideC;
  const int nk = (int)((kend - kbeg) / BK);  // the launcher guarantees BK | K, BK | kc

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NSTAGE) * STAGE;
    stage(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    stage(Bp, ldb, nb0, NB, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
  };
#pragma unroll
  for (int q = 0; q < NSTAGE - 1; ++q)
    if (q < nk) issue(q);

  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;
    if (ahead >= 2) g256::wait_vm<2>();
    else if (ahead == 1) g256::wait_vm<1>();
    else g256::wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1);
    const unsigned char* sa = smem + (kt % NSTAGE) * STAGE;
    const unsigned char* sb = sa + IMG;
    bf16x8v b0[2], b1[2], b2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) frag3(sb, wn + j * 32 + li, lh, b0[j], b1[j], b2[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8v a0, a1, a2;
      frag3(sa, wm + i * 32 + li, lh, a0, a1, a2);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16v c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0[j], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split == 0) {
      if (n < bias.nsplit) {
        if (bias.a1) bv += bias.a1[n];
        if (bias.a2) bv += bias.a2[n];
      } else {
        if (bias.b1) bv += bias.b1[n - bias.nsplit];
        if (bias.b2) bv += bias.b2[n - bias.nsplit];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}

// Split-pass variant (the one ainp_gemm_x6nt_256 launches): each fp32 K-tile
// is split ONCE per workgroup -- every thread splits 8 values of one A row and
// one B row into three bf16 plane images (24 KB per operand, 32-byte rows,
// halves swapped on rows 8..15 mod 16 against bank conflicts) between two
// barriers -- instead of per fragment in every wave that reads it (4x for A,
// 2x for B).  Three fp32 stages (two tiles in flight) + the planes = 144 KB.
// Same split, products and order: bit-identical to gemm_x6nt_256_kernel
// (tools/x6split_lab.hip: 10688 x 1024 x 16448 split 3, 2.158 -> 1.938 ms).
constexpr int NST = 3;                     // fp32 ring of the split-pass kernel
constexpr int PROW = 32, PLANE = BM * PROW;                      // bf16 planes: 16 k per row
constexpr int PLANES = 2 * 3 * PLANE;                            // A0..A2, B0..B2
constexpr int LDS_BYTES_S = NST * STAGE + PLANES;               // 96 + 48 KB
static_assert(LDS_BYTES_S <= 160 * 1024, "fits");

// plane chunk h (k = 8h..8h+7) of row r, swizzled so rows r and r+8 differ
__device__ __forceinline__ int pofs(int row, int h) { return row * PROW + 16 * (h ^ ((row >> 3) & 1)); }

// thread t splits row t>>1, k = 8*(t&1) .. +7 of one operand's fp32 image
__device__ __forceinline__ void split_row(const unsigned char* img, unsigned char* planes, int t) {
  const int row = t >> 1, h = t & 1;
  const float4 u = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h));
  const float4 v = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h + 1));
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  uint32_t q0[4], q1[4], q2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    q0[e] = cvt_pk(a, b);
    const float ra = a - __uint_as_float(q0[e] << 16), rb = b - __uint_as_float(q0[e] & 0xffff0000u);
    q1[e] = cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(q1[e] << 16), sb = rb - __uint_as_float(q1[e] & 0xffff0000u);
    q2[e] = cvt_pk(sa, sb);
  }
  const int o = pofs(row, h);
  *reinterpret_cast<uint4*>(planes + o) = make_uint4(q0[0], q0[1], q0[2], q0[3]);
  *reinterpret_cast<uint4*>(planes + PLANE + o) = make_uint4(q1[0], q1[1], q1[2], q1[3]);
  *reinterpret_cast<uint4*>(planes + 2 * PLANE + o) = make_uint4(q2[0], q2[1], q2[2], q2[3]);
}

__device__ __forceinline__ bf16x8v pfrag(const unsigned char* plane, int row, int h) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(plane + pofs(row, h)));
}

__global__ __launch_bounds__(THREADS, 1) void gemm_x6nt_256s_kernel(
    int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
    const float* __restrict__ B1, const float* __restrict__ B2, int64_t ldb, int64_t bsplit,
    float* __restrict__ C, int64_t ldc, int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* planes = smem + NST * STAGE;
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  const bool hi = n0 >= bsplit;
  const float* Bp = hi ? B2 : B1;
  const int64_t nb0 = hi ? n0 - bsplit : n0, NB = hi ? N - bsplit : bsplit;
  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  float* Cs = C + split * strideC;
  const int nk = (int)((kend - kbeg) / BK);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NST) * STAGE;
    stage(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    stage(Bp, ldb, nb0, NB, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
  };
#pragma unroll
  for (int q = 0; q < NST - 1; ++q)
    if (q < nk) issue(q);

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (tile kt+1 may stay in flight); every wave is done with
    // the planes of tile kt-1 and with its fp32 stage
    if (nk - 1 - kt >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) issue(kt + NST - 1);
    const unsigned char* st = smem + (kt % NST) * STAGE;
    split_row(st, planes, tid);                       // A rows
    split_row(st + IMG, planes + 3 * PLANE, tid);     // B rows
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8v b0[2], b1[2], b2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn + j * 32 + li;
      b0[j] = pfrag(planes + 3 * PLANE, row, lh);
      b1[j] = pfrag(planes + 4 * PLANE, row, lh);
      b2[j] = pfrag(planes + 5 * PLANE, row, lh);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm + i * 32 + li;
      const bf16x8v a0 = pfrag(planes, row, lh), a1 = pfrag(planes + PLANE, row, lh),
                    a2 = pfrag(planes + 2 * PLANE, row, lh);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16v c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0[j], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split == 0) {
      if (n < bias.nsplit) {
        if (bias.a1) bv += bias.a1[n];
        if (bias.a2) bv += bias.a2[n];
      } else {
        if (bias.b1) bv += bias.b1[n - bias.nsplit];
        if (bias.b2) bv += bias.b2[n - bias.nsplit];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}
}  // namespace x6_256

}  // namespace ainp

using namespace ainp;

// AINP_G256_BK64=0: the 32-deep 4-stage ring for every g256 GEMM (A/B)
static bool g256_bk64() {
  static const bool v = [] {
    const char* e = getenv("AINP_G256_BK64");
    return !(e && e[0] == '0');
  }();
  return v;
}

extern "C" int ainp_gemm_bf16nt(int64_t M, int64_t N, int64_t K, const uint16_t* A, int64_t lda,
                                const uint16_t* B, int64_t ldb, float* C, int64_t ldc,
                                const float* bias_a1, const float* bias_a2, const float* bias_b1,
                                const float* bias_b2, int64_t bias_nsplit, int nsplit, int64_t kc,
                                int64_t strideC, void* stream) {
  if (M < 0 || N < 0 || K < 0 || !A || !B || !C || nsplit < 1 || nsplit > 65535 ||
      lda % 8 || ldb % 8 || lda < K || ldb < K || ldc < N || (K % 8) ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return record_msg("ainp_gemm_bf16nt: bad argument (16-byte aligned rows, K % 8 == 0)");
  if (nsplit > 1 && (kc < g16::BK || kc % g16::BK || (int64_t)nsplit * kc < K ||
                     (int64_t)(nsplit - 1) * kc >= K || strideC < M * ldc))
    return record_msg("ainp_gemm_bf16nt: split-K needs kc % 64 == 0 covering K, strideC >= M*ldc");
  if (nsplit == 1) kc = K;
  if (M == 0 || N == 0) return AINP_OK;
  g16::Bias b{bias_a1, bias_a2, bias_b1, bias_b2, bias_nsplit};
  // large GEMMs on the 256 x 256 LDS-DMA kernel (bit-identical: same MFMA, same
  // k order); ops._splitk_bf16 mirrors this rule for its split choice
  static const bool use256 = [] {  // AINP_GEMM16_256=0 keeps every GEMM on g16 (A/B runs)
    const char* e = getenv("AINP_GEMM16_256");
    return !(e && e[0] == '0');
  }();
  // Routing: the 256 x 256 tile (one workgroup per CU, 128 KB of LDS) only
  // for unsplit GEMMs whose 128 x 128 grid is at most two rounds of its 768
  // resident slots -- the layer-0 projection (672 tiles): 522 -> 482 us inside
  // the step.  Measured inside the step it loses where another GEMM runs beside
  // it on the side stream: the data gradient (10836 tiles) 706 -> 891 us, the
  // split-K weight gradient 621 -> 1325 us (it cannot co-reside with the
  // 3-workgroups-per-CU kernel next to it).
  // A split tall-and-narrow GEMM (M >= 8N: the layer-0 projection, 168 tiles
  // of 256 x 256 -> 504 workgroups at split 3) also runs on g256.
  const int64_t tiles128 = cdiv(M, g16::BM) * cdiv(N, g16::BN);
  if (use256 && (nsplit == 1 || M >= 8 * N) && M >= 512 && N >= 512 && tiles128 <= 1536 &&
      K % g256::BK == 0) {
    static const bool lds_ok =
        hipFuncSetAttribute((const void*)g256::gemm_bf16nt_256_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            g256::LDS_BYTES) == hipSuccess &&
        hipFuncSetAttribute((const void*)g256::gemm_bf16nt_256b_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            g256::LDS_BYTES) == hipSuccess;
    if (!lds_ok) return record_msg("ainp_gemm_bf16nt: cannot reserve 128 KB of LDS");
    const int64_t tn = cdiv(N, g256::BN);
    const dim3 grid((unsigned)(cdiv(M, g256::BM) * tn), (unsigned)nsplit);
    if (g256_bk64() && K % g256::b64::BK == 0 && kc % g256::b64::BK == 0)
      hipLaunchKernelGGL(g256::gemm_bf16nt_256b_kernel, grid, dim3(g256::THREADS), g256::LDS_BYTES,
                         as_stream(stream), M, N, K, A, lda, B, ldb, C, ldc, kc, strideC, b,
                         (int)tn);
    else
      hipLaunchKernelGGL(g256::gemm_bf16nt_256_kernel, grid, dim3(g256::THREADS), g256::LDS_BYTES,
                         as_stream(stream), M, N, K, A, lda, B, ldb, C, ldc, kc, strideC, b,
                         (int)tn);
    return check_launch("gemm_bf16nt_256");
  }
  const int64_t tiles_n = cdiv(N, g16::BN);
  const dim3 grid((unsigned)(cdiv(M, g16::BM) * tiles_n), (unsigned)nsplit);
  hipLaunchKernelGGL(g16::gemm_bf16nt_kernel, grid, dim3(g16::THREADS), 0, as_stream(stream), M, N,
                     K, A, lda, B, ldb, C, ldc, kc, strideC, b, (int)tiles_n);
  return check_launch("gemm_bf16nt");
}

extern "C" int ainp_gemm_bf16nt_multi(const ainp_bf16_problem* probs, int nprobs, void* stream) {
  if (!probs || nprobs < 1 || nprobs > g256::MAXP)
    return record_msg("ainp_gemm_bf16nt_multi: 1..3 problems");
  g256::MJob job{};
  job.np = nprobs;
  int64_t first = 0;
  for (int q = 0; q < nprobs; ++q) {
    const ainp_bf16_problem& s = probs[q];
    const int nsplit = s.nsplit < 1 ? 1 : s.nsplit;
    const int64_t kc = nsplit == 1 ? s.K : s.kc;
    if (!s.A || !s.B || !s.C || s.M < 1 || s.N < 1 || s.K < g256::BK || s.K % g256::BK ||
        s.lda % 8 || s.ldb % 8 || s.lda < (s.a_kmajor ? s.M : s.K) ||
        s.ldb < (s.b_kmajor ? s.N : s.K) || s.ldc < s.N || (s.a_kmajor && s.M % 8) ||
        (s.b_kmajor && s.N % 8) ||
        ((uintptr_t)s.A & 15) || ((uintptr_t)s.B & 15) || nsplit > 65535 ||
        (nsplit > 1 && (kc < g256::BK || kc % g256::BK || (int64_t)nsplit * kc < s.K ||
                        (int64_t)(nsplit - 1) * kc >= s.K || s.strideC < s.M * s.ldc)))
      return record_msg("ainp_gemm_bf16nt_multi: bad problem (K, kc % 32 == 0 covering K; "
                        "16-byte aligned k-contiguous rows; strideC >= M*ldc when split)");
    g256::MProb& d = job.p[q];
    d.A = s.A; d.B = s.B; d.C = s.C;
    d.lda = s.lda; d.ldb = s.ldb; d.ldc = s.ldc;
    d.M = s.M; d.N = s.N; d.K = s.K; d.kc = kc; d.strideC = s.strideC;
    d.tiles_m = (int)cdiv(s.M, g256::BM);
    d.tiles_n = (int)cdiv(s.N, g256::BN);
    d.nsplit = nsplit;
    d.a_km = s.a_kmajor ? 1 : 0;
    d.b_km = s.b_kmajor ? 1 : 0;
    d.items = (int64_t)d.tiles_m * d.tiles_n * nsplit;
    d.first = first;
    first += (d.items + 7) / 8 * 8;
  }
  job.bk64 = g256_bk64() ? 1 : 0;
  for (int q = 0; q < nprobs; ++q)
    if (job.p[q].K % g256::b64::BK || job.p[q].kc % g256::b64::BK) job.bk64 = 0;
  static const bool lds_ok =
      hipFuncSetAttribute((const void*)g256::gemm_bf16nt_256_multi_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, g256::LDS_BYTES) == hipSuccess;
  if (!lds_ok) return record_msg("ainp_gemm_bf16nt_multi: cannot reserve 128 KB of LDS");
  if (first > 0x7fffffff) return record_msg("ainp_gemm_bf16nt_multi: grid too large");
  hipLaunchKernelGGL(g256::gemm_bf16nt_256_multi_kernel, dim3((unsigned)first), dim3(g256::THREADS),
                     g256::LDS_BYTES, as_stream(stream), job);
  return check_launch("gemm_bf16nt_256_multi");
}

extern "C" int ainp_wgrad16_nhwc(const uint16_t* gA, int64_t ldA, int Cout, const uint16_t* x16,
                                 int64_t N, int Cin, int H, int W, int k, int stride, int pad,
                                 float* G, int nsplit, int64_t kc, void* stream) {
  if (!gA || !x16 || !G || Cout < 1 || N < 1 || Cin < 8 || Cin % 8 || k < 1 || stride < 1 ||
      pad < 0 || ldA % 8 || ((uintptr_t)gA & 15) || ((uintptr_t)x16 & 15) || nsplit < 1 ||
      nsplit > 65535)
    return record_msg("ainp_wgrad16_nhwc: bad argument (Cin % 8 == 0, 16-byte aligned)");
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t NP = N * (int64_t)Ho * Wo;
  if (Ho < 1 || Wo < 1 || ldA < NP) return record_msg("ainp_wgrad16_nhwc: bad shape (ldA >= N*Ho*Wo)");
  const int64_t K = ldA;   // gA is zero past N*Ho*Wo, as im2col16's columns
  if (nsplit > 1 && (kc < g16::BK || kc % g16::BK || (int64_t)nsplit * kc < K ||
                     (int64_t)(nsplit - 1) * kc >= K))
    return record_msg("ainp_wgrad16_nhwc: split-K needs kc % 64 == 0 covering ldA");
  if (nsplit == 1) kc = K;
  const int64_t Ncol = (int64_t)Cin * k * k + 1;
  g16::WgGeom geo{x16, (int)N, Cin, H, W, k, k * k, stride, pad, Ho, Wo, NP};
  const int64_t tiles_n = cdiv(Ncol, g16::BN);
  const int64_t nwg = cdiv(Cout, g16::BM) * tiles_n * nsplit;
  if (nwg > 0x7fffffff) return record_msg("ainp_wgrad16_nhwc: grid too large");
  const dim3 grid((unsigned)nwg);
  hipLaunchKernelGGL(g16::wgrad16_nhwc_kernel, grid, dim3(g16::THREADS), 0, as_stream(stream),
                     (int64_t)Cout, Ncol, K, gA, ldA, geo, G, Ncol, kc, (int64_t)Cout * Ncol,
                     (int)tiles_n);
  return check_launch("wgrad16_nhwc");
}

extern "C" int ainp_gemm_x6nt_256(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                  const float* B1, const float* B2, int64_t ldb, int64_t bsplit,
                                  float* C, int64_t ldc, const float* bias_a1,
                                  const float* bias_a2, const float* bias_b1,
                                  const float* bias_b2, int64_t bias_nsplit, int nsplit,
                                  int64_t kc, int64_t strideC, void* stream) {
  if (nsplit < 1 || nsplit > 65535 ||
      (nsplit > 1 && (kc < x6_256::BK || kc % x6_256::BK || (int64_t)nsplit * kc < K ||
                      (int64_t)(nsplit - 1) * kc >= K || strideC < M * ldc)))
    return record_msg("ainp_gemm_x6nt_256: split-K needs kc % 16 == 0 covering K, strideC >= M*ldc");
  if (nsplit == 1) kc = K;
  if (M < 0 || N < 0 || K < 0 || !A || !B1 || !C || lda % 4 || ldb % 4 || lda < K || ldb < K ||
      ldc < N || K % x6_256::BK || ((uintptr_t)A & 15) || ((uintptr_t)B1 & 15) ||
      bsplit < 0 || bsplit > N || (bsplit % x6_256::BN && bsplit != N) ||
      (bsplit < N && (!B2 || ((uintptr_t)B2 & 15))))
    return record_msg("ainp_gemm_x6nt_256: bad argument (16-byte aligned k-contiguous rows, "
                      "K % 16 == 0, bsplit % 256 == 0 or bsplit == N)");
  if (M == 0 || N == 0) return AINP_OK;
  // AINP_X6_SPLITPASS=0 keeps the per-fragment-split kernel (A/B runs)
  static const bool splitpass = [] {
    const char* e = getenv("AINP_X6_SPLITPASS");
    return !(e && e[0] == '0');
  }();
  static const bool lds_ok =
      hipFuncSetAttribute((const void*)x6_256::gemm_x6nt_256_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          x6_256::LDS_BYTES) == hipSuccess &&
      hipFuncSetAttribute((const void*)x6_256::gemm_x6nt_256s_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize,
                          x6_256::LDS_BYTES_S) == hipSuccess;
  if (!lds_ok) return record_msg("ainp_gemm_x6nt_256: cannot reserve 144 KB of LDS");
  g16::Bias b{bias_a1, bias_a2, bias_b1, bias_b2, bias_nsplit};
  const int64_t tn = cdiv(N, x6_256::BN);
  const dim3 grid((unsigned)(cdiv(M, x6_256::BM) * tn), (unsigned)nsplit);
  if (splitpass)
    hipLaunchKernelGGL(x6_256::gemm_x6nt_256s_kernel, grid, dim3(x6_256::THREADS),
                       x6_256::LDS_BYTES_S, as_stream(stream), M, N, K, A, lda, B1, B2, ldb,
                       bsplit, C, ldc, kc, strideC, b, (int)tn);
  else
    hipLaunchKernelGGL(x6_256::gemm_x6nt_256_kernel, grid, dim3(x6_256::THREADS),
                       x6_256::LDS_BYTES, as_stream(stream), M, N, K, A, lda, B1, B2, ldb, bsplit,
                       C, ldc, kc, strideC, b, (int)tn);
  return check_launch("gemm_x6nt_256");
}

extern "C" int ainp_cast_bf16_t(const float* x, int64_t R, int64_t C, int64_t ld_in,
                                uint16_t* out, int64_t ld_out, uint16_t* outT, int64_t ld_t,
                                void* stream) {
  if (!x || R < 0 || C < 0 || ld_in < C || (!out && !outT) || (out && ld_out < C) ||
      (outT && ld_t < R))
    return record_msg("ainp_cast_bf16_t: bad argument");
  if (R == 0 || C == 0) return AINP_OK;
  hipLaunchKernelGGL(g16::cast_bf16_t_kernel, dim3((unsigned)cdiv(C, 64), (unsigned)cdiv(R, 64)),
                     dim3(256), 0, as_stream(stream), x, R, C, ld_in, out, ld_out, outT, ld_t);
  return check_launch("cast_bf16_t");
}

extern "C" int ainp_transpose_f32(const float* x, int64_t R, int64_t C, int64_t ld_in, float* outT,
                                  int64_t ld_t, void* stream) {
  if (R < 0 || C < 0 || !x || !outT || ld_in < C || ld_t < R)
    return record_msg("ainp_transpose_f32: bad argument");
  if (R == 0 || C == 0) return AINP_OK;
  hipLaunchKernelGGL(g16::transpose_f32_kernel, dim3((unsigned)cdiv(C, 64), (unsigned)cdiv(R, 64)),
                     dim3(256), 0, as_stream(stream), x, R, C, ld_in, outT, ld_t);
  return check_launch("transpose_f32");
}
