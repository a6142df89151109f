// gan.hip — kernels of the GAN training path:
// PConvUNet (models/GAN/networks.py:10-345), the spectral-norm Discriminator
// (networks.py:352-409), VGGLoss (models/GAN/loss.py) and calculate_losses /
// the D step (models/GAN/train.py:33-88, 341-378).
//
// conv_gen_fwd is the workhorse: an implicit-GEMM convolution on
// v_mfma_f32_16x16x4_f32 (exact fp32) for any kernel size / stride / zero
// padding, whose im2col gather reads up to two NCHW sources (the decoder's
// nearest-x2-upsampled input and the encoder skip: the torch.cat of
// networks.py:297-298,317-318 is never materialised), multiplies each element
// by its source's partial-conv mask plane, and whose epilogue applies the
// spectral-norm 1/sigma, the partial-conv window ratio, the bias, BatchNorm
// statistics partials and ReLU / LeakyReLU.
//
// GEMM view: C[co][p] = sum_k W'[co][k] * X[k][p], p = (n, oy, ox) flattened,
// k = tap * Cin + ci (tap-major).  When Cin and the concat split are
// multiples of 32 every 32-deep K tile has ONE tap, so the gather's bounds,
// mask and address arithmetic are per tile, not per element ("fast" path).
#include <stdlib.h>

#include "common.h"

namespace ainp {

struct ConvSrcDev {
  const float* x;   // [N, C, Hs, Ws]
  const float* m;   // mask plane [N, Hs, Ws] (same for every channel) or null
  int C, Hs, Ws;
  int up;           // 0: Hs==Hin; 1: exact nearest x2 (i>>1); 2: nearest i*Hs/Hin
};

struct ConvGenParams {
  ConvSrcDev s0, s1;        // channels [0, s0.C) then [s0.C, s0.C + s1.C)
  const float* w;           // [Cout][Cin][KH][KW]
  const float* bias;        // [Cout] or null
  const float* ratio;       // [N][Ho][Wo] partial-conv window ratio or null
  const float* scale;       // device scalar multiplier (1/sigma) or null
  float* y;                 // [N][Cout][Ho][Wo]
  double* stats;            // [px_tiles][2][Cout] (sum, sumsq of the stored y) or null
  float* partial;           // split-K: raw sums [gridDim.z][Cout][N*Ho*Wo], epilogue deferred
  uint16_t* y16;            // optional bf16 channel-last copy of y: [N][Ho][Wo][Cout] (nhwc16
                            // and few-input-channel kernels)
  int ktiles_per_split;     // K tiles per blockIdx.z
  int N, Cin, Cout, Hin, Win, Ho, Wo, KH, KW, stride, pad;
  float slope;              // LeakyReLU negative slope (act == 2)
};

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_LEAKY = 2, ACT_TANH = 3 };

__device__ __forceinline__ int src_coord(int i, int S, int L, int up) {
  return up == 0 ? i : (up == 1 ? (i >> 1) : (int)(((int64_t)i * S) / L));
}

__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_LEAKY) return v > 0.f ? v : v * slope;
  if (act == ACT_TANH) return tanhf(v);
  return v;
}

// The optional channel-last bf16 copy (nearest-even) of an MFMA epilogue's
// outputs: register r of a 32x32 accumulator holds channel (r&3) + 8(r>>2) +
// 4(lane>>5), so registers 4q..4q+3 are 4 consecutive channels of the lane's
// pixel -- one 8-byte store each (Cout % 4 == 0; else element stores).  The
// value is recomputed exactly as the fp32 store's (same operations, same order).
__device__ __forceinline__ void store_y16_quad(const ConvGenParams& p, int64_t pg, int co,
                                               const float (&o)[4]) {
  uint16_t* d = p.y16 + pg * p.Cout + co;
  if ((p.Cout & 3) == 0 && co + 3 < p.Cout) {
    uint2 u;
    u.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)o[0]) |
          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)o[1]) << 16);
    u.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)o[2]) |
          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)o[3]) << 16);
    *reinterpret_cast<uint2*>(d) = u;
  } else {
    for (int e = 0; e < 4; ++e)
      if (co + e < p.Cout) d[e] = __builtin_bit_cast(uint16_t, (__bf16)o[e]);
  }
}
template <int MI, int NJ>
__device__ __forceinline__ void epilogue_y16(const ConvGenParams& p, const f32x16 (&acc)[MI][NJ],
                                             int act, int64_t px_w, int co_w, const bool* ok,
                                             const float* rt, int lh, int l31) {
  const float sc = p.scale ? *p.scale : 1.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (!ok[j]) continue;
    const int64_t pg = px_w + 32 * j + l31;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = co_w + 32 * i + 8 * q + 4 * lh;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float bv = (co + e < p.Cout && p.bias) ? p.bias[co + e] : 0.f;
          float v = acc[i][j][4 * q + e] * sc;
          v *= rt[j];
          v += bv;
          o[e] = apply_act(v, act, p.slope);
        }
        store_y16_quad(p, pg, co, o);
      }
  }
}

// The same copy through a wave-private LDS transpose (the wide kernel's free
// ring): per 32-pixel group the wave stages [32 px][MI*32 co] bf16 (144-byte
// rows) and stores whole 128-byte pixel rows, 16 bytes per lane, instead of
// 8-byte pieces 2*Cout bytes apart.  Edge tiles (Cout % 8, last co tile) use
// epilogue_y16.
template <int MI, int NJ>
__device__ __forceinline__ void epilogue_y16_lds(const ConvGenParams& p,
                                                 const f32x16 (&acc)[MI][NJ], int act,
                                                 int64_t px_w, int co_w, const bool* ok,
                                                 const float* rt, int lh, int l31, int lane,
                                                 uint16_t* stg, int64_t NP) {
  constexpr int RS = MI * 32 + 8;                 // staging row stride (bf16)
  constexpr int CPR = MI * 32 / 8;                // 16-byte chunks per pixel row
  if ((p.Cout & 7) || co_w + MI * 32 > p.Cout) {
    epilogue_y16<MI, NJ>(p, acc, act, px_w, co_w, ok, rt, lh, l31);
    return;
  }
  const float sc = p.scale ? *p.scale : 1.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cl = 32 * i + 8 * q + 4 * lh;
        uint32_t h[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float bv = p.bias ? p.bias[co_w + cl + e] : 0.f;
          float v = acc[i][j][4 * q + e] * sc;
          v *= rt[j];
          v += bv;
          h[e] = __builtin_bit_cast(uint16_t, (__bf16)apply_act(v, act, p.slope));
        }
        *reinterpret_cast<uint2*>(stg + l31 * RS + cl) =
            make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 32 * CPR / 64; ++it) {
      const int c = it * 64 + lane, px = c / CPR, cb = (c % CPR) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(stg + px * RS + cb);
      const int64_t pg = px_w + 32 * j + px;
      if (pg < NP) *reinterpret_cast<uint4*>(p.y16 + pg * p.Cout + co_w + cb) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

constexpr int CG_BK = 32;

typedef float f32x16 __attribute__((ext_vector_type(16)));
// v_mfma_f32_32x32x2_f32: lane l holds A[row l&31][k l>>5], B[k l>>5][col l&31];
// D[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31] in register r.
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// K order: source region 0 (k = tap*C0 + ci) then region 1 (k = KK*C0 + tap*C1 + ci).
// wt[k][co] = w[co][cbase(s) + ci][tap]   (k-major, co contiguous)
__global__ void conv_weight_kmajor_kernel(const float* w, int Cout, int C0, int C1, int KK,
                                          float* wt) {
  const int Cin = C0 + C1;
  const int64_t total = (int64_t)Cin * KK * Cout;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int co = (int)(t % Cout);
  const int k = (int)(t / Cout);
  const int K0 = KK * C0;
  int tap, c;
  if (k < K0) {
    tap = k / C0;
    c = k - tap * C0;
  } else {
    tap = (k - K0) / C1;
    c = C0 + (k - K0 - tap * C1);
  }
  wt[t] = w[((int64_t)co * Cin + c) * KK + tap];
}

// Shared epilogue of the implicit-GEMM convolutions (both main loops):
// split-K partial slab, or 1/sigma, partial-conv ratio, bias, BatchNorm
// statistics (fixed order) and activation.  red: >= WN*BM*2 doubles of LDS.
template <int BM>
__device__ __forceinline__ void conv_gen_epilogue(const ConvGenParams& p, f32x16 (&acc)[2][2],
                                                  int act, double* red) {
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, lh = lane >> 5;
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  const int co0 = blockIdx.y * BM;
  if (p.partial) {   // split-K: raw partial sums, the epilogue kernel finishes
    float* pb = p.partial + (int64_t)blockIdx.z * p.Cout * NP;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t pg = px0 + wn * 64 + 32 * j + l31;
      if (pg >= NP) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (co < p.Cout) pb[(int64_t)co * NP + pg] = acc[i][j][r];
        }
    }
    return;
  }
  // ---------------- epilogue
  const float sc = p.scale ? *p.scale : 1.f;
  bool ok[2];
  float rt[2];
  float* yb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t pg = px0 + wn * 64 + 32 * j + l31;
    ok[j] = pg < NP;
    int pn = 0, prem = 0;
    if (ok[j]) {
      pn = (int)(pg / HWo);
      prem = (int)(pg - (int64_t)pn * HWo);
    }
    rt[j] = (ok[j] && p.ratio) ? p.ratio[pg] : 1.f;
    yb[j] = p.y + (int64_t)pn * p.Cout * HWo + prem;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cl = wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int co = co0 + cl;
      const bool cok = co < p.Cout;
      const float bv = (cok && p.bias) ? p.bias[co] : 0.f;
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!ok[j] || !cok) continue;
        float v = acc[i][j][r] * sc;
        v *= rt[j];
        v += bv;
        a += (double)v;
        b += (double)v * (double)v;
        yb[j][(int64_t)co * HWo] = apply_act(v, act, p.slope);
      }
      if (p.stats) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
        }
        if (l31 == 0) {
          red[(wn * BM + cl) * 2 + 0] = a;
          red[(wn * BM + cl) * 2 + 1] = b;
        }
      }
    }
  }
  if (p.y16) epilogue_y16<2, 2>(p, acc, act, px0 + wn * 64, co0 + wm * 64, ok, rt, lh, l31);
  if (p.stats) {
    __syncthreads();
    if (tid < BM) {
      const int co = co0 + tid;
      if (co < p.Cout) {
        double a = 0.0, b = 0.0;
        for (int q = 0; q < WN; ++q) {
          a += red[(q * BM + tid) * 2];
          b += red[(q * BM + tid) * 2 + 1];
        }
        p.stats[((int64_t)blockIdx.x * 2 + 0) * p.Cout + co] = a;
        p.stats[((int64_t)blockIdx.x * 2 + 1) * p.Cout + co] = b;
      }
    }
  }
}

// Implicit-GEMM convolution: block tile BM (co) x BN (pixels) x 32 (k), four
// waves each owning a 64x64 sub-tile (2x2 v_mfma_f32_32x32x2_f32).  BM=128,
// BN=128 (waves 2x2) for Cout > 64; BM=64, BN=256 (waves 1x4) otherwise, so
// narrow layers do not waste half the MFMA work.  The next K tile is gathered
// into registers while the current one is multiplied (one LDS image each).
template <int BM>
__global__ __launch_bounds__(256, 2) void conv_gen_fwd_kernel(ConvGenParams p, const float* wt,
                                                              int act) {
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;                 // waves along pixels (2 or 4)
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int AR = CG_BK * BM / 256;        // A elements per thread per tile (16 / 8)
  constexpr int BR = CG_BK * BN / 256;        // B elements per thread per tile (16 / 32)
  constexpr int AKS = 256 / BM;               // k-row step of the A staging map
  constexpr int BKS = 256 / BN;               // k-row step of the B staging map (2 / 1)
  __shared__ __attribute__((aligned(16))) float sA[CG_BK * LDA];
  __shared__ __attribute__((aligned(16))) float sB[CG_BK * LDB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = p.KH * p.KW;
  const int K0 = KK * p.s0.C;
  const int K = KK * p.Cin;
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  const int co0 = blockIdx.y * BM;
  const int kt_begin = blockIdx.z * p.ktiles_per_split;
  int kt_end = kt_begin + p.ktiles_per_split;
  const int nkt_all = (K + CG_BK - 1) / CG_BK;
  if (kt_end > nkt_all) kt_end = nkt_all;

  // B staging: pixel = tid % BN, k rows = tid / BN + BKS*i (wave-uniform)
  const int bpx = tid % BN, bk0 = tid / BN;
  const int64_t pix = px0 + bpx;
  const bool pv = pix < NP;
  int n = 0, by = 0, bx = 0;
  if (pv) {
    n = (int)(pix / HWo);
    const int r = (int)(pix - (int64_t)n * HWo);
    const int oy = r / p.Wo, ox = r - oy * p.Wo;
    by = oy * p.stride - p.pad;
    bx = ox * p.stride - p.pad;
  }
  // A staging: co = tid % BM, k rows = tid / BM + AKS*i
  const int aco = tid % BM, ak0 = tid / BM;
  const bool acok = co0 + aco < p.Cout;

  float ra[AR], rb[BR];
  auto gather1 = [&](int k) -> float {        // generic: one element of X[k][pix]
    if (!pv || k >= K) return 0.f;
    const bool first = k < K0;
    const ConvSrcDev& s = first ? p.s0 : p.s1;
    const int kr = first ? k : k - K0;
    const int tap = kr / s.C, cs = kr - tap * s.C;
    const int ky = tap / p.KW, kx = tap - ky * p.KW;
    const int iy = by + ky, ix = bx + kx;
    if (iy < 0 || iy >= p.Hin || ix < 0 || ix >= p.Win) return 0.f;
    const int sy = src_coord(iy, s.Hs, p.Hin, s.up), sx = src_coord(ix, s.Ws, p.Win, s.up);
    const int64_t plane = (int64_t)s.Hs * s.Ws;
    const int64_t off = (int64_t)sy * s.Ws + sx;
    float v = s.x[((int64_t)n * s.C + cs) * plane + off];
    if (s.m) v *= s.m[(int64_t)n * plane + off];
    return v;
  };
  auto fetch = [&](int kt) {
    const int k0 = kt * CG_BK;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = k0 + ak0 + AKS * i;
      ra[i] = (acok && k < K) ? wt[(int64_t)k * p.Cout + co0 + aco] : 0.f;
    }
    // a tile lies in one region; in a region with C % 32 == 0 it has one tap
    const bool first = k0 < K0;
    const ConvSrcDev& s = first ? p.s0 : p.s1;
    if (s.C % CG_BK == 0) {
      const int kr = first ? k0 : k0 - K0;
      const int tap = kr / s.C, ci0 = kr - tap * s.C;
      const int ky = tap / p.KW, kx = tap - ky * p.KW;
      const int iy = by + ky, ix = bx + kx;
      const bool inb = pv && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int sy = inb ? src_coord(iy, s.Hs, p.Hin, s.up) : 0;
      const int sx = inb ? src_coord(ix, s.Ws, p.Win, s.up) : 0;
      const int64_t plane = (int64_t)s.Hs * s.Ws;
      const int64_t off = (int64_t)sy * s.Ws + sx;
      const float mv = (inb && s.m) ? s.m[(int64_t)n * plane + off] : 1.f;
      const float* base = s.x + ((int64_t)n * s.C + ci0 + bk0) * plane + off;
#pragma unroll
      for (int i = 0; i < BR; ++i) rb[i] = inb ? base[(int64_t)(BKS * i) * plane] * mv : 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < BR; ++i)
        rb[i] = gather1(__builtin_amdgcn_readfirstlane(k0 + bk0 + BKS * i));
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < AR; ++i) sA[(ak0 + AKS * i) * LDA + aco] = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i) sB[(bk0 + BKS * i) * LDB + bpx] = rb[i];
  };

  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt_begin < kt_end) fetch(kt_begin);
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    commit();
    __syncthreads();
    if (kt + 1 < kt_end) fetch(kt + 1);
    const float* pa = sA + lh * LDA + wm * 64 + l31;
    const float* pb = sB + lh * LDB + wn * 64 + l31;
#pragma unroll
    for (int s = 0; s < CG_BK / 2; ++s) {
      const float a0 = pa[2 * s * LDA], a1 = pa[2 * s * LDA + 32];
      const float b0 = pb[2 * s * LDB], b1 = pb[2 * s * LDB + 32];
      acc[0][0] = mfma32x32x2(a0, b0, acc[0][0]);
      acc[0][1] = mfma32x32x2(a0, b1, acc[0][1]);
      acc[1][0] = mfma32x32x2(a1, b0, acc[1][0]);
      acc[1][1] = mfma32x32x2(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }

  conv_gen_epilogue<BM>(p, acc, act, reinterpret_cast<double*>(sA));
}

// ---------------------------------------------------------------- x6 variant
// The same implicit GEMM with gemm.hip's fp32-accurate split-bf16 main loop:
// every staged element x = x0 + x1 + x2 (three bf16 pieces, round-to-nearest,
// exact), six cross products of order >= 2^-16 per product on
// v_mfma_f32_32x32x16_bf16 (dropped terms <= ~2^-23 |a||b|).  Staging maps
// give each thread ONE row (output channel for A, pixel for B) and a run of
// consecutive k, so the split pieces go to LDS as 16-byte vectors of three
// bf16 planes [row][32 k] with 80-byte rows (conflict-free ds_read_b128
// fragments: lane (row r, half h) reads k = 16s + 8h..+7).  The gather, the
// one-tap-per-tile fast path and the epilogue are conv_gen_fwd_kernel's.
namespace cgx {
__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
// split 8 consecutive-k values into one 16-byte vector per piece, exactly
__device__ __forceinline__ void split8(const float* v, uint4& p0, uint4& p1, uint4& p2) {
  uint32_t q0[4], q1[4], q2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = v[2 * e], b = v[2 * e + 1];
    q0[e] = cvt_pk(a, b);
    const float ra = a - __uint_as_float(q0[e] << 16), rb = b - __uint_as_float(q0[e] & 0xffff0000u);
    q1[e] = cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(q1[e] << 16), sb = rb - __uint_as_float(q1[e] & 0xffff0000u);
    q2[e] = cvt_pk(sa, sb);
  }
  p0 = make_uint4(q0[0], q0[1], q0[2], q0[3]);
  p1 = make_uint4(q1[0], q1[1], q1[2], q1[3]);
  p2 = make_uint4(q2[0], q2[1], q2[2], q2[3]);
}
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ bf16x8 frag(const unsigned char* q) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(q));
}
}  // namespace cgx

// XBK = 16: 16-deep K-tiles with 48-byte image rows (37-46 KB of LDS and
// <= 168 VGPRs: three workgroups per CU); XBK = 32: 80-byte rows, two.
// Split-K ranges (p.ktiles_per_split) stay in CG_BK units.
// NPL = 3: the fp32-accurate split; NPL = 1 (AINP_CONV_BF16): one bf16 plane
// per operand (operands rounded to bf16, fp32 accumulation).
template <int BM, int XBK, int NPL>
__global__ __launch_bounds__(256, XBK == 16 ? 3 : 2) void conv_gen_x6_kernel(ConvGenParams p,
                                                                             const float* wt,
                                                                             int act) {
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;                 // waves along pixels (2 or 4)
  constexpr int AR = XBK * BM / 256;          // consecutive k per thread, A
  constexpr int BR = XBK * BN / 256;          // consecutive k per thread, B
  constexpr int RS = XBK * 2 + 16;            // image row: XBK bf16 + 16-byte pad
  constexpr int APL = BM * RS, BPL = BN * RS;   // plane bytes
  constexpr int ESCR = WN * BM * 2 * (int)sizeof(double);   // epilogue scratch (in sA)
  __shared__ __attribute__((aligned(16))) unsigned char sA[NPL * APL > ESCR ? NPL * APL : ESCR];
  __shared__ __attribute__((aligned(16))) unsigned char sB[NPL * BPL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = p.KH * p.KW;
  const int K0 = KK * p.s0.C;
  const int K = KK * p.Cin;
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  const int co0 = blockIdx.y * BM;
  // split-K ranges are in CG_BK units (the host keeps them XBK-aligned)
  const int nkt_all = (K + XBK - 1) / XBK;
  const int64_t kb = (int64_t)blockIdx.z * p.ktiles_per_split * CG_BK / XBK;
  const int64_t ke = kb + (int64_t)p.ktiles_per_split * CG_BK / XBK;
  const int kt_begin = (int)(kb < nkt_all ? kb : nkt_all);
  const int kt_end = (int)(ke < nkt_all ? ke : nkt_all);

  // B staging: pixel bpx = tid % BN, k run [bkq*BR, bkq*BR + BR) (wave-uniform)
  const int bpx = tid % BN, bkq = tid / BN;
  const int64_t pix = px0 + bpx;
  const bool pv = pix < NP;
  int n = 0, by = 0, bx = 0;
  if (pv) {
    n = (int)(pix / HWo);
    const int r = (int)(pix - (int64_t)n * HWo);
    const int oy = r / p.Wo, ox = r - oy * p.Wo;
    by = oy * p.stride - p.pad;
    bx = ox * p.stride - p.pad;
  }
  // A staging: output channel aco = tid % BM, k run [akq*AR, akq*AR + AR)
  const int aco = tid % BM, akq = tid / BM;
  const bool acok = co0 + aco < p.Cout;

  float ra[AR], rb[BR];
  auto gather1 = [&](int k) -> float {        // generic: one element of X[k][pix]
    if (!pv || k >= K) return 0.f;
    const bool first = k < K0;
    const ConvSrcDev& s = first ? p.s0 : p.s1;
    const int kr = first ? k : k - K0;
    const int tap = kr / s.C, cs = kr - tap * s.C;
    const int ky = tap / p.KW, kx = tap - ky * p.KW;
    const int iy = by + ky, ix = bx + kx;
    if (iy < 0 || iy >= p.Hin || ix < 0 || ix >= p.Win) return 0.f;
    const int sy = src_coord(iy, s.Hs, p.Hin, s.up), sx = src_coord(ix, s.Ws, p.Win, s.up);
    const int64_t plane = (int64_t)s.Hs * s.Ws;
    const int64_t off = (int64_t)sy * s.Ws + sx;
    float v = s.x[((int64_t)n * s.C + cs) * plane + off];
    if (s.m) v *= s.m[(int64_t)n * plane + off];
    return v;
  };
  auto fetch = [&](int kt) {
    const int k0 = kt * XBK;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int k = k0 + akq * AR + i;
      ra[i] = (acok && k < K) ? wt[(int64_t)k * p.Cout + co0 + aco] : 0.f;
    }
    const bool first = k0 < K0;
    const ConvSrcDev& s = first ? p.s0 : p.s1;
    if (s.C % XBK == 0) {                     // the whole tile is one tap of one source
      const int kr = first ? k0 : k0 - K0;
      const int tap = kr / s.C, ci0 = kr - tap * s.C;
      const int ky = tap / p.KW, kx = tap - ky * p.KW;
      const int iy = by + ky, ix = bx + kx;
      const bool inb = pv && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int sy = inb ? src_coord(iy, s.Hs, p.Hin, s.up) : 0;
      const int sx = inb ? src_coord(ix, s.Ws, p.Win, s.up) : 0;
      const int64_t plane = (int64_t)s.Hs * s.Ws;
      const int64_t off = (int64_t)sy * s.Ws + sx;
      const float mv = (inb && s.m) ? s.m[(int64_t)n * plane + off] : 1.f;
      const float* base = s.x + ((int64_t)n * s.C + ci0 + bkq * BR) * plane + off;
#pragma unroll
      for (int i = 0; i < BR; ++i) rb[i] = inb ? base[(int64_t)i * plane] * mv : 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < BR; ++i)
        rb[i] = gather1(__builtin_amdgcn_readfirstlane(k0 + bkq * BR + i));
    }
  };
  // 8 consecutive-k values -> NP planes (the exact split, or one bf16 rounding)
  auto pieces = [&](const float* v, uint4& q0, uint4& q1, uint4& q2) {
    if (NPL == 3) {
      cgx::split8(v, q0, q1, q2);
    } else {
      q0 = make_uint4(cgx::cvt_pk(v[0], v[1]), cgx::cvt_pk(v[2], v[3]), cgx::cvt_pk(v[4], v[5]),
                      cgx::cvt_pk(v[6], v[7]));
      q1 = q2 = q0;
    }
  };
  auto commit = [&]() {
    if (AR >= 8) {
#pragma unroll
      for (int i = 0; i < AR; i += 8) {
        uint4 q0, q1, q2;
        pieces(ra + i, q0, q1, q2);
        unsigned char* q = sA + aco * RS + (akq * AR + i) * 2;
        *reinterpret_cast<uint4*>(q) = q0;
        if (NPL == 3) {
          *reinterpret_cast<uint4*>(q + APL) = q1;
          *reinterpret_cast<uint4*>(q + 2 * APL) = q2;
        }
      }
    } else {                                  // AR == 4: one 8-byte piece per plane
      float v8[8] = {ra[0 % AR], ra[1 % AR], ra[2 % AR], ra[3 % AR], 0.f, 0.f, 0.f, 0.f};
      uint4 q0, q1, q2;
      pieces(v8, q0, q1, q2);
      unsigned char* q = sA + aco * RS + (akq * AR) * 2;
      *reinterpret_cast<uint2*>(q) = make_uint2(q0.x, q0.y);
      if (NPL == 3) {
        *reinterpret_cast<uint2*>(q + APL) = make_uint2(q1.x, q1.y);
        *reinterpret_cast<uint2*>(q + 2 * APL) = make_uint2(q2.x, q2.y);
      }
    }
#pragma unroll
    for (int i = 0; i < BR; i += 8) {
      uint4 q0, q1, q2;
      pieces(rb + i, q0, q1, q2);
      unsigned char* q = sB + bpx * RS + (bkq * BR + i) * 2;
      *reinterpret_cast<uint4*>(q) = q0;
      if (NPL == 3) {
        *reinterpret_cast<uint4*>(q + BPL) = q1;
        *reinterpret_cast<uint4*>(q + 2 * BPL) = q2;
      }
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt_begin < kt_end) fetch(kt_begin);
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    commit();
    __syncthreads();
    if (kt + 1 < kt_end) fetch(kt + 1);
#pragma unroll
    for (int st = 0; st < XBK / 16; ++st) {
      cgx::bf16x8 a[NPL][2], b[NPL][2];
#pragma unroll
      for (int q = 0; q < NPL; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          a[q][i] = cgx::frag(sA + q * APL + (wm * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh);
          b[q][i] = cgx::frag(sB + q * BPL + (wn * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 c = acc[i][j];
          if (NPL == 3) {   // six cross terms, smallest first
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2 % NPL][i], b[0][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1 % NPL][i], b[1 % NPL][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2 % NPL][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1 % NPL][i], b[0][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1 % NPL][j], c, 0, 0, 0);
          }
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], c, 0, 0, 0);
          acc[i][j] = c;
        }
    }
    __syncthreads();
  }
  conv_gen_epilogue<BM>(p, acc, act, reinterpret_cast<double*>(sA));
}

// Split-K epilogue: y[n][co][p] = act(sum_z partial[z][co][px] * scale * ratio + bias),
// one block = 256 pixels of one channel; stats per (pixel block, channel).
__global__ __launch_bounds__(256) void conv_gen_splitk_epilogue(ConvGenParams p, int nsplit,
                                                                int act) {
  const int co = blockIdx.y;
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double a = 0.0, b = 0.0;
  if (px < NP) {
    float v = 0.f;
    for (int z = 0; z < nsplit; ++z) v += p.partial[((int64_t)z * p.Cout + co) * NP + px];
    v *= p.scale ? *p.scale : 1.f;
    if (p.ratio) v *= p.ratio[px];
    if (p.bias) v += p.bias[co];
    a = v;
    b = (double)v * (double)v;
    const int n = (int)(px / HWo);
    const int r = (int)(px - (int64_t)n * HWo);
    p.y[((int64_t)n * p.Cout + co) * HWo + r] = apply_act(v, act, p.slope);
  }
  if (p.stats) {
    __shared__ double red[2][4];
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    if ((threadIdx.x & 63) == 0) {
      red[0][threadIdx.x >> 6] = a;
      red[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      p.stats[((int64_t)blockIdx.x * 2 + 0) * p.Cout + co] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      p.stats[((int64_t)blockIdx.x * 2 + 1) * p.Cout + co] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
  }
}

// Split-K epilogue over 64-pixel x 64-channel tiles (the default; the
// per-channel kernel above under AINP_SPLITK_TILE=0): 16 lanes per channel
// row each own four consecutive pixels, so the nsplit partial rows arrive as
// 16-byte loads issued together (the per-pixel kernel's serial loads were
// latency bound), and the same per-pixel sums in the same z order -- y is
// bit-identical.  The BatchNorm partials are per (64-pixel block, channel);
// Y16: the bf16 channel-last copy of act(y) from an LDS transpose of the tile,
// replacing the nchw_to_nhwc16 pass after the split layers.
constexpr int SKT_P = 64, SKT_C = 64;
template <bool Y16>
__global__ __launch_bounds__(256) void conv_gen_splitk_tile_epilogue(ConvGenParams p, int nsplit,
                                                                     int act) {
  __shared__ uint16_t tile[Y16 ? SKT_P : 1][SKT_C + 2];
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * SKT_P;
  const int co0 = blockIdx.y * SKT_C;
  const int pl = threadIdx.x & 15, rr = threadIdx.x >> 4;
  const int64_t px = px0 + 4 * pl;
  const bool vec = (NP & 3) == 0 && px + 3 < NP;
  const float sc = p.scale ? *p.scale : 1.f;
  float rat[4] = {1.f, 1.f, 1.f, 1.f};
  if (p.ratio)
#pragma unroll
    for (int e = 0; e < 4; ++e) rat[e] = px + e < NP ? p.ratio[px + e] : 1.f;
  int nn[4], rq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    nn[e] = (int)((px + e) / HWo);
    rq[e] = (int)(px + e - (int64_t)nn[e] * HWo);
  }
#pragma unroll 1
  for (int j = 0; j < SKT_C / 16; ++j) {
    const int cl = rr + 16 * j, co = co0 + cl;
    double a = 0.0, b = 0.0;
    if (co < p.Cout && px < NP) {
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      const float* src = p.partial + (int64_t)co * NP + px;
      const int64_t zs = (int64_t)p.Cout * NP;
      if (vec) {
        int z = 0;
        for (; z + 4 <= nsplit; z += 4) {
          float4 q[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) q[u] = *reinterpret_cast<const float4*>(src + (z + u) * zs);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v[0] += q[u].x;
            v[1] += q[u].y;
            v[2] += q[u].z;
            v[3] += q[u].w;
          }
        }
        for (; z < nsplit; ++z) {
          const float4 q = *reinterpret_cast<const float4*>(src + z * zs);
          v[0] += q.x;
          v[1] += q.y;
          v[2] += q.z;
          v[3] += q.w;
        }
      } else {
        for (int z = 0; z < nsplit; ++z)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (px + e < NP) v[e] += src[z * zs + e];
      }
      const float bias = p.bias ? p.bias[co] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (px + e >= NP) continue;
        float t = v[e] * sc;
        if (p.ratio) t *= rat[e];
        if (p.bias) t += bias;
        a += t;
        b += (double)t * (double)t;
        const float o = apply_act(t, act, p.slope);
        p.y[((int64_t)nn[e] * p.Cout + co) * HWo + rq[e]] = o;
        if (Y16) tile[4 * pl + e][cl] = __builtin_bit_cast(uint16_t, (__bf16)o);
      }
    }
    if (p.stats) {
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        a += __shfl_xor(a, m, 16);
        b += __shfl_xor(b, m, 16);
      }
      if (pl == 0 && co < p.Cout) {
        p.stats[((int64_t)blockIdx.x * 2 + 0) * p.Cout + co] = a;
        p.stats[((int64_t)blockIdx.x * 2 + 1) * p.Cout + co] = b;
      }
    }
  }
  if (!Y16) return;
  __syncthreads();
  // rows = pixels, lanes along the channels (bf16 pairs): 32 lanes per pixel
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
  const int c = co0 + 2 * l;
#pragma unroll
  for (int i = r; i < SKT_P; i += 8) {
    const int64_t q = px0 + i;
    if (q >= NP || c >= p.Cout) continue;
    uint16_t* d = p.y16 + q * p.Cout + c;
    if (c + 1 < p.Cout && (p.Cout & 1) == 0)
      *reinterpret_cast<uint32_t*>(d) = (uint32_t)tile[i][2 * l] | ((uint32_t)tile[i][2 * l + 1] << 16);
    else {
      d[0] = tile[i][2 * l];
      if (c + 1 < p.Cout) d[1] = tile[i][2 * l + 1];
    }
  }
}

static bool splitk_tile() {
  static const bool on = [] {
    const char* e = getenv("AINP_SPLITK_TILE");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int splitk_epilogue_launch(const ConvGenParams& p, int64_t NP, int nsplit, int act,
                                  hipStream_t s) {
  if (!splitk_tile()) {
    hipLaunchKernelGGL(conv_gen_splitk_epilogue, dim3((unsigned)cdiv(NP, 256), p.Cout), dim3(256),
                       0, s, p, nsplit, act);
  } else if (p.y16) {
    hipLaunchKernelGGL(conv_gen_splitk_tile_epilogue<true>,
                       dim3((unsigned)cdiv(NP, SKT_P), (unsigned)cdiv(p.Cout, SKT_C)), dim3(256), 0,
                       s, p, nsplit, act);
  } else {
    hipLaunchKernelGGL(conv_gen_splitk_tile_epilogue<false>,
                       dim3((unsigned)cdiv(NP, SKT_P), (unsigned)cdiv(p.Cout, SKT_C)), dim3(256), 0,
                       s, p, nsplit, act);
  }
  return check_launch("conv_gen_splitk_epilogue");
}

// Direct convolution for Cout == 1 (the generator's last PartialConv2d and
// the discriminator's logit conv).  Stage 1: grid (pixel blocks, channel
// chunks of C1_CC) -- each thread sums its pixel over one chunk of the
// concatenated input channels x taps (weights of the chunk in LDS); stage 2
// adds the chunk partials in fixed order, applies 1/sigma, the partial-conv
// ratio, bias and activation, and writes the (optionally cropped, networks.py:334)
// output.
constexpr int C1_CC = 32;

__global__ __launch_bounds__(256) void conv_cout1_partial_kernel(ConvGenParams p, int Hc, int Wc,
                                                                 float* partial) {
  __shared__ float sw[C1_CC * 64];
  const int KK = p.KH * p.KW;
  const int c0 = blockIdx.y * C1_CC;
  const int cn = min(C1_CC, p.Cin - c0);
  for (int i = threadIdx.x; i < cn * KK; i += blockDim.x) sw[i] = p.w[(int64_t)c0 * KK + i];
  __syncthreads();
  const int64_t np = (int64_t)p.N * Hc * Wc;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  const int n = (int)(t / ((int64_t)Hc * Wc));
  const int r = (int)(t - (int64_t)n * Hc * Wc);
  const int oy = r / Wc, ox = r - oy * Wc;
  const int by = oy * p.stride - p.pad, bx = ox * p.stride - p.pad;
  float acc = 0.f;
  for (int src = 0; src < 2; ++src) {
    const ConvSrcDev& s = src == 0 ? p.s0 : p.s1;
    const int sc0 = src == 0 ? 0 : p.s0.C;          // first concat channel of this source
    const int lo = max(c0, sc0), hi = min(c0 + cn, sc0 + s.C);
    if (lo >= hi) continue;
    const int64_t plane = (int64_t)s.Hs * s.Ws;
    for (int ky = 0; ky < p.KH; ++ky) {
      const int iy = by + ky;
      if (iy < 0 || iy >= p.Hin) continue;
      const int sy = src_coord(iy, s.Hs, p.Hin, s.up);
      for (int kx = 0; kx < p.KW; ++kx) {
        const int ix = bx + kx;
        if (ix < 0 || ix >= p.Win) continue;
        const int sx = src_coord(ix, s.Ws, p.Win, s.up);
        const int64_t off = (int64_t)sy * s.Ws + sx;
        const float mv = s.m ? s.m[(int64_t)n * plane + off] : 1.f;
        const float* xb = s.x + ((int64_t)n * s.C + (lo - sc0)) * plane + off;
        const float* wb = sw + (lo - c0) * KK + ky * p.KW + kx;
        float a = 0.f;
        if (hi - lo == C1_CC) {   // a full chunk: 32 loads in flight, 4 partial chains
          float a4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < C1_CC; ++c)
            a4[c & 3] = fmaf(wb[c * KK], xb[(int64_t)c * plane], a4[c & 3]);
          a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        } else {
          for (int c = 0; c < hi - lo; ++c) a = fmaf(wb[c * KK], xb[(int64_t)c * plane], a);
        }
        acc = fmaf(a, mv, acc);
      }
    }
  }
  partial[(int64_t)blockIdx.y * np + t] = acc;
}

// Round 6: the same stage 1 for one plain source (no concatenation, no
// upsampling; the generator's last PartialConv2d, 64 -> 1, 3 x 3, and the
// discriminator's logit conv, 512 -> 1, 4 x 4) with every tap's loads of CG
// channels in flight together: the loop above waits out one load round trip
// per tap (9 / 16 per chunk; C4: 311 us for the generator's 1.29 M pixels).
// Each tap keeps its four channel chains (c & 3, c ascending) and the taps are
// folded in (ky, kx) order with the same fmaf(a, mask, acc), so the partials
// are bit-identical to conv_cout1_partial_kernel's.  Taps outside the input
// load a clamped in-image element and are not folded in.
template <int KT, int CG>
__global__ __launch_bounds__(256) void conv_cout1_partial_b_kernel(ConvGenParams p, int Hc, int Wc,
                                                                  float* partial) {
  constexpr int KK = KT * KT;
  __shared__ float sw[C1_CC * KK];
  const int c0 = blockIdx.y * C1_CC;
  for (int i = threadIdx.x; i < C1_CC * KK; i += blockDim.x) sw[i] = p.w[(int64_t)c0 * KK + i];
  __syncthreads();
  const int64_t np = (int64_t)p.N * Hc * Wc;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  const int n = (int)(t / ((int64_t)Hc * Wc));
  const int r = (int)(t - (int64_t)n * Hc * Wc);
  const int oy = r / Wc, ox = r - oy * Wc;
  const int by = oy * p.stride - p.pad, bx = ox * p.stride - p.pad;
  const ConvSrcDev& s = p.s0;
  const int64_t plane = (int64_t)s.Hs * s.Ws;
  int off[KK];
  bool ok[KK];
#pragma unroll
  for (int ky = 0; ky < KT; ++ky)
#pragma unroll
    for (int kx = 0; kx < KT; ++kx) {
      const int iy = by + ky, ix = bx + kx;
      const bool v = iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      ok[ky * KT + kx] = v;
      off[ky * KT + kx] = v ? iy * s.Ws + ix : 0;
    }
  // one buffer resource over the source, 32-bit byte offsets (the launcher
  // checks the tensor is < 2 GB): the pixel's tap offsets per lane, the
  // channel step as a wave-uniform scalar offset
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(s.x), (short)0, 0x7fffffff, 0x00020000);
  const int pb = (int)(((int64_t)n * s.C + c0) * plane * 4);
  int vo[KK];
#pragma unroll
  for (int k = 0; k < KK; ++k) vo[k] = pb + off[k] * 4;
  int cstep = (int)(plane * 4);
  asm volatile("" : "+s"(cstep));
  float a4[KK][4];
#pragma unroll
  for (int k = 0; k < KK; ++k) a4[k][0] = a4[k][1] = a4[k][2] = a4[k][3] = 0.f;
#pragma unroll 1
  for (int cg = 0; cg < C1_CC; cg += CG) {
    float v[CG][KK];
#pragma unroll
    for (int c = 0; c < CG; ++c)
#pragma unroll
      for (int k = 0; k < KK; ++k)
        v[c][k] = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rx, vo[k], (cg + c) * cstep, 0));
#pragma unroll
    for (int c = 0; c < CG; ++c)
#pragma unroll
      for (int k = 0; k < KK; ++k) {
        // CG % 4 == 0, so channel cg + c's chain is c & 3 (compile-time)
        a4[k][c & 3] = fmaf(sw[(cg + c) * KK + k], v[c][k], a4[k][c & 3]);
      }
  }
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < KK; ++k) {
    if (!ok[k]) continue;
    const float a = (a4[k][0] + a4[k][1]) + (a4[k][2] + a4[k][3]);
    const float mv = s.m ? s.m[(int64_t)n * plane + off[k]] : 1.f;
    acc = fmaf(a, mv, acc);
  }
  partial[(int64_t)blockIdx.y * np + t] = acc;
}

__global__ void conv_cout1_finish_kernel(ConvGenParams p, int act, int Hc, int Wc, int nchunk,
                                         const float* partial) {
  const int64_t np = (int64_t)p.N * Hc * Wc;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  float acc = 0.f;
  for (int c = 0; c < nchunk; ++c) acc += partial[(int64_t)c * np + t];
  const int n = (int)(t / ((int64_t)Hc * Wc));
  const int r = (int)(t - (int64_t)n * Hc * Wc);
  const int oy = r / Wc, ox = r - oy * Wc;
  float v = acc * (p.scale ? *p.scale : 1.f);
  if (p.ratio) v *= p.ratio[((int64_t)n * p.Ho + oy) * p.Wo + ox];
  if (p.bias) v += p.bias[0];
  p.y[t] = apply_act(v, act, p.slope);
}

// Partial-conv mask update (networks.py:83-104): count = sum over the window
// of the channel-repeated masks = C0 * win(m0) + C1 * win(m1) (exact integers
// in fp32), ratio = (Cin*k*k) / (count + 1e-8), new mask = clamp(count, 0, 1).
// KT > 0: a KT x KT window, unrolled, with every tap's load issued
// unconditionally from a clamped in-image position (zero weight outside), so a
// thread's window loads are in flight together (the runtime-bounds loop waited
// out one load latency per tap: 30-34 us for the generator's two largest).
template <int KT>
__global__ __launch_bounds__(256) void pconv_mask_kernel(ConvSrcDev s0, ConvSrcDev s1, int N,
                                                         int Hin, int Win, int KH, int KW,
                                                         int stride, int pad, int Ho, int Wo,
                                                         float winsize, float* ratio,
                                                         float* newmask) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t np = (int64_t)N * Ho * Wo;
  if (t >= np) return;
  const int n = (int)(t / ((int64_t)Ho * Wo));
  const int r = (int)(t - (int64_t)n * Ho * Wo);
  const int oy = r / Wo, ox = r - oy * Wo;
  int c0 = 0, c1 = 0;
  if (KT > 0) {
    const float* m0 = s0.m + (int64_t)n * s0.Hs * s0.Ws;
    const float* m1 = s1.C ? s1.m + (int64_t)n * s1.Hs * s1.Ws : m0;
#pragma unroll
    for (int ky = 0; ky < KT; ++ky) {
      const int iy = oy * stride - pad + ky;
      const bool oky = iy >= 0 && iy < Hin;
      const int cy = min(max(iy, 0), Hin - 1);
      const int sy0 = src_coord(cy, s0.Hs, Hin, s0.up), sy1 = src_coord(cy, s1.Hs, Hin, s1.up);
#pragma unroll
      for (int kx = 0; kx < KT; ++kx) {
        const int ix = ox * stride - pad + kx;
        const bool ok = oky && ix >= 0 && ix < Win;
        const int cx = min(max(ix, 0), Win - 1);
        const float v0 = m0[sy0 * s0.Ws + src_coord(cx, s0.Ws, Win, s0.up)];
        c0 += ok ? (int)v0 : 0;
        if (s1.C) {
          const float v1 = m1[sy1 * s1.Ws + src_coord(cx, s1.Ws, Win, s1.up)];
          c1 += ok ? (int)v1 : 0;
        }
      }
    }
  } else {
    for (int ky = 0; ky < KH; ++ky) {
      const int iy = oy * stride - pad + ky;
      if (iy < 0 || iy >= Hin) continue;
      for (int kx = 0; kx < KW; ++kx) {
        const int ix = ox * stride - pad + kx;
        if (ix < 0 || ix >= Win) continue;
        if (s0.C) {
          const int sy = src_coord(iy, s0.Hs, Hin, s0.up), sx = src_coord(ix, s0.Ws, Win, s0.up);
          c0 += (int)s0.m[((int64_t)n * s0.Hs + sy) * s0.Ws + sx];
        }
        if (s1.C) {
          const int sy = src_coord(iy, s1.Hs, Hin, s1.up), sx = src_coord(ix, s1.Ws, Win, s1.up);
          c1 += (int)s1.m[((int64_t)n * s1.Hs + sy) * s1.Ws + sx];
        }
      }
    }
  }
  const float cnt = (float)(s0.C * c0 + s1.C * c1);
  if (ratio) ratio[t] = winsize / (cnt + 1e-8f);
  if (newmask) newmask[t] = fminf(fmaxf(cnt, 0.f), 1.f);
}

// PConvUNet input padding (networks.py:255-261): features reflect-padded,
// mask constant-1 padded, bottom / right only.
__global__ void gan_pad_input_kernel(const float* x, const float* m, int N, int H, int W,
                                     int Hp, int Wp, float* xp, float* mp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * Hp * Wp) return;
  const int n = (int)(t / ((int64_t)Hp * Wp));
  const int r = (int)(t - (int64_t)n * Hp * Wp);
  const int y = r / Wp, xx = r - y * Wp;
  const int ry = y < H ? y : 2 * (H - 1) - y;
  const int rx = xx < W ? xx : 2 * (W - 1) - xx;
  xp[t] = x[((int64_t)n * H + ry) * W + rx];
  mp[t] = (y < H && xx < W) ? m[((int64_t)n * H + y) * W + xx] : 1.f;
}

// y = act(y * scale[c] + shift[c]) in place (BatchNorm2d train/eval + activation).
__global__ void affine_act_kernel(float* y, const float* scale, const float* shift, int C,
                                  int64_t HW, int64_t total, int act, float slope) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c = (int)((t / HW) % C);
  y[t] = apply_act(fmaf(y[t], scale[c], shift[c]), act, slope);
}

__global__ void maxpool2_kernel(const float* x, float* y, int64_t NC, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= NC * Ho * Wo) return;
  const int64_t nc = t / ((int64_t)Ho * Wo);
  const int r = (int)(t - nc * Ho * Wo);
  const int oy = r / Wo, ox = r - oy * Wo;
  const float* b = x + nc * H * W + (int64_t)(2 * oy) * W + 2 * ox;
  y[t] = fmaxf(fmaxf(b[0], b[1]), fmaxf(b[W], b[W + 1]));
}

// maxpool2_kernel's values plus, in the same pass, their channel-last bf16
// copy out [N][Ho][Wo][C] (nchw_to_nhwc16_kernel's conversion and write-out):
// the VGG19 conv after each max-pool (loss.py:41-51) reads that copy, so no
// separate nchw_to_nhwc16 pass re-reads the pooled plane.  Block (64 output
// columns, output row, image x 64-channel chunk).
__global__ __launch_bounds__(256) void maxpool2_nhwc16_kernel(const float* __restrict__ x,
                                                              float* __restrict__ y, int C,
                                                              int H, int W,
                                                              uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][66];   // [w][c]
  const int Ho = H / 2, Wo = W / 2;
  const int w0 = blockIdx.x * 64, h = blockIdx.y;
  const int cb = (C + 63) / 64;
  const int n = blockIdx.z / cb, c0 = (blockIdx.z % cb) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int w = w0 + tx;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i;
    float v = 0.f;
    if (c < C && w < Wo) {
      const int64_t nc = (int64_t)n * C + c;
      const float* b = x + nc * H * W + (int64_t)(2 * h) * W + 2 * w;
      v = fmaxf(fmaxf(b[0], b[1]), fmaxf(b[W], b[W + 1]));
      y[(nc * Ho + h) * Wo + w] = v;
    }
    tile[tx][i] = __builtin_bit_cast(uint16_t, (__bf16)v);
  }
  __syncthreads();
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
#pragma unroll
  for (int i = r; i < 64; i += 8) {
    const int ww = w0 + i, c = c0 + 2 * l;
    if (ww >= Wo || c >= C) continue;
    uint16_t* q = out + (((int64_t)n * Ho + h) * Wo + ww) * C + c;
    if (c + 1 < C && !(C & 1)) {
      *reinterpret_cast<uint32_t*>(q) = (uint32_t)tile[i][2 * l] | ((uint32_t)tile[i][2 * l + 1] << 16);
    } else {   // odd C: 2-byte stores keep every access aligned
      q[0] = tile[i][2 * l];
      if (c + 1 < C) q[1] = tile[i][2 * l + 1];
    }
  }
}

// ---------------------------------------------------------------- VGG input
// max(clamp(x, 0)) over the whole batch (loss.py:77-78).  Values are >= 0,
// so the float ordering equals the uint ordering of their bit patterns.
__global__ void clamp_max_kernel(const float* x, int64_t n, unsigned int* out) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, x[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// loss.py:74-86 scaling + ImageClassification: antialiased bilinear resize
// (separable weights precomputed by the host for the cropped rows/cols),
// centre crop, ImageNet normalisation; out [N, 3, 224, 224].
__global__ void vgg_prep_kernel(const float* x, int N, int H, int W, int generated,
                                const unsigned int* maxbits, const int* ry0, const int* rn,
                                const float* rw, int rtaps, const int* cx0, const int* cn,
                                const float* cw, int ctaps, int S, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * S * S) return;
  const int n = (int)(t / ((int64_t)S * S));
  const int r = (int)(t - (int64_t)n * S * S);
  const int oy = r / S, ox = r - oy * S;
  float div = 1.f;
  bool use_div = false;
  if (!generated) {
    const double mx = (double)__uint_as_float(*maxbits) + 1e-6;
    use_div = mx > 1e-5;
    div = (float)mx;
  }
  const float* xb = x + (int64_t)n * H * W;
  float acc = 0.f;
  for (int a = 0; a < rn[oy]; ++a) {
    const int yy = ry0[oy] + a;
    float row = 0.f;
    for (int b = 0; b < cn[ox]; ++b) {
      float v = xb[(int64_t)yy * W + cx0[ox] + b];
      if (generated) {
        v = (v + 1.0f) / 2.0f;
      } else {
        v = fmaxf(v, 0.f);
        if (use_div) v = v / div;
      }
      v = fminf(fmaxf(v, 0.f), 1.f);
      row = fmaf(cw[ox * ctaps + b], v, row);
    }
    acc = fmaf(rw[oy * rtaps + a], row, acc);
  }
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  for (int c = 0; c < 3; ++c)
    out[(((int64_t)n * 3 + c) * S + oy) * S + ox] = (acc - mean[c]) / stdv[c];
}

// ------------------------------------------------------------ reductions
// out[0] += sum |a-b| (fixed-order block partials -> one atomic per block is
// not deterministic; use two stages: partial[block] then a single block).
__global__ void absdiff_partial_kernel(const float* a, const float* b, int64_t n,
                                       double* partial) {
  double s = 0.0;
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0) {
    // 16-byte loads, four of each operand in flight per thread (the one-float
    // grid-stride loop waited out a load latency per element)
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const float4* b4 = reinterpret_cast<const float4*>(b);
    const int64_t n4 = n >> 2;
    int64_t i = t0;
    for (; i + 3 * T < n4; i += 4 * T) {
      float4 x[4], y[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x[u] = a4[i + u * T];
        y[u] = b4[i + u * T];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += (double)fabsf(x[u].x - y[u].x);
        s += (double)fabsf(x[u].y - y[u].y);
        s += (double)fabsf(x[u].z - y[u].z);
        s += (double)fabsf(x[u].w - y[u].w);
      }
    }
    for (; i < n4; i += T) {
      const float4 x = a4[i], y = b4[i];
      s += (double)fabsf(x.x - y.x);
      s += (double)fabsf(x.y - y.y);
      s += (double)fabsf(x.z - y.z);
      s += (double)fabsf(x.w - y.w);
    }
    if (t0 < n - 4 * n4) s += (double)fabsf(a[4 * n4 + t0] - b[4 * n4 + t0]);
  } else {
    for (int64_t i = t0; i < n; i += T) s += (double)fabsf(a[i] - b[i]);
  }
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void sum_partials_kernel(const double* partial, int np, double scale, double* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += partial[i];
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1] + red[2] + red[3]) * scale;
}

// BCEWithLogits (torch's stable form) against a constant target y, mean over
// n, optional gradient g = gscale * (sigmoid(x) - y).
__global__ void bce_logits_partial_kernel(const float* x, int64_t n, float y, double* partial,
                                          float* grad, float gscale) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    const float mx = fmaxf(-v, 0.f);
    const float l = (1.f - y) * v + mx + logf(expf(-mx) + expf(-v - mx));
    s += (double)l;
    if (grad) grad[i] = gscale * (1.f / (1.f + expf(-v)) - y);
  }
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// calculate_losses' reconstruction terms (train.py:49-63) in one pass:
// partial[block][0..4] = sum|g*m - o*m|, sum m, sum|g*h - o*h|, sum h,
// sum |g - o| * |o|   (h = 1 - m)
__global__ void gan_recon_partial_kernel(const float* g, const float* o, const float* m,
                                         int64_t n, double* partial) {
  double s[5] = {0, 0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gv = g[i], ov = o[i], mv = m[i], hv = 1.f - mv;
    s[0] += (double)fabsf(gv * mv - ov * mv);
    s[1] += (double)mv;
    s[2] += (double)fabsf(gv * hv - ov * hv);
    s[3] += (double)hv;
    s[4] += (double)(fabsf(gv - ov) * fabsf(ov));
  }
  __shared__ double red[5][4];
  for (int q = 0; q < 5; ++q) {
    const double v = wave_sum_d(s[q]);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 5)
    partial[(int64_t)blockIdx.x * 5 + threadIdx.x] =
        red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
}

// The 5 sums over the block partials in a fixed order: thread t adds partials
// t, t+256, ... (one load in flight per iteration of 256 threads, not one
// thread walking all np rows), then a fixed wave / cross-wave tree.
__device__ __forceinline__ void recon_reduce5(const double* partial, int np, double (&tot)[5]) {
  double s[5] = {0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < np; b += blockDim.x)
#pragma unroll
    for (int q = 0; q < 5; ++q) s[q] += partial[(int64_t)b * 5 + q];
  __shared__ double red[5][4];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const double v = wave_sum_d(s[q]);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 5; ++q) tot[q] = red[q][0] + red[q][1] + red[q][2] + red[q][3];
}

__global__ __launch_bounds__(256) void gan_recon_final_kernel(const double* partial, int np,
                                                              int64_t n, double* out3) {
  double tot[5];
  recon_reduce5(partial, np, tot);
  if (threadIdx.x == 0) {
    // torch: fp32 sums / (fp32 sum + 1e-8); the fp64 sums are rounded once
    const float nv = (float)tot[1] + 1e-8f, nh = (float)tot[3] + 1e-8f;
    out3[0] = (double)((float)tot[0] / nv);
    out3[1] = (double)((float)tot[2] / nh);
    out3[2] = (double)((float)(tot[4] / (double)n));
  }
}

// -------------------------------------------------------------- spectral norm
// torch.nn.utils.spectral_norm, n_power_iterations = 1 (per train forward):
//   v = normalize(W^T u), t = W v, u = normalize(t), sigma = u . t
struct SnLayers {
  const float* w[8];
  float* u[8];
  float* v[8];
  int h[8], wd[8];
  int nl;
};

// tv[l][j] = sum_i W[i][j] u[i]    (grid: x = blocks of 64 columns, y = layer)
// Each wave of the 256-thread block takes the rows i = q mod 4 of 64
// coalesced columns with four independent FMA chains; the four waves' sums
// are added in fixed order through LDS.
constexpr int SN_TMV_COLS = 64;
__global__ __launch_bounds__(256) void sn_tmv_kernel(SnLayers L, float* tv, int ldt) {
  __shared__ float red[4][SN_TMV_COLS];
  const int l = blockIdx.y;
  if (l >= L.nl) return;                      // uniform over the block
  const int jl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int j = blockIdx.x * SN_TMV_COLS + jl;
  const int wd = L.wd[l], h = L.h[l];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < wd) {
    const float* W = L.w[l] + j;
    const float* u = L.u[l];
    int i = q;
    for (; i + 12 < h; i += 16) {
      s0 = fmaf(W[(int64_t)i * wd], u[i], s0);
      s1 = fmaf(W[(int64_t)(i + 4) * wd], u[i + 4], s1);
      s2 = fmaf(W[(int64_t)(i + 8) * wd], u[i + 8], s2);
      s3 = fmaf(W[(int64_t)(i + 12) * wd], u[i + 12], s3);
    }
    for (; i < h; i += 4) s0 = fmaf(W[(int64_t)i * wd], u[i], s0);
  }
  red[q][jl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q == 0 && j < wd) tv[(int64_t)l * ldt + j] = (red[0][jl] + red[1][jl]) + (red[2][jl] + red[3][jl]);
}

__device__ float block_sum_f(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) s += red[i];
  __syncthreads();
  return s;
}

// v[l] = tv[l] / max(||tv[l]||, eps)     (one block per layer)
__global__ void sn_normalize_v_kernel(SnLayers L, const float* tv, int ldt, float eps) {
  __shared__ float red[16];
  const int l = blockIdx.x;
  const int n = L.wd[l];
  const float* t = tv + (int64_t)l * ldt;
  float s = 0.f;
  for (int j = threadIdx.x; j < n; j += blockDim.x) s += t[j] * t[j];
  const float nrm = sqrtf(block_sum_f(s, red));
  const float d = fmaxf(nrm, eps);
  for (int j = threadIdx.x; j < n; j += blockDim.x) L.v[l][j] = t[j] / d;
}

// tu[l][i] = sum_j W[i][j] v[j]     (one block per (row, layer))
__global__ void sn_mv_kernel(SnLayers L, float* tu, int ldt) {
  __shared__ float red[16];
  const int l = blockIdx.y, i = blockIdx.x;
  if (l >= L.nl || i >= L.h[l]) return;
  const float* W = L.w[l] + (int64_t)i * L.wd[l];
  const float* v = L.v[l];
  float s = 0.f;
  for (int j = threadIdx.x; j < L.wd[l]; j += blockDim.x) s = fmaf(W[j], v[j], s);
  s = block_sum_f(s, red);
  if (threadIdx.x == 0) tu[(int64_t)l * ldt + i] = s;
}

// u = tu / max(||tu||, eps); sigma = u . tu; inv_sigma[l] = 1 / sigma
__global__ void sn_finish_kernel(SnLayers L, const float* tu, int ldt, float eps,
                                 float* inv_sigma) {
  __shared__ float red[16];
  const int l = blockIdx.x;
  const int n = L.h[l];
  const float* t = tu + (int64_t)l * ldt;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += t[i] * t[i];
  const float nrm = sqrtf(block_sum_f(s, red));
  const float d = fmaxf(nrm, eps);
  float dotp = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float uu = t[i] / d;
    L.u[l][i] = uu;
    dotp = fmaf(uu, t[i], dotp);
  }
  const float sigma = block_sum_f(dotp, red);
  if (threadIdx.x == 0) inv_sigma[l] = 1.f / sigma;
}

// eval mode (no power iteration): sigma = u . (W v) with the stored u, v
__global__ void sn_sigma_kernel(SnLayers L, const float* tu, int ldt, float* inv_sigma) {
  __shared__ float red[16];
  const int l = blockIdx.x;
  const float* t = tu + (int64_t)l * ldt;
  float dotp = 0.f;
  for (int i = threadIdx.x; i < L.h[l]; i += blockDim.x) dotp = fmaf(L.u[l][i], t[i], dotp);
  const float sigma = block_sum_f(dotp, red);
  if (threadIdx.x == 0) inv_sigma[l] = 1.f / sigma;
}

// dW_orig = G * inv_sigma - (sum G*W_orig) * inv_sigma^2 * u v^T
// stage 1: partial[block] = sum G*W  (fixed order), stage 2: apply.
__global__ void sn_gdot_partial_kernel(const float* G, int ldg, const float* W, int wd, int64_t n,
                                       double* partial) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / wd, c = i - r * wd;
    s += (double)G[r * ldg + c] * (double)W[i];
  }
  __shared__ double red[4];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void sn_wgrad_apply_kernel(const float* G, int ldg, const double* partial, int np,
                                      const float* u, const float* v, const float* inv_sigma,
                                      int h, int wd, float* out, float* out_bias) {
  __shared__ float gw;
  if (threadIdx.x < 64) {   // wave 0: strided lane sums + butterfly, same order in every block
    double s = 0.0;
    for (int b = threadIdx.x; b < np; b += 64) s += partial[b];
    s = wave_sum_d(s);
    if (threadIdx.x == 0) gw = (float)s;
  }
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)h * wd) return;
  const int i = (int)(t / wd), j = (int)(t - (int64_t)i * wd);
  const float is = *inv_sigma;
  out[t] = G[(int64_t)i * ldg + j] * is - gw * is * is * u[i] * v[j];
  if (out_bias && j == 0) out_bias[i] = G[(int64_t)i * ldg + wd];
}

// ------------------------------------------------------------ D backward glue
// col[n][ci*KK + tap][oy*Wo + ox] = x[n][ci][oy*s-p+ky][ox*s-p+kx] (0 outside)
// ones_row: an extra row k = C*KK of 1.0 (the bias column of the weight-grad GEMM)
// col[n][k][p], p < ldp (row stride; p >= Ho*Wo is zero padding so a GEMM can
// use 16-byte loads), k = ci*KH*KW + tap, plus a row of ones when ones_row;
// grid = (pixel blocks, Kr, N): no 64-bit division per element.
__global__ void im2col_kernel(const float* x, int N, int C, int H, int W, int KH, int KW,
                              int stride, int pad, int Ho, int Wo, int ones_row, int ldp,
                              float* col) {
  const int KK = KH * KW;
  const int P = Ho * Wo;
  const int Kr = C * KK + ones_row;
  const int pp = blockIdx.x * blockDim.x + threadIdx.x;
  if (pp >= ldp) return;
  const int k = blockIdx.y, n = blockIdx.z;
  float* dst = col + ((int64_t)n * Kr + k) * ldp + pp;
  if (pp >= P) {
    *dst = 0.f;
    return;
  }
  if (k == C * KK) {
    *dst = 1.f;
    return;
  }
  const int ci = k / KK, tap = k - ci * KK;
  const int ky = tap / KW, kx = tap - ky * KW;
  const int oy = pp / Wo, ox = pp - oy * Wo;
  const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
  *dst = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? x[(((int64_t)n * C + ci) * H + iy) * W + ix]
                                                  : 0.f;
}

// im2col with 4 consecutive pixels x IM2COL_IK consecutive rows k per thread
// and 16-byte stores (ldp % 4 == 0): the row/column split of the first pixel
// is the only division, and 4*IM2COL_IK loads are in flight (clamped
// addresses, masked values).  Same values as im2col_kernel.
constexpr int IM2COL_IK = 4;
__global__ void im2col4_kernel(const float* x, int C, int H, int W, int KH, int KW, int stride,
                               int pad, int Ho, int Wo, int ones_row, int ldp, float* col) {
  const int KK = KH * KW;
  const int P = Ho * Wo;
  const int Kr = C * KK + ones_row;
  const int pp0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (pp0 >= ldp) return;
  const int n = blockIdx.z;
  const int oy0 = pp0 / Wo, ox0 = pp0 - oy0 * Wo;
  float v[IM2COL_IK][4];
#pragma unroll
  for (int j = 0; j < IM2COL_IK; ++j) {
    const int k = blockIdx.y * IM2COL_IK + j;
    if (k >= C * KK) {                       // the ones row, or past the end
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = (k == C * KK && pp0 + e < P) ? 1.f : 0.f;
      continue;
    }
    const int ci = k / KK, tap = k - ci * KK;
    const int ky = tap / KW, kx = tap - ky * KW;
    const float* xp = x + ((int64_t)n * C + ci) * H * W;
    int oy = oy0, ox = ox0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
      const bool ok = pp0 + e < P && iy >= 0 && iy < H && ix >= 0 && ix < W;
      const float t = xp[ok ? iy * W + ix : 0];
      v[j][e] = ok ? t : 0.f;
      if (++ox == Wo) {
        ox = 0;
        ++oy;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < IM2COL_IK; ++j) {
    const int k = blockIdx.y * IM2COL_IK + j;
    if (k < Kr)
      *reinterpret_cast<float4*>(col + ((int64_t)n * Kr + k) * ldp + pp0) =
          make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
  }
}

// col2im for a KSxKS kernel at stride S (the Discriminator's 4x4, stride 2 or
// 1): one (n, ci) plane per blockIdx.y.  At stride 2 only the taps of the
// pixel's parity contribute, so (KS/S)^2 loads, all issued before the sum
// (clamped addresses, masked values); the sum runs in ascending (ky, kx) order
// like col2im_kernel.
template <int KS, int S>
__global__ void col2im_ks_kernel(const float* dcol, int C, int H, int W, int pad, int Ho,
                                 int Wo, int64_t P, float* dx) {
  constexpr int KT = KS / S;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= H * W) return;
  const int nc = blockIdx.y;
  const int iy = r / W, ix = r - iy * W;
  const int by = iy + pad, bx = ix + pad;
  const float* dp = dcol + (int64_t)nc * KS * KS * P;
  float v[KT][KT];
#pragma unroll
  for (int a = 0; a < KT; ++a) {
    const int ky = (S == 2 ? (by & 1) : 0) + S * a;
    const int ty = by - ky;
    const int oy = S == 2 ? ty >> 1 : ty;
    const bool vy = ty >= 0 && oy < Ho;
#pragma unroll
    for (int b = 0; b < KT; ++b) {
      const int kx = (S == 2 ? (bx & 1) : 0) + S * b;
      const int tx = bx - kx;
      const int ox = S == 2 ? tx >> 1 : tx;
      const bool ok = vy && tx >= 0 && ox < Wo;
      const float t = dp[ok ? (int64_t)(ky * KS + kx) * P + oy * Wo + ox : 0];
      v[a][b] = ok ? t : 0.f;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < KT; ++a)
#pragma unroll
    for (int b = 0; b < KT; ++b) s += v[a][b];
  dx[(int64_t)nc * H * W + r] = s;
}

// dx[n][ci][iy][ix] = sum over taps with (iy+p-ky)/s, (ix+p-kx)/s integral and
// in range of dcol[n][ci*KK+tap][oy*Wo+ox]   (gather: deterministic, no atomics)
__global__ void col2im_kernel(const float* dcol, int N, int C, int H, int W, int KH, int KW,
                              int stride, int pad, int Ho, int Wo, int64_t P, float* dx) {
  // P: row stride of dcol (>= Ho*Wo)
  const int KK = KH * KW;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * C * H * W) return;
  const int ix = (int)(t % W);
  const int iy = (int)((t / W) % H);
  const int64_t nc = t / ((int64_t)H * W);
  const int ci = (int)(nc % C);
  const int n = (int)(nc / C);
  float s = 0.f;
  for (int ky = 0; ky < KH; ++ky) {
    const int ty = iy + pad - ky;
    if (ty < 0 || ty % stride) continue;
    const int oy = ty / stride;
    if (oy >= Ho) continue;
    for (int kx = 0; kx < KW; ++kx) {
      const int tx = ix + pad - kx;
      if (tx < 0 || tx % stride) continue;
      const int ox = tx / stride;
      if (ox >= Wo) continue;
      s += dcol[(((int64_t)n * C + ci) * KK + ky * KW + kx) * P + (int64_t)oy * Wo + ox];
    }
  }
  dx[t] = s;
}

// g_pre = g * (y > 0 ? 1 : slope)    (LeakyReLU backward from its output)
__global__ void leaky_bwd_kernel(const float* g, const float* y, int64_t n, float slope,
                                 float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  out[t] = y[t] > 0.f ? g[t] : g[t] * slope;
}

// rows of P elements -> rows of ldo (zero padded), grid = (column blocks, rows)
__global__ void leaky_bwd_ld_kernel(const float* g, const float* y, int P, float slope, int ldo,
                                    float* out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ldo) return;
  const int64_t r = blockIdx.y;
  float v = 0.f;
  if (p < P) {
    const float gv = g[r * P + p];
    v = y[r * P + p] > 0.f ? gv : gv * slope;
  }
  out[r * ldo + p] = v;
}

// standalone PartialConv2d with a per-channel mask: x*m and sum_c m
__global__ void mul_kernel(const float* a, const float* b, int64_t n, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = a[t] * b[t];
}
__global__ void channel_sum_kernel(const float* m, int64_t N, int C, int64_t HW, float* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * HW) return;
  const int64_t n = t / HW, p = t - n * HW;
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += m[(n * C + c) * HW + p];
  out[t] = s;
}


// ------------------------------------------------------- few input channels
// The first layers (G's 7x7 encoder conv on the 1-channel spectrogram, D's
// 4x4 conv on it, VGG's conv1_1 on 3 channels): K = Cin*KH*KW <= 256 and
// Cout <= 64 (K <= 160 here), so the implicit GEMM is all gather and no MFMA work.  Direct
// form: one thread per output pixel holds all Cout accumulators; per k it
// gathers one input value (x * mask) and FMAs it against the k-th weight
// column read from LDS as broadcast float4s; the epilogue writes each
// channel's plane with lane-consecutive pixels.  bf16 (AINP_CONV_BF16): the
// input value and the weights are rounded to bf16 first, so every product is
// the exact bf16 x bf16 product the MFMA would form (fp32 accumulation).
constexpr int SC_K = 160, SC_CO = 64;   // 40 KB of weights in LDS

template <bool B16, bool L16>
__global__ __launch_bounds__(256) void conv_gen_smallcin_kernel(ConvGenParams p, int act) {
  __shared__ __attribute__((aligned(16))) float sw[SC_K][SC_CO];   // [k][co]
  const int KK = p.KH * p.KW, K = KK * p.Cin, Cout = p.Cout;
  for (int i = threadIdx.x; i < K * SC_CO; i += 256) {
    const int k = i / SC_CO, co = i - k * SC_CO;
    float v = 0.f;
    if (co < Cout) {
      // k = tap * Cin + ci (the kmajor order of source 0)
      const int tap = k / p.Cin, ci = k - tap * p.Cin;
      v = p.w[((int64_t)co * p.Cin + ci) * KK + tap];
      if (B16) v = (float)(__bf16)v;
    }
    sw[k][co] = v;
  }
  __syncthreads();
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t pix0 = (int64_t)blockIdx.x * 256;
  const int64_t pix = pix0 + threadIdx.x;
  // y16 (bf16) is written through LDS below, so every thread reaches its barriers
  if (pix >= NP && !(p.y16 && L16)) return;
  const bool valid = pix < NP;
  const int64_t pixc = valid ? pix : NP - 1;
  const int n = (int)(pixc / HWo);
  const int r = (int)(pixc - (int64_t)n * HWo);
  const int oy = r / p.Wo, ox = r - oy * p.Wo;
  const int by = oy * p.stride - p.pad, bx = ox * p.stride - p.pad;
  const ConvSrcDev& s = p.s0;
  const int64_t plane = (int64_t)s.Hs * s.Ws;
  const float* xn = s.x + (int64_t)n * s.C * plane;
  const float* mn = s.m ? s.m + (int64_t)n * plane : nullptr;
  float acc[SC_CO];
#pragma unroll
  for (int c = 0; c < SC_CO; ++c) acc[c] = 0.f;
  int k = 0;
  for (int ky = 0; ky < p.KH; ++ky) {
    const int iy = by + ky;
    for (int kx = 0; kx < p.KW; ++kx) {
      const int ix = bx + kx;
      const bool inb = iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int64_t off = inb ? (int64_t)iy * s.Ws + ix : 0;
      const float mv = (inb && mn) ? mn[off] : 1.f;
      for (int ci = 0; ci < p.Cin; ++ci, ++k) {
        float v = inb ? xn[ci * plane + off] * mv : 0.f;
        if (B16) v = (float)(__bf16)v;
        const float4* wk = reinterpret_cast<const float4*>(sw[k]);
#pragma unroll
        for (int c4 = 0; c4 < SC_CO / 4; ++c4) {
          const float4 w4 = wk[c4];
          acc[4 * c4 + 0] = fmaf(w4.x, v, acc[4 * c4 + 0]);
          acc[4 * c4 + 1] = fmaf(w4.y, v, acc[4 * c4 + 1]);
          acc[4 * c4 + 2] = fmaf(w4.z, v, acc[4 * c4 + 2]);
          acc[4 * c4 + 3] = fmaf(w4.w, v, acc[4 * c4 + 3]);
        }
      }
    }
  }
  const float sc = p.scale ? *p.scale : 1.f;
  const float rt = p.ratio ? p.ratio[pixc] : 1.f;
  float* yb = p.y + (int64_t)n * Cout * HWo + r;
#pragma unroll
  for (int c = 0; c < SC_CO; ++c) {
    if (c < Cout) {
      float v = acc[c] * sc;
      v *= rt;
      if (p.bias) v += p.bias[c];
      acc[c] = apply_act(v, act, p.slope);
      if (valid) yb[(int64_t)c * HWo] = acc[c];
    }
  }
  if (p.y16 && L16) {
    // the block's [256 pixels][Cout] bf16 run staged in the weights' LDS (rows
    // padded by 16 bytes against bank conflicts), then copied out as
    // consecutive 16-byte chunks: fully coalesced stores (each lane's own
    // 128-byte row store touched 8 lines per instruction at 16 bytes each)
    constexpr int RS = SC_CO * 2 + 16;   // bytes per staged pixel row
    static_assert(256 * RS <= (int)sizeof(sw), "y16 staging fits the weight LDS");
    __syncthreads();                     // every wave done with the weights
    unsigned char* st = reinterpret_cast<unsigned char*>(&sw[0][0]);
#pragma unroll
    for (int c = 0; c < SC_CO; c += 8) {
      if (c < Cout) {
        uint32_t h[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          h[j] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[c + 2 * j]) |
                 ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[c + 2 * j + 1]) << 16);
        *reinterpret_cast<uint4*>(st + threadIdx.x * RS + 2 * c) = make_uint4(h[0], h[1], h[2], h[3]);
      }
    }
    __syncthreads();
    const int cpp = Cout / 8;            // 16-byte chunks per pixel
    const int nblk = (int)min<int64_t>(256, NP - pix0);
    uint4* o = reinterpret_cast<uint4*>(p.y16 + pix0 * Cout);
    for (int q = threadIdx.x; q < nblk * cpp; q += 256) {
      const int pl = q / cpp, part = q - pl * cpp;
      o[q] = *reinterpret_cast<const uint4*>(st + pl * RS + 16 * part);
    }
    return;
  }
  // the next conv's channel-last bf16 source (Cout % 8 == 0): this pixel's
  // Cout values as one contiguous run of 16-byte stores
  if (p.y16) {
    uint16_t* o = p.y16 + pix * Cout;
#pragma unroll
    for (int c = 0; c < SC_CO; c += 8) {
      if (c < Cout) {
        uint32_t h[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          h[j] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[c + 2 * j]) |
                 ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)acc[c + 2 * j + 1]) << 16);
        *reinterpret_cast<uint4*>(o + c) = make_uint4(h[0], h[1], h[2], h[3]);
      }
    }
  }
}

// ------------------------------------------------------- bf16 NHWC variant
// The bf16 configurations (C4 / C5) of every conv whose sources have
// channel counts % 32 == 0: the sources are first written channel-last in bf16
// with their partial-conv mask already applied (nchw_to_nhwc16_kernel: the
// masks are channel-uniform per source, so x*m folds in exactly), the weights
// as bf16 [Cout][K] (k = tap*C + ci per source, the fast path's order), so a
// K-tile of 32 channels of ONE tap is, per pixel, 64 contiguous bytes: four
// 16-byte loads per thread per tile instead of 16 scalar gathers and a mask
// load each, at half the bytes.  Same tiles, LDS images (80-byte rows),
// one-plane MFMA loop, split-K and epilogue as conv_gen_x6_kernel<BM, 32, 1>.
// A source with C % 32 != 0 (the U-Net's 1-channel input and mask planes)
// owns KK*C k-values padded up to whole 32-deep tiles (zero weights in the
// pad) and arrives already expanded per output pixel (im2col_nhwc16_kernel:
// [N*Ho*Wo][seg] bf16, mask applied), so its tiles are plain row loads too.
struct Src16 {
  const uint16_t* x;   // [N][Hs][Ws][C] bf16 (mask applied), or [N*Ho*Wo][seg] if exp
  int C, Hs, Ws, up, exp;
};

// k-values one source contributes to the nhwc16 weight rows
__host__ __device__ inline int nhwc16_seg(int C, int KK) {
  return (C & 31) ? (KK * C + 31) / 32 * 32 : KK * C;
}

template <int BM, bool EXP>
__global__ __launch_bounds__(256, 4) void conv_gen_nhwc16_kernel(ConvGenParams p, Src16 s0,
                                                                 Src16 s1,
                                                                 const uint16_t* __restrict__ wt16,
                                                                 int act) {
  constexpr int XBK = 32;
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;
  constexpr int RS = XBK * 2 + 16;
  constexpr int APL = BM * RS, BPL = BN * RS;
  constexpr int ESCR = WN * BM * 2 * (int)sizeof(double);
  __shared__ __attribute__((aligned(16))) unsigned char sA[APL > ESCR ? APL : ESCR];
  __shared__ __attribute__((aligned(16))) unsigned char sB[BPL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = p.KH * p.KW;
  const int K0 = nhwc16_seg(s0.C, KK);
  const int K = K0 + nhwc16_seg(s1.C, KK);
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  const int co0 = blockIdx.y * BM;
  const int nkt_all = K / XBK;
  const int64_t kb = (int64_t)blockIdx.z * p.ktiles_per_split;
  const int64_t ke = kb + p.ktiles_per_split;
  const int kt_begin = (int)(kb < nkt_all ? kb : nkt_all);
  const int kt_end = (int)(ke < nkt_all ? ke : nkt_all);

  // loads: lanes 4r..4r+3 read the four 16-byte chunks of one row's 64-byte
  // K-tile slice (a pixel's 32 channels of one tap, or a weight row), so a
  // wave's load touches 16 rows, not 64; rows r + 64 i, i < BN/64 (BM/64)
  constexpr int NBI = BN / 64, NAI = BM / 64;
  const int ch = tid & 3, rr = tid >> 2;
  // per pixel row: n (-1 past the end) and the packed window origin (by, bx)
  int n_[NBI], byx_[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    const int64_t pix = px0 + rr + 64 * i;
    n_[i] = -1;
    byx_[i] = 0;
    if (pix < NP) {
      n_[i] = (int)(pix / HWo);
      const int r = (int)(pix - (int64_t)n_[i] * HWo);
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      byx_[i] = ((oy * p.stride - p.pad) << 16) | ((ox * p.stride - p.pad) & 0xffff);
    }
  }
  const uint16_t* wrow = wt16 + (int64_t)(co0 + rr) * K + 8 * ch;
  const int arows = p.Cout - co0 - rr;     // row rr + 64 i is valid iff 64 i < arows
  uint4 ra[NAI], rb[NBI];
  auto fetch = [&](int kt) {
    const int k0 = kt * XBK;
#pragma unroll
    for (int i = 0; i < NAI; ++i)
      ra[i] = 64 * i < arows ? *reinterpret_cast<const uint4*>(wrow + (int64_t)64 * i * K + k0)
                             : make_uint4(0, 0, 0, 0);
    const bool first = k0 < K0;
    const Src16& s = first ? s0 : s1;
    const int kr = first ? k0 : k0 - K0;
    if (EXP && s.exp) {   // pre-expanded few-channel source: row pix, k-values kr...
      const int seg = nhwc16_seg(s.C, KK);
#pragma unroll
      for (int i = 0; i < NBI; ++i)
        rb[i] = n_[i] >= 0 ? *reinterpret_cast<const uint4*>(
                                 s.x + (px0 + rr + 64 * i) * seg + kr + 8 * ch)
                           : make_uint4(0, 0, 0, 0);
      return;
    }
    const int tap = kr / s.C, ci0 = kr - tap * s.C;
    const int ky = tap / p.KW, kx = tap - ky * p.KW;
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int iy = (byx_[i] >> 16) + ky, ix = (int)(short)(byx_[i] & 0xffff) + kx;
      const bool inb = n_[i] >= 0 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int sy = inb ? src_coord(iy, s.Hs, p.Hin, s.up) : 0;
      const int sx = inb ? src_coord(ix, s.Ws, p.Win, s.up) : 0;
      const uint16_t* src =
          s.x + (((int64_t)n_[i] * s.Hs + sy) * s.Ws + sx) * s.C + ci0 + 8 * ch;
      rb[i] = inb ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < NAI; ++i)
      *reinterpret_cast<uint4*>(sA + (rr + 64 * i) * RS + 16 * ch) = ra[i];
#pragma unroll
    for (int i = 0; i < NBI; ++i)
      *reinterpret_cast<uint4*>(sB + (rr + 64 * i) * RS + 16 * ch) = rb[i];
  };

  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt_begin < kt_end) fetch(kt_begin);
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    commit();
    __syncthreads();
    if (kt + 1 < kt_end) fetch(kt + 1);
#pragma unroll
    for (int st = 0; st < XBK / 16; ++st) {
      cgx::bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = cgx::frag(sA + (wm * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh);
        b[i] = cgx::frag(sB + (wn * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  conv_gen_epilogue<BM>(p, acc, act, reinterpret_cast<double*>(sA));
}

// LDS-DMA ring variant (opt-in, AINP_CONV16_RING=1; measured slower than the
// kernel above on the C4 bf16 step, 11.66 vs 10.59 ms, profiles/r03_ab1_*): the same tiles, K order, MFMA and epilogue, but the operand rows
// (a weight row's or a pixel's 64-byte K-tile slice) go straight from global
// memory into a 4-stage LDS ring by global_load_lds_dwordx4 -- lane l of a
// wave instruction moves 16 bytes of row 16i + l/4, the chunk XOR-swizzled on
// the source address (g256's image layout: conflict-free ds_read_b128
// fragments) -- with two K-tiles in flight across each barrier (counted
// vmcnt, raw s_barrier): one barrier per K-tile instead of two, and the
// gathers' latency spread over three K-tiles instead of hidden by occupancy
// alone.  Window taps outside the input read a 64-byte zero row.
namespace cgr {
constexpr int NST = 4, ROWB = 64;
__device__ __attribute__((aligned(64))) uint16_t zero_row[32];   // zero-initialised
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
}  // namespace cgr

template <int BM, bool EXP>
__global__ __launch_bounds__(256, 2) void conv_gen_nhwc16_ring_kernel(ConvGenParams p, Src16 s0,
                                                                      Src16 s1,
                                                                      const uint16_t* __restrict__ wt16,
                                                                      int act) {
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;
  constexpr int IMGA = BM * cgr::ROWB, STAGE = (BM + BN) * cgr::ROWB;   // 16 / 20 KB
  constexpr int NA = BM / 64, NB = BN / 64;        // DMA instructions per wave per K-tile
  constexpr int L = NA + NB;
  static_assert(WN * BM * 2 * 8 <= cgr::NST * STAGE, "epilogue scratch fits the ring");
  __shared__ __attribute__((aligned(1024))) unsigned char ring[cgr::NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int KK = p.KH * p.KW;
  const int K0 = nhwc16_seg(s0.C, KK);
  const int K = K0 + nhwc16_seg(s1.C, KK);
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  const int co0 = blockIdx.y * BM;
  const int nkt_all = K / CG_BK;
  const int64_t kb = (int64_t)blockIdx.z * p.ktiles_per_split;
  const int64_t ke = kb + p.ktiles_per_split;
  const int kt_begin = (int)(kb < nkt_all ? kb : nkt_all);
  const int kt_end = (int)(ke < nkt_all ? ke : nkt_all);

  // this lane's rows: A (weights) rows 16 (NA wave + i) + lane/4, B (pixels)
  // rows 16 (NB wave + i) + lane/4; physical chunk lane % 4 holds logical
  // chunk swz(row, lane % 4)
  const int cl = lane & 3;
  const uint16_t* wsrc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = 16 * (NA * wave + i) + (lane >> 2);
    int co = co0 + row;
    co = co < p.Cout ? co : p.Cout - 1;          // rows past Cout: never stored
    wsrc[i] = wt16 + (int64_t)co * K + 8 * cgr::swz(row, cl);
  }
  int n_[NB], byx_[NB], brow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = 16 * (NB * wave + i) + (lane >> 2);
    brow[i] = row;
    const int64_t pix = px0 + row;
    n_[i] = -1;
    byx_[i] = 0;
    if (pix < NP) {
      n_[i] = (int)(pix / HWo);
      const int r = (int)(pix - (int64_t)n_[i] * HWo);
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      byx_[i] = ((oy * p.stride - p.pad) << 16) | ((ox * p.stride - p.pad) & 0xffff);
    }
  }
  const uint16_t* zero = cgr::zero_row + 8 * cl;

  auto issue = [&](int kt) {
    unsigned char* st = ring + (kt & (cgr::NST - 1)) * STAGE;
    const int k0 = kt * CG_BK;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0),
                                       (__attribute__((address_space(3))) void*)(
                                           st + (NA * wave + i) * 1024),
                                       16, 0, 0);
    const bool first = k0 < K0;
    const Src16& s = first ? s0 : s1;
    const int kr = first ? k0 : k0 - K0;
    if (EXP && s.exp) {   // pre-expanded few-channel source: row pix, k-values kr...
      const int seg = nhwc16_seg(s.C, KK);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const uint16_t* src = n_[i] >= 0 ? s.x + (px0 + brow[i]) * seg + kr +
                                               8 * cgr::swz(brow[i], cl)
                                         : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(
                                             st + IMGA + (NB * wave + i) * 1024),
                                         16, 0, 0);
      }
      return;
    }
    const int tap = kr / s.C, ci0 = kr - tap * s.C;
    const int ky = tap / p.KW, kx = tap - ky * p.KW;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int iy = (byx_[i] >> 16) + ky, ix = (int)(short)(byx_[i] & 0xffff) + kx;
      const bool inb = n_[i] >= 0 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int sy = inb ? src_coord(iy, s.Hs, p.Hin, s.up) : 0;
      const int sx = inb ? src_coord(ix, s.Ws, p.Win, s.up) : 0;
      const uint16_t* src = inb ? s.x + (((int64_t)n_[i] * s.Hs + sy) * s.Ws + sx) * s.C + ci0 +
                                      8 * cgr::swz(brow[i], cl)
                                : zero;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(
                                           st + IMGA + (NB * wave + i) * 1024),
                                       16, 0, 0);
    }
  };

  const int wm = wave / WN, wn = wave % WN;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int q = 0; q < cgr::NST - 1; ++q)
    if (kt_begin + q < kt_end) issue(kt_begin + q);
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    // tile kt landed (kt+1, kt+2 may stay in flight); stage of kt-1 free
    const int ahead = kt_end - 1 - kt;
    if (ahead >= 2) __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * L));
    else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | L);
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    const unsigned char* sa = ring + (kt & (cgr::NST - 1)) * STAGE;
    const unsigned char* sb = sa + IMGA;
#pragma unroll
    for (int st = 0; st < CG_BK / 16; ++st) {
      // the next DMA's address arithmetic runs under the first MFMAs
      if (st == 1 && kt + cgr::NST - 1 < kt_end) issue(kt + cgr::NST - 1);
      cgx::bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = wm * 64 + i * 32 + l31, rb = wn * 64 + i * 32 + l31;
        a[i] = cgx::frag(sa + ra * cgr::ROWB + 16 * cgr::swz(ra, 2 * st + lh));
        b[i] = cgx::frag(sb + rb * cgr::ROWB + 16 * cgr::swz(rb, 2 * st + lh));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  __syncthreads();     // every wave done with the ring: the epilogue reuses it
  conv_gen_epilogue<BM>(p, acc, act, reinterpret_cast<double*>(ring));
}

// ------------------------------------------------ bf16 NHWC, wide-tile ring
// conv_gen_nhwc16 on twice the tile area (AINP_CONV16=2 / ainp_conv16_set_variant):
// the kernels above stage 16 KB of operand rows per 1 MFLOP (128 x 128 or
// 64 x 256 tiles, 32-deep K-tiles), so at the layers' re-use they are bound
// by the L2 -> LDS row traffic and the latency of the gathers.  Here:
//  * Cout > 128: 256 (co) x 128 (pixels); Cout 65..128: 128 x 256; both with
//    four waves of 128 x 64 (4 x 2 v_mfma_f32_32x32x16_bf16: 16 MFMAs and 12
//    ds_read_b128 per wave per K-tile), 8 KB of rows per MFLOP;
//  * Cout <= 64: 64 x 256, waves of 64 x 64 (the previous kernels' tile);
//  * rows go global -> LDS by global_load_lds_dwordx4 into a 3-stage ring
//    (two K-tiles in flight across the one raw barrier per K-tile, counted
//    vmcnt; g256's XOR-swizzled 64-byte row image), 60-72 KB: two
//    workgroups (8 waves) per CU;
//  * workgroups are numbered XCD-major (each XCD's L2 owns a contiguous range
//    of pixel tiles) and, within it, co-tile fastest, so the co-tiles that
//    gather the same pixel rows run side by side on one L2.
// Same K order and per-output MFMA chain as conv_gen_nhwc16_kernel (so the
// same sums, bit for bit); the BatchNorm partials keep that kernel's
// per-128/256-pixel slot layout (ainp_conv_gen_stat_parts).
namespace cgw {
constexpr int NST = 3, ROWB = 64;
// NW = 4: waves of 128 x 64 (64 x 64 for BM = 64); NW = 8 (BM >= 128): waves
// of 64 x 64, two workgroups of 8 waves per CU.
template <int BM, int NW>
struct Cfg {
  static constexpr int WM = (NW == 4 && BM >= 128) ? 128 : 64;   // wave tile (co)
  static constexpr int WGM = BM / WM;                            // waves along co
  static constexpr int WGN = NW / WGM;                           // waves along pixels
  static constexpr int WNP = 64;                                 // wave tile (pixels)
  static constexpr int BN = WGN * WNP;                           // tile pixels
  static constexpr int MI = WM / 32, NJ = WNP / 32;
  static constexpr int NA = BM / 16 / NW, NB = BN / 16 / NW;     // 1 KB DMA blocks per wave
  static constexpr int L = NA + NB;
  static constexpr int STAGE = (BM + BN) * ROWB;
  static constexpr int OLD_BN = 16384 / (BM > 64 ? 128 : 64);   // stats slot width
  static_assert(NA * NW * 16 == BM && NB * NW * 16 == BN, "whole DMA blocks per wave");
};
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
}  // namespace cgw

template <int BM, int NW, bool EXP, bool PF = true>
__global__ __launch_bounds__(NW * 64, 2) void conv_gen_nhwc16_wide_kernel(ConvGenParams p, Src16 s0,
                                                                      Src16 s1,
                                                                      const uint16_t* __restrict__ wt16,
                                                                      int act, int tiles_co,
                                                                      int tiles_px) {
  using C = cgw::Cfg<BM, NW>;
  constexpr int BN = C::BN, MI = C::MI, NJ = C::NJ, NA = C::NA, NB = C::NB, L = C::L;
  constexpr int IMGA = BM * cgw::ROWB;
  static_assert(C::WGN * BM * 2 * 8 <= cgw::NST * C::STAGE, "epilogue scratch fits the ring");
  __shared__ __attribute__((aligned(1024))) unsigned char ring[cgw::NST * C::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-major numbering: hardware XCD = blockIdx.x % 8 owns a contiguous range
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int xcd = b0 & 7, slot = b0 >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int co_t = bid % tiles_co, px_t = bid / tiles_co;
  const int KK = p.KH * p.KW;
  const int K0 = nhwc16_seg(s0.C, KK);
  const int K = K0 + nhwc16_seg(s1.C, KK);
  const int HWo = p.Ho * p.Wo;
  const int64_t NP = (int64_t)p.N * HWo;
  const int64_t px0 = (int64_t)px_t * BN;
  const int co0 = co_t * BM;
  const int nkt_all = K / CG_BK;
  const int64_t kb = (int64_t)blockIdx.y * p.ktiles_per_split;
  const int64_t ke = kb + p.ktiles_per_split;
  const int kt_begin = (int)(kb < nkt_all ? kb : nkt_all);
  const int kt_end = (int)(ke < nkt_all ? ke : nkt_all);

  // DMA blocks of this wave: block 4i + wave (16 image rows); i < NA: weight
  // rows, else pixel rows.  Lane: row 16 blk + lane/4, physical chunk lane%4
  // holding logical chunk swz(row, lane%4).
  const int cl = lane & 3;
  const uint16_t* wsrc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = 16 * (NW * i + wave) + (lane >> 2);
    int co = co0 + row;
    co = co < p.Cout ? co : p.Cout - 1;          // rows past Cout: never stored
    wsrc[i] = wt16 + (int64_t)co * K + 8 * cgw::swz(row, cl);
  }
  int n_[NB], byx_[NB], brow[NB], bchunk[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = 16 * (NW * (NA + i) + wave) + (lane >> 2) - BM;   // pixel row in the tile
    brow[i] = row;
    bchunk[i] = 8 * cgw::swz(row + BM, cl);
    const int64_t pix = px0 + row;
    n_[i] = -1;
    byx_[i] = 0;
    if (pix < NP) {
      n_[i] = (int)(pix / HWo);
      const int r = (int)(pix - (int64_t)n_[i] * HWo);
      const int oy = r / p.Wo, ox = r - oy * p.Wo;
      byx_[i] = ((oy * p.stride - p.pad) << 16) | ((ox * p.stride - p.pad) & 0xffff);
    }
  }
  const uint16_t* zero = cgr::zero_row + 8 * cl;

  auto issue = [&](int kt) {
    unsigned char* st = ring + (kt % cgw::NST) * C::STAGE;
    const int k0 = kt * CG_BK;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0),
                                       (__attribute__((address_space(3))) void*)(
                                           st + (NW * i + wave) * 1024),
                                       16, 0, 0);
    const bool first = k0 < K0;
    const Src16& s = first ? s0 : s1;
    const int kr = first ? k0 : k0 - K0;
    if (EXP && s.exp) {   // pre-expanded few-channel source: row pix, k-values kr...
      const int seg = nhwc16_seg(s.C, KK);
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const uint16_t* src = n_[i] >= 0 ? s.x + (px0 + brow[i]) * seg + kr + bchunk[i] : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(
                                             st + (NW * (NA + i) + wave) * 1024),
                                         16, 0, 0);
      }
      return;
    }
    const int tap = kr / s.C, ci0 = kr - tap * s.C;
    const int ky = tap / p.KW, kx = tap - ky * p.KW;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int iy = (byx_[i] >> 16) + ky, ix = (int)(short)(byx_[i] & 0xffff) + kx;
      const bool inb = n_[i] >= 0 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const int sy = inb ? src_coord(iy, s.Hs, p.Hin, s.up) : 0;
      const int sx = inb ? src_coord(ix, s.Ws, p.Win, s.up) : 0;
      const uint16_t* src = inb ? s.x + (((int64_t)n_[i] * s.Hs + sy) * s.Ws + sx) * s.C + ci0 +
                                      bchunk[i]
                                : zero;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(
                                           st + (NW * (NA + i) + wave) * 1024),
                                       16, 0, 0);
    }
  };

  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const int l31 = lane & 31, lh = lane >> 5;
  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int q = 0; q < cgw::NST - 1; ++q)
    if (kt_begin + q < kt_end) issue(kt_begin + q);
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    // tile kt landed (kt+1 may stay in flight); every wave is past tile kt-1,
    // whose stage the DMA of kt+2 reuses
    if (kt + 1 < kt_end) {
      if (L == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (L == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + cgw::NST - 1 < kt_end) issue(kt + cgw::NST - 1);
    const unsigned char* sa = ring + (kt % cgw::NST) * C::STAGE;
    const unsigned char* sb = sa + IMGA;
    // round 6 (PF): both k-steps' fragments read up front, the second
    // k-step's reads overlapping the first one's MFMAs (!PF, AINP_WIDE_PF=0:
    // each k-step's read right before its MFMAs) -- the same MFMAs in the
    // same order either way
    cgx::bf16x8 a[2][MI], b[2][NJ];
#pragma unroll
    for (int st = 0; st < CG_BK / 16; ++st) {
      if (!PF && st > 0) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[st - 1][i], b[st - 1][j],
                                                                acc[i][j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int rb = wn * C::WNP + j * 32 + l31;
        b[st][j] = cgx::frag(sb + rb * cgw::ROWB + 16 * cgw::swz(rb + BM, 2 * st + lh));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int ra = wm * C::WM + i * 32 + l31;
        a[st][i] = cgx::frag(sa + ra * cgw::ROWB + 16 * cgw::swz(ra, 2 * st + lh));
      }
    }
#pragma unroll
    for (int st = PF ? 0 : CG_BK / 16 - 1; st < CG_BK / 16; ++st) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[st][i], b[st][j], acc[i][j], 0,
                                                              0, 0);
    }
  }
  __syncthreads();     // every wave done with the ring: the epilogue reuses it
  double* red = reinterpret_cast<double*>(ring);

  // ---------------- epilogue (conv_gen_epilogue's arithmetic on this tile)
  if (p.partial) {   // split-K: raw partial sums, the epilogue kernel finishes
    float* pb = p.partial + (int64_t)blockIdx.y * p.Cout * NP;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t pg = px0 + wn * C::WNP + 32 * j + l31;
      if (pg >= NP) continue;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + wm * C::WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (co < p.Cout) pb[(int64_t)co * NP + pg] = acc[i][j][r];
        }
    }
    return;
  }
  const float sc = p.scale ? *p.scale : 1.f;
  bool ok[NJ];
  float rt[NJ];
  float* yb[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int64_t pg = px0 + wn * C::WNP + 32 * j + l31;
    ok[j] = pg < NP;
    int pn = 0, prem = 0;
    if (ok[j]) {
      pn = (int)(pg / HWo);
      prem = (int)(pg - (int64_t)pn * HWo);
    }
    rt[j] = (ok[j] && p.ratio) ? p.ratio[pg] : 1.f;
    yb[j] = p.y + (int64_t)pn * p.Cout * HWo + prem;
  }
  // stats: one (sum, sumsq) per co per OLD_BN-pixel slot; a wave's 64 pixels
  // lie in one slot (OLD_BN is 128 or 256)
  constexpr int SPT = BN / C::OLD_BN > 1 ? BN / C::OLD_BN : 1;   // slots per tile
  constexpr int WPS = C::WGN / SPT;                              // waves per slot
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cll = wm * C::WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int co = co0 + cll;
      const bool cok = co < p.Cout;
      const float bv = (cok && p.bias) ? p.bias[co] : 0.f;
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (!ok[j] || !cok) continue;
        float v = acc[i][j][r] * sc;
        v *= rt[j];
        v += bv;
        a += (double)v;
        b += (double)v * (double)v;
        yb[j][(int64_t)co * HWo] = apply_act(v, act, p.slope);
      }
      if (p.stats) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
        }
        if (l31 == 0) {
          red[(wn * BM + cll) * 2 + 0] = a;
          red[(wn * BM + cll) * 2 + 1] = b;
        }
      }
    }
  }
  if (p.y16) {
    // the ring past the statistics scratch (WGN * BM * 16 bytes): 32 rows of
    // (MI*32 + 8) bf16 per wave
    static_assert(C::WGN * BM * 16 + NW * 32 * (MI * 32 + 8) * 2 <= cgw::NST * C::STAGE,
                  "y16 staging fits the ring");
    uint16_t* stg = reinterpret_cast<uint16_t*>(ring + C::WGN * BM * 16) +
                    wave * 32 * (MI * 32 + 8);
    if (MI == 2)
      epilogue_y16_lds<MI, NJ>(p, acc, act, px0 + wn * C::WNP, co0 + wm * C::WM, ok, rt, lh,
                               l31, lane, stg, NP);
    else
      epilogue_y16<MI, NJ>(p, acc, act, px0 + wn * C::WNP, co0 + wm * C::WM, ok, rt, lh, l31);
  }
  if (p.stats) {
    __syncthreads();
    const int64_t nslots = (NP + C::OLD_BN - 1) / C::OLD_BN;
    for (int e = tid; e < BM * SPT; e += NW * 64) {
      const int cll = e % BM, sl = e / BM;
      const int co = co0 + cll;
      const int64_t slot = (int64_t)px_t * SPT + sl;
      if (co >= p.Cout || slot >= nslots) continue;
      double a = 0.0, b = 0.0;
      for (int q = sl * WPS; q < (sl + 1) * WPS; ++q) {
        a += red[(q * BM + cll) * 2];
        b += red[(q * BM + cll) * 2 + 1];
      }
      p.stats[(slot * 2 + 0) * p.Cout + co] = a;
      p.stats[(slot * 2 + 1) * p.Cout + co] = b;
    }
  }
}

// x [N][C][H][W] fp32 (* mask plane m [N][H][W] if given) -> out [N][H][W][C]
// bf16 (nearest-even): 64 channels x 64 columns of one row per block.
__global__ __launch_bounds__(256) void nchw_to_nhwc16_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ m, int C,
                                                             int H, int W,
                                                             uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][66];   // [w][c]
  const int w0 = blockIdx.x * 64, h = blockIdx.y;
  const int cb = (C + 63) / 64;
  const int n = blockIdx.z / cb, c0 = (blockIdx.z % cb) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int w = w0 + tx;
  const float mv = (m && w < W) ? m[((int64_t)n * H + h) * W + w] : 1.f;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i;
    float v = 0.f;
    if (c < C && w < W) v = x[(((int64_t)n * C + c) * H + h) * W + w] * mv;
    tile[tx][i] = __builtin_bit_cast(uint16_t, (__bf16)v);
  }
  __syncthreads();
  // rows w, lanes along c (bf16 pairs): 32 lanes cover one pixel's 64 channels
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
#pragma unroll
  for (int i = r; i < 64; i += 8) {
    const int ww = w0 + i, c = c0 + 2 * l;
    if (ww >= W || c >= C) continue;
    uint16_t* q = out + (((int64_t)n * H + h) * W + ww) * C + c;
    if (c + 1 < C)
      *reinterpret_cast<uint32_t*>(q) = (uint32_t)tile[i][2 * l] | ((uint32_t)tile[i][2 * l + 1] << 16);
    else
      q[0] = tile[i][2 * l];
  }
}

// BatchNorm affine + activation in place (affine_act_kernel's arithmetic) and,
// in the same pass, the channel-last bf16 copy of act(y) times the mask plane
// (nchw_to_nhwc16_kernel's conversion): the bf16 U-Net's block outputs feed
// the next conv without a separate conversion pass.
// KEEP_Y = false: y is only read (a caller whose consumers all take the
// channel-last copy skips the fp32 write-back, a third of the pass's bytes).
template <bool KEEP_Y>
__global__ __launch_bounds__(256) void affine_act_nhwc16_kernel(
    float* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    int act, float slope, const float* __restrict__ m, int C, int H, int W,
    uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][66];   // [w][c]
  const int w0 = blockIdx.x * 64, h = blockIdx.y;
  const int cb = (C + 63) / 64;
  const int n = blockIdx.z / cb, c0 = (blockIdx.z % cb) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int w = w0 + tx;
  const float mv = (m && w < W) ? m[((int64_t)n * H + h) * W + w] : 1.f;
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i;
    float v = 0.f;
    if (c < C && w < W) {
      float* q = y + (((int64_t)n * C + c) * H + h) * W + w;
      v = apply_act(fmaf(*q, scale[c], shift[c]), act, slope);
      if (KEEP_Y) *q = v;
      v *= mv;
    }
    tile[tx][i] = __builtin_bit_cast(uint16_t, (__bf16)v);
  }
  __syncthreads();
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
#pragma unroll
  for (int i = r; i < 64; i += 8) {
    const int ww = w0 + i, c = c0 + 2 * l;
    if (ww >= W || c >= C) continue;
    uint16_t* q = out + (((int64_t)n * H + h) * W + ww) * C + c;
    if (c + 1 < C)
      *reinterpret_cast<uint32_t*>(q) = (uint32_t)tile[i][2 * l] | ((uint32_t)tile[i][2 * l + 1] << 16);
    else
      q[0] = tile[i][2 * l];
  }
}

// few-channel source x [N][C][Hs][Ws] fp32 (x mask plane m [N][Hs][Ws]),
// resampled to Hin x Win as src_coord -> bf16 rows out [N*Ho*Wo][seg],
// k = tap*C + ci < KK*C, zero past it; one thread = 8 k-values of a pixel
__global__ __launch_bounds__(256) void im2col_nhwc16_kernel(
    const float* __restrict__ x, const float* __restrict__ m, int C, int Hs, int Ws, int up,
    int Hin, int Win, int KH, int KW, int stride, int pad, int Ho, int Wo, int64_t NP, int seg,
    uint16_t* __restrict__ out) {
  const int chunks = seg / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= NP * chunks) return;
  const int64_t pix = t / chunks;
  const int k0 = (int)(t - pix * chunks) * 8;
  const int HWo = Ho * Wo;
  const int n = (int)(pix / HWo);
  const int r = (int)(pix - (int64_t)n * HWo);
  const int oy = r / Wo, ox = r - oy * Wo;
  const int KK = KH * KW;
  uint32_t g[4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    const int tap = k / C, ci = k - tap * C;
    const int ky = tap / KW, kx = tap - ky * KW;
    const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    float v = 0.f;
    if (tap < KK && iy >= 0 && iy < Hin && ix >= 0 && ix < Win) {
      const int sy = src_coord(iy, Hs, Hin, up), sx = src_coord(ix, Ws, Win, up);
      v = x[(((int64_t)n * C + ci) * Hs + sy) * Ws + sx];
      if (m) v *= m[((int64_t)n * Hs + sy) * Ws + sx];
    }
    const uint32_t b = __builtin_bit_cast(uint16_t, (__bf16)v);
    if (j & 1) g[j >> 1] |= b << 16;
    else g[j >> 1] = b;
  }
  *reinterpret_cast<uint4*>(out + pix * seg + k0) = make_uint4(g[0], g[1], g[2], g[3]);
}

// Row-staged im2col_nhwc16_kernel (same values bit for bit): a workgroup owns
// IMN_P consecutive output pixels of one output row; the KH input rows x C
// channels they read (x * m, resampled, zero outside) are staged in LDS with
// coalesced loads, a per-k LDS offset table replaces the per-element tap /
// channel divisions, and each thread writes 16-byte chunks of the [pix][seg]
// rows (consecutive threads: consecutive chunks, one contiguous run per block).
constexpr int IMN_P = 64, IMN_LDS = 4096, IMN_SEG = 256;
__global__ __launch_bounds__(256) void im2col_nhwc16_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ m, int C, int Hs, int Ws, int up,
    int Hin, int Win, int KH, int KW, int stride, int pad, int Ho, int Wo, int seg,
    uint16_t* __restrict__ out) {
  __shared__ float patch[IMN_LDS];   // [ci][ky][PW]
  __shared__ int koff[IMN_SEG];      // k -> patch offset of pixel 0, or -1 past KK*C
  const int ox0 = blockIdx.x * IMN_P, oy = blockIdx.y, n = blockIdx.z;
  const int np = min(IMN_P, Wo - ox0);
  const int PW = (np - 1) * stride + KW;
  const int KK = KH * KW;
  const int iy0 = oy * stride - pad, ix0 = ox0 * stride - pad;
  for (int k = threadIdx.x; k < seg; k += 256) {
    const int tap = k / C, ci = k - tap * C;
    const int ky = tap / KW, kx = tap - ky * KW;
    koff[k] = tap < KK ? (ci * KH + ky) * PW + kx : -1;
  }
  for (int e = threadIdx.x; e < C * KH * PW; e += 256) {
    const int ci = e / (KH * PW), rem = e - ci * KH * PW;
    const int ky = rem / PW, c = rem - ky * PW;
    const int iy = iy0 + ky, ix = ix0 + c;
    float v = 0.f;
    if (iy >= 0 && iy < Hin && ix >= 0 && ix < Win) {
      const int sy = src_coord(iy, Hs, Hin, up), sx = src_coord(ix, Ws, Win, up);
      v = x[(((int64_t)n * C + ci) * Hs + sy) * Ws + sx];
      if (m) v *= m[((int64_t)n * Hs + sy) * Ws + sx];
    }
    patch[e] = v;
  }
  __syncthreads();
  const int chunks = seg / 8;
  uint16_t* ob = out + (((int64_t)n * Ho + oy) * Wo + ox0) * seg;
  for (int t = threadIdx.x; t < np * chunks; t += 256) {
    const int p = t / chunks, k0 = (t - p * chunks) * 8;
    uint32_t g[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = koff[k0 + j];
      const float v = o >= 0 ? patch[o + p * stride] : 0.f;
      const uint32_t b = __builtin_bit_cast(uint16_t, (__bf16)v);
      if (j & 1) g[j >> 1] |= b << 16;
      else g[j >> 1] = b;
    }
    *reinterpret_cast<uint4*>(ob + (int64_t)p * seg + k0) = make_uint4(g[0], g[1], g[2], g[3]);
  }
}

// w [Cout][C0+C1][KH][KW] fp32 -> wt16 [Cout][K] bf16, k = tap*C0 + ci (source 0)
// then seg0 + tap*C1 + ci (source 1), each source padded to nhwc16_seg k-values
// with zeros
__global__ void conv_weight_nhwc16_kernel(const float* __restrict__ w, int Cout, int C0, int C1,
                                          int KK, uint16_t* __restrict__ wt16) {
  const int Cin = C0 + C1;
  const int S0 = nhwc16_seg(C0, KK), K = S0 + nhwc16_seg(C1, KK);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)Cout * K) return;
  const int co = (int)(t / K), k = (int)(t % K);
  int tap, c;
  if (k < S0) {
    tap = k / C0;
    c = k - tap * C0;
  } else {
    tap = (k - S0) / C1;
    c = C0 + (k - S0 - tap * C1);
  }
  const float v = tap < KK ? w[((int64_t)co * Cin + c) * KK + tap] : 0.f;
  wt16[t] = __builtin_bit_cast(uint16_t, (__bf16)v);
}

}  // namespace ainp


// ============================================================== C ABI
using namespace ainp;

static ConvSrcDev make_src(const float* x, const float* m, int C, int Hs, int Ws, int Hin,
                           int Win) {
  ConvSrcDev s;
  s.x = x;
  s.m = m;
  s.C = C;
  s.Hs = Hs;
  s.Ws = Ws;
  if (Hs == Hin && Ws == Win) s.up = 0;
  else if (2 * Hs == Hin && 2 * Ws == Win) s.up = 1;
  else s.up = 2;
  return s;
}

static int conv_gen_bm(int Cout) { return Cout > 64 ? 128 : 64; }

// K splits for a launch: small tile grids with long K (the U-Net bottleneck,
// VGG's last blocks) are split so ~768 workgroups run; >= 8 K tiles per split.
// For Cout > 64 count the workgroups of the bf16 wide-tile kernel (256 x 128 /
// 128 x 256 tiles, two per CU) and split grids under 384 of them to ~512: the
// U-Net decoder's 240-tile layers ran on half the CUs' slots (C4 9.34-9.37 ->
// 9.24-9.25, C5 11.98-12.00 -> 11.78-11.80 ms/step, profiles/r04t_summary.txt).
// AINP_CONV_SPLIT_WIDE=0: the old-tile count for every Cout; =3: ~768.
static int conv_gen_nsplit(int64_t NP, int Cout, int K) {
  if (Cout == 1) return 1;
  const int BM = conv_gen_bm(Cout);
  const int64_t blocks = cdiv(NP, 16384 / BM) * cdiv(Cout, BM);
  const int nkt = (int)cdiv(K, CG_BK);
  static const int wide_target = [] {
    const char* e = getenv("AINP_CONV_SPLIT_WIDE");
    return (e && e[0] == '0') ? 0 : (e && e[0] == '3') ? 768 : 512;
  }();
  if (wide_target && Cout > 64) {
    const int64_t bw = Cout > 128 ? cdiv(NP, 128) * cdiv(Cout, 256) : cdiv(NP, 256) * cdiv(Cout, 128);
    if (bw >= 384 || nkt < 16) return 1;
    int64_t sw = wide_target / bw;
    if (sw > nkt / 8) sw = nkt / 8;
    if (sw < 1) sw = 1;
    const int per = (int)cdiv(nkt, sw);
    return (int)cdiv(nkt, per);
  }
  if (blocks >= 384 || nkt < 16) return 1;
  int64_t s = cdiv(768, blocks);
  if (s > nkt / 8) s = nkt / 8;
  if (s < 1) s = 1;
  const int per = (int)cdiv(nkt, s);
  return (int)cdiv(nkt, per);   // no empty split
}

extern "C" int ainp_conv_gen_stat_parts(int64_t N, int Cin, int KH, int KW, int Cout, int64_t Ho,
                                        int64_t Wo) {
  const int64_t NP = N * Ho * Wo;
  if (conv_gen_nsplit(NP, Cout, Cin * KH * KW) > 1)
    return (int)cdiv(NP, splitk_tile() ? SKT_P : 256);
  return (int)cdiv(NP, 16384 / conv_gen_bm(Cout));
}

extern "C" int ainp_conv_weight_kmajor(const float* w, int Cout, int C0, int C1, int KH, int KW,
                                       float* wt, void* stream) {
  if (!w || !wt || Cout < 1 || C0 < 1 || C1 < 0 || KH < 1 || KW < 1)
    return record_msg("ainp_conv_weight_kmajor: bad argument");
  const int64_t total = (int64_t)(C0 + C1) * KH * KW * Cout;
  hipLaunchKernelGGL(conv_weight_kmajor_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), w, Cout, C0, C1, KH * KW, wt);
  return check_launch("conv_weight_kmajor");
}

extern "C" size_t ainp_conv_gen_workspace(int64_t N, int Cin, int KH, int KW, int Cout,
                                          int64_t Ho, int64_t Wo) {
  if (Cout == 1) return (size_t)cdiv(Cin, C1_CC) * N * Ho * Wo * sizeof(float);
  const int64_t NP = N * Ho * Wo;
  const int ns = conv_gen_nsplit(NP, Cout, Cin * KH * KW);
  return ns > 1 ? (size_t)ns * Cout * NP * sizeof(float) : 0;
}

extern "C" int ainp_conv_gen_fwd(const float* x0, const float* m0, int C0, int H0, int W0,
                                 const float* x1, const float* m1, int C1, int H1, int W1,
                                 const float* w, const float* wt, const float* bias,
                                 const float* ratio, const float* scale, float* y, double* stats,
                                 int64_t N,
                                 int Cout, int Hin, int Win, int KH, int KW, int stride,
                                 int pad, int act, float slope, int crop_h, int crop_w,
                                 void* workspace, void* stream) {
  return ainp_conv_gen_fwd_ex(x0, m0, C0, H0, W0, x1, m1, C1, H1, W1, w, wt, bias, ratio, scale, y,
                              stats, N, Cout, Hin, Win, KH, KW, stride, pad, act, slope, crop_h,
                              crop_w, 0, workspace, stream);
}

extern "C" int ainp_conv_gen_fwd_ex(const float* x0, const float* m0, int C0, int H0, int W0,
                                    const float* x1, const float* m1, int C1, int H1, int W1,
                                    const float* w, const float* wt, const float* bias,
                                    const float* ratio, const float* scale, float* y,
                                    double* stats, int64_t N, int Cout, int Hin, int Win, int KH,
                                    int KW, int stride, int pad, int act, float slope, int crop_h,
                                    int crop_w, int flags, void* workspace, void* stream) {
  return ainp_conv_gen_fwd_out16(x0, m0, C0, H0, W0, x1, m1, C1, H1, W1, w, wt, bias, ratio,
                                 scale, y, stats, N, Cout, Hin, Win, KH, KW, stride, pad, act,
                                 slope, crop_h, crop_w, flags, nullptr, workspace, stream);
}

extern "C" int ainp_conv_gen_fwd_out16(const float* x0, const float* m0, int C0, int H0, int W0,
                                       const float* x1, const float* m1, int C1, int H1, int W1,
                                       const float* w, const float* wt, const float* bias,
                                       const float* ratio, const float* scale, float* y,
                                       double* stats, int64_t N, int Cout, int Hin, int Win,
                                       int KH, int KW, int stride, int pad, int act, float slope,
                                       int crop_h, int crop_w, int flags, uint16_t* y16,
                                       void* workspace, void* stream) {
  if (!x0 || C0 < 1 || C1 < 0 || (C1 > 0 && !x1) || !w || !y || N < 1 || Cout < 1 ||
      Hin < 1 || Win < 1 || KH < 1 || KW < 1 || stride < 1 || pad < 0 || act < 0 || act > 3 ||
      (flags & ~AINP_CONV_BF16) || (y16 && (Cout % 8 || ((uintptr_t)y16 & 15))))
    return record_msg("ainp_conv_gen_fwd: bad argument (y16: Cout % 8 == 0, 16-byte aligned)");
  const bool b16 = (flags & AINP_CONV_BF16) != 0;
  const int Ho = (Hin + 2 * pad - KH) / stride + 1;
  const int Wo = (Win + 2 * pad - KW) / stride + 1;
  if (Ho < 1 || Wo < 1) return record_msg("ainp_conv_gen_fwd: empty output");
  ConvGenParams p;
  p.s0 = make_src(x0, m0, C0, H0, W0, Hin, Win);
  p.s1 = make_src(x1, m1, C1, C1 ? H1 : Hin, C1 ? W1 : Win, Hin, Win);
  if ((p.s0.up == 1 && (H0 * 2 != Hin)) || H0 < 1 || W0 < 1)
    return record_msg("ainp_conv_gen_fwd: bad source size");
  p.w = w;
  p.bias = bias;
  p.ratio = ratio;
  p.scale = scale;
  p.y = y;
  p.stats = stats;
  p.partial = nullptr;
  p.y16 = nullptr;
  p.ktiles_per_split = 1 << 30;
  p.N = (int)N;
  p.Cin = C0 + C1;
  p.Cout = Cout;
  p.Hin = Hin;
  p.Win = Win;
  p.Ho = Ho;
  p.Wo = Wo;
  p.KH = KH;
  p.KW = KW;
  p.stride = stride;
  p.pad = pad;
  p.slope = slope;
  hipStream_t s = as_stream(stream);
  if (Cout == 1) {
    const int Hc = crop_h > 0 ? crop_h : Ho, Wc = crop_w > 0 ? crop_w : Wo;
    if (stats || Hc > Ho || Wc > Wo || !workspace || KH * KW > 64)
      return record_msg("ainp_conv_gen_fwd: Cout=1 options (workspace, kernel <= 8x8)");
    const int64_t np = N * (int64_t)Hc * Wc;
    const int nchunk = (int)cdiv(p.Cin, C1_CC);
    float* part = reinterpret_cast<float*>(workspace);
    // one plain source, whole 32-channel chunks, square 3 / 4 kernels: the
    // batched-tap variant (AINP_COUT1_B=0: the loop kernel, A/B)
    static const bool c1b = [] {
      const char* e = getenv("AINP_COUT1_B");
      return !(e && e[0] == '0');
    }();
    const bool plain = p.s1.C == 0 && p.s0.up == 0 && p.Cin % C1_CC == 0 && KH == KW &&
                       (int64_t)N * p.Cin * p.s0.Hs * p.s0.Ws * 4 < ((int64_t)1 << 31);
    if (c1b && plain && KH == 3)
      hipLaunchKernelGGL((conv_cout1_partial_b_kernel<3, 4>), dim3((unsigned)cdiv(np, 256), nchunk),
                         dim3(256), 0, s, p, Hc, Wc, part);
    else if (c1b && plain && KH == 4)
      hipLaunchKernelGGL((conv_cout1_partial_b_kernel<4, 4>), dim3((unsigned)cdiv(np, 256), nchunk),
                         dim3(256), 0, s, p, Hc, Wc, part);
    else
      hipLaunchKernelGGL(conv_cout1_partial_kernel, dim3((unsigned)cdiv(np, 256), nchunk),
                         dim3(256), 0, s, p, Hc, Wc, part);
    hipLaunchKernelGGL(conv_cout1_finish_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, s, p,
                       act, Hc, Wc, nchunk, part);
    return check_launch("conv_cout1");
  }
  if (crop_h > 0 || crop_w > 0) return record_msg("ainp_conv_gen_fwd: crop needs Cout=1");
  // few input channels, one plain source, no BN statistics: the direct kernel
  static const bool small_ok = [] {
    const char* e = getenv("AINP_CONV_SMALLCIN");
    return !(e && e[0] == '0');
  }();
  if (small_ok && C1 == 0 && p.s0.up == 0 && !stats && Cout <= SC_CO &&
      (int64_t)C0 * KH * KW <= SC_K && C0 <= 4) {
    const int64_t NPs = N * (int64_t)Ho * Wo;
    p.y16 = y16;
    // AINP_SMALLCIN_LDS16=0: each thread stores its own pixel's bf16 row (A/B)
    static const bool l16 = [] {
      const char* e = getenv("AINP_SMALLCIN_LDS16");
      return !(e && e[0] == '0');
    }();
    const dim3 g((unsigned)cdiv(NPs, 256));
    if (b16 && l16 && y16 && Cout % 8 == 0)
      hipLaunchKernelGGL((conv_gen_smallcin_kernel<true, true>), g, dim3(256), 0, s, p, act);
    else if (b16)
      hipLaunchKernelGGL((conv_gen_smallcin_kernel<true, false>), g, dim3(256), 0, s, p, act);
    else if (l16 && y16 && Cout % 8 == 0)
      hipLaunchKernelGGL((conv_gen_smallcin_kernel<false, true>), g, dim3(256), 0, s, p, act);
    else
      hipLaunchKernelGGL((conv_gen_smallcin_kernel<false, false>), g, dim3(256), 0, s, p, act);
    return check_launch("conv_gen_smallcin");
  }
  if (y16) return record_msg("ainp_conv_gen_fwd: y16 is written by the few-input-channel kernel only");
  if (!wt) return record_msg("ainp_conv_gen_fwd: k-major weights (ainp_conv_weight_kmajor) required");
  const int BM = conv_gen_bm(Cout);
  const int64_t NP = N * (int64_t)Ho * Wo;
  const int K = p.Cin * KH * KW;
  const int nsplit = conv_gen_nsplit(NP, Cout, K);
  if (nsplit > 1) {
    if (!workspace) return record_msg("ainp_conv_gen_fwd: split-K needs ainp_conv_gen_workspace");
    p.partial = reinterpret_cast<float*>(workspace);
    p.ktiles_per_split = (int)cdiv(cdiv(K, CG_BK), nsplit);
  }
  const int64_t tiles = cdiv(NP, 16384 / BM);
  dim3 grid((unsigned)tiles, (unsigned)cdiv(Cout, BM), (unsigned)nsplit);
  // fp32-accurate split-bf16 main loop unless AINP_CONV_EXACT=1 (exact f32 MFMA)
  static const bool exact = [] {
    const char* e = getenv("AINP_CONV_EXACT");
    return e && e[0] == '1';
  }();
  static const int xbk = [] {
    const char* e = getenv("AINP_CONV_GEN_BK");
    return (e && e[0] == '3') ? 32 : 16;
  }();
  // bf16 operands: one plane, 32-deep K-tiles (measured: 64-deep tiles at
  // 184-212 VGPRs ran the C4 step's convs 1.6x slower); AINP_CONV_GEN_B16_BK
  // = 16 / 64 selects the other depths
  static const int b16bk = [] {
    const char* e = getenv("AINP_CONV_GEN_B16_BK");
    return (e && e[0] == '6') ? 64 : (e && e[0] == '1') ? 16 : 32;
  }();
  const int bk = !b16 ? 0 : (b16bk == 64 && nsplit > 1 && p.ktiles_per_split % 2) ? 32 : b16bk;
  if (bk == 64 && BM == 128)
    hipLaunchKernelGGL((conv_gen_x6_kernel<128, 64, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (bk == 64)
    hipLaunchKernelGGL((conv_gen_x6_kernel<64, 64, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (bk == 16 && BM == 128)
    hipLaunchKernelGGL((conv_gen_x6_kernel<128, 16, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (bk == 16)
    hipLaunchKernelGGL((conv_gen_x6_kernel<64, 16, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (b16 && BM == 128)
    hipLaunchKernelGGL((conv_gen_x6_kernel<128, 32, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (b16)
    hipLaunchKernelGGL((conv_gen_x6_kernel<64, 32, 1>), grid, dim3(256), 0, s, p, wt, act);
  else if (!exact && BM == 128 && xbk == 16)
    hipLaunchKernelGGL((conv_gen_x6_kernel<128, 16, 3>), grid, dim3(256), 0, s, p, wt, act);
  else if (!exact && xbk == 16)
    hipLaunchKernelGGL((conv_gen_x6_kernel<64, 16, 3>), grid, dim3(256), 0, s, p, wt, act);
  else if (!exact && BM == 128)
    hipLaunchKernelGGL((conv_gen_x6_kernel<128, 32, 3>), grid, dim3(256), 0, s, p, wt, act);
  else if (!exact)
    hipLaunchKernelGGL((conv_gen_x6_kernel<64, 32, 3>), grid, dim3(256), 0, s, p, wt, act);
  else if (BM == 128)
    hipLaunchKernelGGL(conv_gen_fwd_kernel<128>, grid, dim3(256), 0, s, p, wt, act);
  else
    hipLaunchKernelGGL(conv_gen_fwd_kernel<64>, grid, dim3(256), 0, s, p, wt, act);
  int rc = check_launch("conv_gen_fwd");
  if (rc || nsplit == 1) return rc;
  return splitk_epilogue_launch(p, NP, nsplit, act, s);
}

extern "C" int ainp_nchw_to_nhwc16(const float* x, const float* m, int64_t N, int C, int H, int W,
                                   uint16_t* out, void* stream) {
  if (!x || !out || N < 1 || C < 1 || H < 1 || W < 1 || N * ((C + 63) / 64) > 65535 || H > 65535)
    return record_msg("ainp_nchw_to_nhwc16: bad argument");
  hipLaunchKernelGGL(nchw_to_nhwc16_kernel, dim3((unsigned)cdiv(W, 64), (unsigned)H,
                                                 (unsigned)(N * cdiv(C, 64))),
                     dim3(256), 0, as_stream(stream), x, m, C, H, W, out);
  return check_launch("nchw_to_nhwc16");
}

extern "C" int ainp_affine_act_nhwc16(float* y, const float* scale, const float* shift,
                                     int64_t N, int C, int H, int W, int act, float slope,
                                     const float* m, uint16_t* out, void* stream) {
  return ainp_affine_act_nhwc16_ex(y, scale, shift, N, C, H, W, act, slope, m, out, 0, stream);
}

extern "C" int ainp_affine_act_nhwc16_ex(float* y, const float* scale, const float* shift,
                                        int64_t N, int C, int H, int W, int act, float slope,
                                        const float* m, uint16_t* out, int flags, void* stream) {
  if (!y || !scale || !shift || !out || N < 1 || C < 1 || H < 1 || W < 1 ||
      N * ((C + 63) / 64) > 65535 || H > 65535 || (flags & ~AINP_AFFINE_NO_Y))
    return record_msg("ainp_affine_act_nhwc16: bad argument");
  const dim3 grid((unsigned)cdiv(W, 64), (unsigned)H, (unsigned)(N * cdiv(C, 64)));
  if (flags & AINP_AFFINE_NO_Y)
    hipLaunchKernelGGL(affine_act_nhwc16_kernel<false>, grid, dim3(256), 0, as_stream(stream), y,
                       scale, shift, act, slope, m, C, H, W, out);
  else
    hipLaunchKernelGGL(affine_act_nhwc16_kernel<true>, grid, dim3(256), 0, as_stream(stream), y,
                       scale, shift, act, slope, m, C, H, W, out);
  return check_launch("affine_act_nhwc16");
}

extern "C" int ainp_im2col_nhwc16(const float* x, const float* m, int64_t N, int C, int Hs,
                                  int Ws, int Hin, int Win, int KH, int KW, int stride, int pad,
                                  uint16_t* out, void* stream) {
  if (!x || !out || N < 1 || C < 1 || Hs < 1 || Ws < 1 || Hin < 1 || Win < 1 || KH < 1 ||
      KW < 1 || stride < 1 || pad < 0 || ((uintptr_t)out & 15))
    return record_msg("ainp_im2col_nhwc16: bad argument");
  const int Ho = (Hin + 2 * pad - KH) / stride + 1, Wo = (Win + 2 * pad - KW) / stride + 1;
  if (Ho < 1 || Wo < 1) return record_msg("ainp_im2col_nhwc16: empty output");
  const ConvSrcDev sd = make_src(x, m, C, Hs, Ws, Hin, Win);
  if (sd.up == 1 && Hs * 2 != Hin) return record_msg("ainp_im2col_nhwc16: bad source size");
  const int seg = nhwc16_seg(C, KH * KW);
  const int64_t NP = N * (int64_t)Ho * Wo;
  // row-staged kernel where its LDS holds the patch (AINP_IM2COL_NHWC16_ROWS=0:
  // the per-chunk kernel)
  static const bool rows_env = [] {
    const char* e = getenv("AINP_IM2COL_NHWC16_ROWS");
    return !(e && e[0] == '0');
  }();
  const int PWmax = (IMN_P - 1) * stride + KW;
  if (rows_env && (int64_t)C * KH * PWmax <= IMN_LDS && seg <= IMN_SEG && N <= 65535 &&
      Ho <= 65535) {
    hipLaunchKernelGGL(im2col_nhwc16_rows_kernel,
                       dim3((unsigned)cdiv(Wo, IMN_P), (unsigned)Ho, (unsigned)N), dim3(256), 0,
                       as_stream(stream), x, m, C, Hs, Ws, sd.up, Hin, Win, KH, KW, stride, pad,
                       Ho, Wo, seg, out);
    return check_launch("im2col_nhwc16_rows");
  }
  hipLaunchKernelGGL(im2col_nhwc16_kernel, dim3((unsigned)cdiv(NP * (seg / 8), 256)), dim3(256), 0,
                     as_stream(stream), x, m, C, Hs, Ws, sd.up, Hin, Win, KH, KW, stride, pad, Ho,
                     Wo, NP, seg, out);
  return check_launch("im2col_nhwc16");
}

extern "C" int ainp_conv_weight_nhwc16(const float* w, int Cout, int C0, int C1, int KH, int KW,
                                       uint16_t* wt16, void* stream) {
  if (!w || !wt16 || Cout < 1 || C0 < 1 || C1 < 0 || KH < 1 || KW < 1)
    return record_msg("ainp_conv_weight_nhwc16: bad argument");
  const int64_t total =
      (int64_t)Cout * (nhwc16_seg(C0, KH * KW) + nhwc16_seg(C1, KH * KW));
  hipLaunchKernelGGL(conv_weight_nhwc16_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), w, Cout, C0, C1, KH * KW, wt16);
  return check_launch("conv_weight_nhwc16");
}

// conv_gen_nhwc16 main loop: 0 register-staged, 1 LDS-DMA ring, 2 wide-tile
// ring of 4 waves, 3 (default) wide-tile ring of 8 waves for Cout > 64 and the
// register-staged kernel below (tools/conv16_lab.py, profiles/r03_c16b_*: the
// C4 step's 30 launches 3.98 -> 3.59 ms, all bit-identical).  Initial value
// from AINP_CONV16 (or AINP_CONV16_RING=1).
static int g_conv16_variant = -1;
static int conv16_variant() {
  if (g_conv16_variant < 0) {
    const char* e = getenv("AINP_CONV16");
    const char* r = getenv("AINP_CONV16_RING");
    g_conv16_variant = (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : ((r && r[0] == '1') ? 1 : 3);
  }
  return g_conv16_variant;
}

extern "C" int ainp_conv16_set_variant(int v) {
  const int prev = conv16_variant();
  if (v >= 0 && v <= 3) g_conv16_variant = v;
  return prev;
}

extern "C" int ainp_conv_gen_fwd_nhwc16_ex(const uint16_t* x0, int C0, int H0, int W0,
                                        const uint16_t* x1, int C1, int H1, int W1,
                                        const uint16_t* wt16, const float* bias, const float* ratio,
                                        const float* scale, float* y, double* stats, int64_t N,
                                        int Cout, int Hin, int Win, int KH, int KW, int stride,
                                        int pad, int act, float slope, uint16_t* y16, void* workspace,
                                        void* stream) {
  if (!x0 || C0 < 1 || C1 < 0 || (C1 > 0 && !x1) || !wt16 || !y || N < 1 || Cout < 2 ||
      Hin < 1 || Win < 1 || KH < 1 || KW < 1 || stride < 1 || pad < 0 || act < 0 || act > 3 ||
      (C0 % 32 == 0 && ((uintptr_t)x0 & 15)) || (C1 % 32 == 0 && ((uintptr_t)x1 & 15)) ||
      ((uintptr_t)wt16 & 15))
    return record_msg("ainp_conv_gen_fwd_nhwc16: bad argument (Cout > 1, 16-B aligned)");
  const int Ho = (Hin + 2 * pad - KH) / stride + 1;
  const int Wo = (Win + 2 * pad - KW) / stride + 1;
  if (Ho < 1 || Wo < 1) return record_msg("ainp_conv_gen_fwd_nhwc16: empty output");
  Src16 a{x0, C0, H0, W0, 0, C0 % 32 != 0}, b{x1, C1, C1 ? H1 : Hin, C1 ? W1 : Win, 0, C1 % 32 != 0};
  const ConvSrcDev sa = make_src(nullptr, nullptr, C0, H0, W0, Hin, Win);
  const ConvSrcDev sb = make_src(nullptr, nullptr, C1, b.Hs, b.Ws, Hin, Win);
  a.up = sa.up;
  b.up = sb.up;
  if (a.up == 1 && H0 * 2 != Hin) return record_msg("ainp_conv_gen_fwd_nhwc16: bad source size");
  ConvGenParams p;
  p.s0 = sa;
  p.s1 = sb;
  p.w = nullptr;
  p.bias = bias;
  p.ratio = ratio;
  p.scale = scale;
  p.y = y;
  p.stats = stats;
  p.partial = nullptr;
  p.y16 = y16;
  p.ktiles_per_split = 1 << 30;
  p.N = (int)N;
  p.Cin = C0 + C1;
  p.Cout = Cout;
  p.Hin = Hin;
  p.Win = Win;
  p.Ho = Ho;
  p.Wo = Wo;
  p.KH = KH;
  p.KW = KW;
  p.stride = stride;
  p.pad = pad;
  p.slope = slope;
  const int BM = conv_gen_bm(Cout);
  const int64_t NP = N * (int64_t)Ho * Wo;
  // the split count follows the unpadded K (ainp_conv_gen_workspace /
  // _stat_parts); the padded tiles are spread over those splits
  const int nsplit = conv_gen_nsplit(NP, Cout, p.Cin * KH * KW);
  const int Kp = nhwc16_seg(C0, KH * KW) + nhwc16_seg(C1, KH * KW);
  if (nsplit > 1) {
    if (!workspace) return record_msg("ainp_conv_gen_fwd_nhwc16: split-K needs ainp_conv_gen_workspace");
    p.partial = reinterpret_cast<float*>(workspace);
    p.ktiles_per_split = (int)cdiv(Kp / CG_BK, nsplit);
  }
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)cdiv(NP, 16384 / BM), (unsigned)cdiv(Cout, BM), (unsigned)nsplit);
  const bool exp = a.exp || b.exp;
  const int variant = conv16_variant();
  // AINP_CONV16_SMALLCO=2: Cout <= 64 on the 4-wave 64 x 256 wide ring under
  // the default variant too (A/B)
  static const bool small_wide = [] {
    const char* e = getenv("AINP_CONV16_SMALLCO");
    return e && e[0] == '2';
  }();
  if (variant == 2 || (variant == 3 && (Cout > 64 || small_wide))) {
    const int BW = Cout > 128 ? 256 : (Cout > 64 ? 128 : 64);
    const int BNW = BW == 256 ? 128 : 256;       // both NW: 256x128 / 128x256 / 64x256
    const int tco = (int)cdiv(Cout, BW), tpx = (int)cdiv(NP, BNW);
    const dim3 gw((unsigned)(tco * tpx), (unsigned)nsplit);
#define AINP_CGW(BMV, NWV, EXPV)                                                                 \
  hipLaunchKernelGGL((conv_gen_nhwc16_wide_kernel<BMV, NWV, EXPV>), gw, dim3(NWV * 64), 0, s, p, a, \
                     b, wt16, act, tco, tpx)
    static const bool wide_pf = [] {
      const char* e = getenv("AINP_WIDE_PF");
      return !(e && e[0] == '0');
    }();
#define AINP_CGW8(BMV, EXPV)                                                                      \
  do {                                                                                           \
    if (wide_pf)                                                                                 \
      hipLaunchKernelGGL((conv_gen_nhwc16_wide_kernel<BMV, 8, EXPV, true>), gw, dim3(512), 0, s, p, \
                         a, b, wt16, act, tco, tpx);                                             \
    else                                                                                         \
      hipLaunchKernelGGL((conv_gen_nhwc16_wide_kernel<BMV, 8, EXPV, false>), gw, dim3(512), 0, s,  \
                         p, a, b, wt16, act, tco, tpx);                                          \
  } while (0)
    if (variant == 3 && BW > 64) {
      if (BW == 256) { if (exp) AINP_CGW8(256, true); else AINP_CGW8(256, false); }
      else { if (exp) AINP_CGW8(128, true); else AINP_CGW8(128, false); }
#undef AINP_CGW8
    } else if (BW == 256) { if (exp) AINP_CGW(256, 4, true); else AINP_CGW(256, 4, false); }
    else if (BW == 128) { if (exp) AINP_CGW(128, 4, true); else AINP_CGW(128, 4, false); }
    else { if (exp) AINP_CGW(64, 4, true); else AINP_CGW(64, 4, false); }
#undef AINP_CGW
  } else if (variant == 1) {
    if (BM == 128 && exp)
      hipLaunchKernelGGL((conv_gen_nhwc16_ring_kernel<128, true>), grid, dim3(256), 0, s, p, a, b,
                         wt16, act);
    else if (BM == 128)
      hipLaunchKernelGGL((conv_gen_nhwc16_ring_kernel<128, false>), grid, dim3(256), 0, s, p, a,
                         b, wt16, act);
    else if (exp)
      hipLaunchKernelGGL((conv_gen_nhwc16_ring_kernel<64, true>), grid, dim3(256), 0, s, p, a, b,
                         wt16, act);
    else
      hipLaunchKernelGGL((conv_gen_nhwc16_ring_kernel<64, false>), grid, dim3(256), 0, s, p, a, b,
                         wt16, act);
  } else if (BM == 128 && exp)
    hipLaunchKernelGGL((conv_gen_nhwc16_kernel<128, true>), grid, dim3(256), 0, s, p, a, b, wt16, act);
  else if (BM == 128)
    hipLaunchKernelGGL((conv_gen_nhwc16_kernel<128, false>), grid, dim3(256), 0, s, p, a, b, wt16, act);
  else if (exp)
    hipLaunchKernelGGL((conv_gen_nhwc16_kernel<64, true>), grid, dim3(256), 0, s, p, a, b, wt16, act);
  else
    hipLaunchKernelGGL((conv_gen_nhwc16_kernel<64, false>), grid, dim3(256), 0, s, p, a, b, wt16, act);
  int rc = check_launch("conv_gen_nhwc16");
  if (rc || nsplit == 1) return rc;
  rc = splitk_epilogue_launch(p, NP, nsplit, act, s);
  if (rc || !y16 || splitk_tile()) return rc;
  // split-K layers are small: their bf16 copy by the coalesced transpose kernel
  // (the per-channel epilogue blocks would store it 2 bytes at a time)
  return ainp_nchw_to_nhwc16(y, nullptr, N, Cout, Ho, Wo, y16, stream);
}

extern "C" int ainp_conv_gen_fwd_nhwc16(const uint16_t* x0, int C0, int H0, int W0,
                                        const uint16_t* x1, int C1, int H1, int W1,
                                        const uint16_t* wt16, const float* bias, const float* ratio,
                                        const float* scale, float* y, double* stats, int64_t N,
                                        int Cout, int Hin, int Win, int KH, int KW, int stride,
                                        int pad, int act, float slope, void* workspace,
                                        void* stream) {
  return ainp_conv_gen_fwd_nhwc16_ex(x0, C0, H0, W0, x1, C1, H1, W1, wt16, bias, ratio, scale, y,
                                     stats, N, Cout, Hin, Win, KH, KW, stride, pad, act, slope,
                                     nullptr, workspace, stream);
}

extern "C" int ainp_pconv_mask(const float* m0, int C0, int H0, int W0, const float* m1, int C1,
                               int H1, int W1, int64_t N, int Hin, int Win, int KH, int KW,
                               int stride, int pad, float winsize, float* ratio, float* newmask,
                               void* stream) {
  if (!m0 || C0 < 1 || (C1 > 0 && !m1) || N < 1 || KH < 1 || KW < 1 || stride < 1)
    return record_msg("ainp_pconv_mask: bad argument");
  const int Ho = (Hin + 2 * pad - KH) / stride + 1;
  const int Wo = (Win + 2 * pad - KW) / stride + 1;
  ConvSrcDev s0 = make_src(nullptr, m0, C0, H0, W0, Hin, Win);
  ConvSrcDev s1 = make_src(nullptr, m1, C1, C1 ? H1 : Hin, C1 ? W1 : Win, Hin, Win);
  if (winsize <= 0.f) winsize = (float)((C0 + C1) * KH * KW);
  const int64_t np = N * (int64_t)Ho * Wo;
  const dim3 grid((unsigned)cdiv(np, 256));
  hipStream_t st = as_stream(stream);
#define AINP_PCM(KT)                                                                          \
  hipLaunchKernelGGL(pconv_mask_kernel<KT>, grid, dim3(256), 0, st, s0, s1, (int)N, Hin, Win, KH, \
                     KW, stride, pad, Ho, Wo, winsize, ratio, newmask)
  static const bool unroll = [] {   // AINP_PCONV_MASK_UNROLL=0: the loop kernel (A/B)
    const char* e = getenv("AINP_PCONV_MASK_UNROLL");
    return !(e && e[0] == '0');
  }();
  const int kt = unroll && KH == KW ? KH : 0;
  if (kt == 3) AINP_PCM(3);
  else if (kt == 4) AINP_PCM(4);
  else if (kt == 5) AINP_PCM(5);
  else if (kt == 7) AINP_PCM(7);
  else AINP_PCM(0);
#undef AINP_PCM
  return check_launch("pconv_mask");
}

extern "C" int ainp_gan_pad_input(const float* x, const float* m, int64_t N, int H, int W,
                                  int Hp, int Wp, float* xp, float* mp, void* stream) {
  if (!x || !m || !xp || !mp || N < 1 || Hp < H || Wp < W || Hp - H >= H || Wp - W >= W)
    return record_msg("ainp_gan_pad_input: bad argument (reflect pad must be < size)");
  const int64_t n = N * (int64_t)Hp * Wp;
  hipLaunchKernelGGL(gan_pad_input_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), x, m, (int)N, H, W, Hp, Wp, xp, mp);
  return check_launch("gan_pad_input");
}

extern "C" int ainp_affine_act(float* y, const float* scale, const float* shift, int64_t N,
                               int C, int64_t HW, int act, float slope, void* stream) {
  if (!y || !scale || !shift || N < 1 || C < 1 || HW < 1 || act < 0 || act > 3)
    return record_msg("ainp_affine_act: bad argument");
  const int64_t total = N * C * HW;
  hipLaunchKernelGGL(affine_act_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), y, scale, shift, C, HW, total, act, slope);
  return check_launch("affine_act");
}

extern "C" int ainp_maxpool2_nhwc16(const float* x, float* y, int64_t N, int C, int H, int W,
                                    uint16_t* out, void* stream) {
  if (!x || !y || !out || N < 1 || C < 1 || H < 2 || W < 2 || ((uintptr_t)out & 3) ||
      N * ((C + 63) / 64) > 65535 || H / 2 > 65535)
    return record_msg("ainp_maxpool2_nhwc16: bad argument");
  hipLaunchKernelGGL(maxpool2_nhwc16_kernel, dim3((unsigned)cdiv(W / 2, 64), (unsigned)(H / 2),
                                                  (unsigned)(N * cdiv(C, 64))),
                     dim3(256), 0, as_stream(stream), x, y, C, H, W, out);
  return check_launch("maxpool2_nhwc16");
}

extern "C" int ainp_maxpool2(const float* x, float* y, int64_t NC, int H, int W, void* stream) {
  if (!x || !y || NC < 1 || H < 2 || W < 2) return record_msg("ainp_maxpool2: bad argument");
  const int64_t n = NC * (H / 2) * (W / 2);
  hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), x, y, NC, H, W);
  return check_launch("maxpool2");
}

extern "C" int ainp_vgg_prep(const float* x, int64_t N, int H, int W, int generated,
                             unsigned int* max_ws, const int* ry0, const int* rn,
                             const float* rw, int rtaps, const int* cx0, const int* cn,
                             const float* cw, int ctaps, int S, float* out, void* stream) {
  if (!x || N < 1 || !ry0 || !rn || !rw || !cx0 || !cn || !cw || !out || S < 1 ||
      generated < 0 || generated > 2 || (generated != 1 && !max_ws))
    return record_msg("ainp_vgg_prep: bad argument");
  hipStream_t s = as_stream(stream);
  if (generated == 2) generated = 0;  // target whose batch max max_ws already holds
  else if (!generated) {
    hipError_t me = hipMemsetAsync(max_ws, 0, sizeof(unsigned int), s);
    if (me != hipSuccess) return record_error(me, "vgg_prep memset");
    hipLaunchKernelGGL(clamp_max_kernel, dim3(256), dim3(256), 0, s, x, N * (int64_t)H * W,
                       max_ws);
  }
  const int64_t n = N * (int64_t)S * S;
  hipLaunchKernelGGL(vgg_prep_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, x, (int)N,
                     H, W, generated, max_ws, ry0, rn, rw, rtaps, cx0, cn, cw, ctaps, S, out);
  return check_launch("vgg_prep");
}

extern "C" int ainp_vgg_target_max(const float* x, int64_t n, unsigned int* max_ws,
                                   void* stream) {
  if (!x || n < 1 || !max_ws) return record_msg("ainp_vgg_target_max: bad argument");
  hipStream_t s = as_stream(stream);
  hipError_t me = hipMemsetAsync(max_ws, 0, sizeof(unsigned int), s);
  if (me != hipSuccess) return record_error(me, "vgg_target_max memset");
  hipLaunchKernelGGL(clamp_max_kernel, dim3(256), dim3(256), 0, s, x, n, max_ws);
  return check_launch("vgg_target_max");
}

static const int kRedBlocks = 512;

extern "C" size_t ainp_reduce_workspace(void) { return (size_t)kRedBlocks * 5 * sizeof(double); }

extern "C" int ainp_absdiff_mean(const float* a, const float* b, int64_t n, void* workspace,
                                 double* out, void* stream) {
  if (!a || !b || n < 1 || !workspace || !out) return record_msg("ainp_absdiff_mean: bad argument");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(absdiff_partial_kernel, dim3(kRedBlocks), dim3(256), 0, s, a, b, n, part);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, part, kRedBlocks,
                     1.0 / (double)n, out);
  return check_launch("absdiff_mean");
}

extern "C" int ainp_bce_logits(const float* x, int64_t n, float target, float* grad,
                               float grad_scale, void* workspace, double* out_mean,
                               void* stream) {
  if (!x || n < 1 || !workspace || !out_mean) return record_msg("ainp_bce_logits: bad argument");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(bce_logits_partial_kernel, dim3(kRedBlocks), dim3(256), 0, s, x, n, target,
                     part, grad, grad_scale);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, part, kRedBlocks,
                     1.0 / (double)n, out_mean);
  return check_launch("bce_logits");
}

extern "C" int ainp_gan_recon_losses(const float* g, const float* o, const float* m, int64_t n,
                                     void* workspace, double* out3, void* stream) {
  if (!g || !o || !m || n < 1 || !workspace || !out3)
    return record_msg("ainp_gan_recon_losses: bad argument");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(gan_recon_partial_kernel, dim3(kRedBlocks), dim3(256), 0, s, g, o, m, n, part);
  hipLaunchKernelGGL(gan_recon_final_kernel, dim3(1), dim3(256), 0, s, part, kRedBlocks, n, out3);
  return check_launch("gan_recon_losses");
}

__global__ __launch_bounds__(256) void gan_recon_sums_kernel(const double* partial, int np,
                                                             double* out5) {
  double tot[5];
  recon_reduce5(partial, np, tot);
  if (threadIdx.x < 5) out5[threadIdx.x] = tot[threadIdx.x];
}

extern "C" int ainp_gan_recon_sums(const float* g, const float* o, const float* m, int64_t n,
                                   void* workspace, double* out5, void* stream) {
  if (!g || !o || !m || n < 1 || !workspace || !out5)
    return record_msg("ainp_gan_recon_sums: bad argument");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(gan_recon_partial_kernel, dim3(kRedBlocks), dim3(256), 0, s, g, o, m, n, part);
  hipLaunchKernelGGL(gan_recon_sums_kernel, dim3(1), dim3(256), 0, s, part, kRedBlocks, out5);
  return check_launch("gan_recon_sums");
}

extern "C" size_t ainp_sn_workspace(int nl, int maxdim) {
  return (size_t)2 * nl * maxdim * sizeof(float);
}

extern "C" int ainp_sn_power(const float* const* w, float* const* u, float* const* v,
                             const int* h, const int* wd, int nl, float eps, void* workspace,
                             int maxdim, float* inv_sigma, int update, void* stream) {
  if (nl < 1 || nl > 8 || !w || !u || !v || !h || !wd || !workspace || !inv_sigma)
    return record_msg("ainp_sn_power: bad argument");
  SnLayers L;
  int maxh = 0, maxw = 0;
  for (int l = 0; l < nl; ++l) {
    if (!w[l] || !u[l] || !v[l] || h[l] < 1 || wd[l] < 1 || h[l] > maxdim || wd[l] > maxdim)
      return record_msg("ainp_sn_power: bad layer");
    L.w[l] = w[l];
    L.u[l] = u[l];
    L.v[l] = v[l];
    L.h[l] = h[l];
    L.wd[l] = wd[l];
    maxh = h[l] > maxh ? h[l] : maxh;
    maxw = wd[l] > maxw ? wd[l] : maxw;
  }
  L.nl = nl;
  float* tv = reinterpret_cast<float*>(workspace);
  float* tu = tv + (size_t)nl * maxdim;
  hipStream_t s = as_stream(stream);
  if (update) {
    hipLaunchKernelGGL(sn_tmv_kernel, dim3((unsigned)cdiv(maxw, SN_TMV_COLS), nl), dim3(256), 0, s, L,
                       tv, maxdim);
    hipLaunchKernelGGL(sn_normalize_v_kernel, dim3(nl), dim3(1024), 0, s, L, tv, maxdim, eps);
  }
  hipLaunchKernelGGL(sn_mv_kernel, dim3(maxh, nl), dim3(256), 0, s, L, tu, maxdim);
  if (update)
    hipLaunchKernelGGL(sn_finish_kernel, dim3(nl), dim3(1024), 0, s, L, tu, maxdim, eps,
                       inv_sigma);
  else
    hipLaunchKernelGGL(sn_sigma_kernel, dim3(nl), dim3(1024), 0, s, L, tu, maxdim, inv_sigma);
  return check_launch("sn_power");
}

extern "C" int ainp_sn_weight_grad(const float* G, int ldg, const float* w_orig, const float* u,
                                   const float* v, const float* inv_sigma, int h, int wd,
                                   void* workspace, float* out, float* out_bias, void* stream) {
  if (!G || !w_orig || !u || !v || !inv_sigma || h < 1 || wd < 1 || !workspace || !out ||
      ldg < wd || (out_bias && ldg < wd + 1))
    return record_msg("ainp_sn_weight_grad: bad argument");
  hipStream_t s = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  const int64_t n = (int64_t)h * wd;
  hipLaunchKernelGGL(sn_gdot_partial_kernel, dim3(kRedBlocks), dim3(256), 0, s, G, ldg, w_orig, wd,
                     n, part);
  hipLaunchKernelGGL(sn_wgrad_apply_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s, G, ldg,
                     part, kRedBlocks, u, v, inv_sigma, h, wd, out, out_bias);
  return check_launch("sn_weight_grad");
}

extern "C" int ainp_im2col_ld(const float* x, int64_t N, int C, int H, int W, int KH, int KW,
                              int stride, int pad, int ones_row, int64_t ldp, float* col,
                              void* stream) {
  if (!x || !col || N < 1 || N > 65535 || C < 1 || KH < 1 || KW < 1 || stride < 1 ||
      ones_row < 0 || ones_row > 1)
    return record_msg("ainp_im2col: bad argument");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  const int64_t Kr = (int64_t)C * KH * KW + ones_row;
  if (Ho < 1 || Wo < 1 || ldp < (int64_t)Ho * Wo || ldp > (1 << 30) || Kr > 65535)
    return record_msg("ainp_im2col: bad shape");
  if (ldp % 4 == 0 && ((uintptr_t)col & 15) == 0)
    hipLaunchKernelGGL(im2col4_kernel, dim3((unsigned)cdiv(ldp / 4, 256),
                                            (unsigned)cdiv(Kr, IM2COL_IK), (unsigned)N),
                       dim3(256), 0, as_stream(stream), x, C, H, W, KH, KW, stride, pad, Ho, Wo,
                       ones_row, (int)ldp, col);
  else
    hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)cdiv(ldp, 256), (unsigned)Kr, (unsigned)N),
                       dim3(256), 0, as_stream(stream), x, (int)N, C, H, W, KH, KW, stride, pad,
                       Ho, Wo, ones_row, (int)ldp, col);
  return check_launch("im2col");
}

extern "C" int ainp_im2col(const float* x, int64_t N, int C, int H, int W, int KH, int KW,
                           int stride, int pad, int ones_row, float* col, void* stream) {
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  return ainp_im2col_ld(x, N, C, H, W, KH, KW, stride, pad, ones_row, (int64_t)Ho * Wo, col,
                        stream);
}

extern "C" int ainp_col2im_ld(const float* dcol, int64_t N, int C, int H, int W, int KH,
                              int KW, int stride, int pad, int64_t ldp, float* dx, void* stream) {
  if (!dcol || !dx || N < 1 || C < 1 || KH < 1 || KW < 1 || stride < 1)
    return record_msg("ainp_col2im: bad argument");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (ldp < (int64_t)Ho * Wo) return record_msg("ainp_col2im: ldp < Ho*Wo");
  const int64_t total = N * C * (int64_t)H * W;
  if (KH == 4 && KW == 4 && (stride == 1 || stride == 2) && N * C <= 65535 &&
      (int64_t)H * W < (1 << 30)) {
    const dim3 grid((unsigned)cdiv((int64_t)H * W, 256), (unsigned)(N * C));
    if (stride == 2)
      hipLaunchKernelGGL((col2im_ks_kernel<4, 2>), grid, dim3(256), 0, as_stream(stream), dcol,
                         C, H, W, pad, Ho, Wo, ldp, dx);
    else
      hipLaunchKernelGGL((col2im_ks_kernel<4, 1>), grid, dim3(256), 0, as_stream(stream), dcol,
                         C, H, W, pad, Ho, Wo, ldp, dx);
    return check_launch("col2im");
  }
  hipLaunchKernelGGL(col2im_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), dcol, (int)N, C, H, W, KH, KW, stride, pad, Ho, Wo, ldp,
                     dx);
  return check_launch("col2im");
}

extern "C" int ainp_col2im(const float* dcol, int64_t N, int C, int H, int W, int KH, int KW,
                           int stride, int pad, float* dx, void* stream) {
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  return ainp_col2im_ld(dcol, N, C, H, W, KH, KW, stride, pad, (int64_t)Ho * Wo, dx, stream);
}

extern "C" int ainp_leaky_bwd_ld(const float* g, const float* y, int64_t rows, int64_t P,
                                 float slope, int64_t ldo, float* out, void* stream) {
  if (!g || !y || !out || rows < 1 || rows > 65535 || P < 1 || ldo < P || ldo > (1 << 30))
    return record_msg("ainp_leaky_bwd_ld: bad argument");
  hipLaunchKernelGGL(leaky_bwd_ld_kernel, dim3((unsigned)cdiv(ldo, 256), (unsigned)rows),
                     dim3(256), 0, as_stream(stream), g, y, (int)P, slope, (int)ldo, out);
  return check_launch("leaky_bwd_ld");
}

extern "C" int ainp_leaky_bwd(const float* g, const float* y, int64_t n, float slope, float* out,
                              void* stream) {
  if (!g || !y || !out || n < 1) return record_msg("ainp_leaky_bwd: bad argument");
  hipLaunchKernelGGL(leaky_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), g, y, n, slope, out);
  return check_launch("leaky_bwd");
}

extern "C" int ainp_mul(const float* a, const float* b, int64_t n, float* out, void* stream) {
  if (!a || !b || !out || n < 1) return record_msg("ainp_mul: bad argument");
  hipLaunchKernelGGL(mul_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream),
                     a, b, n, out);
  return check_launch("mul");
}

extern "C" int ainp_channel_sum(const float* m, int64_t N, int C, int64_t HW, float* out,
                                void* stream) {
  if (!m || !out || N < 1 || C < 1 || HW < 1) return record_msg("ainp_channel_sum: bad argument");
  hipLaunchKernelGGL(channel_sum_kernel, dim3((unsigned)cdiv(N * HW, 256)), dim3(256), 0,
                     as_stream(stream), m, N, C, HW, out);
  return check_launch("channel_sum");
}
