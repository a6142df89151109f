// dconv16.hip — the spectral-norm Discriminator's backward in the bf16
// configurations (BASELINE C4 / C5): networks.py:375-409 convs (k4, stride 2
// / 1, pad 1) differentiated for the D step of models/GAN/train.py:341-378.
//
// Per layer, with g = dL/d(conv output) [N][Cout][Ho][Wo]:
//   d_prep16     LeakyReLU backward (of the layer's own activation) fused with
//                the bf16 cast into the two operand layouts below, summing the
//                split-K slabs of the layer above's data gradient on the way:
//                  gA [Cout][ldA]  pixel-contiguous (q = n*Ho*Wo + oy*Wo + ox)
//                  gT [N*Ho*Wo][Cout] channel-contiguous (NHWC)
//   im2col16     the layer input's columns, bf16 [Cin*k*k + 1][ldA] (last row
//                ones: the bias gradient), pixel-contiguous
//   weight grad  [dW | db] = gA . col^T: one k-contiguous bf16 GEMM over all N
//                images (gemm16.hip, split-K), into sn_weight_grad as before
//   dgrad16      the data gradient as an implicit GEMM over gT: the transposed
//                convolution split into stride^2 output parity classes, each a
//                stride-1 convolution of g with a (k/s) x (k/s) sub-kernel, so no
//                MFMA work multiplies the zeros of the upsampled gradient; K =
//                taps x Cout with 32 channels of one tap per K-tile (one 64-byte
//                NHWC run per pixel), 1/sigma applied in the epilogue.
// The fp32 path (im2col + x6 GEMM + col2im in gan.hip) stays the fp32 one.
#include "common.h"

namespace ainp {
namespace d16 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint16_t to_bf16(float v) {
  return __builtin_bit_cast(uint16_t, (__bf16)v);
}

// k-values a source of C channels x KK taps occupies in a weight row (tiles of 32)
__host__ __device__ inline int seg32(int C, int KK) {
  return (C & 31) ? (KK * C + 31) / 32 * 32 : KK * C;
}

// sum_z g[z] (* leaky') -> gA [C][ldA] (zero past N*P), gT [N*P][C]
__global__ __launch_bounds__(256) void d_prep16_kernel(const float* __restrict__ g, int nslab,
                                                       int64_t slab_stride,
                                                       const float* __restrict__ y, float slope,
                                                       int C, int64_t P, int64_t NP,
                                                       uint16_t* __restrict__ gA, int64_t ldA,
                                                       uint16_t* __restrict__ gT) {
  __shared__ uint16_t tile[64][66];   // [q][c]
  const int64_t q0 = (int64_t)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t q = q0 + tx;
  int64_t base = 0;
  if (q < NP) {
    const int64_t n = q / P;
    base = n * C * P + (q - n * P);
  }
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i;
    float v = 0.f;
    if (c < C && q < NP) {
      const int64_t idx = base + (int64_t)c * P;
      for (int z = 0; z < nslab; ++z) v += g[z * slab_stride + idx];
      if (y && !(y[idx] > 0.f)) v *= slope;
    }
    const uint16_t b = to_bf16(v);
    if (c < C && q < ldA) gA[(int64_t)c * ldA + q] = b;
    tile[tx][i] = b;
  }
  if (!gT) return;
  __syncthreads();
#pragma unroll 4
  for (int i = ty; i < 64; i += 4) {
    const int64_t qq = q0 + i;
    const int c = c0 + tx;
    if (qq < NP && c < C) gT[qq * C + c] = tile[i][tx];
  }
}

// x [N][C][H][W] fp32 -> col [C*KK (+1)][ldA] bf16, q = n*Ho*Wo + oy*Wo + ox,
// zero past N*Ho*Wo.  A thread owns two consecutive q of one input channel
// and writes all KK taps (4-byte stores, 256 contiguous bytes per wave and
// row); the window reads of neighbouring lanes overlap in L1.  blockIdx.y ==
// C is the ones row.
__global__ __launch_bounds__(256) void im2col16_kernel(const float* __restrict__ x, int C, int H,
                                                       int W, int KH, int KW, int stride, int pad,
                                                       int Ho, int Wo, int64_t NP, int ones_row,
                                                       uint16_t* __restrict__ col, int64_t ldA) {
  const int64_t q0 = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (q0 >= ldA) return;
  const int ci = blockIdx.y;
  const int KK = KH * KW;
  if (ci == C) {
    const uint32_t lo = q0 < NP ? 0x3F80u : 0u, hi = q0 + 1 < NP ? 0x3F80u : 0u;
    *reinterpret_cast<uint32_t*>(col + (int64_t)C * KK * ldA + q0) = lo | (hi << 16);
    return;
  }
  const int64_t P = (int64_t)Ho * Wo;
  const float* xp[2];
  int by[2], bx[2];
  bool v[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int64_t q = q0 + e;
    v[e] = q < NP;
    const int64_t n = v[e] ? q / P : 0;
    const int r = v[e] ? (int)(q - n * P) : 0;
    const int oy = r / Wo, ox = r - oy * Wo;
    xp[e] = x + (n * C + ci) * H * W;
    by[e] = oy * stride - pad;
    bx[e] = ox * stride - pad;
  }
  uint16_t* cp = col + (int64_t)ci * KK * ldA + q0;
  for (int ky = 0; ky < KH; ++ky)
    for (int kx = 0; kx < KW; ++kx) {
      uint32_t h[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int iy = by[e] + ky, ix = bx[e] + kx;
        h[e] = (v[e] && iy >= 0 && iy < H && ix >= 0 && ix < W)
                   ? to_bf16(xp[e][(int64_t)iy * W + ix]) : 0u;
      }
      *reinterpret_cast<uint32_t*>(cp + (int64_t)(ky * KW + kx) * ldA) = h[0] | (h[1] << 16);
    }
}

// Parity class (py, px) of a stride-s transposed conv: output rows y = s*i + py
// read gradient rows i + dy0 + a, a < nt = k/s, through kernel row
// ky = ky0 + s*(nt-1-a), ky0 = (py+pad) % s.
struct Cls {
  int py, px, ky0, kx0, dy0, dx0;
};
__host__ __device__ inline Cls make_cls(int cls, int s, int k, int pad) {
  Cls c;
  c.py = cls / s;
  c.px = cls - c.py * s;
  const int nt = k / s;
  c.ky0 = (c.py + pad) % s;
  c.kx0 = (c.px + pad) % s;
  c.dy0 = (c.py + pad - c.ky0 - s * (nt - 1)) / s;
  c.dx0 = (c.px + pad - c.kx0 - s * (nt - 1)) / s;
  return c;
}

// wd [s*s][Cin][Kc] bf16, Kc = seg32(Cout, nt*nt), k = (a*nt + b)*Cout + co ->
// w[co][ci][ky(a)][kx(b)] (zero in the pad)
__global__ void dgrad16_weight_kernel(const float* __restrict__ w, int Cout, int Cin, int k, int s,
                                      int pad, uint16_t* __restrict__ wd) {
  const int nt = k / s, Kc = seg32(Cout, nt * nt);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)s * s * Cin * Kc) return;
  const int kk = (int)(t % Kc);
  const int64_t r = t / Kc;
  const int ci = (int)(r % Cin), cls = (int)(r / Cin);
  const int tap = kk / Cout, co = kk - tap * Cout;
  float v = 0.f;
  if (tap < nt * nt) {
    const Cls c = make_cls(cls, s, k, pad);
    const int a = tap / nt, b = tap - a * nt;
    const int ky = c.ky0 + s * (nt - 1 - a), kx = c.kx0 + s * (nt - 1 - b);
    v = w[(((int64_t)co * Cin + ci) * k + ky) * k + kx];
  }
  wd[t] = to_bf16(v);
}

struct DgradArgs {
  const uint16_t* gT;   // [N][Ho][Wo][Cout]
  const uint16_t* wd;   // [s*s][Cin][Kc]
  const float* scale;   // 1/sigma (device scalar) or null
  float* out;           // [nsplit][N][Cin][H][W]
  int64_t slab;         // elements per split slab
  int N, Cout, Ho, Wo, Cin, H, W, k, s, pad, ktiles_per_split;
  // PREP epilogue (ainp_dgrad16_prep, nsplit 1): d_prep16_kernel's outputs of
  // dx instead of dx -- times LeakyReLU'(y) (y == null: none), bf16 gA
  // [Cin][ldA] (q = n*H*W + pixel) and, if gTo, gTo [N*H*W][Cin]
  const float* y;
  float slope;
  uint16_t* gA;
  int64_t ldA;
  uint16_t* gTo;
};

// grid (pixel tiles of the largest class, Cin / BM, s*s * nsplit)
template <int BM, bool GATHER, bool PREP = false>
__global__ __launch_bounds__(256, 4) void dgrad16_kernel(DgradArgs d) {
  constexpr int XBK = 32;
  constexpr int BN = 16384 / BM;
  constexpr int WN = BN / 64;
  constexpr int RS = XBK * 2 + 16;
  __shared__ __attribute__((aligned(16))) unsigned char sA[BM * RS];
  __shared__ __attribute__((aligned(16))) unsigned char sB[BN * RS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncls = d.s * d.s;
  const int cls = blockIdx.z % ncls, split = blockIdx.z / ncls;
  const Cls c = make_cls(cls, d.s, d.k, d.pad);
  const int nt = d.k / d.s;
  const int Hc = (d.H - c.py + d.s - 1) / d.s, Wc = (d.W - c.px + d.s - 1) / d.s;
  const int64_t HWc = (int64_t)Hc * Wc;
  const int64_t NPc = (int64_t)d.N * HWc;
  const int64_t px0 = (int64_t)blockIdx.x * BN;
  if (px0 >= NPc) return;   // smaller classes: whole block idle (uniform)
  const int co0 = blockIdx.y * BM;   // rows of the GEMM = input channels ci
  const int Kc = seg32(d.Cout, nt * nt);
  const int nkt = Kc / XBK;
  const int kt_begin = min(split * d.ktiles_per_split, nkt);
  const int kt_end = min(kt_begin + d.ktiles_per_split, nkt);

  // loads: lanes 4r..4r+3 read the four 16-byte chunks of one row's 64-byte
  // K-tile slice, rows r + 64 i (gan.hip conv_gen_nhwc16_kernel)
  constexpr int NBI = BN / 64, NAI = BM / 64;
  const int ch = tid & 3, rr = tid >> 2;
  int n_[NBI], byx_[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    const int64_t pix = px0 + rr + 64 * i;
    n_[i] = -1;
    byx_[i] = 0;
    if (pix < NPc) {
      n_[i] = (int)(pix / HWc);
      const int r = (int)(pix - (int64_t)n_[i] * HWc);
      const int ii = r / Wc, jj = r - ii * Wc;
      byx_[i] = ((ii + c.dy0) << 16) | ((jj + c.dx0) & 0xffff);
    }
  }
  const uint16_t* wrow = d.wd + ((int64_t)cls * d.Cin + co0 + rr) * Kc + 8 * ch;
  const int arows = d.Cin - co0 - rr;

  uint4 ra[NAI], rb[NBI];
  auto fetch = [&](int kt) {
    const int k0 = kt * XBK;
#pragma unroll
    for (int i = 0; i < NAI; ++i)
      ra[i] = 64 * i < arows ? *reinterpret_cast<const uint4*>(wrow + (int64_t)64 * i * Kc + k0)
                             : make_uint4(0, 0, 0, 0);
    if (GATHER) return;   // the logit layer's 1-channel gradient: gather_commit
    const int tap = k0 / d.Cout, c0k = k0 - tap * d.Cout;
    const int a = tap / nt, b = tap - a * nt;
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int iy = (byx_[i] >> 16) + a, ix = (int)(short)(byx_[i] & 0xffff) + b;
      const bool inb = n_[i] >= 0 && iy >= 0 && iy < d.Ho && ix >= 0 && ix < d.Wo;
      const uint16_t* src =
          d.gT + (((int64_t)n_[i] * d.Ho + iy) * d.Wo + ix) * d.Cout + c0k + 8 * ch;
      rb[i] = inb ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
    }
  };
  // Cout % 32 != 0: element gather straight into the LDS image (gan.hip
  // conv_gen_nhwc16_kernel's gather_commit)
  auto gather_commit = [&](int kt) {
    constexpr int BRg = XBK * BN / 256;
    const int k0 = kt * XBK;
    const int row = tid % BN, kq = tid / BN;
    const int64_t pix = px0 + row;
    int n = -1, by = 0, bx = 0;
    if (pix < NPc) {
      n = (int)(pix / HWc);
      const int r = (int)(pix - (int64_t)n * HWc);
      const int ii = r / Wc, jj = r - ii * Wc;
      by = ii + c.dy0;
      bx = jj + c.dx0;
    }
#pragma unroll 1
    for (int j0 = 0; j0 < BRg; j0 += 8) {
      uint32_t g[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = k0 + kq * BRg + j0 + j;
        const int tap = kk / d.Cout, co = kk - tap * d.Cout;
        const int a = tap / nt, b = tap - a * nt;
        const int iy = by + a, ix = bx + b;
        uint32_t v = 0;
        if (n >= 0 && tap < nt * nt && iy >= 0 && iy < d.Ho && ix >= 0 && ix < d.Wo)
          v = d.gT[(((int64_t)n * d.Ho + iy) * d.Wo + ix) * d.Cout + co];
        if (j & 1) g[j >> 1] |= v << 16;
        else g[j >> 1] = v;
      }
      *reinterpret_cast<uint4*>(sB + row * RS + (kq * BRg + j0) * 2) =
          make_uint4(g[0], g[1], g[2], g[3]);
    }
  };
  auto commit = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NAI; ++i)
      *reinterpret_cast<uint4*>(sA + (rr + 64 * i) * RS + 16 * ch) = ra[i];
    if (GATHER) {
      gather_commit(kt);
      return;
    }
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
    commit(kt);
    __syncthreads();
    if (kt + 1 < kt_end) fetch(kt + 1);
#pragma unroll
    for (int st = 0; st < XBK / 16; ++st) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uint4*>(sA + (wm * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh));
        fb[i] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const uint4*>(sB + (wn * 64 + i * 32 + l31) * RS + 32 * st + 16 * lh));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: D[row ci][col pixel]; pixel (n, i, j) of the class -> (s*i+py, s*j+px)
  const float sc = d.scale ? *d.scale : 1.f;
  float* ob = d.out + (int64_t)split * d.slab;
  const int64_t HW = (int64_t)d.H * d.W;
  if (PREP) {
    // rows ci0 .. ci0+3 of a lane's accumulators are 4 consecutive channels:
    // one 8-byte gTo store per 4 values (Cin % 4 == 0, checked on the host)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t pg = px0 + wn * 64 + 32 * j + l31;
      if (pg >= NPc) continue;
      const int pn = (int)(pg / HWc);
      const int r = (int)(pg - (int64_t)pn * HWc);
      const int i = r / Wc, jj = r - i * Wc;
      const int64_t pix = (int64_t)(d.s * i + c.py) * d.W + d.s * jj + c.px;
      const int64_t q = (int64_t)pn * HW + pix;
      const float* yb = d.y ? d.y + (int64_t)pn * d.Cin * HW + pix : nullptr;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int ci0 = co0 + wm * 64 + 32 * ii + 8 * r4 + 4 * lh;
          if (ci0 >= d.Cin) continue;
          uint32_t h[2];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[ii][j][4 * r4 + e] * sc;
            if (yb && !(yb[(int64_t)(ci0 + e) * HW] > 0.f)) v *= d.slope;
            const uint16_t b = to_bf16(v);
            d.gA[(int64_t)(ci0 + e) * d.ldA + q] = b;
            if (e & 1) h[e >> 1] |= (uint32_t)b << 16;
            else h[e >> 1] = b;
          }
          if (d.gTo) *reinterpret_cast<uint2*>(d.gTo + q * d.Cin + ci0) = make_uint2(h[0], h[1]);
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t pg = px0 + wn * 64 + 32 * j + l31;
    if (pg >= NPc) continue;
    const int pn = (int)(pg / HWc);
    const int r = (int)(pg - (int64_t)pn * HWc);
    const int i = r / Wc, jj = r - i * Wc;
    float* o = ob + (int64_t)pn * d.Cin * HW + (int64_t)(d.s * i + c.py) * d.W + d.s * jj + c.px;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int ci = co0 + wm * 64 + 32 * ii + (rr & 3) + 8 * (rr >> 2) + 4 * lh;
        if (ci < d.Cin) o[(int64_t)ci * HW] = acc[ii][j][rr] * sc;
      }
  }
}

// Weight gradient of a Cout = 1 conv (the discriminator's logit conv,
// networks.py:403-406): [dW | db] [Cin*KK + 1] with
//   dW[ci][ky][kx] = sum_q g[q] x[n][ci][oy*s+ky-p][ox*s+kx-p],  db = sum_q g[q],
// g = sum of nslab slabs (x LeakyReLU'(y)) as in d_prep16_kernel.  With
// Cout = 1 the im2col16 + GEMM route materialises Cin*KK*N*P bf16 columns
// (299 MB at C4) for a GEMV; here block (ci, z) keeps its KK tap sums over
// pixel slice z in registers (fp32 products, the input read once through L1,
// WC1_U pixels' loads in flight per iteration) and writes them to partial row z;
// wgrad_cout1_sum adds the WC1_S rows in fixed order (bit-reproducible).
// Channel index Cin is the bias.
constexpr int WC1_S = 8, WC1_U = 2;   // pixel slices per channel, pixels in flight per thread

template <int K>
__global__ __launch_bounds__(256) void wgrad_cout1_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ g, int nslab,
                                                          int64_t slab_stride,
                                                          const float* __restrict__ y, float slope,
                                                          int Cin, int H, int W, int Ho, int Wo,
                                                          int stride, int pad, int64_t NP,
                                                          float* __restrict__ part) {
  constexpr int KK = K * K;
  __shared__ float red[4][KK];
  const int ci = blockIdx.x, z = blockIdx.y;
  const int P = Ho * Wo;   // NP < 2^31 (host check): 32-bit index arithmetic
  const int chunk = (int)((NP + WC1_S - 1) / WC1_S);
  const int qa = z * chunk, qb = min((int)NP, qa + chunk);
  float acc[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) acc[t] = 0.f;
  for (int q0 = qa + threadIdx.x; q0 < qb; q0 += 256 * WC1_U) {
    float gv[WC1_U], xv[WC1_U][KK];
#pragma unroll
    for (int e = 0; e < WC1_U; ++e) {
      const int q = q0 + 256 * e;
      const bool vq = q < qb;
      float gq = 0.f;
      if (vq) {
        for (int zz = 0; zz < nslab; ++zz) gq += g[zz * slab_stride + q];
        if (y && !(y[q] > 0.f)) gq *= slope;
      }
      gv[e] = gq;
      if (ci == Cin) continue;
      const int n = vq ? q / P : 0;
      const int r = vq ? q - n * P : 0;
      const int oy = r / Wo, ox = r - oy * Wo;
      const int by = vq ? oy * stride - pad : -(1 << 28), bx = ox * stride - pad;
      const float* xp = x + ((int64_t)n * Cin + ci) * (int64_t)H * W;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int iy = by + ky;
        const bool vy = iy >= 0 && iy < H;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int ix = bx + kx;
          xv[e][ky * K + kx] = (vy && ix >= 0 && ix < W) ? xp[(int64_t)iy * W + ix] : 0.f;
        }
      }
    }
    if (ci == Cin) {
#pragma unroll
      for (int e = 0; e < WC1_U; ++e) acc[0] += gv[e];
      continue;
    }
#pragma unroll
    for (int e = 0; e < WC1_U; ++e)
#pragma unroll
      for (int t = 0; t < KK; ++t) acc[t] = fmaf(gv[e], xv[e][t], acc[t]);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) red[wv][t] = v;
  }
  __syncthreads();
  const int64_t row = (int64_t)Cin * KK + 1;
  if (threadIdx.x < KK) {
    const int t = threadIdx.x;
    const float v = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    if (ci < Cin) part[z * row + (int64_t)ci * KK + t] = v;
    else if (t == 0) part[z * row + (int64_t)Cin * KK] = v;
  }
}

__global__ __launch_bounds__(256) void wgrad_cout1_sum(const float* __restrict__ part, int64_t row,
                                                       float* __restrict__ gw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= row) return;
  float v = 0.f;
#pragma unroll
  for (int z = 0; z < WC1_S; ++z) v += part[z * row + i];
  gw[i] = v;
}

}  // namespace d16
}  // namespace ainp

using namespace ainp;

extern "C" int ainp_d_prep16(const float* g, int nslab, int64_t slab_stride, const float* y,
                             float slope, int64_t N, int C, int64_t P, uint16_t* gA, int64_t ldA,
                             uint16_t* gT, void* stream) {
  if (!g || nslab < 1 || (nslab > 1 && slab_stride < N * C * P) || N < 1 || C < 1 || P < 1 ||
      !gA || ldA < N * P || cdiv(C, 64) > 65535)
    return record_msg("ainp_d_prep16: bad argument");
  hipLaunchKernelGGL(d16::d_prep16_kernel, dim3((unsigned)cdiv(ldA, 64), (unsigned)cdiv(C, 64)),
                     dim3(256), 0, as_stream(stream), g, nslab, slab_stride, y, slope, C, P, N * P,
                     gA, ldA, gT);
  return check_launch("d_prep16");
}

extern "C" int ainp_im2col16(const float* x, int64_t N, int C, int H, int W, int KH, int KW,
                             int stride, int pad, int ones_row, uint16_t* col, int64_t ldA,
                             void* stream) {
  if (!x || !col || N < 1 || C < 1 || KH < 1 || KW < 1 || stride < 1 || pad < 0 || ldA % 8 ||
      ((uintptr_t)col & 15))
    return record_msg("ainp_im2col16: bad argument (ldA % 8, 16-byte aligned)");
  // (ldA % 8: the rows are the 16-byte-aligned k-contiguous operand of ainp_gemm_bf16nt)
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  const int64_t NP = N * Ho * Wo;
  const int Kr = C * KH * KW + (ones_row ? 1 : 0);
  if (Ho < 1 || Wo < 1 || ldA < NP || Kr > 65535) return record_msg("ainp_im2col16: bad shape");
  hipLaunchKernelGGL(d16::im2col16_kernel,
                     dim3((unsigned)cdiv(ldA / 2, 256), (unsigned)(C + (ones_row ? 1 : 0))),
                     dim3(256), 0, as_stream(stream), x, C, H, W, KH, KW, stride, pad, Ho, Wo, NP,
                     ones_row, col, ldA);
  return check_launch("im2col16");
}

extern "C" int ainp_wgrad_cout1(const float* x, const float* g, int nslab, int64_t slab_stride,
                                const float* y, float slope, int64_t N, int Cin, int H, int W,
                                int k, int stride, int pad, float* gw, float* ws, void* stream) {
  if (!x || !g || !gw || !ws || nslab < 1 || N < 1 || Cin < 1 || stride < 1 || pad < 0 ||
      (k != 3 && k != 4) || Cin >= 65535)
    return record_msg("ainp_wgrad_cout1: bad argument (k 3 or 4, workspace)");
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t NP = N * Ho * Wo;
  if (Ho < 1 || Wo < 1 || (nslab > 1 && slab_stride < NP) || NP >= (int64_t)1 << 31)
    return record_msg("ainp_wgrad_cout1: bad shape (N*Ho*Wo < 2^31)");
  const dim3 grid((unsigned)(Cin + 1), d16::WC1_S);
  hipStream_t s = as_stream(stream);
  if (k == 4)
    hipLaunchKernelGGL(d16::wgrad_cout1_kernel<4>, grid, dim3(256), 0, s, x, g, nslab,
                       slab_stride, y, slope, Cin, H, W, Ho, Wo, stride, pad, NP, ws);
  else
    hipLaunchKernelGGL(d16::wgrad_cout1_kernel<3>, grid, dim3(256), 0, s, x, g, nslab,
                       slab_stride, y, slope, Cin, H, W, Ho, Wo, stride, pad, NP, ws);
  const int64_t row = (int64_t)Cin * k * k + 1;
  hipLaunchKernelGGL(d16::wgrad_cout1_sum, dim3((unsigned)cdiv(row, 256)), dim3(256), 0, s, ws, row,
                     gw);
  return check_launch("wgrad_cout1");
}

extern "C" int64_t ainp_wgrad_cout1_workspace(int Cin, int k) {
  return (int64_t)d16::WC1_S * ((int64_t)Cin * k * k + 1) * (int64_t)sizeof(float);
}

// the grid of ainp_dgrad16 / ainp_dgrad16_prep
static int dgrad16_grid(int64_t N, int Cin, int H, int W, int stride, int nsplit, int BM,
                        dim3* grid) {
  const int64_t Hc = cdiv(H, stride), Wc = cdiv(W, stride);   // class (0, 0): the largest
  const int64_t tiles = cdiv(N * Hc * Wc, 16384 / BM);
  const int64_t gz = (int64_t)stride * stride * nsplit;
  if (tiles > 0x7fffffff || gz > 65535) return record_msg("ainp_dgrad16: grid too large");
  *grid = dim3((unsigned)tiles, (unsigned)cdiv(Cin, BM), (unsigned)gz);
  return AINP_OK;
}

extern "C" int ainp_dgrad16_weight(const float* w, int Cout, int Cin, int k, int stride, int pad,
                                   uint16_t* wd, void* stream) {
  if (!w || !wd || Cout < 1 || Cin < 1 || k < 1 || stride < 1 || k % stride || pad < 0 ||
      pad >= k)
    return record_msg("ainp_dgrad16_weight: bad argument (k % stride == 0)");
  const int nt = k / stride;
  const int64_t total = (int64_t)stride * stride * Cin * d16::seg32(Cout, nt * nt);
  hipLaunchKernelGGL(d16::dgrad16_weight_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                     as_stream(stream), w, Cout, Cin, k, stride, pad, wd);
  return check_launch("dgrad16_weight");
}

extern "C" int ainp_dgrad16(const uint16_t* gT, int64_t N, int Cout, int Ho, int Wo,
                            const uint16_t* wd, int Cin, int H, int W, int k, int stride, int pad,
                            const float* scale, float* out, int nsplit, int64_t slab_stride,
                            void* stream) {
  if (!gT || !wd || !out || N < 1 || Cout < 1 || Cin < 1 || k < 1 || stride < 1 ||
      k % stride || pad < 0 || pad >= k || nsplit < 1 || ((uintptr_t)wd & 15) ||
      ((Cout % 32 == 0) && ((uintptr_t)gT & 15)) ||
      (nsplit > 1 && slab_stride < N * Cin * (int64_t)H * W))
    return record_msg("ainp_dgrad16: bad argument");
  if ((H + 2 * pad - k) / stride + 1 != Ho || (W + 2 * pad - k) / stride + 1 != Wo)
    return record_msg("ainp_dgrad16: Ho/Wo do not match the forward conv of H/W");
  const int nt = k / stride;
  const int nkt = d16::seg32(Cout, nt * nt) / 32;
  const int per = (int)cdiv(nkt, nsplit);
  d16::DgradArgs a{gT, wd, scale, out, slab_stride, (int)N, Cout, Ho, Wo, Cin, H, W, k, stride,
                   pad, per, nullptr, 0.f, nullptr, 0, nullptr};
  const int BM = Cin > 64 ? 128 : 64;
  dim3 grid;
  if (const int rc = dgrad16_grid(N, Cin, H, W, stride, nsplit, BM, &grid)) return rc;
  const bool gather = Cout % 32 != 0;
  if (BM == 128 && gather)
    hipLaunchKernelGGL((d16::dgrad16_kernel<128, true>), grid, dim3(256), 0, as_stream(stream), a);
  else if (BM == 128)
    hipLaunchKernelGGL((d16::dgrad16_kernel<128, false>), grid, dim3(256), 0, as_stream(stream), a);
  else if (gather)
    hipLaunchKernelGGL((d16::dgrad16_kernel<64, true>), grid, dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL((d16::dgrad16_kernel<64, false>), grid, dim3(256), 0, as_stream(stream), a);
  return check_launch("dgrad16");
}

extern "C" int ainp_dgrad16_prep(const uint16_t* gT, int64_t N, int Cout, int Ho, int Wo,
                                 const uint16_t* wd, int Cin, int H, int W, int k, int stride,
                                 int pad, const float* scale, const float* y, float slope,
                                 uint16_t* gA, int64_t ldA, uint16_t* gTo, void* stream) {
  const int64_t NP = N * (int64_t)H * W;
  if (!gT || !wd || !gA || N < 1 || Cout < 1 || Cin < 1 || Cin % 4 || k < 1 || stride < 1 ||
      k % stride || pad < 0 || pad >= k || ((uintptr_t)wd & 15) ||
      ((Cout % 32 == 0) && ((uintptr_t)gT & 15)) || ldA < NP || ((uintptr_t)gTo & 7))
    return record_msg("ainp_dgrad16_prep: bad argument (Cin % 4 == 0, ldA >= N*H*W)");
  if ((H + 2 * pad - k) / stride + 1 != Ho || (W + 2 * pad - k) / stride + 1 != Wo)
    return record_msg("ainp_dgrad16_prep: Ho/Wo do not match the forward conv of H/W");
  const int nkt = d16::seg32(Cout, (k / stride) * (k / stride)) / 32;
  d16::DgradArgs a{gT, wd, scale, nullptr, 0, (int)N, Cout, Ho, Wo, Cin, H, W, k, stride,
                   pad, nkt, y, slope, gA, ldA, gTo};
  const int BM = Cin > 64 ? 128 : 64;
  dim3 grid;
  if (const int rc = dgrad16_grid(N, Cin, H, W, stride, 1, BM, &grid)) return rc;
  hipStream_t s = as_stream(stream);
  if (ldA > NP) {   // the zero tail of every gA row
    const hipError_t e = hipMemset2DAsync(gA + NP, (size_t)ldA * 2, 0, (size_t)(ldA - NP) * 2,
                                          (size_t)Cin, s);
    if (e != hipSuccess) return record_error(e, "dgrad16_prep tail");
  }
  const bool gather = Cout % 32 != 0;
  if (BM == 128 && gather)
    hipLaunchKernelGGL((d16::dgrad16_kernel<128, true, true>), grid, dim3(256), 0, s, a);
  else if (BM == 128)
    hipLaunchKernelGGL((d16::dgrad16_kernel<128, false, true>), grid, dim3(256), 0, s, a);
  else if (gather)
    hipLaunchKernelGGL((d16::dgrad16_kernel<64, true, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((d16::dgrad16_kernel<64, false, true>), grid, dim3(256), 0, s, a);
  return check_launch("dgrad16_prep");
}
