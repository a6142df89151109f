// bn.hip — BatchNorm2d (train/eval) + ReLU for [N, C, H, W] activations.
//
// Replaces nn.BatchNorm2d + nn.ReLU of models/CNNBLSTM/model.py:36-59 and the
// permute/reshape layout bridge of model.py:73-74 (the last encoder block's
// output is written straight into the LSTM's [N, T, C*F] layout).
// Statistics are reduced in float64 from per-workgroup partials in a fixed
// order, so results are deterministic run to run.
#include <initializer_list>

#include "common.h"

namespace ainp {

// --------------------------------------------------------------- finalize
// One workgroup per channel: sum the conv epilogue partials
// stats[part][0:C] = sum y, stats[part][C:2C] = sum y^2  ->  sums[c], sums[C+c].
__global__ void bn_stats_reduce_kernel(const double* __restrict__ stats,
                                       int nparts, double* __restrict__ sums,
                                       int C) {
  const int c = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    s += stats[(int64_t)p * 2 * C + c];
    q += stats[(int64_t)p * 2 * C + C + c];
  }
  __shared__ double rs[4], rq[4];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sums[c] = rs[0] + rs[1] + rs[2] + rs[3];
    sums[C + c] = rq[0] + rq[1] + rq[2] + rq[3];
  }
}

// Per channel: mean/var (biased) from the (possibly all-reduced) sums;
// running stats with the unbiased variance (torch BatchNorm2d train mode).
__device__ __forceinline__ void bn_finalize_channel(double sum, double sumsq, int c,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta,
                                                    float* __restrict__ running_mean,
                                                    float* __restrict__ running_var,
                                                    float momentum, float eps, int64_t count,
                                                    float* __restrict__ scale,
                                                    float* __restrict__ shift,
                                                    float* __restrict__ save, int C);

__global__ void bn_finalize_kernel(const double* __restrict__ sums,
                                   const float* __restrict__ gamma,
                                   const float* __restrict__ beta,
                                   float* __restrict__ running_mean,
                                   float* __restrict__ running_var,
                                   float momentum, float eps, int64_t count,
                                   float* __restrict__ scale,
                                   float* __restrict__ shift,
                                   float* __restrict__ save, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // count <= 0: the element count travels with the sums (sums[2C], all-reduced
  // with them by a data-parallel caller, so uneven shards normalise correctly)
  if (count <= 0) count = (int64_t)sums[2 * C];
  bn_finalize_channel(sums[c], sums[C + c], c, gamma, beta, running_mean, running_var, momentum,
                      eps, count, scale, shift, save, C);
}

// bn_stats_reduce_kernel + bn_finalize_kernel in one launch (single process:
// no all-reduce between them): workgroup c reduces channel c's partials and
// its thread 0 finalises the channel -- the same arithmetic, bit for bit.
__global__ void bn_reduce_finalize_kernel(const double* __restrict__ stats, int nparts,
                                          const float* __restrict__ gamma,
                                          const float* __restrict__ beta,
                                          float* __restrict__ running_mean,
                                          float* __restrict__ running_var, float momentum,
                                          float eps, int64_t count, float* __restrict__ scale,
                                          float* __restrict__ shift, float* __restrict__ save,
                                          int C) {
  const int c = blockIdx.x;
  double s = 0.0, q = 0.0;
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
    s += stats[(int64_t)p * 2 * C + c];
    q += stats[(int64_t)p * 2 * C + C + c];
  }
  __shared__ double rs[4], rq[4];
  s = wave_sum_d(s);
  q = wave_sum_d(q);
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rq[threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    bn_finalize_channel(rs[0] + rs[1] + rs[2] + rs[3], rq[0] + rq[1] + rq[2] + rq[3], c, gamma,
                        beta, running_mean, running_var, momentum, eps, count, scale, shift,
                        save, C);
}

__device__ __forceinline__ void bn_finalize_channel(double sum, double sumsq, int c,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta,
                                                    float* __restrict__ running_mean,
                                                    float* __restrict__ running_var,
                                                    float momentum, float eps, int64_t count,
                                                    float* __restrict__ scale,
                                                    float* __restrict__ shift,
                                                    float* __restrict__ save, int C) {
  const double mean = sum / (double)count;
  double var = sumsq / (double)count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * rstd;
  shift[c] = b - (float)mean * g * rstd;
  save[c] = (float)mean;
  save[C + c] = rstd;
  if (running_mean) {
    const double unbiased = count > 1 ? var * (double)count / (double)(count - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

__global__ void bn_eval_affine_kernel(const float* gamma, const float* beta,
                                      const float* rm, const float* rv,
                                      float eps, float* scale, float* shift,
                                      int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float rstd = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  scale[c] = g * rstd;
  shift[c] = b - rm[c] * g * rstd;
}

// --------------------------------------------------------------- tiles
// A tile is 32 (h) x 64 (w) of one (n, c) plane.  NCHW side: lanes along w;
// NTCF side ([n][w][c*H+h]): lanes along h, staged through LDS.
constexpr int TH = 32, TW = 64;

struct TileIdx {
  int n, c, h0, w0;
};
__device__ __forceinline__ TileIdx tile_of(int64_t b, int C, int64_t H,
                                           int64_t W) {
  const int th = (int)((H + TH - 1) / TH), tw = (int)((W + TW - 1) / TW);
  TileIdx t;
  t.w0 = (int)(b % tw) * TW;
  t.h0 = (int)((b / tw) % th) * TH;
  t.c = (int)((b / ((int64_t)tw * th)) % C);
  t.n = (int)(b / ((int64_t)tw * th * C));
  return t;
}

// out = relu(x*scale+shift); NCHW -> NCHW or NCHW -> NTCF
template <bool NTCF>
__global__ __launch_bounds__(256) void bn_relu_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ scale,
    const float* __restrict__ shift, float* __restrict__ out, int C, int64_t H,
    int64_t W) {
  __shared__ float tile[TW][TH + 1];
  const TileIdx ti = tile_of(blockIdx.x, C, H, W);
  const float sc = scale[ti.c], sh = shift[ti.c];
  const int tid = threadIdx.x;
  const float* xp = x + ((int64_t)ti.n * C + ti.c) * H * W;
  if (!NTCF) {
    float* op = out + ((int64_t)ti.n * C + ti.c) * H * W;
    const int tx = tid & 63, ty = tid >> 6;
    for (int i = 0; i < TH / 4; ++i) {
      const int64_t h = ti.h0 + ty + 4 * i, w = ti.w0 + tx;
      if (h < H && w < W) op[h * W + w] = fmaxf(fmaf(xp[h * W + w], sc, sh), 0.f);
    }
  } else {
    const int tx = tid & 63, ty = tid >> 6;
    for (int i = 0; i < TH / 4; ++i) {
      const int hh = ty + 4 * i;
      const int64_t h = ti.h0 + hh, w = ti.w0 + tx;
      float v = 0.f;
      if (h < H && w < W) v = fmaxf(fmaf(xp[h * W + w], sc, sh), 0.f);
      tile[tx][hh] = v;
    }
    __syncthreads();
    // write [n][w][c*H + h], lanes along h
    const int hx = tid & 31, wy = tid >> 5;  // 32 x 8
    const int64_t CH = (int64_t)C * H;
    for (int i = 0; i < TW / 8; ++i) {
      const int ww = wy + 8 * i;
      const int64_t h = ti.h0 + hx, w = ti.w0 + ww;
      if (h < H && w < W) out[((int64_t)ti.n * W + w) * CH + (int64_t)ti.c * H + h] = tile[ww][hx];
    }
  }
}

// Sum tile partials per channel: sums[c] = sum gz, sums[C+c] = sum gz*xhat
__global__ void bn_bwd_sum_kernel(const double* __restrict__ partial, int N,
                                  int C, int tiles_per_plane,
                                  double* __restrict__ sums) {
  const int c = blockIdx.x;
  double s1 = 0.0, s2 = 0.0;
  const int per = N * tiles_per_plane;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const int n = i / tiles_per_plane, t = i % tiles_per_plane;
    const int64_t b = ((int64_t)n * C + c) * tiles_per_plane + t;
    s1 += partial[b * 2];
    s2 += partial[b * 2 + 1];
  }
  __shared__ double r1[4], r2[4];
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  if ((threadIdx.x & 63) == 0) {
    r1[threadIdx.x >> 6] = s1;
    r2[threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    s1 = r1[0] + r1[1] + r1[2] + r1[3];
    s2 = r2[0] + r2[1] + r2[2] + r2[3];
    sums[c] = s1;
    sums[C + c] = s2;
  }
}

// Pre-BatchNorm input y in fp32 or bf16 storage (YB16, AINP_BN_Y16: the bf16
// configuration's conv outputs, AINP_CONV_Y16); e = element index (even for
// the pair load).
template <bool YB16>
__device__ __forceinline__ float2 ld_y2(const float* y, int64_t e) {
  if constexpr (YB16) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(y) + e);
    return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
  } else {
    return *reinterpret_cast<const float2*>(y + e);
  }
}
template <bool YB16>
__device__ __forceinline__ float ld_y1(const float* y, int64_t e) {
  if constexpr (YB16)
    return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(y)[e] << 16);
  else
    return y[e];
}

// BatchNorm-backward output stores: fp32, or bf16 (GY16, nearest-even: the
// bf16 configuration's gy, which its consumers round to bf16 anyway)
template <bool GY16>
__device__ __forceinline__ void gy_st2(void* gy, int64_t e, float a, float b) {   // e even
  if constexpr (GY16) {
    const uint32_t lo = __builtin_bit_cast(uint16_t, (__bf16)a);
    const uint32_t hi = __builtin_bit_cast(uint16_t, (__bf16)b);
    *reinterpret_cast<uint32_t*>(reinterpret_cast<uint16_t*>(gy) + e) = lo | (hi << 16);
  } else {
    *reinterpret_cast<float2*>(reinterpret_cast<float*>(gy) + e) = make_float2(a, b);
  }
}
template <bool GY16>
__device__ __forceinline__ void gy_st1(void* gy, int64_t e, float a) {
  if constexpr (GY16)
    reinterpret_cast<uint16_t*>(gy)[e] = __builtin_bit_cast(uint16_t, (__bf16)a);
  else
    reinterpret_cast<float*>(gy)[e] = a;
}

// ---------------------------------------------------------- flat NCHW path
// g and y both NCHW: a block owns BN_CHUNK contiguous elements of one (n, c)
// plane -- float2 loads/stores straight from HBM, no LDS staging.  The
// partial layout [n][c][chunk] is what bn_bwd_sum_kernel reduces.
constexpr int BN_CHUNK = 4096;

template <bool VEC, bool YB16 = false>
__global__ __launch_bounds__(256) void bn_relu_bwd_reduce_flat(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ save, double* __restrict__ partial,
    int C, int64_t HW, int chunks) {
  __shared__ double red[2][4];
  const int64_t plane = blockIdx.x / chunks;
  const int ch = blockIdx.x % chunks;
  const int c = (int)(plane % C);
  const int64_t o0 = (int64_t)ch * BN_CHUNK;
  const int len = (int)((HW - o0) < BN_CHUNK ? (HW - o0) : BN_CHUNK);
  const float* gp = g + plane * HW + o0;
  const int64_t yo = plane * HW + o0;
  const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    const float2* g2 = reinterpret_cast<const float2*>(gp);
#pragma unroll
    for (int i = 0; i < BN_CHUNK / 512; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (2 * e < len) {
        const float2 gv = g2[e], yv = ld_y2<YB16>(y, yo + 2 * e);
        const float gz0 = fmaf(yv.x, sc, sh) > 0.f ? gv.x : 0.f;
        const float gz1 = fmaf(yv.y, sc, sh) > 0.f ? gv.y : 0.f;
        s1 += gz0 + gz1;
        s2 += gz0 * ((yv.x - mean) * rstd) + gz1 * ((yv.y - mean) * rstd);
      }
    }
  } else {
    for (int e = threadIdx.x; e < len; e += 256) {
      const float yv = ld_y1<YB16>(y, yo + e);
      const float gz = fmaf(yv, sc, sh) > 0.f ? gp[e] : 0.f;
      s1 += gz;
      s2 += gz * ((yv - mean) * rstd);
    }
  }
  const double d1 = wave_sum_d((double)s1), d2 = wave_sum_d((double)s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = d1;
    red[1][threadIdx.x >> 6] = d2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[(int64_t)blockIdx.x * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partial[(int64_t)blockIdx.x * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

template <bool VEC, bool GY16 = false, bool YB16 = false>
__global__ __launch_bounds__(256) void bn_relu_bwd_apply_flat(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ save, const double* __restrict__ sums, void* __restrict__ gy,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int C, int64_t HW, int chunks,
    double inv_count) {
  if (blockIdx.x < (unsigned)C && threadIdx.x == 0) {
    if (dbeta) dbeta[blockIdx.x] = (float)sums[blockIdx.x];
    if (dgamma) dgamma[blockIdx.x] = (float)sums[C + blockIdx.x];
  }
  const int64_t plane = blockIdx.x / chunks;
  const int ch = blockIdx.x % chunks;
  const int c = (int)(plane % C);
  const int64_t o0 = (int64_t)ch * BN_CHUNK;
  const int len = (int)((HW - o0) < BN_CHUNK ? (HW - o0) : BN_CHUNK);
  const int64_t off = plane * HW + o0;
  const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
  const float k = (gamma ? gamma[c] : 1.f) * rstd;
  const double ic = inv_count > 0.0 ? inv_count : 1.0 / sums[2 * C];   // see bn_finalize
  const float m1 = (float)(sums[c] * ic);
  const float m2 = (float)(sums[C + c] * ic);
  if (VEC) {
    const float2* g2 = reinterpret_cast<const float2*>(g + off);
#pragma unroll
    for (int i = 0; i < BN_CHUNK / 512; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (2 * e < len) {
        const float2 gv = g2[e], yv = ld_y2<YB16>(y, off + 2 * e);
        const float gz0 = fmaf(yv.x, sc, sh) > 0.f ? gv.x : 0.f;
        const float gz1 = fmaf(yv.y, sc, sh) > 0.f ? gv.y : 0.f;
        gy_st2<GY16>(gy, off + 2 * e, k * (gz0 - m1 - ((yv.x - mean) * rstd) * m2),
                     k * (gz1 - m1 - ((yv.y - mean) * rstd) * m2));
      }
    }
  } else {
    for (int e = threadIdx.x; e < len; e += 256) {
      const float yv = ld_y1<YB16>(y, off + e);
      const float gz = fmaf(yv, sc, sh) > 0.f ? g[off + e] : 0.f;
      gy_st1<GY16>(gy, off + e, k * (gz - m1 - ((yv - mean) * rstd) * m2));
    }
  }
}



// ---------------------------------------------------- channel-last path
// Round 5: g, y and gy channel-last ([N][H][W][C], C a multiple of 8): a
// thread owns 8 consecutive channels (one or two 16-byte loads per operand)
// of every (256 / (C/8))-th pixel of its block's range, so its per-channel
// constants stay in registers.  Partials [block][2C] (sum gz, sum gz*xhat),
// summed in fixed order by bn_cl_partials_sum.
constexpr int BNC_PIX = 2048;   // pixels per reduce block

template <bool B16>
__device__ __forceinline__ void bnc_ld8(const void* p, int64_t e, float (&v)[8]) {
  if constexpr (B16) {
    const uint4 q = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p) + e);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + e);
    const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + e + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

template <int C, bool GB16, bool YB16>
__global__ __launch_bounds__(256) void bn_relu_bwd_reduce_cl(
    const void* __restrict__ g, const void* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ save, double* __restrict__ partial,
    int64_t P) {
  constexpr int G = C / 8, PPI = 256 / G;
  __shared__ double red[4][2 * C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = tid % G;
  float sc[8], sh[8], mu[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int ch = 8 * grp + c;
    sc[c] = scale[ch];
    sh[c] = shift[ch];
    mu[c] = save[ch];
    rs[c] = save[C + ch];
    s1[c] = s2[c] = 0.f;
  }
  const int64_t p0 = (int64_t)blockIdx.x * BNC_PIX + tid / G;
#pragma unroll 4
  for (int it = 0; it < BNC_PIX / PPI; ++it) {
    const int64_t p = p0 + (int64_t)it * PPI;
    if (p < P) {
      float gv[8], yv[8];
      bnc_ld8<GB16>(g, p * C + 8 * grp, gv);
      bnc_ld8<YB16>(y, p * C + 8 * grp, yv);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float gz = fmaf(yv[c], sc[c], sh[c]) > 0.f ? gv[c] : 0.f;
        s1[c] += gz;
        s2[c] += gz * ((yv[c] - mu[c]) * rs[c]);
      }
    }
  }
  // lanes of one channel group: xor offsets G, 2G, .. 32 (fixed order)
#pragma unroll
  for (int o = G; o < 64; o <<= 1)
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      s1[c] += __shfl_xor(s1[c], o, 64);
      s2[c] += __shfl_xor(s2[c], o, 64);
    }
  if (lane < G) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      red[wave][8 * lane + c] = s1[c];
      red[wave][C + 8 * lane + c] = s2[c];
    }
  }
  __syncthreads();
  if (tid < 2 * C)
    partial[(int64_t)blockIdx.x * 2 * C + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

// sums[o] = sum over blocks of partial[block][o], o < C2: one 256-thread
// block per output, each thread a strided subset of the blocks (in flight
// together), then a fixed-order tree over the 256 per-thread sums
__global__ __launch_bounds__(256) void bn_cl_partials_sum(const double* __restrict__ partial,
                                                          int nblk, int C2,
                                                          double* __restrict__ sums) {
  __shared__ double red[256];
  const int tid = threadIdx.x, o = blockIdx.x;
  double a = 0.0;
  for (int b = tid; b < nblk; b += 256) a += partial[(int64_t)b * C2 + o];
  red[tid] = a;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) sums[o] = red[0];
}

int bn_cl_sum_partials(const double* partial, int nblk, int C2, double* sums, hipStream_t s) {
  hipLaunchKernelGGL(bn_cl_partials_sum, dim3(C2), dim3(256), 0, s, partial, nblk, C2, sums);
  return check_launch("bn_cl_partials_sum");
}

constexpr int BNA_UNR = 2;   // pixels per thread per pass of bn_relu_bwd_apply_cl

template <int C, bool GB16, bool YB16, bool OB16>
__global__ __launch_bounds__(256, 4) void bn_relu_bwd_apply_cl(
    const void* __restrict__ g, const void* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ save, const double* __restrict__ sums, void* __restrict__ gy,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int64_t P, double inv_count) {
  constexpr int G = C / 8, PPI = 256 / G, UNR = BNA_UNR;
  const int tid = threadIdx.x, grp = tid % G;
  if (blockIdx.x == 0 && tid < C) {
    if (dbeta) dbeta[tid] = (float)sums[tid];
    if (dgamma) dgamma[tid] = (float)sums[C + tid];
  }
  // per-channel constants in LDS (7 x 8 registers per thread would cost the
  // pass its occupancy): scale, shift, mean, rstd, k = gamma * rstd, m1, m2
  __shared__ float cst[7][C];
  if (tid < C) {
    const double ic = inv_count > 0.0 ? inv_count : 1.0 / sums[2 * C];   // see bn_finalize
    cst[0][tid] = scale[tid];
    cst[1][tid] = shift[tid];
    cst[2][tid] = save[tid];
    cst[3][tid] = save[C + tid];
    cst[4][tid] = (gamma ? gamma[tid] : 1.f) * save[C + tid];
    cst[5][tid] = (float)(sums[tid] * ic);
    cst[6][tid] = (float)(sums[C + tid] * ic);
  }
  __syncthreads();
  for (int64_t pb = (int64_t)blockIdx.x * PPI * UNR; pb < P; pb += (int64_t)gridDim.x * PPI * UNR) {
    // re-read the constants per iteration (an opaque base keeps the compiler
    // from hoisting 56 of them into registers for the whole loop)
    int cb = 8 * grp;
    asm volatile("" : "+v"(cb));
    float gv[UNR][8], yv[UNR][8];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = pb + u * PPI + tid / G;
      if (p < P) {
        bnc_ld8<GB16>(g, p * C + 8 * grp, gv[u]);
        bnc_ld8<YB16>(y, p * C + 8 * grp, yv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t p = pb + u * PPI + tid / G;
      if (p >= P) continue;
      float o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int ch = cb + c;
        const float gz = fmaf(yv[u][c], cst[0][ch], cst[1][ch]) > 0.f ? gv[u][c] : 0.f;
        o[c] = cst[4][ch] * (gz - cst[5][ch] - ((yv[u][c] - cst[2][ch]) * cst[3][ch]) * cst[6][ch]);
      }
      const int64_t e = p * C + 8 * grp;
      if constexpr (OB16) {
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(gy) + e) =
            make_uint4(cvt_pk_bf16(o[0], o[1]), cvt_pk_bf16(o[2], o[3]), cvt_pk_bf16(o[4], o[5]),
                       cvt_pk_bf16(o[6], o[7]));
      } else {
        float* d = reinterpret_cast<float*>(gy) + e;
        *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
    }
  }
}


// Channel-last <-> NTCF (round 5): the encoder's last block with y channel-
// last [N][H][W][64] and the LSTM side in [N][W][64*H] (feature c*H + h,
// model.py:73-74).  Tiles of 64 pixels x 64 channels transposed through LDS
// ([c][pixel], rows padded to 65 floats): a thread owns 16 consecutive
// channels of one pixel (4 threads per pixel, 64- / 32-byte loads), a wave
// then writes 16 channel rows of 64 pixels (256 / 128-byte runs).
//  * bridge, X role: tile (n, t, 64 rows h): X[n][t][c*H + h] fp32 and / or
//    bf16 -- 64 consecutive h per channel;
//  * bridge, XT role (bf16): tile (n, h, 64 columns t): XT[c*H + h][n*W + t]
//    -- 64 consecutive t per channel (the weight gradient's k-contiguous
//    operand, gemm16.hip);
//  * backward: tile (n, t, 64 rows h); g (NTCF) into LDS, y (channel-last)
//    in registers; reduce accumulates per channel across a persistent
//    block's tiles, apply writes gy channel-last.  The next tile's loads are
//    issued before the current tile is processed.
constexpr int CLN_C = 64;

template <bool YB16>
__device__ __forceinline__ void cln_ld16(const void* y, int64_t e, float (&v)[16]) {
  if constexpr (YB16) {
    const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(y) + e);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4 q = p[h];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[8 * h + 2 * j] = __uint_as_float(w[j] << 16);
        v[8 * h + 2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      }
    }
  } else {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(y) + e);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float4 a = p[h];
      v[4 * h] = a.x; v[4 * h + 1] = a.y; v[4 * h + 2] = a.z; v[4 * h + 3] = a.w;
    }
  }
}

template <bool YB16>
__global__ __launch_bounds__(256) void bn_relu_apply_ntcf_cl(
    const void* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    float* __restrict__ out, uint16_t* __restrict__ out16, uint16_t* __restrict__ outT,
    int64_t ld_t, int H, int W, int64_t nx, int ntf, int ntt) {
  __shared__ float tile[CLN_C][65];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pr = tid >> 2, q = tid & 3;
  int64_t b = blockIdx.x;
  const bool xt = b >= nx;
  int n, h0, t0;
  if (!xt) {                       // (n, t, 64 rows)
    t0 = (int)(b % W);
    h0 = (int)((b / W) % ntf) * 64;
    n = (int)(b / ((int64_t)W * ntf));
  } else {                         // (n, h, 64 columns)
    b -= nx;
    t0 = (int)(b % ntt) * 64;
    h0 = (int)((b / ntt) % H);
    n = (int)(b / ((int64_t)ntt * H));
  }
  const int h = xt ? h0 : h0 + pr, t = xt ? t0 + pr : t0;
  float v[16];
  if (h < H && t < W) {
    cln_ld16<YB16>(y, (((int64_t)n * H + h) * W + t) * CLN_C + 16 * q, v);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = fmaxf(fmaf(v[j], scale[16 * q + j], shift[16 * q + j]), 0.f);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) tile[16 * q + j][pr] = v[j];
  __syncthreads();
  if (!xt) {
    const int hh = h0 + lane;
    if (hh < H) {
      const int64_t row = ((int64_t)n * W + t0) * CLN_C * H + hh;
#pragma unroll 4
      for (int it = 0; it < 16; ++it) {
        const int c = 16 * wave + it;
        const float val = tile[c][lane];
        if (out) out[row + (int64_t)c * H] = val;
        if (out16) out16[row + (int64_t)c * H] = __builtin_bit_cast(uint16_t, (__bf16)val);
      }
    }
  } else {
    const int tt = t0 + lane;
    if (tt < W) {
#pragma unroll 4
      for (int it = 0; it < 16; ++it) {
        const int c = 16 * wave + it;
        outT[((int64_t)c * H + h0) * ld_t + (int64_t)n * W + tt] =
            __builtin_bit_cast(uint16_t, (__bf16)tile[c][lane]);
      }
    }
  }
}

template <bool APPLY, bool YB16, bool GY16>
__global__ __launch_bounds__(256, 4) void bn_relu_bwd_ntcf_cl(
    const float* __restrict__ g, const void* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ save, const double* __restrict__ sums, double* __restrict__ partial,
    void* __restrict__ gy, float* __restrict__ dgamma, float* __restrict__ dbeta, int H, int W,
    int ntf, int64_t ntiles, double inv_count) {
  __shared__ float tile[CLN_C][65];
  __shared__ double red[4][2 * CLN_C];
  // per-channel constants in LDS (registers would hold 6 x 16 of them per
  // thread and cap the pass at two workgroups per CU): scale, shift, mean,
  // rstd and, for the apply, k = gamma * rstd, m1, m2
  __shared__ float cst[7][CLN_C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pr = tid >> 2, q = tid & 3;
  if (APPLY && blockIdx.x == 0 && tid < CLN_C) {
    if (dbeta) dbeta[tid] = (float)sums[tid];
    if (dgamma) dgamma[tid] = (float)sums[CLN_C + tid];
  }
  if (tid < CLN_C) {
    const int c = tid;
    cst[0][c] = scale[c];
    cst[1][c] = shift[c];
    cst[2][c] = save[c];
    cst[3][c] = save[CLN_C + c];
    if (APPLY) {
      const double ic = inv_count > 0.0 ? inv_count : 1.0 / sums[2 * CLN_C];   // see bn_finalize
      cst[4][c] = (gamma ? gamma[c] : 1.f) * save[CLN_C + c];
      cst[5][c] = (float)(sums[c] * ic);                          // m1
      cst[6][c] = (float)(sums[CLN_C + c] * ic);                  // m2
    }
  }
  float a1[APPLY ? 1 : 16], a2[APPLY ? 1 : 16];                   // s1, s2
#pragma unroll
  for (int j = 0; j < (APPLY ? 1 : 16); ++j) a1[j] = a2[j] = 0.f;
  // 32-bit tile coordinates (the launcher checks ntiles < 2^31); clamped,
  // branch-free loads selected to zero past H.  g through a buffer resource
  // per tile (one VGPR offset, the channel rows as scalar offsets); y kept as
  // raw words until used -- the pass is held to 128 VGPRs (4 workgroups / CU)
  constexpr int YW = YB16 ? 2 : 4;               // 16-byte words of y per thread
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  auto coords = [&](int b, int& n, int& h0, int& t) {
    const int bw = b / W;
    t = b - bw * W;
    n = bw / ntf;
    h0 = (bw - n * ntf) * 64;
  };
  float gr[16];
  uint4 yr[YW];
  auto load = [&](int b) {
    int n, h0, t;
    coords(b, n, h0, t);
    const int hh = h0 + lane;
    const bool hok = hh < H;
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g + ((int64_t)n * W + t) * CLN_C * H + (int64_t)16 * wv * H), (short)0,
        0x7fffffff, 0x00020000);
    const int vo = (hok ? hh : H - 1) * 4;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, vo, it * H * 4, 0));
      gr[it] = hok ? v : 0.f;
    }
    const int h = h0 + pr;
    const int64_t e = (((int64_t)n * H + (h < H ? h : H - 1)) * W + t) * CLN_C + 16 * q;
    const uint4* yp = YB16 ? reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(y) + e)
                           : reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(y) + e);
#pragma unroll
    for (int k = 0; k < YW; ++k) yr[k] = yp[k];
  };
  auto ydec = [&](const uint4 (&w)[YW], int j) -> float {   // channel 16 q + j
    const uint4 u = w[YB16 ? j / 8 : j / 4];
    const int k = YB16 ? (j % 8) / 2 : j % 4;
    const uint32_t x = k == 0 ? u.x : k == 1 ? u.y : k == 2 ? u.z : u.w;
    if constexpr (YB16) return __uint_as_float((j & 1) ? (x & 0xffff0000u) : (x << 16));
    return __uint_as_float(x);
  };
  const int nt32 = (int)ntiles;
  int b = blockIdx.x;
  if (b < nt32) load(b);
  for (; b < nt32; b += gridDim.x) {
#pragma unroll
    for (int it = 0; it < 16; ++it) tile[16 * wave + it][lane] = gr[it];
    uint4 yc[YW];
#pragma unroll
    for (int k = 0; k < YW; ++k) yc[k] = yr[k];
    int n, h0, t;
    coords(b, n, h0, t);
    __syncthreads();
    if (b + (int)gridDim.x < nt32) load(b + gridDim.x);   // in flight during this tile
    const int h = h0 + pr;
    const int64_t e = (((int64_t)n * H + h) * W + t) * CLN_C + 16 * q;
    // two halves of 8 channels: computed, then stored
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      float o[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = 8 * hf + jj, c = 16 * q + j;
        const float yv = ydec(yc, j);
        const float gz = fmaf(yv, cst[0][c], cst[1][c]) > 0.f ? tile[c][pr] : 0.f;
        const float xh = (yv - cst[2][c]) * cst[3][c];
        if constexpr (APPLY) {
          o[jj] = cst[4][c] * (gz - cst[5][c] - xh * cst[6][c]);
        } else if (h < H) {
          a1[j] += gz;
          a2[j] += gz * xh;
        }
      }
      if (APPLY && h < H) {
        if constexpr (GY16) {
          reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(gy) + e)[hf] =
              make_uint4(cvt_pk_bf16(o[0], o[1]), cvt_pk_bf16(o[2], o[3]),
                         cvt_pk_bf16(o[4], o[5]), cvt_pk_bf16(o[6], o[7]));
        } else {
          float4* d = reinterpret_cast<float4*>(reinterpret_cast<float*>(gy) + e) + 2 * hf;
          d[0] = make_float4(o[0], o[1], o[2], o[3]);
          d[1] = make_float4(o[4], o[5], o[6], o[7]);
        }
      }
    }
    __syncthreads();   // the tile is re-written next iteration
  }
  if constexpr (APPLY) return;
  // lanes of one channel quarter (== q mod 4): xor 4 .. 32, fixed order
#pragma unroll
  for (int o = 4; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < (APPLY ? 1 : 16); ++j) {
      a1[j] += __shfl_xor(a1[j], o, 64);
      a2[j] += __shfl_xor(a2[j], o, 64);
    }
  if (lane < 4) {
#pragma unroll
    for (int j = 0; j < (APPLY ? 1 : 16); ++j) {
      red[wave][16 * lane + j] = a1[j];
      red[wave][CLN_C + 16 * lane + j] = a2[j];
    }
  }
  __syncthreads();
  if (tid < 2 * CLN_C)
    partial[(int64_t)blockIdx.x * 2 * CLN_C + tid] =
        red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}
// persistent blocks of the NTCF backward passes (AINP_CLN_BLOCKS, <= the
// CLN_BLOCKS_MAX partial rows the workspace holds)
constexpr int CLN_BLOCKS_MAX = 2048;
static int cln_blocks() {
  static const int v = [] {
    const char* e = getenv("AINP_CLN_BLOCKS");
    const int b = e ? atoi(e) : 768;
    return b < 256 ? 256 : (b > CLN_BLOCKS_MAX ? CLN_BLOCKS_MAX : b);
  }();
  return v;
}

// ----------------------------------------------------------- NTCF path
// The encoder's last BatchNorm+ReLU reads / writes the LSTM layout
// [n][w][c*H + h] (model.py:73-74) while y is NCHW: 64(h) x 64(w) tiles of one
// (n, c), transposed through LDS; every global load of a tile is issued
// before the barrier (both operands in flight together).
constexpr int NT_T = 64;

__device__ __forceinline__ void ntcf_tile(int64_t b, int C, int64_t H, int64_t W, int& n, int& c,
                                          int& h0, int& w0) {
  const int th = (int)((H + NT_T - 1) / NT_T), tw = (int)((W + NT_T - 1) / NT_T);
  w0 = (int)(b % tw) * NT_T;
  h0 = (int)((b / tw) % th) * NT_T;
  c = (int)((b / ((int64_t)tw * th)) % C);
  n = (int)(b / ((int64_t)tw * th * C));
}

__global__ __launch_bounds__(256) void bn_relu_apply_ntcf(const float* __restrict__ x,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          float* __restrict__ out, int C, int64_t H,
                                                          int64_t W) {
  __shared__ float tile[NT_T][NT_T + 1];   // [w][h]
  int n, c, h0, w0;
  ntcf_tile(blockIdx.x, C, H, W, n, c, h0, w0);
  const float sc = scale[c], sh = shift[c];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const float* xp = x + ((int64_t)n * C + c) * H * W;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t h = h0 + q + 4 * i, w = w0 + lane;
    v[i] = (h < H && w < W) ? fmaxf(fmaf(xp[h * W + w], sc, sh), 0.f) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) tile[lane][q + 4 * i] = v[i];
  __syncthreads();
  const int64_t CH = (int64_t)C * H;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t h = h0 + lane, w = w0 + q + 4 * i;
    if (h < H && w < W) out[((int64_t)n * W + w) * CH + (int64_t)c * H + h] = tile[q + 4 * i][lane];
  }
}

template <bool APPLY, bool GY16 = false, bool YB16 = false>
__global__ __launch_bounds__(256) void bn_relu_bwd_ntcf(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ save, const double* __restrict__ sums, double* __restrict__ partial,
    void* __restrict__ gy, float* __restrict__ dgamma, float* __restrict__ dbeta, int C,
    int64_t H, int64_t W, double inv_count) {
  __shared__ float tile[NT_T][NT_T + 1];   // g as [w][h]
  __shared__ double red[2][4];
  if (APPLY && blockIdx.x < (unsigned)C && threadIdx.x == 0) {
    if (dbeta) dbeta[blockIdx.x] = (float)sums[blockIdx.x];
    if (dgamma) dgamma[blockIdx.x] = (float)sums[C + blockIdx.x];
  }
  int n, c, h0, w0;
  ntcf_tile(blockIdx.x, C, H, W, n, c, h0, w0);
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t CH = (int64_t)C * H;
  const int64_t off = ((int64_t)n * C + c) * H * W;
  float gv[16], yv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {            // g: lanes along h (NTCF rows)
    const int64_t h = h0 + lane, w = w0 + q + 4 * i;
    gv[i] = (h < H && w < W) ? g[((int64_t)n * W + w) * CH + (int64_t)c * H + h] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {            // y: lanes along w (NCHW rows)
    const int64_t h = h0 + q + 4 * i, w = w0 + lane;
    yv[i] = (h < H && w < W) ? ld_y1<YB16>(y, off + h * W + w) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) tile[q + 4 * i][lane] = gv[i];
  __syncthreads();
  const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
  if (APPLY) {
    const float k = (gamma ? gamma[c] : 1.f) * rstd;
    const double ic = inv_count > 0.0 ? inv_count : 1.0 / sums[2 * C];   // see bn_finalize
    const float m1 = (float)(sums[c] * ic);
    const float m2 = (float)(sums[C + c] * ic);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t h = h0 + q + 4 * i, w = w0 + lane;
      if (h < H && w < W) {
        const float gz = fmaf(yv[i], sc, sh) > 0.f ? tile[lane][q + 4 * i] : 0.f;
        gy_st1<GY16>(gy, off + h * W + w, k * (gz - m1 - ((yv[i] - mean) * rstd) * m2));
      }
    }
  } else {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t h = h0 + q + 4 * i, w = w0 + lane;
      if (h < H && w < W) {
        const float gz = fmaf(yv[i], sc, sh) > 0.f ? tile[lane][q + 4 * i] : 0.f;
        s1 += gz;
        s2 += gz * ((yv[i] - mean) * rstd);
      }
    }
    const double d1 = wave_sum_d((double)s1), d2 = wave_sum_d((double)s2);
    if (lane == 0) {
      red[0][q] = d1;
      red[1][q] = d2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      partial[(int64_t)blockIdx.x * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      partial[(int64_t)blockIdx.x * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
  }
}

// NTCF v2 for C*H % 64 == 0 and even W (the model: C*H = 64*257): the NCHW
// tensor is [n][k = c*H + h][w] and the NTCF one [n][w][k], so the layout
// bridge is a batched 2-D transpose tiled 64 (k) x 64 (w) -- no 1-row h
// tiles, 8-byte vectors on both sides (a wave moves two 256-byte rows per
// instruction); the channel of row k is k / H.
// kfirst: consecutive workgroups walk k (the NTCF rows' contiguous dimension)
// rather than w (default; AINP_NTCF_KFIRST=0: w first.  bwd_apply 0.609 ->
// 0.588 ms in tools/bn_probe.py, profiles/r04kl_summary.txt)
__device__ __forceinline__ void ntcf2_tile(int64_t b, int64_t K, int64_t W, int& n, int& k0,
                                           int& w0, int kfirst = 0) {
  const int tw = (int)((W + NT_T - 1) / NT_T), tk = (int)(K / NT_T);
  if (kfirst) {
    k0 = (int)(b % tk) * NT_T;
    w0 = (int)((b / tk) % tw) * NT_T;
  } else {
    w0 = (int)(b % tw) * NT_T;
    k0 = (int)((b / tw) % tk) * NT_T;
  }
  n = (int)(b / ((int64_t)tw * tk));
}
static int ntcf_kfirst() {
  static const int v = [] {
    const char* e = getenv("AINP_NTCF_KFIRST");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

__global__ __launch_bounds__(256) void bn_relu_apply_ntcf2(const float* __restrict__ x,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           float* __restrict__ out, int C, int64_t H,
                                                           int64_t W, int kfirst) {
  __shared__ float tile[NT_T][NT_T + 1];   // [w][k]
  const int64_t K = (int64_t)C * H;
  int n, k0, w0;
  ntcf2_tile(blockIdx.x, K, W, n, k0, w0, kfirst);
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
  const float* xn = x + (int64_t)n * K * W;
#pragma unroll
  for (int i = 0; i < 8; ++i) {                 // rows k, lanes along w (float2)
    const int kk = r + 8 * i;
    const int64_t k = k0 + kk;
    const int c = (int)(k / H);
    const int w = w0 + 2 * l;
    float2 v = make_float2(0.f, 0.f);
    if (w < W) v = *reinterpret_cast<const float2*>(xn + k * W + w);
    const float sc = scale[c], sh = shift[c];
    tile[2 * l][kk] = fmaxf(fmaf(v.x, sc, sh), 0.f);
    tile[2 * l + 1][kk] = fmaxf(fmaf(v.y, sc, sh), 0.f);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8; ++i) {                 // rows w, lanes along k (float2)
    const int ww = r + 8 * i;
    const int64_t w = w0 + ww;
    if (w < W)
      *reinterpret_cast<float2*>(out + ((int64_t)n * W + w) * K + k0 + 2 * l) =
          make_float2(tile[ww][2 * l], tile[ww][2 * l + 1]);
  }
}

template <bool GY16 = false, bool YB16 = false>
__global__ __launch_bounds__(256) void bn_relu_bwd_apply_ntcf2(
    const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ gamma,
    const float* __restrict__ save, const double* __restrict__ sums, void* __restrict__ gy,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int C, int64_t H, int64_t W,
    double inv_count, int64_t ntiles, int kfirst) {
  __shared__ float tile[NT_T][NT_T + 1];   // g as [w][k]
  if (blockIdx.x < (unsigned)C && threadIdx.x == 0) {
    if (dbeta) dbeta[blockIdx.x] = (float)sums[blockIdx.x];
    if (dgamma) dgamma[blockIdx.x] = (float)sums[C + blockIdx.x];
  }
  if (blockIdx.x >= ntiles) return;         // a dgamma / dbeta writer only
  const int64_t K = (int64_t)C * H;
  int n, k0, w0;
  ntcf2_tile(blockIdx.x, K, W, n, k0, w0, kfirst);
  const int l = threadIdx.x & 31, r = threadIdx.x >> 5;
  float2 yv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {                 // g: rows w, lanes along k
    const int ww = r + 8 * i;
    const int64_t w = w0 + ww;
    float2 v = make_float2(0.f, 0.f);
    if (w < W) v = *reinterpret_cast<const float2*>(g + ((int64_t)n * W + w) * K + k0 + 2 * l);
    tile[ww][2 * l] = v.x;
    tile[ww][2 * l + 1] = v.y;
  }
  const int64_t yn = (int64_t)n * K * W;
#pragma unroll
  for (int i = 0; i < 8; ++i) {                 // y: rows k, lanes along w
    const int64_t k = k0 + r + 8 * i;
    const int w = w0 + 2 * l;
    yv[i] = w < W ? ld_y2<YB16>(y, yn + k * W + w) : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const int64_t gn = (int64_t)n * K * W;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int kk = r + 8 * i;
    const int64_t k = k0 + kk;
    const int w = w0 + 2 * l;
    if (w >= W) continue;
    const int c = (int)(k / H);
    const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
    const float kc = (gamma ? gamma[c] : 1.f) * rstd;
    const double ic = inv_count > 0.0 ? inv_count : 1.0 / sums[2 * C];   // see bn_finalize
    const float m1 = (float)(sums[c] * ic);
    const float m2 = (float)(sums[C + c] * ic);
    const float gz0 = fmaf(yv[i].x, sc, sh) > 0.f ? tile[2 * l][kk] : 0.f;
    const float gz1 = fmaf(yv[i].y, sc, sh) > 0.f ? tile[2 * l + 1][kk] : 0.f;
    gy_st2<GY16>(gy, gn + k * W + w, kc * (gz0 - m1 - ((yv[i].x - mean) * rstd) * m2),
                 kc * (gz1 - m1 - ((yv[i].y - mean) * rstd) * m2));
  }
}

// The bf16 configuration's layer-0 LSTM operands straight from the encoder
// (gemm16.hip): relu(x*scale+shift) rounded to bf16 (nearest-even), written
// both as X [n][w][k] (the NTCF input of the projection GEMM) and X^T
// [k][n*W + w] (ld_t per row: the k-contiguous operand of the weight-gradient
// GEMM).  128 (k) x 128 (w) tiles (even C*H and W): X^T rows of 128 w and X
// rows of 128 k are 256-byte stores per wave instruction (64 x 64 tiles store
// 128-byte pieces: 0.437 -> 0.412 ms at the C3 shape, tools/bn_probe.py).  A
// thread converts the k pair (2p, 2p+1) at columns (w, w+1): X^T takes the
// (w, w+1) pairs of each row, the LDS tile the (k, k+1) pairs of each column,
// packed bf16x2 both ways.
constexpr int B2K = 128, B2W = 128;
template <bool YB16 = false>
__global__ __launch_bounds__(256) void bn_relu_apply_ntcf_bf16(
    const float* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
    uint16_t* __restrict__ out, uint16_t* __restrict__ outT, int64_t ld_t, int C, int64_t H,
    int64_t W) {
  __shared__ uint32_t tile[B2W][B2K / 2 + 1];   // [w][k pair]
  const int64_t K = (int64_t)C * H;
  const int tw = (int)((W + B2W - 1) / B2W), tk = (int)((K + B2K - 1) / B2K);
  const int64_t b = blockIdx.x;
  const int w0 = (int)(b % tw) * B2W;
  const int64_t k0 = ((b / tw) % tk) * B2K;
  const int n = (int)(b / ((int64_t)tw * tk));
  const int l = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t xn = (int64_t)n * K * W;
  const int w = w0 + 2 * l;
  const bool wok = w < W;
  float2 v[16][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {                  // k pairs p = q + 4 i: rows 2p, 2p+1
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t k = k0 + 2 * (q + 4 * i) + e;
      v[i][e] = (wok && k < K) ? ld_y2<YB16>(x, xn + k * W + w) : make_float2(0.f, 0.f);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int p = q + 4 * i;
    uint32_t u[2][2];   // [row e][column]
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t k = k0 + 2 * p + e;
      const int c = (int)((k < K ? k : K - 1) / H);
      const float sc = scale[c], sh = shift[c];
      u[e][0] = __builtin_bit_cast(uint16_t, (__bf16)fmaxf(fmaf(v[i][e].x, sc, sh), 0.f));
      u[e][1] = __builtin_bit_cast(uint16_t, (__bf16)fmaxf(fmaf(v[i][e].y, sc, sh), 0.f));
      if (wok && k < K)
        *reinterpret_cast<uint32_t*>(outT + k * ld_t + (int64_t)n * W + w) =
            u[e][0] | (u[e][1] << 16);
    }
    tile[2 * l][p] = u[0][0] | (u[1][0] << 16);
    tile[2 * l + 1][p] = u[0][1] | (u[1][1] << 16);
  }
  __syncthreads();
  const bool kok = k0 + 2 * l < K;
#pragma unroll 8
  for (int i = 0; i < B2W / 4; ++i) {             // rows w, lanes along k pairs
    const int ww = q + 4 * i;
    const int64_t wr = w0 + ww;
    if (wr < W && kok)
      *reinterpret_cast<uint32_t*>(out + ((int64_t)n * W + wr) * K + k0 + 2 * l) = tile[ww][l];
  }
}

static bool ntcf2_ok(int C, int64_t H, int64_t W, std::initializer_list<const void*> ptrs) {
  if (((int64_t)C * H) % NT_T != 0 || W % 2 != 0) return false;
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 8 != 0) return false;
  return true;
}

static int64_t tiles_per_plane(int64_t H, int64_t W) {
  return cdiv(H, TH) * cdiv(W, TW);
}

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_bn_stats_reduce(const double* stats, int nparts,
                                    double* sums, int C, void* stream) {
  if (!stats || nparts < 1 || !sums || C < 1)
    return record_msg("ainp_bn_stats_reduce: bad argument");
  hipLaunchKernelGGL(bn_stats_reduce_kernel, dim3(C), dim3(256), 0,
                     as_stream(stream), stats, nparts, sums, C);
  return check_launch("bn_stats_reduce");
}

extern "C" int ainp_bn_reduce_finalize(const double* stats, int nparts, int64_t count,
                                       const float* gamma, const float* beta,
                                       float* running_mean, float* running_var, float momentum,
                                       float eps, float* scale, float* shift,
                                       float* save_mean_rstd, int C, void* stream) {
  if (!stats || nparts < 1 || !scale || !shift || !save_mean_rstd || C < 1 || count < 1 ||
      ((running_mean == nullptr) != (running_var == nullptr)))
    return record_msg("ainp_bn_reduce_finalize: bad argument");
  hipLaunchKernelGGL(bn_reduce_finalize_kernel, dim3(C), dim3(256), 0, as_stream(stream), stats,
                     nparts, gamma, beta, running_mean, running_var, momentum, eps, count, scale,
                     shift, save_mean_rstd, C);
  return check_launch("bn_reduce_finalize");
}

extern "C" int ainp_bn_finalize(const double* sums, int64_t count,
                                const float* gamma, const float* beta,
                                float* running_mean, float* running_var,
                                float momentum, float eps, float* scale,
                                float* shift, float* save_mean_rstd, int C,
                                void* stream) {
  if (!sums || !scale || !shift || !save_mean_rstd || C < 1 || count < 0 ||
      ((running_mean == nullptr) != (running_var == nullptr)))
    return record_msg("ainp_bn_finalize: bad argument");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(64), 0,
                     as_stream(stream), sums, gamma, beta, running_mean,
                     running_var, momentum, eps, count, scale, shift,
                     save_mean_rstd, C);
  return check_launch("bn_finalize");
}

extern "C" int ainp_bn_eval_affine(const float* gamma, const float* beta,
                                   const float* running_mean,
                                   const float* running_var, float eps,
                                   float* scale, float* shift, int C,
                                   void* stream) {
  if (!running_mean || !running_var || !scale || !shift || C < 1)
    return record_msg("ainp_bn_eval_affine: bad argument");
  hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 63) / 64), dim3(64), 0,
                     as_stream(stream), gamma, beta, running_mean, running_var,
                     eps, scale, shift, C);
  return check_launch("bn_eval_affine");
}

extern "C" int ainp_bn_relu_apply(const float* x, const float* scale,
                                  const float* shift, float* out, int64_t N,
                                  int C, int64_t H, int64_t W, int out_ntcf,
                                  void* stream) {
  if (!x || !scale || !shift || !out || N < 0 || C < 1 || H < 1 || W < 1)
    return record_msg("ainp_bn_relu_apply: bad argument");
  if (N == 0) return AINP_OK;
  const int64_t blocks = N * C * tiles_per_plane(H, W);
  hipStream_t s = as_stream(stream);
  if (out_ntcf && ntcf2_ok(C, H, W, {x, out}))
    hipLaunchKernelGGL(bn_relu_apply_ntcf2,
                       dim3((unsigned)(N * (C * H / NT_T) * cdiv(W, NT_T))), dim3(256), 0, s, x,
                       scale, shift, out, C, H, W, ntcf_kfirst());
  else if (out_ntcf)
    hipLaunchKernelGGL(bn_relu_apply_ntcf, dim3((unsigned)(N * C * cdiv(H, NT_T) * cdiv(W, NT_T))),
                       dim3(256), 0, s, x, scale, shift, out, C, H, W);
  else
    hipLaunchKernelGGL(bn_relu_apply_kernel<false>, dim3((unsigned)blocks),
                       dim3(256), 0, s, x, scale, shift, out, C, H, W);
  return check_launch("bn_relu_apply");
}

extern "C" int ainp_bn_relu_apply_ntcf_bf16_ex(const float* x, const float* scale,
                                               const float* shift, uint16_t* out, uint16_t* outT,
                                               int64_t ld_t, int64_t N, int C, int64_t H,
                                               int64_t W, int flags, void* stream) {
  if (!x || !scale || !shift || !out || !outT || N < 1 || C < 1 || H < 1 || W < 1 ||
      ld_t < N * W || !ntcf2_ok(C, H, W, {x}) || (reinterpret_cast<uintptr_t>(out) & 3) ||
      (reinterpret_cast<uintptr_t>(outT) & 3) || (ld_t & 1) || (flags & ~AINP_BN_Y16))
    return record_msg("ainp_bn_relu_apply_ntcf_bf16: bad argument (C*H % 64, even W and ld_t)");
  const dim3 grid((unsigned)(N * cdiv(C * H, B2K) * cdiv(W, B2W)));
  if (flags & AINP_BN_Y16)
    hipLaunchKernelGGL(bn_relu_apply_ntcf_bf16<true>, grid, dim3(256), 0, as_stream(stream), x,
                       scale, shift, out, outT, ld_t, C, H, W);
  else
    hipLaunchKernelGGL(bn_relu_apply_ntcf_bf16<false>, grid, dim3(256), 0, as_stream(stream), x,
                       scale, shift, out, outT, ld_t, C, H, W);
  return check_launch("bn_relu_apply_ntcf_bf16");
}

// Round 5: the bridge from a channel-last y ([N][H][W][64], AINP_BN_Y16: bf16
// storage): out (fp32) / out16 (bf16) = relu(y*scale+shift) as [N][W][64*H],
// outT (bf16) as [64*H][ld_t] (column n*W + w); NULL outputs are skipped.
extern "C" int ainp_bn_relu_apply_ntcf_cl(const float* y, const float* scale, const float* shift,
                                          float* out, uint16_t* out16, uint16_t* outT,
                                          int64_t ld_t, int64_t N, int C, int64_t H, int64_t W,
                                          int flags, void* stream) {
  if (!y || !scale || !shift || (!out && !out16 && !outT) || N < 1 || C != CLN_C || H < 1 ||
      W < 1 || (outT && ld_t < N * W) || (reinterpret_cast<uintptr_t>(y) & 15) ||
      (flags & ~AINP_BN_Y16) || H * W * C >= ((int64_t)1 << 31))
    return record_msg("ainp_bn_relu_apply_ntcf_cl: bad argument (C = 64, 16-byte aligned y)");
  const int ntf = (int)cdiv(H, 64), ntt = (int)cdiv(W, 64);
  const int64_t nx = (out || out16) ? N * W * ntf : 0;
  const int64_t nxt = outT ? N * H * ntt : 0;
  const dim3 grid((unsigned)(nx + nxt));
  if (flags & AINP_BN_Y16)
    hipLaunchKernelGGL(bn_relu_apply_ntcf_cl<true>, grid, dim3(256), 0, as_stream(stream), y,
                       scale, shift, out, out16, outT, ld_t, (int)H, (int)W, nx, ntf, ntt);
  else
    hipLaunchKernelGGL(bn_relu_apply_ntcf_cl<false>, grid, dim3(256), 0, as_stream(stream), y,
                       scale, shift, out, out16, outT, ld_t, (int)H, (int)W, nx, ntf, ntt);
  return check_launch("bn_relu_apply_ntcf_cl");
}

extern "C" int ainp_bn_relu_apply_ntcf_bf16(const float* x, const float* scale,
                                            const float* shift, uint16_t* out, uint16_t* outT,
                                            int64_t ld_t, int64_t N, int C, int64_t H, int64_t W,
                                            void* stream) {
  return ainp_bn_relu_apply_ntcf_bf16_ex(x, scale, shift, out, outT, ld_t, N, C, H, W, 0, stream);
}

extern "C" size_t ainp_bn_relu_bwd_workspace(int64_t N, int C, int64_t H,
                                             int64_t W) {
  const int64_t tiled = N * C * tiles_per_plane(H, W) * 2;
  int64_t cl = cdiv(N * H * W, BNC_PIX) * 2 * C;   // channel-last partials
  if (cl < (int64_t)CLN_BLOCKS_MAX * 2 * C) cl = (int64_t)CLN_BLOCKS_MAX * 2 * C;
  return (size_t)(tiled > cl ? tiled : cl) * sizeof(double);
}

template <bool YB16>
static int bn_bwd_reduce_launch(const float* g, const float* y, const float* scale,
                                const float* shift, const float* save_mean_rstd, void* workspace,
                                double* sums, int64_t N, int C, int64_t H, int64_t W, int g_ntcf,
                                hipStream_t s) {
  double* partial = reinterpret_cast<double*>(workspace);
  if (!g_ntcf) {
    const int64_t HW = H * W;
    const int chunks = (int)cdiv(HW, BN_CHUNK);   // <= tiles_per_plane: fits the workspace
    const bool vec = (HW % 2 == 0) && ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y)) % 8 == 0);
    const dim3 grid((unsigned)(N * C * chunks));
    if (vec)
      hipLaunchKernelGGL((bn_relu_bwd_reduce_flat<true, YB16>), grid, dim3(256), 0, s, g, y,
                         scale, shift, save_mean_rstd, partial, C, HW, chunks);
    else
      hipLaunchKernelGGL((bn_relu_bwd_reduce_flat<false, YB16>), grid, dim3(256), 0, s, g, y,
                         scale, shift, save_mean_rstd, partial, C, HW, chunks);
    int rc = check_launch("bn_relu_bwd_reduce_flat");
    if (rc) return rc;
    hipLaunchKernelGGL(bn_bwd_sum_kernel, dim3(C), dim3(256), 0, s, partial, (int)N, C, chunks, sums);
    return check_launch("bn_bwd_sum");
  }
  const int64_t tpp = cdiv(H, NT_T) * cdiv(W, NT_T);   // <= tiles_per_plane: fits
  hipLaunchKernelGGL((bn_relu_bwd_ntcf<false, false, YB16>), dim3((unsigned)(N * C * tpp)),
                     dim3(256), 0, s, g, y, scale, shift, nullptr, save_mean_rstd, nullptr,
                     partial, nullptr, nullptr, nullptr, C, H, W, 0.0);
  int rc = check_launch("bn_relu_bwd_reduce_ntcf");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_bwd_sum_kernel, dim3(C), dim3(256), 0, s, partial,
                     (int)N, C, (int)tpp, sums);
  return check_launch("bn_bwd_sum");
}

// channel-last launchers (AINP_BN_CL; AINP_BN_G16: g in bf16 storage)
static bool bn_cl_ok(int C, std::initializer_list<const void*> ptrs) {
  if (C % 8 != 0 || C > 64) return false;
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 16 != 0) return false;
  return true;
}

static int bn_cl_reduce(const float* g, const float* y, const float* scale, const float* shift,
                        const float* save, void* workspace, double* sums, int64_t N, int64_t H,
                        int64_t W, int C, int g_ntcf, int flags, hipStream_t s) {
  const int64_t P = N * H * W;
  double* partial = reinterpret_cast<double*>(workspace);
  const bool g16 = flags & AINP_BN_G16, y16 = flags & AINP_BN_Y16;
  if ((flags & AINP_BN_CL) && g_ntcf) {   // g NTCF fp32, y channel-last (64 channels)
    if (C != CLN_C || g16 || !bn_cl_ok(C, {y}) || H * W * C >= ((int64_t)1 << 31) ||
        N * W * cdiv(H, 64) >= ((int64_t)1 << 31))
      return record_msg("ainp_bn_relu_bwd_reduce: NTCF g with channel-last y needs C = 64, "
                        "fp32 g, 16-byte aligned y");
    const int ntf = (int)cdiv(H, 64);
    const int64_t ntiles = N * W * ntf;
#define AINP_BNN(YV)                                                                             \
    hipLaunchKernelGGL((bn_relu_bwd_ntcf_cl<false, YV, false>), dim3(cln_blocks()), dim3(256), 0, s, \
                       g, y, scale, shift, nullptr, save, nullptr, partial, nullptr, nullptr,     \
                       nullptr, (int)H, (int)W, ntf, ntiles, 0.0)
    if (y16) AINP_BNN(true); else AINP_BNN(false);
#undef AINP_BNN
    int rc = check_launch("bn_relu_bwd_ntcf_cl");
    if (rc) return rc;
    hipLaunchKernelGGL(bn_cl_partials_sum, dim3(2 * C), dim3(256), 0, s, partial, cln_blocks(),
                       2 * C, sums);
    return check_launch("bn_cl_partials_sum");
  }
  if (!(flags & AINP_BN_CL) || g_ntcf || !bn_cl_ok(C, {g, y}))
    return record_msg("ainp_bn_relu_bwd_reduce: AINP_BN_CL needs C % 8 == 0 (<= 64), 16-byte "
                      "aligned g / y and no NTCF layout (AINP_BN_G16 needs AINP_BN_CL)");
  const int64_t nblk = cdiv(P, BNC_PIX);
#define AINP_BNCR(CV, GV, YV)                                                                   \
  if (C == CV && g16 == GV && y16 == YV)                                                        \
    hipLaunchKernelGGL((bn_relu_bwd_reduce_cl<CV, GV, YV>), dim3((unsigned)nblk), dim3(256), 0, s, \
                       g, y, scale, shift, save, partial, P);
#define AINP_BNCR4(CV) AINP_BNCR(CV, false, false) AINP_BNCR(CV, true, false) \
  AINP_BNCR(CV, false, true) AINP_BNCR(CV, true, true)
  AINP_BNCR4(16) AINP_BNCR4(32) AINP_BNCR4(64)
  if (C != 16 && C != 32 && C != 64)
    return record_msg("ainp_bn_relu_bwd_reduce: AINP_BN_CL serves C = 16, 32, 64");
#undef AINP_BNCR4
#undef AINP_BNCR
  int rc = check_launch("bn_relu_bwd_reduce_cl");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_cl_partials_sum, dim3(2 * C), dim3(256), 0, s, partial, (int)nblk, 2 * C,
                     sums);
  return check_launch("bn_cl_partials_sum");
}

static int bn_cl_apply(const float* g, const float* y, const float* scale, const float* shift,
                       const float* gamma, const float* save, const double* sums, int64_t count,
                       void* gy, float* dgamma, float* dbeta, int64_t N, int64_t H, int64_t W,
                       int C, int g_ntcf, int flags, hipStream_t s) {
  const int64_t P = N * H * W;
  const double inv_count = count > 0 ? 1.0 / (double)count : 0.0;   // 0: sums[2C]
  if ((flags & AINP_BN_CL) && g_ntcf) {   // g NTCF fp32, y / gy channel-last (64 channels)
    if (C != CLN_C || (flags & AINP_BN_G16) || !bn_cl_ok(C, {y, gy}) ||
        H * W * C >= ((int64_t)1 << 31) || N * W * cdiv(H, 64) >= ((int64_t)1 << 31))
      return record_msg("ainp_bn_relu_bwd_apply: NTCF g with channel-last y needs C = 64, "
                        "fp32 g, 16-byte aligned y / gy");
    const int ntf = (int)cdiv(H, 64);
    const int64_t ntiles = N * W * ntf;
    const bool y16 = flags & AINP_BN_Y16, o16 = flags & AINP_BN_GY16;
#define AINP_BNN(YV, OV)                                                                         \
    hipLaunchKernelGGL((bn_relu_bwd_ntcf_cl<true, YV, OV>), dim3(cln_blocks()), dim3(256), 0, s, g, \
                       y, scale, shift, gamma, save, sums, nullptr, gy, dgamma, dbeta, (int)H,    \
                       (int)W, ntf, ntiles, inv_count)
    if (y16 && o16) AINP_BNN(true, true);
    else if (y16) AINP_BNN(true, false);
    else if (o16) AINP_BNN(false, true);
    else AINP_BNN(false, false);
#undef AINP_BNN
    return check_launch("bn_relu_bwd_ntcf_cl");
  }
  if (!(flags & AINP_BN_CL) || g_ntcf || !bn_cl_ok(C, {g, y, gy}))
    return record_msg("ainp_bn_relu_bwd_apply: AINP_BN_CL needs C % 8 == 0 (<= 64), 16-byte "
                      "aligned g / y / gy and no NTCF layout (AINP_BN_G16 needs AINP_BN_CL)");
  const int ppb = 256 / (C / 8) * BNA_UNR;                           // pixels per block pass
  int64_t nb = cdiv(P, ppb);
  if (nb > 2048) nb = 2048;
  const bool g16 = flags & AINP_BN_G16, y16 = flags & AINP_BN_Y16, o16 = flags & AINP_BN_GY16;
#define AINP_BNCA(CV, GV, YV, OV)                                                              \
  if (C == CV && g16 == GV && y16 == YV && o16 == OV)                                          \
    hipLaunchKernelGGL((bn_relu_bwd_apply_cl<CV, GV, YV, OV>), dim3((unsigned)nb), dim3(256), 0, \
                       s, g, y, scale, shift, gamma, save, sums, gy, dgamma, dbeta, P, inv_count);
#define AINP_BNCA8(CV) AINP_BNCA(CV, false, false, false) AINP_BNCA(CV, false, false, true) \
  AINP_BNCA(CV, true, false, false) AINP_BNCA(CV, true, false, true)                        \
  AINP_BNCA(CV, false, true, false) AINP_BNCA(CV, false, true, true)                        \
  AINP_BNCA(CV, true, true, false) AINP_BNCA(CV, true, true, true)
  AINP_BNCA8(16) AINP_BNCA8(32) AINP_BNCA8(64)
  if (C != 16 && C != 32 && C != 64)
    return record_msg("ainp_bn_relu_bwd_apply: AINP_BN_CL serves C = 16, 32, 64");
#undef AINP_BNCA8
#undef AINP_BNCA
  return check_launch("bn_relu_bwd_apply_cl");
}

extern "C" int ainp_bn_relu_bwd_reduce_ex(const float* g, const float* y, const float* scale,
                                          const float* shift, const float* save_mean_rstd,
                                          void* workspace, double* sums, int64_t N, int C,
                                          int64_t H, int64_t W, int g_ntcf, int flags,
                                          void* stream) {
  if (!g || !y || !scale || !shift || !save_mean_rstd || !workspace || !sums ||
      N < 1 || C < 1 || H < 1 || W < 1 || (flags & ~(AINP_BN_Y16 | AINP_BN_CL | AINP_BN_G16)))
    return record_msg("ainp_bn_relu_bwd_reduce: bad argument");
  if (flags & (AINP_BN_CL | AINP_BN_G16))
    return bn_cl_reduce(g, y, scale, shift, save_mean_rstd, workspace, sums, N, H, W, C,
                        g_ntcf, flags, as_stream(stream));
  if (flags & AINP_BN_Y16)
    return bn_bwd_reduce_launch<true>(g, y, scale, shift, save_mean_rstd, workspace, sums, N, C,
                                      H, W, g_ntcf, as_stream(stream));
  return bn_bwd_reduce_launch<false>(g, y, scale, shift, save_mean_rstd, workspace, sums, N, C, H,
                                     W, g_ntcf, as_stream(stream));
}

extern "C" int ainp_bn_relu_bwd_reduce(const float* g, const float* y,
                                       const float* scale, const float* shift,
                                       const float* save_mean_rstd,
                                       void* workspace, double* sums,
                                       int64_t N, int C, int64_t H, int64_t W,
                                       int g_ntcf, void* stream) {
  return ainp_bn_relu_bwd_reduce_ex(g, y, scale, shift, save_mean_rstd, workspace, sums, N, C, H,
                                    W, g_ntcf, 0, stream);
}

template <bool GY16, bool YB16>
static int bn_bwd_apply_launch(const float* g, const float* y, const float* scale,
                               const float* shift, const float* gamma,
                               const float* save_mean_rstd, const double* sums, int64_t count,
                               void* gy, float* dgamma, float* dbeta, int64_t N, int C, int64_t H,
                               int64_t W, int g_ntcf, hipStream_t s);

extern "C" int ainp_bn_relu_bwd_apply_ex(const float* g, const float* y, const float* scale,
                                         const float* shift, const float* gamma,
                                         const float* save_mean_rstd, const double* sums,
                                         int64_t count, void* gy, float* dgamma, float* dbeta,
                                         int64_t N, int C, int64_t H, int64_t W, int g_ntcf,
                                         int flags, void* stream) {
  if (!g || !y || !scale || !shift || !save_mean_rstd || !sums || !gy ||
      N < 1 || C < 1 || H < 1 || W < 1 || count < 0 ||
      (flags & ~(AINP_BN_GY16 | AINP_BN_Y16 | AINP_BN_CL | AINP_BN_G16)))
    return record_msg("ainp_bn_relu_bwd_apply: bad argument");
  hipStream_t s = as_stream(stream);
  if (flags & (AINP_BN_CL | AINP_BN_G16))
    return bn_cl_apply(g, y, scale, shift, gamma, save_mean_rstd, sums, count, gy, dgamma, dbeta,
                       N, H, W, C, g_ntcf, flags, s);
#define AINP_BNA(GV, YV)                                                                       \
  return bn_bwd_apply_launch<GV, YV>(g, y, scale, shift, gamma, save_mean_rstd, sums, count, gy, \
                                     dgamma, dbeta, N, C, H, W, g_ntcf, s)
  const bool g16 = flags & AINP_BN_GY16, y16 = flags & AINP_BN_Y16;
  if (g16 && y16) AINP_BNA(true, true);
  if (g16) AINP_BNA(true, false);
  if (y16) AINP_BNA(false, true);
  AINP_BNA(false, false);
#undef AINP_BNA
}

extern "C" int ainp_bn_relu_bwd_apply(const float* g, const float* y,
                                      const float* scale, const float* shift,
                                      const float* gamma,
                                      const float* save_mean_rstd,
                                      const double* sums, int64_t count,
                                      float* gy, float* dgamma, float* dbeta,
                                      int64_t N, int C, int64_t H, int64_t W,
                                      int g_ntcf, void* stream) {
  return ainp_bn_relu_bwd_apply_ex(g, y, scale, shift, gamma, save_mean_rstd, sums, count, gy,
                                   dgamma, dbeta, N, C, H, W, g_ntcf, 0, stream);
}

template <bool GY16, bool YB16>
static int bn_bwd_apply_launch(const float* g, const float* y, const float* scale,
                               const float* shift, const float* gamma,
                               const float* save_mean_rstd, const double* sums, int64_t count,
                               void* gy, float* dgamma, float* dbeta, int64_t N, int C, int64_t H,
                               int64_t W, int g_ntcf, hipStream_t s) {
  const int64_t blocks = N * C * tiles_per_plane(H, W);
  const double inv_count = count > 0 ? 1.0 / (double)count : 0.0;   // 0: sums[2C]
  if (!g_ntcf) {
    const int64_t HW = H * W;
    const int chunks = (int)cdiv(HW, BN_CHUNK);
    const bool vec = (HW % 2 == 0) && ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y) |
                                        reinterpret_cast<uintptr_t>(gy)) % 8 == 0);
    int64_t nb = N * C * chunks;
    if (nb < C) nb = C;   // the dgamma / dbeta writers
    if (vec)
      hipLaunchKernelGGL((bn_relu_bwd_apply_flat<true, GY16, YB16>), dim3((unsigned)nb), dim3(256), 0, s, g, y,
                         scale, shift, gamma, save_mean_rstd, sums, gy, dgamma, dbeta, C, HW,
                         chunks, inv_count);
    else
      hipLaunchKernelGGL((bn_relu_bwd_apply_flat<false, GY16, YB16>), dim3((unsigned)nb), dim3(256), 0, s, g, y,
                         scale, shift, gamma, save_mean_rstd, sums, gy, dgamma, dbeta, C, HW,
                         chunks, inv_count);
    return check_launch("bn_relu_bwd_apply_flat");
  }
  (void)blocks;
  if (ntcf2_ok(C, H, W, {g, y, gy})) {
    const int64_t nt2 = N * (C * H / NT_T) * cdiv(W, NT_T);
    const int64_t nb2 = nt2 < C ? C : nt2;   // >= C blocks: the dgamma / dbeta writers
    hipLaunchKernelGGL((bn_relu_bwd_apply_ntcf2<GY16, YB16>), dim3((unsigned)nb2), dim3(256), 0, s, g, y, scale,
                       shift, gamma, save_mean_rstd, sums, gy, dgamma, dbeta, C, H, W, inv_count,
                       nt2, ntcf_kfirst());
    return check_launch("bn_relu_bwd_apply_ntcf2");
  }
  int64_t nb = N * C * cdiv(H, NT_T) * cdiv(W, NT_T);
  if (nb < C) nb = C;
  hipLaunchKernelGGL((bn_relu_bwd_ntcf<true, GY16, YB16>), dim3((unsigned)nb), dim3(256), 0, s, g, y, scale,
                     shift, gamma, save_mean_rstd, sums, nullptr, gy, dgamma, dbeta, C, H, W,
                     inv_count);
  return check_launch("bn_relu_bwd_apply_ntcf");
}
