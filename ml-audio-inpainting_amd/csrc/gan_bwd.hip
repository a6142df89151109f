// gan_bwd.hip — the generator backward of the GAN path (opt-in
// `fix_generator_grad`): PartialConv2d / BatchNorm2d + LeakyReLU /
// Tanh + crop backward for PConvUNet (models/GAN/networks.py:63-106,139-168,
// 247-345), the VGG19 input gradient of VGGLoss (models/GAN/loss.py:65-131)
// and the reconstruction-loss gradient of calculate_losses
// (models/GAN/train.py:49-63).
//
// The reference trains G only if its loop drops the torch.no_grad() around
// the generator (train.py:349-350); these kernels are the pieces
// torch autograd would run for it.  They are HBM-bound elementwise /
// reduction passes; the GEMM-shaped parts (weight gradients, data gradients)
// run on the existing MFMA GEMM / conv kernels (ainp/gan.py).  Every
// reduction is a fixed-order partial sum, so results are deterministic.
#include "common.h"

namespace ainp {

// ------------------------------------------------------------ PartialConv sources
// out [N, C0 + C1, Hin, Win] = cat(nearest(x0) * nearest(m0), x1 * m1): the
// input the reference's PartialConv2d convolves (networks.py:81,85), with the
// decoder's x2 nearest upsample (networks.py:297-301) folded in.
__global__ void pconv_src_materialize_kernel(const float* __restrict__ x0,
                                             const float* __restrict__ m0, int C0, int H0, int W0,
                                             const float* __restrict__ x1,
                                             const float* __restrict__ m1, int C1, int Hin,
                                             int Win, int64_t total, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int C = C0 + C1;
  const int x = (int)(t % Win);
  const int y = (int)((t / Win) % Hin);
  const int c = (int)((t / ((int64_t)Win * Hin)) % C);
  const int64_t n = t / ((int64_t)Win * Hin * C);
  float v;
  if (c < C0) {
    const int ys = (int)(((int64_t)y * H0) / Hin), xs = (int)(((int64_t)x * W0) / Win);
    const int64_t p = (int64_t)ys * W0 + xs;
    v = x0[(n * C0 + c) * H0 * W0 + p];
    if (m0) v *= m0[n * H0 * W0 + p];
  } else {
    const int64_t p = (int64_t)y * Win + x;
    v = x1[(n * C1 + (c - C0)) * (int64_t)Hin * Win + p];
    if (m1) v *= m1[n * (int64_t)Hin * Win + p];
  }
  out[t] = v;
}

// Gradient of one source from the gradient of the materialised input:
// dxs[n][c][ys][xs] (+)= ms[n][ys][xs] * sum of dxin[n][c_off + c] over the
// (Hin/Hs) x (Win/Ws) block that source pixel was replicated to (nearest
// upsample backward = block sum; the mask product's backward = x mask).
__global__ void pconv_src_grad_kernel(const float* __restrict__ dxin, int Cin, int Hin, int Win,
                                      int c_off, int C, int Hs, int Ws,
                                      const float* __restrict__ ms, int64_t total,
                                      float* __restrict__ dxs, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int xs = (int)(t % Ws);
  const int ys = (int)((t / Ws) % Hs);
  const int c = (int)((t / ((int64_t)Ws * Hs)) % C);
  const int64_t n = t / ((int64_t)Ws * Hs * C);
  const int fy = Hin / Hs, fx = Win / Ws;
  const float* src = dxin + (n * Cin + c_off + c) * (int64_t)Hin * Win;
  float s = 0.f;
  for (int a = 0; a < fy; ++a)
    for (int b = 0; b < fx; ++b) s += src[(int64_t)(ys * fy + a) * Win + xs * fx + b];
  if (ms) s *= ms[n * (int64_t)Hs * Ws + (int64_t)ys * Ws + xs];
  if (accumulate) s += dxs[t];
  dxs[t] = s;
}

// ------------------------------------------------------------ activation (+crop) backward
// act (ainp's ACT_* codes): 0 none, 1 ReLU, 2 LeakyReLU(slope) (derivative
// from the output's sign, as torch's inplace ReLU / LeakyReLU backward),
// 3 Tanh (1 - a^2).  g / a are
// [N, C, gH, gW] (the cropped output for the generator's last layer); the
// result lives on the conv grid [N, C, H, W] (zero outside the crop):
// gz = g * act'(a) and gc = gz * ratio[n][pixel] in rows of ldo.
__global__ void gen_act_bwd_kernel(const float* __restrict__ g, int gH, int gW,
                                   const float* __restrict__ a, int act, float slope,
                                   const float* __restrict__ ratio, int C, int H, int W,
                                   int64_t ldo, int64_t total, float* __restrict__ gz,
                                   float* __restrict__ gc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // total = N * C * ldo
  const int64_t row = t / ldo;
  const int64_t p = t - row * ldo;
  const int64_t P = (int64_t)H * W;
  if (p >= P) {
    gc[t] = 0.f;
    return;
  }
  const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
  float v = 0.f;
  if (y < gH && x < gW) {
    const int64_t i = row * gH * gW + (int64_t)y * gW + x;
    v = g[i];
    if (act == 1) {
      v = a[i] > 0.f ? v : 0.f;
    } else if (act == 2) {
      v = a[i] > 0.f ? v : v * slope;
    } else if (act == 3) {
      const float o = a[i];
      v = v * (1.f - o * o);
    }
  }
  if (gz) gz[row * P + p] = v;
  if (ratio) {
    const int64_t n = row / C;
    v *= ratio[n * P + p];
  }
  gc[t] = v;
}

// ------------------------------------------------------------ BatchNorm2d + LeakyReLU backward
// y: pre-BN conv output, z = y * scale + shift the BN output, a = leaky(z);
// ga the gradient w.r.t. a.  g' = ga * leaky'(z).  Train-mode BN backward
// (batch statistics save = [mean | rstd]):
//   dbeta = sum g',  dgamma = sum g' xhat,
//   dy = gamma rstd (g' - dbeta / M - xhat dgamma / M),  xhat = (y - mean) rstd.
constexpr int BA_CHUNK = 4096;

__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(
    const float* __restrict__ ga, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ save, float slope, int C,
    int64_t P, int chunks, double* __restrict__ partial) {
  const int64_t plane = blockIdx.x / chunks;
  const int ch = blockIdx.x % chunks;
  const int c = (int)(plane % C);
  const int64_t o0 = (int64_t)ch * BA_CHUNK;
  const int len = (int)((P - o0) < BA_CHUNK ? (P - o0) : BA_CHUNK);
  const float* gp = ga + plane * P + o0;
  const float* yp = y + plane * P + o0;
  const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
  float s1 = 0.f, s2 = 0.f;
  for (int e = threadIdx.x; e < len; e += 256) {
    const float yv = yp[e];
    const float gv = gp[e];
    const float gz = fmaf(yv, sc, sh) > 0.f ? gv : gv * slope;
    s1 += gz;
    s2 += gz * ((yv - mean) * rstd);
  }
  __shared__ double red[2][4];
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

// sums[c] = sum g', sums[C + c] = sum g' xhat over the [n][c][chunk] partials
__global__ void bn_act_bwd_sum_kernel(const double* __restrict__ partial, int N, int C,
                                      int chunks, double* __restrict__ sums) {
  const int c = blockIdx.x;
  double s1 = 0.0, s2 = 0.0;
  const int per = N * chunks;
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const int n = i / chunks, k = i % chunks;
    const int64_t b = ((int64_t)n * C + c) * chunks + k;
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
    sums[c] = r1[0] + r1[1] + r1[2] + r1[3];
    sums[C + c] = r2[0] + r2[1] + r2[2] + r2[3];
  }
}

// gc [N, C, ldo] = dy * ratio[n][p] (zero-padded rows), dgamma / dbeta
__global__ __launch_bounds__(256) void bn_act_bwd_apply_kernel(
    const float* __restrict__ ga, const float* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ save,
    const float* __restrict__ gamma, const double* __restrict__ sums, double inv_count,
    int eval, float slope, const float* __restrict__ ratio, int C, int64_t P, int64_t ldo,
    int64_t total, float* __restrict__ gc, float* __restrict__ dgamma,
    float* __restrict__ dbeta) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < C) {
    if (dbeta) dbeta[t] = (float)sums[t];
    if (dgamma) dgamma[t] = (float)sums[C + t];
  }
  if (t >= total) return;   // total = N * C * ldo
  const int64_t row = t / ldo;
  const int64_t p = t - row * ldo;
  if (p >= P) {
    gc[t] = 0.f;
    return;
  }
  const int c = (int)(row % C);
  const float sc = scale[c], sh = shift[c], mean = save[c], rstd = save[C + c];
  const float k = (gamma ? gamma[c] : 1.f) * rstd;
  // eval mode (running statistics): the statistics are constants, so the
  // batch-mean terms vanish
  const double ic = eval ? 0.0 : (inv_count > 0.0 ? inv_count : 1.0 / sums[2 * C]);
  const float m1 = (float)(sums[c] * ic);
  const float m2 = (float)(sums[C + c] * ic);
  const float yv = y[row * P + p];
  const float gv = ga[row * P + p];
  const float gz = fmaf(yv, sc, sh) > 0.f ? gv : gv * slope;
  float v = k * (gz - m1 - ((yv - mean) * rstd) * m2);
  if (ratio) v *= ratio[(row / C) * P + p];
  gc[t] = v;
}

// ------------------------------------------------------------ VGG19 input gradient
// MaxPool2d(2, 2) backward with torch's CPU argmax rule (first maximum in
// row-major window order; NaN wins): g [NC, H/2, W/2] -> gx [NC, H, W].
__global__ void maxpool2_bwd_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                    int H, int W, int64_t total, float* __restrict__ gx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // total = NC * H * W
  const int xx = (int)(t % W);
  const int yy = (int)((t / W) % H);
  const int64_t nc = t / ((int64_t)W * H);
  const int Ho = H / 2, Wo = W / 2;
  const int oy = yy >> 1, ox = xx >> 1;
  float v = 0.f;
  if (oy < Ho && ox < Wo) {
    const float* xp = x + nc * H * W;
    int best = 0;
    float mx = xp[(int64_t)(2 * oy) * W + 2 * ox];
    for (int k = 1; k < 4; ++k) {
      const float c = xp[(int64_t)(2 * oy + (k >> 1)) * W + 2 * ox + (k & 1)];
      if (c > mx || isnan(c)) {
        mx = c;
        best = k;
        if (isnan(c)) break;
      }
    }
    if (best == ((yy & 1) << 1 | (xx & 1))) v = g[(nc * Ho + oy) * Wo + ox];
  }
  gx[t] = v;
}

// gacc[n][i][j] = sum_c g[n][c][i][j] / std_c  (the ImageNet normalisation and
// the x3 channel repeat of loss.py:81 / ImageClassification, transposed)
__global__ void vgg_prep_bwd_norm_kernel(const float* __restrict__ g, int S, int64_t total,
                                         float* __restrict__ gacc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // N * S * S
  const int64_t SS = (int64_t)S * S;
  const int64_t n = t / SS, r = t - n * SS;
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  float s = 0.f;
  for (int c = 0; c < 3; ++c) s += g[(n * 3 + c) * SS + r] / stdv[c];
  gacc[t] = s;
}

// tmp[n][i][x] = sum_j cw(j, x) gacc[n][i][j]: the column pass of the
// antialiased bilinear resize, transposed (input column x gets every output
// column j whose taps cover it)
__global__ void vgg_prep_bwd_cols_kernel(const float* __restrict__ gacc, int S, int W,
                                         const int* __restrict__ cx0, const int* __restrict__ cn,
                                         const float* __restrict__ cw, int ctaps, int64_t total,
                                         float* __restrict__ tmp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // N * S * W
  const int x = (int)(t % W);
  const int64_t ni = t / W;   // n * S + i
  const float* gr = gacc + ni * S;
  float s = 0.f;
  for (int j = 0; j < S; ++j) {
    const int b = x - cx0[j];
    if (b >= 0 && b < cn[j]) s = fmaf(cw[j * ctaps + b], gr[j], s);
  }
  tmp[t] = s;
}

// gx[n][y][x] = 0.5 * [0 <= (x+1)/2 <= 1] * sum_i rw(i, y) tmp[n][i][x]: the
// row pass transposed, then clamp((x+1)/2, 0, 1)'s backward (loss.py:71,79)
__global__ void vgg_prep_bwd_rows_kernel(const float* __restrict__ tmp, const float* __restrict__ x,
                                         int S, int H, int W, const int* __restrict__ ry0,
                                         const int* __restrict__ rn, const float* __restrict__ rw,
                                         int rtaps, int64_t total, float* __restrict__ gx) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // N * H * W
  const int xx = (int)(t % W);
  const int yy = (int)((t / W) % H);
  const int64_t n = t / ((int64_t)W * H);
  const float* tp = tmp + n * S * W;
  float s = 0.f;
  for (int i = 0; i < S; ++i) {
    const int a = yy - ry0[i];
    if (a >= 0 && a < rn[i]) s = fmaf(rw[i * rtaps + a], tp[(int64_t)i * W + xx], s);
  }
  const float v = (x[t] + 1.0f) / 2.0f;
  gx[t] = (v >= 0.f && v <= 1.f) ? 0.5f * s : 0.f;
}

// out (+)= gs * scale * sign(a - b)   (nn.L1Loss backward; sign(0) = 0)
__global__ void absdiff_grad_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                    int64_t n, const float* __restrict__ gs, float scale,
                                    float* __restrict__ out, int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float d = a[t] - b[t];
  const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  float v = sg * scale * (gs ? *gs : 1.f);
  if (accumulate) v += out[t];
  out[t] = v;
}

// out[b][i][j] = gs * scale * (sign(Ga - Gb)[i][j] + sign(Ga - Gb)[j][i]): the
// Gram L1 gradient dG + dG^T that bmm(F, F^T)'s backward multiplies by F
__global__ void gram_sign_sym_kernel(const float* __restrict__ Ga, const float* __restrict__ Gb,
                                     int C, int64_t total, const float* __restrict__ gs,
                                     float scale, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;   // B * C * C
  const int j = (int)(t % C);
  const int i = (int)((t / C) % C);
  const int64_t b = t / ((int64_t)C * C);
  const int64_t tt = (b * C + j) * C + i;
  const float d0 = Ga[t] - Gb[t], d1 = Ga[tt] - Gb[tt];
  const float s0 = d0 > 0.f ? 1.f : (d0 < 0.f ? -1.f : 0.f);
  const float s1 = d1 > 0.f ? 1.f : (d1 < 0.f ? -1.f : 0.f);
  out[t] = (s0 + s1) * scale * (gs ? *gs : 1.f);
}

// calculate_losses' reconstruction terms (train.py:49-63) backward:
//   d/dg = gout0 sign(gm - om) m / (sum m + 1e-8)
//        + gout1 sign(gh - oh) h / (sum h + 1e-8) + gout2 sign(g - o) |o| / n_total
// with the forward's (all-reduced) sums s[5] and h = 1 - m.
__global__ void gan_recon_bwd_kernel(const float* __restrict__ g, const float* __restrict__ o,
                                     const float* __restrict__ m, int64_t n,
                                     const double* __restrict__ s5, const float* __restrict__ gout,
                                     double n_total, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float nv = (float)s5[1] + 1e-8f, nh = (float)s5[3] + 1e-8f;
  const float gv = g[t], ov = o[t], mv = m[t], hv = 1.f - mv;
  const float dv = gv * mv - ov * mv, dh = gv * hv - ov * hv, dw = gv - ov;
  auto sgn = [](float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); };
  float r = gout[0] * (sgn(dv) * mv / nv);
  r += gout[1] * (sgn(dh) * hv / nh);
  r += gout[2] * (float)((double)(sgn(dw) * fabsf(ov)) / n_total);
  out[t] = r;
}

// out[ci][co][kh][kw] = w[co][ci][K-1-kh][K-1-kw]: a stride-1 'same' conv's
// data gradient as a forward conv (conv_gen) over the output gradient
__global__ void conv_weight_flip_t_kernel(const float* __restrict__ w, int Cout, int Cin, int K,
                                          int64_t total, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int kw = (int)(t % K);
  const int kh = (int)((t / K) % K);
  const int co = (int)((t / ((int64_t)K * K)) % Cout);
  const int ci = (int)(t / ((int64_t)K * K * Cout));
  out[t] = w[(((int64_t)co * Cin + ci) * K + (K - 1 - kh)) * K + (K - 1 - kw)];
}

// out = leaky(y * scale[c] + shift[c]) (affine_act_kernel's arithmetic, out of
// place): the generator forward under autograd keeps the pre-BN y for the
// BatchNorm backward
__global__ void affine_leaky_out_kernel(const float* __restrict__ y,
                                        const float* __restrict__ scale,
                                        const float* __restrict__ shift, int C, int64_t HW,
                                        int64_t total, float slope, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int c = (int)((t / HW) % C);
  const float v = fmaf(y[t], scale[c], shift[c]);
  out[t] = v > 0.f ? v : v * slope;
}

inline dim3 grid1(int64_t n) { return dim3((unsigned)cdiv(n, 256)); }

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_affine_leaky_out(const float* y, const float* scale, const float* shift,
                                     int64_t N, int C, int64_t HW, float slope, float* out,
                                     void* stream) {
  if (!y || !scale || !shift || !out || N < 1 || C < 1 || HW < 1)
    return record_msg("ainp_affine_leaky_out: bad argument");
  const int64_t total = N * C * HW;
  hipLaunchKernelGGL(affine_leaky_out_kernel, grid1(total), dim3(256), 0, as_stream(stream), y,
                     scale, shift, C, HW, total, slope, out);
  return check_launch("affine_leaky_out");
}

extern "C" int ainp_pconv_src_materialize(const float* x0, const float* m0, int64_t N, int C0,
                                          int H0, int W0, const float* x1, const float* m1,
                                          int C1, int Hin, int Win, float* out, void* stream) {
  if (!x0 || !out || N < 1 || C0 < 1 || C1 < 0 || H0 < 1 || W0 < 1 || Hin < H0 || Win < W0 ||
      Hin % H0 || Win % W0 || (C1 > 0 && !x1))
    return record_msg("ainp_pconv_src_materialize: bad argument");
  const int64_t total = N * (C0 + C1) * (int64_t)Hin * Win;
  if (total >= ((int64_t)1 << 40)) return record_msg("ainp_pconv_src_materialize: too large");
  hipLaunchKernelGGL(pconv_src_materialize_kernel, grid1(total), dim3(256), 0, as_stream(stream),
                     x0, m0, C0, H0, W0, x1, m1, C1, Hin, Win, total, out);
  return check_launch("pconv_src_materialize");
}

extern "C" int ainp_pconv_src_grad(const float* dxin, int64_t N, int Cin, int Hin, int Win,
                                   int c_off, int C, int Hs, int Ws, const float* ms, float* dxs,
                                   int accumulate, void* stream) {
  if (!dxin || !dxs || N < 1 || C < 1 || c_off < 0 || c_off + C > Cin || Hs < 1 || Ws < 1 ||
      Hin % Hs || Win % Ws || accumulate < 0 || accumulate > 1)
    return record_msg("ainp_pconv_src_grad: bad argument");
  const int64_t total = N * C * (int64_t)Hs * Ws;
  hipLaunchKernelGGL(pconv_src_grad_kernel, grid1(total), dim3(256), 0, as_stream(stream), dxin,
                     Cin, Hin, Win, c_off, C, Hs, Ws, ms, total, dxs, accumulate);
  return check_launch("pconv_src_grad");
}

extern "C" int ainp_gen_act_bwd(const float* g, int gH, int gW, const float* a, int act,
                                float slope, const float* ratio, int64_t N, int C, int H, int W,
                                int64_t ldo, float* gz, float* gc, void* stream) {
  if (!g || !gc || N < 1 || C < 1 || gH < 1 || gW < 1 || gH > H || gW > W ||
      ldo < (int64_t)H * W || act < 0 || act > 3 || (act && !a))
    return record_msg("ainp_gen_act_bwd: bad argument");
  const int64_t total = N * C * ldo;
  hipLaunchKernelGGL(gen_act_bwd_kernel, grid1(total), dim3(256), 0, as_stream(stream), g, gH,
                     gW, a, act, slope, ratio, C, H, W, ldo, total, gz, gc);
  return check_launch("gen_act_bwd");
}

extern "C" size_t ainp_bn_act_bwd_workspace(int64_t N, int C, int64_t P) {
  return (size_t)(N * C * cdiv(P, BA_CHUNK)) * 2 * sizeof(double);
}

extern "C" int ainp_bn_act_bwd_reduce(const float* ga, const float* y, const float* scale,
                                      const float* shift, const float* save, float slope,
                                      int64_t N, int C, int64_t P, void* workspace, double* sums,
                                      void* stream) {
  if (!ga || !y || !scale || !shift || !save || !workspace || !sums || N < 1 || C < 1 || P < 1)
    return record_msg("ainp_bn_act_bwd_reduce: bad argument");
  const int chunks = (int)cdiv(P, BA_CHUNK);
  hipStream_t s = as_stream(stream);
  double* partial = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(bn_act_bwd_reduce_kernel, dim3((unsigned)(N * C * chunks)), dim3(256), 0, s,
                     ga, y, scale, shift, save, slope, C, P, chunks, partial);
  int rc = check_launch("bn_act_bwd_reduce");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_act_bwd_sum_kernel, dim3(C), dim3(256), 0, s, partial, (int)N, C, chunks,
                     sums);
  return check_launch("bn_act_bwd_sum");
}

extern "C" int ainp_bn_act_bwd_apply(const float* ga, const float* y, const float* scale,
                                     const float* shift, const float* save, const float* gamma,
                                     const double* sums, int64_t count, float slope,
                                     const float* ratio, int64_t N, int C, int64_t P, int64_t ldo,
                                     float* gc, float* dgamma, float* dbeta, void* stream) {
  if (!ga || !y || !scale || !shift || !save || !sums || !gc || N < 1 || C < 1 || P < 1 ||
      ldo < P || count < -1)
    return record_msg("ainp_bn_act_bwd_apply: bad argument");
  const int64_t total = N * C * ldo;
  // count: > 0 batch statistics over count elements; 0: the count is sums[2C];
  // -1: eval mode (save = running mean | rstd)
  const double inv = count > 0 ? 1.0 / (double)count : 0.0;
  const int eval = count < 0 ? 1 : 0;
  const int64_t launch = total > C ? total : C;
  hipLaunchKernelGGL(bn_act_bwd_apply_kernel, grid1(launch), dim3(256), 0, as_stream(stream), ga,
                     y, scale, shift, save, gamma, sums, inv, eval, slope, ratio, C, P, ldo, total,
                     gc,
                     dgamma, dbeta);
  return check_launch("bn_act_bwd_apply");
}

extern "C" int ainp_maxpool2_bwd(const float* g, const float* x, int64_t NC, int H, int W,
                                 float* gx, void* stream) {
  if (!g || !x || !gx || NC < 1 || H < 2 || W < 2)
    return record_msg("ainp_maxpool2_bwd: bad argument");
  const int64_t total = NC * (int64_t)H * W;
  hipLaunchKernelGGL(maxpool2_bwd_kernel, grid1(total), dim3(256), 0, as_stream(stream), g, x, H,
                     W, total, gx);
  return check_launch("maxpool2_bwd");
}

extern "C" size_t ainp_vgg_prep_bwd_workspace(int64_t N, int W, int S) {
  return (size_t)(N * (int64_t)S * S + N * (int64_t)S * W) * sizeof(float);
}

extern "C" int ainp_vgg_prep_bwd(const float* g, const float* x, int64_t N, int H, int W,
                                 const int* ry0, const int* rn, const float* rw, int rtaps,
                                 const int* cx0, const int* cn, const float* cw, int ctaps, int S,
                                 void* workspace, float* gx, void* stream) {
  if (!g || !x || !ry0 || !rn || !rw || !cx0 || !cn || !cw || !workspace || !gx || N < 1 ||
      H < 1 || W < 1 || S < 1 || rtaps < 1 || ctaps < 1)
    return record_msg("ainp_vgg_prep_bwd: bad argument");
  hipStream_t s = as_stream(stream);
  float* gacc = reinterpret_cast<float*>(workspace);
  float* tmp = gacc + N * (int64_t)S * S;
  const int64_t t0 = N * (int64_t)S * S, t1 = N * (int64_t)S * W, t2 = N * (int64_t)H * W;
  hipLaunchKernelGGL(vgg_prep_bwd_norm_kernel, grid1(t0), dim3(256), 0, s, g, S, t0, gacc);
  int rc = check_launch("vgg_prep_bwd_norm");
  if (rc) return rc;
  hipLaunchKernelGGL(vgg_prep_bwd_cols_kernel, grid1(t1), dim3(256), 0, s, gacc, S, W, cx0, cn, cw,
                     ctaps, t1, tmp);
  rc = check_launch("vgg_prep_bwd_cols");
  if (rc) return rc;
  hipLaunchKernelGGL(vgg_prep_bwd_rows_kernel, grid1(t2), dim3(256), 0, s, tmp, x, S, H, W, ry0,
                     rn, rw, rtaps, t2, gx);
  return check_launch("vgg_prep_bwd_rows");
}

extern "C" int ainp_absdiff_grad(const float* a, const float* b, int64_t n, const float* gscale,
                                 float scale, float* out, int accumulate, void* stream) {
  if (!a || !b || !out || n < 1 || accumulate < 0 || accumulate > 1)
    return record_msg("ainp_absdiff_grad: bad argument");
  hipLaunchKernelGGL(absdiff_grad_kernel, grid1(n), dim3(256), 0, as_stream(stream), a, b, n,
                     gscale, scale, out, accumulate);
  return check_launch("absdiff_grad");
}

extern "C" int ainp_gram_sign_sym(const float* Ga, const float* Gb, int64_t B, int C,
                                  const float* gscale, float scale, float* out, void* stream) {
  if (!Ga || !Gb || !out || B < 1 || C < 1) return record_msg("ainp_gram_sign_sym: bad argument");
  const int64_t total = B * (int64_t)C * C;
  hipLaunchKernelGGL(gram_sign_sym_kernel, grid1(total), dim3(256), 0, as_stream(stream), Ga, Gb,
                     C, total, gscale, scale, out);
  return check_launch("gram_sign_sym");
}

extern "C" int ainp_gan_recon_bwd(const float* g, const float* o, const float* m, int64_t n,
                                  const double* sums5, const float* gout3, double n_total,
                                  float* out, void* stream) {
  if (!g || !o || !m || !sums5 || !gout3 || !out || n < 1 || !(n_total > 0))
    return record_msg("ainp_gan_recon_bwd: bad argument");
  hipLaunchKernelGGL(gan_recon_bwd_kernel, grid1(n), dim3(256), 0, as_stream(stream), g, o, m, n,
                     sums5, gout3, n_total, out);
  return check_launch("gan_recon_bwd");
}

extern "C" int ainp_conv_weight_flip_t(const float* w, int Cout, int Cin, int K, float* out,
                                       void* stream) {
  if (!w || !out || Cout < 1 || Cin < 1 || K < 1)
    return record_msg("ainp_conv_weight_flip_t: bad argument");
  const int64_t total = (int64_t)Cout * Cin * K * K;
  hipLaunchKernelGGL(conv_weight_flip_t_kernel, grid1(total), dim3(256), 0, as_stream(stream), w,
                     Cout, Cin, K, total, out);
  return check_launch("conv_weight_flip_t");
}
