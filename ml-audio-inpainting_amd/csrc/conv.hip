// conv.hip — 3x3 / stride 1 / pad 1 convolution over [N, C, F, T] on the
// gfx950 f32-input MFMA (v_mfma_f32_16x16x4_f32, exact fp32).
//
// Replaces nn.Conv2d(k=3, p=1) of models/CNNBLSTM/model.py:35-60 (forward,
// data gradient, weight gradient).  Implicit GEMM, nothing im2col'd in HBM:
//   forward  D[pixel][co]       = sum_{ci,tap} act(x)[ci][pixel+tap] * w[co][ci][tap]
//   dgrad    same kernel on dy with w'[ci][co][tap] = w[co][ci][8-tap]
//   wgrad    D[co][(tap,ci)]    = sum_pixel dy[co][pixel] * act(x)[ci][pixel+tap]
// act(x) = relu(x*scale[c]+shift[c]) is the previous BatchNorm2d+ReLU applied
// while staging the input tile into LDS (never materialised in HBM); zero
// padding is applied after act, as nn.Conv2d pads its post-ReLU input.
//
// Forward tile: one workgroup = one example, 8 rows (f) x 48 columns (t);
// each of the 4 waves owns 2 rows x 3 sixteen-pixel MFMA row tiles x CT
// sixteen-channel column tiles (CT = ceil(Cout/16)).  K = Cin*9 is walked in
// chunks of 8 input channels; LDS k order inside a chunk is (tap, ci) so the
// A-operand address is lane-constant + compile-time immediate.
#include <stdlib.h>

#include "common.h"

namespace ainp {

// ---------------------------------------------------------------- forward
constexpr int CV_FT = 8;          // rows per tile
constexpr int CV_TT = 48;         // columns per tile (3 MFMA tiles)
constexpr int CV_CK = 8;          // input channels per K chunk
constexpr int CV_LDT = 52;        // LDS row length (>= TT+2)
constexpr int CV_PLANE = 528;     // >= (FT+2)*LDT, == 16 mod 32 (conflict-free A)
constexpr int CV_KCH = CV_CK * 9; // k per chunk = 72

template <int CT>
struct FwdLds {
  static constexpr int LDW = (CT * 16) % 32 == 0 ? CT * 16 + 16 : CT * 16;
  static constexpr int IN = CV_CK * CV_PLANE;
  static constexpr int WT = CV_KCH * LDW;
};

// Staging is register double-buffered: chunk c+1's global loads are issued
// right after chunk c is committed to LDS, so they are in flight during
// chunk c's MFMAs (a load->store loop per element would serialise one HBM
// round trip per element).
// EX (exact shapes: Cin % 8 == 0, Cout == 16*CT, a sample's planes within
// 2^31 bytes): staging without per-element predicates -- clamped-address
// buffer loads, out-of-image values selected to zero at commit -- so the
// compiler emits no branch/vmcnt(0) per element.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ int clampi(int v, int lo, int hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

template <int CT, bool DGRAD, bool EX = false>
__global__ __launch_bounds__(256, 2) void conv3x3_fwd_mfma(
    const float* __restrict__ x, const float* __restrict__ w,
    const float* __restrict__ bias, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, float* __restrict__ y,
    double* __restrict__ stats, int Cin, int Cout, int H, int W) {
  using L = FwdLds<CT>;
  __shared__ __attribute__((aligned(16))) float s_in[L::IN];
  __shared__ __attribute__((aligned(16))) float s_w[L::WT];
  __shared__ double s_red[2 * 4 * CT * 16];

  const int n = blockIdx.z;
  const int f0 = blockIdx.y * CV_FT;
  const int t0 = blockIdx.x * CV_TT;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, kq = lane >> 4;
  const int64_t HW = (int64_t)H * W;
  const float* xn = x + (int64_t)n * Cin * HW;

  f32x4 acc[2][3][CT];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int c = 0; c < CT; ++c) acc[r][p][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Staging map (no per-element index decode): lane = tile column (50 of 64
  // lanes active), input row r = wave + 4*i with row order (rr, ci):
  // rr = i>>1, ci = wave + 4*(i&1); weight row k = wave + 4*i with
  // tap = i>>1, ci = wave + 4*(i&1), lane = output channel.
  constexpr int NIR = CV_CK * (CV_FT + 2) / 4;   // 20 input rows per thread
  constexpr int NWR = CV_KCH / 4;                // 18 weight rows per thread
  float pin[NIR], pw[NWR];
  const int tcol = t0 - 1 + lane;                // input column of this lane
  const bool col_ok = lane < CV_TT + 2 && tcol >= 0 && tcol < W;
  auto fetch = [&](int ci0) {
    const int cg0 = ci0 + wave;
    if constexpr (EX) {
      int plane = (int)(HW * 4);
      asm volatile("" : "+s"(plane));  // per-plane offsets stay per chunk, not hoisted
      const __amdgpu_buffer_rsrc_t rx = buf_rsrc(xn);
      const int tcl = clampi(tcol, 0, W - 1);
#pragma unroll
      for (int i = 0; i < NIR; ++i) {
        const int rr = i >> 1, f = clampi(f0 - 1 + rr, 0, H - 1);
        pin[i] = buf_ld(rx, (f * W + tcl) * 4, (cg0 + 4 * (i & 1)) * plane);
      }
      const int lc = lane < CT * 16 ? lane : CT * 16 - 1;
#pragma unroll
      for (int i = 0; i < NWR; ++i) {
        const int tap = i >> 1, cg = cg0 + 4 * (i & 1);
        pw[i] = DGRAD ? w[((int64_t)cg * Cout + lc) * 9 + (8 - tap)]
                      : w[((int64_t)lc * Cin + cg) * 9 + tap];
      }
      return;
    }
    const float* xb = xn + (int64_t)cg0 * HW + (int64_t)(f0 - 1) * W + tcol;
#pragma unroll
    for (int i = 0; i < NIR; ++i) {
      const int rr = i >> 1, cg = cg0 + 4 * (i & 1), f = f0 - 1 + rr;
      float v = 0.f;
      if (col_ok && cg < Cin && f >= 0 && f < H)
        v = xb[(int64_t)(4 * (i & 1)) * HW + (int64_t)rr * W];
      pin[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NWR; ++i) {
      const int tap = i >> 1, cg = cg0 + 4 * (i & 1);
      float v = 0.f;
      if (lane < CT * 16 && lane < Cout && cg < Cin)
        v = DGRAD ? w[((int64_t)cg * Cout + lane) * 9 + (8 - tap)]   // w'[co][cg] = w[cg][co] flipped
                  : w[((int64_t)lane * Cin + cg) * 9 + tap];
      pw[i] = v;
    }
  };
  auto commit = [&](int ci0) {
    const int cg0 = ci0 + wave;
    if constexpr (EX) {
#pragma unroll
      for (int i = 0; i < NIR; ++i) {
        const int rr = i >> 1, ci = wave + 4 * (i & 1), cg = cg0 + 4 * (i & 1);
        const int f = f0 - 1 + rr;
        const bool ok = col_ok && f >= 0 && f < H;
        float v = pin[i];
        if (in_scale) v = fmaxf(fmaf(v, in_scale[cg], in_shift[cg]), 0.f);
        if (lane < CV_TT + 2) s_in[ci * CV_PLANE + rr * CV_LDT + lane] = ok ? v : 0.f;
      }
#pragma unroll
      for (int i = 0; i < NWR; ++i) {
        const int k = (i >> 1) * 8 + wave + 4 * (i & 1);
        if (lane < CT * 16) s_w[k * L::LDW + lane] = pw[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NIR; ++i) {
      const int rr = i >> 1, ci = wave + 4 * (i & 1), cg = cg0 + 4 * (i & 1);
      float v = pin[i];
      if (in_scale) {
        const int f = f0 - 1 + rr;
        const bool ok = col_ok && cg < Cin && f >= 0 && f < H;
        v = ok ? fmaxf(fmaf(v, in_scale[cg], in_shift[cg]), 0.f) : 0.f;
      }
      if (lane < CV_TT + 2) s_in[ci * CV_PLANE + rr * CV_LDT + lane] = v;
    }
#pragma unroll
    for (int i = 0; i < NWR; ++i) {
      const int k = (i >> 1) * 8 + wave + 4 * (i & 1);
      if (lane < CT * 16) s_w[k * L::LDW + lane] = pw[i];
    }
  };

  const int nchunk = (Cin + CV_CK - 1) / CV_CK;
  fetch(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    if (ch > 0) __syncthreads();  // previous chunk's LDS reads are done
    commit(ch * CV_CK);
    __syncthreads();
    if (ch + 1 < nchunk) fetch((ch + 1) * CV_CK);

    const float* a_base = s_in + kq * CV_PLANE + li;
    const float* b_base = s_w + kq * L::LDW + li;
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int tap = s >> 1, cb = (s & 1) * 4;
      const int df = tap / 3, dt = tap % 3;
      float bf[CT];
#pragma unroll
      for (int c = 0; c < CT; ++c) bf[c] = b_base[(s * 4) * L::LDW + c * 16];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const float af =
              a_base[cb * CV_PLANE + (wave * 2 + r + df) * CV_LDT + p * 16 + dt];
#pragma unroll
          for (int c = 0; c < CT; ++c) acc[r][p][c] = mfma16x16x4(af, bf[c], acc[r][p][c]);
        }
    }
  }

  // epilogue: D[pixel = 4*kq + j][co = li] in register j
  float* yn = y + (int64_t)n * Cout * HW;
  float psum[CT], psq[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    psum[c] = 0.f;
    psq[c] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < CT; ++c) {
    const int co = c * 16 + li;
    const bool cok = co < Cout;
    const float bv = (bias && cok) ? bias[co] : 0.f;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int f = f0 + wave * 2 + r;
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int t = t0 + p * 16 + kq * 4 + j;
          if (cok && f < H && t < W) {
            const float v = acc[r][p][c][j] + bv;
            yn[(int64_t)co * HW + (int64_t)f * W + t] = v;
            psum[c] += v;
            psq[c] += v * v;
          }
        }
    }
  }
  if (stats) {
    // reduce over the 4 lane groups sharing a channel, then over waves
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      double a = psum[c], b = psq[c];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if (kq == 0) {
        s_red[(wave * CT + c) * 16 + li] = a;
        s_red[4 * CT * 16 + (wave * CT + c) * 16 + li] = b;
      }
    }
    __syncthreads();
    const int64_t part = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    for (int co = tid; co < Cout; co += 256) {
      const int c = co >> 4, l = co & 15;
      double a = 0.0, b = 0.0;
      for (int wv = 0; wv < 4; ++wv) {
        a += s_red[(wv * CT + c) * 16 + l];
        b += s_red[4 * CT * 16 + (wv * CT + c) * 16 + l];
      }
      stats[part * 2 * Cout + co] = a;
      stats[part * 2 * Cout + Cout + co] = b;
    }
  }
}

// ---------------------------------------------------------------- wgrad
// Persistent workgroups each reduce a strided set of 2x64 pixel tiles into
// register accumulators D[co][j], j = tap*Cin + ci, then write one partial
// slab; a two-stage kernel sums the slabs in fixed order (deterministic).
// Tile t+1's act(x) halo and dy are prefetched into registers while tile t's
// MFMAs run.
constexpr int WG_FT = 2, WG_TT = 64;
constexpr int WG_LDT = 68;         // >= TT+2
constexpr int WG_XPLANE = 290;     // >= (FT+2)*LDT = 272, == 2 mod 32
constexpr int WG_GPLANE = 130;     // >= FT*TT = 128, == 2 mod 32 (dy tile)
constexpr int WG_CIMAX = 32;       // input channels staged per pass

template <int CT, int JT>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_mfma(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int N, int Cin, int Cout, int H, int W,
    int ci0, int cin_pass) {
  // this pass covers input channels [ci0, ci0+cin_pass), j = tap*cin_pass+ci
  __shared__ __attribute__((aligned(16))) float s_x[WG_CIMAX * WG_XPLANE];
  __shared__ __attribute__((aligned(16))) float s_g[CT * 16 * WG_GPLANE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, kq = lane >> 4;
  // wave -> (co tile, subset of j tiles)
  constexpr int WPC = 4 / CT;                 // waves per co tile
  constexpr int JPW = (JT + WPC - 1) / WPC;   // j tiles per wave
  const int ct = wave / WPC;
  const int jt0 = (wave % WPC) * JPW;
  const int J = 9 * cin_pass;

  // per-lane B offsets (ci, tap) for each of the wave's j tiles
  int boff[JPW];
#pragma unroll
  for (int q = 0; q < JPW; ++q) {
    const int j = (jt0 + q) * 16 + li;
    int o = 0;
    if (j < J) {
      const int tap = j / cin_pass, ci = j % cin_pass;
      o = ci * WG_XPLANE + (tap / 3) * WG_LDT + (tap % 3);
    }
    boff[q] = o;
  }
  f32x4 acc[JPW];
#pragma unroll
  for (int q = 0; q < JPW; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f;

  const int tiles_t = (W + WG_TT - 1) / WG_TT;
  const int tiles_f = (H + WG_FT - 1) / WG_FT;
  const int64_t ntiles = (int64_t)N * tiles_f * tiles_t;
  const int64_t HW = (int64_t)H * W;
  const bool ct_ok = ct < CT && wave < CT * WPC;

  // Staging map: lane = tile column.  act(x) interior: wave = halo row rr
  // (0..3), loop index = input channel; the 2 halo columns x 4 rows x
  // cin_pass are one element per thread.  dy: rr = wave&1, co = (wave>>1)+2i.
  constexpr int NGR = CT * 8;                    // dy rows per thread
  float px[WG_CIMAX], pxh, pg[NGR];
  const int hside = tid & 1, hrr = (tid >> 1) & 3, hci = tid >> 3;  // halo element
  auto tile_coords = [&](int64_t tile, int& n, int& f0, int& t0) {
    const int tt = tile % tiles_t;
    const int tf = (tile / tiles_t) % tiles_f;
    n = (int)(tile / ((int64_t)tiles_t * tiles_f));
    f0 = tf * WG_FT;
    t0 = tt * WG_TT;
  };
  auto fetch = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    const int f = f0 - 1 + wave, t = t0 + lane;
    const bool ok = f >= 0 && f < H && t < W;
    const float* xb = x + ((int64_t)n * Cin + ci0) * HW + (int64_t)f * W + t;
#pragma unroll
    for (int i = 0; i < WG_CIMAX; ++i)
      px[i] = (ok && i < cin_pass) ? xb[(int64_t)i * HW] : 0.f;
    {
      const int fh = f0 - 1 + hrr, th = hside ? t0 + WG_TT : t0 - 1;
      pxh = (hci < cin_pass && fh >= 0 && fh < H && th >= 0 && th < W)
                ? x[((int64_t)n * Cin + ci0 + hci) * HW + (int64_t)fh * W + th]
                : 0.f;
    }
    const int fg = f0 + (wave & 1);
    const bool gok = fg < H && t < W;
    const float* gb = dy + ((int64_t)n * Cout + (wave >> 1)) * HW + (int64_t)fg * W + t;
#pragma unroll
    for (int i = 0; i < NGR; ++i) {
      const int co = (wave >> 1) + 2 * i;
      pg[i] = (gok && co < Cout) ? gb[(int64_t)(2 * i) * HW] : 0.f;
    }
  };
  auto commit = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    const int f = f0 - 1 + wave, t = t0 + lane;
    const bool ok = f >= 0 && f < H && t < W;
#pragma unroll
    for (int i = 0; i < WG_CIMAX; ++i) {
      if (i < cin_pass) {
        float v = px[i];
        if (in_scale) v = ok ? fmaxf(fmaf(v, in_scale[ci0 + i], in_shift[ci0 + i]), 0.f) : 0.f;
        s_x[i * WG_XPLANE + wave * WG_LDT + lane + 1] = v;
      }
    }
    if (hci < cin_pass) {
      float v = pxh;
      if (in_scale) {
        const int fh = f0 - 1 + hrr, th = hside ? t0 + WG_TT : t0 - 1;
        const bool hok = fh >= 0 && fh < H && th >= 0 && th < W;
        v = hok ? fmaxf(fmaf(v, in_scale[ci0 + hci], in_shift[ci0 + hci]), 0.f) : 0.f;
      }
      s_x[hci * WG_XPLANE + hrr * WG_LDT + (hside ? WG_TT + 1 : 0)] = v;
    }
#pragma unroll
    for (int i = 0; i < NGR; ++i) {
      const int co = (wave >> 1) + 2 * i;
      s_g[co * WG_GPLANE + (wave & 1) * WG_TT + lane] = pg[i];
    }
  };

  int64_t tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    commit(tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
    if (ct_ok) {
      const float* ga = s_g + (ct * 16 + li) * WG_GPLANE + kq;
#pragma unroll 4
      for (int s = 0; s < WG_FT * WG_TT / 4; ++s) {
        // pixel for this lane: p = 4s + kq  -> (row, col)
        const int p = 4 * s + kq;
        const int rr = p / WG_TT, cc = p % WG_TT;
        const float af = ga[4 * s];
        dbias += af;
        const float* xb = s_x + rr * WG_LDT + cc;
#pragma unroll
        for (int q = 0; q < JPW; ++q) acc[q] = mfma16x16x4(af, xb[boff[q]], acc[q]);
      }
    }
    __syncthreads();
  }
  // write partial slab: [Cout_pad=CT*16][J+1] for this block (+ bias column)
  float* slab = partial + (int64_t)blockIdx.x * (CT * 16) * (J + 1);
  if (ct_ok) {
#pragma unroll
    for (int q = 0; q < JPW; ++q) {
      const int j = (jt0 + q) * 16 + li;
      if (jt0 + q < JT && j < J) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = ct * 16 + kq * 4 + r;
          slab[co * (J + 1) + j] = acc[q][r];
        }
      }
    }
    // bias partial: lanes li hold co = ct*16+li summed over their kq pixels
    float d = dbias;
    d += __shfl_xor(d, 16, 64);
    d += __shfl_xor(d, 32, 64);
    if (kq == 0 && (wave % WPC) == 0) slab[(ct * 16 + li) * (J + 1) + J] = d;
  }
}

// Specialised weight gradient for the model's channel pairs: CP input channels
// per pass (16 or 32) and CO = Cout (16, 32 or 64) are compile-time, so
//  * staging has no per-element predicates: every load is a buffer load at a
//    clamped (always in-range) address, channel planes addressed by a scalar
//    soffset, and out-of-image values are selected to zero at commit;
//  * every LDS fragment address is a per-lane base + compile-time immediate,
//    and each 4-pixel step issues all of its B-fragment reads before its MFMAs
//    (the generic kernel above ran out of registers and serialised one LDS
//    round trip per MFMA).
// Same tiles, partial-slab format and deterministic reduction as
// conv3x3_wgrad_mfma.

template <int CP, int CO>
struct WgradT {
  static constexpr int CT = CO / 16;                      // co tiles
  static constexpr int JT = 9 * CP / 16;                  // j tiles
  static constexpr int WPC0 = 4 / CT, WPC1 = (JT + 8) / 9;
  static constexpr int WPC = WPC0 > WPC1 ? WPC0 : WPC1;   // waves per co tile
  static constexpr int NW = CT * WPC;                     // waves (4 or 8)
  static constexpr int JPW = (JT + WPC - 1) / WPC;        // j tiles per wave (<= 9)
};

template <int CP, int CO>
__global__ __launch_bounds__((WgradT<CP, CO>::NW * 64), (WgradT<CP, CO>::NW / 2)) void conv3x3_wgrad_t(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int N, int Cin, int H, int W, int ci0) {
  using T = WgradT<CP, CO>;
  constexpr int J = 9 * CP, JT = T::JT, WPC = T::WPC, JPW = T::JPW, NW = T::NW;
  constexpr int XH = NW / 4;                  // channel groups of the x interior rows
  constexpr int NXR = CP / XH;                // x rows per thread
  constexpr int NGR = CO * 2 / NW;            // dy rows per thread
  static_assert(CP % 16 == 0 && CP <= WG_CIMAX && CO % 16 == 0 && CO <= 64, "shape");
  static_assert(8 * CP <= NW * 64, "halo: one element per thread");
  __shared__ __attribute__((aligned(16))) float s_x[CP * WG_XPLANE];
  __shared__ __attribute__((aligned(16))) float s_g[CO * WG_GPLANE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, kq = lane >> 4;
  const int ct = wave / WPC;
  const int jt0 = (wave % WPC) * JPW;

  // B offset of j tile q for this lane (ci = li within the tile), row 0 col 0
  int boff[JPW];
#pragma unroll
  for (int q = 0; q < JPW; ++q) {
    const int jt = jt0 + q;
    const int tap = CP == 32 ? (jt >> 1) : jt;
    const int cih = CP == 32 ? (jt & 1) * 16 : 0;
    boff[q] = (cih + li) * WG_XPLANE + (tap / 3) * WG_LDT + (tap % 3) + kq;
  }
  f32x4 acc[JPW];
#pragma unroll
  for (int q = 0; q < JPW; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f;

  const int tiles_t = (W + WG_TT - 1) / WG_TT;
  const int tiles_f = (H + WG_FT - 1) / WG_FT;
  const int64_t ntiles = (int64_t)N * tiles_f * tiles_t;
  const int64_t HW = (int64_t)H * W;

  // staging map: x interior row xr = wave&3 (halo rows f0-1..f0+2), channels
  // xc0 + XH*i; dy row gr = wave&1, channels gc0 + (NW/2)*i; one x halo-column
  // element per thread
  const int xr = wave & 3, xc0 = wave >> 2;
  const int gr = wave & 1, gc0 = wave >> 1;
  float px[NXR], pxh, pg[NGR];
  const int hside = tid & 1, hrr = (tid >> 1) & 3, hci = tid >> 3;
  auto tile_coords = [&](int64_t tile, int& n, int& f0, int& t0) {
    const int tt = tile % tiles_t;
    const int tf = (tile / tiles_t) % tiles_f;
    n = (int)(tile / ((int64_t)tiles_t * tiles_f));
    f0 = tf * WG_FT;
    t0 = tt * WG_TT;
  };
  auto fetch = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    int plane = (int)(HW * 4);
    asm volatile("" : "+s"(plane));  // keep the per-plane offsets out of the tile loop
    const int tc = clampi(t0 + lane, 0, W - 1);
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x + ((int64_t)n * Cin + ci0) * HW);
    const int vo = (clampi(f0 - 1 + xr, 0, H - 1) * W + tc) * 4;
#pragma unroll
    for (int i = 0; i < NXR; ++i) px[i] = buf_ld(rx, vo, (xc0 + XH * i) * plane);
    {
      const int fh = clampi(f0 - 1 + hrr, 0, H - 1);
      const int th = clampi(hside ? t0 + WG_TT : t0 - 1, 0, W - 1);
      pxh = buf_ld(rx, (fh * W + th) * 4, (hci < CP ? hci : CP - 1) * plane);
    }
    const __amdgpu_buffer_rsrc_t rg = buf_rsrc(dy + (int64_t)n * CO * HW);
    const int vg = (clampi(f0 + gr, 0, H - 1) * W + tc) * 4;
#pragma unroll
    for (int i = 0; i < NGR; ++i) pg[i] = buf_ld(rg, vg, (gc0 + (NW / 2) * i) * plane);
  };
  auto commit = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    const int f = f0 - 1 + xr, t = t0 + lane;
    const bool ok = f >= 0 && f < H && t < W;
    if (in_scale) {
#pragma unroll
      for (int i = 0; i < NXR; ++i) {
        const int ci = xc0 + XH * i;
        s_x[ci * WG_XPLANE + xr * WG_LDT + lane + 1] =
            ok ? fmaxf(fmaf(px[i], in_scale[ci0 + ci], in_shift[ci0 + ci]), 0.f) : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NXR; ++i)
        s_x[(xc0 + XH * i) * WG_XPLANE + xr * WG_LDT + lane + 1] = ok ? px[i] : 0.f;
    }
    if (hci < CP) {
      const int fh = f0 - 1 + hrr, th = hside ? t0 + WG_TT : t0 - 1;
      const bool hok = fh >= 0 && fh < H && th >= 0 && th < W;
      float v = pxh;
      if (in_scale) v = fmaxf(fmaf(v, in_scale[ci0 + hci], in_shift[ci0 + hci]), 0.f);
      s_x[hci * WG_XPLANE + hrr * WG_LDT + (hside ? WG_TT + 1 : 0)] = hok ? v : 0.f;
    }
    const bool gok = f0 + gr < H && t < W;
#pragma unroll
    for (int i = 0; i < NGR; ++i)
      s_g[(gc0 + (NW / 2) * i) * WG_GPLANE + gr * WG_TT + lane] = gok ? pg[i] : 0.f;
  };

  const float* ga = s_g + (ct * 16 + li) * WG_GPLANE + kq;
  int64_t tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    commit(tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
#pragma unroll
    for (int s = 0; s < WG_FT * WG_TT / 4; ++s) {
      // pixel p = 4s + kq -> row s/16, column 4(s%16) + kq (kq folded into the bases)
      const int roff = (s >> 4) * WG_LDT + (s & 15) * 4;
      const float af = ga[4 * s];
      dbias += af;
      float bv[JPW];
#pragma unroll
      for (int q = 0; q < JPW; ++q) bv[q] = s_x[boff[q] + roff];
#pragma unroll
      for (int q = 0; q < JPW; ++q)
        if (JPW * WPC == JT || jt0 + q < JT) acc[q] = mfma16x16x4(af, bv[q], acc[q]);
    }
    __syncthreads();
  }
  float* slab = partial + (int64_t)blockIdx.x * CO * (J + 1);
#pragma unroll
  for (int q = 0; q < JPW; ++q) {
    const int j = (jt0 + q) * 16 + li;
    if (jt0 + q < JT) {
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(ct * 16 + kq * 4 + r) * (J + 1) + j] = acc[q][r];
    }
  }
  float d = dbias;
  d += __shfl_xor(d, 16, 64);
  d += __shfl_xor(d, 32, 64);
  if (kq == 0 && (wave % WPC) == 0) slab[(ct * 16 + li) * (J + 1) + J] = d;
}

// Stage 1: tmp[g][idx] = sum of slabs [g*per_group, (g+1)*per_group), fp64
// (the first conv's weight gradient is a heavily cancelling sum: its input
// sits near log10(1e-9) while the BatchNorm-backward output sums to ~0).
__global__ void wgrad_reduce1(const float* __restrict__ partial, int nparts,
                              int per, int per_group, double* __restrict__ tmp) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= per) return;
  const int g = blockIdx.y;
  const int b0 = g * per_group;
  int b1 = b0 + per_group;
  if (b1 > nparts) b1 = nparts;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    a0 += partial[(int64_t)(b + 0) * per + idx];
    a1 += partial[(int64_t)(b + 1) * per + idx];
    a2 += partial[(int64_t)(b + 2) * per + idx];
    a3 += partial[(int64_t)(b + 3) * per + idx];
  }
  for (; b < b1; ++b) a0 += partial[(int64_t)b * per + idx];
  tmp[(int64_t)g * per + idx] = (a0 + a1) + (a2 + a3);
}

// Stage 2: sum the group partials; out dw[co][ci0+ci][tap], dbias[co].
__global__ void wgrad_reduce(const double* __restrict__ partial, int nparts,
                             int CTp, int J, int cin_pass, int ci0, int Cin,
                             int Cout, float* __restrict__ dw,
                             float* __restrict__ dbias, int write_bias) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int per = CTp * (J + 1);
  if (idx >= per) return;
  const int co = idx / (J + 1), j = idx % (J + 1);
  if (co >= Cout) return;
  double s = 0.0;
  for (int b = 0; b < nparts; ++b) s += partial[(int64_t)b * per + idx];
  if (j == J) {
    if (write_bias && dbias) dbias[co] = (float)s;
  } else {
    const int tap = j / cin_pass, ci = j % cin_pass;
    dw[((int64_t)co * Cin + ci0 + ci) * 9 + tap] = (float)s;
  }
}

constexpr int WG_BLOCKS = 512;
constexpr int WG_GROUPS = 16;  // stage-1 groups of WG_BLOCKS/WG_GROUPS slabs

static int wgrad_ct(int Cout) { return (Cout + 15) / 16; }
static int wgrad_pass(int Cin) { return Cin < WG_CIMAX ? Cin : WG_CIMAX; }


// ------------------------------------------------------------ small channels
// Convolutions whose one side has 1-2 channels (the encoder's first conv
// 1->16, the decoder's last 16->1 and its dgrad: models/CNNBLSTM/model.py:35,59)
// are HBM-bound: the 16-row MFMA tiles above would waste 15/16 of their work.
// fwd/dgrad: an 8x48 tile per block (the same tiling and stats-part
// numbering as conv3x3_fwd_mfma), 128 threads = 8 rows x 16 x 3 pixels, input
// tile + weights in LDS.  The tile is staged with every global load issued
// before the first LDS store (no per-element load->store latency chain).
// XL (round 5): x channel-last [N][H][W][CIN]; element e then walks the
// channels of a pixel fastest (contiguous loads) and lands in the same
// [c][row][col] LDS image.
template <int CIN, bool PRO, int NT, bool XL = false>
__device__ __forceinline__ void stage_small_tile(const float* __restrict__ x,
                                                 const float* __restrict__ in_scale,
                                                 const float* __restrict__ in_shift,
                                                 float* sx, int n, int f0, int t0, int H, int W) {
  constexpr int LR = CV_TT + 2, ROWS = CV_FT + 2, E = CIN * ROWS * LR;
  constexpr int PER = (E + NT - 1) / NT;
  // loads in flight per thread: the whole tile in one round trip up to 32
  constexpr int BATCH = PER <= 32 ? PER : 16;
  const int64_t HW = (int64_t)H * W;
  // a thread's channel is the same for all its elements when CIN = 1 or, channel-
  // last, when NT is a multiple of CIN: the prologue constants are then loaded
  // once (round 6: per-element loads of in_scale[c] / in_shift[c] cost the
  // 16 -> 1 forward 40 % of its time)
  constexpr bool CFIX = CIN == 1 || (XL && NT % CIN == 0);
  float fsc = 1.f, fsh = 0.f;
  if (PRO && CFIX) {
    const int c = CIN == 1 ? 0 : (int)(threadIdx.x % CIN);
    fsc = in_scale[c];
    fsh = in_shift[c];
  }
  auto decode = [&](int e, int& c, int& rr, int& cc) {
    if constexpr (XL) {
      c = e % CIN;
      rr = (e / CIN) / LR;
      cc = (e / CIN) % LR;
    } else {
      c = e / (ROWS * LR);
      rr = (e / LR) % ROWS;
      cc = e % LR;
    }
  };
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += BATCH) {
    float v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int e = threadIdx.x + NT * (b0 + i);
      int c, rr, cc;
      decode(e, c, rr, cc);
      const int f = f0 - 1 + rr, t = t0 - 1 + cc;
      const bool ok = b0 + i < PER && e < E && f >= 0 && f < H && t >= 0 && t < W;
      const int64_t off = XL ? ((int64_t)n * HW + (int64_t)f * W + t) * CIN + c
                             : ((int64_t)n * CIN + c) * HW + (int64_t)f * W + t;
      v[i] = ok ? x[off] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int e = threadIdx.x + NT * (b0 + i);
      if (b0 + i >= PER || e >= E) break;
      int c, rr, cc;
      decode(e, c, rr, cc);
      float a = v[i];
      if (PRO) {
        const int f = f0 - 1 + rr, t = t0 - 1 + cc;
        // BatchNorm+ReLU of the previous layer; zero padding stays zero
        if (f >= 0 && f < H && t >= 0 && t < W)
          a = fmaxf(fmaf(a, CFIX ? fsc : in_scale[c], CFIX ? fsh : in_shift[c]), 0.f);
      }
      sx[(c * ROWS + rr) * LR + cc] = a;
    }
  }
}

// PX pixels per thread: 3 (128 threads) when COUT is wide (per-thread outputs
// amortise the stats reduction), 1 (384 threads) when it is 1-2 (more waves
// in flight for the 16-channel staging).
template <int CIN, int COUT, bool DGRAD, bool PRO, int PX, bool XL = false, bool YL = false>
__global__ __launch_bounds__(384 / PX) void conv3x3_small_fwd(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, int H, int W, Bnr bnr) {
  constexpr int TR = CV_FT, TC = CV_TT, LR = TC + 2, NT = 384 / PX, TPR = TC / PX, NWV = NT / 64;
  __shared__ float sx[CIN * (TR + 2) * LR];
  __shared__ float sw[COUT][CIN][9];
  __shared__ double sred[2][NWV][COUT];
  // fused BatchNorm-backward reduce of a channel-last dx (Bnr): the (gz,
  // gz * xhat) terms replace (v, v^2); y is loaded before the tile is staged
  // and the constants sit in LDS
  constexpr bool FZ = DGRAD && YL && COUT % 4 == 0;
  __shared__ float sbn[FZ ? 4 * COUT : 1];
  const int n = blockIdx.z, f0 = blockIdx.y * TR, t0 = blockIdx.x * TC;
  const int tid = threadIdx.x;
  const int64_t HW = (int64_t)H * W;
  const bool fused = FZ && stats && bnr.y != nullptr;
  uint4 yr[FZ ? PX : 1][FZ ? COUT / 4 : 1];
  if constexpr (FZ) {
    if (fused) {
      bnr_stage(bnr, sbn, COUT, COUT, tid, NT);
      const int f = f0 + tid / TPR;
#pragma unroll
      for (int q = 0; q < PX; ++q) {
        const int t = t0 + tid % TPR + TPR * q;
        const bool ok = f < H && t < W;
#pragma unroll
        for (int c4 = 0; c4 < COUT / 4; ++c4)
          yr[q][c4] = bnr_ld4(bnr, ok ? ((int64_t)n * HW + (int64_t)f * W + t) * COUT + 4 * c4 : 0);
      }
    }
  }
  stage_small_tile<CIN, PRO, NT, XL>(x, in_scale, in_shift, sx, n, f0, t0, H, W);
  for (int i = tid; i < COUT * CIN * 9; i += blockDim.x) {
    const int co = i / (CIN * 9), ci = (i / 9) % CIN, tap = i % 9;
    sw[co][ci][tap] = DGRAD ? w[(ci * COUT + co) * 9 + 8 - tap] : w[(co * CIN + ci) * 9 + tap];
  }
  __syncthreads();
  const int r = tid / TPR, c0 = tid % TPR;       // pixels (r, c0 + TPR*q), q < PX
  const int f = f0 + r;
  float acc[PX][COUT];
#pragma unroll
  for (int q = 0; q < PX; ++q)
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[q][co] = bias ? bias[co] : 0.f;
  constexpr int CUNR = CIN <= 2 ? CIN : 2;   // bound the hoisted weights per iteration
#pragma unroll CUNR
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float* xr = sx + (ci * (TR + 2) + r + tap / 3) * LR + c0 + tap % 3;
      float v[PX];
#pragma unroll
      for (int q = 0; q < PX; ++q) v[q] = xr[TPR * q];
#pragma unroll
      for (int co = 0; co < COUT; ++co) {
        const float wv = sw[co][ci][tap];
#pragma unroll
        for (int q = 0; q < PX; ++q) acc[q][co] = fmaf(wv, v[q], acc[q][co]);
      }
    }
  bool ok[PX];
#pragma unroll
  for (int q = 0; q < PX; ++q) {
    const int t = t0 + c0 + TPR * q;
    ok[q] = f < H && t < W;
    if (ok[q]) {
      if constexpr (YL && COUT % 4 == 0) {   // channel-last: a pixel's COUT channels
        float4* yp = reinterpret_cast<float4*>(y + ((int64_t)n * HW + (int64_t)f * W + t) * COUT);
#pragma unroll
        for (int c4 = 0; c4 < COUT / 4; ++c4)
          yp[c4] = make_float4(acc[q][4 * c4], acc[q][4 * c4 + 1], acc[q][4 * c4 + 2],
                               acc[q][4 * c4 + 3]);
      } else {
#pragma unroll
        for (int co = 0; co < COUT; ++co)
          y[YL ? ((int64_t)n * HW + (int64_t)f * W + t) * COUT + co
               : ((int64_t)n * COUT + co) * HW + (int64_t)f * W + t] = acc[q][co];
      }
    }
  }
  if (stats) {
    const int wave = tid >> 6;
    float ts[FZ ? PX : 1][FZ ? COUT : 1], tq[FZ ? PX : 1][FZ ? COUT : 1];
    if constexpr (FZ) {
      if (fused) {
#pragma unroll
        for (int q = 0; q < PX; ++q)
#pragma unroll
          for (int c4 = 0; c4 < COUT / 4; ++c4) {
            const float v4[4] = {acc[q][4 * c4], acc[q][4 * c4 + 1], acc[q][4 * c4 + 2],
                                 acc[q][4 * c4 + 3]};
            float yv[4];
            bnr_dec4(bnr.y16, yr[q][c4], yv);
            bnr_terms4<COUT>(sbn, 4 * c4, yv, v4, ok[q], &ts[q][4 * c4], &tq[q][4 * c4]);
          }
      }
    }
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int q = 0; q < PX; ++q)
        if (FZ && fused) {
          a += ts[FZ ? q : 0][FZ ? co : 0];
          b += tq[FZ ? q : 0][FZ ? co : 0];
        } else if (ok[q]) {
          a += acc[q][co];
          b = fmaf(acc[q][co], acc[q][co], b);   // explicit: every instance rounds alike
        }
      a = wave_sum(a);
      b = wave_sum(b);
      if ((tid & 63) == 0) {
        sred[0][wave][co] = a;
        sred[1][wave][co] = b;
      }
    }
    __syncthreads();
    if (tid < COUT) {
      const int64_t part = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
      double a = 0.0, b = 0.0;
      for (int q = 0; q < NWV; ++q) {
        a += sred[0][q][tid];
        b += sred[1][q][tid];
      }
      stats[part * 2 * COUT + tid] = a;
      stats[part * 2 * COUT + COUT + tid] = b;
    }
  }
}

// wgrad: one thread per (co, ci, tap) output (+ COUT bias outputs) summing
// dy * act(x) over the block's 8x48 pixels from LDS; one slab per block,
// reduced by wgrad_reduce1 + small_wgrad_final in fixed order (fp64).
template <int CIN, int COUT, bool PRO>
__global__ __launch_bounds__(256) void conv3x3_small_wgrad(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int H, int W) {
  constexpr int TR = CV_FT, TC = CV_TT, LR = TC + 2, GP = TR * TC + 1;
  constexpr int NOUT = COUT * CIN * 9 + COUT;
  constexpr int GE = COUT * TR * TC, GPER = (GE + 255) / 256;
  __shared__ float sx[CIN * (TR + 2) * LR];
  __shared__ float sg[COUT * GP];
  const int n = blockIdx.z, f0 = blockIdx.y * TR, t0 = blockIdx.x * TC;
  const int tid = threadIdx.x;
  const int64_t HW = (int64_t)H * W;
  {
    float v[GPER];
#pragma unroll
    for (int i = 0; i < GPER; ++i) {
      const int e = tid + 256 * i;
      const int co = e / (TR * TC), p = e % (TR * TC);
      const int f = f0 + p / TC, t = t0 + p % TC;
      v[i] = (e < GE && f < H && t < W) ? dy[((int64_t)n * COUT + co) * HW + (int64_t)f * W + t] : 0.f;
    }
    stage_small_tile<CIN, PRO, 256>(x, in_scale, in_shift, sx, n, f0, t0, H, W);
#pragma unroll
    for (int i = 0; i < GPER; ++i) {
      const int e = tid + 256 * i;
      if (e < GE) sg[(e / (TR * TC)) * GP + e % (TR * TC)] = v[i];
    }
  }
  __syncthreads();
  const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (int o = tid; o < NOUT; o += blockDim.x) {
    float s = 0.f;
    if (o < COUT * CIN * 9) {
      const int co = o / (CIN * 9), ci = (o / 9) % CIN, tap = o % 9;
      const int ky = tap / 3, kx = tap % 3;
      const float* g = sg + co * GP;
      for (int r = 0; r < TR; ++r) {
        const float* xr = sx + (ci * (TR + 2) + r + ky) * LR + kx;
#pragma unroll 8
        for (int c = 0; c < TC; ++c) s = fmaf(g[r * TC + c], xr[c], s);
      }
    } else {
      const float* g = sg + (o - COUT * CIN * 9) * GP;
      for (int p = 0; p < TR * TC; ++p) s += g[p];
    }
    partial[blk * NOUT + o] = s;
  }
}

// wgrad of the 1-2-channel-sided convs as row strips (round 5): one wave per
// (input channel ca, output channel cg) pair walks a strip of SW_RS rows of
// one image; its 64 lanes cover columns t0-1 .. t0+62 and lanes 1..62 own the
// output columns t0 .. t0+61.  Each loaded row of act(x)[ca] is shifted by one
// lane both ways (the kx = 0 / 2 taps), the last three rows stay in registers
// (the ky taps), so every input element is read from HBM once per pair and
// every lane does 9 FMAs per pixel -- no LDS, no partially idle threads (the
// 8x48-tile kernel above keeps 145 of 256 threads busy and re-stages the
// halo per tile; in the C2 step its 16->1 instance ran 1.8 ms beside the
// layer-0 GEMM pair on the side stream).  Rows are loaded SW_RB at a time.
// Partial slabs: [tile][NOUT] with the old kernel's output order, reduced by
// the same fixed-order wgrad_reduce1 + small_wgrad_final.
constexpr int SW_RS = 32;          // rows per strip
constexpr int SW_TW = 62;          // output columns per wave
constexpr int SW_RB = 8;           // rows loaded per batch

template <int CA, int CG, bool PRO>
__global__ __launch_bounds__(256) void conv3x3_strip_wgrad(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int H, int W, int ntf, int ntt) {
  constexpr int NOUT = CG * CA * 9 + CG;
  const int lane = threadIdx.x & 63;
  const int pair = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (pair >= CA * CG) return;                 // whole waves only: no barrier below
  const int ca = pair % CA, cg = pair / CA;
  const int tile = blockIdx.x;                 // (n, strip, column block)
  const int tt = tile % ntt, fs = (tile / ntt) % ntf, n = tile / (ntt * ntf);
  const int f0 = fs * SW_RS, t = tt * SW_TW - 1 + lane;
  const bool tin = t >= 0 && t < W;
  const bool own = lane >= 1 && lane <= SW_TW && tin;
  const int64_t HW = (int64_t)H * W;
  const float* xa = x + ((int64_t)n * CA + ca) * HW + t;
  const float* gg = dy + ((int64_t)n * CG + cg) * HW + t;
  float sc = 1.f, sh = 0.f;
  if (PRO) {
    sc = in_scale[ca];
    sh = in_shift[ca];
  }
  float acc[9], accb = 0.f;
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = 0.f;
  // window rows f-1, f, f+1 of act(x): (left, centre, right) per lane
  float w0l = 0.f, w0c = 0.f, w0r = 0.f, w1l = 0.f, w1c = 0.f, w1r = 0.f;
  // row f0-1 and f0 prime the window
  {
    const int f = f0 - 1;
    float a = (f >= 0 && tin) ? xa[(int64_t)f * W] : 0.f;
    if (PRO && f >= 0 && tin) a = fmaxf(fmaf(a, sc, sh), 0.f);
    w1c = a;
    w1l = __shfl_up(a, 1, 64);
    w1r = __shfl_down(a, 1, 64);
  }
  {
    const int f = f0;
    float a = (f < H && tin) ? xa[(int64_t)f * W] : 0.f;
    if (PRO && f < H && tin) a = fmaxf(fmaf(a, sc, sh), 0.f);
    w0l = w1l; w0c = w1c; w0r = w1r;
    w1c = a;
    w1l = __shfl_up(a, 1, 64);
    w1r = __shfl_down(a, 1, 64);
  }
  const int rows = (H - f0) < SW_RS ? (H - f0) : SW_RS;
  for (int r0 = 0; r0 < rows; r0 += SW_RB) {
    float va[SW_RB], vg[SW_RB];
#pragma unroll
    for (int i = 0; i < SW_RB; ++i) {
      const int f = f0 + r0 + i;              // output row; a needs row f+1
      const bool rok = r0 + i < rows;
      va[i] = (rok && f + 1 < H && tin) ? xa[(int64_t)(f + 1) * W] : 0.f;
      vg[i] = (rok && own) ? gg[(int64_t)f * W] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < SW_RB; ++i) {
      const int f = f0 + r0 + i;
      float a = va[i];
      if (PRO && f + 1 < H && tin) a = fmaxf(fmaf(a, sc, sh), 0.f);
      const float al = __shfl_up(a, 1, 64), ar = __shfl_down(a, 1, 64);
      const float g = vg[i];
      // rows f-1 (w0), f (w1), f+1 (a)
      acc[0] = fmaf(g, w0l, acc[0]);
      acc[1] = fmaf(g, w0c, acc[1]);
      acc[2] = fmaf(g, w0r, acc[2]);
      acc[3] = fmaf(g, w1l, acc[3]);
      acc[4] = fmaf(g, w1c, acc[4]);
      acc[5] = fmaf(g, w1r, acc[5]);
      acc[6] = fmaf(g, al, acc[6]);
      acc[7] = fmaf(g, a, acc[7]);
      acc[8] = fmaf(g, ar, acc[8]);
      accb += g;
      w0l = w1l; w0c = w1c; w0r = w1r;
      w1l = al; w1c = a; w1r = ar;
    }
  }
  float* out = partial + (int64_t)tile * NOUT;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float s = wave_sum(acc[i]);
    if (lane == 0) out[(cg * CA + ca) * 9 + i] = s;
  }
  if (ca == 0) {
    const float s = wave_sum(accb);
    if (lane == 0) out[CG * CA * 9 + cg] = s;
  }
}

// The same row strips with the 16-channel side channel-last (round 5): a lane
// holds 4 consecutive channels (one 16-byte load) of one pixel, a wave 16
// pixels (columns t0-1 .. t0+14; lanes of pixels 1..14 own outputs) x 4
// channel quads; the column shifts are lane shifts by 4.  ACL: act(x) is the
// 16-channel side (16 -> 1 conv, dy one plane); else dy is (1 -> 16).
constexpr int SWC_TW = 14;         // output columns per wave

// Round 6, BNA (1 -> 16 only, !ACL): dy is not read but formed per element
// from the BatchNorm+ReLU backward of the 16-channel layer -- g (the gradient
// of its output) and y (its pre-BN input), both channel-last fp32 -- with
// bn_relu_bwd_apply_cl's constants and arithmetic, so the values are that
// pass's gy bit for bit and gy is never written: the encoder's first conv,
// whose input needs no gradient, is the only consumer of its gy.
struct BnApply {
  const float* g;       // [N][H][W][16]
  const float* y;       // [N][H][W][16]
  const float* scale;   // forward BatchNorm scale / shift (ReLU mask)
  const float* shift;
  const float* gamma;   // nullable
  const float* save;    // mean [16], rstd [16]
  const double* sums;   // [sum gz | sum gz*xhat] (16 each), [2C] = count if inv_count == 0
  float* dgamma;
  float* dbeta;
  double inv_count;
};

template <bool ACL, bool PRO, bool BNA = false>
__global__ __launch_bounds__(256) void conv3x3_strip_wgrad_cl(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int H, int W, int ntf, int ntt, int ntiles, BnApply bna = {}) {
  static_assert(!(BNA && ACL), "the fused BatchNorm apply forms the 16-channel dy");
  constexpr int NOUT = 16 * 9 + (ACL ? 1 : 16);
  const int lane = threadIdx.x & 63, q = lane & 3, pj = lane >> 2;
  if (BNA && blockIdx.x == 0 && threadIdx.x < 16) {   // as bn_relu_bwd_apply_cl
    if (bna.dbeta) bna.dbeta[threadIdx.x] = (float)bna.sums[threadIdx.x];
    if (bna.dgamma) bna.dgamma[threadIdx.x] = (float)bna.sums[16 + threadIdx.x];
  }
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);     // one tile per wave
  if (tile >= ntiles) return;                               // whole waves: no barrier below
  const int tt = tile % ntt, fs = (tile / ntt) % ntf, n = tile / (ntt * ntf);
  const int f0 = fs * SW_RS, t = tt * SWC_TW - 1 + pj;
  const bool tin = t >= 0 && t < W;
  const bool own = pj >= 1 && pj <= SWC_TW && tin;
  const int64_t HW = (int64_t)H * W;
  // the 16-channel side: element (pixel, 4q..4q+3); the 1-channel side: pixel
  const float* vsrc = (ACL ? x : (BNA ? bna.g : dy)) + ((int64_t)n * HW + t) * 16 + 4 * q;
  const float* ysrc = BNA ? bna.y + ((int64_t)n * HW + t) * 16 + 4 * q : nullptr;
  const float* ssrc = (ACL ? dy : x) + (int64_t)n * HW + t;
  // BNA: this lane's four channels' constants (scale, shift, mean, rstd,
  // k = gamma * rstd, m1, m2), computed as bn_relu_bwd_apply_cl stages them
  float bc[7][4];
  if constexpr (BNA) {
    const double ic = bna.inv_count > 0.0 ? bna.inv_count : 1.0 / bna.sums[32];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * q + e;
      bc[0][e] = bna.scale[c];
      bc[1][e] = bna.shift[c];
      bc[2][e] = bna.save[c];
      bc[3][e] = bna.save[16 + c];
      bc[4][e] = (bna.gamma ? bna.gamma[c] : 1.f) * bna.save[16 + c];
      bc[5][e] = (float)(bna.sums[c] * ic);
      bc[6][e] = (float)(bna.sums[16 + c] * ic);
    }
  }
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
  float ssc = 1.f, ssh = 0.f;
  if (PRO) {
    if (ACL) {
      sc = *reinterpret_cast<const float4*>(in_scale + 4 * q);
      sh = *reinterpret_cast<const float4*>(in_shift + 4 * q);
    } else {
      ssc = in_scale[0];
      ssh = in_shift[0];
    }
  }
  // act(x) of row f (zero outside the image): 4 channels (ACL) or 1 (x 4 lanes)
  auto load_a = [&](int f, float (&a)[4]) {
    const bool ok = f >= 0 && f < H && tin;
    if (ACL) {
      float4 v = ok ? *reinterpret_cast<const float4*>(vsrc + (int64_t)f * W * 16)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
      if (PRO && ok) {
        v.x = fmaxf(fmaf(v.x, sc.x, sh.x), 0.f);
        v.y = fmaxf(fmaf(v.y, sc.y, sh.y), 0.f);
        v.z = fmaxf(fmaf(v.z, sc.z, sh.z), 0.f);
        v.w = fmaxf(fmaf(v.w, sc.w, sh.w), 0.f);
      }
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
      float v = ok ? ssrc[(int64_t)f * W] : 0.f;
      if (PRO && ok) v = fmaxf(fmaf(v, ssc, ssh), 0.f);
      a[0] = a[1] = a[2] = a[3] = v;
    }
  };
  auto load_g = [&](int f, float (&g)[4]) {
    const bool ok = f < H && own;
    if (ACL) {
      const float v = ok ? ssrc[(int64_t)f * W] : 0.f;
      g[0] = g[1] = g[2] = g[3] = v;
    } else {
      const float4 v = ok ? *reinterpret_cast<const float4*>(vsrc + (int64_t)f * W * 16)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      g[0] = v.x; g[1] = v.y; g[2] = v.z; g[3] = v.w;
      if constexpr (BNA) {   // gy of the BatchNorm+ReLU backward (0 outside the image)
        const float4 u = ok ? *reinterpret_cast<const float4*>(ysrc + (int64_t)f * W * 16)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        const float yv[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gz = fmaf(yv[e], bc[0][e], bc[1][e]) > 0.f ? g[e] : 0.f;
          const float o = bc[4][e] * (gz - bc[5][e] - ((yv[e] - bc[2][e]) * bc[3][e]) * bc[6][e]);
          g[e] = ok ? o : 0.f;
        }
      }
    }
  };
  float acc[9][4], accb[4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[i][e] = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) accb[e] = 0.f;
  // window rows f-1 (w0) and f (w1): (left, centre, right) per channel
  float w0l[4], w0c[4], w0r[4], w1l[4], w1c[4], w1r[4];
  auto shift = [&](const float (&a)[4], float (&l)[4], float (&r)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      l[e] = __shfl_up(a[e], 4, 64);
      r[e] = __shfl_down(a[e], 4, 64);
    }
  };
  load_a(f0 - 1, w0c);
  shift(w0c, w0l, w0r);
  load_a(f0, w1c);
  shift(w1c, w1l, w1r);
  const int rows = (H - f0) < SW_RS ? (H - f0) : SW_RS;
  for (int r0 = 0; r0 < rows; r0 += 4) {
    float va[4][4], vg[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + r0 + i;
      const bool rok = r0 + i < rows;
      load_a(rok ? f + 1 : H, va[i]);
      load_g(rok ? f : H, vg[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float al[4], ar[4];
      shift(va[i], al, ar);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = vg[i][e];
        acc[0][e] = fmaf(g, w0l[e], acc[0][e]);
        acc[1][e] = fmaf(g, w0c[e], acc[1][e]);
        acc[2][e] = fmaf(g, w0r[e], acc[2][e]);
        acc[3][e] = fmaf(g, w1l[e], acc[3][e]);
        acc[4][e] = fmaf(g, w1c[e], acc[4][e]);
        acc[5][e] = fmaf(g, w1r[e], acc[5][e]);
        acc[6][e] = fmaf(g, al[e], acc[6][e]);
        acc[7][e] = fmaf(g, va[i][e], acc[7][e]);
        acc[8][e] = fmaf(g, ar[e], acc[8][e]);
        accb[e] += g;
        w0l[e] = w1l[e]; w0c[e] = w1c[e]; w0r[e] = w1r[e];
        w1l[e] = al[e]; w1c[e] = va[i][e]; w1r[e] = ar[e];
      }
    }
  }
  // sum the 16 pixels of each channel quad (lanes == q mod 4), fixed order
  auto qsum = [&](float v) {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  float* out = partial + (int64_t)tile * NOUT;
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float s = qsum(acc[i][e]);
      // (16 -> 1): o = ci*9 + tap; (1 -> 16): o = co*9 + tap -- channel 4q + e
      if (pj == 0) out[(4 * q + e) * 9 + i] = s;
    }
  if (ACL) {
    const float s = qsum(accb[0]);
    if (lane == 0) out[144] = s;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float s = qsum(accb[e]);
      if (pj == 0) out[144 + 4 * q + e] = s;
    }
  }
}

// Round 6: the 16 -> 1 forward (decoder.6, models/CNNBLSTM/model.py:59-60)
// on row strips, its 16-channel input channel-last.  conv3x3_small_fwd stages
// a 16 x 10 x 50 halo per 8 x 48 tile (32 KB of LDS: four workgroups per CU)
// and reads it back 144 times per pixel: 106 us at the C2 shape (1.7 TB/s of
// its 176 MB input).  Here a wave walks a strip of R1_RS rows x R1_TW output
// columns.  Lane 4p + q holds pixel column t0 - 1 + p (p < 16; p = 1 .. 14
// own outputs) and channels 4q .. 4q+3: one 16-byte load per row (a wave: 1
// KB contiguous; rows prefetched three ahead), its 36 weights in VGPRs.  Per
// input row it forms the nine tap partials u[ky][dx] = sum over its four
// channels of w[c][ky][dx] act(x)[c] and adds them to the three output rows
// the row feeds; a finished output row is summed over the four channel
// quads (two DPP steps) and over its three columns (two one-pixel lane
// shifts).  Every input element comes from HBM once per strip (halo: 16/14
// columns, (R1_RS+2)/R1_RS rows).  BatchNorm partials: one [sum y, sum y^2]
// row per workgroup of four strips (fp32 per lane and wave, fp64 across
// waves).  Another summation order than conv3x3_small_fwd (within 1e-6).
constexpr int R1_TW = 14;   // output columns per wave
constexpr int R1_RS = 16;   // rows per strip

template <bool PRO>
__global__ __launch_bounds__(256) void conv3x3_rows_16to1(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, int H, int W, int nfs, int nts,
    int nstrips) {
  __shared__ double red[4][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, p = lane >> 2, q = lane & 3;
  const int strip = blockIdx.x * 4 + wave;
  float s1 = 0.f, s2 = 0.f;
  if (strip < nstrips) {
    const int ts = strip % nts, fs = (strip / nts) % nfs, n = strip / (nts * nfs);
    const int f0 = fs * R1_RS, t = ts * R1_TW - 1 + p;
    const bool tin = t >= 0 && t < W;
    const bool own = p >= 1 && p <= R1_TW && tin;
    const int64_t HW = (int64_t)H * W;
    const float4* src =
        reinterpret_cast<const float4*>(x + ((int64_t)n * HW + (tin ? t : 0)) * 16 + 4 * q);
    const int rows = (H - f0) < R1_RS ? (H - f0) : R1_RS;
    const float bv = bias ? bias[0] : 0.f;
    float wr[4][9];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k) wr[c][k] = w[(4 * q + c) * 9 + k];
    float4 sc4 = make_float4(1.f, 1.f, 1.f, 1.f), sh4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (PRO) {
      sc4 = *reinterpret_cast<const float4*>(in_scale + 4 * q);
      sh4 = *reinterpret_cast<const float4*>(in_shift + 4 * q);
    }
    auto load = [&](int r) -> float4 {
      return (r >= 0 && r < H && tin) ? src[(int64_t)r * W * 4] : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    float A[3][3];   // output rows r-1, r, r+1 of input row r: per dx, unshifted
#pragma unroll
    for (int k = 0; k < 3; ++k) A[0][k] = A[1][k] = A[2][k] = 0.f;
    const int nrow = rows + 2;
    float4 b0 = load(f0 - 1), b1 = load(f0), b2 = load(f0 + 1);   // three rows in flight
    auto step = [&](int i, float4& buf) {
      const int r = f0 - 1 + i;
      float a[4] = {buf.x, buf.y, buf.z, buf.w};
      if (i + 3 < nrow) buf = load(r + 3);
      if (PRO && r >= 0 && r < H && tin) {   // zero padding stays zero
        a[0] = fmaxf(fmaf(a[0], sc4.x, sh4.x), 0.f);
        a[1] = fmaxf(fmaf(a[1], sc4.y, sh4.y), 0.f);
        a[2] = fmaxf(fmaf(a[2], sc4.z, sh4.z), 0.f);
        a[3] = fmaxf(fmaf(a[3], sc4.w, sh4.w), 0.f);
      }
      float u[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float v = wr[0][k] * a[0];
        v = fmaf(wr[1][k], a[1], v);
        v = fmaf(wr[2][k], a[2], v);
        u[k] = fmaf(wr[3][k], a[3], v);
      }
      // ky = 0 feeds output row r+1, ky = 1 row r, ky = 2 row r-1
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        A[2][dx] += u[dx];
        A[1][dx] += u[3 + dx];
        A[0][dx] += u[6 + dx];
      }
      if (i >= 2) {   // output row r-1 (>= f0) is complete
        float v3[3];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {   // sum over the quad's channel groups
          float v = A[0][dx];
          v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
          v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
          v3[dx] = v;
        }
        const float l = __shfl_up(v3[0], 4, 64), rr = __shfl_down(v3[2], 4, 64);
        const float v = bv + ((l + v3[1]) + rr);
        if (own && q == 0) {
          y[(int64_t)n * HW + (int64_t)(r - 1) * W + t] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        A[0][dx] = A[1][dx];
        A[1][dx] = A[2][dx];
        A[2][dx] = 0.f;
      }
    };
    for (int i = 0; i < nrow; i += 3) {
      step(i, b0);
      if (i + 1 < nrow) step(i + 1, b1);
      if (i + 2 < nrow) step(i + 2, b2);
    }
  }
  if (!stats) return;   // uniform: no barrier without statistics
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    red[wave][0] = s1;
    red[wave][1] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += red[k][threadIdx.x];
    stats[(int64_t)blockIdx.x * 2 + threadIdx.x] = v;
  }
}

// Round 6: the 1 -> 16 convs on row strips, their 16-channel side channel-
// last: the encoder's first forward (encoder.0, models/CNNBLSTM/model.py:35-36)
// with its BatchNorm partials, and the decoder's last data gradient (dy of one
// channel -> dx of 16, decoder.6, model.py:59-60) with the fused BatchNorm-
// backward reduce of the layer it feeds (Bnr).  conv3x3_small_fwd took 86 /
// 126 us for them at the C2 shape.  Lane 4p + q of a wave: pixel column
// t0 - 1 + p (p < 16; p = 1 .. 14 own outputs) and channels 4q .. 4q+3, whose
// 36 weights, biases and BatchNorm constants sit in its VGPRs; each output
// pixel row is one float4 per lane (a wave: 1 KB contiguous).  The one-channel
// input row is read by the four lanes of a pixel and shifted by one pixel
// (four lanes) for the outer taps: a rolling 3 x 3 window, rows prefetched two
// ahead.  Per output the fma chain of conv3x3_small_fwd (bias, then the nine
// taps in order; data gradient: flipped taps, no bias), so y / dx are bit-
// identical to it.  BatchNorm partials: one row per workgroup of four strips,
// [sum | sum of squares] (forward) or [sum gz | sum gz * xhat] (Bnr) x 16
// channels, lanes in fp32, workgroup in fp64 (<= exact_stat_parts rows).
constexpr int R16_TW = 14;   // output columns per wave
constexpr int R16_RS = 16;   // rows per strip

// OUT (data gradient of Conv2d(16, 1) feeding a BatchNorm+ReLU, decoder.5 ->
// decoder.6): 0 = store dx; 1 = store nothing (the fused reduce's partials
// only: the apply pass recomputes dx); 2 / 3 = the BatchNorm+ReLU backward
// apply of the recomputed dx (bna: constants as bn_relu_bwd_apply_cl forms
// them, y = bnr.y fp32) stored as gy in fp32 / bf16 -- dx is never written.
template <bool DG, bool PRO, bool FZ, int OUT = 0>
__global__ __launch_bounds__(256) void conv3x3_rows_1to16(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, Bnr bnr, int H, int W, int nfs, int nts,
    int nstrips, BnApply bna = {}) {
  static_assert(OUT < 2 || (DG && !FZ), "the apply mode is a data gradient without partials");
  constexpr bool LY = FZ || OUT >= 2;   // y of each output pixel loaded (prefetched a row ahead)
  __shared__ double red[4][32];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, p = lane >> 2, q = lane & 3;
  if (OUT >= 2 && blockIdx.x == 0 && threadIdx.x < 16) {   // as bn_relu_bwd_apply_cl
    if (bna.dbeta) bna.dbeta[threadIdx.x] = (float)bna.sums[threadIdx.x];
    if (bna.dgamma) bna.dgamma[threadIdx.x] = (float)bna.sums[16 + threadIdx.x];
  }
  const int strip = blockIdx.x * 4 + wave;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (strip < nstrips) {
    const int ts = strip % nts, fs = (strip / nts) % nfs, n = strip / (nts * nfs);
    const int f0 = fs * R16_RS, t = ts * R16_TW - 1 + p;
    const bool tin = t >= 0 && t < W;
    const bool own = p >= 1 && p <= R16_TW && tin;
    const int64_t HW = (int64_t)H * W;
    const float* xs = x + (int64_t)n * HW + (tin ? t : 0);
    float wr[4][9], bq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int k = 0; k < 9; ++k) wr[c][k] = w[(4 * q + c) * 9 + (DG ? 8 - k : k)];
      bq[c] = (!DG && bias) ? bias[4 * q + c] : 0.f;
    }
    const float sc0 = PRO ? in_scale[0] : 1.f, sh0 = PRO ? in_shift[0] : 0.f;
    float bsc[4], bsh[4], bmu[4], brs[4], bk[4], bm1[4], bm2[4];
    if constexpr (FZ) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bsc[c] = bnr.sc[4 * q + c];
        bsh[c] = bnr.sh[4 * q + c];
        bmu[c] = bnr.save[4 * q + c];
        brs[c] = bnr.save[16 + 4 * q + c];
      }
    }
    if constexpr (OUT >= 2) {   // bn_relu_bwd_apply_cl's staging, per lane
      const double ic = bna.inv_count > 0.0 ? bna.inv_count : 1.0 / bna.sums[32];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int ch = 4 * q + c;
        bsc[c] = bna.scale[ch];
        bsh[c] = bna.shift[ch];
        bmu[c] = bna.save[ch];
        brs[c] = bna.save[16 + ch];
        bk[c] = (bna.gamma ? bna.gamma[ch] : 1.f) * bna.save[16 + ch];
        bm1[c] = (float)(bna.sums[ch] * ic);
        bm2[c] = (float)(bna.sums[16 + ch] * ic);
      }
    }
    const int rows = (H - f0) < R16_RS ? (H - f0) : R16_RS;
    auto ldx = [&](int r) -> float { return (r >= 0 && r < H && tin) ? xs[(int64_t)r * W] : 0.f; };
    auto act = [&](int r, float v) -> float {   // zero padding stays zero
      return (PRO && r >= 0 && r < H && tin) ? fmaxf(fmaf(v, sc0, sh0), 0.f) : v;
    };
    auto ldy = [&](int f) -> uint4 {   // Bnr: y of output row f, channels 4q .. 4q+3
      const int64_t e = ((((int64_t)n * H + (f < H ? f : H - 1)) * W) + (tin ? t : 0)) * 16 + 4 * q;
      return bnr_ld4(bnr, e);
    };
    // window rows f-1, f, f+1 (left, centre, right)
    float wl[3], wc[3], wrr[3];
    wc[0] = act(f0 - 1, ldx(f0 - 1));
    wc[1] = act(f0, ldx(f0));
    wl[0] = __shfl_up(wc[0], 4, 64); wrr[0] = __shfl_down(wc[0], 4, 64);
    wl[1] = __shfl_up(wc[1], 4, 64); wrr[1] = __shfl_down(wc[1], 4, 64);
    float nx0 = ldx(f0 + 1), nx1 = ldx(f0 + 2);   // raw rows f+1, f+2 in flight
    uint4 ny = make_uint4(0u, 0u, 0u, 0u);
    if (LY) ny = ldy(f0);
    for (int i = 0; i < rows; ++i) {
      const int f = f0 + i;
      const float cv = act(f + 1, nx0);
      nx0 = nx1;
      nx1 = ldx(f + 3);
      uint4 yc = ny;
      if (LY && i + 1 < rows) ny = ldy(f + 1);
      wc[2] = cv;
      wl[2] = __shfl_up(cv, 4, 64);
      wrr[2] = __shfl_down(cv, 4, 64);
      float o[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float acc = bq[c];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          acc = fmaf(wr[c][3 * ky], wl[ky], acc);
          acc = fmaf(wr[c][3 * ky + 1], wc[ky], acc);
          acc = fmaf(wr[c][3 * ky + 2], wrr[ky], acc);
        }
        o[c] = acc;
      }
      if (own) {
        float* yo = y + ((((int64_t)n * H + f) * W) + t) * 16 + 4 * q;
        if constexpr (OUT == 0) {
          *reinterpret_cast<float4*>(yo) = make_float4(o[0], o[1], o[2], o[3]);
        } else if constexpr (OUT >= 2) {
          float yv[4], gy[4];
          bnr_dec4(0, yc, yv);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float gz = fmaf(yv[c], bsc[c], bsh[c]) > 0.f ? o[c] : 0.f;
            gy[c] = bk[c] * (gz - bm1[c] - ((yv[c] - bmu[c]) * brs[c]) * bm2[c]);
          }
          if constexpr (OUT == 3) {
            uint16_t* yb = reinterpret_cast<uint16_t*>(y) + ((((int64_t)n * H + f) * W) + t) * 16 + 4 * q;
            *reinterpret_cast<uint2*>(yb) = make_uint2(cvt_pk_bf16(gy[0], gy[1]), cvt_pk_bf16(gy[2], gy[3]));
          } else {
            *reinterpret_cast<float4*>(yo) = make_float4(gy[0], gy[1], gy[2], gy[3]);
          }
        }
        if constexpr (FZ) {
          float yv[4];
          bnr_dec4(bnr.y16, yc, yv);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float gz = fmaf(yv[c], bsc[c], bsh[c]) > 0.f ? o[c] : 0.f;
            s1[c] += gz;
            s2[c] += gz * ((yv[c] - bmu[c]) * brs[c]);
          }
        } else if constexpr (OUT < 2) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            s1[c] += o[c];
            s2[c] = fmaf(o[c], o[c], s2[c]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        wl[k] = wl[k + 1];
        wc[k] = wc[k + 1];
        wrr[k] = wrr[k + 1];
      }
    }
  }
  if (!stats) return;   // uniform: no barrier without statistics
  // the 16 pixel lanes of each channel quad, fixed butterfly order
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {
      s1[c] += __shfl_xor(s1[c], o, 64);
      s2[c] += __shfl_xor(s2[c], o, 64);
    }
  if (p == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      red[wave][4 * q + c] = s1[c];
      red[wave][16 + 4 * q + c] = s2[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += red[k][threadIdx.x];
    stats[(int64_t)blockIdx.x * 32 + threadIdx.x] = v;
  }
}

// AINP_SMALL_ROWS=0: the 8 x 48 LDS tile kernel for the 16 -> 1 forward (A/B)
static bool small_rows_env() {
  static const bool v = [] {
    const char* e = getenv("AINP_SMALL_ROWS");
    return !(e && e[0] == '0');
  }();
  return v;
}

static int64_t rows16to1_strips(int64_t N, int64_t H, int64_t W) {
  return N * cdiv(H, R1_RS) * cdiv(W, R1_TW);
}

// dw[o] (o < COUT*CIN*9, [co][ci][tap] order) and dbias from the group sums
// first-stage groups of the small weight gradients' slab sum: their slabs are
// only 145-160 floats wide, so WG_GROUPS (16) groups left one thread per
// output summing 430 rows one after another (47 us at the C2 shape, on the
// critical path at the end of the backward); 128 groups of ~54 rows
constexpr int SWG_GROUPS = 128, SWG_GROUPS_MAX = 128;

__global__ __launch_bounds__(SWG_GROUPS_MAX) void small_wgrad_final(
    const double* __restrict__ tmp, int ngroups, int nw, int nout, float* __restrict__ dw,
    float* __restrict__ dbias) {
  // one workgroup per output o: group g's partial in thread g, then a fixed
  // pairwise tree in LDS (round 6: a serial loop over the 128 groups took 32 us)
  __shared__ double red[SWG_GROUPS_MAX];
  const int o = blockIdx.x, g = threadIdx.x;
  red[g] = g < ngroups ? tmp[(int64_t)g * nout + o] : 0.0;
  __syncthreads();
  for (int h = SWG_GROUPS_MAX / 2; h > 0; h >>= 1) {
    if (g < h) red[g] += red[g + h];
    __syncthreads();
  }
  if (g == 0) {
    const double v = red[0];
    if (o < nw) dw[o] = (float)v;
    else if (dbias) dbias[o - nw] = (float)v;
  }
}

// (Cin, Cout) pairs with a dedicated small-channel kernel
static bool small_pair(int a, int b) {
  return ((a == 1 || a == 2) && b == 16) || ((b == 1 || b == 2) && a == 16);
}

template <int CIN, int COUT, bool XL, bool YL>
static void launch_small_fwd_l(bool dgrad, const float* x, const float* w, const float* bias,
                               const float* sc, const float* sh, float* y, double* stats,
                               int64_t N, int64_t H, int64_t W, hipStream_t s, const Bnr& bnr) {
  dim3 grid((unsigned)cdiv(W, CV_TT), (unsigned)cdiv(H, CV_FT), (unsigned)N);
  constexpr int PX = COUT >= 16 ? 3 : 1;
  const dim3 block(384 / PX);
  if (dgrad)
    hipLaunchKernelGGL((conv3x3_small_fwd<CIN, COUT, true, false, PX, XL, YL>), grid, block, 0, s,
                       x, w, bias, sc, sh, y, stats, (int)H, (int)W, bnr);
  else if (sc)
    hipLaunchKernelGGL((conv3x3_small_fwd<CIN, COUT, false, true, PX, XL, YL>), grid, block, 0, s,
                       x, w, bias, sc, sh, y, stats, (int)H, (int)W, Bnr{});
  else
    hipLaunchKernelGGL((conv3x3_small_fwd<CIN, COUT, false, false, PX, XL, YL>), grid, block, 0,
                       s, x, w, bias, sc, sh, y, stats, (int)H, (int)W, Bnr{});
}

// lay (round 5): bit 0 = input channel-last (a 16-channel input), bit 1 =
// output channel-last (a 16-channel output); 1-2-channel tensors are the
// same in both layouts
template <int CIN, int COUT>
static void launch_small_fwd(bool dgrad, const float* x, const float* w, const float* bias,
                             const float* sc, const float* sh, float* y, double* stats,
                             int64_t N, int64_t H, int64_t W, hipStream_t s, int lay,
                             const Bnr& bnr) {
  const bool xl = (lay & 1) && CIN >= 16, yl = (lay & 2) && COUT >= 16;
  if (xl) launch_small_fwd_l<CIN, COUT, true, false>(dgrad, x, w, bias, sc, sh, y, stats, N, H, W, s, bnr);
  else if (yl) launch_small_fwd_l<CIN, COUT, false, true>(dgrad, x, w, bias, sc, sh, y, stats, N, H, W, s, bnr);
  else launch_small_fwd_l<CIN, COUT, false, false>(dgrad, x, w, bias, sc, sh, y, stats, N, H, W, s, bnr);
}

// *used: the BatchNorm partial rows written (<= exact_stat_parts)
static int small_fwd_dispatch(bool dgrad, const float* x, const float* w, const float* bias,
                              const float* sc, const float* sh, float* y, double* stats,
                              int64_t N, int Cin, int Cout, int64_t H, int64_t W, hipStream_t s,
                              int lay = 0, const Bnr& bnr = Bnr{}, int64_t* used = nullptr) {
  if (used) *used = N * cdiv(H, CV_FT) * cdiv(W, CV_TT);   // exact_stat_parts
  // (the BatchNorm partial rows of a row-strip launch stay within
  // exact_stat_parts; otherwise the tile kernel runs)
  if (!dgrad && Cin == 16 && Cout == 1 && (lay & 1) && small_rows_env() &&
      N * H * W * 16 < ((int64_t)1 << 40) && rows16to1_strips(N, H, W) < ((int64_t)1 << 31) &&
      cdiv(rows16to1_strips(N, H, W), 4) <= N * cdiv(H, CV_FT) * cdiv(W, CV_TT)) {
    const int nfs = (int)cdiv(H, R1_RS), nts = (int)cdiv(W, R1_TW);
    const int64_t ns = rows16to1_strips(N, H, W), nb = cdiv(ns, 4);
    if (used) *used = nb;
    const dim3 grid((unsigned)nb);
    if (sc)
      hipLaunchKernelGGL(conv3x3_rows_16to1<true>, grid, dim3(256), 0, s, x, w, bias, sc, sh, y,
                         stats, (int)H, (int)W, nfs, nts, (int)ns);
    else
      hipLaunchKernelGGL(conv3x3_rows_16to1<false>, grid, dim3(256), 0, s, x, w, bias, sc, sh, y,
                         stats, (int)H, (int)W, nfs, nts, (int)ns);
    return check_launch("conv3x3_rows_16to1");
  }
  if (Cin == 1 && Cout == 16 && (lay & 2) && small_rows_env() &&
      N * H * W * 16 < ((int64_t)1 << 40) && (dgrad || !bnr.y)) {
    const int nfs = (int)cdiv(H, R16_RS), nts = (int)cdiv(W, R16_TW);
    const int64_t ns = N * nfs * nts, nb = cdiv(ns, 4);
    if (nb <= N * cdiv(H, CV_FT) * cdiv(W, CV_TT) && ns < ((int64_t)1 << 31)) {
      if (used) *used = nb;
      const bool fz = dgrad && bnr.y && stats;
#define AINP_R16(DGV, PROV, FZV, ...)                                                              \
  hipLaunchKernelGGL((conv3x3_rows_1to16<DGV, PROV, FZV, ##__VA_ARGS__>), dim3((unsigned)nb),      \
                     dim3(256), 0, s, x, w, bias, sc, sh, y, stats, bnr, (int)H, (int)W, nfs, nts, \
                     (int)ns)
      if (dgrad && fz && !y) AINP_R16(true, false, true, 1);   // partials only (dx recomputed)
      else if (dgrad && fz) AINP_R16(true, false, true);
      else if (dgrad) AINP_R16(true, false, false);
      else if (sc) AINP_R16(false, true, false);
      else AINP_R16(false, false, false);
#undef AINP_R16
      return check_launch("conv3x3_rows_1to16");
    }
  }
  if (!y) return record_msg("conv3x3: a partials-only data gradient needs the row-strip kernel");
#define AINP_SF(A, B) \
  if (Cin == A && Cout == B) { launch_small_fwd<A, B>(dgrad, x, w, bias, sc, sh, y, stats, N, H, W, s, lay, bnr); return check_launch("conv3x3_small_fwd"); }
  AINP_SF(1, 16) AINP_SF(2, 16) AINP_SF(16, 1) AINP_SF(16, 2)
#undef AINP_SF
  return record_msg("conv3x3: no small-channel kernel for this pair");
}

// AINP_SMALL_WGRAD_TILE=1: the 8x48-tile kernel for every small pair (A/B)
static bool small_wgrad_tile_env() {
  const char* e = getenv("AINP_SMALL_WGRAD_TILE");
  return e && e[0] == '1';
}


static int64_t strip_tiles(int64_t N, int64_t H, int64_t W) {
  return N * cdiv(H, SW_RS) * cdiv(W, SW_TW);
}

static size_t small_wgrad_ws(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  int64_t nblk = N * cdiv(H, CV_FT) * cdiv(W, CV_TT);
  const int64_t ns = strip_tiles(N, H, W), nc = N * cdiv(H, SW_RS) * cdiv(W, SWC_TW);
  if (ns > nblk) nblk = ns;
  if (nc > nblk) nblk = nc;
  const int nout = Cout * Cin * 9 + Cout;
  return (size_t)nblk * nout * sizeof(float) + (size_t)SWG_GROUPS * nout * sizeof(double) + 16;
}

static int64_t strip_cl_tiles(int64_t N, int64_t H, int64_t W) {
  return N * cdiv(H, SW_RS) * cdiv(W, SWC_TW);
}

// lay (round 5): bit 0 = x channel-last (its 16 channels: the 16 -> 1 conv),
// bit 2 = dy channel-last (the 1 -> 16 conv); 1-channel tensors are the same
// in both layouts
static int small_wgrad(const float* x, const float* sc, const float* sh, const float* dy,
                       float* dw, float* dbias, void* workspace, int64_t N, int Cin, int Cout,
                       int64_t H, int64_t W, hipStream_t s, int lay = 0,
                       const BnApply* bna = nullptr) {
  const int nout = Cout * Cin * 9 + Cout;
  float* partial = reinterpret_cast<float*>(workspace);
  int64_t nblk;
  const bool acl = (lay & 1) && Cin == 16, gcl = (lay & 4) && Cout == 16;
  if (bna && !(gcl && Cin == 1)) return record_msg("conv3x3_wgrad: fused BatchNorm apply: 1 -> 16 only");
  if ((acl && Cout == 1) || (gcl && Cin == 1)) {
    const int ntf = (int)cdiv(H, SW_RS), ntt = (int)cdiv(W, SWC_TW);
    nblk = strip_cl_tiles(N, H, W);
    const dim3 grid((unsigned)cdiv(nblk, 4));
    if (bna && sc)
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<false, true, true>), grid, dim3(256), 0, s, x, sc,
                         sh, dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk, *bna);
    else if (bna)
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<false, false, true>), grid, dim3(256), 0, s, x, sc,
                         sh, dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk, *bna);
    else if (acl && sc)
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<true, true>), grid, dim3(256), 0, s, x, sc, sh,
                         dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk);
    else if (acl)
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<true, false>), grid, dim3(256), 0, s, x, sc, sh,
                         dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk);
    else if (sc)
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<false, true>), grid, dim3(256), 0, s, x, sc, sh,
                         dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk);
    else
      hipLaunchKernelGGL((conv3x3_strip_wgrad_cl<false, false>), grid, dim3(256), 0, s, x, sc, sh,
                         dy, partial, (int)H, (int)W, ntf, ntt, (int)nblk);
  } else if (acl || gcl) {
    return record_msg("conv3x3_wgrad: no channel-last small-channel kernel for this pair");
  } else if (!small_wgrad_tile_env() && H * W < ((int64_t)1 << 31)) {
    const int ntf = (int)cdiv(H, SW_RS), ntt = (int)cdiv(W, SW_TW);
    nblk = strip_tiles(N, H, W);
    const dim3 grid((unsigned)nblk, (unsigned)cdiv(Cin * Cout, 4));
#define AINP_SW(A, B) \
  else if (Cin == A && Cout == B && sc) hipLaunchKernelGGL((conv3x3_strip_wgrad<A, B, true>), grid, dim3(256), 0, s, x, sc, sh, dy, partial, (int)H, (int)W, ntf, ntt); \
  else if (Cin == A && Cout == B) hipLaunchKernelGGL((conv3x3_strip_wgrad<A, B, false>), grid, dim3(256), 0, s, x, sc, sh, dy, partial, (int)H, (int)W, ntf, ntt);
    if (false) {}
    AINP_SW(1, 16) AINP_SW(2, 16) AINP_SW(16, 1) AINP_SW(16, 2)
    else return record_msg("conv3x3_wgrad: no small-channel kernel for this pair");
#undef AINP_SW
  } else {
    dim3 grid((unsigned)cdiv(W, CV_TT), (unsigned)cdiv(H, CV_FT), (unsigned)N);
    nblk = (int64_t)grid.x * grid.y * grid.z;
#define AINP_SW(A, B) \
  else if (Cin == A && Cout == B && sc) hipLaunchKernelGGL((conv3x3_small_wgrad<A, B, true>), grid, dim3(256), 0, s, x, sc, sh, dy, partial, (int)H, (int)W); \
  else if (Cin == A && Cout == B) hipLaunchKernelGGL((conv3x3_small_wgrad<A, B, false>), grid, dim3(256), 0, s, x, sc, sh, dy, partial, (int)H, (int)W);
    if (false) {}
    AINP_SW(1, 16) AINP_SW(2, 16) AINP_SW(16, 1) AINP_SW(16, 2)
    else return record_msg("conv3x3_wgrad: no small-channel kernel for this pair");
#undef AINP_SW
  }
  int rc = check_launch("conv3x3_small_wgrad");
  if (rc) return rc;
  uintptr_t tp = reinterpret_cast<uintptr_t>(partial + nblk * nout);
  tp = (tp + 15) & ~(uintptr_t)15;
  double* tmp = reinterpret_cast<double*>(tp);
  const int per_group = (int)cdiv(nblk, SWG_GROUPS);
  hipLaunchKernelGGL(wgrad_reduce1, dim3((nout + 255) / 256, SWG_GROUPS), dim3(256), 0, s, partial,
                     (int)nblk, nout, per_group, tmp);
  rc = check_launch("wgrad_reduce1");
  if (rc) return rc;
  hipLaunchKernelGGL(small_wgrad_final, dim3(nout), dim3(SWG_GROUPS_MAX), 0, s, tmp, SWG_GROUPS,
                     Cout * Cin * 9, nout, dw, dbias);
  return check_launch("small_wgrad_final");
}

template <int CT, int JT>
static void launch_wgrad(const float* x, const float* sc, const float* sh,
                         const float* dy, float* partial, int N, int Cin,
                         int Cout, int H, int W, int ci0, int cp,
                         hipStream_t s) {
  hipLaunchKernelGGL((conv3x3_wgrad_mfma<CT, JT>), dim3(WG_BLOCKS), dim3(256),
                     0, s, x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp);
}

}  // namespace ainp

using namespace ainp;

namespace ainp {
int64_t conv_x6_stat_parts(int64_t N, int64_t H, int64_t W);
int64_t conv_x6_stat_rows(bool dgrad, int Cin, int Cout, int64_t N, int64_t H, int64_t W,
                          bool b16);
bool conv_x6_dgrad16_ok(int Cin, int Cout, int64_t H, int64_t W);
bool conv_x6_fwd16_ok(int Cin, int Cout, int64_t H, int64_t W);
bool conv_x6_dgrad_cfnt_ok(int Cin, int Cout, int64_t N, int64_t H, int64_t W);
int conv_wgrad_x6_launch(const float* x, const float* sc, const float* sh, const float* dy,
                         float* partial, int64_t N, int Cin, int Cout, int64_t H, int64_t W,
                         int ci0, int cp, int grid, hipStream_t s, bool b16, bool g16, bool x16,
                         int lay, int* grid_used);
int conv_x6_launch(bool dgrad, const float* x, const float* w, const float* bias,
                   const float* sc, const float* sh, float* y, double* stats, int64_t N, int Cin,
                   int Cout, int64_t H, int64_t W, hipStream_t s, int64_t* parts, bool b16,
                   bool x16, bool y16, int lay, const Bnr* bnr = nullptr);

// conv_x6.hip (fp32-accurate split-bf16 MFMA) serves every pair it has an
// instantiation for unless AINP_CONV_EXACT=1 selects the exact f32 kernels.
static bool conv_exact_env() {
  static const bool v = [] {
    const char* e = getenv("AINP_CONV_EXACT");
    return e && e[0] == '1';
  }();
  return v;
}

static int64_t exact_stat_parts(int64_t N, int64_t H, int64_t W) {
  return N * cdiv(H, CV_FT) * cdiv(W, CV_TT);
}
}  // namespace ainp

// Upper bound over both kernel families' tilings; the launch zero-fills the
// partials its tiling does not produce, so the fixed-order sum is unchanged.
extern "C" int ainp_conv3x3_fwd_stat_parts(int64_t N, int64_t H, int64_t W) {
  const int64_t a = exact_stat_parts(N, H, W), b = conv_x6_stat_parts(N, H, W);
  return (int)(a > b ? a : b);
}

// The BatchNorm partial rows ainp_conv3x3_fwd writes for this shape (the
// kernel the dispatch below selects; fewer than the bound above when a
// persistent kernel serves it).
extern "C" int64_t ainp_conv3x3_fwd_stat_rows_ex(int64_t N, int Cin, int Cout, int64_t H,
                                                 int64_t W, int flags) {
  if (!small_pair(Cin, Cout) && !conv_exact_env()) {
    const int64_t r =
        conv_x6_stat_rows(false, Cin, Cout, N, H, W, (flags & AINP_CONV_BF16) != 0);
    if (r) return r;
  }
  return exact_stat_parts(N, H, W);
}

extern "C" int64_t ainp_conv3x3_fwd_stat_rows(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  return ainp_conv3x3_fwd_stat_rows_ex(N, Cin, Cout, H, W, 0);
}

template <bool DG>
static int conv_fwd_dispatch(const float* x, const float* w, const float* bias,
                             const float* sc, const float* sh, float* y,
                             double* stats, int64_t N, int Cin, int Cout,
                             int64_t H, int64_t W, hipStream_t s, bool b16, bool x16 = false,
                             bool y16 = false, int lay = 0) {
  // partials [used, rows) of the BatchNorm statistics are zero
  auto zero_tail = [&](int64_t used) -> int {
    if (!stats) return AINP_OK;
    const int64_t bound =
        ainp_conv3x3_fwd_stat_rows_ex(N, Cin, Cout, H, W, b16 ? AINP_CONV_BF16 : 0);
    if (used >= bound) return AINP_OK;
    hipError_t e = hipMemsetAsync(stats + used * 2 * Cout, 0,
                                  (size_t)(bound - used) * 2 * Cout * sizeof(double), s);
    return e == hipSuccess ? AINP_OK : record_error(e, "conv3x3 stats tail");
  };
  static const char* kNo16 =
      "conv3x3: bf16 storage (AINP_CONV_DY16 / _X16 / _Y16) needs a split-bf16 kernel for this pair";
  if (small_pair(Cin, Cout)) {
    if (x16 || y16) return record_msg(kNo16);
    int64_t used = 0;
    const int rc = small_fwd_dispatch(DG, x, w, bias, sc, sh, y, stats, N, Cin, Cout, H, W, s,
                                      lay, Bnr{}, &used);
    return rc ? rc : zero_tail(used);
  }
  if (!conv_exact_env()) {
    int64_t parts = 0;
    const int rc = conv_x6_launch(DG, x, w, bias, sc, sh, y, stats, N, Cin, Cout, H, W, s,
                                  &parts, b16, x16, y16, lay);
    if (rc == 2) return record_msg(lay ? "conv3x3: no channel-last / bf16-storage kernel for this pair"
                                       : kNo16);
    if (rc != 1) return rc ? rc : zero_tail(parts);
  }
  if (x16 || y16) return record_msg(kNo16);
  if (lay) return record_msg("conv3x3: channel-last activations need a split-bf16 kernel for this pair");
  {
    const int rc = zero_tail(exact_stat_parts(N, H, W));
    if (rc) return rc;
  }
  dim3 grid((unsigned)cdiv(W, CV_TT), (unsigned)cdiv(H, CV_FT), (unsigned)N);
  const int ct = (Cout + 15) / 16;
  const bool ex = Cin % CV_CK == 0 && Cout % 16 == 0 &&
                  (int64_t)Cin * H * W * 4 < ((int64_t)1 << 31);
#define AINP_FWD(CTV)                                                                  \
  do {                                                                                 \
    if (ex)                                                                            \
      hipLaunchKernelGGL((conv3x3_fwd_mfma<CTV, DG, true>), grid, dim3(256), 0, s, x, w, \
                         bias, sc, sh, y, stats, Cin, Cout, (int)H, (int)W);           \
    else                                                                               \
      hipLaunchKernelGGL((conv3x3_fwd_mfma<CTV, DG, false>), grid, dim3(256), 0, s, x, \
                         w, bias, sc, sh, y, stats, Cin, Cout, (int)H, (int)W);        \
  } while (0)
  switch (ct) {
    case 1: AINP_FWD(1); break;
    case 2: AINP_FWD(2); break;
    case 3: AINP_FWD(3); break;
    case 4: AINP_FWD(4); break;
    default: return record_msg("conv3x3: Cout > 64 unsupported");
  }
#undef AINP_FWD
  return check_launch("conv3x3_fwd_mfma");
}

static bool conv_flags_ok(int flags) { return (flags & ~AINP_CONV_BF16) == 0; }
// forward: the act(x) source and / or y in bf16 storage (with the bf16 arithmetic);
// either may be channel-last
static bool conv_fwd_flags_ok(int flags) {
  const int cl = flags & (AINP_CONV_XCL | AINP_CONV_YCL);
  flags &= ~cl;
  return (flags & ~(AINP_CONV_BF16 | AINP_CONV_X16 | AINP_CONV_Y16)) == 0 &&
         (!(flags & (AINP_CONV_X16 | AINP_CONV_Y16)) || (flags & AINP_CONV_BF16));
}
// data / weight gradients: dy may be bf16 storage (with the bf16 arithmetic);
// data gradient: dy / dx channel-last; weight gradient: x / dy channel-last
static bool conv_grad_flags_ok(int flags, bool wgrad) {
  // data gradient: dx [C][H][N][W] (AINP_CONV_YCFNT) instead of channel-last
  if ((flags & AINP_CONV_YCFNT) && (wgrad || (flags & AINP_CONV_YCL))) return false;
  if (!wgrad) flags &= ~AINP_CONV_YCFNT;
  const int cl = flags & (wgrad ? (AINP_CONV_XCL | AINP_CONV_GCL) : (AINP_CONV_XCL | AINP_CONV_YCL));
  flags &= ~cl;
  const int extra = AINP_CONV_DY16 | (wgrad ? AINP_CONV_X16 : 0);
  return (flags & ~(AINP_CONV_BF16 | extra)) == 0 &&
         (!(flags & extra) || (flags & AINP_CONV_BF16));
}
// ABI layout flags -> the kernels' layout bits (bit 0 input, bit 1 output,
// bit 2 the weight gradient's dy)
static int conv_lay(int flags) {
  return ((flags & AINP_CONV_XCL) ? 1 : 0) | ((flags & AINP_CONV_YCL) ? 2 : 0) |
         ((flags & AINP_CONV_GCL) ? 4 : 0) | ((flags & AINP_CONV_YCFNT) ? 8 : 0);
}

extern "C" int ainp_conv3x3_fwd_ex(const float* x, const float* w,
                                   const float* bias, const float* in_scale,
                                   const float* in_shift, float* y, double* stats,
                                   int64_t N, int Cin, int Cout, int64_t H,
                                   int64_t W, int flags, void* stream) {
  if (!x || !w || !y || N < 0 || Cin < 1 || Cout < 1 || H < 1 || W < 1 ||
      N > 65535 || H > (1 << 24) || W > (1 << 24) || !conv_fwd_flags_ok(flags))
    return record_msg("ainp_conv3x3_fwd: bad argument");
  if ((in_scale == nullptr) != (in_shift == nullptr))
    return record_msg("ainp_conv3x3_fwd: in_scale/in_shift must both be set");
  if (N == 0) return AINP_OK;
  return conv_fwd_dispatch<false>(x, w, bias, in_scale, in_shift, y, stats, N,
                                  Cin, Cout, H, W, as_stream(stream),
                                  (flags & AINP_CONV_BF16) != 0, (flags & AINP_CONV_X16) != 0,
                                  (flags & AINP_CONV_Y16) != 0, conv_lay(flags));
}

extern "C" int ainp_conv3x3_fwd(const float* x, const float* w,
                                const float* bias, const float* in_scale,
                                const float* in_shift, float* y, double* stats,
                                int64_t N, int Cin, int Cout, int64_t H,
                                int64_t W, void* stream) {
  return ainp_conv3x3_fwd_ex(x, w, bias, in_scale, in_shift, y, stats, N, Cin, Cout, H, W, 0,
                             stream);
}

extern "C" int ainp_conv3x3_dgrad_ex(const float* dy, const float* w, float* dx,
                                     float* workspace, int64_t N, int Cin,
                                     int Cout, int64_t H, int64_t W, int flags,
                                     void* stream) {
  (void)workspace;
  if (!dy || !w || !dx || N < 0 || Cin < 1 || Cout < 1 || H < 1 || W < 1 ||
      N > 65535 || !conv_grad_flags_ok(flags, false))
    return record_msg("ainp_conv3x3_dgrad: bad argument");
  if ((flags & AINP_CONV_YCFNT) && ainp_conv3x3_dgrad_cfnt_ok(N, Cin, Cout, H, W) != 1)
    return record_msg("ainp_conv3x3_dgrad: AINP_CONV_YCFNT serves the 32 -> 16 channel data "
                      "gradient only (see ainp_conv3x3_dgrad_cfnt_ok)");
  if (N == 0) return AINP_OK;
  // conv over dy (Cout channels) producing Cin channels, flipped weights
  return conv_fwd_dispatch<true>(dy, w, nullptr, nullptr, nullptr, dx, nullptr,
                                 N, Cout, Cin, H, W, as_stream(stream),
                                 (flags & AINP_CONV_BF16) != 0, (flags & AINP_CONV_DY16) != 0,
                                 false, conv_lay(flags));
}

extern "C" int ainp_conv3x3_dgrad_cfnt_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  if (N < 0 || Cin < 1 || Cout < 1 || H < 1 || W < 1 || conv_exact_env()) return 0;
  return conv_x6_dgrad_cfnt_ok(Cout, Cin, N, H, W) ? 1 : 0;
}

extern "C" int ainp_conv3x3_dgrad(const float* dy, const float* w, float* dx,
                                  float* workspace, int64_t N, int Cin,
                                  int Cout, int64_t H, int64_t W,
                                  void* stream) {
  return ainp_conv3x3_dgrad_ex(dy, w, dx, workspace, N, Cin, Cout, H, W, 0, stream);
}

// Round 5: the data gradient with the consuming BatchNorm's backward reduce
// fused into its epilogue (conv_x6.hip Bnr): the split-bf16 data-gradient
// kernels with a channel-last dx sum (gz, gz * xhat) of the value they just
// computed into per-workgroup partials, so the separate reduce pass over dx
// and y disappears.  Pairs without such a kernel run the data gradient and
// then the channel-last reduce (same results, two passes).
static bool dgrad_bnr_env() {
  static const bool v = [] {
    const char* e = getenv("AINP_DGRAD_BNR");
    return !(e && e[0] == '0');
  }();
  return v;
}

extern "C" int64_t ainp_conv3x3_dgrad_bnr_workspace(int64_t N, int Cin, int Cout, int64_t H,
                                                    int64_t W) {
  (void)Cout;
  if (N < 0 || Cin < 1 || H < 1 || W < 1) return 0;
  int64_t rows = N * cdiv(H, 8) * cdiv(W, 32);            // 8-row tiles
  const int64_t pers = 512 * (int64_t)X6_OCC_MAX;         // persistent grids
  if (rows < pers) rows = pers;
  if (rows < exact_stat_parts(N, H, W)) rows = exact_stat_parts(N, H, W);   // small convs
  const int64_t fused = rows * 2 * Cin * (int64_t)sizeof(double);
  const int64_t sep = (int64_t)ainp_bn_relu_bwd_workspace(N, Cin, H, W);
  return fused > sep ? fused : sep;
}

extern "C" int ainp_conv3x3_dgrad_bnr(const float* dy, const float* w, float* dx, int64_t N,
                                      int Cin, int Cout, int64_t H, int64_t W, int flags,
                                      const void* y, const float* scale, const float* shift,
                                      const float* save_mean_rstd, void* workspace, double* sums,
                                      int bn_flags, void* stream) {
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  // dx == nullptr (round 6): the partials only, for the 1 -> 16 data gradient
  // whose dx the apply recomputes (ainp_conv3x3_dgrad_bnapply)
  const bool nodx = !dx && small_pair(Cout, Cin) && Cin == 16 && dgrad_bnr_env() &&
                    !(flags & AINP_CONV_DY16);
  if (!dy || !w || (!dx && !nodx) || !y || !scale || !shift || !save_mean_rstd || !workspace ||
      !sums || N < 1 || Cin < 1 || Cout < 1 || H < 1 || W < 1 || N > 65535 ||
      !conv_grad_flags_ok(flags, false) || !(flags & AINP_CONV_YCL) ||
      (bn_flags & ~AINP_BN_Y16) || !(Cin == 16 || Cin == 32 || Cin == 64) ||
      !al16(dx) || !al16(y) || !al16(scale) || !al16(shift) || !al16(save_mean_rstd))
    return record_msg("ainp_conv3x3_dgrad_bnr: bad argument (channel-last dx and y, C in "
                      "{16, 32, 64}, 16-byte aligned dx / y / scale / shift / save)");
  const hipStream_t s = as_stream(stream);
  const Bnr bnr{y, scale, shift, save_mean_rstd, (bn_flags & AINP_BN_Y16) ? 1 : 0};
  double* partial = reinterpret_cast<double*>(workspace);
  if (dgrad_bnr_env() && small_pair(Cout, Cin) && Cin % 4 == 0 && !(flags & AINP_CONV_DY16)) {
    // 1 -> 16 channels: the small kernel's channel-last epilogue
    int64_t used = 0;
    const int rc = small_fwd_dispatch(true, dy, w, nullptr, nullptr, nullptr, dx, partial, N,
                                      Cout, Cin, H, W, s, conv_lay(flags), bnr, &used);
    if (rc) return rc;
    return bn_cl_sum_partials(partial, (int)used, 2 * Cin, sums, s);
  }
  if (dgrad_bnr_env() && !small_pair(Cout, Cin) && !conv_exact_env()) {
    int64_t parts = 0;
    const int rc = conv_x6_launch(true, dy, w, nullptr, nullptr, nullptr, dx, partial, N, Cout,
                                  Cin, H, W, s, &parts, (flags & AINP_CONV_BF16) != 0,
                                  (flags & AINP_CONV_DY16) != 0, false, conv_lay(flags), &bnr);
    if (rc == AINP_OK) return bn_cl_sum_partials(partial, (int)parts, 2 * Cin, sums, s);
    if (rc < 0) return rc;
  }
  const int rc = ainp_conv3x3_dgrad_ex(dy, w, dx, nullptr, N, Cin, Cout, H, W, flags, stream);
  if (rc) return rc;
  return ainp_bn_relu_bwd_reduce_ex(dx, reinterpret_cast<const float*>(y), scale, shift,
                                    save_mean_rstd, workspace, sums, N, Cin, H, W, 0,
                                    AINP_BN_CL | (bn_flags & AINP_BN_Y16), stream);
}

// Round 6: Conv2d(16, 1)'s data gradient (dy one channel -> dx 16, decoder.6)
// through the BatchNorm+ReLU backward apply of the 16-channel layer it feeds
// (decoder.5), one row-strip pass: gy = apply(dx recomputed, y), dx never
// written.  The reduce's sums come from ainp_conv3x3_dgrad_bnr with dx null.
extern "C" int ainp_conv3x3_dgrad_bnapply(const float* dy, const float* w, const float* y,
                                          const float* scale, const float* shift,
                                          const float* gamma, const float* save_mean_rstd,
                                          const double* sums, int64_t count, void* gy, int gy16,
                                          float* dgamma, float* dbeta, int64_t N, int Cin,
                                          int Cout, int64_t H, int64_t W, void* stream) {
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  const int nfs = (int)cdiv(H > 0 ? H : 1, R16_RS), nts = (int)cdiv(W > 0 ? W : 1, R16_TW);
  const int64_t ns = N * nfs * nts;
  if (!dy || !w || !y || !scale || !shift || !save_mean_rstd || !sums || !gy || N < 1 || H < 1 ||
      W < 1 || Cin != 16 || Cout != 1 || count < 0 || !al16(y) || !al16(gy) ||
      ns >= ((int64_t)1 << 31) || N * H * W * 16 >= ((int64_t)1 << 40))
    return record_msg("ainp_conv3x3_dgrad_bnapply: bad argument (Conv2d(16, 1), channel-last "
                      "16-byte aligned fp32 y, gy)");
  const Bnr bnr{y, scale, shift, save_mean_rstd, 0};
  const BnApply bna{nullptr, y, scale, shift, gamma, save_mean_rstd, sums, dgamma, dbeta,
                    count > 0 ? 1.0 / (double)count : 0.0};
  const dim3 grid((unsigned)cdiv(ns, 4));
  if (gy16)
    hipLaunchKernelGGL((conv3x3_rows_1to16<true, false, false, 3>), grid, dim3(256), 0,
                       as_stream(stream), dy, w, nullptr, nullptr, nullptr,
                       reinterpret_cast<float*>(gy), nullptr, bnr, (int)H, (int)W, nfs, nts,
                       (int)ns, bna);
  else
    hipLaunchKernelGGL((conv3x3_rows_1to16<true, false, false, 2>), grid, dim3(256), 0,
                       as_stream(stream), dy, w, nullptr, nullptr, nullptr,
                       reinterpret_cast<float*>(gy), nullptr, bnr, (int)H, (int)W, nfs, nts,
                       (int)ns, bna);
  return check_launch("conv3x3_rows_1to16 (apply)");
}

extern "C" int ainp_conv3x3_dy16_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  (void)N;
  if (Cin < 1 || Cout < 1 || H < 1 || W < 1 || small_pair(Cin, Cout) || conv_exact_env())
    return 0;
  // weight gradient: one 32-channel pass on conv3x3_wgrad_x6(s) (conv_wgrad_x6_launch)
  const bool fits =
      (int64_t)H * W * 4 * (Cout > WG_CIMAX ? Cout : WG_CIMAX) < ((int64_t)1 << 31);
  const int cp = wgrad_pass(Cin);
  if (!fits || Cin > WG_CIMAX ||
      !((cp == 32 && Cout == 16) || (cp == 16 && Cout == 32) || (cp == 32 && Cout == 64)))
    return 0;
  // data gradient: the conv over dy (Cout channels) producing Cin
  return conv_x6_dgrad16_ok(Cout, Cin, H, W) ? 1 : 0;
}

extern "C" int ainp_conv3x3_io16_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  (void)N;
  if (Cin < 1 || Cout < 1 || H < 1 || W < 1 || small_pair(Cin, Cout) || conv_exact_env())
    return 0;
  const bool fits =
      (int64_t)H * W * 4 * (Cout > WG_CIMAX ? Cout : WG_CIMAX) < ((int64_t)1 << 31);
  const int cp = wgrad_pass(Cin);
  if (!fits || Cin > WG_CIMAX ||
      !((cp == 32 && Cout == 16) || (cp == 16 && Cout == 32) || (cp == 32 && Cout == 64)))
    return 0;
  return conv_x6_fwd16_ok(Cin, Cout, H, W) ? 1 : 0;
}

// Round 5: 1 if every conv3x3 entry point of this nn.Conv2d(Cin, Cout) takes
// channel-last activations (AINP_CONV_XCL / _YCL / _GCL; host-only)
extern "C" int ainp_conv3x3_cl_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W) {
  (void)N;
  if (Cin < 1 || Cout < 1 || H < 1 || W < 1 || conv_exact_env()) return 0;
  const int64_t cmax = Cin > Cout ? Cin : Cout;
  if (H * W * cmax * 4 >= ((int64_t)1 << 31)) return 0;
  if (small_pair(Cin, Cout)) return (Cin == 16 && Cout == 1) || (Cin == 1 && Cout == 16);
  // forward (persistent x6p / x6q), data gradient (x6p / x6q / 8-row tiled),
  // weight gradient (one 32-channel pass on wgrad_x6 / x6s)
  const bool fwd = (Cin == 16 && Cout == 32) || (Cin == 32 && Cout == 64) ||
                   (Cin == 32 && Cout == 16);
  const bool dgr = (Cout == 32 && Cin == 16) || (Cout == 16 && Cin == 32) ||
                   (Cout == 64 && Cin == 32);
  return fwd && dgr ? 1 : 0;
}

extern "C" size_t ainp_conv3x3_wgrad_workspace(int64_t N, int Cin, int Cout,
                                               int64_t H, int64_t W) {
  if (small_pair(Cin, Cout)) return small_wgrad_ws(N, Cin, Cout, H, W);
  const int cp = wgrad_pass(Cin);
  int ct = wgrad_ct(Cout);
  if (ct == 3) ct = 4;
  // slabs for the largest grid (the bf16 x6 kernels' multiplier, conv_x6_occ16)
  return (size_t)(WG_BLOCKS * X6_OCC_MAX + 2 * WG_GROUPS) * ct * 16 * (9 * cp + 1) *
         sizeof(float);
}

extern "C" int ainp_conv3x3_wgrad(const float* x, const float* in_scale,
                                  const float* in_shift, const float* dy,
                                  float* dw, float* dbias, void* workspace,
                                  int64_t N, int Cin, int Cout, int64_t H,
                                  int64_t W, void* stream) {
  return ainp_conv3x3_wgrad_ex(x, in_scale, in_shift, dy, dw, dbias, workspace, N, Cin, Cout, H,
                               W, 0, stream);
}

// Round 6: the 1 -> 16 conv's weight gradient with the BatchNorm+ReLU
// backward apply of its output fused in (conv3x3_strip_wgrad_cl<BNA>): gy is
// formed per element from g and y instead of read, and never written.
extern "C" int ainp_conv3x3_wgrad_bnapply(const float* x, const float* in_scale,
                                          const float* in_shift, const float* g, const float* y,
                                          const float* scale, const float* shift,
                                          const float* gamma, const float* save_mean_rstd,
                                          const double* sums, int64_t count, float* dw,
                                          float* dbias, float* dgamma, float* dbeta,
                                          void* workspace, int64_t N, int Cin, int Cout, int64_t H,
                                          int64_t W, void* stream) {
  auto al16 = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (!x || !g || !y || !scale || !shift || !save_mean_rstd || !sums || !dw || !workspace ||
      N < 1 || H < 1 || W < 1 || Cin != 1 || Cout != 16 || count < 0 || !al16(g) || !al16(y) ||
      (in_scale == nullptr) != (in_shift == nullptr))
    return record_msg("ainp_conv3x3_wgrad_bnapply: bad argument (Conv2d(1, 16), channel-last "
                      "16-byte aligned fp32 g / y)");
  const BnApply bna{g, y, scale, shift, gamma, save_mean_rstd, sums, dgamma, dbeta,
                    count > 0 ? 1.0 / (double)count : 0.0};
  return small_wgrad(x, in_scale, in_shift, nullptr, dw, dbias, workspace, N, Cin, Cout, H, W,
                     as_stream(stream), 4, &bna);
}

extern "C" int ainp_conv3x3_wgrad_ex(const float* x, const float* in_scale,
                                     const float* in_shift, const float* dy,
                                     float* dw, float* dbias, void* workspace,
                                     int64_t N, int Cin, int Cout, int64_t H,
                                     int64_t W, int flags, void* stream) {
  if (!x || !dy || !dw || !workspace || N < 1 || Cin < 1 || Cout < 1 ||
      H < 1 || W < 1 || !conv_grad_flags_ok(flags, true))
    return record_msg("ainp_conv3x3_wgrad: bad argument");
  const bool b16 = (flags & AINP_CONV_BF16) != 0;
  const bool g16 = (flags & AINP_CONV_DY16) != 0;
  const bool x16 = (flags & AINP_CONV_X16) != 0;
  static const char* kNo16 =
      "ainp_conv3x3_wgrad: bf16 storage (AINP_CONV_DY16 / _X16) needs a split-bf16 "
      "weight-gradient kernel for this pair";
  if ((in_scale == nullptr) != (in_shift == nullptr))
    return record_msg("ainp_conv3x3_wgrad: in_scale/in_shift must both be set");
  const int lay = conv_lay(flags);
  if (small_pair(Cin, Cout)) {
    if (g16 || x16) return record_msg(kNo16);
    return small_wgrad(x, in_scale, in_shift, dy, dw, dbias, workspace, N, Cin, Cout, H, W,
                       as_stream(stream), lay);
  }
  const int CT = wgrad_ct(Cout);
  if (CT > 4) return record_msg("ainp_conv3x3_wgrad: Cout > 64 unsupported");
  const int CTp = CT == 3 ? 4 : CT;  // kernel co-tiles (waves split evenly)
  hipStream_t s = as_stream(stream);
  float* partial = reinterpret_cast<float*>(workspace);
  for (int ci0 = 0; ci0 < Cin; ci0 += WG_CIMAX) {
    const int cp = (Cin - ci0) < WG_CIMAX ? (Cin - ci0) : WG_CIMAX;
    const int JT = (9 * cp + 15) / 16;  // 1..18
#define AINP_WG(CTV)                                                                \
  do {                                                                              \
    if (JT <= 1) launch_wgrad<CTV, 1>(x, in_scale, in_shift, dy, partial, (int)N,  \
                                      Cin, Cout, (int)H, (int)W, ci0, cp, s);       \
    else if (JT <= 4) launch_wgrad<CTV, 4>(x, in_scale, in_shift, dy, partial,     \
                                           (int)N, Cin, Cout, (int)H, (int)W, ci0, \
                                           cp, s);                                  \
    else if (JT <= 9) launch_wgrad<CTV, 9>(x, in_scale, in_shift, dy, partial,     \
                                           (int)N, Cin, Cout, (int)H, (int)W, ci0, \
                                           cp, s);                                  \
    else launch_wgrad<CTV, 18>(x, in_scale, in_shift, dy, partial, (int)N, Cin,    \
                               Cout, (int)H, (int)W, ci0, cp, s);                   \
  } while (0)
    // specialised kernel: 32-bit buffer offsets must cover a sample's planes
    const bool fits = (int64_t)H * W * 4 * (Cout > WG_CIMAX ? Cout : WG_CIMAX) < ((int64_t)1 << 31);
    const int key = fits ? cp * 100 + Cout : 0;
#define AINP_WGT(CPV, COV)                                                           \
  hipLaunchKernelGGL((conv3x3_wgrad_t<CPV, COV>), dim3(WG_BLOCKS),                    \
                     dim3(WgradT<CPV, COV>::NW * 64), 0, s, x,                          \
                     in_scale, in_shift, dy, partial, (int)N, Cin, (int)H, (int)W, ci0)
    // split-bf16 kernel where it is instantiated (conv_x6.hip), unless
    // AINP_CONV_EXACT=1; same slab format
    int nblk_x6 = b16 ? WG_BLOCKS * conv_x6_occ16() : WG_BLOCKS;
    int rc = (fits && !conv_exact_env())
                 ? conv_wgrad_x6_launch(x, in_scale, in_shift, dy, partial, N, Cin, Cout, H, W,
                                        ci0, cp, nblk_x6, s, b16, g16, x16, lay, &nblk_x6)
                 : 1;
    if (rc == 1 && (g16 || x16)) return record_msg(kNo16);
    if (rc == 1 && lay)
      return record_msg("ainp_conv3x3_wgrad: channel-last activations need a split-bf16 kernel");
    const int nblk = rc == 0 ? nblk_x6 : WG_BLOCKS;   // slabs the launch writes
    if (rc == 1) switch (key) {
      case 1616: AINP_WGT(16, 16); break;
      case 1632: AINP_WGT(16, 32); break;
      case 1664: AINP_WGT(16, 64); break;
      case 3216: AINP_WGT(32, 16); break;
      case 3232: AINP_WGT(32, 32); break;
      case 3264: AINP_WGT(32, 64); break;
      default:
        switch (CTp) {
          case 1: AINP_WG(1); break;
          case 2: AINP_WG(2); break;
          default: AINP_WG(4); break;
        }
    }
#undef AINP_WGT
#undef AINP_WG
    if (rc == 1) rc = check_launch("conv3x3_wgrad_mfma");
    if (rc) return rc;
    const int J = 9 * cp;
    const int per = CTp * 16 * (J + 1);
    double* tmp = reinterpret_cast<double*>(partial + (size_t)nblk * per);
    hipLaunchKernelGGL(wgrad_reduce1, dim3((per + 255) / 256, WG_GROUPS), dim3(256), 0, s,
                       partial, nblk, per, nblk / WG_GROUPS, tmp);
    rc = check_launch("wgrad_reduce1");
    if (rc) return rc;
    hipLaunchKernelGGL(wgrad_reduce, dim3((per + 255) / 256), dim3(256), 0, s,
                       tmp, WG_GROUPS, CTp * 16, J, cp, ci0, Cin, Cout, dw,
                       dbias, ci0 == 0 ? 1 : 0);
    rc = check_launch("wgrad_reduce");
    if (rc) return rc;
  }
  return AINP_OK;
}
