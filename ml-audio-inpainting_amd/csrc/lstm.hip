// lstm.hip — BLSTM recurrence (forward and backward through time).
//
// Replaces the recurrent part of nn.LSTM(bidirectional=True, batch_first=True)
// of models/CNNBLSTM/model.py:46-47,77.  The input projections x W_ih^T + b
// are one big MFMA GEMM (gemm.hip) done before the recurrence; what remains
// per time step is h_{t-1} W_hh^T (4H x H) plus the gate nonlinearities.
//
// Mapping: one workgroup of 2H lanes per (sequence, direction) pair, W_hh held
// in VGPRs for the whole sequence (2H floats per lane: at H=128 that is 256
// VGPRs, one wave per SIMD), h_{t-1} broadcast from LDS.  Lane pair (2j,2j+1)
// owns hidden unit j: lane 2j the (i,f) gate rows, lane 2j+1 the (g,o) rows;
// the pair swaps pre-activations with one xor-shuffle and both finish the cell
// update.  No inter-workgroup traffic at all: the 2*N sequence-directions run
// as independent workgroups, one step = one LDS barrier.
// Per-step inputs (zx rows, and for the backward the saved gates/cells/dh) are
// staged 16 steps at a time through LDS by register-prefetched chunk loads.
//
// Arithmetic: fp32, PyTorch gate order i,f,g,o; c' = f c + i g; h' = o tanh c'.
#include "common.h"

namespace ainp {

constexpr int LCH = 16;  // steps per staged chunk

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

template <int H>
__global__ __launch_bounds__(2 * H, 1) void lstm_fwd_kernel(
    const float* __restrict__ zx, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ h_out,
    float* __restrict__ gates, float* __restrict__ cell, int T) {
  constexpr int NT = 2 * H;         // threads
  constexpr int G4 = 4 * H;         // gate rows
  constexpr int PF = LCH * G4 / 4 / NT;  // float4 prefetched per thread (=8)
  __shared__ __attribute__((aligned(16))) float zs[2][LCH][G4];
  __shared__ __attribute__((aligned(16))) float hb[2][H];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, j = tid >> 1, half = tid & 1;
  const float* whh = dir ? whh_r : whh_f;
  const int row0 = half ? 2 * H + j : j;
  const int row1 = half ? 3 * H + j : H + j;

  float w0[H], w1[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    w0[k] = whh[(int64_t)row0 * H + k];
    w1[k] = whh[(int64_t)row1 * H + k];
  }
  if (tid < H) hb[1][tid] = 0.f;

  const int64_t zrow = 8 * H;  // zx row length (both directions)
  const float* zbase = zx + (int64_t)n * T * zrow + dir * G4;
  auto tix = [&](int t) { return dir ? (T - 1 - t) : t; };

  float4 pf[PF];
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int idx = tid + i * NT;  // float4 index within chunk
      const int s = idx / (G4 / 4), r = (idx % (G4 / 4)) * 4;
      const int t = ch * LCH + s;
      pf[i] = (t < T) ? *reinterpret_cast<const float4*>(zbase + (int64_t)tix(t) * zrow + r)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / (G4 / 4), r = (idx % (G4 / 4)) * 4;
      *reinterpret_cast<float4*>(&zs[buf][s][r]) = pf[i];
    }
  };

  const int nch = (T + LCH - 1) / LCH;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  float c = 0.f;
  float* hrow = h_out + (int64_t)n * T * 2 * H + dir * H + j;
  float* crow = cell ? cell + (int64_t)n * T * 2 * H + dir * H + j : nullptr;
  float* grow = gates ? gates + (int64_t)n * T * 8 * H + dir * G4 : nullptr;

  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load_chunk(ch + 1);
    for (int s = 0; s < LCH; ++s) {
      const int t = ch * LCH + s;
      if (t >= T) break;  // uniform across the block
      const float* hp = hb[(t + 1) & 1];
      float a0 = zs[buf][s][row0], a1 = zs[buf][s][row1];
      float b0 = 0.f, b1 = 0.f, c0 = 0.f, c1 = 0.f, d0 = 0.f, d1 = 0.f;
#pragma unroll
      for (int k = 0; k < H; k += 4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hp + k);
        a0 = fmaf(w0[k + 0], h4.x, a0);
        a1 = fmaf(w1[k + 0], h4.x, a1);
        b0 = fmaf(w0[k + 1], h4.y, b0);
        b1 = fmaf(w1[k + 1], h4.y, b1);
        c0 = fmaf(w0[k + 2], h4.z, c0);
        c1 = fmaf(w1[k + 2], h4.z, c1);
        d0 = fmaf(w0[k + 3], h4.w, d0);
        d1 = fmaf(w1[k + 3], h4.w, d1);
      }
      const float p0 = (a0 + b0) + (c0 + d0);
      const float p1 = (a1 + b1) + (c1 + d1);
      const float q0 = __shfl_xor(p0, 1, 64);
      const float q1 = __shfl_xor(p1, 1, 64);
      const float ip = half ? q0 : p0, fp = half ? q1 : p1;
      const float gp = half ? p0 : q0, op = half ? p1 : q1;
      const float ig = sigm(ip), fg = sigm(fp), gg = tanhf(gp), og = sigm(op);
      c = fmaf(fg, c, ig * gg);
      const float h = og * tanhf(c);
      const int64_t tt = tix(t);
      if (!half) {
        hb[t & 1][j] = h;
        hrow[tt * 2 * H] = h;
        if (crow) crow[tt * 2 * H] = c;
        if (grow) {
          grow[tt * 8 * H + j] = ig;
          grow[tt * 8 * H + H + j] = fg;
        }
      } else if (grow) {
        grow[tt * 8 * H + 2 * H + j] = gg;
        grow[tt * 8 * H + 3 * H + j] = og;
      }
      __syncthreads();
    }
    if (ch + 1 < nch) store_chunk(buf ^ 1);
    __syncthreads();
  }
}

// Backward through time.  Bwd step u walks the forward steps in reverse:
// forward step t = T-1-u, time index tt(t).  Lane pair (2k,2k+1) also owns
// the recurrent matvec output dh_rec[k] = sum_g dG[g] W[g][k]: lane 2k sums
// g in [0,2H) (i,f rows), lane 2k+1 g in [2H,4H) (g,o rows).
template <int H>
__global__ __launch_bounds__(2 * H, 1) void lstm_bwd_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates,
    const float* __restrict__ cell, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ dgates, int T) {
  constexpr int NT = 2 * H;
  constexpr int G4 = 4 * H;
  constexpr int PG = LCH * G4 / 4 / NT;            // float4 of gates per thread (8)
  constexpr int PC = ((LCH + 1) * H + NT - 1) / NT;  // cell floats per thread (9)
  constexpr int PD = LCH * H / NT;                 // dh floats per thread (8)
  __shared__ __attribute__((aligned(16))) float gsm[2][LCH][G4];
  __shared__ float csm[2][LCH + 1][H];
  __shared__ float dsm[2][LCH][H];
  __shared__ __attribute__((aligned(16))) float dgb[2][G4];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, j = tid >> 1, half = tid & 1;
  const float* whh = dir ? whh_r : whh_f;
  // lane holds W[2H*half + q][j], q in [0, 2H)
  float wt[2 * H];
#pragma unroll
  for (int q = 0; q < 2 * H; ++q) wt[q] = whh[(int64_t)(2 * H * half + q) * H + j];

  auto tix = [&](int t) { return dir ? (T - 1 - t) : t; };
  const float* gbase = gates + (int64_t)n * T * 8 * H + dir * G4;
  const float* cbase = cell + (int64_t)n * T * 2 * H + dir * H;
  const float* dbase = dh_out + (int64_t)n * T * 2 * H + dir * H;

  float4 pg[PG];
  float pc[PC], pd[PD];
  // chunk ch covers bwd steps u in [ch*LCH, ch*LCH+LCH); forward step
  // t = T-1-u; cells for u..u+LCH (the extra row is c_{t-1} of the last step)
  auto load_chunk = [&](int ch) {
#pragma unroll
    for (int i = 0; i < PG; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / (G4 / 4), r = (idx % (G4 / 4)) * 4;
      const int t = T - 1 - (ch * LCH + s);
      pg[i] = (t >= 0) ? *reinterpret_cast<const float4*>(gbase + (int64_t)tix(t) * 8 * H + r)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PC; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / H, r = idx % H;
      const int t = T - 1 - (ch * LCH + s);
      pc[i] = (s <= LCH && t >= 0) ? cbase[(int64_t)tix(t) * 2 * H + r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / H, r = idx % H;
      const int t = T - 1 - (ch * LCH + s);
      pd[i] = (t >= 0) ? dbase[(int64_t)tix(t) * 2 * H + r] : 0.f;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PG; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / (G4 / 4), r = (idx % (G4 / 4)) * 4;
      *reinterpret_cast<float4*>(&gsm[buf][s][r]) = pg[i];
    }
#pragma unroll
    for (int i = 0; i < PC; ++i) {
      const int idx = tid + i * NT;
      const int s = idx / H, r = idx % H;
      if (s <= LCH) csm[buf][s][r] = pc[i];
    }
#pragma unroll
    for (int i = 0; i < PD; ++i) {
      const int idx = tid + i * NT;
      dsm[buf][idx / H][idx % H] = pd[i];
    }
  };

  const int nch = (T + LCH - 1) / LCH;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  float dh_rec = 0.f, dc_next = 0.f;
  float* dgrow = dgates + (int64_t)n * T * 8 * H + dir * G4;
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load_chunk(ch + 1);
    for (int s = 0; s < LCH; ++s) {
      const int u = ch * LCH + s;
      if (u >= T) break;
      const int t = T - 1 - u;
      const float ig = gsm[buf][s][j], fg = gsm[buf][s][H + j];
      const float gg = gsm[buf][s][2 * H + j], og = gsm[buf][s][3 * H + j];
      const float cc = csm[buf][s][j];
      const float cp = (t > 0) ? csm[buf][s + 1][j] : 0.f;
      const float dh = dsm[buf][s][j] + dh_rec;
      const float tc = tanhf(cc);
      const float dog = dh * tc;
      const float dc = fmaf(dh * og, 1.f - tc * tc, dc_next);
      const float dig = dc * gg, dgg = dc * ig, dfg = dc * cp;
      dc_next = dc * fg;
      const float dai = dig * ig * (1.f - ig);
      const float daf = dfg * fg * (1.f - fg);
      const float dag = dgg * (1.f - gg * gg);
      const float dao = dog * og * (1.f - og);
      const int64_t tt = tix(t);
      float* dgr = dgrow + tt * 8 * H;
      float* db = dgb[u & 1];
      if (!half) {
        db[j] = dai;
        db[H + j] = daf;
        dgr[j] = dai;
        dgr[H + j] = daf;
      } else {
        db[2 * H + j] = dag;
        db[3 * H + j] = dao;
        dgr[2 * H + j] = dag;
        dgr[3 * H + j] = dao;
      }
      __syncthreads();
      const float* dq = db + 2 * H * half;
      float a = 0.f, b = 0.f, c = 0.f, d = 0.f;
#pragma unroll
      for (int q = 0; q < 2 * H; q += 4) {
        const float4 v = *reinterpret_cast<const float4*>(dq + q);
        a = fmaf(wt[q + 0], v.x, a);
        b = fmaf(wt[q + 1], v.y, b);
        c = fmaf(wt[q + 2], v.z, c);
        d = fmaf(wt[q + 3], v.w, d);
      }
      const float part = (a + b) + (c + d);
      dh_rec = part + __shfl_xor(part, 1, 64);
    }
    if (ch + 1 < nch) store_chunk(buf ^ 1);
    __syncthreads();
  }
}

// hprev[n][t][dir*H + k] = h of the previous forward step (0 at the start):
// dir 0 -> h_out[n][t-1][k], dir 1 -> h_out[n][t+1][H+k].
__global__ void lstm_hprev_kernel(const float* __restrict__ h_out,
                                  float* __restrict__ hprev, int64_t N,
                                  int64_t T, int H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = N * T * 2 * H;
  if (i >= total) return;
  const int64_t col = i % (2 * H);
  const int64_t t = (i / (2 * H)) % T;
  const int dir = col >= H;
  float v = 0.f;
  if (!dir && t > 0) v = h_out[i - 2 * H];
  if (dir && t < T - 1) v = h_out[i + 2 * H];
  hprev[i] = v;
}

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_lstm_rec_fwd(const float* zx, const float* const* w_hh,
                                 float* h_out, float* gates, float* cell,
                                 int64_t N, int64_t T, int H, void* stream) {
  if (!zx || !w_hh || !w_hh[0] || !w_hh[1] || !h_out || N < 0 || T < 0 ||
      N > 32768)
    return record_msg("ainp_lstm_rec_fwd: bad argument");
  if (N == 0 || T == 0) return AINP_OK;
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)(2 * N));
  switch (H) {
    case 32: hipLaunchKernelGGL(lstm_fwd_kernel<32>, grid, dim3(64), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
    case 64: hipLaunchKernelGGL(lstm_fwd_kernel<64>, grid, dim3(128), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
    case 128: hipLaunchKernelGGL(lstm_fwd_kernel<128>, grid, dim3(256), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
    default: return record_msg("ainp_lstm_rec_fwd: H must be 32, 64 or 128");
  }
  return check_launch("lstm_fwd_kernel");
}

extern "C" int ainp_lstm_rec_bwd(const float* dh_out, const float* gates,
                                 const float* cell, const float* const* w_hh,
                                 float* dgates, int64_t N, int64_t T, int H,
                                 void* stream) {
  if (!dh_out || !gates || !cell || !w_hh || !w_hh[0] || !w_hh[1] || !dgates ||
      N < 0 || T < 0 || N > 32768)
    return record_msg("ainp_lstm_rec_bwd: bad argument");
  if (N == 0 || T == 0) return AINP_OK;
  hipStream_t s = as_stream(stream);
  dim3 grid((unsigned)(2 * N));
  switch (H) {
    case 32: hipLaunchKernelGGL(lstm_bwd_kernel<32>, grid, dim3(64), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
    case 64: hipLaunchKernelGGL(lstm_bwd_kernel<64>, grid, dim3(128), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
    case 128: hipLaunchKernelGGL(lstm_bwd_kernel<128>, grid, dim3(256), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
    default: return record_msg("ainp_lstm_rec_bwd: H must be 32, 64 or 128");
  }
  return check_launch("lstm_bwd_kernel");
}

extern "C" int ainp_lstm_hprev(const float* h_out, float* hprev, int64_t N,
                               int64_t T, int H, void* stream) {
  if (!h_out || !hprev || N < 0 || T < 0 || H < 1)
    return record_msg("ainp_lstm_hprev: bad argument");
  const int64_t total = N * T * 2 * H;
  if (total == 0) return AINP_OK;
  hipLaunchKernelGGL(lstm_hprev_kernel, dim3((unsigned)cdiv(total, 256)),
                     dim3(256), 0, as_stream(stream), h_out, hprev, N, T, H);
  return check_launch("lstm_hprev");
}
