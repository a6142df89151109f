// lstm.hip — BLSTM recurrence (forward and backward through time).
//
// Replaces the recurrent part of nn.LSTM(bidirectional=True, batch_first=True)
// of models/CNNBLSTM/model.py:46-47,77.  The input projections x W_ih^T + b
// are one big MFMA GEMM (gemm.hip) done before the recurrence; what remains
// per time step is h_{t-1} W_hh^T (4H x H) plus the gate nonlinearities.
//
// Mapping: one workgroup of 4H lanes per (sequence, direction) pair, W_hh held
// in VGPRs for the whole sequence (one gate row = H floats per lane: 128 VGPRs
// at H=128, two waves per SIMD), h_{t-1} broadcast from LDS.  The lane quad
// (4u..4u+3) owns hidden unit u's gates i,f,g,o and exchanges them with DPP.
// No inter-workgroup traffic at all: the 2*N sequence-directions run as
// independent workgroups, one step = one LDS barrier.
// Per-step inputs (zx rows, and for the backward the saved gates/cells/dh) are
// staged 16 steps at a time through LDS by register-prefetched chunk loads.
//
// Arithmetic: fp32, PyTorch gate order i,f,g,o; c' = f c + i g; h' = o tanh c'.
#include "common.h"

namespace ainp {

constexpr int LCH = 16;  // steps per staged chunk

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// Per-step workgroup barrier that orders LDS only.  __syncthreads() would also
// wait (vmcnt(0)) for the step's global stores of h/c/gates, putting a full
// store round trip on the sequential critical path of every time step.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Quad broadcast: value of lane (4*(lane/4) + Q) to every lane of the quad.
// Packed fp32 pair: v_pk_fma_f32 issues two FMAs per instruction on gfx950,
// halving the issue cost of the per-step W_hh matvec.  Lanes .x/.y of the two
// accumulators are the same k mod 4 chains as four scalar accumulators, so the
// result is bit-identical to the scalar form.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int Q>
__device__ __forceinline__ float quad_bcast(float v) {
  constexpr int ctrl = Q | (Q << 2) | (Q << 4) | (Q << 6);  // DPP quad_perm
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
}

// Forward recurrence.  4H lanes per (sequence, direction): lane = 4u + g owns
// gate row r = g*H + u of W_hh (H VGPRs; at H=128 no accumulator-file round
// trips), so a hidden unit's four gates (i,f,g,o) sit in one lane quad and are
// exchanged with DPP quad broadcasts.  h_{t-1} is read from LDS as broadcast
// ds_read_b128.  One LDS barrier per step.
template <int H>
__global__ __launch_bounds__(4 * H, 1) void lstm_fwd_kernel(
    const float* __restrict__ zx, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ h_out,
    float* __restrict__ gates, float* __restrict__ cell, int T) {
  constexpr int NT = 4 * H;         // threads
  constexpr int G4 = 4 * H;         // gate rows
  constexpr int PF = LCH * G4 / 4 / NT;  // float4 prefetched per thread (=LCH/4)
  __shared__ __attribute__((aligned(16))) float zs[2][LCH][G4];
  __shared__ __attribute__((aligned(16))) float hb[2][H];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, u = tid >> 2, g = tid & 3;
  const int row = g * H + u;
  const float* whh = dir ? whh_r : whh_f;

  f2 w[H / 2];
#pragma unroll
  for (int k = 0; k < H; k += 4) {
    const float4 v = *reinterpret_cast<const float4*>(whh + (int64_t)row * H + k);
    w[k / 2] = f2{v.x, v.y}; w[k / 2 + 1] = f2{v.z, v.w};
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
  float* hrow = h_out + (int64_t)n * T * 2 * H + dir * H + u;
  float* crow = cell ? cell + (int64_t)n * T * 2 * H + dir * H + u : nullptr;
  float* grow = gates ? gates + (int64_t)n * T * 8 * H + dir * G4 + row : nullptr;

  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load_chunk(ch + 1);
    for (int s = 0; s < LCH; ++s) {
      const int t = ch * LCH + s;
      if (t >= T) break;  // uniform across the block
      const float* hp = hb[(t + 1) & 1];
      f2 a01 = f2{zs[buf][s][row], 0.f}, a23 = f2{0.f, 0.f};
#pragma unroll
      for (int k = 0; k < H; k += 4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hp + k);
        a01 = pk_fma(w[k / 2], f2{h4.x, h4.y}, a01);
        a23 = pk_fma(w[k / 2 + 1], f2{h4.z, h4.w}, a23);
      }
      const float pre = (a01.x + a01.y) + (a23.x + a23.y);
      const float act = (g == 2) ? tanhf(pre) : sigm(pre);
      const float ig = quad_bcast<0>(act), fg = quad_bcast<1>(act);
      const float gg = quad_bcast<2>(act), og = quad_bcast<3>(act);
      c = fmaf(fg, c, ig * gg);
      const float h = og * tanhf(c);
      const int64_t tt = tix(t);
      if (g == 0) {
        hb[t & 1][u] = h;
        hrow[tt * 2 * H] = h;
        if (crow) crow[tt * 2 * H] = c;
      }
      if (grow) grow[tt * 8 * H] = act;
      lds_barrier();
    }
    if (ch + 1 < nch) store_chunk(buf ^ 1);
    __syncthreads();
  }
}

// Backward through time.  Bwd step u walks the forward steps in reverse:
// forward step t = T-1-u, time index tt(t).  Lane = 4k + q: the quad of
// hidden unit k computes the four gate gradients of unit k (lane q -> gate
// q) and the recurrent matvec dh_rec[k] = sum_g dG[g] W[g][k], lane q summing
// the gate block g in [qH, qH+H) with W[qH+m][k] (m < H) held in VGPRs; the
// four partials are combined with DPP quad broadcasts.
template <int H>
__global__ __launch_bounds__(4 * H, 1) void lstm_bwd_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates,
    const float* __restrict__ cell, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ dgates, int T) {
  constexpr int NT = 4 * H;
  constexpr int G4 = 4 * H;
  constexpr int DGS = H + 4;                        // padded gate-block stride (banks)
  constexpr int PG = LCH * G4 / 4 / NT;             // float4 of gates per thread
  constexpr int PC = ((LCH + 1) * H + NT - 1) / NT; // cell floats per thread
  constexpr int PD = (LCH * H + NT - 1) / NT;       // dh floats per thread
  __shared__ __attribute__((aligned(16))) float gsm[2][LCH][G4];
  __shared__ float csm[2][LCH + 1][H];
  __shared__ float dsm[2][LCH][H];
  __shared__ __attribute__((aligned(16))) float dgb[2][4 * DGS];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, k = tid >> 2, q = tid & 3;
  const float* whh = dir ? whh_r : whh_f;
  f2 wt[H / 2];  // W[q*H + m][k], m pairs
#pragma unroll
  for (int m = 0; m < H; m += 2)
    wt[m / 2] = f2{whh[(int64_t)(q * H + m) * H + k], whh[(int64_t)(q * H + m + 1) * H + k]};

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
      pd[i] = (s < LCH && t >= 0) ? dbase[(int64_t)tix(t) * 2 * H + r] : 0.f;
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
      const int s = idx / H, r = idx % H;
      if (s < LCH) dsm[buf][s][r] = pd[i];
    }
  };

  const int nch = (T + LCH - 1) / LCH;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  float dh_rec = 0.f, dc_next = 0.f;
  float* dgrow = dgates + (int64_t)n * T * 8 * H + dir * G4 + q * H + k;
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load_chunk(ch + 1);
    for (int s = 0; s < LCH; ++s) {
      const int uu = ch * LCH + s;
      if (uu >= T) break;
      const int t = T - 1 - uu;
      const float ig = gsm[buf][s][k], fg = gsm[buf][s][H + k];
      const float gg = gsm[buf][s][2 * H + k], og = gsm[buf][s][3 * H + k];
      const float cc = csm[buf][s][k];
      const float cp = (t > 0) ? csm[buf][s + 1][k] : 0.f;
      const float dh = dsm[buf][s][k] + dh_rec;
      const float tc = tanhf(cc);
      const float dc = fmaf(dh * og, 1.f - tc * tc, dc_next);
      dc_next = dc * fg;
      float da;
      if (q == 0) da = (dc * gg) * ig * (1.f - ig);            // d pre_i
      else if (q == 1) da = (dc * cp) * fg * (1.f - fg);       // d pre_f
      else if (q == 2) da = (dc * ig) * (1.f - gg * gg);       // d pre_g
      else da = (dh * tc) * og * (1.f - og);                   // d pre_o
      const int64_t tt = tix(t);
      float* db = dgb[uu & 1];
      db[q * DGS + k] = da;
      dgrow[tt * 8 * H] = da;
      lds_barrier();
      const float* dq = db + q * DGS;
      f2 ab = f2{0.f, 0.f}, cd = f2{0.f, 0.f};
#pragma unroll
      for (int m = 0; m < H; m += 4) {
        const float4 v = *reinterpret_cast<const float4*>(dq + m);
        ab = pk_fma(wt[m / 2], f2{v.x, v.y}, ab);
        cd = pk_fma(wt[m / 2 + 1], f2{v.z, v.w}, cd);
      }
      const float part = (ab.x + ab.y) + (cd.x + cd.y);
      dh_rec = (quad_bcast<0>(part) + quad_bcast<1>(part)) +
               (quad_bcast<2>(part) + quad_bcast<3>(part));
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
    case 32: hipLaunchKernelGGL(lstm_fwd_kernel<32>, grid, dim3(128), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
    case 64: hipLaunchKernelGGL(lstm_fwd_kernel<64>, grid, dim3(256), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
    case 128: hipLaunchKernelGGL(lstm_fwd_kernel<128>, grid, dim3(512), 0, s, zx, w_hh[0], w_hh[1], h_out, gates, cell, (int)T); break;
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
    case 32: hipLaunchKernelGGL(lstm_bwd_kernel<32>, grid, dim3(128), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
    case 64: hipLaunchKernelGGL(lstm_bwd_kernel<64>, grid, dim3(256), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
    case 128: hipLaunchKernelGGL(lstm_bwd_kernel<128>, grid, dim3(512), 0, s, dh_out, gates, cell, w_hh[0], w_hh[1], dgates, (int)T); break;
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
