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

// Gate nonlinearities on the hardware transcendental units (v_exp_f32,
// v_rcp_f32, ~1 ulp each) instead of libm's expf / IEEE division / tanhf: they
// sit on the serial per-step critical path.  tanh(x) = 2*sigmoid(2x) - 1 is
// within ~1.5e-7 absolute of tanhf (the tolerance of fp32 O(1) values); the
// i,f,g,o quad evaluates ONE sigmoid per lane (g's argument doubled) instead of
// a divergent tanhf/sigmoid pair.
__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
__device__ __forceinline__ float tanh_hw(float x) { return 2.f * sigm(2.f * x) - 1.f; }

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

// Forward recurrence.  4H lanes per (sequence, direction): the lane quad
// 4u..4u+3 owns hidden unit u, and lane q of the quad holds the k-quarter
// [q*H/4, (q+1)*H/4) of all four of its gate rows (i,f,g,o) of W_hh (H VGPRs;
// at H=128 no accumulator-file round trips).  Per step each lane reads only its
// quarter of h_{t-1} (8 broadcast ds_read_b128 at H=128 instead of 32 for a
// whole row: the LDS issue was the step's critical resource), forms four
// partial dot products, and a two-stage DPP reduce-scatter inside the quad
// leaves lane q with the full pre-activation of gate q.  One LDS barrier per
// step.
template <int Q0, int Q1, int Q2, int Q3>
__device__ __forceinline__ float quad_perm(float v) {
  constexpr int ctrl = Q0 | (Q1 << 2) | (Q2 << 4) | (Q3 << 6);
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xF, 0xF, false));
}

// p[g] = lane's partial of gate g; returns the quad total of gate q (fixed
// addition order: pairs (0,1),(2,3) first, then (0,2),(1,3)).
__device__ __forceinline__ float quad_reduce_scatter4(const float (&p)[4], int q) {
  const bool b0 = q & 1, b1 = q >> 1;
  const float s0 = b0 ? p[0] : p[1], s1 = b0 ? p[2] : p[3];
  const float k0 = (b0 ? p[1] : p[0]) + quad_perm<1, 0, 3, 2>(s0);   // gate b0
  const float k1 = (b0 ? p[3] : p[2]) + quad_perm<1, 0, 3, 2>(s1);   // gate b0 + 2
  const float s2 = b1 ? k0 : k1;
  return (b1 ? k1 : k0) + quad_perm<2, 3, 0, 1>(s2);                 // gate q
}

template <int H>
__global__ __launch_bounds__(4 * H, 1) void lstm_fwd_kernel(
    const float* __restrict__ zx, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ h_out,
    float* __restrict__ gates, float* __restrict__ cell, int T) {
  constexpr int NT = 4 * H;         // threads
  constexpr int G4 = 4 * H;         // gate rows
  constexpr int KQ = H / 4;         // k per lane
  constexpr int HP = H + 16;        // padded h: k -> k + 4*(k/KQ) (conflict-free quarters)
  constexpr int PF = LCH * G4 / 4 / NT;  // float4 prefetched per thread (=LCH/4)
  __shared__ __attribute__((aligned(16))) float zs[2][LCH][G4];
  __shared__ __attribute__((aligned(16))) float hb[2][HP];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, u = tid >> 2, q = tid & 3;
  const int row = q * H + u;        // the gate row this lane finishes (gate q of unit u)
  const float* whh = dir ? whh_r : whh_f;

  f2 w[4][KQ / 2];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int k = 0; k < KQ; k += 4) {
      const float4 v = *reinterpret_cast<const float4*>(whh + (int64_t)(g * H + u) * H + q * KQ + k);
      w[g][k / 2] = f2{v.x, v.y};
      w[g][k / 2 + 1] = f2{v.z, v.w};
    }
  if (tid < HP) hb[1][tid] = 0.f;

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
      const float* hp = hb[(t + 1) & 1] + q * (KQ + 4);
      f2 a[4], b[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) a[g] = b[g] = f2{0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KQ; k += 4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hp + k);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          a[g] = pk_fma(w[g][k / 2], f2{h4.x, h4.y}, a[g]);
          b[g] = pk_fma(w[g][k / 2 + 1], f2{h4.z, h4.w}, b[g]);
        }
      }
      float part[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) part[g] = (a[g].x + a[g].y) + (b[g].x + b[g].y);
      const float pre = quad_reduce_scatter4(part, q) + zs[buf][s][row];
      const float sg = sigm(q == 2 ? 2.f * pre : pre);
      const float act = (q == 2) ? 2.f * sg - 1.f : sg;
      const float ig = quad_bcast<0>(act), fg = quad_bcast<1>(act);
      const float gg = quad_bcast<2>(act), og = quad_bcast<3>(act);
      c = fmaf(fg, c, ig * gg);
      const float h = og * tanh_hw(c);
      const int64_t tt = tix(t);
      if (q == 0) {
        hb[t & 1][u + 4 * (u / KQ)] = h;
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
// forward step t = T-1-u, time index tt(t).  Lane = 4k + q computes gate q's
// gradient of hidden unit k (elementwise part).  The recurrent matvec
// dh_rec[k] = sum_r dG[r] W[r][k] (r over the 4H gate rows) uses a different
// split of the same lanes: lane l = 16*kg + rg holds W[rg*H/4 + j][4kg + kk]
// (j < H/4, kk < 4: H VGPRs), reads only its H/4 gradients (8 broadcast
// ds_read_b128 at H=128 instead of 32), and the 16 lanes of the DPP row all-
// reduce their four partials (rotations 8,4,2,1: every lane ends with the
// bitwise-identical sums) -- lane 4k+q is in the row of k = 4kg + rg/4.
template <int R>
__device__ __forceinline__ float row_ror(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + R, 0xF, 0xF, false));
}

template <int H>
__global__ __launch_bounds__(4 * H, 1) void lstm_bwd_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates,
    const float* __restrict__ cell, const float* __restrict__ whh_f,
    const float* __restrict__ whh_r, float* __restrict__ dgates, int T) {
  constexpr int NT = 4 * H;
  constexpr int G4 = 4 * H;
  constexpr int PG = LCH * G4 / 4 / NT;             // float4 of gates per thread
  constexpr int PC = ((LCH + 1) * H + NT - 1) / NT; // cell floats per thread
  constexpr int PD = (LCH * H + NT - 1) / NT;       // dh floats per thread
  __shared__ __attribute__((aligned(16))) float gsm[2][LCH][G4];
  __shared__ float csm[2][LCH + 1][H];
  __shared__ float dsm[2][LCH][H];
  constexpr int RPG = H / 4;                        // gate rows per lane (matvec)
  constexpr int DGP = 4 * H + 64;                   // padded dG: r -> r + 4*(r/RPG)
  __shared__ __attribute__((aligned(16))) float dgb[2][DGP];

  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int tid = threadIdx.x, k = tid >> 2, q = tid & 3;
  const int kg = tid >> 4, rg = tid & 15;           // matvec split
  const float* whh = dir ? whh_r : whh_f;
  f2 wt[4][RPG / 2];  // W[rg*RPG + j][4kg + kk], j pairs
#pragma unroll
  for (int j = 0; j < RPG; j += 2) {
    const float4 v0 = *reinterpret_cast<const float4*>(whh + (int64_t)(rg * RPG + j) * H + 4 * kg);
    const float4 v1 = *reinterpret_cast<const float4*>(whh + (int64_t)(rg * RPG + j + 1) * H + 4 * kg);
    wt[0][j / 2] = f2{v0.x, v1.x};
    wt[1][j / 2] = f2{v0.y, v1.y};
    wt[2][j / 2] = f2{v0.z, v1.z};
    wt[3][j / 2] = f2{v0.w, v1.w};
  }

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
    // Everything of a step that does not depend on dh_rec (the previous
    // step's matvec) is loaded and folded into two coefficients one step
    // ahead, while that matvec runs; the serial chain per step is then
    // dh -> dc -> da -> LDS -> barrier -> matvec -> DPP reduce.
    float ca = 0.f, cq = 0.f, cf = 0.f, dd = 0.f;  // og*(1-tc^2), gate-q factor, fg, dh_out
    auto prep = [&](int s, int t) {
      const float ig = gsm[buf][s][k], fg = gsm[buf][s][H + k];
      const float gg = gsm[buf][s][2 * H + k], og = gsm[buf][s][3 * H + k];
      const float tc = tanh_hw(csm[buf][s][k]);
      const float cp = (t > 0) ? csm[buf][s + 1][k] : 0.f;
      ca = og * (1.f - tc * tc);
      cf = fg;
      dd = dsm[buf][s][k];
      if (q == 0) cq = gg * (ig * (1.f - ig));            // d pre_i = dc * cq
      else if (q == 1) cq = cp * (fg * (1.f - fg));       // d pre_f = dc * cq
      else if (q == 2) cq = ig * (1.f - gg * gg);         // d pre_g = dc * cq
      else cq = tc * (og * (1.f - og));                   // d pre_o = dh * cq
    };
    if (ch * LCH < T) prep(0, T - 1 - ch * LCH);
    for (int s = 0; s < LCH; ++s) {
      const int uu = ch * LCH + s;
      if (uu >= T) break;
      const int t = T - 1 - uu;
      const float dh = dd + dh_rec;
      const float dc = fmaf(dh, ca, dc_next);
      dc_next = dc * cf;
      const float da = (q == 3 ? dh : dc) * cq;
      const int64_t tt = tix(t);
      float* db = dgb[uu & 1];
      {
        const int r = q * H + k;
        db[r + 4 * (r / RPG)] = da;
      }
      dgrow[tt * 8 * H] = da;
      lds_barrier();
      if (s + 1 < LCH && uu + 1 < T) prep(s + 1, t - 1);
      const float* dq = db + rg * (RPG + 4);
      f2 a[4], b[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) a[kk] = b[kk] = f2{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < RPG; j += 4) {
        const float4 v = *reinterpret_cast<const float4*>(dq + j);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          a[kk] = pk_fma(wt[kk][j / 2], f2{v.x, v.y}, a[kk]);
          b[kk] = pk_fma(wt[kk][j / 2 + 1], f2{v.z, v.w}, b[kk]);
        }
      }
      float part[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        float v = (a[kk].x + a[kk].y) + (b[kk].x + b[kk].y);
        v += row_ror<8>(v);
        v += row_ror<4>(v);
        v += row_ror<2>(v);
        v += row_ror<1>(v);
        part[kk] = v;
      }
      const int sel = rg >> 2;                      // k = 4kg + sel
      dh_rec = sel == 0 ? part[0] : (sel == 1 ? part[1] : (sel == 2 ? part[2] : part[3]));
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
