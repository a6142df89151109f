// stft.hip — fused STFT + spectrogram features + gap mask.
//
// One wave owns one (example, frame) item at a time.  The frame's clean and
// gapped windowed samples are packed as two half-length complex sequences
// z[m] = x[2m] + i x[2m+1] (real-FFT-via-half-size-complex-FFT), transformed
// with a radix-2 Stockham FFT in float64 in the wave's LDS slice, then
// unpacked to the n_fft/2+1 real-FFT bins.  Everything stays float64 until the
// single rounding to the output type: the reference's gapped CNNBLSTM STFT is
// complex128 (utils.py:180-183 promotes to float64) and its clean
// STFT is computed by numpy in float64 before being stored as complex64.
//
// Frame semantics follow librosa>=0.10 stft(center=True, pad_mode='constant')
// as called by utils.extract_spectrogram (utils.py:225-232): frame t covers
// padded samples [t*hop, t*hop+n_fft) of the signal zero-padded by n_fft/2 on
// both sides; X[f,t] = sum_n w[n] x_pad[t*hop+n] e^{-2 pi i f n / n_fft}.
#include "common.h"

#include <stdlib.h>

namespace ainp {

struct cd {
  double re, im;
};
__device__ __forceinline__ cd cmul(cd a, cd b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// Mask frame range, CNNBLSTM rule (models/CNNBLSTM/dataset.py:116-119):
// librosa.time_to_frames(start_sample/sr) = int((s/sr)*sr)//hop, in IEEE double.
__device__ __forceinline__ int64_t time_to_frame(int64_t sample, int64_t sr,
                                                 int hop) {
  double secs = (double)sample / (double)sr;  // utils.py:186
  double samp = secs * (double)sr;            // librosa time_to_samples
  return ((int64_t)samp) / hop;               // astype(int) then // hop
}

template <int MODE>
__global__ __launch_bounds__(256) void stft_features_kernel(
    const float* __restrict__ audio, int64_t n_samples,
    const int32_t* __restrict__ clip_index,
    const int64_t* __restrict__ gap_start, int64_t batch, int64_t gap_len,
    int64_t sample_rate, const double* __restrict__ window, int n_fft,
    int log2m, int hop, int64_t n_frames, float* __restrict__ out0,
    float* __restrict__ out1, float* __restrict__ out2,
    float* __restrict__ out3) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = n_fft >> 1;        // complex FFT length
  const int F = M + 1;             // real-FFT bins
  // LDS carve: twiddles tw[q] = exp(-2 pi i q / n_fft), q in [0, M]
  cd* tw = reinterpret_cast<cd*>(smem);
  double* win = reinterpret_cast<double*>(tw + (M + 1));
  // per-wave work buffers: 2 signals x 2 ping-pong x M complex
  cd* wbase = reinterpret_cast<cd*>(win + n_fft);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  cd* bufA = wbase + (size_t)wave * 4 * M;  // [2][M]
  cd* bufB = bufA + 2 * M;                  // [2][M]

  for (int q = threadIdx.x; q <= M; q += blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)q / (double)n_fft, &s, &c);
    tw[q] = {c, s};
  }
  for (int n = threadIdx.x; n < n_fft; n += blockDim.x) win[n] = window[n];
  __syncthreads();

  const int64_t n_avail = 1 + n_samples / hop;  // frames librosa produces
  const int64_t total = batch * n_frames;
  const int nw = blockDim.x >> 6;
  for (int64_t base = (int64_t)blockIdx.x * nw; base < total;
       base += (int64_t)gridDim.x * nw) {
    const int64_t item = base + wave;
    const bool valid = item < total;
    const int64_t b = valid ? item / n_frames : 0;
    const int64_t t = valid ? item % n_frames : 0;
    const int64_t clip = clip_index ? (int64_t)clip_index[b] : b;
    const float* x = audio + clip * n_samples;
    const int64_t gs = gap_start[b];
    const int64_t ge = gs + gap_len;
    const int64_t s0 = t * hop - (n_fft >> 1);
    const bool in_range = valid && t < n_avail;

    // 1. windowed load, packed as z[m] = x[2m] + i x[2m+1]
    for (int m = lane; m < M; m += 64) {
      double xc[2], xg[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int n = 2 * m + e;
        const int64_t s = s0 + n;
        double v = 0.0;
        if (in_range && s >= 0 && s < n_samples) v = (double)x[s];
        const double vg = (s >= gs && s < ge) ? 0.0 : v;
        xc[e] = v * win[n];
        xg[e] = vg * win[n];
      }
      bufA[m] = {xc[0], xc[1]};
      bufA[M + m] = {xg[0], xg[1]};
    }
    __syncthreads();

    // 2. radix-2 Stockham FFT of length M on both signals (natural order out)
    cd* src = bufA;
    cd* dst = bufB;
    for (int st = 0; st < log2m; ++st) {
      const int Ns = 1 << st;
      for (int j = lane; j < (M >> 1); j += 64) {
        const int k = j & (Ns - 1);
        const cd w = tw[(k << (log2m - st))];  // exp(-2 pi i k / (2 Ns))
        const int o = (j << 1) - k;
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const cd a = src[sg * M + j];
          const cd bb = cmul(w, src[sg * M + j + (M >> 1)]);
          dst[sg * M + o] = {a.re + bb.re, a.im + bb.im};
          dst[sg * M + o + Ns] = {a.re - bb.re, a.im - bb.im};
        }
      }
      __syncthreads();
      cd* tmp = src;
      src = dst;
      dst = tmp;
    }

    // 3. unpack the real FFTs: X[k] = Ze + W^k Zo, k = 0..M
    if (valid) {
      const size_t obase = (size_t)b * F * n_frames + t;
      float maskv;
      if (MODE == AINP_FEAT_CNNBLSTM) {
        const int64_t fs = time_to_frame(gs, sample_rate, hop);
        const int64_t fe = time_to_frame(ge, sample_rate, hop);
        maskv = (t >= fs && t < fe) ? 1.f : 0.f;
      } else {
        int64_t fs = gs / hop;
        int64_t fe = (ge + hop - 1) / hop;  // ceil(end/hop)
        if (fs < 0) fs = 0;
        if (fe > n_avail) fe = n_avail;
        maskv = (fe > fs && t >= fs && t < fe) ? 0.f : 1.f;
      }
      for (int k = lane; k < F; k += 64) {
        cd X[2];
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const cd zk = src[sg * M + (k & (M - 1))];
          const cd zm = src[sg * M + ((M - k) & (M - 1))];
          // Ze = (zk + conj(zm))/2, Zo = (zk - conj(zm))/(2i)
          const cd ze = {0.5 * (zk.re + zm.re), 0.5 * (zk.im - zm.im)};
          const cd zo = {0.5 * (zk.im + zm.im), -0.5 * (zk.re - zm.re)};
          const cd r = cmul(tw[k], zo);
          X[sg] = {ze.re + r.re, ze.im + r.im};
        }
        const size_t o = obase + (size_t)k * n_frames;
        if (MODE == AINP_FEAT_CNNBLSTM) {
          if (out0) out0[o] = in_range ? (float)log10(hypot(X[1].re, X[1].im) + 1e-9) : 0.f;
          if (out1) {
            float2 v = in_range ? make_float2((float)X[0].re, (float)X[0].im)
                                : make_float2(0.f, 0.f);
            reinterpret_cast<float2*>(out1)[o] = v;
          }
          if (out2) out2[o] = maskv;
        } else {
          // complex64 rounding first, then |.|, log1p, angle (dataset.py:121-135)
          const float cr = (float)X[0].re, ci = (float)X[0].im;
          const float ir = (float)X[1].re, ii = (float)X[1].im;
          const float mc = (float)hypot((double)cr, (double)ci);
          const float mi = (float)hypot((double)ir, (double)ii);
          if (out0) out0[o] = (float)log1p((double)mc);
          if (out1) out1[o] = (float)log1p((double)mi);
          if (out2) out2[o] = (float)atan2((double)ci, (double)cr);
          if (out3) out3[o] = maskv;
        }
      }
    }
    __syncthreads();  // buffers are reused by the next item
  }
}

// ---------------------------------------------------------------------------
// n_fft = 512 fast path (every configuration of BASELINE.json): tiles of 16
// consecutive frames of one example per workgroup, outputs staged in LDS and
// written as contiguous runs along t (the [B][F][T] layout), so every store is
// a coalesced 64-B (f32) / 128-B (complex64) row segment instead of one
// 4-byte scatter per bin.
//
// FFT: the 512-point real FFT is a 256-point complex FFT of
// z[m] = x[2m] + i x[2m+1], computed four-step as 16 x 16 in float64:
// 16 lanes per FFT, lane j holds z[16 n1 + j] (n1 = 0..15; a coalesced 128-B
// load per n1), a 16-point DFT in registers (radix 4 x 4), the twiddle
// W256^{j k1} (per-lane registers, read once from an LDS table), a dword-wise
// 16 x 16 transpose through the wave's own LDS slice (no block barrier), and a
// second in-register 16-point DFT.  Lane j then holds Z[j + 16 k2]; the
// real-FFT unpack takes Z[256 - k] from lane 16 - j by ds_bpermute.
//
// Work: one clean FFT per frame; a gapped FFT only for frames whose window
// [t*hop - 256, t*hop + 256) intersects the gap -- elsewhere the gapped and
// clean signals are the same float64 values, so the clean FFT is bit-identical
// to the gapped one and feeds the log-magnitude directly.
namespace f512 {
constexpr int M = 256, F = 257, TF = 16, NW = 4, NT = 64 * NW;
constexpr int XROW = 17;                 // transpose row stride (dwords)
constexpr int XSLOT = 16 * XROW;         // per-FFT transpose buffer (dwords)
constexpr int PROW = 17;                 // staging row stride (floats) per bin
constexpr int PLANE = F * PROW;          // floats per staged output plane
constexpr size_t LDS_WIN = 512 * sizeof(double);
constexpr size_t LDS_XCH = (size_t)NW * 4 * XSLOT * sizeof(uint32_t);
constexpr size_t LDS_STAGE = (size_t)3 * PLANE * sizeof(float);
constexpr size_t LDS_TW = (size_t)M * 2 * sizeof(double);
constexpr size_t LDS_BYTES = LDS_WIN + LDS_TW + LDS_XCH + LDS_STAGE;
static_assert(LDS_BYTES * 2 <= 160 * 1024, "two workgroups per CU");

constexpr double C1 = 0.9807852804032304, S1 = 0.19509032201612825;  // cos/sin(pi/16)
constexpr double C2 = 0.9238795325112867, S2 = 0.3826834323650898;   // cos/sin(pi/8)
constexpr double C3 = 0.8314696123025452, S3 = 0.5555702330196022;   // cos/sin(3pi/16)
constexpr double RH = 0.7071067811865476;                            // sqrt(1/2)
// W32^k = exp(-2 pi i k / 32), k = 0..15
__device__ constexpr double W32R[16] = {1.0, C1, C2, C3, RH, S3, S2, S1,
                                        0.0, -S1, -S2, -S3, -RH, -C3, -C2, -C1};
__device__ constexpr double W32I[16] = {0.0, -S1, -S2, -S3, -RH, -C3, -C2, -C1,
                                        -1.0, -C1, -C2, -C3, -RH, -S3, -S2, -S1};

__device__ __forceinline__ void dft4(double& ar, double& ai, double& br, double& bi,
                                     double& cr, double& ci, double& dr, double& di) {
  const double t0r = ar + cr, t0i = ai + ci, t1r = ar - cr, t1i = ai - ci;
  const double t2r = br + dr, t2i = bi + di, t3r = br - dr, t3i = bi - di;
  ar = t0r + t2r; ai = t0i + t2i;     // X0
  cr = t0r - t2r; ci = t0i - t2i;     // X2
  br = t1r + t3i; bi = t1i - t3r;     // X1 = (x0-x2) - i(x1-x3)
  dr = t1r - t3i; di = t1i + t3r;     // X3 = (x0-x2) + i(x1-x3)
}

__device__ __forceinline__ void cmul_c(double& r, double& i, double wr, double wi) {
  const double t = r * wr - i * wi;
  i = r * wi + i * wr;
  r = t;
}

// In-register 16-point forward DFT of v[n] (n = 4 n1 + n2).  Output X[k] is
// left at position pos(k) = 4 (k & 3) + (k >> 2).
__device__ __forceinline__ void dft16(double (&re)[16], double (&im)[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2)
    dft4(re[n2], im[n2], re[4 + n2], im[4 + n2], re[8 + n2], im[8 + n2], re[12 + n2],
         im[12 + n2]);
  // Y[k1][n2] sits at 4 k1 + n2; twiddle W16^{n2 k1}
  cmul_c(re[5], im[5], C2, -S2);     // k1=1,n2=1: W16^1
  cmul_c(re[6], im[6], RH, -RH);     // k1=1,n2=2: W16^2
  cmul_c(re[7], im[7], S2, -C2);     // k1=1,n2=3: W16^3
  cmul_c(re[9], im[9], RH, -RH);     // k1=2,n2=1: W16^2
  { const double t = re[10]; re[10] = im[10]; im[10] = -t; }   // W16^4 = -i
  cmul_c(re[11], im[11], -RH, -RH);  // k1=2,n2=3: W16^6
  cmul_c(re[13], im[13], S2, -C2);   // k1=3,n2=1: W16^3
  cmul_c(re[14], im[14], -RH, -RH);  // k1=3,n2=2: W16^6
  cmul_c(re[15], im[15], -C2, S2);   // k1=3,n2=3: W16^9
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1)
    dft4(re[4 * k1], im[4 * k1], re[4 * k1 + 1], im[4 * k1 + 1], re[4 * k1 + 2],
         im[4 * k1 + 2], re[4 * k1 + 3], im[4 * k1 + 3]);
}
__device__ __forceinline__ constexpr int pos(int k) { return 4 * (k & 3) + (k >> 2); }

__device__ __forceinline__ uint32_t dw(double v, int hi) {
  const uint64_t u = __double_as_longlong(v);
  return hi ? (uint32_t)(u >> 32) : (uint32_t)u;
}
__device__ __forceinline__ double set_dw(double v, int hi, uint32_t x) {
  uint64_t u = __double_as_longlong(v);
  u = hi ? ((u & 0xffffffffull) | ((uint64_t)x << 32)) : ((u & ~0xffffffffull) | x);
  return __longlong_as_double(u);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// blockIdx -> tile so that consecutive tiles of one example share an XCD
// (workgroups are dealt round-robin over the 8 XCDs); bijective on [0, n).
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t n) {
  const int64_t per = n / 8, rem = n % 8, x = b % 8, i = b / 8;
  return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// Per-tile scalars (uniform over the workgroup).
struct Tile {
  int b, t0, ncomp, nvalid, ga, gb, njobs;
  int64_t gs64, ge64;
  const float* x;
};

template <int MODE>
__device__ __forceinline__ Tile make_tile(int v, int ntiles, int ntt, int NF, int ns, int hop,
                                          const float* audio, int64_t n_samples,
                                          const int32_t* clip_index, const int64_t* gap_start,
                                          int64_t gap_len, bool want_lm, bool want_fft) {
  Tile T;
  const int tile = (int)xcd_tile(v, ntiles);
  T.b = tile / ntt;
  T.t0 = (tile - T.b * ntt) * TF;
  const int64_t clip = clip_index ? (int64_t)clip_index[T.b] : T.b;
  T.x = audio + clip * n_samples;
  T.gs64 = gap_start[T.b];
  T.ge64 = T.gs64 + gap_len;
  const int n_avail = 1 + ns / hop;
  T.nvalid = min(TF, NF - T.t0);
  T.ncomp = max(0, min(T.nvalid, n_avail - T.t0));
  // tile columns [ga, gb) whose window [t*hop - 256, t*hop + 256) meets the gap
  T.ga = 0;
  T.gb = 0;
  if (want_lm && gap_len > 0 && T.ncomp > 0) {
    const int64_t lo = T.gs64 - 256;  // t*hop > lo  <=>  t >= floor(lo/hop) + 1
    const int64_t tlo = (lo >= 0 ? lo / hop : -((-lo + hop - 1) / hop)) + 1;
    const int64_t thi = (T.ge64 + 256 + hop - 1) / hop;  // first t: t*hop - 256 >= ge
    T.ga = (int)max((int64_t)0, min((int64_t)T.ncomp, tlo - T.t0));
    T.gb = (int)max((int64_t)T.ga, min((int64_t)T.ncomp, thi - T.t0));
  }
  T.njobs = want_fft ? T.ncomp + (T.gb - T.ga) : 0;
  return T;
}

// Job q of a tile: columns 0..ncomp-1 clean, then ga..gb-1 gapped.  Lane j of
// the job's 16-lane group loads x[s0 + 32 n1 + {0,1}], s0 = t*hop - 256 + 2j;
// samples outside the signal, and gap samples of gapped jobs, read as 0 (an
// exact zero, as the reference's multiply / concatenate gives).
template <bool VEC2>
__device__ __forceinline__ void load_raw(const Tile& T, int q, int j, int ns, int hop,
                                         int64_t gap_len, float (&raw0)[16],
                                         float (&raw1)[16]) {
  q = min(q, max(T.njobs - 1, 0));
  const int c = q < T.ncomp ? q : T.ga + (q - T.ncomp);
  const int s0 = (T.t0 + c) * hop - 256 + 2 * j;
  const int gs = (int)max((int64_t)-(1 << 30), min((int64_t)1 << 30, T.gs64));
  const int gl = q >= T.ncomp ? (int)gap_len : 0;
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const int s = s0 + 32 * n1;
    const bool in0 = (unsigned)s < (unsigned)ns && (unsigned)(s - gs) >= (unsigned)gl;
    const bool in1 = (unsigned)(s + 1) < (unsigned)ns && (unsigned)(s + 1 - gs) >= (unsigned)gl;
    if (VEC2) {
      const float2 p = *reinterpret_cast<const float2*>(T.x + min(max(s, 0), ns - 2));
      raw0[n1] = in0 ? p.x : 0.f;
      raw1[n1] = in1 ? p.y : 0.f;
    } else {
      const float p0 = T.x[min(max(s, 0), ns - 1)];
      const float p1 = T.x[min(max(s + 1, 0), ns - 1)];
      raw0[n1] = in0 ? p0 : 0.f;
      raw1[n1] = in1 ? p1 : 0.f;
    }
  }
}

// Persistent: each workgroup walks tiles v = blockIdx.x, + gridDim.x, ...;
// the next tile's samples are loaded while the current tile is written out.
template <int MODE, bool VEC2>
__global__ __launch_bounds__(NT, 2) void stft512_kernel(
    const float* __restrict__ audio, int64_t n_samples,
    const int32_t* __restrict__ clip_index, const int64_t* __restrict__ gap_start,
    int64_t batch, int64_t gap_len, int64_t sample_rate,
    const double* __restrict__ window, int hop, int64_t n_frames, int64_t n_tiles_t,
    float* __restrict__ out0, float* __restrict__ out1, float* __restrict__ out2,
    float* __restrict__ out3) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* win = reinterpret_cast<double*>(smem);
  double2* tw256 = reinterpret_cast<double2*>(smem + LDS_WIN);  // W256^q
  uint32_t* xch = reinterpret_cast<uint32_t*>(smem + LDS_WIN + LDS_TW);
  float* stage = reinterpret_cast<float*>(smem + LDS_WIN + LDS_TW + LDS_XCH);
  float* P0 = stage;
  float* P1 = stage + PLANE;
  float* P2 = stage + 2 * PLANE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = lane >> 4, j = lane & 15;
  // the launcher guarantees n_samples, n_frames * hop and gap_len < 2^30
  const int ntt = (int)n_tiles_t, NF = (int)n_frames, ns = (int)n_samples;
  const int ntiles = (int)(batch * n_tiles_t);
  const bool want_lm = MODE == AINP_FEAT_CNNBLSTM ? out0 != nullptr : out1 != nullptr;
  const bool want_fft = MODE == AINP_FEAT_CNNBLSTM ? (out0 || out1) : (out0 || out1 || out2);
  float* mask_out = MODE == AINP_FEAT_CNNBLSTM ? out2 : out3;
  const int n_avail = 1 + ns / hop;
  const int myjob = wave * 4 + slot;

  int v = blockIdx.x;
  Tile T = make_tile<MODE>(v, ntiles, ntt, NF, ns, hop, audio, n_samples, clip_index,
                           gap_start, gap_len, want_lm, want_fft);
  float raw0[16], raw1[16];
  load_raw<VEC2>(T, myjob, j, ns, hop, gap_len, raw0, raw1);

  // window / 2 (the unpack's 1/2 factors, exact) and W256^q into LDS, once
  for (int n = tid; n < 512; n += NT) win[n] = 0.5 * window[n];
  {
    double s, c;
    sincospi(-(double)tid / 128.0, &s, &c);
    tw256[tid] = make_double2(c, s);
  }
  double ujr, uji;  // W512^j
  sincospi(-(double)j / 256.0, &uji, &ujr);
  uint32_t* xs = xch + myjob * XSLOT;

  while (true) {
    if (T.ncomp < TF) {  // frames past the end of the signal (t >= 1 + S//hop) are zero
      for (int i = tid; i < F * TF; i += NT) {
        const int c = i % TF, f = i / TF;
        if (c >= T.ncomp) {
          P0[f * PROW + c] = 0.f;
          P1[f * PROW + c] = 0.f;
          P2[f * PROW + c] = 0.f;
        }
      }
    }
    __syncthreads();  // tables ready / previous tile written out

    for (int q0 = 0; q0 < T.njobs; q0 += 4 * NW) {
      const int q = q0 + myjob;
      const bool active = q < T.njobs;
      const bool gapped = q >= T.ncomp;
      if (q0 > 0) load_raw<VEC2>(T, q, j, ns, hop, gap_len, raw0, raw1);
      const int c = active ? (gapped ? T.ga + (q - T.ncomp) : q) : 0;
      double re[16], im[16];
      // 1. window: z[16 n1 + j] = w x[32 n1 + 2j] + i w x[32 n1 + 2j + 1]
#pragma unroll
      for (int n1 = 0; n1 < 16; ++n1) {
        const double2 w = *reinterpret_cast<const double2*>(win + 32 * n1 + 2 * j);
        re[n1] = (double)raw0[n1] * w.x;
        im[n1] = (double)raw1[n1] * w.y;
      }
      // 2. DFT over n1, twiddle W256^{j k1}
      dft16(re, im);
      double br[16], bi[16];
#pragma unroll
      for (int k1 = 0; k1 < 16; ++k1) {
        br[k1] = re[pos(k1)];
        bi[k1] = im[pos(k1)];
        if (k1) {
          const double2 w = tw256[(j * k1) & 255];
          cmul_c(br[k1], bi[k1], w.x, w.y);
        }
      }
      // 3. transpose Y[k1][n2=j] -> lane j gets Y[k1=j][n2], one dword plane at a time
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hi = r & 1;
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) xs[k1 * XROW + j] = dw(r < 2 ? br[k1] : bi[k1], hi);
        wave_sync();
#pragma unroll
        for (int n2 = 0; n2 < 16; ++n2) {
          const uint32_t u = xs[j * XROW + n2];
          if (r < 2) re[n2] = set_dw(re[n2], hi, u);
          else im[n2] = set_dw(im[n2], hi, u);
        }
        wave_sync();
      }
      // 4. DFT over n2: lane j now holds Z[j + 16 k2] at pos(k2)
      dft16(re, im);
      // 5. real-FFT unpack; partner Z[(256 - k) & 255] lives in lane (16 - j) & 15.
      // Stores are unconditional: a lane whose value is not wanted writes the
      // padding column TF of its row.
      const bool in_gap = c >= T.ga && c < T.gb;
      const int c_clean = active && !gapped ? c : TF;           // target / orig / phase
      const int c_lm = active && (gapped || !in_gap) ? c : TF;   // log-magnitude of X_gap
      const int c_lm2 = MODE == AINP_FEAT_GAN && active && !gapped && !in_gap ? c : TF;
      const int src = (lane & ~15) | ((16 - j) & 15);
#pragma unroll
      for (int k2 = 0; k2 < 16; ++k2) {
        const double zr = re[pos(k2)], zi = im[pos(k2)];
        const double sr = __shfl(re[pos(15 - k2)], src, 64);
        const double si = __shfl(im[pos(15 - k2)], src, 64);
        const double pr = j == 0 ? re[pos((16 - k2) & 15)] : sr;
        const double pi = j == 0 ? im[pos((16 - k2) & 15)] : si;
        // Z carries a factor 1/2 (window): Ze = Z + conj(Zp), Zo = -i (Z - conj(Zp))
        const double er = zr + pr, ei = zi - pi;
        double orr = zi + pi, oi = pr - zr;
        double wr = ujr, wi = uji;  // W512^{j + 16 k2} = W512^j * W32^{k2}
        cmul_c(wr, wi, W32R[k2], W32I[k2]);
        cmul_c(orr, oi, wr, wi);
        const double Xr = er + orr, Xi = ei + oi;
        const int row = (j + 16 * k2) * PROW;
        if (MODE == AINP_FEAT_CNNBLSTM) {
          P1[row + c_clean] = (float)Xr;
          P2[row + c_clean] = (float)Xi;
          P0[row + c_lm] = __log10f(__builtin_amdgcn_sqrtf((float)(Xr * Xr + Xi * Xi)) + 1e-9f);
        } else {
          const float cr = (float)Xr, ci = (float)Xi;
          const float lm = log1pf(hypotf(cr, ci));
          P0[row + c_clean] = lm;
          P2[row + c_clean] = atan2f(ci, cr);
          P1[row + (gapped ? c_lm : c_lm2)] = lm;
        }
      }
      // Nyquist bin 256 = Re Z0 - Im Z0 (lane j = 0)
      if (j == 0) {
        const double Xr = 2.0 * (re[0] - im[0]);
        const int row = 256 * PROW;
        if (MODE == AINP_FEAT_CNNBLSTM) {
          P1[row + c_clean] = (float)Xr;
          P2[row + c_clean] = 0.f;
          P0[row + c_lm] = __log10f(fabsf((float)Xr) + 1e-9f);
        } else {
          const float cr = (float)Xr;
          const float lm = log1pf(fabsf(cr));
          P0[row + c_clean] = lm;
          P2[row + c_clean] = atan2f(0.f, cr);
          P1[row + (gapped ? c_lm : c_lm2)] = lm;
        }
      }
    }

    // next tile: its first-pass samples load while this tile is written out
    const Tile cur = T;
    v += gridDim.x;
    const bool more = v < ntiles;
    if (more) {
      T = make_tile<MODE>(v, ntiles, ntt, NF, ns, hop, audio, n_samples, clip_index,
                          gap_start, gap_len, want_lm, want_fft);
      load_raw<VEC2>(T, myjob, j, ns, hop, gap_len, raw0, raw1);
    }
    __syncthreads();

    // coalesced write-out: thread (row, col) -> rows of TF consecutive frames
    const int col = tid % TF, row0 = tid / TF;
    if (col < cur.nvalid) {
      const int t = cur.t0 + col;
      float maskv;
      if (MODE == AINP_FEAT_CNNBLSTM) {
        const int64_t fs = time_to_frame(cur.gs64, sample_rate, hop);
        const int64_t fe = time_to_frame(cur.ge64, sample_rate, hop);
        maskv = (t >= fs && t < fe) ? 1.f : 0.f;
      } else {
        int64_t fs = cur.gs64 / hop;
        int64_t fe = (cur.ge64 + hop - 1) / hop;
        if (fs < 0) fs = 0;
        if (fe > n_avail) fe = n_avail;
        maskv = (fe > fs && t >= fs && t < fe) ? 0.f : 1.f;
      }
      const size_t base = (size_t)cur.b * F * n_frames + t;
      for (int f = row0; f < F; f += NT / TF) {
        const size_t o = base + (size_t)f * n_frames;
        const int l = f * PROW + col;
        if (MODE == AINP_FEAT_CNNBLSTM) {
          if (out0) out0[o] = P0[l];
          if (out1) reinterpret_cast<float2*>(out1)[o] = make_float2(P1[l], P2[l]);
        } else {
          if (out0) out0[o] = P0[l];
          if (out1) out1[o] = P1[l];
          if (out2) out2[o] = P2[l];
        }
        if (mask_out) mask_out[o] = maskv;
      }
    }
    if (!more) break;
    __syncthreads();  // staging is rewritten by the next tile
  }
}
}  // namespace f512

// Plain STFT (utils.extract_spectrogram / librosa.stft): one wave per
// (signal, frame); real input of type Tin, output complex<Tin> [F][T] per
// signal (real-FFT via one half-length complex FFT).  center: frames start at t*hop -
// n_fft/2 with zero padding (librosa>=0.10 'constant'), else at t*hop.
template <typename Tin>
__global__ __launch_bounds__(256) void stft_plain_kernel(
    const Tin* __restrict__ audio, int64_t n_samples, int64_t n_sig,
    const double* __restrict__ window, int n_fft, int log2m, int hop,
    int center, int64_t n_frames, Tin* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = n_fft >> 1;
  const int F = M + 1;
  cd* tw = reinterpret_cast<cd*>(smem);
  double* win = reinterpret_cast<double*>(tw + (M + 1));
  cd* wbase = reinterpret_cast<cd*>(win + n_fft);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  cd* bufA = wbase + (size_t)wave * 2 * M;
  cd* bufB = bufA + M;
  for (int q = threadIdx.x; q <= M; q += blockDim.x) {
    double sn, cs;
    sincospi(-2.0 * (double)q / (double)n_fft, &sn, &cs);
    tw[q] = {cs, sn};
  }
  for (int n = threadIdx.x; n < n_fft; n += blockDim.x) win[n] = window[n];
  __syncthreads();
  const int64_t total = n_sig * n_frames;
  const int nw = blockDim.x >> 6;
  for (int64_t base = (int64_t)blockIdx.x * nw; base < total;
       base += (int64_t)gridDim.x * nw) {
    const int64_t item = base + wave;
    const bool valid = item < total;
    const int64_t b = valid ? item / n_frames : 0;
    const int64_t t = valid ? item % n_frames : 0;
    const Tin* x = audio + b * n_samples;
    const int64_t s0 = t * hop - (center ? (n_fft >> 1) : 0);
    for (int m = lane; m < M; m += 64) {
      double v[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int n = 2 * m + e;
        const int64_t sidx = s0 + n;
        const double a = (valid && sidx >= 0 && sidx < n_samples) ? (double)x[sidx] : 0.0;
        v[e] = a * win[n];
      }
      bufA[m] = {v[0], v[1]};
    }
    __syncthreads();
    cd* src = bufA;
    cd* dst = bufB;
    for (int st = 0; st < log2m; ++st) {
      const int Ns = 1 << st;
      for (int j = lane; j < (M >> 1); j += 64) {
        const int k = j & (Ns - 1);
        const cd w = tw[(k << (log2m - st))];
        const int o = (j << 1) - k;
        const cd aa = src[j];
        const cd bb = cmul(w, src[j + (M >> 1)]);
        dst[o] = {aa.re + bb.re, aa.im + bb.im};
        dst[o + Ns] = {aa.re - bb.re, aa.im - bb.im};
      }
      __syncthreads();
      cd* tmp = src;
      src = dst;
      dst = tmp;
    }
    if (valid) {
      Tin* o = out + (b * F * n_frames + t) * 2;
      for (int k = lane; k < F; k += 64) {
        const cd zk = src[k & (M - 1)];
        const cd zm = src[(M - k) & (M - 1)];
        const cd ze = {0.5 * (zk.re + zm.re), 0.5 * (zk.im - zm.im)};
        const cd zo = {0.5 * (zk.im + zm.im), -0.5 * (zk.re - zm.re)};
        const cd r = cmul(tw[k], zo);
        o[(size_t)k * n_frames * 2] = (Tin)(ze.re + r.re);
        o[(size_t)k * n_frames * 2 + 1] = (Tin)(ze.im + r.im);
      }
    }
    __syncthreads();
  }
}

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_stft_features(const float* audio, int64_t n_clips,
                                  int64_t n_samples, const int32_t* clip_index,
                                  const int64_t* gap_start, int64_t batch,
                                  int64_t gap_len, int64_t sample_rate,
                                  const double* window, int n_fft, int hop,
                                  int64_t n_frames, int mode, float* out0,
                                  float* out1, float* out2, float* out3,
                                  void* stream) {
  if (!audio || !gap_start || !window || batch < 0 || n_clips <= 0 ||
      n_samples <= 0 || hop <= 0 || n_frames < 0 || sample_rate <= 0)
    return record_msg("ainp_stft_features: bad argument");
  if (n_fft < 16 || n_fft > 2048 || (n_fft & (n_fft - 1)))
    return record_msg("ainp_stft_features: n_fft must be a power of two in [16,2048]");
  if (mode != AINP_FEAT_CNNBLSTM && mode != AINP_FEAT_GAN)
    return record_msg("ainp_stft_features: bad mode");
  if (batch == 0 || n_frames == 0) return AINP_OK;
  hipStream_t s = as_stream(stream);
  const char* gen = getenv("AINP_STFT_GENERIC");  // 1: force the generic kernel (tests)
  if (n_fft == 512 && !(gen && gen[0] == '1')) {
    if (n_samples >= (1 << 30) || n_frames * hop >= (1 << 30) || gap_len >= (1 << 30))
      return record_msg("ainp_stft_features: signal too long for the n_fft=512 kernel");
    const int64_t ntt = cdiv(n_frames, f512::TF);
    const int64_t ntiles = batch * ntt;
    if (ntiles > 0x7fffffff) return record_msg("ainp_stft_features: too many frames");
    // persistent: at most two workgroups per CU (LDS-limited); pstride env for tuning
    int64_t grid = ntiles;
    const char* ps = getenv("AINP_STFT_GRID");
    if (ps && atoi(ps) > 0) grid = min(grid, (int64_t)atoi(ps));
    const bool vec2 = (hop % 2 == 0) && (n_samples % 2 == 0) &&
                      ((reinterpret_cast<uintptr_t>(audio) & 7) == 0);
#define AINP_F512(MODE, V)                                                              \
  hipLaunchKernelGGL((f512::stft512_kernel<MODE, V>), dim3(grid), dim3(f512::NT),       \
                     f512::LDS_BYTES, s, audio, n_samples, clip_index, gap_start, batch, \
                     gap_len, sample_rate, window, hop, n_frames, ntt, out0, out1, out2, \
                     out3)
    if (mode == AINP_FEAT_CNNBLSTM) {
      if (vec2) AINP_F512(AINP_FEAT_CNNBLSTM, true);
      else AINP_F512(AINP_FEAT_CNNBLSTM, false);
    } else {
      if (vec2) AINP_F512(AINP_FEAT_GAN, true);
      else AINP_F512(AINP_FEAT_GAN, false);
    }
#undef AINP_F512
    return check_launch("ainp_stft_features");
  }
  const int M = n_fft / 2;
  int log2m = 0;
  while ((1 << log2m) < M) ++log2m;
  // waves per block limited by LDS: 64*M bytes per wave
  int nw = 4;
  while (nw > 1 && (size_t)nw * 64 * M + 16 * (M + 1) + 8 * n_fft > 160 * 1024) nw >>= 1;
  const size_t lds = (size_t)nw * 64 * M + 16 * (M + 1) + 8 * n_fft;
  const int64_t total = batch * n_frames;
  int64_t grid = cdiv(total, nw);
  if (grid > 4096) grid = 4096;
  if (mode == AINP_FEAT_CNNBLSTM)
    hipLaunchKernelGGL(stft_features_kernel<AINP_FEAT_CNNBLSTM>, dim3(grid),
                       dim3(64 * nw), lds, s, audio, n_samples, clip_index,
                       gap_start, batch, gap_len, sample_rate, window, n_fft,
                       log2m, hop, n_frames, out0, out1, out2, out3);
  else
    hipLaunchKernelGGL(stft_features_kernel<AINP_FEAT_GAN>, dim3(grid),
                       dim3(64 * nw), lds, s, audio, n_samples, clip_index,
                       gap_start, batch, gap_len, sample_rate, window, n_fft,
                       log2m, hop, n_frames, out0, out1, out2, out3);
  return check_launch("ainp_stft_features");
}

extern "C" int ainp_stft(const void* audio, int dtype, int64_t n_signals,
                         int64_t n_samples, const double* window, int n_fft,
                         int hop, int center, int64_t n_frames, void* out,
                         void* stream) {
  if (!audio || !window || !out || n_signals < 0 || n_samples < 0 || hop <= 0 ||
      n_frames < 0 || (dtype != 0 && dtype != 1))
    return record_msg("ainp_stft: bad argument");
  if (n_fft < 16 || n_fft > 2048 || (n_fft & (n_fft - 1)))
    return record_msg("ainp_stft: n_fft must be a power of two in [16,2048]");
  if (n_signals == 0 || n_frames == 0) return AINP_OK;
  const int M = n_fft / 2;
  int log2m = 0;
  while ((1 << log2m) < M) ++log2m;
  int nw = 4;
  while (nw > 1 && (size_t)nw * 32 * M + 16 * (M + 1) + 8 * n_fft > 160 * 1024) nw >>= 1;
  const size_t lds = (size_t)nw * 32 * M + 16 * (M + 1) + 8 * n_fft;
  int64_t grid = cdiv(n_signals * n_frames, nw);
  if (grid > 4096) grid = 4096;
  hipStream_t s = as_stream(stream);
  if (dtype == 0)
    hipLaunchKernelGGL(stft_plain_kernel<float>, dim3(grid), dim3(64 * nw), lds, s,
                       (const float*)audio, n_samples, n_signals, window, n_fft,
                       log2m, hop, center, n_frames, (float*)out);
  else
    hipLaunchKernelGGL(stft_plain_kernel<double>, dim3(grid), dim3(64 * nw), lds, s,
                       (const double*)audio, n_samples, n_signals, window, n_fft,
                       log2m, hop, center, n_frames, (double*)out);
  return check_launch("ainp_stft");
}
