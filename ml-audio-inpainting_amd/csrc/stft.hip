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
// consecutive frames of one example per workgroup of 4 waves, one frame per
// 16-lane group; outputs staged in LDS and written as contiguous runs along t
// (the [B][F][T] layout), so every store is a coalesced 64-B (f32) / 128-B
// (complex64) row segment instead of one 4-byte scatter per bin.
//
// FFT: the 512-point real FFT is a 256-point complex FFT of
// z[m] = x[2m] + i x[2m+1], computed four-step as 16 x 16 in float64:
// lane j holds z[16 n1 + j] (n1 = 0..15), a 16-point DFT in registers
// (radix 4 x 4), the twiddle W256^{j k1} (LDS table), a 16 x 16 transpose
// through the group's own LDS slot (wave-local sync), a second 16-point DFT.
// Lane j then holds Z[j + 16 k2]; the real-FFT unpack pairs bins k and 256 - k
// (X[256 - k] = conj(Ze - W^k Zo)), so each lane forms 16 bins from 8 partner
// values fetched from lane 16 - j -- half the fp64 work of one bin per value.
//
// Work: one clean FFT per frame; a gapped FFT only for frames whose window
// [t*hop - 256, t*hop + 256) intersects the gap -- elsewhere the gapped and
// clean signals are the same float64 values, so the clean FFT is bit-identical
// to the gapped one and feeds the log-magnitude directly.  The kernel is
// fp64-VALU-bound (gfx950 issues a wave64 fp64 op at half the fp32 rate,
// measured 30 T lane-ops/s, tools/fp64_rate.hip) and store-bound in turn;
// tools/stft_lab.hip holds the measured alternatives.
namespace f512 {
constexpr int M = 256, F = 257, TF = 16, NW = 4, NT = 64 * NW;
constexpr int XROW = 17;                 // transpose row stride (dwords)
constexpr int XSLOT = 16 * XROW;         // per-FFT transpose buffer (dwords)
// LDS: log-magnitude plane P0 [257][16] f32 | complex plane PC [257][16] float2
// (during the FFT phase PC's bytes hold the transpose slots and the window) |
// W256 twiddle table.  53.4 KB: two workgroups per CU (VGPR-limited).
constexpr size_t LDS_P0 = (size_t)F * TF * sizeof(float);
constexpr size_t LDS_PC = (size_t)F * TF * sizeof(float2);
constexpr size_t LDS_TW = 256 * sizeof(double2);
constexpr size_t LDS_BYTES = LDS_P0 + LDS_PC + LDS_TW;
constexpr size_t XCH_BYTES = (size_t)NW * 4 * XSLOT * sizeof(uint32_t);
static_assert(XCH_BYTES + 512 * sizeof(double) <= LDS_PC, "xch + window fit in PC");

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
  int b, t0, ncomp, nvalid, ga, gb;
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
  T.gs64 = gap_start ? gap_start[T.b] : 0;
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
  return T;
}

// staged element (bin f, tile column c): columns XOR-swizzled by the bin's low
// bits, so the unpack's 16 lanes (16 bins, one column) hit 16 banks and the
// write-out's 16 lanes (one bin, 16 columns) read one contiguous row.
__device__ __forceinline__ int sw(int f, int c) { return f * TF + (c ^ (f & 15)); }

template <bool VEC2>
__device__ __forceinline__ void load_frame(const float* __restrict__ x, int s0, int ns, int gs,
                                           int gl, bool check, float (&r0)[16],
                                           float (&r1)[16]) {
  if (!check) {
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) {
      if (VEC2) {
        const float2 p = *reinterpret_cast<const float2*>(x + s0 + 32 * n1);
        r0[n1] = p.x;
        r1[n1] = p.y;
      } else {
        r0[n1] = x[s0 + 32 * n1];
        r1[n1] = x[s0 + 32 * n1 + 1];
      }
    }
    return;
  }
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const int s = s0 + 32 * n1;
    const bool in0 = (unsigned)s < (unsigned)ns && (unsigned)(s - gs) >= (unsigned)gl;
    const bool in1 = (unsigned)(s + 1) < (unsigned)ns && (unsigned)(s + 1 - gs) >= (unsigned)gl;
    if (VEC2) {
      const float2 p = *reinterpret_cast<const float2*>(x + min(max(s, 0), ns - 2));
      r0[n1] = in0 ? p.x : 0.f;
      r1[n1] = in1 ? p.y : 0.f;
    } else {
      const float p0 = x[min(max(s, 0), ns - 1)];
      const float p1 = x[min(max(s + 1, 0), ns - 1)];
      r0[n1] = in0 ? p0 : 0.f;
      r1[n1] = in1 ? p1 : 0.f;
    }
  }
}

// window (x 1/2, exact), 16-point DFT over n1, twiddle W256^{j k1}, wave-local
// 16 x 16 transpose (four dword planes, in place: each round moves one plane),
// 16-point DFT over n2.  Lane j ends with Z[j + 16 k2] at pos(k2).
__device__ __forceinline__ void fft256(const float (&r0)[16], const float (&r1)[16],
                                       const double2* win2, int j,
                                       const double2* tw256, uint32_t* xs, double (&re)[16],
                                       double (&im)[16], int tstride = 1) {
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) {
    const double2 w = win2[16 * n1 + j];
    re[n1] = (double)r0[n1] * w.x;
    im[n1] = (double)r1[n1] * w.y;
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the twiddle loads below the first DFT
  dft16(re, im);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) {
    const double2 w = tw256[((j * k1) & 255) * tstride];
    cmul_c(re[pos(k1)], im[pos(k1)], w.x, w.y);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int hi = r & 1;
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1)
      xs[k1 * XROW + j] = dw(r < 2 ? re[pos(k1)] : im[pos(k1)], hi);
    wave_sync();
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const uint32_t u = xs[j * XROW + n2];
      if (r < 2) re[n2] = set_dw(re[n2], hi, u);
      else im[n2] = set_dw(im[n2], hi, u);
    }
    wave_sync();
  }
  dft16(re, im);
}

// Real-FFT unpack by conjugate pairs: lane j forms X[k] and X[256 - k] for
// k = j + 16 k2, k2 = 0..7 (X[256 - k] = conj(Ze - W^k Zo)), and lane 0 also
// X[128].  Z's partner Z[256 - k] lives in lane 16 - j (lane 0: itself).
template <typename Out>
__device__ __forceinline__ void unpack(const double (&re)[16], const double (&im)[16], int j,
                                       int lane, double ujr, double uji, Out out,
                                       const double2* Wt = nullptr) {
  const int src = (lane & ~15) | ((16 - j) & 15);
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    const double zr = re[pos(k2)], zi = im[pos(k2)];
    const double sr = __shfl(re[pos(15 - k2)], src, 64);
    const double si = __shfl(im[pos(15 - k2)], src, 64);
    const double pr = j == 0 ? re[pos((16 - k2) & 15)] : sr;
    const double pi = j == 0 ? im[pos((16 - k2) & 15)] : si;
    const double er = zr + pr, ei = zi - pi;
    double orr = zi + pi, oi = pr - zr;
    double wr = ujr, wi = uji;
    if (Wt) {
      const double2 w = Wt[j + 16 * k2];
      wr = w.x;
      wi = w.y;
    } else {
      cmul_c(wr, wi, W32R[k2], W32I[k2]);
    }
    cmul_c(orr, oi, wr, wi);
    out(j + 16 * k2, er + orr, ei + oi);
    out(256 - j - 16 * k2, er - orr, oi - ei);
  }
  if (j == 0) {
    const double zr = re[pos(8)], zi = im[pos(8)];
    const double er = zr + zr, orr = zi + zi;
    double wr = ujr, wi = uji, o_r = orr, o_i = zr - zr;
    if (Wt) {
      wr = Wt[128].x;
      wi = Wt[128].y;
    } else {
      cmul_c(wr, wi, W32R[8], W32I[8]);
    }
    cmul_c(o_r, o_i, wr, wi);
    out(128, er + o_r, (zi - zi) + o_i);
  }
}

// log10(|X| + 1e-9) of the complex64-rounded bin: |X|^2 in fp32 (the
// cancellation-prone arithmetic is the fp64 FFT before it); the argument of the
// log is >= 1e-9, so the raw v_log_f32 needs no denormal scaling.
__device__ __forceinline__ float lm_cnn(double Xr, double Xi) {
  const float r = (float)Xr, i = (float)Xi;
  return __builtin_amdgcn_logf(__builtin_amdgcn_sqrtf(r * r + i * i) + 1e-9f) *
         0.30102999566398120f;
}

// Modes beyond the two feature modes (include/ainp.h):
//   F512_PLAIN  out0 = complex64 X [batch][257][n_frames] (librosa.stft, center,
//               zero padding) -- ainp_stft for n_fft = 512 float32
//   F512_GL     one Griffin-Lim phase update fused into the write-out
//               (librosa griffinlim): rebuilt = X; a = rebuilt - m/(1+m) tprev
//               (not on the first iteration); angles (out1) = a / (|a| + tiny);
//               tprev (out0, read and written) = rebuilt
constexpr int F512_PLAIN = 2, F512_GL = 3;

template <int MODE, bool VEC2>
__global__ __launch_bounds__(NT, 2) void stft512_kernel(
    const float* __restrict__ audio, int64_t n_samples, const int32_t* __restrict__ clip_index,
    const int64_t* __restrict__ gap_start, int64_t batch, int64_t gap_len, int64_t sample_rate,
    const double* __restrict__ window, int hop, int64_t n_frames, int64_t n_tiles_t,
    float* __restrict__ out0, float* __restrict__ out1, float* __restrict__ out2,
    float* __restrict__ out3, float gl_c = 0.f, int gl_first = 0) {
  constexpr bool FEAT = MODE == AINP_FEAT_CNNBLSTM || MODE == AINP_FEAT_GAN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P0 = reinterpret_cast<float*>(smem);
  float2* PC = reinterpret_cast<float2*>(smem + LDS_P0);
  // FFT phase: transpose slots and the window (x 1/2) live in PC's bytes
  uint32_t* xch = reinterpret_cast<uint32_t*>(smem + LDS_P0);
  double2* win2 = reinterpret_cast<double2*>(smem + LDS_P0 + XCH_BYTES);
  double2* tw256 = reinterpret_cast<double2*>(smem + LDS_P0 + LDS_PC);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = lane & 15, myjob0 = wave * 4 + (lane >> 4);
  const int ntt = (int)n_tiles_t, NF = (int)n_frames, ns = (int)n_samples;
  const int ntiles = (int)(batch * n_tiles_t);
  const bool want_lm = !FEAT ? false
                       : MODE == AINP_FEAT_CNNBLSTM ? out0 != nullptr : out1 != nullptr;
  const bool want_fft = MODE == F512_GL ? true
                        : MODE == F512_PLAIN ? out0 != nullptr
                        : MODE == AINP_FEAT_CNNBLSTM ? (out0 || out1) : (out0 || out1 || out2);
  float* mask_out = !FEAT ? nullptr : MODE == AINP_FEAT_CNNBLSTM ? out2 : out3;
  const int n_avail = 1 + ns / hop;
  {
    double s, c;
    sincospi(-(double)tid / 128.0, &s, &c);
    tw256[tid] = make_double2(c, s);
  }
  double ujr, uji;  // W512^j
  sincospi(-(double)j0 / 256.0, &uji, &ujr);
  double2 wreg = make_double2(window[2 * tid], window[2 * tid + 1]);
  wreg.x *= 0.5;  // the unpack's 1/2 factors (exact)
  wreg.y *= 0.5;

  for (int v = blockIdx.x; v < ntiles; v += gridDim.x) {
    const Tile T = make_tile<MODE>(v, ntiles, ntt, NF, ns, hop, audio, n_samples,
                                               clip_index, gap_start, gap_len, want_lm, want_fft);
    if (want_fft) {
      win2[tid] = wreg;  // the previous tile's unpack overwrote it
      // lane indices laundered per tile: keeps the compiler from hoisting ~100
      // per-lane LDS addresses out of the tile loop into registers
      int j = j0, myjob = myjob0;
      asm volatile("" : "+v"(j), "+v"(myjob));
      __syncthreads();
      const int cb = min(myjob, max(T.ncomp - 1, 0));
      const bool act_b = myjob < T.ncomp;
      const bool interior = T.ncomp == TF && T.t0 * hop >= 256 && (T.t0 + TF - 1) * hop + 256 <= ns;
      double re[16], im[16];
      uint32_t* xs = xch + myjob * XSLOT;
      // pass A: gapped FFTs of the columns whose window meets the gap (log-magnitude only)
      if (T.gb > T.ga) {
        const int ca = min(T.ga + myjob, T.gb - 1);
        const bool act_a = T.ga + myjob < T.gb;
        const int gs = (int)max((int64_t)-(1 << 30), min((int64_t)1 << 30, T.gs64));
        float ra0[16], ra1[16];
        load_frame<VEC2>(T.x, (T.t0 + ca) * hop - 256 + 2 * j, ns, gs, (int)gap_len, true, ra0,
                         ra1);
        fft256(ra0, ra1, win2, j, tw256, xs, re, im);
        if (MODE == AINP_FEAT_CNNBLSTM) {
          unpack(re, im, j, lane, ujr, uji, [&](int f, double Xr, double Xi) {
            if (act_a) P0[sw(f, ca)] = lm_cnn(Xr, Xi);
          });
        } else {
          unpack(re, im, j, lane, ujr, uji, [&](int f, double Xr, double Xi) {
            if (act_a) P0[sw(f, ca)] = log1pf(hypotf((float)Xr, (float)Xi));
          });
        }
      }
      // pass B: clean FFTs
      float rb0[16], rb1[16];
      load_frame<VEC2>(T.x, (T.t0 + cb) * hop - 256 + 2 * j, ns, 0, 0, !interior, rb0, rb1);
      fft256(rb0, rb1, win2, j, tw256, xs, re, im);
      __syncthreads();  // every transpose slot is read (they alias PC)
      const bool own_lm = act_b && !(myjob >= T.ga && myjob < T.gb);
      const bool zero_lm = !act_b;
      if (!FEAT) {
        unpack(re, im, j, lane, ujr, uji, [&](int f, double Xr, double Xi) {
          PC[sw(f, myjob)] = act_b ? make_float2((float)Xr, (float)Xi) : make_float2(0.f, 0.f);
        });
      } else if (MODE == AINP_FEAT_CNNBLSTM) {
        unpack(re, im, j, lane, ujr, uji, [&](int f, double Xr, double Xi) {
          const int l = sw(f, myjob);
          PC[l] = act_b ? make_float2((float)Xr, (float)Xi) : make_float2(0.f, 0.f);
          if (own_lm || zero_lm) P0[l] = act_b ? lm_cnn(Xr, Xi) : 0.f;
        });
      } else {
        unpack(re, im, j, lane, ujr, uji, [&](int f, double Xr, double Xi) {
          const int l = sw(f, myjob);
          const float cr = (float)Xr, ci = (float)Xi;
          const float lm = log1pf(hypotf(cr, ci));
          PC[l] = act_b ? make_float2(lm, atan2f(ci, cr)) : make_float2(0.f, 0.f);
          if (own_lm || zero_lm) P0[l] = act_b ? lm : 0.f;
        });
      }
    }
    __syncthreads();

    // coalesced write-out: thread (row, col) -> runs of TF consecutive frames
    int col = tid % TF, row0 = tid / TF;
    asm volatile("" : "+v"(col), "+v"(row0));
    if (!FEAT && col < T.nvalid) {
      const size_t base = (size_t)T.b * F * n_frames + T.t0 + col;
      float2* o0 = reinterpret_cast<float2*>(out0);
      float2* o1 = reinterpret_cast<float2*>(out1);
      for (int f = row0; f < F; f += NT / TF) {
        const size_t o = base + (size_t)f * n_frames;
        const float2 x = PC[sw(f, col)];
        if (MODE == F512_PLAIN) {
          o0[o] = x;
        } else {
          float ar = x.x, ai = x.y;
          if (!gl_first) {
            const float2 tp = o0[o];
            ar -= gl_c * tp.x;
            ai -= gl_c * tp.y;
          }
          const float mag = sqrtf(ar * ar + ai * ai) + 1.17549435e-38f;
          o1[o] = make_float2(ar / mag, ai / mag);
          o0[o] = x;
        }
      }
    } else if (FEAT && col < T.nvalid) {
      const int t = T.t0 + col;
      float maskv;
      if (MODE == AINP_FEAT_CNNBLSTM) {
        const int64_t fs = time_to_frame(T.gs64, sample_rate, hop);
        const int64_t fe = time_to_frame(T.ge64, sample_rate, hop);
        maskv = (t >= fs && t < fe) ? 1.f : 0.f;
      } else {
        int64_t fs = T.gs64 / hop;
        int64_t fe = (T.ge64 + hop - 1) / hop;
        if (fs < 0) fs = 0;
        if (fe > n_avail) fe = n_avail;
        maskv = (fe > fs && t >= fs && t < fe) ? 0.f : 1.f;
      }
      const size_t base = (size_t)T.b * F * n_frames + t;
      for (int f = row0; f < F; f += NT / TF) {
        const size_t o = base + (size_t)f * n_frames;
        const int l = sw(f, col);
        if (MODE == AINP_FEAT_CNNBLSTM) {
          if (out0) out0[o] = P0[l];
          if (out1) reinterpret_cast<float2*>(out1)[o] = PC[l];
        } else {
          const float2 p = PC[l];
          if (out0) out0[o] = p.x;
          if (out1) out1[o] = P0[l];
          if (out2) out2[o] = p.y;
        }
        if (mask_out) mask_out[o] = maskv;
      }
    }
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

// persistent grid of the n_fft = 512 kernel: two workgroups per CU
static int64_t f512_grid(int64_t ntiles) {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      n_cu = cu > 0 ? cu : 256;
    else
      n_cu = 256;
  }
  return min(ntiles, (int64_t)2 * n_cu);
}

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
    // persistent: two workgroups per CU walk the tiles (more do not fit the
    // VGPR budget); AINP_STFT_GRID overrides for tuning
    int64_t grid = f512_grid(ntiles);
    const char* ps = getenv("AINP_STFT_GRID");
    if (ps && atoi(ps) > 0) grid = min(ntiles, (int64_t)atoi(ps));
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

// n_fft = 512, center, float32 input on the tiled kernel (MODE F512_PLAIN or F512_GL)
template <int MODE>
static int f512_launch(const float* audio, int64_t n_signals, int64_t n_samples,
                       const double* window, int hop, int64_t n_frames, float* out0, float* out1,
                       float gl_c, int gl_first, hipStream_t s) {
  if (n_samples >= (1 << 30) || n_frames * hop >= (1 << 30))
    return record_msg("ainp_stft: signal too long for the n_fft=512 kernel");
  const int64_t ntt = cdiv(n_frames, f512::TF);
  const int64_t ntiles = n_signals * ntt;
  if (ntiles > 0x7fffffff) return record_msg("ainp_stft: too many frames");
  const int64_t grid = f512_grid(ntiles);
  const bool vec2 = (hop % 2 == 0) && (n_samples % 2 == 0) &&
                    ((reinterpret_cast<uintptr_t>(audio) & 7) == 0);
  if (vec2)
    hipLaunchKernelGGL((f512::stft512_kernel<MODE, true>), dim3(grid), dim3(f512::NT),
                       f512::LDS_BYTES, s, audio, n_samples, nullptr, nullptr, n_signals,
                       (int64_t)0, (int64_t)1, window, hop, n_frames, ntt, out0, out1, nullptr,
                       nullptr, gl_c, gl_first);
  else
    hipLaunchKernelGGL((f512::stft512_kernel<MODE, false>), dim3(grid), dim3(f512::NT),
                       f512::LDS_BYTES, s, audio, n_samples, nullptr, nullptr, n_signals,
                       (int64_t)0, (int64_t)1, window, hop, n_frames, ntt, out0, out1, nullptr,
                       nullptr, gl_c, gl_first);
  return check_launch("ainp_stft (n_fft 512)");
}

extern "C" int ainp_gl_stft_update(const float* audio, int64_t n_signals, int64_t n_samples,
                                   const double* window, int hop, int64_t n_frames,
                                   float* tprev, float* angles, float momentum, int first,
                                   void* stream) {
  if (!audio || !window || !tprev || !angles || n_signals < 0 || n_samples <= 0 || hop <= 0 ||
      n_frames < 0 || n_frames > 1 + n_samples / hop)
    return record_msg("ainp_gl_stft_update: bad argument");
  if (n_signals == 0 || n_frames == 0) return AINP_OK;
  return f512_launch<f512::F512_GL>(audio, n_signals, n_samples, window, hop, n_frames, tprev,
                                    angles, momentum / (1.f + momentum), first,
                                    as_stream(stream));
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
  const char* gen = getenv("AINP_STFT_GENERIC");  // 1: force the generic kernel (tests)
  if (n_fft == 512 && dtype == 0 && center && n_frames <= 1 + n_samples / hop &&
      !(gen && gen[0] == '1'))
    return f512_launch<f512::F512_PLAIN>((const float*)audio, n_signals, n_samples, window, hop,
                                         n_frames, (float*)out, nullptr, 0.f, 0,
                                         as_stream(stream));
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
