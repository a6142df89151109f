// istft.hip — inverse STFT and the Griffin-Lim phase update:
// utils.spectrogram_to_audio (utils.py:279-333) -> librosa>=0.10 istft /
// griffinlim.
//
// istft: every frame's spectrum (n_fft/2+1 bins) is inverse real-FFT'd in
// float64 (numpy irfft semantics: the imaginary parts of the DC and Nyquist
// bins are ignored) through a half-length complex IFFT in the wave's LDS,
// multiplied by the synthesis window and stored; a second kernel overlap-adds
// the frames as a gather (each output sample sums its <= n_fft/hop frames in
// fixed order), divides by the window sum-square where it exceeds tiny, and
// drops n_fft/2 samples on each side (center=True): output length
// hop*(T-1) (center) or n_fft + hop*(T-1).
#include "common.h"

namespace ainp {

struct cdi {
  double re, im;
};
__device__ __forceinline__ cdi cmuli(cdi a, cdi b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// input modes
enum { IST_C64 = 0, IST_C128 = 1, IST_MAG_ANGLES = 2, IST_MAG_PHASE = 3 };

__global__ __launch_bounds__(256) void istft_frames_kernel(
    const void* __restrict__ in0, const void* __restrict__ in1, int mode, int64_t n_signals,
    int64_t n_frames, const double* __restrict__ window, int n_fft, int log2m,
    double* __restrict__ frames) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = n_fft >> 1;
  const int F = M + 1;
  cdi* tw = reinterpret_cast<cdi*>(smem);                 // exp(+2 pi i q / n_fft), q in [0, M]
  cdi* wbase = tw + (M + 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cdi* bufA = wbase + (size_t)wave * 2 * M;
  cdi* bufB = bufA + M;
  for (int q = threadIdx.x; q <= M; q += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)q / (double)n_fft, &s, &c);
    tw[q] = {c, s};
  }
  __syncthreads();
  const int64_t total = n_signals * n_frames;
  const int nw = blockDim.x >> 6;
  for (int64_t base = (int64_t)blockIdx.x * nw; base < total; base += (int64_t)gridDim.x * nw) {
    const int64_t item = base + wave;
    const bool valid = item < total;
    const int64_t b = valid ? item / n_frames : 0;
    const int64_t t = valid ? item % n_frames : 0;
    auto bin = [&](int k) -> cdi {       // X[k] of (b, t), spectra laid out [b][F][T]
      if (!valid) return {0.0, 0.0};
      const int64_t idx = ((int64_t)b * F + k) * n_frames + t;
      cdi x;
      if (mode == IST_C64) {
        const float* p = reinterpret_cast<const float*>(in0);
        x = {(double)p[2 * idx], (double)p[2 * idx + 1]};
      } else if (mode == IST_C128) {
        const double* p = reinterpret_cast<const double*>(in0);
        x = {p[2 * idx], p[2 * idx + 1]};
      } else if (mode == IST_MAG_ANGLES) {
        const float mg = reinterpret_cast<const float*>(in0)[idx];
        const float* a = reinterpret_cast<const float*>(in1);
        // S * angles in complex64 arithmetic, as numpy does before irfft
        x = {(double)(mg * a[2 * idx]), (double)(mg * a[2 * idx + 1])};
      } else {
        const float mg = reinterpret_cast<const float*>(in0)[idx];
        const float ph = reinterpret_cast<const float*>(in1)[idx];
        double s, c;
        sincos((double)ph, &s, &c);
        x = {(double)mg * c, (double)mg * s};
      }
      if (k == 0 || k == M) x.im = 0.0;   // numpy irfft ignores them
      return x;
    };
    // pack: Z[k] = Xe[k] + i Xo[k], Xe = (A + B)/2, Xo = (A - B) e^{+2 pi i k/N} / 2,
    // A = X[k], B = conj(X[M-k])
    for (int k = lane; k < M; k += 64) {
      const cdi A = bin(k);
      const cdi Bc = bin(M - k);
      const cdi B = {Bc.re, -Bc.im};
      const cdi e = {0.5 * (A.re + B.re), 0.5 * (A.im + B.im)};
      const cdi o = cmuli({0.5 * (A.re - B.re), 0.5 * (A.im - B.im)}, tw[k]);
      bufA[k] = {e.re - o.im, e.im + o.re};
    }
    __syncthreads();
    // inverse complex FFT of length M (Stockham, conjugate twiddles)
    cdi* src = bufA;
    cdi* dst = bufB;
    for (int st = 0; st < log2m; ++st) {
      const int Ns = 1 << st;
      for (int j = lane; j < (M >> 1); j += 64) {
        const int k = j & (Ns - 1);
        const cdi w = tw[(k << (log2m - st))];
        const int o = (j << 1) - k;
        const cdi a = src[j];
        const cdi bb = cmuli(w, src[j + (M >> 1)]);
        dst[o] = {a.re + bb.re, a.im + bb.im};
        dst[o + Ns] = {a.re - bb.re, a.im - bb.im};
      }
      __syncthreads();
      cdi* tmp = src;
      src = dst;
      dst = tmp;
    }
    if (valid) {
      double* fr = frames + item * n_fft;
      const double inv = 1.0 / (double)M;
      for (int m = lane; m < M; m += 64) {
        fr[2 * m] = src[m].re * inv * window[2 * m];
        fr[2 * m + 1] = src[m].im * inv * window[2 * m + 1];
      }
    }
    __syncthreads();
  }
}

// y[b][o] = sum_t frames[b][t][j - t*hop] / wss[j], j = o + off (off = n_fft/2 if center)
template <typename Tout>
__global__ void istft_ola_kernel(const double* __restrict__ frames, const double* __restrict__ window,
                                 int64_t n_signals, int64_t n_frames, int n_fft, int hop,
                                 int64_t out_len, int64_t off, double tiny, Tout* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_signals * out_len) return;
  const int64_t b = i / out_len;
  const int64_t j = i - b * out_len + off;
  int64_t t_lo = j - n_fft + 1 <= 0 ? 0 : (j - n_fft + hop) / hop;   // ceil((j-n_fft+1)/hop)
  int64_t t_hi = j / hop;
  if (t_hi > n_frames - 1) t_hi = n_frames - 1;
  double s = 0.0, wss = 0.0;
  for (int64_t t = t_lo; t <= t_hi; ++t) {
    const int64_t n = j - t * hop;
    if (n < 0 || n >= n_fft) continue;
    s += frames[(b * n_frames + t) * n_fft + n];
    wss += window[n] * window[n];
  }
  if (wss > tiny) s /= wss;
  y[i] = (Tout)s;
}

// Griffin-Lim phase update (librosa griffinlim, momentum form):
//   a = rebuilt - (m / (1 + m)) * tprev   (no tprev term on the first iteration)
//   angles = a / (|a| + eps);   tprev = rebuilt
// complex64 interleaved arrays, eps = tiny(float32) as librosa uses for complex64.
__global__ void gl_update_kernel(const float* __restrict__ rebuilt, float* __restrict__ tprev,
                                 float* __restrict__ angles, int64_t n, float momentum, int first) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float rr = rebuilt[2 * i], ri = rebuilt[2 * i + 1];
  float ar = rr, ai = ri;
  if (!first) {
    const float c = momentum / (1.f + momentum);
    ar -= c * tprev[2 * i];
    ai -= c * tprev[2 * i + 1];
  }
  const float mag = sqrtf(ar * ar + ai * ai) + 1.17549435e-38f;
  angles[2 * i] = ar / mag;
  angles[2 * i + 1] = ai / mag;
  tprev[2 * i] = rr;
  tprev[2 * i + 1] = ri;
}

}  // namespace ainp

using namespace ainp;

extern "C" size_t ainp_istft_workspace(int64_t n_signals, int64_t n_frames, int n_fft) {
  return (size_t)n_signals * n_frames * n_fft * sizeof(double);
}

extern "C" int ainp_istft(const void* in0, const void* in1, int mode, int64_t n_signals,
                          int n_bins, int64_t n_frames, const double* window, int n_fft, int hop,
                          int center, void* workspace, void* out, void* stream) {
  int log2n = 0;
  while ((1 << log2n) < n_fft) ++log2n;
  if (!in0 || (mode >= 2 && !in1) || mode < 0 || mode > 3 || n_signals < 1 || n_frames < 1 ||
      !window || n_fft < 16 || n_fft > 2048 || (1 << log2n) != n_fft || n_bins != n_fft / 2 + 1 ||
      hop < 1 || hop > n_fft || !workspace || !out)
    return record_msg("ainp_istft: bad argument (n_fft power of two 16..2048, bins n_fft/2+1)");
  hipStream_t s = as_stream(stream);
  const int M = n_fft / 2;
  int nw = 4;   // waves per block: each needs 2*M complex doubles of LDS (160 KB on gfx950)
  while (nw > 1 && (size_t)nw * 32 * M + 16 * (M + 1) > 160 * 1024) nw >>= 1;
  const size_t lds = (size_t)nw * 32 * M + 16 * (M + 1);
  const int64_t items = n_signals * n_frames;
  int64_t blocks = cdiv(items, nw);
  if (blocks > 8192) blocks = 8192;
  double* frames = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(istft_frames_kernel, dim3((unsigned)blocks), dim3(64 * nw), lds, s, in0, in1,
                     mode, n_signals, n_frames, window, n_fft, log2n - 1, frames);
  int rc = check_launch("istft_frames");
  if (rc) return rc;
  const int64_t full = (int64_t)n_fft + (int64_t)hop * (n_frames - 1);
  const int64_t off = center ? n_fft / 2 : 0;
  const int64_t out_len = center ? full - 2 * (n_fft / 2) : full;
  const int64_t total = n_signals * out_len;
  if (mode == IST_C128)
    hipLaunchKernelGGL(istft_ola_kernel<double>, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       s, frames, window, n_signals, n_frames, n_fft, hop, out_len, off,
                       2.2250738585072014e-308, reinterpret_cast<double*>(out));
  else
    hipLaunchKernelGGL(istft_ola_kernel<float>, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, s,
                       frames, window, n_signals, n_frames, n_fft, hop, out_len, off,
                       (double)1.17549435e-38f, reinterpret_cast<float*>(out));
  return check_launch("istft_ola");
}

extern "C" int ainp_gl_update(const float* rebuilt, float* tprev, float* angles, int64_t n,
                              float momentum, int first, void* stream) {
  if (!rebuilt || !tprev || !angles || n < 1) return record_msg("ainp_gl_update: bad argument");
  hipLaunchKernelGGL(gl_update_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), rebuilt, tprev, angles, n, momentum, first);
  return check_launch("gl_update");
}
