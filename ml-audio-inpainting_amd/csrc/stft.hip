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
  hipStream_t s = as_stream(stream);
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
