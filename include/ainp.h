/*
 * ainp.h — C ABI of the MI355X-native spectrogram-inpainting training path.
 *
 * Drop-in boundary.  The reference
 * (savage-hacker14/ml-audio-inpainting) is pure Python: its "operator API" is
 * the Python surface of utils.py / models/CNNBLSTM/{model,dataset,train}.py.
 * Every entry point below replaces one implicit librosa / numpy / ATen kernel
 * that surface launches today; the reference call site is cited per function.
 *
 * Conventions (all functions):
 *   - every pointer is a caller-owned DEVICE buffer unless stated otherwise;
 *     the library never allocates, frees or synchronises;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *   - layouts are dense row-major (C order) in the shapes stated;
 *   - return 0 on success or a negative AINP_E* code; nothing throws across
 *     the ABI; launches are asynchronous on `stream`.
 * Callers: the Python host layer (ml-audio-inpainting_amd/ainp/_lib.py) via
 * ctypes; see INTEGRATION.md for the binding stub.
 */
#ifndef AINP_H
#define AINP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AINP_OK 0
#define AINP_EINVAL (-1)     /* bad shape / argument */
#define AINP_ELAUNCH (-2)    /* kernel launch failed */
#define AINP_EUNSUPPORTED (-3)

/* ------------------------------------------------------------------------ */
/* Library identity                                                          */
/* ------------------------------------------------------------------------ */
/* ABI version: bumped on any signature change. */
int ainp_abi_version(void);
/* Name of the gfx target the code objects were built for ("gfx950"). */
const char* ainp_build_target(void);
/* Last hip error string recorded by a failing launch in this thread. */
const char* ainp_last_error(void);

/* ------------------------------------------------------------------------ */
/* (a5/a6/a7) STFT + spectrogram features + gap mask, one fused kernel.      */
/* ------------------------------------------------------------------------ */
/* Replaces, per example:
 *   utils.extract_spectrogram -> librosa.stft(center=True, window='hann',
 *       pad_mode='constant')                           (utils.py:192-234)
 *   CNNBLSTM mode: models/CNNBLSTM/dataset.py:95-119  (target STFT of the clean
 *       clip, log10(|STFT(gapped clip)|+1e-9), time_to_frames gap mask, 1=gap)
 *   GAN mode:      models/GAN/dataset.py:104-152      (log1p|STFT| of clean and
 *       impaired clip, angle of the clean STFT, frame mask 1=valid)
 * Arithmetic: both STFTs are computed in float64 (the reference's gapped CNNBLSTM
 * path is complex128) and rounded once to the output type.
 *
 * audio      [n_clips, n_samples] f32 clean clips
 * clip_index [batch] int32 clip used by each example (NULL: example b uses clip b)
 * gap_start  [batch] int64 first zeroed sample of each example's gap
 * window     [n_fft] f64 analysis window, already centre-padded to n_fft
 *            (librosa get_window(...,fftbins=True) + util.pad_center)
 * n_fft      power of two, 16..2048;   F = n_fft/2+1
 * n_frames   frames written per example (<= 1 + n_samples/hop); CNNBLSTM slices
 *            to ceil(sr*max_len_s/hop) (dataset.py:89,110-111)
 * mode 0 (AINP_FEAT_CNNBLSTM):
 *   out0 [batch,F,n_frames] f32  log10(|X_gap|+1e-9)
 *   out1 [batch,F,n_frames,2] f32 complex64 target X_clean (re,im interleaved)
 *   out2 [batch,F,n_frames] f32  mask, 1 on frames [fs,fe) with
 *        fs = int((s/sr)*sr)//hop, fe = int(((s+g)/sr)*sr)//hop in IEEE double
 *        (librosa.time_to_frames of the float seconds)
 *   out3 unused (may be NULL)
 * mode 1 (AINP_FEAT_GAN):
 *   out0 log1p(|X_clean|)   out1 log1p(|X_imp|)   out2 angle(X_clean)
 *   out3 mask 1=valid, 0 on [s//hop, min(T, ceil((s+g)/hop)))
 * Any out pointer may be NULL to skip that output.
 */
#define AINP_FEAT_CNNBLSTM 0
#define AINP_FEAT_GAN 1
int ainp_stft_features(const float* audio, int64_t n_clips, int64_t n_samples,
                       const int32_t* clip_index, const int64_t* gap_start,
                       int64_t batch, int64_t gap_len, int64_t sample_rate,
                       const double* window, int n_fft, int hop,
                       int64_t n_frames, int mode, float* out0, float* out1,
                       float* out2, float* out3, void* stream);

/* Plain STFT, utils.extract_spectrogram -> librosa.stft (utils.py:192-234):
 * audio [n_signals, n_samples] of dtype 0 = float32 or 1 = float64 (device);
 * out complex64 (dtype 0) / complex128 (dtype 1) [n_signals, n_fft/2+1,
 * n_frames], computed in float64.  center != 0: frame t starts at
 * t*hop - n_fft/2 with zero padding (n_frames = 1 + n_samples/hop); else at
 * t*hop (n_frames = 1 + (n_samples-n_fft)/hop). */
int ainp_stft(const void* audio, int dtype, int64_t n_signals,
              int64_t n_samples, const double* window, int n_fft, int hop,
              int center, int64_t n_frames, void* out, void* stream);

/* Inverse STFT, librosa>=0.10 istft (utils.spectrogram_to_audio, utils.py:317-326):
 * spectra [n_signals][n_bins = n_fft/2+1][n_frames] given as mode
 *   0: complex64 (in0)            1: complex128 (in0, output float64)
 *   2: magnitude f32 (in0) * complex64 unit angles (in1)  -- the Griffin-Lim inner istft
 *   3: magnitude f32 (in0) * exp(i * phase f32 (in1))    -- spectrogram_to_audio with phase
 * frames: float64 irfft (imaginary DC / Nyquist ignored, as numpy) x window;
 * overlap-add gather, divided by the window sum-square where > tiny; center != 0
 * trims n_fft/2 per side: out [n_signals][hop*(n_frames-1)] (center) or
 * [n_signals][n_fft + hop*(n_frames-1)].  workspace: ainp_istft_workspace bytes.
 * window: [n_fft] f64, centre-padded (as for ainp_stft). */
size_t ainp_istft_workspace(int64_t n_signals, int64_t n_frames, int n_fft);
int ainp_istft(const void* in0, const void* in1, int mode, int64_t n_signals, int n_bins,
               int64_t n_frames, const double* window, int n_fft, int hop, int center,
               void* workspace, void* out, void* stream);
/* One Griffin-Lim phase update (librosa griffinlim, utils.py:330): a = rebuilt -
 * m/(1+m) * tprev (no tprev term when first != 0), angles = a / (|a| + tiny),
 * tprev = rebuilt; n complex64 elements (interleaved). */
/* Griffin-Lim STFT + phase update in one launch (n_fft = 512, center, float32
 * audio [n_signals][n_samples] -> n_frames frames; the tiled n_fft=512 STFT
 * kernel with ainp_gl_update's arithmetic in its write-out): rebuilt =
 * stft(audio); a = rebuilt - m/(1+m) * tprev (not when first != 0); angles =
 * a / (|a| + tiny); tprev = rebuilt.  tprev / angles: complex64
 * [n_signals][257][n_frames].  ainp_stft routes n_fft = 512 float32 center
 * STFTs to the same kernel. */
int ainp_gl_stft_update(const float* audio, int64_t n_signals, int64_t n_samples,
                        const double* window, int hop, int64_t n_frames, float* tprev,
                        float* angles, float momentum, int first, void* stream);
int ainp_gl_update(const float* rebuilt, float* tprev, float* angles, int64_t n,
                   float momentum, int first, void* stream);

/* ------------------------------------------------------------------------ */
/* fp32 GEMM on MFMA (fp32-accurate bf16 split by default, exact f32 on flag) */
/* ------------------------------------------------------------------------ */
/* C = alpha * op(A) * op(B) + beta * C + bias1 + bias2   (bias along n)
 * Replaces the ATen GEMMs behind nn.LSTM's input projections and nn.Linear
 * (models/CNNBLSTM/model.py:46-50,77,80) and their backward.
 * Element (m,k) of op(A) is A[m*sam + k*sak]; (k,n) of op(B) is
 * B[k*sbk + n*sbn]; (m,n) of C is C[m*scm + n*scn].  One of (sam,sak), one
 * of (sbk,sbn) and one of (scm,scn) must be 1 (the contiguous dimension).
 * Batches: nptr pointer batches (host arrays of device pointers, nptr <= 8)
 * times nstrided strided batches; batch b uses pointer entry b % nptr offset
 * by (b / nptr) * stride{A,B,C}.  bias1/bias2: host arrays (may be NULL, or
 * hold NULL entries) of per-pointer-batch bias vectors of length N.
 * ksplit == 1: all nptr*nstrided (A,B) pairs are summed into C[0]
 * (K-concatenation across separate buffers / strided slabs).
 * ksplit == 2: for each pointer batch p, its nstrided (A,B) pairs are summed
 * into C[p] (split-K with one partial slab per pointer batch). */
int ainp_gemm_f32(int64_t M, int64_t N, int64_t K, float alpha,
                  const float* const* A, int64_t sam, int64_t sak,
                  int64_t strideA, const float* const* B, int64_t sbk,
                  int64_t sbn, int64_t strideB, float beta, float* const* C,
                  int64_t scm, int64_t scn, int64_t strideC,
                  const float* const* bias1, const float* const* bias2,
                  int nptr, int64_t nstrided, int ksplit, void* stream);

/* Same GEMM with a caller-provided workspace.  When the 128x128 tile grid
 * would leave the resident workgroup slots unevenly filled (ksplit == 0 and
 * K long), the work is split stream-K style into equal (tile, k) ranges;
 * pieces of tiles that straddle two ranges go through the workspace and are
 * summed in fixed order (deterministic).  ainp_gemm_f32_workspace returns the
 * bytes needed (0 = the plain grid is used and workspace may be NULL); a
 * smaller or NULL workspace silently selects the plain grid.  A workspace must
 * not be shared by calls in flight on different streams.  Stream-K is used by
 * the exact f32 main loop only (AINP_GEMM_EXACT_F32 below); the default split
 * bf16 loop always runs the plain grid and ignores the workspace. */
size_t ainp_gemm_f32_workspace(int64_t M, int64_t N, int64_t K, int nptr,
                               int64_t nstrided, int ksplit);
int ainp_gemm_f32_ws(int64_t M, int64_t N, int64_t K, float alpha,
                     const float* const* A, int64_t sam, int64_t sak,
                     int64_t strideA, const float* const* B, int64_t sbk,
                     int64_t sbn, int64_t strideB, float beta, float* const* C,
                     int64_t scm, int64_t scn, int64_t strideC,
                     const float* const* bias1, const float* const* bias2,
                     int nptr, int64_t nstrided, int ksplit, void* workspace,
                     size_t ws_bytes, void* stream);

/* Same GEMM with a precision flag.  flags == 0 (what ainp_gemm_f32 and
 * ainp_gemm_f32_ws use): each fp32 operand is split exactly into three bf16
 * pieces and the six cross products of order >= 2^-16 are accumulated in f32
 * on the bf16 MFMA (dropped terms <= ~2^-23 |a||b| per product, the level of
 * f32 rounding); flags == AINP_GEMM_EXACT_F32: exact f32 MFMA (k-ordered fmaf
 * chain); flags == AINP_GEMM_BF16: every operand element rounded to bf16
 * (nearest-even), f32 accumulation -- the bf16 configurations (BASELINE
 * configs C3-C5, torch autocast(bfloat16) arithmetic for nn.LSTM / nn.Linear,
 * models/CNNBLSTM/model.py:46-50). */
#define AINP_GEMM_EXACT_F32 1
#define AINP_GEMM_BF16 2
int ainp_gemm_f32_ex(int64_t M, int64_t N, int64_t K, float alpha,
                     const float* const* A, int64_t sam, int64_t sak,
                     int64_t strideA, const float* const* B, int64_t sbk,
                     int64_t sbn, int64_t strideB, float beta, float* const* C,
                     int64_t scm, int64_t scn, int64_t strideC,
                     const float* const* bias1, const float* const* bias2,
                     int nptr, int64_t nstrided, int ksplit, int flags, void* workspace,
                     size_t ws_bytes, void* stream);

/* fp32 layer-0 LSTM input projection (models/CNNBLSTM/model.py:46-47,77,
 * nn.LSTM's x W_ih^T + b_ih + b_hh for both directions in one launch) on the
 * 256x256 LDS-DMA tile: C[m][n] = sum_k A[m][k] B[n][k] + bias(n), A [M][lda]
 * fp32 k-contiguous, B rows n < bsplit from B1 [bsplit][ldb], the rest from
 * B2 [N - bsplit][ldb] (the two directions' W_ih), 16-byte aligned rows
 * (lda, ldb % 4 == 0), K % 16 == 0, bsplit % 256 == 0; bias as
 * ainp_gemm_bf16nt.  Arithmetic and summation order are those of
 * ainp_gemm_f32's default main loop (the exact three-piece bf16 split, six
 * cross products per 16-k step), so with nsplit == 1 C is bit-identical to
 * it.  nsplit > 1: split-K, split s sums k in [s*kc, min(K, (s+1)*kc))
 * (kc % 16 == 0) into slab C + s*strideC, the bias into slab 0 only (combine
 * with ainp_sum_slabs). */
int ainp_gemm_x6nt_256(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                       const float* B1, const float* B2, int64_t ldb, int64_t bsplit,
                       float* C, int64_t ldc, const float* bias_a1, const float* bias_a2,
                       const float* bias_b1, const float* bias_b2, int64_t bias_nsplit,
                       int nsplit, int64_t kc, int64_t strideC, void* stream);

/* fp32-accurate ("x6") GEMMs on the 256 x 256 split-plane tile
 * (csrc/gemm_x6r.hip): 1..3 problems in ONE launch (one grid, problem q's
 * work items after problem q-1's), so e.g. the layer-0 LSTM data gradient and
 * weight gradient (models/CNNBLSTM/model.py:46-47,77 backward) share the chip
 * without a second stream.  Per problem:
 *   C(m, n) = sum_k A(m, k) B(n, k) + bias(n)          m < M, n < N, k < K
 *   A(m, k) = a_kmajor ? A[k*lda + m] : A[m*lda + k]; if A2, columns
 *             k >= a_ksplit come from A2 at k - a_ksplit
 *   B(n, k) = b_kmajor ? B[k*ldb + n] : B[n*ldb + k]; if B2 and b_ksplit > 0,
 *             columns k >= b_ksplit come from B2 (k - b_ksplit); if B2 and
 *             b_ksplit <= 0, rows n >= b_nsplit come from B2 (n - b_nsplit)
 *   C rows m >= c_msplit go to C2 (m - c_msplit) when C2 != NULL; ldc for both
 *   bias: (bias_a1 + bias_a2)[n] for n < bias_nsplit, (bias_b1 + bias_b2)
 *         [n - bias_nsplit] after (any may be NULL), slab 0 only
 *   nsplit > 1: split-K, split s sums k in [s*kc, min(K, (s+1)*kc)) into
 *         C + s*strideC (and C2 + s*strideC)
 * Requirements: K, kc, a_ksplit, b_ksplit % 16 == 0; b_nsplit, c_msplit %
 * 256 == 0; operands 16-byte aligned with ld % 4 == 0; k-major operands have
 * a row count % 4 == 0.  Arithmetic: the exact three-piece bf16 split, six
 * cross products per 16-k step (ainp_gemm_f32's default main loop): with
 * nsplit == 1 and k-contiguous operands bit-identical to ainp_gemm_x6nt_256. */
typedef struct {
  const float* A; const float* A2; int64_t lda; int64_t a_ksplit; int a_kmajor;
  const float* B; const float* B2; int64_t ldb; int64_t b_nsplit; int64_t b_ksplit; int b_kmajor;
  float* C; float* C2; int64_t ldc; int64_t c_msplit;
  const float* bias_a1; const float* bias_a2; const float* bias_b1; const float* bias_b2;
  int64_t bias_nsplit;
  int64_t M, N, K; int nsplit; int64_t kc; int64_t strideC;
} ainp_x6_problem;
int ainp_gemm_x6_multi(const ainp_x6_problem* probs, int nprobs, void* stream);

/* bf16-operand GEMM (the bf16 configuration's layer-0 LSTM GEMMs,
 * models/CNNBLSTM/model.py:46-47,77: input projection, data and weight
 * gradients): C[m][n] (+ split s * strideC) = sum_k A[m][k] B[n][k] + bias(n),
 * A [M][lda] and B [N][ldb] bf16 (uint16 bit patterns), both k-contiguous,
 * 16-byte aligned rows (lda, ldb % 8 == 0), K % 8 == 0; fp32 accumulation
 * on the bf16 MFMA; C fp32 row-major with ldc.  bias(n) = a1[n] + a2[n] for
 * n < bias_nsplit, else b1[n - bias_nsplit] + b2[n - bias_nsplit] (NULLs = 0:
 * the two LSTM directions' b_ih + b_hh).  nsplit > 1: split-K, split s sums k
 * in [s*kc, min(K, (s+1)*kc)) (kc % 64 == 0) into slab C + s*strideC with
 * no bias (combine with ainp_sum_slabs). */
int ainp_gemm_bf16nt(int64_t M, int64_t N, int64_t K, const uint16_t* A, int64_t lda,
                     const uint16_t* B, int64_t ldb, float* C, int64_t ldc,
                     const float* bias_a1, const float* bias_a2, const float* bias_b1,
                     const float* bias_b2, int64_t bias_nsplit, int nsplit, int64_t kc,
                     int64_t strideC, void* stream);
/* Up to 3 bf16-operand GEMMs in ONE launch on the 256 x 256 LDS-DMA tile
 * (csrc/gemm16.hip gemm_bf16nt_256_multi_kernel): the bf16 configuration's
 * layer-0 LSTM backward pair dW_cat = dg^T X beside dX = dg W_cat
 * (models/CNNBLSTM/model.py:46-47,77), the long-K weight-gradient items first.
 * Per problem C[m][n] (+ split s * strideC) = sum_k A[m][k] B[n][k], A [M][lda]
 * and B [N][ldb] bf16 bit patterns (k-contiguous, 16-byte aligned rows, lda,
 * ldb % 8 == 0), K % 32 == 0, fp32 C row-major; nsplit > 1: split s sums k in
 * [s*kc, min(K, (s+1)*kc)) (kc % 32 == 0) into slab C + s*strideC (combine
 * with ainp_sum_slabs).  a_kmajor / b_kmajor: the operand is given k-major
 * ([K][ld], ld >= M or N; rows transposed in LDS by ds_read_b64_tr_b16), e.g.
 * dW_cat = dg^T X straight from dg [NT, 8H] and X [NT, I].  Same MFMA and k
 * order as ainp_gemm_bf16nt in every layout: with equal splits the results
 * are bit-identical. */
typedef struct {
  const uint16_t* A; int64_t lda;
  const uint16_t* B; int64_t ldb;
  float* C; int64_t ldc;
  int64_t M, N, K; int nsplit; int64_t kc; int64_t strideC;
  int a_kmajor, b_kmajor;   /* 1: A(m, k) = A[k*lda + m] (M % 8 == 0), likewise B */
} ainp_bf16_problem;
int ainp_gemm_bf16nt_multi(const ainp_bf16_problem* probs, int nprobs, void* stream);
/* fp32 x [R][ld_in] -> bf16 (nearest-even) out [R][ld_out] and/or its
 * transpose outT [C][ld_t] (either may be NULL): the BPTT gradient and the
 * layer-0 weights as bf16 GEMM operands. */
int ainp_cast_bf16_t(const float* x, int64_t R, int64_t C, int64_t ld_in, uint16_t* out,
                     int64_t ld_out, uint16_t* outT, int64_t ld_t, void* stream);

/* fp32 x [R][ld_in] -> outT [C][ld_t] (64 x 64 LDS tiles).  Builds the
 * k-contiguous W_ih^T operand of the fp32 layer-0 data gradient
 * dX = dgates . W_ih (models/CNNBLSTM/model.py:46-47 backward, via
 * ainp_gemm_x6nt_256 with bsplit == N). */
int ainp_transpose_f32(const float* x, int64_t R, int64_t C, int64_t ld_in, float* outT,
                       int64_t ld_t, void* stream);

/* ------------------------------------------------------------------------ */
/* 3x3 / stride 1 / pad 1 convolution over [N, C, F, T] spectrogram tiles    */
/* ------------------------------------------------------------------------ */
/* Replaces nn.Conv2d(kernel_size=3, padding=1) of models/CNNBLSTM/model.py:
 * 35-60 with the preceding nn.BatchNorm2d + nn.ReLU fused into its input load.
 * Forward: y = conv(act(x)) + bias, act(x) = relu(x*in_scale+in_shift) per
 * input channel when in_scale != NULL, identity otherwise; zero padding is
 * applied to act(x) as nn.Conv2d pads its (post-ReLU) input.
 * w: [Cout, Cin, 3, 3]; bias: [Cout] or NULL; Cout <= 64.
 * stats (may be NULL): double[ainp_conv3x3_fwd_stat_rows(N,Cin,Cout,H,W) *
 * 2*Cout] (ainp_conv3x3_fwd_stat_parts(N,H,W) is an upper bound over all
 * channel counts); row p receives a workgroup's [sum y (Cout) | sum y^2
 * (Cout)] for the following BatchNorm (reduced by ainp_bn_stats_reduce);
 * rows a kernel does not produce are zeroed. */
int ainp_conv3x3_fwd_stat_parts(int64_t N, int64_t H, int64_t W);
int64_t ainp_conv3x3_fwd_stat_rows(int64_t N, int Cin, int Cout, int64_t H, int64_t W);
/* The rows for a given ainp_conv3x3_fwd_ex `flags` (AINP_CONV_BF16: the bf16
 * kernels run a larger persistent grid, one row per workgroup). */
int64_t ainp_conv3x3_fwd_stat_rows_ex(int64_t N, int Cin, int Cout, int64_t H, int64_t W,
                                      int flags);
int ainp_conv3x3_fwd(const float* x, const float* w, const float* bias,
                     const float* in_scale, const float* in_shift, float* y,
                     double* stats, int64_t N, int Cin, int Cout, int64_t H,
                     int64_t W, void* stream);
/* Data gradient dx = conv_transpose(dy, w): [N,Cout,H,W] -> [N,Cin,H,W].
 * workspace unused (may be NULL); Cin <= 64. */
int ainp_conv3x3_dgrad(const float* dy, const float* w, float* dx,
                       float* workspace, int64_t N, int Cin, int Cout,
                       int64_t H, int64_t W, void* stream);
/* Weight gradient dw[co,ci,ky,kx] = sum_{n,h,w} dy[n,co,h,w] *
 *   act(x)[n,ci,h+ky-1,w+kx-1]; dbias[co] = sum dy (dbias may be NULL).
 * act as in the forward.  Overwrites dw / dbias; deterministic.
 * workspace: ainp_conv3x3_wgrad_workspace(...) bytes. */
size_t ainp_conv3x3_wgrad_workspace(int64_t N, int Cin, int Cout, int64_t H,
                                    int64_t W);
int ainp_conv3x3_wgrad(const float* x, const float* in_scale,
                       const float* in_shift, const float* dy, float* dw,
                       float* dbias, void* workspace, int64_t N, int Cin,
                       int Cout, int64_t H, int64_t W, void* stream);
/* The three entry points above with a precision flag (the plain ones pass 0:
 * fp32-accurate split-bf16 MFMA, or exact f32 for the 1- and 16-channel
 * pairs).  AINP_CONV_BF16: the 16/32/64-channel pairs round every activation /
 * weight / gradient operand to bf16 (nearest-even) and accumulate in f32 --
 * the bf16 configurations C3-C5 (torch autocast(bfloat16) nn.Conv2d of
 * models/CNNBLSTM/model.py:35-60); BatchNorm statistics, biases and outputs
 * stay fp32.  The 1 <-> 16 channel convs stay fp32 (HBM-bound). */
#define AINP_CONV_BF16 2
/* With AINP_CONV_BF16, data / weight gradients only: dy holds bf16 values
 * (uint16 storage, passed through the float* argument) -- the bf16
 * configuration's BatchNorm-backward outputs (ainp_bn_relu_bwd_apply_ex with
 * AINP_BN_GY16), which these kernels round to bf16 anyway, so dx and dw are
 * those of fp32 dy (dbias sums the stored bf16 values).  Supported by the
 * pairs with split-bf16 kernels (16/32/64 channels); other pairs return an
 * error. */
#define AINP_CONV_DY16 4
/* With AINP_CONV_BF16: forward, and the weight gradient's act(x) source: x
 * holds bf16 values (uint16 storage through the float* argument) -- the bf16
 * configuration's pre-BatchNorm activations, written by a forward with
 * AINP_CONV_Y16 (y as bf16, nearest-even; its BatchNorm partials sum the
 * stored values).  Supported by the pairs with persistent split-bf16
 * forwards and split-bf16 weight gradients (ainp_conv3x3_io16_ok). */
#define AINP_CONV_X16 8
#define AINP_CONV_Y16 16
/* Round 5: channel-last activations, [N][H][W][C] (a pixel's channels
 * contiguous; 1-2-channel tensors are the same in either layout).  The
 * input (forward: x; data gradient: dy; weight gradient: x) is channel-last
 * with AINP_CONV_XCL, the output (forward: y; data gradient: dx) with
 * AINP_CONV_YCL, the weight gradient's dy with AINP_CONV_GCL.  Every
 * combination with the bf16 flags above; served for the pairs
 * ainp_conv3x3_cl_ok accepts (the model's 1/16/32/64-channel convs).
 * Replaces the NCHW convs of models/CNNBLSTM/model.py:34-61. */
#define AINP_CONV_XCL 32
#define AINP_CONV_YCL 64
#define AINP_CONV_GCL 128
/* Round 6, data gradient only (not with AINP_CONV_YCL): dx written
 * [Cin][H][N][W] -- for the decoder input, the [C*F, N*T] k-major operand of
 * the fp32 output projection's backward GEMMs (nn.Linear + view/permute of
 * models/CNNBLSTM/model.py:51-53,79-80), which otherwise needs a transposing
 * copy of the whole gradient.  Served for the 32 -> 16 channel data gradient
 * (dy 32 channels, dx 16) only; ainp_conv3x3_dgrad_cfnt_ok says when
 * (host-only), and ainp_conv3x3_dgrad_ex refuses it otherwise. */
#define AINP_CONV_YCFNT 256
int ainp_conv3x3_dgrad_cfnt_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W);
int ainp_conv3x3_cl_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W);
int ainp_conv3x3_fwd_ex(const float* x, const float* w, const float* bias,
                        const float* in_scale, const float* in_shift, float* y,
                        double* stats, int64_t N, int Cin, int Cout, int64_t H,
                        int64_t W, int flags, void* stream);
int ainp_conv3x3_dgrad_ex(const float* dy, const float* w, float* dx,
                          float* workspace, int64_t N, int Cin, int Cout,
                          int64_t H, int64_t W, int flags, void* stream);
int ainp_conv3x3_wgrad_ex(const float* x, const float* in_scale,
                          const float* in_shift, const float* dy, float* dw,
                          float* dbias, void* workspace, int64_t N, int Cin,
                          int Cout, int64_t H, int64_t W, int flags, void* stream);
/* Round 6: the weight gradient of Conv2d(1, 16) (x one channel; the encoder's
 * first conv, models/CNNBLSTM/model.py:35-36) with the step-2 apply of the
 * BatchNorm+ReLU backward of its output fused in: dy = gy is formed per
 * element from g (gradient of the BatchNorm+ReLU output) and y (its pre-BN
 * input), both channel-last [N][H][W][16] fp32, 16-byte aligned, with the
 * constants and arithmetic of ainp_bn_relu_bwd_apply_ex (scale / shift /
 * gamma / save_mean_rstd / sums / count as there) -- the values are that
 * apply's gy bit for bit -- and gy is not written (for a conv whose input needs
 * no gradient it has no other consumer).  dw / dbias as ainp_conv3x3_wgrad_ex
 * (lay: dy channel-last), dgamma / dbeta as the apply writes them.  workspace:
 * ainp_conv3x3_wgrad_workspace(N, 1, 16, H, W) bytes. */
int ainp_conv3x3_wgrad_bnapply(const float* x, const float* in_scale, const float* in_shift,
                               const float* g, const float* y, const float* scale,
                               const float* shift, const float* gamma,
                               const float* save_mean_rstd, const double* sums, int64_t count,
                               float* dw, float* dbias, float* dgamma, float* dbeta,
                               void* workspace, int64_t N, int Cin, int Cout, int64_t H,
                               int64_t W, void* stream);
/* 1 if both ainp_conv3x3_dgrad_ex and ainp_conv3x3_wgrad_ex of this
 * nn.Conv2d(Cin, Cout) accept AINP_CONV_BF16 | AINP_CONV_DY16 (host-only). */
int ainp_conv3x3_dy16_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W);
/* 1 if ainp_conv3x3_fwd_ex of this nn.Conv2d(Cin, Cout) accepts AINP_CONV_X16
 * and AINP_CONV_Y16 and its ainp_conv3x3_wgrad_ex accepts AINP_CONV_X16
 * (host-only; with AINP_CONV_BF16). */
int ainp_conv3x3_io16_ok(int64_t N, int Cin, int Cout, int64_t H, int64_t W);

/* ------------------------------------------------------------------------ */
/* BatchNorm2d (training statistics) + ReLU                                   */
/* ------------------------------------------------------------------------ */
/* Reduce the conv epilogue partials to per-channel sums:
 * sums[0:C] = sum y, sums[C:2C] = sum y^2 (double).  Between this and
 * ainp_bn_finalize a data-parallel caller all-reduces `sums` (SyncBN). */
int ainp_bn_stats_reduce(const double* stats, int nparts, double* sums, int C,
                         void* stream);
/* ainp_bn_stats_reduce followed by ainp_bn_finalize (count > 0) in one
 * launch, for a single process (no all-reduce of the sums between them):
 * the same scale / shift / save / running statistics, bit for bit. */
int ainp_bn_reduce_finalize(const double* stats, int nparts, int64_t count, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            float momentum, float eps, float* scale, float* shift,
                            float* save_mean_rstd, int C, void* stream);
/* Finalise batch statistics into the affine form used by the next kernel:
 * scale = gamma*rstd, shift = beta-mean*scale; save_mean_rstd (float[2*C])
 * keeps mean / rstd for the backward; running stats updated in place with
 * momentum and the unbiased variance, as torch.nn.BatchNorm2d in train mode
 * (running_* may both be NULL).  count = elements per channel summed into
 * `sums` (N*H*W, times the world size after an all-reduce); count == 0: the
 * count is read from sums[2*C] (a data-parallel caller appends its local
 * N*H*W to the sums and all-reduces it with them: uneven shards then
 * normalise with the true global count).  ainp_bn_relu_bwd_apply takes count
 * the same way (count == 0: its sums[2*C] holds the forward's global count). */
int ainp_bn_finalize(const double* sums, int64_t count, const float* gamma,
                     const float* beta, float* running_mean,
                     float* running_var, float momentum, float eps,
                     float* scale, float* shift, float* save_mean_rstd, int C,
                     void* stream);
/* Eval-mode affine from running statistics. */
int ainp_bn_eval_affine(const float* gamma, const float* beta,
                        const float* running_mean, const float* running_var,
                        float eps, float* scale, float* shift, int C,
                        void* stream);
/* out = relu(x*scale[c] + shift[c]) over x [N,C,H,W].  If out_ntcf != 0 the
 * result is written as [N, W, C*H] (feature c*H+h at time w): the LSTM input
 * layout produced by model.py:73-74's permute(0,3,1,2).reshape. */
int ainp_bn_relu_apply(const float* x, const float* scale, const float* shift,
                       float* out, int64_t N, int C, int64_t H, int64_t W,
                       int out_ntcf, void* stream);
/* BatchNorm+ReLU backward.  z = relu(y*scale+shift); gz = g*(z>0).
 * Step 1 (reduce): sums[0:C] = sum(gz), sums[C:2C] = sum(gz*xhat) (double),
 *   xhat = (y-mean)*rstd.  workspace: ainp_bn_relu_bwd_workspace(...) bytes.
 *   A data-parallel caller all-reduces `sums` before step 2 (SyncBN).
 * Step 2 (apply): gy = gamma*rstd*(gz - sums0/count - xhat*sums1/count),
 *   written [N,C,H,W]; dgamma = sums1, dbeta = sums0 (float[C], may be NULL).
 * g is [N,C,H,W], or [N,W,C*H] (LSTM input layout) if g_ntcf != 0. */
size_t ainp_bn_relu_bwd_workspace(int64_t N, int C, int64_t H, int64_t W);
int ainp_bn_relu_bwd_reduce(const float* g, const float* y, const float* scale,
                            const float* shift, const float* save_mean_rstd,
                            void* workspace, double* sums, int64_t N, int C,
                            int64_t H, int64_t W, int g_ntcf, void* stream);
int ainp_bn_relu_bwd_apply(const float* g, const float* y, const float* scale,
                           const float* shift, const float* gamma,
                           const float* save_mean_rstd, const double* sums,
                           int64_t count, float* gy, float* dgamma,
                           float* dbeta, int64_t N, int C, int64_t H,
                           int64_t W, int g_ntcf, void* stream);
/* Step 2 with flags: AINP_BN_GY16 writes gy as bf16 (nearest-even, uint16
 * storage) -- the bf16 configuration, whose data / weight gradient kernels
 * round gy to bf16 when staging it (ainp_conv3x3_dgrad_ex / _wgrad_ex with
 * AINP_CONV_DY16 read that storage; see ainp_conv3x3_dy16_ok). */
#define AINP_BN_GY16 1
/* AINP_BN_Y16 (reduce / apply / the bf16 NTCF bridge): the pre-BN input y holds
 * bf16 values (uint16 storage through the float* argument; a forward with
 * AINP_CONV_Y16 wrote it). */
#define AINP_BN_Y16 2
/* Round 5: g, y and gy channel-last ([N][H][W][C], C = 16 / 32 / 64, 16-byte
 * aligned; g_ntcf must be 0) -- the layout the AINP_CONV_XCL / _YCL convs
 * read and write.  AINP_BN_G16 (with AINP_BN_CL): g in bf16 storage. */
#define AINP_BN_CL 4
#define AINP_BN_G16 8
int ainp_bn_relu_bwd_reduce_ex(const float* g, const float* y, const float* scale,
                               const float* shift, const float* save_mean_rstd, void* workspace,
                               double* sums, int64_t N, int C, int64_t H, int64_t W, int g_ntcf,
                               int flags, void* stream);
int ainp_bn_relu_bwd_apply_ex(const float* g, const float* y, const float* scale,
                              const float* shift, const float* gamma,
                              const float* save_mean_rstd, const double* sums,
                              int64_t count, void* gy, float* dgamma, float* dbeta,
                              int64_t N, int C, int64_t H, int64_t W, int g_ntcf, int flags,
                              void* stream);
/* Round 5: ainp_conv3x3_dgrad_ex followed by the step-1 reduce of the
 * BatchNorm+ReLU the data gradient feeds, in one pass where a split-bf16
 * data-gradient kernel serves the pair: its epilogue sums (gz, gz*xhat) of
 * the dx it just computed (y = that BatchNorm's pre-BN input, channel-last,
 * AINP_BN_Y16: bf16 storage), so dx and y are not read again.  dx is written
 * as ainp_conv3x3_dgrad_ex writes it; sums as ainp_bn_relu_bwd_reduce_ex
 * with AINP_BN_CL would (same terms, another fixed summation order).  flags:
 * ainp_conv3x3_dgrad_ex's, AINP_CONV_YCL required; Cin in {16, 32, 64}
 * (the channel-last BatchNorm reduce's instances; others are refused up front);
 * dx / y / scale / shift / save 16-byte aligned.  Pairs without a fused
 * kernel (or AINP_DGRAD_BNR=0) run the two passes.  Replaces the
 * conv-backward + BatchNorm2d-backward pair of autograd on
 * models/CNNBLSTM/model.py:35-60.  workspace:
 * ainp_conv3x3_dgrad_bnr_workspace(...) bytes. */
int64_t ainp_conv3x3_dgrad_bnr_workspace(int64_t N, int Cin, int Cout, int64_t H, int64_t W);
/* Round 6: with dx == NULL, ainp_conv3x3_dgrad_bnr writes only the sums, for
 * Conv2d(16, 1) (dy one channel -> dx 16): its dx is recomputed by
 * ainp_conv3x3_dgrad_bnapply, which forms the data gradient again (the same
 * fma chains) and writes the BatchNorm+ReLU backward apply of it, gy
 * (channel-last [N][H][W][16]; gy16: bf16 nearest-even storage), as
 * ainp_bn_relu_bwd_apply_ex would from that dx and y (fp32 channel-last),
 * with dgamma / dbeta -- dx is never written or read back (decoder.5 ->
 * decoder.6 of models/CNNBLSTM/model.py:57-60).  sums / count as the apply. */
int ainp_conv3x3_dgrad_bnapply(const float* dy, const float* w, const float* y,
                               const float* scale, const float* shift, const float* gamma,
                               const float* save_mean_rstd, const double* sums, int64_t count,
                               void* gy, int gy16, float* dgamma, float* dbeta, int64_t N,
                               int Cin, int Cout, int64_t H, int64_t W, void* stream);
int ainp_conv3x3_dgrad_bnr(const float* dy, const float* w, float* dx, int64_t N, int Cin,
                           int Cout, int64_t H, int64_t W, int flags, const void* y,
                           const float* scale, const float* shift, const float* save_mean_rstd,
                           void* workspace, double* sums, int bn_flags, void* stream);

/* bf16 configuration (BASELINE C3): the encoder's last BN+ReLU writes the
 * layer-0 LSTM input directly as bf16 (nearest-even) in both layouts the
 * bf16-operand GEMMs read: out [N][W][C*H] (the NTCF input, model.py:73-74)
 * and outT [C*H][ld_t] with element (k, n*W + w) (its transpose, the weight
 * gradient's k-contiguous operand).  Needs C*H % 64 == 0, W and ld_t even. */
int ainp_bn_relu_apply_ntcf_bf16(const float* x, const float* scale, const float* shift,
                                 uint16_t* out, uint16_t* outT, int64_t ld_t, int64_t N, int C,
                                 int64_t H, int64_t W, void* stream);
/* Round 5: the same bridge from a channel-last y [N][H][W][64] (AINP_BN_Y16:
 * bf16 storage): out (fp32) and / or out16 (bf16) = relu(y*scale+shift) as
 * [N][W][64*H], outT (bf16) as [64*H][ld_t] (element (k, n*W + w)); NULL
 * outputs are skipped.  With AINP_BN_CL, ainp_bn_relu_bwd_reduce_ex /
 * _apply_ex take g_ntcf = 1 for this block: g [N,W,64*H] fp32, y and gy
 * channel-last. */
int ainp_bn_relu_apply_ntcf_cl(const float* y, const float* scale, const float* shift,
                               float* out, uint16_t* out16, uint16_t* outT, int64_t ld_t,
                               int64_t N, int C, int64_t H, int64_t W, int flags, void* stream);
/* flags: AINP_BN_Y16 (x in bf16 storage) */
int ainp_bn_relu_apply_ntcf_bf16_ex(const float* x, const float* scale, const float* shift,
                                    uint16_t* out, uint16_t* outT, int64_t ld_t, int64_t N,
                                    int C, int64_t H, int64_t W, int flags, void* stream);

/* ------------------------------------------------------------------------ */
/* BLSTM recurrence (one layer, both directions), batch_first                */
/* ------------------------------------------------------------------------ */
/* Replaces the recurrent part of nn.LSTM(bidirectional=True, batch_first)
 * (models/CNNBLSTM/model.py:46-47,77). Gate order i,f,g,o; c'=f*c+i*g;
 * h'=o*tanh(c'); h0=c0=0.
 * zx    [N, T, 8H]  input projections x W_ih^T + b_ih + b_hh; forward
 *       direction in columns [0,4H), reverse direction in [4H,8H)
 * w_hh  host array of 2 device pointers to the [4H, H] recurrent weights
 * h_out [N, T, 2H]  output (forward in [0,H), reverse in [H,2H))
 * gates [N, T, 8H]  saved post-activation gates (needed by the backward)
 * cell  [N, T, 2H]  saved cell states (needed by the backward)
 * H in {32, 64, 128}. */
int ainp_lstm_rec_fwd(const float* zx, const float* const* w_hh, float* h_out,
                      float* gates, float* cell, int64_t N, int64_t T, int H,
                      void* stream);
/* Backward through time: dh_out [N,T,2H] -> dgates [N,T,8H] (gradient of the
 * pre-activation gates, i.e. of zx). */
int ainp_lstm_rec_bwd(const float* dh_out, const float* gates,
                      const float* cell, const float* const* w_hh,
                      float* dgates, int64_t N, int64_t T, int H,
                      void* stream);
/* hprev[n,t,:H] = h_out[n,t-1,:H], hprev[n,t,H:] = h_out[n,t+1,H:] (0 at the
 * sequence start): the right-hand operand of dW_hh = dgates^T * hprev. */
int ainp_lstm_hprev(const float* h_out, float* hprev, int64_t N, int64_t T,
                    int H, void* stream);

/* ------------------------------------------------------------------------ */
/* Tracing: per-phase roctx ranges (data / fwd / bwd / all-reduce / */
/* optimizer) for rocprofv3 --marker-trace.  push returns the nesting depth.  */
/* ------------------------------------------------------------------------ */
int ainp_range_push(const char* name);
int ainp_range_pop(void);
void ainp_mark(const char* name);

/* ------------------------------------------------------------------------ */
/* Loss, reductions, optimizer                                               */
/* ------------------------------------------------------------------------ */
/* CNNBLSTM training loss (models/CNNBLSTM/train.py:70,104):
 *   L = sum | 10^y * m - |target| * m |    (nn.L1Loss(reduction='sum'))
 * y, mask [n] f32; target [n] complex64 (interleaved).
 * loss: double[ainp_l1_pow10_loss_slots(n)], caller-allocated (no zeroing):
 * on completion loss[0] = L, loss[1..] is the per-workgroup partial scratch.
 * Deterministic: fixed-order two-pass reduction, no atomics (bit-reproducible
 * from run to run).  dy (may be NULL): dL/dy * grad_scale. */
int64_t ainp_l1_pow10_loss_slots(int64_t n);
int ainp_l1_pow10_loss(const float* y, const float* mask, const float* target,
                       int64_t n, double* loss, float* dy, float grad_scale,
                       void* stream);
/* out[i] = x[i] * scalar[0] (scalar is a device pointer: scales a gradient
 * by the autograd grad_output without a host sync). */
int ainp_scale_by_dev(const float* x, float* out, int64_t n,
                      const float* scalar, void* stream);
/* out[i] = sum_s x[s*n + i] over nslabs slabs (split-K combine, fixed order). */
int ainp_sum_slabs(const float* x, int64_t nslabs, int64_t n, float* out,
                   void* stream);
/* out[r] = sum_b sum_c x[(b*rows + r)*cols + c] (bias gradient of a layer
 * whose output is [nb, rows, cols]). */
int ainp_rowsum_batched(const float* x, int64_t nb, int64_t rows, int64_t cols,
                        float* out, void* stream);
/* Column sums: out[j] (+)= sum_i x[i*ld + j], i<rows, j<cols.  Row slabs are
 * combined with float atomics, so the summation order can vary run to run;
 * ainp_colsum_slabs + ainp_sum_slabs is the fixed-order form. */
int ainp_colsum(const float* x, int64_t rows, int64_t cols, int64_t ld,
                float* out, int accumulate, void* stream);
/* partial[s*cols + j] = sum of x[i*ld + j] over rows i of slab s (nslabs
 * slabs of ceil(rows/nslabs) rows, fixed order).  Bias gradients of
 * nn.LSTM (models/CNNBLSTM/model.py:46-47) then = ainp_sum_slabs(partial). */
int ainp_colsum_slabs(const float* x, int64_t rows, int64_t cols, int64_t ld,
                      int64_t nslabs, float* partial, void* stream);
/* Multi-tensor Adam with torch.optim.Adam arithmetic (amsgrad=False,
 * maximize=False): m = lerp(m, g, 1-b1); v = b2*v + (1-b2)*g*g;
 * p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps); bc_i = 1 - b_i^step.
 * weight_decay adds wd*p to g first (torch's L2 form).  Host arrays of
 * n_tensors device pointers and element counts; step is 1-based. */
int ainp_adam(float* const* params, const float* const* grads,
              float* const* exp_avg, float* const* exp_avg_sq,
              const int64_t* numel, int n_tensors, double lr, double beta1,
              double beta2, double eps, double weight_decay, int64_t step,
              void* stream);
/* Same with the step counter on the device (HIP-graph capturable, torch's
 * Adam(capturable=True) contract): step_dev (float[1]) is incremented by the
 * launch and the bias corrections are formed from it on the device, in the
 * same double arithmetic as the host form; scalars_dev (float[2]) is scratch.
 * step_dev == NULL: the host `step` is used, as ainp_adam. */
int ainp_adam_ex(float* const* params, const float* const* grads,
                 float* const* exp_avg, float* const* exp_avg_sq,
                 const int64_t* numel, int n_tensors, double lr, double beta1,
                 double beta2, double eps, double weight_decay, int64_t step,
                 float* step_dev, float* scalars_dev, void* stream);

/* ------------------------------------------------------------------------ */
/* (a15-a20) GAN path: PConvUNet, spectral-norm Discriminator, VGG loss      */
/* ------------------------------------------------------------------------ */
/* Generic convolution, implicit GEMM on f32 MFMA (exact fp32).  Replaces:
 *   PartialConv2d.conv + mask_ratio + bias (models/GAN/networks.py:77-96),
 *   the Discriminator's spectral-norm Conv2d + LeakyReLU (networks.py:359-370,
 *   402-405), the frozen VGG19 Conv2d+ReLU (models/GAN/loss.py:21,45-46),
 *   and the torch.cat / nn.Upsample feeding each decoder block
 *   (networks.py:282-298, 306-318): the input is read from two NCHW sources,
 *   channels [0,C0) from x0 (H0 x W0; nearest-resampled to Hin x Win when
 *   smaller, i.e. the x2 Upsample) and [C0,C0+C1) from x1 (H1 x W1 == Hin x Win),
 *   each multiplied by its mask plane m0 / m1 ([N,H0,W0] / [N,H1,W1], NULL = 1).
 * w [Cout][C0+C1][KH][KW] (used by the Cout == 1 path); wt = the same weights
 * k-major from ainp_conv_weight_kmajor (required when Cout > 1; cacheable while
 * w is unchanged); y [N][Cout][Ho][Wo];
 * y = act(conv * (*scale) * ratio[n][oy][ox] + bias[co]); scale / ratio / bias
 * may be NULL.  act: 0 none, 1 ReLU, 2 LeakyReLU(slope), 3 tanh.
 * stats (NULL or double[ainp_conv_gen_stat_parts(...)][2][Cout]): fixed-order
 * per-tile (sum, sumsq) of the value before act, for ainp_bn_stats_reduce.
 * workspace: ainp_conv_gen_workspace(...) bytes (0 = may be NULL): the Cout == 1
 * direct channel-chunked kernel and split-K launches (small tile grids with a
 * long K) keep their partial sums there.  crop_h / crop_w (> 0, Cout == 1
 * only) write only the top-left crop (networks.py:334), else pass 0. */
int ainp_conv_gen_stat_parts(int64_t N, int Cin, int KH, int KW, int Cout, int64_t Ho,
                             int64_t Wo);
size_t ainp_conv_gen_workspace(int64_t N, int Cin, int KH, int KW, int Cout, int64_t Ho,
                               int64_t Wo);
/* wt[k][co] for the implicit GEMM: k runs over source 0 (k = tap*C0 + ci), then
 * source 1 (k = KH*KW*C0 + tap*C1 + ci); wt[k][co] = w[co][ci (+C0)][tap]. */
int ainp_conv_weight_kmajor(const float* w, int Cout, int C0, int C1, int KH, int KW,
                            float* wt, void* stream);
int ainp_conv_gen_fwd(const float* x0, const float* m0, int C0, int H0, int W0,
                      const float* x1, const float* m1, int C1, int H1, int W1,
                      const float* w, const float* wt, const float* bias, const float* ratio,
                      const float* scale, float* y, double* stats, int64_t N,
                      int Cout, int Hin, int Win, int KH, int KW, int stride,
                      int pad, int act, float slope, int crop_h, int crop_w,
                      void* workspace, void* stream);
/* Same with a precision flag: AINP_CONV_BF16 rounds the gathered activations
 * and the weights to bf16 (fp32 accumulation, fp32 epilogue) -- the GAN bf16
 * configurations C4 / C5 (models/GAN/networks.py:63-106,359-405, loss.py). */
int ainp_conv_gen_fwd_ex(const float* x0, const float* m0, int C0, int H0, int W0,
                         const float* x1, const float* m1, int C1, int H1, int W1,
                         const float* w, const float* wt, const float* bias,
                         const float* ratio, const float* scale, float* y, double* stats,
                         int64_t N, int Cout, int Hin, int Win, int KH, int KW, int stride,
                         int pad, int act, float slope, int crop_h, int crop_w, int flags,
                         void* workspace, void* stream);
/* ainp_conv_gen_fwd_ex that also writes y16 (may be NULL; Cout % 8 == 0,
 * 16-byte aligned): the result after the activation as a bf16 (nearest-even)
 * channel-last copy [N][Ho][Wo][Cout], the next conv's channel-last source
 * (what ainp_nchw_to_nhwc16 would write from y).  Only the direct
 * few-input-channel route writes it (one plain source of <= 4 channels,
 * C0*KH*KW <= 160, Cout <= 64, no statistics: the discriminator's first conv
 * on the spectrogram, networks.py:359-373, and VGG19's conv1_1, loss.py:41-51);
 * any other route returns an error when y16 is given. */
int ainp_conv_gen_fwd_out16(const float* x0, const float* m0, int C0, int H0, int W0,
                            const float* x1, const float* m1, int C1, int H1, int W1,
                            const float* w, const float* wt, const float* bias,
                            const float* ratio, const float* scale, float* y, double* stats,
                            int64_t N, int Cout, int Hin, int Win, int KH, int KW, int stride,
                            int pad, int act, float slope, int crop_h, int crop_w, int flags,
                            uint16_t* y16, void* workspace, void* stream);
/* bf16 configurations (C4 / C5), channel-last variant: ainp_nchw_to_nhwc16
 * writes a source x [N][C][H][W] times its mask plane m [N][H][W] (may be
 * NULL) as bf16 (nearest-even) out [N][H][W][C]; ainp_conv_weight_nhwc16
 * writes the weights as bf16 wt16 [Cout][S0 + S1] (k = tap*C0 + ci, then
 * S0 + tap*C1 + ci), where a source of C channels spans S = KK*C k-values,
 * rounded up to a multiple of 32 (zero weights) when C % 32 != 0; such a
 * source is passed expanded per output pixel by ainp_im2col_nhwc16
 * (x [N][C][Hs][Ws] fp32 times its mask plane m, resampled to Hin x Win like
 * source 0 -> bf16 rows [N*Ho*Wo][S], k = tap*C + ci, zero past KK*C); then
 * ainp_conv_gen_fwd_nhwc16 is ainp_conv_gen_fwd_ex(AINP_CONV_BF16) on those
 * operands (same resampling of source 0, ratio / scale / bias / stats /
 * activation epilogue and split-K workspace; no crop, Cout > 1).  16-byte
 * aligned buffers. */
int ainp_nchw_to_nhwc16(const float* x, const float* m, int64_t N, int C, int H, int W,
                        uint16_t* out, void* stream);
int ainp_conv_weight_nhwc16(const float* w, int Cout, int C0, int C1, int KH, int KW,
                            uint16_t* wt16, void* stream);
int ainp_im2col_nhwc16(const float* x, const float* m, int64_t N, int C, int Hs, int Ws, int Hin,
                       int Win, int KH, int KW, int stride, int pad, uint16_t* out, void* stream);
int ainp_conv_gen_fwd_nhwc16(const uint16_t* x0, int C0, int H0, int W0, const uint16_t* x1,
                             int C1, int H1, int W1, const uint16_t* wt16, const float* bias,
                             const float* ratio, const float* scale, float* y, double* stats,
                             int64_t N, int Cout, int Hin, int Win, int KH, int KW, int stride,
                             int pad, int act, float slope, void* workspace, void* stream);
/* ainp_conv_gen_fwd_nhwc16 that also writes y16 (may be NULL): the result
 * after the activation as a bf16 (nearest-even) channel-last copy
 * [N][Ho][Wo][Cout] -- the next conv's channel-last source, written by this
 * epilogue instead of a separate ainp_nchw_to_nhwc16 pass (VGG19 and the
 * discriminator, whose convs have no partial-conv mask;
 * models/GAN/loss.py:41-51, networks.py:352-409). */
int ainp_conv_gen_fwd_nhwc16_ex(const uint16_t* x0, int C0, int H0, int W0, const uint16_t* x1,
                                int C1, int H1, int W1, const uint16_t* wt16, const float* bias,
                                const float* ratio, const float* scale, float* y, double* stats,
                                int64_t N, int Cout, int Hin, int Win, int KH, int KW, int stride,
                                int pad, int act, float slope, uint16_t* y16, void* workspace,
                                void* stream);
/* Main loop of ainp_conv_gen_fwd_nhwc16 (same sums, bit for bit, in every
 * variant): 0 register-staged 128x128 / 64x256 tiles, 1 the same tiles on an
 * LDS-DMA ring, 2 wide tiles (256x128 / 128x256 / 64x256) of 4 waves on a
 * 3-stage LDS-DMA ring with XCD-major workgroup order, 3 the same tiles with 8
 * waves of 64x64 (Cout > 64; variant 0 below; the default).  Returns the
 * previous variant; an out-of-range v only queries.  Initial value: env
 * AINP_CONV16. */
int ainp_conv16_set_variant(int v);
/* PartialConv2d mask update (networks.py:83-104, multi_channel=False):
 * count = C0*window_sum(m0) + C1*window_sum(m1) over the conv's window (masks
 * are planes of integer counts -- 0/1, or a channel sum -- repeated over their
 * channels), ratio = winsize / (count + 1e-8) with winsize = C_in*KH*KW (pass
 * <= 0 for (C0+C1)*KH*KW), newmask = clamp(count, 0, 1); both [N][Ho][Wo]
 * (NULL skips). */
int ainp_pconv_mask(const float* m0, int C0, int H0, int W0, const float* m1, int C1,
                    int H1, int W1, int64_t N, int Hin, int Win, int KH, int KW,
                    int stride, int pad, float winsize, float* ratio, float* newmask,
                    void* stream);
/* PConvUNet input padding (networks.py:255-261): x reflect, mask constant 1,
 * bottom/right to Hp x Wp (pad < size, as F.pad(mode='reflect') requires). */
int ainp_gan_pad_input(const float* x, const float* m, int64_t N, int H, int W,
                       int Hp, int Wp, float* xp, float* mp, void* stream);
/* y = act(y*scale[c] + shift[c]) in place: BatchNorm2d + LeakyReLU of the
 * Encoder/DecoderBlocks (networks.py:149-151, 165-167). */
int ainp_affine_act(float* y, const float* scale, const float* shift, int64_t N, int C,
                    int64_t HW, int act, float slope, void* stream);
/* ainp_affine_act on y [N][C][H][W] and, in the same pass, the bf16
 * configurations' channel-last copy of the result times the mask plane
 * m [N][H][W] (may be NULL): out [N][H][W][C] bf16, exactly what
 * ainp_nchw_to_nhwc16(y, m) gives afterwards (the next PartialConv2d's source). */
int ainp_affine_act_nhwc16(float* y, const float* scale, const float* shift, int64_t N, int C,
                           int H, int W, int act, float slope, const float* m, uint16_t* out,
                           void* stream);
/* ainp_affine_act_nhwc16 with flags: AINP_AFFINE_NO_Y leaves y unchanged (only
 * the channel-last copy is written) for a caller whose consumers all read the
 * copy -- the bf16 U-Net's no-grad forward (networks.py:139-152, 247-345). */
#define AINP_AFFINE_NO_Y 1
int ainp_affine_act_nhwc16_ex(float* y, const float* scale, const float* shift, int64_t N, int C,
                              int H, int W, int act, float slope, const float* m, uint16_t* out,
                              int flags, void* stream);
/* nn.MaxPool2d(2, 2) of VGG19.features (loss.py:21). */
int ainp_maxpool2(const float* x, float* y, int64_t NC, int H, int W, void* stream);
/* ainp_maxpool2 on x [N][C][H][W] that also writes the pooled values' bf16
 * (nearest-even) channel-last copy out [N][H/2][W/2][C] (4-byte aligned): the
 * next VGG19 conv's source (loss.py:41-51), as ainp_nchw_to_nhwc16 would. */
int ainp_maxpool2_nhwc16(const float* x, float* y, int64_t N, int C, int H, int W,
                         uint16_t* out, void* stream);
/* VGGLoss._prepare_input_for_vgg + weights.transforms() (loss.py:65-86,104-106):
 * generated: (x+1)/2; target: clamp(x,0)/(max+1e-6) with the batch max found on
 * the device (max_ws: 1 uint scratch); clamp to [0,1]; antialiased bilinear
 * resize evaluated only at the SxS centre-crop outputs with the separable
 * tables (ry0, rn, rw[S][rtaps]) / (cx0, cn, cw[S][ctaps]) built by the host
 * (torch's _upsample_bilinear2d_aa weights); ImageNet normalisation;
 * out [N,3,S,S].  generated: 1 generated, 0 target (max found here), 2 target
 * whose max max_ws already holds (ainp_vgg_target_max + a MAX all-reduce). */
int ainp_vgg_prep(const float* x, int64_t N, int H, int W, int generated,
                  unsigned int* max_ws, const int* ry0, const int* rn, const float* rw,
                  int rtaps, const int* cx0, const int* cn, const float* cw, int ctaps,
                  int S, float* out, void* stream);
/* Fixed-order reductions (workspace: ainp_reduce_workspace() bytes).
 * absdiff_mean: *out = mean |a-b|  (nn.L1Loss(), loss.py:117,128).
 * bce_logits: *out_mean = mean BCEWithLogits(x, target) (train.py:41-42,355-359),
 *   grad (NULL to skip) = grad_scale * (sigmoid(x) - target).
 * gan_recon_losses: out3 = {Lv, Lh, Lw} of calculate_losses (train.py:49-63). */
size_t ainp_reduce_workspace(void);
int ainp_absdiff_mean(const float* a, const float* b, int64_t n, void* workspace,
                      double* out, void* stream);
int ainp_bce_logits(const float* x, int64_t n, float target, float* grad, float grad_scale,
                    void* workspace, double* out_mean, void* stream);
int ainp_gan_recon_losses(const float* g, const float* o, const float* m, int64_t n,
                          void* workspace, double* out3, void* stream);
/* Data-parallel forms: the raw fp64 sums behind
 * ainp_gan_recon_losses, out5 = [sum|(g-o)m|, sum m, sum|(g-o)(1-m)|, sum(1-m),
 * sum|g-o||o|], to be SUM-all-reduced before the ratios; and the VGG target's
 * batch max (clamp(x,0) bits, loss.py:78) alone, to be MAX-all-reduced and then
 * passed to ainp_vgg_prep with generated == 2. */
int ainp_gan_recon_sums(const float* g, const float* o, const float* m, int64_t n,
                        void* workspace, double* out5, void* stream);
int ainp_vgg_target_max(const float* x, int64_t n, unsigned int* max_ws, void* stream);
/* torch.nn.utils.spectral_norm for nl (<= 8) layers at once (networks.py:
 * 360-361,403-404), W viewed [h][wd]: update != 0 (train-mode forward) runs one
 * power iteration v = normalize(W^T u), u = normalize(W v) in place; always
 * inv_sigma[l] = 1 / (u . W v).  workspace: ainp_sn_workspace(nl, maxdim)
 * bytes, maxdim >= every h and wd. */
size_t ainp_sn_workspace(int nl, int maxdim);
int ainp_sn_power(const float* const* w, float* const* u, float* const* v, const int* h,
                  const int* wd, int nl, float eps, void* workspace, int maxdim,
                  float* inv_sigma, int update, void* stream);
/* Gradient through W = W_orig / sigma with u, v held constant:
 * out = G*inv_sigma - (sum G*W_orig) * inv_sigma^2 * u v^T, G [h][ldg] (its
 * first wd columns are dL/dW); out_bias (may be NULL) = G[:, wd] (the bias
 * gradient computed as the ones-row column of the weight-grad GEMM).
 * workspace: ainp_reduce_workspace() bytes. */
int ainp_sn_weight_grad(const float* G, int ldg, const float* w_orig, const float* u,
                        const float* v, const float* inv_sigma, int h, int wd, void* workspace,
                        float* out, float* out_bias, void* stream);
/* Discriminator backward glue: im2col col[N][C*KH*KW + ones_row][Ho*Wo]
 * (k = ci*KH*KW + tap; ones_row = 1 appends a row of 1.0), its adjoint col2im
 * as a gather (deterministic), LeakyReLU backward from the activation output. */
int ainp_im2col(const float* x, int64_t N, int C, int H, int W, int KH, int KW, int stride,
                int pad, int ones_row, float* col, void* stream);
int ainp_col2im(const float* dcol, int64_t N, int C, int H, int W, int KH, int KW, int stride,
                int pad, float* dx, void* stream);
int ainp_leaky_bwd(const float* g, const float* y, int64_t n, float slope, float* out,
                   void* stream);
/* Row-padded forms (rows of Ho*Wo / P elements stored with stride ldp / ldo,
 * the padding zeroed) so the D weight-gradient GEMM over pixels can use
 * 16-byte loads (ld % 4 == 0). */
int ainp_im2col_ld(const float* x, int64_t N, int C, int H, int W, int KH, int KW, int stride,
                   int pad, int ones_row, int64_t ldp, float* col, void* stream);
int ainp_leaky_bwd_ld(const float* g, const float* y, int64_t rows, int64_t P, float slope,
                      int64_t ldo, float* out, void* stream);
int ainp_col2im_ld(const float* dcol, int64_t N, int C, int H, int W, int KH, int KW, int stride,
                   int pad, int64_t ldp, float* dx, void* stream);
/* ---- Generator backward (opt-in fix_generator_grad; csrc/gan_bwd.hip).
 * The reference's PConvUNet / VGGLoss / calculate_losses are differentiable
 * nn.Modules (networks.py:247-345, loss.py:89-131, train.py:33-88); only its
 * loop's torch.no_grad() (train.py:349-350) keeps G untrained (Q1). */
/* out = LeakyReLU(y * scale[c] + shift[c]) out of place (EncoderBlock /
 * DecoderBlock BatchNorm + activation, networks.py:150-151; the pre-BN y is
 * kept for the backward). */
int ainp_affine_leaky_out(const float* y, const float* scale, const float* shift, int64_t N,
                          int C, int64_t HW, float slope, float* out, void* stream);
/* PartialConv2d's convolved input cat(nearest(x0) * nearest(m0), x1 * m1)
 * [N, C0+C1, Hin, Win] (networks.py:79-82 with the decoder's x2 nearest
 * upsample and torch.cat, networks.py:297-313); m0 / m1 [N, Hs, Ws] planes
 * or NULL, x1 NULL when C1 == 0. */
int ainp_pconv_src_materialize(const float* x0, const float* m0, int64_t N, int C0, int H0,
                               int W0, const float* x1, const float* m1, int C1, int Hin, int Win,
                               float* out, void* stream);
/* Backward of the above for one source (channels [c_off, c_off+C) of dxin,
 * resolution Hs x Ws, Hin % Hs == 0): dxs (+)= ms * block sum of dxin. */
int ainp_pconv_src_grad(const float* dxin, int64_t N, int Cin, int Hin, int Win, int c_off, int C,
                        int Hs, int Ws, const float* ms, float* dxs, int accumulate,
                        void* stream);
/* Activation (+crop) backward of a PartialConv2d output (act 0 none, 1 ReLU,
 * 2 LeakyReLU, 3 Tanh; a = the activation's output, [N, C, gH, gW]): gz [N, C, H*W] =
 * g * act'(a) (zero outside the gH x gW crop; may be NULL), gc [N, C, ldo] =
 * gz * ratio[n][pixel] (ratio may be NULL), rows zero-padded to ldo. */
int ainp_gen_act_bwd(const float* g, int gH, int gW, const float* a, int act, float slope,
                     const float* ratio, int64_t N, int C, int H, int W, int64_t ldo, float* gz,
                     float* gc, void* stream);
/* BatchNorm2d (train mode) + LeakyReLU backward of a generator block
 * (save = [mean | rstd] from ainp_bn_finalize; y the pre-BN conv output):
 * reduce -> sums[0:C] = sum g', sums[C:2C] = sum g' xhat (fixed order, f64;
 * all-reduce them for SyncBN); apply -> gc [N, C, ldo] = dy * ratio (the
 * PartialConv2d window ratio, may be NULL), dgamma, dbeta.  count == 0: the
 * element count is sums[2C] (ainp_bn_stats_reduce's DP form); count == -1:
 * eval mode (save = [running_mean | 1/sqrt(running_var + eps)]). */
size_t ainp_bn_act_bwd_workspace(int64_t N, int C, int64_t P);
int ainp_bn_act_bwd_reduce(const float* ga, const float* y, const float* scale, const float* shift,
                           const float* save, float slope, int64_t N, int C, int64_t P,
                           void* workspace, double* sums, void* stream);
int ainp_bn_act_bwd_apply(const float* ga, const float* y, const float* scale, const float* shift,
                          const float* save, const float* gamma, const double* sums, int64_t count,
                          float slope, const float* ratio, int64_t N, int C, int64_t P,
                          int64_t ldo, float* gc, float* dgamma, float* dbeta, void* stream);
/* nn.MaxPool2d(2, 2) backward (torch's first-maximum rule), g [NC, H/2, W/2]. */
int ainp_maxpool2_bwd(const float* g, const float* x, int64_t NC, int H, int W, float* gx,
                      void* stream);
/* VGG input preparation backward for the generated batch (loss.py:71,79-81 +
 * ImageClassification): g [N, 3, S, S] -> gx [N, 1, H, W] through the
 * normalisation, the x3 repeat, the antialiased resize + crop (the
 * ainp_vgg_prep tables) and clamp((x+1)/2, 0, 1). */
size_t ainp_vgg_prep_bwd_workspace(int64_t N, int W, int S);
int ainp_vgg_prep_bwd(const float* g, const float* x, int64_t N, int H, int W, const int* ry0,
                      const int* rn, const float* rw, int rtaps, const int* cx0, const int* cn,
                      const float* cw, int ctaps, int S, void* workspace, float* gx,
                      void* stream);
/* nn.L1Loss backward: out (+)= (*gscale) * scale * sign(a - b) (gscale: a
 * device float, e.g. autograd's incoming gradient, or NULL = 1). */
int ainp_absdiff_grad(const float* a, const float* b, int64_t n, const float* gscale, float scale,
                      float* out, int accumulate, void* stream);
/* L1 of two Gram batches [B, C, C] backward, symmetrised for bmm(F, F^T):
 * out = (*gscale) * scale * (sign(Ga - Gb) + sign(Ga - Gb)^T). */
int ainp_gram_sign_sym(const float* Ga, const float* Gb, int64_t B, int C, const float* gscale,
                       float scale, float* out, void* stream);
/* calculate_losses' Lv / Lh / Lw (train.py:49-63) backward w.r.t. the
 * generated magnitude, from the forward's sums (ainp_gan_recon_sums, after
 * a DP all-reduce) and the three losses' incoming gradients gout3 (device). */
int ainp_gan_recon_bwd(const float* g, const float* o, const float* m, int64_t n,
                       const double* sums5, const float* gout3, double n_total, float* out,
                       void* stream);
/* out [Cin][Cout][K][K] = w[co][ci] flipped: a stride-1 'same' conv's data
 * gradient as a forward conv (VGG19 input gradient). */
int ainp_conv_weight_flip_t(const float* w, int Cout, int Cin, int K, float* out, void* stream);
/* The Discriminator backward in the bf16 configurations (C4 / C5; the same
 * networks.py:375-409 convs as the row-padded fp32 forms above).
 * ainp_d_prep16: g = sum of nslab slabs [N][C][P] (slab_stride apart; the
 * split-K partials of ainp_dgrad16), times LeakyReLU'(y) when y != NULL
 * (y = the layer's activation output, y > 0 ? 1 : slope), cast to bf16 as
 * gA [C][ldA] (q = n*P + p; zero for N*P <= q < ldA) and, when gT != NULL,
 * gT [N*P][C].  ainp_im2col16: ainp_im2col_ld in bf16 with every image's
 * pixels in one row: col [C*KH*KW (+1 ones row)][ldA], q = n*Ho*Wo + p, zero
 * past N*Ho*Wo (ldA % 8 == 0, 16-byte aligned); the weight gradient is then
 * ainp_gemm_bf16nt(gA, col) over K = ldA.  ainp_dgrad16_weight: the weights
 * w [Cout][Cin][k][k] regrouped for the data gradient, bf16
 * wd [s*s][Cin][Kc], Kc = taps*Cout rounded up to 32 when Cout % 32 != 0,
 * taps = (k/s)^2 (k % s == 0).  ainp_dgrad16: dx [N][Cin][H][W] of the conv
 * (k, stride s, pad) from gT [N][Ho][Wo][Cout] and wd, times *scale (1/sigma;
 * NULL = 1), as stride^2 parity-class implicit GEMMs; nsplit > 1 writes nsplit
 * partial slabs slab_stride apart (summed by ainp_d_prep16 or ainp_sum_slabs). */
int ainp_d_prep16(const float* g, int nslab, int64_t slab_stride, const float* y, float slope,
                  int64_t N, int C, int64_t P, uint16_t* gA, int64_t ldA, uint16_t* gT,
                  void* stream);
int ainp_im2col16(const float* x, int64_t N, int C, int H, int W, int KH, int KW, int stride,
                  int pad, int ones_row, uint16_t* col, int64_t ldA, void* stream);
/* ainp_wgrad16_nhwc: the weight gradient ainp_im2col16 + ainp_gemm_bf16nt
 * compute, [dW | db] = gA . [col ; 1]^T over K = ldA, without materialising
 * the columns: the GEMM's B operand is gathered from the layer input's
 * channel-last bf16 copy x16 [N][H][W][Cin] (Cin % 8 == 0; the copy the
 * forward conv read).  G [nsplit][Cout][Cin*k*k + 1] (column ci*k*k + tap,
 * then the bias), split-K slabs kc apart in K as ainp_gemm_bf16nt's (kc % 64
 * == 0; nsplit 1: kc ignored); bit-identical to the two-call route with the
 * same split. */
int ainp_wgrad16_nhwc(const uint16_t* gA, int64_t ldA, int Cout, const uint16_t* x16, int64_t N,
                      int Cin, int H, int W, int k, int stride, int pad, float* G, int nsplit,
                      int64_t kc, void* stream);
/* ainp_wgrad_cout1: the weight gradient of a Cout = 1 conv (k = 3 or 4; the
 * discriminator's logit conv, networks.py:403-406) straight from the fp32
 * input x [N][Cin][H][W] and g = sum of nslab slabs [N][1][Ho][Wo] (times
 * LeakyReLU'(y) when y != NULL): gw [Cin*k*k + 1] = [dW | db], fp32 products,
 * fixed-order reduction -- replaces ainp_im2col16 + ainp_gemm_bf16nt (a GEMV
 * over materialised columns) for that layer.  ws: ainp_wgrad_cout1_workspace
 * bytes (the per-pixel-slice partial rows). */
int ainp_wgrad_cout1(const float* x, const float* g, int nslab, int64_t slab_stride,
                     const float* y, float slope, int64_t N, int Cin, int H, int W, int k,
                     int stride, int pad, float* gw, float* ws, void* stream);
int64_t ainp_wgrad_cout1_workspace(int Cin, int k);
int ainp_dgrad16_weight(const float* w, int Cout, int Cin, int k, int stride, int pad,
                        uint16_t* wd, void* stream);
int ainp_dgrad16(const uint16_t* gT, int64_t N, int Cout, int Ho, int Wo, const uint16_t* wd,
                 int Cin, int H, int W, int k, int stride, int pad, const float* scale,
                 float* out, int nsplit, int64_t slab_stride, void* stream);
/* ainp_dgrad16 (nsplit 1) followed by ainp_d_prep16 of its dx, in one pass:
 * the data-gradient epilogue multiplies by LeakyReLU'(y) (y [N][Cin][H][W],
 * NULL = none), rounds to bf16 and writes gA [Cin][ldA] (q = n*H*W + pixel,
 * zero for N*H*W <= q < ldA) and, when gTo != NULL, gTo [N*H*W][Cin] -- the
 * next (lower) discriminator layer's two gradient operands, bit for bit what
 * the two calls give, without the fp32 dx round trip.  Cin % 4 == 0,
 * gTo 8-byte aligned. */
int ainp_dgrad16_prep(const uint16_t* gT, int64_t N, int Cout, int Ho, int Wo,
                      const uint16_t* wd, int Cin, int H, int W, int k, int stride, int pad,
                      const float* scale, const float* y, float slope, uint16_t* gA,
                      int64_t ldA, uint16_t* gTo, void* stream);
/* PartialConv2d called with a per-channel mask (networks.py:74-85 when
 * mask.shape[1] == C_in): out = a*b elementwise, and the channel sum of the
 * mask [N,C,HW] -> [N,HW] whose window sum is the mask_conv count. */
int ainp_mul(const float* a, const float* b, int64_t n, float* out, void* stream);
int ainp_channel_sum(const float* m, int64_t N, int C, int64_t HW, float* out, void* stream);

/* ------------------------------------------------------------------------ */
/* (f2) FLAC ingest -- HOST code, host pointers                              */
/* ------------------------------------------------------------------------ */
/* Replaces soundfile/libsndfile behind utils.load_audio -> librosa.load
 * (utils.py:36).  data: the whole file in host memory.  ainp_flac_info parses
 * STREAMINFO (md5: 16 bytes, may be NULL); ainp_flac_decode writes the
 * interleaved signed samples [frames][channels] as int32 (as encoded: scale by
 * 2^-(bps-1) for libsndfile's float), verifying every frame's CRC-8/CRC-16. */
int ainp_flac_info(const uint8_t* data, size_t n, int* sample_rate, int* channels,
                   int* bits_per_sample, int64_t* total_samples, uint8_t* md5);
int ainp_flac_decode(const uint8_t* data, size_t n, int32_t* out, int64_t max_frames,
                     int64_t* n_frames);
/* Writer behind utils.save_audio (utils.py:84-87: soundfile FLAC, PCM_16)
 * for add_gaps.py / pre_process_dataset.py: interleaved signed samples
 * [frames][channels] -> a complete .flac file image in out[0..*out_len)
 * (STREAMINFO with the samples' MD5; 4096-sample blocks; CONSTANT / FIXED
 * 0-4 + partitioned Rice / VERBATIM subframes).  bits 8, 16 or 24.
 * ainp_flac_encode_bound: a sufficient `cap`. */
size_t ainp_flac_encode_bound(int64_t frames, int channels, int bits_per_sample);
int ainp_flac_encode(const int32_t* samples, int64_t frames, int channels, int bits_per_sample,
                     int sample_rate, uint8_t* out, size_t cap, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* AINP_H */
