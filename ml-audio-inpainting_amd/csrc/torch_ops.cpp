// torch_ops.cpp — TORCH_LIBRARY registration of the libainp C ABI.
//
// Every GPU entry point of include/ainp.h is registered as a PyTorch custom
// operator torch.ops.ainp.<name> (the C name without the ainp_ prefix), with
// the same argument meaning: device pointers become Tensors, `stream` becomes
// PyTorch's current HIP stream of the operand's device, dimensions are read
// from the tensor shapes (checked here, on the host, before any launch) where
// the C signature takes them separately.  Operators follow the out= style of
// the C ABI: outputs are caller-allocated mutable arguments (Tensor(a!)), so
// the Python layer (ainp/ops.py) keeps the allocation policy and the caching
// allocator / HIP-graph memory pools own every buffer.  Kernels are
// registered for the CUDA dispatch key (ROCm PyTorch's HIP device), so a CPU
// tensor fails in the dispatcher -- there is no CPU path.
//
// Host-only queries (workspace sizes, stat-part counts) and the FLAC codec
// stay on the plain C ABI (ctypes); they launch nothing.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <optional>
#include <vector>

#include "ainp.h"

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void chk(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "ainp_", what, " failed (", rc, "): ", ainp_last_error());
}

void* stream_of(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

// device tensor of the given dtype (unit-stride rows if contig); returns its pointer
template <typename T = float>
T* dev(const Tensor& t, const char* name, at::ScalarType st = at::kFloat, bool contig = true) {
  TORCH_CHECK(t.defined(), name, " is required");
  TORCH_CHECK(t.is_cuda(), name, " must live on the GPU (ainp has no CPU path), got ",
              t.device());
  TORCH_CHECK(t.scalar_type() == st, name, " must be ", st, ", got ", t.scalar_type());
  TORCH_CHECK(!contig || t.is_contiguous(), name, " must be contiguous");
  return static_cast<T*>(t.data_ptr());
}
template <typename T = float>
T* opt(const OptT& t, const char* name, at::ScalarType st = at::kFloat, bool contig = true) {
  return (t.has_value() && t->defined()) ? dev<T>(*t, name, st, contig) : nullptr;
}
void numel_is(const Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.numel() == n, name, " has ", t.numel(), " elements, expected ", n);
}
void same_device(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(a.device() == b.device(), "operands on different devices: ", a.device(), " vs ",
              b.device());
}
#define GUARD(t) c10::hip::HIPGuardMasqueradingAsCUDA guard_((t).device())

// ------------------------------------------------------------------- STFT
void stft_features(const Tensor& audio, const OptT& clip_index, const Tensor& gap_start,
                   int64_t gap_len, int64_t sample_rate, const Tensor& window, int64_t n_fft,
                   int64_t hop, int64_t n_frames, int64_t mode, const OptT& out0,
                   const OptT& out1, const OptT& out2, const OptT& out3) {
  GUARD(audio);
  TORCH_CHECK(audio.dim() == 2, "audio must be [n_clips, n_samples]");
  const int64_t n_clips = audio.size(0), S = audio.size(1);
  const int32_t* ci = opt<int32_t>(clip_index, "clip_index", at::kInt);
  const int64_t batch = ci ? clip_index->numel() : n_clips;
  numel_is(gap_start, batch, "gap_start");
  numel_is(window, n_fft, "window");
  const int64_t plane = batch * (n_fft / 2 + 1) * n_frames;
  // out1 is complex64 in the CNNBLSTM mode (interleaved re/im floats)
  auto optf = [&](const OptT& t, const char* nm, bool cplx) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    if (cplx) {
      numel_is(*t, plane, nm);
      return reinterpret_cast<float*>(dev<void>(*t, nm, at::kComplexFloat));
    }
    numel_is(*t, plane, nm);
    return dev(*t, nm);
  };
  chk(ainp_stft_features(dev(audio, "audio"), n_clips, S, ci,
                         dev<int64_t>(gap_start, "gap_start", at::kLong), batch, gap_len,
                         sample_rate, dev<double>(window, "window", at::kDouble), (int)n_fft,
                         (int)hop, n_frames, (int)mode, optf(out0, "out0", false),
                         optf(out1, "out1", mode == AINP_FEAT_CNNBLSTM), optf(out2, "out2", false),
                         optf(out3, "out3", false), stream_of(audio)),
      "stft_features");
}

void stft(const Tensor& audio, const Tensor& window, int64_t n_fft, int64_t hop, bool center,
          int64_t n_frames, const Tensor& out) {
  GUARD(audio);
  TORCH_CHECK(audio.dim() == 2, "audio must be [n_signals, n_samples]");
  const bool f64 = audio.scalar_type() == at::kDouble;
  const void* a = f64 ? (const void*)dev<double>(audio, "audio", at::kDouble)
                      : (const void*)dev(audio, "audio");
  void* o = dev<void>(out, "out", f64 ? at::kComplexDouble : at::kComplexFloat);
  numel_is(out, audio.size(0) * (n_fft / 2 + 1) * n_frames, "out");
  numel_is(window, n_fft, "window");
  chk(ainp_stft(a, f64 ? 1 : 0, audio.size(0), audio.size(1),
                dev<double>(window, "window", at::kDouble), (int)n_fft, (int)hop, center ? 1 : 0,
                n_frames, o, stream_of(audio)),
      "stft");
}

void istft(const Tensor& in0, const OptT& in1, int64_t mode, int64_t n_bins, int64_t n_frames,
           const Tensor& window, int64_t n_fft, int64_t hop, bool center, const Tensor& workspace,
           const Tensor& out) {
  GUARD(in0);
  const void* p0;
  const void* p1 = nullptr;
  if (mode == 0) p0 = dev<void>(in0, "spec", at::kComplexFloat);
  else if (mode == 1) p0 = dev<void>(in0, "spec", at::kComplexDouble);
  else {
    p0 = dev(in0, "mag");
    TORCH_CHECK(in1.has_value() && in1->defined(), "istft modes 2/3 need angles / phase");
    p1 = mode == 2 ? (const void*)dev<void>(*in1, "angles", at::kComplexFloat)
                   : (const void*)dev(*in1, "phase");
    numel_is(*in1, in0.numel(), "angles/phase");
  }
  TORCH_CHECK(in0.numel() % (n_bins * n_frames) == 0, "spectrum is not [..., F, T]");
  const int64_t nsig = in0.numel() / (n_bins * n_frames);
  const int64_t full = n_fft + hop * (n_frames - 1);
  numel_is(out, nsig * (center ? full - 2 * (n_fft / 2) : full), "out");
  TORCH_CHECK((size_t)workspace.nbytes() >= ainp_istft_workspace(nsig, n_frames, (int)n_fft),
              "istft workspace too small");
  chk(ainp_istft(p0, p1, (int)mode, nsig, (int)n_bins, n_frames,
                 dev<double>(window, "window", at::kDouble), (int)n_fft, (int)hop, center ? 1 : 0,
                 workspace.data_ptr(), out.data_ptr(), stream_of(in0)),
      "istft");
}

void gl_stft_update(const Tensor& audio, const Tensor& window, int64_t hop, int64_t n_frames,
                    const Tensor& tprev, const Tensor& angles, double momentum, bool first) {
  GUARD(audio);
  TORCH_CHECK(audio.dim() == 2, "audio must be [n_signals, n_samples]");
  const int64_t n = audio.size(0) * 257 * n_frames;
  numel_is(tprev, n, "tprev");
  numel_is(angles, n, "angles");
  numel_is(window, 512, "window");
  chk(ainp_gl_stft_update(dev(audio, "audio"), audio.size(0), audio.size(1),
                          dev<double>(window, "window", at::kDouble), (int)hop, n_frames,
                          (float*)dev<void>(tprev, "tprev", at::kComplexFloat),
                          (float*)dev<void>(angles, "angles", at::kComplexFloat), (float)momentum,
                          first ? 1 : 0, stream_of(audio)),
      "gl_stft_update");
}

void gl_update(const Tensor& rebuilt, const Tensor& tprev, const Tensor& angles, double momentum,
               bool first) {
  GUARD(rebuilt);
  const int64_t n = angles.numel();
  numel_is(rebuilt, n, "rebuilt");
  numel_is(tprev, n, "tprev");
  chk(ainp_gl_update((const float*)dev<void>(rebuilt, "rebuilt", at::kComplexFloat),
                     (float*)dev<void>(tprev, "tprev", at::kComplexFloat),
                     (float*)dev<void>(angles, "angles", at::kComplexFloat), n, (float)momentum,
                     first ? 1 : 0, stream_of(rebuilt)),
      "gl_update");
}

// ------------------------------------------------------------------- GEMM
void gemm(int64_t M, int64_t N, int64_t K, double alpha, at::TensorList A, int64_t sam,
          int64_t sak, int64_t strideA, at::TensorList B, int64_t sbk, int64_t sbn,
          int64_t strideB, double beta, at::TensorList C, int64_t scm, int64_t scn,
          int64_t strideC, const c10::List<OptT>& bias1, const c10::List<OptT>& bias2,
          int64_t nstrided, int64_t ksplit, int64_t flags, const OptT& workspace) {
  const int64_t nptr = (int64_t)A.size();
  TORCH_CHECK(nptr >= 1 && nptr <= 8 && (int64_t)B.size() == nptr && (int64_t)C.size() == nptr,
              "gemm: 1..8 pointer batches with as many A, B and C");
  TORCH_CHECK(bias1.size() == 0 || (int64_t)bias1.size() == nptr, "gemm: bias1 per pointer batch");
  TORCH_CHECK(bias2.size() == 0 || (int64_t)bias2.size() == nptr, "gemm: bias2 per pointer batch");
  GUARD(C[0]);
  const float* pa[8];
  const float* pb[8];
  float* pc[8];
  const float* b1[8];
  const float* b2[8];
  for (int64_t i = 0; i < nptr; ++i) {
    // views are allowed: the pointer carries the view's offset, strides are explicit
    pa[i] = dev(A[i], "A", at::kFloat, false);
    pb[i] = dev(B[i], "B", at::kFloat, false);
    pc[i] = dev(C[i], "C", at::kFloat, false);
    same_device(A[i], C[0]);
    same_device(B[i], C[0]);
    same_device(C[i], C[0]);
    b1[i] = bias1.size() ? opt(bias1.get(i), "bias1") : nullptr;
    b2[i] = bias2.size() ? opt(bias2.get(i), "bias2") : nullptr;
  }
  void* ws = nullptr;
  size_t wsb = 0;
  if (workspace.has_value() && workspace->defined()) {
    ws = dev<void>(*workspace, "workspace", workspace->scalar_type());
    wsb = workspace->nbytes();
  }
  chk(ainp_gemm_f32_ex(M, N, K, (float)alpha, pa, sam, sak, strideA, pb, sbk, sbn, strideB,
                       (float)beta, pc, scm, scn, strideC, bias1.size() ? b1 : nullptr,
                       bias2.size() ? b2 : nullptr, (int)nptr, nstrided, (int)ksplit, (int)flags,
                       ws, wsb, stream_of(C[0])),
      "gemm_f32_ex");
}

// An fp32 tensor's data, or (bf16 = the flag bit is set) a bf16 tensor's uint16
// storage passed through the ABI's float* argument (AINP_CONV_X16 / _Y16 /
// _DY16, AINP_BN_Y16 / _GY16).
const float* f32_or_16(const Tensor& t, const char* name, bool bf16) {
  return bf16 ? reinterpret_cast<const float*>(dev<c10::BFloat16>(t, name, at::kBFloat16))
              : dev(t, name);
}
float* f32_or_16_mut(const Tensor& t, const char* name, bool bf16) {
  return bf16 ? reinterpret_cast<float*>(dev<c10::BFloat16>(t, name, at::kBFloat16))
              : dev(t, name);
}

// ------------------------------------------------------------------- conv3x3
void conv3x3_fwd(const Tensor& x, const Tensor& w, const OptT& bias, const OptT& in_scale,
                 const OptT& in_shift, const Tensor& y, const OptT& stats, int64_t flags) {
  GUARD(x);
  // channel-last activations (AINP_CONV_XCL): x [N,H,W,Cin]
  const bool xcl = flags & AINP_CONV_XCL;
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(1) == x.size(xcl ? 3 : 1) && w.size(2) == 3 &&
                  w.size(3) == 3,
              "conv3x3_fwd: x [N,Cin,H,W] (channel-last: [N,H,W,Cin]), w [Cout,Cin,3,3]");
  const int64_t N = x.size(0), Cin = w.size(1), H = x.size(xcl ? 1 : 2), W = x.size(xcl ? 2 : 3),
                Cout = w.size(0);
  numel_is(y, N * Cout * H * W, "y");
  double* st = opt<double>(stats, "stats", at::kDouble);
  if (st)
    numel_is(*stats,
             ainp_conv3x3_fwd_stat_rows_ex(N, (int)Cin, (int)Cout, H, W, (int)flags) * 2 * Cout,
             "stats");
  chk(ainp_conv3x3_fwd_ex(f32_or_16(x, "x", flags & AINP_CONV_X16), dev(w, "w"),
                          opt(bias, "bias"), opt(in_scale, "in_scale"), opt(in_shift, "in_shift"),
                          f32_or_16_mut(y, "y", flags & AINP_CONV_Y16), st, N, (int)Cin,
                          (int)Cout, H, W, (int)flags, stream_of(x)),
      "conv3x3_fwd_ex");
}

void conv3x3_dgrad(const Tensor& dy, const Tensor& w, const Tensor& dx, int64_t flags) {
  GUARD(dy);
  const bool gcl = flags & AINP_CONV_XCL;   // dy [N,H,W,Cout]
  TORCH_CHECK(dy.dim() == 4 && w.dim() == 4 && w.size(0) == dy.size(gcl ? 3 : 1),
              "conv3x3_dgrad: dy [N,Cout,H,W] (channel-last: [N,H,W,Cout]), w [Cout,Cin,3,3]");
  const int64_t N = dy.size(0), Cout = w.size(0), H = dy.size(gcl ? 1 : 2),
                W = dy.size(gcl ? 2 : 3), Cin = w.size(1);
  numel_is(dx, N * Cin * H * W, "dx");
  const float* dyp = f32_or_16(dy, "dy", flags & AINP_CONV_DY16);
  chk(ainp_conv3x3_dgrad_ex(dyp, dev(w, "w"), dev(dx, "dx"), nullptr, N, (int)Cin,
                            (int)Cout, H, W, (int)flags, stream_of(dy)),
      "conv3x3_dgrad_ex");
}

// dx channel-last [N,H,W,Cin] (AINP_CONV_YCL) + the BatchNorm-backward sums
// of the layer it feeds (y [N,H,W,Cin], AINP_BN_Y16: bf16 storage)
void conv3x3_dgrad_bnr(const Tensor& dy, const Tensor& w, const Tensor& dx, int64_t flags,
                       const Tensor& y, const Tensor& scale, const Tensor& shift,
                       const Tensor& save, const Tensor& workspace, const Tensor& sums,
                       int64_t bn_flags) {
  GUARD(dy);
  const bool gcl = flags & AINP_CONV_XCL;   // dy [N,H,W,Cout]
  TORCH_CHECK(dy.dim() == 4 && w.dim() == 4 && w.size(0) == dy.size(gcl ? 3 : 1),
              "conv3x3_dgrad_bnr: dy [N,Cout,H,W] (channel-last: [N,H,W,Cout]), w [Cout,Cin,3,3]");
  const int64_t N = dy.size(0), Cout = w.size(0), H = dy.size(gcl ? 1 : 2),
                W = dy.size(gcl ? 2 : 3), Cin = w.size(1);
  // an empty dx: the sums only (ainp_conv3x3_dgrad_bnr with dx NULL, round 6)
  const bool nodx = dx.numel() == 0;
  if (!nodx) numel_is(dx, N * Cin * H * W, "dx");
  numel_is(y, N * Cin * H * W, "y");
  // the kernels stage 4*Cin BatchNorm constants (scale, shift, mean, rstd)
  numel_is(scale, Cin, "scale");
  numel_is(shift, Cin, "shift");
  numel_is(save, 2 * Cin, "save");
  for (const Tensor* t : {&w, &dx, &y, &scale, &shift, &save, &workspace, &sums})
    same_device(*t, dy);
  TORCH_CHECK(sums.numel() >= 2 * Cin, "sums needs 2C entries");
  TORCH_CHECK((int64_t)workspace.nbytes() >=
                  ainp_conv3x3_dgrad_bnr_workspace(N, (int)Cin, (int)Cout, H, W),
              "conv3x3_dgrad_bnr workspace too small");
  chk(ainp_conv3x3_dgrad_bnr(f32_or_16(dy, "dy", flags & AINP_CONV_DY16), dev(w, "w"),
                             nodx ? nullptr : dev(dx, "dx"), N, (int)Cin, (int)Cout, H, W,
                             (int)flags,
                             f32_or_16(y, "y", bn_flags & AINP_BN_Y16), dev(scale, "scale"),
                             dev(shift, "shift"), dev(save, "save"), workspace.data_ptr(),
                             dev<double>(sums, "sums", at::kDouble), (int)bn_flags,
                             stream_of(dy)),
      "conv3x3_dgrad_bnr");
}

void conv3x3_wgrad(const Tensor& x, const OptT& in_scale, const OptT& in_shift, const Tensor& dy,
                   const Tensor& dw, const OptT& dbias, const Tensor& workspace, int64_t flags) {
  GUARD(x);
  // channel-last: x [N,H,W,Cin] (AINP_CONV_XCL), dy [N,H,W,Cout] (AINP_CONV_GCL)
  const bool xcl = flags & AINP_CONV_XCL, gcl = flags & AINP_CONV_GCL;
  const int64_t N = x.size(0), Cin = x.size(xcl ? 3 : 1), H = x.size(xcl ? 1 : 2),
                W = x.size(xcl ? 2 : 3), Cout = dy.size(gcl ? 3 : 1);
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dy.size(0) == N && dy.size(gcl ? 1 : 2) == H &&
                  dy.size(gcl ? 2 : 3) == W,
              "conv3x3_wgrad: x [N,Cin,H,W], dy [N,Cout,H,W] (or channel-last [N,H,W,C])");
  numel_is(dw, Cout * Cin * 9, "dw");
  TORCH_CHECK((size_t)workspace.nbytes() >= ainp_conv3x3_wgrad_workspace(N, (int)Cin, (int)Cout, H, W),
              "conv3x3_wgrad workspace too small");
  const float* dyp = f32_or_16(dy, "dy", flags & AINP_CONV_DY16);
  chk(ainp_conv3x3_wgrad_ex(f32_or_16(x, "x", flags & AINP_CONV_X16), opt(in_scale, "in_scale"),
                            opt(in_shift, "in_shift"),
                            dyp, dev(dw, "dw"), opt(dbias, "dbias"),
                            workspace.data_ptr(), N, (int)Cin, (int)Cout, H, W, (int)flags,
                            stream_of(x)),
      "conv3x3_wgrad_ex");
}

// Conv2d(16, 1)'s data gradient through the BatchNorm+ReLU backward apply
// (ainp_conv3x3_dgrad_bnapply): dy [N,1,H,W], y fp32 / gy [N,H,W,16]
void conv3x3_dgrad_bnapply(const Tensor& dy, const Tensor& w, const Tensor& y,
                           const Tensor& scale, const Tensor& shift, const OptT& gamma,
                           const Tensor& save, const Tensor& sums, int64_t count, const Tensor& gy,
                           const Tensor& dgamma, const Tensor& dbeta) {
  GUARD(dy);
  TORCH_CHECK(dy.dim() == 4 && dy.size(1) == 1 && w.dim() == 4 && w.size(0) == 1 &&
                  w.size(1) == 16 && y.dim() == 4 && y.size(3) == 16,
              "conv3x3_dgrad_bnapply: dy [N,1,H,W], w [1,16,3,3], y / gy [N,H,W,16]");
  const int64_t N = dy.size(0), H = dy.size(2), W = dy.size(3);
  numel_is(y, N * H * W * 16, "y");
  numel_is(gy, N * H * W * 16, "gy");
  numel_is(scale, 16, "scale");
  numel_is(shift, 16, "shift");
  numel_is(save, 32, "save");
  numel_is(dgamma, 16, "dgamma");
  numel_is(dbeta, 16, "dbeta");
  TORCH_CHECK(sums.numel() >= 32 && sums.scalar_type() == at::kDouble, "sums: >= 32 doubles");
  for (const Tensor* t : {&w, &y, &scale, &shift, &save, &sums, &gy, &dgamma, &dbeta})
    same_device(*t, dy);
  const bool g16 = gy.scalar_type() == at::kBFloat16;
  TORCH_CHECK(g16 || gy.scalar_type() == at::kFloat, "gy: float32 or bfloat16");
  TORCH_CHECK(gy.is_contiguous(), "gy must be contiguous");
  chk(ainp_conv3x3_dgrad_bnapply(dev(dy, "dy"), dev(w, "w"), dev(y, "y"), dev(scale, "scale"),
                                 dev(shift, "shift"), opt(gamma, "gamma"), dev(save, "save"),
                                 dev<double>(sums, "sums", at::kDouble), count, gy.data_ptr(),
                                 g16 ? 1 : 0, dev(dgamma, "dgamma"), dev(dbeta, "dbeta"), N, 16,
                                 1, H, W, stream_of(dy)),
      "conv3x3_dgrad_bnapply");
}

// the 1 -> 16 weight gradient with the BatchNorm+ReLU backward apply fused
// (ainp_conv3x3_wgrad_bnapply): x [N,1,H,W], g / y [N,H,W,16] fp32
void conv3x3_wgrad_bnapply(const Tensor& x, const OptT& in_scale, const OptT& in_shift,
                           const Tensor& g, const Tensor& y, const Tensor& scale,
                           const Tensor& shift, const OptT& gamma, const Tensor& save,
                           const Tensor& sums, int64_t count, const Tensor& dw,
                           const OptT& dbias, const Tensor& dgamma, const Tensor& dbeta,
                           const Tensor& workspace) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1 && g.dim() == 4 && g.size(3) == 16 &&
                  g.size(0) == x.size(0) && g.size(1) == x.size(2) && g.size(2) == x.size(3),
              "conv3x3_wgrad_bnapply: x [N,1,H,W], g / y [N,H,W,16]");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  numel_is(y, N * H * W * 16, "y");
  numel_is(dw, 16 * 9, "dw");
  numel_is(scale, 16, "scale");
  numel_is(shift, 16, "shift");
  numel_is(save, 32, "save");
  numel_is(dgamma, 16, "dgamma");
  numel_is(dbeta, 16, "dbeta");
  TORCH_CHECK(sums.numel() >= 32 && sums.scalar_type() == at::kDouble, "sums: >= 32 doubles");
  for (const Tensor* t : {&g, &y, &scale, &shift, &save, &sums, &dw, &dgamma, &dbeta, &workspace})
    same_device(*t, x);
  TORCH_CHECK((size_t)workspace.nbytes() >= ainp_conv3x3_wgrad_workspace(N, 1, 16, H, W),
              "conv3x3_wgrad_bnapply workspace too small");
  chk(ainp_conv3x3_wgrad_bnapply(dev(x, "x"), opt(in_scale, "in_scale"), opt(in_shift, "in_shift"),
                                 dev(g, "g"), dev(y, "y"), dev(scale, "scale"),
                                 dev(shift, "shift"), opt(gamma, "gamma"), dev(save, "save"),
                                 dev<double>(sums, "sums", at::kDouble), count, dev(dw, "dw"),
                                 opt(dbias, "dbias"), dev(dgamma, "dgamma"), dev(dbeta, "dbeta"),
                                 workspace.data_ptr(), N, 1, 16, H, W, stream_of(x)),
      "conv3x3_wgrad_bnapply");
}

// ------------------------------------------------------------------- BatchNorm
void bn_stats_reduce(const Tensor& stats, const Tensor& sums, int64_t C) {
  GUARD(stats);
  // [parts, 2C] (conv3x3 epilogue) or [parts, 2, C] (conv_gen): rows of 2C
  TORCH_CHECK(C > 0 && stats.numel() % (2 * C) == 0 && stats.size(-1) * (stats.dim() == 3 ? 2 : 1) == 2 * C,
              "stats must be [parts, 2C] or [parts, 2, C]");
  TORCH_CHECK(sums.numel() >= 2 * C, "sums needs 2C entries");
  chk(ainp_bn_stats_reduce(dev<double>(stats, "stats", at::kDouble), (int)(stats.numel() / (2 * C)),
                           dev<double>(sums, "sums", at::kDouble), (int)C, stream_of(stats)),
      "bn_stats_reduce");
}

void bn_finalize(const Tensor& sums, int64_t count, const OptT& gamma, const OptT& beta,
                 const OptT& running_mean, const OptT& running_var, double momentum, double eps,
                 const Tensor& scale, const Tensor& shift, const Tensor& save) {
  GUARD(sums);
  const int64_t C = scale.numel();
  TORCH_CHECK(sums.numel() >= 2 * C + (count == 0 ? 1 : 0), "sums too short");
  numel_is(shift, C, "shift");
  numel_is(save, 2 * C, "save");
  chk(ainp_bn_finalize(dev<double>(sums, "sums", at::kDouble), count, opt(gamma, "gamma"),
                       opt(beta, "beta"), opt(running_mean, "running_mean"),
                       opt(running_var, "running_var"), (float)momentum, (float)eps,
                       dev(scale, "scale"), dev(shift, "shift"), dev(save, "save"), (int)C,
                       stream_of(sums)),
      "bn_finalize");
}

void bn_reduce_finalize(const Tensor& stats, int64_t count, const OptT& gamma, const OptT& beta,
                        const OptT& running_mean, const OptT& running_var, double momentum,
                        double eps, const Tensor& scale, const Tensor& shift, const Tensor& save) {
  GUARD(stats);
  const int64_t C = scale.numel();
  TORCH_CHECK(C > 0 && stats.numel() % (2 * C) == 0 &&
                  stats.size(-1) * (stats.dim() == 3 ? 2 : 1) == 2 * C,
              "stats must be [parts, 2C] or [parts, 2, C]");
  numel_is(shift, C, "shift");
  numel_is(save, 2 * C, "save");
  chk(ainp_bn_reduce_finalize(dev<double>(stats, "stats", at::kDouble),
                              (int)(stats.numel() / (2 * C)), count, opt(gamma, "gamma"),
                              opt(beta, "beta"), opt(running_mean, "running_mean"),
                              opt(running_var, "running_var"), (float)momentum, (float)eps,
                              dev(scale, "scale"), dev(shift, "shift"), dev(save, "save"),
                              (int)C, stream_of(stats)),
      "bn_reduce_finalize");
}

void bn_eval_affine(const OptT& gamma, const OptT& beta, const Tensor& running_mean,
                    const Tensor& running_var, double eps, const Tensor& scale,
                    const Tensor& shift) {
  GUARD(running_mean);
  const int64_t C = running_mean.numel();
  numel_is(running_var, C, "running_var");
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  chk(ainp_bn_eval_affine(opt(gamma, "gamma"), opt(beta, "beta"), dev(running_mean, "running_mean"),
                          dev(running_var, "running_var"), (float)eps, dev(scale, "scale"),
                          dev(shift, "shift"), (int)C, stream_of(running_mean)),
      "bn_eval_affine");
}

void bn_relu_apply(const Tensor& x, const Tensor& scale, const Tensor& shift, const Tensor& out,
                   bool ntcf) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  numel_is(out, x.numel(), "out");
  chk(ainp_bn_relu_apply(dev(x, "x"), dev(scale, "scale"), dev(shift, "shift"), dev(out, "out"), N,
                         (int)C, H, W, ntcf ? 1 : 0, stream_of(x)),
      "bn_relu_apply");
}

void bn_relu_bwd_reduce(const Tensor& g, const Tensor& y, const Tensor& scale, const Tensor& shift,
                        const Tensor& save, const Tensor& workspace, const Tensor& sums, bool ntcf,
                        int64_t flags) {
  GUARD(y);
  // AINP_BN_CL: y (and g) channel-last [N,H,W,C]; AINP_BN_G16: g bf16 storage
  const bool cl = flags & AINP_BN_CL;
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W] (channel-last: [N,H,W,C])");
  const int64_t N = y.size(0), C = y.size(cl ? 3 : 1), H = y.size(cl ? 1 : 2),
                W = y.size(cl ? 2 : 3);
  numel_is(g, y.numel(), "g");
  TORCH_CHECK(sums.numel() >= 2 * C, "sums needs 2C entries");
  TORCH_CHECK((size_t)workspace.nbytes() >= ainp_bn_relu_bwd_workspace(N, (int)C, H, W),
              "bn_relu_bwd workspace too small");
  chk(ainp_bn_relu_bwd_reduce_ex(f32_or_16(g, "g", flags & AINP_BN_G16),
                                 f32_or_16(y, "y", flags & AINP_BN_Y16),
                                 dev(scale, "scale"), dev(shift, "shift"), dev(save, "save"),
                                 workspace.data_ptr(), dev<double>(sums, "sums", at::kDouble), N,
                                 (int)C, H, W, ntcf ? 1 : 0, (int)flags, stream_of(y)),
      "bn_relu_bwd_reduce_ex");
}

void bn_relu_bwd_apply(const Tensor& g, const Tensor& y, const Tensor& scale, const Tensor& shift,
                       const OptT& gamma, const Tensor& save, const Tensor& sums, int64_t count,
                       const Tensor& gy, const OptT& dgamma, const OptT& dbeta, bool ntcf,
                       int64_t flags) {
  GUARD(y);
  const bool cl = flags & AINP_BN_CL;
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W] (channel-last: [N,H,W,C])");
  const int64_t N = y.size(0), C = y.size(cl ? 3 : 1), H = y.size(cl ? 1 : 2),
                W = y.size(cl ? 2 : 3);
  numel_is(g, y.numel(), "g");
  numel_is(gy, y.numel(), "gy");
  TORCH_CHECK(sums.numel() >= 2 * C + (count == 0 ? 1 : 0), "sums too short");
  // AINP_BN_GY16: gy is bf16 storage
  void* gyp = (flags & AINP_BN_GY16) ? (void*)dev<c10::BFloat16>(gy, "gy", at::kBFloat16)
                                     : (void*)dev(gy, "gy");
  chk(ainp_bn_relu_bwd_apply_ex(f32_or_16(g, "g", flags & AINP_BN_G16),
                                f32_or_16(y, "y", flags & AINP_BN_Y16),
                                dev(scale, "scale"),
                                dev(shift, "shift"), opt(gamma, "gamma"), dev(save, "save"),
                                dev<double>(sums, "sums", at::kDouble), count, gyp,
                                opt(dgamma, "dgamma"), opt(dbeta, "dbeta"), N, (int)C, H, W,
                                ntcf ? 1 : 0, (int)flags, stream_of(y)),
      "bn_relu_bwd_apply_ex");
}

// ------------------------------------------------------------------- BLSTM
void lstm_rec_fwd(const Tensor& zx, const Tensor& whh_f, const Tensor& whh_r, const Tensor& h_out,
                  const OptT& gates, const OptT& cell, int64_t H) {
  GUARD(zx);
  TORCH_CHECK(zx.dim() == 3 && zx.size(2) == 8 * H, "zx must be [N,T,8H]");
  const int64_t N = zx.size(0), T = zx.size(1);
  numel_is(whh_f, 4 * H * H, "whh_f");
  numel_is(whh_r, 4 * H * H, "whh_r");
  numel_is(h_out, N * T * 2 * H, "h_out");
  float* gp = opt(gates, "gates");
  float* cp = opt(cell, "cell");
  if (gp) numel_is(*gates, N * T * 8 * H, "gates");
  if (cp) numel_is(*cell, N * T * 2 * H, "cell");
  const float* w[2] = {dev(whh_f, "whh_f"), dev(whh_r, "whh_r")};
  chk(ainp_lstm_rec_fwd(dev(zx, "zx"), w, dev(h_out, "h_out"), gp, cp, N, T, (int)H, stream_of(zx)),
      "lstm_rec_fwd");
}

void lstm_rec_bwd(const Tensor& dh_out, const Tensor& gates, const Tensor& cell,
                  const Tensor& whh_f, const Tensor& whh_r, const Tensor& dgates, int64_t H) {
  GUARD(dh_out);
  TORCH_CHECK(dh_out.dim() == 3 && dh_out.size(2) == 2 * H, "dh_out must be [N,T,2H]");
  const int64_t N = dh_out.size(0), T = dh_out.size(1);
  numel_is(gates, N * T * 8 * H, "gates");
  numel_is(cell, N * T * 2 * H, "cell");
  numel_is(dgates, N * T * 8 * H, "dgates");
  numel_is(whh_f, 4 * H * H, "whh_f");
  numel_is(whh_r, 4 * H * H, "whh_r");
  const float* w[2] = {dev(whh_f, "whh_f"), dev(whh_r, "whh_r")};
  chk(ainp_lstm_rec_bwd(dev(dh_out, "dh_out"), dev(gates, "gates"), dev(cell, "cell"), w,
                        dev(dgates, "dgates"), N, T, (int)H, stream_of(dh_out)),
      "lstm_rec_bwd");
}

void lstm_hprev(const Tensor& h_out, const Tensor& hprev, int64_t H) {
  GUARD(h_out);
  TORCH_CHECK(h_out.dim() == 3 && h_out.size(2) == 2 * H, "h_out must be [N,T,2H]");
  numel_is(hprev, h_out.numel(), "hprev");
  chk(ainp_lstm_hprev(dev(h_out, "h_out"), dev(hprev, "hprev"), h_out.size(0), h_out.size(1),
                      (int)H, stream_of(h_out)),
      "lstm_hprev");
}

// ------------------------------------------------------------------- loss / reductions / Adam
void l1_pow10_loss(const Tensor& y, const Tensor& mask, const Tensor& target, const Tensor& loss,
                   const OptT& dy, double grad_scale) {
  GUARD(y);
  const int64_t n = y.numel();
  numel_is(mask, n, "mask");
  numel_is(target, n, "target");
  float* d = opt(dy, "dy");
  if (d) numel_is(*dy, n, "dy");
  TORCH_CHECK(loss.numel() >= ainp_l1_pow10_loss_slots(n),
              "l1_pow10_loss: loss needs ainp_l1_pow10_loss_slots(n) doubles");
  chk(ainp_l1_pow10_loss(dev(y, "y"), dev(mask, "mask"),
                         (const float*)dev<void>(target, "target", at::kComplexFloat), n,
                         dev<double>(loss, "loss", at::kDouble), d, (float)grad_scale,
                         stream_of(y)),
      "l1_pow10_loss");
}

void scale_by_dev(const Tensor& x, const Tensor& out, const Tensor& scalar) {
  GUARD(x);
  numel_is(out, x.numel(), "out");
  chk(ainp_scale_by_dev(dev(x, "x"), dev(out, "out"), x.numel(), dev(scalar, "scalar"),
                        stream_of(x)),
      "scale_by_dev");
}

void sum_slabs(const Tensor& x, int64_t nslabs, int64_t n, const Tensor& out) {
  GUARD(x);
  TORCH_CHECK(x.numel() >= nslabs * n && out.numel() >= n, "sum_slabs: extents");
  chk(ainp_sum_slabs(dev(x, "x", at::kFloat, false), nslabs, n, dev(out, "out", at::kFloat, false),
                     stream_of(x)),
      "sum_slabs");
}

void rowsum_batched(const Tensor& x, const Tensor& out) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 3, "x must be [nb, rows, cols]");
  numel_is(out, x.size(1), "out");
  chk(ainp_rowsum_batched(dev(x, "x"), x.size(0), x.size(1), x.size(2), dev(out, "out"),
                          stream_of(x)),
      "rowsum_batched");
}

void colsum(const Tensor& x, int64_t rows, int64_t cols, int64_t ld, const Tensor& out,
            bool accumulate) {
  GUARD(x);
  TORCH_CHECK(out.numel() >= cols, "colsum: out too short");
  chk(ainp_colsum(dev(x, "x", at::kFloat, false), rows, cols, ld, dev(out, "out", at::kFloat, false),
                  accumulate ? 1 : 0, stream_of(x)),
      "colsum");
}

void colsum_slabs(const Tensor& x, int64_t rows, int64_t cols, int64_t ld, int64_t nslabs,
                  const Tensor& partial) {
  GUARD(x);
  numel_is(partial, nslabs * cols, "partial");
  chk(ainp_colsum_slabs(dev(x, "x", at::kFloat, false), rows, cols, ld, nslabs,
                        dev(partial, "partial"), stream_of(x)),
      "colsum_slabs");
}

void adam(at::TensorList params, at::TensorList grads, at::TensorList exp_avg,
          at::TensorList exp_avg_sq, double lr, double beta1, double beta2, double eps,
          double weight_decay, int64_t step, const OptT& step_dev, const OptT& scalars_dev) {
  const size_t n = params.size();
  if (n == 0) return;
  TORCH_CHECK(grads.size() == n && exp_avg.size() == n && exp_avg_sq.size() == n,
              "adam: params, grads, exp_avg, exp_avg_sq differ in length");
  GUARD(params[0]);
  std::vector<float*> p(n), m(n), v(n);
  std::vector<const float*> g(n);
  std::vector<int64_t> ne(n);
  for (size_t i = 0; i < n; ++i) {
    p[i] = dev(params[i], "param");
    g[i] = dev(grads[i], "grad");
    m[i] = dev(exp_avg[i], "exp_avg");
    v[i] = dev(exp_avg_sq[i], "exp_avg_sq");
    ne[i] = params[i].numel();
    numel_is(grads[i], ne[i], "grad");
    numel_is(exp_avg[i], ne[i], "exp_avg");
    numel_is(exp_avg_sq[i], ne[i], "exp_avg_sq");
    same_device(params[i], params[0]);
  }
  float* sd = opt(step_dev, "step_dev");
  float* sc = opt(scalars_dev, "scalars_dev");
  chk(ainp_adam_ex(p.data(), g.data(), m.data(), v.data(), ne.data(), (int)n, lr, beta1, beta2,
                   eps, weight_decay, step, sd, sc, stream_of(params[0])),
      "adam_ex");
}

// ------------------------------------------------------------------- GAN
void conv_weight_kmajor(const Tensor& w, int64_t C0, int64_t C1, const Tensor& wt) {
  GUARD(w);
  TORCH_CHECK(w.dim() == 4 && w.size(1) == C0 + C1, "w must be [Cout, C0+C1, KH, KW]");
  numel_is(wt, w.numel(), "wt");
  chk(ainp_conv_weight_kmajor(dev(w, "w"), (int)w.size(0), (int)C0, (int)C1, (int)w.size(2),
                              (int)w.size(3), dev(wt, "wt"), stream_of(w)),
      "conv_weight_kmajor");
}

uint16_t* bf16p(const Tensor& t, const char* name, bool contig);

void conv_gen_fwd(const Tensor& x0, const OptT& m0, const OptT& x1, const OptT& m1,
                  const Tensor& w, const OptT& wt, const OptT& bias, const OptT& ratio,
                  const OptT& scale, const Tensor& y, const OptT& stats, int64_t Hin, int64_t Win,
                  int64_t stride, int64_t pad, int64_t act, double slope, int64_t crop_h,
                  int64_t crop_w, int64_t flags, const OptT& workspace, const OptT& y16) {
  GUARD(x0);
  TORCH_CHECK(x0.dim() == 4 && w.dim() == 4, "conv_gen: x0 [N,C0,H0,W0], w [Cout,Cin,KH,KW]");
  const int64_t N = x0.size(0), C0 = x0.size(1), H0 = x0.size(2), W0 = x0.size(3);
  int64_t C1 = 0, H1 = 0, W1 = 0;
  const float* px1 = opt(x1, "x1");
  if (px1) {
    TORCH_CHECK(x1->dim() == 4 && x1->size(0) == N, "x1 must be [N,C1,H1,W1]");
    C1 = x1->size(1);
    H1 = x1->size(2);
    W1 = x1->size(3);
  }
  const int64_t Cout = w.size(0), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(w.size(1) == C0 + C1, "conv_gen: weight expects ", w.size(1),
              " input channels, sources give ", C0 + C1);
  const float* pm0 = opt(m0, "m0");
  const float* pm1 = opt(m1, "m1");
  if (pm0) numel_is(*m0, N * H0 * W0, "m0");
  if (pm1) numel_is(*m1, N * H1 * W1, "m1");
  const int64_t Ho = (Hin + 2 * pad - KH) / stride + 1, Wo = (Win + 2 * pad - KW) / stride + 1;
  if (Cout == 1 && crop_h > 0) numel_is(y, N * crop_h * crop_w, "y");
  else numel_is(y, N * Cout * Ho * Wo, "y");
  const float* pwt = opt(wt, "wt");
  TORCH_CHECK(Cout == 1 || pwt, "conv_gen: Cout > 1 needs the k-major weights wt");
  double* st = opt<double>(stats, "stats", at::kDouble);
  if (st)
    numel_is(*stats,
             (int64_t)ainp_conv_gen_stat_parts(N, (int)(C0 + C1), (int)KH, (int)KW, (int)Cout, Ho, Wo) *
                 2 * Cout,
             "stats");
  const size_t need = ainp_conv_gen_workspace(N, (int)(C0 + C1), (int)KH, (int)KW, (int)Cout,
                                              (Cout == 1 && crop_h > 0) ? crop_h : Ho,
                                              (Cout == 1 && crop_w > 0) ? crop_w : Wo);
  void* ws = nullptr;
  if (workspace.has_value() && workspace->defined()) {
    ws = dev<void>(*workspace, "workspace", workspace->scalar_type());
    TORCH_CHECK((size_t)workspace->nbytes() >= need, "conv_gen workspace too small");
  } else {
    TORCH_CHECK(need == 0, "conv_gen needs a workspace of ", need, " bytes");
  }
  uint16_t* o16 = nullptr;
  if (y16.has_value() && y16->defined()) {
    numel_is(*y16, N * Cout * Ho * Wo, "y16");
    o16 = bf16p(*y16, "y16", true);
  }
  chk(ainp_conv_gen_fwd_out16(dev(x0, "x0"), pm0, (int)C0, (int)H0, (int)W0, px1, pm1, (int)C1,
                              (int)H1, (int)W1, dev(w, "w"), pwt, opt(bias, "bias"),
                              opt(ratio, "ratio"), opt(scale, "scale"), dev(y, "y"), st, N,
                              (int)Cout, (int)Hin, (int)Win, (int)KH, (int)KW, (int)stride,
                              (int)pad, (int)act, (float)slope, (int)crop_h, (int)crop_w,
                              (int)flags, o16, ws, stream_of(x0)),
      "conv_gen_fwd_out16");
}

void pconv_mask(const Tensor& m0, int64_t C0, const OptT& m1, int64_t C1, int64_t N, int64_t Hin,
                int64_t Win, int64_t k, int64_t stride, int64_t pad, double winsize,
                const OptT& ratio, const OptT& newmask) {
  GUARD(m0);
  TORCH_CHECK(m0.dim() >= 2, "m0 must be [..., H, W]");
  const int64_t H0 = m0.size(-2), W0 = m0.size(-1);
  numel_is(m0, N * H0 * W0, "m0");
  const float* p1 = opt(m1, "m1");
  int64_t H1 = 0, W1 = 0;
  if (p1) {
    H1 = m1->size(-2);
    W1 = m1->size(-1);
    numel_is(*m1, N * H1 * W1, "m1");
  }
  const int64_t Ho = (Hin + 2 * pad - k) / stride + 1, Wo = (Win + 2 * pad - k) / stride + 1;
  float* pr = opt(ratio, "ratio");
  float* pn = opt(newmask, "newmask");
  if (pr) numel_is(*ratio, N * Ho * Wo, "ratio");
  if (pn) numel_is(*newmask, N * Ho * Wo, "newmask");
  chk(ainp_pconv_mask(dev(m0, "m0"), (int)C0, (int)H0, (int)W0, p1, (int)C1, (int)H1, (int)W1, N,
                      (int)Hin, (int)Win, (int)k, (int)k, (int)stride, (int)pad, (float)winsize, pr,
                      pn, stream_of(m0)),
      "pconv_mask");
}

void gan_pad_input(const Tensor& x, const Tensor& m, const Tensor& xp, const Tensor& mp) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4 && xp.dim() == 3, "x [N,1,H,W], xp [N,Hp,Wp]");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3), Hp = xp.size(1), Wp = xp.size(2);
  numel_is(m, N * H * W, "mask");
  numel_is(mp, N * Hp * Wp, "mp");
  chk(ainp_gan_pad_input(dev(x, "x"), dev(m, "mask"), N, (int)H, (int)W, (int)Hp, (int)Wp,
                         dev(xp, "xp"), dev(mp, "mp"), stream_of(x)),
      "gan_pad_input");
}

void affine_act(const Tensor& y, const Tensor& scale, const Tensor& shift, int64_t act,
                double slope) {
  GUARD(y);
  TORCH_CHECK(y.dim() >= 2, "y must be [N, C, ...]");
  const int64_t N = y.size(0), C = y.size(1);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  chk(ainp_affine_act(dev(y, "y"), dev(scale, "scale"), dev(shift, "shift"), N, (int)C,
                      y.numel() / (N * C), (int)act, (float)slope, stream_of(y)),
      "affine_act");
}

void maxpool2(const Tensor& x, const Tensor& y, const OptT& out16) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  numel_is(y, x.size(0) * x.size(1) * (x.size(2) / 2) * (x.size(3) / 2), "y");
  if (out16.has_value() && out16->defined()) {
    numel_is(*out16, y.numel(), "out16");
    chk(ainp_maxpool2_nhwc16(dev(x, "x"), dev(y, "y"), x.size(0), (int)x.size(1),
                             (int)x.size(2), (int)x.size(3), bf16p(*out16, "out16", true),
                             stream_of(x)),
        "maxpool2_nhwc16");
    return;
  }
  chk(ainp_maxpool2(dev(x, "x"), dev(y, "y"), x.size(0) * x.size(1), (int)x.size(2),
                    (int)x.size(3), stream_of(x)),
      "maxpool2");
}

void check_reduce_ws(const Tensor& ws) {
  TORCH_CHECK((size_t)ws.nbytes() >= ainp_reduce_workspace(), "reduction workspace too small");
}

void absdiff_mean(const Tensor& a, const Tensor& b, const Tensor& workspace, const Tensor& out) {
  GUARD(a);
  numel_is(b, a.numel(), "b");
  check_reduce_ws(workspace);
  chk(ainp_absdiff_mean(dev(a, "a"), dev(b, "b"), a.numel(), workspace.data_ptr(),
                        dev<double>(out, "out", at::kDouble), stream_of(a)),
      "absdiff_mean");
}

void bce_logits(const Tensor& x, double target, const OptT& grad, double grad_scale,
                const Tensor& workspace, const Tensor& out) {
  GUARD(x);
  float* gp = opt(grad, "grad");
  if (gp) numel_is(*grad, x.numel(), "grad");
  check_reduce_ws(workspace);
  chk(ainp_bce_logits(dev(x, "logits"), x.numel(), (float)target, gp, (float)grad_scale,
                      workspace.data_ptr(), dev<double>(out, "out", at::kDouble), stream_of(x)),
      "bce_logits");
}

void gan_recon_losses(const Tensor& g, const Tensor& o, const Tensor& m, const Tensor& workspace,
                      const Tensor& out) {
  GUARD(g);
  numel_is(o, g.numel(), "original");
  numel_is(m, g.numel(), "mask");
  numel_is(out, 3, "out");
  check_reduce_ws(workspace);
  chk(ainp_gan_recon_losses(dev(g, "generated"), dev(o, "original"), dev(m, "mask"), g.numel(),
                            workspace.data_ptr(), dev<double>(out, "out", at::kDouble),
                            stream_of(g)),
      "gan_recon_losses");
}

void gan_recon_sums(const Tensor& g, const Tensor& o, const Tensor& m, const Tensor& workspace,
                    const Tensor& out) {
  GUARD(g);
  numel_is(o, g.numel(), "original");
  numel_is(m, g.numel(), "mask");
  numel_is(out, 5, "out");
  check_reduce_ws(workspace);
  chk(ainp_gan_recon_sums(dev(g, "generated"), dev(o, "original"), dev(m, "mask"), g.numel(),
                          workspace.data_ptr(), dev<double>(out, "out", at::kDouble),
                          stream_of(g)),
      "gan_recon_sums");
}

void vgg_target_max(const Tensor& x, const Tensor& max_ws) {
  GUARD(x);
  chk(ainp_vgg_target_max(dev(x, "x"), x.numel(),
                          (unsigned int*)dev<int32_t>(max_ws, "max_ws", at::kInt), stream_of(x)),
      "vgg_target_max");
}

void vgg_prep(const Tensor& x, int64_t generated, const Tensor& max_ws, const Tensor& ry0,
              const Tensor& rn, const Tensor& rw, const Tensor& cx0, const Tensor& cn,
              const Tensor& cw, int64_t S, const Tensor& out) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,1,H,W]");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  numel_is(out, N * 3 * S * S, "out");
  TORCH_CHECK(rw.dim() == 2 && cw.dim() == 2 && rw.size(0) == S && cw.size(0) == S,
              "vgg_prep: weight tables [S, taps]");
  numel_is(ry0, S, "ry0");
  numel_is(rn, S, "rn");
  numel_is(cx0, S, "cx0");
  numel_is(cn, S, "cn");
  chk(ainp_vgg_prep(dev(x, "x"), N, (int)H, (int)W, (int)generated,
                    (unsigned int*)dev<int32_t>(max_ws, "max_ws", at::kInt),
                    dev<int32_t>(ry0, "ry0", at::kInt), dev<int32_t>(rn, "rn", at::kInt),
                    dev(rw, "rw"), (int)rw.size(1), dev<int32_t>(cx0, "cx0", at::kInt),
                    dev<int32_t>(cn, "cn", at::kInt), dev(cw, "cw"), (int)cw.size(1), (int)S,
                    dev(out, "out"), stream_of(x)),
      "vgg_prep");
}

void sn_power(at::TensorList w, at::TensorList u, at::TensorList v, double eps,
              const Tensor& workspace, const Tensor& inv_sigma, bool update) {
  const size_t nl = w.size();
  TORCH_CHECK(nl >= 1 && nl <= 8 && u.size() == nl && v.size() == nl, "sn_power: 1..8 layers");
  GUARD(w[0]);
  std::vector<const float*> pw(nl);
  std::vector<float*> pu(nl), pv(nl);
  std::vector<int> h(nl), wd(nl);
  int maxdim = 0;
  for (size_t i = 0; i < nl; ++i) {
    pw[i] = dev(w[i], "weight");
    pu[i] = dev(u[i], "u");
    pv[i] = dev(v[i], "v");
    h[i] = (int)w[i].size(0);
    wd[i] = (int)(w[i].numel() / w[i].size(0));
    numel_is(u[i], h[i], "u");
    numel_is(v[i], wd[i], "v");
    maxdim = std::max(maxdim, std::max(h[i], wd[i]));
  }
  numel_is(inv_sigma, (int64_t)nl, "inv_sigma");
  TORCH_CHECK((size_t)workspace.nbytes() >= ainp_sn_workspace((int)nl, maxdim),
              "sn workspace too small");
  chk(ainp_sn_power(pw.data(), pu.data(), pv.data(), h.data(), wd.data(), (int)nl, (float)eps,
                    workspace.data_ptr(), maxdim, dev(inv_sigma, "inv_sigma"), update ? 1 : 0,
                    stream_of(w[0])),
      "sn_power");
}

void sn_weight_grad(const Tensor& G, const Tensor& w_orig, const Tensor& u, const Tensor& v,
                    const Tensor& inv_sigma, const Tensor& workspace, const Tensor& out,
                    const OptT& out_bias) {
  GUARD(G);
  const int64_t h = w_orig.size(0), wd = w_orig.numel() / h;
  TORCH_CHECK(G.dim() == 2 && G.size(0) == h && G.size(1) >= wd, "G must be [h, ldg >= wd]");
  numel_is(out, w_orig.numel(), "out");
  numel_is(u, h, "u");
  numel_is(v, wd, "v");
  float* ob = opt(out_bias, "out_bias");
  if (ob) {
    numel_is(*out_bias, h, "out_bias");
    TORCH_CHECK(G.size(1) > wd, "the bias gradient needs the ones-row column of G");
  }
  check_reduce_ws(workspace);
  chk(ainp_sn_weight_grad(dev(G, "G"), (int)G.size(1), dev(w_orig, "w_orig"), dev(u, "u"),
                          dev(v, "v"), dev(inv_sigma, "inv_sigma", at::kFloat, false), (int)h,
                          (int)wd, workspace.data_ptr(), dev(out, "out"), ob, stream_of(G)),
      "sn_weight_grad");
}

void im2col_ld(const Tensor& x, int64_t k, int64_t stride, int64_t pad, bool ones_row, int64_t ldp,
               const Tensor& col) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  TORCH_CHECK(ldp >= Ho * Wo, "ldp < Ho*Wo");
  numel_is(col, N * (C * k * k + (ones_row ? 1 : 0)) * ldp, "col");
  chk(ainp_im2col_ld(dev(x, "x"), N, (int)C, (int)H, (int)W, (int)k, (int)k, (int)stride, (int)pad,
                     ones_row ? 1 : 0, ldp, dev(col, "col"), stream_of(x)),
      "im2col_ld");
}

void col2im_ld(const Tensor& dcol, int64_t k, int64_t stride, int64_t pad, const Tensor& dx) {
  GUARD(dcol);
  TORCH_CHECK(dx.dim() == 4 && dcol.dim() == 3, "dcol [N, C*k*k, ldp], dx [N,C,H,W]");
  const int64_t N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  const int64_t ldp = dcol.size(2);
  TORCH_CHECK(dcol.size(0) == N && dcol.size(1) >= C * k * k && ldp >= Ho * Wo,
              "col2im: dcol shape");
  chk(ainp_col2im_ld(dev(dcol, "dcol"), N, (int)C, (int)H, (int)W, (int)k, (int)k, (int)stride,
                     (int)pad, ldp, dev(dx, "dx"), stream_of(dcol)),
      "col2im_ld");
}

void leaky_bwd(const Tensor& g, const Tensor& y, double slope, const Tensor& out) {
  GUARD(g);
  numel_is(y, g.numel(), "y");
  numel_is(out, g.numel(), "out");
  chk(ainp_leaky_bwd(dev(g, "g"), dev(y, "y"), g.numel(), (float)slope, dev(out, "out"),
                     stream_of(g)),
      "leaky_bwd");
}

void leaky_bwd_ld(const Tensor& g, const Tensor& y, int64_t rows, double slope, int64_t ldo,
                  const Tensor& out) {
  GUARD(g);
  TORCH_CHECK(rows > 0 && g.numel() % rows == 0, "leaky_bwd_ld: rows");
  const int64_t P = g.numel() / rows;
  TORCH_CHECK(ldo >= P, "ldo < P");
  numel_is(y, g.numel(), "y");
  numel_is(out, rows * ldo, "out");
  chk(ainp_leaky_bwd_ld(dev(g, "g"), dev(y, "y"), rows, P, (float)slope, ldo, dev(out, "out"),
                        stream_of(g)),
      "leaky_bwd_ld");
}

void mul(const Tensor& a, const Tensor& b, const Tensor& out) {
  GUARD(a);
  numel_is(b, a.numel(), "b");
  numel_is(out, a.numel(), "out");
  chk(ainp_mul(dev(a, "a"), dev(b, "b"), a.numel(), dev(out, "out"), stream_of(a)), "mul");
}

void channel_sum(const Tensor& m, const Tensor& out) {
  GUARD(m);
  TORCH_CHECK(m.dim() == 4, "mask must be [N,C,H,W]");
  const int64_t N = m.size(0), C = m.size(1), HW = m.size(2) * m.size(3);
  numel_is(out, N * HW, "out");
  chk(ainp_channel_sum(dev(m, "mask"), N, (int)C, HW, dev(out, "out"), stream_of(m)),
      "channel_sum");
}


// ------------------------------------------------------------------- bf16 GEMM operands
uint16_t* bf16p(const Tensor& t, const char* name, bool contig = true) {
  return reinterpret_cast<uint16_t*>(dev<void>(t, name, at::kBFloat16, contig));
}

// Round 5: the bridge from a channel-last y [N,H,W,64]; any of out (fp32
// [N,W,64*H]), out16 (bf16, same), outT (bf16 [64*H, >= N*W]) may be absent.
void bn_relu_apply_ntcf_cl(const Tensor& y, const Tensor& scale, const Tensor& shift,
                           const OptT& out, const OptT& out16, const OptT& outT, int64_t flags) {
  GUARD(y);
  TORCH_CHECK(y.dim() == 4, "y must be channel-last [N,H,W,C]");
  const int64_t N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  float* o = nullptr;
  if (out.has_value() && out->defined()) {
    numel_is(*out, y.numel(), "out");
    o = dev(*out, "out");
  }
  uint16_t* o16 = nullptr;
  if (out16.has_value() && out16->defined()) {
    numel_is(*out16, y.numel(), "out16");
    o16 = bf16p(*out16, "out16");
  }
  uint16_t* oT = nullptr;
  int64_t ld_t = 0;
  if (outT.has_value() && outT->defined()) {
    TORCH_CHECK(outT->dim() == 2 && outT->size(0) == C * H && outT->size(1) >= N * W &&
                    outT->stride(1) == 1,
                "outT must be [C*H, >= N*W] with contiguous rows");
    oT = bf16p(*outT, "outT", false);
    ld_t = outT->stride(0);
  }
  chk(ainp_bn_relu_apply_ntcf_cl(f32_or_16(y, "y", flags & AINP_BN_Y16), dev(scale, "scale"),
                                 dev(shift, "shift"), o, o16, oT, ld_t, N, (int)C, H, W,
                                 (int)flags, stream_of(y)),
      "bn_relu_apply_ntcf_cl");
}

void bn_relu_apply_ntcf_bf16(const Tensor& x, const Tensor& scale, const Tensor& shift,
                             const Tensor& out, const Tensor& outT, int64_t flags) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  numel_is(out, x.numel(), "out");
  TORCH_CHECK(outT.dim() == 2 && outT.size(0) == C * H && outT.size(1) >= N * W,
              "outT must be [C*H, >= N*W]");
  TORCH_CHECK(outT.stride(1) == 1, "outT rows must be contiguous");
  chk(ainp_bn_relu_apply_ntcf_bf16_ex(f32_or_16(x, "x", flags & AINP_BN_Y16), dev(scale, "scale"),
                                      dev(shift, "shift"), bf16p(out, "out"),
                                      bf16p(outT, "outT", false), outT.stride(0), N, (int)C, H, W,
                                      (int)flags, stream_of(x)),
      "bn_relu_apply_ntcf_bf16_ex");
}

// Split-column bias of the NT GEMMs: bias_a1/a2 cover columns [0, nsplit),
// bias_b1/b2 columns [nsplit, N); every bias given must have that many entries.
void check_nt_bias(const OptT& a1, const OptT& a2, const OptT& b1, const OptT& b2,
                   int64_t nsplit, int64_t N, const char* op) {
  const bool any = (a1.has_value() && a1->defined()) || (a2.has_value() && a2->defined()) ||
                   (b1.has_value() && b1->defined()) || (b2.has_value() && b2->defined());
  if (!any) return;
  TORCH_CHECK(nsplit >= 0 && nsplit <= N, op, ": bias_nsplit must be in [0, N]");
  if (a1.has_value() && a1->defined()) numel_is(*a1, nsplit, "bias_a1");
  if (a2.has_value() && a2->defined()) numel_is(*a2, nsplit, "bias_a2");
  if (b1.has_value() && b1->defined()) numel_is(*b1, N - nsplit, "bias_b1");
  if (b2.has_value() && b2->defined()) numel_is(*b2, N - nsplit, "bias_b2");
}

// ainp_gemm_bf16nt_multi: problem q = A[q] [M, >=K] (or k-major [>=K, >=M]),
// B[q] [N, >=K] (or k-major [>=K, >=N]) (bf16, unit-stride rows), C[q] [M, N] or
// split-K slabs [nsplit, M, N]; ints[5q .. 5q+4] = K, nsplit, kc, a_kmajor, b_kmajor.
void gemm_bf16nt_multi(const std::vector<Tensor>& A, const std::vector<Tensor>& B,
                       const std::vector<Tensor>& C, const std::vector<int64_t>& ints) {
  const int64_t np = (int64_t)C.size();
  TORCH_CHECK(np >= 1 && np <= 3 && (int64_t)A.size() == np && (int64_t)B.size() == np &&
                  (int64_t)ints.size() == 5 * np,
              "gemm_bf16nt_multi: 1..3 problems (A, B, C each, 5 ints)");
  GUARD(C[0]);
  std::vector<ainp_bf16_problem> pr(np);
  for (int64_t q = 0; q < np; ++q) {
    const int64_t K = ints[5 * q], nsplit = ints[5 * q + 1], kc = ints[5 * q + 2];
    const bool akm = ints[5 * q + 3] != 0, bkm = ints[5 * q + 4] != 0;
    const Tensor &a = A[q], &b = B[q], &c = C[q];
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1,
                "gemm_bf16nt_multi: 2-D operands with unit-stride rows");
    TORCH_CHECK((c.dim() == 2 && nsplit == 1) || (c.dim() == 3 && c.size(0) == nsplit),
                "gemm_bf16nt_multi: C [M, N] or split-K slabs [nsplit, M, N]");
    TORCH_CHECK(c.stride(-1) == 1, "gemm_bf16nt_multi: C rows must be unit-stride");
    const int64_t M = c.size(-2), N = c.size(-1);
    TORCH_CHECK(akm ? (a.size(0) >= K && a.size(1) == M) : (a.size(0) == M && a.size(1) >= K),
                "gemm_bf16nt_multi: A must be [M, >=K] (or k-major [>=K, M])");
    TORCH_CHECK(bkm ? (b.size(0) >= K && b.size(1) == N) : (b.size(0) == N && b.size(1) >= K),
                "gemm_bf16nt_multi: B must be [N, >=K] (or k-major [>=K, N])");
    same_device(a, C[0]);
    same_device(b, C[0]);
    same_device(c, C[0]);
    ainp_bf16_problem& p = pr[q];
    p.A = bf16p(a, "A", false);
    p.lda = a.stride(0);
    p.B = bf16p(b, "B", false);
    p.ldb = b.stride(0);
    p.C = dev(c, "C", at::kFloat, false);
    p.ldc = c.stride(-2);
    p.M = M; p.N = N; p.K = K;
    p.nsplit = (int)nsplit; p.kc = kc;
    p.strideC = c.dim() == 3 ? c.stride(0) : 0;
    p.a_kmajor = akm ? 1 : 0;
    p.b_kmajor = bkm ? 1 : 0;
  }
  chk(ainp_gemm_bf16nt_multi(pr.data(), (int)np, stream_of(C[0])), "gemm_bf16nt_multi");
}

void gemm_bf16nt(const Tensor& A, const Tensor& B, const Tensor& C, int64_t K,
                 const OptT& bias_a1, const OptT& bias_a2, const OptT& bias_b1,
                 const OptT& bias_b2, int64_t bias_nsplit, int64_t nsplit, int64_t kc) {
  GUARD(C);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1,
              "gemm_bf16nt: A [M, >=K], B [N, >=K] with unit-stride rows");
  TORCH_CHECK(A.size(1) >= K && B.size(1) >= K, "gemm_bf16nt: K exceeds the operand rows");
  const int64_t M = A.size(0), N = B.size(0);
  TORCH_CHECK((C.dim() == 2 && nsplit == 1) || (C.dim() == 3 && C.size(0) == nsplit),
              "gemm_bf16nt: C [M, N] or split-K slabs [nsplit, M, N]");
  TORCH_CHECK(C.size(-2) == M && C.size(-1) == N && C.stride(-1) == 1, "gemm_bf16nt: C shape");
  same_device(A, C);
  same_device(B, C);
  check_nt_bias(bias_a1, bias_a2, bias_b1, bias_b2, bias_nsplit, N, "gemm_bf16nt");
  chk(ainp_gemm_bf16nt(M, N, K, bf16p(A, "A", false), A.stride(0), bf16p(B, "B", false),
                       B.stride(0), dev(C, "C", at::kFloat, false), C.stride(-2),
                       opt(bias_a1, "bias_a1"), opt(bias_a2, "bias_a2"), opt(bias_b1, "bias_b1"),
                       opt(bias_b2, "bias_b2"), bias_nsplit, (int)nsplit, kc,
                       C.dim() == 3 ? C.stride(0) : 0, stream_of(C)),
      "gemm_bf16nt");
}

void gemm_x6nt_256(const Tensor& A, const Tensor& B1, const Tensor& B2, const Tensor& C,
                   const OptT& bias_a1, const OptT& bias_a2, const OptT& bias_b1,
                   const OptT& bias_b2, int64_t bias_nsplit, int64_t nsplit, int64_t kc) {
  GUARD(C);
  TORCH_CHECK(A.dim() == 2 && B1.dim() == 2 && B2.dim() == 2 && A.stride(1) == 1 &&
                  B1.stride(1) == 1 && B2.stride(1) == 1 && B1.stride(0) == B2.stride(0),
              "gemm_x6nt_256: A [M, K], B1 [N1, K], B2 [N2, K] with unit-stride rows");
  const int64_t M = A.size(0), K = A.size(1), N1 = B1.size(0), N = N1 + B2.size(0);
  TORCH_CHECK(B1.size(1) == K && B2.size(1) == K, "gemm_x6nt_256: operand K mismatch");
  TORCH_CHECK((C.dim() == 2 && nsplit == 1) || (C.dim() == 3 && C.size(0) == nsplit),
              "gemm_x6nt_256: C [M, N] or split-K slabs [nsplit, M, N]");
  TORCH_CHECK(C.size(-2) == M && C.size(-1) == N && C.stride(-1) == 1, "gemm_x6nt_256: C shape");
  same_device(A, C);
  same_device(B1, C);
  same_device(B2, C);
  check_nt_bias(bias_a1, bias_a2, bias_b1, bias_b2, bias_nsplit, N, "gemm_x6nt_256");
  chk(ainp_gemm_x6nt_256(M, N, K, dev(A, "A", at::kFloat, false), A.stride(0),
                         dev(B1, "B1", at::kFloat, false), dev(B2, "B2", at::kFloat, false),
                         B1.stride(0), N1, dev(C, "C", at::kFloat, false), C.stride(-2),
                         opt(bias_a1, "bias_a1"), opt(bias_a2, "bias_a2"), opt(bias_b1, "bias_b1"),
                         opt(bias_b2, "bias_b2"), bias_nsplit, (int)nsplit, kc,
                         C.dim() == 3 ? C.stride(0) : 0, stream_of(C)),
      "gemm_x6nt_256");
}

// ainp_gemm_x6_multi: per problem q, ins[8q .. 8q+7] = A, A2, B, B2, bias_a1,
// bias_a2, bias_b1, bias_b2 (optional), outs[2q], outs[2q+1] = C, C2 (C2 with
// no elements = none), ints[16q .. 16q+15] = a_ksplit, a_kmajor, b_nsplit,
// b_ksplit, b_kmajor, c_msplit, bias_nsplit, M, N, K, nsplit, kc, strideC,
// lda, ldb, ldc.  Every operand extent is checked against its tensor.
void gemm_x6_multi(const std::vector<std::optional<Tensor>>& ins, const std::vector<Tensor>& outs,
                   const std::vector<int64_t>& ints) {
  const int64_t np = (int64_t)outs.size() / 2;
  TORCH_CHECK(np >= 1 && np <= 3 && (int64_t)ins.size() == 8 * np && (int64_t)ints.size() == 16 * np,
              "gemm_x6_multi: 1..3 problems of 8 inputs, 2 outputs, 16 ints");
  GUARD(outs[0]);
  std::vector<ainp_x6_problem> pr(np);
  auto fp = [&](const std::optional<Tensor>& t, const char* nm) -> const float* {
    if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat, nm, " must be a float32 GPU tensor");
    same_device(*t, outs[0]);
    return t->data_ptr<float>();
  };
  // an operand of R rows x Kx cols (k-major or not) with leading dim ld must fit t
  auto fits = [](const std::optional<Tensor>& t, bool km, int64_t R, int64_t Kx, int64_t ld,
                 const char* nm) {
    if (!t.has_value() || !t->defined() || t->numel() == 0) return;
    TORCH_CHECK(t->is_contiguous() || t->dim() == 2, nm, ": contiguous or 2-D strided");
    const int64_t need = km ? (Kx - 1) * ld + R : (R - 1) * ld + Kx;
    const int64_t have = t->dim() == 2 && !t->is_contiguous()
                             ? (t->size(0) - 1) * t->stride(0) + t->size(1) : t->numel();
    TORCH_CHECK(R > 0 && Kx > 0 && need <= have, nm, " is too small for its extent (", need,
                " > ", have, ")");
  };
  for (int64_t q = 0; q < np; ++q) {
    const int64_t* v = ints.data() + 16 * q;
    const auto* in = ins.data() + 8 * q;
    ainp_x6_problem& p = pr[q];
    p.a_ksplit = v[0]; p.a_kmajor = (int)v[1]; p.b_nsplit = v[2]; p.b_ksplit = v[3];
    p.b_kmajor = (int)v[4]; p.c_msplit = v[5]; p.bias_nsplit = v[6];
    p.M = v[7]; p.N = v[8]; p.K = v[9]; p.nsplit = (int)v[10]; p.kc = v[11]; p.strideC = v[12];
    p.lda = v[13]; p.ldb = v[14]; p.ldc = v[15];
    p.A = fp(in[0], "A"); p.A2 = fp(in[1], "A2"); p.B = fp(in[2], "B"); p.B2 = fp(in[3], "B2");
    p.bias_a1 = fp(in[4], "bias_a1"); p.bias_a2 = fp(in[5], "bias_a2");
    p.bias_b1 = fp(in[6], "bias_b1"); p.bias_b2 = fp(in[7], "bias_b2");
    const Tensor& C = outs[2 * q];
    const Tensor& C2 = outs[2 * q + 1];
    p.C = const_cast<float*>(fp(C, "C"));
    p.C2 = const_cast<float*>(fp(C2, "C2"));
    TORCH_CHECK(p.A && p.B && p.C, "gemm_x6_multi: A, B, C are required");
    const bool a2 = p.A2 != nullptr, b2 = p.B2 != nullptr, c2 = p.C2 != nullptr;
    TORCH_CHECK(!a2 || (p.a_ksplit > 0 && p.a_ksplit < p.K), "a_ksplit out of range");
    TORCH_CHECK(!c2 || (p.c_msplit > 0 && p.c_msplit < p.M), "c_msplit out of range");
    TORCH_CHECK(!b2 || (p.b_ksplit > 0 ? p.b_ksplit < p.K : (p.b_nsplit > 0 && p.b_nsplit < p.N)),
                "B split out of range");
    fits(in[0], p.a_kmajor, p.M, a2 ? p.a_ksplit : p.K, p.lda, "A");
    if (a2) fits(in[1], p.a_kmajor, p.M, p.K - p.a_ksplit, p.lda, "A2");
    const bool bk = b2 && p.b_ksplit > 0;
    const int64_t nb1 = (b2 && !bk) ? p.b_nsplit : p.N;
    fits(in[2], p.b_kmajor, nb1, bk ? p.b_ksplit : p.K, p.ldb, "B");
    if (b2) fits(in[3], p.b_kmajor, bk ? p.N : p.N - p.b_nsplit, bk ? p.K - p.b_ksplit : p.K,
                 p.ldb, "B2");
    const int64_t ns = p.nsplit < 1 ? 1 : p.nsplit;
    const int64_t m1 = c2 ? p.c_msplit : p.M;
    fits(C, false, (ns - 1) * (p.strideC / std::max<int64_t>(p.ldc, 1)) + m1, p.N, p.ldc, "C");
    if (c2) fits(C2, false, (ns - 1) * (p.strideC / std::max<int64_t>(p.ldc, 1)) + p.M - m1, p.N,
                 p.ldc, "C2");
    if (p.bias_a1) numel_is(*in[4], p.bias_nsplit, "bias_a1");
    if (p.bias_a2) numel_is(*in[5], p.bias_nsplit, "bias_a2");
    if (p.bias_b1) numel_is(*in[6], p.N - p.bias_nsplit, "bias_b1");
    if (p.bias_b2) numel_is(*in[7], p.N - p.bias_nsplit, "bias_b2");
  }
  chk(ainp_gemm_x6_multi(pr.data(), (int)np, stream_of(outs[0])), "gemm_x6_multi");
}

void transpose_f32(const Tensor& x, const Tensor& outT) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be 2-D with unit-stride rows");
  TORCH_CHECK(outT.dim() == 2 && outT.size(0) == x.size(1) && outT.size(1) == x.size(0) &&
                  outT.stride(1) == 1,
              "outT must be [C, R] with unit-stride rows");
  same_device(x, outT);
  chk(ainp_transpose_f32(dev(x, "x", at::kFloat, false), x.size(0), x.size(1), x.stride(0),
                         dev(outT, "outT", at::kFloat, false), outT.stride(0), stream_of(x)),
      "transpose_f32");
}

void cast_bf16_t(const Tensor& x, const OptT& out, const OptT& outT) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be 2-D with unit-stride rows");
  const int64_t R = x.size(0), Cc = x.size(1);
  uint16_t* o = nullptr;
  uint16_t* ot = nullptr;
  int64_t ldo = Cc, ldt = R;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(out->dim() == 2 && out->size(0) == R && out->size(1) == Cc && out->stride(1) == 1,
                "out must be [R, C]");
    o = bf16p(*out, "out", false);
    ldo = out->stride(0);
  }
  if (outT.has_value() && outT->defined()) {
    TORCH_CHECK(outT->dim() == 2 && outT->size(0) == Cc && outT->size(1) == R &&
                    outT->stride(1) == 1,
                "outT must be [C, R]");
    ot = bf16p(*outT, "outT", false);
    ldt = outT->stride(0);
  }
  chk(ainp_cast_bf16_t(dev(x, "x", at::kFloat, false), R, Cc, x.stride(0), o, ldo, ot, ldt,
                       stream_of(x)),
      "cast_bf16_t");
}

// k-values one source contributes to an nhwc16 weight row (gan.hip nhwc16_seg)
int64_t nhwc16_seg(int64_t C, int64_t KK) { return (C % 32) ? (KK * C + 31) / 32 * 32 : KK * C; }

void nchw_to_nhwc16(const Tensor& x, const OptT& m, const Tensor& out) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const float* mp = opt(m, "mask");
  if (mp) numel_is(*m, N * H * W, "mask");
  numel_is(out, x.numel(), "out");
  chk(ainp_nchw_to_nhwc16(dev(x, "x"), mp, N, (int)C, (int)H, (int)W, bf16p(out, "out"),
                          stream_of(x)),
      "nchw_to_nhwc16");
}

void affine_act_nhwc16(const Tensor& y, const Tensor& scale, const Tensor& shift, int64_t act,
                       double slope, const OptT& m, const Tensor& out, bool keep_y) {
  GUARD(y);
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W]");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  const float* mp = opt(m, "mask");
  if (mp) numel_is(*m, N * H * W, "mask");
  numel_is(out, y.numel(), "out");
  chk(ainp_affine_act_nhwc16_ex(dev(y, "y"), dev(scale, "scale"), dev(shift, "shift"), N,
                                (int)C, (int)H, (int)W, (int)act, (float)slope, mp,
                                bf16p(out, "out", true), keep_y ? 0 : AINP_AFFINE_NO_Y,
                                stream_of(y)),
      "affine_act_nhwc16");
}

void im2col_nhwc16(const Tensor& x, const OptT& m, int64_t Hin, int64_t Win, int64_t KH,
                   int64_t KW, int64_t stride, int64_t pad, const Tensor& out) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,Hs,Ws]");
  const int64_t N = x.size(0), C = x.size(1), Hs = x.size(2), Ws = x.size(3);
  const float* mp = opt(m, "mask");
  if (mp) numel_is(*m, N * Hs * Ws, "mask");
  const int64_t Ho = (Hin + 2 * pad - KH) / stride + 1, Wo = (Win + 2 * pad - KW) / stride + 1;
  numel_is(out, N * Ho * Wo * nhwc16_seg(C, KH * KW), "out");
  chk(ainp_im2col_nhwc16(dev(x, "x"), mp, N, (int)C, (int)Hs, (int)Ws, (int)Hin, (int)Win, (int)KH,
                         (int)KW, (int)stride, (int)pad, bf16p(out, "out"), stream_of(x)),
      "im2col_nhwc16");
}

void conv_weight_nhwc16(const Tensor& w, int64_t C0, int64_t C1, const Tensor& wt16) {
  GUARD(w);
  TORCH_CHECK(w.dim() == 4 && w.size(1) == C0 + C1, "w must be [Cout, C0+C1, KH, KW]");
  const int64_t KK = w.size(2) * w.size(3);
  numel_is(wt16, w.size(0) * (nhwc16_seg(C0, KK) + nhwc16_seg(C1, KK)), "wt16");
  chk(ainp_conv_weight_nhwc16(dev(w, "w"), (int)w.size(0), (int)C0, (int)C1, (int)w.size(2),
                              (int)w.size(3), bf16p(wt16, "wt16"), stream_of(w)),
      "conv_weight_nhwc16");
}

void conv_gen_fwd_nhwc16(const Tensor& x0, const OptT& x1, const Tensor& wt16, int64_t Cout,
                         int64_t KH, int64_t KW, const OptT& bias, const OptT& ratio,
                         const OptT& scale, const Tensor& y, const OptT& stats, int64_t Hin,
                         int64_t Win, int64_t stride, int64_t pad, int64_t act, double slope,
                         const OptT& workspace, at::IntArrayRef dims, const OptT& y16) {
  // dims = [N, C0, H0, W0, C1, H1, W1] (required when a source has C % 32 != 0:
  // such a source is the [N*Ho*Wo, seg] rows of im2col_nhwc16), else from the
  // [N, Hs, Ws, C] channel-last tensors
  GUARD(x0);
  const int64_t Ho = (Hin + 2 * pad - KH) / stride + 1, Wo = (Win + 2 * pad - KW) / stride + 1;
  int64_t N, C0, H0, W0, C1 = 0, H1 = 0, W1 = 0;
  const uint16_t* p1 = nullptr;
  if (!dims.empty()) {
    TORCH_CHECK(dims.size() == 7, "dims must be [N, C0, H0, W0, C1, H1, W1]");
    N = dims[0]; C0 = dims[1]; H0 = dims[2]; W0 = dims[3]; C1 = dims[4]; H1 = dims[5]; W1 = dims[6];
  } else {
    TORCH_CHECK(x0.dim() == 4, "x0 must be [N,H0,W0,C0] (channel-last bf16)");
    N = x0.size(0); H0 = x0.size(1); W0 = x0.size(2); C0 = x0.size(3);
    if (x1.has_value() && x1->defined()) {
      TORCH_CHECK(x1->dim() == 4 && x1->size(0) == N, "x1 must be [N,H1,W1,C1]");
      H1 = x1->size(1); W1 = x1->size(2); C1 = x1->size(3);
    }
  }
  auto src_numel = [&](int64_t C, int64_t H, int64_t W) {
    return (C % 32) ? N * Ho * Wo * nhwc16_seg(C, KH * KW) : N * H * W * C;
  };
  numel_is(x0, src_numel(C0, H0, W0), "x0");
  if (C1 > 0) {
    TORCH_CHECK(x1.has_value() && x1->defined(), "x1 required for C1 > 0");
    numel_is(*x1, src_numel(C1, H1, W1), "x1");
    p1 = bf16p(*x1, "x1");
  }
  numel_is(wt16, Cout * (nhwc16_seg(C0, KH * KW) + nhwc16_seg(C1, KH * KW)), "wt16");
  numel_is(y, N * Cout * Ho * Wo, "y");
  double* st = opt<double>(stats, "stats", at::kDouble);
  if (st)
    numel_is(*stats,
             (int64_t)ainp_conv_gen_stat_parts(N, (int)(C0 + C1), (int)KH, (int)KW, (int)Cout, Ho, Wo) *
                 2 * Cout,
             "stats");
  const size_t need = ainp_conv_gen_workspace(N, (int)(C0 + C1), (int)KH, (int)KW, (int)Cout, Ho, Wo);
  void* ws = nullptr;
  if (workspace.has_value() && workspace->defined()) {
    ws = dev<void>(*workspace, "workspace", workspace->scalar_type());
    TORCH_CHECK((size_t)workspace->nbytes() >= need, "conv_gen workspace too small");
  } else {
    TORCH_CHECK(need == 0, "conv_gen needs a workspace of ", need, " bytes");
  }
  uint16_t* o16 = nullptr;
  if (y16.has_value() && y16->defined()) {
    numel_is(*y16, N * Cout * Ho * Wo, "y16");
    o16 = bf16p(*y16, "y16");
  }
  chk(ainp_conv_gen_fwd_nhwc16_ex(bf16p(x0, "x0"), (int)C0, (int)H0, (int)W0, p1, (int)C1,
                                  (int)H1, (int)W1, bf16p(wt16, "wt16"), opt(bias, "bias"),
                                  opt(ratio, "ratio"), opt(scale, "scale"), dev(y, "y"), st, N,
                                  (int)Cout, (int)Hin, (int)Win, (int)KH, (int)KW, (int)stride,
                                  (int)pad, (int)act, (float)slope, o16, ws, stream_of(x0)),
      "conv_gen_fwd_nhwc16");
}

void d_prep16(const Tensor& g, int64_t nslab, const OptT& y, double slope, int64_t N, int64_t C,
              int64_t P, const Tensor& gA, const OptT& gT) {
  GUARD(g);
  numel_is(g, nslab * N * C * P, "g");
  const float* yp = opt(y, "y");
  if (yp) numel_is(*y, N * C * P, "y");
  TORCH_CHECK(gA.dim() == 2 && gA.size(0) == C && gA.size(1) >= N * P, "gA must be [C, >= N*P]");
  uint16_t* gt = nullptr;
  if (gT.has_value() && gT->defined()) {
    numel_is(*gT, N * P * C, "gT");
    gt = bf16p(*gT, "gT");
  }
  chk(ainp_d_prep16(dev(g, "g"), (int)nslab, N * C * P, yp, (float)slope, N, (int)C, P,
                    bf16p(gA, "gA"), gA.size(1), gt, stream_of(g)),
      "d_prep16");
}

void wgrad_cout1(const Tensor& x, const Tensor& g, int64_t nslab, const OptT& y, double slope,
                 int64_t k, int64_t stride, int64_t pad, const Tensor& gw, const Tensor& ws) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  numel_is(g, nslab * N * Ho * Wo, "g");
  const float* yp = opt(y, "y");
  if (yp) numel_is(*y, N * Ho * Wo, "y");
  numel_is(gw, C * k * k + 1, "gw");
  TORCH_CHECK(ws.numel() * 4 >= ainp_wgrad_cout1_workspace((int)C, (int)k),
              "ws smaller than ainp_wgrad_cout1_workspace");
  chk(ainp_wgrad_cout1(dev(x, "x"), dev(g, "g"), (int)nslab, N * Ho * Wo, yp, (float)slope, N,
                       (int)C, (int)H, (int)W, (int)k, (int)stride, (int)pad, dev(gw, "gw"),
                       dev(ws, "ws"), stream_of(x)),
      "wgrad_cout1");
}

void im2col16(const Tensor& x, int64_t k, int64_t stride, int64_t pad, bool ones_row,
              const Tensor& col) {
  GUARD(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(col.dim() == 2 && col.size(0) == C * k * k + (ones_row ? 1 : 0),
              "col must be [C*k*k (+1), ldA]");
  chk(ainp_im2col16(dev(x, "x"), N, (int)C, (int)H, (int)W, (int)k, (int)k, (int)stride, (int)pad,
                    ones_row ? 1 : 0, bf16p(col, "col"), col.size(1), stream_of(x)),
      "im2col16");
}

void dgrad16_weight(const Tensor& w, int64_t stride, int64_t pad, const Tensor& wd) {
  GUARD(w);
  TORCH_CHECK(w.dim() == 4 && w.size(2) == w.size(3), "w must be [Cout, Cin, k, k]");
  const int64_t Cout = w.size(0), Cin = w.size(1), k = w.size(2);
  TORCH_CHECK(stride >= 1 && k % stride == 0, "dgrad16_weight: k % stride == 0");
  const int64_t nt = k / stride;
  numel_is(wd, stride * stride * Cin * nhwc16_seg(Cout, nt * nt), "wd");
  chk(ainp_dgrad16_weight(dev(w, "w"), (int)Cout, (int)Cin, (int)k, (int)stride, (int)pad,
                          bf16p(wd, "wd"), stream_of(w)),
      "dgrad16_weight");
}

void dgrad16(const Tensor& gT, const Tensor& wd, int64_t Cin, int64_t H, int64_t W, int64_t k,
             int64_t stride, int64_t pad, const OptT& scale, const Tensor& out, int64_t nsplit) {
  GUARD(gT);
  TORCH_CHECK(gT.dim() == 4, "gT must be [N, Ho, Wo, Cout] (channel-last bf16)");
  const int64_t N = gT.size(0), Ho = gT.size(1), Wo = gT.size(2), Cout = gT.size(3);
  TORCH_CHECK(stride >= 1 && k % stride == 0, "dgrad16: k % stride == 0");
  const int64_t nt = k / stride;
  numel_is(wd, stride * stride * Cin * nhwc16_seg(Cout, nt * nt), "wd");
  numel_is(out, nsplit * N * Cin * H * W, "out");
  chk(ainp_dgrad16(bf16p(gT, "gT"), N, (int)Cout, (int)Ho, (int)Wo, bf16p(wd, "wd"), (int)Cin,
                   (int)H, (int)W, (int)k, (int)stride, (int)pad, opt(scale, "scale"),
                   dev(out, "out"), (int)nsplit, N * Cin * H * W, stream_of(gT)),
      "dgrad16");
}
void wgrad16_nhwc(const Tensor& gA, const Tensor& x16, int64_t k, int64_t stride, int64_t pad,
                  const Tensor& G, int64_t nsplit, int64_t kc) {
  GUARD(gA);
  TORCH_CHECK(gA.dim() == 2 && x16.dim() == 4, "wgrad16_nhwc: gA [Cout, ldA], x16 [N, H, W, Cin]");
  const int64_t Cout = gA.size(0), N = x16.size(0), H = x16.size(1), W = x16.size(2),
                Cin = x16.size(3);
  numel_is(G, nsplit * Cout * (Cin * k * k + 1), "G");
  chk(ainp_wgrad16_nhwc(bf16p(gA, "gA", false), gA.stride(0), (int)Cout, bf16p(x16, "x16"), N,
                        (int)Cin, (int)H, (int)W, (int)k, (int)stride, (int)pad, dev(G, "G"),
                        (int)nsplit, kc, stream_of(gA)),
      "wgrad16_nhwc");
}

void dgrad16_prep(const Tensor& gT, const Tensor& wd, int64_t Cin, int64_t H, int64_t W,
                  int64_t k, int64_t stride, int64_t pad, const OptT& scale, const OptT& y,
                  double slope, const Tensor& gA, const OptT& gTo) {
  GUARD(gT);
  TORCH_CHECK(gT.dim() == 4, "gT must be [N, Ho, Wo, Cout] (channel-last bf16)");
  const int64_t N = gT.size(0), Ho = gT.size(1), Wo = gT.size(2), Cout = gT.size(3);
  TORCH_CHECK(stride >= 1 && k % stride == 0, "dgrad16_prep: k % stride == 0");
  const int64_t nt = k / stride;
  numel_is(wd, stride * stride * Cin * nhwc16_seg(Cout, nt * nt), "wd");
  TORCH_CHECK(gA.dim() == 2 && gA.size(0) == Cin && gA.size(1) >= N * H * W,
              "gA must be [Cin, ldA >= N*H*W]");
  const float* py = opt(y, "y");
  if (py) numel_is(*y, N * Cin * H * W, "y");
  uint16_t* pt = nullptr;
  if (gTo.has_value() && gTo->defined()) {
    numel_is(*gTo, N * H * W * Cin, "gTo");
    pt = bf16p(*gTo, "gTo");
  }
  chk(ainp_dgrad16_prep(bf16p(gT, "gT"), N, (int)Cout, (int)Ho, (int)Wo, bf16p(wd, "wd"),
                        (int)Cin, (int)H, (int)W, (int)k, (int)stride, (int)pad,
                        opt(scale, "scale"), py, (float)slope, bf16p(gA, "gA"), gA.size(1), pt,
                        stream_of(gT)),
      "dgrad16_prep");
}
// ---------------------------------------------------------------- generator backward
// (csrc/gan_bwd.hip; opt-in fix_generator_grad)
void affine_leaky_out(const Tensor& y, const Tensor& scale, const Tensor& shift, double slope,
                      const Tensor& out) {
  GUARD(y);
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W]");
  const int64_t N = y.size(0), C = y.size(1), HW = y.size(2) * y.size(3);
  numel_is(scale, C, "scale");
  numel_is(shift, C, "shift");
  numel_is(out, y.numel(), "out");
  chk(ainp_affine_leaky_out(dev(y, "y"), dev(scale, "scale"), dev(shift, "shift"), N, (int)C, HW,
                            (float)slope, dev(out, "out"), stream_of(y)),
      "affine_leaky_out");
}

void pconv_src_materialize(const Tensor& x0, const OptT& m0, const OptT& x1, const OptT& m1,
                           int64_t Hin, int64_t Win, const Tensor& out) {
  GUARD(x0);
  TORCH_CHECK(x0.dim() == 4, "x0 must be [N,C0,H0,W0]");
  const int64_t N = x0.size(0), C0 = x0.size(1), H0 = x0.size(2), W0 = x0.size(3);
  int64_t C1 = 0;
  if (x1.has_value() && x1->defined()) {
    TORCH_CHECK(x1->dim() == 4 && x1->size(0) == N && x1->size(2) == Hin && x1->size(3) == Win,
                "x1 must be [N,C1,Hin,Win]");
    C1 = x1->size(1);
  }
  if (m0.has_value() && m0->defined()) numel_is(*m0, N * H0 * W0, "m0");
  if (m1.has_value() && m1->defined()) numel_is(*m1, N * Hin * Win, "m1");
  numel_is(out, N * (C0 + C1) * Hin * Win, "out");
  chk(ainp_pconv_src_materialize(dev(x0, "x0"), opt(m0, "m0"), N, (int)C0, (int)H0, (int)W0,
                                 opt(x1, "x1"), opt(m1, "m1"), (int)C1, (int)Hin, (int)Win,
                                 dev(out, "out"), stream_of(x0)),
      "pconv_src_materialize");
}

void pconv_src_grad(const Tensor& dxin, int64_t c_off, const OptT& ms, bool accumulate,
                    const Tensor& dxs) {
  GUARD(dxin);
  TORCH_CHECK(dxin.dim() == 4 && dxs.dim() == 4, "dxin / dxs must be 4-d");
  const int64_t N = dxin.size(0), Cin = dxin.size(1), Hin = dxin.size(2), Win = dxin.size(3);
  const int64_t C = dxs.size(1), Hs = dxs.size(2), Ws = dxs.size(3);
  TORCH_CHECK(dxs.size(0) == N && c_off >= 0 && c_off + C <= Cin, "pconv_src_grad: channels");
  if (ms.has_value() && ms->defined()) numel_is(*ms, N * Hs * Ws, "ms");
  chk(ainp_pconv_src_grad(dev(dxin, "dxin"), N, (int)Cin, (int)Hin, (int)Win, (int)c_off, (int)C,
                          (int)Hs, (int)Ws, opt(ms, "ms"), dev(dxs, "dxs"), accumulate ? 1 : 0,
                          stream_of(dxin)),
      "pconv_src_grad");
}

void gen_act_bwd(const Tensor& g, const OptT& a, int64_t act, double slope, const OptT& ratio,
                 int64_t H, int64_t W, int64_t ldo, const OptT& gz, const Tensor& gc) {
  GUARD(g);
  TORCH_CHECK(g.dim() == 4, "g must be [N,C,gH,gW]");
  const int64_t N = g.size(0), C = g.size(1), gH = g.size(2), gW = g.size(3);
  if (a.has_value() && a->defined()) numel_is(*a, g.numel(), "a");
  if (ratio.has_value() && ratio->defined()) numel_is(*ratio, N * H * W, "ratio");
  if (gz.has_value() && gz->defined()) numel_is(*gz, N * C * H * W, "gz");
  numel_is(gc, N * C * ldo, "gc");
  chk(ainp_gen_act_bwd(dev(g, "g"), (int)gH, (int)gW, opt(a, "a"), (int)act, (float)slope,
                       opt(ratio, "ratio"), N, (int)C, (int)H, (int)W, ldo, opt(gz, "gz"),
                       dev(gc, "gc"), stream_of(g)),
      "gen_act_bwd");
}

void bn_act_bwd_reduce(const Tensor& ga, const Tensor& y, const Tensor& scale,
                       const Tensor& shift, const Tensor& save, double slope,
                       const Tensor& workspace, const Tensor& sums) {
  GUARD(ga);
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W]");
  const int64_t N = y.size(0), C = y.size(1), P = y.size(2) * y.size(3);
  numel_is(ga, y.numel(), "ga");
  numel_is(save, 2 * C, "save");
  TORCH_CHECK(sums.numel() >= 2 * C, "sums");
  TORCH_CHECK(workspace.numel() * workspace.element_size() >=
                  (int64_t)ainp_bn_act_bwd_workspace(N, (int)C, P), "workspace too small");
  chk(ainp_bn_act_bwd_reduce(dev(ga, "ga"), dev(y, "y"), dev(scale, "scale"), dev(shift, "shift"),
                             dev(save, "save"), (float)slope, N, (int)C, P, workspace.data_ptr(),
                             dev<double>(sums, "sums", at::kDouble), stream_of(ga)),
      "bn_act_bwd_reduce");
}

void bn_act_bwd_apply(const Tensor& ga, const Tensor& y, const Tensor& scale, const Tensor& shift,
                      const Tensor& save, const OptT& gamma, const Tensor& sums, int64_t count,
                      double slope, const OptT& ratio, int64_t ldo, const Tensor& gc,
                      const OptT& dgamma, const OptT& dbeta) {
  GUARD(ga);
  TORCH_CHECK(y.dim() == 4, "y must be [N,C,H,W]");
  const int64_t N = y.size(0), C = y.size(1), P = y.size(2) * y.size(3);
  numel_is(ga, y.numel(), "ga");
  numel_is(save, 2 * C, "save");
  TORCH_CHECK(sums.numel() >= 2 * C + (count == 0 ? 1 : 0), "sums");
  if (ratio.has_value() && ratio->defined()) numel_is(*ratio, N * P, "ratio");
  numel_is(gc, N * C * ldo, "gc");
  chk(ainp_bn_act_bwd_apply(dev(ga, "ga"), dev(y, "y"), dev(scale, "scale"), dev(shift, "shift"),
                            dev(save, "save"), opt(gamma, "gamma"),
                            dev<double>(sums, "sums", at::kDouble), count, (float)slope,
                            opt(ratio, "ratio"), N, (int)C, P, ldo, dev(gc, "gc"),
                            opt(dgamma, "dgamma"), opt(dbeta, "dbeta"), stream_of(ga)),
      "bn_act_bwd_apply");
}

void maxpool2_bwd(const Tensor& g, const Tensor& x, const Tensor& gx) {
  GUARD(g);
  TORCH_CHECK(x.dim() == 4, "x must be [N,C,H,W]");
  const int64_t NC = x.size(0) * x.size(1), H = x.size(2), W = x.size(3);
  numel_is(g, NC * (H / 2) * (W / 2), "g");
  numel_is(gx, x.numel(), "gx");
  chk(ainp_maxpool2_bwd(dev(g, "g"), dev(x, "x"), NC, (int)H, (int)W, dev(gx, "gx"),
                        stream_of(g)),
      "maxpool2_bwd");
}

void vgg_prep_bwd(const Tensor& g, const Tensor& x, const Tensor& ry0, const Tensor& rn,
                  const Tensor& rw, const Tensor& cx0, const Tensor& cn, const Tensor& cw,
                  int64_t S, const Tensor& workspace, const Tensor& gx) {
  GUARD(g);
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1, "x must be [N,1,H,W]");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  numel_is(g, N * 3 * S * S, "g");
  numel_is(gx, x.numel(), "gx");
  TORCH_CHECK(rw.dim() == 2 && cw.dim() == 2 && rw.size(0) == S && cw.size(0) == S,
              "vgg_prep_bwd: weight tables [S, taps]");
  numel_is(ry0, S, "ry0");
  numel_is(rn, S, "rn");
  numel_is(cx0, S, "cx0");
  numel_is(cn, S, "cn");
  TORCH_CHECK(workspace.numel() * workspace.element_size() >=
                  (int64_t)ainp_vgg_prep_bwd_workspace(N, (int)W, (int)S), "workspace too small");
  chk(ainp_vgg_prep_bwd(dev(g, "g"), dev(x, "x"), N, (int)H, (int)W,
                        dev<int32_t>(ry0, "ry0", at::kInt), dev<int32_t>(rn, "rn", at::kInt),
                        dev(rw, "rw"), (int)rw.size(1), dev<int32_t>(cx0, "cx0", at::kInt),
                        dev<int32_t>(cn, "cn", at::kInt), dev(cw, "cw"), (int)cw.size(1), (int)S,
                        workspace.data_ptr(), dev(gx, "gx"), stream_of(g)),
      "vgg_prep_bwd");
}

void absdiff_grad(const Tensor& a, const Tensor& b, const OptT& gscale, double scale,
                  bool accumulate, const Tensor& out) {
  GUARD(a);
  numel_is(b, a.numel(), "b");
  numel_is(out, a.numel(), "out");
  if (gscale.has_value() && gscale->defined()) numel_is(*gscale, 1, "gscale");
  chk(ainp_absdiff_grad(dev(a, "a"), dev(b, "b"), a.numel(), opt(gscale, "gscale"), (float)scale,
                        dev(out, "out"), accumulate ? 1 : 0, stream_of(a)),
      "absdiff_grad");
}

void gram_sign_sym(const Tensor& Ga, const Tensor& Gb, const OptT& gscale, double scale,
                   const Tensor& out) {
  GUARD(Ga);
  TORCH_CHECK(Ga.dim() == 3 && Ga.size(1) == Ga.size(2), "Ga must be [B,C,C]");
  numel_is(Gb, Ga.numel(), "Gb");
  numel_is(out, Ga.numel(), "out");
  if (gscale.has_value() && gscale->defined()) numel_is(*gscale, 1, "gscale");
  chk(ainp_gram_sign_sym(dev(Ga, "Ga"), dev(Gb, "Gb"), Ga.size(0), (int)Ga.size(1),
                         opt(gscale, "gscale"), (float)scale, dev(out, "out"), stream_of(Ga)),
      "gram_sign_sym");
}

void gan_recon_bwd(const Tensor& g, const Tensor& o, const Tensor& m, const Tensor& sums5,
                   const Tensor& gout3, double n_total, const Tensor& out) {
  GUARD(g);
  numel_is(o, g.numel(), "original");
  numel_is(m, g.numel(), "mask");
  numel_is(sums5, 5, "sums5");
  numel_is(gout3, 3, "gout3");
  numel_is(out, g.numel(), "out");
  chk(ainp_gan_recon_bwd(dev(g, "generated"), dev(o, "original"), dev(m, "mask"), g.numel(),
                         dev<double>(sums5, "sums5", at::kDouble), dev(gout3, "gout3"), n_total,
                         dev(out, "out"), stream_of(g)),
      "gan_recon_bwd");
}

void conv_weight_flip_t(const Tensor& w, const Tensor& out) {
  GUARD(w);
  TORCH_CHECK(w.dim() == 4 && w.size(2) == w.size(3), "w must be [Cout,Cin,K,K]");
  numel_is(out, w.numel(), "out");
  chk(ainp_conv_weight_flip_t(dev(w, "w"), (int)w.size(0), (int)w.size(1), (int)w.size(2),
                              dev(out, "out"), stream_of(w)),
      "conv_weight_flip_t");
}

}  // namespace

TORCH_LIBRARY(ainp, m) {
  m.def("stft_features(Tensor audio, Tensor? clip_index, Tensor gap_start, int gap_len, "
        "int sample_rate, Tensor window, int n_fft, int hop, int n_frames, int mode, "
        "Tensor(a!)? out0, Tensor(b!)? out1, Tensor(c!)? out2, Tensor(d!)? out3) -> ()");
  m.def("stft(Tensor audio, Tensor window, int n_fft, int hop, bool center, int n_frames, "
        "Tensor(a!) out) -> ()");
  m.def("istft(Tensor in0, Tensor? in1, int mode, int n_bins, int n_frames, Tensor window, "
        "int n_fft, int hop, bool center, Tensor(a!) workspace, Tensor(b!) out) -> ()");
  m.def("gl_update(Tensor rebuilt, Tensor(a!) tprev, Tensor(b!) angles, float momentum, "
        "bool first) -> ()");
  m.def("gemm_x6_multi(Tensor?[] ins, Tensor(a!)[] outs, int[] ints) -> ()");
  m.def("gl_stft_update(Tensor audio, Tensor window, int hop, int n_frames, Tensor(a!) tprev, "
        "Tensor(b!) angles, float momentum, bool first) -> ()");
  m.def("gemm(int M, int N, int K, float alpha, Tensor[] A, int sam, int sak, int strideA, "
        "Tensor[] B, int sbk, int sbn, int strideB, float beta, Tensor(a!)[] C, int scm, int scn, "
        "int strideC, Tensor?[] bias1, Tensor?[] bias2, int nstrided, int ksplit, int flags, "
        "Tensor(b!)? workspace) -> ()");
  m.def("conv3x3_fwd(Tensor x, Tensor w, Tensor? bias, Tensor? in_scale, Tensor? in_shift, "
        "Tensor(a!) y, Tensor(b!)? stats, int flags) -> ()");
  m.def("conv3x3_dgrad(Tensor dy, Tensor w, Tensor(a!) dx, int flags) -> ()");
  m.def("conv3x3_dgrad_bnr(Tensor dy, Tensor w, Tensor(a!) dx, int flags, Tensor y, Tensor scale, "
        "Tensor shift, Tensor save, Tensor(b!) workspace, Tensor(c!) sums, int bn_flags) -> ()");
  m.def("conv3x3_dgrad_bnapply(Tensor dy, Tensor w, Tensor y, Tensor scale, Tensor shift, "
        "Tensor? gamma, Tensor save, Tensor sums, int count, Tensor(a!) gy, Tensor(b!) dgamma, "
        "Tensor(c!) dbeta) -> ()");
  m.def("conv3x3_wgrad_bnapply(Tensor x, Tensor? in_scale, Tensor? in_shift, Tensor g, Tensor y, "
        "Tensor scale, Tensor shift, Tensor? gamma, Tensor save, Tensor sums, int count, "
        "Tensor(a!) dw, Tensor(b!)? dbias, Tensor(c!) dgamma, Tensor(d!) dbeta, "
        "Tensor(e!) workspace) -> ()");
  m.def("conv3x3_wgrad(Tensor x, Tensor? in_scale, Tensor? in_shift, Tensor dy, Tensor(a!) dw, "
        "Tensor(b!)? dbias, Tensor(c!) workspace, int flags) -> ()");
  m.def("bn_stats_reduce(Tensor stats, Tensor(a!) sums, int C) -> ()");
  m.def("bn_reduce_finalize(Tensor stats, int count, Tensor? gamma, Tensor? beta, "
        "Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, float eps, "
        "Tensor(c!) scale, Tensor(d!) shift, Tensor(e!) save) -> ()");
  m.def("bn_finalize(Tensor sums, int count, Tensor? gamma, Tensor? beta, "
        "Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, float eps, "
        "Tensor(c!) scale, Tensor(d!) shift, Tensor(e!) save) -> ()");
  m.def("bn_eval_affine(Tensor? gamma, Tensor? beta, Tensor running_mean, Tensor running_var, "
        "float eps, Tensor(a!) scale, Tensor(b!) shift) -> ()");
  m.def("bn_relu_apply(Tensor x, Tensor scale, Tensor shift, Tensor(a!) out, bool ntcf) -> ()");
  m.def("bn_relu_bwd_reduce(Tensor g, Tensor y, Tensor scale, Tensor shift, Tensor save, "
        "Tensor(a!) workspace, Tensor(b!) sums, bool ntcf, int flags=0) -> ()");
  m.def("bn_relu_bwd_apply(Tensor g, Tensor y, Tensor scale, Tensor shift, Tensor? gamma, "
        "Tensor save, Tensor sums, int count, Tensor(a!) gy, Tensor(b!)? dgamma, "
        "Tensor(c!)? dbeta, bool ntcf, int flags=0) -> ()");
  m.def("lstm_rec_fwd(Tensor zx, Tensor whh_f, Tensor whh_r, Tensor(a!) h_out, "
        "Tensor(b!)? gates, Tensor(c!)? cell, int H) -> ()");
  m.def("lstm_rec_bwd(Tensor dh_out, Tensor gates, Tensor cell, Tensor whh_f, Tensor whh_r, "
        "Tensor(a!) dgates, int H) -> ()");
  m.def("lstm_hprev(Tensor h_out, Tensor(a!) hprev, int H) -> ()");
  m.def("l1_pow10_loss(Tensor y, Tensor mask, Tensor target, Tensor(a!) loss, Tensor(b!)? dy, "
        "float grad_scale) -> ()");
  m.def("scale_by_dev(Tensor x, Tensor(a!) out, Tensor scalar) -> ()");
  m.def("sum_slabs(Tensor x, int nslabs, int n, Tensor(a!) out) -> ()");
  m.def("rowsum_batched(Tensor x, Tensor(a!) out) -> ()");
  m.def("colsum(Tensor x, int rows, int cols, int ld, Tensor(a!) out, bool accumulate) -> ()");
  m.def("colsum_slabs(Tensor x, int rows, int cols, int ld, int nslabs, Tensor(a!) partial) -> ()");
  m.def("adam(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avg, "
        "Tensor(c!)[] exp_avg_sq, float lr, float beta1, float beta2, float eps, "
        "float weight_decay, int step, Tensor(d!)? step_dev, Tensor(e!)? scalars_dev) -> ()");
  m.def("conv_weight_kmajor(Tensor w, int C0, int C1, Tensor(a!) wt) -> ()");
  m.def("conv_gen_fwd(Tensor x0, Tensor? m0, Tensor? x1, Tensor? m1, Tensor w, Tensor? wt, "
        "Tensor? bias, Tensor? ratio, Tensor? scale, Tensor(a!) y, Tensor(b!)? stats, int Hin, "
        "int Win, int stride, int pad, int act, float slope, int crop_h, int crop_w, int flags, "
        "Tensor(c!)? workspace, Tensor(d!)? y16=None) -> ()");
  m.def("pconv_mask(Tensor m0, int C0, Tensor? m1, int C1, int N, int Hin, int Win, int k, "
        "int stride, int pad, float winsize, Tensor(a!)? ratio, Tensor(b!)? newmask) -> ()");
  m.def("gan_pad_input(Tensor x, Tensor m, Tensor(a!) xp, Tensor(b!) mp) -> ()");
  m.def("affine_act(Tensor(a!) y, Tensor scale, Tensor shift, int act, float slope) -> ()");
  m.def("maxpool2(Tensor x, Tensor(a!) y, Tensor(b!)? out16=None) -> ()");
  m.def("absdiff_mean(Tensor a, Tensor b, Tensor(a!) workspace, Tensor(b!) out) -> ()");
  m.def("bce_logits(Tensor x, float target, Tensor(a!)? grad, float grad_scale, "
        "Tensor(b!) workspace, Tensor(c!) out) -> ()");
  m.def("gan_recon_losses(Tensor g, Tensor o, Tensor m, Tensor(a!) workspace, Tensor(b!) out) -> ()");
  m.def("gan_recon_sums(Tensor g, Tensor o, Tensor m, Tensor(a!) workspace, Tensor(b!) out) -> ()");
  m.def("vgg_target_max(Tensor x, Tensor(a!) max_ws) -> ()");
  m.def("vgg_prep(Tensor x, int generated, Tensor(a!) max_ws, Tensor ry0, Tensor rn, Tensor rw, "
        "Tensor cx0, Tensor cn, Tensor cw, int S, Tensor(b!) out) -> ()");
  m.def("sn_power(Tensor[] w, Tensor(a!)[] u, Tensor(b!)[] v, float eps, Tensor(c!) workspace, "
        "Tensor(d!) inv_sigma, bool update) -> ()");
  m.def("sn_weight_grad(Tensor G, Tensor w_orig, Tensor u, Tensor v, Tensor inv_sigma, "
        "Tensor(a!) workspace, Tensor(b!) out, Tensor(c!)? out_bias) -> ()");
  m.def("im2col_ld(Tensor x, int k, int stride, int pad, bool ones_row, int ldp, "
        "Tensor(a!) col) -> ()");
  m.def("col2im_ld(Tensor dcol, int k, int stride, int pad, Tensor(a!) dx) -> ()");
  m.def("leaky_bwd(Tensor g, Tensor y, float slope, Tensor(a!) out) -> ()");
  m.def("leaky_bwd_ld(Tensor g, Tensor y, int rows, float slope, int ldo, Tensor(a!) out) -> ()");
  m.def("mul(Tensor a, Tensor b, Tensor(a!) out) -> ()");
  m.def("channel_sum(Tensor m, Tensor(a!) out) -> ()");
  m.def("bn_relu_apply_ntcf_cl(Tensor y, Tensor scale, Tensor shift, Tensor(a!)? out, "
        "Tensor(b!)? out16, Tensor(c!)? outT, int flags) -> ()");
  m.def("bn_relu_apply_ntcf_bf16(Tensor x, Tensor scale, Tensor shift, Tensor(a!) out, "
        "Tensor(b!) outT, int flags=0) -> ()");
  m.def("gemm_bf16nt_multi(Tensor[] A, Tensor[] B, Tensor(a!)[] C, int[] ints) -> ()");
  m.def("gemm_bf16nt(Tensor A, Tensor B, Tensor(a!) C, int K, Tensor? bias_a1, Tensor? bias_a2, "
        "Tensor? bias_b1, Tensor? bias_b2, int bias_nsplit, int nsplit, int kc) -> ()");
  m.def("cast_bf16_t(Tensor x, Tensor(a!)? out, Tensor(b!)? outT) -> ()");
  m.def("transpose_f32(Tensor x, Tensor(a!) outT) -> ()");
  m.def("gemm_x6nt_256(Tensor A, Tensor B1, Tensor B2, Tensor(a!) C, Tensor? bias_a1, "
        "Tensor? bias_a2, Tensor? bias_b1, Tensor? bias_b2, int bias_nsplit, int nsplit, "
        "int kc) -> ()");
  m.def("nchw_to_nhwc16(Tensor x, Tensor? m, Tensor(a!) out) -> ()");
  m.def("affine_act_nhwc16(Tensor(a!) y, Tensor scale, Tensor shift, int act, float slope, "
        "Tensor? m, Tensor(b!) out, bool keep_y=True) -> ()");
  m.def("conv_weight_nhwc16(Tensor w, int C0, int C1, Tensor(a!) wt16) -> ()");
  m.def("conv_gen_fwd_nhwc16(Tensor x0, Tensor? x1, Tensor wt16, int Cout, int KH, int KW, "
        "Tensor? bias, Tensor? ratio, Tensor? scale, Tensor(a!) y, Tensor(b!)? stats, int Hin, "
        "int Win, int stride, int pad, int act, float slope, Tensor(c!)? workspace, "
        "int[] dims=[], Tensor(d!)? y16=None) -> ()");
  m.def("im2col_nhwc16(Tensor x, Tensor? m, int Hin, int Win, int KH, int KW, int stride, "
        "int pad, Tensor(a!) out) -> ()");
  m.def("d_prep16(Tensor g, int nslab, Tensor? y, float slope, int N, int C, int P, "
        "Tensor(a!) gA, Tensor(b!)? gT) -> ()");
  m.def("wgrad_cout1(Tensor x, Tensor g, int nslab, Tensor? y, float slope, int k, int stride, "
        "int pad, Tensor(a!) gw, Tensor(b!) ws) -> ()");
  m.def("im2col16(Tensor x, int k, int stride, int pad, bool ones_row, Tensor(a!) col) -> ()");
  m.def("dgrad16_weight(Tensor w, int stride, int pad, Tensor(a!) wd) -> ()");
  m.def("dgrad16(Tensor gT, Tensor wd, int Cin, int H, int W, int k, int stride, int pad, "
        "Tensor? scale, Tensor(a!) out, int nsplit) -> ()");
  m.def("wgrad16_nhwc(Tensor gA, Tensor x16, int k, int stride, int pad, Tensor(a!) G, "
        "int nsplit, int kc) -> ()");
  m.def("dgrad16_prep(Tensor gT, Tensor wd, int Cin, int H, int W, int k, int stride, int pad, "
        "Tensor? scale, Tensor? y, float slope, Tensor(a!) gA, Tensor(b!)? gTo) -> ()");
  m.def("affine_leaky_out(Tensor y, Tensor scale, Tensor shift, float slope, Tensor(a!) out) -> ()");
  m.def("pconv_src_materialize(Tensor x0, Tensor? m0, Tensor? x1, Tensor? m1, int Hin, int Win, "
        "Tensor(a!) out) -> ()");
  m.def("pconv_src_grad(Tensor dxin, int c_off, Tensor? ms, bool accumulate, Tensor(a!) dxs) -> ()");
  m.def("gen_act_bwd(Tensor g, Tensor? a, int act, float slope, Tensor? ratio, int H, int W, "
        "int ldo, Tensor(a!)? gz, Tensor(b!) gc) -> ()");
  m.def("bn_act_bwd_reduce(Tensor ga, Tensor y, Tensor scale, Tensor shift, Tensor save, "
        "float slope, Tensor(a!) workspace, Tensor(b!) sums) -> ()");
  m.def("bn_act_bwd_apply(Tensor ga, Tensor y, Tensor scale, Tensor shift, Tensor save, "
        "Tensor? gamma, Tensor sums, int count, float slope, Tensor? ratio, int ldo, "
        "Tensor(a!) gc, Tensor(b!)? dgamma, Tensor(c!)? dbeta) -> ()");
  m.def("maxpool2_bwd(Tensor g, Tensor x, Tensor(a!) gx) -> ()");
  m.def("vgg_prep_bwd(Tensor g, Tensor x, Tensor ry0, Tensor rn, Tensor rw, Tensor cx0, Tensor cn, "
        "Tensor cw, int S, Tensor(a!) workspace, Tensor(b!) gx) -> ()");
  m.def("absdiff_grad(Tensor a, Tensor b, Tensor? gscale, float scale, bool accumulate, "
        "Tensor(a!) out) -> ()");
  m.def("gram_sign_sym(Tensor Ga, Tensor Gb, Tensor? gscale, float scale, Tensor(a!) out) -> ()");
  m.def("gan_recon_bwd(Tensor g, Tensor o, Tensor m, Tensor sums5, Tensor gout3, float n_total, "
        "Tensor(a!) out) -> ()");
  m.def("conv_weight_flip_t(Tensor w, Tensor(a!) out) -> ()");
}

TORCH_LIBRARY_IMPL(ainp, CUDA, m) {
  m.impl("stft_features", &stft_features);
  m.impl("stft", &stft);
  m.impl("istft", &istft);
  m.impl("gl_update", &gl_update);
  m.impl("gl_stft_update", &gl_stft_update);
  m.impl("gemm_x6_multi", &gemm_x6_multi);
  m.impl("gemm_bf16nt_multi", &gemm_bf16nt_multi);
  m.impl("gemm", &gemm);
  m.impl("conv3x3_fwd", &conv3x3_fwd);
  m.impl("conv3x3_dgrad", &conv3x3_dgrad);
  m.impl("conv3x3_dgrad_bnr", &conv3x3_dgrad_bnr);
  m.impl("conv3x3_wgrad", &conv3x3_wgrad);
  m.impl("conv3x3_wgrad_bnapply", &conv3x3_wgrad_bnapply);
  m.impl("conv3x3_dgrad_bnapply", &conv3x3_dgrad_bnapply);
  m.impl("bn_stats_reduce", &bn_stats_reduce);
  m.impl("bn_finalize", &bn_finalize);
  m.impl("bn_reduce_finalize", &bn_reduce_finalize);
  m.impl("bn_eval_affine", &bn_eval_affine);
  m.impl("bn_relu_apply", &bn_relu_apply);
  m.impl("bn_relu_bwd_reduce", &bn_relu_bwd_reduce);
  m.impl("bn_relu_bwd_apply", &bn_relu_bwd_apply);
  m.impl("lstm_rec_fwd", &lstm_rec_fwd);
  m.impl("lstm_rec_bwd", &lstm_rec_bwd);
  m.impl("lstm_hprev", &lstm_hprev);
  m.impl("l1_pow10_loss", &l1_pow10_loss);
  m.impl("scale_by_dev", &scale_by_dev);
  m.impl("sum_slabs", &sum_slabs);
  m.impl("rowsum_batched", &rowsum_batched);
  m.impl("colsum", &colsum);
  m.impl("colsum_slabs", &colsum_slabs);
  m.impl("adam", &adam);
  m.impl("conv_weight_kmajor", &conv_weight_kmajor);
  m.impl("conv_gen_fwd", &conv_gen_fwd);
  m.impl("pconv_mask", &pconv_mask);
  m.impl("gan_pad_input", &gan_pad_input);
  m.impl("affine_act", &affine_act);
  m.impl("affine_act_nhwc16", &affine_act_nhwc16);
  m.impl("maxpool2", &maxpool2);
  m.impl("absdiff_mean", &absdiff_mean);
  m.impl("bce_logits", &bce_logits);
  m.impl("gan_recon_losses", &gan_recon_losses);
  m.impl("gan_recon_sums", &gan_recon_sums);
  m.impl("vgg_target_max", &vgg_target_max);
  m.impl("vgg_prep", &vgg_prep);
  m.impl("sn_power", &sn_power);
  m.impl("sn_weight_grad", &sn_weight_grad);
  m.impl("im2col_ld", &im2col_ld);
  m.impl("col2im_ld", &col2im_ld);
  m.impl("leaky_bwd", &leaky_bwd);
  m.impl("leaky_bwd_ld", &leaky_bwd_ld);
  m.impl("mul", &mul);
  m.impl("channel_sum", &channel_sum);
  m.impl("bn_relu_apply_ntcf_bf16", &bn_relu_apply_ntcf_bf16);
  m.impl("bn_relu_apply_ntcf_cl", &bn_relu_apply_ntcf_cl);
  m.impl("gemm_bf16nt", &gemm_bf16nt);
  m.impl("cast_bf16_t", &cast_bf16_t);
  m.impl("transpose_f32", &transpose_f32);
  m.impl("gemm_x6nt_256", &gemm_x6nt_256);
  m.impl("nchw_to_nhwc16", &nchw_to_nhwc16);
  m.impl("conv_weight_nhwc16", &conv_weight_nhwc16);
  m.impl("conv_gen_fwd_nhwc16", &conv_gen_fwd_nhwc16);
  m.impl("im2col_nhwc16", &im2col_nhwc16);
  m.impl("d_prep16", &d_prep16);
  m.impl("wgrad_cout1", &wgrad_cout1);
  m.impl("im2col16", &im2col16);
  m.impl("dgrad16_weight", &dgrad16_weight);
  m.impl("dgrad16", &dgrad16);
  m.impl("dgrad16_prep", &dgrad16_prep);
  m.impl("wgrad16_nhwc", &wgrad16_nhwc);
  m.impl("affine_leaky_out", &affine_leaky_out);
  m.impl("pconv_src_materialize", &pconv_src_materialize);
  m.impl("pconv_src_grad", &pconv_src_grad);
  m.impl("gen_act_bwd", &gen_act_bwd);
  m.impl("bn_act_bwd_reduce", &bn_act_bwd_reduce);
  m.impl("bn_act_bwd_apply", &bn_act_bwd_apply);
  m.impl("maxpool2_bwd", &maxpool2_bwd);
  m.impl("vgg_prep_bwd", &vgg_prep_bwd);
  m.impl("absdiff_grad", &absdiff_grad);
  m.impl("gram_sign_sym", &gram_sign_sym);
  m.impl("gan_recon_bwd", &gan_recon_bwd);
  m.impl("conv_weight_flip_t", &conv_weight_flip_t);
}

// The ops write through raw device pointers like the C ABI; autograd is the
// Python autograd.Function layer above them (ainp/cnnblstm.py, ainp/gan.py),
// so the Autograd key falls through to the device kernel.
TORCH_LIBRARY_IMPL(ainp, Autograd, m) {
  m.impl("stft_features", torch::CppFunction::makeFallthrough());
  m.impl("stft", torch::CppFunction::makeFallthrough());
  m.impl("istft", torch::CppFunction::makeFallthrough());
  m.impl("gl_update", torch::CppFunction::makeFallthrough());
  m.impl("gl_stft_update", torch::CppFunction::makeFallthrough());
  m.impl("gemm_x6_multi", torch::CppFunction::makeFallthrough());
  m.impl("gemm_bf16nt_multi", torch::CppFunction::makeFallthrough());
  m.impl("gemm", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_fwd", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_dgrad", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_dgrad_bnr", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_wgrad", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_wgrad_bnapply", torch::CppFunction::makeFallthrough());
  m.impl("conv3x3_dgrad_bnapply", torch::CppFunction::makeFallthrough());
  m.impl("bn_stats_reduce", torch::CppFunction::makeFallthrough());
  m.impl("bn_finalize", torch::CppFunction::makeFallthrough());
  m.impl("bn_reduce_finalize", torch::CppFunction::makeFallthrough());
  m.impl("bn_eval_affine", torch::CppFunction::makeFallthrough());
  m.impl("bn_relu_apply", torch::CppFunction::makeFallthrough());
  m.impl("bn_relu_bwd_reduce", torch::CppFunction::makeFallthrough());
  m.impl("bn_relu_bwd_apply", torch::CppFunction::makeFallthrough());
  m.impl("lstm_rec_fwd", torch::CppFunction::makeFallthrough());
  m.impl("lstm_rec_bwd", torch::CppFunction::makeFallthrough());
  m.impl("lstm_hprev", torch::CppFunction::makeFallthrough());
  m.impl("l1_pow10_loss", torch::CppFunction::makeFallthrough());
  m.impl("scale_by_dev", torch::CppFunction::makeFallthrough());
  m.impl("sum_slabs", torch::CppFunction::makeFallthrough());
  m.impl("rowsum_batched", torch::CppFunction::makeFallthrough());
  m.impl("colsum", torch::CppFunction::makeFallthrough());
  m.impl("colsum_slabs", torch::CppFunction::makeFallthrough());
  m.impl("adam", torch::CppFunction::makeFallthrough());
  m.impl("conv_weight_kmajor", torch::CppFunction::makeFallthrough());
  m.impl("conv_gen_fwd", torch::CppFunction::makeFallthrough());
  m.impl("pconv_mask", torch::CppFunction::makeFallthrough());
  m.impl("gan_pad_input", torch::CppFunction::makeFallthrough());
  m.impl("affine_act", torch::CppFunction::makeFallthrough());
  m.impl("affine_act_nhwc16", torch::CppFunction::makeFallthrough());
  m.impl("maxpool2", torch::CppFunction::makeFallthrough());
  m.impl("absdiff_mean", torch::CppFunction::makeFallthrough());
  m.impl("bce_logits", torch::CppFunction::makeFallthrough());
  m.impl("gan_recon_losses", torch::CppFunction::makeFallthrough());
  m.impl("gan_recon_sums", torch::CppFunction::makeFallthrough());
  m.impl("vgg_target_max", torch::CppFunction::makeFallthrough());
  m.impl("vgg_prep", torch::CppFunction::makeFallthrough());
  m.impl("sn_power", torch::CppFunction::makeFallthrough());
  m.impl("sn_weight_grad", torch::CppFunction::makeFallthrough());
  m.impl("im2col_ld", torch::CppFunction::makeFallthrough());
  m.impl("col2im_ld", torch::CppFunction::makeFallthrough());
  m.impl("leaky_bwd", torch::CppFunction::makeFallthrough());
  m.impl("leaky_bwd_ld", torch::CppFunction::makeFallthrough());
  m.impl("mul", torch::CppFunction::makeFallthrough());
  m.impl("channel_sum", torch::CppFunction::makeFallthrough());
  m.impl("bn_relu_apply_ntcf_bf16", torch::CppFunction::makeFallthrough());
  m.impl("bn_relu_apply_ntcf_cl", torch::CppFunction::makeFallthrough());
  m.impl("gemm_bf16nt", torch::CppFunction::makeFallthrough());
  m.impl("cast_bf16_t", torch::CppFunction::makeFallthrough());
  m.impl("transpose_f32", torch::CppFunction::makeFallthrough());
  m.impl("gemm_x6nt_256", torch::CppFunction::makeFallthrough());
  m.impl("nchw_to_nhwc16", torch::CppFunction::makeFallthrough());
  m.impl("conv_weight_nhwc16", torch::CppFunction::makeFallthrough());
  m.impl("conv_gen_fwd_nhwc16", torch::CppFunction::makeFallthrough());
  m.impl("im2col_nhwc16", torch::CppFunction::makeFallthrough());
  m.impl("d_prep16", torch::CppFunction::makeFallthrough());
  m.impl("wgrad_cout1", torch::CppFunction::makeFallthrough());
  m.impl("im2col16", torch::CppFunction::makeFallthrough());
  m.impl("dgrad16_weight", torch::CppFunction::makeFallthrough());
  m.impl("dgrad16", torch::CppFunction::makeFallthrough());
  m.impl("dgrad16_prep", torch::CppFunction::makeFallthrough());
  m.impl("wgrad16_nhwc", torch::CppFunction::makeFallthrough());
  m.impl("affine_leaky_out", torch::CppFunction::makeFallthrough());
  m.impl("pconv_src_materialize", torch::CppFunction::makeFallthrough());
  m.impl("pconv_src_grad", torch::CppFunction::makeFallthrough());
  m.impl("gen_act_bwd", torch::CppFunction::makeFallthrough());
  m.impl("bn_act_bwd_reduce", torch::CppFunction::makeFallthrough());
  m.impl("bn_act_bwd_apply", torch::CppFunction::makeFallthrough());
  m.impl("maxpool2_bwd", torch::CppFunction::makeFallthrough());
  m.impl("vgg_prep_bwd", torch::CppFunction::makeFallthrough());
  m.impl("absdiff_grad", torch::CppFunction::makeFallthrough());
  m.impl("gram_sign_sym", torch::CppFunction::makeFallthrough());
  m.impl("gan_recon_bwd", torch::CppFunction::makeFallthrough());
  m.impl("conv_weight_flip_t", torch::CppFunction::makeFallthrough());
}
