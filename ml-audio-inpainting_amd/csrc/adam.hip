// adam.hip — multi-tensor Adam, torch.optim.Adam arithmetic.
//
// Replaces optim.Adam(model.parameters(), lr) of models/CNNBLSTM/train.py:71-72
// (step at :108).  Per element, in the order torch's single-tensor and
// foreach paths use (torch/optim/adam.py):
//   m = m + (1-b1)*(g-m)            (exp_avg.lerp_(grad, 1-beta1))
//   v = v*b2 + (1-b2)*g*g           (exp_avg_sq.mul_(beta2).addcmul_(g,g,1-b2))
//   p = p - step_size * m / (sqrt(v)/sqrt(bc2) + eps),  step_size = lr/bc1
// with optional L2 weight decay g += wd*p (torch's non-decoupled form).
#include "common.h"

namespace ainp {

constexpr int ADAM_MAX = 32;
struct AdamList {
  float* p[ADAM_MAX];
  const float* g[ADAM_MAX];
  float* m[ADAM_MAX];
  float* v[ADAM_MAX];
  int64_t n[ADAM_MAX];
  int64_t block_start[ADAM_MAX + 1];
  int count;
};

constexpr int ADAM_CHUNK = 256 * 8;

// Device-step form (HIP-graph capturable): one thread advances the step
// counter kept on the device and forms step_size / sqrt(bc2) exactly as the
// host path does (double pow, one rounding to f32), so a captured step
// replays with the right bias corrections.
__global__ void adam_prologue(float* step_dev, float* scalars, double lr, double beta1,
                              double beta2) {
  const float step = step_dev[0] + 1.0f;
  step_dev[0] = step;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  scalars[0] = (float)(lr / bc1);
  scalars[1] = (float)sqrt(bc2);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamList L, float step_size,
                                                   float w1, float b2, float w2,
                                                   float bc2_sqrt, float eps,
                                                   float wd, const float* scalars) {
  if (scalars) {
    step_size = scalars[0];
    bc2_sqrt = scalars[1];
  }
  const int64_t b = blockIdx.x;
  int ti = 0;
  while (ti + 1 < L.count && L.block_start[ti + 1] <= b) ++ti;
  const int64_t base = (b - L.block_start[ti]) * ADAM_CHUNK;
  float* p = L.p[ti];
  const float* g = L.g[ti];
  float* m = L.m[ti];
  float* v = L.v[ti];
  const int64_t n = L.n[ti];
  for (int e = threadIdx.x; e < ADAM_CHUNK; e += 256) {
    const int64_t i = base + e;
    if (i >= n) break;
    float gi = g[i];
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2;
    vi = vi + w2 * (gi * gi);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi - step_size * (mi / denom);
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_adam(float* const* params, const float* const* grads,
                         float* const* exp_avg, float* const* exp_avg_sq,
                         const int64_t* numel, int n_tensors, double lr,
                         double beta1, double beta2, double eps,
                         double weight_decay, int64_t step, void* stream) {
  return ainp_adam_ex(params, grads, exp_avg, exp_avg_sq, numel, n_tensors, lr, beta1, beta2,
                      eps, weight_decay, step, nullptr, nullptr, stream);
}

extern "C" int ainp_adam_ex(float* const* params, const float* const* grads,
                            float* const* exp_avg, float* const* exp_avg_sq,
                            const int64_t* numel, int n_tensors, double lr,
                            double beta1, double beta2, double eps,
                            double weight_decay, int64_t step, float* step_dev,
                            float* scalars_dev, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !numel || n_tensors < 0 ||
      (!step_dev && step < 1) || (!step_dev != !scalars_dev))
    return record_msg("ainp_adam: bad argument");
  // scalars exactly as torch/optim/adam.py forms them (Python doubles),
  // rounded once to the f32 op math
  const double st = step_dev ? 1.0 : (double)step;
  const double bc1 = 1.0 - pow(beta1, st);
  const double bc2 = 1.0 - pow(beta2, st);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  hipStream_t s = as_stream(stream);
  if (step_dev) {
    hipLaunchKernelGGL(adam_prologue, dim3(1), dim3(1), 0, s, step_dev, scalars_dev, lr, beta1,
                       beta2);
    const int rc = check_launch("adam_prologue");
    if (rc) return rc;
  }
  for (int base = 0; base < n_tensors; base += ADAM_MAX) {
    AdamList L;
    L.count = 0;
    int64_t blocks = 0;
    for (int i = base; i < n_tensors && L.count < ADAM_MAX; ++i) {
      const int c = L.count++;
      L.p[c] = params[i];
      L.g[c] = grads[i];
      L.m[c] = exp_avg[i];
      L.v[c] = exp_avg_sq[i];
      L.n[c] = numel[i];
      L.block_start[c] = blocks;
      blocks += cdiv(numel[i], ADAM_CHUNK);
    }
    L.block_start[L.count] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, L,
                       step_size, (float)(1.0 - beta1), (float)beta2,
                       (float)(1.0 - beta2), bc2_sqrt, (float)eps,
                       (float)weight_decay, (const float*)scalars_dev);
    const int rc = check_launch("adam");
    if (rc) return rc;
  }
  return AINP_OK;
}
