// fp64 / fp32 VALU issue-rate microbenchmark (8 independent FMA chains per lane).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <typename T>
__global__ __launch_bounds__(256) void fma_chain(T* out, T a, T b, int iters) {
  T v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = v[i] * a + b;
  }
  T s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  if (s == (T)12345.678) out[threadIdx.x] = s;
}
template <typename T>
__global__ __launch_bounds__(256) void add_chain(T* out, T a, int iters) {
  T v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = v[i] + a;
  }
  T s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i];
  if (s == (T)12345.678) out[threadIdx.x] = s;
}
int main() {
  double* d;
  hipMalloc(&d, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096, grid = 256 * 8;
  for (int k = 0; k < 4; ++k) {
    for (int w = 0; w < 2; ++w) {
      hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(fma_chain<double>, grid, 256, 0, 0, d, 1.0000001, 1e-9, iters);
      if (k == 1) hipLaunchKernelGGL(fma_chain<float>, grid, 256, 0, 0, (float*)d, 1.0000001f, 1e-9f, iters);
      if (k == 2) hipLaunchKernelGGL(add_chain<double>, grid, 256, 0, 0, d, 1e-9, iters);
      if (k == 3) hipLaunchKernelGGL(add_chain<float>, grid, 256, 0, 0, (float*)d, 1e-9f, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)grid * 256 * iters * 8;
    const char* nm[] = {"fma f64", "fma f32", "add f64", "add f32"};
    printf("%s: %.2f ms, %.1f T lane-ops/s (%.1f TFLOP/s if FMA)\n", nm[k], ms, ops / ms / 1e9,
           2 * ops / ms / 1e9);
  }
  return 0;
}
