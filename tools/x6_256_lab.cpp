// x6_256_lab.cpp -- ainp_gemm_x6nt_256 vs ainp_gemm_f32 (default x6 main loop)
// at the fp32 layer-0 projection shape (M=10688, N=1024 as two 512-row W_ih
// halves, K=16448, bias per direction): bit-exactness and time, via libainp.so.
//   hipcc -O3 -std=c++17 -I include tools/x6_256_lab.cpp -o tools/x6_256_lab \
//     -L ml-audio-inpainting_amd/ainp -lainp -Wl,-rpath,'$ORIGIN/../ml-audio-inpainting_amd/ainp'
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "ainp.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atol(argv[1]) : 10688, H = 128, N = 8 * H,
                K = argc > 2 ? atol(argv[2]) : 16448;
  std::vector<float> ha(M * K), hw(N * K), hb(4 * 4 * H);
  uint32_t s = 99u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) * (1.0f / 16777216.0f) - 0.5f);
  };
  for (auto& v : ha) v = fmaxf(rnd(), 0.f) * 3.f;  // BN+ReLU-like activations
  for (auto& v : hw) v = rnd() * 0.02f;
  for (auto& v : hb) v = rnd() * 0.1f;
  float *A, *W, *bias, *C0, *C1;
  CK(hipMalloc(&A, ha.size() * 4));
  CK(hipMalloc(&W, hw.size() * 4));
  CK(hipMalloc(&bias, hb.size() * 4));
  CK(hipMalloc(&C0, M * N * 4));
  CK(hipMalloc(&C1, M * N * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  const float* Wf = W;
  const float* Wr = W + 4 * H * K;
  const float *bif = bias, *bhf = bias + 4 * H, *bir = bias + 8 * H, *bhr = bias + 12 * H;
  // product path: pointer batches (A, W_ih) and (A, W_ih_rev) into zx[:, :4H], zx[:, 4H:]
  const float* Ap[2] = {A, A};
  const float* Bp[2] = {Wf, Wr};
  float* Cp[2] = {C0, C0 + 4 * H};
  const float* b1[2] = {bif, bir};
  const float* b2[2] = {bhf, bhr};
  auto prod = [&] {
    if (ainp_gemm_f32(M, 4 * H, K, 1.f, Ap, K, 1, 0, Bp, 1, K, 0, 0.f, Cp, N, 1, 0, b1, b2, 2, 1,
                      0, nullptr))
      exit(2);
  };
  const int S = argc > 3 ? atoi(argv[3]) : 1;
  const int64_t kc = S > 1 ? ((K / S + 15) / 16) * 16 : K;
  float* slabs = nullptr;
  if (S > 1) CK(hipMalloc(&slabs, (size_t)S * M * N * 4));
  auto x6 = [&] {
    if (ainp_gemm_x6nt_256(M, N, K, A, K, Wf, Wr, K, 4 * H, S > 1 ? slabs : C1, N, bif, bhf, bir,
                           bhr, 4 * H, S, kc, M * N, nullptr) ||
        (S > 1 && ainp_sum_slabs(slabs, S, M * N, C1, nullptr))) {
      fprintf(stderr, "%s\n", ainp_last_error());
      exit(2);
    }
  };
  CK(hipMemset(C1, 0xff, M * N * 4));
  prod();
  x6();
  CK(hipDeviceSynchronize());
  std::vector<float> r0(M * N), r1(M * N);
  CK(hipMemcpy(r0.data(), C0, M * N * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), C1, M * N * 4, hipMemcpyDeviceToHost));
  size_t nd = 0;
  double mx = 0;
  for (size_t i = 0; i < r0.size(); ++i) {
    if (memcmp(&r0[i], &r1[i], 4)) ++nd;
    const double e = fabs((double)r0[i] - (double)r1[i]);
    if (!(e <= mx)) mx = e;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto tm = [&](auto f) {
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 10;
  };
  const double tp = tm(prod), tx = tm(x6), fl = 2.0 * M * N * K;
  printf("split %d  M=%ld N=%ld K=%ld: product x6 %.3f ms (%.1f TF)  x6_256 %.3f ms (%.1f TF)  "
         "differing %zu / %zu (max |d| %.3g)\n",
         S, (long)M, (long)N, (long)K, tp, fl / tp / 1e9, tx, fl / tx / 1e9, nd, r0.size(), mx);
  return S == 1 && nd != 0;
}
