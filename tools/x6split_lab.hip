// x6split_lab.hip — the split-pass fp32 x6 256x256 tile
// (gemm16.hip x6_256::gemm_x6nt_256s_kernel: each fp32 K-tile split ONCE per
// workgroup into three bf16 plane images) against the per-fragment-split
// kernel (gemm_x6nt_256_kernel) at the C2 layer-0 projection shape: bit
// equality and time.  Measured (MI355X): unsplit 2.868 -> 2.853 ms, split 3
// 2.158 -> 1.938 ms, 0 differing values.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/x6split_lab.hip -o tools/x6split_lab
#include "../ml-audio-inpainting_amd/csrc/gemm16.hip"

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>

namespace ainp {
int record_error(hipError_t e, const char* where) {
  fprintf(stderr, "%s: %s\n", where, hipGetErrorString(e));
  return -1;
}
int record_msg(const char* msg) {
  fprintf(stderr, "%s\n", msg);
  return -1;
}

}  // namespace ainp

using namespace ainp;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main() {
  const int64_t M = 10688, H = 128, N = 8 * H, K = 16448;
  std::vector<float> ha(M * K), hw(N * K);
  uint32_t s = 99u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) * (1.0f / 16777216.0f) - 0.5f);
  };
  for (auto& v : ha) v = fmaxf(rnd(), 0.f) * 3.f;
  for (auto& v : hw) v = rnd() * 0.02f;
  float *A, *W, *C0, *C1;
  CK(hipMalloc(&A, ha.size() * 4));
  CK(hipMalloc(&W, hw.size() * 4));
  CK(hipMalloc(&C0, 3 * M * N * 4));
  CK(hipMalloc(&C1, 3 * M * N * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)x6_256::gemm_x6nt_256_kernel,
                         hipFuncAttributeMaxDynamicSharedMemorySize, x6_256::LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)x6_256::gemm_x6nt_256s_kernel,
                         hipFuncAttributeMaxDynamicSharedMemorySize, x6_256::LDS_BYTES_S));
  g16::Bias b{nullptr, nullptr, nullptr, nullptr, 0};
  const int64_t tn = N / 256, tm = (M + 255) / 256;
  for (int S : {1, 3}) {
    const int64_t kc = S > 1 ? ((K / S + 15) / 16) * 16 : K;
    auto l0 = [&] {
      hipLaunchKernelGGL(x6_256::gemm_x6nt_256_kernel, dim3((unsigned)(tm * tn), S), dim3(512),
                         x6_256::LDS_BYTES, 0, M, N, K, A, K, W, W + 4 * H * K, K, 4 * H, C0, N,
                         kc, M * N, b, (int)tn);
    };
    auto l1 = [&] {
      hipLaunchKernelGGL(x6_256::gemm_x6nt_256s_kernel, dim3((unsigned)(tm * tn), S), dim3(512),
                         x6_256::LDS_BYTES_S, 0, M, N, K, A, K, W, W + 4 * H * K, K, 4 * H, C1, N, kc,
                         M * N, b, (int)tn);
    };
    CK(hipMemset(C1, 0xff, 3 * M * N * 4));
    l0();
    l1();
    CK(hipDeviceSynchronize());
    std::vector<float> r0(S * M * N), r1(S * M * N);
    CK(hipMemcpy(r0.data(), C0, r0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r1.data(), C1, r1.size() * 4, hipMemcpyDeviceToHost));
    size_t nd = 0;
    for (size_t i = 0; i < r0.size(); ++i) nd += memcmp(&r0[i], &r1[i], 4) != 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto tm_ = [&](auto f) {
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
    const double t0 = tm_(l0), t1 = tm_(l1);
    printf("split %d: x6_256 %.3f ms  x6split %.3f ms  differing %zu / %zu\n", S, t0, t1, nd,
           r0.size());
  }
  return 0;
}
