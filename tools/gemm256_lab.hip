// gemm256_lab.hip — the 256x256 LDS-DMA bf16 NT GEMM (gemm16.hip g256) vs
// the product kernel (gemm16.hip, 128x128x64 register-staged) at the layer-0
// LSTM shapes of the bf16 configuration: bit-exactness (same MFMA, same k
// order) and time.  Measured (MI355X): fwd 611 -> 763 TF (split 3: 892),
// dX 597 -> 722 TF, dW split 2 624 -> 744 TF, all bit-identical; s_setprio
// around the MFMAs and all-fragments-first reads measured no better.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/gemm256_lab.hip -o tools/gemm256_lab
#include "../ml-audio-inpainting_amd/csrc/gemm16.hip"

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

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <typename L>
static double time_ms(L launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

static void run(const char* name, int64_t M, int64_t N, int64_t K, int nsplit) {
  const int64_t kc = nsplit > 1 ? ((K / nsplit + 63) / 64) * 64 : K;
  std::vector<uint16_t> ha(M * K), hb(N * K);
  uint32_t s = 777u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    const float f = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f);
    const __bf16 h = (__bf16)f;
    return __builtin_bit_cast(uint16_t, h);
  };
  for (auto& v : ha) v = rnd();
  for (auto& v : hb) v = rnd();
  uint16_t *A, *B;
  float *C0, *C1;
  const size_t csz = (size_t)nsplit * M * N;
  CK(hipMalloc(&A, ha.size() * 2));
  CK(hipMalloc(&B, hb.size() * 2));
  CK(hipMalloc(&C0, csz * 4));
  CK(hipMalloc(&C1, csz * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  g16::Bias b16{nullptr, nullptr, nullptr, nullptr, 0};
  g256::Bias b256{nullptr, nullptr, nullptr, nullptr, 0};
  const int64_t tn16 = (N + 127) / 128, tn256 = (N + 255) / 256;
  auto l16 = [&] {
    hipLaunchKernelGGL(g16::gemm_bf16nt_kernel, dim3((unsigned)(((M + 127) / 128) * tn16), nsplit),
                       dim3(256), 0, 0, M, N, K, A, K, B, K, C0, N, kc, M * N, b16, (int)tn16);
  };
  auto l256 = [&] {
    hipLaunchKernelGGL(g256::gemm_bf16nt_256_kernel,
                       dim3((unsigned)(((M + 255) / 256) * tn256), nsplit), dim3(512),
                       g256::LDS_BYTES, 0, M, N, K, A, K, B, K, C1, N, kc, M * N, b256,
                       (int)tn256);
  };
  CK(hipMemset(C0, 0, csz * 4));
  CK(hipMemset(C1, 0xff, csz * 4));
  l16();
  l256();
  CK(hipDeviceSynchronize());
  std::vector<float> r0(csz), r1(csz);
  CK(hipMemcpy(r0.data(), C0, csz * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), C1, csz * 4, hipMemcpyDeviceToHost));
  size_t ndiff = 0;
  double mx = 0;
  for (size_t i = 0; i < csz; ++i) {
    if (memcmp(&r0[i], &r1[i], 4)) ++ndiff;
    const double e = fabs((double)r0[i] - (double)r1[i]);
    if (!(e <= mx)) mx = e;
  }
  const double flop = 2.0 * M * N * K;
  const double t16 = time_ms(l16, 10), t256 = time_ms(l256, 10);
  printf("%-6s M=%ld N=%ld K=%ld split=%d: gemm16 %.3f ms (%.0f TF)  g256 %.3f ms (%.0f TF)  "
         "differing %zu / %zu (max |d| %.3g)\n",
         name, (long)M, (long)N, (long)K, nsplit, t16, flop / t16 / 1e9, t256,
         flop / t256 / 1e9, ndiff, csz, mx);
  fflush(stdout);
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(C0));
  CK(hipFree(C1));
}

int main() {
  CK(hipFuncSetAttribute((const void*)g256::gemm_bf16nt_256_kernel,
                         hipFuncAttributeMaxDynamicSharedMemorySize, g256::LDS_BYTES));
  run("small", 512, 768, 256, 1);
  run("fwd", 10688, 1024, 16448, 1);
  run("fwd", 10688, 1024, 16448, 3);
  run("dX", 10688, 16448, 1024, 1);
  run("dW", 1024, 16448, 10688, 1);
  run("dW", 1024, 16448, 10688, 2);
  printf("done\n");
  return 0;
}
