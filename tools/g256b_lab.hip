// g256b_lab.hip — round 6 lab: the bf16 layer-0 GEMM tile (gemm16.hip g256,
// 256 x 256, 32-deep K-tiles, 4-stage LDS-DMA ring, one barrier per K-tile,
// fragments read right before their MFMAs) against a 64-deep K-tile variant:
// two 64 KB stages (128-byte image rows, 16-byte chunks XOR-swizzled by the
// row's low 3 bits), 32 MFMAs per wave between barriers, the next k-step's
// fragments read while the current k-step's MFMAs run.  Same MFMA, same k
// order, so the results must be bit-identical.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/g256b_lab.hip -o tools/g256b_lab
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

namespace g64 {
constexpr int BM = 256, BN = 256, BK = 64, NST = 2;
constexpr int ROWB = BK * 2;          // 128-byte image rows
constexpr int IMG = BM * ROWB;        // 32 KB per operand per stage
constexpr int STAGE = 2 * IMG;
constexpr int LDS_BYTES = NST * STAGE;   // 128 KB
using g16::bf16x8v;
using g16::f32x16v;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

// one operand's 256 x 64 K-tile: wave w, instruction i covers rows
// 8 (4w + i) .. +8; lane L -> row + L/8, physical chunk L % 8
template <int NW>
__device__ __forceinline__ void stage(const uint16_t* __restrict__ P, int64_t ld, int64_t r0,
                                      int64_t R, int64_t k0, unsigned char* img, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 32 / NW; ++i) {
    const int blk = (32 / NW) * wave + i;
    const int row = 8 * blk + (lane >> 3);
    const int c = swz(row, lane & 7);
    int64_t gr = r0 + row;
    gr = gr < R ? gr : R - 1;
    const uint16_t* src = P + gr * ld + k0 + 8 * c;
    __builtin_amdgcn_global_load_lds(
        (const void*)src, (__attribute__((address_space(3))) void*)(img + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8v frag(const unsigned char* img, int row, int chunk) {
  return __builtin_bit_cast(bf16x8v,
                            *reinterpret_cast<const uint4*>(img + row * ROWB + 16 * swz(row, chunk)));
}

template <int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_bf16nt_g64_kernel(
    int64_t M, int64_t N, int64_t K, const uint16_t* __restrict__ A, int64_t lda,
    const uint16_t* __restrict__ B, int64_t ldb, float* __restrict__ C, int64_t ldc, int64_t kc,
    int64_t strideC, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  const int nk = (int)((kend - kbeg) / BK);
  float* Cs = C + split * strideC;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = WGM * WGN, TI = 256 / WGM / 32, TJ = 256 / WGN / 32;
  const int wm = (wave / WGN) * (32 * TI), wn = (wave % WGN) * (32 * TJ);
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NST) * STAGE;
    stage<NW>(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    stage<NW>(B, ldb, n0, N, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
  };
  if (nk > 0) issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile kt (the only DMA in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's DMAs of kt; every wave done with kt-1
    asm volatile("" ::: "memory");
    if (kt + 1 < nk) issue(kt + 1);  // into kt-1's stage
    const unsigned char* sa = smem + (kt % NST) * STAGE;
    const unsigned char* sb = sa + IMG;
    bf16x8v fa[2][TI], fb[2][TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[0][j] = frag(sb, wn + j * 32 + li, lh);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[0][i] = frag(sa, wm + i * 32 + li, lh);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[cur ^ 1][j] = frag(sb, wn + j * 32 + li, 2 * (ks + 1) + lh);
#pragma unroll
        for (int i = 0; i < TI; ++i) fa[cur ^ 1][i] = frag(sa, wm + i * 32 + li, 2 * (ks + 1) + lh);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][i], fb[cur][j], acc[i][j], 0,
                                                              0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r];
      }
  }
}
}  // namespace g64
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
  // split length a multiple of 64 (both kernels' K-tiles)
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
  g256::Bias b256{nullptr, nullptr, nullptr, nullptr, 0};
  const int64_t tn256 = (N + 255) / 256;
  const unsigned grid = (unsigned)(((M + 255) / 256) * tn256);
  auto l256 = [&] {
    hipLaunchKernelGGL(g256::gemm_bf16nt_256_kernel, dim3(grid, nsplit), dim3(512),
                       g256::LDS_BYTES, 0, M, N, K, A, K, B, K, C0, N, kc, M * N, b256,
                       (int)tn256);
  };
  auto l64 = [&] {
    hipLaunchKernelGGL((g64::gemm_bf16nt_g64_kernel<2, 4>), dim3(grid, nsplit), dim3(512),
                       g64::LDS_BYTES, 0, M, N, K, A, K, B, K, C1, N, kc, M * N, (int)tn256);
  };
  auto l64w4 = [&] {
    hipLaunchKernelGGL((g64::gemm_bf16nt_g64_kernel<2, 2>), dim3(grid, nsplit), dim3(256),
                       g64::LDS_BYTES, 0, M, N, K, A, K, B, K, C1, N, kc, M * N, (int)tn256);
  };
  CK(hipMemset(C0, 0, csz * 4));
  CK(hipMemset(C1, 0xff, csz * 4));
  l256();
  l64();
  CK(hipDeviceSynchronize());
  std::vector<float> r0(csz), r1(csz);
  CK(hipMemcpy(r0.data(), C0, csz * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), C1, csz * 4, hipMemcpyDeviceToHost));
  size_t ndiff = 0;
  for (size_t i = 0; i < csz; ++i)
    if (memcmp(&r0[i], &r1[i], 4)) ++ndiff;
  CK(hipMemset(C1, 0xff, csz * 4));
  l64w4();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(r1.data(), C1, csz * 4, hipMemcpyDeviceToHost));
  size_t ndiff4 = 0;
  for (size_t i = 0; i < csz; ++i)
    if (memcmp(&r0[i], &r1[i], 4)) ++ndiff4;
  const double flop = 2.0 * M * N * K;
  const double t256 = time_ms(l256, 10), t64 = time_ms(l64, 10), t4 = time_ms(l64w4, 10);
  printf("%-6s M=%ld N=%ld K=%ld split=%d: g256 %.3f ms (%.0f TF)  g64 %.3f ms (%.0f TF, diff %zu)"
         "  g64w4 %.3f ms (%.0f TF, diff %zu) of %zu\n",
         name, (long)M, (long)N, (long)K, nsplit, t256, flop / t256 / 1e9, t64, flop / t64 / 1e9,
         ndiff, t4, flop / t4 / 1e9, ndiff4, csz);
  fflush(stdout);
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(C0));
  CK(hipFree(C1));
}

int main() {
  CK(hipFuncSetAttribute((const void*)g256::gemm_bf16nt_256_kernel,
                         hipFuncAttributeMaxDynamicSharedMemorySize, g256::LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)g64::gemm_bf16nt_g64_kernel<2, 4>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, g64::LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)g64::gemm_bf16nt_g64_kernel<2, 2>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, g64::LDS_BYTES));
  run("small", 512, 768, 256, 1);
  run("fwd", 10688, 1024, 16448, 3);
  run("dX", 10688, 16448, 1024, 1);
  run("sq8k", 8192, 8192, 8192, 1);
  printf("done\n");
  return 0;
}
