// x6split_lab.hip — variant of the fp32 x6 256x256 tile (gemm16.hip x6_256)
// that splits each fp32 K-tile into its three bf16 planes ONCE per workgroup
// (a split pass into an LDS plane buffer between two barriers) instead of
// per fragment in every wave that reads it (4x for A, 2x for B).  Same
// products and order, so the result must be bit-identical to x6_256.
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

namespace x6s {
using g16::bf16x8v;
using g16::Bias;
using g16::f32x16v;
constexpr int BM = 256, BN = 256, BK = 16, THREADS = 512, NST = 3;
constexpr int ROWB = 64, IMG = BM * ROWB, STAGE = 2 * IMG;       // fp32 ring
constexpr int PROW = 32, PLANE = BM * PROW;                      // bf16 planes: 16 k per row
constexpr int PLANES = 2 * 3 * PLANE;                            // A0..A2, B0..B2
constexpr int LDS_BYTES = NST * STAGE + PLANES;                  // 96 + 48 KB
static_assert(LDS_BYTES <= 160 * 1024, "fits");

// plane chunk h (k = 8h..8h+7) of row r, swizzled so rows r and r+8 differ
__device__ __forceinline__ int pofs(int row, int h) { return row * PROW + 16 * (h ^ ((row >> 3) & 1)); }

__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// thread t splits row t>>1, k = 8*(t&1) .. +7 of one operand's fp32 image
__device__ __forceinline__ void split_row(const unsigned char* img, unsigned char* planes, int t) {
  const int row = t >> 1, h = t & 1;
  const float4 u = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h));
  const float4 v = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * g256::swz(row, 2 * h + 1));
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  uint32_t q0[4], q1[4], q2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = x[2 * e], b = x[2 * e + 1];
    q0[e] = cvt_pk(a, b);
    const float ra = a - __uint_as_float(q0[e] << 16), rb = b - __uint_as_float(q0[e] & 0xffff0000u);
    q1[e] = cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(q1[e] << 16), sb = rb - __uint_as_float(q1[e] & 0xffff0000u);
    q2[e] = cvt_pk(sa, sb);
  }
  const int o = pofs(row, h);
  *reinterpret_cast<uint4*>(planes + o) = make_uint4(q0[0], q0[1], q0[2], q0[3]);
  *reinterpret_cast<uint4*>(planes + PLANE + o) = make_uint4(q1[0], q1[1], q1[2], q1[3]);
  *reinterpret_cast<uint4*>(planes + 2 * PLANE + o) = make_uint4(q2[0], q2[1], q2[2], q2[3]);
}

__device__ __forceinline__ bf16x8v pfrag(const unsigned char* plane, int row, int h) {
  return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(plane + pofs(row, h)));
}

__global__ __launch_bounds__(THREADS, 1) void gemm_x6nt_split_kernel(
    int64_t M, int64_t N, int64_t K, const float* __restrict__ A, int64_t lda,
    const float* __restrict__ B1, const float* __restrict__ B2, int64_t ldb, int64_t bsplit,
    float* __restrict__ C, int64_t ldc, int64_t kc, int64_t strideC, Bias bias, int tiles_n) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];
  unsigned char* planes = smem + NST * STAGE;
  const int64_t nwg = gridDim.x, bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8, q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t per_group = 8 * tiles_m;
  const int64_t first_n = (bid / per_group) * 8;
  const int64_t gsize = (tiles_n - first_n) < 8 ? (tiles_n - first_n) : 8;
  const int64_t in_g = bid % per_group;
  const int64_t m0 = (in_g / gsize) * BM, n0 = (first_n + in_g % gsize) * BN;
  const bool hi = n0 >= bsplit;
  const float* Bp = hi ? B2 : B1;
  const int64_t nb0 = hi ? n0 - bsplit : n0, NB = hi ? N - bsplit : bsplit;
  const int64_t split = blockIdx.y;
  const int64_t kbeg = split * kc;
  const int64_t kend = (kbeg + kc) < K ? (kbeg + kc) : K;
  float* Cs = C + split * strideC;
  const int nk = (int)((kend - kbeg) / BK);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 2) * 128, wn = (wave & 3) * 64;
  const int li = lane & 31, lh = lane >> 5;
  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NST) * STAGE;
    x6_256::stage(A, lda, m0, M, kbeg + (int64_t)kt * BK, st, wave, lane);
    x6_256::stage(Bp, ldb, nb0, NB, kbeg + (int64_t)kt * BK, st + IMG, wave, lane);
  };
#pragma unroll
  for (int q = 0; q < NST - 1; ++q)
    if (q < nk) issue(q);

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (tile kt+1 may stay in flight); every wave is done with
    // the planes of tile kt-1 and with its fp32 stage
    if (nk - 1 - kt >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) issue(kt + NST - 1);
    const unsigned char* st = smem + (kt % NST) * STAGE;
    split_row(st, planes, tid);                       // A rows
    split_row(st + IMG, planes + 3 * PLANE, tid);     // B rows
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8v b0[2], b1[2], b2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn + j * 32 + li;
      b0[j] = pfrag(planes + 3 * PLANE, row, lh);
      b1[j] = pfrag(planes + 4 * PLANE, row, lh);
      b2[j] = pfrag(planes + 5 * PLANE, row, lh);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm + i * 32 + li;
      const bf16x8v a0 = pfrag(planes, row, lh), a1 = pfrag(planes + PLANE, row, lh),
                    a2 = pfrag(planes + 2 * PLANE, row, lh);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x16v c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0[j], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn + j * 32 + li;
    if (n >= N) continue;
    float bv = 0.f;
    if (split == 0) {
      if (n < bias.nsplit) {
        if (bias.a1) bv += bias.a1[n];
        if (bias.a2) bv += bias.a2[n];
      } else {
        if (bias.b1) bv += bias.b1[n - bias.nsplit];
        if (bias.b2) bv += bias.b2[n - bias.nsplit];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cs[m * ldc + n] = acc[i][j][r] + bv;
      }
  }
}
}  // namespace x6s
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
  CK(hipFuncSetAttribute((const void*)x6s::gemm_x6nt_split_kernel,
                         hipFuncAttributeMaxDynamicSharedMemorySize, x6s::LDS_BYTES));
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
      hipLaunchKernelGGL(x6s::gemm_x6nt_split_kernel, dim3((unsigned)(tm * tn), S), dim3(512),
                         x6s::LDS_BYTES, 0, M, N, K, A, K, W, W + 4 * H * K, K, 4 * H, C1, N, kc,
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
