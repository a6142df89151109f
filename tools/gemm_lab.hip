// gemm_lab.hip — A/B bench of f32 MFMA GEMM main-loop structures against the
// shipped ainp_gemm_f32 on the CNNBLSTM layer-0 shapes (tools only, not the
// product).  Build: tools/gemm_lab.sh.  Each variant must be bit-identical to
// the shipped kernel (same per-MFMA k order), which the lab checks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/ainp.h"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ f32x16v mfma32(float a, float b, f32x16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Operand tile staged by glds into a lane-linear LDS image.
//  KC (k contiguous in memory): image [row][BK] with the 16-byte granule index
//     XOR-swizzled by (row / (64/BK)) so ds_read_b128 fragment reads are
//     conflict-free (source address pre-swizzled).
//  MC (rows contiguous): image [BK][R], no swizzle (ds_read_b32 halves).
template <int R, int BK, bool KC, int WAVES>
struct GOp {
  static constexpr int BYTES = R * BK * 4;
  static constexpr int NI = BYTES / 1024 / WAVES;  // glds per wave per tile
  static_assert(NI * 1024 * WAVES == BYTES, "tile must split into 1 KB wave pieces");
  static constexpr int GPR = KC ? BK / 4 : R / 4;  // granules per image row
  static constexpr int RPS = 64 / BK;              // KC rows per 256-byte bank sweep

  __device__ static __forceinline__ int swz(int row) { return (row / RPS) & (GPR - 1); }

  // issue this wave's glds for one tile
  __device__ static __forceinline__ void stage(const float* __restrict__ p, int64_t ld, int64_t r0,
                                               int64_t k0, int64_t Rtot, unsigned char* img,
                                               int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = j * WAVES + wave;
      const int idx = c * 64 + lane;
      const float* src;
      if (KC) {
        const int row = idx / GPR, pp = idx % GPR;
        const int g = pp ^ swz(row);
        int64_t gr = r0 + row;
        if (gr > Rtot - 1) gr = Rtot - 1;
        src = p + gr * ld + k0 + 4 * g;
      } else {
        const int kk = idx / GPR, q = idx % GPR;
        int64_t gr = r0 + 4 * q;
        if (gr > Rtot - 4) gr = Rtot - 4;
        src = p + (k0 + kk) * ld + gr;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(img + c * 1024), 16, 0, 0);
    }
  }

  // LDS byte offset of the fragment (KC: one b128; MC: base of 4 b32 at stride R*4)
  __device__ static __forceinline__ int frag_off(int r, int kg, int h) {
    if (KC) return (r * BK + 4 * ((kg * 2 + h) ^ swz(r))) * 4;
    return ((kg * 8 + 4 * h) * R + r) * 4;
  }
  // fragment of k-group kg (8 k): lane (row r, half h) gets k = 8kg + 4h + e
  __device__ static __forceinline__ float4 frag(const float* s, int r, int kg, int h) {
    if (KC) {
      const int g = (kg * 2 + h) ^ swz(r);
      return *reinterpret_cast<const float4*>(&s[r * BK + 4 * g]);
    }
    const int k = kg * 8 + 4 * h;
    return make_float4(s[(k + 0) * R + r], s[(k + 1) * R + r], s[(k + 2) * R + r],
                       s[(k + 3) * R + r]);
  }
};

// Fragment read hidden from the compiler (it would otherwise guard every LDS
// read behind vmcnt(0) for the in-flight LDS-DMA); the caller waits lgkmcnt.
template <bool KC, int R>
__device__ __forceinline__ void frag_asm(float4& f, unsigned addr) {
  if (KC) {
    asm volatile("ds_read_b128 %0, %1" : "=v"(f) : "v"(addr));
  } else {
    asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:%5\n\t"
                 "ds_read_b32 %2, %4 offset:%6\n\tds_read_b32 %3, %4 offset:%7"
                 : "=v"(f.x), "=v"(f.y), "=v"(f.z), "=v"(f.w)
                 : "v"(addr), "n"(R * 4), "n"(2 * R * 4), "n"(3 * R * 4));
  }
}

template <int N>
__device__ __forceinline__ void lgkm_n(float4& a, float4& b, float4& c, float4& d) {
  constexpr int n = N > 15 ? 15 : N;
  asm volatile("s_waitcnt lgkmcnt(%16)"
               : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z),
                 "+v"(b.w), "+v"(c.x), "+v"(c.y), "+v"(c.z), "+v"(c.w), "+v"(d.x), "+v"(d.y),
                 "+v"(d.z), "+v"(d.w)
               : "n"(n));
}
template <int PER, int NKG>
__device__ __forceinline__ void lgkm_wait(int kg, float4& a, float4& b, float4& c, float4& d) {
  // kg is a compile-time constant after unrolling
  if (kg == NKG - 1) lgkm_n<0>(a, b, c, d);
  else if (kg == NKG - 2) lgkm_n<PER>(a, b, c, d);
  else if (kg == NKG - 3) lgkm_n<2 * PER>(a, b, c, d);
  else lgkm_n<3 * PER>(a, b, c, d);
}

template <int BM, int BK, int NBUF, bool AKC, bool BKC, bool ASMR = false>
__global__ __launch_bounds__(BM / 64 * 2 * 64) void gemm_glds(int64_t M, int64_t N, int64_t K,
                                                             const float* __restrict__ A, int64_t lda,
                                                             const float* __restrict__ B, int64_t ldb,
                                                             float* __restrict__ C, int64_t ldc) {
  constexpr int BN = 128;
  constexpr int WAVES = BM / 64 * 2;
  using OA = GOp<BM, BK, AKC, WAVES>;
  using OB = GOp<BN, BK, BKC, WAVES>;
  constexpr int BUF = OA::BYTES + OB::BYTES;
  constexpr int NLD = OA::NI + OB::NI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NBUF * BUF];

  const int64_t nwg = gridDim.x;
  const int64_t bid0 = blockIdx.x;
  const int64_t xcd = bid0 % 8, slot = bid0 / 8;
  const int64_t q8 = nwg / 8, r8 = nwg % 8;
  const int64_t bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int64_t tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int64_t group = 8;
  const int64_t per_group = group * tiles_m;
  const int64_t g = bid / per_group;
  const int64_t first_n = g * group;
  const int64_t gsize = (tiles_n - first_n) < group ? (tiles_n - first_n) : group;
  const int64_t in_g = bid % per_group;
  const int64_t tn = first_n + (in_g % gsize);
  const int64_t tm = in_g / gsize;
  const int64_t m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int li = lane & 31, lh = lane >> 5;

  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int64_t nk = K / BK;
  auto stage = [&](int64_t it) {
    unsigned char* b = smem + (int)((uint64_t)it % NBUF) * BUF;
    OA::stage(A, lda, m0, it * BK, M, b, wave, lane);
    OB::stage(B, ldb, n0, it * BK, N, b + OA::BYTES, wave, lane);
  };
#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (p < nk) stage(p);

  for (int64_t it = 0; it < nk; ++it) {
    // tiles it .. it+NBUF-2 are in flight; retire tile it (this wave's part)
    const int64_t ahead = nk - 1 - it;  // tiles after it already issued (capped)
    if (NBUF == 3) {
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (NBUF == 4) {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NLD) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // every wave's part of tile it has landed, every wave is done with tile it-1
    asm volatile("s_barrier" ::: "memory");
    if (it + NBUF - 1 < nk) stage(it + NBUF - 1);
    const int cur = (int)((uint64_t)it % NBUF);
    const float* As = reinterpret_cast<const float*>(smem + cur * BUF);
    const float* Bs = reinterpret_cast<const float*>(smem + cur * BUF + OA::BYTES);
    float4 fa[BK / 8][2], fb[BK / 8][2];
    if (ASMR) {
      const unsigned base = (unsigned)(uintptr_t)(smem + cur * BUF);
#pragma unroll
      for (int kg = 0; kg < BK / 8; ++kg) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          frag_asm<AKC, BM>(fa[kg][i], base + OA::frag_off(wm + i * 32 + li, kg, lh));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          frag_asm<BKC, BN>(fb[kg][j], base + OA::BYTES + OB::frag_off(wn + j * 32 + li, kg, lh));
      }
    }
#pragma unroll
    for (int kg = 0; kg < BK / 8; ++kg) {
      float4 af[2], bf[2];
      if (ASMR) {
        // reads retire in issue order: wait until only the later groups' reads
        // are in flight (lgkmcnt saturates at 15, a stronger wait is still correct)
        constexpr int PER = (AKC ? 2 : 8) + (BKC ? 2 : 8);
        lgkm_wait<PER, BK / 8>(kg, fa[kg][0], fa[kg][1], fb[kg][0], fb[kg][1]);
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = fa[kg][i];
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = fb[kg][j];
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = OA::frag(As, wm + i * 32 + li, kg, lh);
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = OB::frag(Bs, wn + j * 32 + li, kg, lh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma32(af[i].x, bf[j].x, acc[i][j]);
          acc[i][j] = mfma32(af[i].y, bf[j].y, acc[i][j]);
          acc[i][j] = mfma32(af[i].z, bf[j].z, acc[i][j]);
          acc[i][j] = mfma32(af[i].w, bf[j].w, acc[i][j]);
        }
    }
    if (NBUF == 2) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn + j * 32 + li;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) C[m * ldc + n] = acc[i][j][r];
      }
    }
}

struct Shape {
  const char* name;
  int64_t M, N, K;
  bool akc, bkc;
};

static void fill(float* d, size_t n, unsigned seed) {
  std::vector<float> h(n);
  uint32_t s = seed * 2654435761u + 1;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
}

typedef void (*Launch)(const Shape&, const float*, const float*, float*, hipStream_t);

template <int BM, int BK, int NBUF, bool AKC, bool BKC, bool ASMR>
static void launch_v(const Shape& s, const float* A, const float* B, float* C, hipStream_t st) {
  const int64_t lda = AKC ? s.K : s.M, ldb = BKC ? s.K : s.N;
  dim3 grid((unsigned)(((s.M + BM - 1) / BM) * ((s.N + 127) / 128)));
  hipLaunchKernelGGL((gemm_glds<BM, BK, NBUF, AKC, BKC, ASMR>), grid, dim3(BM / 64 * 2 * 64), 0, st,
                     s.M, s.N, s.K, A, lda, B, ldb, C, s.N);
}

static void launch_ref(const Shape& s, const float* A, const float* B, float* C, hipStream_t st) {
  // A(m,k): KC -> A[m*K + k]; MC -> A[k*M + m].  B(k,n): KC -> B[n*K + k]; MC -> B[k*N + n]
  const float* Ap[1] = {A};
  const float* Bp[1] = {B};
  float* Cp[1] = {C};
  int rc = ainp_gemm_f32(s.M, s.N, s.K, 1.f, Ap, s.akc ? s.K : 1, s.akc ? 1 : s.M, 0, Bp,
                         s.bkc ? 1 : s.N, s.bkc ? s.K : 1, 0, 0.f, Cp, s.N, 1, 0, nullptr, nullptr,
                         1, 1, 0, st);
  if (rc) {
    fprintf(stderr, "ref gemm rc %d\n", rc);
    exit(1);
  }
}

struct Variant {
  const char* name;
  Launch fn[4];  // [akc*2 + bkc]
};

#define VARIANT(NAME, BM, BK, NB, AS)                                                      \
  {NAME,                                                                                   \
   {launch_v<BM, BK, NB, false, false, AS>, launch_v<BM, BK, NB, false, true, AS>,         \
    launch_v<BM, BK, NB, true, false, AS>, launch_v<BM, BK, NB, true, true, AS>}}

int main(int argc, char** argv) {
  Shape shapes[] = {
      {"fwd  X W^T   M10688 N1024 K16448 (KC,KC)", 10688, 1024, 16448, true, true},
      {"dX   dG W    M10688 N16448 K1024 (KC,MC)", 10688, 16448, 1024, true, false},
      {"dW   dG^T X  M1024 N16448 K10688 (MC,MC)", 1024, 16448, 10688, false, false},
  };
  Variant vars[] = {
      VARIANT("glds 128x128 BK16 3buf", 128, 16, 3, false),
      VARIANT("glds 128x128 BK32 2buf", 128, 32, 2, false),
      VARIANT("glds 128x128 BK16 3buf asm", 128, 16, 3, true),
      VARIANT("glds 128x128 BK16 4buf asm", 128, 16, 4, true),
      VARIANT("glds 128x128 BK32 3buf asm", 128, 32, 3, true),
      VARIANT("glds 256x128 BK16 3buf asm", 256, 16, 3, true),
      VARIANT("glds 256x128 BK32 3buf asm", 256, 32, 3, true),
  };
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    float *A, *B, *C, *Cr;
    CK(hipMalloc(&A, s.M * s.K * 4));
    CK(hipMalloc(&B, s.K * s.N * 4));
    CK(hipMalloc(&C, s.M * s.N * 4));
    CK(hipMalloc(&Cr, s.M * s.N * 4));
    fill(A, s.M * s.K, 1);
    fill(B, s.K * s.N, 2);
    const double flop = 2.0 * s.M * s.N * s.K;
    auto timeit = [&](auto&& fn, float* out) {
      fn(out);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) fn(out);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      return ms / reps;
    };
    const float mr = timeit([&](float* o) { launch_ref(s, A, B, o, st); }, Cr);
    printf("%s\n  %-26s %8.3f ms %7.1f TF\n", s.name, "shipped gemm_f32_kernel", mr,
           flop / mr / 1e9);
    std::vector<float> hr(s.M * s.N), hc(s.M * s.N);
    CK(hipMemcpy(hr.data(), Cr, s.M * s.N * 4, hipMemcpyDeviceToHost));
    for (const Variant& v : vars) {
      Launch fn = v.fn[(s.akc ? 2 : 0) + (s.bkc ? 1 : 0)];
      CK(hipMemset(C, 0, s.M * s.N * 4));
      const float ms = timeit([&](float* o) { fn(s, A, B, o, st); }, C);
      CK(hipGetLastError());
      CK(hipMemcpy(hc.data(), C, s.M * s.N * 4, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < hc.size(); ++i) bad += memcmp(&hc[i], &hr[i], 4) != 0;
      printf("  %-26s %8.3f ms %7.1f TF  mismatches %zu\n", v.name, ms, flop / ms / 1e9, bad);
    }
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(Cr));
  }
  return 0;
}
