// gemm_x6r.hip — fp32-accurate ("x6") GEMMs on a 256 x 256 tile with the
// bf16 split pass overlapped with the MFMAs, and several GEMMs in one launch.
//
// Replaces, for the fp32 configuration (BASELINE C2), the three layer-0 GEMMs
// of nn.LSTM(16448 -> 128, bidirectional) (models/CNNBLSTM/model.py:46-47,77):
// the input projection X W_cat^T, and the backward pair dX = dg W_cat beside
// dW_cat = dg^T X -- launched together as one grid, so neither has to share
// CUs with a second kernel on another stream.
//
// Arithmetic: gemm.hip's x6 scheme -- every fp32 operand element split
// exactly into three bf16 pieces (x = x0 + x1 + x2), the six cross products of
// order >= 2^-16 accumulated per 16-k step as a2b0 + a1b1 + a0b2 + a1b0 + a0b1
// + a0b0 on v_mfma_f32_32x32x16_bf16 (f32 accumulate); with the same k order,
// results are bit-identical to the x6_256 kernels (gemm16.hip).
//
// Tile: 512 threads = 8 waves (2 m x 4 n), each 128 x 64 outputs = 4 x 2
// 32x32 accumulators.  Per 16-deep K-tile:
//   LDS   (static, 160 KB) fp32 ring of 2 stages (A + B, 32 KB each) filled by
//         global_load_lds_dwordx4 (16 B per lane), and two sets of bf16 split
//         planes (3 pieces x (A + B) x 256 rows x 32 B = 48 KB each): 160 KB;
//   step  one barrier: the split of tile kt+1 (fp32 stage -> planes) runs
//         between the MFMA groups of tile kt, the DMA of tile kt+2 flies over
//         the whole iteration.
// Operands may be k-contiguous ("N": element (r,k) at P[r*ld + k]) or
// k-major ("T": P[k*ld + r]) -- the transposition happens in the split pass,
// so dW = dg^T X reads dg and X as they lie.  Per-problem pointer splits
// cover the two LSTM directions (B rows n >= b_nsplit, B or A columns
// k >= *_ksplit from a second tensor; C rows m >= c_msplit to a second one).
#include "common.h"

#include <stdlib.h>

namespace ainp {
namespace x6r {

constexpr int BM = 256, BN = 256, BK = 16, THREADS = 512;
constexpr int ROWB = BK * 4;                 // fp32 N image: 64-byte rows
constexpr int IMG = BM * ROWB;               // 16 KB per operand per stage
constexpr int STAGE = 2 * IMG;               // A + B
constexpr int PROW = 32, PLANE = BM * PROW;  // bf16 plane: 16 k per row
constexpr int PSET = 6 * PLANE;              // A0..A2, B0..B2 = 48 KB
constexpr int LDS_BYTES = 2 * STAGE + 2 * PSET;
static_assert(LDS_BYTES == 160 * 1024, "the whole LDS of a CU");
constexpr int MAXP = 3;

typedef float f32x16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

struct Prob {
  const float* A; const float* A2; int64_t lda, a_ksplit; int a_km;
  const float* B; const float* B2; int64_t ldb, b_nsplit, b_ksplit; int b_km;
  float* C; float* C2; int64_t ldc, c_msplit;
  const float* bias_a1; const float* bias_a2; const float* bias_b1; const float* bias_b2;
  int64_t bias_nsplit;
  int64_t M, N, K, kc, strideC;
  int nsplit, tiles_m, tiles_n;
  int mfast;                 // groups of 8 tiles walk m first (see gemm_x6r_kernel)
  int64_t items, first;      // work items (tiles x splits), first blockIdx (multiple of 8)
};
struct Job {
  Prob p[MAXP];
  int np;
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
__device__ __forceinline__ int pofs(int row, int h) { return row * PROW + 16 * (h ^ ((row >> 3) & 1)); }

__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// DMA of one operand's 256 x 16 fp32 K-tiles into the stage images.
//  N: 16 image rows per wave instruction (lanes 4r..4r+3 = one 64-byte row,
//     chunks XOR-swizzled on the source address);
//  T: one k-row of 256 fp32 (1 KB) per wave instruction, lane l = rows 4l..4l+3.
// The per-lane part of each address is computed once (off[i]); a K-tile adds
// the wave-uniform k offset (and switches to the second tensor past ksplit).
struct Dma {
  const float* p1;    // tensor holding k < ksplit (or all k)
  const float* p2;    // tensor holding k >= ksplit (nullptr: none)
  int64_t ksplit, kbeg, dk;   // dk: floats per unit of k (1: N layout, ld: T layout)
  int64_t off[2];             // per-lane offset of instruction i at k = 0
};

__device__ __forceinline__ Dma dma_setup(const float* P, const float* P2, int64_t ld,
                                         int64_t ksplit, int km, int64_t r0, int64_t R,
                                         int64_t kbeg, int wave, int lane) {
  Dma d;
  d.p1 = P;
  d.p2 = P2;
  d.ksplit = ksplit;
  d.kbeg = kbeg;
  d.dk = km ? ld : 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = 2 * wave + i;
    if (!km) {
      const int row = 16 * blk + (lane >> 2);
      int64_t gr = r0 + row;
      gr = gr < R ? gr : R - 1;
      d.off[i] = gr * ld + 4 * swz(row, lane & 3);
    } else {
      int64_t gr = r0 + 4 * lane;
      gr = gr + 4 <= R ? gr : R - 4;       // R % 4 == 0 (launcher)
      d.off[i] = (int64_t)blk * ld + gr;
    }
  }
  return d;
}

__device__ __forceinline__ void dma_issue(const Dma& d, int64_t k0, unsigned char* img, int wave) {
  const float* base = d.p1;
  int64_t kk = k0;
  if (d.p2 && k0 >= d.ksplit) {    // K-tiles never straddle ksplit (launcher)
    base = d.p2;
    kk = k0 - d.ksplit;
  }
  const float* b = base + kk * d.dk;
#pragma unroll
  for (int i = 0; i < 2; ++i)
    __builtin_amdgcn_global_load_lds(
        (const void*)(b + d.off[i]),
        (__attribute__((address_space(3))) void*)(img + (2 * wave + i) * 1024), 16, 0, 0);
}

// Split-pass operand values of thread t: 8 fp32 of one row (k = 8h .. 8h+7).
//  N image: row = t >> 1, h = t & 1 (two ds_read_b128);
//  T image: row = t & 255, h = t >> 8 (eight ds_read_b32, consecutive rows per wave).
template <int KM>
__device__ __forceinline__ void split_read(const unsigned char* img, int t, float (&x)[8],
                                           int& row, int& h) {
  if (!KM) {
    row = t >> 1;
    h = t & 1;
    const float4 u = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * swz(row, 2 * h));
    const float4 v = *reinterpret_cast<const float4*>(img + row * ROWB + 16 * swz(row, 2 * h + 1));
    x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
    x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
  } else {
    row = t & 255;
    h = t >> 8;
    const float* f = reinterpret_cast<const float*>(img);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = f[(8 * h + e) * 256 + row];
  }
}

__device__ __forceinline__ void split_write(const float (&x)[8], int row, int h,
                                            unsigned char* planes) {
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

__device__ __forceinline__ void mfma6(f32x16v& c, const bf16x8v& a0, const bf16x8v& a1,
                                      const bf16x8v& a2, const bf16x8v& b0, const bf16x8v& b1,
                                      const bf16x8v& b2) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, c, 0, 0, 0);
}

// Static LDS objects (not one dynamic array): the compiler's wait insertion
// can then tell an in-flight LDS-DMA into one fp32 stage from reads of the
// other stage and of the planes, instead of draining vmcnt(0) before every
// ds_read (cdna_hip_programming.md §5: the second-object / glds traps).  The
// K loop is unrolled by two so every buffer index is a compile-time constant.
__shared__ __attribute__((aligned(1024))) unsigned char st_a[STAGE];
__shared__ __attribute__((aligned(1024))) unsigned char st_b[STAGE];
__shared__ __attribute__((aligned(1024))) unsigned char ps_a[PSET];
__shared__ __attribute__((aligned(1024))) unsigned char ps_b[PSET];

template <int PAR>
__device__ __forceinline__ unsigned char* stage_of() { return PAR ? st_b : st_a; }
template <int PAR>
__device__ __forceinline__ unsigned char* planes_of() { return PAR ? ps_b : ps_a; }

// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] |
// vmcnt_hi[15:14]); "max" in the other fields
constexpr int WAIT_VM0 = 0x0F70, WAIT_VM4 = 0x0F74, WAIT_LGKM0 = 0xC07F;

struct Ctx {
  Dma da, db;
  int64_t kbeg;
  int nk, a_km, b_km, tid, wave, wm, wn, li, lh;
};

template <int PAR>
__device__ __forceinline__ void issue_tile(const Ctx& c, int kt) {   // kt & 1 == PAR
  const int64_t k0 = c.kbeg + (int64_t)kt * BK;
  dma_issue(c.da, k0, stage_of<PAR>(), c.wave);
  dma_issue(c.db, k0, stage_of<PAR>() + IMG, c.wave);
}

// one K-tile kt (kt & 1 == PAR): MFMAs on planes PAR; meanwhile tile kt+2's
// DMA into stage PAR and the split of tile kt+1 (stage PAR^1 -> planes PAR^1)
template <int PAR, int AKM, int BKM, bool APF>
__device__ __forceinline__ void ktile(const Ctx& c, int kt, f32x16v (&acc)[4][2]) {
  // tile kt+1's DMA landed (every wave), planes PAR complete, every wave done
  // with tile kt-1 (planes PAR^1) and with the split of tile kt (stage PAR)
  // (the builtin, not inline asm: the compiler's wait insertion then knows
  // the stage PAR^1 DMA has landed and adds no vmcnt(0) before the split reads)
  __builtin_amdgcn_s_waitcnt(WAIT_VM0);
  __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
  __builtin_amdgcn_s_barrier();
  const unsigned char* ps = planes_of<PAR>();
  const unsigned char* st = stage_of<PAR ^ 1>();
  unsigned char* pn = planes_of<PAR ^ 1>();
  // APF: the split runs on every tile, the last included (it then reads a
  // stale stage and writes planes nobody reads again -- every wave is past
  // tile kt-1): the LDS op counts agree on every path, so the compiler's
  // waits before the MFMA groups stay partial instead of lgkmcnt(0)
  const bool nxt = APF || kt + 1 < c.nk;
  bf16x8v b0[2], b1[2], b2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = c.wn + j * 32 + c.li;
    b0[j] = pfrag(ps + 3 * PLANE, row, c.lh);
    b1[j] = pfrag(ps + 4 * PLANE, row, c.lh);
    b2[j] = pfrag(ps + 5 * PLANE, row, c.lh);
  }
  float xa[8], xb[8];
  int ra = 0, ha = 0, rb = 0, hb = 0;
  // APF: the A fragments of row group i+1 are read before group i's MFMAs,
  // so their LDS latency hides under those MFMAs
  bf16x8v a0, a1, a2;
  if (APF) {
    const int row = c.wm + c.li;
    a0 = pfrag(ps, row, c.lh);
    a1 = pfrag(ps + PLANE, row, c.lh);
    a2 = pfrag(ps + 2 * PLANE, row, c.lh);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bf16x8v n0, n1, n2;
    if (APF) {
      if (i < 3) {
        const int row = c.wm + (i + 1) * 32 + c.li;
        n0 = pfrag(ps, row, c.lh);
        n1 = pfrag(ps + PLANE, row, c.lh);
        n2 = pfrag(ps + 2 * PLANE, row, c.lh);
      }
    } else {
      const int row = c.wm + i * 32 + c.li;
      a0 = pfrag(ps, row, c.lh);
      a1 = pfrag(ps + PLANE, row, c.lh);
      a2 = pfrag(ps + 2 * PLANE, row, c.lh);
    }
    __builtin_amdgcn_s_setprio(1);
    mfma6(acc[i][0], a0, a1, a2, b0[0], b1[0], b2[0]);
    mfma6(acc[i][1], a0, a1, a2, b0[1], b1[1], b2[1]);
    __builtin_amdgcn_s_setprio(0);
    if (APF && i < 3) {
      a0 = n0;
      a1 = n1;
      a2 = n2;
    }
    if (i == 0 && kt + 2 < c.nk) issue_tile<PAR>(c, kt + 2);
    if (nxt) {
      if (i == 0) split_read<AKM>(st, c.tid, xa, ra, ha);
      if (i == 1) split_write(xa, ra, ha, pn);
      if (i == 2) split_read<BKM>(st + IMG, c.tid, xb, rb, hb);
      if (i == 3) split_write(xb, rb, hb, pn + 3 * PLANE);
    }
  }
}

template <int AKM, int BKM, bool APF>
__device__ __forceinline__ void kloop(const Ctx& c, f32x16v (&acc)[4][2]) {
  // prologue: tile 0 landed and split into planes 0, tile 1 in flight
  if (c.nk > 0) {
    issue_tile<0>(c, 0);
    if (c.nk > 1) issue_tile<1>(c, 1);
    if (c.nk > 1) __builtin_amdgcn_s_waitcnt(WAIT_VM4);
    else __builtin_amdgcn_s_waitcnt(WAIT_VM0);
    __builtin_amdgcn_s_barrier();
    float x[8];
    int row, h;
    split_read<AKM>(st_a, c.tid, x, row, h);
    split_write(x, row, h, ps_a);
    split_read<BKM>(st_a + IMG, c.tid, x, row, h);
    split_write(x, row, h, ps_a + 3 * PLANE);
  }
  for (int kt = 0; kt < c.nk; kt += 2) {
    ktile<0, AKM, BKM, APF>(c, kt, acc);
    if (kt + 1 < c.nk) ktile<1, AKM, BKM, APF>(c, kt + 1, acc);
  }
}

template <bool APF>
__global__ __launch_bounds__(THREADS, 1) void gemm_x6r_kernel(Job job) {
  // ---- which problem / tile / split (uniform per workgroup)
  const int64_t bid0 = blockIdx.x;
  int pi = 0;
#pragma unroll
  for (int q = 1; q < MAXP; ++q)
    if (q < job.np && bid0 >= job.p[q].first) pi = q;
  const Prob& P = job.p[pi];
  const int64_t n8 = (P.items + 7) / 8 * 8;          // items padded to whole XCD rounds
  const int64_t loc0 = bid0 - P.first;
  const int64_t loc = (loc0 % 8) * (n8 / 8) + loc0 / 8;   // contiguous range per XCD
  if (loc >= P.items) return;
  const int64_t tiles = (int64_t)P.tiles_m * P.tiles_n;
  const int64_t split = loc / tiles, t = loc - split * tiles;
  int64_t m0, n0;
  if (P.mfast) {
    // few m-tiles (the layer-0 weight gradient dW = dg^T X: 4 gate-row tiles):
    // a group of 8 consecutive items on one XCD = all tiles_m m-tiles of
    // 8 / tiles_m n-tiles, so every X panel is streamed into that XCD's L2
    // once for its 4 m-tiles instead of once per m-tile (the small dg panels
    // are re-read from the Infinity Cache)
    const int64_t gn = 8 / P.tiles_m;
    const int64_t per = (int64_t)P.tiles_m * gn;
    const int64_t in_g = t % per;
    m0 = (in_g % P.tiles_m) * BM;
    n0 = ((t / per) * gn + in_g / P.tiles_m) * BN;
  } else {
    const int64_t per_group = 8 * (int64_t)P.tiles_m;
    const int64_t first_n = (t / per_group) * 8;
    const int64_t gsize = (P.tiles_n - first_n) < 8 ? (P.tiles_n - first_n) : 8;
    const int64_t in_g = t % per_group;
    m0 = (in_g / gsize) * BM;
    n0 = (first_n + in_g % gsize) * BN;
  }
  const int64_t kbeg = split * P.kc;
  const int64_t kend = (kbeg + P.kc) < P.K ? (kbeg + P.kc) : P.K;
  // this n-tile's B half (b_nsplit % 256 == 0)
  const bool bhi = P.B2 && P.b_ksplit <= 0 && n0 >= P.b_nsplit;
  const float* Bp = bhi ? P.B2 : P.B;
  const float* Bk2 = (P.B2 && P.b_ksplit > 0) ? P.B2 : nullptr;
  const int64_t nb0 = bhi ? n0 - P.b_nsplit : n0;
  const int64_t NB = bhi ? P.N - P.b_nsplit : ((P.B2 && P.b_ksplit <= 0) ? P.b_nsplit : P.N);
  const float* Ak2 = (P.A2 && P.a_ksplit > 0) ? P.A2 : nullptr;

  Ctx c;
  c.tid = threadIdx.x;
  const int lane = c.tid & 63;
  c.wave = c.tid >> 6;
  c.wm = (c.wave >> 2) * 128;
  c.wn = (c.wave & 3) * 64;
  c.li = lane & 31;
  c.lh = lane >> 5;
  c.kbeg = kbeg;
  c.nk = (int)((kend - kbeg) / BK);
  c.a_km = P.a_km;
  c.b_km = P.b_km;
  c.da = dma_setup(P.A, Ak2, P.lda, P.a_ksplit, P.a_km, m0, P.M, kbeg, c.wave, lane);
  c.db = dma_setup(Bp, Bk2, P.ldb, P.b_ksplit, P.b_km, nb0, NB, kbeg, c.wave, lane);

  f32x16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // operand layouts as template parameters: no runtime branch (and no merged
  // LDS address the compiler cannot attribute) inside the K loop
  if (c.a_km) {
    if (c.b_km) kloop<1, 1, APF>(c, acc);
    else kloop<1, 0, APF>(c, acc);
  } else {
    if (c.b_km) kloop<0, 1, APF>(c, acc);
    else kloop<0, 0, APF>(c, acc);
  }
  // ---- epilogue: D[row=(r&3)+8*(r>>2)+4*lh][col=li] of each 32x32 tile
  float* Cs = P.C;
  float* Cs2 = P.C2;
  if (split) {
    Cs += split * P.strideC;
    if (Cs2) Cs2 += split * P.strideC;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + c.wn + j * 32 + c.li;
    if (n >= P.N) continue;
    float bv = 0.f;
    if (split == 0) {
      if (n < P.bias_nsplit) {
        if (P.bias_a1) bv += P.bias_a1[n];
        if (P.bias_a2) bv += P.bias_a2[n];
      } else {
        if (P.bias_b1) bv += P.bias_b1[n - P.bias_nsplit];
        if (P.bias_b2) bv += P.bias_b2[n - P.bias_nsplit];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + c.wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * c.lh;
        if (m >= P.M) continue;
        float* dst = (Cs2 && m >= P.c_msplit) ? Cs2 + (m - P.c_msplit) * P.ldc
                                              : Cs + m * P.ldc;
        dst[n] = acc[i][j][r] + bv;
      }
  }
}

}  // namespace x6r
}  // namespace ainp

using namespace ainp;

static bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int ainp_gemm_x6_multi(const ainp_x6_problem* probs, int nprobs, void* stream) {
  if (!probs || nprobs < 1 || nprobs > x6r::MAXP)
    return record_msg("ainp_gemm_x6_multi: 1..3 problems");
  x6r::Job job{};
  job.np = nprobs;
  int64_t first = 0;
  for (int q = 0; q < nprobs; ++q) {
    const ainp_x6_problem& s = probs[q];
    x6r::Prob& d = job.p[q];
    const int64_t M = s.M, N = s.N, K = s.K;
    const int nsplit = s.nsplit < 1 ? 1 : s.nsplit;
    const int64_t kc = nsplit == 1 ? K : s.kc;
    bool ok = M > 0 && N > 0 && K > 0 && K % x6r::BK == 0 && s.A && s.B && s.C &&
              a16(s.A) && a16(s.B) && s.lda % 4 == 0 && s.ldb % 4 == 0 && s.ldc >= N &&
              nsplit <= 65535;
    // k-contiguous operands: rows of >= K floats; k-major ones: R % 4 == 0
    const int64_t arows = (s.A2 && s.a_ksplit > 0) ? M : M;
    ok = ok && (s.a_kmajor ? (s.lda >= arows && M % 4 == 0) : s.lda >= (s.A2 ? s.a_ksplit : K));
    const bool bn = s.B2 && s.b_ksplit <= 0;   // B split along n
    ok = ok && (s.b_kmajor ? (s.ldb >= (bn ? s.b_nsplit : N) && N % 4 == 0 &&
                              (!bn || (N - s.b_nsplit) % 4 == 0))
                           : s.ldb >= ((s.B2 && s.b_ksplit > 0) ? s.b_ksplit : K));
    if (s.A2) ok = ok && a16(s.A2) && s.a_ksplit > 0 && s.a_ksplit % x6r::BK == 0 && s.a_ksplit < K;
    if (s.B2)
      ok = ok && a16(s.B2) &&
           (s.b_ksplit > 0 ? (s.b_ksplit % x6r::BK == 0 && s.b_ksplit < K)
                           : (s.b_nsplit > 0 && s.b_nsplit % x6r::BN == 0 && s.b_nsplit < N));
    if (s.C2) ok = ok && s.c_msplit > 0 && s.c_msplit % x6r::BM == 0 && s.c_msplit < M;
    if (nsplit > 1)
      ok = ok && kc >= x6r::BK && kc % x6r::BK == 0 && (int64_t)nsplit * kc >= K &&
           (int64_t)(nsplit - 1) * kc < K && s.strideC >= (s.C2 ? s.c_msplit : M) * s.ldc;
    if (s.A2 && nsplit > 1) ok = ok && s.a_ksplit % kc == 0;   // no K-tile straddles
    if (!ok)
      return record_msg("ainp_gemm_x6_multi: bad problem (K % 16, 16-byte aligned operands, "
                        "ld % 4, k-major rows % 4, splits on tile boundaries, split-K cover)");
    d.A = s.A; d.A2 = s.A2; d.lda = s.lda; d.a_ksplit = s.A2 ? s.a_ksplit : 0; d.a_km = s.a_kmajor;
    d.B = s.B; d.B2 = s.B2; d.ldb = s.ldb; d.b_nsplit = s.b_nsplit;
    d.b_ksplit = s.B2 ? s.b_ksplit : 0; d.b_km = s.b_kmajor;
    d.C = s.C; d.C2 = s.C2; d.ldc = s.ldc; d.c_msplit = s.C2 ? s.c_msplit : M;
    d.bias_a1 = s.bias_a1; d.bias_a2 = s.bias_a2; d.bias_b1 = s.bias_b1; d.bias_b2 = s.bias_b2;
    d.bias_nsplit = s.bias_nsplit;
    d.M = M; d.N = N; d.K = K; d.kc = kc; d.strideC = s.strideC; d.nsplit = nsplit;
    d.tiles_m = (int)cdiv(M, x6r::BM);
    d.tiles_n = (int)cdiv(N, x6r::BN);
    // m-first groups where 8 / tiles_m n-tiles x tiles_m tiles fill a group of
    // 8 exactly (AINP_X6R_MFAST=0: n-first everywhere, A/B)
    static const bool mfast_env = [] {
      const char* e = getenv("AINP_X6R_MFAST");
      return !(e && e[0] == '0');
    }();
    d.mfast = (mfast_env && (d.tiles_m == 2 || d.tiles_m == 4 || d.tiles_m == 8) &&
               d.tiles_n >= 8) ? 1 : 0;
    d.items = (int64_t)d.tiles_m * d.tiles_n * nsplit;
    d.first = first;
    first += (d.items + 7) / 8 * 8;
  }
  if (first > 0x7fffffff) return record_msg("ainp_gemm_x6_multi: grid too large");
  // AINP_X6R_APF=0: A fragments read right before their MFMA group and the
  // split skipped past the last tile (the round-4 main loop), for A/B
  static const bool apf = [] {
    const char* e = getenv("AINP_X6R_APF");
    return !(e && e[0] == '0');
  }();
  if (apf)
    hipLaunchKernelGGL(x6r::gemm_x6r_kernel<true>, dim3((unsigned)first), dim3(x6r::THREADS), 0,
                       as_stream(stream), job);
  else
    hipLaunchKernelGGL(x6r::gemm_x6r_kernel<false>, dim3((unsigned)first), dim3(x6r::THREADS), 0,
                       as_stream(stream), job);
  return check_launch("gemm_x6_multi");
}
