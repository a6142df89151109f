// conv_x6.hip — 3x3 / stride 1 / pad 1 convolution (forward and data gradient)
// of models/CNNBLSTM/model.py:35-60 on the bf16 MFMA with fp32 accuracy.
//
// Same arithmetic idea as gemm.hip's x6 loop: every fp32 operand element is
// split exactly into three bf16 pieces (x = x0 + x1 + x2, round-to-nearest at
// each step) when it is staged into LDS, and each product is accumulated as
// the six cross terms of order >= 2^-16 on v_mfma_f32_32x32x16_bf16 (f32
// accumulation; dropped terms <= ~2^-23 |a||b|, the level of f32 rounding).
//
// Implicit GEMM D[co][pixel] = sum_{tap, ci} w[co][ci][tap] * act(x)[ci][pixel + tap]:
//  * workgroup = 8 waves = one example's 16 rows x 32 columns of output; wave w
//    owns rows 2w, 2w+1 (one 32-pixel MFMA column tile each) x COP channels
//    (COP/32 MFMA row tiles);
//  * K is walked in chunks of 16 input channels; per chunk the halo tile
//    (18 x 34 pixels x 16 channels) is staged channel-last -- each pixel's 16
//    channels are 32 contiguous bytes per piece, the 16-byte halves XOR-swizzled
//    by column bit 3 -- so the B fragment of tap (dy, dx) is ONE ds_read_b128
//    per lane at pixel (row+dy, col+dx), conflict-free for every shift;
//  * the chunk's weights [co][tap][16 ci] (304-byte rows) are split and staged
//    the same way (the A fragment of a tap is one ds_read_b128);
//  * one MFMA k-step = one tap x 16 channels: 9 k-steps per chunk;
//  * act(x) = relu(x*scale+shift) (the previous BatchNorm2d + ReLU) is applied
//    while staging, and zero padding after it (nn.Conv2d pads its post-ReLU
//    input);
//  * epilogue: bias, store, per-workgroup (sum, sum of squares) partials of
//    each output channel for the following BatchNorm (fp64, fixed order).
// dgrad is the same kernel over dy with w'[ci][co][tap] = w[co][ci][8 - tap].
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace ainp {

namespace cx6 {
constexpr int TR = 16, TC = 32;          // output rows x columns per workgroup
constexpr int HR = TR + 2, HC = TC + 2;  // halo tile
constexpr int CK = 16;                   // input channels per K chunk
constexpr int XROW = HC * 32;            // bytes per halo row per piece (16 bf16 / pixel)
constexpr int XPLANE = HR * XROW;        // 19584
constexpr int WROW = 9 * 32 + 16;        // bytes per weight row (9 taps x 16 bf16 + pad)
constexpr int NT = 512;                  // threads (8 waves)
constexpr int XU = 2 * HR * HC;          // halo staging units (pixel, channel half)
constexpr int XI = (XU + NT - 1) / NT;   // units per thread (3)
}  // namespace cx6

typedef __bf16 bf16x8c __attribute__((ext_vector_type(8)));

// activation layouts of a launch (bitmask): input / output / dy channel-last
constexpr int CL_X = 1, CL_Y = 2, CL_G = 4;
// round 6: a data gradient's dx written [C][H][N][W] (AINP_CONV_YCFNT) -- the
// [C*F, N*T] operand of the fp32 output projection's backward GEMMs, so the
// transposing copy of the decoder input gradient disappears (x6q only)
constexpr int CL_CF = 8;

__device__ __forceinline__ int wx6_clamp(int v, int lo, int hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
// buffer loads: 32-bit per-lane offsets + a scalar channel-plane offset, so no
// per-load 64-bit addresses are kept live across the tile loop
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wx6_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ float wx6_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// Activation / gradient operands stored as fp32 or, G16, as bf16 (the bf16
// configuration's BatchNorm-backward outputs, AINP_CONV_DY16): element size,
// the buffer over element e0 of p, and one element load at byte offsets.
template <bool G16>
constexpr int act_es() { return G16 ? 2 : 4; }
template <bool G16>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t act_rsrc(const float* p, int64_t e0) {
  const char* b = reinterpret_cast<const char*>(p) + e0 * act_es<G16>();
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(b), (short)0, 0x7fffffff,
                                           0x00020000);
}
// Forward output y in bf16 storage (Y16, AINP_CONV_Y16: the bf16
// configuration's pre-BatchNorm activations): the value as stored, whose
// BatchNorm partials the epilogue then sums.
__device__ __forceinline__ float y16_round(float v) { return (float)(__bf16)v; }
__device__ __forceinline__ void y16_st(float* y, int64_t e, float vr) {
  reinterpret_cast<uint16_t*>(y)[e] = __builtin_bit_cast(uint16_t, (__bf16)vr);
}
template <bool G16>
__device__ __forceinline__ float act_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  if constexpr (G16)
    return __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0) << 16);
  else
    return wx6_ld(r, voff, soff);
}
typedef __bf16 bf16x4c __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t cx6_cvt_pk(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

// Channel-last activations (round 5): [N][H][W][C], a pixel's channels
// contiguous.  8 consecutive channels are one 16-byte (bf16 storage) or two
// 16-byte (fp32) buffer loads at byte offset voff -- the staging units of
// the kernels below are (pixel, 8-channel group), so a unit is one or two
// vector loads instead of 8 plane-strided scalar ones, and consecutive lanes
// read consecutive bytes.
template <bool G16>
__device__ __forceinline__ void cl_ld8(__amdgpu_buffer_rsrc_t r, int voff, float (&v)[8]) {
  if constexpr (G16) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(q[j] << 16);
      v[2 * j + 1] = __uint_as_float(q[j] & 0xffff0000u);
    }
  } else {
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = __uint_as_float(a[j]);
      v[4 + j] = __uint_as_float(b[j]);
    }
  }
}
// 4 consecutive channels of one channel-last pixel: fp32 (16 B) or bf16
// (8 B, round-to-nearest-even; exact for values already rounded by y16_round)
template <bool Y16>
__device__ __forceinline__ void cl_st4(float* y, int64_t e, float a, float b, float c, float d) {
  if constexpr (Y16) {
    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + e) =
        make_uint2(cx6_cvt_pk(a, b), cx6_cvt_pk(c, d));
  } else {
    *reinterpret_cast<float4*>(y + e) = make_float4(a, b, c, d);
  }
}

// Round 5: the BatchNorm-backward reduce of the layer a data gradient feeds
// (bn.hip bn_relu_bwd_reduce_cl), fused into the data gradient's epilogue.
// With y = that layer's pre-BatchNorm output (channel-last, fp32 or bf16
// storage) and v the dx value just computed, the epilogue sums
//   gz = v if y * scale + shift > 0 else 0   and   gz * (y - mean) * rstd
// in the (sum, sum of squares) slots of the forward's BatchNorm partials --
// the [part][2C] rows bn_cl_partials_sum reduces -- so the separate reduce
// pass (a full re-read of dx and y) goes away.  Bnr: common.h.
// 16 values per lane of a 32x32 MFMA accumulator -> lane li (of its 32-lane
// half) holds the sum over the half of value li >> 1 (fixed butterfly order)
__device__ __forceinline__ float x6_reduce16(const float (&v)[16], int li) {
  float t8[8], t4[4], t2[2];
  const bool b4 = li & 16, b3 = li & 8, b2 = li & 4, b1 = li & 2;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    t8[k] = (b4 ? v[k + 8] : v[k]) + __shfl_xor(b4 ? v[k] : v[k + 8], 16, 64);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    t4[k] = (b3 ? t8[k + 4] : t8[k]) + __shfl_xor(b3 ? t8[k] : t8[k + 4], 8, 64);
#pragma unroll
  for (int k = 0; k < 2; ++k)
    t2[k] = (b2 ? t4[k + 2] : t4[k]) + __shfl_xor(b2 ? t4[k] : t4[k + 2], 4, 64);
  const float t1 = (b1 ? t2[1] : t2[0]) + __shfl_xor(b1 ? t2[0] : t2[1], 2, 64);
  return t1 + __shfl_xor(t1, 1, 64);
}

// split 8 floats into three packed bf16 vectors (8 x bf16 each), exactly
__device__ __forceinline__ void cx6_split8(const float (&v)[8], uint4& p0, uint4& p1, uint4& p2) {
  uint32_t q0[4], q1[4], q2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a = v[2 * e], b = v[2 * e + 1];
    q0[e] = cx6_cvt_pk(a, b);
    const float ra = a - __uint_as_float(q0[e] << 16), rb = b - __uint_as_float(q0[e] & 0xffff0000u);
    q1[e] = cx6_cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(q1[e] << 16), sb = rb - __uint_as_float(q1[e] & 0xffff0000u);
    q2[e] = cx6_cvt_pk(sa, sb);
  }
  p0 = make_uint4(q0[0], q0[1], q0[2], q0[3]);
  p1 = make_uint4(q1[0], q1[1], q1[2], q1[3]);
  p2 = make_uint4(q2[0], q2[1], q2[2], q2[3]);
}

// Stage 8 activation / weight values as NP bf16 planes `plane` bytes apart:
// NP = 3 -- the exact split (fp32-accurate path); NP = 1 -- one bf16 rounding
// (round-to-nearest-even: the bf16 configurations' operand precision).
template <int NP>
__device__ __forceinline__ void cx6_stage(const float (&v)[8], unsigned char* d, int plane) {
  if (NP == 1) {
    *reinterpret_cast<uint4*>(d) = make_uint4(cx6_cvt_pk(v[0], v[1]), cx6_cvt_pk(v[2], v[3]),
                                              cx6_cvt_pk(v[4], v[5]), cx6_cvt_pk(v[6], v[7]));
  } else {
    uint4 p0, p1, p2;
    cx6_split8(v, p0, p1, p2);
    *reinterpret_cast<uint4*>(d) = p0;
    *reinterpret_cast<uint4*>(d + plane) = p1;
    *reinterpret_cast<uint4*>(d + 2 * plane) = p2;
  }
}
// MFMA terms per product: the six cross terms of order >= 2^-16, smallest
// first (plane of A, plane of B), or the single bf16 product
__host__ __device__ constexpr int cx6_terms(int NP) { return NP == 3 ? 6 : 1; }
__host__ __device__ constexpr int cx6_pa(int NP, int t) {
  return NP == 1 ? 0 : (t == 0 ? 2 : (t == 1 || t == 3) ? 1 : 0);
}
__host__ __device__ constexpr int cx6_pb(int NP, int t) {
  return NP == 1 ? 0 : (t == 2 ? 2 : (t == 1 || t == 4) ? 1 : 0);
}

__device__ __forceinline__ bf16x8c cx6_ld(const unsigned char* p) {
  return __builtin_bit_cast(bf16x8c, *reinterpret_cast<const uint4*>(p));
}

// bf16 channel-last data gradient fed by LDS-DMA (round 5): the 64 -> 32
// channel data gradient of the bf16 configuration (dy = the BatchNorm-backward
// output gy, bf16 channel-last, no prologue: nothing to transform on the way
// into LDS).  The conv3x3_x6_kernel<64, 32, dgrad, RPW 1, NP 1> instance
// stages each 16-channel chunk's halo through registers and waits for it
// once per chunk (SQ: MFMA busy 0.14, waits 0.69); here one persistent
// workgroup per CU keeps the chunk images of the whole 64-channel halo in
// LDS, double-buffered: global_load_lds_dwordx4 brings tile i+1's halo while
// tile i's 36 MFMA steps run.  Same LDS image layout (per 16-channel plane:
// [row][col][16], halves swizzled by column bit 3), same weights image, same
// chunk -> tap MFMA order as the register-staged kernel: bit-identical.
namespace cdd {
constexpr int CI = 64, COP = 32, TR = 8, TC = 32, HR = TR + 2, HC = TC + 2;
constexpr int XROW = HC * 32, XPLANE = HR * XROW;           // 1088, 10880
constexpr int NPIX = HR * HC;                                // 340 halo pixels
constexpr int XBLK = (NPIX * 32 + 1023) / 1024;              // 11 DMA blocks per plane
constexpr int XPP = XBLK * 1024;                             // padded plane
constexpr int NCK = CI / 16;                                 // 4 planes
constexpr int XBUF = NCK * XPP;                              // 45056 per halo buffer
constexpr int WROW = 9 * 32 + 16, WPLANE = COP * WROW;       // 304, 9728
constexpr int NT = 512;
constexpr int YBLK = TR * TC * COP * 2 / 1024;              // 16 blocks: bf16 y of a tile
}  // namespace cdd
__device__ __attribute__((aligned(64))) uint16_t cdd_zero[8];   // zero-initialised

// global_load_lds_dwordx4 issued from inline asm (the recipe of
// cdna_hip_programming.md, M0 saved and restored in the statement): hipcc does
// not track it, so it neither drains it with vmcnt(0) before the LDS reads of
// other ring stages nor counts it -- the kernel's own counted vmcnt waits do.
__device__ __forceinline__ void glds16_asm(const void* gsrc, const unsigned char* lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(dst)
               : "memory");
}


// WREG (round 6): the wave's 36 weight fragments held in VGPRs (144) for the
// whole kernel instead of re-read from LDS per tile -- half the LDS read
// traffic of the MFMA loop (the LDS, 162 KB, allows one workgroup per CU
// either way)
template <bool WREG>
__global__ __launch_bounds__(cdd::NT, WREG ? 1 : 2) void conv3x3_dgrad_b16dma_kernel(
    const uint16_t* __restrict__ gy, const float* __restrict__ w, float* __restrict__ dx,
    double* __restrict__ stats, Bnr bnr, int N, int H, int W, int ntr, int ntc, int64_t ntiles) {
  using namespace cdd;
  __shared__ __attribute__((aligned(1024))) unsigned char sxa[XBUF];
  __shared__ __attribute__((aligned(1024))) unsigned char sxb[XBUF];
  __shared__ __attribute__((aligned(16))) unsigned char sw[NCK * WPLANE];
  // fused BatchNorm-backward reduce (stats != nullptr, bf16 y): the tile's y
  // [8 x 32 pixels][32 channels] rides the halo DMA into a second double
  // buffer, the layer's constants sit in sbn -- the epilogue waits on LDS only
  __shared__ __attribute__((aligned(1024))) unsigned char sya[YBLK * 1024];
  __shared__ __attribute__((aligned(1024))) unsigned char syb[YBLK * 1024];
  __shared__ float sbn[4 * COP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const bool fz = stats != nullptr;
  if (fz) bnr_stage(bnr, sbn, COP, COP, tid, NT);
  // weights once: plane kc, row co, tap, half -> w'[co][kc*16 + 8h + c][tap]
  // = w[kc*16 + 8h + c][co][8 - tap] (the forward weight [64][32][3][3])
  for (int u = tid; u < NCK * COP * 18; u += NT) {
    const int half = u & 1, tap = (u >> 1) % 9, co = (u / 18) % COP, kc = u / (18 * COP);
    float pw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int ci = kc * 16 + 8 * half + c;
      pw[c] = w[((int64_t)ci * COP + co) * 9 + (8 - tap)];
    }
    cx6_stage<1>(pw, sw + kc * WPLANE + co * WROW + tap * 32 + 16 * half, WPLANE);
  }
  // halo DMA of tile t into buffer buf: plane kc, block j (32 linear halo
  // pixels, 1 KB); lane L -> pixel 32 j + L/2, physical half L % 2 holding
  // the logical half (L % 2) ^ (col bit 3)
  // y block j of the tile (fz): lane L -> pixel 16 j + L/4, channels 8 (L % 4) ..
  const uint16_t* yg = reinterpret_cast<const uint16_t*>(bnr.y);
  auto issue = [&](int64_t t, unsigned char* buf, unsigned char* ybuf) {
    const int tc = (int)(t % ntc), tr = (int)((t / ntc) % ntr), n = (int)(t / ((int64_t)ntc * ntr));
    const int r0 = tr * TR, c0 = tc * TC;
    const int nblk = NCK * XBLK + (fz ? YBLK : 0);
    for (int q = wave; q < nblk; q += NT / 64) {
      const uint16_t* src = cdd_zero;
      unsigned char* dst;
      if (q < NCK * XBLK) {
        const int kc = q / XBLK, j = q % XBLK;
        const int lp = 32 * j + (lane >> 1);
        if (lp < NPIX) {
          const int row = lp / HC, col = lp % HC;
          const int gr = r0 - 1 + row, gc = c0 - 1 + col;
          const int hl = (lane & 1) ^ ((col >> 3) & 1);
          if (gr >= 0 && gr < H && gc >= 0 && gc < W)
            src = gy + (((int64_t)n * H + gr) * W + gc) * CI + kc * 16 + 8 * hl;
        }
        dst = buf + kc * XPP + j * 1024;
      } else {
        const int j = q - NCK * XBLK, p = 16 * j + (lane >> 2);
        const int gr = r0 + (p >> 5), gc = c0 + (p & 31);
        if (gr < H && gc < W) src = yg + (((int64_t)n * H + gr) * W + gc) * COP + 8 * (lane & 3);
        dst = ybuf + j * 1024;
      }
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  // fused BatchNorm-backward reduce (stats != nullptr): lane li of half lh
  // ends up holding channel row li >> 1's sums (x6p's butterfly)
  double bs = 0.0, bq = 0.0;
  bf16x8c wa[WREG ? NCK : 1][WREG ? 9 : 1];
  if constexpr (WREG) {
    __syncthreads();   // the staged weights
#pragma unroll
    for (int kc = 0; kc < NCK; ++kc)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        wa[kc][tap] = cx6_ld(sw + kc * WPLANE + li * WROW + tap * 32 + 16 * lh);
  }
  int64_t t = blockIdx.x;
  if (t < ntiles) issue(t, sxa, sya);
  bool cur_a = true;
  for (; t < ntiles; t += gridDim.x) {
    unsigned char* sx = cur_a ? sxa : sxb;
    const unsigned char* sy = cur_a ? sya : syb;
    // this tile's halo landed (every wave's DMA), the weights are staged
    __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0)
    __syncthreads();
    const int64_t tn = t + gridDim.x;
    if (tn < ntiles) issue(tn, cur_a ? sxb : sxa, cur_a ? syb : sya);   // lands during this tile
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int kc = 0; kc < NCK; ++kc) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dxx = tap % 3;
        const int hcol = li + dxx;
        const bf16x8c a = WREG ? wa[WREG ? kc : 0][WREG ? tap : 0]
                               : cx6_ld(sw + kc * WPLANE + li * WROW + tap * 32 + 16 * lh);
        const bf16x8c b = cx6_ld(sx + kc * XPP + (wave + dy) * XROW + hcol * 32 +
                                 16 * (lh ^ ((hcol >> 3) & 1)));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
      }
    }
    // epilogue: D[co = (r&3) + 8(r>>2) + 4lh][pixel col li] of output row
    // r0 + wave; channel-last, 4 consecutive channels per 16-byte store
    const int tc = (int)(t % ntc), tr = (int)((t / ntc) % ntr), n = (int)(t / ((int64_t)ntc * ntr));
    const int row = tr * TR + wave, col = tc * TC + li;
    const bool pok = row < H && col < W;
    const int64_t e0 = (((int64_t)n * H + row) * W + col) * COP;
    if (pok) {
      float* d = dx + e0;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int co0 = 8 * rb + 4 * lh;
        *reinterpret_cast<float4*>(d + co0) =
            make_float4(acc[4 * rb], acc[4 * rb + 1], acc[4 * rb + 2], acc[4 * rb + 3]);
      }
    }
    if (fz) {
      float s1[16], s2[16];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int co0 = 8 * rb + 4 * lh;
        const uint2 u = *reinterpret_cast<const uint2*>(sy + (wave * 32 + li) * 64 + co0 * 2);
        float yv[4];
        bnr_dec4(1, make_uint4(u.x, u.y, 0u, 0u), yv);
        const float v4[4] = {acc[4 * rb], acc[4 * rb + 1], acc[4 * rb + 2], acc[4 * rb + 3]};
        bnr_terms4<COP>(sbn, co0, yv, v4, pok, s1 + 4 * rb, s2 + 4 * rb);
      }
      bs += (double)x6_reduce16(s1, li);
      bq += (double)x6_reduce16(s2, li);
    }
    __syncthreads();   // every wave is done with sx before it is re-filled
    cur_a = !cur_a;
  }
  if (!fz) return;
  // [wave][sum, sum of products][32] in the (now free) halo buffer, then the
  // 8 waves in fixed order
  double* red = reinterpret_cast<double*>(sxa);
  if ((li & 1) == 0) {
    const int r = li >> 1;
    const int co = (r & 3) + 8 * (r >> 2) + 4 * lh;
    red[(wave * 2 + 0) * COP + co] = bs;
    red[(wave * 2 + 1) * COP + co] = bq;
  }
  __syncthreads();
  if (tid < 2 * COP) {
    const int k = tid / COP, co = tid % COP;
    double a = 0.0;
    for (int wv = 0; wv < NT / 64; ++wv) a += red[(wv * 2 + k) * COP + co];
    stats[(int64_t)blockIdx.x * 2 * COP + tid] = a;
  }
}

// Round 6: the bf16 configuration's forward convs (encoder 16 -> 32 and
// 32 -> 64, decoder 16 -> 32; models/CNNBLSTM/model.py:35-43,53-55) on the
// same LDS-DMA structure: one persistent grid as conv3x3_x6p_kernel's (same
// tiles, same tile order per workgroup, same wave -> (output row, 32-channel
// tile) map), the tile's whole CI-channel halo brought by
// global_load_lds_dwordx4 into one of two LDS buffers while the previous
// tile's MFMAs run, the weights staged once.  The input is the previous
// layer's pre-BatchNorm y (bf16 channel-last): its BatchNorm+ReLU is applied
// in LDS before the tile's barrier, each lane rewriting the 16 bytes its own
// DMA wrote (the same fmaf / max / RNE rounding as x6p's staging; zeros
// outside the image stay zero).  Same LDS images, the same chunk -> tap ->
// channel-tile MFMA order, the same epilogue (bias, bf16 rounding, channel-
// last store, fixed-order BatchNorm partials): bit-identical to x6p<CI, COP,
// NP = 1, G16, Y16, XL, YL>.  (The DMA is issued from inline asm, so hipcc
// adds no vmcnt(0) before the LDS reads; the loop's own vmcnt(0) at the top
// retires the tile's DMA and the previous epilogue's stores.)
namespace cdf {
constexpr int TR = 8, TC = 32, HR = TR + 2, HC = TC + 2;
constexpr int XROW = HC * 32;                                // 1088
constexpr int NPIX = HR * HC;                                // 340 halo pixels
constexpr int XBLK = (NPIX * 32 + 1023) / 1024;              // 11 DMA blocks per plane
constexpr int XPP = XBLK * 1024;                             // padded plane
constexpr int WROW = 9 * 32 + 16;                            // 304
}  // namespace cdf

// s_waitcnt vmcnt(n) for a run-time n (immediates 0..15; larger: 0, which
// waits for more than needed)
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
#define AINP_VMW(K) \
  case K: asm volatile("s_waitcnt vmcnt(" #K ")" ::: "memory"); break;
    AINP_VMW(1) AINP_VMW(2) AINP_VMW(3) AINP_VMW(4) AINP_VMW(5) AINP_VMW(6) AINP_VMW(7)
    AINP_VMW(8) AINP_VMW(9) AINP_VMW(10) AINP_VMW(11) AINP_VMW(12) AINP_VMW(13) AINP_VMW(14)
    AINP_VMW(15)
#undef AINP_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// NS = 2: one tile's DMA in flight beside the MFMAs, vmcnt(0) at the top of
// each tile; NS = 3: two, with the epilogue's stores issued as buffer stores
// by every lane (masked lanes write past the buffer's end, which drops them)
// so each wave's vmcnt counts are exact and the top-of-tile wait leaves the
// younger DMA and the stores in flight
template <int CI, int COP, int NT, int NS = 2, int NKREG = -1>
__global__ __launch_bounds__(NT, 1) void conv3x3_fwd_b16dma_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    uint16_t* __restrict__ y, double* __restrict__ stats, int N, int Cout, int H, int W) {
  using namespace cdf;
  constexpr int NCK = CI / 16, NI = COP / 32, NW = NT / 64, NIW = NI * TR / NW;
  static_assert(CI % 16 == 0 && (COP == 32 || COP == 64) && NIW >= 1 && NIW * NW == NI * TR,
                "shape");
  constexpr int XBUF = NCK * XPP, WPLANE = COP * WROW;
  constexpr int NBLK = NCK * XBLK;                         // DMA blocks per tile
  constexpr int QMAX = (NBLK + NW - 1) / NW;
  constexpr int QFULL = NBLK - (QMAX - 1) * NW;            // waves < QFULL issue QMAX
  constexpr int OFF_W = NS * XBUF, OFF_SS = OFF_W + NCK * WPLANE, OFF_B = OFF_SS + 2 * CI * 4;
  constexpr int LDS = OFF_B + COP * 4;
  static_assert(NS == 2 || NS == 3, "ring");
  static_assert(2 * XBUF >= TR * 2 * COP * 8, "BatchNorm row sums reuse the halo buffers");
  // one LDS object: [halo buffers 0 .. NS-1 | weights | scale, shift | bias]
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS];
  unsigned char* sw = smem + OFF_W;
  float* sss = reinterpret_cast<float*>(smem + OFF_SS);
  float* s_b = reinterpret_cast<float*>(smem + OFF_B);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int wrow = wave % TR, wco = (wave / TR) * NIW;
  const bool pro = in_scale != nullptr;

  for (int u = tid; u < NCK * COP * 18; u += NT) {
    const int half = u & 1, tap = (u >> 1) % 9, co = (u / 18) % COP, ch = u / (18 * COP);
    float pw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int ci = ch * 16 + 8 * half + c;
      pw[c] = co < Cout ? w[((int64_t)co * CI + ci) * 9 + tap] : 0.f;
    }
    cx6_stage<1>(pw, sw + ch * WPLANE + co * WROW + tap * 32 + 16 * half, WPLANE);
  }
  if (tid < 2 * CI) sss[tid] = pro ? (tid < CI ? in_scale[tid] : in_shift[tid - CI]) : 0.f;
  if (tid < COP) s_b[tid] = (bias && tid < Cout) ? bias[tid] : 0.f;
  __syncthreads();   // weights and constants, before any DMA is in flight
  // the wave's A (weight) fragments stay in VGPRs for the whole kernel
  // (NCK x 9 x NIW x 4 VGPRs): per tile only the activations are read from LDS
  // (the first NKR chunks, NKREG < 0: all; the rest read from LDS per tile.
  // 32 -> 64: 16 waves reading every weight fragment from LDS measured faster
  // than 8 waves holding half of them, r06o: 0.264 vs 0.277 ms)
  constexpr int NKR = NKREG < 0 ? NCK : NKREG;
  bf16x8c wa[NKR > 0 ? NKR : 1][9][NIW];
#pragma unroll
  for (int kc = 0; kc < NKR; ++kc)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int i = 0; i < NIW; ++i)
        wa[kc][tap][i] = cx6_ld(sw + kc * WPLANE + li * WROW + 16 * lh + (wco + i) * 32 * WROW +
                                tap * 32);

  const int tiles_c = (W + TC - 1) / TC, tiles_r = (H + TR - 1) / TR;
  // 32-bit tile arithmetic (the launcher checks N * tiles < 2^31)
  const int ntiles = N * tiles_r * tiles_c;
  auto coords = [&](int t, int& n, int& r0, int& c0) {
    const unsigned q = (unsigned)t / (unsigned)tiles_c;
    c0 = (int)((unsigned)t - q * (unsigned)tiles_c) * TC;
    n = (int)(q / (unsigned)tiles_r);
    r0 = (int)(q - (unsigned)n * (unsigned)tiles_r) * TR;
  };
  // DMA unit k of this wave: block qb = wave + NW k (plane qb / XBLK, block
  // qb % XBLK); lane L -> halo pixel 32 j + L/2, physical half L % 2 holding
  // the logical half (L % 2) ^ (column bit 3)
  auto issue = [&](int t, unsigned char* buf) {
    int n, r0, c0;
    coords(t, n, r0, c0);
#pragma unroll
    for (int k = 0; k < QMAX; ++k) {
      const int qb = wave + NW * k;
      if (qb >= NBLK) break;
      const int kc = qb / XBLK, j = qb % XBLK;
      const int lp = 32 * j + (lane >> 1);
      const uint16_t* src = cdd_zero;
      if (lp < NPIX) {
        const int row = lp / HC, col = lp % HC;
        const int gr = r0 - 1 + row, gc = c0 - 1 + col;
        const int hl = (lane & 1) ^ ((col >> 3) & 1);
        if ((unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W)
          src = x + (((int64_t)n * H + gr) * W + gc) * CI + kc * 16 + 8 * hl;
      }
      glds16_asm(src, buf + kc * XPP + j * 1024);
    }
  };
  // BatchNorm+ReLU of the lane's own DMA units, in place
  auto prologue = [&](int t, unsigned char* buf) {
    int n, r0, c0;
    coords(t, n, r0, c0);
#pragma unroll
    for (int k = 0; k < QMAX; ++k) {
      const int qb = wave + NW * k;
      if (qb >= NBLK) break;
      const int kc = qb / XBLK, j = qb % XBLK;
      const int lp = 32 * j + (lane >> 1);
      const int row = lp / HC, col = lp % HC;
      const int gr = r0 - 1 + row, gc = c0 - 1 + col;
      if (lp < NPIX && (unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W) {
        const int ci0 = kc * 16 + 8 * ((lane & 1) ^ ((col >> 3) & 1));
        uint4* p = reinterpret_cast<uint4*>(buf + kc * XPP + j * 1024 + 16 * lane);
        const uint4 v = *p;
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = ci0 + 2 * e;
          const float a = fmaxf(fmaf(__uint_as_float(w4[e] << 16), sss[c], sss[CI + c]), 0.f);
          const float b = fmaxf(fmaf(__uint_as_float(w4[e] & 0xffff0000u), sss[c + 1],
                                     sss[CI + c + 1]), 0.f);
          o[e] = cx6_cvt_pk(a, b);
        }
        *p = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  };

  f32x16 acc[NIW];
  double bs[NIW], bq[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i) bs[i] = bq[i] = 0.0;
  // this workgroup's tiles: blockIdx.x + i * gridDim.x, i < cnt
  const int cnt = (int)blockIdx.x < ntiles ? (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  constexpr int S = NIW * 4;                               // stores per tile per wave
  const int Q = wave < QFULL ? QMAX : QMAX - 1;            // DMAs per tile per wave
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      y, (short)0, (int)((int64_t)N * H * W * Cout * 2), 0x00020000);
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < cnt) issue((int)blockIdx.x + i * (int)gridDim.x, smem + i * XBUF);
  for (int it = 0; it < cnt; ++it) {
    const int t = (int)blockIdx.x + it * (int)gridDim.x;
    unsigned char* sx = smem + (it % NS) * XBUF;
    // this wave's DMAs of tile t retired; NS = 3: what was issued after them
    // (the next tile's DMA, the last two epilogues' stores) may stay in flight
    if constexpr (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      const int younger = it == 0 ? (cnt > 1 ? Q : 0)
                        : it == 1 ? S + (cnt > 2 ? Q : 0)
                                  : 2 * S + (it + 1 < cnt ? Q : 0);
      vm_wait_rt(younger);
    }
    if (pro) prologue(t, sx);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // tile t complete in LDS; the oldest buffer is free
    asm volatile("" ::: "memory");
    if (it + NS - 1 < cnt)
      issue((int)blockIdx.x + (it + NS - 1) * (int)gridDim.x, smem + ((it + NS - 1) % NS) * XBUF);
#pragma unroll
    for (int i = 0; i < NIW; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
    for (int kc = 0; kc < NCK; ++kc) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dxx = tap % 3;
        const int hcol = li + dxx;
        const bf16x8c b = cx6_ld(sx + kc * XPP + (wrow + dy) * XROW + hcol * 32 +
                                 16 * (lh ^ ((hcol >> 3) & 1)));
#pragma unroll
        for (int i = 0; i < NIW; ++i) {
          const bf16x8c a = kc < NKR ? wa[kc < NKR ? kc : 0][tap][i]
                                     : cx6_ld(sw + kc * WPLANE + li * WROW + 16 * lh +
                                              (wco + i) * 32 * WROW + tap * 32);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
        }
      }
    }
    // epilogue (conv3x3_x6p_kernel's, Y16 + YL): bias, bf16 rounding,
    // channel-last stores of 4 channels, BatchNorm sums of the stored values
    int n, r0, c0;
    coords(t, n, r0, c0);
    const int row = r0 + wrow, col = c0 + li;
    const bool pok = row < H && col < W;
    const int64_t ycl = (((int64_t)n * H + row) * W + col) * Cout;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      float s[16], q[16], vv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * (wco + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const bool ok = pok && co < Cout;
        const float v = y16_round(acc[i][r] + s_b[co]);
        vv[r] = v;
        s[r] = ok ? v : 0.f;
        q[r] = s[r] * s[r];
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int co0 = 32 * (wco + i) + 8 * rb + 4 * lh;
        if constexpr (NS == 2) {
          if (pok && co0 < Cout)
            cl_st4<true>(reinterpret_cast<float*>(y), ycl + co0, vv[4 * rb], vv[4 * rb + 1],
                         vv[4 * rb + 2], vv[4 * rb + 3]);
        } else {
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          u32x2 d;
          d[0] = cx6_cvt_pk(vv[4 * rb], vv[4 * rb + 1]);
          d[1] = cx6_cvt_pk(vv[4 * rb + 2], vv[4 * rb + 3]);
          const int vo = (pok && co0 < Cout) ? (int)((ycl + co0) * 2) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b64(d, ry, vo, 0, 0);
        }
      }
      if (stats) {
        bs[i] += (double)x6_reduce16(s, li);
        bq[i] += (double)x6_reduce16(q, li);
      }
    }
  }
  if (!stats) return;
  // per-row sums -> [row][sum, sum of squares][COP] (the halo buffers are free)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
  if ((li & 1) == 0) {
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int r = li >> 1;
      const int co = 32 * (wco + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
      red[(wrow * 2 + 0) * COP + co] = bs[i];
      red[(wrow * 2 + 1) * COP + co] = bq[i];
    }
  }
  __syncthreads();
  for (int co = tid; co < Cout; co += NT) {
    double sm = 0.0, sq = 0.0;
    for (int wv = 0; wv < TR; ++wv) {
      sm += red[(wv * 2 + 0) * COP + co];
      sq += red[(wv * 2 + 1) * COP + co];
    }
    stats[(int64_t)blockIdx.x * 2 * Cout + co] = sm;
    stats[(int64_t)blockIdx.x * 2 * Cout + Cout + co] = sq;
  }
}

// AINP_CONV16_DMA=0: the register-staged x6p forwards (A/B)
static bool conv16_dma() {
  static const bool v = [] {
    const char* e = getenv("AINP_CONV16_DMA");
    return !(e && e[0] == '0');
  }();
  return v;
}

// AINP_DGRAD16_DMA=0: the register-staged kernel for that data gradient (A/B)
static bool dgrad16_dma() {
  static const bool v = [] {
    const char* e = getenv("AINP_DGRAD16_DMA");
    return !(e && e[0] == '0');
  }();
  return v;
}

// RPW output rows per wave: 2 (16-row tiles, one workgroup per CU) or 1
// (8-row tiles: half the halo LDS, two workgroups per CU).
template <int CI, int COP, bool DGRAD, int RPW, int NP, bool G16 = false, bool XL = false,
          bool YL = false>
__global__ __launch_bounds__(cx6::NT, RPW == 1 ? 4 : 2) void conv3x3_x6_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, int Cout, int H, int W, Bnr bnr) {
  using cx6::HC;
  using cx6::TC;
  using cx6::CK;
  using cx6::XROW;
  using cx6::WROW;
  using cx6::NT;
  constexpr int TR = 8 * RPW, HR = TR + 2, XPLANE = HR * XROW;
  constexpr int XU = 2 * HR * HC, XI = (XU + NT - 1) / NT;
  static_assert(CI % CK == 0 && (COP == 32 || COP == 64), "shape");
  constexpr int NI = COP / 32;
  constexpr int WPLANE = COP * WROW;
  constexpr int WU = COP * 18;                // weight staging units (co, tap, half)
  constexpr int WI = (WU + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) unsigned char sx[NP * XPLANE];
  __shared__ __attribute__((aligned(16))) unsigned char sw[NP * WPLANE];
  __shared__ double red[8 * 2 * COP];          // BatchNorm partials per wave
  // fused BatchNorm-backward reduce (Bnr, the 8-row channel-last data
  // gradient): the layer's constants in LDS, this lane's y loaded up front
  constexpr bool FZ = DGRAD && YL && RPW == 1 && COP == 32;
  __shared__ float sbn[FZ ? 4 * COP : 1];

  const int n = blockIdx.z, r0 = blockIdx.y * TR, c0 = blockIdx.x * TC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t HW = (int64_t)H * W;
  constexpr int ES = act_es<G16>();
  const bool fused = FZ && bnr.y != nullptr;
  uint4 yr[FZ ? NI : 1][4];
  if constexpr (FZ) {
    if (fused) {
      bnr_stage(bnr, sbn, Cout, COP, tid, NT);
      const int row = r0 + wave, col = c0 + li;
      const bool pok = row < H && col < W;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int co0 = 32 * i + 8 * rb + 4 * lh;
          yr[i][rb] = bnr_ld4(bnr, (pok && co0 < Cout)
                                       ? ((int64_t)n * HW + (int64_t)row * W + col) * Cout + co0
                                       : 0);
        }
    }
  }

  float px[XI][8];
  // staging unit -> (halo column, halo row, channel half); channel-last (XL):
  // the two lanes of a pixel read its chunk's channels as contiguous bytes
  auto unit = [&](int u, int& col, int& row, int& half) {
    if constexpr (XL) {
      half = u & 1;
      const int hp = u >> 1;
      col = hp % HC;
      row = hp / HC;
    } else {
      col = u % HC;
      row = (u / HC) % HR;
      half = u / (HR * HC);
    }
  };
  // clamped-address buffer loads (selected to zero at commit); valid while a
  // sample's CI planes span < 2^31 bytes (the launcher checks)
  auto fetch = [&](int ci0) {
    if constexpr (XL) {
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, (int64_t)n * HW * CI + ci0);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        int col, row, half;
        unit(u < XU ? u : XU - 1, col, row, half);
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        cl_ld8<G16>(rx, ((gr * W + gc) * CI + 8 * half) * ES, px[i]);
      }
    } else {
      int plane = (int)(HW * ES);
      asm volatile("" : "+s"(plane));
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, ((int64_t)n * CI + ci0) * HW);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        const int col = u % HC, row = (u / HC) % HR, half = u < XU ? u / (HR * HC) : 1;
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        const int vo = 8 * half * plane + (gr * W + gc) * ES;
#pragma unroll
        for (int c = 0; c < 8; ++c) px[i][c] = act_ld<G16>(rx, vo, c * plane);
      }
    }
  };
  auto commit = [&](int ci0) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int u = tid + NT * i;
      if (u < XU) {
        int col, row, half;
        unit(u, col, row, half);
        const int gr = r0 - 1 + row, gc = c0 - 1 + col;
        const bool inb = gr >= 0 && gr < H && gc >= 0 && gc < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = px[i][c];
          if (in_scale) {
            const int ci = ci0 + 8 * half + c;
            t = fmaxf(fmaf(t, in_scale[ci], in_shift[ci]), 0.f);
          }
          v[c] = inb ? t : 0.f;
        }
        cx6_stage<NP>(v, sx + row * XROW + col * 32 + 16 * (half ^ ((col >> 3) & 1)), XPLANE);
      }
    }
    // weights: L2-resident gathers loaded here rather than prefetched (the
    // registers are needed by the halo prefetch and the accumulators)
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int u = tid + NT * i;
      if (u < WU) {
        const int half = u & 1, tap = (u >> 1) % 9, co = u / 18;
        float pw[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int ci = ci0 + 8 * half + c;
          pw[c] = co < Cout ? (DGRAD ? w[((int64_t)ci * Cout + co) * 9 + (8 - tap)]
                                     : w[((int64_t)co * CI + ci) * 9 + tap])
                            : 0.f;
        }
        cx6_stage<NP>(pw, sw + co * WROW + tap * 32 + 16 * half, WPLANE);
      }
    }
  };

  f32x16 acc[NI][RPW];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < RPW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int NCH = CI / CK;
  fetch(0);
#pragma unroll 1
  for (int ch = 0; ch < NCH; ++ch) {
    if (ch > 0) __syncthreads();  // previous chunk's fragment reads are done
    commit(ch * CK);
    __syncthreads();
    if (ch + 1 < NCH) fetch((ch + 1) * CK);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
      bf16x8c a[NP][NI], b[NP][RPW];
      const int hcol = li + dx;
      const unsigned char* xb = sx + (RPW * wave + dy) * XROW + hcol * 32 + 16 * (lh ^ ((hcol >> 3) & 1));
      const unsigned char* wb = sw + li * WROW + tap * 32 + 16 * lh;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < NI; ++i) a[p][i] = cx6_ld(wb + p * WPLANE + i * 32 * WROW);
#pragma unroll
        for (int j = 0; j < RPW; ++j) b[p][j] = cx6_ld(xb + p * XPLANE + j * XROW);
      }
      // term-major over the NI x 2 accumulators: no back-to-back dependent MFMAs
#pragma unroll
      for (int t = 0; t < cx6_terms(NP); ++t) {
        const int pa = cx6_pa(NP, t), pb = cx6_pb(NP, t);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < RPW; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa][i], b[pb][j], acc[i][j], 0,
                                                                0, 0);
      }
    }
  }

  // epilogue: D[co = 32i + (r&3) + 8(r>>2) + 4lh][pixel col li] of row 2*wave + j;
  // BatchNorm partials reduced over the 32 lanes of each half (one channel
  // set), then over the 8 waves in fixed order
  float* yn = y + (int64_t)n * Cout * HW;
  const int col = c0 + li;
  if constexpr (YL) {   // channel-last: 4 consecutive channels per store (Cout % 4 == 0)
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int row = r0 + RPW * wave + j;
        if (row < H && col < W) {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            const int co0 = 32 * i + 8 * rb + 4 * lh;
            if (co0 < Cout) {
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * rb + e] + (bias ? bias[co0 + e] : 0.f);
              cl_st4<false>(yn, ((int64_t)row * W + col) * Cout + co0, v[0], v[1], v[2], v[3]);
            }
          }
        }
      }
  }
  if constexpr (FZ) {
    // fused BatchNorm-backward reduce (Bnr): (gz, gz * xhat) per channel,
    // summed over the wave's 32 pixels by a float butterfly
    if (fused) {
      const int row = r0 + wave;
      const bool pok = row < H && col < W;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float s1[16], s2[16];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int co0 = 32 * i + 8 * rb + 4 * lh;
          const float v4[4] = {acc[i][0][4 * rb], acc[i][0][4 * rb + 1], acc[i][0][4 * rb + 2],
                               acc[i][0][4 * rb + 3]};
          float yv[4];
          bnr_dec4(bnr.y16, yr[FZ ? i : 0][rb], yv);
          bnr_terms4<COP>(sbn, co0, yv, v4, pok && co0 < Cout, s1 + 4 * rb, s2 + 4 * rb);
        }
        const float t1 = x6_reduce16(s1, li), t2 = x6_reduce16(s2, li);
        const int r = li >> 1, co = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if ((li & 1) == 0 && co < Cout) {
          red[(wave * 2 + 0) * COP + co] = t1;
          red[(wave * 2 + 1) * COP + co] = t2;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI && !fused; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const bool cok = co < Cout;
      const float bv = (bias && cok) ? bias[co] : 0.f;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int row = r0 + RPW * wave + j;
        if (cok && row < H && col < W) {
          const float v = acc[i][j][r] + bv;
          if constexpr (!YL) yn[(int64_t)co * HW + (int64_t)row * W + col] = v;
          s += v;
          q += v * v;
        }
      }
      if (stats) {
        double ds = s, dq = q;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          ds += __shfl_xor(ds, o, 64);
          dq += __shfl_xor(dq, o, 64);
        }
        if (li == 0) {
          red[(wave * 2 + 0) * COP + co] = ds;
          red[(wave * 2 + 1) * COP + co] = dq;
        }
      }
    }
  if (!stats) return;
  __syncthreads();
  const int64_t part = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (int co = tid; co < Cout; co += NT) {
    double s = 0.0, q = 0.0;
    for (int wv = 0; wv < 8; ++wv) {
      s += red[(wv * 2 + 0) * COP + co];
      q += red[(wv * 2 + 1) * COP + co];
    }
    stats[part * 2 * Cout + co] = s;
    stats[part * 2 * Cout + Cout + co] = q;
  }
}

// Upper bound on the BatchNorm partials an x6 launch writes for [N, H, W]
// outputs: one per workgroup of the persistent kernel (<= 512), one per tile
// of the tiled kernel.
int64_t conv_x6_stat_parts(int64_t N, int64_t H, int64_t W) {
  const int64_t tiled = N * cdiv(H, cx6::TR) * cdiv(W, cx6::TC);
  return tiled > 512 ? tiled : 512;
}

int conv_x6p_launch(bool dgrad, const float* x, const float* w, const float* bias,
                    const float* sc, const float* sh, float* y, double* stats, int64_t N, int Cin,
                    int Cout, int64_t H, int64_t W, hipStream_t s, int64_t* parts, bool b16,
                    bool x16, bool y16, int lay, const Bnr& bnr);

// Persistent-grid multiplier of the bf16 (NP = 1) kernels: their LDS (21-50
// KB) and VGPR (48-80) footprints let 2-4x the fp32 kernels' workgroups stay
// resident, and they are bound by the loads a CU keeps in flight (SQ passes:
// MFMA busy 0.05-0.10, waves parked on s_waitcnt 0.5-0.67 of their cycles,
// profiles/r04e_*).  AINP_X6_OCC16 overrides (1 .. X6_OCC_MAX).
int conv_x6_occ16() {
  static const int v = [] {
    const char* e = getenv("AINP_X6_OCC16");
    const int o = e ? atoi(e) : 1;
    return o < 1 ? 1 : (o > X6_OCC_MAX ? X6_OCC_MAX : o);
  }();
  return v;
}

// Launch if (Cin, Cout) has an x6 instantiation; returns 1 if not handled.
// *parts = the number of BatchNorm partials written.  The persistent kernel
// serves every pair it has (32-bit buffer offsets permitting); the tiled one
// is kept for AINP_CONV_X6_TILED=1.
// BatchNorm partial rows the x6 launch below writes for this shape (0: no x6
// kernel serves it); mirrors conv_x6_launch / conv_x6p_launch.
int64_t conv_x6_stat_rows(bool dgrad, int Cin, int Cout, int64_t N, int64_t H, int64_t W,
                          bool b16) {
  const int occ = b16 ? conv_x6_occ16() : 1;
  if (Cout > 64 || Cout < 16) return 0;
  const int cop = Cout <= 32 ? 32 : 64;
  static const bool tiled_env = getenv("AINP_CONV_X6_TILED") != nullptr;
  if (!tiled_env && (int64_t)(Cin > Cout ? Cin : Cout) * H * W * 4 < ((int64_t)1 << 31)) {
    // one row per persistent workgroup (bf16: the multiplied grid)
    if (!dgrad && Cin == 32 && cop == 64) return 256 * occ;
    if (Cin == 16 && cop == 32) return 512 * occ;
    if (Cin == 32 && Cout == 16) return 512 * occ;
  }
  if (((Cin == 32 && cop == 64) || (Cin == 64 && cop == 32)) &&
      (int64_t)Cin * H * W * 4 < ((int64_t)1 << 31))    // 32-bit buffer offsets
    return N * cdiv(H, cx6::TR) * cdiv(W, cx6::TC);
  return 0;
}

// 1 if conv_x6_launch(dgrad = true, stats = nullptr, b16, x16) takes bf16 dy
// for this (dy channels, dx channels) pair; mirrors its routing.
bool conv_x6_dgrad16_ok(int Cin, int Cout, int64_t H, int64_t W) {
  const int cop = Cout <= 32 ? 32 : 64;
  static const bool tiled_env = getenv("AINP_CONV_X6_TILED") != nullptr;
  if (Cout > 64 || Cout < 16) return false;
  if (!tiled_env && (int64_t)(Cin > Cout ? Cin : Cout) * H * W * 4 < ((int64_t)1 << 31) &&
      ((Cin == 16 && cop == 32) || (Cin == 32 && Cout == 16)))
    return true;   // persistent x6p / x6q
  return ((Cin == 32 && cop == 64) || (Cin == 64 && cop == 32)) &&
         (int64_t)Cin * H * W * 4 < ((int64_t)1 << 31);   // tiled, 8-row tiles
}

// 1 if conv_x6_launch(dgrad = true, lay with CL_CF) serves this (dy channels,
// dx channels) pair: the persistent 32 -> 16 data gradient (x6q)
bool conv_x6_dgrad_cfnt_ok(int Cin, int Cout, int64_t N, int64_t H, int64_t W) {
  static const bool tiled_env = getenv("AINP_CONV_X6_TILED") != nullptr;
  return !tiled_env && Cin == 32 && Cout == 16 && N * H * W * 16 < ((int64_t)1 << 40) &&
         (int64_t)Cin * H * W * 4 < ((int64_t)1 << 31);
}

// 1 if conv_x6_launch(dgrad = false, b16) serves this pair on a persistent
// kernel, the only forwards with bf16-storage input / output (x16 / y16)
bool conv_x6_fwd16_ok(int Cin, int Cout, int64_t H, int64_t W) {
  const int cop = Cout <= 32 ? 32 : 64;
  static const bool tiled_env = getenv("AINP_CONV_X6_TILED") != nullptr;
  if (Cout > 64 || Cout < 16 || tiled_env ||
      (int64_t)(Cin > Cout ? Cin : Cout) * H * W * 4 >= ((int64_t)1 << 31))
    return false;
  return (Cin == 32 && cop == 64) || (Cin == 16 && cop == 32) || (Cin == 32 && Cout == 16);
}

// Instantiate f for the run-time layout bits: f(xl, yl) with integral-constant
// booleans (input / output channel-last)
template <typename F>
static void cl_dispatch(int lay, F&& f) {
  if ((lay & CL_X) && (lay & CL_Y)) f(std::true_type{}, std::true_type{});
  else if (lay & CL_X) f(std::true_type{}, std::false_type{});
  else if (lay & CL_Y) f(std::false_type{}, std::true_type{});
  else f(std::false_type{}, std::false_type{});
}

int conv_x6_launch(bool dgrad, const float* x, const float* w, const float* bias,
                   const float* sc, const float* sh, float* y, double* stats, int64_t N, int Cin,
                   int Cout, int64_t H, int64_t W, hipStream_t s, int64_t* parts, bool b16,
                   bool x16, bool y16, int lay, const Bnr* bnrp) {
  const Bnr bnr = bnrp ? *bnrp : Bnr{};
  // fused BatchNorm-backward reduce: a data gradient writing channel-last dx,
  // whose partials are the (sum gz, sum gz * xhat) rows
  const bool fused = bnr.y != nullptr;
  // (dx of at most 32 channels: the fused instances)
  if (fused && !(dgrad && stats && (lay & CL_Y) && !bias && Cout <= 32)) return 2;
  if (conv_x6_stat_rows(dgrad, Cin, Cout, N, H, W, b16) == 0) return (lay & CL_CF) ? 2 : 1;
  static const bool tiled_env = getenv("AINP_CONV_X6_TILED") != nullptr;
  if (!tiled_env && (int64_t)(Cin > Cout ? Cin : Cout) * H * W * 4 < ((int64_t)1 << 31)) {
    const int rc = conv_x6p_launch(dgrad, x, w, bias, sc, sh, y, stats, N, Cin, Cout, H, W, s,
                                   parts, b16, x16, y16, lay, bnr);
    if (rc != 1) return rc;
  }
  if (lay & CL_CF) return 2;   // only the persistent x6q writes [C][H][N][W]
  if ((int64_t)Cin * H * W * 4 >= ((int64_t)1 << 31)) return 1;   // 32-bit buffer offsets
  // the data gradient without forward statistics: 8-row tiles (channel-last,
  // bf16 dy, the fused reduce)
  const bool dg8 = dgrad && (!stats || fused);
  if (y16 || (x16 && !(dg8 && b16))) return 2;   // bf16 storage: no such kernel
  if (lay && !dg8) return 2;
  if (dg8 && b16 && x16 && lay == (CL_X | CL_Y) && Cin == cdd::CI && Cout == cdd::COP && !bias &&
      !sc && (!fused || bnr.y16) && dgrad16_dma()) {
    const int ntr = (int)cdiv(H, cdd::TR), ntc = (int)cdiv(W, cdd::TC);
    const int64_t nt = N * (int64_t)ntr * ntc;
    const int grid = (int)(nt < 256 ? nt : 256);   // one persistent workgroup per CU
    *parts = grid;
    // AINP_DGRAD16_WREG=0: weight fragments re-read from LDS per tile (A/B)
    static const bool wreg = [] {
      const char* e = getenv("AINP_DGRAD16_WREG");
      return !(e && e[0] == '0');
    }();
    if (wreg)
      hipLaunchKernelGGL(conv3x3_dgrad_b16dma_kernel<true>, dim3(grid), dim3(cdd::NT), 0, s,
                         reinterpret_cast<const uint16_t*>(x), w, y, stats, bnr, (int)N, (int)H,
                         (int)W, ntr, ntc, nt);
    else
      hipLaunchKernelGGL(conv3x3_dgrad_b16dma_kernel<false>, dim3(grid), dim3(cdd::NT), 0, s,
                         reinterpret_cast<const uint16_t*>(x), w, y, stats, bnr, (int)N, (int)H,
                         (int)W, ntr, ntc, nt);
    return check_launch("conv3x3_dgrad_b16dma");
  }
  *parts = dg8 ? N * cdiv(H, 8) * cdiv(W, cx6::TC) : N * cdiv(H, cx6::TR) * cdiv(W, cx6::TC);
  const dim3 grid((unsigned)cdiv(W, cx6::TC), (unsigned)cdiv(H, cx6::TR), (unsigned)N);
  const int cop = Cout <= 32 ? 32 : 64;
#define AINP_X6N(CIV, COV, NPV)                                                                \
  if (Cin == CIV && cop == COV) {                                                               \
    if (dg8) {   /* 8-row tiles, two workgroups per CU */                                       \
      const dim3 g8((unsigned)cdiv(W, cx6::TC), (unsigned)cdiv(H, 8), (unsigned)N);             \
      cl_dispatch(lay, [&](auto xl, auto yl) {                                                  \
        constexpr bool XL = decltype(xl)::value, YL = decltype(yl)::value;                      \
        if (NPV == 1 && x16)                                                                    \
          hipLaunchKernelGGL((conv3x3_x6_kernel<CIV, COV, true, 1, NPV, true, XL, YL>), g8,     \
                             dim3(cx6::NT), 0, s, x, w, bias, sc, sh, y, stats, Cout, (int)H,   \
                             (int)W, bnr);                                                      \
        else                                                                                    \
          hipLaunchKernelGGL((conv3x3_x6_kernel<CIV, COV, true, 1, NPV, false, XL, YL>), g8,    \
                             dim3(cx6::NT), 0, s, x, w, bias, sc, sh, y, stats, Cout, (int)H,   \
                             (int)W, bnr);                                                      \
      });                                                                                       \
    } else if (dgrad)                                                                           \
      hipLaunchKernelGGL((conv3x3_x6_kernel<CIV, COV, true, 2, NPV>), grid, dim3(cx6::NT), 0, s, \
                         x, w, bias, sc, sh, y, stats, Cout, (int)H, (int)W, bnr);              \
    else                                                                                        \
      hipLaunchKernelGGL((conv3x3_x6_kernel<CIV, COV, false, 2, NPV>), grid, dim3(cx6::NT), 0,  \
                         s, x, w, bias, sc, sh, y, stats, Cout, (int)H, (int)W, bnr);           \
    return check_launch("conv3x3_x6");                                                          \
  }
#define AINP_X6(CIV, COV)                                                                     \
  if (b16) {                                                                                  \
    AINP_X6N(CIV, COV, 1)                                                                     \
  } else {                                                                                    \
    AINP_X6N(CIV, COV, 3)                                                                     \
  }
  // Only the pairs where this kernel beats the exact f32 kernels on the model's
  // shapes (r01_v9 op timings): the encoder's 32->64 conv (1.17 vs 1.21 ms) and
  // its 64->32 data gradient (0.83 vs 0.98 ms).  With 16 input channels (one K
  // chunk) or a padded 16-channel output, the single resident workgroup per CU
  // leaves the staging latency exposed and the exact kernels are faster.
  AINP_X6(32, 64) AINP_X6(64, 32)
#undef AINP_X6
#undef AINP_X6N
  return 1;
}

// ------------------------------------------------------------------ wgrad
// Weight gradient D[co][(tap, ci)] = sum_pixel dy[co][pixel] * act(x)[ci][pixel + tap]
// of a 32-input-channel pass, on the same split-bf16 arithmetic:
//  * persistent workgroups walk strided sets of 4 x 24-pixel tiles (the
//    reduction dimension, 6 k-steps of 16 pixels = two 8-pixel row segments)
//    and write one fp32 partial slab each, in the slab format of conv.hip's
//    wgrad kernels, summed there by wgrad_reduce1/wgrad_reduce in fixed order;
//  * both operands are staged channel-last, three bf16 planes each, so every
//    global load is coalesced along pixels and every fragment is two
//    ds_read_b64_tr_b16 transposing reads (4 consecutive pixels x 16
//    channels), conflict-free and 8-byte aligned for every tap shift:
//      act(x): 6 x 26 halo, [pixel][32 ci], halo rows 32 pixels apart, the
//              16-byte channel groups XOR-swizzled by pixel bits 1-2;
//      dy:     [96 pixels][64 co], 16-byte groups swizzled by pixel bits 0-2;
//  * wave = (co tile, tap row): the three taps of a row share the A fragments
//    and interleave their accumulators;
//  * the next tile's x and dy are prefetched into registers during the MFMAs;
//  * dbias[co] = sum of dy, per staging unit in fp32, reduced in fixed order.
namespace wx6 {
constexpr int FT = 4, TT = 24, NPX = FT * TT;  // tile: 96 pixels, 6 k-steps
constexpr int HR = FT + 2, HC = TT + 2;        // halo 6 x 26
constexpr int HS = 32;                         // halo row stride (pixels, == 0 mod 8)
constexpr int XPL = ((HR - 1) * HS + HC) * 64; // one plane: [pixel][32 ci] bf16
constexpr int XU = HR * HC * 4;                // x staging units (pixel, 8-ci group)
}  // namespace wx6

typedef short v4s16 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ v4s16 wx6_tr(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s16*)(p));
}
__device__ __forceinline__ bf16x8c wx6_cat(v4s16 lo, v4s16 hi) {
  return __builtin_shufflevector(__builtin_bit_cast(bf16x4c, lo), __builtin_bit_cast(bf16x4c, hi),
                                 0, 1, 2, 3, 4, 5, 6, 7);
}
// dy image: 16-byte group swizzle of a pixel (bijective on pixel bits 0-2;
// pixels 2 apart use opposite 64-byte halves of their rows)
__device__ __forceinline__ int wx6_gswz(int px) {
  return (((px >> 1) & 1) << 2) | (((px >> 2) & 1) << 1) | (px & 1);
}

// XL / GL (round 5): act(x)'s source / dy channel-last ([N][H][W][C]): a unit
// (pixel, 8-channel group) is one or two vector loads, consecutive lanes on
// consecutive groups of a pixel.
template <int CO, int NP, bool G16 = false, bool XG16 = false, bool XL = false, bool GL = false>
__global__ __launch_bounds__(CO / 32 * 3 * 64, 3) void conv3x3_wgrad_x6(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int N, int Cin, int H, int W, int ci0) {
  using namespace wx6;
  constexpr int CP = 32, J = 9 * CP, NI = CO / 32;
  constexpr int NT = NI * 3 * 64;
  constexpr int XI = (XU + NT - 1) / NT;
  constexpr int NG = CO / 8;                   // dy 16-byte groups per pixel
  constexpr int GU = NPX * NG, GI = (GU + NT - 1) / NT;
  constexpr int GPX = CO * 2;                  // dy image bytes per pixel
  constexpr int GPL = NPX * GPX;
  static_assert(CO == 64 && NT % NPX == 0, "dy staging map: units of one thread share a pixel");
  // sx doubles as the bias reduction buffer [CO][NPX] floats after the loop
  constexpr int SXB = NP * XPL > CO * NPX * 4 ? NP * XPL : CO * NPX * 4;
  __shared__ __attribute__((aligned(16))) unsigned char sx[SXB];
  __shared__ __attribute__((aligned(16))) unsigned char sg[NP * GPL];
  __shared__ __attribute__((aligned(16))) float s_ss[2 * CP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int ct = wave % NI, dyt = wave / NI;  // co tile, tap row
  // transposing reads: lane 4q+p of 16-lane group g supplies pixel q (+4 for
  // the second read) of its 8-pixel segment at channels 16*(g&1) + 4p .. +3
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  int bx[3][2];  // x: halo pixel dyt*HS + dx + q + 4s (segment origin added per k-step)
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const int hp = dyt * HS + dx + q + 4 * sh;
      bx[dx][sh] = hp * 64 + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((hp >> 1) & 3)) + 8 * (pp & 1);
    }
  int ba[2];     // dy: pixel 8*lh + q + 4s of the k-step, channels of co tile ct
#pragma unroll
  for (int sh = 0; sh < 2; ++sh) {
    const int px = 8 * lh + q + 4 * sh;
    ba[sh] = px * GPX + 16 * ((4 * ct + 2 * (g & 1) + (pp >> 1)) ^ wx6_gswz(px)) + 8 * (pp & 1);
  }

  if (tid < 2 * CP)
    s_ss[tid] = in_scale ? (tid < CP ? in_scale[ci0 + tid] : in_shift[ci0 + tid - CP]) : 0.f;

  f32x16 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum[GI][8];
#pragma unroll
  for (int i = 0; i < GI; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) bsum[i][c] = 0.f;

  const int tiles_t = (W + TT - 1) / TT, tiles_f = (H + FT - 1) / FT;
  const int64_t ntiles = (int64_t)N * tiles_f * tiles_t;
  const int64_t HW = (int64_t)H * W;
  auto tile_coords = [&](int64_t tile, int& n, int& f0, int& t0) {
    t0 = (int)(tile % tiles_t) * TT;
    f0 = (int)((tile / tiles_t) % tiles_f) * FT;
    n = (int)(tile / ((int64_t)tiles_t * tiles_f));
  };
  // dy unit i of this thread: staging pixel and 8-channel group (NCHW: one
  // pixel for all of a thread's units; channel-last: consecutive groups)
  auto gunit = [&](int i, int& px_, int& grp_) {
    const int gu = tid + NT * i;
    if constexpr (GL) {
      px_ = gu / NG;
      grp_ = gu % NG;
    } else {
      px_ = tid % NPX;
      grp_ = gu / NPX;
    }
  };
  // x unit -> (halo pixel, 8-channel group)
  auto xunit = [&](int u, int& hp_, int& grp_) {
    if constexpr (XL) {
      hp_ = u >> 2;
      grp_ = u & 3;
    } else {
      hp_ = u % (HR * HC);
      grp_ = u / (HR * HC);
    }
  };

  float px[XI][8], pg[GI][8];
  auto fetch = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    // act(x) input: fp32 or bf16 storage (XG16)
    constexpr int XES = act_es<XG16>();
    if constexpr (XL) {
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<XG16>(x, (int64_t)n * HW * Cin + ci0);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        int hp, grp;
        xunit(u < XU ? u : XU - 1, hp, grp);
        const int gr = wx6_clamp(f0 - 1 + hp / HC, 0, H - 1);
        const int gc = wx6_clamp(t0 - 1 + hp % HC, 0, W - 1);
        cl_ld8<XG16>(rx, ((gr * W + gc) * Cin + 8 * grp) * XES, px[i]);
      }
    } else {
      int plane = (int)(HW * XES);
      asm volatile("" : "+s"(plane));  // keep c * plane out of the tile loop
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<XG16>(x, ((int64_t)n * Cin + ci0) * HW);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        const int hp = u % (HR * HC), grp = u < XU ? u / (HR * HC) : 3;
        const int gr = wx6_clamp(f0 - 1 + hp / HC, 0, H - 1);
        const int gc = wx6_clamp(t0 - 1 + hp % HC, 0, W - 1);
        const int vo = 8 * grp * plane + (gr * W + gc) * XES;
#pragma unroll
        for (int c = 0; c < 8; ++c) px[i][c] = act_ld<XG16>(rx, vo, c * plane);
      }
    }
    // dy: fp32 or bf16 storage (G16)
    constexpr int GES = act_es<G16>();
    if constexpr (GL) {
      const __amdgpu_buffer_rsrc_t rg = act_rsrc<G16>(dy, (int64_t)n * HW * CO);
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        int gp, grp;
        gunit(i, gp, grp);
        const int gr = wx6_clamp(f0 + gp / TT, 0, H - 1), gc = wx6_clamp(t0 + gp % TT, 0, W - 1);
        cl_ld8<G16>(rg, ((gr * W + gc) * CO + 8 * grp) * GES, pg[i]);
      }
    } else {
      int gplane = (int)(HW * GES);
      asm volatile("" : "+s"(gplane));
      const __amdgpu_buffer_rsrc_t rg = act_rsrc<G16>(dy, (int64_t)n * CO * HW);
      const int gpx = tid % NPX;
      const int gr = wx6_clamp(f0 + gpx / TT, 0, H - 1), gc = wx6_clamp(t0 + gpx % TT, 0, W - 1);
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        const int grp = (tid + NT * i) / NPX;
        const int vo = 8 * grp * gplane + (gr * W + gc) * GES;
#pragma unroll
        for (int c = 0; c < 8; ++c) pg[i][c] = act_ld<G16>(rg, vo, c * gplane);
      }
    }
  };
  auto commit = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int u = tid + NT * i;
      if (u < XU) {
        int hp, grp;
        xunit(u, hp, grp);
        const int hr = hp / HC, hc = hp % HC;
        const int gr = f0 - 1 + hr, gc = t0 - 1 + hc;
        const bool inb = gr >= 0 && gr < H && gc >= 0 && gc < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = px[i][c];
          if (in_scale) t = fmaxf(fmaf(t, s_ss[8 * grp + c], s_ss[CP + 8 * grp + c]), 0.f);
          v[c] = inb ? t : 0.f;
        }
        const int sp = hr * HS + hc;
        cx6_stage<NP>(v, sx + sp * 64 + 16 * (grp ^ ((sp >> 1) & 3)), XPL);
      }
    }
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      int gpx, grp;
      gunit(i, gpx, grp);
      const bool pok = f0 + gpx / TT < H && t0 + gpx % TT < W;
      float v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        v[c] = pok ? pg[i][c] : 0.f;
        bsum[i][c] += v[c];
      }
      cx6_stage<NP>(v, sg + gpx * GPX + 16 * (grp ^ wx6_gswz(gpx)), GPL);
    }
  };

  __syncthreads();  // s_ss
  int64_t tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    commit(tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
#pragma unroll
    for (int ks = 0; ks < NPX / 16; ++ks) {
      // this lane's 8-pixel segment: G = 2ks + lh -> tile row G/3, column 8(G%3)
      const int G0 = 2 * ks, G1 = 2 * ks + 1;
      const int seg = lh ? (G1 / 3) * HS + (G1 % 3) * 8 : (G0 / 3) * HS + (G0 % 3) * 8;
      bf16x8c a[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p)
        a[p] = wx6_cat(wx6_tr(sg + p * GPL + ba[0] + ks * 16 * GPX),
                       wx6_tr(sg + p * GPL + ba[1] + ks * 16 * GPX));
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int o0 = bx[dx][0] + seg * 64, o1 = bx[dx][1] + seg * 64;
        bf16x8c b[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          b[p] = wx6_cat(wx6_tr(sx + p * XPL + o0), wx6_tr(sx + p * XPL + o1));
        // six cross terms smallest first (NP = 3), or the bf16 product
        f32x16 c = acc[dx];
#pragma unroll
        for (int t = 0; t < cx6_terms(NP); ++t)
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cx6_pa(NP, t)], b[cx6_pb(NP, t)], c, 0,
                                                      0, 0);
        acc[dx] = c;
      }
    }
    __syncthreads();
  }

  // slab [CO][J + 1]: D[co = 32ct + (r&3) + 8(r>>2) + 4lh][ci = li] of tap 3dyt+dx
  float* slab = partial + (int64_t)blockIdx.x * CO * (J + 1);
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      slab[co * (J + 1) + (3 * dyt + dx) * CP + li] = acc[dx][r];
    }
  // bias: [co][staging pixel] partials (free LDS after the loop's last barrier)
  float* red = reinterpret_cast<float*>(sx);
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    int gpx, grp;
    gunit(i, gpx, grp);
#pragma unroll
    for (int c = 0; c < 8; ++c) red[(8 * grp + c) * NPX + gpx] = bsum[i][c];
  }
  __syncthreads();
  if (tid < CO) {
    float sum = 0.f;
    for (int k = 0; k < NPX; ++k) sum += red[tid * NPX + k];
    slab[tid * (J + 1) + J] = sum;
  }
}

// Round 6: the bf16 configuration's 32 -> 64 weight gradient fed by LDS-DMA
// (models/CNNBLSTM/model.py:40-42 backward).  conv3x3_wgrad_x6<64, NP = 1>
// stages each 96-pixel tile through registers behind two barriers and runs
// only 18 MFMAs per wave per tile (SQ: MFMA busy 0.06, waits 0.7).  Here both
// bf16 channel-last operands go global -> LDS by global_load_lds_dwordx4
// into a 3-stage ring (one tile in flight across each barrier, counted
// vmcnt, raw s_barrier), in the register kernel's LDS images (same swizzles,
// same transposing fragment reads), on 192-pixel tiles (8 x 24) walked
// down the frequency axis so consecutive tiles share two halo rows in L2:
//  * the BatchNorm+ReLU prologue act(x) = relu(x*scale+shift) (zero outside
//    the image) is applied once per tile in place, an LDS pass between the
//    two barriers of the tile -- the same fp32 fmaf/max and RNE rounding as
//    the register kernel's staging, so the staged operands are identical;
//  * the 18 output tiles (2 co tiles x 9 taps) plus the bias: 8 waves = 4
//    groups of 5 accumulator tiles (co tile x taps 0-4 / taps 5-8 + bias)
//    x 2 k-halves of the tile, 2 waves per SIMD, one A (dy) fragment per
//    k-step shared by a wave's 5 MFMAs;
//  * db[co] = sum dy on the MFMA: A times a ones B fragment (fp32
//    accumulation of the bf16 dy);
//  * epilogue: the k-halves combined through LDS, one slab per workgroup in
//    conv.hip's [CO][9*32 + 1] slab format (wgrad_reduce1 / wgrad_reduce).
// The per-pixel work is HBM-bound (2*9*32*64 FLOP per 192 B of bf16 x + dy).
namespace wdm {
constexpr int TT = 24;                             // tile columns (3 row segments of 8)
constexpr int HS = 32;                             // halo row stride (pixels)
constexpr int NT = 512;                            // 8 waves
constexpr int NW = NT / 64;
constexpr int CP = 32, CO = 64, J = 9 * CP;
constexpr int NA = 5;                              // accumulator tiles per wave
// tile geometry / ring depth per variant (FT tile rows, NS ring stages)
template <int FT, int NS>
struct Geo {
  static constexpr int NPX = FT * TT;                      // pixels per tile (k)
  static constexpr int HR = FT + 2, HC = TT + 2;           // halo
  static constexpr int XPIX = (HR - 1) * HS + HC;          // halo pixel slots
  static constexpr int XBLK = (XPIX * 64 + 1023) / 1024;   // DMA blocks (16 pixels each)
  static constexpr int GBLK = NPX * 128 / 1024;            // DMA blocks (8 pixels each)
  static constexpr int XB = XBLK * 1024;
  static constexpr int STAGE = XB + GBLK * 1024;
  static constexpr int NBLK = XBLK + GBLK;                 // DMA blocks per tile
  static constexpr int QMAX = (NBLK + NW - 1) / NW;        // DMA instructions per wave
  static constexpr int QFULL = NBLK - (QMAX - 1) * NW;     // waves < QFULL issue QMAX
  static constexpr int LDS = NS * STAGE + 2 * CP * 4;
  static_assert(FT % 4 == 0 && NPX % 32 == 0, "two k-halves of whole k-steps");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(4 * NA * 16 * 64 * 4 <= NS * STAGE, "k-half reduction buffer");
};
}  // namespace wdm

// s_waitcnt vmcnt(n * Q), n = DMA tiles left in flight (0..4), Q = this
// wave's DMA instructions per tile
template <int Q>
__device__ __forceinline__ void wdm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Q) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * Q) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * Q) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * Q) : "memory"); break;
  }
}

// dbg (measurement only, AINP_WDM_DBG; wrong results): 1 = no MFMAs,
// 2 = no prologue pass -- what the DMA ring / the pass alone cost
template <int FT, int NS>
__global__ __launch_bounds__(wdm::NT, 1) void conv3x3_wgrad_b16dma_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const uint16_t* __restrict__ dy,
    float* __restrict__ partial, int N, int H, int W, int dbg) {
  using namespace wdm;
  using G = Geo<FT, NS>;
  constexpr int NPX = G::NPX, HC = G::HC, XPIX = G::XPIX, XBLK = G::XBLK, XB = G::XB;
  constexpr int STAGE = G::STAGE, NBLK = G::NBLK, QMAX = G::QMAX, QFULL = G::QFULL;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[G::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int ct = wave & 1, th = (wave >> 1) & 1, kh = wave >> 2;   // co tile, tap half, k-half
  const bool pro = in_scale != nullptr;
  // transposing-read offsets: the register kernel's (conv3x3_wgrad_x6); slot
  // j of tap half th is tap 5 th + j (th = 1, j = 4: the bias, no B read)
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  int bx[NA][2];
#pragma unroll
  for (int j = 0; j < NA; ++j)
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
      const int tap = 5 * th + j < 9 ? 5 * th + j : 8;
      const int hp = (tap / 3) * HS + tap % 3 + q + 4 * sh;
      bx[j][sh] = hp * 64 + 16 * ((2 * (g & 1) + (pp >> 1)) ^ ((hp >> 1) & 3)) + 8 * (pp & 1);
    }
  int ba[2];   // pixel q + 4 sh of the lane's segment (segment offsets added below)
#pragma unroll
  for (int sh = 0; sh < 2; ++sh) {
    const int px = q + 4 * sh;
    ba[sh] = px * 128 + 16 * ((4 * ct + 2 * (g & 1) + (pp >> 1)) ^ wx6_gswz(px)) + 8 * (pp & 1);
  }
  const int tg = tid & 3;
  // prologue constants [scale 32 | shift 32] behind the ring
  float* sss = reinterpret_cast<float*>(smem + NS * STAGE);
  if (pro && tid < 2 * CP) {
    float v = tid < CP ? in_scale[tid] : in_shift[tid - CP];
    asm volatile("" : "+v"(v));
    sss[tid] = v;
  }
  __syncthreads();   // sss, before any DMA is in flight

  // 32-bit tile arithmetic (the launcher checks N * tiles < 2^31)
  const unsigned tiles_t = (W + TT - 1) / TT, tiles_f = (H + FT - 1) / FT;
  const unsigned ntiles = (unsigned)N * tiles_f * tiles_t;
  // contiguous tile ranges per workgroup, frequency tiles fastest
  const unsigned per = ntiles / gridDim.x, rem = ntiles % gridDim.x;
  const unsigned tbeg = blockIdx.x * per + (blockIdx.x < rem ? blockIdx.x : rem);
  const int cnt = (int)(per + (blockIdx.x < rem ? 1 : 0));
  auto coords = [&](unsigned t, int& n, int& f0, int& t0) {
    const unsigned qd = t / tiles_f;
    f0 = (int)(t - qd * tiles_f) * FT;
    n = (int)(qd / tiles_t);
    t0 = (int)(qd - (unsigned)n * tiles_t) * TT;
  };
  // lane unit k of this wave's DMAs: the pixel's (row, col) relative to the
  // tile origin and its byte offset from the origin's pixel.  hole: one of
  // the halo image's unused columns (never read by the MFMAs)
  auto unit = [&](int k, int& rr, int& cc, int& off, bool& hole) {
    const int qb = wave + NW * k;
    if (qb < XBLK) {
      // halo pixel slot sp = 16 qb + lane/4, physical 16-byte group lane % 4
      const int sp = 16 * qb + (lane >> 2), hc = sp & 31;
      const int grp = (lane & 3) ^ ((sp >> 1) & 3);
      hole = hc >= HC;
      rr = (sp >> 5) - 1;
      cc = hole ? 0 : hc - 1;
      off = (rr * W + cc) * (CP * 2) + 16 * grp;
    } else {
      // dy pixel px = 8 j + lane/8, physical 16-byte group lane % 8
      const int px = 8 * (qb - XBLK) + (lane >> 3);
      const int grp = (lane & 7) ^ wx6_gswz(px);
      hole = false;
      rr = px / TT;
      cc = px - rr * TT;
      off = (rr * W + cc) * (CO * 2) + 16 * grp;
    }
  };
  // interior tiles (halo inside the image, the large majority): the source
  // is the tile origin plus a per-lane offset fixed across tiles
  int loff[QMAX];
#pragma unroll
  for (int k = 0; k < QMAX; ++k) {
    int rr, cc;
    bool hole;
    unit(k, rr, cc, loff[k], hole);
  }
  auto interior = [&](int f0, int t0) {
    return f0 >= 1 && f0 + FT + 1 <= H && t0 >= 1 && t0 + TT + 1 <= W;
  };
  auto issue = [&](int i) {
    int n, f0, t0;
    coords(tbeg + i, n, f0, t0);
    const int64_t org = ((int64_t)n * H + f0) * W + t0;
    const char* xo = reinterpret_cast<const char*>(x) + org * (CP * 2);
    const char* go = reinterpret_cast<const char*>(dy) + org * (CO * 2);
    unsigned char* st = smem + (i % NS) * STAGE;
    if (interior(f0, t0)) {
#pragma unroll
      for (int k = 0; k < QMAX; ++k) {
        const int qb = wave + NW * k;
        if (qb >= NBLK) break;
        glds16_asm((qb < XBLK ? xo : go) + loff[k], st + qb * 1024);
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < QMAX; ++k) {
      const int qb = wave + NW * k;
      if (qb >= NBLK) break;
      int rr, cc, off;
      bool hole;
      unit(k, rr, cc, off, hole);
      const bool ok = !hole && (unsigned)(f0 + rr) < (unsigned)H && (unsigned)(t0 + cc) < (unsigned)W;
      glds16_asm(ok ? (qb < XBLK ? xo : go) + off : reinterpret_cast<const char*>(cdd_zero),
                 st + qb * 1024);
    }
  };

  f32x16 acc[NA];
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  bf16x8c ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < cnt) issue(i);
  for (int i = 0; i < cnt; ++i) {
    // tile i landed (this wave's DMAs); tiles i+1 .. i+NS-2 may stay in flight
    const int ahead = cnt - 1 - i < NS - 2 ? cnt - 1 - i : NS - 2;
    if (wave < QFULL) wdm_wait<QMAX>(ahead);
    else wdm_wait<QMAX - 1>(ahead);
    unsigned char* sx = smem + (i % NS) * STAGE;
    const unsigned char* sg = sx + XB;
    if (pro && !(dbg & 2)) {
      // act(x) in place, before the tile's barrier: each lane rewrites the 16
      // bytes its own DMA wrote (its vmcnt wait above retired them), so no
      // other wave's data is read here and the pass overlaps the other waves'
      // MFMAs of the previous tile.  Outside the image the DMA wrote zeros,
      // which stay (nn.Conv2d pads after the ReLU).
      int n, f0, t0;
      coords(tbeg + i, n, f0, t0);
      const bool inner = interior(f0, t0);   // every lane's pixel in the image
#pragma unroll
      for (int k = 0; k < QMAX; ++k) {
        const int qb = wave + NW * k;
        if (qb >= XBLK) break;
        const int sp = 16 * qb + (lane >> 2), hr = sp >> 5, hc = sp & 31;
        const int grp = (lane & 3) ^ ((sp >> 1) & 3);
        const int gr = f0 - 1 + hr, gc = t0 - 1 + hc;
        if (inner || (hc < HC && (unsigned)gr < (unsigned)H && (unsigned)gc < (unsigned)W)) {
          uint4* p = reinterpret_cast<uint4*>(sx + qb * 1024 + 16 * lane);
          const uint4 v = *p;
          const float4 c0 = reinterpret_cast<const float4*>(sss)[2 * grp];
          const float4 c1 = reinterpret_cast<const float4*>(sss)[2 * grp + 1];
          const float4 h0 = reinterpret_cast<const float4*>(sss + CP)[2 * grp];
          const float4 h1 = reinterpret_cast<const float4*>(sss + CP)[2 * grp + 1];
          const float ssc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
          const float ssh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = fmaxf(fmaf(__uint_as_float(w4[e] << 16), ssc[2 * e], ssh[2 * e]), 0.f);
            const float b = fmaxf(fmaf(__uint_as_float(w4[e] & 0xffff0000u), ssc[2 * e + 1],
                                       ssh[2 * e + 1]), 0.f);
            o[e] = cx6_cvt_pk(a, b);
          }
          *p = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // tile i (DMAs + prologue) visible; stage i-1 free
    asm volatile("" ::: "memory");
    if (i + NS - 1 < cnt) issue(i + NS - 1);
    if (dbg & 1) continue;
    // fragments of k-step ks+1 are read while the MFMAs of ks run (two
    // register sets); the bias slot's ones fragment is selected, not branched
    constexpr int KS = NPX / 32;
    // per-lane fragment bases of this stage, once per tile; the k-step and
    // segment offsets below are compile-time (ds_read offset fields)
    // k-step kk takes 8-pixel row segment G = kk (lanes 0-31) and
    // G = kk + NG/2 (lanes 32-63, NG/2 segments = whole tile rows later), so
    // the lane-half part of every fragment address is a per-lane constant
    // folded into these bases and the k-step part is compile-time
    // (the k-half kh likewise: its KS k-steps are KS / 3 whole tile rows)
    constexpr int NG = NPX / 8, HROWS = NG / 2 / 3;
    static_assert((NPX / 32) % 3 == 0, "k-half = whole tile rows");
    const int ao = (lh * (NG / 2) + kh * (NPX / 32)) * 8 * 128;
    const int bo = (lh * HROWS + kh * (NPX / 32) / 3) * HS * 64;
    const unsigned char* pa0 = sg + ba[0] + ao;
    const unsigned char* pa1 = sg + ba[1] + ao;
    const unsigned char* pb[NA][2];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      pb[j][0] = sx + bx[j][0] + bo;
      pb[j][1] = sx + bx[j][1] + bo;
    }
    auto frag_a = [&](int kk) {
      return wx6_cat(wx6_tr(pa0 + kk * 8 * 128), wx6_tr(pa1 + kk * 8 * 128));
    };
    auto frag_b = [&](int kk, int j) {
      const int seg = (kk / 3) * HS + (kk % 3) * 8;
      return wx6_cat(wx6_tr(pb[j][0] + seg * 64), wx6_tr(pb[j][1] + seg * 64));
    };
    bf16x8c fa[2], fb[2][NA];
    fa[0] = frag_a(0);
#pragma unroll
    for (int j = 0; j < NA; ++j) fb[0][j] = frag_b(0, j);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < KS) {
        fa[cur ^ 1] = frag_a(ks + 1);
#pragma unroll
        for (int j = 0; j < NA; ++j) fb[cur ^ 1][j] = frag_b(ks + 1, j);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the MFMAs
#pragma unroll
      for (int j = 0; j < NA - 1; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], fb[cur][j], acc[j], 0, 0, 0);
      acc[NA - 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur], th ? ones : fb[cur][NA - 1],
                                                            acc[NA - 1], 0, 0, 0);
    }
  }
  // combine the k-halves through the (now idle) ring, then one slab
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  const int wg = wave & 3;
  if (kh == 1) {
#pragma unroll
    for (int t = 0; t < NA; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wg * NA + t) * 16 + r) * 64 + lane] = acc[t][r];
  }
  __syncthreads();
  if (kh == 1) return;
  float* slab = partial + (int64_t)blockIdx.x * CO * (J + 1);
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int tap = 5 * th + j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const float v = acc[j][r] + red[((wg * NA + j) * 16 + r) * 64 + lane];
      if (tap < 9) slab[co * (J + 1) + tap * CP + li] = v;
      else if (li == 0) slab[co * (J + 1) + J] = v;    // the ones column: db
    }
  }
}

// AINP_WGRAD16_DMA=0: the register-staged kernel for that weight gradient (A/B)
static bool wgrad16_dma() {
  static const bool v = [] {
    const char* e = getenv("AINP_WGRAD16_DMA");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Small-channel variant for (Cin pass, Cout) = (32, 16) and (16, 32): one of
// the two GEMM dimensions is 16, so the 32x32 tiles above would be half
// empty.  Same tiles, staging, slabs and bias as conv3x3_wgrad_x6, on
// v_mfma_f32_16x16x32_bf16 (16 x 16 outputs, 32 pixels per k-step):
//  * 6 waves = (16-channel block of the 32-wide side, tap row) x 3 taps;
//  * A (dy) and B (act(x)) fragments are two transposing reads each: lane
//    group g (= lane >> 4) takes the k-step's 8-pixel segment 4ks + g;
//  * both images keep 64 bytes per pixel; the 16-byte group swizzle
//    f(px) = px bit 1 | (px bit 2 ^ px bit 3) << 1 keeps the writes
//    (8 consecutive pixels) and the reads (two groups 8 pixels apart, the
//    halo row stride being == 8 mod 16) conflict-free.
namespace wx6s {
constexpr int TT = 24, HC = TT + 2;            // tile columns (3 segments of 8), halo columns
constexpr int HS = 40;                         // halo row stride (pixels, == 8 mod 16)
// FT tile rows: NPX = 24 FT pixels, 3 FT / 4 k-steps of 32
template <int FT> constexpr int npx() { return FT * TT; }
template <int FT> constexpr int xpl() { return (FT + 1) * HS * 64 + HC * 64; }
template <int FT> constexpr int gpl() { return npx<FT>() * 64; }
}  // namespace wx6s

__device__ __forceinline__ int wx6s_swz(int px) {
  return ((px >> 1) & 1) | ((((px >> 2) ^ (px >> 3)) & 1) << 1);
}

template <int CP, int CO, int NP, bool G16 = false, bool XG16 = false, bool XL = false,
          bool GL = false, int FT = 4>
__global__ __launch_bounds__(384, FT == 4 ? 3 : NP == 1 ? 2 : 1) void conv3x3_wgrad_x6s(
    const float* __restrict__ x, const float* __restrict__ in_scale,
    const float* __restrict__ in_shift, const float* __restrict__ dy,
    float* __restrict__ partial, int N, int Cin, int H, int W, int ci0) {
  using namespace wx6s;
  static_assert((CP == 32 && CO == 16) || (CP == 16 && CO == 32), "shape");
  constexpr int NPX = npx<FT>(), HR = FT + 2, XPL = xpl<FT>(), GPL = gpl<FT>();
  constexpr int J = 9 * CP, NT = 384;
  constexpr int XG = CP / 8, XU = HR * HC * XG, XI = (XU + NT - 1) / NT;
  constexpr int GG = CO / 8, GU = NPX * GG;     // dy units (pixel, 8-co group)
  constexpr int GI = (GU + NT - 1) / NT;         // dy units per thread (unit tid + NT i)
  static_assert(NT % NPX == 0 && NT % GG == 0, "a thread's dy units share a pixel (NCHW) / a group (CL)");
  // sx doubles as the bias reduction buffer [CO][NPX] floats after the loop
  constexpr int SXB = NP * XPL > CO * NPX * 4 ? NP * XPL : CO * NPX * 4;
  __shared__ __attribute__((aligned(16))) unsigned char sx[SXB];
  __shared__ __attribute__((aligned(16))) unsigned char sg[NP * GPL];
  __shared__ __attribute__((aligned(16))) float s_ss[2 * CP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = wave & 1, dyt = wave >> 1;
  const int cob = CO == 32 ? blk : 0, cib = CP == 32 ? blk : 0;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  // transposing-read address of a pixel for this lane (lane 4q+pp of its
  // group supplies pixel q (+4) at channels 4pp..4pp+3 of its 16-block)
  auto xaddr = [&](int hp) {
    return hp * 64 + 16 * ((2 * cib + (pp >> 1)) ^ wx6s_swz(hp)) + 8 * (pp & 1);
  };
  auto gaddr = [&](int px) {
    return px * 64 + 16 * ((2 * cob + (pp >> 1)) ^ wx6s_swz(px)) + 8 * (pp & 1);
  };

  if (tid < 2 * CP)
    s_ss[tid] = in_scale ? (tid < CP ? in_scale[ci0 + tid] : in_shift[ci0 + tid - CP]) : 0.f;

  f32x4 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[GI][8];
#pragma unroll
  for (int i = 0; i < GI; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) bsum[i][c] = 0.f;

  const int tiles_t = (W + TT - 1) / TT, tiles_f = (H + FT - 1) / FT;
  const int64_t ntiles = (int64_t)N * tiles_f * tiles_t;
  const int64_t HW = (int64_t)H * W;
  auto tile_coords = [&](int64_t tile, int& n, int& f0, int& t0) {
    t0 = (int)(tile % tiles_t) * TT;
    f0 = (int)((tile / tiles_t) % tiles_f) * FT;
    n = (int)(tile / ((int64_t)tiles_t * tiles_f));
  };
  // dy unit i of this thread (unit tid + NT i < GU): pixel and 8-channel
  // group; the channel-last order puts a pixel's groups on consecutive lanes
  auto gunit = [&](int i, int& px_, int& grp_) {
    const int gu = tid + NT * i;
    px_ = GL ? gu / GG : gu % NPX;
    grp_ = GL ? gu % GG : gu / NPX;
  };
  auto xunit = [&](int u, int& hp_, int& grp_) {
    if constexpr (XL) {
      hp_ = u / XG;
      grp_ = u % XG;
    } else {
      hp_ = u % (HR * HC);
      grp_ = u / (HR * HC);
    }
  };

  float px[XI][8], pg[GI][8];
  auto fetch = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
    // act(x) input: fp32 or bf16 storage (XG16)
    constexpr int XES = act_es<XG16>();
    if constexpr (XL) {
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<XG16>(x, (int64_t)n * HW * Cin + ci0);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        int hp, grp;
        xunit(u < XU ? u : XU - 1, hp, grp);
        const int gr = wx6_clamp(f0 - 1 + hp / HC, 0, H - 1);
        const int gc = wx6_clamp(t0 - 1 + hp % HC, 0, W - 1);
        cl_ld8<XG16>(rx, ((gr * W + gc) * Cin + 8 * grp) * XES, px[i]);
      }
    } else {
      int plane = (int)(HW * XES);
      asm volatile("" : "+s"(plane));
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<XG16>(x, ((int64_t)n * Cin + ci0) * HW);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        const int hp = u % (HR * HC), grp = u < XU ? u / (HR * HC) : XG - 1;
        const int gr = wx6_clamp(f0 - 1 + hp / HC, 0, H - 1);
        const int gc = wx6_clamp(t0 - 1 + hp % HC, 0, W - 1);
        const int vo = 8 * grp * plane + (gr * W + gc) * XES;
#pragma unroll
        for (int c = 0; c < 8; ++c) px[i][c] = act_ld<XG16>(rx, vo, c * plane);
      }
    }
    // dy: fp32 or bf16 storage (G16)
    constexpr int GES = act_es<G16>();
    int gplane = (int)(HW * GES);
    asm volatile("" : "+s"(gplane));
    const __amdgpu_buffer_rsrc_t rg =
        act_rsrc<G16>(dy, GL ? (int64_t)n * HW * CO : (int64_t)n * CO * HW);
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      int gpx, ggrp;
      gunit(i, gpx, ggrp);
      const int gpc = gpx < NPX ? gpx : NPX - 1, ggc = ggrp < GG ? ggrp : GG - 1;
      const int gr = wx6_clamp(f0 + gpc / TT, 0, H - 1), gc = wx6_clamp(t0 + gpc % TT, 0, W - 1);
      if constexpr (GL) {
        cl_ld8<G16>(rg, ((gr * W + gc) * CO + 8 * ggc) * GES, pg[i]);
      } else {
        const int vo = 8 * ggc * gplane + (gr * W + gc) * GES;
#pragma unroll
        for (int c = 0; c < 8; ++c) pg[i][c] = act_ld<G16>(rg, vo, c * gplane);
      }
    }
  };
  auto commit = [&](int64_t tile) {
    int n, f0, t0;
    tile_coords(tile, n, f0, t0);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int u = tid + NT * i;
      if (u < XU) {
        int hp, grp;
        xunit(u, hp, grp);
        const int hr = hp / HC, hc = hp % HC;
        const int gr = f0 - 1 + hr, gc = t0 - 1 + hc;
        const bool inb = gr >= 0 && gr < H && gc >= 0 && gc < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = px[i][c];
          if (in_scale) t = fmaxf(fmaf(t, s_ss[8 * grp + c], s_ss[CP + 8 * grp + c]), 0.f);
          v[c] = inb ? t : 0.f;
        }
        const int sp = hr * HS + hc;
        cx6_stage<NP>(v, sx + sp * 64 + 16 * (grp ^ wx6s_swz(sp)), XPL);
      }
    }
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      if (tid + NT * i < GU) {
        int gpx, ggrp;
        gunit(i, gpx, ggrp);
        const bool pok = f0 + gpx / TT < H && t0 + gpx % TT < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = pok ? pg[i][c] : 0.f;
          bsum[i][c] += v[c];
        }
        cx6_stage<NP>(v, sg + gpx * 64 + 16 * (ggrp ^ wx6s_swz(gpx)), GPL);
      }
    }
  };

  __syncthreads();  // s_ss
  int64_t tile = blockIdx.x;
  if (tile < ntiles) fetch(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    commit(tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
#pragma unroll
    for (int ks = 0; ks < NPX / 32; ++ks) {
      // this lane group's 8-pixel segment G = 4ks + g: tile row G/3, column 8(G%3)
      const int G = 4 * ks + g;
      const int srow = G / 3, scol = (G % 3) * 8;
      bf16x8c a[NP];
      {
        const int o0 = gaddr(8 * G + q), o1 = gaddr(8 * G + q + 4);
#pragma unroll
        for (int p = 0; p < NP; ++p)
          a[p] = wx6_cat(wx6_tr(sg + p * GPL + o0), wx6_tr(sg + p * GPL + o1));
      }
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int hp = (srow + dyt) * HS + scol + dx + q;
        const int o0 = xaddr(hp), o1 = xaddr(hp + 4);
        bf16x8c b[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          b[p] = wx6_cat(wx6_tr(sx + p * XPL + o0), wx6_tr(sx + p * XPL + o1));
        // D[co][ci]: A = dy (rows co), B = act(x) (columns ci); six cross
        // terms smallest first (NP = 3), or the bf16 product
        f32x4 c = acc[dx];
#pragma unroll
        for (int t = 0; t < cx6_terms(NP); ++t)
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cx6_pa(NP, t)], b[cx6_pb(NP, t)], c, 0,
                                                      0, 0);
        acc[dx] = c;
      }
    }
    __syncthreads();
  }

  // slab [CO][J + 1]: D[co = 16cob + 4g + r][ci = 16cib + (lane & 15)] of tap 3dyt+dx
  float* slab = partial + (int64_t)blockIdx.x * CO * (J + 1);
#pragma unroll
  for (int dx = 0; dx < 3; ++dx)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * cob + 4 * g + r;
      slab[co * (J + 1) + (3 * dyt + dx) * CP + 16 * cib + (lane & 15)] = acc[dx][r];
    }
  float* red = reinterpret_cast<float*>(sx);
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    if (tid + NT * i < GU) {
      int gpx, ggrp;
      gunit(i, gpx, ggrp);
#pragma unroll
      for (int c = 0; c < 8; ++c) red[(8 * ggrp + c) * NPX + gpx] = bsum[i][c];
    }
  }
  __syncthreads();
  if (tid < CO) {
    float sum = 0.f;
    for (int k = 0; k < NPX; ++k) sum += red[tid * NPX + k];
    slab[tid * (J + 1) + J] = sum;
  }
}

// ------------------------------------------------------- persistent fwd/dgrad
// Forward / data gradient as a persistent kernel: one workgroup per CU walks
// a strided set of 8 x 32-pixel output tiles, so that
//  * every K chunk's split weights stay resident in LDS for the whole launch
//    (staged and split once, not per tile);
//  * the next (tile, chunk) halo is prefetched into registers (buffer loads,
//    32-bit offsets) while the current chunk's MFMAs run, across tile
//    boundaries too;
//  * the BatchNorm partials are accumulated per workgroup in fixed tile
//    order (fp32 over a tile row's 32 pixels by a lane reduce-scatter, fp64
//    across tiles) and written once: the partial count is the fixed grid.
// Wave w owns output row w of the tile (32 pixels x COP channels); fragments,
// layouts and the six-product arithmetic are those of conv3x3_x6_kernel.
namespace cxp {
constexpr int TC = 32, HC = TC + 2;      // tile columns, halo columns
constexpr int CK = 16;                   // input channels per K chunk
constexpr int XROW = HC * 32;            // halo row bytes per plane (16 bf16 per pixel)
constexpr int WROW = 9 * 32 + 16;        // weight row bytes per chunk and plane
}  // namespace cxp

// XL / YL (round 5): input / output channel-last ([N][H][W][C]) instead of
// NCHW.  A channel-last staging unit u is (pixel u >> 1, 8-channel half u & 1):
// the two lanes of a pixel read its chunk's 16 channels as contiguous bytes.
template <int CI, int COP, bool DGRAD, int NT, int TR, int NP, bool G16 = false, bool Y16 = false,
          bool XL = false, bool YL = false>
__global__ __launch_bounds__(NT, NT / 256) void conv3x3_x6p_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, int N, int Cout, int H, int W, Bnr bnr) {
  using namespace cxp;
  static_assert(CI % CK == 0 && (COP == 32 || COP == 64), "shape");
  constexpr int NI = COP / 32, NCH = CI / CK;
  // tile TR x 32 pixels; wave w = output row w % TR and 32-channel tiles
  // [(w / TR) * NIW, +NIW): 8 waves of 8 rows x COP channels, or 16 waves
  // (twice the waves to hide the staging) as 8 rows x 2 channel halves
  // (COP = 64) or 16 rows (COP = 32)
  constexpr int HR = TR + 2, XPLANE = HR * XROW, XU = 2 * HR * HC;
  constexpr int NW = NT / 64, NIW = NI * TR / NW;
  constexpr int XI = (XU + NT - 1) / NT;
  static_assert(NIW >= 1 && NIW * NW == NI * TR, "waves");
  constexpr int WPLANE = COP * WROW, WCH = NP * WPLANE;
  constexpr int WU = NCH * COP * 18;       // weight units (chunk, co, tap, half)
  __shared__ __attribute__((aligned(16))) unsigned char sw[NCH * WCH];
  __shared__ __attribute__((aligned(16))) unsigned char sx[NP * XPLANE];
  __shared__ float s_ss[2 * CI];
  static_assert(NP * XPLANE >= TR * 2 * COP * 8, "BatchNorm row sums reuse the halo image");
  // fused BatchNorm-backward reduce (Bnr): constants in LDS; the tile's y
  // is loaded in one batch at the top of the epilogue (holding it across the
  // MFMA loop would cost this kernel its second workgroup per CU)
  constexpr bool FZ = DGRAD && YL;
  __shared__ float sbn[FZ ? 4 * COP : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int wrow = wave % TR, wco = (wave / TR) * NIW;  // output row, first 32-channel tile
  const int64_t HW = (int64_t)H * W;
  const bool fused = FZ && bnr.y != nullptr;
  if (fused) bnr_stage(bnr, sbn, Cout, COP, tid, NT);

  for (int u = tid; u < WU; u += NT) {
    const int half = u & 1, tap = (u >> 1) % 9, co = (u / 18) % COP, ch = u / (18 * COP);
    float pw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int ci = ch * CK + 8 * half + c;
      pw[c] = co < Cout ? (DGRAD ? w[((int64_t)ci * Cout + co) * 9 + (8 - tap)]
                                 : w[((int64_t)co * CI + ci) * 9 + tap])
                        : 0.f;
    }
    cx6_stage<NP>(pw, sw + ch * WCH + co * WROW + tap * 32 + 16 * half, WPLANE);
  }
  if (tid < 2 * CI)
    s_ss[tid] = in_scale ? (tid < CI ? in_scale[tid] : in_shift[tid - CI]) : 0.f;
  // bias from LDS: a global load in the epilogue would make it wait for the
  // next tile's halo prefetch (vmcnt is in order)
  __shared__ float s_b[COP];
  if (tid < COP) s_b[tid] = (bias && tid < Cout) ? bias[tid] : 0.f;

  const int tiles_c = (W + TC - 1) / TC, tiles_r = (H + TR - 1) / TR;
  const int64_t ntiles = (int64_t)N * tiles_r * tiles_c;
  auto tile_coords = [&](int64_t tile, int& n, int& r0, int& c0) {
    c0 = (int)(tile % tiles_c) * TC;
    r0 = (int)((tile / tiles_c) % tiles_r) * TR;
    n = (int)(tile / ((int64_t)tiles_c * tiles_r));
  };

  float px[XI][8];
  // staging unit -> (halo column, halo row, channel half)
  auto unit = [&](int u, int& col, int& row, int& half) {
    if constexpr (XL) {
      half = u & 1;
      const int hp = u >> 1;
      col = hp % HC;
      row = hp / HC;
    } else {
      col = u % HC;
      row = (u / HC) % HR;
      half = u / (HR * HC);
    }
  };
  auto fetch = [&](int64_t tile, int ch) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
    constexpr int ES = act_es<G16>();
    if constexpr (XL) {
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, (int64_t)n * HW * CI + ch * CK);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        int col, row, half;
        unit(u < XU ? u : XU - 1, col, row, half);
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        cl_ld8<G16>(rx, ((gr * W + gc) * CI + 8 * half) * ES, px[i]);
      }
    } else {
      int plane = (int)(HW * ES);
      asm volatile("" : "+s"(plane));  // keep c * plane out of the loop
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, ((int64_t)n * CI + ch * CK) * HW);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        const int col = u % HC, row = (u / HC) % HR, half = u < XU ? u / (HR * HC) : 1;
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        const int vo = 8 * half * plane + (gr * W + gc) * ES;
#pragma unroll
        for (int c = 0; c < 8; ++c) px[i][c] = act_ld<G16>(rx, vo, c * plane);
      }
    }
  };
  auto commit = [&](int64_t tile, int ch) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int u = tid + NT * i;
      if (u < XU) {
        int col, row, half;
        unit(u, col, row, half);
        const int gr = r0 - 1 + row, gc = c0 - 1 + col;
        const bool inb = gr >= 0 && gr < H && gc >= 0 && gc < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = px[i][c];
          if (in_scale) {
            const int ci = ch * CK + 8 * half + c;
            t = fmaxf(fmaf(t, s_ss[ci], s_ss[CI + ci]), 0.f);
          }
          v[c] = inb ? t : 0.f;
        }
        cx6_stage<NP>(v, sx + row * XROW + col * 32 + 16 * (half ^ ((col >> 3) & 1)), XPLANE);
      }
    }
  };

  f32x16 acc[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  double bs[NIW], bq[NIW];   // BatchNorm sums of channel row li>>1 (see epilogue)
#pragma unroll
  for (int i = 0; i < NIW; ++i) bs[i] = bq[i] = 0.0;

  // 16 values per lane -> lane li holds the sum over the 32 lanes of its half
  // of value li >> 1 (fixed butterfly order)
  auto reduce16 = [&](const float (&v)[16]) {
    float t8[8], t4[4], t2[2];
    const bool b4 = li & 16, b3 = li & 8, b2 = li & 4, b1 = li & 2;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      t8[k] = (b4 ? v[k + 8] : v[k]) + __shfl_xor(b4 ? v[k] : v[k + 8], 16, 64);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      t4[k] = (b3 ? t8[k + 4] : t8[k]) + __shfl_xor(b3 ? t8[k] : t8[k + 4], 8, 64);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      t2[k] = (b2 ? t4[k + 2] : t4[k]) + __shfl_xor(b2 ? t4[k] : t4[k + 2], 4, 64);
    const float t1 = (b1 ? t2[1] : t2[0]) + __shfl_xor(b1 ? t2[0] : t2[1], 2, 64);
    return t1 + __shfl_xor(t1, 1, 64);
  };

  auto epilogue = [&](int64_t tile) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
    const int row = r0 + wrow, col = c0 + li;
    const bool pok = row < H && col < W;
    const int64_t yo = (int64_t)n * Cout * HW + (int64_t)row * W + col;
    const int64_t ycl = ((int64_t)n * HW + (int64_t)row * W + col) * Cout;
    uint4 yr[FZ ? NIW : 1][4];
    if constexpr (FZ) {
      if (fused) {
#pragma unroll
        for (int i = 0; i < NIW; ++i)
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            const int co0 = 32 * (wco + i) + 8 * rb + 4 * lh;
            yr[i][rb] = bnr_ld4(bnr, (pok && co0 < Cout) ? ycl + co0 : 0);
          }
      }
    }
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      float s[16], q[16], vv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * (wco + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const bool ok = pok && co < Cout;
        float v = acc[i][r] + s_b[co];
        if constexpr (Y16) v = y16_round(v);
        if constexpr (!YL) {
          if constexpr (Y16) {
            if (ok) y16_st(y, yo + (int64_t)co * HW, v);
          } else {
            if (ok) y[yo + (int64_t)co * HW] = v;
          }
        }
        vv[r] = v;
        s[r] = ok ? v : 0.f;
        q[r] = s[r] * s[r];
      }
      if constexpr (FZ) {   // fused BatchNorm-backward reduce (Bnr)
        if (fused) {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            const int co0 = 32 * (wco + i) + 8 * rb + 4 * lh;
            const float v4[4] = {vv[4 * rb], vv[4 * rb + 1], vv[4 * rb + 2], vv[4 * rb + 3]};
            float yv[4];
            bnr_dec4(bnr.y16, yr[FZ ? i : 0][rb], yv);
            bnr_terms4<COP>(sbn, co0, yv, v4, pok && co0 < Cout, s + 4 * rb, q + 4 * rb);
          }
        }
      }
      if constexpr (YL) {   // 4 consecutive channels per store (Cout % 4 == 0)
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int co0 = 32 * (wco + i) + 8 * rb + 4 * lh;
          if (pok && co0 < Cout)
            cl_st4<Y16>(y, ycl + co0, vv[4 * rb], vv[4 * rb + 1], vv[4 * rb + 2], vv[4 * rb + 3]);
        }
      }
      if (stats) {
        bs[i] += (double)reduce16(s);
        bq[i] += (double)reduce16(q);
      }
    }
  };

  __syncthreads();  // weights, s_ss
  int64_t tile = blockIdx.x;
  int ch = 0;
  if (tile < ntiles) fetch(tile, 0);
  while (tile < ntiles) {
    commit(tile, ch);
    __syncthreads();
    int nch = ch + 1;
    int64_t ntile = tile;
    if (nch == NCH) {
      nch = 0;
      ntile += gridDim.x;
    }
    if (ntile < ntiles) fetch(ntile, nch);
    const unsigned char* wb0 = sw + ch * WCH + li * WROW + 16 * lh;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
      const int hcol = li + dx;
      const unsigned char* xb =
          sx + (wrow + dy) * XROW + hcol * 32 + 16 * (lh ^ ((hcol >> 3) & 1));
      bf16x8c a[NP][NIW], b[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < NIW; ++i)
          a[p][i] = cx6_ld(wb0 + p * WPLANE + (wco + i) * 32 * WROW + tap * 32);
        b[p] = cx6_ld(xb + p * XPLANE);
      }
      // six cross terms smallest first, term-major over the NI accumulators
#pragma unroll
      for (int t = 0; t < cx6_terms(NP); ++t) {
        const int pa = cx6_pa(NP, t), pb = cx6_pb(NP, t);
#pragma unroll
        for (int i = 0; i < NIW; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa][i], b[pb], acc[i], 0, 0, 0);
      }
    }
    if (nch == 0) {  // the tile's last chunk: store, BatchNorm sums, restart
      epilogue(tile);
#pragma unroll
      for (int i = 0; i < NIW; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    }
    __syncthreads();
    tile = ntile;
    ch = nch;
  }

  if (!stats) return;
  // per-row sums -> [row][sum, sum of squares][COP] (the halo image is free)
  double* red = reinterpret_cast<double*>(sx);
  if ((li & 1) == 0) {
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int r = li >> 1;
      const int co = 32 * (wco + i) + (r & 3) + 8 * (r >> 2) + 4 * lh;
      red[(wrow * 2 + 0) * COP + co] = bs[i];
      red[(wrow * 2 + 1) * COP + co] = bq[i];
    }
  }
  __syncthreads();
  for (int co = tid; co < Cout; co += NT) {
    double s = 0.0, q = 0.0;
    for (int wv = 0; wv < TR; ++wv) {
      s += red[(wv * 2 + 0) * COP + co];
      q += red[(wv * 2 + 1) * COP + co];
    }
    stats[(int64_t)blockIdx.x * 2 * Cout + co] = s;
    stats[(int64_t)blockIdx.x * 2 * Cout + Cout + co] = q;
  }
}

// 16-output-channel variant (decoder 32->16 and the 16->32 convs' data
// gradients): the persistent kernel above on v_mfma_f32_16x16x32_bf16, so no
// half of a 32-wide tile is wasted.  A k-step is two taps x 16 channels of one
// chunk (lane group g = lane >> 4 takes tap 2s + (g >> 1), channels
// 8 (g & 1) .. +7); the tenth tap slot of a weight row is zero.  Wave = one
// output row as two 16-pixel tiles sharing the A fragments.  Weight rows are
// 336 bytes (10 tap slots + pad: conflict-free 16-lane b128 reads).
namespace cxq {
constexpr int TR = 8, HR = TR + 2;
constexpr int WROW = 10 * 32 + 16;
constexpr int XPLANE = HR * cxp::XROW;
constexpr int XU = 2 * HR * cxp::HC;
}  // namespace cxq

template <int CI, bool DGRAD, int NP, bool G16 = false, bool Y16 = false, bool XL = false,
          bool YL = false>
__global__ __launch_bounds__(512, 2) void conv3x3_x6q_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
    float* __restrict__ y, double* __restrict__ stats, int N, int Cout, int H, int W, Bnr bnr,
    int ycf) {
  using cxp::CK;
  using cxp::HC;
  using cxp::TC;
  using cxp::XROW;
  using namespace cxq;
  constexpr int NT = 512, CO = 16, NCH = CI / CK;
  constexpr int WPLANE = CO * WROW, WCH = NP * WPLANE;
  constexpr int WU = NCH * CO * 20;          // weight units (chunk, co, tap slot, half)
  constexpr int XI = (XU + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) unsigned char sw[NCH * WCH];
  __shared__ __attribute__((aligned(16))) unsigned char sx[NP * XPLANE];
  __shared__ float s_ss[2 * CI];
  static_assert(NP * XPLANE >= TR * 2 * CO * 8, "BatchNorm row sums reuse the halo image");
  // fused BatchNorm-backward reduce (Bnr): as in conv3x3_x6p_kernel
  constexpr bool FZ = DGRAD && YL;
  __shared__ float sbn[FZ ? 4 * CO : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int64_t HW = (int64_t)H * W;
  const bool fused = FZ && bnr.y != nullptr;
  if (fused) bnr_stage(bnr, sbn, Cout, CO, tid, NT);
  uint4 yr[2];

  for (int u = tid; u < WU; u += NT) {
    const int half = u & 1, tap = (u >> 1) % 10, co = (u / 20) % CO, ch = u / (20 * CO);
    float pw[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int ci = ch * CK + 8 * half + c;
      pw[c] = (co < Cout && tap < 9) ? (DGRAD ? w[((int64_t)ci * Cout + co) * 9 + (8 - tap)]
                                              : w[((int64_t)co * CI + ci) * 9 + tap])
                                     : 0.f;
    }
    cx6_stage<NP>(pw, sw + ch * WCH + co * WROW + tap * 32 + 16 * half, WPLANE);
  }
  if (tid < 2 * CI)
    s_ss[tid] = in_scale ? (tid < CI ? in_scale[tid] : in_shift[tid - CI]) : 0.f;
  // bias from LDS (see conv3x3_x6p_kernel)
  __shared__ float s_b[CO];
  if (tid < CO) s_b[tid] = (bias && tid < Cout) ? bias[tid] : 0.f;

  const int tiles_c = (W + TC - 1) / TC, tiles_r = (H + TR - 1) / TR;
  const int64_t ntiles = (int64_t)N * tiles_r * tiles_c;
  auto tile_coords = [&](int64_t tile, int& n, int& r0, int& c0) {
    c0 = (int)(tile % tiles_c) * TC;
    r0 = (int)((tile / tiles_c) % tiles_r) * TR;
    n = (int)(tile / ((int64_t)tiles_c * tiles_r));
  };

  float px[XI][8];
  // staging unit -> (halo column, halo row, channel half); channel-last: the
  // two lanes of a pixel read its chunk's channels as contiguous bytes
  auto unit = [&](int u, int& col, int& row, int& half) {
    if constexpr (XL) {
      half = u & 1;
      const int hp = u >> 1;
      col = hp % HC;
      row = hp / HC;
    } else {
      col = u % HC;
      row = (u / HC) % HR;
      half = u / (HR * HC);
    }
  };
  auto fetch = [&](int64_t tile, int ch) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
    constexpr int ES = act_es<G16>();
    if constexpr (XL) {
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, (int64_t)n * HW * CI + ch * CK);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        int col, row, half;
        unit(u < XU ? u : XU - 1, col, row, half);
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        cl_ld8<G16>(rx, ((gr * W + gc) * CI + 8 * half) * ES, px[i]);
      }
    } else {
      int plane = (int)(HW * ES);
      asm volatile("" : "+s"(plane));
      const __amdgpu_buffer_rsrc_t rx = act_rsrc<G16>(x, ((int64_t)n * CI + ch * CK) * HW);
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int u = tid + NT * i;
        const int col = u % HC, row = (u / HC) % HR, half = u < XU ? u / (HR * HC) : 1;
        const int gr = wx6_clamp(r0 - 1 + row, 0, H - 1), gc = wx6_clamp(c0 - 1 + col, 0, W - 1);
        const int vo = 8 * half * plane + (gr * W + gc) * ES;
#pragma unroll
        for (int c = 0; c < 8; ++c) px[i][c] = act_ld<G16>(rx, vo, c * plane);
      }
    }
  };
  auto commit = [&](int64_t tile, int ch) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int u = tid + NT * i;
      if (u < XU) {
        int col, row, half;
        unit(u, col, row, half);
        const int gr = r0 - 1 + row, gc = c0 - 1 + col;
        const bool inb = gr >= 0 && gr < H && gc >= 0 && gc < W;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float t = px[i][c];
          if (in_scale) {
            const int ci = ch * CK + 8 * half + c;
            t = fmaxf(fmaf(t, s_ss[ci], s_ss[CI + ci]), 0.f);
          }
          v[c] = inb ? t : 0.f;
        }
        cx6_stage<NP>(v, sx + row * XROW + col * 32 + 16 * (half ^ ((col >> 3) & 1)), XPLANE);
      }
    }
  };

  f32x4 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  double bs = 0.0, bq = 0.0;   // BatchNorm sums of channel 4g + ((lane >> 2) & 3)

  // 4 values per lane -> lane holds the sum over its 16-lane group of value
  // (lane >> 2) & 3 (fixed butterfly order)
  auto reduce4 = [&](const float (&v)[4]) {
    const bool b3 = lane & 8, b2 = lane & 4;
    float t2[2];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      t2[k] = (b3 ? v[k + 2] : v[k]) + __shfl_xor(b3 ? v[k] : v[k + 2], 8, 64);
    float t1 = (b2 ? t2[1] : t2[0]) + __shfl_xor(b2 ? t2[0] : t2[1], 4, 64);
    t1 += __shfl_xor(t1, 2, 64);
    return t1 + __shfl_xor(t1, 1, 64);
  };

  auto epilogue = [&](int64_t tile) {
    int n, r0, c0;
    tile_coords(tile, n, r0, c0);
    const int row = r0 + wave;
    // NCHW, or (ycf) [C][H][N][W]: the same contiguous rows of W, other strides
    const int64_t yo = ycf ? ((int64_t)row * N + n) * W : (int64_t)n * Cout * HW + (int64_t)row * W;
    const int64_t cs = ycf ? (int64_t)N * HW : HW;
    float s[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = c0 + 16 * j + l16;
      const bool pok = row < H && col < W;
      float vv[4], ts[4], tq[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 4 * g + r;
        const bool ok = pok && co < Cout;
        float v = acc[j][r] + s_b[co];
        if constexpr (Y16) v = y16_round(v);
        if constexpr (!YL) {
          if constexpr (Y16) {
            if (ok) y16_st(y, yo + (int64_t)co * cs + col, v);
          } else {
            if (ok) y[yo + (int64_t)co * cs + col] = v;
          }
        }
        vv[r] = v;
        const float sv = ok ? v : 0.f;
        ts[r] = sv;
        tq[r] = sv * sv;
      }
      if constexpr (FZ) {   // fused BatchNorm-backward reduce (Bnr)
        if (fused) {
          float yv[4];
          bnr_dec4(bnr.y16, yr[j], yv);
          bnr_terms4<CO>(sbn, 4 * g, yv, vv, pok && 4 * g < Cout, ts, tq);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[r] += ts[r];
        q[r] += tq[r];
      }
      if constexpr (YL) {   // channels 4g .. 4g+3 of pixel (row, col)
        if (pok && 4 * g < Cout)
          cl_st4<Y16>(y, ((int64_t)n * HW + (int64_t)row * W + col) * Cout + 4 * g, vv[0], vv[1],
                      vv[2], vv[3]);
      }
    }
    if (stats) {
      bs += (double)reduce4(s);
      bq += (double)reduce4(q);
    }
  };

  __syncthreads();  // weights, s_ss
  int64_t tile = blockIdx.x;
  int ch = 0;
  if (tile < ntiles) fetch(tile, 0);
  while (tile < ntiles) {
    commit(tile, ch);
    __syncthreads();
    int nch = ch + 1;
    int64_t ntile = tile;
    if (nch == NCH) {
      nch = 0;
      ntile += gridDim.x;
    }
    if constexpr (FZ) {
      if (fused && nch == 0) {   // this tile's y (its last chunk)
        int n, r0, c0;
        tile_coords(tile, n, r0, c0);
        const int row = r0 + wave;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = c0 + 16 * j + l16;
          const bool ok = row < H && col < W && 4 * g < Cout;
          yr[j] = bnr_ld4(bnr, ok ? ((int64_t)n * HW + (int64_t)row * W + col) * Cout + 4 * g : 0);
        }
      }
      // unconditional (see conv3x3_x6p_kernel)
      fetch(ntile < ntiles ? ntile : tile, nch);
    } else {
      if (ntile < ntiles) fetch(ntile, nch);
    }
    const unsigned char* wb0 = sw + ch * WCH + l16 * WROW + 16 * (g & 1);
#pragma unroll
    for (int ks = 0; ks < 5; ++ks) {
      const int tap = 2 * ks + (g >> 1);            // 9 = the zero slot
      const int tp = tap < 9 ? tap : 8;             // its (unused) pixel shift
      const int dy = tp / 3, dx = tp % 3;
      bf16x8c a[NP], b[NP][2];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        a[p] = cx6_ld(wb0 + p * WPLANE + tap * 32);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int hcol = 16 * j + l16 + dx;
          b[p][j] = cx6_ld(sx + p * XPLANE + (wave + dy) * XROW + hcol * 32 +
                           16 * ((g & 1) ^ ((hcol >> 3) & 1)));
        }
      }
#pragma unroll
      for (int t = 0; t < cx6_terms(NP); ++t) {
        const int pa = cx6_pa(NP, t), pb = cx6_pb(NP, t);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[pa], b[pb][j], acc[j], 0, 0, 0);
      }
    }
    if (nch == 0) {
      epilogue(tile);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    tile = ntile;
    ch = nch;
  }

  if (!stats) return;
  double* red = reinterpret_cast<double*>(sx);   // [row][sum, sum of squares][16]
  if ((lane & 3) == 0) {
    const int co = 4 * g + ((lane >> 2) & 3);
    red[(wave * 2 + 0) * CO + co] = bs;
    red[(wave * 2 + 1) * CO + co] = bq;
  }
  __syncthreads();
  for (int co = tid; co < Cout; co += NT) {
    double sm = 0.0, sq = 0.0;
    for (int wv = 0; wv < TR; ++wv) {
      sm += red[(wv * 2 + 0) * CO + co];
      sq += red[(wv * 2 + 1) * CO + co];
    }
    stats[(int64_t)blockIdx.x * 2 * Cout + co] = sm;
    stats[(int64_t)blockIdx.x * 2 * Cout + Cout + co] = sq;
  }
}

// Persistent launcher (conv_x6_launch routes here); returns 1 if (CI, COP)
// has no instantiation.  x16 / y16 (bf16 configuration, NP = 1 only): the
// input (dy of a data gradient, act(x) source of a forward) / the forward
// output in bf16 storage.  lay: CL_X (input channel-last) | CL_Y (output
// channel-last).
template <int CIV, int COV, bool DG, int NTV, int TRV>
static void x6p_go(dim3 g, hipStream_t s, bool b16, bool x16, bool y16, int lay, const float* x,
                   const float* w, const float* bias, const float* sc, const float* sh, float* y,
                   double* stats, int N, int Cout, int H, int W, const Bnr& bnr) {
  cl_dispatch(lay, [&](auto xl, auto yl) {
    constexpr bool XL = decltype(xl)::value, YL = decltype(yl)::value;
#define AINP_X6PK(NPV, GV, YV)                                                                   \
  hipLaunchKernelGGL((conv3x3_x6p_kernel<CIV, COV, DG, NTV, TRV, NPV, GV, YV, XL, YL>), g,       \
                     dim3(NTV), 0, s, x, w, bias, sc, sh, y, stats, N, Cout, H, W, bnr)
    if (!b16) {
      AINP_X6PK(3, false, false);
    } else if constexpr (DG) {
      if (x16) AINP_X6PK(1, true, false);
      else AINP_X6PK(1, false, false);
    } else {
      if (x16 && y16) AINP_X6PK(1, true, true);
      else if (x16) AINP_X6PK(1, true, false);
      else if (y16) AINP_X6PK(1, false, true);
      else AINP_X6PK(1, false, false);
    }
#undef AINP_X6PK
  });
}

template <bool DG>
static void x6q_go(dim3 g, hipStream_t s, bool b16, bool x16, bool y16, int lay, const float* x,
                   const float* w, const float* bias, const float* sc, const float* sh, float* y,
                   double* stats, int N, int Cout, int H, int W, const Bnr& bnr) {
  const int ycf = (lay & CL_CF) ? 1 : 0;
  cl_dispatch(lay, [&](auto xl, auto yl) {
    constexpr bool XL = decltype(xl)::value, YL = decltype(yl)::value;
#define AINP_X6QK(NPV, GV, YV)                                                                \
  hipLaunchKernelGGL((conv3x3_x6q_kernel<32, DG, NPV, GV, YV, XL, YL>), g, dim3(512), 0, s, x, \
                     w, bias, sc, sh, y, stats, N, Cout, H, W, bnr, ycf)
    if (!b16) {
      AINP_X6QK(3, false, false);
    } else if constexpr (DG) {
      if (x16) AINP_X6QK(1, true, false);
      else AINP_X6QK(1, false, false);
    } else {
      if (x16 && y16) AINP_X6QK(1, true, true);
      else if (x16) AINP_X6QK(1, true, false);
      else if (y16) AINP_X6QK(1, false, true);
      else AINP_X6QK(1, false, false);
    }
#undef AINP_X6QK
  });
}

int conv_x6p_launch(bool dgrad, const float* x, const float* w, const float* bias,
                    const float* sc, const float* sh, float* y, double* stats, int64_t N, int Cin,
                    int Cout, int64_t H, int64_t W, hipStream_t s, int64_t* parts, bool b16,
                    bool x16, bool y16, int lay, const Bnr& bnr) {
  const int cop = Cout <= 32 ? 32 : 64;
  if ((lay & CL_CF) && !(dgrad && Cin == 32 && Cout == 16 && !(lay & CL_Y)))
    return 2;   // [C][H][N][W] dx: the 32 -> 16 data gradient (x6q) only
  // bf16 channel-last forward with bf16 source and output: the LDS-DMA
  // kernel, on x6p's grid (the same BatchNorm partial rows, bit-identical)
  if (!dgrad && b16 && x16 && y16 && lay == (CL_X | CL_Y) && Cout % 4 == 0 && conv16_dma() &&
      ((Cin == 32 && cop == 64) || (Cin == 16 && cop == 32))) {
    const int g = (Cin == 32 ? 256 : 512) * conv_x6_occ16();
    *parts = g;
    const uint16_t* x16p = reinterpret_cast<const uint16_t*>(x);
    uint16_t* y16p = reinterpret_cast<uint16_t*>(y);
    // AINP_CONV16_RING=3: three halo buffers (exact-count buffer stores), A/B;
    // default two (r06n / r06o: equal or faster, the DMA is not the limit)
    static const int ring = [] {
      const char* e = getenv("AINP_CONV16_RING");
      return (e && e[0] == '3') ? 3 : 2;
    }();
    if (N * cdiv(H, cdf::TR) * cdiv(W, cdf::TC) >= ((int64_t)1 << 31))
      return record_msg("conv3x3_fwd_b16dma: too many tiles");
    const bool r3 = ring == 3 && N * H * W * Cout * 2 < ((int64_t)1 << 31) - 64;
#define AINP_CF(CIV, COV, NTV, KR)                                                             \
  do {                                                                                         \
    if (r3)                                                                                    \
      hipLaunchKernelGGL((conv3x3_fwd_b16dma_kernel<CIV, COV, NTV, 3, KR>), dim3(g), dim3(NTV), \
                         0, s, x16p, w, bias, sc, sh, y16p, stats, (int)N, Cout, (int)H,        \
                         (int)W);                                                               \
    else                                                                                       \
      hipLaunchKernelGGL((conv3x3_fwd_b16dma_kernel<CIV, COV, NTV, 2, KR>), dim3(g), dim3(NTV), \
                         0, s, x16p, w, bias, sc, sh, y16p, stats, (int)N, Cout, (int)H,        \
                         (int)W);                                                               \
  } while (0)
    if (Cin == 32) AINP_CF(32, 64, 1024, 0);
    else AINP_CF(16, 32, 512, -1);
#undef AINP_CF
    return check_launch("conv3x3_fwd_b16dma");
  }
  // two workgroups per CU where the LDS allows it (one 16-channel chunk)
#define AINP_X6P(CIV, COV, DG, G, NTV, TRV)                                                      \
  if (dgrad == DG && Cin == CIV && cop == COV) {                                                 \
    const int g2 = b16 ? (G) * conv_x6_occ16() : (G);                                            \
    x6p_go<CIV, COV, DG, NTV, TRV>(dim3(g2), s, b16, x16, y16, lay, x, w, bias, sc, sh, y,      \
                                   stats, (int)N, Cout, (int)H, (int)W, bnr);                    \
    *parts = g2;                                                                                 \
    return check_launch("conv3x3_x6p");                                                          \
  }
  AINP_X6P(32, 64, false, 256, 1024, 8)
  AINP_X6P(16, 32, false, 512, 512, 8) AINP_X6P(16, 32, true, 512, 512, 8)
  if (Cin == 32 && Cout == 16) {   // two workgroups per CU (65 KB of LDS; bf16: more)
    const int gq = b16 ? 512 * conv_x6_occ16() : 512;
    if (dgrad)
      x6q_go<true>(dim3(gq), s, b16, x16, y16, lay, x, w, bias, sc, sh, y, stats, (int)N, Cout,
                   (int)H, (int)W, bnr);
    else
      x6q_go<false>(dim3(gq), s, b16, x16, y16, lay, x, w, bias, sc, sh, y, stats, (int)N, Cout,
                    (int)H, (int)W, bnr);
    *parts = gq;
    return check_launch("conv3x3_x6q");
  }
#undef AINP_X6P
  return 1;
}

// conv3x3_wgrad_x6s tile rows, per plane count (AINP_X6S_FT1 for the bf16
// configuration's NP = 1: 4, 8 or 16; AINP_X6S_FT3 for NP = 3: 4 or 8).
// Defaults from profiles/r06_x6s_ft_lab.txt (standalone, C2 shape): NP = 3
// 8-row tiles 0.304 -> 0.262 ms (16 -> 32) and 0.338 -> 0.293 ms (32 -> 16),
// one workgroup per CU (111 KB of LDS); C2 14.16 -> 14.07 ms/step on one box
// (profiles/r06_ab_x6s_ft.txt).  NP = 1: 4 rows stay fastest (0.166 ms vs
// 0.210 / 0.201).
static int x6s_ft(int np) {
  auto rd = [](const char* name, int def) {
    const char* e = getenv(name);
    const int v = e ? atoi(e) : def;
    return v == 8 || v == 16 ? v : 4;
  };
  return np == 1 ? rd("AINP_X6S_FT1", 4) : rd("AINP_X6S_FT3", 8);   // read per launch (tests)
}

// the split-bf16 weight-gradient kernels of one pass (NP planes, storage
// G16 / XG16) for the (cp, Cout) pair; returns 1 if it has none
template <int NP, bool G16, bool XG16>
static int wgrad_x6_go(const float* x, const float* sc, const float* sh, const float* dy,
                       float* partial, int64_t N, int Cin, int Cout, int64_t H, int64_t W,
                       int ci0, int cp, int grid, hipStream_t s, int lay) {
  int rc = 1;
  const int ft = x6s_ft(NP);
  auto go = [&](auto xlc, auto glc) {
    constexpr bool XL = decltype(xlc)::value, GL = decltype(glc)::value;
    if ((cp == 32 && Cout == 16) || (cp == 16 && Cout == 32)) {
#define AINP_X6S(CPV, COV, FTV)                                                                  \
  hipLaunchKernelGGL((conv3x3_wgrad_x6s<CPV, COV, NP, G16, XG16, XL, GL, FTV>), dim3(grid),     \
                     dim3(384), 0, s, x, sc, sh, dy, partial, (int)N, Cin, (int)H, (int)W, ci0)
      if (cp == 32) {
        if (NP == 1 && ft == 16) AINP_X6S(32, 16, NP == 1 ? 16 : 8);
        else if (ft == 8) AINP_X6S(32, 16, 8);
        else AINP_X6S(32, 16, 4);
      } else {
        if (NP == 1 && ft == 16) AINP_X6S(16, 32, NP == 1 ? 16 : 8);
        else if (ft == 8) AINP_X6S(16, 32, 8);
        else AINP_X6S(16, 32, 4);
      }
#undef AINP_X6S
      rc = check_launch("conv3x3_wgrad_x6s");
    } else if (cp == 32 && Cout == 64) {
      hipLaunchKernelGGL((conv3x3_wgrad_x6<64, NP, G16, XG16, XL, GL>), dim3(grid), dim3(384), 0,
                         s, x, sc, sh, dy, partial, (int)N, Cin, (int)H, (int)W, ci0);
      rc = check_launch("conv3x3_wgrad_x6");
    }
  };
  const bool xl = (lay & CL_X) != 0, gl = (lay & CL_G) != 0;
  if (xl && gl) go(std::true_type{}, std::true_type{});
  else if (xl) go(std::true_type{}, std::false_type{});
  else if (gl) go(std::false_type{}, std::true_type{});
  else go(std::false_type{}, std::false_type{});
  return rc;
}

// Launch the split-bf16 weight gradient of one 32-channel pass if Cout has an
// instantiation; returns 1 if not handled.  grid = persistent workgroups.
// g16 / x16 (bf16 configuration): dy / act(x)'s source in bf16 storage.
// lay: CL_X (act(x) source channel-last) | CL_G (dy channel-last).
int conv_wgrad_x6_launch(const float* x, const float* sc, const float* sh, const float* dy,
                         float* partial, int64_t N, int Cin, int Cout, int64_t H, int64_t W,
                         int ci0, int cp, int grid, hipStream_t s, bool b16, bool g16, bool x16,
                         int lay, int* grid_used) {
  *grid_used = grid;
  // bf16 channel-last 32 -> 64 (the bf16 configuration's encoder conv): the
  // LDS-DMA kernel, one workgroup per CU (its slabs: grid_used)
  if (b16 && g16 && x16 && lay == (CL_X | CL_G) && Cin == 32 && cp == 32 && ci0 == 0 &&
      Cout == 64 && wgrad16_dma()) {
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int g = ncu >= 16 ? ncu / 16 * 16 : 16;   // a multiple of WG_GROUPS (16)
    if (N * ((H + 3) / 4) * ((W + wdm::TT - 1) / wdm::TT) >= ((int64_t)1 << 31))
      return record_msg("conv3x3_wgrad_b16dma: too many tiles");
    *grid_used = g;
    static const int var = [] {
      const char* e = getenv("AINP_WDM_VARIANT");
      return e ? atoi(e) : 0;
    }();
    static const int dbg = [] {
      const char* e = getenv("AINP_WDM_DBG");
      return e ? atoi(e) : 0;
    }();
#define AINP_WDM(FTV, NSV)                                                                   \
  hipLaunchKernelGGL((conv3x3_wgrad_b16dma_kernel<FTV, NSV>), dim3(g), dim3(wdm::NT), 0, s, \
                     reinterpret_cast<const uint16_t*>(x), sc, sh,                          \
                     reinterpret_cast<const uint16_t*>(dy), partial, (int)N, (int)H, (int)W, dbg)
    // default: 8-row tiles, 2 stages (r06h sweep, standalone at the C3 shape:
    // <8,2> 174 us, <4,4> 218, <4,5> 230, <4,6> 232; <8,3> needs more than
    // 256 VGPRs with the fragment double buffer and spills)
    switch (var) {
      case 1: AINP_WDM(4, 5); break;
      case 2: AINP_WDM(4, 6); break;
      case 3: AINP_WDM(4, 4); break;
      default: AINP_WDM(8, 2); break;
    }
#undef AINP_WDM
    return check_launch("conv3x3_wgrad_b16dma");
  }
  if (b16) {
    if (g16 && x16) return wgrad_x6_go<1, true, true>(x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp, grid, s, lay);
    if (g16) return wgrad_x6_go<1, true, false>(x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp, grid, s, lay);
    if (x16) return wgrad_x6_go<1, false, true>(x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp, grid, s, lay);
    return wgrad_x6_go<1, false, false>(x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp, grid, s, lay);
  }
  return wgrad_x6_go<3, false, false>(x, sc, sh, dy, partial, N, Cin, Cout, H, W, ci0, cp, grid, s,
                                      lay);
}

}  // namespace ainp
