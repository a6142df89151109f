// loss.hip — fused CNNBLSTM reconstruction loss and small reductions.
#include "common.h"

namespace ainp {

// L = sum |10^y*m - |target|*m|  (models/CNNBLSTM/train.py:70,104:
// nn.L1Loss(reduction='sum') on (10 ** y) * mask vs abs(target) * mask)
// dL/dy = sign(d) * m * 10^y * ln(10), sign(0) = 0 as in torch's L1 backward.
// Deterministic: each workgroup writes its fp64 partial to partial[blockIdx.x]
// (fixed grid-stride order, fixed wave/LDS combine); l1_sum_partials_kernel
// adds the partials in a fixed order.  No atomics: the loss is bit-reproducible.
__global__ __launch_bounds__(256) void l1_pow10_kernel(
    const float* __restrict__ y, const float* __restrict__ mask,
    const float2* __restrict__ target, int64_t n, double* __restrict__ partial,
    float* __restrict__ dy, float grad_scale) {
  const float LN10 = 2.302585092994046f;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float m = mask[i];
    const float p = powf(10.f, y[i]);
    const float2 t = target[i];
    const float a = p * m;
    const float b = hypotf(t.x, t.y) * m;
    const float d = a - b;
    acc += (double)fabsf(d);
    if (dy) {
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      dy[i] = grad_scale * (sg * m) * (p * LN10);
    }
  }
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = sum of partial[0..np) in a fixed order (one workgroup of 256).
__global__ __launch_bounds__(256) void l1_sum_partials_kernel(const double* __restrict__ partial,
                                                              int64_t np, double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < np; i += 256) acc += partial[i];
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

static int64_t l1_grid(int64_t n) {
  int64_t grid = cdiv(n, 256 * 8);
  return grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
}

// out[j] (+)= sum_i x[i*ld + j]; one thread per column, rows split over
// blockIdx.y slabs reduced with atomics when more than one slab.
__global__ void colsum_kernel(const float* __restrict__ x, int64_t rows,
                              int64_t cols, int64_t ld, float* __restrict__ out,
                              int64_t rows_per) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  const int64_t r0 = blockIdx.y * rows_per;
  int64_t r1 = r0 + rows_per;
  if (r1 > rows) r1 = rows;
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += x[r * ld + j];
  atomicAdd(&out[j], s);
}

// partial[s*cols + j] = sum of x[r*ld + j] over the rows of slab s, in a fixed
// order (four interleaved partial sums); the slabs are combined by
// sum_slabs_kernel, so the column sums are deterministic.
__global__ void colsum_slabs_kernel(const float* __restrict__ x, int64_t rows, int64_t cols,
                                    int64_t ld, int64_t rows_per, float* __restrict__ partial) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < rows ? r0 + rows_per : rows;
  const float* p = x + j;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int64_t r = r0;
  // 8 rows in flight; the adds keep the 4-accumulator order of the loop below.
  for (; r + 7 < r1; r += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(r + u) * ld];
    a0 += v[0]; a1 += v[1]; a2 += v[2]; a3 += v[3];
    a0 += v[4]; a1 += v[5]; a2 += v[6]; a3 += v[7];
  }
  for (; r + 3 < r1; r += 4) {
    a0 += p[r * ld];
    a1 += p[(r + 1) * ld];
    a2 += p[(r + 2) * ld];
    a3 += p[(r + 3) * ld];
  }
  for (; r < r1; ++r) a0 += p[r * ld];
  partial[(int64_t)blockIdx.y * cols + j] = (a0 + a1) + (a2 + a3);
}

__global__ void zero_kernel(float* p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

__global__ void scale_by_dev_kernel(const float* __restrict__ x,
                                    float* __restrict__ out, int64_t n,
                                    const float* __restrict__ s) {
  const float v = s[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = x[i] * v;
}

// out[i] = sum_s x[s*n + i]  (fixed order: deterministic split-K combine)
__global__ void sum_slabs_kernel(const float* __restrict__ x, int64_t nslabs,
                                 int64_t n, float* __restrict__ out) {
  for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i4 * 4 < n;
       i4 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i4 * 4;
    if (i + 3 < n && (n & 3) == 0) {
      float4 a = *reinterpret_cast<const float4*>(x + i);
      int64_t s = 1;
      // 4 slab loads in flight per iteration; the adds keep slab order.
      for (; s + 3 < nslabs; s += 4) {
        float4 b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          b[u] = *reinterpret_cast<const float4*>(x + (s + u) * n + i);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w;
        }
      }
      for (; s < nslabs; ++s) {
        const float4 b = *reinterpret_cast<const float4*>(x + s * n + i);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      *reinterpret_cast<float4*>(out + i) = a;
    } else {
      for (int64_t e = i; e < i + 4 && e < n; ++e) {
        float a = 0.f;
        for (int64_t s = 0; s < nslabs; ++s) a += x[s * n + e];
        out[e] = a;
      }
    }
  }
}

// sum_slabs for few elements over many slabs (a split-K GEMM with a tiny
// output: the discriminator's first-layer weight gradient, 64 x 17 over 512
// slabs): a workgroup owns SS_E elements, its SS_G slab groups each sum the
// slabs g, g + SS_G, ... in order, and the group partials are added in
// fixed order g = 0 .. SS_G-1 (deterministic; a different order than
// sum_slabs_kernel's, so only taken where that kernel would run a handful of
// workgroups through hundreds of dependent loads).
constexpr int SS_E = 8, SS_G = 32;
__global__ __launch_bounds__(256) void sum_slabs_groups_kernel(const float* __restrict__ x,
                                                               int64_t nslabs, int64_t n,
                                                               float* __restrict__ out) {
  __shared__ float part[SS_G][SS_E];
  const int e = threadIdx.x % SS_E, g = threadIdx.x / SS_E;
  const int64_t i = (int64_t)blockIdx.x * SS_E + e;
  float a = 0.f;
  if (i < n) {
    int64_t s = g;
    for (; s + 3 * SS_G < nslabs; s += 4 * SS_G) {
      float b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) b[u] = x[(s + u * SS_G) * n + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) a += b[u];
    }
    for (; s < nslabs; s += SS_G) a += x[s * n + i];
  }
  part[g][e] = a;
  __syncthreads();
  if (g == 0 && i < n) {
    float t = part[0][e];
    for (int q = 1; q < SS_G; ++q) t += part[q][e];
    out[i] = t;
  }
}

// out[r] = sum_b sum_c x[(b*rows + r)*cols + c]; one wave per row.
__global__ __launch_bounds__(256) void rowsum_batched_kernel(
    const float* __restrict__ x, int64_t nb, int64_t rows, int64_t cols,
    float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int64_t b = 0; b < nb; ++b) {
    const float* p = x + (b * rows + r) * cols;
    for (int64_t c = lane; c < cols; c += 64) s += p[c];
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s;
}

}  // namespace ainp

using namespace ainp;

extern "C" int ainp_sum_slabs(const float* x, int64_t nslabs, int64_t n,
                              float* out, void* stream) {
  if (!x || !out || nslabs < 1 || n < 0) return record_msg("ainp_sum_slabs: bad argument");
  if (n == 0) return AINP_OK;
  int64_t grid = cdiv(cdiv(n, 4), 256);
  if (grid > 4096) grid = 4096;
  if (grid < 16 && nslabs >= 64) {
    hipLaunchKernelGGL(sum_slabs_groups_kernel, dim3((unsigned)cdiv(n, SS_E)), dim3(256), 0,
                       as_stream(stream), x, nslabs, n, out);
    return check_launch("sum_slabs_groups");
  }
  hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)grid), dim3(256), 0,
                     as_stream(stream), x, nslabs, n, out);
  return check_launch("sum_slabs");
}

extern "C" int ainp_rowsum_batched(const float* x, int64_t nb, int64_t rows,
                                   int64_t cols, float* out, void* stream) {
  if (!x || !out || nb < 1 || rows < 0 || cols < 1)
    return record_msg("ainp_rowsum_batched: bad argument");
  if (rows == 0) return AINP_OK;
  hipLaunchKernelGGL(rowsum_batched_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256),
                     0, as_stream(stream), x, nb, rows, cols, out);
  return check_launch("rowsum_batched");
}

extern "C" int ainp_scale_by_dev(const float* x, float* out, int64_t n,
                                 const float* scalar, void* stream) {
  if (!x || !out || !scalar || n < 0) return record_msg("ainp_scale_by_dev: bad argument");
  if (n == 0) return AINP_OK;
  int64_t grid = cdiv(n, 256 * 4);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(scale_by_dev_kernel, dim3((unsigned)grid), dim3(256), 0,
                     as_stream(stream), x, out, n, scalar);
  return check_launch("scale_by_dev");
}

extern "C" int64_t ainp_l1_pow10_loss_slots(int64_t n) { return 1 + l1_grid(n); }

extern "C" int ainp_l1_pow10_loss(const float* y, const float* mask,
                                  const float* target, int64_t n, double* loss,
                                  float* dy, float grad_scale, void* stream) {
  if (!loss || n < 0 || (n > 0 && (!y || !mask || !target)))
    return record_msg("ainp_l1_pow10_loss: bad argument");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    hipLaunchKernelGGL(l1_sum_partials_kernel, dim3(1), dim3(256), 0, s, loss + 1, 0, loss);
    return check_launch("l1_pow10_loss");
  }
  const int64_t grid = l1_grid(n);
  hipLaunchKernelGGL(l1_pow10_kernel, dim3((unsigned)grid), dim3(256), 0, s, y, mask,
                     reinterpret_cast<const float2*>(target), n, loss + 1, dy, grad_scale);
  hipLaunchKernelGGL(l1_sum_partials_kernel, dim3(1), dim3(256), 0, s, loss + 1, grid, loss);
  return check_launch("l1_pow10_loss");
}

extern "C" int ainp_colsum(const float* x, int64_t rows, int64_t cols,
                           int64_t ld, float* out, int accumulate,
                           void* stream) {
  if (!x || !out || rows < 0 || cols < 0 || ld < cols)
    return record_msg("ainp_colsum: bad argument");
  hipStream_t s = as_stream(stream);
  if (!accumulate && cols > 0)
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)cdiv(cols, 256)), dim3(256),
                       0, s, out, cols);
  if (rows == 0 || cols == 0) return check_launch("colsum");
  const int64_t rows_per = 128;
  dim3 grid((unsigned)cdiv(cols, 256), (unsigned)cdiv(rows, rows_per));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, s, x, rows, cols, ld,
                     out, rows_per);
  return check_launch("colsum");
}

extern "C" int ainp_colsum_slabs(const float* x, int64_t rows, int64_t cols, int64_t ld,
                                 int64_t nslabs, float* partial, void* stream) {
  if (!x || !partial || rows < 0 || cols < 1 || ld < cols || nslabs < 1 || nslabs > 65535)
    return record_msg("ainp_colsum_slabs: bad argument");
  const int64_t rows_per = cdiv(rows, nslabs);
  dim3 grid((unsigned)cdiv(cols, 256), (unsigned)nslabs);
  hipLaunchKernelGGL(colsum_slabs_kernel, grid, dim3(256), 0, as_stream(stream), x, rows, cols,
                     ld, rows_per, partial);
  return check_launch("colsum_slabs");
}
