// Bias + GELU epilogue (forward/backward) for gfx950 transformer MLPs.
//
// Forward: y = gelu(x + bias) over [N, D] (bf16/fp32), erf form (ViT) or tanh form (GPT-2
// "gelu_new"); the pre-activation is NOT stored — backward recomputes it from x + bias.
// Backward: dx = dy * gelu'(x + bias); dbias accumulated per workgroup (column partials,
// fixed order) and reduced by a small finalize kernel. The same column-strip kernel without the
// GELU part is the bias gradient of every Linear layer (pdt_colsum, ops/linear.py).
#include "../common.h"
#include "../gelu_math.h"

using namespace pdt;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const T* __restrict__ x, const float* __restrict__ bias,
                                                            T* __restrict__ y, int64_t nvec, int D, int tanh_form) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c = (int)((i * 4) % D);
    float v[4], b[4];
    Vec4<T>::ld(x, i * 4, v);
    if (bias) Vec4<float>::ld(bias, c, b);
    else b[0] = b[1] = b[2] = b[3] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const gf2 r = gelu2(gf2{v[j] + b[j], v[j + 1] + b[j + 1]}, tanh_form);
      v[j] = r.x;
      v[j + 1] = r.y;
    }
    Vec4<T>::st(y, i * 4, v);
  }
}

// 8 consecutive elements <-> 8 floats (16 B for bf16, 2 x 16 B for fp32).
template <typename T> struct Vec8;
template <> struct Vec8<uint16_t> {
  __device__ __forceinline__ static void ld(const uint16_t* p, float (&v)[8]) { ld8_bf16(p, v); }
  __device__ __forceinline__ static void st(uint16_t* p, const float (&v)[8]) { st8_bf16(p, v); }
};
template <> struct Vec8<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// Column-strip kernel for [N, D] row-major tensors (D % 8 == 0):
//   blockIdx.x = 512-column strip (a wave covers it with 8 columns per lane, 16-byte accesses),
//   blockIdx.y = row chunk; the 4 waves of a workgroup take interleaved rows of the chunk, two
//   rows in flight per wave, and combine their column sums through LDS into one partial row.
// GELU=true : dx = dy * gelu'(x + bias) is written and dx is column-summed (bias gradient).
// GELU=false: dy is only column-summed (a Linear layer's bias gradient).
// ~2048 workgroups (8 waves/CU) keep enough loads in flight to stream at HBM rate; the
// per-chunk partials (nchunk x D fp32) are reduced in a fixed order by colsum_finalize.
constexpr int kStrip = 512;
// 8 bias values at column c: fp32, or the bf16 parameter itself (bb: a bf16 model's bias needs no fp32 copy — the
// cast and its backward were two aten kernels per MLP per step)
__device__ __forceinline__ void ld_bias8(const void* bias, int bb, int c, float (&b)[8]) {
  if (bb) {
    const uint4 q = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(bias) + c);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      b[2 * k] = __uint_as_float(w[k] << 16);
      b[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
  } else {
    Vec4<float>::ld(reinterpret_cast<const float*>(bias), c, *reinterpret_cast<float(*)[4]>(b));
    Vec4<float>::ld(reinterpret_cast<const float*>(bias), c + 4, *reinterpret_cast<float(*)[4]>(b + 4));
  }
}

template <typename T, bool GELU>
__global__ __launch_bounds__(256) void strip_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                    const void* __restrict__ bias, T* __restrict__ dx,
                                                    float* __restrict__ part, int64_t N, int D, int rows_per_chunk,
                                                    int tanh_form, int bb) {
  __shared__ float red[4][kStrip + 4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * kStrip + lane * 8;
  const bool valid = c < D;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(N, r0 + rows_per_chunk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (valid) {
    if (GELU && bias) ld_bias8(bias, bb, c, b);
    int64_t r = r0 + wv;
    for (; r + 4 < r1; r += 8) {  // two rows in flight
      float g0[8], g1[8];
      Vec8<T>::ld(dy + r * D + c, g0);
      Vec8<T>::ld(dy + (r + 4) * D + c, g1);
      if (GELU) {
        float v0[8], v1[8];
        Vec8<T>::ld(x + r * D + c, v0);
        Vec8<T>::ld(x + (r + 4) * D + c, v1);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const gf2 d0 = gf2{g0[j], g0[j + 1]} * gelu_grad2(gf2{v0[j] + b[j], v0[j + 1] + b[j + 1]}, tanh_form);
          const gf2 d1 = gf2{g1[j], g1[j + 1]} * gelu_grad2(gf2{v1[j] + b[j], v1[j + 1] + b[j + 1]}, tanh_form);
          g0[j] = d0.x; g0[j + 1] = d0.y;
          g1[j] = d1.x; g1[j + 1] = d1.y;
        }
        Vec8<T>::st(dx + r * D + c, g0);
        Vec8<T>::st(dx + (r + 4) * D + c, g1);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += g0[j] + g1[j];
    }
    for (; r < r1; r += 4) {
      float g0[8];
      Vec8<T>::ld(dy + r * D + c, g0);
      if (GELU) {
        float v0[8];
        Vec8<T>::ld(x + r * D + c, v0);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const gf2 d0 = gf2{g0[j], g0[j + 1]} * gelu_grad2(gf2{v0[j] + b[j], v0[j + 1] + b[j + 1]}, tanh_form);
          g0[j] = d0.x; g0[j + 1] = d0.y;
        }
        Vec8<T>::st(dx + r * D + c, g0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += g0[j];
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wv][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int q = threadIdx.x; q < kStrip; q += 256) {
    const int cc = blockIdx.x * kStrip + q;
    if (cc < D) part[(int64_t)blockIdx.y * D + cc] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
  }
}

// Forward over the same strip mapping (no per-element div/mod for the bias column, 16-byte
// accesses, two rows in flight per wave).
template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_strip_kernel(const T* __restrict__ x, const void* __restrict__ bias,
                                                             T* __restrict__ y, int64_t N, int D, int rows_per_chunk,
                                                             int tanh_form, int bb) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * kStrip + lane * 8;
  if (c >= D) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(N, r0 + rows_per_chunk);
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) ld_bias8(bias, bb, c, b);
  int64_t r = r0 + wv;
  for (; r + 4 < r1; r += 8) {
    float v0[8], v1[8];
    Vec8<T>::ld(x + r * D + c, v0);
    Vec8<T>::ld(x + (r + 4) * D + c, v1);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const gf2 q0 = gelu2(gf2{v0[j] + b[j], v0[j + 1] + b[j + 1]}, tanh_form);
      const gf2 q1 = gelu2(gf2{v1[j] + b[j], v1[j + 1] + b[j + 1]}, tanh_form);
      v0[j] = q0.x; v0[j + 1] = q0.y;
      v1[j] = q1.x; v1[j + 1] = q1.y;
    }
    Vec8<T>::st(y + r * D + c, v0);
    Vec8<T>::st(y + (r + 4) * D + c, v1);
  }
  for (; r < r1; r += 4) {
    float v0[8];
    Vec8<T>::ld(x + r * D + c, v0);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const gf2 q0 = gelu2(gf2{v0[j] + b[j], v0[j + 1] + b[j + 1]}, tanh_form);
      v0[j] = q0.x; v0[j + 1] = q0.y;
    }
    Vec8<T>::st(y + r * D + c, v0);
  }
}

// Fixed-order column sums of the per-chunk partials: 16 columns x 16 chunk-groups per workgroup.
template <typename TO>
__global__ __launch_bounds__(256) void colsum_finalize_kernel(const float* __restrict__ part, int nblk, int D,
                                                              TO* __restrict__ out) {
  __shared__ float red[16][17];
  const int grp = threadIdx.x >> 4, cl = threadIdx.x & 15;
  const int c = blockIdx.x * 16 + cl;
  float a = 0.f;
  if (c < D)
    for (int blk = grp; blk < nblk; blk += 16) a += part[(int64_t)blk * D + c];
  red[grp][cl] = a;
  __syncthreads();
  if (grp == 0 && c < D) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += red[q][cl];
    Elt<TO>::st(out, c, s);
  }
}

// Row chunks so that strips x chunks ~ 1024 workgroups (4 waves/CU, 2 rows in flight each) with
// >= 64 rows per chunk: enough bytes in flight to stream at HBM rate while keeping the partial
// slab (and its fixed-order finalize) small.
inline int strip_chunks(int64_t N, int D, int& rpc) {
  if (N <= 0) {
    rpc = 0;
    return 0;
  }
  const int strips = (D + kStrip - 1) / kStrip;
  int64_t nchunk = 1024 / strips;
  const int64_t by_rows = (N + 63) / 64;
  if (nchunk > by_rows) nchunk = by_rows;
  if (nchunk < 1) nchunk = 1;
  rpc = (int)((N + nchunk - 1) / nchunk);
  return (int)((N + rpc - 1) / rpc);
}

template <typename T, bool GELU>
void launch_strip(const T* dy, const T* x, const void* bias, T* dx, float* part, int64_t N, int D, int tanh_form,
                  int& nchunk, hipStream_t s, int bb = 0) {
  int rpc;
  nchunk = strip_chunks(N, D, rpc);
  const dim3 grid((D + kStrip - 1) / kStrip, nchunk);
  hipLaunchKernelGGL((strip_kernel<T, GELU>), grid, dim3(256), 0, s, dy, x, bias, dx, part, N, D, rpc, tanh_form, bb);
}

}  // namespace

extern "C" {

int64_t pdt_gelu_workspace_floats(int64_t N, int D) {
  int rpc;
  return (int64_t)strip_chunks(N, D, rpc) * D;
}

// bias_bf16: bias is bf16 (the strip path, D % 8 == 0, only)
int pdt_bias_gelu_fwd(const void* x, int dtype, const void* bias, void* y, int64_t N, int D, int tanh_form,
                      hipStream_t s, int bias_bf16) {
  if (D % 8 == 0) {
    if (N == 0) return 0;
    int rpc;
    const int nchunk = strip_chunks(N, D, rpc);
    const dim3 grid((D + kStrip - 1) / kStrip, nchunk);
    if (dtype == 0)
      hipLaunchKernelGGL(gelu_fwd_strip_kernel<float>, grid, dim3(256), 0, s, (const float*)x, bias, (float*)y, N, D,
                         rpc, tanh_form, bias_bf16);
    else
      hipLaunchKernelGGL(gelu_fwd_strip_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)x, bias,
                         (uint16_t*)y, N, D, rpc, tanh_form, bias_bf16);
    return 0;
  }
  if (D % 4 != 0 || bias_bf16) return -1;
  const int64_t nvec = N * D / 4;
  if (nvec == 0) return 0;
  int64_t grid = (nvec + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (dtype == 0)
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, (const float*)bias,
                       (float*)y, nvec, D, tanh_form);
  else
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)x,
                       (const float*)bias, (uint16_t*)y, nvec, D, tanh_form);
  return 0;
}

// bias_bf16: bias is bf16 and dbias is written as bf16 too
int pdt_bias_gelu_bwd(const void* dy, const void* x, int dtype, const void* bias, void* dx, void* dbias,
                      int64_t N, int D, int tanh_form, float* ws, hipStream_t s, int bias_bf16) {
  if (D % 8 != 0) return -1;
  if (N == 0) return 0;
  float* part = dbias ? ws : nullptr;
  int nchunk;
  if (dtype == 0)
    launch_strip<float, true>((const float*)dy, (const float*)x, bias, (float*)dx, part, N, D, tanh_form, nchunk, s,
                              bias_bf16);
  else
    launch_strip<uint16_t, true>((const uint16_t*)dy, (const uint16_t*)x, bias, (uint16_t*)dx, part, N, D,
                                 tanh_form, nchunk, s, bias_bf16);
  if (dbias && bias_bf16)
    hipLaunchKernelGGL(colsum_finalize_kernel<uint16_t>, dim3((D + 15) / 16), dim3(256), 0, s, ws, nchunk, D,
                       (uint16_t*)dbias);
  else if (dbias)
    hipLaunchKernelGGL(colsum_finalize_kernel<float>, dim3((D + 15) / 16), dim3(256), 0, s, ws, nchunk, D,
                       (float*)dbias);
  return 0;
}

// Fixed-order sum of nblk per-chunk column partials [nblk, D] fp32 into out (odtype 0 fp32, 1 bf16).
int pdt_colsum_finalize(const float* part, int nblk, int D, void* out, int odtype, hipStream_t s) {
  if (D <= 0) return 0;
  if (odtype == 0)
    hipLaunchKernelGGL(colsum_finalize_kernel<float>, dim3((D + 15) / 16), dim3(256), 0, s, part, nblk, D, (float*)out);
  else
    hipLaunchKernelGGL(colsum_finalize_kernel<uint16_t>, dim3((D + 15) / 16), dim3(256), 0, s, part, nblk, D,
                       (uint16_t*)out);
  return 0;
}

// Column sum of a [N, D] tensor (a Linear layer's bias gradient) into `out` (fp32 or bf16, odtype).
int pdt_colsum(const void* x, int dtype, int64_t N, int D, void* out, int odtype, float* ws, hipStream_t s) {
  if (D % 8 != 0) return -1;
  int nchunk = 1;
  if (N > 0) {
    if (dtype == 0)
      launch_strip<float, false>((const float*)x, nullptr, nullptr, nullptr, ws, N, D, 0, nchunk, s);
    else
      launch_strip<uint16_t, false>((const uint16_t*)x, nullptr, nullptr, nullptr, ws, N, D, 0, nchunk, s);
  } else {
    nchunk = 0;
  }
  if (odtype == 0)
    hipLaunchKernelGGL(colsum_finalize_kernel<float>, dim3((D + 15) / 16), dim3(256), 0, s, ws, nchunk, D,
                       (float*)out);
  else
    hipLaunchKernelGGL(colsum_finalize_kernel<uint16_t>, dim3((D + 15) / 16), dim3(256), 0, s, ws, nchunk, D,
                       (uint16_t*)out);
  return 0;
}

}  // extern "C"
