// Bias + GELU epilogue (forward/backward) for gfx950 transformer MLPs.
//
// Forward: y = gelu(x + bias) over [N, D] (bf16/fp32), erf form (ViT) or tanh form (GPT-2
// "gelu_new"); the pre-activation is NOT stored — backward recomputes it from x + bias.
// Backward: dx = dy * gelu'(x + bias); dbias accumulated per workgroup (column partials,
// fixed order) and reduced by a small finalize kernel.
#include "../common.h"

using namespace pdt;

namespace {

__device__ __forceinline__ float gelu_f(float v, int tanh_form) {
  if (tanh_form) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float t = tanhf(k0 * (v + k1 * v * v * v));
    return 0.5f * v * (1.f + t);
  }
  return 0.5f * v * (1.f + erff(v * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_grad(float v, int tanh_form) {
  if (tanh_form) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float u = k0 * (v + k1 * v * v * v);
    const float t = tanhf(u);
    const float du = k0 * (1.f + 3.f * k1 * v * v);
    return 0.5f * (1.f + t) + 0.5f * v * (1.f - t * t) * du;
  }
  const float cdf = 0.5f * (1.f + erff(v * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * v * v);
  return cdf + v * pdf;
}

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
    for (int j = 0; j < 4; ++j) v[j] = gelu_f(v[j] + b[j], tanh_form);
    Vec4<T>::st(y, i * 4, v);
  }
}

// One workgroup per row block; each lane owns 4 columns and walks rows.
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ bias, T* __restrict__ dx,
                                                            float* __restrict__ part, int64_t N, int D,
                                                            int rows_per_block, int tanh_form) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  for (int c = threadIdx.x * 4; c < D; c += 1024) {
    float b[4], acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) Vec4<float>::ld(bias, c, b);
    else b[0] = b[1] = b[2] = b[3] = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      float g[4], v[4];
      Vec4<T>::ld(dy, r * D + c, g);
      Vec4<T>::ld(x, r * D + c, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) { g[j] *= gelu_grad(v[j] + b[j], tanh_form); acc[j] += g[j]; }
      Vec4<T>::st(dx, r * D + c, g);
    }
    if (part) Vec4<float>::st(part, (int64_t)blockIdx.x * D + c, acc);
  }
}

__global__ __launch_bounds__(256) void colsum_finalize_kernel(const float* __restrict__ part, int nblk, int D,
                                                              float* __restrict__ out) {
  __shared__ float red[16][17];  // 16 columns x 16 row-groups (fixed order)
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
    out[c] = s;
  }
}

inline int gelu_bwd_blocks(int64_t N, int& rpb) {
  int64_t nblk = (N + 31) / 32;
  if (nblk > 256) nblk = 256;
  if (nblk < 1) nblk = 1;
  rpb = (int)((N + nblk - 1) / nblk);
  return (int)((N + rpb - 1) / rpb);
}

}  // namespace

extern "C" {

int64_t pdt_gelu_workspace_floats(int64_t N, int D) {
  int rpb;
  return (int64_t)gelu_bwd_blocks(N, rpb) * D;
}

int pdt_bias_gelu_fwd(const void* x, int dtype, const float* bias, void* y, int64_t N, int D, int tanh_form,
                      hipStream_t s) {
  if (D % 4 != 0) return -1;
  const int64_t nvec = N * D / 4;
  if (nvec == 0) return 0;
  int64_t grid = (nvec + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (dtype == 0)
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, bias, (float*)y,
                       nvec, D, tanh_form);
  else
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)x, bias,
                       (uint16_t*)y, nvec, D, tanh_form);
  return 0;
}

int pdt_bias_gelu_bwd(const void* dy, const void* x, int dtype, const float* bias, void* dx, float* dbias,
                      int64_t N, int D, int tanh_form, float* ws, hipStream_t s) {
  if (D % 4 != 0) return -1;
  if (N == 0) return 0;
  int rpb;
  const int nblk = gelu_bwd_blocks(N, rpb);
  float* part = dbias ? ws : nullptr;
  if (dtype == 0)
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<float>, dim3(nblk), dim3(256), 0, s, (const float*)dy, (const float*)x,
                       bias, (float*)dx, part, N, D, rpb, tanh_form);
  else
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<uint16_t>, dim3(nblk), dim3(256), 0, s, (const uint16_t*)dy,
                       (const uint16_t*)x, bias, (uint16_t*)dx, part, N, D, rpb, tanh_form);
  if (dbias)
    hipLaunchKernelGGL(colsum_finalize_kernel, dim3((D + 15) / 16), dim3(256), 0, s, ws, nblk, D, dbias);
  return 0;
}

}  // extern "C"
