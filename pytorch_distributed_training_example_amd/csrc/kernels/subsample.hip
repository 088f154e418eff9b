// Stride-s pixel subsampling of a channels_last tensor and its adjoint, for the ResNet stride-2 1x1
// shortcut run as gather + GEMM (ops/conv.py _Conv1x1StridedFn):
//   gather : xs[n, i, j, :] = x[n, s*i, s*j, :]
//   scatter-add (the gradient): full[n, s*i, s*j, :] += t[n, i, j, :]
// aten's strided copy / strided add_ ran these at ~2-2.5 TB/s (0.8 + 0.4 ms per ResNet-50 step at
// 1024 images/GPU, profiles/r2/steady_resnet50_b1024_ours.md); here one lane moves 16 B per
// iteration, consecutive lanes along the contiguous channel run, a grid-stride loop over
// (output pixel, 8-channel chunk). Not in the reference (LeNet has no strided shortcut).
#include "../common.h"

namespace {

__global__ __launch_bounds__(256) void gather_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ xs, int H,
                                                     int W, int Hs, int Ws, int C8, int s, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(v % C8);
    const int64_t p = v / C8;
    const int j = (int)(p % Ws);
    const int64_t q = p / Ws;
    const int i = (int)(q % Hs);
    const int64_t n = q / Hs;
    const int64_t src = ((n * H + (int64_t)i * s) * W + (int64_t)j * s) * C8 + c8;
    reinterpret_cast<uint4*>(xs)[v] = reinterpret_cast<const uint4*>(x)[src];
  }
}

__global__ __launch_bounds__(256) void scatter_add_kernel(const uint16_t* __restrict__ t, uint16_t* __restrict__ full,
                                                          int H, int W, int Hs, int Ws, int C8, int s, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(v % C8);
    const int64_t p = v / C8;
    const int j = (int)(p % Ws);
    const int64_t q = p / Ws;
    const int i = (int)(q % Hs);
    const int64_t n = q / Hs;
    const int64_t dst = ((n * H + (int64_t)i * s) * W + (int64_t)j * s) * C8 + c8;
    float a[8], b[8];
    pdt::ld8_bf16(full + dst * 8, a);
    pdt::ld8_bf16(t + v * 8, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += b[k];
    pdt::st8_bf16(full + dst * 8, a);
  }
}

inline int grid_for(int64_t nvec) {
  int64_t g = (nvec + 255) / 256;
  return (int)(g > 256 * 8 ? 256 * 8 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

// x [N, H, W, C] -> xs [N, Hs, Ws, C] (bf16, channels_last storage), Hs = (H-1)/s+1; C % 8 == 0.
int pdt_subsample_gather(const uint16_t* x, uint16_t* xs, int N, int H, int W, int C, int s, hipStream_t st) {
  if (C % 8 != 0 || s < 1 || N < 1) return -1;
  const int Hs = (H - 1) / s + 1, Ws = (W - 1) / s + 1;
  const int64_t nvec = (int64_t)N * Hs * Ws * (C / 8);
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(nvec)), dim3(256), 0, st, x, xs, H, W, Hs, Ws, C / 8, s, nvec);
  return 0;
}

// full[N, H, W, C] += scatter of t [N, Hs, Ws, C] at the stride-s pixels.
int pdt_subsample_scatter_add(const uint16_t* t, uint16_t* full, int N, int H, int W, int C, int s, hipStream_t st) {
  if (C % 8 != 0 || s < 1 || N < 1) return -1;
  const int Hs = (H - 1) / s + 1, Ws = (W - 1) / s + 1;
  const int64_t nvec = (int64_t)N * Hs * Ws * (C / 8);
  hipLaunchKernelGGL(scatter_add_kernel, dim3(grid_for(nvec)), dim3(256), 0, st, t, full, H, W, Hs, Ws, C / 8, s,
                     nvec);
  return 0;
}

}  // extern "C"
