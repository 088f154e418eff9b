// Standalone correctness + timing harness for csrc/kernels/conv3x3_wgrad.hip (no torch):
// random bf16 NHWC x / dy, a naive fp32 reference weight gradient, max relative error, and time
// per call at the ResNet-50 stride-1 3x3 shapes for each tuning variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/convbench/wgrad3x3_bench.cpp -o /tmp/wgb
#include "../../pytorch_distributed_training_example_amd/csrc/kernels/conv3x3_wgrad.hip"

#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_kernel(uint16_t* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float v = ((h & 0xffff) / 65535.f - 0.5f) * 2.f * scale;
    p[i] = __builtin_bit_cast(uint16_t, (__bf16)v);
  }
}

__global__ void ref_wgrad_kernel(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int Ci, int Co) {
  const int64_t total = (int64_t)Co * 9 * Ci;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Ci), t = (int)((i / Ci) % 9), co = (int)(i / (9 * Ci));
    const int kh = t / 3, kw = t % 3;
    float acc = 0.f;
    for (int n = 0; n < N; ++n)
      for (int oh = 0; oh < H; ++oh)
        for (int ow = 0; ow < W; ++ow) {
          const int ih = oh + kh - 1, iw = ow + kw - 1;
          if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
          acc += bf2f(dy[(((int64_t)n * H + oh) * W + ow) * Co + co]) * bf2f(x[(((int64_t)n * H + ih) * W + iw) * Ci + ci]);
        }
    dw[i] = acc;  // [co][t][ci]
  }
}

static float bfh(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

static bool check(int N, int H, int W, int Ci, int Co) {
  const int64_t nx = (int64_t)N * H * W * Ci, ny = (int64_t)N * H * W * Co, nw = (int64_t)Co * 9 * Ci;
  uint16_t *x, *dy, *dw; float *ref, *ws;
  CK(hipMalloc(&x, nx * 2)); CK(hipMalloc(&dy, ny * 2)); CK(hipMalloc(&dw, nw * 2)); CK(hipMalloc(&ref, nw * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, x, nx, 1u, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, dy, ny, 7u, 1.f);
  hipLaunchKernelGGL(ref_wgrad_kernel, dim3(1024), dim3(256), 0, 0, x, dy, ref, N, H, W, Ci, Co);
  int ns = 0;
  const int64_t wsf = pdt_conv3x3_wgrad_ws_floats(N, H, W, Ci, Co, &ns);
  if (wsf == 0) { printf("unsupported %d %d %d %d %d\n", N, H, W, Ci, Co); return false; }
  CK(hipMalloc(&ws, wsf * 4));
  const int rc = pdt_conv3x3s1_wgrad(x, dy, dw, ws, N, H, W, Ci, Co, 0);
  CK(hipDeviceSynchronize());
  std::vector<uint16_t> h(nw); std::vector<float> r(nw);
  CK(hipMemcpy(h.data(), dw, nw * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(r.data(), ref, nw * 4, hipMemcpyDeviceToHost));
  double num = 0, den = 0, mx = 0;
  for (int64_t i = 0; i < nw; ++i) { const double d = bfh(h[i]) - r[i]; num += d * d; den += (double)r[i] * r[i]; mx = fmax(mx, fabs(d)); }
  const double rel = sqrt(num / (den + 1e-30));
  printf("check N=%d H=%d W=%d Ci=%d Co=%d rc=%d nsplit=%d rel=%.2e maxabs=%.3e %s\n", N, H, W, Ci, Co, rc, ns, rel, mx,
         rel < 1e-2 && rc == 0 ? "OK" : "FAIL");
  CK(hipFree(x)); CK(hipFree(dy)); CK(hipFree(dw)); CK(hipFree(ref)); CK(hipFree(ws));
  return rel < 1e-2 && rc == 0;
}

static void timeit(int N, int H, int W, int Ci, int Co, int iters) {
  const int64_t nx = (int64_t)N * H * W * Ci, ny = (int64_t)N * H * W * Co, nw = (int64_t)Co * 9 * Ci;
  uint16_t *x, *dy, *dw; float* ws;
  CK(hipMalloc(&x, nx * 2)); CK(hipMalloc(&dy, ny * 2)); CK(hipMalloc(&dw, nw * 2));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, x, nx, 1u, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, dy, ny, 7u, 1.f);
  const int cots[2] = {64, 128};
  const int wgs[2] = {256, 512};
  for (int ci = 0; ci < 2; ++ci) {
    if (Co % cots[ci]) continue;
    for (int wi = 0; wi < 2; ++wi) {
      pdt_conv3x3_wgrad_tune(wgs[wi], cots[ci]);
      int ns = 0;
      const int64_t wsf = pdt_conv3x3_wgrad_ws_floats(N, H, W, Ci, Co, &ns);
      CK(hipMalloc(&ws, wsf * 4));
      hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
      for (int i = 0; i < 3; ++i) pdt_conv3x3s1_wgrad(x, dy, dw, ws, N, H, W, Ci, Co, 0);
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) pdt_conv3x3s1_wgrad(x, dy, dw, ws, N, H, W, Ci, Co, 0);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / iters;
      const double tf = 2.0 * N * H * W * (double)Co * 9 * Ci / (us * 1e-6) / 1e12;
      printf("time N=%d H=%d W=%d Ci=%d Co=%d co_t=%d wgs=%d nsplit=%d: %.1f us  %.0f TF/s\n", N, H, W, Ci, Co, cots[ci],
             wgs[wi], ns, us, tf);
      CK(hipFree(ws));
    }
  }
  pdt_conv3x3_wgrad_tune(0, 0);
  CK(hipFree(x)); CK(hipFree(dy)); CK(hipFree(dw));
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  bool ok = true;
  ok &= check(2, 13, 11, 64, 64);
  ok &= check(3, 56, 56, 64, 64);
  ok &= check(2, 28, 28, 128, 128);
  ok &= check(4, 14, 14, 256, 256);
  ok &= check(9, 7, 7, 512, 512);
  ok &= check(2, 9, 5, 64, 192);
  ok &= check(1, 3, 3, 128, 64);
  ok &= check(5, 7, 7, 128, 256);
  if (!ok) { printf("CHECK FAILED\n"); return 1; }
  if (getenv("PROBE")) {  // 1 = staging only, 2 = MFMA only
    pdt_conv3x3_wgrad_probe(atoi(getenv("PROBE")));
    printf("PROBE %s\n", getenv("PROBE"));
  }
  if (getenv("ONLY")) {  // one layer (1..4), default tuning, for counter collection
    const int l = atoi(getenv("ONLY"));
    const int hw[5] = {0, 56, 28, 14, 7}, c[5] = {0, 64, 128, 256, 512};
    const int64_t n = (int64_t)B * hw[l] * hw[l];
    uint16_t *x, *dy, *dw; float* ws; int ns = 0;
    CK(hipMalloc(&x, n * c[l] * 2)); CK(hipMalloc(&dy, n * c[l] * 2)); CK(hipMalloc(&dw, (int64_t)c[l] * 9 * c[l] * 2));
    CK(hipMalloc(&ws, pdt_conv3x3_wgrad_ws_floats(B, hw[l], hw[l], c[l], c[l], &ns) * 4));
    for (int i = 0; i < 5; ++i) pdt_conv3x3s1_wgrad(x, dy, dw, ws, B, hw[l], hw[l], c[l], c[l], 0);
    CK(hipDeviceSynchronize());
    printf("ONLY layer %d done\n", l);
    return 0;
  }
  timeit(B, 56, 56, 64, 64, 20);
  timeit(B, 28, 28, 128, 128, 20);
  timeit(B, 14, 14, 256, 256, 20);
  timeit(B, 7, 7, 512, 512, 20);
  return 0;
}
