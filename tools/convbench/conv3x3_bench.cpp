// Standalone correctness + timing harness for csrc/kernels/conv3x3.hip (no torch):
// random bf16 NHWC input / weights, a naive fp32 reference conv kernel, max error, and time per
// call at the ResNet-50 stride-1 shapes (batch 512). build (see tools/gpu_conv3x3.sh):
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/convbench/conv3x3_bench.cpp -o conv3x3_bench
#include "../../pytorch_distributed_training_example_amd/csrc/kernels/conv3x3.hip"

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

// naive reference: one thread per output, fp32 accumulate; w layout [Co][3][3][Ci]
__global__ void ref_kernel(const uint16_t* x, const uint16_t* w, float* y, int N, int H, int W, int Ci, int Co) {
  const int64_t total = (int64_t)N * H * W * Co;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % Co);
    const int64_t m = i / Co;
    const int ow = (int)(m % W), oh = (int)((m / W) % H), n = (int)(m / ((int64_t)H * W));
    float acc = 0.f;
    for (int kh = 0; kh < 3; ++kh)
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = oh + kh - 1, iw = ow + kw - 1;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        const uint16_t* xp = x + (((int64_t)n * H + ih) * W + iw) * Ci;
        const uint16_t* wp = w + ((int64_t)co * 9 + kh * 3 + kw) * Ci;
        for (int c = 0; c < Ci; ++c) acc += bf2f(xp[c]) * bf2f(wp[c]);
      }
    y[i] = acc;
  }
}


static float h_bf(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

static void check(int N, int H, int W, int Ci, int Co, bool dgrad, int iters) {
  const int64_t M = (int64_t)N * H * W;
  uint16_t *x, *w, *wf, *y;
  float* yr;
  CK(hipMalloc(&x, M * Ci * 2)); CK(hipMalloc(&w, (int64_t)Co * 9 * Ci * 2)); CK(hipMalloc(&wf, (int64_t)Co * 9 * Ci * 2));
  CK(hipMalloc(&y, M * Co * 2)); CK(hipMalloc(&yr, M * Co * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, x, M * Ci, 17u, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, w, (int64_t)Co * 9 * Ci, 99u, 0.1f);
  const uint16_t* wk = w;
  int cin = Ci, cout = Co;
  if (dgrad) {  // treat x as dY [N,H,W,Co'=Ci]... the flip maps w[Co][9][Ci] -> wf[Ci][9][Co]
    pdt_conv3x3_flip_weights(w, wf, Co, Ci, 0);
    wk = wf;
    cin = Co; cout = Ci;  // dX = conv(dY (Co channels), wf): here x plays dY with Co channels
  }
  if (dgrad) { CK(hipFree(x)); CK(hipMalloc(&x, M * cin * 2)); hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, x, M * cin, 17u, 1.f);
               CK(hipFree(y)); CK(hipMalloc(&y, M * cout * 2)); CK(hipFree(yr)); CK(hipMalloc(&yr, M * cout * 4)); }
  int rc = pdt_conv3x3s1_fwd(x, wk, y, N, H, W, cin, cout, 0);
  if (rc) { printf("skip (launch rc %d) N=%d H=%d Ci=%d Co=%d\n", rc, N, H, cin, cout); CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(wf)); CK(hipFree(y)); CK(hipFree(yr)); return; }
  if (getenv("NOREF")) {  // profiling: timing only
    CK(hipDeviceSynchronize());
    for (int i = 0; i < iters; ++i) pdt_conv3x3s1_fwd(x, wk, y, N, H, W, cin, cout, 0);
    CK(hipDeviceSynchronize());
    printf("ran %d iters N=%d H=%d Ci=%d Co=%d\n", iters, N, H, cin, cout);
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(wf)); CK(hipFree(y)); CK(hipFree(yr));
    return;
  }
  hipLaunchKernelGGL(ref_kernel, dim3(4096), dim3(256), 0, 0, x, wk, yr, N, H, W, cin, cout);
  CK(hipDeviceSynchronize());
  // check (sampled for big shapes)
  const int64_t tot = M * cout;
  std::vector<uint16_t> hy(tot);
  std::vector<float> hr(tot);
  CK(hipMemcpy(hy.data(), y, tot * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), yr, tot * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  int64_t bad = 0;
  for (int64_t i = 0; i < tot; ++i) {
    const double d = fabs((double)h_bf(hy[i]) - hr[i]);
    maxerr = d > maxerr ? d : maxerr;
    maxref = fabs(hr[i]) > maxref ? fabs(hr[i]) : maxref;
    if (d > 0.02 * fabs(hr[i]) + 0.02) ++bad;
  }
  double us = 0;
  if (iters > 0) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) pdt_conv3x3s1_fwd(x, wk, y, N, H, W, cin, cout, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) pdt_conv3x3s1_fwd(x, wk, y, N, H, W, cin, cout, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    us = ms * 1e3 / iters;
  }
  const double flops = 2.0 * M * cin * cout * 9;
  printf("%s N=%4d H=%3d Ci=%4d Co=%4d  maxerr %.3e (max|ref| %.2f) bad %lld  %8.1f us  %6.0f TF/s\n",
         dgrad ? "dgrad" : "fwd  ", N, H, cin, cout, maxerr, maxref, (long long)bad, us, us > 0 ? flops / us / 1e6 : 0.0);
  fflush(stdout);
  CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(wf)); CK(hipFree(y)); CK(hipFree(yr));
  if (bad && !getenv("PROBE")) exit(2);
}


int main(int argc, char** argv) {
  // (the weight gradient has its own harness: tools/convbench/wgrad3x3_bench.cpp)
  if (getenv("ONLY")) {  // one ResNet-50 layer (1..4), forward, for counter collection
    const int l = atoi(getenv("ONLY"));
    const int hw[5] = {0, 56, 28, 14, 7}, c[5] = {0, 64, 128, 256, 512};
    check(512, hw[l], hw[l], c[l], c[l], false, argc > 1 ? atoi(argv[1]) : 3);
    return 0;
  }
  // correctness: odd sizes, pixel-tile tails, both BN variants, dgrad weights
  check(3, 13, 11, 64, 64, false, 0);
  check(2, 9, 7, 128, 256, false, 0);
  check(3, 13, 11, 64, 128, true, 0);
  check(1, 5, 5, 192, 64, false, 0);
  // ResNet-50 stride-1 shapes, batch 512
  const int it = argc > 1 ? atoi(argv[1]) : 20;
  check(512, 56, 56, 64, 64, false, it);
  check(512, 28, 28, 128, 128, false, it);
  check(512, 14, 14, 256, 256, false, it);
  check(512, 7, 7, 512, 512, false, it);
  check(512, 56, 56, 64, 64, true, it);
  check(512, 14, 14, 256, 256, true, it);
  return 0;
}
