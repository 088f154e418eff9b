// Standalone correctness + timing harness for csrc/kernels/conv_stem.hip (no torch): batch-512
// 224x224 bf16 NHWC input, [64][7][7][3] weights, a naive fp32 reference on a few images, time
// per call. -DPDT_STEM_PROBE=1/2/3 builds the diagnostic variants (no stores / no MFMA / no loads).
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/convbench/stem_bench.cpp -o stem_bench
#include "../../pytorch_distributed_training_example_amd/csrc/kernels/conv_stem.hip"

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
    p[i] = __builtin_bit_cast(uint16_t, (__bf16)(((h & 0xffff) / 65535.f - 0.5f) * 2.f * scale));
  }
}

__global__ void fill_one(uint16_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0x3f80;
}

__global__ void ref_kernel(const uint16_t* x, const uint16_t* w, float* y, int N, int H, int W, int OH, int OW) {
  const int64_t total = (int64_t)N * OH * OW * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % 64);
    const int64_t m = i / 64;
    const int ow = (int)(m % OW), oh = (int)((m / OW) % OH), n = (int)(m / ((int64_t)OH * OW));
    float acc = 0.f;
    for (int kh = 0; kh < 7; ++kh)
      for (int kw = 0; kw < 7; ++kw) {
        const int ih = 2 * oh - 3 + kh, iw = 2 * ow - 3 + kw;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        for (int c = 0; c < 3; ++c)
          acc += bf2f(x[(((int64_t)n * H + ih) * W + iw) * 3 + c]) * bf2f(w[((co * 7 + kh) * 7 + kw) * 3 + c]);
      }
    y[i] = acc;
  }
}

__global__ void ref_wgrad_kernel(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int OH, int OW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 147) return;
  const int co = i / 147, r = i % 147, kh = r / 21, kw = (r % 21) / 3, c = r % 3;
  float acc = 0.f;
  for (int n = 0; n < N; ++n)
    for (int oh = 0; oh < OH; ++oh)
      for (int ow = 0; ow < OW; ++ow) {
        const int ih = 2 * oh - 3 + kh, iw = 2 * ow - 3 + kw;
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
        acc += bf2f(dy[(((int64_t)n * OH + oh) * OW + ow) * 64 + co]) * bf2f(x[(((int64_t)n * H + ih) * W + iw) * 3 + c]);
      }
  dw[i] = acc;
}

static float bf_host(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

static int wgrad_main(int N, int H, int W, bool ref, int iters) {
  const int OH = (H - 1) / 2 + 1, OW = W / 2;
  const int64_t nx = (int64_t)N * H * W * 3, ny = (int64_t)N * OH * OW * 64;
  uint16_t *x, *dy, *dw;
  float *ws, *dwr;
  CK(hipMalloc(&x, nx * 2)); CK(hipMalloc(&dy, ny * 2)); CK(hipMalloc(&dw, 64 * 147 * 2));
  CK(hipMalloc(&ws, pdt_stem_wgrad_ws_floats() * 4)); CK(hipMalloc(&dwr, 64 * 147 * 4));
  fill_kernel<<<1024, 256>>>(x, nx, 5, 1.f);
  fill_kernel<<<1024, 256>>>(dy, ny, 6, 1.f);
  if (getenv("ONESX")) fill_one<<<1024, 256>>>(x, nx);
  if (getenv("ONESDY")) fill_one<<<1024, 256>>>(dy, ny);
  int rc = pdt_stem_conv_wgrad(x, dy, dw, ws, N, H, W, 0);
  CK(hipDeviceSynchronize());
  if (rc) { printf("wgrad rc %d\n", rc); return 1; }
  double md = 0, mr = 0;
  if (ref) {
    ref_wgrad_kernel<<<(64 * 147 + 255) / 256, 256>>>(x, dy, dwr, N, H, W, OH, OW);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> h(64 * 147);
    std::vector<float> r(64 * 147);
    CK(hipMemcpy(h.data(), dw, 64 * 147 * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), dwr, 64 * 147 * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < 64 * 147; ++i) {
      md = std::max(md, (double)std::fabs(bf_host(h[i]) - r[i]));
      mr = std::max(mr, (double)std::fabs(r[i]));
    }
    if (getenv("DUMP"))
      for (int i = 0; i < 147; i += 1) printf("co0 kh%d kw%d ci%d: ours %8.3f ref %8.3f\n", i / 21, (i % 21) / 3, i % 3, bf_host(h[i]), r[i]);
  }
  double us = 0;
  if (iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) pdt_stem_conv_wgrad(x, dy, dw, ws, N, H, W, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) pdt_stem_conv_wgrad(x, dy, dw, ws, N, H, W, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    us = ms * 1e3 / iters;
  }
  printf("stem wgrad N=%d H=%d W=%d: %.1f us  %.2f TB/s  max|err| %.3g (max|ref| %.3g)\n", N, H, W, us,
         us > 0 ? (nx + ny) * 2 / us / 1e6 : 0.0, md, mr);
  CK(hipFree(x)); CK(hipFree(dy)); CK(hipFree(dw)); CK(hipFree(ws)); CK(hipFree(dwr));
  return md > 0.02 * mr + 0.05 ? 2 : 0;
}

int main(int argc, char** argv) {
  if (getenv("WGRAD")) {
    int rc = 0;
    rc |= wgrad_main(2, 32, 32, true, 0);
    if (!getenv("DUMP")) rc |= wgrad_main(3, 17, 64, true, 0);
    if (!getenv("DUMP")) rc |= wgrad_main(2, 224, 224, true, 0);
    if (!getenv("DUMP")) rc |= wgrad_main(512, 224, 224, false, 20);
    return rc;
  }
  const int N = argc > 1 ? atoi(argv[1]) : 512, H = 224, W = 224, OH = 112, OW = 112;
  const int64_t nx = (int64_t)N * H * W * 3, ny = (int64_t)N * OH * OW * 64;
  uint16_t *x, *w, *wp, *y;
  float* yr;
  CK(hipMalloc(&x, nx * 2)); CK(hipMalloc(&w, 64 * 147 * 2)); CK(hipMalloc(&wp, pdt_stem_conv_wprep_elems() * 2));
  CK(hipMalloc(&y, ny * 2));
  fill_kernel<<<1024, 256>>>(x, nx, 1, 1.f);
  fill_kernel<<<64, 256>>>(w, 64 * 147, 2, 0.2f);
  int rc = pdt_stem_conv_fwd(x, w, wp, y, N, H, W, 0);
  CK(hipDeviceSynchronize());
  if (rc) { printf("rc %d\n", rc); return 1; }
  const int NR = 2;
  const int64_t nr = (int64_t)NR * OH * OW * 64;
  CK(hipMalloc(&yr, nr * 4));
  ref_kernel<<<1024, 256>>>(x, w, yr, NR, H, W, OH, OW);
  CK(hipDeviceSynchronize());
  std::vector<uint16_t> hy(nr);
  std::vector<float> hr(nr);
  CK(hipMemcpy(hy.data(), y, nr * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), yr, nr * 4, hipMemcpyDeviceToHost));
  double md = 0, mr = 0;
  for (int64_t i = 0; i < nr; ++i) {
    md = std::max(md, (double)std::fabs(bf_host(hy[i]) - hr[i]));
    mr = std::max(mr, (double)std::fabs(hr[i]));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) pdt_stem_conv_fwd(x, w, wp, y, N, H, W, 0);
  const int it = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < it; ++i) pdt_stem_conv_fwd(x, w, wp, y, N, H, W, 0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  printf("stem probe=%d N=%d: %.1f us  %.2f TB/s  max|err| %.3g (max|ref| %.3g)\n", PDT_STEM_PROBE, N, us,
         (nx + ny) * 2 / us / 1e6, md, mr);
  return 0;
}
