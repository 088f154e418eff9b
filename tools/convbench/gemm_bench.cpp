// Standalone timing harness for csrc/kernels/gemm.hip (no torch): random bf16 operands, a sampled
// fp32 check of C, and time per call on the ViT-B/16 / GPT-2-medium Linear shapes. Build variants
// with -DPDT_GEMM_PROBE=1 (no MFMA) / 2 (no DMA) to split the time between the load path and MFMA.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip tools/convbench/gemm_bench.cpp -o /tmp/gemmb
#include "../../pytorch_distributed_training_example_amd/csrc/kernels/gemm.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static float bfh(uint16_t v) { uint32_t u = (uint32_t)v << 16; float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
  struct S { const char* name; int M, K, N; } shapes[] = {
      {"gpt2_qkv", 8192, 1024, 3072}, {"gpt2_proj", 8192, 1024, 1024}, {"gpt2_fc1", 8192, 1024, 4096},
      {"gpt2_fc2", 8192, 4096, 1024}, {"vit_qkv", 25216, 768, 2304},  {"vit_proj", 25216, 768, 768},
      {"vit_fc1", 25216, 768, 3072},  {"vit_fc2", 25216, 3072, 768},  {"sq8k", 8192, 8192, 8192}};
  const int iters = 20;
  for (const S& s : shapes) {
    if (argc > 1 && strcmp(argv[1], s.name) != 0) continue;  // one shape (PMC runs)
    uint16_t *a, *b, *c;
    CK(hipMalloc(&a, (int64_t)s.M * s.K * 2)); CK(hipMalloc(&b, (int64_t)s.N * s.K * 2)); CK(hipMalloc(&c, (int64_t)s.M * s.N * 2));
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, a, (int64_t)s.M * s.K, 1u, 1.f);
    hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, b, (int64_t)s.N * s.K, 7u, 1.f);
    CK(pdt_gemm_nt(a, b, c, nullptr, nullptr, 0, 0, 0, s.M, s.N, s.K, 0) == 0 ? hipSuccess : hipErrorInvalidValue);
    CK(hipDeviceSynchronize());
    double err = 0;
    if (PDT_GEMM_PROBE == 0) {  // 64 sampled outputs against an fp64 host dot product
      std::vector<uint16_t> ha((size_t)s.K), hb((size_t)s.K), hc(1);
      for (int t = 0; t < 64; ++t) {
        const int m = (int)((t * 7919LL) % s.M), n = (int)((t * 104729LL) % s.N);
        CK(hipMemcpy(ha.data(), a + (int64_t)m * s.K, s.K * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), b + (int64_t)n * s.K, s.K * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), c + (int64_t)m * s.N + n, 2, hipMemcpyDeviceToHost));
        double ref = 0;
        for (int k = 0; k < s.K; ++k) ref += (double)bfh(ha[k]) * bfh(hb[k]);
        err = fmax(err, fabs(bfh(hc[0]) - ref) / sqrt((double)s.K));
      }
    }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) pdt_gemm_nt(a, b, c, nullptr, nullptr, 0, 0, 0, s.M, s.N, s.K, 0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = fminf(best, ms / iters);
    }
    printf("probe=%d %-10s M=%5d K=%5d N=%5d  %8.1f us  %7.1f TF/s  err/sqrtK=%.3g\n", PDT_GEMM_PROBE, s.name, s.M, s.K,
           s.N, best * 1e3, 2.0 * s.M * s.N * s.K / (best * 1e-3) / 1e12, err);
    CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c));
  }
  return 0;
}
