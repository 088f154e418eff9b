// Micro-benchmark: how fast can a column reduction over an [M, C] bf16 NHWC tensor stream HBM on
// gfx950, and what access pattern does it need? (BN statistics at the ResNet-50 shapes.)
// Variants: per-block contiguous row chunks vs grid-interleaved passes, blocks per CU, rows in
// flight per lane. Sums are written per block (no finalize) — this measures the streaming part.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/read_reduce tools/membench/read_reduce.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void acc8(const uint4& t, float (&s1)[8], float (&s2)[8]) {
  const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = __uint_as_float(w[k] << 16), b = __uint_as_float(w[k] & 0xffff0000u);
    s1[2 * k] += a; s2[2 * k] = fmaf(a, a, s2[2 * k]);
    s1[2 * k + 1] += b; s2[2 * k + 1] = fmaf(b, b, s2[2 * k + 1]);
  }
}

// LPR lanes per row (8 channels each); R = 256/LPR rows per pass; U passes per iteration.
// INTERLEAVE=0: block b owns passes [b*ppb, (b+1)*ppb); 1: pass p = it*nblocks + b.
template <int LPR, int U, int INTERLEAVE>
__global__ __launch_bounds__(256) void rr_kernel(const uint16_t* __restrict__ x, int64_t M, int C, int64_t ppb,
                                                 float* __restrict__ out) {
  constexpr int R = 256 / LPR;
  const int tid = threadIdx.x, l = tid % LPR, r = tid / LPR;
  const int c = blockIdx.y * LPR * 8 + l * 8;
  float s1[8] = {}, s2[8] = {};
  const int64_t npass = M / R;
  const int64_t nit = ppb / U;
  for (int64_t it = 0; it < nit; ++it) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t p = INTERLEAVE ? ((it * U + u) * gridDim.x + blockIdx.x) : (blockIdx.x * ppb + it * U + u);
      if (p >= npass) p = npass - 1;
      v[u] = *reinterpret_cast<const uint4*>(x + (p * R + r) * (int64_t)C + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc8(v[u], s1, s2);
  }
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) a += s1[j] + s2[j];
  out[(int64_t)blockIdx.x * 256 + tid] = a;
}

template <int LPR, int U, int IL>
int run(uint16_t* const* xs, int64_t M, int C, int nblocks, float* out, const char* name) {
  constexpr int R = 256 / LPR;
  const int nchunk = C / (LPR * 8);
  const int64_t npass = M / R;
  int64_t ppb = (npass + nblocks - 1) / nblocks;
  ppb = (ppb + U - 1) / U * U;
  dim3 grid(nblocks, nchunk);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // 4 rotating 205-MB buffers (> the 256-MiB Infinity Cache): every launch streams from HBM
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rr_kernel<LPR, U, IL>), grid, dim3(256), 0, 0, xs[i & 3], M, C, ppb, out);
  CK(hipEventRecord(e0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((rr_kernel<LPR, U, IL>), grid, dim3(256), 0, 0, xs[i & 3], M, C, ppb, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / it;
  printf("%-34s C=%4d blocks=%5d x %2d  %7.1f us  %5.2f TB/s\n", name, C, nblocks, nchunk, us,
         (double)M * C * 2 / us / 1e6);
  return 0;
}

int main() {
  const int64_t bytes = 205520896;  // 512 x 56 x 56 x 64 bf16
  uint16_t* x[4]; float* out;
  for (int i = 0; i < 4; ++i) { CK(hipMalloc(&x[i], bytes)); CK(hipMemset(x[i], 0x3f, bytes)); }
  CK(hipMalloc(&out, 4096 * 256 * sizeof(float) * 8));
  for (int C : {64, 256, 1024}) {
    const int64_t M = bytes / 2 / C;
    for (int nb : {256, 512, 1024, 2048}) {
      const int nbk = C == 64 ? nb : (C == 256 ? nb : nb / 2);
      if (C == 64) {
        run<8, 8, 0>(x, M, C, nbk, out, "chunk LPR8 U8");
        run<8, 8, 1>(x, M, C, nbk, out, "interleave LPR8 U8");
        run<8, 4, 1>(x, M, C, nbk, out, "interleave LPR8 U4");
        run<8, 16, 1>(x, M, C, nbk, out, "interleave LPR8 U16");
      } else if (C == 256) {
        run<8, 8, 0>(x, M, C, nbk / 4, out, "chunk LPR8 U8 (64-ch chunks)");
        run<32, 8, 0>(x, M, C, nbk, out, "chunk LPR32 U8");
        run<32, 8, 1>(x, M, C, nbk, out, "interleave LPR32 U8");
      } else {
        run<64, 8, 0>(x, M, C, nbk, out, "chunk LPR64 U8");
        run<64, 8, 1>(x, M, C, nbk, out, "interleave LPR64 U8");
        run<8, 8, 1>(x, M, C, nbk / 8, out, "interleave LPR8 U8 (64-ch chunks)");
      }
    }
  }
  return 0;
}
