// Sum of S equal slices: out[i] = sum_s x[s * n + i] (bf16 in, fp32 accumulate, bf16 out).
//
// The second half of the split-K weight gradients (ops/conv.py _wgrad_splitk, ops/linear.py): a
// batched GEMM leaves S partial dW slices [S][Co*Ci]; aten's dim-0 sum of that [S, N] tensor ran at
// ~2.5 TB/s (10 us per GPT-2-medium weight, 97 calls = 1 ms/step, profiles/r2/transformer).
// Here one lane owns 8 consecutive outputs: S independent 16-B loads in flight (all issued before
// the first add), one 16-B store, a grid-stride loop of 8 workgroups per CU.
// Not in the reference (no weight-gradient code there: torch autograd, /root/reference/train.py:49).
#include "../common.h"

using namespace pdt;

namespace {

__device__ __forceinline__ void unpack8(const uint4& t, float (&v)[8]) {
  const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

template <int S>
__global__ __launch_bounds__(256) void slice_sum_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out,
                                                        int64_t nvec, int64_t n) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    uint4 p[S];
#pragma unroll
    for (int s = 0; s < S; ++s) p[s] = *reinterpret_cast<const uint4*>(x + s * n + v * 8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float f[8];
      unpack8(p[s], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    st8_bf16(out + v * 8, acc);
  }
}

}  // namespace

extern "C" {

// x: [S][n] bf16 contiguous, n % 8 == 0, S in {2, 4, 8, 16, 32, 64}; out: [n] bf16.
int pdt_slice_sum_bf16(const uint16_t* x, uint16_t* out, int S, int64_t n, hipStream_t s) {
  if (n % 8 != 0 || n < 8) return -1;
  const int64_t nvec = n / 8;
  int64_t grid = (nvec + 255) / 256;
  if (grid > 256 * 8) grid = 256 * 8;
#define PDT_SS(SS) hipLaunchKernelGGL(slice_sum_kernel<SS>, dim3((unsigned)grid), dim3(256), 0, s, x, out, nvec, n)
  switch (S) {
    case 2: PDT_SS(2); break;
    case 4: PDT_SS(4); break;
    case 8: PDT_SS(8); break;
    case 16: PDT_SS(16); break;
    case 32: PDT_SS(32); break;
    case 64: PDT_SS(64); break;
    default: return -1;
  }
#undef PDT_SS
  return 0;
}

}  // extern "C"
