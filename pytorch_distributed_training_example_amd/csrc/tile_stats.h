// BatchNorm statistics of a conv output tile, taken in the producing kernel's epilogue from the
// bf16 tile staged in LDS (the values actually written), so the BatchNorm that consumes the
// output never re-reads it for its statistics (bn_fwd_train_tiles in kernels/batchnorm.hip).
//
// Partials layout: part[0 .. T*N)  = per-tile channel sums, part[T*N .. 2*T*N) = per-tile CENTRED
// sums of squares (sum (y - tile mean)^2), T = ceil(M / BM) tiles of BM rows. The finalize
// combines them in double: var = (sum_t (M2_t + S_t^2 / n_t)) / M - mean^2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdt {

// Threads = (channel pair, row group); `red` needs (THREADS / (BN/2)) * BN floats of LDS not
// overlapping the tile. Contains __syncthreads: every thread of the block must call it.
template <int BM, int BN, int THREADS, int STRIDE>
__device__ __forceinline__ void tile_bn_stats(const char* tile, float* red, int nvalid, float* __restrict__ part,
                                              int mt, int T, int N, int n0) {
  constexpr int kGroups = THREADS / (BN / 2);
  constexpr int kRows = BM / kGroups;
  static_assert(BM % kGroups == 0, "row groups");
  const int tid = threadIdx.x;
  const int cp = tid % (BN / 2), g = tid / (BN / 2);
  const char* col = tile + cp * 4;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll 8
  for (int rr = 0; rr < kRows; ++rr) {
    const int r = g * kRows + rr;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(col + r * STRIDE);
    if (r < nvalid) { s0 += __uint_as_float(v << 16); s1 += __uint_as_float(v & 0xffff0000u); }
  }
  red[g * BN + 2 * cp] = s0;
  red[g * BN + 2 * cp + 1] = s1;
  __syncthreads();
  float t0 = 0.f, t1 = 0.f;
#pragma unroll
  for (int q = 0; q < kGroups; ++q) { t0 += red[q * BN + 2 * cp]; t1 += red[q * BN + 2 * cp + 1]; }
  const float inv_n = 1.f / (float)nvalid;
  const float mu0 = t0 * inv_n, mu1 = t1 * inv_n;
  __syncthreads();
  float q0 = 0.f, q1 = 0.f;
#pragma unroll 8
  for (int rr = 0; rr < kRows; ++rr) {
    const int r = g * kRows + rr;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(col + r * STRIDE);
    const float d0 = __uint_as_float(v << 16) - mu0, d1 = __uint_as_float(v & 0xffff0000u) - mu1;
    if (r < nvalid) { q0 += d0 * d0; q1 += d1 * d1; }
  }
  red[g * BN + 2 * cp] = q0;
  red[g * BN + 2 * cp + 1] = q1;
  __syncthreads();
  if (g == 0) {
    float m20 = 0.f, m21 = 0.f;
#pragma unroll
    for (int q = 0; q < kGroups; ++q) { m20 += red[q * BN + 2 * cp]; m21 += red[q * BN + 2 * cp + 1]; }
    *reinterpret_cast<float2*>(part + (int64_t)mt * N + n0 + 2 * cp) = make_float2(t0, t1);
    *reinterpret_cast<float2*>(part + ((int64_t)T + mt) * N + n0 + 2 * cp) = make_float2(m20, m21);
  }
}

template <int BM, int BN, int THREADS>
constexpr int tile_bn_stats_lds() { return (THREADS / (BN / 2)) * BN * 4; }

}  // namespace pdt
