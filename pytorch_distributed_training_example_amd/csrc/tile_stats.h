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

// ---- The same partials from the values an epilogue thread already holds (no extra pass over the
// staged tile): every thread keeps sums of (y - K) and (y - K)^2 for one 8-channel chunk over its
// rows, K = the tile's first row (the same shift for every thread of the block, read once from the
// staged tile); the block sums them in a fixed order and stores S = n K + sum(y - K) and the centred
// M2 = sum (y - K)^2 - sum(y - K)^2 / n. Packed fp32 math (v_pk_add / v_pk_fma): ~3 VALU per value.
typedef float pdt_f2 __attribute__((ext_vector_type(2)));

struct RowStats8 {
  pdt_f2 k[4], s[4], q[4];
};

// K: the 8 channels' values in the tile's first row (as stored).
__device__ __forceinline__ void rs8_init(RowStats8& t, const uint4& k) {
  const uint32_t w[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t.k[j] = pdt_f2{__uint_as_float(w[j] << 16), __uint_as_float(w[j] & 0xffff0000u)};
    t.s[j] = pdt_f2{0.f, 0.f};
    t.q[j] = pdt_f2{0.f, 0.f};
  }
}

// One row's 8 bf16 values (as stored).
__device__ __forceinline__ void rs8_add(RowStats8& t, const uint4& v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const pdt_f2 d = pdt_f2{__uint_as_float(w[j] << 16), __uint_as_float(w[j] & 0xffff0000u)} - t.k[j];
    t.s[j] += d;
    t.q[j] = d * d + t.q[j];
  }
}

// Tile partials of the chunk (tid % (BN/8)) every thread accumulated over its rows; K = the tile's first-row
// value of channel tid (threads tid < BN; read before the tile's LDS was released), nvalid = the tile's valid
// rows; `red`: WAVES * (BN/8) * 16 floats of LDS nobody reads any more. Contains __syncthreads: every thread of
// the block must call it.
template <int BN, int WAVES>
__device__ __forceinline__ void rs8_tile_store(RowStats8& t, float K, float* red, float* __restrict__ part,
                                               int nvalid, int T, int mt, int N, int n0) {
  constexpr int kChunks = BN / 8;
  static_assert(64 % kChunks == 0, "chunk lanes");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto xr = [](float v) {  // v + v[lane ^ sh] for sh = kChunks .. 32 (VALU cross-lane forms)
    if constexpr (kChunks <= 8) v = xor_add<8>(v);
    if constexpr (kChunks <= 16) v = xor_add<16>(v);
    return xor_add<32>(v);
  };
  static_assert(kChunks >= 8, "xor_add distances");
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t.s[j] = pdt_f2{xr(t.s[j].x), xr(t.s[j].y)};
    t.q[j] = pdt_f2{xr(t.q[j].x), xr(t.q[j].y)};
  }
  if (lane < kChunks) {
    float* r = red + (wid * kChunks + lane) * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[2 * j] = t.s[j].x; r[2 * j + 1] = t.s[j].y;
      r[8 + 2 * j] = t.q[j].x; r[8 + 2 * j + 1] = t.q[j].y;
    }
  }
  __syncthreads();
  if (tid < BN) {
    const int c = tid >> 3, j = tid & 7;
    float S = 0.f, Q = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      S += red[(w * kChunks + c) * 16 + j];
      Q += red[(w * kChunks + c) * 16 + 8 + j];
    }
    const float n = (float)nvalid;
    part[(int64_t)mt * N + n0 + tid] = fmaf(n, K, S);
    part[((int64_t)T + mt) * N + n0 + tid] = fmaxf(Q - S * S / n, 0.f);
  }
}

template <int BN, int WAVES>
constexpr int rs8_tile_store_lds() { return WAVES * (BN / 8) * 16 * 4; }

// ---- BatchNorm BACKWARD reduction in the epilogue of the kernel that writes dy (the gradient at a
// BatchNorm's output): per tile, per channel, sum(dz) and sum(dz * (x - mean)), dz = dy * ReLU mask.
// part layout as above ([T][N] sums of dz, then [T][N] sums of dz (x - mean)); the finalize is
// bn_bwd_train_tiles (kernels/batchnorm.hip).
struct BnSrc {
  const uint16_t* x;    // the BatchNorm's input [M, N] bf16
  const uint8_t* mask;  // its ReLU bit-mask (bit j of byte (m*N + n)/8) or null
  const float* mean;    // its batch mean [N]
  float* part;          // [2][T][N] output
};

// One 8-channel piece of the written tile: dy (bf16 x 8, as stored), the BatchNorm input at the same
// place and its mask byte; mu = the 8 channels' means.
__device__ __forceinline__ void bn_bwd_accum8(uint4 v, uint4 xb, unsigned mk, const float (&mu)[8], float (&s1)[8],
                                              float (&s2)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w}, xw[4] = {xb.x, xb.y, xb.z, xb.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t gb = k & 1 ? (w[k >> 1] & 0xffff0000u) : (w[k >> 1] << 16);
    const uint32_t xv = k & 1 ? (xw[k >> 1] & 0xffff0000u) : (xw[k >> 1] << 16);
    const float g = (mk >> k) & 1u ? __uint_as_float(gb) : 0.f;
    s1[k] += g;
    s2[k] += g * (__uint_as_float(xv) - mu[k]);
  }
}

// The 8 bf16 values of v with the lanes whose ReLU bit is clear set to +0: a BSTATS epilogue stores the
// gradient at a BatchNorm + ReLU output already masked (every consumer multiplies by that mask anyway,
// so the stored values are bit-identical in effect, and the ALG backward of conv3 + bn3 needs g = dy m
// as a plain GEMM operand: ops/conv.py _bwd_alg).
__device__ __forceinline__ uint4 mask8(uint4 v, unsigned mk) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lo = (mk >> (2 * k)) & 1u ? 0x0000ffffu : 0u, hi = (mk >> (2 * k + 1)) & 1u ? 0xffff0000u : 0u;
    w[k] &= lo | hi;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Block-wide sum of every thread's (s1, s2) for its chunk (tid % CHUNKS; CHUNKS = BN/8 divides 64)
// and the tile's partials store. `red`: WAVES * 2 * BN floats of LDS no one reads any more
// (contains __syncthreads: every thread of the block must call it).
template <int BN, int WAVES>
__device__ __forceinline__ void bn_bwd_tile_store(float (&s1)[8], float (&s2)[8], float* red, float* __restrict__ part,
                                                  int T, int mt, int N, int n0) {
  constexpr int kChunks = BN / 8;
  static_assert(64 % kChunks == 0, "chunk lanes");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // lanes of one wave holding the same chunk differ in the lane bits >= log2(kChunks)
  static_assert(kChunks >= 8, "xor_add distances");
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if constexpr (kChunks <= 8) { s1[k] = xor_add<8>(s1[k]); s2[k] = xor_add<8>(s2[k]); }
    if constexpr (kChunks <= 16) { s1[k] = xor_add<16>(s1[k]); s2[k] = xor_add<16>(s2[k]); }
    s1[k] = xor_add<32>(s1[k]);
    s2[k] = xor_add<32>(s2[k]);
  }
  __syncthreads();
  if (lane < kChunks) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[(wid * 2) * BN + lane * 8 + k] = s1[k];
      red[(wid * 2 + 1) * BN + lane * 8 + k] = s2[k];
    }
  }
  __syncthreads();
  for (int q = tid; q < 2 * BN; q += WAVES * 64) {
    const int st = q / BN, ch = q % BN;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) t += red[(w * 2 + st) * BN + ch];
    part[((int64_t)st * T + mt) * N + n0 + ch] = t;
  }
}

}  // namespace pdt
