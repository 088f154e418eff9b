// LayerNorm forward/backward for gfx950 (ViT-B/16 D=768, GPT-2-medium D=1024).
//
// Not in the reference (no transformer); required by the ViT / GPT-2 north-star configs.
// One wave64 per row: the row stays in registers (D/64 values per lane, 8-byte bf16
// vectors), so the forward is an exact two-pass mean/variance with a single HBM read and
// write. The backward computes dx per row in registers and per-workgroup partial
// dgamma/dbeta (fixed-order second pass: deterministic, no atomics).
//
// Residual fusion (pre-norm transformer blocks): the forward optionally adds a residual branch
// first, s = x + h (rounded to the storage dtype, exactly as a separate add would store it),
// writes s (the new residual stream) and normalises it; the backward optionally adds the
// residual stream's own gradient, dx = LN'(dy) + ds. That removes the separate add kernels
// (2 per block forward, 2 per block backward) and one full read of s.
#include "../common.h"
#include "../fp8_pack.h"

using namespace pdt;

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves, one row each

template <typename T> __device__ __forceinline__ float round_to(float v) { return v; }
template <> __device__ __forceinline__ float round_to<uint16_t>(float v) { return bf2f(f2bf(v)); }

// Row statistics and the normalised value, shared by ln_fwd_kernel and ln_fwd_fp8_kernel with FP
// contraction off, so both produce the same bits (the fp8 form quantizes exactly the bf16 y).
template <int K>
__device__ __forceinline__ void ln_stats(const float (&v)[K][4], float eps, float& mean, float& rstd) {
#pragma clang fp contract(off)
  constexpr int D = 256 * K;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) s += v[k][0] + v[k][1] + v[k][2] + v[k][3];
  mean = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[k][j] - mean;
      q += d * d;
    }
  rstd = rsqrtf(wave_sum(q) * (1.f / D) + eps);
}
__device__ __forceinline__ float ln_val(float v, float mean, float rstd, float w, float b) {
#pragma clang fp contract(off)
  return (v - mean) * rstd * w + b;
}

// K = D / 256: 4-element groups per lane (D = 256*K)
template <typename T, int K>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     T* __restrict__ y, T* __restrict__ sum_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t N, float eps) {
  constexpr int D = 256 * K;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= N) return;
  const T* xr = x + row * D;
  float v[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Vec4<T>::ld(xr, (int64_t)(k * 256 + lane * 4), v[k]);
    if (res != nullptr) {  // s = x + h, stored and normalised at storage precision
      float hv[4];
      Vec4<T>::ld(res + row * D, (int64_t)(k * 256 + lane * 4), hv);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[k][j] = round_to<T>(v[k][j] + hv[j]);
      Vec4<T>::st(sum_out + row * D, (int64_t)(k * 256 + lane * 4), v[k]);
    }
  }
  float mean, rstd;
  ln_stats<K>(v, eps, mean, rstd);
  T* yr = y + row * D;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = k * 256 + lane * 4;
    float wv[4], bv[4], o[4];
    Vec4<float>::ld(w, c, wv);
    Vec4<float>::ld(b, c, bv);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = ln_val(v[k][j], mean, rstd, wv[j], bv[j]);
    Vec4<T>::st(yr, (int64_t)c, o);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// LayerNorm (+ residual add) whose output goes straight to e4m3 for the fp8 GEMM that consumes it
// (ops/fp8.py Fp8Act: a transformer block's qkv and fc1 inputs). Unfused, the bf16 y was written
// here and read back by a cast-transpose pass; now the kernel writes y as fp8 row-major AND
// transposed (the layouts the forward and the weight-gradient GEMMs take), scaled by the consumer's
// delayed scale, with |y|max folded into its amax slot. y is rounded to bf16 before quantizing, so
// the bytes equal the unfused chain's. A workgroup owns 32 rows (8 waves x 4 rows, every row's loads
// issued before any row's math: one exposed latency per wave); the fp8 rows also go to an LDS image (row pitch D + 4 bytes: the transposed
// readers' 8-row blocks hit distinct banks) from which the transposed 32-B row segments are written.
// Tiles are placed XCD-aware so the four tiles sharing a 128-B line of y^T write it through one L2.
template <int K>
__global__ __launch_bounds__(512) void ln_fwd_fp8_kernel(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ res,
                                                         const float* __restrict__ w, const float* __restrict__ b,
                                                         uint16_t* __restrict__ sum_out, uint8_t* __restrict__ yq,
                                                         uint8_t* __restrict__ yqt, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out, int64_t N, float eps,
                                                         const float* __restrict__ scale, float* __restrict__ amax,
                                                         int striped) {
  constexpr int D = 256 * K, kRows = 32, kPitch = D + 4;
  __shared__ __attribute__((aligned(16))) uint8_t tile[kRows * kPitch];
  __shared__ float red[8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * kRows;
  const float s8 = *scale;
  float wr[K][4], br[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Vec4<float>::ld(w, k * 256 + lane * 4, wr[k]);
    Vec4<float>::ld(b, k * 256 + lane * 4, br[k]);
  }
  float am = 0.f;
  {
    constexpr int r0 = 0;
    uint2 xv[4][K], hv[4][K];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = m0 + wv * 4 + r0 + q;
      if (row < N) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          xv[q][k] = *reinterpret_cast<const uint2*>(x + row * D + k * 256 + lane * 4);
          if (res != nullptr) hv[q][k] = *reinterpret_cast<const uint2*>(res + row * D + k * 256 + lane * 4);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int tr = wv * 4 + r0 + q;
      const int64_t row = m0 + tr;
      if (row >= N) continue;  // wave-uniform
      float v[K][4];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        v[k][0] = __uint_as_float(xv[q][k].x << 16); v[k][1] = __uint_as_float(xv[q][k].x & 0xffff0000u);
        v[k][2] = __uint_as_float(xv[q][k].y << 16); v[k][3] = __uint_as_float(xv[q][k].y & 0xffff0000u);
        if (res != nullptr) {  // s = x + h, stored and normalised at storage precision (as ln_fwd_kernel)
          const float hh[4] = {__uint_as_float(hv[q][k].x << 16), __uint_as_float(hv[q][k].x & 0xffff0000u),
                               __uint_as_float(hv[q][k].y << 16), __uint_as_float(hv[q][k].y & 0xffff0000u)};
#pragma unroll
          for (int j = 0; j < 4; ++j) v[k][j] = round_to<uint16_t>(v[k][j] + hh[j]);
          Vec4<uint16_t>::st(sum_out + row * D, (int64_t)(k * 256 + lane * 4), v[k]);
        }
      }
      float mean, rstd;
      ln_stats<K>(v, eps, mean, rstd);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = round_to<uint16_t>(ln_val(v[k][j], mean, rstd, wr[k][j], br[k][j]));
          am = fmaxf(am, fabsf(o[j]));
        }
        const uint32_t pk = pack4_fp8(o[0] * s8, o[1] * s8, o[2] * s8, o[3] * s8);
        *reinterpret_cast<uint32_t*>(yq + row * D + k * 256 + lane * 4) = pk;
        *reinterpret_cast<uint32_t*>(tile + tr * kPitch + k * 256 + lane * 4) = pk;
      }
      if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
    }
  }
  __syncthreads();
  // y^T: item (word column g, 8-row block rb) -> 4 rows of y^T, 8 bytes each; N % 16 == 0 keeps
  // 8-row blocks whole
  for (int it = threadIdx.x; it < (D / 4) * 4; it += 512) {
    const int rb = it & 3, g = it >> 2;
    if (m0 + rb * 8 < N) {
      uint32_t t8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) t8[i] = *reinterpret_cast<const uint32_t*>(tile + (rb * 8 + i) * kPitch + g * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<uint2*>(yqt + (int64_t)(g * 4 + j) * N + m0 + rb * 8) =
            make_uint2(byte_col(t8[0], t8[1], t8[2], t8[3], j), byte_col(t8[4], t8[5], t8[6], t8[7], j));
    }
  }
  am = wave_max(am);
  if (lane == 0) red[wv] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    float bm = red[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) bm = fmaxf(bm, red[i]);
    if (bm > 0.f) atomicMax(reinterpret_cast<int*>(amax_slot(amax, striped, blockIdx.x)), __float_as_int(bm));
  }
}

// Backward: dx per row; per-block partial dgamma/dbeta written to part[blk][2][D].
template <typename T, int K>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ dres,
                                                     const float* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, T* __restrict__ dx,
                                                     float* __restrict__ part, int64_t N, int rows_per_block) {
  constexpr int D = 256 * K;
  __shared__ float sdw[4][D];
  __shared__ float sdb[4][D];
  const int lane = threadIdx.x & 63, wv_id = threadIdx.x >> 6;
  float dw[K][4], db[K][4], wr[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Vec4<float>::ld(w, k * 256 + lane * 4, wr[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) { dw[k][j] = 0.f; db[k][j] = 0.f; }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  // RF rows per wave in flight (rows r, r + 4, ...): all loads of them are issued before any
  // row's math, so a wave exposes the memory latency once per RF rows (single-row: 2.5 TB/s)
  constexpr int RF = K <= 4 ? 4 : 2;
  for (int64_t row0 = r0 + wv_id; row0 < r1; row0 += 4 * RF) {
    float g[RF][K][4], xh[RF][K][4], rr[RF][K][4];
    float mu[RF], rs[RF];
    bool ok[RF];
#pragma unroll
    for (int q = 0; q < RF; ++q) {
      const int64_t row = row0 + 4 * q;
      ok[q] = row < r1;
      const int64_t rw = ok[q] ? row : row0;  // duplicate load for a missing second row, result unused
      mu[q] = mean[rw];
      rs[q] = rstd[rw];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int64_t c = rw * D + k * 256 + lane * 4;
        Vec4<T>::ld(dy, c, g[q][k]);
        Vec4<T>::ld(x, c, xh[q][k]);
        if (dres != nullptr) Vec4<T>::ld(dres, c, rr[q][k]);
      }
    }
#pragma unroll
    for (int q = 0; q < RF; ++q) {
      if (!ok[q]) continue;
      const int64_t row = row0 + 4 * q;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[q][k][j] = (xh[q][k][j] - mu[q]) * rs[q];
          db[k][j] += g[q][k][j];
          dw[k][j] += g[q][k][j] * xh[q][k][j];
          const float gw = g[q][k][j] * wr[k][j];
          s1 += gw;
          s2 += gw * xh[q][k][j];
        }
      s1 = wave_sum(s1) * (1.f / D);
      s2 = wave_sum(s2) * (1.f / D);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = rs[q] * (g[q][k][j] * wr[k][j] - s1 - xh[q][k][j] * s2);
          if (dres != nullptr) o[j] += rr[q][k][j];  // + the residual stream's own gradient
        }
        Vec4<T>::st(dx, row * D + k * 256 + lane * 4, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sdw[wv_id][k * 256 + lane * 4 + j] = dw[k][j];
      sdb[wv_id][k * 256 + lane * 4 + j] = db[k][j];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    part[((int64_t)blockIdx.x * 2 + 0) * D + c] = sdw[0][c] + sdw[1][c] + sdw[2][c] + sdw[3][c];
    part[((int64_t)blockIdx.x * 2 + 1) * D + c] = sdb[0][c] + sdb[1][c] + sdb[2][c] + sdb[3][c];
  }
}

// Fixed-order column sums of the per-block partials: 16 columns x 16 row-groups per workgroup,
// so each thread sums only nblk/16 independent values (latency-bound otherwise).
__global__ __launch_bounds__(256) void ln_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int D,
                                                              float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[2][16][17];
  const int grp = threadIdx.x >> 4, cl = threadIdx.x & 15;
  const int c = blockIdx.x * 16 + cl;
  float a = 0.f, b = 0.f;
  if (c < D)
    for (int blk = grp; blk < nblk; blk += 16) {
      a += part[((int64_t)blk * 2 + 0) * D + c];
      b += part[((int64_t)blk * 2 + 1) * D + c];
    }
  red[0][grp][cl] = a;
  red[1][grp][cl] = b;
  __syncthreads();
  if (grp == 0 && c < D) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) { sa += red[0][q][cl]; sb += red[1][q][cl]; }
    dw[c] = sa;
    db[c] = sb;
  }
}

// Workgroup cap (PDT_LN_BWD_BLOCKS, read once; A/B): 512 = 2 workgroups per CU.
inline int64_t ln_bwd_cap() {
  static int64_t cap = 0;
  if (cap == 0) {
    const char* e = getenv("PDT_LN_BWD_BLOCKS");
    const int64_t v = (e && e[0]) ? strtol(e, nullptr, 10) : 512;
    cap = v >= 64 && v <= 4096 ? v : 512;
  }
  return cap;
}

// Minimum rows per workgroup (PDT_LN_BWD_ROWS, read once; A/B): 32 = 8 rows per wave.
inline int64_t ln_bwd_min_rows() {
  static int64_t r = 0;
  if (r == 0) {
    const char* e = getenv("PDT_LN_BWD_ROWS");
    const int64_t v = (e && e[0]) ? strtol(e, nullptr, 10) : 32;
    r = v >= 4 && v <= 256 ? v : 32;
  }
  return r;
}

inline int ln_bwd_blocks(int64_t N, int& rows_per_block) {
  int64_t nblk = (N + ln_bwd_min_rows() - 1) / ln_bwd_min_rows();
  if (nblk > ln_bwd_cap()) nblk = ln_bwd_cap();  // the dgamma/dbeta slab is nblk x 2 x D floats
  if (nblk < 1) nblk = 1;
  rows_per_block = (int)((N + nblk - 1) / nblk);
  return (int)((N + rows_per_block - 1) / rows_per_block);
}

}  // namespace

extern "C" {

int64_t pdt_ln_workspace_floats(int64_t N, int D) {
  int rpb;
  return (int64_t)ln_bwd_blocks(N, rpb) * 2 * D;
}

#define PDT_LN_SWITCH(MACRO) \
  switch (D / 256) {         \
    case 1: MACRO(1); break; \
    case 2: MACRO(2); break; \
    case 3: MACRO(3); break; \
    case 4: MACRO(4); break; \
    case 5: MACRO(5); break; \
    case 6: MACRO(6); break; \
    case 8: MACRO(8); break; \
    case 10: MACRO(10); break; \
    case 12: MACRO(12); break; \
    case 16: MACRO(16); break; \
    default: return -1;      \
  }

// res / sum_out: optional residual branch h and the stored sum s = x + h (both or neither).
int pdt_ln_fwd(const void* x, const void* res, int dtype, const float* w, const float* b, void* y, void* sum_out,
               float* mean, float* rstd, int64_t N, int D, float eps, hipStream_t s) {
  if ((res == nullptr) != (sum_out == nullptr)) return -2;
  if (D % 256 != 0) return -1;
  if (N == 0) return 0;
  const dim3 grid((unsigned)((N + kRowsPerBlock - 1) / kRowsPerBlock));
#define PDT_LNF(K)                                                                                           \
  if (dtype == 0)                                                                                            \
    hipLaunchKernelGGL((ln_fwd_kernel<float, K>), grid, dim3(256), 0, s, (const float*)x, (const float*)res, w, \
                       b, (float*)y, (float*)sum_out, mean, rstd, N, eps);                                    \
  else                                                                                                       \
    hipLaunchKernelGGL((ln_fwd_kernel<uint16_t, K>), grid, dim3(256), 0, s, (const uint16_t*)x,               \
                       (const uint16_t*)res, w, b, (uint16_t*)y, (uint16_t*)sum_out, mean, rstd, N, eps);
  PDT_LN_SWITCH(PDT_LNF)
#undef PDT_LNF
  return 0;
}

// bf16 x (+ res -> sum_out) -> LayerNorm -> e4m3 yq [N, D] and yq^T [D, N] (scale / amax: the
// consumer's fp8 state row). N % 16 == 0; D = 256 K, K in {2, .., 6} (K = 8 would spill).
int pdt_ln_fwd_fp8(const uint16_t* x, const uint16_t* res, const float* w, const float* b, uint16_t* sum_out,
                   uint8_t* yq, uint8_t* yqt, float* mean, float* rstd, int64_t N, int D, float eps,
                   const float* scale, float* amax, int striped, hipStream_t s) {
  if ((res == nullptr) != (sum_out == nullptr)) return -2;
  if (D % 256 != 0 || N % 16 != 0) return -1;
  if (N == 0) return 0;
  const dim3 grid((unsigned)((N + 31) / 32));
#define PDT_LNF8(K)                                                                                          \
  hipLaunchKernelGGL((ln_fwd_fp8_kernel<K>), grid, dim3(512), 0, s, x, res, w, b, sum_out, yq, yqt, mean, rstd, N, \
                     eps, scale, amax, striped);
  switch (D / 256) {
    case 2: PDT_LNF8(2); break;
    case 3: PDT_LNF8(3); break;
    case 4: PDT_LNF8(4); break;
    case 5: PDT_LNF8(5); break;
    case 6: PDT_LNF8(6); break;
    default: return -1;
  }
#undef PDT_LNF8
  return 0;
}

// dres: optional gradient added into dx (residual stream), same dtype/layout as dx.
int pdt_ln_bwd(const void* dy, const void* x, const void* dres, int dtype, const float* w, const float* mean,
               const float* rstd, void* dx, float* dw, float* db, int64_t N, int D, float* ws, hipStream_t s) {
  if (D % 256 != 0 || D > 2048) return -1;  // LDS: 2 x 4 x D floats
  if (N == 0) return 0;
  int rpb;
  const int nblk = ln_bwd_blocks(N, rpb);
#define PDT_LNB(K)                                                                                            \
  if (dtype == 0)                                                                                             \
    hipLaunchKernelGGL((ln_bwd_kernel<float, K>), dim3(nblk), dim3(256), 0, s, (const float*)dy, (const float*)x, \
                       (const float*)dres, w, mean, rstd, (float*)dx, ws, N, rpb);                            \
  else                                                                                                        \
    hipLaunchKernelGGL((ln_bwd_kernel<uint16_t, K>), dim3(nblk), dim3(256), 0, s, (const uint16_t*)dy,         \
                       (const uint16_t*)x, (const uint16_t*)dres, w, mean, rstd, (uint16_t*)dx, ws, N, rpb);
  switch (D / 256) {
    case 1: PDT_LNB(1); break;
    case 2: PDT_LNB(2); break;
    case 3: PDT_LNB(3); break;
    case 4: PDT_LNB(4); break;
    case 5: PDT_LNB(5); break;
    case 6: PDT_LNB(6); break;
    case 8: PDT_LNB(8); break;
    default: return -1;
  }
#undef PDT_LNB
  hipLaunchKernelGGL(ln_bwd_finalize_kernel, dim3((D + 15) / 16), dim3(256), 0, s, ws, nblk, D, dw, db);
  return 0;
}

}  // extern "C"
