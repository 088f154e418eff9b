// LayerNorm forward/backward for gfx950 (ViT-B/16 D=768, GPT-2-medium D=1024).
//
// Not in the reference (no transformer); required by the ViT / GPT-2 north-star configs.
// One wave64 per row: the row stays in registers (D/64 values per lane, 8-byte bf16
// vectors), so the forward is an exact two-pass mean/variance with a single HBM read and
// write. The backward computes dx per row in registers and per-workgroup partial
// dgamma/dbeta (fixed-order second pass: deterministic, no atomics).
#include "../common.h"

using namespace pdt;

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves, one row each

// K = D / 256: 4-element groups per lane (D = 256*K)
template <typename T, int K>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t N, float eps) {
  constexpr int D = 256 * K;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= N) return;
  const T* xr = x + row * D;
  float v[K][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Vec4<T>::ld(xr, (int64_t)(k * 256 + lane * 4), v[k]);
    s += v[k][0] + v[k][1] + v[k][2] + v[k][3];
  }
  const float mean = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) { const float d = v[k][j] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / D) + eps);
  T* yr = y + row * D;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = k * 256 + lane * 4;
    float wv[4], bv[4], o[4];
    Vec4<float>::ld(w, c, wv);
    Vec4<float>::ld(b, c, bv);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = (v[k][j] - mean) * rstd * wv[j] + bv[j];
    Vec4<T>::st(yr, (int64_t)c, o);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// Backward: dx per row; per-block partial dgamma/dbeta written to part[blk][2][D].
template <typename T, int K>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
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
  for (int64_t row = r0 + wv_id; row < r1; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float g[K][4], xh[K][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t c = row * D + k * 256 + lane * 4;
      Vec4<T>::ld(dy, c, g[k]);
      Vec4<T>::ld(x, c, xh[k]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xh[k][j] = (xh[k][j] - mu) * rs;
        db[k][j] += g[k][j];
        dw[k][j] += g[k][j] * xh[k][j];
        const float gw = g[k][j] * wr[k][j];
        s1 += gw;
        s2 += gw * xh[k][j];
      }
    }
    s1 = wave_sum(s1) * (1.f / D);
    s2 = wave_sum(s2) * (1.f / D);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = rs * (g[k][j] * wr[k][j] - s1 - xh[k][j] * s2);
      Vec4<T>::st(dx, row * D + k * 256 + lane * 4, o);
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

inline int ln_bwd_blocks(int64_t N, int& rows_per_block) {
  int64_t nblk = (N + 31) / 32;  // >= 8 rows per wave
  if (nblk > 256) nblk = 256;
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

int pdt_ln_fwd(const void* x, int dtype, const float* w, const float* b, void* y, float* mean, float* rstd,
               int64_t N, int D, float eps, hipStream_t s) {
  if (D % 256 != 0) return -1;
  if (N == 0) return 0;
  const dim3 grid((unsigned)((N + kRowsPerBlock - 1) / kRowsPerBlock));
#define PDT_LNF(K)                                                                                           \
  if (dtype == 0)                                                                                            \
    hipLaunchKernelGGL((ln_fwd_kernel<float, K>), grid, dim3(256), 0, s, (const float*)x, w, b, (float*)y, mean, \
                       rstd, N, eps);                                                                        \
  else                                                                                                       \
    hipLaunchKernelGGL((ln_fwd_kernel<uint16_t, K>), grid, dim3(256), 0, s, (const uint16_t*)x, w, b,         \
                       (uint16_t*)y, mean, rstd, N, eps);
  PDT_LN_SWITCH(PDT_LNF)
#undef PDT_LNF
  return 0;
}

int pdt_ln_bwd(const void* dy, const void* x, int dtype, const float* w, const float* mean, const float* rstd,
               void* dx, float* dw, float* db, int64_t N, int D, float* ws, hipStream_t s) {
  if (D % 256 != 0 || D > 2048) return -1;  // LDS: 2 x 4 x D floats
  if (N == 0) return 0;
  int rpb;
  const int nblk = ln_bwd_blocks(N, rpb);
#define PDT_LNB(K)                                                                                            \
  if (dtype == 0)                                                                                             \
    hipLaunchKernelGGL((ln_bwd_kernel<float, K>), dim3(nblk), dim3(256), 0, s, (const float*)dy, (const float*)x, \
                       w, mean, rstd, (float*)dx, ws, N, rpb);                                                \
  else                                                                                                        \
    hipLaunchKernelGGL((ln_bwd_kernel<uint16_t, K>), dim3(nblk), dim3(256), 0, s, (const uint16_t*)dy,         \
                       (const uint16_t*)x, w, mean, rstd, (uint16_t*)dx, ws, N, rpb);
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
