// Small-matrix assembly of the ALGEBRAIC backward of a ResNet bottleneck's conv3 + bn3 (gfx950).
//
// conv3: z = a W^T (a [M, CW] = bn2's output, W [C4, CW]); bn3's backward gives its input gradient as
//   dz = A g + B (z - mu) + D          (per channel c of C4; g = dy * relu mask, A B D = bn_bwd_coef)
// Substituting z = a W^T (the conv's own forward) removes z and dz from the backward entirely:
//   da = dz W     = g (diag(A) W) + a G + c,      G = W^T diag(B) W [CW, CW],  c = E W,  E = D - B mu
//   dW = dz^T a   = diag(A) P + diag(B) W Gram + E (x) S
// with P = g^T a [C4, CW], Gram = a^T a [CW, CW] and S = column sums of a — all three from ONE pass of
// the 1x1 weight-gradient kernel over (g, a) (conv1x1_wgrad.hip SEG), and da from ONE GEMM over the
// K-concatenation [g | a | a | 1] against b = [diag(A) W | G_hi | G_lo | c_hi, c_lo, 0...]^T rows
// (conv1x1.hip SEG; G and c split into bf16 hi + lo parts: the a G term can cancel part of g diag(A) W).
// The BatchNorm's backward apply pass (read dy, z, mask; write dz) and both re-reads of dz are gone:
// per bottleneck of ResNet-50 layers 2-4 one 4C-channel tensor is read twice instead of five times.
//
// This file: one launch that writes b (bf16 [CW, Kt], Kt = C4 + 2 CW + 32) and dW (bf16 [C4, CW]) from
// W, the coefficients and the fp32 products G (= W^T diag(B) W) and BWG (= diag(B) W Gram).
// Not in the reference (LeNet has no BatchNorm, /root/reference/cnn.py:9-23).
#include "../common.h"

#include <stdlib.h>

using namespace pdt;

namespace {

__device__ __forceinline__ float bfv(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

constexpr int kSK = 128;  // K rows per split-K slice of the small products (bn_alg_small_gemm_kernel)
// BWG's K is CW: one 64-row slice when CW == 64 (ResNet layer 1), 128-row slices otherwise
__host__ __device__ __forceinline__ int bwg_len(int CW) { return CW < kSK ? CW : kSK; }
__host__ __device__ __forceinline__ int bwg_slices(int CW) { return CW / bwg_len(CW); }

// blocks [0, CW): row k of b; blocks [CW, ...): 256-element slices of dW
__global__ __launch_bounds__(256) void bn_alg_assemble_kernel(const uint16_t* __restrict__ W, const float* __restrict__ coef,
                                                              const float* __restrict__ mean, const float* __restrict__ G,
                                                              const float* __restrict__ wg, const float* __restrict__ BWG,
                                                              uint16_t* __restrict__ bcat, uint16_t* __restrict__ dW,
                                                              int C4, int CW, int rep) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int Kt = C4 + rep * CW + 32;
  const float* A = coef;
  const float* Bc = coef + C4;
  const float* D = coef + 2 * C4;
  if ((int)blockIdx.x < CW) {
    const int k = blockIdx.x;
    uint16_t* row = bcat + (int64_t)k * Kt;
    float cs = 0.f;
    for (int c = tid; c < C4; c += 256) {
      const float w = bfv(W[(int64_t)c * CW + k]);
      row[c] = f2bf(w * A[c]);
      cs += (D[c] - Bc[c] * mean[c]) * w;
    }
    for (int j = tid; j < CW; j += 256) {
      float gv = 0.f;  // the split-K slices of G in order (bn_alg_small_gemm_kernel)
      for (int sl = 0; sl < C4 / kSK; ++sl) gv += G[((int64_t)sl * CW + k) * CW + j];
      const uint16_t hi = f2bf(gv);
      row[C4 + j] = hi;
      if (rep == 2) row[C4 + CW + j] = f2bf(gv - bfv(hi));
    }
    cs = block_sum(cs, red);
    if (tid < 32) {
      const uint16_t hi = f2bf(cs);
      row[C4 + rep * CW + tid] = tid == 0 ? hi : (tid == 1 ? f2bf(cs - bfv(hi)) : (uint16_t)0);
    }
    return;
  }
  const int64_t e = (int64_t)(blockIdx.x - CW) * 256 + tid;
  if (e >= (int64_t)C4 * CW) return;
  const int c = (int)(e / CW), k = (int)(e % CW);
  const float S = wg[(int64_t)(C4 + CW) * CW + k];  // first row of the ones block: column sums of a
  const float E = D[c] - Bc[c] * mean[c];
  float bwg = 0.f;
  for (int sl = 0; sl < bwg_slices(CW); ++sl) bwg += BWG[(int64_t)sl * C4 * CW + e];
  dW[e] = f2bf(A[c] * wg[e] + bwg + E * S);
}

// Sum-only producer (conv1x1.hip / gap_bwd with the BatchNorm input not read): each tile's centred-sum entry
// is sum(g (0 - mean)) = -mean sum(g). The true one is sum(g (z - mean)) = sum_k P[c, k] W[c, k] - mean sum(g)
// (z = a W^T): adding rowsum(P * W) to one tile's entry completes the reduction the finalize sums.
// One wave per channel: lanes stride the (contiguous) row, then a fixed-order wave sum.
__global__ __launch_bounds__(256) void bn_alg_fix_s2_kernel(float* __restrict__ part, int T, const float* __restrict__ wg,
                                                            const uint16_t* __restrict__ W, int C4, int CW) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C4) return;
  float s = 0.f;
  for (int k = lane; k < CW; k += 64) s += wg[(int64_t)c * CW + k] * bfv(W[(int64_t)c * CW + k]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) part[(int64_t)T * C4 + c] += s;  // part[1][0][c]
}

// A downsample shortcut BatchNorm's backward partials in one "tile" (ops/batchnorm.py _alg_ds_prelude): part[0][0] =
// s1 = sum(g) (bn3's bias gradient: the same g), part[1][0] = -mean s1 + rowsum(P * W) — the same fp32 operations as
// building -(mean * s1) and then bn_alg_fix_s2_kernel's add (one launch instead of four).
__global__ __launch_bounds__(256) void bn_alg_ds_part_kernel(float* __restrict__ part, const float* __restrict__ s1,
                                                             const float* __restrict__ mean, const float* __restrict__ wg,
                                                             const uint16_t* __restrict__ W, int C4, int CW) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C4) return;
  float s = 0.f;
  for (int k = lane; k < CW; k += 64) s += wg[(int64_t)c * CW + k] * bfv(W[(int64_t)c * CW + k]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) {
#pragma clang fp contract(off)
    const float v = s1[c];
    part[c] = v;
    const float mv = mean[c] * v;  // rounded on its own (no fma): the two-step form's product
    part[C4 + c] = -mv + s;
  }
}

// The two small fp32 products of the ALG backward in one launch, as split-K partials (64 x 64 output tiles,
// 256 threads x 4 x 4, K slices of 128 rows: 8 steps of 16 with the next step's operands loaded into registers
// before the current step's FMAs — a serial K loop of C4 / 16 latency-bound steps ran 110-200 us):
//   Gp[s]  [CW, CW] = sum over rows c of slice s: W[c, i] Bc[c] W[c, j]        (s < C4 / 128)
//   Bp[s]  [C4, CW] = Bc[c] sum over rows j of slice s: W[c, j] Gram[j, k]       (s < CW / 128)
// bn_alg_assemble_kernel sums the slices in a fixed order (deterministic).
__global__ __launch_bounds__(256) void bn_alg_small_gemm_kernel(const uint16_t* __restrict__ W, const float* __restrict__ coef,
                                                                const float* __restrict__ wg, float* __restrict__ Gp,
                                                                float* __restrict__ Bp, int C4, int CW) {
  __shared__ float sa[16][68], sb[16][68];
  const float* Bc = coef + C4;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int tcw = CW / 64, nG = tcw * tcw;
  const int t = blockIdx.x, sl = blockIdx.y;
  const bool isG = t < nG;
  if (isG ? sl >= C4 / kSK : sl >= bwg_slices(CW)) return;
  const int klen = isG ? kSK : bwg_len(CW);
  const int k0 = sl * klen;
  const float* Gram = wg + (int64_t)C4 * CW;
  int i0, j0;
  if (isG) { i0 = (t / tcw) * 64; j0 = (t % tcw) * 64; }
  else { i0 = ((t - nG) / tcw) * 64; j0 = ((t - nG) % tcw) * 64; }  // (c rows, k cols)
  // this thread's 4 (a, b) operand elements of one 16-row step: e = tid + 256 u
  float ra[4], rb[4];
  auto load = [&](int kk) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      if (isG) {
        const int r = e >> 6, q = e & 63, c = kk + r;
        ra[u] = bfv(W[(int64_t)c * CW + i0 + q]) * Bc[c];
        rb[u] = bfv(W[(int64_t)c * CW + j0 + q]);
      } else {
        const int r = e & 15, q = e >> 4;  // a: W[c = i0 + q, j = kk + r] (16 consecutive j per row)
        ra[u] = bfv(W[(int64_t)(i0 + q) * CW + kk + r]);
        const int r2 = e >> 6, q2 = e & 63;
        rb[u] = Gram[(int64_t)(kk + r2) * CW + j0 + q2];
      }
    }
  };
  float acc[4][4] = {};
  load(k0);
  for (int kk = k0; kk < k0 + klen; kk += 16) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      if (isG) { sa[e >> 6][e & 63] = ra[u]; }
      else { sa[e & 15][e >> 4] = ra[u]; }
      sb[e >> 6][e & 63] = rb[u];
    }
    __syncthreads();
    if (kk + 16 < k0 + klen) load(kk + 16);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float4 av = *reinterpret_cast<const float4*>(&sa[r][ty * 4]);
      const float4 bv = *reinterpret_cast<const float4*>(&sb[r][tx * 4]);
      const float a4[4] = {av.x, av.y, av.z, av.w}, b4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] += a4[u] * b4[v];
    }
  }
  if (isG) {
    float* o = Gp + (int64_t)sl * CW * CW;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<float4*>(o + (int64_t)(i0 + ty * 4 + u) * CW + j0 + tx * 4) =
          make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
  } else {
    float* o = Bp + (int64_t)sl * C4 * CW;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = i0 + ty * 4 + u;
      const float bcv = Bc[c];
      *reinterpret_cast<float4*>(o + (int64_t)c * CW + j0 + tx * 4) =
          make_float4(bcv * acc[u][0], bcv * acc[u][1], bcv * acc[u][2], bcv * acc[u][3]);
    }
  }
}

// The same split-K partials on the matrix cores (v_mfma_f32_16x16x32_bf16) with every non-bf16 operand carried as
// a bf16 hi + lo pair (two MFMAs; products exact, sums fp32: ~1e-5 relative, the VALU kernel above is the oracle in
// tests/test_bwd_alg_gpu.py). No LDS: every fragment is 8 K-contiguous elements of one row —
//   Gp: X = W^T rows i (the dgrad GEMM's prepared transpose), Y = (Bc W^T) rows j, K = c (slice of 128);
//   Bp: X = W rows c, Y = Gram rows k (Gram is symmetric: its row k is its column k), K = j.
// 256 threads = 4 waves, each a 32 x 32 quarter of the 64 x 64 tile (2 x 2 16 x 16 blocks). The VALU kernel ran
// 17-44 us per launch at ResNet-50's shapes, latency-bound.
typedef __bf16 bf16x8a __attribute__((ext_vector_type(8)));
typedef float f4a __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8a& hi, bf16x8a& lo) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 h, l;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint16_t h0 = f2bf(v[2 * k]), h1 = f2bf(v[2 * k + 1]);
    const uint16_t l0 = f2bf(v[2 * k] - bfv(h0)), l1 = f2bf(v[2 * k + 1] - bfv(h1));
    h[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    l[k] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
  hi = __builtin_bit_cast(bf16x8a, h);
  lo = __builtin_bit_cast(bf16x8a, l);
}

__global__ __launch_bounds__(256) void bn_alg_small_mfma_kernel(const uint16_t* __restrict__ W,
                                                                const uint16_t* __restrict__ Wt,
                                                                const float* __restrict__ coef,
                                                                const float* __restrict__ wg, float* __restrict__ Gp,
                                                                float* __restrict__ Bp, int C4, int CW) {
  const float* Bc = coef + C4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const int tcw = CW / 64, nG = tcw * tcw;
  const int t = blockIdx.x, sl = blockIdx.y;
  const bool isG = t < nG;
  if (isG ? sl >= C4 / kSK : sl >= bwg_slices(CW)) return;
  const int klen = isG ? kSK : bwg_len(CW);
  const int k0 = sl * klen;
  const float* Gram = wg + (int64_t)C4 * CW;
  int i0, j0;
  if (isG) { i0 = (t / tcw) * 64; j0 = (t % tcw) * 64; }
  else { i0 = ((t - nG) / tcw) * 64; j0 = ((t - nG) % tcw) * 64; }  // (c rows, k cols)
  i0 += 32 * (w >> 1);
  j0 += 32 * (w & 1);
  f4a acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f4a{0.f, 0.f, 0.f, 0.f};
  for (int kk = k0; kk < k0 + klen; kk += 32) {
    const int kc = kk + 8 * lq;  // this lane's 8 K elements
    bf16x8a x[2], yh[2], yl[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int r = i0 + 16 * a + lr;
      x[a] = *reinterpret_cast<const bf16x8a*>(isG ? Wt + (int64_t)r * C4 + kc : W + (int64_t)r * CW + kc);
    }
    float bsc[8];
    if (isG) {
      *reinterpret_cast<float4*>(bsc) = *reinterpret_cast<const float4*>(Bc + kc);
      *reinterpret_cast<float4*>(bsc + 4) = *reinterpret_cast<const float4*>(Bc + kc + 4);
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = j0 + 16 * b + lr;
      float v[8];
      if (isG) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 q = *reinterpret_cast<const u4*>(Wt + (int64_t)r * C4 + kc);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] = __uint_as_float(q[k] << 16) * bsc[2 * k];
          v[2 * k + 1] = __uint_as_float(q[k] & 0xffff0000u) * bsc[2 * k + 1];
        }
      } else {
        *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(Gram + (int64_t)r * CW + kc);
        *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(Gram + (int64_t)r * CW + kc + 4);
      }
      split8(v, yh[b], yl[b]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[a], yh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[a], yl[b], acc[a][b], 0, 0, 0);
      }
  }
  // lane's acc[r] = D[row = block row 4 lq + r][col = lr]
  if (isG) {
    float* o = Gp + (int64_t)sl * CW * CW;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(int64_t)(i0 + 16 * a + 4 * lq + r) * CW + j0 + 16 * b + lr] = acc[a][b][r];
  } else {
    float* o = Bp + (int64_t)sl * C4 * CW;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = i0 + 16 * a + 4 * lq + r;
        const float bcv = Bc[c];
#pragma unroll
        for (int b = 0; b < 2; ++b) o[(int64_t)c * CW + j0 + 16 * b + lr] = bcv * acc[a][b][r];
      }
  }
}

int g_small_mfma = -1;  // PDT_ALG_SMALL_MFMA (default 1), read once

}  // namespace

extern "C" {

// part [2, T, C4] fp32 (a sum-only producer's BatchNorm backward partials), wg: pdt_conv1x1_wgrad_seg's output
// (rows 0..C4-1 = P), W [C4, CW] bf16: completes part's centred sums in place (see bn_alg_fix_s2_kernel).
int pdt_bn_alg_fix_s2(float* part, int T, const float* wg, const uint16_t* W, int C4, int CW, hipStream_t s) {
  if (T < 1 || C4 < 1 || CW < 1) return -1;
  hipLaunchKernelGGL(bn_alg_fix_s2_kernel, dim3((C4 + 3) / 4), dim3(256), 0, s, part, T, wg, W, C4, CW);
  return 0;
}

// part [2, 1, C4] fp32 of a downsample BatchNorm on the ALG backward (see bn_alg_ds_part_kernel).
int pdt_bn_alg_ds_part(float* part, const float* s1, const float* mean, const float* wg, const uint16_t* W, int C4,
                       int CW, hipStream_t s) {
  if (C4 < 1 || CW < 1) return -1;
  hipLaunchKernelGGL(bn_alg_ds_part_kernel, dim3((C4 + 3) / 4), dim3(256), 0, s, part, s1, mean, wg, W, C4, CW);
  return 0;
}

// Gp [C4 / 128, CW, CW] and Bp [max(1, CW / 128), C4, CW] fp32 split-K slices (see bn_alg_small_gemm_kernel);
// C4 % 128 == 0, CW == 64 or CW % 128 == 0.
// Wt (nullable): W^T [CW, C4] bf16 — with it the products run on the matrix cores (bn_alg_small_mfma_kernel,
// PDT_ALG_SMALL_MFMA=0 keeps the fp32 VALU kernel).
int pdt_bn_alg_small_gemm(const uint16_t* W, const uint16_t* Wt, const float* coef, const float* wg, float* G,
                          float* BWG, int C4, int CW, hipStream_t s) {
  if (C4 % kSK || CW % 64 || (CW > 64 && CW % kSK)) return -1;
  if (g_small_mfma < 0) {
    const char* e = getenv("PDT_ALG_SMALL_MFMA");
    g_small_mfma = (e && e[0] == '0') ? 0 : 1;
  }
  const int tcw = CW / 64;
  const int sy = C4 / kSK > bwg_slices(CW) ? C4 / kSK : bwg_slices(CW);
  if (Wt && g_small_mfma)
    hipLaunchKernelGGL(bn_alg_small_mfma_kernel, dim3(tcw * tcw + (C4 / 64) * tcw, sy), dim3(256), 0, s, W, Wt, coef,
                       wg, G, BWG, C4, CW);
  else
    hipLaunchKernelGGL(bn_alg_small_gemm_kernel, dim3(tcw * tcw + (C4 / 64) * tcw, sy), dim3(256), 0, s, W, coef, wg,
                       G, BWG, C4, CW);
  return 0;
}

// bcat [CW, C4 + 2 CW + 32] bf16, dW [C4, CW] bf16; W [C4, CW] bf16 row-major; coef [3, C4] (A, B, D), mean [C4],
// G [CW, CW], BWG [C4, CW] fp32; wg: pdt_conv1x1_wgrad_seg's output (rows 0..C4-1 = P, row C4 + CW = S).
// rep = 2: G as a bf16 hi + lo pair (bcat [CW, C4 + 2 CW + 32], the data-gradient GEMM repeats a twice);
// rep = 1: G's hi half only (bcat [CW, C4 + CW + 32]: PDT_ALG_GLO=0).
int pdt_bn_alg_assemble(const uint16_t* W, const float* coef, const float* mean, const float* G, const float* wg,
                        const float* BWG, uint16_t* bcat, uint16_t* dW, int C4, int CW, int rep, hipStream_t s) {
  if (C4 < 1 || CW < 1 || rep < 1 || rep > 2) return -1;
  const int64_t nd = ((int64_t)C4 * CW + 255) / 256;
  hipLaunchKernelGGL(bn_alg_assemble_kernel, dim3((unsigned)(CW + nd)), dim3(256), 0, s, W, coef, mean, G, wg, BWG,
                     bcat, dW, C4, CW, rep);
  return 0;
}

}  // extern "C"
