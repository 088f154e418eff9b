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
                                                              int C4, int CW) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const int Kt = C4 + 2 * CW + 32;
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
      row[C4 + CW + j] = f2bf(gv - bfv(hi));
    }
    cs = block_sum(cs, red);
    if (tid < 32) {
      const uint16_t hi = f2bf(cs);
      row[C4 + 2 * CW + tid] = tid == 0 ? hi : (tid == 1 ? f2bf(cs - bfv(hi)) : (uint16_t)0);
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

}  // namespace

extern "C" {

// part [2, T, C4] fp32 (a sum-only producer's BatchNorm backward partials), wg: pdt_conv1x1_wgrad_seg's output
// (rows 0..C4-1 = P), W [C4, CW] bf16: completes part's centred sums in place (see bn_alg_fix_s2_kernel).
int pdt_bn_alg_fix_s2(float* part, int T, const float* wg, const uint16_t* W, int C4, int CW, hipStream_t s) {
  if (T < 1 || C4 < 1 || CW < 1) return -1;
  hipLaunchKernelGGL(bn_alg_fix_s2_kernel, dim3((C4 + 3) / 4), dim3(256), 0, s, part, T, wg, W, C4, CW);
  return 0;
}

// Gp [C4 / 128, CW, CW] and Bp [max(1, CW / 128), C4, CW] fp32 split-K slices (see bn_alg_small_gemm_kernel);
// C4 % 128 == 0, CW == 64 or CW % 128 == 0.
int pdt_bn_alg_small_gemm(const uint16_t* W, const float* coef, const float* wg, float* G, float* BWG, int C4, int CW,
                          hipStream_t s) {
  if (C4 % kSK || CW % 64 || (CW > 64 && CW % kSK)) return -1;
  const int tcw = CW / 64;
  const int sy = C4 / kSK > bwg_slices(CW) ? C4 / kSK : bwg_slices(CW);
  hipLaunchKernelGGL(bn_alg_small_gemm_kernel, dim3(tcw * tcw + (C4 / 64) * tcw, sy), dim3(256), 0, s, W, coef, wg, G,
                     BWG, C4, CW);
  return 0;
}

// bcat [CW, C4 + 2 CW + 32] bf16, dW [C4, CW] bf16; W [C4, CW] bf16 row-major; coef [3, C4] (A, B, D), mean [C4],
// G [CW, CW], BWG [C4, CW] fp32; wg: pdt_conv1x1_wgrad_seg's output (rows 0..C4-1 = P, row C4 + CW = S).
int pdt_bn_alg_assemble(const uint16_t* W, const float* coef, const float* mean, const float* G, const float* wg,
                        const float* BWG, uint16_t* bcat, uint16_t* dW, int C4, int CW, hipStream_t s) {
  if (C4 < 1 || CW < 1) return -1;
  const int64_t nd = ((int64_t)C4 * CW + 255) / 256;
  hipLaunchKernelGGL(bn_alg_assemble_kernel, dim3((unsigned)(CW + nd)), dim3(256), 0, s, W, coef, mean, G, wg, BWG,
                     bcat, dW, C4, CW);
  return 0;
}

}  // extern "C"
