// Channels-last (NHWC) bf16 BatchNorm for gfx950, training + eval, with fused ReLU and
// fused residual add (ResNet bottleneck tail: relu(bn3(x) + identity)).
//
// Not in the reference (LeNet has no BN, /root/reference/cnn.py:9-23); required by the
// ResNet-50 north-star config (BASELINE.json). Activations are [M = N*H*W, C] bf16 with C
// contiguous, so every lane moves 8 channels (16 B) per access and a wave reads whole rows.
//
// Forward (train):   reduce  -> per-block (Σ(x-k), Σ(x-k)²) partials, k = x[0, c] shift
//                    finalize-> mean, invstd, running stats, per-channel (a, b)
//                    apply   -> y = x*a + b (+ residual) (relu), bf16 out
// Backward (train):  reduce  -> per-block (Σdz, Σdz(x-mean)), dz = dy * (y > 0)
//                    finalize-> dgamma, dbeta and per-channel dx coefficients
//                    apply   -> dx = A dz + B (x-mean) + D, (dres = dz)
// Partials are summed in a fixed order (deterministic, no float atomics). The apply passes
// use a grid-stride of a multiple of C so each lane's 8-channel coefficients are loaded once.
#include "../common.h"

using namespace pdt;

namespace {

constexpr int kThreads = 256;
constexpr int kChunkC = 2048;  // channels per workgroup in the reduce pass (256 lanes x 8)

struct Geo {
  int CC, L, R;  // channels in this chunk, lanes per row, rows per pass
};
__device__ __forceinline__ Geo geo(int C, int chunk) {
  Geo g;
  const int c0 = chunk * kChunkC;
  g.CC = min(kChunkC, C - c0);
  g.L = g.CC / 8;
  g.R = kThreads / g.L;
  return g;
}

// MODE 0: forward stats. MODE 1: backward reduce (no relu). MODE 2: backward reduce w/ relu mask.
template <int MODE>
__global__ __launch_bounds__(kThreads) void bn_reduce_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, int64_t M, int C, int64_t rows_per_block,
    float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sm[2][kChunkC];
  const Geo g = geo(C, blockIdx.y);
  const int tid = threadIdx.x;
  const int r = tid / g.L, l = tid % g.L;
  const int c = blockIdx.y * kChunkC + l * 8;
  const bool active = r < g.R;
  const int64_t m0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t m1 = min(M, m0 + rows_per_block);
  float k[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (active) {
    if (MODE == 0) ld8_bf16(x + c, k);  // shift: first row of the tensor (same for all blocks)
    else {
      const float4 a = *reinterpret_cast<const float4*>(mean + c);
      const float4 b = *reinterpret_cast<const float4*>(mean + c + 4);
      k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
    }
    int64_t m = m0 + r;
    // 2-deep unroll: two independent rows in flight per lane
    for (; m + g.R < m1; m += 2 * g.R) {
      float xa[8], xb[8];
      ld8_bf16(x + m * C + c, xa);
      ld8_bf16(x + (m + g.R) * C + c, xb);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float da = xa[j] - k[j], db = xb[j] - k[j];
          s1[j] += da + db;
          s2[j] += da * da + db * db;
        }
      } else {
        float ga[8], gb[8];
        ld8_bf16(dy + m * C + c, ga);
        ld8_bf16(dy + (m + g.R) * C + c, gb);
        if (MODE == 2) {
          float ya[8], yb[8];
          ld8_bf16(y + m * C + c, ya);
          ld8_bf16(y + (m + g.R) * C + c, yb);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            ga[j] = ya[j] > 0.f ? ga[j] : 0.f;
            gb[j] = yb[j] > 0.f ? gb[j] : 0.f;
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1[j] += ga[j] + gb[j];
          s2[j] += ga[j] * (xa[j] - k[j]) + gb[j] * (xb[j] - k[j]);
        }
      }
    }
    for (; m < m1; m += g.R) {
      float xa[8];
      ld8_bf16(x + m * C + c, xa);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = xa[j] - k[j]; s1[j] += d; s2[j] += d * d; }
      } else {
        float ga[8];
        ld8_bf16(dy + m * C + c, ga);
        if (MODE == 2) {
          float ya[8];
          ld8_bf16(y + m * C + c, ya);
#pragma unroll
          for (int j = 0; j < 8; ++j) ga[j] = ya[j] > 0.f ? ga[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) { s1[j] += ga[j]; s2[j] += ga[j] * (xa[j] - k[j]); }
      }
    }
  }
  // reduce the R row-groups of the block through LDS (rows of width CC)
  const int CC = g.CC;
  if (g.R == 1) {
    if (active) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        part[((int64_t)blockIdx.x * 2 + 0) * C + c + j] = s1[j];
        part[((int64_t)blockIdx.x * 2 + 1) * C + c + j] = s2[j];
      }
    }
    return;
  }
  // tree over r: sm holds R x CC partials only when R*CC <= kChunkC (always: R*L*8 <= 2048)
  if (active) {
    float* d0 = &sm[0][r * CC + l * 8];
    float* d1 = &sm[1][r * CC + l * 8];
    *reinterpret_cast<float4*>(d0) = make_float4(s1[0], s1[1], s1[2], s1[3]);
    *reinterpret_cast<float4*>(d0 + 4) = make_float4(s1[4], s1[5], s1[6], s1[7]);
    *reinterpret_cast<float4*>(d1) = make_float4(s2[0], s2[1], s2[2], s2[3]);
    *reinterpret_cast<float4*>(d1 + 4) = make_float4(s2[4], s2[5], s2[6], s2[7]);
  }
  __syncthreads();
  for (int cc = tid; cc < CC; cc += kThreads) {
    float a = 0.f, b = 0.f;
    for (int rr = 0; rr < g.R; ++rr) { a += sm[0][rr * CC + cc]; b += sm[1][rr * CC + cc]; }
    part[((int64_t)blockIdx.x * 2 + 0) * C + blockIdx.y * kChunkC + cc] = a;
    part[((int64_t)blockIdx.x * 2 + 1) * C + blockIdx.y * kChunkC + cc] = b;
  }
}

// Sum nblk partials for 64 channels per workgroup (4 groups of 64 lanes, fixed order).
__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int nblk, int C, int c,
                                             float& S1, float& S2) {
  __shared__ float red[2][4][64];
  const int grp = threadIdx.x / 64, ln = threadIdx.x % 64;
  float a = 0.f, b = 0.f;
  if (c < C) {
    for (int blk = grp; blk < nblk; blk += 4) {
      a += part[((int64_t)blk * 2 + 0) * C + c];
      b += part[((int64_t)blk * 2 + 1) * C + c];
    }
  }
  red[0][grp][ln] = a;
  red[1][grp][ln] = b;
  __syncthreads();
  S1 = red[0][0][ln] + red[0][1][ln] + red[0][2][ln] + red[0][3][ln];
  S2 = red[1][0][ln] + red[1][1][ln] + red[1][2][ln] + red[1][3][ln];
}

__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(
    const float* __restrict__ part, int nblk, int C, int64_t M, const uint16_t* __restrict__ x,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ mean_out,
    float* __restrict__ invstd_out, float* __restrict__ a_out, float* __restrict__ b_out,
    float* __restrict__ running_mean, float* __restrict__ running_var, float momentum, float eps) {
  const int c = blockIdx.x * 64 + (threadIdx.x % 64);
  float S1, S2;
  sum_partials(part, nblk, C, c, S1, S2);
  if (threadIdx.x >= 64 || c >= C) return;
  const float k = bf2f(x[c]);
  const double inv_m = 1.0 / (double)M;
  const double d1 = (double)S1 * inv_m;
  double var = (double)S2 * inv_m - d1 * d1;
  var = var < 0.0 ? 0.0 : var;
  const float mean = (float)(k + d1);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = mean;
  invstd_out[c] = invstd;
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  a_out[c] = gm * invstd;
  b_out[c] = bt - mean * gm * invstd;
  if (running_mean) running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
  if (running_var) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unbiased;
  }
}

__global__ void bn_eval_coef_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                    float* __restrict__ a_out, float* __restrict__ b_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  a_out[c] = gm * invstd;
  b_out[c] = bt - rm[c] * gm * invstd;
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    const float* __restrict__ part, int nblk, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ A, float* __restrict__ B, float* __restrict__ D) {
  const int c = blockIdx.x * 64 + (threadIdx.x % 64);
  float S1, S2;
  sum_partials(part, nblk, C, c, S1, S2);
  if (threadIdx.x >= 64 || c >= C) return;
  const float is = invstd[c];
  const float gm = gamma ? gamma[c] : 1.f;
  const float db = S1, dg = S2 * is;
  if (dgamma) dgamma[c] = dg;
  if (dbeta) dbeta[c] = db;
  const float inv_m = 1.f / (float)M;
  A[c] = gm * is;
  B[c] = -gm * is * is * dg * inv_m;
  D[c] = -gm * is * db * inv_m;
}

__device__ __forceinline__ void ld8_f32(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <bool RELU, bool RES>
__global__ __launch_bounds__(256) void bn_apply_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const float* __restrict__ a,
    const float* __restrict__ b, uint16_t* __restrict__ y, int64_t nvec, int C, int fixed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float av[8], bv[8];
  if (fixed && i < nvec) {
    const int c = (int)((i * 8) % C);
    ld8_f32(a + c, av);
    ld8_f32(b + c, bv);
  }
  for (; i < nvec; i += stride) {
    if (!fixed) {
      const int c = (int)((i * 8) % C);
      ld8_f32(a + c, av);
      ld8_f32(b + c, bv);
    }
    float v[8];
    ld8_bf16(x + i * 8, v);
    float rv[8];
    if (RES) ld8_bf16(res + i * 8, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[j] * av[j] + bv[j];
      if (RES) t += rv[j];
      if (RELU) t = t > 0.f ? t : 0.f;
      v[j] = t;
    }
    st8_bf16(y + i * 8, v);
  }
}

template <bool RELU, bool RES>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ A, const float* __restrict__ B,
    const float* __restrict__ D, uint16_t* __restrict__ dx, uint16_t* __restrict__ dres, int64_t nvec,
    int C, int fixed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float mv[8], av[8], bv[8], dv[8];
  auto load_coef = [&](int64_t ii) {
    const int c = (int)((ii * 8) % C);
    ld8_f32(mean + c, mv);
    ld8_f32(A + c, av);
    ld8_f32(B + c, bv);
    ld8_f32(D + c, dv);
  };
  if (fixed && i < nvec) load_coef(i);
  for (; i < nvec; i += stride) {
    if (!fixed) load_coef(i);
    float g[8], xv[8];
    ld8_bf16(dy + i * 8, g);
    ld8_bf16(x + i * 8, xv);
    if (RELU) {
      float yv[8];
      ld8_bf16(y + i * 8, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    if (RES) st8_bf16(dres + i * 8, g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = av[j] * g[j] + bv[j] * (xv[j] - mv[j]) + dv[j];
    st8_bf16(dx + i * 8, o);
  }
}

inline int num_reduce_blocks(int64_t M, int C, int64_t& rows_per_block) {
  const int CC = C < kChunkC ? C : kChunkC;
  const int R = kThreads / (CC / 8);
  const int nchunks = (C + kChunkC - 1) / kChunkC;
  int64_t nblk = (M + (int64_t)R * 8 - 1) / ((int64_t)R * 8);  // >= 8 row-passes per lane
  const int64_t cap = 512 / nchunks > 0 ? 512 / nchunks : 1;
  if (nblk > cap) nblk = cap;
  if (nblk < 1) nblk = 1;
  rows_per_block = (M + nblk - 1) / nblk;
  nblk = (M + rows_per_block - 1) / rows_per_block;
  return (int)nblk;
}

inline int apply_grid(int64_t nvec) {
  int64_t g = (nvec + 255) / 256;
  const int64_t cap = 256 * 8;  // 8 workgroups per CU, grid-stride the rest
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

}  // namespace

extern "C" {

// Workspace size (floats) for the partial sums of a reduce pass.
int64_t pdt_bn_workspace_floats(int64_t M, int C) {
  int64_t rpb;
  const int nblk = num_reduce_blocks(M, C, rpb);
  return (int64_t)nblk * 2 * C;
}

// Training forward. Outputs: y (bf16), mean/invstd (f32 [C]); updates running stats.
// ws: >= pdt_bn_workspace_floats(M,C) + 2*C floats.
int pdt_bn_fwd_train(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int64_t M,
                     int C, int relu, uint16_t* y, float* mean, float* invstd, float* ws,
                     hipStream_t s) {
  if (C % 8 != 0) return -1;
  int64_t rpb;
  const int nblk = num_reduce_blocks(M, C, rpb);
  const int nchunks = (C + kChunkC - 1) / kChunkC;
  float* part = ws;
  float* a = ws + (int64_t)nblk * 2 * C;
  float* b = a + C;
  hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(nblk, nchunks), dim3(kThreads), 0, s, x, nullptr, nullptr,
                     nullptr, M, C, rpb, part);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, s, part, nblk, C, M, x,
                     gamma, beta, mean, invstd, a, b, running_mean, running_var, momentum, eps);
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec);
#define PDT_APPLY(RL, RS) \
  hipLaunchKernelGGL((bn_apply_kernel<RL, RS>), dim3(grid), dim3(256), 0, s, x, res, a, b, y, nvec, C, fixed)
  if (relu && res) PDT_APPLY(true, true);
  else if (relu) PDT_APPLY(true, false);
  else if (res) PDT_APPLY(false, true);
  else PDT_APPLY(false, false);
  return 0;
}

// Eval forward with running statistics. ws: >= 2*C floats.
int pdt_bn_fwd_eval(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                    const float* running_mean, const float* running_var, float eps, int64_t M, int C,
                    int relu, uint16_t* y, float* ws, hipStream_t s) {
  if (C % 8 != 0) return -1;
  float* a = ws;
  float* b = ws + C;
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta,
                     running_mean, running_var, eps, a, b);
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec);
  if (relu && res) PDT_APPLY(true, true);
  else if (relu) PDT_APPLY(true, false);
  else if (res) PDT_APPLY(false, true);
  else PDT_APPLY(false, false);
#undef PDT_APPLY
  return 0;
}

// Training backward. y is the forward OUTPUT (used for the relu mask when relu != 0).
// Outputs dx (bf16), dres (bf16, when has_res), dgamma/dbeta (f32 [C]).
// ws: >= pdt_bn_workspace_floats(M,C) + 3*C floats.
int pdt_bn_bwd_train(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* gamma,
                     const float* mean, const float* invstd, int64_t M, int C, int relu, int has_res,
                     uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, float* ws, hipStream_t s) {
  if (C % 8 != 0) return -1;
  int64_t rpb;
  const int nblk = num_reduce_blocks(M, C, rpb);
  const int nchunks = (C + kChunkC - 1) / kChunkC;
  float* part = ws;
  float* A = ws + (int64_t)nblk * 2 * C;
  float* B = A + C;
  float* D = B + C;
  if (relu)
    hipLaunchKernelGGL(bn_reduce_kernel<2>, dim3(nblk, nchunks), dim3(kThreads), 0, s, x, dy, y, mean, M, C,
                       rpb, part);
  else
    hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(nblk, nchunks), dim3(kThreads), 0, s, x, dy, y, mean, M, C,
                       rpb, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, s, part, nblk, C, M, gamma,
                     invstd, dgamma, dbeta, A, B, D);
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec);
#define PDT_BAPPLY(RL, RS)                                                                             \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, RS>), dim3(grid), dim3(256), 0, s, dy, x, y, mean, A, B, D, \
                     dx, dres, nvec, C, fixed)
  if (relu && has_res) PDT_BAPPLY(true, true);
  else if (relu) PDT_BAPPLY(true, false);
  else if (has_res) PDT_BAPPLY(false, true);
  else PDT_BAPPLY(false, false);
#undef PDT_BAPPLY
  return 0;
}

}  // extern "C"
