// FP8 (OCP e4m3fn, gfx950) training casts with delayed per-tensor scaling.
//
// BASELINE.json config 3 ("ViT-B/16 DDP + AMP (bf16/fp8)"). Not in the reference (LeNet, fp32).
// gfx950's fp8 is the OCP encoding (e4m3fn: max 448, has NaN, no inf) — NOT MI300's fnuz
// (cdna_hip_programming.md §4). hipBLASLt's fp8 GEMMs on gfx950 run 1.4-2.3x the bf16 rate on
// ViT/GPT-2 linear shapes (tools/fp8_bench.py), so every Linear's three GEMMs (fwd, dgrad,
// wgrad) take fp8 operands; the casts are the memory-bound part and live here:
//
//   fp8_cast_transpose: one pass over a bf16 [M, K] tensor writes BOTH the row-major fp8 copy
//     and its transpose (the operand layouts hipBLASLt needs for the fwd / dgrad / wgrad GEMMs),
//     scales by the tensor's current scale (read from device memory: capture-safe, no host sync)
//     and folds |x|max into the tensor's amax slot (atomicMax on the float bits — the values are
//     non-negative so integer order == float order), one atomic per workgroup. 64x64 tiles
//     staged through LDS, persistent grid.
//   fp8_update_scales: one launch per step for ALL fp8 tensors of a model: push amax into the
//     history (shift register), scale = 448 / (max(history) * 2^margin), scale_inv = 1/scale, reset amax.
#include "../common.h"
#include "../gelu_math.h"

using namespace pdt;

namespace {

constexpr float kE4M3Max = 448.f;
constexpr int kTile = 64;

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, kE4M3Max, -kE4M3Max);
  b = __builtin_amdgcn_fmed3f(b, kE4M3Max, -kE4M3Max);
  c = __builtin_amdgcn_fmed3f(c, kE4M3Max, -kE4M3Max);
  d = __builtin_amdgcn_fmed3f(d, kE4M3Max, -kE4M3Max);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);  // bytes 0,1
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);        // bytes 2,3
  return (uint32_t)w;
}

// Persistent grid over 64x64 tiles (grid-stride); 256 threads; thread t handles row t/4 of a tile,
// 16 columns. amax is kept in registers across tiles and reduced once per workgroup: one atomic
// per workgroup (a per-wave atomic on the single amax word serialises in L2 — 19k atomics on a
// ViT activation cost ~250 us). Requires M % 16 == 0 and K % 16 == 0.
__global__ __launch_bounds__(256) void fp8_cast_transpose_kernel(const uint16_t* __restrict__ x, int64_t M, int64_t K,
                                                                 const float* __restrict__ scale,
                                                                 uint8_t* __restrict__ out,
                                                                 uint8_t* __restrict__ out_t,
                                                                 float* __restrict__ amax) {
  __shared__ uint32_t tile[kTile][kTile / 4 + 1];  // fp8 bytes, 4 per word, padded rows
  __shared__ float red[4];
  const int64_t ntk = (K + kTile - 1) / kTile, ntiles = ntk * ((M + kTile - 1) / kTile);
  const int r = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
  const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 16;
  const float s = *scale;
  float am = 0.f;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t m0 = (t / ntk) * kTile, k0 = (t % ntk) * kTile;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if ((m0 + r < M) && (k0 + cc < K)) {
      const uint16_t* src = x + (m0 + r) * K + k0 + cc;
      float v[16];
      ld8_bf16(src, *reinterpret_cast<float(*)[8]>(v));
      ld8_bf16(src + 8, *reinterpret_cast<float(*)[8]>(v + 8));
#pragma unroll
      for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[q] = pack4_fp8(v[4 * q] * s, v[4 * q + 1] * s, v[4 * q + 2] * s, v[4 * q + 3] * s);
      *reinterpret_cast<uint4*>(out + (m0 + r) * K + k0 + cc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (out_t) {
#pragma unroll
      for (int q = 0; q < 4; ++q) tile[r][(cc >> 2) + q] = w[q];
      __syncthreads();
      // transposed: thread t writes 16 bytes of row (k0 + t/4) of out_t, i.e. column t/4 of the tile
      if (k0 + c < K && m0 + rr < M) {
        const int wsel = c >> 2, sh = (c & 3) * 8;
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t v = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) v |= ((tile[rr + 4 * q + j][wsel] >> sh) & 0xffu) << (8 * j);
          o[q] = v;
        }
        *reinterpret_cast<uint4*>(out_t + (k0 + c) * M + m0 + rr) = make_uint4(o[0], o[1], o[2], o[3]);
      }
      __syncthreads();  // tile is reused by the next iteration
    }
  }
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (b > 0.f) atomicMax(reinterpret_cast<int*>(amax), __float_as_int(b));
  }
}

// The MLP's activation in fp8, produced where it is computed (fp8.py _Fp8MlpFn):
//   forward  (BWD = false): g  = gelu(h + bias)            -> g  as e4m3 [M, D] + its transpose
//   backward (BWD = true):  dh = dg * gelu'(h + bias)      -> dh as e4m3 [M, D] + its transpose,
//                                                             and sum_m dh (bias gradient partials)
// Unfused, each was a bias+GELU strip kernel writing a bf16 [M, D] tensor and a cast-transpose pass
// reading it back: 2 x 2 B of traffic per element less here (ViT-B/16: [25216, 3072] per block).
// The value quantized is the bf16-rounded activation, exactly what the unfused chain quantized
// (same gelu_math.h functions, same scale product), so gq / dhq are bit-identical to it; the bias
// gradient sums the unrounded fp32 dh, as the strip kernel does (different summation order).
// A workgroup owns one 64-column strip and a chunk of 64-row tiles: the bias and the column sums
// stay in registers; the next tile's operands are loaded before the current tile's transposed write.
// D % 64 == 0, M % 16 == 0.
template <bool BWD>
__global__ __launch_bounds__(256) void fp8_gelu_cast_kernel(const uint16_t* __restrict__ h,
                                                            const uint16_t* __restrict__ dg,
                                                            const float* __restrict__ bias, int64_t M, int D,
                                                            int rows_per_chunk, int tanh_form,
                                                            const float* __restrict__ scale,
                                                            uint8_t* __restrict__ out, uint8_t* __restrict__ out_t,
                                                            float* __restrict__ amax, float* __restrict__ part) {
  __shared__ uint32_t tile[kTile][kTile / 4 + 1];
  __shared__ float red[4];
  __shared__ float cred[4][BWD ? kTile : 1];
  const int r = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
  const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 16;
  const int k0 = blockIdx.x * kTile;
  const int64_t mbeg = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t mend = min(M, mbeg + rows_per_chunk);
  const float s = *scale;
  float b[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) b[j] = bias ? bias[k0 + cc + j] : 0.f;
  float am = 0.f, cs[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) cs[j] = 0.f;
  uint4 hv[2], gv[2];
  auto load = [&](int64_t m0) {
    if (m0 + r < mend) {
      const int64_t off = (m0 + r) * D + k0 + cc;
      hv[0] = *reinterpret_cast<const uint4*>(h + off);
      hv[1] = *reinterpret_cast<const uint4*>(h + off + 8);
      if (BWD) {
        gv[0] = *reinterpret_cast<const uint4*>(dg + off);
        gv[1] = *reinterpret_cast<const uint4*>(dg + off + 8);
      }
    }
  };
  load(mbeg);
  for (int64_t m0 = mbeg; m0 < mend; m0 += kTile) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (m0 + r < mend) {
      float v[16], g[16];
      ld8_bf16(reinterpret_cast<const uint16_t*>(&hv[0]), *reinterpret_cast<float(*)[8]>(v));
      ld8_bf16(reinterpret_cast<const uint16_t*>(&hv[1]), *reinterpret_cast<float(*)[8]>(v + 8));
      if (BWD) {
        ld8_bf16(reinterpret_cast<const uint16_t*>(&gv[0]), *reinterpret_cast<float(*)[8]>(g));
        ld8_bf16(reinterpret_cast<const uint16_t*>(&gv[1]), *reinterpret_cast<float(*)[8]>(g + 8));
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float a;
        if (BWD) {
          a = g[j] * gelu_grad(v[j] + b[j], tanh_form);
          cs[j] += a;
        } else {
          a = gelu_f(v[j] + b[j], tanh_form);
        }
        v[j] = bf2f(f2bf(a));
        am = fmaxf(am, fabsf(v[j]));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[q] = pack4_fp8(v[4 * q] * s, v[4 * q + 1] * s, v[4 * q + 2] * s, v[4 * q + 3] * s);
      *reinterpret_cast<uint4*>(out + (m0 + r) * D + k0 + cc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (m0 + kTile < mend) load(m0 + kTile);  // in flight during the transposed write
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[r][(cc >> 2) + q] = w[q];
    __syncthreads();
    if (m0 + rr < mend) {
      const int wsel = c >> 2, sh = (c & 3) * 8;
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) t |= ((tile[rr + 4 * q + j][wsel] >> sh) & 0xffu) << (8 * j);
        o[q] = t;
      }
      *reinterpret_cast<uint4*>(out_t + (int64_t)(k0 + c) * M + m0 + rr) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
  }
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  if (BWD) {  // column sums: lanes with equal (lane & 3) share the columns; fixed butterfly order
#pragma unroll
    for (int j = 0; j < 16; ++j) {
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) cs[j] += __shfl_xor(cs[j], o, 64);
    }
    if ((threadIdx.x & 63) < 4) {
#pragma unroll
      for (int j = 0; j < 16; ++j) cred[threadIdx.x >> 6][cc + j] = cs[j];
    }
  }
  __syncthreads();
  if constexpr (BWD)
    if (threadIdx.x < kTile) part[(int64_t)blockIdx.y * D + k0 + threadIdx.x] =
        (cred[0][threadIdx.x] + cred[1][threadIdx.x]) + (cred[2][threadIdx.x] + cred[3][threadIdx.x]);
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f) atomicMax(reinterpret_cast<int*>(amax), __float_as_int(bm));
  }
}

// Row chunks of whole 64-row tiles so that strips x chunks ~ 1024 workgroups.
inline int gelu_cast_chunks(int64_t M, int D, int& rpc) {
  const int64_t tiles = (M + kTile - 1) / kTile, strips = D / kTile;
  int64_t n = 1024 / strips;
  if (n > tiles) n = tiles;
  if (n < 1) n = 1;
  rpc = (int)(((tiles + n - 1) / n) * kTile);
  return (int)((M + rpc - 1) / rpc);
}

// Weight casts of a whole model in one launch: a table of tensors, one workgroup-range per tensor
// (each runs fp8_cast_transpose's tile loop over its own tiles). A step casts every fp8 Linear's
// weight once (48 tensors on ViT-B/16): one launch instead of 48 launches of a few microseconds.
struct CastJob {
  const uint16_t* x;
  uint8_t* out;
  uint8_t* out_t;
  float* st;  // state row: amax, scale, ...
  int M, K;
  int blk0;   // first workgroup of this job
};
constexpr int kMaxJobs = 64;
struct CastTable {
  CastJob j[kMaxJobs];
  int n;
};

__global__ __launch_bounds__(256) void fp8_cast_multi_kernel(CastTable tab) {
  __shared__ uint32_t tile[kTile][kTile / 4 + 1];
  __shared__ float red[4];
  int ji = 0;
  for (int q = 1; q < tab.n; ++q)
    if ((int)blockIdx.x >= tab.j[q].blk0) ji = q;
  const CastJob& J = tab.j[ji];
  const int nb = (ji + 1 < tab.n ? tab.j[ji + 1].blk0 : (int)gridDim.x) - J.blk0;
  const int bid = blockIdx.x - J.blk0;
  const int64_t M = J.M, K = J.K;
  const int64_t ntk = (K + kTile - 1) / kTile, ntiles = ntk * ((M + kTile - 1) / kTile);
  const int r = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
  const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 16;
  const float s = J.st[1];
  float am = 0.f;
  for (int64_t t = bid; t < ntiles; t += nb) {
    const int64_t m0 = (t / ntk) * kTile, k0 = (t % ntk) * kTile;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if ((m0 + r < M) && (k0 + cc < K)) {
      const uint16_t* src = J.x + (m0 + r) * K + k0 + cc;
      float v[16];
      ld8_bf16(src, *reinterpret_cast<float(*)[8]>(v));
      ld8_bf16(src + 8, *reinterpret_cast<float(*)[8]>(v + 8));
#pragma unroll
      for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(v[j]));
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[q] = pack4_fp8(v[4 * q] * s, v[4 * q + 1] * s, v[4 * q + 2] * s, v[4 * q + 3] * s);
      *reinterpret_cast<uint4*>(J.out + (m0 + r) * K + k0 + cc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[r][(cc >> 2) + q] = w[q];
    __syncthreads();
    if (k0 + c < K && m0 + rr < M) {
      const int wsel = c >> 2, sh = (c & 3) * 8;
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v |= ((tile[rr + 4 * q + j][wsel] >> sh) & 0xffu) << (8 * j);
        o[q] = v;
      }
      *reinterpret_cast<uint4*>(J.out_t + (k0 + c) * M + m0 + rr) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
  }
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f) atomicMax(reinterpret_cast<int*>(J.st), __float_as_int(bm));
  }
}

// state rows: [amax_cur, scale, scale_inv, hist_0 .. hist_{L-1}] per tensor (stride 3 + L floats).
// The history is a shift register (newest first), so no ring position has to live on the host —
// the update is identical on every replay of a captured step.
__global__ void fp8_update_scales_kernel(float* __restrict__ state, int n, int L, float margin_scale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* st = state + (int64_t)i * (3 + L);
  float m = st[0];
  for (int j = L - 1; j > 0; --j) {
    st[3 + j] = st[3 + j - 1];
    m = fmaxf(m, st[3 + j]);
  }
  st[3] = st[0];
  if (m > 0.f && isfinite(m)) {
    const float sc = kE4M3Max / (m * margin_scale);
    st[1] = sc;
    st[2] = 1.f / sc;
  }
  st[0] = 0.f;
}

}  // namespace

extern "C" {

int pdt_fp8_cast_transpose(const uint16_t* x, int64_t M, int64_t K, const float* scale, uint8_t* out,
                           uint8_t* out_t, float* amax, hipStream_t s) {
  if (M % 16 != 0 || K % 16 != 0) return -1;
  if (M == 0 || K == 0) return 0;
  const int64_t ntiles = ((K + kTile - 1) / kTile) * ((M + kTile - 1) / kTile);
  const unsigned grid = (unsigned)(ntiles < 1024 ? ntiles : 1024);  // 4 workgroups per CU
  hipLaunchKernelGGL(fp8_cast_transpose_kernel, dim3(grid), dim3(256), 0, s, x, M, K, scale, out, out_t, amax);
  return 0;
}

int64_t pdt_fp8_gelu_cast_workspace_floats(int64_t M, int D) {
  if (D % kTile != 0 || M <= 0) return 0;
  int rpc;
  return (int64_t)gelu_cast_chunks(M, D, rpc) * D;
}

// bwd = 0: out = fp8(gelu(h + bias)); bwd = 1: out = fp8(dg * gelu'(h + bias)) and part[nchunk][D]
// = per-chunk column sums of it (fp32, unrounded). out_t = the transpose. Returns the chunk count
// (>= 1), or < 0 when the shape is not served (D % 64, M % 16).
int pdt_fp8_gelu_cast(const uint16_t* h, const uint16_t* dg, const float* bias, int64_t M, int D, int tanh_form,
                      const float* scale, uint8_t* out, uint8_t* out_t, float* amax, float* part, hipStream_t s) {
  if (D % kTile != 0 || M % 16 != 0 || M <= 0 || D <= 0) return -1;
  if (dg && !part) return -1;
  int rpc;
  const int nchunk = gelu_cast_chunks(M, D, rpc);
  const dim3 grid(D / kTile, nchunk);
  if (dg)
    hipLaunchKernelGGL(fp8_gelu_cast_kernel<true>, grid, dim3(256), 0, s, h, dg, bias, M, D, rpc, tanh_form, scale,
                       out, out_t, amax, part);
  else
    hipLaunchKernelGGL(fp8_gelu_cast_kernel<false>, grid, dim3(256), 0, s, h, dg, bias, M, D, rpc, tanh_form, scale,
                       out, out_t, amax, part);
  return nchunk;
}

// n bf16 [M_i, K_i] tensors -> fp8 row-major + transposed copies, scaled by their state rows, amax
// folded in; one launch. Returns 0, or < 0 when a shape is not served.
int pdt_fp8_cast_multi(int n, const uint16_t* const* x, const int* M, const int* K, float* const* st,
                       uint8_t* const* out, uint8_t* const* out_t, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kMaxJobs) return -2;
  CastTable tab;
  tab.n = n;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 16 != 0 || K[i] % 16 != 0 || M[i] <= 0 || K[i] <= 0) return -1;
    const int64_t tiles = (int64_t)((K[i] + kTile - 1) / kTile) * ((M[i] + kTile - 1) / kTile);
    tab.j[i] = CastJob{x[i], out[i], out_t[i], st[i], M[i], K[i], blk};
    blk += (int)(tiles < 64 ? tiles : 64);  // <= 64 workgroups per tensor, tiles grid-strided
  }
  hipLaunchKernelGGL(fp8_cast_multi_kernel, dim3(blk), dim3(256), 0, s, tab);
  return 0;
}

int pdt_fp8_update_scales(float* state, int n, int L, float margin_scale, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(fp8_update_scales_kernel, dim3((n + 255) / 256), dim3(256), 0, s, state, n, L, margin_scale);
  return 0;
}

}  // extern "C"
