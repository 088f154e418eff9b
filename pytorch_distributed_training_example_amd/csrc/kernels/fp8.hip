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
//     non-negative so integer order == float order), one atomic per workgroup. 128x64 tiles
//     staged through LDS, persistent grid.
//   fp8_update_scales: one launch per step for ALL fp8 tensors of a model: push amax into the
//     history (shift register), scale = 448 / (max(history) * 2^margin), scale_inv = 1/scale, reset amax.
#include "../common.h"
#include "../fp8_pack.h"
#include "../gelu_math.h"

using namespace pdt;

namespace {

constexpr int kTile = 64;

// ---- the tile engine shared by every cast kernel ----
// A tile is 128 rows x 64 columns. Row-major phase: thread t converts 16 columns (cc = 16 (t & 3))
// of rows t / 4 and t / 4 + 64 (two 32-B loads per row in flight per thread, prefetched one tile
// ahead) and stores the 16 fp8 bytes; the bytes also go to an LDS image of the tile. Transposed
// phase: thread t reads one 4-column word from each row of an 8-row block (rb = t & 15, word
// gq = t / 16), transposes the 8 x 4 bytes in registers and stores 8 B into each of 4 rows of the
// transposed output: the 16 lanes of a word column write 128 contiguous bytes of one out_t row
// (the 64-row version wrote 64-B halves of lines with 16-B stores and ran at 3.4-4.1 TB/s).
// LDS: word g of row r at r * 16 + (g ^ ((r >> 3) & 15)) — the transposed reads then see 2-way
// bank conflicts instead of 16-way.
constexpr int kTM = 128;
__device__ __forceinline__ int t8(int r, int g) { return r * 16 + (g ^ ((r >> 3) & 15)); }

struct Pre {
  uint4 x[2][2], g[2][2];  // [row half][16-B piece]: the operand and (GELU backward) its gradient
};

enum { M_CAST = 0, M_GELU = 1, M_GELU_BWD = 2, M_CAST_SUM = 3 };  // M_CAST_SUM: cast + column sums

template <int MODE>
__device__ __forceinline__ void tile_load(Pre& p, const uint16_t* __restrict__ x, const uint16_t* __restrict__ dg,
                                          int64_t rows, int64_t K, int64_t m0, int64_t k0, int ra, int cc) {
  if (k0 + cc >= K) return;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int64_t row = m0 + ra + 64 * hh;
    if (row < rows) {
      const int64_t off = row * K + k0 + cc;
      p.x[hh][0] = *reinterpret_cast<const uint4*>(x + off);
      p.x[hh][1] = *reinterpret_cast<const uint4*>(x + off + 8);
      if (MODE == M_GELU_BWD) {
        p.g[hh][0] = *reinterpret_cast<const uint4*>(dg + off);
        p.g[hh][1] = *reinterpret_cast<const uint4*>(dg + off + 8);
      }
    }
  }
}

// rows: rows of this tile's range that exist (M, or the end of a row chunk); M: out_t's row length.
template <int MODE>
__device__ __forceinline__ void tile_emit(const Pre& p, const float* bl, float s, int tanh_form, int64_t rows,
                                          int64_t M, int64_t K, int64_t m0, int64_t k0, int ra, int cc,
                                          uint8_t* __restrict__ out, uint8_t* __restrict__ out_t, uint32_t* lds,
                                          float& am, float (&cs)[16], int probe) {
  const bool colok = k0 + cc < K;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int64_t row = m0 + ra + 64 * hh;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (row < rows && colok) {
      float v[16], g[16];
      ld8_bf16(reinterpret_cast<const uint16_t*>(&p.x[hh][0]), *reinterpret_cast<float(*)[8]>(v));
      ld8_bf16(reinterpret_cast<const uint16_t*>(&p.x[hh][1]), *reinterpret_cast<float(*)[8]>(v + 8));
      if (MODE == M_GELU_BWD) {
        ld8_bf16(reinterpret_cast<const uint16_t*>(&p.g[hh][0]), *reinterpret_cast<float(*)[8]>(g));
        ld8_bf16(reinterpret_cast<const uint16_t*>(&p.g[hh][1]), *reinterpret_cast<float(*)[8]>(g + 8));
      }
      float b[16];  // the strip's bias (GELU modes), from LDS: 16 VGPRs fewer through the tile loop
      if (MODE == M_GELU || MODE == M_GELU_BWD) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(b + 4 * q) = reinterpret_cast<const float4*>(bl + cc)[q];
      }
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        if (MODE == M_GELU) {
          const gf2 r = gelu2(gf2{v[j] + b[j], v[j + 1] + b[j + 1]}, tanh_form);
          v[j] = bf2f(f2bf(r.x));
          v[j + 1] = bf2f(f2bf(r.y));
        } else if (MODE == M_GELU_BWD) {
          const gf2 a = gf2{g[j], g[j + 1]} * gelu_grad2(gf2{v[j] + b[j], v[j + 1] + b[j + 1]}, tanh_form);
          cs[j] += a.x;
          cs[j + 1] += a.y;
          v[j] = bf2f(f2bf(a.x));
          v[j + 1] = bf2f(f2bf(a.y));
        } else if (MODE == M_CAST_SUM) {
          cs[j] += v[j];
          cs[j + 1] += v[j + 1];
        }
        am = fmaxf(am, fabsf(v[j]));
        am = fmaxf(am, fabsf(v[j + 1]));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[q] = pack4_fp8(v[4 * q] * s, v[4 * q + 1] * s, v[4 * q + 2] * s, v[4 * q + 3] * s);
      if (!(probe & 2)) *reinterpret_cast<uint4*>(out + row * K + k0 + cc) = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) lds[t8(ra + 64 * hh, (cc >> 2) + q)] = w[q];
  }
  __syncthreads();
  const int rb = threadIdx.x & 15, gq = threadIdx.x >> 4;
  if (!(probe & 1) && m0 + rb * 8 < rows && k0 + 4 * gq < K) {  // rows and K are multiples of 8 / 16: whole blocks
    uint32_t wv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[i] = lds[t8(rb * 8 + i, gq)];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = byte_col(wv[0], wv[1], wv[2], wv[3], j), hi = byte_col(wv[4], wv[5], wv[6], wv[7], j);
      *reinterpret_cast<uint2*>(out_t + (k0 + 4 * gq + j) * M + m0 + rb * 8) = make_uint2(lo, hi);
    }
  }
  __syncthreads();  // the LDS image is rewritten by the next tile
}

// amax: the state row. Striped rows (Fp8State, fp8_pack.h kAmaxStripes) take workgroup b's maximum
// in stripe b % 16 (64-B apart, 16 L2 lines): one amax word took every workgroup's atomic in turn,
// ~7 ns each — 8.6 us of a 23 us cast over 1,182 workgroups (profiles/r5/fp8_amax_atomics.txt).
__device__ __forceinline__ void amax_commit(float am, float* red, float* amax, int striped, int wg) {
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f && amax) atomicMax(reinterpret_cast<int*>(amax_slot(amax, striped, wg)), __float_as_int(bm));
  }
}

// Plain cast over tiles tb, tb + step, ... of a bf16 [M, K] tensor (k tiles fastest).
__device__ __forceinline__ void cast_tiles(const uint16_t* __restrict__ x, int64_t M, int64_t K, float s,
                                           uint8_t* __restrict__ out, uint8_t* __restrict__ out_t, float* amax,
                                           int striped, int64_t tb, int64_t step, uint32_t* lds, float* red) {
  const int64_t ntk = (K + kTile - 1) / kTile, ntiles = ntk * ((M + kTM - 1) / kTM);
  const int ra = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
  float am = 0.f, cs[16];
  Pre p;
  if (tb < ntiles) tile_load<M_CAST>(p, x, nullptr, M, K, (tb / ntk) * kTM, (tb % ntk) * kTile, ra, cc);
  for (int64_t t = tb; t < ntiles; t += step) {
    const int64_t m0 = (t / ntk) * kTM, k0 = (t % ntk) * kTile;
    const Pre cur = p;
    if (t + step < ntiles)
      tile_load<M_CAST>(p, x, nullptr, M, K, ((t + step) / ntk) * kTM, ((t + step) % ntk) * kTile, ra, cc);
    tile_emit<M_CAST>(cur, nullptr, s, 0, M, M, K, m0, k0, ra, cc, out, out_t, lds, am, cs, striped >> 1);
  }
  amax_commit(am, red, amax, striped & 1, (int)tb);
}

// Persistent grid over 128x64 tiles (grid-stride); amax kept in registers and committed with one
// atomic per workgroup (a per-wave atomic on the single amax word serialises in L2 — 19k atomics on
// a ViT activation cost ~250 us). Requires M % 16 == 0 and K % 16 == 0.
__global__ __launch_bounds__(256) void fp8_cast_transpose_kernel(const uint16_t* __restrict__ x, int64_t M, int64_t K,
                                                                 const float* __restrict__ scale,
                                                                 uint8_t* __restrict__ out,
                                                                 uint8_t* __restrict__ out_t,
                                                                 float* __restrict__ amax, int striped) {
  __shared__ uint32_t lds[kTM * 16];
  __shared__ float red[4];
  cast_tiles(x, M, K, *scale, out, out_t, amax, striped, blockIdx.x, gridDim.x, lds, red);
}

// The MLP's activation in fp8, produced where it is computed (fp8.py _Fp8MlpFn):
//   forward  (MODE = M_GELU):     g  = gelu(h + bias)        -> g  as e4m3 [M, D] + its transpose
//   backward (MODE = M_GELU_BWD): dh = dg * gelu'(h + bias)  -> dh as e4m3 [M, D] + its transpose,
//                                                               and sum_m dh (bias gradient partials)
// Unfused, each was a bias+GELU strip kernel writing a bf16 [M, D] tensor and a cast-transpose pass
// reading it back: 2 x 2 B of traffic per element less here (ViT-B/16: [25216, 3072] per block).
// The value quantized is the bf16-rounded activation, exactly what the unfused chain quantized
// (same gelu_math.h functions, same scale product), so gq / dhq are bit-identical to it; the bias
// gradient sums the unrounded fp32 dh, as the strip kernel does (different summation order).
// A workgroup owns one 64-column strip and a chunk of 128-row tiles: the bias and the column sums
// stay in registers. D % 64 == 0, M % 16 == 0.
template <int MODE>
__global__ __launch_bounds__(256) void fp8_gelu_cast_kernel(const uint16_t* __restrict__ h,
                                                            const uint16_t* __restrict__ dg,
                                                            const float* __restrict__ bias, int64_t M, int D,
                                                            int rows_per_chunk, int tanh_form,
                                                            const float* __restrict__ scale,
                                                            uint8_t* __restrict__ out, uint8_t* __restrict__ out_t,
                                                            float* __restrict__ amax, float* __restrict__ part,
                                                            int striped) {
  constexpr bool BWD = MODE == M_GELU_BWD || MODE == M_CAST_SUM;  // column partial sums
  __shared__ uint32_t lds[kTM * 16];
  __shared__ float red[4];
  __shared__ float cred[4][BWD ? kTile : 1];
  __shared__ __attribute__((aligned(16))) float bl[kTile];
  const int ra = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
  const int64_t k0 = (int64_t)blockIdx.x * kTile;
  const int64_t mbeg = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t mend = min(M, mbeg + rows_per_chunk);
  const float s = *scale;
  float cs[16], am = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) cs[j] = 0.f;
  if (threadIdx.x < kTile) bl[threadIdx.x] = (MODE != M_CAST_SUM && bias) ? bias[k0 + threadIdx.x] : 0.f;
  __syncthreads();
  Pre p;
  tile_load<MODE>(p, h, dg, mend, D, mbeg, k0, ra, cc);
  for (int64_t m0 = mbeg; m0 < mend; m0 += kTM) {
    const Pre cur = p;
    if (m0 + kTM < mend) tile_load<MODE>(p, h, dg, mend, D, m0 + kTM, k0, ra, cc);
    tile_emit<MODE>(cur, bl, s, tanh_form, mend, M, D, m0, k0, ra, cc, out, out_t, lds, am, cs, striped >> 1);
  }
  if constexpr (BWD) {  // column sums: lanes with equal (lane & 3) share the columns; fixed butterfly order
#pragma unroll
    for (int j = 0; j < 16; ++j) {
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) cs[j] += __shfl_xor(cs[j], o, 64);
    }
    if ((threadIdx.x & 63) < 4) {
#pragma unroll
      for (int j = 0; j < 16; ++j) cred[threadIdx.x >> 6][cc + j] = cs[j];
    }
    __syncthreads();
    if (threadIdx.x < kTile)
      part[(int64_t)blockIdx.y * D + k0 + threadIdx.x] =
          (cred[0][threadIdx.x] + cred[1][threadIdx.x]) + (cred[2][threadIdx.x] + cred[3][threadIdx.x]);
  }
  amax_commit(am, red, amax, striped & 1, blockIdx.y * gridDim.x + blockIdx.x);
}

// Row chunks of whole 128-row tiles so that strips x chunks ~ one resident wave of workgroups: 1024
// for the forward (4 per CU), 768 for the backward (162 VGPRs: 3 per CU) — a second partial round
// of workgroups would run at a fraction of the occupancy.
inline int gelu_cast_chunks(int64_t M, int D, bool bwd, int& rpc) {
  const int64_t tiles = (M + kTM - 1) / kTM, strips = D / kTile;
  int64_t n = (bwd ? 768 : 1024) / strips;
  if (n > tiles) n = tiles;
  if (n < 1) n = 1;
  rpc = (int)(((tiles + n - 1) / n) * kTM);
  return (int)((M + rpc - 1) / rpc);
}

// (the same kernel with MODE = M_CAST_SUM is the cast of a Linear's output gradient dy that also
// yields the bias gradient sum_m dy: the separate column-strip pass over dy is gone.)

// Weight casts of a whole model in one launch: a table of tensors, one workgroup range per tensor
// (each runs the cast tile loop over its own tiles). A step casts every fp8 Linear's weight once
// (48 tensors on ViT-B/16): one launch instead of 48 launches of a few microseconds.
struct CastJob {
  const uint16_t* x;
  uint8_t* out;
  uint8_t* out_t;
  float* st;  // state row: amax, scale, ...
  int M, K, striped;
  int blk0;   // first workgroup of this job
};
constexpr int kMaxJobs = 64;
struct CastTable {
  CastJob j[kMaxJobs];
  int n;
};

__global__ __launch_bounds__(256) void fp8_cast_multi_kernel(CastTable tab) {
  __shared__ uint32_t lds[kTM * 16];
  __shared__ float red[4];
  int ji = 0;
  for (int q = 1; q < tab.n; ++q)
    if ((int)blockIdx.x >= tab.j[q].blk0) ji = q;
  const CastJob& J = tab.j[ji];
  const int nb = (ji + 1 < tab.n ? tab.j[ji + 1].blk0 : (int)gridDim.x) - J.blk0;
  cast_tiles(J.x, J.M, J.K, J.st[1], J.out, J.out_t, J.st, J.striped, blockIdx.x - J.blk0, nb, lds, red);
}

// state rows: [amax_cur, scale, scale_inv, hist_0 .. hist_{L-1}] per tensor (stride 3 + L floats), or
// striped (fp8_pack.h): [amax_cur, scale, scale_inv, pad, 16 amax stripes 16 floats apart, hist...]
// (stride kAmaxHist + L). The history is a shift register (newest first), so no ring position has to
// live on the host — the update is identical on every replay of a captured step.
__global__ void fp8_update_scales_kernel(float* __restrict__ state, int n, int L, float margin_scale, int striped) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int h0 = striped ? kAmaxHist : 3;
  float* st = state + (int64_t)i * (h0 + L);
  float cur = st[0];
  if (striped) {
#pragma unroll
    for (int j = 0; j < kAmaxStripes; ++j) {
      cur = fmaxf(cur, st[kAmaxStripe0 + j * kAmaxStripeStride]);
      st[kAmaxStripe0 + j * kAmaxStripeStride] = 0.f;
    }
  }
  float m = cur;
  for (int j = L - 1; j > 0; --j) {
    st[h0 + j] = st[h0 + j - 1];
    m = fmaxf(m, st[h0 + j]);
  }
  st[h0] = cur;
  if (m > 0.f && isfinite(m)) {
    const float sc = kE4M3Max / (m * margin_scale);
    st[1] = sc;
    st[2] = 1.f / sc;
  }
  st[0] = 0.f;
}

}  // namespace

// diagnosis only: PDT_FP8_AMAX_PROBE=1 drops the amax atomics (times their cost; scales go stale)
inline bool amax_probe() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_FP8_AMAX_PROBE");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}
// diagnosis only: PDT_FP8_STORE_PROBE = 1 skips the transposed stores, 2 the row-major ones (bits of the
// kernels' flags argument above the stripe bit)
inline int store_probe() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PDT_FP8_STORE_PROBE");
    v = (e && e[0]) ? (int)strtol(e, nullptr, 10) & 3 : 0;
  }
  return v << 1;
}

extern "C" {

int pdt_fp8_cast_transpose(const uint16_t* x, int64_t M, int64_t K, const float* scale, uint8_t* out,
                           uint8_t* out_t, float* amax, int striped, hipStream_t s) {
  if (M % 16 != 0 || K % 16 != 0) return -1;
  if (M == 0 || K == 0) return 0;
  const int64_t ntiles = ((K + kTile - 1) / kTile) * ((M + kTM - 1) / kTM);
  // every workgroup resident at once (74 VGPRs: 6 per CU) with an equal tile count each
  const int64_t per = (ntiles + 1535) / 1536;
  const unsigned grid = (unsigned)((ntiles + per - 1) / per);
  hipLaunchKernelGGL(fp8_cast_transpose_kernel, dim3(grid), dim3(256), 0, s, x, M, K, scale, out, out_t,
                     amax_probe() ? nullptr : amax, striped | store_probe());
  return 0;
}

int64_t pdt_fp8_gelu_cast_workspace_floats(int64_t M, int D) {
  if (D % kTile != 0 || M <= 0) return 0;
  int rpc;
  return (int64_t)gelu_cast_chunks(M, D, true, rpc) * D;
}

// bwd = 0: out = fp8(gelu(h + bias)); bwd = 1: out = fp8(dg * gelu'(h + bias)) and part[nchunk][D]
// = per-chunk column sums of it (fp32, unrounded). out_t = the transpose. Returns the chunk count
// (>= 1), or < 0 when the shape is not served (D % 64, M % 16).
int pdt_fp8_gelu_cast(const uint16_t* h, const uint16_t* dg, const float* bias, int64_t M, int D, int tanh_form,
                      const float* scale, uint8_t* out, uint8_t* out_t, float* amax, float* part, int striped,
                      hipStream_t s) {
  if (D % kTile != 0 || M % 16 != 0 || M <= 0 || D <= 0) return -1;
  if (dg && !part) return -1;
  int rpc;
  const int nchunk = gelu_cast_chunks(M, D, dg != nullptr, rpc);
  const dim3 grid(D / kTile, nchunk);
  if (dg)
    hipLaunchKernelGGL(fp8_gelu_cast_kernel<M_GELU_BWD>, grid, dim3(256), 0, s, h, dg, bias, M, D, rpc, tanh_form, scale,
                       out, out_t, amax_probe() ? nullptr : amax, part, striped | store_probe());
  else
    hipLaunchKernelGGL(fp8_gelu_cast_kernel<M_GELU>, grid, dim3(256), 0, s, h, dg, bias, M, D, rpc, tanh_form, scale,
                       out, out_t, amax_probe() ? nullptr : amax, part, striped | store_probe());
  return nchunk;
}

// x bf16 [M, D] -> fp8 + transpose (scale, amax as pdt_fp8_cast_transpose) and part[nchunk][D] =
// per-chunk column sums of x (fp32). Returns the chunk count, or < 0 (D % 64, M % 16).
int pdt_fp8_cast_colsum(const uint16_t* x, int64_t M, int D, const float* scale, uint8_t* out, uint8_t* out_t,
                        float* amax, float* part, int striped, hipStream_t s) {
  if (D % kTile != 0 || M % 16 != 0 || M <= 0 || D <= 0 || !part) return -1;
  int rpc;
  const int nchunk = gelu_cast_chunks(M, D, true, rpc);
  hipLaunchKernelGGL(fp8_gelu_cast_kernel<M_CAST_SUM>, dim3(D / kTile, nchunk), dim3(256), 0, s, x, nullptr, nullptr,
                     M, D, rpc, 0, scale, out, out_t, amax_probe() ? nullptr : amax, part, striped | store_probe());
  return nchunk;
}

// n bf16 [M_i, K_i] tensors -> fp8 row-major + transposed copies, scaled by their state rows, amax
// folded in; one launch. Returns 0, or < 0 when a shape is not served.
int pdt_fp8_cast_multi(int n, const uint16_t* const* x, const int* M, const int* K, float* const* st,
                       const int* striped, uint8_t* const* out, uint8_t* const* out_t, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kMaxJobs) return -2;
  CastTable tab;
  tab.n = n;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] % 16 != 0 || K[i] % 16 != 0 || M[i] <= 0 || K[i] <= 0) return -1;
    const int64_t tiles = (int64_t)((K[i] + kTile - 1) / kTile) * ((M[i] + kTM - 1) / kTM);
    tab.j[i] = CastJob{x[i], out[i], out_t[i], st[i], M[i], K[i], striped[i], blk};
    blk += (int)(tiles < 64 ? tiles : 64);  // <= 64 workgroups per tensor, tiles grid-strided
  }
  hipLaunchKernelGGL(fp8_cast_multi_kernel, dim3(blk), dim3(256), 0, s, tab);
  return 0;
}

int pdt_fp8_update_scales(float* state, int n, int L, float margin_scale, int striped, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(fp8_update_scales_kernel, dim3((n + 255) / 256), dim3(256), 0, s, state, n, L, margin_scale,
                     striped);
  return 0;
}

}  // extern "C"
