// Channels-last (NHWC) bf16 BatchNorm for gfx950, training + eval, with fused ReLU and
// fused residual add (ResNet bottleneck tail: relu(bn3(x) + identity)).
//
// Not in the reference (LeNet has no BN, /root/reference/cnn.py:9-23); required by the
// ResNet-50 north-star config (BASELINE.json). Activations are [M = N*H*W, C] bf16 with C
// contiguous.
//
// Forward (train): 2 kernels
//   reduce+finalize : grid (row blocks, C/64 chunks); a lane owns 8 channels (one 16-B load)
//                     of a 64-channel chunk, 32 rows per pass; per-block shifted sums
//                     (Σ(x-k), Σ(x-k)², k = x[0,c]) go to a partial slab, and the LAST block to
//                     arrive for a chunk (agent-scope release → relaxed ticket → agent-scope
//                     acquire, cdna_hip_programming.md §6 G16) reduces the slab in a fixed
//                     order (deterministic) and writes mean / invstd / running stats and the
//                     per-channel affine (a, b) — no separate finalize launch.
//   apply           : y = relu?(x*a + b + residual?) in bf16, plus a 1-bit ReLU mask
//                     (1/16 of y's bytes) so backward never re-reads y.
// Backward (train): 2 kernels, same structure
//   reduce+finalize : Σdz, Σdz(x-mean) with dz = dy·mask → dgamma, dbeta, dx coefficients
//   apply           : dx = A·dz + B·(x-mean) + D (and dres = dz for the residual branch)
#include "../common.h"
#include <algorithm>
#include "../tile_stats.h"

using namespace pdt;

namespace {

constexpr int kThreads = 256;
constexpr int kCC = 64;   // channels per reduce workgroup
constexpr int kL = 8;     // lanes per row (8 channels each)
constexpr int kR = 32;    // rows per pass

struct FinArgs {
  // forward
  const uint16_t* x;          // shift source (row 0)
  const float* gamma;
  const float* beta;
  float* mean_out;
  float* invstd_out;
  float* a_out;
  float* b_out;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  // backward
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* A;
  float* B;
  float* D;
  int64_t M;
};

__device__ __forceinline__ void ld8_f32(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// MODE 0: forward stats. MODE 1: backward, no relu. MODE 2: backward with relu mask.
template <int MODE>
__device__ __forceinline__ void accum_row(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                          const uint8_t* __restrict__ mask, int64_t m, int C, int c,
                                          const float (&k)[8], float (&s1)[8], float (&s2)[8]) {
  float xv[8];
  ld8_bf16(x + m * C + c, xv);
  if (MODE == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = xv[j] - k[j]; s1[j] += d; s2[j] += d * d; }
  } else {
    float g[8];
    ld8_bf16(dy + m * C + c, g);
    if (MODE == 2) {
      const unsigned mb = mask[(m * C + c) >> 3];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = (mb >> j) & 1u ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] += g[j]; s2[j] += g[j] * (xv[j] - k[j]); }
  }
}

// Forward outputs of one channel from its batch mean and (biased) variance: mean / invstd,
// the apply coefficients y = a*x + b, and the running statistics (unbiased variance).
// (fp contraction off here and in fin_fwd_sums: every finalize kernel that inlines these must round
// identically — with contraction the compiler picked different fma pairings in the one- and two-launch
// tile finalizes, and running_var differed in the last bit)
__device__ __forceinline__ void bn_set_fwd(int ch, double mu_d, double var, const FinArgs& fa) {
#pragma clang fp contract(off)
  const int64_t Mt = fa.M;
  var = var < 0.0 ? 0.0 : var;
  const float mu = (float)mu_d;
  const float is = (float)(1.0 / sqrt(var + (double)fa.eps));
  fa.mean_out[ch] = mu;
  fa.invstd_out[ch] = is;
  const float gm = fa.gamma ? fa.gamma[ch] : 1.f, bt = fa.beta ? fa.beta[ch] : 0.f;
  fa.a_out[ch] = gm * is;
  fa.b_out[ch] = bt - mu * gm * is;
  if (fa.running_mean) fa.running_mean[ch] = (1.f - fa.momentum) * fa.running_mean[ch] + fa.momentum * mu;
  if (fa.running_var) {
    const double unb = Mt > 1 ? var * (double)Mt / (double)(Mt - 1) : var;
    fa.running_var[ch] = (1.f - fa.momentum) * fa.running_var[ch] + fa.momentum * (float)unb;
  }
}

// Per-channel finalize from the full sums (S1, S2): forward -> mean/invstd/affine/running stats,
// backward -> dgamma/dbeta and the dx coefficients.
template <int MODE>
__device__ __forceinline__ void bn_finalize(int ch, float S1, float S2, const FinArgs& fa) {
  const int64_t Mt = fa.M;
  if (MODE == 0) {
    const float kk = bf2f(fa.x[ch]);
    const double inv_m = 1.0 / (double)Mt;
    const double d1 = (double)S1 * inv_m;
    bn_set_fwd(ch, (double)kk + d1, (double)S2 * inv_m - d1 * d1, fa);
  } else {
    const float is = fa.invstd[ch];
    const float gm = fa.gamma ? fa.gamma[ch] : 1.f;
    const float db = S1, dg = S2 * is;
    if (fa.dgamma) fa.dgamma[ch] = dg;
    if (fa.dbeta) fa.dbeta[ch] = db;
    const float inv_m = 1.f / (float)Mt;
    fa.A[ch] = gm * is;
    fa.B[ch] = -gm * is * is * dg * inv_m;
    fa.D[ch] = -gm * is * db * inv_m;
  }
}

// ---- deterministic two-level finalize (the v1 single-level and v2 fixed-64-channel reduce kernels
// were measured slower and removed: v2 3.0-3.8 TB/s vs v3's 5.2-5.6, tools/r50_roofline.py).
// Blocks of a chunk are grouped kG at a time: the last block to arrive in a group sums the
// group's slabs (fixed order) into a group slab, and the last group to arrive sums the group
// slabs (fixed order) and finalizes. The serial tail is then <= kG + nrow/kG slab reads instead
// of nrow (512 slabs = 256 KB of cross-XCD reads for C = 64 in v1).
constexpr int kG = 16;

// Sum `n` slabs of 2*kCC floats (stride 2*kCC) in index order into thread tid's column
// (tid < 2*kCC); loads are issued 8 at a time so the cross-XCD round trips overlap.
__device__ __forceinline__ float sum_slabs(const float* __restrict__ base, int n, int tid) {
  float a = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base[(int64_t)(i + u) * (2 * kCC) + tid];
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  for (; i < n; ++i) a += base[(int64_t)i * (2 * kCC) + tid];
  return a;
}

// ---- v3 reduce: wide channel chunks + software-pipelined loads.
// v2 measured 3.0-3.8 TB/s on the ResNet-50 shapes (tools/r50_roofline.py): every lane issued its
// U loads, waited for all of them, accumulated, and only then issued the next U, so the bytes in
// flight per CU fell to zero once per iteration; for C >= 256 each wave also read 8 separate
// 128-B row pieces. v3:
//   * a chunk is CC = min(C, 512) channels, LPR = CC/8 lanes per row, so one wave load instruction
//     always reads 1 KB of contiguous memory (8 rows of C=64, ..., 1 row of C>=512);
//   * the loads of iteration i+1 are issued before iteration i is accumulated (two register
//     sets; the last iteration re-loads valid rows instead of branching around its loads, so
//     hipcc's counted vmcnt waits stay intact — cdna_hip_programming.md §5 item 4(c));
//   * the same deterministic two-level last-arriver finalize as v2, generalised to 2*CC columns.
template <int MODE, int U>
struct RowSet {
  uint4 x[U];
  uint4 g[U];
  uint8_t mk[U];
};

template <int MODE, int U>
__device__ __forceinline__ void load_set(RowSet<MODE, U>& s, const uint16_t* __restrict__ x,
                                         const uint16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                                         int64_t m, int64_t step, int C, int c) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t o = (m + u * step) * C + c;
    s.x[u] = *reinterpret_cast<const uint4*>(x + o);
    if (MODE != 0) s.g[u] = *reinterpret_cast<const uint4*>(dy + o);
    if (MODE == 2) s.mk[u] = mask[o >> 3];
  }
}

__device__ __forceinline__ void unpack8(const uint4& t, float (&v)[8]) {
  const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

template <int MODE, int U>
__device__ __forceinline__ void accum_set(const RowSet<MODE, U>& s, const float (&k)[8], float (&s1)[8],
                                          float (&s2)[8]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float xv[8];
    unpack8(s.x[u], xv);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = xv[j] - k[j]; s1[j] += d; s2[j] = fmaf(d, d, s2[j]); }
    } else {
      float g[8];
      unpack8(s.g[u], g);
      if (MODE == 2) {
        const unsigned mb = s.mk[u];
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = (mb >> j) & 1u ? g[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += g[j]; s2[j] = fmaf(g[j], xv[j] - k[j], s2[j]); }
    }
  }
}

template <int LPR>
__device__ __forceinline__ void sum_slabs3(const float* __restrict__ base, int n, int tid, float (&tot)[4]) {
  constexpr int W = 2 * 8 * LPR;  // floats per slab
  constexpr int NV = (W + kThreads - 1) / kThreads;
#pragma unroll
  for (int q = 0; q < NV; ++q) tot[q] = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int v = tid + q * kThreads;
      if (v < W) {
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = base[(int64_t)(i + u) * W + v];
#pragma unroll
        for (int u = 0; u < 8; ++u) tot[q] += t[u];
      }
    }
  }
  for (; i < n; ++i) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int v = tid + q * kThreads;
      if (v < W) tot[q] += base[(int64_t)i * W + v];
    }
  }
}

template <int MODE, int LPR, int U>
__global__ __launch_bounds__(kThreads) void bn_reduce3_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
    const float* __restrict__ mean, int64_t M, int C, int64_t rows_per_block, int nrow,
    float* __restrict__ part, float* __restrict__ gpart, unsigned* __restrict__ counters, FinArgs fa,
    int split_fin) {
  constexpr int CC = 8 * LPR;            // channels per chunk
  constexpr int R = kThreads / LPR;      // rows per pass
  constexpr int W = 2 * CC;              // floats per slab
  constexpr int NV = (W + kThreads - 1) / kThreads;
  __shared__ __attribute__((aligned(16))) float sm[2 * R * CC + 4];
  const int tid = threadIdx.x;
  const int chunk = blockIdx.y;
  const int l = tid % LPR, r = tid / LPR;
  const int c = chunk * CC + l * 8;
  const int64_t m0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t m1 = min(M, m0 + rows_per_block);
  float k[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (MODE == 0) ld8_bf16(x + c, k);  // shift: row 0 (same for every block)
  else ld8_f32(mean + c, k);
  const int64_t per_it = (int64_t)U * R;
  const int64_t nfull = (m1 - m0) / per_it;
  if (nfull > 0) {
    RowSet<MODE, U> a, b;
    load_set<MODE, U>(a, x, dy, mask, m0 + r, R, C, c);
    for (int64_t it = 0; it < nfull; it += 2) {
      // prefetch it+1 (clamped: the tail re-loads valid rows, never branches around loads)
      const int64_t n1 = it + 1 < nfull ? it + 1 : nfull - 1;
      load_set<MODE, U>(b, x, dy, mask, m0 + n1 * per_it + r, R, C, c);
      accum_set<MODE, U>(a, k, s1, s2);
      if (it + 1 >= nfull) break;
      const int64_t n2 = it + 2 < nfull ? it + 2 : nfull - 1;
      load_set<MODE, U>(a, x, dy, mask, m0 + n2 * per_it + r, R, C, c);
      accum_set<MODE, U>(b, k, s1, s2);
    }
  }
  for (int64_t m = m0 + nfull * per_it + r; m < m1; m += R) {
    RowSet<MODE, 1> t;
    load_set<MODE, 1>(t, x, dy, mask, m, R, C, c);
    accum_set<MODE, 1>(t, k, s1, s2);
  }

  float* d0 = &sm[r * CC + l * 8];
  float* d1 = &sm[R * CC + r * CC + l * 8];
  *reinterpret_cast<float4*>(d0) = make_float4(s1[0], s1[1], s1[2], s1[3]);
  *reinterpret_cast<float4*>(d0 + 4) = make_float4(s1[4], s1[5], s1[6], s1[7]);
  *reinterpret_cast<float4*>(d1) = make_float4(s2[0], s2[1], s2[2], s2[3]);
  *reinterpret_cast<float4*>(d1 + 4) = make_float4(s2[4], s2[5], s2[6], s2[7]);
  __syncthreads();
  const int ngroups = (nrow + kG - 1) / kG;
  const int g = blockIdx.x / kG;
  const int gsize = min(kG, nrow - g * kG);
  float* slabs = part + (int64_t)chunk * nrow * W;
  float* gslabs = gpart + (int64_t)chunk * ngroups * W;
  unsigned* ctr = counters + chunk * (ngroups + 1);
  float tot[4];
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    tot[q] = 0.f;
    const int v = tid + q * kThreads;
    if (v < W) {
      const int which = v / CC, cl = v % CC;
      const float* src = &sm[which * R * CC + cl];
#pragma unroll 4
      for (int rr = 0; rr < R; ++rr) tot[q] += src[rr * CC];
      if (gsize > 1 || split_fin) slabs[(int64_t)blockIdx.x * W + v] = tot[q];
    }
  }
  if (split_fin) return;  // bn_fin_kernel reduces the slabs (next launch on the stream)
  if (gsize > 1) {  // level 1: last arriver of the group of kG blocks
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&ctr[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm[2 * R * CC] = (t == (unsigned)(gsize - 1)) ? 1.f : 0.f;
    }
    __syncthreads();
    if (sm[2 * R * CC] == 0.f) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ctr[g] = 0u;  // self-reset (stream-ordered for the next launch)
    }
    __syncthreads();
    sum_slabs3<LPR>(slabs + (int64_t)g * kG * W, gsize, tid, tot);
  }
  if (ngroups > 1) {  // level 2: last group
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int v = tid + q * kThreads;
      if (v < W) gslabs[(int64_t)g * W + v] = tot[q];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = __hip_atomic_fetch_add(&ctr[ngroups], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm[2 * R * CC + 1] = (t == (unsigned)(ngroups - 1)) ? 1.f : 0.f;
    }
    __syncthreads();
    if (sm[2 * R * CC + 1] == 0.f) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ctr[ngroups] = 0u;
    }
    __syncthreads();
    sum_slabs3<LPR>(gslabs, ngroups, tid, tot);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int v = tid + q * kThreads;
    if (v < W) sm[v] = tot[q];
  }
  __syncthreads();
  for (int ch = tid; ch < CC; ch += kThreads) bn_finalize<MODE>(chunk * CC + ch, sm[ch], sm[CC + ch], fa);
}

// Split finalize (bn_tune variant 5, default): the reduce kernel only writes one slab per block and
// this kernel, next on the stream, sums them. Measured on the ResNet-50 shapes (tools/bn_trace.py):
// the in-kernel last-arriver finalize (agent release fence, ticket, acquire fence, cross-XCD slab
// reads, twice) cost 10-20 us per call on top of 12-160 us of streaming; a kernel boundary plus
// this launch costs a few us. One block per 64 channels, summed in a fixed order (deterministic).
template <int MODE>
__global__ __launch_bounds__(1024) void bn_fin_kernel(const float* __restrict__ part, int nrow, int CC, FinArgs fa) {
  // 1024 threads = 128 columns (S1, S2 of 64 channels) x 8 slab subsets; every thread issues its
  // loads 16 at a time (clamped indices, no branches around loads) so one block's serial part is
  // a few cross-XCD round trips, not nrow/2 of them
  __shared__ float sm[8 * 128];
  const int tid = threadIdx.x;
  const int ch0 = blockIdx.x * 64;
  const int chunk = ch0 / CC, off = ch0 % CC;
  const int W = 2 * CC;
  const int col = tid & 127, j = tid >> 7;
  const int v = (col >> 6) * CC + off + (col & 63);
  const float* base = part + (int64_t)chunk * nrow * W + v;
  float a = 0.f;
  for (int b0 = j; b0 < nrow; b0 += 8 * 16) {
    float t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int b = b0 + 8 * u;
      t[u] = base[(int64_t)(b < nrow ? b : j) * W];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) a += (b0 + 8 * u < nrow) ? t[u] : 0.f;
  }
  sm[j * 128 + col] = a;
  __syncthreads();
  if (tid < 128) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += sm[q * 128 + tid];
    sm[tid] = s;
  }
  __syncthreads();
  if (tid < 64) bn_finalize<MODE>(ch0 + tid, sm[tid], sm[64 + tid], fa);
}

// Statistics from the per-tile partials of a producer kernel's epilogue (conv1x1.hip STATS:
// part = [T][C] tile sums, then [T][C] centred tile sums of squares, tiles of BMt rows). Level 1:
// block (64 channels, tile range) -> double (S, Q) with Q = sum_t (M2_t + S_t^2 / n_t) — the
// between-tile term in double, so E[x^2] - mean^2 never cancels in fp32. Level 2 finalizes.
// CENTRED = false (backward partials: sum dz, sum dz (x - mean)): plain double sums, Q = sum_t q_t.
// NCNT: partial t covers part[2 T C + t] rows (float) instead of BMt (the stem conv's per-wave partials).
// Tiles per level-1 block (PDT_BN_TILES_PER_BLOCK, read once; a multiple of 16): 128. 32 (each of a block's
// 16 row groups sums two tiles, one round of loads, 4x the blocks) measured no faster — 10,874-10,914 vs
// 10,909-10,925 img/s at 128 / GPU graphed, 15,309 vs 15,387 at 1024 (profiles/r5/bn_tiles_per_block.txt):
// the ~5-12 us of these launches is launch / tail latency, not their loads.
int g_tiles_per_block = 0;
inline int tiles_per_block() {
  if (g_tiles_per_block == 0) {
    const char* e = getenv("PDT_BN_TILES_PER_BLOCK");
    const int v = (e && e[0]) ? (int)strtol(e, nullptr, 10) : 128;
    g_tiles_per_block = (v >= 16 && v % 16 == 0) ? v : 128;
  }
  return g_tiles_per_block;
}
int g_tiles_fused = 1;  // pdt_bn_tiles_fused(0): the two-launch finalize (A/B)

template <bool CENTRED, bool NCNT = false>
__global__ __launch_bounds__(1024) void bn_tiles_l1_kernel(const float* __restrict__ part, int T, int BMt, int64_t M,
                                                           int C, double* __restrict__ out, int tpb) {
  __shared__ double sm[2][16][64];
  const int tid = threadIdx.x, cl = tid & 63, j = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int t0 = blockIdx.y * tpb, t1 = min(T, t0 + tpb);
  double S = 0.0, Q = 0.0;
#pragma unroll 4
  for (int t = t0 + j; t < t1; t += 16) {
    const float s = part[(int64_t)t * C + c];
    const float q = part[((int64_t)T + t) * C + c];
    const int64_t rem = M - (int64_t)t * BMt;
    const double n = NCNT ? (double)part[2 * (int64_t)T * C + t] : (double)(rem < BMt ? rem : BMt);
    S += (double)s;
    Q += CENTRED ? (double)q + (n > 0.0 ? (double)s * (double)s / n : 0.0) : (double)q;
  }
  sm[0][j][cl] = S;
  sm[1][j][cl] = Q;
  __syncthreads();
  if (j == 0) {
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) { s += sm[0][u][cl]; q += sm[1][u][cl]; }
    out[((int64_t)blockIdx.y * C + c) * 2] = s;
    out[((int64_t)blockIdx.y * C + c) * 2 + 1] = q;
  }
}

// Forward finalize from the double sums S = sum x, Q = sum x^2 (about the tile means, recombined).
__device__ __forceinline__ void fin_fwd_sums(int c, double s, double q, const FinArgs& fa) {
#pragma clang fp contract(off)
  const double inv_m = 1.0 / (double)fa.M;
  const double mu = s * inv_m;
  bn_set_fwd(c, mu, q * inv_m - mu * mu, fa);
}

// The P level-1 entries of channel c in the one-launch finalize's order (bn_tiles_fin_kernel): 16
// strided groups (p = j, j + 16, ...), then the group sums in order — so both paths agree bit for bit.
__device__ __forceinline__ void sum_level1(const double* __restrict__ in, int P, int C, int c, double& s, double& q) {
  s = 0.0;
  q = 0.0;
  for (int j = 0; j < 16; ++j) {
    double sj = 0.0, qj = 0.0;
    for (int p = j; p < P; p += 16) { sj += in[((int64_t)p * C + c) * 2]; qj += in[((int64_t)p * C + c) * 2 + 1]; }
    s += sj;
    q += qj;
  }
}

// Levels 1 + 2 in ONE launch (the finalize was a second ~5 us launch per BatchNorm, 94 per ResNet-50
// step: 0.45 ms at 1024 images, 0.9 ms of a 12.8 ms step at 128): the block of tile range p writes its
// level-1 sums, and the LAST block of its 64-channel column to arrive (release fence, ticket on a
// self-resetting counter, acquire fence — the reduce kernels' pattern) sums the P entries in index
// order and finalizes. P == 1: no ticket. Deterministic: fixed summation order either way.
__device__ unsigned g_tiles_ctr[64];  // one per 64-channel column (C <= 4096), zero at load, self-resetting

template <bool CENTRED, bool NCNT = false>
__global__ __launch_bounds__(1024) void bn_tiles_fin_kernel(const float* __restrict__ part, int T, int BMt, int64_t M,
                                                            int C, double* __restrict__ lv, FinArgs fa, int tpb) {
  __shared__ double sm[2][16][64];
  __shared__ int last;
  const int tid = threadIdx.x, cl = tid & 63, j = tid >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int P = gridDim.y;
  const int t0 = blockIdx.y * tpb, t1 = min(T, t0 + tpb);
  double S = 0.0, Q = 0.0;
#pragma unroll 4
  for (int t = t0 + j; t < t1; t += 16) {
    const float s = part[(int64_t)t * C + c];
    const float q = part[((int64_t)T + t) * C + c];
    const int64_t rem = M - (int64_t)t * BMt;
    const double n = NCNT ? (double)part[2 * (int64_t)T * C + t] : (double)(rem < BMt ? rem : BMt);
    S += (double)s;
    Q += CENTRED ? (double)q + (n > 0.0 ? (double)s * (double)s / n : 0.0) : (double)q;
  }
  sm[0][j][cl] = S;
  sm[1][j][cl] = Q;
  __syncthreads();
  double s = 0.0, q = 0.0;
  if (j == 0) {
#pragma unroll
    for (int u = 0; u < 16; ++u) { s += sm[0][u][cl]; q += sm[1][u][cl]; }
  }
  if (P > 1) {
    if (j == 0) {
      lv[((int64_t)blockIdx.y * C + c) * 2] = s;
      lv[((int64_t)blockIdx.y * C + c) * 2 + 1] = q;
    }
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tk = __hip_atomic_fetch_add(&g_tiles_ctr[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      last = tk == (unsigned)(P - 1);
    }
    __syncthreads();
    if (!last) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      g_tiles_ctr[blockIdx.x] = 0u;
    }
    __syncthreads();
    // the P level-1 entries of the column, combined by all 16 row groups (group j takes p = j, j + 16, ...
    // in order, then group sums in order: a fixed order, deterministic). One thread per channel walking all
    // P entries serially made this tail ~10 us of dependent loads at layer 1 (P = 98).
    // Loads 8 entries at a time (clamped indices, no branch around a load), added in the same p order.
    s = 0.0;
    q = 0.0;
    for (int p0 = j; p0 < P; p0 += 16 * 8) {
      double ts[8], tq[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = min(p0 + 16 * u, P - 1);
        ts[u] = __builtin_nontemporal_load(&lv[((int64_t)p * C + c) * 2]);
        tq[u] = __builtin_nontemporal_load(&lv[((int64_t)p * C + c) * 2 + 1]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + 16 * u < P) {
          s += ts[u];
          q += tq[u];
        }
    }
    sm[0][j][cl] = s;
    sm[1][j][cl] = q;
    __syncthreads();
    if (j != 0) return;
    s = 0.0;
    q = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) { s += sm[0][u][cl]; q += sm[1][u][cl]; }
  } else if (j != 0) {
    return;
  }
  if (CENTRED) {
    fin_fwd_sums(c, s, q, fa);
  } else {
    bn_finalize<1>(c, (float)s, (float)q, fa);
  }
}

__global__ void bn_tiles_l2_kernel(const double* __restrict__ in, int P, int C, FinArgs fa) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s, q;
  sum_level1(in, P, C, c, s, q);
  fin_fwd_sums(c, s, q, fa);
}

// Backward finalize from the level-1 sums: S = sum dz, Q = sum dz (x - mean) -> dgamma / dbeta / A, B, D.
__global__ void bn_tiles_l2b_kernel(const double* __restrict__ in, int P, int C, FinArgs fa) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s, q;
  sum_level1(in, P, C, c, s, q);
  bn_finalize<1>(c, (float)s, (float)q, fa);
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

// Apply passes: grid-stride over 16-B vectors (8 workgroups of 256 per CU), U vectors per thread
// per iteration with all loads issued first. U = 1 is used: U = 4 (apply) / 2 (backward) measured
// 5-10 % SLOWER on the ResNet-50 shapes (tools/bn_trace.py, 822 MB: 350 vs 318 us, 520 vs 469 us).
// RA: the residual is a BatchNorm's INPUT whose apply was deferred to here (ResNet downsample
// shortcut): the added term is ra*res + rb per channel, so that BN's output is never written.
// SubOut (y != null): the output's stride-s subsample [N, Hs, Ws, C] is written as well (the input of the next
// ResNet stage's strided 1x1 shortcut, whose gather pass over y then never runs: ops/conv.py _Conv1x1StridedFn).
struct SubOut {
  uint16_t* y;
  int H, W, Hs, Ws, s;
  float inv_w, inv_h;  // 1 / W, 1 / H (pixel index decomposition in fp32, corrected: exact below 2^24 pixels)
};

__device__ __forceinline__ int div_fix(int v, int d, float inv) {
  int q = (int)((float)v * inv);
  q -= q * d > v ? 1 : 0;
  q += (q + 1) * d <= v ? 1 : 0;
  return q;
}

template <bool RELU, bool RES, bool MASK, int U, bool RA = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const float* __restrict__ a,
    const float* __restrict__ b, uint16_t* __restrict__ y, uint8_t* __restrict__ mask, int64_t nvec, int C,
    int fixed, const float* __restrict__ ra = nullptr, const float* __restrict__ rb = nullptr, SubOut so = SubOut{}) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float av[8], bv[8], rav[8], rbv[8];
  if (fixed && i < nvec) {  // stride % (C/8) == 0: every vector of this thread has the same channels
    const int c = (int)((i * 8) % C);
    ld8_f32(a + c, av);
    ld8_f32(b + c, bv);
    if (RA) { ld8_f32(ra + c, rav); ld8_f32(rb + c, rbv); }
  }
  for (; i < nvec; i += U * stride) {
    uint4 xv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k < nvec) {
        xv[u] = *reinterpret_cast<const uint4*>(x + k * 8);
        if (RES) rv[u] = *reinterpret_cast<const uint4*>(res + k * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k >= nvec) break;
      if (!fixed) {
        const int c = (int)((k * 8) % C);
        ld8_f32(a + c, av);
        ld8_f32(b + c, bv);
        if (RA) { ld8_f32(ra + c, rav); ld8_f32(rb + c, rbv); }
      }
      float v[8], r[8];
      unpack8(xv[u], v);
      if (RES) unpack8(rv[u], r);
      unsigned mb = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = v[j] * av[j] + bv[j];
        if (RES) t += RA ? r[j] * rav[j] + rbv[j] : r[j];
        if (RELU) {
          mb |= (t > 0.f ? 1u : 0u) << j;
          t = t > 0.f ? t : 0.f;
        }
        v[j] = t;
      }
      st8_bf16(y + k * 8, v);
      if (MASK) mask[k] = (uint8_t)mb;
      if (so.y) {  // (uniform) the stride-s subsample too
        const int e = (int)(k * 8);  // (M C < 2^31: checked by the host)
        const int row = e / C, cc = e - row * C;
        const int t = div_fix(row, so.W, so.inv_w), w = row - t * so.W;
        const int n = div_fix(t, so.H, so.inv_h), h = t - n * so.H;
        if (h % so.s == 0 && w % so.s == 0)
          st8_bf16(so.y + (((int64_t)n * so.Hs + h / so.s) * so.Ws + w / so.s) * C + cc, v);
      }
    }
  }
}

template <bool RELU, bool RES, int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint8_t* __restrict__ mask,
    const float* __restrict__ mean, const float* __restrict__ A, const float* __restrict__ B,
    const float* __restrict__ D, uint16_t* __restrict__ dx, uint16_t* __restrict__ dres, int64_t nvec, int C,
    int fixed) {
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
  for (; i < nvec; i += U * stride) {
    uint4 gv[U], xv[U];
    unsigned mk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k < nvec) {
        gv[u] = *reinterpret_cast<const uint4*>(dy + k * 8);
        xv[u] = *reinterpret_cast<const uint4*>(x + k * 8);
        if (RELU) mk[u] = mask[k];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + u * stride;
      if (k >= nvec) break;
      if (!fixed) load_coef(k);
      float g[8], xf[8];
      unpack8(gv[u], g);
      unpack8(xv[u], xf);
      if (RELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = (mk[u] >> j) & 1u ? g[j] : 0.f;
      }
      if (RES) st8_bf16(dres + k * 8, g);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = av[j] * g[j] + bv[j] * (xf[j] - mv[j]) + dv[j];
      st8_bf16(dx + k * 8, o);
    }
  }
}

// ---- ResNet stem: BN apply + ReLU + 3x3/s2/p1 max-pool in one pass (NHWC bf16).
// The [N,112,112,64] BN output is never written: each pooled output applies the BN affine to its
// 3x3 window, keeps the max of the pre-ReLU values (ReLU is monotone: max(relu(z)) = relu(max z))
// and records a 1-byte code per (output, channel): the window index 0..8 of the winner, or 15
// when the max is <= 0 (ReLU kills the gradient). Ties keep the first element in (kh, kw) scan
// order, like aten's max_pool2d.
__global__ __launch_bounds__(256) void bn_apply_pool_kernel(const uint16_t* __restrict__ x,
                                                            const float* __restrict__ a,
                                                            const float* __restrict__ b, uint16_t* __restrict__ y,
                                                            uint8_t* __restrict__ code, int N, int H, int W, int C,
                                                            int Ho, int Wo, int contig) {
  // one workgroup per output row (n, oh), threads over (ow, c8): 32-bit index math per element.
  // contig: a workgroup walks a CONTIGUOUS run of output rows, so the input row two neighbouring
  // windows share (2 oh + 1) is an L2 hit on the workgroup's own XCD (grid-stride rows land on
  // different XCDs and fetch it from HBM twice)
  const int C8 = C >> 3;
  const int per_row = Wo * C8;
  const int64_t nrows = (int64_t)N * Ho;
  const int64_t rper = contig ? (nrows + gridDim.x - 1) / gridDim.x : 1;
  const int64_t rbeg = contig ? (int64_t)blockIdx.x * rper : blockIdx.x;
  const int64_t rend = contig ? std::min<int64_t>(nrows, rbeg + rper) : nrows;
  const int64_t rstep = contig ? 1 : gridDim.x;
  for (int64_t row = rbeg; row < rend; row += rstep) {
   const int oh = (int)(row % Ho);
   const int n = (int)(row / Ho);
   for (int e = threadIdx.x; e < per_row; e += blockDim.x) {
    const int ow = e / C8, c8 = e - ow * C8;
    const int64_t i = row * per_row + e;
    float av[8], bv[8];
    Vec4<float>::ld(a, c8 * 8, *reinterpret_cast<float(*)[4]>(av));
    Vec4<float>::ld(a, c8 * 8 + 4, *reinterpret_cast<float(*)[4]>(av + 4));
    Vec4<float>::ld(b, c8 * 8, *reinterpret_cast<float(*)[4]>(bv));
    Vec4<float>::ld(b, c8 * 8 + 4, *reinterpret_cast<float(*)[4]>(bv + 4));
    float m[8];
    int k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { m[j] = -INFINITY; k[j] = 15; }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        ld8_bf16(x + (((int64_t)n * H + ih) * W + iw) * C + c8 * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float z = fmaf(v[j], av[j], bv[j]);
          if (z > m[j]) { m[j] = z; k[j] = kh * 3 + kw; }
        }
      }
    }
    float o[8];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool pos = m[j] > 0.f;
      o[j] = pos ? m[j] : 0.f;
      const uint32_t cj = pos ? (uint32_t)k[j] : 15u;
      if (j < 4) lo |= cj << (8 * j);
      else hi |= cj << (8 * (j - 4));
    }
    st8_bf16(y + i * 8, o);
    *reinterpret_cast<uint2*>(code + i * 8) = make_uint2(lo, hi);
   }
  }
}

// Gradient of the fused stem w.r.t. the BN output's pre-ReLU value: a gather over the (up to 4)
// pooled windows that contain each input position — every input written exactly once, no atomics,
// fixed summation order.
// BNRED (C == 64): also the stem BatchNorm's backward reduction — sum dz, sum dz (x - mean) of every
// dz it writes (x: the BN input at the same place), per workgroup into part [2][gridDim.x][64] (the
// tiles layout, tile_stats.h): the reduce pass over (dz, x) disappears (bn_bwd_from_partials).
template <bool BNRED>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ code, uint16_t* __restrict__ dz,
                                                          int N, int H, int W, int C, int Ho, int Wo,
                                                          const uint16_t* __restrict__ xb, const float* __restrict__ mean,
                                                          float* __restrict__ part) {
  // one workgroup per input row (n, ih), threads over (iw, c8): 32-bit index math per element
  // (64-bit div/mod per element made this kernel VALU-bound: 545 us at 1.5 TB/s, batch 512)
  const int C8 = C >> 3;
  const int per_row = W * C8;
  float s1[8], s2[8], mu[8];
  if constexpr (BNRED) {  // blockDim 256 is a multiple of C8 = 8: a thread's channel chunk never changes
    const int c8 = threadIdx.x % 8;
    ld8_f32(mean + c8 * 8, mu);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  }
  for (int64_t row = blockIdx.x; row < (int64_t)N * H; row += gridDim.x) {
   const int ih = (int)(row % H);
   const int n = (int)(row / H);
   for (int e = threadIdx.x; e < per_row; e += blockDim.x) {
    const int iw = e / C8, c8 = e - iw * C8;
    const int64_t i = row * per_row + e;
    // the (up to) 2 x 2 pooled windows containing (ih, iw): all loads issued before any use
    // (clamped duplicates count once: window index idx never matches for a duplicate)
    const int oh0 = ih >> 1, oh1 = min(Ho - 1, (ih + 1) >> 1);
    const int ow0 = iw >> 1, ow1 = min(Wo - 1, (iw + 1) >> 1);
    uint2 cw[4];
    uint4 dv[4];
    uint4 xv;
    if constexpr (BNRED) xv = *reinterpret_cast<const uint4*>(xb + i * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = q < 2 ? oh0 : oh1, ow = (q & 1) ? ow1 : ow0;
      const int64_t o = (((int64_t)n * Ho + oh) * Wo + ow) * C + c8 * 8;
      cw[q] = *reinterpret_cast<const uint2*>(code + o);
      dv[q] = *reinterpret_cast<const uint4*>(dy + o);
    }
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = q < 2 ? oh0 : oh1, ow = (q & 1) ? ow1 : ow0;
      const bool dup = (q >= 2 && oh1 == oh0) || ((q & 1) && ow1 == ow0);
      const uint32_t idx = dup ? 0xffu : (uint32_t)((ih - (2 * oh - 1)) * 3 + (iw - (2 * ow - 1)));
      float v[8];
      unpack8(dv[q], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t cj = ((j < 4 ? cw[q].x : cw[q].y) >> (8 * (j & 3))) & 0xffu;
        g[j] += cj == idx ? v[j] : 0.f;
      }
    }
    uint4 st;  // the rounded values the BN backward reads back
    st.x = (uint32_t)f2bf(g[0]) | ((uint32_t)f2bf(g[1]) << 16);
    st.y = (uint32_t)f2bf(g[2]) | ((uint32_t)f2bf(g[3]) << 16);
    st.z = (uint32_t)f2bf(g[4]) | ((uint32_t)f2bf(g[5]) << 16);
    st.w = (uint32_t)f2bf(g[6]) | ((uint32_t)f2bf(g[7]) << 16);
    if (dz) *reinterpret_cast<uint4*>(dz + i * 8) = st;  // null: the reduction only (its consumer re-forms dz)
    if constexpr (BNRED) bn_bwd_accum8(st, xv, 0xffu, mu, s1, s2);
   }
  }
  if constexpr (BNRED) {
    __shared__ float red[4 * 2 * 64];
    bn_bwd_tile_store<64, 4>(s1, s2, red, part, (int)gridDim.x, (int)blockIdx.x, 64, 0);
  }
}

// The same gradient, one thread per 2 x 2 block of input positions (2a + r, 2b + s) and 8 channels:
// the block's positions lie only in the pooled windows (a .. a+1, b .. b+1), so the four (dy, code)
// loads serve four outputs (maxpool_bwd_kernel loads them per position: 4x the load instructions and
// L2 traffic, 980 us at batch 1024 = 4 TB/s). Each position sums its matching windows in the same
// (a, b), (a, b+1), (a+1, b), (a+1, b+1) order, so dz is bit-identical to maxpool_bwd_kernel's.
int g_pool_bwd_v2 = 1;  // pdt_maxpool_bwd_v2(0): maxpool_bwd_kernel (A/B)
// pdt_pool_fwd_contig(1): contiguous row / element runs per workgroup in the stem pool kernels. Measured
// SLOWER than grid-stride (batch 1024: forward 836-850 vs 811 us, gradient 805-818 vs 748 us,
// profiles/r4/pool_bwd_bench_b1024.txt): neighbouring workgroups in flight together share the rows in
// MALL / L2 anyway, and one run per workgroup serialises its rows' latency. Off; kept for the A/B.
int g_pool_contig = 0;

template <bool BNRED>
__global__ __launch_bounds__(256) void maxpool_bwd2_kernel(const uint16_t* __restrict__ dy,
                                                           const uint8_t* __restrict__ code, uint16_t* __restrict__ dz,
                                                           int N, int H, int W, int C, int Ho, int Wo,
                                                           const uint16_t* __restrict__ xb, const float* __restrict__ mean,
                                                           float* __restrict__ part, int contig) {
  const int C8 = C >> 3;
  float s1[8], s2[8], mu[8];
  if constexpr (BNRED) {  // C8 == 8 divides the thread stride: a thread's channel chunk never changes
    ld8_f32(mean + (threadIdx.x % 8) * 8, mu);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  }
  const int64_t total = (int64_t)N * Ho * Wo * C8;
  // contig: a workgroup walks one contiguous run of (a multiple of 256) elements, so the dy / code rows that
  // neighbouring pooled rows share stay in its XCD's L2 (as in bn_apply_pool_kernel)
  const int64_t per = contig ? ((total + gridDim.x - 1) / gridDim.x + 255) / 256 * 256 : 0;
  const int64_t ebeg = contig ? (int64_t)blockIdx.x * per + threadIdx.x : (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t eend = contig ? std::min<int64_t>(total, (int64_t)blockIdx.x * per + per) : total;
  const int64_t estep = contig ? blockDim.x : (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = ebeg; e < eend; e += estep) {
    const int c8 = (int)(e % C8);
    const int64_t pix = e / C8;  // pooled position (n, a, b)
    const int b = (int)(pix % Wo);
    const int64_t na = pix / Wo;
    const int a = (int)(na % Ho), n = (int)(na / Ho);
    const int a1 = min(Ho - 1, a + 1), b1 = min(Wo - 1, b + 1);
    uint2 cw[4];
    uint4 dv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = q < 2 ? a : a1, ow = (q & 1) ? b1 : b;
      const int64_t o = (((int64_t)n * Ho + oh) * Wo + ow) * C + c8 * 8;
      cw[q] = *reinterpret_cast<const uint2*>(code + o);
      dv[q] = *reinterpret_cast<const uint4*>(dy + o);
    }
    uint4 xv[4];
    if constexpr (BNRED) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ih = 2 * a + (t >> 1), iw = 2 * b + (t & 1);
        if (ih < H && iw < W) xv[t] = *reinterpret_cast<const uint4*>(xb + (((int64_t)n * H + ih) * W + iw) * C + c8 * 8);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // input position (2a + r, 2b + s)
      const int r = t >> 1, sc = t & 1;
      const int ih = 2 * a + r, iw = 2 * b + sc;
      if (ih >= H || iw >= W) continue;
      float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dr = q >> 1, ds = q & 1;  // window (a + dr, b + ds)
        if ((dr && !r) || (ds && !sc)) continue;  // (2a, .) lies in window row a only; likewise columns
        if ((dr && a1 == a) || (ds && b1 == b)) continue;  // past the last window (clamped duplicate)
        const uint32_t idx = (uint32_t)((dr ? 0 : r + 1) * 3 + (ds ? 0 : sc + 1));
        float v[8];
        unpack8(dv[q], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t cj = ((j < 4 ? cw[q].x : cw[q].y) >> (8 * (j & 3))) & 0xffu;
          g[j] += cj == idx ? v[j] : 0.f;
        }
      }
      uint4 st;
      st.x = (uint32_t)f2bf(g[0]) | ((uint32_t)f2bf(g[1]) << 16);
      st.y = (uint32_t)f2bf(g[2]) | ((uint32_t)f2bf(g[3]) << 16);
      st.z = (uint32_t)f2bf(g[4]) | ((uint32_t)f2bf(g[5]) << 16);
      st.w = (uint32_t)f2bf(g[6]) | ((uint32_t)f2bf(g[7]) << 16);
      if (dz) *reinterpret_cast<uint4*>(dz + (((int64_t)n * H + ih) * W + iw) * C + c8 * 8) = st;  // null: sums only
      if constexpr (BNRED) bn_bwd_accum8(st, xv[t], 0xffu, mu, s1, s2);
    }
  }
  if constexpr (BNRED) {
    __shared__ float red[4 * 2 * 64];
    bn_bwd_tile_store<64, 4>(s1, s2, red, part, (int)gridDim.x, (int)blockIdx.x, 64, 0);
  }
}

// ---- ResNet head: the global-average-pool gradient dy[n, h, w, c] = bf16(g[n, c] / (H W)) written
// channels_last, with the backward reduction of the BatchNorm whose output was pooled (sum dz, sum dz
// (x - mean), dz = dy * ReLU mask) from the values written: that BatchNorm (the last bn3) skips its
// reduce pass, and the aten broadcast-copy kernel that wrote dy before is gone. Thread chunk c8 =
// tid % C8 is fixed (C8 divides 256); part [2][gridDim.x][C], fixed-order sums (deterministic).
template <bool BNRED>
__global__ __launch_bounds__(256) void gap_bwd_kernel(const uint16_t* __restrict__ g, float scale, int HW, int C,
                                                      int64_t M, uint16_t* __restrict__ dy,
                                                      const uint16_t* __restrict__ xb, const uint8_t* __restrict__ mask,
                                                      const float* __restrict__ mean, float* __restrict__ part) {
  const int C8 = C >> 3;
  float s1[8], s2[8], mu[8];
  if constexpr (BNRED) {  // C8 divides 256 and the stride: e % C8 == threadIdx.x % C8 throughout
    ld8_f32(mean + (threadIdx.x % C8) * 8, mu);
#pragma unroll
    for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  }
  const int64_t total = M * C8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = e / C8;
    const int c8 = (int)(e - m * C8);
    const int n = (int)(m / HW);
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(g + (int64_t)n * C + c8 * 8), v);
    uint4 st;  // the same rounding as bf16 (gy * scale) in PyTorch
    st.x = (uint32_t)f2bf(v[0] * scale) | ((uint32_t)f2bf(v[1] * scale) << 16);
    st.y = (uint32_t)f2bf(v[2] * scale) | ((uint32_t)f2bf(v[3] * scale) << 16);
    st.z = (uint32_t)f2bf(v[4] * scale) | ((uint32_t)f2bf(v[5] * scale) << 16);
    st.w = (uint32_t)f2bf(v[6] * scale) | ((uint32_t)f2bf(v[7] * scale) << 16);
    if constexpr (BNRED) {
      // (xb null: sum-only, the ALG backward derives the centred sum itself; see conv1x1.hip)
      const uint4 xv = xb ? *reinterpret_cast<const uint4*>(xb + e * 8) : make_uint4(0u, 0u, 0u, 0u);
      const unsigned mk = mask ? mask[e] : 0xffu;
      bn_bwd_accum8(st, xv, mk, mu, s1, s2);
      st = mask8(st, mk);  // stored masked, as the 1x1 GEMM's BSTATS epilogue (tile_stats.h mask8)
    }
    *reinterpret_cast<uint4*>(dy + e * 8) = st;
  }
  if constexpr (BNRED) {
    __shared__ float red[256 * 16];
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[threadIdx.x * 16 + j] = s1[j]; red[threadIdx.x * 16 + 8 + j] = s2[j]; }
    __syncthreads();
    if ((int)threadIdx.x < C8) {
      const int c8 = threadIdx.x;
      float t1[8], t2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { t1[j] = 0.f; t2[j] = 0.f; }
      for (int k = threadIdx.x; k < 256; k += C8)
#pragma unroll
        for (int j = 0; j < 8; ++j) { t1[j] += red[k * 16 + j]; t2[j] += red[k * 16 + 8 + j]; }
      const int T = gridDim.x;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        part[(int64_t)blockIdx.x * C + c8 * 8 + j] = t1[j];
        part[((int64_t)T + blockIdx.x) * C + c8 * 8 + j] = t2[j];
      }
    }
  }
}

struct ReduceGeo {
  int nrow, nchunks;
  int64_t rows_per_block;
};

// Reduce-kernel tuning (bn_tune): variant 3/4 = in-kernel last-arriver finalize (4: also the
// centred second pass), 5 = separate finalize kernel; total workgroups targeted per call; rows in
// flight per lane for the forward / backward reduce.
struct BnTune {
  int variant = 5;
  int target_blocks = 512;  // tools/bn_reduce_sweep.py: 2 workgroups per CU beat 4-16 (10.5 vs 11.5+ ms/step)
  int u_fwd = 8;
  int u_bwd = 4;
};
BnTune g_tune;

// v3: chunk = min(C, 512) channels (C is a multiple of 64; chunks must tile C exactly)
inline int chunk3(int C) {
  for (int cc = 512; cc > 64; cc >>= 1)
    if (C % cc == 0) return cc;
  return 64;
}

inline ReduceGeo reduce_geo3(int64_t M, int C, int U) {
  ReduceGeo g;
  const int cc = chunk3(C);
  g.nchunks = C / cc;
  const int R = kThreads / (cc / 8);
  int64_t nrow = g_tune.target_blocks / g.nchunks;
  if (nrow > 1024) nrow = 1024;
  const int64_t max_rows = (M + 2 * (int64_t)U * R - 1) / (2 * (int64_t)U * R);  // >= 2 pipelined iterations
  if (nrow > max_rows) nrow = max_rows;
  if (nrow < 1) nrow = 1;
  g.rows_per_block = (M + nrow - 1) / nrow;
  g.nrow = (int)((M + g.rows_per_block - 1) / g.rows_per_block);
  return g;
}

inline int64_t slab_floats3(const ReduceGeo& g, int C) {
  const int ngroups = (g.nrow + kG - 1) / kG;
  return (int64_t)(g.nrow + ngroups) * 2 * C;  // nchunks * (nrow + ngroups) * 2 * cc
}

// Launch the reduce (+ fused finalize) of MODE; returns the float offset in ws where the
// per-channel coefficient arrays start.
template <int MODE>
int64_t launch_reduce(const uint16_t* x, const uint16_t* dy, const uint8_t* mask, const float* mean, int64_t M,
                      int C, float* ws, unsigned* counters, const FinArgs& fa, hipStream_t s) {
  const int U = MODE == 0 ? g_tune.u_fwd : g_tune.u_bwd;
  {
    const ReduceGeo g = reduce_geo3(M, C, U);
    float* part = ws;
    float* gpart = ws + (int64_t)g.nrow * 2 * C;
    const int cc = chunk3(C);
#define PDT_R3(LPR, UU)                                                                                      \
  hipLaunchKernelGGL((bn_reduce3_kernel<MODE, LPR, UU>), dim3(g.nrow, g.nchunks), dim3(kThreads), 0, s, x, dy, \
                     mask, mean, M, C, g.rows_per_block, g.nrow, part, gpart, counters, fa, g_tune.variant >= 4)
#define PDT_R3U(LPR)              \
  if (U >= 8) PDT_R3(LPR, 8);     \
  else if (U >= 4) PDT_R3(LPR, 4); \
  else PDT_R3(LPR, 2)
    if (cc == 512) { PDT_R3U(64); }
    else if (cc == 256) { PDT_R3U(32); }
    else if (cc == 128) { PDT_R3U(16); }
    else { PDT_R3U(8); }
#undef PDT_R3U
#undef PDT_R3
    if (g_tune.variant == 5)
      hipLaunchKernelGGL(bn_fin_kernel<MODE>, dim3(C / 64), dim3(1024), 0, s, part, g.nrow, cc, fa);
    return slab_floats3(g, C);
  }
}

int g_row_wgs = 16;  // pdt_bn_row_wgs(n): A/B of the stem pool kernels' grid cap (workgroups per CU)

inline int row_grid(int64_t rows) {  // row-wise stem kernels: <= 16 workgroups per CU, grid-stride
  const int64_t cap = 256 * (int64_t)g_row_wgs;
  return (int)(rows < cap ? (rows < 1 ? 1 : rows) : cap);
}

// Workgroups per CU before the apply passes grid-stride (tools/bn_apply_grid_sweep.py, 1024 images, ResNet-50
// shapes): the residual forward apply and the backward apply run fastest at 2 per CU, the plain forward apply
// at 3-4 (8 before: 5-15 % slower, e.g. C = 512 at 28 x 28: residual 715 -> 611 us, backward 804 -> 748 us,
// plain 520 -> 491 us, each with its reduce pass). pdt_bn_apply_wgs(n) forces n for all three (A/B).
enum ApplyKind { kApplyPlain = 0, kApplyRes = 1, kApplyBwd = 2 };
int g_apply_wgs[3] = {4, 2, 2};

inline int apply_grid(int64_t nvec, ApplyKind kind) {
  int64_t g = (nvec + 255) / 256;
  const int64_t cap = 256 * (int64_t)g_apply_wgs[kind];
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

// Backward finalize (from per-tile / per-workgroup partials [2][T][C]: sum dz, sum dz (x - mean)) + apply.
int bn_bwd_from_partials(const float* part, int T, int BMt, const uint16_t* dy, const uint16_t* x,
                         const uint8_t* mask, const float* gamma, const float* mean, const float* invstd, int64_t M,
                         int C, int relu, int has_res, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta,
                         float* ws, hipStream_t s, float* coef = nullptr) {
  if (relu && !mask) return -2;
  const int P = (T + tiles_per_block() - 1) / tiles_per_block();
  double* lv = reinterpret_cast<double*>(ws);
  float* A = coef ? coef : ws + 4 * (int64_t)P * C;  // coef: the caller's [3][C] (A, B, D)
  float* B = A + C;
  float* D = B + C;
  FinArgs fa{};
  fa.gamma = gamma; fa.invstd = invstd; fa.dgamma = dgamma; fa.dbeta = dbeta; fa.A = A; fa.B = B; fa.D = D;
  fa.M = M;
  if (g_tiles_fused && C / 64 <= 64) {
    hipLaunchKernelGGL(bn_tiles_fin_kernel<false>, dim3(C / 64, P), dim3(1024), 0, s, part, T, BMt, M, C, lv, fa, tiles_per_block());
  } else {
    hipLaunchKernelGGL(bn_tiles_l1_kernel<false>, dim3(C / 64, P), dim3(1024), 0, s, part, T, BMt, M, C, lv, tiles_per_block());
    hipLaunchKernelGGL(bn_tiles_l2b_kernel, dim3((C + 255) / 256), dim3(256), 0, s, lv, P, C, fa);
  }
  if (!dx) return 0;  // coefficients only: the consumer applies them (pdt_stem_conv_wgrad_bn)
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec, kApplyBwd);
#define PDT_BAPPLY(RL, RS)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, RS, 1>), dim3(grid), dim3(256), 0, s, dy, x, mask, mean, A, B, D, \
                     dx, dres, nvec, C, fixed)
  if (relu && has_res) PDT_BAPPLY(true, true);
  else if (relu) PDT_BAPPLY(true, false);
  else if (has_res) PDT_BAPPLY(false, true);
  else PDT_BAPPLY(false, false);
#undef PDT_BAPPLY
  return 0;
}

}  // namespace

extern "C" {

// Workspace floats needed by a train fwd/bwd call (partial slabs + per-channel coefficients).
int64_t pdt_bn_workspace_floats(int64_t M, int C) {
  return slab_floats3(reduce_geo3(M, C, 2), C) + 4 * (int64_t)C;  // U = 2 gives the most rows
}

// 1: one-launch tile finalize (bn_tiles_fin_kernel, default); 0: level-1 + level-2 launches.
void pdt_bn_tiles_fused(int on) { g_tiles_fused = on; }

// Select the reduce implementation / grid (benchmarking). Values <= 0 keep the current setting.
void pdt_bn_tune(int variant, int target_blocks, int u_fwd, int u_bwd) {
  if (variant >= 3 && variant <= 5) g_tune.variant = variant;
  if (target_blocks > 0) g_tune.target_blocks = target_blocks;
  if (u_fwd > 0) g_tune.u_fwd = u_fwd;
  if (u_bwd > 0) g_tune.u_bwd = u_bwd;
}

// Training forward. Outputs: y (bf16), mask (uint8, M*C/8, when relu), mean/invstd (f32 [C]);
// updates running stats. counters: >= C/64 zeroed uint32 (self-resetting).
// res_a / res_b (nullable): the residual is a deferred BatchNorm's input, added as res_a*res + res_b.
// y == nullptr: statistics and coefficients only (a, b at ws + pdt_bn_workspace_floats - 4C), no apply.
int pdt_bn_fwd_train(const uint16_t* x, const uint16_t* res, const float* res_a, const float* res_b,
                     const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int64_t M, int C,
                     int relu, uint16_t* y, uint8_t* mask, float* mean, float* invstd, float* ws,
                     unsigned* counters, hipStream_t s) {
  if (C % kCC != 0 || M < 1) return -1;
  // coefficients live at the tail of ws (past the largest slab area)
  float* a = ws + pdt_bn_workspace_floats(M, C) - 4 * (int64_t)C;
  float* b = a + C;
  FinArgs fa{};
  fa.x = x; fa.gamma = gamma; fa.beta = beta; fa.mean_out = mean; fa.invstd_out = invstd; fa.a_out = a;
  fa.b_out = b; fa.running_mean = running_mean; fa.running_var = running_var; fa.momentum = momentum;
  fa.eps = eps; fa.M = M;
  launch_reduce<0>(x, nullptr, nullptr, nullptr, M, C, ws, counters, fa, s);
  if (!y) return 0;
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec, res ? kApplyRes : kApplyPlain);
  const SubOut so{};
#define PDT_APPLY(RL, RS, MK)                                                                                 \
  hipLaunchKernelGGL((bn_apply_kernel<RL, RS, MK, 1>), dim3(grid), dim3(256), 0, s, x, res, a, b, y, mask, \
                     nvec, C, fixed, nullptr, nullptr, so)
#define PDT_APPLY_RA()                                                                                         \
  hipLaunchKernelGGL((bn_apply_kernel<true, true, true, 1, true>), dim3(grid), dim3(256), 0, s, x, res, a, b, y, \
                     mask, nvec, C, fixed, res_a, res_b, so)
  const bool mk = mask != nullptr;
  if (res_a && !(relu && res && mk)) return -3;  // the deferred-residual form exists for relu+res+mask only
  if (res_a) PDT_APPLY_RA();
  else if (relu && res) { if (mk) PDT_APPLY(true, true, true); else PDT_APPLY(true, true, false); }
  else if (relu) { if (mk) PDT_APPLY(true, false, true); else PDT_APPLY(true, false, false); }
  else if (res) PDT_APPLY(false, true, false);
  else PDT_APPLY(false, false, false);
  return 0;
}

// Workspace floats of pdt_bn_fwd_train_tiles.
int64_t pdt_bn_tiles_ws_floats(int T, int C) {
  const int64_t P = (T + tiles_per_block() - 1) / tiles_per_block();
  return 4 * P * C + 2 * (int64_t)C;
}

// Training forward whose statistics come from a producer's per-tile partials (see
// bn_tiles_l1_kernel) instead of a reduce pass over x: finalize (2 small launches) + apply.
int pdt_bn_fwd_train_tiles(const float* part, int T, int BMt, const uint16_t* x, const uint16_t* res,
                           const float* res_a, const float* res_b,
                           const float* gamma, const float* beta, float* running_mean, float* running_var,
                           float momentum, float eps, int64_t M, int C, int relu, uint16_t* y, uint8_t* mask,
                           float* mean, float* invstd, float* ws, hipStream_t s, uint16_t* sub_y, int sub_H,
                           int sub_W, int sub_s) {
  if (C % kCC != 0 || M < 1 || T != (int)((M + BMt - 1) / BMt)) return -1;
  if (sub_y && (sub_s < 2 || sub_H < 1 || sub_W < 1 || M % ((int64_t)sub_H * sub_W) != 0 || M >= (1 << 24) ||
                M * C >= ((int64_t)1 << 31)))
    return -4;  // (the fp32 index decomposition is exact below 2^24 pixels)
  const int P = (T + tiles_per_block() - 1) / tiles_per_block();
  double* lv = reinterpret_cast<double*>(ws);
  float* a = ws + 4 * (int64_t)P * C;
  float* b = a + C;
  FinArgs fa{};
  fa.gamma = gamma; fa.beta = beta; fa.mean_out = mean; fa.invstd_out = invstd; fa.a_out = a;
  fa.b_out = b; fa.running_mean = running_mean; fa.running_var = running_var; fa.momentum = momentum;
  fa.eps = eps; fa.M = M;
  if (g_tiles_fused && C / 64 <= 64) {
    hipLaunchKernelGGL(bn_tiles_fin_kernel<true>, dim3(C / 64, P), dim3(1024), 0, s, part, T, BMt, M, C, lv, fa, tiles_per_block());
  } else {
    hipLaunchKernelGGL(bn_tiles_l1_kernel<true>, dim3(C / 64, P), dim3(1024), 0, s, part, T, BMt, M, C, lv, tiles_per_block());
    hipLaunchKernelGGL(bn_tiles_l2_kernel, dim3((C + 255) / 256), dim3(256), 0, s, lv, P, C, fa);
  }
  if (!y) return 0;
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec, res ? kApplyRes : kApplyPlain);
  const bool mk = mask != nullptr;
  if (res_a && !(relu && res && mk)) return -3;
  const SubOut so = sub_y ? SubOut{sub_y, sub_H, sub_W, (sub_H - 1) / sub_s + 1, (sub_W - 1) / sub_s + 1, sub_s,
                                   1.f / (float)sub_W, 1.f / (float)sub_H}
                          : SubOut{};
  if (res_a) PDT_APPLY_RA();
  else if (relu && res) { if (mk) PDT_APPLY(true, true, true); else PDT_APPLY(true, true, false); }
  else if (relu) { if (mk) PDT_APPLY(true, false, true); else PDT_APPLY(true, false, false); }
  else if (res) PDT_APPLY(false, true, false);
  else PDT_APPLY(false, false, false);
  return 0;
}

// Training forward of the ResNet stem tail: BN statistics (same reduce as pdt_bn_fwd_train), then
// BN apply + ReLU + 3x3/s2/p1 max-pool fused. x: NHWC [N,H,W,C]; y: [N,Ho,Wo,C]; code: N*Ho*Wo*C bytes.
int pdt_bn_relu_maxpool_fwd_train(const uint16_t* x, const float* gamma, const float* beta, float* running_mean,
                                  float* running_var, float momentum, float eps, int N, int H, int W, int C,
                                  uint16_t* y, uint8_t* code, float* mean, float* invstd, float* ws,
                                  unsigned* counters, hipStream_t s) {
  const int64_t M = (int64_t)N * H * W;
  if (C % kCC != 0 || M < 1) return -1;
  // coefficients live at the tail of ws (past the largest slab area)
  float* a = ws + pdt_bn_workspace_floats(M, C) - 4 * (int64_t)C;
  float* b = a + C;
  FinArgs fa{};
  fa.x = x; fa.gamma = gamma; fa.beta = beta; fa.mean_out = mean; fa.invstd_out = invstd; fa.a_out = a;
  fa.b_out = b; fa.running_mean = running_mean; fa.running_var = running_var; fa.momentum = momentum;
  fa.eps = eps; fa.M = M;
  launch_reduce<0>(x, nullptr, nullptr, nullptr, M, C, ws, counters, fa, s);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t nvec = (int64_t)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(bn_apply_pool_kernel, dim3(row_grid((int64_t)N * Ho)), dim3(256), 0, s, x, a, b, y, code, N, H, W, C,
                     Ho, Wo, g_pool_contig);
  return 0;
}

// pdt_bn_relu_maxpool_fwd_train with the statistics from the stem conv's partials (conv_stem.hip
// pdt_stem_conv_fwd_stats: P partials with row counts, C == 64) instead of a reduce pass over x.
// ws: pdt_bn_parts_ws_floats(P, C) floats.
int64_t pdt_bn_parts_ws_floats(int P, int C) { return pdt_bn_tiles_ws_floats(P, C); }

int pdt_bn_relu_maxpool_fwd_train_parts(const float* part, int P, const uint16_t* x, const float* gamma,
                                        const float* beta, float* running_mean, float* running_var, float momentum,
                                        float eps, int N, int H, int W, int C, uint16_t* y, uint8_t* code, float* mean,
                                        float* invstd, float* ws, hipStream_t s) {
  const int64_t M = (int64_t)N * H * W;
  if (C % kCC != 0 || C / 64 > 64 || M < 1 || P < 1) return -1;
  const int PB = (P + tiles_per_block() - 1) / tiles_per_block();
  double* lv = reinterpret_cast<double*>(ws);
  float* a = ws + 4 * (int64_t)PB * C;
  float* b = a + C;
  FinArgs fa{};
  fa.gamma = gamma; fa.beta = beta; fa.mean_out = mean; fa.invstd_out = invstd; fa.a_out = a;
  fa.b_out = b; fa.running_mean = running_mean; fa.running_var = running_var; fa.momentum = momentum;
  fa.eps = eps; fa.M = M;
  // BMt = 1: unused (NCNT) but keeps the kernel's tail arithmetic in range
  hipLaunchKernelGGL((bn_tiles_fin_kernel<true, true>), dim3(C / 64, PB), dim3(1024), 0, s, part, P, 1, M, C, lv, fa, tiles_per_block());
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipLaunchKernelGGL(bn_apply_pool_kernel, dim3(row_grid((int64_t)N * Ho)), dim3(256), 0, s, x, a, b, y, code, N, H, W, C,
                     Ho, Wo, g_pool_contig);
  return 0;
}

// dz [N,H,W,C] (gradient at the BN output, ReLU folded in) from the pooled gradient dy [N,Ho,Wo,C].
int pdt_maxpool3s2_bwd(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                       hipStream_t s) {
  if (C % 8 != 0) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t nvec = (int64_t)N * H * W * (C / 8);
  if (nvec == 0) return 0;
  hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(row_grid((int64_t)N * H)), dim3(256), 0, s, dy, code, dz, N, H, W,
                     C, Ho, Wo, nullptr, nullptr, nullptr);
  return 0;
}

// Eval forward with running statistics. ws: >= 2*C floats.
int pdt_bn_fwd_eval(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                    const float* running_mean, const float* running_var, float eps, int64_t M, int C, int relu,
                    uint16_t* y, float* ws, hipStream_t s) {
  if (C % 8 != 0) return -1;
  float* a = ws;
  float* b = ws + C;
  uint8_t* mask = nullptr;
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, running_mean,
                     running_var, eps, a, b);
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec, res ? kApplyRes : kApplyPlain);
  const SubOut so{};
  if (relu && res) PDT_APPLY(true, true, false);
  else if (relu) PDT_APPLY(true, false, false);
  else if (res) PDT_APPLY(false, true, false);
  else PDT_APPLY(false, false, false);
#undef PDT_APPLY
#undef PDT_APPLY_RA
  return 0;
}

// Training backward. mask: the forward's relu bit-mask (required when relu != 0).
// Outputs dx (bf16), dres (bf16, when has_res), dgamma/dbeta (f32 [C]).
int pdt_bn_bwd_train(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* gamma,
                     const float* mean, const float* invstd, int64_t M, int C, int relu, int has_res,
                     uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, float* ws, unsigned* counters,
                     hipStream_t s) {
  if (C % kCC != 0 || M < 1) return -1;
  if (relu && !mask) return -2;
  float* A = ws + pdt_bn_workspace_floats(M, C) - 4 * (int64_t)C;
  float* B = A + C;
  float* D = B + C;
  FinArgs fa{};
  fa.gamma = gamma; fa.invstd = invstd; fa.dgamma = dgamma; fa.dbeta = dbeta; fa.A = A; fa.B = B; fa.D = D;
  fa.M = M;
  if (relu) launch_reduce<2>(x, dy, mask, mean, M, C, ws, counters, fa, s);
  else launch_reduce<1>(x, dy, mask, mean, M, C, ws, counters, fa, s);
  const int64_t nvec = M * C / 8;
  const int fixed = (2048 % C) == 0;
  const int grid = apply_grid(nvec, kApplyBwd);
#define PDT_BAPPLY(RL, RS)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, RS, 1>), dim3(grid), dim3(256), 0, s, dy, x, mask, mean, A, B, D, \
                     dx, dres, nvec, C, fixed)
  if (relu && has_res) PDT_BAPPLY(true, true);
  else if (relu) PDT_BAPPLY(true, false);
  else if (has_res) PDT_BAPPLY(false, true);
  else PDT_BAPPLY(false, false);
#undef PDT_BAPPLY
  return 0;
}

// Training backward WITHOUT the apply: the reduction (a pass over dy, x, mask) and the finalize into
// coef [3][C] = A, B, D (dx = A dy m + B (x - mean) + D) + dgamma / dbeta, for a consumer that forms
// dx while loading its operand (conv1x1_bwd_fused.hip). ws: pdt_bn_workspace_floats(M, C).
int pdt_bn_bwd_coef(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* gamma, const float* mean,
                    const float* invstd, int64_t M, int C, int relu, float* coef, float* dgamma, float* dbeta, float* ws,
                    unsigned* counters, hipStream_t s) {
  if (C % kCC != 0 || M < 1 || !coef) return -1;
  if (relu && !mask) return -2;
  FinArgs fa{};
  fa.gamma = gamma; fa.invstd = invstd; fa.dgamma = dgamma; fa.dbeta = dbeta;
  fa.A = coef; fa.B = coef + C; fa.D = coef + 2 * C;
  fa.M = M;
  if (relu) launch_reduce<2>(x, dy, mask, mean, M, C, ws, counters, fa, s);
  else launch_reduce<1>(x, dy, mask, mean, M, C, ws, counters, fa, s);
  return 0;
}

// Same from a producer's per-tile partials [2][T][C] (no pass over dy): finalize only.
// ws: pdt_bn_tiles_ws_floats(T, C) floats.
int pdt_bn_bwd_coef_tiles(const float* part, int T, const float* gamma, const float* invstd, int64_t M, int C,
                          float* coef, float* dgamma, float* dbeta, float* ws, hipStream_t s) {
  if (C % kCC != 0 || M < 1 || T < 1 || !coef) return -1;
  return bn_bwd_from_partials(part, T, 1, nullptr, nullptr, nullptr, gamma, nullptr, invstd, M, C, 0, 0, nullptr,
                              nullptr, dgamma, dbeta, ws, s, coef);
}

// Training backward whose reduction (sum dz, sum dz (x - mean), dz = dy * mask) comes from the
// per-tile partials [2][T][C] written by the kernel that produced dy (conv1x1.hip BSTATS): finalize
// (2 small launches) + apply, no reduce pass over (dy, x). ws: pdt_bn_tiles_ws_floats(T, C) + 2C floats.
// The backward partials are plain sums, so T is free (the stride-2 data gradient writes 4 phases of
// ceil(M/4/256) tiles, conv3x3_s2.hip); BMt is unused here.
int pdt_bn_bwd_train_tiles(const float* part, int T, int BMt, const uint16_t* dy, const uint16_t* x,
                           const uint8_t* mask, const float* gamma, const float* mean, const float* invstd, int64_t M,
                           int C, int relu, int has_res, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta,
                           float* ws, hipStream_t s) {
  if (C % kCC != 0 || M < 1 || T < 1) return -1;
  return bn_bwd_from_partials(part, T, BMt, dy, x, mask, gamma, mean, invstd, M, C, relu, has_res, dx, dres, dgamma,
                              dbeta, ws, s);
}

// Workgroups (= BN partial tiles) of pdt_gap_bwd: 0 when the reduction does not apply (C / 8 must divide 256).
int pdt_gap_bwd_parts(int64_t M, int C) {
  if (C % 8 != 0 || C > 2048 || 256 % (C / 8) != 0 || M < 1) return 0;
  return (int)std::min<int64_t>((M * (C / 8) + 255) / 256, 1024);
}

// dy [M = N H W, C] channels_last from g [N, C] (bf16) scaled by 1 / (H W); with xb (the pooled BatchNorm's
// input), its ReLU mask (or null) and mean: that BatchNorm's backward partials into part [2][T][C],
// T = pdt_gap_bwd_parts(M, C).
int pdt_gap_bwd(const uint16_t* g, int N, int HW, int C, uint16_t* dy, const uint16_t* xb, const uint8_t* mask,
                const float* mean, float* part, hipStream_t s) {
  const int64_t M = (int64_t)N * HW;
  if (C % 8 != 0 || M < 1) return -1;
  const float scale = (float)(1.0 / (double)HW);
  if (part) {  // the pooled BatchNorm's backward partials (xb null: sum-only)
    const int T = pdt_gap_bwd_parts(M, C);
    if (T == 0 || !mean) return -2;
    hipLaunchKernelGGL(gap_bwd_kernel<true>, dim3(T), dim3(256), 0, s, g, scale, HW, C, M, dy, xb, mask, mean, part);
  } else {
    const int grid = (int)std::min<int64_t>((M * (C / 8) + 255) / 256, 4096);
    hipLaunchKernelGGL(gap_bwd_kernel<false>, dim3(grid), dim3(256), 0, s, g, scale, HW, C, M, dy, nullptr, nullptr,
                       nullptr, nullptr);
  }
  return 0;
}

// A/B switch of the max-pool gradient kernel (maxpool_bwd2_kernel by default).
void pdt_maxpool_bwd_v2(int on) { g_pool_bwd_v2 = on; }
void pdt_pool_fwd_contig(int on) { g_pool_contig = on; }
void pdt_bn_row_wgs(int n) { g_row_wgs = n > 0 ? n : 16; }

void pdt_bn_apply_wgs(int n) {  // n <= 0: the measured defaults
  g_apply_wgs[kApplyPlain] = n > 0 ? n : 4;
  g_apply_wgs[kApplyRes] = n > 0 ? n : 2;
  g_apply_wgs[kApplyBwd] = n > 0 ? n : 2;
}

static void launch_pool_bwd_bn(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C, int Ho,
                               int Wo, const uint16_t* x, const float* mean, float* part, int T, hipStream_t s) {
  // v2 covers input positions < (2 Ho, 2 Wo): every one when H <= 2 Ho and W <= 2 Wo (always, for 3x3/s2/p1)
  if (g_pool_bwd_v2 && H <= 2 * Ho && W <= 2 * Wo)
    hipLaunchKernelGGL(maxpool_bwd2_kernel<true>, dim3(T), dim3(256), 0, s, dy, code, dz, N, H, W, C, Ho, Wo, x, mean,
                       part, g_pool_contig);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(T), dim3(256), 0, s, dy, code, dz, N, H, W, C, Ho, Wo, x, mean,
                       part);
}

// Stem backward: max-pool gradient dz (written) with the stem BatchNorm's backward reduction fused,
// then the BN finalize + apply -> dx. C == 64. ws: pdt_bn_tiles_ws_floats(pdt_maxpool_bn_parts(), C)
// + 2C floats; part: 2 * pdt_maxpool_bn_parts() * C floats.
int pdt_maxpool_bn_parts(int N, int H) { return row_grid((int64_t)N * H); }

int pdt_maxpool3s2_bwd_bn(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                          const uint16_t* x, const float* gamma, const float* mean, const float* invstd, uint16_t* dx,
                          float* dgamma, float* dbeta, float* part, float* ws, hipStream_t s) {
  if (C != 64) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t M = (int64_t)N * H * W;
  if (M < 1) return -1;
  const int T = pdt_maxpool_bn_parts(N, H);
  launch_pool_bwd_bn(dy, code, dz, N, H, W, C, Ho, Wo, x, mean, part, T, s);
  return bn_bwd_from_partials(part, T, 1, dz, x, nullptr, gamma, mean, invstd, M, C, 0, 0, dx, nullptr, dgamma, dbeta,
                              ws, s);
}

// Same, without the apply: dz and the dx coefficients coef [3][C] = A, B, D (dx = A dz + B (x - mean)
// + D) for a consumer that applies them on load (the stem weight gradient). dz = null: not written
// (pdt_stem_conv_wgrad_bn_pool forms it again from dy and the codes).
int pdt_maxpool3s2_bwd_bn_coef(const uint16_t* dy, const uint8_t* code, uint16_t* dz, int N, int H, int W, int C,
                               const uint16_t* x, const float* gamma, const float* mean, const float* invstd,
                               float* coef, float* dgamma, float* dbeta, float* part, float* ws, hipStream_t s) {
  if (C != 64 || !coef) return -1;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int64_t M = (int64_t)N * H * W;
  if (M < 1) return -1;
  const int T = pdt_maxpool_bn_parts(N, H);
  launch_pool_bwd_bn(dy, code, dz, N, H, W, C, Ho, Wo, x, mean, part, T, s);
  return bn_bwd_from_partials(part, T, 1, dz, x, nullptr, gamma, mean, invstd, M, C, 0, 0, nullptr, nullptr, dgamma,
                              dbeta, ws, s, coef);
}

}  // extern "C"
