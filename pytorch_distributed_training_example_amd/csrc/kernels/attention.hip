// Flash attention (forward + backward) for gfx950, head dim 64, bf16 in / bf16 out, fp32 accumulate.
//
// Not in the reference (no transformer, /root/reference/cnn.py); serves the ViT-B/16 and
// GPT-2-medium north-star configs ("attention fwd/bwd (flash-style, MFMA)").
//
// MFMA: v_mfma_f32_16x16x32_bf16. Operand lane maps (cdna_hip_programming.md §3):
//   A[row = l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col = l&15], C/D: col = l&15, row = 4(l>>4)+r.
// Layout trick ("swapped" QK^T): the forward computes S^T = K·Q^T, so each lane owns ONE query
// (the accumulator column) and 4 keys per 16-key subtile in registers. Row statistics (max,
// sum) are per-lane plus 2 cross-group shuffles, the online-softmax rescale is a per-lane
// scalar, and P^T feeds O^T = V^T·P^T as the B operand straight from the accumulators (the
// MFMA's k order is permuted consistently on both operands: element j of lane group g is key
// 4g+j (j<4) / 16+4g+j-4 (j>=4)). The V^T operand comes from a row-major LDS tile through
// ds_read_b64_tr_b16 (hardware transposed read, T10). The backward uses:
//   dK/dV kernel: S = Q·K^T (lane = key), dV^T += dO^T·P, dK^T += Q^T·dS  (dO^T, Q^T by tr reads)
//   dQ kernel:    forward structure, dQ^T += K^T·dS^T
// so dQ needs no atomics and no cross-workgroup reduction (deterministic).
#include "../common.h"

#include <type_traits>

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int D = 64;
constexpr int ROW_BYTES = D * 2;  // 128 B per LDS row
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
#ifndef DKDV_MINW
#define DKDV_MINW 2
#endif

struct Tensor4 {  // bf16 [B, H, T, D] view with arbitrary (b, h, t) strides, d stride 1
  const uint16_t* p;
  int64_t sb, sh, st;
};

// ---------------------------------------------------------------- LDS tile helpers
// Tile: ROWS x 64 bf16, row-major, 16-B chunks XOR-swizzled by (row >> 1) & 7 so that 16
// lanes reading 16 different rows at one logical chunk hit 16 different bank slots.
__device__ __forceinline__ int swz(int row, int chunk) { return row * ROW_BYTES + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ bf16x8 lds_row8(const char* tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(tile + swz(row, chunk));
}

// Transposed read: 4 consecutive rows r0..r0+3 of the tile, columns col0 + 0..15 distributed over
// the 16 lanes of each lane group; lane i gets column col0+i of the 4 rows (element q = row r0+q).
__device__ __forceinline__ s4 lds_tr4(const char* tile, int r0, int col0, int lane) {
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int row = r0 + q;
  const int col = col0 + 4 * p;  // element column, multiple of 4
  const int off = swz(row, col >> 3) + ((col & 4) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(tile + off));
}

__device__ __forceinline__ bf16x8 cat8(s4 a, s4 b) {
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ bf16x8 pack8(f4 a, f4 b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

// Raw v_exp_f32 (2^x): exp2f() adds a denormal range-reduction (cmp, 2 cndmask, add, ldexp)
// around every exponential — 4 extra VALU ops per score for results that underflow to 0 in
// bf16 anyway. exp2(-inf) = 0 holds for the masked scores.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 gload8(const uint16_t* p, bool ok) {
  if (ok) return *reinterpret_cast<const bf16x8*>(p);
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

// Buffer resource over one (batch, head) slice of a [B, H, T, 64] view: rows 0..T-1 at stride
// `st` elements. Loads past row T-1 fall outside num_records and return 0 in hardware, so tile
// staging needs no per-row bounds branch (raw buffer, stride 0; dword3 = gfx9 raw-buffer format).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const uint16_t* base, int T, int64_t st) {
  const uint32_t bytes = (uint32_t)(((int64_t)(T - 1) * st + D) * 2);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), (short)0, bytes, 0x00020000);
}

// Stage a 64-row tile (rows r0.. of a [T, 64] head slice) into LDS: 512 16-B chunks, 2 per thread.
struct Stage {
  bf16x8 v[2];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int64_t st, int r0, int tid) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = tid + 256 * u, row = id >> 3, ch = id & 7;
      const uint32_t off = (uint32_t)(((int64_t)(r0 + row) * st + ch * 8) * 2);
      v[u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  }
  __device__ __forceinline__ void store(char* tile, int tid) const {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = tid + 256 * u, row = id >> 3, ch = id & 7;
      *reinterpret_cast<bf16x8*>(tile + swz(row, ch)) = v[u];
    }
  }
};

// ============================================================================ forward
// grid (ceil(T/128), H, B), 256 threads; wave w owns queries [blk*128 + 32w, +32) as 2 x 16.
// ~155 VGPRs: 3 waves per SIMD. Measured alternatives (tools/attn_bench.py, GPT-2 shape): forcing
// 4 waves/SIMD spills (-14%); prefetching K/V two tiles ahead (+24 VGPR) is -7%.
template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(Tensor4 Q, Tensor4 K, Tensor4 V, uint16_t* __restrict__ O,
                                                       int64_t o_sb, int64_t o_sh, int64_t o_st,
                                                       float* __restrict__ LSE, int H, int T, float sl2) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 64 * ROW_BYTES];
  char* Ks = lds;
  char* Vs = lds + 64 * ROW_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int qblk = blockIdx.x * 128;
  const int qbase = qblk + 32 * w;
  const int64_t qoff = (int64_t)b * Q.sb + (int64_t)h * Q.sh;
  const int64_t koff = (int64_t)b * K.sb + (int64_t)h * K.sh;
  const int64_t voff = (int64_t)b * V.sb + (int64_t)h * V.sh;
  const __amdgpu_buffer_rsrc_t krs = slice_rsrc(K.p + koff, T, K.st), vrs = slice_rsrc(V.p + voff, T, V.st);

  // Q^T as B operand, held in registers: [qb][k-step]
  bf16x8 bq[2][2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qr = qbase + 16 * qb + c;
      bq[qb][s] = gload8(Q.p + qoff + (int64_t)qr * Q.st + 32 * s + 8 * g, qr < T);
    }
  f4 oacc[2][4];
  float m[2], l[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    m[qb] = -INFINITY;
    l[qb] = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) oacc[qb][n] = f4{0.f, 0.f, 0.f, 0.f};
  }

  const int kv_end = CAUSAL ? min(T, qblk + 128) : T;
  const int ntiles = (kv_end + 63) / 64;
  // one K/V tile: wait for its staged registers, publish to LDS, prefetch tile `tn`, compute
  auto tile = [&](int t, Stage& sk, Stage& sv, int tn) {
    const int kv0 = t * 64;
    __syncthreads();
    sk.store(Ks, tid);
    sv.store(Vs, tid);
    __syncthreads();
    if (tn < ntiles) {  // prefetch into the registers just drained, while this tile computes
      sk.load(krs, K.st, tn * 64, tid);
      sv.load(vrs, V.st, tn * 64, tid);
    }
    if (qbase >= T || (CAUSAL && kv0 > qbase + 31)) return;  // wave has no query here
    // ---- S^T = K Q^T for 4 key subtiles x 2 query blocks
    f4 st[2][4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a0 = lds_row8(Ks, ks * 16 + c, g);
      const bf16x8 a1 = lds_row8(Ks, ks * 16 + c, 4 + g);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f4 acc = {0.f, 0.f, 0.f, 0.f};
        acc = mfma(a0, bq[qb][0], acc);
        acc = mfma(a1, bq[qb][1], acc);
        st[qb][ks] = acc;
      }
    }
    // ---- online softmax (per lane = per query), P^T packed as the B operand
    // masking only on tiles that cross the sequence end or the causal diagonal (wave-uniform)
    const bool edge = (kv0 + 64 > T) || (CAUSAL && kv0 + 63 > qbase);
    bf16x8 pb[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int qi = qbase + 16 * qb + c;
      if (edge) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kv0 + ks * 16 + 4 * g + r;
            if (key >= T || (CAUSAL && key > qi)) st[qb][ks][r] = -INFINITY;
          }
      }
      float mt = -INFINITY;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) mt = fmaxf(mt, st[qb][ks][r]);
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m[qb], mt * sl2);  // running max in log2-scaled units
      const float alpha = (mn == -INFINITY) ? 1.f : fast_exp2(m[qb] - mn);
      const float msub = (mn == -INFINITY) ? 0.f : mn;
      float ls = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fast_exp2(fmaf(st[qb][ks][r], sl2, -msub));
          st[qb][ks][r] = p;
          ls += p;
        }
      l[qb] = l[qb] * alpha + ls;
      m[qb] = mn;
      if (!__all(alpha == 1.f)) {  // exact skip: no query of the wave moved its max
#pragma unroll
        for (int n = 0; n < 4; ++n) oacc[qb][n] *= alpha;
      }
      pb[qb][0] = pack8(st[qb][0], st[qb][1]);
      pb[qb][1] = pack8(st[qb][2], st[qb][3]);
    }
    // ---- O^T += V^T P^T
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int kst = 0; kst < 2; ++kst) {
        const bf16x8 va = cat8(lds_tr4(Vs, 32 * kst + 4 * g, 16 * n, lane), lds_tr4(Vs, 32 * kst + 16 + 4 * g, 16 * n, lane));
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) oacc[qb][n] = mfma(va, pb[qb][kst], oacc[qb][n]);
      }
    };
  Stage sk, sv;
  sk.load(krs, K.st, 0, tid);
  sv.load(vrs, V.st, 0, tid);
  for (int t = 0; t < ntiles; ++t) tile(t, sk, sv, t + 1);
  // ---- epilogue: normalise, store O (8 B per lane per d-tile) and LSE
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float lt = l[qb] + __shfl_xor(l[qb], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int qi = qbase + 16 * qb + c;
    if (qi >= T) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    uint16_t* orow = O + (int64_t)b * o_sb + (int64_t)h * o_sh + (int64_t)qi * o_st;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float v4[4] = {oacc[qb][n][0] * inv, oacc[qb][n][1] * inv, oacc[qb][n][2] * inv, oacc[qb][n][3] * inv};
      Vec4<uint16_t>::st(orow, 16 * n + 4 * g, v4);
    }
    if (g == 0) LSE[((int64_t)b * H + h) * T + qi] = (m[qb] + log2f(lt)) * LN2;
  }
}

// ============================================================================ backward: delta
// delta[b,h,t] = sum_d dO * O  (fp32). One thread per (row, 8 columns), 8 lanes per row.
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(Tensor4 DO, Tensor4 Ot, float* __restrict__ delta, int H,
                                                           int T, int64_t rows) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid >> 3;
  const int ch = gid & 7;
  float s = 0.f;
  if (row < rows) {
    const int t = (int)(row % T);
    const int64_t bh = row / T;
    const int hh = (int)(bh % H), bb = (int)(bh / H);
    float a[8], o[8];
    ld8_bf16(DO.p + (int64_t)bb * DO.sb + (int64_t)hh * DO.sh + (int64_t)t * DO.st + 8 * ch, a);
    ld8_bf16(Ot.p + (int64_t)bb * Ot.sb + (int64_t)hh * Ot.sh + (int64_t)t * Ot.st + 8 * ch, o);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * o[j];
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (row < rows && ch == 0) delta[row] = s;
}

// ============================================================================ backward: dQ
// Forward structure: S^T = K Q^T, dP^T = V dO^T (lane = query), dS^T = P^T (dP^T - delta),
// dQ^T += K^T dS^T (K^T by transposed LDS reads).
template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(Tensor4 Q, Tensor4 K, Tensor4 V, Tensor4 DO,
                                                          const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                          uint16_t* __restrict__ DQ, int64_t dq_sb, int64_t dq_sh,
                                                          int64_t dq_st, int H, int T, float sl2, float scale) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 64 * ROW_BYTES];
  char* Ks = lds;
  char* Vs = lds + 64 * ROW_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int qblk = blockIdx.x * 128;
  const int qbase = qblk + 32 * w;
  const int64_t qoff = (int64_t)b * Q.sb + (int64_t)h * Q.sh;
  const int64_t dooff = (int64_t)b * DO.sb + (int64_t)h * DO.sh;
  const int64_t koff = (int64_t)b * K.sb + (int64_t)h * K.sh;
  const int64_t voff = (int64_t)b * V.sb + (int64_t)h * V.sh;
  const int64_t rowoff = ((int64_t)b * H + h) * T;

  bf16x8 bq[2][2], bdo[2][2];
  float lse2[2], dlt[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qr = qbase + 16 * qb + c;
    const bool ok = qr < T;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bq[qb][s] = gload8(Q.p + qoff + (int64_t)qr * Q.st + 32 * s + 8 * g, ok);
      bdo[qb][s] = gload8(DO.p + dooff + (int64_t)qr * DO.st + 32 * s + 8 * g, ok);
    }
    lse2[qb] = ok ? LSE[rowoff + qr] * LOG2E : 0.f;
    dlt[qb] = ok ? DELTA[rowoff + qr] : 0.f;
  }
  f4 dq[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int n = 0; n < 4; ++n) dq[qb][n] = f4{0.f, 0.f, 0.f, 0.f};

  const int kv_end = CAUSAL ? min(T, qblk + 128) : T;
  const int ntiles = (kv_end + 63) / 64;
  const __amdgpu_buffer_rsrc_t krs = slice_rsrc(K.p + koff, T, K.st), vrs = slice_rsrc(V.p + voff, T, V.st);
  Stage sk, sv;
  sk.load(krs, K.st, 0, tid);
  sv.load(vrs, V.st, 0, tid);
  for (int t = 0; t < ntiles; ++t) {
    const int kv0 = t * 64;
    __syncthreads();
    sk.store(Ks, tid);
    sv.store(Vs, tid);
    __syncthreads();
    if (t + 1 < ntiles) {
      sk.load(krs, K.st, kv0 + 64, tid);
      sv.load(vrs, V.st, kv0 + 64, tid);
    }
    if (qbase >= T || (CAUSAL && kv0 > qbase + 31)) continue;
    // masking only on tiles that cross the sequence end or the causal diagonal (mask-free
    // instantiation for interior tiles)
    const bool edge = (kv0 + 64 > T) || (CAUSAL && kv0 + 63 > qbase);
    auto tile_body = [&](auto edge_c) {
      constexpr bool EDGE = decltype(edge_c)::value;
      bf16x8 dsb[2][2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 ka0 = lds_row8(Ks, ks * 16 + c, g), ka1 = lds_row8(Ks, ks * 16 + c, 4 + g);
        const bf16x8 va0 = lds_row8(Vs, ks * 16 + c, g), va1 = lds_row8(Vs, ks * 16 + c, 4 + g);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          f4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
          s = mfma(ka0, bq[qb][0], s);
          s = mfma(ka1, bq[qb][1], s);
          dp = mfma(va0, bdo[qb][0], dp);
          dp = mfma(va1, bdo[qb][1], dp);
          const int qi = qbase + 16 * qb + c;
          f4 ds;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float p = fast_exp2(fmaf(s[r], sl2, -lse2[qb]));
            if (EDGE) {
              const int key = kv0 + ks * 16 + 4 * g + r;
              if (key >= T || qi >= T || (CAUSAL && key > qi)) p = 0.f;
            }
            ds[r] = p * (dp[r] - dlt[qb]);
          }
          // stash dS^T (fp32) in the S slot; pack after both halves of a 32-key step exist
          if ((ks & 1) == 0) dsb[qb][ks >> 1] = pack8(ds, f4{0.f, 0.f, 0.f, 0.f});
          else {
            bf16x8 t8 = dsb[qb][ks >> 1];
            t8[4] = (__bf16)ds[0]; t8[5] = (__bf16)ds[1]; t8[6] = (__bf16)ds[2]; t8[7] = (__bf16)ds[3];
            dsb[qb][ks >> 1] = t8;
          }
        }
      }
      // dQ^T += K^T dS^T
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int kst = 0; kst < 2; ++kst) {
          const bf16x8 ka = cat8(lds_tr4(Ks, 32 * kst + 4 * g, 16 * n, lane), lds_tr4(Ks, 32 * kst + 16 + 4 * g, 16 * n, lane));
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) dq[qb][n] = mfma(ka, dsb[qb][kst], dq[qb][n]);
        }
    };
    if (edge) tile_body(std::true_type{});
    else tile_body(std::false_type{});
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int qi = qbase + 16 * qb + c;
    if (qi >= T) continue;
    uint16_t* row = DQ + (int64_t)b * dq_sb + (int64_t)h * dq_sh + (int64_t)qi * dq_st;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float v4[4] = {dq[qb][n][0] * scale, dq[qb][n][1] * scale, dq[qb][n][2] * scale, dq[qb][n][3] * scale};
      Vec4<uint16_t>::st(row, 16 * n + 4 * g, v4);
    }
  }
}

// ============================================================================ backward: dK, dV
// grid (ceil(T/128), H, B); wave w owns keys [blk*128 + 32w, +32) as 2 key subtiles of 16.
// Per 64-query tile (Q, dO staged in LDS): S = Q K^T and dP = dO V^T with lane = key,
// dV^T += dO^T P and dK^T += Q^T dS (dO^T, Q^T via transposed LDS reads).
template <bool CAUSAL>
__global__ __launch_bounds__(256, DKDV_MINW) void attn_bwd_dkdv_kernel(Tensor4 Q, Tensor4 K, Tensor4 V, Tensor4 DO,
                                                            const float* __restrict__ LSE,
                                                            const float* __restrict__ DELTA, uint16_t* __restrict__ DK,
                                                            uint16_t* __restrict__ DV, int64_t g_sb, int64_t g_sh,
                                                            int64_t g_st, int H, int T, float sl2, float scale) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 64 * ROW_BYTES];
  __shared__ float srow[2][64];  // lse2, delta of the staged query tile
  char* Qs = lds;
  char* Ds = lds + 64 * ROW_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int kblk = blockIdx.x * 128;
  const int kbase = kblk + 32 * w;
  const int64_t qoff = (int64_t)b * Q.sb + (int64_t)h * Q.sh;
  const int64_t dooff = (int64_t)b * DO.sb + (int64_t)h * DO.sh;
  const int64_t koff = (int64_t)b * K.sb + (int64_t)h * K.sh;
  const int64_t voff = (int64_t)b * V.sb + (int64_t)h * V.sh;
  const int64_t rowoff = ((int64_t)b * H + h) * T;

  // K^T and V^T as B operands (lane = key column), held in registers: [key subtile][k-step]
  bf16x8 bk[2][2], bv[2][2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int kr = kbase + 16 * kb + c;
    const bool ok = kr < T;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bk[kb][s] = gload8(K.p + koff + (int64_t)kr * K.st + 32 * s + 8 * g, ok);
      bv[kb][s] = gload8(V.p + voff + (int64_t)kr * V.st + 32 * s + 8 * g, ok);
    }
  }
  f4 dk[2][4], dv[2][4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      dk[kb][n] = f4{0.f, 0.f, 0.f, 0.f};
      dv[kb][n] = f4{0.f, 0.f, 0.f, 0.f};
    }

  const int q_start = CAUSAL ? (kblk / 64) * 64 : 0;
  const int ntiles = (T - q_start + 63) / 64;
  const __amdgpu_buffer_rsrc_t qrs = slice_rsrc(Q.p + qoff, T, Q.st), drs = slice_rsrc(DO.p + dooff, T, DO.st);
  Stage sq, sd;
  sq.load(qrs, Q.st, q_start, tid);
  sd.load(drs, DO.st, q_start, tid);
  for (int t = 0; t < ntiles; ++t) {
    const int q0 = q_start + t * 64;
    __syncthreads();
    sq.store(Qs, tid);
    sd.store(Ds, tid);
    if (tid < 64) {
      const int qr = q0 + tid;
      srow[0][tid] = qr < T ? LSE[rowoff + qr] * LOG2E : 0.f;
      srow[1][tid] = qr < T ? DELTA[rowoff + qr] : 0.f;
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      sq.load(qrs, Q.st, q0 + 64, tid);
      sd.load(drs, DO.st, q0 + 64, tid);
    }
    // no key of this wave exists, or every query of the tile precedes this wave's keys
    if (kbase >= T || (CAUSAL && q0 + 63 < kbase)) continue;
    // masking only on tiles that cross the sequence end or the causal diagonal; interior tiles
    // run a mask-free instantiation (no per-score compare/select: ~80 VALU ops per tile)
    const bool edge = (q0 + 64 > T) || (kbase + 32 > T) || (CAUSAL && q0 < kbase + 32);
    auto tile_body = [&](auto edge_c) {
      constexpr bool EDGE = decltype(edge_c)::value;
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {  // 32-query k-step for the dV/dK products
        bf16x8 pb[2], dsb[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          f4 pp[2], dd[2];
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int qs = 2 * kq + half;  // 16-query subtile
            const bf16x8 qa0 = lds_row8(Qs, qs * 16 + c, g), qa1 = lds_row8(Qs, qs * 16 + c, 4 + g);
            const bf16x8 da0 = lds_row8(Ds, qs * 16 + c, g), da1 = lds_row8(Ds, qs * 16 + c, 4 + g);
            f4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
            s = mfma(qa0, bk[kb][0], s);
            s = mfma(qa1, bk[kb][1], s);
            dp = mfma(da0, bv[kb][0], dp);
            dp = mfma(da1, bv[kb][1], dp);
            const int key = kbase + 16 * kb + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int ql = qs * 16 + 4 * g + r;
              const int qi = q0 + ql;
              float p = fast_exp2(fmaf(s[r], sl2, -srow[0][ql]));
              if (EDGE && (qi >= T || key >= T || (CAUSAL && key > qi))) p = 0.f;
              pp[half][r] = p;
              dd[half][r] = p * (dp[r] - srow[1][ql]);
            }
          }
          pb[kb] = pack8(pp[0], pp[1]);
          dsb[kb] = pack8(dd[0], dd[1]);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const bf16x8 doT = cat8(lds_tr4(Ds, 32 * kq + 4 * g, 16 * n, lane), lds_tr4(Ds, 32 * kq + 16 + 4 * g, 16 * n, lane));
          const bf16x8 qT = cat8(lds_tr4(Qs, 32 * kq + 4 * g, 16 * n, lane), lds_tr4(Qs, 32 * kq + 16 + 4 * g, 16 * n, lane));
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            dv[kb][n] = mfma(doT, pb[kb], dv[kb][n]);
            dk[kb][n] = mfma(qT, dsb[kb], dk[kb][n]);
          }
        }
      }
    };
    if (edge) tile_body(std::true_type{});
    else tile_body(std::false_type{});
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int kr = kbase + 16 * kb + c;
    if (kr >= T) continue;
    const int64_t off = (int64_t)b * g_sb + (int64_t)h * g_sh + (int64_t)kr * g_st;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float a4[4] = {dk[kb][n][0] * scale, dk[kb][n][1] * scale, dk[kb][n][2] * scale, dk[kb][n][3] * scale};
      float v4[4] = {dv[kb][n][0], dv[kb][n][1], dv[kb][n][2], dv[kb][n][3]};
      Vec4<uint16_t>::st(DK + off, 16 * n + 4 * g, a4);
      Vec4<uint16_t>::st(DV + off, 16 * n + 4 * g, v4);
    }
  }
}

}  // namespace

extern "C" {

// q/k/v/o/do/dq/dk/dv: bf16 [B, H, T, 64] views given by (b, h, t) strides (d stride 1, 16-B aligned rows).
int pdt_attn_fwd(const uint16_t* q, const int64_t* qs, const uint16_t* k, const int64_t* ks, const uint16_t* v,
                 const int64_t* vs, uint16_t* o, const int64_t* os, float* lse, int B, int H, int T, int Dh,
                 int causal, float scale, hipStream_t s) {
  if (Dh != D) return -1;
  const Tensor4 Q{q, qs[0], qs[1], qs[2]}, K{k, ks[0], ks[1], ks[2]}, V{v, vs[0], vs[1], vs[2]};
  const dim3 grid((T + 127) / 128, H, B);
  const float sl2 = scale * LOG2E;
  if (causal)
    hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, s, Q, K, V, o, os[0], os[1], os[2], lse, H, T, sl2);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, s, Q, K, V, o, os[0], os[1], os[2], lse, H, T, sl2);
  return 0;
}

// delta: fp32 [B*H*T] workspace. dq/dk/dv share the strides gs (e.g. slices of one packed dqkv).
int pdt_attn_bwd(const uint16_t* dout, const int64_t* dos, const uint16_t* q, const int64_t* qs, const uint16_t* k,
                 const int64_t* ks, const uint16_t* v, const int64_t* vs, const uint16_t* o, const int64_t* os,
                 const float* lse, float* delta, uint16_t* dq, uint16_t* dk, uint16_t* dv, const int64_t* gs, int B,
                 int H, int T, int Dh, int causal, float scale, hipStream_t s) {
  if (Dh != D) return -1;
  const Tensor4 Q{q, qs[0], qs[1], qs[2]}, K{k, ks[0], ks[1], ks[2]}, V{v, vs[0], vs[1], vs[2]};
  const Tensor4 DO{dout, dos[0], dos[1], dos[2]}, Ot{o, os[0], os[1], os[2]};
  const int64_t rows = (int64_t)B * H * T;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s, DO, Ot, delta, H,
                     T, rows);
  const dim3 grid((T + 127) / 128, H, B);
  const float sl2 = scale * LOG2E;
  if (causal) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, grid, dim3(256), 0, s, Q, K, V, DO, lse, delta, dq, gs[0], gs[1],
                       gs[2], H, T, sl2, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, grid, dim3(256), 0, s, Q, K, V, DO, lse, delta, dk, dv, gs[0],
                       gs[1], gs[2], H, T, sl2, scale);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, grid, dim3(256), 0, s, Q, K, V, DO, lse, delta, dq, gs[0], gs[1],
                       gs[2], H, T, sl2, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<false>, grid, dim3(256), 0, s, Q, K, V, DO, lse, delta, dk, dv, gs[0],
                       gs[1], gs[2], H, T, sl2, scale);
  }
  return 0;
}

}  // extern "C"
