// Transformer Linear GEMMs on MFMA (gfx950): C[M, N] = A[M, K] · B[N, K]ᵀ, bf16 operands, fp32
// accumulation, bf16 out, with the Linear epilogues fused (SURVEY.md §2.3 "bias + GELU epilogue";
// not in the reference, whose only model is LeNet, /root/reference/cnn.py):
//
//   EPI_NONE  C = A·Bᵀ
//   EPI_BIAS  C = A·Bᵀ + bias                      (bias bf16 or fp32, added in fp32, one rounding)
//   EPI_GELU  C = A·Bᵀ (the pre-activation the backward needs), G = gelu(C + bias)   — the MLP's
//             first layer in one pass: the standalone bias+GELU kernel read C back and wrote G.
//
// Geometry (cdna_hip_programming.md §5, "the 256² 8-phase template", written for this kernel):
//   * 256 x 256 output tile, K-step 64, 512 threads = 8 waves as 2 (M) x 4 (N); a wave owns a
//     128 x 64 piece of C as 8 x 4 blocks of v_mfma_f32_16x16x32_bf16 (128 fp32 accumulators).
//   * A stage is the K-step's [A rows; B rows] image, 512 rows of 128 B, XOR-swizzled on the 16-B
//     chunk ((row >> 1) & 7: conflict-free ds_read_b128 for the 16x16x32 lane map). Two stages
//     (128 KB LDS, one workgroup per CU). Staging is LDS-DMA (global_load_lds_dwordx4): each
//     wave's instruction writes 1 KB = 8 rows linearly; the swizzle is applied to the SOURCE chunk.
//   * A K-step runs as four phases, one C quadrant each (64 rows x 32 columns of the wave's piece,
//     16 MFMAs): (A0,B0) (A0,B1) (A1,B1) (A1,B0) — fragments are read in phases 0-2 only and
//     reused, so a wave holds 32 + 16 + 16 fragment VGPRs.
//   * Every phase is a LOAD section and an MFMA section separated by raw s_barriers, and the two
//     wave rows run one barrier apart (row 1 passes one extra barrier first): on every SIMD one
//     wave issues its fragment reads and DMA while the other runs its 16 MFMAs at raised priority.
//   * Wave row 0 DMAs the B rows of each image, row 1 the A rows. B is last read in phase 1 and A
//     in phase 2, so K-step t+2's shares go out from phase 3 of step t into the stage step t just
//     freed, and are retired by vmcnt(0) in phase 3 of step t+1: each wave keeps its 8 KB share in
//     flight nearly all the time (a drain to zero every K-step cost 10-15 % on the load path).
//   * Measured ceiling (tools/convbench/gemm_bench.cpp, probes): per K-step a CU moves 192 KB of
//     fragment reads + 64 KB of DMA writes through LDS — 256 KB at 128 B/clk is the 2048 cycles of
//     MFMA work itself, so LDS bandwidth, not the matrix pipe, sets the pace (MFMA busy 43 % on
//     the GPT-2 fc1 shape). A 5-slot ring of 32 KB operand parts (all 160 KB of LDS, parts issued
//     up to 1.5 K-steps ahead) sped the load path alone by 20 % but the whole kernel lost 15 %:
//     the extra DMA lands in the LDS-read-heavy phases. Rejected.
//   * Rows of A past M are clamped onto row M-1 (valid memory, results never stored), so any M
//     runs; N % 256 == 0 and K % 64 == 0 (every ViT-B/16 and GPT-2 Linear).
//   * Tiles are ordered in groups of 4 A bands (bands fastest, then N tiles) and the block -> tile
//     map is XCD-aware (xcd_remap): the ~32 tiles resident on one XCD span 4 A bands x 8 B bands
//     and share both in its L2 (8k^3: 1421 vs 1309 TF for plain N-first order).
#include "../common.h"

#include <algorithm>

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

constexpr int kBM = 256, kBK = 64, kThreads = 512;
// Tile 256 x BN: BN = 256, or 128 for shapes with fewer 256 x 256 tiles than ~1.5 waves of CUs
// (gpt2_proj / gpt2_fc2: 128 tiles on 256 CUs; vit_proj: 297) — twice the tiles, wave tiles
// 128 x 32, half the MFMAs per phase.
template <int BN>
struct GT {
  static constexpr int kStage = (kBM + BN) * kBK * 2;  // 64 / 48 KB
  static constexpr int kEpiStride = BN * 2 + 16;       // staged bf16 output rows (padded)
  static constexpr int kLds = 2 * kStage > kBM * kEpiStride ? 2 * kStage : kBM * kEpiStride;
  static constexpr int WC = BN / 4, NJ = WC / 16, NH = NJ / 2;  // wave columns, 16-col blocks, per phase
  static constexpr int kBI = BN / 32;                          // DMA instructions of a B-loading wave
};

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU = 2 };

#ifndef PDT_GEMM_GROUP
#define PDT_GEMM_GROUP 4
#endif
constexpr int kGroup = PDT_GEMM_GROUP;  // A bands per tile group (tile order)

#ifndef PDT_GEMM_PROBE
#define PDT_GEMM_PROBE 0  // diagnostics only (tools/convbench/gemm_bench.cpp): 1 = no MFMA, 2 = no DMA,
                          // 3 = no epilogue (accumulators kept alive, nothing staged or stored)
#endif

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fp8 (F8): the same LDS images hold 128 e4m3 values per 128-B row, so one K-step is ONE block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 per 16 x 16 block (unit scales, e8m0 127) instead of two bf16 MFMAs:
// twice the cycles of one bf16 16x16x32, so the same matrix-pipe time and the same fragment bytes per
// K-step for twice the K — the bf16 kernel's LDS-read bound (header) halved per FLOP. A lane's 32 operand
// bytes are its two bf16 fragments' 16-B chunks (chunks lchk and 4 + lchk of the row): any fixed byte ->
// k placement shared by A and B gives the same dot product, so the hardware's k order within a lane's
// 32 bytes never matters. The per-tensor dequantisation scales multiply the fp32 accumulators in the
// epilogue (torch._scaled_mm semantics: C = (A sa)(B sb)^T + bias).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma8(i32x8 a, i32x8 b, f4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);  // e4m3 x e4m3
}
// a lane's 32-B fp8 fragment: the 16-B chunks lchk and 4 + lchk of an LDS row (loaded straight into the
// two halves of the operand's 8 consecutive VGPRs — no register copies)
__device__ __forceinline__ i32x8 ld_frag8(const char* p0, const char* p1) {
  const i32x4 x = *reinterpret_cast<const i32x4*>(p0), y = *reinterpret_cast<const i32x4*>(p1);
  return __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// GELU with short-latency math (the epilogue runs once per tile with nothing to hide it behind):
// tanh(u) = 1 - 2 / (1 + e^{2u}); erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below
// the bf16 rounding of the result).
__device__ __forceinline__ float gelu_f(float v, int tanh_form) {
  if (tanh_form) {
    const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
    const float t = 1.f - 2.f * __frcp_rn(1.f + __expf(2.f * u));
    return 0.5f * v * (1.f + t);
  }
  const float x = fabsf(v) * 0.7071067811865476f;
  const float t = __frcp_rn(1.f + 0.3275911f * x);
  const float p = ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  const float e = 1.f - p * __expf(-x * x);
  return 0.5f * v * (1.f + copysignf(e, v));
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}

// F8: A / B are e4m3 [M, 2K] / [N, 2K] bytes passed as uint16 rows of K (so every address below is the
// bf16 kernel's), sa / sb their device-side dequantisation scales.
template <int EPI, int BN, bool F8 = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_kernel(const uint16_t* __restrict__ A,
                                                               const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                                                               uint16_t* __restrict__ G, const void* __restrict__ bias,
                                                               int bias_f32, int tanh_form, int M, int N, int K,
                                                               const float* __restrict__ sa, const float* __restrict__ sb,
                                                               float* __restrict__ part, int ksplit) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  using T = GT<BN>;
  constexpr int kStage = T::kStage, kEpiStride = T::kEpiStride, WC = T::WC, NJ = T::NJ, NH = T::NH;
  const int ntn = N / BN, ntm = (M + kBM - 1) / kBM;
  const int id0 = xcd_remap(blockIdx.x, gridDim.x);
  // split-K (F8, ksplit > 1): block id = split * tiles + tile; split s takes K-steps [s nkt / ksplit,
  // (s + 1) nkt / ksplit) and writes its fp32 tile to part[s] (summed by splitk_reduce_kernel)
  const int split = id0 / (ntn * ntm), id = id0 - split * (ntn * ntm);
  // groups of kGroup A bands: consecutive ids (one XCD) cover kGroup bands x a few N tiles, so the
  // tiles resident on an XCD at once share both operands in its L2
  const int gband = (id / (kGroup * ntn)) * kGroup, gsize = min(ntm - gband, kGroup), gi = id % (kGroup * ntn);
  const int m0 = (gband + gi % gsize) * kBM, n0 = (gi / gsize) * BN;
  const int nkt = K / kBK, kb = split * nkt / ksplit;
  const int nk = (split + 1) * nkt / ksplit - kb;

  // DMA: waves 0-3 (wave row 0) stage the B rows of the image, waves 4-7 (row 1) the A rows — each
  // A wave 64 rows as 8 instructions of 8 rows, each B wave BN / 4 rows (8 or 4 instructions); lane ->
  // (row + lane / 8, physical chunk lane % 8). The first half of a wave's instructions is half 0 of
  // its share, the rest half 1.
  const bool loads_b = wid < 4;
  const uint16_t* const src = loads_b ? B : A;
  const int rbase = loads_b ? kBM + wid * WC : (wid - 4) * 64;  // first LDS row of this wave's share
  const int nI = loads_b ? T::kBI : 8;                         // (wave-uniform)
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int R = rbase + j * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((R >> 1) & 7);
    const int grow = loads_b ? n0 + (R - kBM) : min(m0 + R, M - 1);
    off[j] = grow * K + logical * 8 + kb * kBK;
  }
  auto issue = [&](int t, int half) {  // half 0 / 1 of this wave's share of K-step t
    if (PDT_GEMM_PROBE == 2) return;
    char* st = lds + (t & 1) * kStage + rbase * 128;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j >= half * (nI / 2) && j < (half + 1) * (nI / 2))  // (wave-uniform)
        __builtin_amdgcn_global_load_lds(src + (off[j] + t * kBK), (PDT_LDS void*)(st + j * 1024), 16, 0, 0);
  };

  const int lrow = lane & 15, lchk = lane >> 4;
  f4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b0[NH][2], b1[NH][2];
  i32x8 a8[4], b08[NH], b18[NH];  // F8 fragments

  auto read_a = [&](const char* SA, int aq) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wr * 128 + aq * 64 + i * 16 + lrow;
      if constexpr (F8) {
        a8[i] = ld_frag8(SA + swz(r, lchk), SA + swz(r, 4 + lchk));
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) a[i][kk] = *reinterpret_cast<const bf16x8*>(SA + swz(r, kk * 4 + lchk));
      }
    }
  };
  auto read_b = [&](const char* SB, int bq, bf16x8 (&b)[NH][2], i32x8 (&b8)[NH]) {
#pragma unroll
    for (int j = 0; j < NH; ++j) {
      const int r = kBM + wc * WC + bq * (WC / 2) + j * 16 + lrow;
      if constexpr (F8) {
        b8[j] = ld_frag8(SB + swz(r, lchk), SB + swz(r, 4 + lchk));
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) b[j][kk] = *reinterpret_cast<const bf16x8*>(SB + swz(r, kk * 4 + lchk));
      }
    }
  };
  auto quad = [&](int aq, int bq, const bf16x8 (&b)[NH][2], const i32x8 (&b8)[NH]) {
    if (PDT_GEMM_PROBE == 1) {  // keep the fragment reads alive without the MFMAs
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(a[i][0]), "v"(a[i][1]));
#pragma unroll
      for (int j = 0; j < NH; ++j) asm volatile("" ::"v"(b[j][0]), "v"(b[j][1]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NH; ++j) {
        if constexpr (F8) {
          acc[aq * 4 + i][bq * NH + j] = mfma8(b8[j], a8[i], acc[aq * 4 + i][bq * NH + j]);
        } else {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            acc[aq * 4 + i][bq * NH + j] = mfma(b[j][kk], a[i][kk], acc[aq * 4 + i][bq * NH + j]);  // D[n][m]
        }
      }
  };

  // Pipeline (intervals = barrier-delimited; row 0 loads in even ones, row 1 in odd ones): the B
  // part of a stage is last read in phase 1, the A part in phase 2, so K-step t+2's B (row 0) and
  // A (row 1) shares are DMA'd from phase 3 of step t and phase 0 of step t+1 on, and retired by
  // vmcnt(0) in phase 3 of step t+1 — each wave keeps one share in flight almost continuously,
  // ~6-8 barrier intervals ahead of its first read.
  issue(0, 0);
  issue(0, 1);
  if (nk > 1) issue(1, 0);
  if (nk > 1) {  // step 0's share landed: younger are step 1's half 0 (nI / 2 instructions)
    if (nI == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (wr == 1) bar();  // row 1 runs one barrier behind row 0

  for (int k = 0; k < nk; ++k) {
    const char* S = lds + (k & 1) * kStage;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- load section
      if (q == 0) {
        if (k + 1 < nk) issue(k + 1, 1);
        read_b(S, 0, b0, b08);
        read_a(S, 0);
      } else if (q == 1) {
        read_b(S, 1, b1, b18);
      } else if (q == 2) {
        read_a(S, 1);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of K-step k+1 landed
        if (k + 2 < nk) issue(k + 2, 0);
      }
      bar();
      // ---- MFMA section
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      if (q == 0) quad(0, 0, b0, b08);
      else if (q == 1) quad(0, 1, b1, b18);
      else if (q == 2) quad(1, 1, b1, b18);
      else quad(1, 0, b0, b08);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  }
  if (wr == 0) bar();  // balance row 1's extra barrier

  if (PDT_GEMM_PROBE == 3) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) C[tid] = 1;
    return;
  }
  // ---- epilogue: lane holds C[m][n .. n+3] of every block (4 consecutive columns). The bf16 tile
  // is staged through LDS (free now: every read and DMA has retired) and written as whole 512-B
  // row segments — 8-B stores straight from the accumulators hit each 128-B line four times and
  // ran the write-out at ~1 TB/s. EPI_GELU stages H, then G.
  float bv[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wc * WC + j * 16 + 4 * lchk;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = 0.f;
    if constexpr (EPI != EPI_NONE) {
      if (bias) {
        if (bias_f32) {
          const float4 t = *reinterpret_cast<const float4*>(static_cast<const float*>(bias) + n);
          bv[j][0] = t.x; bv[j][1] = t.y; bv[j][2] = t.z; bv[j][3] = t.w;
        } else {
          const uint2 t = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(bias) + n);
          bv[j][0] = bf2f((uint16_t)t.x); bv[j][1] = bf2f((uint16_t)(t.x >> 16));
          bv[j][2] = bf2f((uint16_t)t.y); bv[j][3] = bf2f((uint16_t)(t.y >> 16));
        }
      }
    }
  }
  if constexpr (F8) {
    const float sc = *sa * *sb;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] *= sc;
  }
  bar();
  if constexpr (F8) {
    if (ksplit > 1) {  // fp32 partial tile, staged through LDS one wave row (128 rows) at a time
      constexpr int kPS = BN * 4 + 16;
      float* const pb = part + (int64_t)split * M * N;
#pragma unroll 1
      for (int ph = 0; ph < 2; ++ph) {
        if (wr == ph) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              *reinterpret_cast<f4*>(lds + (i * 16 + lrow) * kPS + (wc * WC + j * 16 + 4 * lchk) * 4) = acc[i][j];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        for (int idx = tid; idx < 128 * (BN / 4); idx += kThreads) {
          const int r = idx / (BN / 4), c = idx % (BN / 4);
          const int m = m0 + ph * 128 + r;
          if (m < M)
            *reinterpret_cast<float4*>(pb + (int64_t)m * N + n0 + c * 4) =
                *reinterpret_cast<const float4*>(lds + r * kPS + c * 16);
        }
        bar();
      }
      return;
    }
  }
  auto stage_out = [&](uint16_t* __restrict__ out, bool gelu_pass) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f4 v = acc[i][j];
        uint2 pk;
        if constexpr (EPI == EPI_GELU) {
          pk = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));  // H
          if (gelu_pass) {
            pk = make_uint2(pack2(gelu_f(bf2f((uint16_t)pk.x) + bv[j][0], tanh_form),
                                  gelu_f(bf2f((uint16_t)(pk.x >> 16)) + bv[j][1], tanh_form)),
                            pack2(gelu_f(bf2f((uint16_t)pk.y) + bv[j][2], tanh_form),
                                  gelu_f(bf2f((uint16_t)(pk.y >> 16)) + bv[j][3], tanh_form)));
          }
        } else {
          pk = make_uint2(pack2(v[0] + bv[j][0], v[1] + bv[j][1]), pack2(v[2] + bv[j][2], v[3] + bv[j][3]));
        }
        *reinterpret_cast<uint2*>(lds + (wr * 128 + i * 16 + lrow) * kEpiStride + (wc * WC + j * 16 + 4 * lchk) * 2) = pk;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    for (int idx = tid; idx < kBM * (BN / 8); idx += kThreads) {
      const int r = idx / (BN / 8), c = idx % (BN / 8);
      const int m = m0 + r;
      if (m < M)
        *reinterpret_cast<uint4*>(out + (int64_t)m * N + n0 + c * 8) =
            *reinterpret_cast<const uint4*>(lds + r * kEpiStride + c * 16);
    }
  };
  stage_out(C, false);
  if constexpr (EPI == EPI_GELU) {
    bar();  // every wave has copied H out of LDS
    stage_out(G, true);
  }
}

template <int EPI, int BN, bool F8 = false>
int launch_bn(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
              int tanh_form, int M, int N, int K, hipStream_t s, const float* sa = nullptr, const float* sb = nullptr,
              float* part = nullptr, int ksplit = 1) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, BN, F8>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, GT<BN>::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  const int64_t grid = (int64_t)((M + kBM - 1) / kBM) * (N / BN) * ksplit;
  hipLaunchKernelGGL((gemm_nt_kernel<EPI, BN, F8>), dim3((unsigned)grid), dim3(kThreads), GT<BN>::kLds, s, A, B, C, G,
                     bias, bias_f32, tanh_form, M, N, K, sa, sb, part, ksplit);
  return hipPeekAtLastError() == hipSuccess ? 0 : -4;  // a refused launch fails loudly, not as garbage
}

// 256 x 256 tiles unless they fill at most one wave of the 256 CUs (then 256 x 128: twice the tiles).
// Measured (profiles/r5/gemm_bn128.txt): 128 tiles of 256 x 256 (GPT-2 proj / fc2) run 18% / 13% faster
// as 256 x 128; 297 tiles (ViT proj / fc2) run 6% / 9% slower. PDT_GEMM_BN=128 / 256 forces one (A/B).
inline int pick_bn(int M, int N) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("PDT_GEMM_BN");
    forced = (e && e[0]) ? (int)strtol(e, nullptr, 10) : 0;
  }
  if (forced == 128 && N % 128 == 0) return 128;
  if (forced == 256 && N % 256 == 0) return 256;
  if (N % 256 != 0) return 128;
  const int64_t tiles = (int64_t)((M + kBM - 1) / kBM) * (N / 256);
  return tiles <= 256 ? 128 : 256;
}

template <int EPI, bool F8 = false>
int launch(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
           int tanh_form, int M, int N, int K, hipStream_t s, const float* sa = nullptr, const float* sb = nullptr,
           float* part = nullptr, int ksplit = 1) {
  return pick_bn(M, N) == 128
             ? launch_bn<EPI, 128, F8>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s, sa, sb, part, ksplit)
             : launch_bn<EPI, 256, F8>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s, sa, sb, part, ksplit);
}

// C = bf16(sum over the ksplit fp32 partial tiles), fixed order (deterministic); 4 elements per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, uint16_t* __restrict__ C,
                                                            int64_t n4, int64_t MN, int ksplit) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = reinterpret_cast<const float4*>(part)[i];
    for (int sp = 1; sp < ksplit; ++sp) {
      const float4 b = reinterpret_cast<const float4*>(part + sp * MN)[i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    reinterpret_cast<uint2*>(C)[i] = make_uint2(pack2(a.x, a.y), pack2(a.z, a.w));
  }
}

// K splits for an fp8 GEMM with few output tiles (PDT_GEMM_KSPLIT forces a count, 1 = off): about 384
// workgroups, at least 8 K-steps of 128 per split, at most 16 splits.
int fp8_ksplit(int M, int N, int K) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = getenv("PDT_GEMM_KSPLIT");
    forced = (e && e[0]) ? (int)strtol(e, nullptr, 10) : 0;
  }
  const int nkt = K / (2 * kBK);
  const int64_t tiles = (int64_t)((M + kBM - 1) / kBM) * (N / pick_bn(M, N));
  int ks = forced > 0 ? forced : (tiles >= 192 ? 1 : (int)((384 + tiles - 1) / tiles));
  ks = std::min(ks, std::min(16, nkt / 8));
  return ks < 1 ? 1 : ks;
}

}  // namespace

extern "C" {

// C[M, N] (and G for epi 2) from A[M, K] and B[N, K], all row-major contiguous bf16; N % 128 == 0.
// epi: 0 none, 1 + bias, 2 C = A·Bᵀ and G = gelu(C + bias) (tanh_form: GPT-2's tanh GELU).
// bias: [N] fp32 (bias_f32 = 1) or bf16, may be null. Returns 0, or < 0 when the shape is not served.
int pdt_gemm_nt(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
                int epi, int tanh_form, int M, int N, int K, hipStream_t s) {
  if (M < 1 || N % 128 != 0 || K % kBK != 0 || N < 128 || K < kBK) return -1;
  if ((int64_t)M * K >= (int64_t)1 << 31 || (int64_t)N * K >= (int64_t)1 << 31) return -2;
  if (epi == EPI_GELU && G == nullptr) return -1;
  switch (epi) {
    case EPI_NONE: return launch<EPI_NONE>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    case EPI_BIAS: return launch<EPI_BIAS>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    case EPI_GELU: return launch<EPI_GELU>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    default: return -1;
  }
}

// fp8 e4m3 operands: C[M, N] bf16 = (A sa)(B sb)^T (+ bias, epi 1) from A [M, K] and B [N, K] row-major e4m3
// bytes and device-side fp32 dequantisation scales sa / sb (torch._scaled_mm's); N % 128 == 0, K % 128 == 0.
// ws / ksplit (epi 0 only): pdt_gemm_nt_fp8_ksplit() splits of K, ws = ksplit * M * N floats (ksplit 1: unused).
int pdt_gemm_nt_fp8_ksplit(int M, int N, int K) {
  if (M < 1 || N % 128 != 0 || K % (2 * kBK) != 0 || N < 128 || K < 2 * kBK) return 1;
  return fp8_ksplit(M, N, K);
}

int pdt_gemm_nt_fp8(const uint8_t* A, const uint8_t* B, uint16_t* C, const float* sa, const float* sb,
                    const void* bias, int bias_f32, int epi, int M, int N, int K, float* ws, int ksplit, hipStream_t s) {
  if (M < 1 || N % 128 != 0 || K % (2 * kBK) != 0 || N < 128 || K < 2 * kBK || !sa || !sb) return -1;
  if ((int64_t)M * K >= (int64_t)1 << 31 || (int64_t)N * K >= (int64_t)1 << 31) return -2;
  if (ksplit < 1 || ksplit > K / (2 * kBK) || (ksplit > 1 && (!ws || epi != EPI_NONE))) return -1;
  const uint16_t* a = reinterpret_cast<const uint16_t*>(A);
  const uint16_t* b = reinterpret_cast<const uint16_t*>(B);
  if (ksplit > 1) {
    const int rc = launch<EPI_NONE, true>(a, b, C, nullptr, nullptr, 0, 0, M, N, K / 2, s, sa, sb, ws, ksplit);
    if (rc) return rc;
    const int64_t MN = (int64_t)M * N, n4 = MN / 4;
    const int64_t g = std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, ws, C, n4, MN, ksplit);
    return hipPeekAtLastError() == hipSuccess ? 0 : -4;
  }
  switch (epi) {  // the kernel addresses 128-B rows of K / 2 uint16
    case EPI_NONE: return launch<EPI_NONE, true>(a, b, C, nullptr, bias, bias_f32, 0, M, N, K / 2, s, sa, sb);
    case EPI_BIAS: return launch<EPI_BIAS, true>(a, b, C, nullptr, bias, bias_f32, 0, M, N, K / 2, s, sa, sb);
    default: return -1;
  }
}

}  // extern "C"
