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

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 512;
constexpr int kStage = (kBM + kBN) * kBK * 2;  // 64 KB
constexpr int kEpiStride = kBN * 2 + 16;       // staged bf16 output rows (padded)
constexpr int kLds = 2 * kStage > kBM * kEpiStride ? 2 * kStage : kBM * kEpiStride;

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

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_kernel(const uint16_t* __restrict__ A,
                                                               const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                                                               uint16_t* __restrict__ G, const void* __restrict__ bias,
                                                               int bias_f32, int tanh_form, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int ntn = N / kBN, ntm = (M + kBM - 1) / kBM;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  // groups of kGroup A bands: consecutive ids (one XCD) cover kGroup bands x a few N tiles, so the
  // tiles resident on an XCD at once share both operands in its L2
  const int gband = (id / (kGroup * ntn)) * kGroup, gsize = min(ntm - gband, kGroup), gi = id % (kGroup * ntn);
  const int m0 = (gband + gi % gsize) * kBM, n0 = (gi / gsize) * kBN;
  const int nk = K / kBK;

  // DMA: waves 0-3 (wave row 0) stage the B rows of the image, waves 4-7 (row 1) the A rows — each
  // wave 64 rows as 8 instructions of 8 rows; lane -> (row + lane / 8, physical chunk lane % 8).
  // Instructions 0-3 are half 0 of the wave's share, 4-7 half 1.
  const bool loads_b = wid < 4;
  const uint16_t* const src = loads_b ? B : A;
  const int rbase = loads_b ? kBM + wid * 64 : (wid - 4) * 64;  // first LDS row of this wave's share
  int off[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int R = rbase + j * 8 + (lane >> 3);
    const int logical = (lane & 7) ^ ((R >> 1) & 7);
    const int grow = loads_b ? n0 + (R - kBM) : min(m0 + R, M - 1);
    off[j] = grow * K + logical * 8;
  }
  auto issue = [&](int t, int half) {  // half 0 / 1 of this wave's share of K-step t
    if (PDT_GEMM_PROBE == 2) return;
    char* st = lds + (t & 1) * kStage + rbase * 128;
#pragma unroll
    for (int j = half * 4; j < half * 4 + 4; ++j)
      __builtin_amdgcn_global_load_lds(src + (off[j] + t * kBK), (PDT_LDS void*)(st + j * 1024), 16, 0, 0);
  };

  const int lrow = lane & 15, lchk = lane >> 4;
  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b0[2][2], b1[2][2];

  auto read_a = [&](const char* SA, int aq) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        a[i][kk] = *reinterpret_cast<const bf16x8*>(SA + swz(wr * 128 + aq * 64 + i * 16 + lrow, kk * 4 + lchk));
  };
  auto read_b = [&](const char* SB, int bq, bf16x8 (&b)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        b[j][kk] = *reinterpret_cast<const bf16x8*>(SB + swz(kBM + wc * 64 + bq * 32 + j * 16 + lrow, kk * 4 + lchk));
  };
  auto quad = [&](int aq, int bq, const bf16x8 (&b)[2][2]) {
    if (PDT_GEMM_PROBE == 1) {  // keep the fragment reads alive without the MFMAs
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(a[i][0]), "v"(a[i][1]));
      asm volatile("" ::"v"(b[0][0]), "v"(b[0][1]), "v"(b[1][0]), "v"(b[1][1]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          acc[aq * 4 + i][bq * 2 + j] = mfma(b[j][kk], a[i][kk], acc[aq * 4 + i][bq * 2 + j]);  // D[n][m]
  };

  // Pipeline (intervals = barrier-delimited; row 0 loads in even ones, row 1 in odd ones): the B
  // part of a stage is last read in phase 1, the A part in phase 2, so K-step t+2's B (row 0) and
  // A (row 1) shares are DMA'd from phase 3 of step t and phase 0 of step t+1 on, and retired by
  // vmcnt(0) in phase 3 of step t+1 — each wave keeps one share in flight almost continuously,
  // ~6-8 barrier intervals ahead of its first read.
  issue(0, 0);
  issue(0, 1);
  if (nk > 1) issue(1, 0);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (wr == 1) bar();  // row 1 runs one barrier behind row 0

  for (int k = 0; k < nk; ++k) {
    const char* S = lds + (k & 1) * kStage;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- load section
      if (q == 0) {
        if (k + 1 < nk) issue(k + 1, 1);
        read_b(S, 0, b0);
        read_a(S, 0);
      } else if (q == 1) {
        read_b(S, 1, b1);
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
      if (q == 0) quad(0, 0, b0);
      else if (q == 1) quad(0, 1, b1);
      else if (q == 2) quad(1, 1, b1);
      else quad(1, 0, b0);
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
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) C[tid] = 1;
    return;
  }
  // ---- epilogue: lane holds C[m][n .. n+3] of every block (4 consecutive columns). The bf16 tile
  // is staged through LDS (free now: every read and DMA has retired) and written as whole 512-B
  // row segments — 8-B stores straight from the accumulators hit each 128-B line four times and
  // ran the write-out at ~1 TB/s. EPI_GELU stages H, then G.
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + 4 * lchk;
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
  bar();
  auto stage_out = [&](uint16_t* __restrict__ out, bool gelu_pass) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
        *reinterpret_cast<uint2*>(lds + (wr * 128 + i * 16 + lrow) * kEpiStride + (wc * 64 + j * 16 + 4 * lchk) * 2) = pk;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    for (int idx = tid; idx < kBM * (kBN / 8); idx += kThreads) {
      const int r = idx / (kBN / 8), c = idx % (kBN / 8);
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

template <int EPI>
int launch(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
           int tanh_form, int M, int N, int K, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  const int64_t grid = (int64_t)((M + kBM - 1) / kBM) * (N / kBN);
  hipLaunchKernelGGL(gemm_nt_kernel<EPI>, dim3((unsigned)grid), dim3(kThreads), kLds, s, A, B, C, G, bias, bias_f32,
                     tanh_form, M, N, K);
  return hipPeekAtLastError() == hipSuccess ? 0 : -4;  // a refused launch fails loudly, not as garbage
}

}  // namespace

extern "C" {

// C[M, N] (and G for epi 2) from A[M, K] and B[N, K], all row-major contiguous bf16.
// epi: 0 none, 1 + bias, 2 C = A·Bᵀ and G = gelu(C + bias) (tanh_form: GPT-2's tanh GELU).
// bias: [N] fp32 (bias_f32 = 1) or bf16, may be null. Returns 0, or < 0 when the shape is not served.
int pdt_gemm_nt(const uint16_t* A, const uint16_t* B, uint16_t* C, uint16_t* G, const void* bias, int bias_f32,
                int epi, int tanh_form, int M, int N, int K, hipStream_t s) {
  if (M < 1 || N % kBN != 0 || K % kBK != 0 || N < kBN || K < kBK) return -1;
  if ((int64_t)M * K >= (int64_t)1 << 31 || (int64_t)N * K >= (int64_t)1 << 31) return -2;
  if (epi == EPI_GELU && G == nullptr) return -1;
  switch (epi) {
    case EPI_NONE: return launch<EPI_NONE>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    case EPI_BIAS: return launch<EPI_BIAS>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    case EPI_GELU: return launch<EPI_GELU>(A, B, C, G, bias, bias_f32, tanh_form, M, N, K, s);
    default: return -1;
  }
}

}  // extern "C"
