// 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on MFMA (gfx950), NHWC bf16, fp32 accumulate.
//
// Not in the reference (LeNet's convs are 5x5 on 1-16 channels, /root/reference/cnn.py:10-16).
// Serves the ResNet-50 north-star config: 13 of its 16 3x3 convs are stride 1, and every one does
// 118 GFLOP per direction at batch 512. MIOpen's kernels ran them at 0.35-0.9 PF
// (tools/r50_roofline.py: fwd 135-255 us, data-gradient 210-296 us vs a 74 us MFMA floor).
//
//   Y[m, co] = sum_{tap, ci} X[pixel(m) + shift(tap), ci] * Wt[co, tap, ci]      (m = (n, oh, ow))
//
// GEMM view: M = N*H*W pixels, N = Co, K = 9 taps x Ci. A k-step is one tap and 64 input
// channels, so every A row is 128 contiguous bytes of one (shifted) input pixel, or zeros when
// the shifted pixel is in the padding. The data gradient of the same conv is this kernel on dY
// with the weights flipped and transposed (conv3x3_flip_weights): Wt'[ci, 8 - tap, co].
//
// Structure (cdna_hip_programming.md §5):
//   * tile 256 pixels x BN (64 | 128) output channels, 512 threads = 8 waves as 4 (M) x 2 (N),
//     each wave 64 x BN/2 as 4 x BN/32 blocks of v_mfma_f32_16x16x32_bf16;
//   * operands staged global -> LDS by LDS-DMA (global_load_lds_dwordx4: 1 KB = 8 rows of 128 B
//     per wave instruction) into a 3-slot ring: the slot for k-step s+2 is issued right after the
//     barrier of step s, while steps s (being read) and s+1 (landing) are resident; ONE raw
//     s_barrier per k-step and a counted vmcnt, so the DMA stays in flight across barriers;
//   * padding rows are DMA'd from a 256-B zero page (per-lane source address), no branches;
//   * rows XOR-swizzled ((row >> 1) & 7 on the 16-B chunk: conflict-free ds_read_b128 for the
//     16x16x32 lane map) by permuting each lane's SOURCE chunk — the DMA writes LDS linearly;
//   * MFMA operands swapped (A = weights, B = pixels) so a lane's accumulator holds 4
//     consecutive channels of one pixel; the epilogue stages the bf16 tile through LDS and
//     writes whole 16-B row pieces;
//   * block -> tile map XCD-aware (xcd_remap): the output-channel tiles of one pixel tile, and
//     neighbouring pixel tiles (which share input rows), run on one XCD's L2.
#include "../common.h"
#include "../tile_stats.h"

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

__device__ __attribute__((aligned(256))) uint4 g_conv_zero[16];  // zero page for padding rows (never written)
__device__ __attribute__((aligned(16))) uint8_t g_conv_ones[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                      0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};  // "no ReLU mask"

// Runtime variant bits for A/B (pdt_conv3x3_opt; env PDT_CONV3X3_OPT read once, default kOptDefault):
//   bit 0: the weight-stationary kernel skips the DMA of halo rows past its tile's extent;
//   bits 1 / 2 (timing probes only, WRONG results): that kernel without its halo DMA after the first
//   chunk / without its MFMA loop — the compute-only and load-only times of its pipeline;
//   bit 3: its fragment-read / MFMA software pipeline pinned with scheduling barriers;
//   bit 4 (probe, WRONG results): its loader waves do not wait for a chunk's DMA before the barrier;
//   bit 5: 64 -> 64 channels at W = 56 on the row-tile kernel (conv3x3wsr_kernel) instead (bits 1 / 2
//   are its timing probes too);
//   bit 6: the halo kernel (conv3x3h, layers 2-4) issues its LDS DMA through inline asm (dma16a);
//   bit 7: the row-tile kernel takes the data gradient's BatchNorm backward reduction (BSTATS).
constexpr int kOptDefault = 41;
int g_c3opt = -1;
inline int conv3x3_opt() {
  if (g_c3opt < 0) {
    const char* e = getenv("PDT_CONV3X3_OPT");
    g_c3opt = (e && e[0]) ? (int)strtol(e, nullptr, 10) : kOptDefault;
    if (g_c3opt < 0) g_c3opt = kOptDefault;
  }
  return g_c3opt;
}

constexpr int kSlots = 3;

// Tile BM pixels x BN channels, WM x WN waves (each (BM/WM) x (BN/WN)), BK input channels per
// k-step (LDS rows of 2*BK bytes), 3-slot LDS ring.
template <int BM_, int BN_, int WM_, int WN_, int BK_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_;
  static constexpr int kThreads = WM * WN * 64;
  static constexpr int kRow = BK * 2;
  static constexpr int kRPI = 1024 / kRow;  // rows per 1-KB DMA instruction
  static constexpr int kABytes = BM * kRow;
  static constexpr int kBBytes = BN * kRow;
  static constexpr int kSlot = kABytes + kBBytes;
  static constexpr int kEpiStride = BN * 2 + 16;
  static constexpr int kLds = (kSlots * kSlot > BM * kEpiStride) ? kSlots * kSlot : BM * kEpiStride;
  static constexpr int kMB = BM / WM / 16;  // 16-row pixel blocks per wave
  static constexpr int kNB = BN / WN / 16;  // 16-wide channel blocks per wave
  static constexpr int kALd = BM / kRPI / (WM * WN);  // DMA instructions per wave per slot
  static constexpr int kBLd = BN / kRPI / (WM * WN);
  static constexpr int kG = kALd + kBLd;
  static_assert(kALd * kRPI * WM * WN == BM && kBLd * kRPI * WM * WN == BN, "DMA split");
};

// 16-B chunk swizzle: conflict-free ds_read_b128 of 16 consecutive rows for the 16x16x32 lane
// map (lanes 16q..16q+15 read chunk q of rows 0..15; ds_read_b128 serves lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... one LDS cycle each). 128-B rows: chunk ^ ((row>>1)&7).
// 64-B rows (4 rows per 256-B bank row): chunk ^ (((row>>2)&1)<<1) — conflict-free for 16
// consecutive rows starting at ANY row (the halo kernel's tap-shifted reads), not just aligned ones:
// in every lane group the 4 rows of one residue mod 4 have consecutive row>>2 and chunks c, c^1,
// c^1, c, which this XOR maps to 4 distinct 16-B slots (checked by hand for all four groups).
template <int ROW>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (ROW == 128) return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4);
}

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (PDT_LDS void*)lds_wave_base, 16, 0, 0);
}

// LDS DMA through inline asm: with the builtin form anywhere in a loop, the compiler's waitcnt pass
// treats the LGKM counter as out of order and turns every fragment-read wait into lgkmcnt(0); hidden
// from it, the DMA is counted by this kernel's own vmcnt waits and the ds_read waits stay exact.
__device__ __forceinline__ void dma16a(const void* src, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(PDT_LDS const char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}

template <bool ASM>
__device__ __forceinline__ void dma16x(const void* src, char* lds_wave_base) {
  if constexpr (ASM) dma16a(src, lds_wave_base);
  else dma16(src, lds_wave_base);
}

template <int G>
__device__ __forceinline__ void wait_vm() {
  static_assert(G >= 0 && G <= 8, "vmcnt");
  if constexpr (G == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (G == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (G == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (G == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (G == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (G == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#ifndef PDT_CONV_PROBE
#define PDT_CONV_PROBE 0  // diagnostics only: 1 = DMA without MFMA, 2 = MFMA without DMA
#endif
template <class Cf>
__global__ __launch_bounds__(Cf::kThreads, Cf::kThreads / 128) void conv3x3s1_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, int N, int H, int W,
    int Ci, int Co) {
  constexpr int BM = Cf::BM, BN = Cf::BN, BK = Cf::BK, ROW = Cf::kRow, RPI = Cf::kRPI, CPR = BK / 8;
  constexpr int WROWS = BM / Cf::WM, WCOLS = BN / Cf::WN;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % Cf::WM, wn = wid / Cf::WM;
  const int HW = H * W;
  const int M = N * HW;
  const int ntiles = Co / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;

  // ---- rows this lane DMAs: A rows (wid*kALd + i)*RPI + lane/CPR, chunk lane%CPR (pre-swizzled)
  const int sub = lane / CPR, p = lane % CPR;
  int aoff[Cf::kALd];
  unsigned amask[Cf::kALd];
#pragma unroll
  for (int i = 0; i < Cf::kALd; ++i) {
    const int r = (wid * Cf::kALd + i) * RPI + sub;
    const int m = m0 + r;
    const int chk = (swz<ROW>(r, p) - r * ROW) >> 4;  // logical chunk stored at physical p
    unsigned mk = 0;
    aoff[i] = chk * 8;
    if (m < M) {
      const int rem = m % HW, oh = rem / W, ow = rem % W;
      aoff[i] += m * Ci;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ih = oh + kh - 1, iw = ow + kw - 1;
          if (ih >= 0 && ih < H && iw >= 0 && iw < W) mk |= 1u << (kh * 3 + kw);
        }
    }
    amask[i] = mk;
  }
  int boff[Cf::kBLd];
#pragma unroll
  for (int j = 0; j < Cf::kBLd; ++j) {
    const int r = (wid * Cf::kBLd + j) * RPI + sub;
    boff[j] = (n0 + r) * 9 * Ci + ((swz<ROW>(r, p) - r * ROW) >> 4) * 8;
  }
  const int kcc = Ci / BK;
  const int S = 9 * kcc;

  auto issue = [&](int s) {
    const int tap = s % 9, cc = s / 9;
    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = ((kh - 1) * W + (kw - 1)) * Ci + cc * BK;
    char* slot = lds + (s % kSlots) * Cf::kSlot;
#pragma unroll
    for (int i = 0; i < Cf::kALd; ++i) {
      const uint16_t* src =
          ((amask[i] >> tap) & 1u) ? X + (aoff[i] + toff) : reinterpret_cast<const uint16_t*>(g_conv_zero);
      dma16(src, slot + (wid * Cf::kALd + i) * 1024);
    }
    const int wo = tap * Ci + cc * BK;
#pragma unroll
    for (int j = 0; j < Cf::kBLd; ++j)
      dma16(Wt + (boff[j] + wo), slot + Cf::kABytes + (wid * Cf::kBLd + j) * 1024);
  };

  f4 acc[Cf::kMB][Cf::kNB];
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (S > 1) issue(1);
  const int lrow = lane & 15, lchk = lane >> 4;
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) wait_vm<Cf::kG>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (PDT_CONV_PROBE != 2 && s + 2 < S) issue(s + 2);
    if (PDT_CONV_PROBE == 1) continue;
    const char* As = lds + (s % kSlots) * Cf::kSlot;
    const char* Bs = As + Cf::kABytes;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 a[Cf::kMB], b[Cf::kNB];
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(As + swz<ROW>(wm * WROWS + i * 16 + lrow, kk * 4 + lchk));
#pragma unroll
      for (int j = 0; j < Cf::kNB; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + swz<ROW>(wn * WCOLS + j * 16 + lrow, kk * 4 + lchk));
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
        for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // D[co][m]
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // ---- epilogue: bf16 tile [BM pixels][BN] through LDS, then 16-B row pieces to Y
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) {
      const int ml = wm * WROWS + i * 16 + lrow;
      const int cl = wn * WCOLS + j * 16 + 4 * lchk;
      const f4 v = acc[i][j];
      uint2 pk;
      pk.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
             ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
      pk.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
             ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
      *reinterpret_cast<uint2*>(lds + ml * Cf::kEpiStride + cl * 2) = pk;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  constexpr int kChunks = BN / 8;
  for (int idx = tid; idx < BM * kChunks; idx += Cf::kThreads) {
    const int r = idx / kChunks, c = idx % kChunks;
    const int m = m0 + r;
    if (m < M)
      *reinterpret_cast<uint4*>(Y + (int64_t)m * Co + n0 + c * 8) =
          *reinterpret_cast<const uint4*>(lds + r * Cf::kEpiStride + c * 16);
  }
}

// ---------------------------------------------------------------- halo variant (default)
// The per-tap kernel above DMAs its A tile once per TAP: every input pixel crosses L2 -> LDS nine
// times, and at 48 KB per k-step the L2 -> LDS path (~60-70 GB/s per CU) bounds it near 0.8 PF
// (SQ_VALU_MFMA_BUSY 37 %). Here the A operand of one 32-channel chunk is staged ONCE as the
// tile's padded input halo — the input rows its 256 output pixels touch, each row W+2 pixels wide
// (pad columns and rows DMA'd from the zero page) — and the nine taps read shifted fragment rows
// out of it: LDS row of (pixel m, tap kh,kw) = base(m) + kh*(W+2) + kw. Only the weights stream
// per tap. LDS: 2 halo buffers (chunk c computes while c+1 lands) + 2 weight slots = 80 KB ->
// two workgroups per CU.
template <int BN_, int WM_, int WN_, int TPS_ = 1>
struct HCfg {
  static constexpr int BM = 256, BN = BN_, WM = WM_, WN = WN_, BK = 32, TPS = TPS_;  // TPS: taps per k-step
  static constexpr int kThreads = WM * WN * 64;
  static constexpr int kWaves = WM * WN;
  static constexpr int kRow = 64;
  static constexpr int kHaloRows = 512;  // >= padded-halo rows of any 256-pixel tile (host-checked)
  static constexpr int kHaloBytes = kHaloRows * kRow;
  static constexpr int kBBytes = TPS * BN * kRow;  // [tap of the step][co] rows
  static constexpr int kHLd = kHaloRows / 16 / kWaves;  // halo DMA instructions per wave
  static constexpr int kBLd = TPS * BN / 16 / kWaves;   // weight DMA instructions per wave per step
  static constexpr int kMB = BM / WM / 16, kNB = BN / WN / 16;
  static constexpr int kEpiStride = BN * 2 + 16;
  static constexpr int kMain = 2 * kHaloBytes + 2 * kBBytes;
  static constexpr int kEpi = BM * kEpiStride + tile_bn_stats_lds<BM, BN, kThreads>();  // staged tile + stats
  static constexpr int kLds = kMain > kEpi ? kMain : kEpi;
  static constexpr int kOcc = (160 * 1024) / kLds;  // workgroups per CU (LDS-limited)
  static constexpr int kMinWaves = kOcc * kThreads / 256 > 0 ? kOcc * kThreads / 256 : 1;  // per SIMD
  static_assert(kHLd * 16 * kWaves == kHaloRows && kBLd * 16 * kWaves == TPS * BN, "DMA split");
  static_assert(9 % TPS == 0 && 9 / TPS >= 3, "halo hand-off needs >= 3 steps per chunk");
};

__device__ __forceinline__ int chk64(int row, int p) { return p ^ (((row >> 2) & 1) << 1); }  // = swz<64>, involution

// BSTATS: Y is the gradient at a BatchNorm's output (this launch is a data gradient): its backward
// reduction is taken in the epilogue (tile_stats.h bn_bwd_accum8 / bn_bwd_tile_store).
template <class Cf, bool STATS = false, bool BSTATS = false, bool AD = false>
__global__ __launch_bounds__(Cf::kThreads, Cf::kMinWaves) void conv3x3h_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ Wt, uint16_t* __restrict__ Y, int N, int H, int W,
    int Ci, int Co, float* __restrict__ part, BnSrc bs) {
  constexpr int BM = Cf::BM, BN = Cf::BN, BK = Cf::BK;
  constexpr int WROWS = BM / Cf::WM, WCOLS = BN / Cf::WN;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % Cf::WM, wn = wid / Cf::WM;
  const int HW = H * W, M = N * HW, W2 = W + 2, H2 = H + 2;
  const int ntiles = Co / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
  const int mlast = min(m0 + BM, M) - 1;
  const int pr0 = (m0 / HW) * H2 + (m0 % HW) / W;  // padded row of (n_first, oh_first - 1)
  const int Q = ((mlast / HW) * H2 + (mlast % HW) / W + 2 - pr0 + 1) * W2;

  const int sub = lane >> 2, p = lane & 3;
  int hoff[Cf::kHLd];  // element offset of this lane's halo piece, -1 = zero page
#pragma unroll
  for (int i = 0; i < Cf::kHLd; ++i) {
    const int q = (wid * Cf::kHLd + i) * 16 + sub;
    int off = -1;
    if (q < Q) {
      const int PR = pr0 + q / W2, col = q % W2;
      const int n = PR / H2, ih = PR % H2 - 1, iw = col - 1;
      if (ih >= 0 && ih < H && iw >= 0 && iw < W && n < N) off = ((n * H + ih) * W + iw) * Ci + chk64(q, p) * 8;
    }
    hoff[i] = off;
  }
  int boff[Cf::kBLd];
#pragma unroll
  for (int j = 0; j < Cf::kBLd; ++j) {
    const int r = (wid * Cf::kBLd + j) * 16 + sub;  // [u][co], u = tap within the step
    boff[j] = (n0 + r % BN) * 9 * Ci + (r / BN) * Ci + chk64(r, p) * 8;
  }
  constexpr int SPC = 9 / Cf::TPS;  // steps per chunk
  const int lrow = lane & 15, lchk = lane >> 4;
  int abase[Cf::kMB];
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i) {
    const int m = min(m0 + wm * WROWS + i * 16 + lrow, mlast);  // rows past M: computed, never stored
    const int n = m / HW, rem = m % HW, oh = rem / W, ow = rem % W;
    abase[i] = (n * H2 + oh - pr0) * W2 + ow;
  }
  const int nch = Ci / BK;
  const int S = SPC * nch;
  char* const halo0 = lds;
  char* const bslot0 = lds + 2 * Cf::kHaloBytes;

  auto issue_halo = [&](int c) {
    char* hb = halo0 + (c & 1) * Cf::kHaloBytes;
#pragma unroll
    for (int i = 0; i < Cf::kHLd; ++i) {
      const uint16_t* src = hoff[i] >= 0 ? X + (hoff[i] + c * BK) : reinterpret_cast<const uint16_t*>(g_conv_zero);
      dma16x<AD>(src, hb + (wid * Cf::kHLd + i) * 1024);
    }
  };
  auto issue_b = [&](int s) {
    const int c = s / SPC, g = s - SPC * c;
    char* bs = bslot0 + (s & 1) * Cf::kBBytes;
#pragma unroll
    for (int j = 0; j < Cf::kBLd; ++j)
      dma16x<AD>(Wt + (boff[j] + g * Cf::TPS * Ci + c * BK), bs + (wid * Cf::kBLd + j) * 1024);
  };

  f4 acc[Cf::kMB][Cf::kNB];
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  issue_halo(0);
  issue_b(0);
  bool pend = false;  // a halo DMA was issued after the last weight DMA (wave-uniform)
  for (int s = 0; s < S; ++s) {
    // weights of step s (issued last step) and, at a chunk start, its halo (issued 8 steps ago
    // and retired two steps after issue by the in-order vmcnt) are resident once every wave has
    // waited for its own DMA and passed the barrier
    if (pend) wait_vm<Cf::kHLd>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    pend = false;
    const int c = s / SPC, g = s - SPC * c;
    if (s + 1 < S) issue_b(s + 1);
    if (g == 1 && c + 1 < nch) {  // buffer (c+1)&1 was last read in chunk c-1: every wave is past it
      issue_halo(c + 1);
      pend = true;
    }
    const char* hb = halo0 + (c & 1) * Cf::kHaloBytes;
    const char* bs = bslot0 + (s & 1) * Cf::kBBytes;
    bf16x8 a[2][Cf::kMB], b[2][Cf::kNB];
    auto rd = [&](int u, int set) {  // fragments of tap g*TPS + u
      const int t = g * Cf::TPS + u;
      const int toff = (t / 3) * W2 + (t % 3);
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i) {
        const int q = abase[i] + toff;
        a[set][i] = *reinterpret_cast<const bf16x8*>(hb + q * 64 + (chk64(q, lchk) << 4));
      }
#pragma unroll
      for (int j = 0; j < Cf::kNB; ++j) {
        const int r = u * BN + wn * WCOLS + j * 16 + lrow;
        b[set][j] = *reinterpret_cast<const bf16x8*>(bs + r * 64 + (chk64(r, lchk) << 4));
      }
    };
    rd(0, 0);
#pragma unroll
    for (int u = 0; u < Cf::TPS; ++u) {
      if (u + 1 < Cf::TPS) rd(u + 1, (u + 1) & 1);  // next tap's reads under this tap's MFMAs
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
        for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = mfma(b[u & 1][j], a[u & 1][i], acc[i][j]);  // D[co][m]
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) {
      const int ml = wm * WROWS + i * 16 + lrow;
      const int cl = wn * WCOLS + j * 16 + 4 * lchk;
      const f4 v = acc[i][j];
      uint2 pk;
      pk.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
             ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
      pk.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
             ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
      *reinterpret_cast<uint2*>(lds + ml * Cf::kEpiStride + cl * 2) = pk;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  constexpr int kChunks = BN / 8;
  static_assert(Cf::kThreads % kChunks == 0, "a thread keeps one 8-channel chunk");
  // STATS: BatchNorm statistics of the stored bf16 values from the epilogue's registers (tile_stats.h
  // RowStats8: no extra passes over the staged tile)
  RowStats8 rst;
  float kst = 0.f;
  if constexpr (STATS) {
    rs8_init(rst, *reinterpret_cast<const uint4*>(lds + (tid % kChunks) * 16));
    if (tid < BN) kst = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(lds + tid * 2) << 16);
  }
  float bs1[8], bs2[8], bmu[8];
  if constexpr (BSTATS) {
    const int c = tid % kChunks;
    *reinterpret_cast<float4*>(bmu) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8);
    *reinterpret_cast<float4*>(bmu + 4) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8 + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) { bs1[k] = 0.f; bs2[k] = 0.f; }
  }
  // Rows in batches whose BN-input loads are all issued before the first use, branch-free (a row past
  // M reads the last valid row and adds nothing; a null mask reads a 0xff byte). Written per row with
  // conditions, every row's loads waited a full memory latency (hipcc branches around a conditional
  // load and waits inside the branch, cdna_hip_programming.md §5 trap (c)): the BN-reduction data
  // gradient ran ~30 us per call slower than the forward (profiles/r5).
  constexpr int kRowIt = BM * kChunks / Cf::kThreads;
  constexpr int kBt = BSTATS && kRowIt > 4 ? 4 : kRowIt;
  static_assert(kRowIt * Cf::kThreads == BM * kChunks && kRowIt % kBt == 0, "epilogue rows");
  const uint8_t* const bm_base = bs.mask ? bs.mask : g_conv_ones;
  const int64_t bm_scale = bs.mask ? 1 : 0;
#pragma unroll 1
  for (int h = 0; h < kRowIt; h += kBt) {
    uint4 xbv[kBt];
    unsigned mkv[kBt];
#pragma unroll
    for (int it = 0; it < kBt; ++it) {
      if constexpr (BSTATS) {
        const int idx = tid + (h + it) * Cf::kThreads, r = idx / kChunks, cc = idx % kChunks;
        const int m = m0 + r, mc = m < M ? m : M - 1;
        const int64_t off = (int64_t)mc * Co + n0 + cc * 8;
        xbv[it] = *reinterpret_cast<const uint4*>(bs.x + off);
        const unsigned mk = bm_base[(off >> 3) * bm_scale];
        mkv[it] = m < M ? mk : 0u;
      }
    }
#pragma unroll
    for (int it = 0; it < kBt; ++it) {
      const int idx = tid + (h + it) * Cf::kThreads, r = idx / kChunks, cc = idx % kChunks;
      const int m = m0 + r;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + r * Cf::kEpiStride + cc * 16);
      if constexpr (BSTATS) bn_bwd_accum8(v, xbv[it], mkv[it], bmu, bs1, bs2);
      if (m >= M) continue;
      if constexpr (STATS) rs8_add(rst, v);
      *reinterpret_cast<uint4*>(Y + (int64_t)m * Co + n0 + cc * 8) = v;
    }
  }
  if constexpr (BSTATS)  // every wave is done reading the staged tile: its LDS holds the block sums
    bn_bwd_tile_store<BN, Cf::kWaves>(bs1, bs2, reinterpret_cast<float*>(lds), bs.part, (M + BM - 1) / BM, m0 / BM,
                                      Co, n0);
  if constexpr (STATS) {
    __syncthreads();  // (likewise)
    rs8_tile_store<BN, Cf::kWaves>(rst, kst, reinterpret_cast<float*>(lds), part, min(BM, M - m0), (M + BM - 1) / BM,
                                   m0 / BM, Co, n0);
  }
}

// ---------------------------------------------------------------- warp-specialised halo variant
// Counters on the two kernels above (SQ_VALU_MFMA_BUSY 37-40 %, SQ_WAIT_ANY 33 %) point at their
// barrier-per-k-step structure: every 16 MFMAs per wave all waves meet, issue DMA, and wait for
// fresh LDS reads before the matrix pipe restarts. Here one workgroup = 4 consumer waves (one per
// SIMD, 64 pixels x 64 channels each) + NL loader waves, and the unit of synchronisation is a whole
// 32-channel chunk: its padded input halo AND the weights of all nine taps (68 KB) sit in one of two
// LDS buffers, so a consumer runs 9 x 16 MFMAs with its fragment reads for tap t+1 issued under the
// MFMAs of tap t and meets the others once per chunk. Loader waves DMA chunk c+1 into the other
// buffer meanwhile (their DMA issue never blocks a consumer's MFMA issue).
template <int NL_>
struct WCfg {
  static constexpr int BM = 256, BN = 64, BK = 32, NL = NL_;
  static constexpr int kThreads = (4 + NL) * 64;
  static constexpr int kHaloRows = 512;
  static constexpr int kHaloBytes = kHaloRows * 64;  // 32 KB
  static constexpr int kBRows = 9 * BN;              // [tap][co]
  static constexpr int kBBytes = kBRows * 64;        // 36 KB
  static constexpr int kBuf = kHaloBytes + kBBytes;
  static constexpr int kHIns = kHaloRows / 16 / NL, kBIns = kBRows / 16 / NL;  // DMA instrs per loader
  static constexpr int kEpiStride = BN * 2 + 16;
  static constexpr int kLds = 2 * kBuf;
  static_assert(kHIns * 16 * NL == kHaloRows && kBIns * 16 * NL == kBRows, "DMA split");
  static_assert(BM * kEpiStride <= kLds, "epilogue");
};

template <class Cf>
__global__ __launch_bounds__(Cf::kThreads, 1) void conv3x3ws_kernel(const uint16_t* __restrict__ X,
                                                                  const uint16_t* __restrict__ Wt,
                                                                  uint16_t* __restrict__ Y, int N, int H, int W,
                                                                  int Ci, int Co) {
  constexpr int BM = Cf::BM, BN = Cf::BN, BK = Cf::BK;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool loader = wid >= 4;
  const int HW = H * W, M = N * HW, W2 = W + 2, H2 = H + 2;
  const int ntiles = Co / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / ntiles) * BM, n0 = (tile % ntiles) * BN;
  const int mlast = min(m0 + BM, M) - 1;
  const int pr0 = (m0 / HW) * H2 + (m0 % HW) / W;
  const int Q = ((mlast / HW) * H2 + (mlast % HW) / W + 2 - pr0 + 1) * W2;
  const int nch = Ci / BK;

  // loader state: element offsets of this lane's halo and weight pieces (-1 = zero page)
  int hoff[Cf::kHIns], boff[Cf::kBIns];
  const int sub = lane >> 2, p = lane & 3;
  if (loader) {
    const int l = wid - 4;
#pragma unroll
    for (int i = 0; i < Cf::kHIns; ++i) {
      const int q = (l * Cf::kHIns + i) * 16 + sub;
      int off = -1;
      if (q < Q) {
        const int PR = pr0 + q / W2, col = q % W2;
        const int n = PR / H2, ih = PR % H2 - 1, iw = col - 1;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W && n < N) off = ((n * H + ih) * W + iw) * Ci + chk64(q, p) * 8;
      }
      hoff[i] = off;
    }
#pragma unroll
    for (int j = 0; j < Cf::kBIns; ++j) {
      const int r = (l * Cf::kBIns + j) * 16 + sub;  // [tap][co] row
      const int t = r / BN, co = r % BN;
      boff[j] = (n0 + co) * 9 * Ci + t * Ci + chk64(r, p) * 8;
    }
  }
  auto dma_chunk = [&](int c) {
    const int l = wid - 4;
    char* buf = lds + (c & 1) * Cf::kBuf;
#pragma unroll
    for (int i = 0; i < Cf::kHIns; ++i) {
      const uint16_t* src = hoff[i] >= 0 ? X + (hoff[i] + c * BK) : reinterpret_cast<const uint16_t*>(g_conv_zero);
      dma16(src, buf + (l * Cf::kHIns + i) * 1024);
    }
#pragma unroll
    for (int j = 0; j < Cf::kBIns; ++j) dma16(Wt + (boff[j] + c * BK), buf + Cf::kHaloBytes + (l * Cf::kBIns + j) * 1024);
  };

  // consumer state
  const int lrow = lane & 15, lchk = lane >> 4;
  int abase[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = min(m0 + wid * 64 + i * 16 + lrow, mlast);
    const int n = m / HW, rem = m % HW, oh = rem / W, ow = rem % W;
    abase[i] = (n * H2 + oh - pr0) * W2 + ow;
  }
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  if (loader) {
    dma_chunk(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int c = 0; c < nch; ++c) {
    if (loader) {
      if (c + 1 < nch) {
        dma_chunk(c + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      const char* hb = lds + (c & 1) * Cf::kBuf;
      const char* bb = hb + Cf::kHaloBytes;
      bf16x8 a[2][4], b[2][4];
      auto rd = [&](int t, int set) {
        const int toff = (t / 3) * W2 + (t % 3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = abase[i] + toff;
          a[set][i] = *reinterpret_cast<const bf16x8*>(hb + q * 64 + (chk64(q, lchk) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = t * BN + j * 16 + lrow;
          b[set][j] = *reinterpret_cast<const bf16x8*>(bb + r * 64 + (chk64(r, lchk) << 4));
        }
      };
      rd(0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t < 8) rd(t + 1, (t + 1) & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma(b[t & 1][j], a[t & 1][i], acc[i][j]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  if (!loader) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ml = wid * 64 + i * 16 + lrow;
        const int cl = j * 16 + 4 * lchk;
        const f4 v = acc[i][j];
        uint2 pk;
        pk.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
               ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
        pk.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
               ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
        *reinterpret_cast<uint2*>(lds + ml * Cf::kEpiStride + cl * 2) = pk;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  constexpr int kChunks = BN / 8;
  for (int idx = tid; idx < BM * kChunks; idx += Cf::kThreads) {
    const int r = idx / kChunks, cc = idx % kChunks;
    const int m = m0 + r;
    if (m < M)
      *reinterpret_cast<uint4*>(Y + (int64_t)m * Co + n0 + cc * 8) =
          *reinterpret_cast<const uint4*>(lds + r * Cf::kEpiStride + cc * 16);
  }
}

// ---------------------------------------------------------------- weight-stationary persistent variant
// For small filters (ResNet-50 layer 1: 64 -> 64 channels, 74 KB of bf16 weights) every variant
// above spends as long on per-tile overhead as on MFMA work: a 256 x 64 tile is only 19 MFLOP, so
// the first DMA's latency, the barriers and the epilogue of every tile sit on the critical path
// (all of them ran layer 1 at 0.45 PF). Here the weights are loaded into LDS ONCE per workgroup,
// one workgroup per CU walks a contiguous range of pixel tiles, and the 32-channel halo chunks of
// consecutive tiles stream through two LDS buffers without a break: loader waves DMA pair k+1
// (tile, chunk) while the consumers compute pair k, and a tile's results go straight from the
// accumulators to HBM (8-B stores, no LDS round trip) while the next tile's halo is landing.
template <int CI_, int CO_>
struct SCfg {
  static constexpr int BM = 256, BK = 32, CI = CI_, CO = CO_, NL = 4;
  static constexpr int kThreads = (4 + NL) * 64;
  static constexpr int kHaloRows = 640, kHaloBytes = kHaloRows * 64;  // W=56 tiles crossing an image: 580
  static constexpr int kNch = CI / BK;
  static constexpr int kWRows = kNch * 9 * CO;  // [chunk][tap][co] rows of 64 B
  static constexpr int kWBytes = kWRows * 64;
  static constexpr int kStatBytes = 4 * 2 * CO * 4;  // per consumer wave: (sum, M2) x CO
  static constexpr int kLds = kWBytes + 2 * kHaloBytes + kStatBytes;
  static constexpr int kHIns = kHaloRows / 16 / NL;
  static_assert(CO == 64, "4 consumer waves x 64 pixels x 64 channels");
  static_assert(kWRows % (16 * (4 + NL)) == 0, "weight DMA split");
  static_assert(kLds <= 160 * 1024, "LDS");
};

// STATS: the BatchNorm statistics of each 256-pixel tile, as in the halo kernel's epilogue
// (tile_stats.h layout, BM = 256 rows per tile), taken from the accumulators: each consumer wave
// reduces its 64 rows across the 16 row lanes (sum, then the CENTRED sum of squares about its own
// mean), parks them in LDS at the tile's end, and consumer wave 0 merges the four 64-row chunks
// (Chan's formula) after the next barrier while the other waves already compute the next tile:
// 437 us per call vs 390 us + a 97 us reduce pass (layer 1, batch 1024). (The backward reduction
// the same way — the BatchNorm input read with 8-B per-lane loads in the epilogue, or prefetched
// under the last chunk's MFMAs — ran 688-771 us vs 385 us + a 140 us reduce pass: not kept.)
template <class Cf, bool STATS = false, bool PIPE = true>
__global__ __launch_bounds__(Cf::kThreads, 1) void conv3x3wst_kernel(const uint16_t* __restrict__ X,
                                                                   const uint16_t* __restrict__ Wt,
                                                                   uint16_t* __restrict__ Y, int N, int H, int W,
                                                                   float* __restrict__ part, int opt) {
  constexpr int BM = Cf::BM, BK = Cf::BK, CI = Cf::CI, CO = Cf::CO, NCH = Cf::kNch;
  const bool kSkipDead = opt & 1;
  constexpr bool kRed = STATS;
  static_assert(!kRed || NCH >= 2, "a parked chunk is merged before the next tile's end overwrites it");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const wlds = lds;
  char* const halo0 = lds + Cf::kWBytes;
  float* const statb = reinterpret_cast<float*>(lds + Cf::kWBytes + 2 * Cf::kHaloBytes);  // [wave][2][CO]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool loader = wid >= 4;
  const int HW = H * W, M = N * HW, W2 = W + 2, H2 = H + 2;
  const int ntile = (M + BM - 1) / BM;
  // contiguous tile range per workgroup: neighbouring tiles share halo rows (L2 hits)
  const int g = gridDim.x, b = blockIdx.x;
  const int t_begin = (int)((int64_t)ntile * b / g), t_end = (int)((int64_t)ntile * (b + 1) / g);
  const int K = (t_end - t_begin) * NCH;  // (tile, chunk) pairs of this workgroup
  const int sub = lane >> 2, p = lane & 3;

  // weights: every wave DMAs its share once
  {
    constexpr int kIns = Cf::kWRows / 16 / (4 + Cf::NL);
#pragma unroll
    for (int i = 0; i < kIns; ++i) {
      const int r = (wid * kIns + i) * 16 + sub;  // [c][t][co]
      const int c = r / (9 * CO), t = (r / CO) % 9, co = r % CO;
      dma16(Wt + (co * 9 + t) * CI + c * BK + chk64(r, p) * 8, wlds + (wid * kIns + i) * 1024);
    }
  }
  auto tile_geo = [&](int tl, int& m0, int& mlast, int& pr0, int& Q) {
    m0 = tl * BM;
    mlast = min(m0 + BM, M) - 1;
    pr0 = (m0 / HW) * H2 + (m0 % HW) / W;
    Q = ((mlast / HW) * H2 + (mlast % HW) / W + 2 - pr0 + 1) * W2;
  };
  auto dma_halo = [&](int k) {
    const int tl = t_begin + k / NCH, c = k % NCH;
    int m0, mlast, pr0, Q;
    tile_geo(tl, m0, mlast, pr0, Q);
    const int l = wid - 4;
    char* hb = halo0 + (k & 1) * Cf::kHaloBytes;
#pragma unroll
    for (int i = 0; i < Cf::kHIns; ++i) {
      // rows past the tile's halo are never read: skip whole 16-row DMA instructions (wave-uniform)
      if (kSkipDead && (l * Cf::kHIns + i) * 16 >= Q) break;
      const int q = (l * Cf::kHIns + i) * 16 + sub;
      const uint16_t* src = reinterpret_cast<const uint16_t*>(g_conv_zero);
      if (q < Q) {
        const int PR = pr0 + q / W2, col = q % W2;
        const int n = PR / H2, ih = PR % H2 - 1, iw = col - 1;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W && n < N)
          src = X + (((n * H + ih) * W + iw) * CI + c * BK + chk64(q, p) * 8);
      }
      dma16(src, hb + (l * Cf::kHIns + i) * 1024);
    }
  };

  const int lrow = lane & 15, lchk = lane >> 4;
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  int abase[4];
  int cur_m0 = 0, cur_mlast = -1;
  const int ntile_all = ntile;
  // merge the four parked 64-row chunks of tile `tl` (consumer wave 0, one channel per lane)
  auto merge = [&](int tl) {
    const int m0 = tl * BM, mlast = min(m0 + BM, M) - 1;
    float S = 0.f, nt = 0.f, Q;
    float sw[4], qw[4], nw[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      nw[w] = (float)max(0, min(64, mlast - (m0 + 64 * w) + 1));
      sw[w] = statb[(w * 2) * CO + lane];
      qw[w] = statb[(w * 2 + 1) * CO + lane];
      S += sw[w];
      nt += nw[w];
    }
    // Chan: M2 = sum M2_w + sum n_w (mu_w - mu)^2
    const float mu = S / nt;
    Q = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      if (nw[w] > 0.f) {
        const float d = sw[w] / nw[w] - mu;
        Q += qw[w] + nw[w] * d * d;
      }
    part[(int64_t)tl * CO + lane] = S;
    part[((int64_t)ntile_all + tl) * CO + lane] = Q;
  };
  int pending = -1;  // tile whose parked chunks wave 0 merges after the next barrier

  if (loader && K > 0) dma_halo(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int k = 0; k < K; ++k) {
    if (loader) {
      if (k + 1 < K && !(opt & 2)) {
        dma_halo(k + 1);
        if (!(opt & 16)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      const int tl = t_begin + k / NCH, c = k % NCH;
      if constexpr (kRed) {
        if (pending >= 0 && wid == 0) merge(pending);
        pending = -1;
      }
      if (c == 0) {  // new tile: fragment row bases
        int pr0, Q;
        tile_geo(tl, cur_m0, cur_mlast, pr0, Q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = min(cur_m0 + wid * 64 + i * 16 + lrow, cur_mlast);
          const int n = m / HW, rem = m % HW, oh = rem / W, ow = rem % W;
          abase[i] = (n * H2 + oh - pr0) * W2 + ow;
        }
      }
      const char* hb = halo0 + (k & 1) * Cf::kHaloBytes;
      const char* wb = wlds + c * 9 * CO * 64;
      bf16x8 a[2][4], bq[2][4];
      auto rd = [&](int t, int set) {
        const int toff = (t / 3) * W2 + (t % 3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = abase[i] + toff;
          a[set][i] = *reinterpret_cast<const bf16x8*>(hb + q * 64 + (chk64(q, lchk) << 4));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = c * 9 * CO + t * CO + j * 16 + lrow;
          bq[set][j] = *reinterpret_cast<const bf16x8*>(wlds + r * 64 + (chk64(r, lchk) << 4));
        }
      };
      (void)wb;
      if (!(opt & 4)) {
      rd(0, 0);
      if constexpr (PIPE) {
        // One consumer wave per SIMD: nothing hides a fragment read's latency but this wave's own
        // MFMAs, so pin the software pipeline (tap t+1's reads issued, then tap t's 16 MFMAs) against
        // the scheduler, which otherwise interleaves reads and MFMAs with a full lgkmcnt(0) wait
        // every 4 MFMAs.
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          if (t < 8) rd(t + 1, (t + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma(bq[t & 1][j], a[t & 1][i], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t < 8) rd(t + 1, (t + 1) & 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma(bq[t & 1][j], a[t & 1][i], acc[i][j]);
      }
      }
      }
      if (c == NCH - 1) {  // tile done: accumulators straight to HBM (4 channels = 8 B per lane)
        float s1[4][4], s2[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) s1[j][e] = s2[j][e] = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = cur_m0 + wid * 64 + i * 16 + lrow;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f4 v = acc[i][j];
            if (m <= cur_mlast) {
              uint2 pk;
              pk.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
                     ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
              pk.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
                     ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
              const int64_t off = (int64_t)m * CO + j * 16 + 4 * lchk;
              *reinterpret_cast<uint2*>(Y + off) = pk;
              // the statistics are of the values written (bf16-rounded)
              v = f4{__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u), __uint_as_float(pk.y << 16),
                     __uint_as_float(pk.y & 0xffff0000u)};
              if constexpr (STATS) {
#pragma unroll
                for (int e = 0; e < 4; ++e) s1[j][e] += v[e];
              }
            }
            acc[i][j] = v;  // STATS: the rounded values, for the centred second pass
          }
        }
        if constexpr (kRed) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              s1[j][e] = row16_sum(s1[j][e]);  // over the 16 pixel lanes (DPP, no LDS)
          {  // centred sum of squares about this wave's 64-row mean
            const int nw = max(0, min(64, cur_mlast - (cur_m0 + wid * 64) + 1));
            const float inv = nw > 0 ? 1.f / (float)nw : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bool ok = cur_m0 + wid * 64 + i * 16 + lrow <= cur_mlast;
#pragma unroll
              for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float d = acc[i][j][e] - s1[j][e] * inv;
                  s2[j][e] += ok ? d * d : 0.f;
                }
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              s2[j][e] = row16_sum(s2[j][e]);
          if (lrow == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                statb[(wid * 2) * CO + j * 16 + 4 * lchk + e] = s1[j][e];
                statb[(wid * 2 + 1) * CO + j * 16 + 4 * lchk + e] = s2[j][e];
              }
          }
          pending = tl;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if constexpr (kRed) {  // the last tile's chunks (parked before the loop's final barrier)
    if (!loader && wid == 0 && pending >= 0) merge(pending);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (probe bit 4 leaves DMA in flight to here)
}

// ---------------------------------------------------------------- weight-stationary row-tile variant
// Layer 1 of ResNet-50 at 224 x 224 (64 -> 64 channels, 56 x 56). The persistent kernel above ran
// 385-436 us per call at 1024 images against a 94 us MFMA floor, and rocprofv3 counters
// (profiles/r5/pmc_conv3x3wst_layer1.md) put it at 24 % MFMA-busy with ~4 VALU instructions per MFMA:
// its 256-pixel tiles cross image rows and images, so every fragment row, halo row and DMA source is
// a runtime-divisor function of the tile (consumer and loader waves alike), and each chunk's halo DMA
// was drained before the next barrier (one chunk of lookahead). Here a tile is R = 224 / W WHOLE rows of
// one image (W = 56: 4 rows = 224 pixels), so
//   * every consumer lane's fragment rows are the same in every tile (computed once per launch) and a
//     halo row's (padded row, column) is a compile-time-divisor split of its index;
//   * the halo of a 32-channel chunk is (R + 2) padded rows with ONE pad column shared by consecutive
//     rows — (R + 2)(W + 1) + 1 = 343 rows of 64 B (21.4 KB) — so FOUR buffers fit next to the 72 KB of
//     stationary weights and loader waves keep three chunks in flight (counted vmcnt);
//   * 4 consumer waves as 2 (pixels) x 2 (channels), 112 x 32 each (7 x 2 v_mfma_f32_16x16x32_bf16),
//     results straight from the accumulators to HBM; BatchNorm statistics per 224-row tile (tile_stats.h
//     layout with BMt = 224: bn_fwd_train_tiles reads the tile height off the partials' row count).
// Requires H % R == 0 (tiles never cross images) and M % 224 == 0 follows.
template <int W_>
struct RCfg {
  static constexpr int W = W_, BM = 224, R = BM / W, CI = 64, CO = 64, BK = 32, NCH = 2, NL = 4, NBUF = 4;
  static constexpr int kThreads = (4 + NL) * 64;
  static constexpr int kStride = W + 1;                    // halo row pitch: one pad column between rows
  static constexpr int kHaloRows = (R + 2) * kStride + 1;  // 343 at W = 56
  static constexpr int kHaloBytes = kHaloRows * 64;
  static constexpr int kHIns = (kHaloRows + 15) / 16;      // 16-row DMA instructions per chunk (4 loaders)
  static constexpr int kWRows = NCH * 9 * CO, kWBytes = kWRows * 64;
  static constexpr int kStatBytes = 2 * 2 * CO * 4;        // [pixel half][sum, M2][co]
  static constexpr int kLds = kWBytes + NBUF * kHaloBytes + kStatBytes;
  static constexpr int kMB = BM / 2 / 16;                  // 16-pixel blocks per consumer wave
  static_assert(R * W == BM && BM % 32 == 0, "whole image rows, two 16-row-block halves");
  static_assert(kWRows % (16 * (4 + NL)) == 0, "weight DMA split");
  static_assert(kLds <= 160 * 1024, "LDS");
};

template <int N>
__device__ __forceinline__ void wait_vm_n() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N < 0, "vmcnt value");
}

// BSTATS: Y is the gradient at a BatchNorm's output (a data gradient): that BatchNorm's backward
// reduction (sum dz, sum dz (x - mean), dz = Y * ReLU mask) per 224-row tile into bs.part; the BN input
// and mask of the tile's pixels are loaded into registers at the start of its second chunk, under the
// MFMAs (28 + 7 VGPRs), and reduced from the accumulators like the forward statistics.
template <class Cf, bool STATS = false, bool BSTATS = false>
__global__ __launch_bounds__(Cf::kThreads, 1) void conv3x3wsr_kernel(const uint16_t* __restrict__ X,
                                                                   const uint16_t* __restrict__ Wt,
                                                                   uint16_t* __restrict__ Y, int N, int H,
                                                                   float* __restrict__ part, int opt, BnSrc bs) {
  static_assert(!(STATS && BSTATS), "one epilogue reduction");
  constexpr int W = Cf::W, R = Cf::R, BM = Cf::BM, BK = Cf::BK, CI = Cf::CI, CO = Cf::CO, NB = Cf::NBUF;
  constexpr int S = Cf::kStride, MB = Cf::kMB, HR = Cf::kHaloRows, HI = Cf::kHIns;
  constexpr int kSplit = 3;  // A blocks in the first read group of a tap
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const wlds = lds;
  char* const halo0 = lds + Cf::kWBytes;
  float* const statb = reinterpret_cast<float*>(lds + Cf::kWBytes + NB * Cf::kHaloBytes);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool loader = wid >= 4;
  const int tpi = H / R, ntile = N * tpi;
  const int g = gridDim.x, b = blockIdx.x;
  const int t_begin = (int)((int64_t)ntile * b / g), t_end = (int)((int64_t)ntile * (b + 1) / g);
  const int K = (t_end - t_begin) * 2;  // (tile, chunk) steps of this workgroup
  const int sub = lane >> 2, p = lane & 3;

  {  // weights [chunk][tap][co] rows of 64 B: every wave DMAs its share once
    constexpr int kIns = Cf::kWRows / 16 / (4 + Cf::NL);
#pragma unroll
    for (int i = 0; i < kIns; ++i) {
      const int r = (wid * kIns + i) * 16 + sub;
      const int c = r / (9 * CO), t = (r / CO) % 9, co = r % CO;
      dma16a(Wt + (co * 9 + t) * CI + c * BK + chk64(r, p) * 8, wlds + (wid * kIns + i) * 1024);
    }
  }
  // loader wave l issues the chunk's DMA instructions l, l + 4, ... (HI in all): nl of them
  const int l = wid - 4;
  const int nl = (HI - l + 3) / 4;
  // the zero page's address once (SGPRs), not a GOT load per DMA instruction inside the loop
  uint64_t zpa = reinterpret_cast<uint64_t>(g_conv_zero);
  asm volatile("" : "+s"(zpa));
  const uint16_t* const zpage = reinterpret_cast<const uint16_t*>(zpa);
  auto dma_halo = [&](int k) {
    const int tl = t_begin + (k >> 1), c = k & 1;
    const int n = tl / tpi, r0 = (tl - n * tpi) * R;
    char* hb = halo0 + (k % NB) * Cf::kHaloBytes;
    // loader and consumer roles share one register allocation: keep the loader's per-lane row math in
    // the loop (not hoisted and held live across the consumers' MFMA code)
    int lsub = sub;
    asm volatile("" : "+v"(lsub));
#pragma unroll
    for (int i = 0; i < (HI + 3) / 4; ++i) {
      const int gi = l + 4 * i;
      if (gi >= HI) break;  // wave-uniform
      const int q = gi * 16 + lsub;
      const int pr = q / S, pc = q - pr * S - 1, ih = r0 - 1 + pr;
      const uint16_t* src = zpage;
      if (pc >= 0 && pc < W && ih >= 0 && ih < H) src = X + (((n * H + ih) * W + pc) * CI + c * BK + chk64(q, p) * 8);
      if (q < HR) dma16a(src, hb + gi * 1024);  // the last instruction's rows past HR stay off
    }
  };
  auto wait_next = [&](int k) {  // chunk k + 1 landed: allow the DMAs of chunks k + 2 .. k + 3 in flight
    const int after = min(K - 1, k + 3) - (k + 1);
    if (after <= 0) wait_vm_n<0>();
    else if (after == 1) { if (nl == 6) wait_vm_n<6>(); else wait_vm_n<5>(); }
    else { if (nl == 6) wait_vm_n<12>(); else wait_vm_n<10>(); }
  };

  // consumer geometry: identical in every tile
  const int lrow = lane & 15, lchk = lane >> 4;
  const int wm = wid & 1, wn = (wid >> 1) & 1;
  // swizzled LDS offsets of every (block, tap) fragment row, relative to the halo buffer: the same in
  // every tile and chunk, so computed once (recomputing them costs ~5 VALU per fragment read, 3 VALU per
  // MFMA in all)
  // two 16-bit offsets per VGPR (offsets < 22 KB): 35 VGPRs instead of 63, unpacked by the address add
  // (BSTATS needs 35 more VGPRs in its epilogue than 256 allow with these held: it recomputes them)
  static_assert(Cf::kHaloBytes <= 65536, "16-bit fragment offsets");
  constexpr bool kHold = !BSTATS;
  uint32_t aoff[MB][5];
  int abase[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int mm = wm * (BM / 2) + i * 16 + lrow;
    const int ab = (mm / W) * S + mm % W;
    abase[i] = ab;
    if constexpr (kHold) {
#pragma unroll
      for (int u = 0; u < 5; ++u) {
        uint32_t v = 0;
#pragma unroll
        for (int h = 0; h < 2 && 2 * u + h < 9; ++h) {
          const int t = 2 * u + h;
          const int q = ab + (t / 3) * S + (t % 3);
          v |= (uint32_t)(q * 64 + (chk64(q, lchk) << 4)) << (16 * h);
        }
        aoff[i][u] = v;
        asm volatile("" : "+v"(aoff[i][u]));
      }
    }
  }
  const int bbase = lrow * 64 + (chk64(lrow, lchk) << 4) + (wn * 32) * 64;  // + (c*9*CO + t*CO + j*16) * 64
  f4 acc[MB][2];
  int pending = -1;
  float* const opart = BSTATS ? bs.part : part;
  auto merge = [&](int tl) {  // consumer wave 0: one channel per lane, over the two pixel halves
    const float S0 = statb[0 * CO + lane], Q0 = statb[1 * CO + lane];
    const float S1 = statb[2 * CO + lane], Q1 = statb[3 * CO + lane];
    opart[(int64_t)tl * CO + lane] = S0 + S1;
    if constexpr (BSTATS) {  // plain sums
      opart[((int64_t)ntile + tl) * CO + lane] = Q0 + Q1;
    } else {  // Chan's formula: centred sums of squares of two 112-row halves
      const float d = (S1 - S0) * (1.f / (BM / 2));
      opart[((int64_t)ntile + tl) * CO + lane] = Q0 + Q1 + d * d * (float)(BM / 4);
    }
  };
  // BSTATS: the mask base (all-ones page when there is no ReLU)
  const uint8_t* const bm_base = BSTATS && bs.mask ? bs.mask : g_conv_ones;
  const int64_t bm_scale = BSTATS && bs.mask ? 1 : 0;
  uint2 bxv[MB][2];
  uint32_t bmk[MB];

  if (loader) {
    for (int j = 0; j < 3 && j < K; ++j) dma_halo(j);
    const int after = min(K - 1, 2);  // chunks issued after chunk 0
    if (after <= 0) wait_vm_n<0>();
    else if (after == 1) { if (nl == 6) wait_vm_n<6>(); else wait_vm_n<5>(); }
    else { if (nl == 6) wait_vm_n<12>(); else wait_vm_n<10>(); }
  } else {
    wait_vm_n<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int tl = t_begin; tl < t_end; ++tl) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int k = (tl - t_begin) * 2 + c;
      if (loader) {
        if (k + 3 < K && !(opt & 2)) dma_halo(k + 3);
        wait_next(k);
      } else {
        if constexpr (STATS || BSTATS) {
          if (pending >= 0 && wid == 0) merge(pending);
          pending = -1;
        }
        // BSTATS: the tile's BN input and mask bits, loaded at the epilogue (held across the MFMAs, the 35
        // VGPRs spill: 256 per wave at two waves per SIMD)
        auto prefetch_bn = [&]() {
          int m0 = tl * BM + wm * (BM / 2) + lrow;
          asm volatile("" : "+v"(m0));  // per-lane address math stays here (hoisted, it would spill)
#pragma unroll
          for (int i = 0; i < MB; ++i) {
            const int64_t m = m0 + i * 16;
#pragma unroll
            for (int j = 0; j < 2; ++j)
              bxv[i][j] = *reinterpret_cast<const uint2*>(bs.x + m * CO + wn * 32 + j * 16 + 4 * lchk);
            bmk[i] = *reinterpret_cast<const uint32_t*>(bm_base + (m * (CO / 8) + wn * 4) * bm_scale);
          }
        };
        const char* hb = halo0 + (k % NB) * Cf::kHaloBytes;
        const char* wb = wlds + bbase + (c * 9 * CO) * 64;
        int ab[MB];
        if constexpr (!kHold) {
#pragma unroll
          for (int i = 0; i < MB; ++i) {
            ab[i] = abase[i];
            asm volatile("" : "+v"(ab[i]));
          }
        }
        auto frag_off = [&](int i, int t) -> uint32_t {
          if constexpr (kHold) {
            return (t & 1) ? (aoff[i][t >> 1] >> 16) : (aoff[i][t >> 1] & 0xffffu);
          } else {
            const int q = ab[i] + (t / 3) * S + (t % 3);
            return (uint32_t)(q * 64 + (chk64(q, lchk) << 4));
          }
        };
        bf16x8 a[2][MB], bq[2][2];
        // fragment reads of tap t in two groups: B + A blocks 0..2, then A blocks 3..6
        auto rd = [&](int t, int set, int part) {
          if (part == 0) {
#pragma unroll
            for (int j = 0; j < 2; ++j) bq[set][j] = *reinterpret_cast<const bf16x8*>(wb + (t * CO + j * 16) * 64);
          }
#pragma unroll
          for (int i = part == 0 ? 0 : kSplit; i < (part == 0 ? kSplit : MB); ++i)
            a[set][i] = *reinterpret_cast<const bf16x8*>(hb + frag_off(i, t));
        };
        auto mm = [&](int t, int i0, int i1) {
#pragma unroll
          for (int i = i0; i < i1; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = (c == 0 && t == 0) ? mfma(bq[0][j], a[0][i], f4{0.f, 0.f, 0.f, 0.f})
                                             : mfma(bq[t & 1][j], a[t & 1][i], acc[i][j]);
        };
        // One consumer wave per SIMD: only this wave's own MFMAs can hide its fragment reads, so the
        // software pipeline is pinned against the scheduler (which otherwise interleaves reads and
        // MFMAs with a full lgkmcnt(0) wait every 2 MFMAs): tap t+1's reads go out in two groups, each
        // ahead of half of tap t's MFMAs, so at most 14 LDS reads are ever outstanding — within the
        // 4-bit lgkmcnt, which lets the compiler wait for exactly the reads an MFMA group consumes
        // (9 per tap in one group would put 18 in flight and force lgkmcnt(0)).
        if (!(opt & 4)) {
        rd(0, 0, 0);
        rd(0, 0, 1);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          if (t < 8) rd(t + 1, (t + 1) & 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          mm(t, 0, kSplit + 1);
          __builtin_amdgcn_sched_barrier(0);
          if (t < 8) rd(t + 1, (t + 1) & 1, 1);
          __builtin_amdgcn_sched_barrier(0);
          mm(t, kSplit + 1, MB);
          __builtin_amdgcn_sched_barrier(0);
        }
        }
        if (c == 1) {  // tile done: bf16 results straight to HBM (4 channels = 8 B per lane)
          const int m0 = tl * BM + wm * (BM / 2);
          float s1[2][4], s2b[2][4];
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) s1[j][e] = s2b[j][e] = 0.f;
          float bmu[2][4];  // this lane's 8 channels' batch means (cache-resident; loaded here, not held)
          if constexpr (BSTATS) {
            prefetch_bn();
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float4 mv = *reinterpret_cast<const float4*>(bs.mean + wn * 32 + j * 16 + 4 * lchk);
              bmu[j][0] = mv.x; bmu[j][1] = mv.y; bmu[j][2] = mv.z; bmu[j][3] = mv.w;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetched BN inputs and the means
          }
#pragma unroll
          for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f4 v = acc[i][j];
              uint2 pk;
              pk.x = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
                     ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
              pk.y = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
                     ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
              *reinterpret_cast<uint2*>(Y + (int64_t)(m0 + i * 16 + lrow) * CO + wn * 32 + j * 16 + 4 * lchk) = pk;
              if constexpr (BSTATS) {  // dz = written value x mask; sums of dz and dz (x - mean)
                const float gv[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                                     __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
                const float xv[4] = {__uint_as_float(bxv[i][j].x << 16), __uint_as_float(bxv[i][j].x & 0xffff0000u),
                                     __uint_as_float(bxv[i][j].y << 16), __uint_as_float(bxv[i][j].y & 0xffff0000u)};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float dz = (bmk[i] >> (j * 16 + 4 * lchk + e)) & 1u ? gv[e] : 0.f;
                  s1[j][e] += dz;
                  s2b[j][e] += dz * (xv[e] - bmu[j][e]);
                }
              }
              if constexpr (STATS) {  // statistics of the values written (bf16-rounded)
                acc[i][j] = f4{__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                               __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
#pragma unroll
                for (int e = 0; e < 4; ++e) s1[j][e] += acc[i][j][e];
              }
            }
          if constexpr (BSTATS) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) {  // every lane takes part in the DPP row sums
                s1[j][e] = row16_sum(s1[j][e]);
                s2b[j][e] = row16_sum(s2b[j][e]);
              }
            if (lrow == 0) {
#pragma unroll
              for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const int co = wn * 32 + j * 16 + 4 * lchk + e;
                  statb[(wm * 2) * CO + co] = s1[j][e];
                  statb[(wm * 2 + 1) * CO + co] = s2b[j][e];
                }
            }
            pending = tl;
          }
          if constexpr (STATS) {
            float s2[2][4];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                s1[j][e] = row16_sum(s1[j][e]);
                const float mu = s1[j][e] * (1.f / (BM / 2));
                float q2 = 0.f;
#pragma unroll
                for (int i = 0; i < MB; ++i) {
                  const float d = acc[i][j][e] - mu;
                  q2 += d * d;
                }
                s2[j][e] = row16_sum(q2);
              }
            if (lrow == 0) {
#pragma unroll
              for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const int co = wn * 32 + j * 16 + 4 * lchk + e;
                  statb[(wm * 2) * CO + co] = s1[j][e];
                  statb[(wm * 2 + 1) * CO + co] = s2[j][e];
                }
            }
            pending = tl;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if constexpr (STATS || BSTATS) {
    if (!loader && wid == 0 && pending >= 0) merge(pending);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// (The weight gradient lives in conv3x3_wgrad.hip: a first version here, register-staged with
// 16x16x32 MFMAs and a 128-pixel tile of arbitrary rows, ran slower than MIOpen and was replaced.)

// Upper bound of the padded-halo rows of a 256-pixel tile (kernel's Q).
inline int64_t halo_rows_bound(int H, int W, int BM) {
  const int64_t rows = (BM - 1) / W + 2;                    // output rows a tile can touch
  const int64_t imgs = rows <= H ? 2 : (rows - 1) / H + 2;  // images those rows can span
  return (rows + 2 * imgs) * (W + 2);
}

template <class Cf, bool STATS = false, bool BSTATS = false>
int launch_h(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co, hipStream_t s,
             float* part = nullptr, const BnSrc& bs = BnSrc{}) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3h_kernel<Cf, STATS, BSTATS, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3h_kernel<Cf, STATS, BSTATS, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  if (Ci % Cf::BK != 0 || Co % Cf::BN != 0) return -1;
  if (halo_rows_bound(H, W, Cf::BM) > Cf::kHaloRows) return -4;
  const int64_t M = (int64_t)N * H * W;
  const int64_t grid = (M + Cf::BM - 1) / Cf::BM * (Co / Cf::BN);
  if (conv3x3_opt() & 64)
    hipLaunchKernelGGL((conv3x3h_kernel<Cf, STATS, BSTATS, true>), dim3((unsigned)grid), dim3(Cf::kThreads), Cf::kLds,
                       s, x, w, y, N, H, W, Ci, Co, part, bs);
  else
    hipLaunchKernelGGL((conv3x3h_kernel<Cf, STATS, BSTATS, false>), dim3((unsigned)grid), dim3(Cf::kThreads), Cf::kLds,
                       s, x, w, y, N, H, W, Ci, Co, part, bs);
  return 0;
}

template <class Cf>
int launch_ws(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3ws_kernel<Cf>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  if (Ci % Cf::BK != 0 || Co % Cf::BN != 0) return -1;
  if (halo_rows_bound(H, W, Cf::BM) > Cf::kHaloRows) return -4;
  const int64_t M = (int64_t)N * H * W;
  const int64_t grid = (M + Cf::BM - 1) / Cf::BM * (Co / Cf::BN);
  hipLaunchKernelGGL(conv3x3ws_kernel<Cf>, dim3((unsigned)grid), dim3(Cf::kThreads), Cf::kLds, s, x, w, y, N, H, W,
                     Ci, Co);
  return 0;
}

template <class Cf, bool STATS = false>
int launch_wst(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co, hipStream_t s,
               float* part = nullptr) {
  static bool attr = false;
  static int ncu = 0;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3wst_kernel<Cf, STATS, true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3wst_kernel<Cf, STATS, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    attr = true;
  }
  if (Ci != Cf::CI || Co != Cf::CO) return -1;
  if (halo_rows_bound(H, W, Cf::BM) > Cf::kHaloRows) return -4;
  const int64_t M = (int64_t)N * H * W;
  const int64_t ntile = (M + Cf::BM - 1) / Cf::BM;
  const int grid = (int)(ntile < ncu ? ntile : ncu);
  const int opt = conv3x3_opt();
  if (opt & 8)
    hipLaunchKernelGGL((conv3x3wst_kernel<Cf, STATS, true>), dim3(grid), dim3(Cf::kThreads), Cf::kLds, s, x, w, y, N, H,
                       W, part, opt);
  else
    hipLaunchKernelGGL((conv3x3wst_kernel<Cf, STATS, false>), dim3(grid), dim3(Cf::kThreads), Cf::kLds, s, x, w, y, N,
                       H, W, part, opt);
  return 0;
}

// The row-tile weight-stationary kernel (conv3x3wsr_kernel): opt bit 5, W = 56 (ResNet-50 layer 1 at
// 224 x 224; other widths keep conv3x3wst), whole-row tiles inside one image, at least one tile per CU.
using RCfg56 = RCfg<56>;
inline bool wsr_applies(int N, int H, int W, int Ci, int Co) {
  return (conv3x3_opt() & 32) && Ci == 64 && Co == 64 && W == RCfg56::W && H % RCfg56::R == 0 &&
         (int64_t)N * (H / RCfg56::R) >= 256;
}

template <bool STATS, bool BSTATS = false>
int launch_wsr(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, hipStream_t s, float* part = nullptr,
               const BnSrc& bs = BnSrc{}) {
  using Cf = RCfg56;
  static bool attr = false;
  static int ncu = 0;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3wsr_kernel<Cf, STATS, BSTATS>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    attr = true;
  }
  const int64_t ntile = (int64_t)N * (H / Cf::R);
  const int grid = (int)(ntile < ncu ? ntile : ncu);
  hipLaunchKernelGGL((conv3x3wsr_kernel<Cf, STATS, BSTATS>), dim3(grid), dim3(Cf::kThreads), Cf::kLds, s, x, w, y, N,
                     H, part, conv3x3_opt(), bs);
  return 0;
}

using HWide = HCfg<128, 4, 2>;   // 8 waves of 64x64
using HNarrow = HCfg<64, 4, 1>;  // 4 waves of 64x64

// Wt'[ci][t][co] = Wt[co][8 - t][ci]: the data gradient of a stride-1 pad-1 3x3 conv is a
// stride-1 pad-1 3x3 conv of dY with these weights.
__global__ void conv3x3_flip_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ wf, int Co, int Ci) {
  const int64_t n = (int64_t)Co * 9 * Ci;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i / (9 * Co));
    const int rem = (int)(i % (9 * Co));
    const int t = rem / Co, co = rem % Co;
    wf[i] = w[((int64_t)co * 9 + (8 - t)) * Ci + ci];
  }
}

template <class Cf>
int launch(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3s1_kernel<Cf>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  if (Ci % Cf::BK != 0 || Co % Cf::BN != 0) return -1;
  const int64_t M = (int64_t)N * H * W;
  const int64_t grid = (M + Cf::BM - 1) / Cf::BM * (Co / Cf::BN);
  hipLaunchKernelGGL(conv3x3s1_kernel<Cf>, dim3((unsigned)grid), dim3(Cf::kThreads), Cf::kLds, s, x, w, y, N, H, W,
                     Ci, Co);
  return 0;
}

// 128-channel tiles unless the grid would leave CUs idle (pdt::small_grid_narrow)
inline bool h_wide(int64_t M, int Co) { return Co % 128 == 0 && !small_grid_narrow((M + 255) / 256 * (Co / 128)); }

using CfWide = Cfg<256, 128, 4, 2, 32>;   // Co % 128 == 0: 8 waves of 64x64, 72 KB LDS -> 2 WG/CU
using CfNarrow = Cfg<256, 64, 4, 1, 32>;  // Co == 64: 4 waves of 64x64, 60 KB LDS

}  // namespace

extern "C" {

// y[N,H,W,Co] = conv3x3(x[N,H,W,Ci], w[Co,3,3,Ci]), stride 1, padding 1 (all NHWC / channels_last
// bf16). Ci % 64 == 0, Co % 64 == 0, N*H*W*max(Ci,Co) < 2^31. Returns 0 on success.
int pdt_conv3x3s1_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, int N, int H, int W, int Ci, int Co,
                      hipStream_t s) {
  if (Ci % 32 != 0 || Co % 64 != 0 || N < 1 || H < 1 || W < 1) return -1;
  const int64_t M = (int64_t)N * H * W;
  if (M * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31 || (int64_t)Co * 9 * Ci >= (int64_t)1 << 31) return -2;
#ifdef PDT_CONV_CFG_OVERRIDE
  return PDT_CONV_LAUNCH<PDT_CONV_CFG_OVERRIDE>(x, w, y, N, H, W, Ci, Co, s);
#endif
  int rc = -1;
  if (wsr_applies(N, H, W, Ci, Co)) return launch_wsr<false>(x, w, y, N, H, s);
  if (Ci == 64 && Co == 64) rc = launch_wst<SCfg<64, 64>>(x, w, y, N, H, W, Ci, Co, s);
  if (rc == -1) rc = h_wide(M, Co) ? launch_h<HWide>(x, w, y, N, H, W, Ci, Co, s) : launch_h<HNarrow>(x, w, y, N, H, W, Ci, Co, s);
  if (rc != -4) return rc;
  // halo larger than the LDS buffer (tiny W): per-tap staging
  if (Co % 128 == 0) return launch<CfWide>(x, w, y, N, H, W, Ci, Co, s);
  return launch<CfNarrow>(x, w, y, N, H, W, Ci, Co, s);
}

// Rows per statistics tile of pdt_conv3x3s1_fwd_stats at this shape: 224 where the row-tile kernel runs
// (part then has M / 224 tiles), else 256.
int pdt_conv3x3s1_stats_tile_rows(int N, int H, int W, int Ci, int Co) {
  return wsr_applies(N, H, W, Ci, Co) ? RCfg56::BM : 256;
}

// Same for the backward reduction of pdt_conv3x3s1_fwd_bnbwd.
int pdt_conv3x3s1_bnbwd_tile_rows(int N, int H, int W, int Ci, int Co) {
  return wsr_applies(N, H, W, Ci, Co) && (conv3x3_opt() & 128) ? RCfg56::BM : 256;
}

// Forward + per-tile BatchNorm statistics of y into part ([2][T][Co] fp32, tile_stats.h; tiles of
// pdt_conv3x3s1_stats_tile_rows rows).
// The halo and weight-stationary (64 -> 64) kernels have the statistics epilogue: returns -5 where
// another kernel would run (tiny W: per-tap staging) — caller falls back.
int pdt_conv3x3s1_fwd_stats(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int N, int H, int W,
                            int Ci, int Co, hipStream_t s) {
  if (Ci % 32 != 0 || Co % 64 != 0 || N < 1 || H < 1 || W < 1) return -1;
  const int64_t M = (int64_t)N * H * W;
  if (M * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31 || (int64_t)Co * 9 * Ci >= (int64_t)1 << 31) return -2;
  if (wsr_applies(N, H, W, Ci, Co)) return launch_wsr<true>(x, w, y, N, H, s, part);  // 224-row tiles
  if (Ci == 64 && Co == 64) {
    const int rc = launch_wst<SCfg<64, 64>, true>(x, w, y, N, H, W, Ci, Co, s, part);
    return rc == -4 ? -5 : rc;
  }
  if (halo_rows_bound(H, W, 256) > 512) return -5;
  return h_wide(M, Co) ? launch_h<HWide, true>(x, w, y, N, H, W, Ci, Co, s, part)
                       : launch_h<HNarrow, true>(x, w, y, N, H, W, Ci, Co, s, part);
}

// Data gradient y = conv3x3(dy, flipped w) whose output y is the gradient at a BatchNorm's output
// (input bn_x [N,H,W,Co] bf16, ReLU bit-mask bn_mask or null, batch mean bn_mean [Co]): also writes
// that BatchNorm's backward per-tile partials bn_part [2][T][Co] (tile_stats.h). Halo kernel only:
// returns -5 where another kernel would run (caller falls back to a plain launch + reduce pass).
int pdt_conv3x3s1_fwd_bnbwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const uint16_t* bn_x,
                            const uint8_t* bn_mask, const float* bn_mean, float* bn_part, int N, int H, int W, int Ci,
                            int Co, hipStream_t s) {
  if (Ci % 32 != 0 || Co % 64 != 0 || N < 1 || H < 1 || W < 1 || !bn_x || !bn_mean || !bn_part) return -1;
  const int64_t M = (int64_t)N * H * W;
  if (M * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31 || (int64_t)Co * 9 * Ci >= (int64_t)1 << 31) return -2;
  const BnSrc bs{bn_x, bn_mask, bn_mean, bn_part};
  // the row-tile kernel takes it (224-row tiles); the 256-pixel weight-stationary one's reduction did not pay
  if (wsr_applies(N, H, W, Ci, Co) && (conv3x3_opt() & 128)) return launch_wsr<false, true>(x, w, y, N, H, s, nullptr, bs);
  if (Ci == 64 && Co == 64) return -5;
  if (halo_rows_bound(H, W, 256) > 512) return -5;
  return h_wide(M, Co) ? launch_h<HWide, false, true>(x, w, y, N, H, W, Ci, Co, s, nullptr, bs)
                       : launch_h<HNarrow, false, true>(x, w, y, N, H, W, Ci, Co, s, nullptr, bs);
}

// Set the 3x3 variant bits (conv3x3_opt); -1 re-reads PDT_CONV3X3_OPT. Returns the previous value.
int pdt_conv3x3_opt(int v) {
  const int old = conv3x3_opt();
  g_c3opt = v;
  (void)conv3x3_opt();
  return old;
}

// wf[Ci,3,3,Co] (the data-gradient weights) from w[Co,3,3,Ci].
int pdt_conv3x3_flip_weights(const uint16_t* w, uint16_t* wf, int Co, int Ci, hipStream_t s) {
  const int64_t n = (int64_t)Co * 9 * Ci;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(conv3x3_flip_kernel, dim3(grid), dim3(256), 0, s, w, wf, Co, Ci);
  return 0;
}

}  // extern "C"
