// 1x1 convolution (an NHWC GEMM) on MFMA for gfx950, with the epilogues ResNet needs fused in:
//
//   Y[m, n] = sum_k A[m, k] * B[n, k]   (+ C[m, n])                     A, B, C, Y bf16, fp32 accumulate
//
//   forward     : A = X [M = N*H*W, Ci], B = W [Co, Ci]          -> Y = conv1x1(X)
//   data grad   : A = dY [M, Co],        B = W^T [Ci, Co]        -> dX (+ C: the other branch's
//                 gradient of X — the ResNet shortcut — accumulated in place, beta = 1)
//   STATS       : per 256-pixel tile, per output channel: the tile's sum and its CENTRED sum of
//                 squares (of the bf16 values written), so the BatchNorm that consumes Y never
//                 re-reads it for its statistics (ops/batchnorm.py, bn_fwd_train_tiles).
//
// Not in the reference (LeNet has no 1x1 convs, /root/reference/cnn.py:10-16). ResNet-50's 1x1
// convs are HBM-bound (K = 64..2048, M = 25K..1.6M at batch 512; tools/r50_roofline.py); the
// library kernels (MIOpen / hipBLASLt) cannot fuse the BatchNorm statistics, which cost a full
// extra read of every conv output (bn_reduce3, ~2 ms of a 44 ms step, profiles/r2).
//
// Structure (same machinery as the per-tap 3x3 kernel, conv3x3.hip):
//   * tile 256 pixels x BN (64 | 128) channels; 4 (M) x BN/64 (N) waves of 64 x 64, each as
//     4 x 4 blocks of v_mfma_f32_16x16x32_bf16 with the operands swapped (A = B-rows, B = pixels)
//     so a lane's accumulator holds 4 consecutive channels of one pixel;
//   * k-steps of 32 channels (64-B LDS rows); A and B staged global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, 1 KB = 16 rows per wave instruction) through a 3-slot ring, one
//     s_barrier per k-step, counted vmcnt so the DMA stays in flight across barriers; ~72 KB of
//     LDS -> 2 workgroups per CU, so one workgroup's epilogue overlaps the other's loads;
//   * rows XOR-swizzled (chunk ^ ((row >> 2) & 1) << 1) by permuting each lane's SOURCE chunk,
//     conflict-free ds_read_b128 for the 16x16x32 lane map; rows past M DMA a zero page;
//   * epilogue: the bf16 tile is staged through LDS, the statistics are taken from the staged
//     (rounded) values, and the tile leaves as whole 16-B row pieces (C added there, fp32);
//   * block -> tile map XCD-aware (xcd_remap): the N-tiles of one pixel tile share an L2.
//
//   ATR (forward only): A is a BatchNorm's INPUT whose apply was deferred to here: every A element is
//                 replaced by relu(a[k] x + b[k]) (the coefficients of that BatchNorm + ReLU, fp32, same
//                 fma and rounding as its apply pass) in registers after the fragment read, so the
//                 BatchNorm's output is never written or read (ResNet bottleneck bn2 -> conv3).
//
//   APPLY (forward only): the GEMM output z is the INPUT of a BatchNorm whose statistics are already
//                 known (the same GEMM ran once before, with STATS, ops/conv.py): the epilogue writes that
//                 BatchNorm's output relu(a z + b + r) and its ReLU bits instead of z, with r the residual
//                 (or ra r + rb, a deferred shortcut BatchNorm). A ResNet bottleneck's bn3 apply pass then
//                 reads conv3's input (C/4 channels) instead of z (C channels): 0.75 of a tensor less
//                 traffic per block; z is still stored by the first run for the backward.
//
//   BSTATS (data grad only): the output Y is the gradient dy at a BatchNorm's output, and that
//                 BatchNorm's backward reduction is taken here instead of in a separate pass over
//                 (dy, x): per 256-pixel tile, per channel, sum(dz) and sum(dz * (xb - mean)) with
//                 dz = dy * relu mask (xb, mask, mean: the BatchNorm's saved input / mask / mean;
//                 dz from the bf16 values written). The pass that would re-read dy is gone; xb is
//                 read once here instead (ops/batchnorm.py GradStatsSource, bn_bwd_train_tiles).
#include "../common.h"
#include "../tile_stats.h"

#include <stdlib.h>

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

__device__ __attribute__((aligned(256))) uint4 g_gemm_zero[16];  // zero page for rows past M (never written)
__device__ __attribute__((aligned(256))) uint4 g_gemm_ones[16] = {  // bf16 1.0 page (SEG's bias segment)
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}};
__device__ uint8_t g_mask_ones[16] = {  // (non-const: global, not constant, address space)
   0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                            0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};  // "no mask"

template <int BN_, int WM_, int WN_>
struct G1 {
  static constexpr int BM = 256, BN = BN_, WM = WM_, WN = WN_, BK = 32, kSlots = 3;
  static constexpr int kWaves = WM * WN, kThreads = kWaves * 64;
  static constexpr int kABytes = BM * 64, kBBytes = BN * 64, kSlot = kABytes + kBBytes;
  static constexpr int kEpiStride = BN * 2 + 16;
  static constexpr int kEpi = BM * kEpiStride;
  static constexpr int kRed = 0;  // (the statistics reduction reuses the released tile: rs8_tile_store)
  static constexpr int kLds = kSlots * kSlot > kEpi + kRed ? kSlots * kSlot : kEpi + kRed;
  static constexpr int kMB = BM / WM / 16, kNB = BN / WN / 16;
  static constexpr int kALd = BM / 16 / kWaves, kBLd = BN / 16 / kWaves, kG = kALd + kBLd;
  static constexpr int kOcc = (160 * 1024) / kLds;
  static constexpr int kMinWaves = kOcc * kThreads / 256 > 0 ? kOcc * kThreads / 256 : 1;
  static_assert(kALd * 16 * kWaves == BM && kBLd * 16 * kWaves == BN, "DMA split");
};

__device__ __forceinline__ int chk64(int row, int p) { return p ^ (((row >> 2) & 1) << 1); }  // involution
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + (chk64(row, chunk) << 4); }

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (PDT_LDS void*)lds_wave_base, 16, 0, 0);
}

template <int G>
__device__ __forceinline__ void wait_vm() {
  static_assert(G >= 0 && G <= 6, "vmcnt");
  if constexpr (G == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (G == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (G == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (G == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (G == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// part (STATS): [T][N] tile sums, then [T][N] centred tile sums of squares (T = ceil(M / 256)).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Strided accumulate source (ACC): Cin is the COMPACT gradient of a stride-s subsampling of Y's
// pixels (a ResNet stride-2 shortcut's data gradient, [N*Hs*Ws, N] with Hs = (H-1)/s+1): Y row
// m = (n, h, w) adds Cin row (n, h/s, w/s) when s divides h and w, nothing otherwise. s = 0: Cin
// has Y's rows (plain accumulate).
struct CGeom {
  int s, H, W, Hs, Ws;
};

// APPLY: the BatchNorm applied in the epilogue. ab = [2][N] (a, then b); rab = [2][N] (ra, rb) or null
// (plain residual); the residual itself comes in Cin; mask [M * N / 8] receives the ReLU bits.
struct ApArgs {
  const float* ab;
  const float* rab;
  uint8_t* mask;
  int probe;  // diagnosis only (pdt_conv1x1_probe): 1 = no output stores, 2 = no MFMA, 4 = no operand DMA,
             // 8 = 64-channel tiles (4 waves) for every N, 64 = no 256-channel tiles
  // SEG (a2 != null; one-tile kernel only): A is the K-concatenation [A (k1 columns) | a2 (k2) repeated rep2
  // times | 32 columns of 1.0] — B holds the matching [N, k1 + rep2 k2 + 32] rows. The ones segment adds a
  // per-column bias (B's columns there); a repeated a2 segment meets a hi / lo split of its B block.
  const uint16_t* a2;
  int k1, k2, rep2;
  // nostore (STATS forward): the statistics only, Y is not written (ops/conv.py: a bottleneck conv3 whose output
  // is consumed only by its BatchNorm's statistics and its recomputed APPLY GEMM, and never by the backward)
  int nostore;
};

int g_probe = 0;

// NT: streaming (non-temporal) output stores. ATR: acoef = [2][K] fp32 (a, then b), see the header.
template <class Cf, bool ACC, bool STATS, bool NT, bool BSTATS, bool ATR = false, bool APPLY = false, bool STR = false>
__global__ __launch_bounds__(Cf::kThreads, Cf::kMinWaves) void conv1x1_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* Y, const uint16_t* Cin,
    const uint8_t* __restrict__ Cmask, float* __restrict__ part, int M, int K, int N, BnSrc bs, CGeom cg,
    const float* __restrict__ acoef, ApArgs ap) {
  static_assert(!(APPLY && (ACC || STATS || BSTATS)), "APPLY is a forward epilogue of its own");
  static_assert(!STR || ACC, "STR: a strided accumulate source");
  constexpr int BM = Cf::BM, BN = Cf::BN;
  constexpr int WROWS = BM / Cf::WM, WCOLS = BN / Cf::WN;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % Cf::WM, wn = wid / Cf::WM;
  const int ntiles = N / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / ntiles;
  const int m0 = mt * BM, n0 = (tile % ntiles) * BN;

  const int sub = lane >> 2, p = lane & 3;
  // SEG: A rows are k1 long (the first segment); a2 rows k2 long (workgroup-uniform)
  const bool seg = ap.a2 != nullptr;
  const int lda = seg ? ap.k1 : K;
  int aoff[Cf::kALd];  // element offset of this lane's A piece, -1 = zero page
  int a2off[Cf::kALd];
#pragma unroll
  for (int i = 0; i < Cf::kALd; ++i) {
    const int r = (wid * Cf::kALd + i) * 16 + sub;
    aoff[i] = m0 + r < M ? (m0 + r) * lda + chk64(r, p) * 8 : -1;
    a2off[i] = (m0 + r) * ap.k2 + chk64(r, p) * 8;
  }
  int boff[Cf::kBLd];
#pragma unroll
  for (int j = 0; j < Cf::kBLd; ++j) {
    const int r = (wid * Cf::kBLd + j) * 16 + sub;
    boff[j] = (n0 + r) * K + chk64(r, p) * 8;
  }
  const int S = K / Cf::BK;

  auto issue = [&](int s) {
    char* slot = lds + (s % Cf::kSlots) * Cf::kSlot;
    const int ko = s * Cf::BK;
    // SEG: which segment this k-step reads (uniform), and the column inside it
    const int ks2 = ko - ap.k1, seg2 = seg && ks2 >= 0 && ks2 < ap.rep2 * ap.k2 ? 1 : (seg && ks2 >= 0 ? 2 : 0);
    const int ko2 = seg2 == 1 ? ks2 % ap.k2 : 0;
#pragma unroll
    for (int i = 0; i < Cf::kALd; ++i) {
      const uint16_t* src = aoff[i] < 0 ? reinterpret_cast<const uint16_t*>(g_gemm_zero)
                            : seg2 == 0 ? A + (aoff[i] + ko)
                            : seg2 == 1 ? ap.a2 + (a2off[i] + ko2)
                                        : reinterpret_cast<const uint16_t*>(g_gemm_ones);
      dma16(src, slot + (wid * Cf::kALd + i) * 1024);
    }
#pragma unroll
    for (int j = 0; j < Cf::kBLd; ++j) dma16(B + (boff[j] + ko), slot + Cf::kABytes + (wid * Cf::kBLd + j) * 1024);
  };
  const int probe = ap.probe;

  f4 acc[Cf::kMB][Cf::kNB];
#pragma unroll
  for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // ATR: the [2][K] coefficient table in LDS past the ring / epilogue area (filled before any DMA)
  float* const ctab = reinterpret_cast<float*>(lds + Cf::kLds);
  if constexpr (ATR) {
    for (int i = tid; i < 2 * K; i += Cf::kThreads) ctab[i] = acoef[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  if (!(probe & 4)) {
    issue(0);
    if (S > 1) issue(1);
  }
  const int lrow = lane & 15, lchk = lane >> 4;
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) wait_vm<Cf::kG>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 2 < S && !(probe & 4)) issue(s + 2);  // slot (s+2)%3 was last read at step s-1: every wave is past it
    const char* As = lds + (s % Cf::kSlots) * Cf::kSlot;
    const char* Bs = As + Cf::kABytes;
    bf16x8 a[Cf::kMB], b[Cf::kNB];
#pragma unroll
    for (int i = 0; i < Cf::kMB; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + swz64(wm * WROWS + i * 16 + lrow, lchk));
#pragma unroll
    for (int j = 0; j < Cf::kNB; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + swz64(wn * WCOLS + j * 16 + lrow, lchk));
    if constexpr (ATR) {  // relu(a x + b) of the fragment's 8 channels, s * 32 + 8 lchk + 0..7
      const int k0 = s * Cf::BK + 8 * lchk;
      float ca[8], cb[8];
      *reinterpret_cast<float4*>(ca) = *reinterpret_cast<const float4*>(ctab + k0);
      *reinterpret_cast<float4*>(ca + 4) = *reinterpret_cast<const float4*>(ctab + k0 + 4);
      *reinterpret_cast<float4*>(cb) = *reinterpret_cast<const float4*>(ctab + K + k0);
      *reinterpret_cast<float4*>(cb + 4) = *reinterpret_cast<const float4*>(ctab + K + k0 + 4);
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 w = __builtin_bit_cast(u4, a[i]);
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[2 * k] = __uint_as_float(w[k] << 16); v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u); }
        u4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float t0 = v[2 * k] * ca[2 * k] + cb[2 * k], t1 = v[2 * k + 1] * ca[2 * k + 1] + cb[2 * k + 1];
          o[k] = (uint32_t)f2bf(t0 > 0.f ? t0 : 0.f) | ((uint32_t)f2bf(t1 > 0.f ? t1 : 0.f) << 16);
        }
        a[i] = __builtin_bit_cast(bf16x8, o);
      }
    }
    if (!(probe & 2)) {
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
        for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // D[n][m]
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // ---- epilogue: bf16 tile [BM pixels][BN] staged in LDS
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
  __syncthreads();

  // STATS: the tile's BatchNorm partials from the rows each thread stores (RowStats8), merged after the loop
  RowStats8 rst;
  float kst = 0.f;  // the tile's first-row value of channel tid (tid < BN), for rs8_tile_store
  if constexpr (STATS) {
    rs8_init(rst, *reinterpret_cast<const uint4*>(lds + (tid % (BN / 8)) * 16));
    if (tid < BN) kst = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(lds + tid * 2) << 16);
  }

  constexpr int kChunks = BN / 8;
  static_assert(Cf::kThreads % kChunks == 0, "a thread keeps one 8-channel chunk");
  float bs1[8], bs2[8], bmu[8];
  float pa[8], pb[8], pra[8], prb[8];  // APPLY: this thread's 8 channels' coefficients
  if constexpr (APPLY) {
    const int c = tid % kChunks;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pa[k] = ap.ab[n0 + c * 8 + k];
      pb[k] = ap.ab[N + n0 + c * 8 + k];
      pra[k] = ap.rab ? ap.rab[n0 + c * 8 + k] : 1.f;
      prb[k] = ap.rab ? ap.rab[N + n0 + c * 8 + k] : 0.f;
    }
  }
  if constexpr (BSTATS) {
    const int c = tid % kChunks;
    *reinterpret_cast<float4*>(bmu) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8);
    *reinterpret_cast<float4*>(bmu + 4) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8 + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) { bs1[k] = 0.f; bs2[k] = 0.f; }
  }
  // A thread keeps one 8-channel chunk c and rows r0 + kRowStep * it. Every global load of the
  // epilogue (the accumulate source, its ReLU mask, the BSTATS input and mask) is issued for all
  // kIt rows before the first use: one memory latency per tile instead of one per row (issued per
  // row, the dgrad+accumulate kernels ran at ~2.7 TB/s, latency bound in this epilogue). The loads
  // of a row precede its store, and no other thread touches it, so c may alias y.
  // (Both sources at 128 VGPRs — the 8-wave tile with ACC and BSTATS — go in two batches of rows:
  // all eight rows at once spilled there.)
  constexpr int kRowStep = Cf::kThreads / kChunks, kIt = BM / kRowStep;
  constexpr int kB = (ACC && BSTATS && Cf::kWaves >= 8) ? kIt / 2 : kIt;
  static_assert(kRowStep * kIt == BM && kIt % kB == 0, "epilogue rows");
  const int r0 = tid / kChunks, c = tid % kChunks;
  // The loads are BRANCH-FREE: a row past M reads the tile's last valid row (its results are dropped),
  // a null mask reads a 0xff byte, and the strided source is a separate instantiation (STR). Written
  // with per-row conditions, hipcc branched around every load and put an s_waitcnt vmcnt(1) / (0)
  // into each row's branch (cdna_hip_programming.md §5, trap (c)): the rows' loads were serialised
  // after all, one memory latency each.
  const uint8_t* const cm_base = Cmask ? Cmask : g_mask_ones;
  const int64_t cm_scale = Cmask ? 1 : 0;
  const uint8_t* const bm_base = bs.mask ? bs.mask : g_mask_ones;
  const int64_t bm_scale = bs.mask ? 1 : 0;
  // BSTATS sum-only (bs.x null): the BatchNorm input is not read (a zero page, stride 0) — only sum(dz) is
  // meaningful then; the ALG backward derives sum(dz (x - mean)) from its weight-gradient pass (bn_alg.hip)
  const uint16_t* const bx_base = bs.x ? bs.x : reinterpret_cast<const uint16_t*>(g_gemm_zero);
  const int64_t bx_scale = bs.x ? 1 : 0;
#pragma unroll 1
  for (int h = 0; h < kIt; h += kB) {
  uint4 cv[kB], xbv[kB];
  unsigned cmk[kB], bmkv[kB];
  bool okv[kB];
#pragma unroll
  for (int it = 0; it < kB; ++it) {
    const int m = m0 + r0 + kRowStep * (h + it);
    const bool ok = m < M;
    okv[it] = ok;
    const int mc = ok ? m : M - 1;
    const int64_t off = (int64_t)mc * N + n0 + c * 8;
    if constexpr (BSTATS) {
      xbv[it] = *reinterpret_cast<const uint4*>(bx_base + off * bx_scale);
      const unsigned b = bm_base[(off >> 3) * bm_scale];
      bmkv[it] = ok ? b : 0u;  // a dropped row adds nothing to the reduction
    }
    if constexpr (APPLY) cv[it] = *reinterpret_cast<const uint4*>(Cin + off);  // the residual
    if constexpr (ACC) {
      const unsigned mk = cm_base[(off >> 3) * cm_scale];  // C = Cin * mask: a ReLU's masked gradient
      if constexpr (STR) {  // compact strided source: rows off the sampling grid add nothing
        const int w = mc % cg.W, t = mc / cg.W, hh = t % cg.H, n = t / cg.H;
        const bool on = hh % cg.s == 0 && w % cg.s == 0;
        const int64_t co = on ? ((int64_t)(n * cg.Hs + hh / cg.s) * cg.Ws + w / cg.s) * N : 0;
        cv[it] = *reinterpret_cast<const uint4*>(Cin + co + n0 + c * 8);
        cmk[it] = on ? mk : 0u;
      } else {
        cv[it] = *reinterpret_cast<const uint4*>(Cin + off);
        cmk[it] = mk;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < kB; ++it) {
    const int r = r0 + kRowStep * (h + it);
    const int m = m0 + r;
    const bool ok = okv[it];
    uint4 v = *reinterpret_cast<const uint4*>(lds + (ok ? r : 0) * Cf::kEpiStride + c * 16);
    const int64_t off = (int64_t)(ok ? m : 0) * N + n0 + c * 8;
    if constexpr (ACC) {
      float a[8], cc[8];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w}, cw[4] = {cv[it].x, cv[it].y, cv[it].z, cv[it].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[2 * k] = __uint_as_float(w[k] << 16); a[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        cc[2 * k] = __uint_as_float(cw[k] << 16); cc[2 * k + 1] = __uint_as_float(cw[k] & 0xffff0000u);
      }
      const unsigned mb = cmk[it];
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += (mb >> k) & 1u ? cc[k] : 0.f;
      v.x = (uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16);
      v.y = (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16);
      v.z = (uint32_t)f2bf(a[4]) | ((uint32_t)f2bf(a[5]) << 16);
      v.w = (uint32_t)f2bf(a[6]) | ((uint32_t)f2bf(a[7]) << 16);
    }
    unsigned amb = 0;
    if constexpr (APPLY) {  // relu(a z + b + r): the same fp32 operations as batchnorm.hip bn_apply_kernel
      float z[8], r[8];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w}, rw[4] = {cv[it].x, cv[it].y, cv[it].z, cv[it].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        z[2 * k] = __uint_as_float(w[k] << 16); z[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        r[2 * k] = __uint_as_float(rw[k] << 16); r[2 * k + 1] = __uint_as_float(rw[k] & 0xffff0000u);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float t = z[k] * pa[k] + pb[k];
        t += ap.rab ? r[k] * pra[k] + prb[k] : r[k];
        amb |= (t > 0.f ? 1u : 0u) << k;
        z[k] = t > 0.f ? t : 0.f;
      }
      v.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
      v.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
      v.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
      v.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
    }
    if constexpr (BSTATS) {
      bn_bwd_accum8(v, xbv[it], bmkv[it], bmu, bs1, bs2);
      v = mask8(v, bmkv[it]);  // stored masked (tile_stats.h mask8)
    }
    if (!ok) continue;
    if constexpr (STATS) rs8_add(rst, v);
    if constexpr (APPLY) {
      if (!(probe & 32)) ap.mask[off >> 3] = (uint8_t)amb;
    }
    if ((probe & 1) || ap.nostore) continue;
    if constexpr (NT) {
      const u32x4 t = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(Y + off));
    } else {
      *reinterpret_cast<uint4*>(Y + off) = v;
    }
  }
  }

  if constexpr (BSTATS)  // every wave is done reading the staged tile: its LDS holds the block sums
    bn_bwd_tile_store<BN, Cf::kWaves>(bs1, bs2, reinterpret_cast<float*>(lds), bs.part, (M + BM - 1) / BM, mt, N, n0);
  if constexpr (STATS) {
    __syncthreads();  // every wave is done reading the staged tile: its LDS takes the reduction
    rs8_tile_store<BN, Cf::kWaves>(rst, kst, reinterpret_cast<float*>(lds), part, min(BM, M - m0), (M + BM - 1) / BM,
                                   mt, N, n0);
  }
}

// ---------------------------------------------------------------------------------------------------
// PERSISTENT variant (PDT_CONV1X1_PERSIST; by default for the kinds where it measured faster, see g_persist): one
// workgroup per CU (two for the 64-channel tile) walks its share of the tiles, and tile t+1's first
// two operand k-steps are DMA'd into the ring WHILE tile t's epilogue runs (its staging area is placed
// past those two slots), so its output stores drain under tile t+1's main loop. Measured reason
// (profiles/r4/conv1x1_probe_b1024.txt): with nothing computed, loaded or stored the one-tile-per-
// workgroup kernel still took ~245 us for 12,544 tiles of 1024 threads (~5 us per tile per CU of launch,
// prologue and epilogue serialisation), and with one 135-KB workgroup per CU every tile ran its DMA
// wait, MFMA and epilogue back to back.
//
// vmcnt accounting (hand-counted waits; the DMAs are inline asm, invisible to hipcc, so its own waits
// for the epilogue's register loads can only over-wait): in issue order a tile's ops are D0, D1 (issued
// by the previous tile's epilogue, or the prologue), that previous epilogue's kStores row stores, then
// D2 (at step 0), D3 (step 1), ... Waiting for D_s leaves younger: D_{s+1} when it exists, plus the
// previous epilogue's row stores while s < 2. Every row store is issued by every thread (rows past M
// go to a sink) so the count is exact; the statistics stores come last and only make a wait stricter.
template <class Cf>
struct PL {
  static constexpr int kStgOff = 2 * Cf::kSlot;              // slots 0 / 1 take tile t+1's D0 / D1
  static constexpr int kFull = Cf::BM * Cf::kEpiStride;
  static constexpr int kHalves = kStgOff + kFull <= 152 * 1024 ? 1 : 2;
  static constexpr int kStg = kFull / kHalves;
  static constexpr int kRed0 = Cf::kWaves * (Cf::BN / 8) * 16 * 4, kRed1 = Cf::kWaves * 2 * Cf::BN * 4;
  static constexpr int kRed = kRed0 > kRed1 ? kRed0 : kRed1;
  static constexpr int kArea = kStg > kRed ? kStg : kRed;
  static constexpr int kLds = 3 * Cf::kSlot > kStgOff + kArea ? 3 * Cf::kSlot : kStgOff + kArea;
  static constexpr int kOcc = (160 * 1024) / kLds;
  static constexpr int kMinWaves = kOcc * Cf::kThreads / 256 > 0 ? kOcc * Cf::kThreads / 256 : 1;
  static_assert(kLds <= 160 * 1024 && kFull % kHalves == 0, "LDS");
};

__device__ __attribute__((aligned(256))) uint4 g_gemm_sink[1024];  // row stores past M (exact vmcnt)
__device__ uint8_t g_mask_sink[1024];

__device__ __forceinline__ void dma16a(const void* src, char* lds_wave_base) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(PDT_LDS const char*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmn() {  // s_waitcnt vmcnt(N), expcnt / lgkmcnt unconstrained
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <class Cf, bool ACC, bool STATS, bool BSTATS, bool ATR, bool APPLY, bool STR>
__global__ __launch_bounds__(Cf::kThreads, PL<Cf>::kMinWaves) void conv1x1p_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* Y, const uint16_t* Cin,
    const uint8_t* __restrict__ Cmask, float* __restrict__ part, int M, int K, int N, BnSrc bs, CGeom cg,
    const float* __restrict__ acoef, ApArgs ap) {
  static_assert(!(APPLY && (ACC || STATS || BSTATS)), "APPLY is a forward epilogue of its own");
  static_assert(!STR || ACC, "STR: a strided accumulate source");
  using L = PL<Cf>;
  constexpr int BM = Cf::BM, BN = Cf::BN, kG = Cf::kG, kHalves = L::kHalves;
  constexpr int WROWS = BM / Cf::WM, WCOLS = BN / Cf::WN;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % Cf::WM, wn = wid / Cf::WM;
  const int ntn = N / BN, T = (M + BM - 1) / BM, total = T * ntn;
  // tiles: 8 contiguous chunks, one per XCD (blocks b, b + 8, ... under round-robin placement — speed
  // only): the N-tiles of a pixel tile run side by side on one L2
  const int G = gridDim.x, xg = blockIdx.x % 8, jg = blockIdx.x / 8, gx = (G - xg + 7) / 8;
  const int c_lo = (int)((int64_t)total * xg / 8), c_hi = (int)((int64_t)total * (xg + 1) / 8);
  int tile = c_lo + jg;
  if (tile >= c_hi) return;  // (uniform: before any barrier)
  const int S = K / Cf::BK;
  char* const stg = lds + L::kStgOff;

  const int sub = lane >> 2, p = lane & 3;
  auto aoff_of = [&](int m0, int i) {
    const int r = (wid * Cf::kALd + i) * 16 + sub;
    return m0 + r < M ? (m0 + r) * K + chk64(r, p) * 8 : -1;
  };
  auto boff_of = [&](int n0, int j) {
    const int r = (wid * Cf::kBLd + j) * 16 + sub;
    return (n0 + r) * K + chk64(r, p) * 8;
  };
  int aoff[Cf::kALd], boff[Cf::kBLd];
  auto issue = [&](int s, int slot_i) {
    char* slot = lds + slot_i * Cf::kSlot;
    const int ko = s * Cf::BK;
#pragma unroll
    for (int i = 0; i < Cf::kALd; ++i)
      dma16a(aoff[i] >= 0 ? (const void*)(A + (aoff[i] + ko)) : (const void*)g_gemm_zero, slot + (wid * Cf::kALd + i) * 1024);
#pragma unroll
    for (int j = 0; j < Cf::kBLd; ++j) dma16a(B + (boff[j] + ko), slot + Cf::kABytes + (wid * Cf::kBLd + j) * 1024);
  };

  float* const ctab = reinterpret_cast<float*>(lds + L::kLds);
  if constexpr (ATR) {
    for (int i = tid; i < 2 * K; i += Cf::kThreads) ctab[i] = acoef[i];
    __syncthreads();  // (no DMA issued yet: a plain barrier)
  }
  // kernel-lifetime epilogue constants
  constexpr int kChunks = BN / 8;
  constexpr int kRowStep = Cf::kThreads / kChunks, kIt = BM / kRowStep;
  constexpr int kItH = kIt / kHalves;
  // rows per batch of loads (registers: 128 per lane at 16 waves, 256 below)
  constexpr int kB = (ACC && BSTATS) ? (Cf::kWaves >= 16 ? 2 : (kItH >= 8 ? kItH / 2 : kItH)) : kItH;
  constexpr int kStores = kIt * (APPLY ? 2 : 1);  // row stores per thread per tile (exact)
  static_assert(kRowStep * kIt == BM && kIt % kHalves == 0 && kItH % kB == 0, "epilogue rows");
  const int r0 = tid / kChunks, c = tid % kChunks;
  const uint8_t* const cm_base = Cmask ? Cmask : g_mask_ones;
  const int64_t cm_scale = Cmask ? 1 : 0;
  const uint8_t* const bm_base = bs.mask ? bs.mask : g_mask_ones;
  const int64_t bm_scale = bs.mask ? 1 : 0;
  // BSTATS sum-only (bs.x null): the BatchNorm input is not read (a zero page, stride 0) — only sum(dz) is
  // meaningful then; the ALG backward derives sum(dz (x - mean)) from its weight-gradient pass (bn_alg.hip)
  const uint16_t* const bx_base = bs.x ? bs.x : reinterpret_cast<const uint16_t*>(g_gemm_zero);
  const int64_t bx_scale = bs.x ? 1 : 0;

  int mt = tile / ntn, n0 = (tile % ntn) * BN, m0 = mt * BM;
#pragma unroll
  for (int i = 0; i < Cf::kALd; ++i) aoff[i] = aoff_of(m0, i);
#pragma unroll
  for (int j = 0; j < Cf::kBLd; ++j) boff[j] = boff_of(n0, j);
  issue(0, 0);
  if (S > 1) issue(1, 1);
  bool first = true;
  const int lrow = lane & 15, lchk = lane >> 4;
  for (;;) {
    f4 acc[Cf::kMB][Cf::kNB];
#pragma unroll
    for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
      for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const bool nxt = s + 1 < S;
      if (s >= 2 || first) {
        if (nxt) wait_vmn<kG>(); else wait_vmn<0>();
      } else {  // s < 2 after an epilogue: its row stores are younger than D_s
        if (nxt) wait_vmn<kG + kStores>(); else wait_vmn<kStores>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + 2 < S) issue(s + 2, (s + 2) % 3);  // slot (s+2)%3 was last read at step s-1
      const char* As = lds + (s % 3) * Cf::kSlot;
      const char* Bs = As + Cf::kABytes;
      bf16x8 a[Cf::kMB], b[Cf::kNB];
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + swz64(wm * WROWS + i * 16 + lrow, lchk));
#pragma unroll
      for (int j = 0; j < Cf::kNB; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + swz64(wn * WCOLS + j * 16 + lrow, lchk));
      if constexpr (ATR) {
        const int k0 = s * Cf::BK + 8 * lchk;
        float ca[8], cb[8];
        *reinterpret_cast<float4*>(ca) = *reinterpret_cast<const float4*>(ctab + k0);
        *reinterpret_cast<float4*>(ca + 4) = *reinterpret_cast<const float4*>(ctab + k0 + 4);
        *reinterpret_cast<float4*>(cb) = *reinterpret_cast<const float4*>(ctab + K + k0);
        *reinterpret_cast<float4*>(cb + 4) = *reinterpret_cast<const float4*>(ctab + K + k0 + 4);
#pragma unroll
        for (int i = 0; i < Cf::kMB; ++i) {
          typedef unsigned u4 __attribute__((ext_vector_type(4)));
          const u4 w = __builtin_bit_cast(u4, a[i]);
          u4 o;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float t0 = __uint_as_float(w[k] << 16) * ca[2 * k] + cb[2 * k];
            const float t1 = __uint_as_float(w[k] & 0xffff0000u) * ca[2 * k + 1] + cb[2 * k + 1];
            o[k] = (uint32_t)f2bf(t0 > 0.f ? t0 : 0.f) | ((uint32_t)f2bf(t1 > 0.f ? t1 : 0.f) << 16);
          }
          a[i] = __builtin_bit_cast(bf16x8, o);
        }
      }
#pragma unroll
      for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
        for (int j = 0; j < Cf::kNB; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // D[n][m]
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    // the accumulators as the bf16 values the tile stores (half the registers to carry into the
    // epilogue: a wave of the second half keeps them through the first half's rows)
    uint2 pk[Cf::kMB][Cf::kNB];
#pragma unroll
    for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
      for (int j = 0; j < Cf::kNB; ++j) {
        const f4 v = acc[i][j];
        pk[i][j].x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        pk[i][j].y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      }
    // ---- epilogue of this tile; the next tile's D0 / D1 go out first (slots 0 / 1: every wave is past
    // its last fragment read after this barrier)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int cur_m0 = m0, cur_n0 = n0, cur_mt = mt;
    const int next = tile + gx;
    const bool has_next = next < c_hi;
    if (has_next) {
      mt = next / ntn; n0 = (next % ntn) * BN; m0 = mt * BM;
#pragma unroll
      for (int i = 0; i < Cf::kALd; ++i) aoff[i] = aoff_of(m0, i);
#pragma unroll
      for (int j = 0; j < Cf::kBLd; ++j) boff[j] = boff_of(n0, j);
      issue(0, 0);
      if (S > 1) issue(1, 1);
    }

    RowStats8 rst;
    float kst = 0.f;
    float bs1[8], bs2[8], bmu[8];
    float pa[8], pb[8], pra[8], prb[8];
    if constexpr (APPLY) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        pa[k] = ap.ab[cur_n0 + c * 8 + k];
        pb[k] = ap.ab[N + cur_n0 + c * 8 + k];
        pra[k] = ap.rab ? ap.rab[cur_n0 + c * 8 + k] : 1.f;
        prb[k] = ap.rab ? ap.rab[N + cur_n0 + c * 8 + k] : 0.f;
      }
    }
    if constexpr (BSTATS) {
      *reinterpret_cast<float4*>(bmu) = *reinterpret_cast<const float4*>(bs.mean + cur_n0 + c * 8);
      *reinterpret_cast<float4*>(bmu + 4) = *reinterpret_cast<const float4*>(bs.mean + cur_n0 + c * 8 + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) { bs1[k] = 0.f; bs2[k] = 0.f; }
    }
#pragma unroll
    for (int hv = 0; hv < kHalves; ++hv) {
      // this half's waves stage their accumulators (bf16) as rows [hv BM/H, (hv+1) BM/H) of the tile
      constexpr int kWH = Cf::WM / kHalves;  // wave rows per half
      if (wm / kWH == hv) {
#pragma unroll
        for (int i = 0; i < Cf::kMB; ++i)
#pragma unroll
          for (int j = 0; j < Cf::kNB; ++j) {
            const int ml = (wm % kWH) * WROWS + i * 16 + lrow;
            const int cl = wn * WCOLS + j * 16 + 4 * lchk;
            *reinterpret_cast<uint2*>(stg + ml * Cf::kEpiStride + cl * 2) = pk[i][j];
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (STATS) {
        if (hv == 0) {
          rs8_init(rst, *reinterpret_cast<const uint4*>(stg + (tid % kChunks) * 16));
          if (tid < BN) kst = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(stg + tid * 2) << 16);
        }
      }
#pragma unroll
      for (int h = hv * kItH; h < (hv + 1) * kItH; h += kB) {
        uint4 cv[kB], xbv[kB];
        unsigned cmk[kB], bmkv[kB];
        bool okv[kB];
#pragma unroll
        for (int it = 0; it < kB; ++it) {
          const int m = cur_m0 + r0 + kRowStep * (h + it);
          const bool ok = m < M;
          okv[it] = ok;
          const int mc = ok ? m : M - 1;
          const int64_t off = (int64_t)mc * N + cur_n0 + c * 8;
          if constexpr (BSTATS) {
            xbv[it] = *reinterpret_cast<const uint4*>(bx_base + off * bx_scale);
            const unsigned b8 = bm_base[(off >> 3) * bm_scale];
            bmkv[it] = ok ? b8 : 0u;
          }
          if constexpr (APPLY) cv[it] = *reinterpret_cast<const uint4*>(Cin + off);
          if constexpr (ACC) {
            const unsigned mk = cm_base[(off >> 3) * cm_scale];
            if constexpr (STR) {
              const int w = mc % cg.W, t = mc / cg.W, hh = t % cg.H, n = t / cg.H;
              const bool on = hh % cg.s == 0 && w % cg.s == 0;
              const int64_t co = on ? ((int64_t)(n * cg.Hs + hh / cg.s) * cg.Ws + w / cg.s) * N : 0;
              cv[it] = *reinterpret_cast<const uint4*>(Cin + co + cur_n0 + c * 8);
              cmk[it] = on ? mk : 0u;
            } else {
              cv[it] = *reinterpret_cast<const uint4*>(Cin + off);
              cmk[it] = mk;
            }
          }
        }
#pragma unroll
        for (int it = 0; it < kB; ++it) {
          const int r = r0 + kRowStep * (h + it);
          const bool ok = okv[it];
          uint4 v = *reinterpret_cast<const uint4*>(stg + (r - hv * (BM / kHalves)) * Cf::kEpiStride + c * 16);
          const int64_t off = (int64_t)(cur_m0 + r) * N + cur_n0 + c * 8;
          if constexpr (ACC) {
            float a8[8], cc[8];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w}, cw[4] = {cv[it].x, cv[it].y, cv[it].z, cv[it].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              a8[2 * k] = __uint_as_float(w[k] << 16); a8[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
              cc[2 * k] = __uint_as_float(cw[k] << 16); cc[2 * k + 1] = __uint_as_float(cw[k] & 0xffff0000u);
            }
            const unsigned mb = cmk[it];
#pragma unroll
            for (int k = 0; k < 8; ++k) a8[k] += (mb >> k) & 1u ? cc[k] : 0.f;
            v.x = (uint32_t)f2bf(a8[0]) | ((uint32_t)f2bf(a8[1]) << 16);
            v.y = (uint32_t)f2bf(a8[2]) | ((uint32_t)f2bf(a8[3]) << 16);
            v.z = (uint32_t)f2bf(a8[4]) | ((uint32_t)f2bf(a8[5]) << 16);
            v.w = (uint32_t)f2bf(a8[6]) | ((uint32_t)f2bf(a8[7]) << 16);
          }
          unsigned amb = 0;
          if constexpr (APPLY) {
            float z[8], rr[8];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w}, rw[4] = {cv[it].x, cv[it].y, cv[it].z, cv[it].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              z[2 * k] = __uint_as_float(w[k] << 16); z[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
              rr[2 * k] = __uint_as_float(rw[k] << 16); rr[2 * k + 1] = __uint_as_float(rw[k] & 0xffff0000u);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              float t = z[k] * pa[k] + pb[k];
              t += ap.rab ? rr[k] * pra[k] + prb[k] : rr[k];
              amb |= (t > 0.f ? 1u : 0u) << k;
              z[k] = t > 0.f ? t : 0.f;
            }
            v.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
            v.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
            v.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
            v.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
          }
          if constexpr (BSTATS) {
            bn_bwd_accum8(v, xbv[it], bmkv[it], bmu, bs1, bs2);
            v = mask8(v, bmkv[it]);  // stored masked (tile_stats.h mask8)
          }
          if constexpr (STATS) {
            if (ok) rs8_add(rst, v);
          }
          // every thread stores every row (past M: the sink) so the vmcnt counts above are exact
          uint4* yp = ok && !ap.nostore ? reinterpret_cast<uint4*>(Y + off) : g_gemm_sink + tid;
          *yp = v;
          if constexpr (APPLY) {
            uint8_t* mp = ok ? ap.mask + (off >> 3) : g_mask_sink + tid;
            *mp = (uint8_t)amb;
          }
        }
      }
      __builtin_amdgcn_s_barrier();  // every wave is done reading this half's staged rows
      asm volatile("" ::: "memory");
    }
    if constexpr (BSTATS)
      bn_bwd_tile_store<BN, Cf::kWaves>(bs1, bs2, reinterpret_cast<float*>(stg), bs.part, T, cur_mt, N, cur_n0);
    if constexpr (STATS)
      rs8_tile_store<BN, Cf::kWaves>(rst, kst, reinterpret_cast<float*>(stg), part, min(BM, M - cur_m0), T, cur_mt, N,
                                     cur_n0);
    if constexpr (BSTATS || STATS) {  // the reduction area is the next epilogue's staging area
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (!has_next) break;
    tile = next;
    first = false;
  }
  wait_vmn<0>();
}

// 0: one tile per workgroup everywhere; 1 (default): persistent where it measured faster — the 16-wave
// 256-channel tile of the plain / statistics forward and of the data gradient without an accumulate source
// (ResNet-50, 1024 images, tools/conv1x1_persist_bench.py, profiles/r5/conv1x1_persist_bench_b1024.txt:
// forward + statistics 64->256 @56 526 -> 430 us, data gradient + BN reduction 64->256 @56 774 -> 725,
// @28 458 -> 401, @14 290 -> 267); the ATR, APPLY and accumulate epilogues hold more registers and spill
// at 128 per lane, and the 8- / 4-wave persistent tiles were slower: there the one-tile kernel stays;
// 2: every kind and tile persistent (A/B). -1: PDT_CONV1X1_PERSIST, read once.
int g_persist = -1;

inline int persist_mode() {
  if (g_persist < 0) {
    const char* e = getenv("PDT_CONV1X1_PERSIST");
    g_persist = (e && e[0]) ? (int)strtol(e, nullptr, 10) : 1;
    if (g_persist < 0 || g_persist > 2) g_persist = 1;
  }
  return g_persist;
}

template <class Cf, bool ACC, bool STATS, bool BSTATS, bool ATR, bool APPLY, bool STR>
int launch_p(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm, float* part, int M,
             int K, int N, const BnSrc& bs, const CGeom& cg, hipStream_t s, const float* acoef, const ApArgs& ap) {
  using L = PL<Cf>;
  static bool attr = false;
  constexpr int kMaxLds = L::kLds + (ATR ? 2 * 512 * 4 : 0);
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1p_kernel<Cf, ACC, STATS, BSTATS, ATR, APPLY, STR>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds) != hipSuccess)
      return -3;
    attr = true;
  }
  const int lds = L::kLds + (ATR ? 2 * K * 4 : 0);
  const int64_t total = (int64_t)(M + Cf::BM - 1) / Cf::BM * (N / Cf::BN);
  const int occ = (160 * 1024) / lds > 0 ? (160 * 1024) / lds : 1;
  int64_t grid = 256 * (int64_t)occ;
  if (grid > total) grid = total;
  hipLaunchKernelGGL((conv1x1p_kernel<Cf, ACC, STATS, BSTATS, ATR, APPLY, STR>), dim3((unsigned)grid),
                     dim3(Cf::kThreads), lds, s, a, b, y, c, cm, part, M, K, N, bs, cg, acoef, ap);
  return 0;
}

constexpr int kMaxATRK = 512;  // ATR coefficient table: [2][K] floats past kLds

template <class Cf, bool ACC, bool STATS, bool NT, bool BSTATS, bool ATR = false, bool APPLY = false, bool STR = false>
int launch_nt(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm, float* part,
              int M, int K, int N, const BnSrc& bs, const CGeom& cg, hipStream_t s, const float* acoef = nullptr,
              const ApArgs& ap = ApArgs{}) {
  static bool attr = false;
  constexpr int kMaxLds = Cf::kLds + (ATR ? 2 * kMaxATRK * 4 : 0);
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_kernel<Cf, ACC, STATS, NT, BSTATS, ATR, APPLY, STR>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds) != hipSuccess)
      return -3;
    attr = true;
  }
  if (ATR && K > kMaxATRK) return -1;
  const int lds = Cf::kLds + (ATR ? 2 * K * 4 : 0);
  const int64_t grid = (int64_t)(M + Cf::BM - 1) / Cf::BM * (N / Cf::BN);
  ApArgs apx = ap;
  apx.probe = g_probe;
  // persistent: from two tiles per workgroup up (probes run on the one-tile kernel)
  if constexpr (!NT) {
    constexpr bool kMeasured = Cf::kWaves >= 16 && !ACC && !ATR && !APPLY;  // see g_persist
    const int pm = persist_mode();
    if ((pm == 2 || (pm == 1 && kMeasured)) && g_probe == 0 && !ap.a2 &&
        grid >= 2 * 256 * (int64_t)((160 * 1024) / PL<Cf>::kLds))
      return launch_p<Cf, ACC, STATS, BSTATS, ATR, APPLY, STR>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef, apx);
  }
  hipLaunchKernelGGL((conv1x1_kernel<Cf, ACC, STATS, NT, BSTATS, ATR, APPLY, STR>), dim3((unsigned)grid),
                     dim3(Cf::kThreads), lds, s, a, b, y, c, cm, part, M, K, N, bs, cg, acoef, apx);
  return 0;
}

template <class Cf, bool ACC, bool STATS, bool BSTATS = false>
int launch(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm, float* part, int M,
           int K, int N, const BnSrc& bs, const CGeom& cg, hipStream_t s, const ApArgs& ap = ApArgs{}) {
  if constexpr (ACC)
    if (cg.s) return launch_nt<Cf, ACC, STATS, false, BSTATS, false, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s,
                                                                                  nullptr, ap);
  // (non-temporal output stores, NT = true, measured no gain: default-policy stores keep the
  // output in L2 for the consuming BatchNorm)
  return launch_nt<Cf, ACC, STATS, false, BSTATS>(a, b, y, c, cm, part, M, K, N, bs, cg, s, nullptr, ap);
}

using GXWide = G1<256, 4, 4>;  // N % 256 == 0 (large M): 16 waves of 64x64, a block writes whole 512-B rows
using GWide = G1<128, 4, 2>;   // N % 128 == 0: 8 waves of 64x64
using GNarrow = G1<64, 4, 1>;  // N == 64 (or odd multiples of 64): 4 waves of 64x64
// 8 waves of 128 x 64 (PDT_CONV1X1_W2=1, A/B): the deep-K forward shapes (layers 3-4) are MFMA-fed, not HBM-bound,
// and a 64 x 64 wave tile reads 2.7x the LDS bytes per MFMA of a 128 x 64 one
using GXWide2 = G1<256, 2, 4>;
inline bool w2_on() {
  static const int v = [] {
    const char* e = getenv("PDT_CONV1X1_W2");
    return (e && e[0]) ? (int)strtol(e, nullptr, 10) : 0;
  }();
  return v != 0;
}

template <class Cf>
int dispatch(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm, float* part,
             int M, int K, int N, const BnSrc& bs, const CGeom& cg, hipStream_t s, const float* acoef = nullptr,
             const ApArgs& ap = ApArgs{}) {
  if ((c && part) || (cm && !c) || (part && bs.part) || (cg.s && (!c || cm))) return -1;  // not instantiated
  if (acoef) {  // forward with the producing BatchNorm's apply deferred here (+ statistics epilogue)
    if (c || bs.part) return -1;
    if (part) return launch_nt<Cf, false, true, false, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef);
    return launch_nt<Cf, false, false, false, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef);
  }
  if (bs.part) {
    if (!bs.mean) return -1;
    if (c) return launch<Cf, true, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s);
    return launch<Cf, false, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s);
  }
  if (c) return launch<Cf, true, false>(a, b, y, c, cm, part, M, K, N, bs, cg, s);
  if (part) return launch<Cf, false, true>(a, b, y, c, cm, part, M, K, N, bs, cg, s, ap);
  return launch<Cf, false, false>(a, b, y, c, cm, part, M, K, N, bs, cg, s);
}

}  // namespace

extern "C" {

int pdt_conv1x1_tile_rows() { return 256; }

// Diagnosis (tools/conv1x1_bw.py --probe): see ApArgs::probe. Results are wrong while set.
void pdt_conv1x1_probe(int probe) { g_probe = probe; }

// A/B hook (see g_persist): 0 = one tile per workgroup, 1 = persistent where measured faster (default),
// 2 = every kind and tile persistent. Returns the previous mode.
int pdt_conv1x1_persist(int mode) {
  const int old = persist_mode();
  g_persist = mode < 0 ? -1 : (mode > 2 ? 2 : mode);
  return old;
}

// y[M,N] = a[M,K] * b[N,K]^T (+ c[M,N], masked by the bit-mask cm when given: bit j of byte
// (m*N + n) / 8 — the BatchNorm ReLU mask layout); part: stats of y per 256-row tile (see above),
// or null. All bf16 row-major, K % 32 == 0, N % 64 == 0, M * max(K, N) < 2^31. c may alias y.
// bn_x / bn_mask / bn_mean / bn_part (BSTATS, all null = off): y is the gradient at the output of a
// BatchNorm with input bn_x [M,N], ReLU mask bn_mask (or null) and mean bn_mean [N]; bn_part
// [2][T][N] receives that BatchNorm's backward per-tile sums (see the header). Not with part.
// c_s, c_H, c_W (c_s > 0): c is the compact gradient of the stride-c_s subsampling of y's pixels
// (y rows = [n][c_H][c_W]), see CGeom; needs c, no cm.
// acoef ([2][K] fp32, or null): A is a BatchNorm input, relu(acoef[0][k] x + acoef[1][k]) is used (ATR).
int pdt_conv1x1_gemm(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* c, const uint8_t* cm,
                     float* part, int M, int K, int N, const uint16_t* bn_x, const uint8_t* bn_mask,
                     const float* bn_mean, float* bn_part, int c_s, int c_H, int c_W, const float* acoef,
                     hipStream_t s, int nostore) {
  ApArgs ap{};
  ap.nostore = nostore && part && !c && !acoef && !bn_part ? 1 : 0;  // statistics-only forward (see ApArgs)
  if (nostore && !ap.nostore) return -1;
  if (M < 1 || K < 32 || K % 32 != 0 || N < 64 || N % 64 != 0) return -1;
  if ((int64_t)M * (K > N ? K : N) >= ((int64_t)1 << 31) || (int64_t)N * K >= ((int64_t)1 << 31)) return -2;
  const BnSrc bs{bn_x, bn_mask, bn_mean, bn_part};
  CGeom cg{0, 1, 1, 1, 1};
  if (c_s > 0) {
    if (c_H < 1 || c_W < 1 || M % (c_H * c_W) != 0) return -1;
    cg = CGeom{c_s, c_H, c_W, (c_H - 1) / c_s + 1, (c_W - 1) / c_s + 1};
  }
  // 256-wide tiles when the grid is deep (>= 8 blocks per CU): contiguous 512-B output rows, A read once
  // (tools/conv1x1_probe.py, 1024 images: 128->512 @28 fwd+stats 293 vs 342 us, 64->256 @56 506-554 vs
  // 553-571; at 512->2048 @7 — 1,568 blocks — 5 % slower, hence the threshold)
  // (the 16-wave tile only for the plain / statistics forward and the data gradient without an accumulate
  // source — with the ATR operand transform or an accumulate source the 8-wave tile, two workgroups per
  // CU, ran 5-10 % faster at every ResNet-50 depth: profiles/r5/conv1x1_tiles_bench_b1024.txt)
  if (w2_on() && N % 256 == 0 && K >= 256 && !c && !acoef && !bs.part && !(g_probe & 64))
    return dispatch<GXWide2>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef, ap);
  if (N % 256 == 0 && (int64_t)((M + 255) / 256) * (N / 256) >= 2048 && !(g_probe & 64) && !c && !acoef)
    return dispatch<GXWide>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef, ap);
  if (N % 128 == 0 && !(g_probe & 8) && !small_grid_narrow((int64_t)((M + 255) / 256) * (N / 128)))
    return dispatch<GWide>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef, ap);
  return dispatch<GNarrow>(a, b, y, c, cm, part, M, K, N, bs, cg, s, acoef, ap);
}

// SEG: y[M,N] = [a1 | a2 (x rep2) | 1] [M, k1 + rep2 k2 + 32] * b[N, k1 + rep2 k2 + 32]^T, with the BSTATS
// epilogue when bn_x is given (as pdt_conv1x1_gemm). a1 [M, k1], a2 [M, k2] row-major bf16, k1 % 32 == 0,
// k2 % 32 == 0 (ops/conv.py _bwd_alg: the data gradient of conv3 with bn3's backward folded into b).
int pdt_conv1x1_gemm_seg(const uint16_t* a1, int k1, const uint16_t* a2, int k2, int rep2, const uint16_t* b,
                         uint16_t* y, int M, int N, const uint16_t* bn_x, const uint8_t* bn_mask, const float* bn_mean,
                         float* bn_part, hipStream_t s) {
  const int K = k1 + rep2 * k2 + 32;
  if (M < 1 || k1 < 32 || k1 % 32 || k2 < 32 || k2 % 32 || rep2 < 1 || N < 64 || N % 64 != 0 || !a2) return -1;
  if ((int64_t)M * (K > N ? K : N) >= ((int64_t)1 << 31) || (int64_t)N * K >= ((int64_t)1 << 31)) return -2;
  const BnSrc bs{bn_x, bn_mask, bn_mean, bn_part};
  const CGeom cg{0, 1, 1, 1, 1};
  ApArgs ap{};
  ap.a2 = a2; ap.k1 = k1; ap.k2 = k2; ap.rep2 = rep2;
  // tile for N % 256 (PDT_SEG_TILE, A/B): 0 = 8 waves of 64 x 64 (256 x 128), 1 = 8 waves of 128 x 64 (256 x 256:
  // half the LDS bytes per MFMA for these deep-K shapes), 2 = 16 waves of 64 x 64 (256 x 256)
  static const int seg_tile = [] {
    const char* e = getenv("PDT_SEG_TILE");
    return (e && e[0]) ? (int)strtol(e, nullptr, 10) : 0;
  }();
  const bool bst = bn_part != nullptr;
  if (bst && !bn_mean) return -1;
  if (N % 256 == 0 && seg_tile == 1) {
    if (bst) return launch_nt<GXWide2, false, false, false, true>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
    return launch_nt<GXWide2, false, false, false, false>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
  }
  if (N % 256 == 0 && seg_tile == 2) {
    if (bst) return launch_nt<GXWide, false, false, false, true>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
    return launch_nt<GXWide, false, false, false, false>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
  }
  if (bst) {
    if (N % 128 == 0) return launch_nt<GWide, false, false, false, true>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
    return launch_nt<GNarrow, false, false, false, true>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
  }
  if (N % 128 == 0) return launch_nt<GWide, false, false, false, false>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
  return launch_nt<GNarrow, false, false, false, false>(a1, b, y, nullptr, nullptr, nullptr, M, K, N, bs, cg, s, nullptr, ap);
}

// APPLY: y[M,N] = relu(ab[0] * (a b^T) + ab[1] + r) with r = res (rab null) or rab[0] res + rab[1], and its
// ReLU bits -> mask [M * N / 8]; acoef as in pdt_conv1x1_gemm (ATR). The GEMM must be the one whose
// statistics gave ab (same a, b, acoef: the z values are recomputed bit for bit).
int pdt_conv1x1_gemm_apply(const uint16_t* a, const uint16_t* b, uint16_t* y, const uint16_t* res, const float* ab,
                           const float* rab, uint8_t* mask, int M, int K, int N, const float* acoef, hipStream_t s) {
  if (M < 1 || K < 32 || K % 32 != 0 || N < 64 || N % 64 != 0 || !res || !ab || !mask) return -1;
  if ((int64_t)M * (K > N ? K : N) >= ((int64_t)1 << 31) || (int64_t)N * K >= ((int64_t)1 << 31)) return -2;
  const BnSrc bs{};
  const CGeom cg{0, 1, 1, 1, 1};
  const ApArgs ap{ab, rab, mask};
  // (APPLY on the 8-wave tile at every size: 892 vs 943 us at 64->256 @56, 505 vs 540 @28, 307 vs 333 @14 on
  // the 16-wave one, profiles/r5/conv1x1_tiles_bench_b1024.txt)
  if (N % 128 == 0 && !(g_probe & 8)) {
    if (acoef) return launch_nt<GWide, false, false, false, false, true, true>(a, b, y, res, nullptr, nullptr, M, K, N, bs, cg, s, acoef, ap);
    return launch_nt<GWide, false, false, false, false, false, true>(a, b, y, res, nullptr, nullptr, M, K, N, bs, cg, s, acoef, ap);
  }
  if (acoef) return launch_nt<GNarrow, false, false, false, false, true, true>(a, b, y, res, nullptr, nullptr, M, K, N, bs, cg, s, acoef, ap);
  return launch_nt<GNarrow, false, false, false, false, false, true>(a, b, y, res, nullptr, nullptr, M, K, N, bs, cg, s, acoef, ap);
}

}  // extern "C"
