// Weight gradient of a 1x1 convolution on MFMA (gfx950), NHWC bf16, fp32 accumulate:
//
//   dW[co, ci] = sum_m dY[m, co] * X[m, ci]          (m = (n, h, w): K = N*H*W pixels)
//
// Not in the reference (LeNet has no 1x1 convs, /root/reference/cnn.py:10-16). Replaces MIOpen's
// igemm_wrw kernels on ResNet-50's layer-1 1x1 convs (M = 3.2M pixels at 1024/GPU; 7 calls,
// 2.6 ms/step with their zero-fill / cast passes, profiles/r3) — the last MIOpen kernels of the
// ResNet-50 step, and the ones whose run-time compile dominated the fresh-box first step.
//
// These shapes are HBM-bound (a 64x256 wgrad reads 2 GB for 105 GFLOP), so the design goal is
// one pass over dY and X at full bandwidth:
//   * a workgroup owns the WHOLE channel block CO_B x CI_B (all of dW for layer-1 shapes) and a
//     contiguous pixel range (split-K over pixels): every dY / X byte crosses HBM once; fp32
//     partials per split are summed in a fixed order by conv1x1_wgrad_reduce_kernel
//     (deterministic, no atomics);
//   * a stage = 32 pixels of dY [32 x CO_B] and X [32 x CI_B] — contiguous global rows — staged
//     by LDS-DMA (global_load_lds_dwordx4) through a 4-slot ring, issued 3 stages ahead, one
//     s_barrier per stage, counted vmcnt so the DMA stays in flight across barriers;
//   * both operands are pixel-major (K-strided); fragments come from LDS through the transposed
//     read ds_read_b64_tr_b16 (4 pixel rows x 16 channels per 16-lane group, each lane receiving one
//     channel's 4 pixels), as in conv3x3_wgrad.hip; rows XOR-swizzled (by permuting each lane's
//     DMA SOURCE chunk — the DMA writes LDS linearly) so 4 consecutive rows hit 4 distinct 64-B
//     bank groups;
//   * waves tile the block as WCO x WCI of v_mfma_f32_32x32x16_bf16 32x32 accumulators.
#include "../common.h"

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef short s4v __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

__device__ __attribute__((aligned(256))) uint4 g_wg1_zero[16];  // zero page for pixels past M (never written)

// KP: pixels per stage; SLOTS: LDS ring depth (SLOTS - 1 stages in flight)
template <int CO_B_, int CI_B_, int WCO_, int WCI_, int KP_ = 32, int SLOTS_ = 4>
struct W1Cfg {
  static constexpr int CO_B = CO_B_, CI_B = CI_B_, WCO = WCO_, WCI = WCI_, kKP = KP_;
  static constexpr int kSlotBytes = kKP * (CO_B + CI_B) * 2;
  static constexpr int kSlots = SLOTS_ * kSlotBytes <= 160 * 1024 ? SLOTS_ : (160 * 1024) / kSlotBytes;
  static constexpr int kAhead = kSlots - 1;
  static constexpr int kWaves = (CO_B / WCO) * (CI_B / WCI), kThreads = kWaves * 64;
  static constexpr int kRowY = CO_B * 2, kRowX = CI_B * 2;  // LDS row bytes
  static constexpr int kYBytes = kKP * kRowY, kXBytes = kKP * kRowX, kSlot = kYBytes + kXBytes;
  static constexpr int kLds = kSlots * kSlot;
  static constexpr int kYLd = kYBytes / 1024 / kWaves, kXLd = kXBytes / 1024 / kWaves;  // DMA per wave per stage
  static constexpr int kG = kYLd + kXLd;
  static constexpr int kMI = WCO / 32, kNJ = WCI / 32;
  static constexpr int kOcc = (160 * 1024) / kLds;  // workgroups per CU (LDS-limited)
  static constexpr int kMinWaves = kOcc * kWaves / 4 < 1 ? 1 : (kOcc * kWaves / 4 > 4 ? 4 : kOcc * kWaves / 4);  // per SIMD
  static_assert(kYLd * 1024 * kWaves == kYBytes && kXLd * 1024 * kWaves == kXBytes, "DMA split");
  static_assert(kWaves <= 8 && kLds <= 160 * 1024, "workgroup");
};

// 16-B chunk swizzle: 4 consecutive rows of a transposed read on 4 distinct 64-B bank groups.
// 128-B rows: rows r, r+1 are the two halves of a 256-B bank row, r+2, r+3 flip chunk bit 2;
// >= 256-B rows: chunk bits 2-3 ^= row & 3. Both are involutions (used to permute DMA sources).
template <int ROWB>
__host__ __device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (ROWB == 128) return ch ^ (((row >> 1) & 1) << 2);
  else return ch ^ ((row & 3) << 2);
}
template <int ROWB>
__device__ __forceinline__ int chunk_off(int row, int ch) { return row * ROWB + (swz<ROWB>(row, ch) << 4); }

// The transposed read as inline asm: for the builtin the compiler cannot tell which LDS bytes it
// reads, so it put an s_waitcnt vmcnt(0) for ALL outstanding LDS-DMA (incl. the stages just issued
// ahead) in front of it, serialising the ring. Completion is tracked by hand instead (lgkm_fence).
__device__ __forceinline__ s4v tr_read(const char* p) {
  s4v r;
  const uint32_t a = (uint32_t)(uintptr_t)(PDT_LDS const char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
__device__ __forceinline__ bf16x8 cat2(s4v a, s4v b) {
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}
__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (PDT_LDS void*)lds_wave_base, 16, 0, 0);
}
template <int MI, int NJ>
__device__ __forceinline__ void lgkm_fence(bf16x8 (&a)[MI], bf16x8 (&b)[NJ]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(b[j]));
}
// s_waitcnt vmcnt(N) leaving expcnt / lgkmcnt unconstrained (gfx9 simm16 encoding)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// wait until at most `later` stages of G DMA instructions each are outstanding (later <= K)
template <int G, int K>
__device__ __forceinline__ void wait_stages(int later) {
  if constexpr (K == 0) {
    wait_vm<0>();
  } else {
    if (later >= K) wait_vm<K * G>();
    else wait_stages<G, K - 1>(later);
  }
}

struct W1Geo {
  int M, Ci, Co, ntiles, tiles_per_split, nsplit, nblk;
  int ilv;  // 1: split k takes stages k, k + nsplit, ... (all workgroups stream neighbouring pixels)
  // SEG (dy2 != null): the dY operand is the channel concatenation [dY (co1) | dy2 (co2) | CO_B columns of
  // 1.0]; Co = co1 + co2 + CO_B. The ones block's rows are the column sums of X (ops/conv.py _bwd_alg).
  const uint16_t* dy2;
  int co1, co2;
};

__device__ __attribute__((aligned(256))) uint4 g_wg1_ones[16] = {  // bf16 1.0 page (SEG)
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u},
    {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}, {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u}};

template <class Cf>
__global__ __launch_bounds__(Cf::kThreads, Cf::kMinWaves) void conv1x1_wgrad_kernel(const uint16_t* __restrict__ X,
                                                                               const uint16_t* __restrict__ dY,
                                                                               float* __restrict__ ws, W1Geo g) {
  constexpr int CO_B = Cf::CO_B, CI_B = Cf::CI_B, RY = Cf::kRowY, RX = Cf::kRowX;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // XCD-aware: consecutive logical ids (one split's channel blocks: same pixels) on one XCD
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / g.nblk, bt = L % g.nblk;
  const int nci = g.Ci / CI_B;
  const int co0 = (bt / nci) * CO_B, ci0 = (bt % nci) * CI_B;
  const int t_begin = g.ilv ? split : split * g.tiles_per_split, t_step = g.ilv ? g.nsplit : 1;
  const int S = g.ilv ? (g.ntiles - split + g.nsplit - 1) / g.nsplit
                      : min(g.ntiles, t_begin + g.tiles_per_split) - t_begin;
  constexpr int kKP = Cf::kKP, kSlots = Cf::kSlots, kAhead = Cf::kAhead;

  // SEG: this workgroup's dY source (uniform): dY, dy2, or the ones page, with its row stride
  const uint16_t* ysrc = dY;
  int ldy = g.Co, ycol = co0;
  bool yones = false;
  if (g.dy2) {
    if (co0 < g.co1) { ldy = g.co1; }
    else if (co0 < g.co1 + g.co2) { ysrc = g.dy2; ldy = g.co2; ycol = co0 - g.co1; }
    else { yones = true; ldy = 0; ycol = 0; }
  }
  // per-lane DMA pieces (stage independent): row in the tile and element offset from its first pixel
  int yrow[Cf::kYLd], yoff[Cf::kYLd], xrow[Cf::kXLd], xoff[Cf::kXLd];
#pragma unroll
  for (int i = 0; i < Cf::kYLd; ++i) {
    const int o = (wid * Cf::kYLd + i) * 1024 + lane * 16, row = o / RY, slot = (o % RY) >> 4;
    yrow[i] = row;
    yoff[i] = row * ldy + ycol + swz<RY>(row, slot) * 8;
  }
#pragma unroll
  for (int i = 0; i < Cf::kXLd; ++i) {
    const int o = (wid * Cf::kXLd + i) * 1024 + lane * 16, row = o / RX, slot = (o % RX) >> 4;
    xrow[i] = row;
    xoff[i] = row * g.Ci + ci0 + swz<RX>(row, slot) * 8;
  }
  auto issue = [&](int s) {
    char* slot = lds + (s % kSlots) * Cf::kSlot;
    const int p0 = (t_begin + s * t_step) * kKP;
    const uint16_t* yb = ysrc + (int64_t)p0 * ldy;
    const uint16_t* xb = X + (int64_t)p0 * g.Ci;
#pragma unroll
    for (int i = 0; i < Cf::kYLd; ++i) {
      const void* src = p0 + yrow[i] < g.M ? (yones ? (const void*)g_wg1_ones : (const void*)(yb + yoff[i]))
                                           : (const void*)g_wg1_zero;
      dma16(src, slot + (wid * Cf::kYLd + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < Cf::kXLd; ++i) {
      const void* src = p0 + xrow[i] < g.M ? (const void*)(xb + xoff[i]) : (const void*)g_wg1_zero;
      dma16(src, slot + Cf::kYBytes + (wid * Cf::kXLd + i) * 1024);
    }
  };

  // wave -> WCO x WCI block; lane roles of the transposed reads (see conv3x3_wgrad.hip)
  constexpr int nwci = CI_B / Cf::WCI;
  const int wco = wid / nwci, wci = wid % nwci;
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int prow = 8 * (grp >> 1) + q;
  const int half8 = (p & 1) * 8;
  int ya[Cf::kMI], xa[Cf::kNJ];  // LDS byte offsets of this lane's pieces in row `prow`
#pragma unroll
  for (int i = 0; i < Cf::kMI; ++i) ya[i] = chunk_off<RY>(prow, (wco * Cf::WCO + 32 * i + 16 * (grp & 1) + 4 * p) >> 3) + half8;
#pragma unroll
  for (int j = 0; j < Cf::kNJ; ++j) xa[j] = chunk_off<RX>(prow, (wci * Cf::WCI + 32 * j + 16 * (grp & 1) + 4 * p) >> 3) + half8;
  // rows prow + 4 and prow + 16 k: the swizzles depend on row bits 0-1 (>= 256-B rows) or bit 1
  // (128-B rows), which adding 4 or 16 leaves alone -> constant offsets
  f16v acc[Cf::kMI][Cf::kNJ];
#pragma unroll
  for (int i = 0; i < Cf::kMI; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNJ; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

#pragma unroll
  for (int s = 0; s < kAhead; ++s)
    if (s < S) issue(s);
  for (int s = 0; s < S; ++s) {
    // this stage's DMA is complete once at most the later in-flight stages' remain outstanding
    wait_stages<Cf::kG, kAhead - 1>(min(S - 1, s + kAhead - 1) - s);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + kAhead < S) issue(s + kAhead);  // its slot was last read at stage s - 1: every wave is past it
    const char* ys = lds + (s % kSlots) * Cf::kSlot;
    const char* xs = ys + Cf::kYBytes;
#pragma unroll
    for (int kk = 0; kk < kKP / 16; ++kk) {
      bf16x8 a[Cf::kMI], b[Cf::kNJ];
#pragma unroll
      for (int i = 0; i < Cf::kMI; ++i) {
        const char* pp = ys + ya[i] + kk * 16 * RY;
        a[i] = cat2(tr_read(pp), tr_read(pp + 4 * RY));
      }
#pragma unroll
      for (int j = 0; j < Cf::kNJ; ++j) {
        const char* pp = xs + xa[j] + kk * 16 * RX;
        b[j] = cat2(tr_read(pp), tr_read(pp + 4 * RX));
      }
      // the reads' results are ready: the wait takes every fragment as an in/out operand, so no MFMA
      // can be scheduled above it
      lgkm_fence(a, b);
#pragma unroll
      for (int i = 0; i < Cf::kMI; ++i)
#pragma unroll
        for (int j = 0; j < Cf::kNJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);  // D[co][ci]
    }
  }
  // partials ws[split][co][ci]; 32x32 accumulator: lane holds ci = l % 32,
  // co = 8 (v / 4) + 4 (l / 32) + v % 4 for v = 0..15
  float* wsp = ws + (int64_t)split * g.Co * g.Ci;
#pragma unroll
  for (int i = 0; i < Cf::kMI; ++i)
#pragma unroll
    for (int j = 0; j < Cf::kNJ; ++j) {
      const int ci = ci0 + wci * Cf::WCI + 32 * j + (lane & 31);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int co = co0 + wco * Cf::WCO + 32 * i + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
        wsp[(int64_t)co * g.Ci + ci] = acc[i][j][v];
      }
    }
}

// dw[co][ci] (bf16) = sum over splits in a fixed order. A workgroup takes 16 float4 columns and
// its 16 wave-quarters split the nsplit partials round-robin (each summed in order), then one
// fixed-order pass over the 16 group sums: deterministic, and 16x the parallelism of one thread per
// column (whose serial 192-deep loads ran 49 us for a 64 KB result).
constexpr int kRedCols = 16, kRedGroups = 16;
template <bool F32>
__global__ __launch_bounds__(256) void conv1x1_wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                   void* __restrict__ dw, int nsplit, int64_t n4) {
  __shared__ float4 part[kRedGroups][kRedCols];
  const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
  const int64_t i = (int64_t)blockIdx.x * kRedCols + col;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4)
    for (int k = grp; k < nsplit; k += kRedGroups) {
      const float4 v = reinterpret_cast<const float4*>(ws + (int64_t)k * n4 * 4)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  part[grp][col] = s;
  __syncthreads();
  if (grp == 0 && i < n4) {
    float4 t = part[0][col];
#pragma unroll
    for (int k = 1; k < kRedGroups; ++k) {
      const float4 v = part[k][col];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    if constexpr (F32) {
      reinterpret_cast<float4*>(dw)[i] = t;
    } else {
      const uint32_t lo = (uint32_t)f2bf(t.x) | ((uint32_t)f2bf(t.y) << 16);
      const uint32_t hi = (uint32_t)f2bf(t.z) | ((uint32_t)f2bf(t.w) << 16);
      reinterpret_cast<uint2*>(dw)[i] = make_uint2(lo, hi);
    }
  }
}

// Channel-block configurations (the block covers all of dW for ResNet-50's layer-1 shapes) x
// pipeline variants (pixels per stage, ring depth; the ring is clamped to the 160 KB of LDS)
enum class Blk { k64x64, k256x64, k64x256, k128x256, k128x128 };
constexpr int kVariants = 5;
constexpr int kVarKP[kVariants] = {32, 32, 64, 64, 32};
constexpr int kVarSlots[kVariants] = {4, 8, 4, 3, 3};  // 4: a 3-slot ring, two 128x256 workgroups per CU (SEG A/B)

template <Blk B, int V>
struct CfgOf;
template <int V>
struct CfgOf<Blk::k64x64, V> { using T = W1Cfg<64, 64, 32, 32, kVarKP[V], kVarSlots[V]>; };     // 4 waves
template <int V>
struct CfgOf<Blk::k256x64, V> { using T = W1Cfg<256, 64, 64, 64, kVarKP[V], kVarSlots[V]>; };   // 4 waves
template <int V>
struct CfgOf<Blk::k64x256, V> { using T = W1Cfg<64, 256, 64, 64, kVarKP[V], kVarSlots[V]>; };   // 4 waves
template <int V>
struct CfgOf<Blk::k128x256, V> { using T = W1Cfg<128, 256, 64, 64, kVarKP[V], kVarSlots[V]>; }; // 8 waves
template <int V>
struct CfgOf<Blk::k128x128, V> { using T = W1Cfg<128, 128, 64, 64, kVarKP[V], kVarSlots[V]>; }; // 4 waves (SEG)

inline Blk pick_block(int Co, int Ci) {
  if (Co % 128 == 0 && Ci % 256 == 0) return Blk::k128x256;
  if (Co % 256 == 0 && Ci % 64 == 0) return Blk::k256x64;
  if (Co % 64 == 0 && Ci % 256 == 0) return Blk::k64x256;
  return Blk::k64x64;
}

struct CfgInfo {
  int cob, cib, occ, kp;
};
template <class Cf>
CfgInfo info_of() { return CfgInfo{Cf::CO_B, Cf::CI_B, Cf::kOcc, Cf::kKP}; }
template <Blk B>
CfgInfo info_var(int v) {
  switch (v) {
    case 4: return info_of<typename CfgOf<B, 4>::T>();
    case 1: return info_of<typename CfgOf<B, 1>::T>();
    case 2: return info_of<typename CfgOf<B, 2>::T>();
    case 3: return info_of<typename CfgOf<B, 3>::T>();
    default: return info_of<typename CfgOf<B, 0>::T>();
  }
}
inline CfgInfo info(Blk b, int v) {
  switch (b) {
    case Blk::k128x128: return info_var<Blk::k128x128>(v);
    case Blk::k128x256: return info_var<Blk::k128x256>(v);
    case Blk::k256x64: return info_var<Blk::k256x64>(v);
    case Blk::k64x256: return info_var<Blk::k64x256>(v);
    default: return info_var<Blk::k64x64>(v);
  }
}
inline void block_dims(Blk b, int& cob, int& cib, int& occ) {
  const CfgInfo i = info(b, 0);
  cob = i.cob; cib = i.cib; occ = i.occ;
}

int g_target_wgs = 0;  // 0: by shape (wgs_default)
int g_variant = -1;    // -1: by shape (variant_default)
int g_ilv = -1;        // -1: by shape; 0 / 1 forced

// Measured on MI355X at ResNet-50 batch 1024 (tools/conv1x1_wgrad_bench.py, profiles/r3/
// conv1x1_wgrad_bench_b1024.txt): FEWER streams than CUs with interleaved stages stream best —
// 192 workgroups taking stages k, k + 192, ... (all of them on neighbouring pixels at any moment)
// reach 362-437 us on the 2.0-2.5 GB layer-1 shapes (MIOpen 380-486 us); 512 separate pixel ranges
// (2 workgroups per CU) ran 1.3x slower. 64x64: 64-pixel stages (4 KB DMA per stage at 32 was too
// little work per barrier).
inline int variant_default(Blk b) { return b == Blk::k64x64 ? 2 : 0; }
inline int wgs_default(const CfgInfo&, int nblk) { return nblk == 1 ? 192 : 256; }

// SEG: a block whose CO_B divides both concatenated segments
inline Blk pick_block_seg(int co1, int co2, int Ci) {
  if (Ci % 256 == 0 && co1 % 128 == 0 && co2 % 128 == 0) return Blk::k128x256;
  if (Ci % 128 == 0 && co1 % 128 == 0 && co2 % 128 == 0) return Blk::k128x128;
  if (Ci % 256 == 0) return Blk::k64x256;
  return Blk::k64x64;
}

// SEG pipeline variant (PDT_WGRAD_SEG_VARIANT, A/B; -1 = the shape default)
inline int seg_variant() {
  static const int v = [] {
    const char* e = getenv("PDT_WGRAD_SEG_VARIANT");
    // default 4 (a 3-slot ring: two 128 x 256 workgroups per CU): 1.08-1.13x variant 0 at ResNet-50's layer 2-4
    // shapes (tools/alg_bench.py, profiles/r6/alg_kernels_bench.txt)
    const int x = (e && e[0]) ? (int)strtol(e, nullptr, 10) : 4;
    return x >= -1 && x < kVariants ? x : 4;
  }();
  return v;
}

inline bool geo_of(int M, int Ci, int Co, W1Geo& g, int seg_co1 = 0, int seg_co2 = 0) {
  if (M < 1 || Ci % 64 != 0 || Co % 64 != 0) return false;
  const Blk b = seg_co1 ? pick_block_seg(seg_co1, seg_co2, Ci) : pick_block(Co, Ci);
  if (seg_co1) {  // Co = co1 + co2 + CO_B (the ones block)
    const CfgInfo i0 = info(b, 0);
    Co = seg_co1 + seg_co2 + i0.cob;
  }
  g.dy2 = nullptr; g.co1 = seg_co1; g.co2 = seg_co2;
  const int var = seg_co1 && seg_variant() >= 0 ? seg_variant() : (g_variant >= 0 ? g_variant : variant_default(b));
  const CfgInfo ci = info(b, var);
  g.M = M; g.Ci = Ci; g.Co = Co;
  g.ntiles = (M + ci.kp - 1) / ci.kp;
  g.nblk = (Co / ci.cob) * (Ci / ci.cib);
  const int target = g_target_wgs > 0 ? g_target_wgs : wgs_default(ci, g.nblk);
  int ns = (target + g.nblk - 1) / g.nblk;
  // SEG (many channel blocks): ONE wave of workgroups — as many splits as fit the CUs' resident slots
  // (256 x LDS occupancy) rather than rounding up past them: 11 blocks x 24 splits = 264 workgroups at one
  // per CU would run 8 of them as a second, full-length wave
  if (seg_co1 && g_target_wgs <= 0) ns = (256 * (ci.occ > 0 ? ci.occ : 1)) / g.nblk;
  if (ns > g.ntiles) ns = g.ntiles;
  if (ns < 1) ns = 1;
  g.tiles_per_split = (g.ntiles + ns - 1) / ns;
  g.nsplit = (g.ntiles + g.tiles_per_split - 1) / g.tiles_per_split;
  g.ilv = g_ilv >= 0 ? g_ilv : 1;
  return true;
}

template <class Cf, bool F32 = false>
int launch(const uint16_t* x, const uint16_t* dy, void* dw, float* ws, const W1Geo& g, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1x1_wgrad_kernel<Cf>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  hipLaunchKernelGGL(conv1x1_wgrad_kernel<Cf>, dim3(g.nsplit * g.nblk), dim3(Cf::kThreads), Cf::kLds, s, x, dy, ws, g);
  const int64_t n4 = (int64_t)g.Co * g.Ci / 4;
  hipLaunchKernelGGL(conv1x1_wgrad_reduce_kernel<F32>, dim3((unsigned)((n4 + kRedCols - 1) / kRedCols)),
                     dim3(kRedCols * kRedGroups), 0, s, ws, dw, g.nsplit, n4);
  return 0;
}

template <Blk B, bool F32 = false>
int launch_var(int v, const uint16_t* x, const uint16_t* dy, void* dw, float* ws, const W1Geo& g, hipStream_t s) {
  switch (v) {
    case 4: return launch<typename CfgOf<B, 4>::T, F32>(x, dy, dw, ws, g, s);
    case 1: return launch<typename CfgOf<B, 1>::T, F32>(x, dy, dw, ws, g, s);
    case 2: return launch<typename CfgOf<B, 2>::T, F32>(x, dy, dw, ws, g, s);
    case 3: return launch<typename CfgOf<B, 3>::T, F32>(x, dy, dw, ws, g, s);
    default: return launch<typename CfgOf<B, 0>::T, F32>(x, dy, dw, ws, g, s);
  }
}

}  // namespace

extern "C" {

// fp32 workspace floats for pdt_conv1x1_wgrad at this shape (0: unsupported shape).
int64_t pdt_conv1x1_wgrad_ws_floats(int M, int Ci, int Co, int* nsplit_out) {
  W1Geo g;
  if (!geo_of(M, Ci, Co, g)) return 0;
  if (nsplit_out) *nsplit_out = g.nsplit;
  return (int64_t)g.nsplit * Co * Ci;
}

// dw[Co, Ci] (bf16) = dy[M, Co]^T x[M, Ci] (row-major bf16: the NHWC views of a stride-1 1x1 conv's
// output gradient and input). ws: pdt_conv1x1_wgrad_ws_floats() floats. Ci, Co % 64 == 0,
// M * max(Ci, Co) < 2^31. Returns 0, or < 0 for an unsupported shape (caller falls back).
int pdt_conv1x1_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int M, int Ci, int Co,
                      hipStream_t s) {
  if ((int64_t)M * (Ci > Co ? Ci : Co) >= ((int64_t)1 << 31)) return -2;
  W1Geo g;
  if (!geo_of(M, Ci, Co, g)) return -1;
  const Blk b = pick_block(Co, Ci);
  const int v = g_variant >= 0 ? g_variant : variant_default(b);
  switch (b) {
    case Blk::k128x256: return launch_var<Blk::k128x256>(v, x, dy, dw, ws, g, s);
    case Blk::k256x64: return launch_var<Blk::k256x64>(v, x, dy, dw, ws, g, s);
    case Blk::k64x256: return launch_var<Blk::k64x256>(v, x, dy, dw, ws, g, s);
    default: return launch_var<Blk::k64x64>(v, x, dy, dw, ws, g, s);
  }
}

// Tuning hook (tools/conv1x1_wgrad_bench.py): target workgroups (0 = by shape) and pipeline
// variant (-1 = by shape; 0..3 = kVarKP / kVarSlots), each left alone when < -1.
// SEG: out[co1 + co2 + cob, Ci] fp32 = [dy1 | dy2 | 1]^T x over M pixels (dy1 [M, co1], dy2 [M, co2], x [M, Ci]
// row-major bf16); rows co1 + co2 .. are the column sums of x. ws: pdt_conv1x1_wgrad_seg_ws_floats() floats;
// *rows_out = co1 + co2 + cob. Fixed-order split reduction (deterministic).
int64_t pdt_conv1x1_wgrad_seg_ws_floats(int M, int Ci, int co1, int co2, int* rows_out) {
  W1Geo g;
  if (co1 < 64 || co2 < 64 || !geo_of(M, Ci, co1 + co2 + 64, g, co1, co2)) return 0;
  if (rows_out) *rows_out = g.Co;
  return (int64_t)g.nsplit * g.Co * Ci;
}

int pdt_conv1x1_wgrad_seg(const uint16_t* x, const uint16_t* dy1, int co1, const uint16_t* dy2, int co2, float* out,
                          float* ws, int M, int Ci, hipStream_t s) {
  if ((int64_t)M * (Ci > co1 ? (Ci > co2 ? Ci : co2) : (co1 > co2 ? co1 : co2)) >= ((int64_t)1 << 31)) return -2;
  W1Geo g;
  if (co1 < 64 || co2 < 64 || !dy2 || !geo_of(M, Ci, co1 + co2 + 64, g, co1, co2)) return -1;
  g.dy2 = dy2;
  const Blk b = pick_block_seg(co1, co2, Ci);
  const int v = seg_variant() >= 0 ? seg_variant() : (g_variant >= 0 ? g_variant : variant_default(b));
  switch (b) {
    case Blk::k128x256: return launch_var<Blk::k128x256, true>(v, x, dy1, out, ws, g, s);
    case Blk::k128x128: return launch_var<Blk::k128x128, true>(v, x, dy1, out, ws, g, s);
    case Blk::k64x256: return launch_var<Blk::k64x256, true>(v, x, dy1, out, ws, g, s);
    default: return launch_var<Blk::k64x64, true>(v, x, dy1, out, ws, g, s);
  }
}

void pdt_conv1x1_wgrad_tune(int target_wgs, int variant, int interleave) {
  if (target_wgs >= 0) g_target_wgs = target_wgs;
  if (variant >= -1 && variant < kVariants) g_variant = variant;
  if (interleave >= -1 && interleave <= 1) g_ilv = interleave;
}

}  // extern "C"
