// ResNet stem convolution: 7x7 / stride 2 / pad 3, 3 -> 64 channels, NHWC bf16 on MFMA (gfx950).
//
// Not in the reference (its CNN is LeNet, /root/reference/cnn.py:10-16); it serves the ResNet-50
// north-star config, where this one layer writes the largest activation of the network
// (512 x 112 x 112 x 64 bf16 = 822 MB) and MIOpen's igemm_fwd kernel took 716 us for it
// (profiles/r2/steady_resnet50_ours.md) against a ~165 us HBM floor (154 MB read + 822 MB written).
//
// Three input channels make every generic implicit GEMM awkward (K = 147, rows of 6 bytes). Here
// the input is padded to 4 channels IN LDS and the kernel width to 8 taps in the (prepped)
// weights, so one k-step of v_mfma_f32_16x16x32_bf16 is one kernel row kh: 8 taps x 4 channels,
// and a lane's 8 k values (2 taps x 4 channels) are 16 contiguous LDS bytes of 2 neighbouring
// padded pixels. The 8th tap and 4th channel carry zero weights (and finite zero inputs).
//
//   * tile = 4 output rows x 112 output columns of one image, 256 threads: wave w computes
//     output row w — 7 pixel blocks x 4 channel blocks of 16x16 accumulators (112 VGPRs);
//   * persistent, 2 workgroups per CU (each a contiguous run of tiles) that drift out of phase,
//     so one's MFMAs overlap the other's loads, stores and barriers: the prepped weights
//     (64 x 7 x 32 bf16, 28 KB) are staged to LDS once; each tile's input window (13 rows x 230
//     columns x 4 channels, 25.6 KB) is loaded into registers after this tile's MFMAs, lands
//     while its stores drain, and replaces the window after a barrier; 7 k-steps of 28 MFMAs
//     per wave per tile. (One 8-wave workgroup per CU with two window buffers ran 277 us: its
//     waves move through the phases in lock step.)
//   * MFMA operands swapped (A = weights, B = pixels): a lane's accumulator is 4 consecutive
//     channels of one pixel; each 16-pixel block goes through a wave-private LDS staging block
//     and out as 16-B pieces, 1 KB contiguous per store instruction. Storing the accumulators
//     directly (8 B per lane, 16 cache lines per instruction) ran the kernel at 2.6 TB/s — the
//     no-store probe took 165 us of its 380;
//   * (A BatchNorm-statistics epilogue here — per-lane sums, Chan merges across lanes and rows —
//     measured 686 us vs 390 us + the 321 us reduce pass it replaces: the extra registers spill
//     in this 250-VGPR kernel; not kept.)
//   * the kernel is HBM-store bound, not MFMA bound (28 MFMAs per 16 x 64 outputs); a first
//     non-persistent version (4-row tiles, 3 workgroups per CU, weights re-staged and the window
//     loaded then waited on per tile) ran 384 us at batch 512 vs MIOpen's 860 us.
#include "../common.h"
#include "../tile_stats.h"

#include <algorithm>

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kCo = 64;
constexpr int kThreads = 256;                 // 4 waves
constexpr int kRowsOut = kThreads / 64;       // output rows per workgroup (one per wave)
constexpr int kTW = 112;                      // output columns per workgroup
constexpr int kMB = kTW / 16;                 // 16-pixel blocks per wave
constexpr int kInRows = 2 * kRowsOut + 5;     // 13 input rows
constexpr int kInCols = 2 * kTW + 6;          // 230 (column 229 only meets the zero 8th tap)
// LDS pixel column c at byte 8c + 16 (c >> 5): the 16-B pad per 32 pixels spreads the window
// writes (8 pixels per lane, 64 B apart across lanes: 16-way bank conflicts unpadded, measured
// as half of all LDS cycles) over all banks, and keeps the fragment reads (pixel pairs) aligned
// and conflict-free.
__host__ __device__ constexpr int pix_off(int c) { return 8 * c + 16 * (c >> 5); }
constexpr int kInPitch = pix_off(kInCols) + 16;  // 1,968 B
constexpr int kGroups = 30;                   // 8-pixel global load groups per input row
constexpr int kWRow = 7 * 64;                 // [kh 7][kw 8][ci 4] bf16
constexpr int kWPitch = kWRow + 16;           // +16 B: conflict-free 16-row fragment reads
constexpr int kLdsIn = kInRows * kInPitch;    // 25,584 B
constexpr int kStPitch = kCo * 2 + 16;        // epilogue staging row (one pixel), +16 B vs bank conflicts
constexpr int kStage = 16 * kStPitch;         // per wave: one 16-pixel block
constexpr int kLds = kLdsIn + kCo * kWPitch + kRowsOut * kStage;  // 64,496 B: window, weights, staging
constexpr int kWPrepElems = kCo * 7 * 32;
constexpr int kLdsStats = kLds + kRowsOut * 64 * 3 * 8;  // + per-lane (K, S, Q) pairs of the statistics variant

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}

// w: [64][7][7][3] (channels_last storage of [64, 3, 7, 7]) -> wp: [64][7][8][4], zero-padded.
__global__ __launch_bounds__(256) void stem_wprep_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ wp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kWPrepElems) return;
  const int co = i / 224, r = i % 224, kh = r / 32, k = r % 32, kw = k >> 2, ci = k & 3;
  wp[i] = (kw < 7 && ci < 3) ? w[((co * 7 + kh) * 7 + kw) * 3 + ci] : (uint16_t)0;
}

// One tile's input window -> registers: 13 rows x 30 groups of 8 pixels (48 B, 16-B aligned since
// W % 8 == 0), at most 2 groups per thread; out-of-image groups are zeros.
struct Window {
  uint4 v[2][3];
};

__device__ __forceinline__ void load_window(Window& wv, const uint16_t* __restrict__ X, int tid, int n, int ih0,
                                            int gb, int H, int W) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * kThreads;
    const int r = i / kGroups, g = i - r * kGroups;
    const int ih = ih0 + r, iw = gb + 8 * g;
    wv.v[u][0] = wv.v[u][1] = wv.v[u][2] = make_uint4(0u, 0u, 0u, 0u);
    if (i < kInRows * kGroups && ih >= 0 && ih < H && iw >= 0 && iw < W) {
      const uint4* src = reinterpret_cast<const uint4*>(X + ((int64_t)(n * H + ih) * W + iw) * 3);
      wv.v[u][0] = src[0];
      wv.v[u][1] = src[1];
      wv.v[u][2] = src[2];
    }
  }
}

// 24 bf16 = 8 pixels x (c0 c1 c2) -> 8 LDS pixels of (c0 c1 c2 0) at LDS columns 8g - 5 + q.
__device__ __forceinline__ void store_window(const Window& wv, char* lin, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + u * kThreads;
    if (i >= kInRows * kGroups) continue;
    const int r = i / kGroups, g = i - r * kGroups;
    const uint32_t w[12] = {wv.v[u][0].x, wv.v[u][0].y, wv.v[u][0].z, wv.v[u][0].w, wv.v[u][1].x, wv.v[u][1].y,
                            wv.v[u][1].z, wv.v[u][1].w, wv.v[u][2].x, wv.v[u][2].y, wv.v[u][2].z, wv.v[u][2].w};
    char* row = lin + r * kInPitch;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = 3 * q;  // bf16 index of channel 0
      const uint32_t c0 = (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
      const uint32_t c1 = (w[(e + 1) >> 1] >> (((e + 1) & 1) * 16)) & 0xffffu;
      const uint32_t c2 = (w[(e + 2) >> 1] >> (((e + 2) & 1) * 16)) & 0xffffu;
      const int col = 8 * g - 5 + q;
      if (col >= 0 && col < kInCols) *reinterpret_cast<uint2*>(row + pix_off(col)) = make_uint2(c0 | (c1 << 16), c2);
    }
  }
}

// Persistent: workgroup b owns a contiguous range of tiles (n, row tile, column tile), column
// tile fastest; the weights are staged once, and the next tile's input window is loaded into
// registers while this tile's MFMAs run (two LDS window buffers, one barrier per tile).
// Requires W % 32 == 0 (OW = W / 2 a multiple of 16; load groups never straddle the image edge).
#ifndef PDT_STEM_PROBE
#define PDT_STEM_PROBE 0  // diagnostics only (tools/convbench/stem_bench.cpp): 1 = no Y stores, 2 = no MFMA, 3 = no window loads
#endif
// STATS (FULL and OW == 112 only): BatchNorm statistics of the stored output, per wave over all its
// tiles — see the comment above pdt_stem_conv_fwd_stats.
template <bool FULL, bool STATS = false>  // FULL: every column tile is 112 wide (OW % 112 == 0): no per-block predicates
__global__ __launch_bounds__(kThreads, 2) void stem_conv_kernel(const uint16_t* __restrict__ X,
                                                          const uint16_t* __restrict__ Wp,
                                                          uint16_t* __restrict__ Y, int H, int W, int OH, int OW,
                                                          int nrt, int nct, int ntiles, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const lw = lds + kLdsIn;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int per = ntiles / gridDim.x, rem = ntiles % gridDim.x;
  const int t0 = blockIdx.x * per + min((int)blockIdx.x, rem);
  const int cnt = per + ((int)blockIdx.x < rem ? 1 : 0);
  if (cnt == 0) return;  // never: grid <= ntiles

  auto coords = [&](int t, int& n, int& oh0, int& ow0) {
    const int ct = t % nct, rt = (t / nct) % nrt;
    n = t / (nct * nrt);
    oh0 = rt * kRowsOut;
    ow0 = ct * kTW;
  };

  // ---- weights (once): 64 rows x 28 16-B pieces
  for (int i = tid; i < kCo * 28; i += kThreads) {
    const int co = i / 28, r = i - co * 28;
    *reinterpret_cast<uint4*>(lw + co * kWPitch + r * 16) = reinterpret_cast<const uint4*>(Wp)[i];
  }
  Window wv;
  int n, oh0, ow0;
  coords(t0, n, oh0, ow0);
  load_window(wv, X, tid, n, 2 * oh0 - 3, 2 * ow0 - 8, H, W);
  store_window(wv, lds, tid);

  const int pl = lane & 15, g = lane >> 4;
  const char* wrow = lw + pl * kWPitch + g * 16;
  char* const stage = lw + kCo * kWPitch + wid * kStage;
  // statistics: lane = channel pair (lane & 31) x 8 of the block's 16 pixels (lane >> 5); shifted
  // sums about K = the wave's first stored value of the pair (packed fp32)
  // (K, S, Q) live in a per-lane LDS slot between tiles, not in registers: this kernel sits at its
  // 256-VGPR budget (carrying them spilled to scratch)
  pdt_f2* const sst = reinterpret_cast<pdt_f2*>(lds + kLds) + (wid * 64 + lane) * 3;
  bool kset = false;
  int nrows = 0;
  const char* const srd = stage + (lane >> 5) * 8 * kStPitch + (lane & 31) * 4;
  for (int k = 0; k < cnt; ++k) {
    const int t = t0 + k;
    coords(t, n, oh0, ow0);
    __syncthreads();  // window k visible

    const char* lin = lds;
    const int nb = min(kMB, (OW - ow0) >> 4);
    f4 acc[kMB][4];
#pragma unroll
    for (int i = 0; i < kMB; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    // pixel pair p = 16 i + pl + g (columns 2p, 2p + 1) at pix_off(2p) = 16 p + 16 (p >> 4)
    const char* arow = lin + 2 * wid * kInPitch + 16 * (pl + g) + 16 * ((pl + g) >> 4);
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      bf16x8 bw[4], av[kMB];
#pragma unroll
      for (int j = 0; j < 4; ++j) bw[j] = *reinterpret_cast<const bf16x8*>(wrow + j * 16 * kWPitch + kh * 64);
#pragma unroll
      for (int i = 0; i < kMB; ++i)  // past-the-edge blocks read in-window LDS and are never stored
        av[i] = *reinterpret_cast<const bf16x8*>(arow + kh * kInPitch + i * 272);
#pragma unroll
      for (int i = 0; i < kMB; ++i) {
        if (FULL || i < nb) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr (PDT_STEM_PROBE == 2) acc[i][j] += f4{(float)av[i][j], (float)bw[j][i], 0.f, 0.f};
            else acc[i][j] = mfma(bw[j], av[i], acc[i][j]);
          }
        }
      }
    }

    // next window -> registers, issued before this tile's stores: the loads land while the stores
    // drain (issued earlier, it made the compiler wait for the previous tile's stores — which
    // share vmcnt and whose data registers the loads reuse — before the MFMAs)
    if (PDT_STEM_PROBE != 3 && k + 1 < cnt) {
      int n1, oh1, ow1;
      coords(t + 1, n1, oh1, ow1);
      load_window(wv, X, tid, n1, 2 * oh1 - 3, 2 * ow1 - 8, H, W);
    }

    // ---- epilogue: lane = pixel pl of each block, channels 16j + 4g .. +3 -> the wave's LDS
    // staging block [16 px][64 ch] -> 16-B pieces, each store instruction 1 KB contiguous of Y
    const int oh = oh0 + wid;
    if (oh < OH) {
      uint16_t* yrow = Y + ((int64_t)(n * OH + oh) * OW + ow0) * kCo;
#pragma unroll
      for (int i = 0; i < kMB; ++i) {
        if (FULL || i < nb) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f4 v = acc[i][j];
            *reinterpret_cast<uint2*>(stage + pl * kStPitch + j * 32 + g * 8) =
                make_uint2(pk2(v[0], v[1]), pk2(v[2], v[3]));
          }
          if constexpr (STATS) {  // the wave's own staging writes above complete in order first
            pdt_f2 sk, ss, sq;
            if (!kset) {
              const uint32_t kw = *reinterpret_cast<const uint32_t*>(stage + (lane & 31) * 4);
              sk = pdt_f2{__uint_as_float(kw << 16), __uint_as_float(kw & 0xffff0000u)};
              ss = sq = pdt_f2{0.f, 0.f};
              kset = true;
            } else {
              sk = sst[0]; ss = sst[1]; sq = sst[2];
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const uint32_t w = *reinterpret_cast<const uint32_t*>(srd + r * kStPitch);
              const pdt_f2 d = pdt_f2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)} - sk;
              ss += d;
              sq = d * d + sq;
            }
            sst[0] = sk; sst[1] = ss; sst[2] = sq;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {  // the wave's own LDS writes above complete in order first
            const int idx = lane + 64 * h, px = idx >> 3, c = idx & 7;
            const uint4 pv = *reinterpret_cast<const uint4*>(stage + px * kStPitch + c * 16);
            if (PDT_STEM_PROBE == 1 && pv.x != 12345u) continue;
            *reinterpret_cast<uint4*>(yrow + (int64_t)(i * 16 + px) * kCo + c * 8) = pv;
          }
        }
      }
      nrows += OW;
    }
    if (PDT_STEM_PROBE != 3 && k + 1 < cnt) {
      __syncthreads();  // every wave is done reading window k
      store_window(wv, lds, tid);
    }
  }
  if constexpr (STATS) {  // partial p = (workgroup, wave): S = n K + sum (y - K), M2 = sum (y - K)^2 - sum (y - K)^2 / n
    pdt_f2 sk = pdt_f2{0.f, 0.f}, ss = sk, sq = sk;
    if (kset) { sk = sst[0]; ss = sst[1]; sq = sst[2]; }
    ss = pdt_f2{xor_add<32>(ss.x), xor_add<32>(ss.y)};
    sq = pdt_f2{xor_add<32>(sq.x), xor_add<32>(sq.y)};
    if (lane < 32) {
      const int P = gridDim.x * kRowsOut, p = blockIdx.x * kRowsOut + wid;
      const float n = (float)nrows;
      const float inv = nrows > 0 ? 1.f / n : 0.f;
      *reinterpret_cast<float2*>(part + (int64_t)p * kCo + 2 * lane) = make_float2(fmaf(n, sk.x, ss.x), fmaf(n, sk.y, ss.y));
      *reinterpret_cast<float2*>(part + (int64_t)(P + p) * kCo + 2 * lane) =
          make_float2(fmaxf(sq.x - ss.x * ss.x * inv, 0.f), fmaxf(sq.y - ss.y * ss.y * inv, 0.f));
      if (lane == 0) part[(int64_t)2 * P * kCo + p] = n;
    }
  }
}


// ---------------------------------------------------------------- weight gradient
//   dW[co, kh, kw, ci] = sum_px dY[px, co] * X[2 oh + kh - 3, 2 ow + kw - 3, ci]
// MIOpen's kernel took 690 us for it at batch 512 (profiles/r2/steady_resnet50_ours.md); the work
// is a GEMM [64 co] x [224 patch k] over K = 6.4M pixels, HBM-bound on reading dY (822 MB).
// Both operands are pixel-major in memory and need pixels along the MFMA k dimension: fragments
// come from transposed LDS reads (ds_read_b64_tr_b16: each lane names one pixel row, the 16 lanes
// of a group receive one column of 4 pixels), as in conv3x3.hip's weight gradient.
//   * tile = 2 output rows of one image (2 x OW <= 224 pixels = up to 7 k-steps of 32), 512
//     threads: wave = k half (patch blocks 0-6 | 7-13) x pixel group (k-steps j with
//     (j + tile) % 4 == group), 4 co blocks x 7 patch blocks = 28 accumulators;
//   * dY tile (contiguous in NHWC: 2 full rows) arrives by LDS-DMA into a double buffer, rows
//     XOR-swizzled on 16-B chunks by ((row >> 1) & 3) << 1 through the SOURCE address so the
//     transposed reads of 8 consecutive rows hit distinct banks; the X window (9 rows, 3 -> 4
//     channels) goes through registers like the forward's; one barrier per tile;
//   * persistent, 1 workgroup per CU; the 4 pixel groups are summed through LDS at the end and
//     each workgroup writes one fp32 partial, summed in a fixed order by stem_wgrad_reduce_kernel.
//   * BNA: the stem BatchNorm's backward apply happens on the way in. dY is then the gradient at
//     the BN output (the max-pool gradient dz) and Xb the BN input: both tiles arrive by LDS-DMA
//     and one in-place pass turns them into dx = A dz + B (xb - mean) + D (the formula and the bf16
//     rounding of bn_bwd_apply_kernel), so the BN's dx — written and re-read once each by the
//     separate apply pass — never exists in HBM.
constexpr int kGThreads = 512;
constexpr int kGRowsOut = 2;
constexpr int kGInRows = 2 * kGRowsOut + 5;  // 9
// window column c <-> input column c - 4 (232 columns): input pixel PAIRS (12 B, 4-B aligned at an
// even input column) go to 16-B aligned LDS pairs, so consecutive lanes write consecutive 16 B
// (8 pixels per lane, 64 B apart across lanes, cost 16-way bank conflicts: 47% of LDS cycles)
constexpr int kGCols = 232;
constexpr int kGInPitch = kGCols * 8;  // unpadded: a patch half (4 pixels) is 32 contiguous B
constexpr int kGMaxPx = kGRowsOut * kTW;     // 224
constexpr int kGDy = kGMaxPx * 128;          // dY tile [224 px][64 co] bf16
constexpr int kGBuf = kGDy + kGInRows * kGInPitch;
constexpr int kGLds = 2 * kGBuf;             // 90,752 B
constexpr int kGBufB = kGBuf + kGDy;         // BNA: + the BN input tile
constexpr int kGLdsB = 2 * kGBufB + 4 * 64 * 4;  // + the coefficient table A, B, D, mean: 148,864 B
constexpr int kGK = 7 * 32;                  // padded patch length (kh x kw 8 x ci 4)
constexpr int kGPairs = kGCols / 2;
constexpr int kGItems = kGInRows * kGPairs;  // 1,044 pixel pairs per window
constexpr int kGRounds = (kGItems + kGThreads - 1) / kGThreads;

__device__ __attribute__((aligned(256))) uint4 g_stem_zero[8];  // zero page for DMA of rows past OH

// LDS-DMA (global_load_lds_dwordx4: lane i's 16 B land at M0 + 16 i) issued from inline asm: the
// builtin form makes the compiler assume the DMA may alias every later LDS read and put a
// vmcnt(0) in front of the next tile's fragment reads — i.e. wait for the prefetch it was meant
// to overlap. Ordering is by the kernel's own counted vmcnt waits and barriers instead.
__device__ __forceinline__ void dma16_opaque(const void* src, const char* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory");
}

// The stem BatchNorm's backward apply dx = A dz + B (x - mean) + D, unfused (no contraction): the
// dz-tile and pooled-gradient forms of the weight gradient evaluate it identically, bit for bit.
__device__ __forceinline__ float bn_apply_dx(float a, float g, float b, float x, float m, float d) {
#pragma clang fp contract(off)
  return a * g + b * (x - m) + d;
}

typedef short s4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 tr8(const char* p0, const char* p1) {
  const s4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)p0);
  const s4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)p1);
  typedef short s8 __attribute__((ext_vector_type(8)));
  const s8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

#ifndef PDT_STEM_WG_PROBE
#define PDT_STEM_WG_PROBE 0  // diagnostics only: 1 = staging without compute, 2 = compute without staging
#endif
// POOL (with BNA): dY is the gradient at the MAX-POOL output [N, PH, PW, 64] with its winner codes
// `pcode` (bn_apply_pool_kernel), not the pool's input gradient: each tile DMAs the two pooled rows its
// two stem rows fall in (dy + codes, 21 KB in place of the 28 KB dz tile) and forms dz per position in
// the apply pass with maxpool_bwd2_kernel's window order and bf16 rounding — so the stem's dz (1.6 GB
// at 1024 images) is neither written by the pool gradient nor read back here.
template <bool BNA, bool POOL = false>
__global__ __launch_bounds__(kGThreads, 1) void stem_wgrad_kernel(const uint16_t* __restrict__ X,
                                                                  const uint16_t* __restrict__ dY,
                                                                  float* __restrict__ ws, int H, int W, int OH,
                                                                  int OW, int nrt, int ntiles,
                                                                  const uint16_t* __restrict__ Xb = nullptr,
                                                                  const float* __restrict__ coef = nullptr,
                                                                  const float* __restrict__ mean = nullptr,
                                                                  const uint8_t* __restrict__ pcode = nullptr) {
  static_assert(!POOL || BNA, "the pooled form is the fused BN apply's");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int kBuf = BNA ? kGBufB : kGBuf;
  float* const ctab = reinterpret_cast<float*>(lds + 2 * kGBufB);  // BNA: [A | B | D | mean][64]
  if (BNA && threadIdx.x < 64) {
    const int c = threadIdx.x;
    ctab[c] = coef[c];
    ctab[64 + c] = coef[64 + c];
    ctab[128 + c] = coef[128 + c];
    ctab[192 + c] = mean[c];
  }
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int per = ntiles / gridDim.x, rem = ntiles % gridDim.x;
  const int t0 = blockIdx.x * per + min((int)blockIdx.x, rem);
  const int cnt = per + ((int)blockIdx.x < rem ? 1 : 0);
  const int P = kGRowsOut * OW;  // pixels per tile (multiple of 32)
  const int nks = P >> 5;

  // ---- staging: dY tile by DMA (P/8 instructions of 8 rows; instruction q by wave q % 8)
  auto dma_tile = [&](const uint16_t* base, int t, char* buf) {
    const int n = t / nrt, oh0 = (t - n * nrt) * kGRowsOut;
    const uint16_t* src0 = base + (int64_t)(n * OH + oh0) * OW * 64;
    const int vrows = min(kGRowsOut, OH - oh0) * OW;  // valid pixel rows of the tile
    for (int q = wid; q < (P >> 3); q += 8) {
      const int r = q * 8 + (lane >> 3), pos = lane & 7;
      const int chunk = pos ^ (((r >> 1) & 3) << 1);
      const void* src = r < vrows ? (const void*)(src0 + (int64_t)r * 64 + chunk * 8) : (const void*)g_stem_zero;
      dma16_opaque(src, buf + q * 1024);
    }
  };
  const int PH = (OH - 1) / 2 + 1, PW = (OW - 1) / 2 + 1;
  // POOL: pooled rows a = oh0 / 2 and min(a + 1, PH - 1): dy at [0, 2 PW * 128), codes after it
  auto dma_pooled = [&](int t, char* buf) {
    const int n = t / nrt, a = (t - n * nrt) * kGRowsOut / 2;
    const int a1 = min(a + 1, PH - 1);
    const int npx = 2 * PW;
    for (int q = wid; q < (npx + 7) / 8; q += 8) {  // dy: 8 pooled pixels (128 B each) per instruction
      const int px = q * 8 + (lane >> 3), pos = lane & 7;
      const int pr = px >= PW, pc = px - pr * PW;
      const void* src = px < npx ? (const void*)(dY + ((int64_t)(n * PH + (pr ? a1 : a)) * PW + pc) * 64 + pos * 8)
                                 : (const void*)g_stem_zero;
      dma16_opaque(src, buf + q * 1024);
    }
    char* cbuf = buf + npx * 128;
    for (int q = wid; q < (npx + 15) / 16; q += 8) {  // codes: 16 pooled pixels (64 B each) per instruction
      const int px = q * 16 + (lane >> 2), pos = lane & 3;
      const int pr = px >= PW, pc = px - pr * PW;
      const void* src = px < npx ? (const void*)(pcode + ((int64_t)(n * PH + (pr ? a1 : a)) * PW + pc) * 64 + pos * 16)
                                 : (const void*)g_stem_zero;
      dma16_opaque(src, cbuf + q * 1024);
    }
  };
  auto dma_dy = [&](int t, char* buf) {
    if constexpr (POOL) dma_pooled(t, buf);
    else dma_tile(dY, t, buf);
    if (BNA) dma_tile(Xb, t, buf + kGBuf);
  };
  // BNA: dz tile (buf) and BN input tile (buf + kGBuf), same swizzled layout -> dx in place of dz.
  // Thread: channel chunk tid % 8 (its 8 coefficients), rows tid / 8 + 64 u; LDS position of its
  // chunk in row r = chunk ^ swizzle(r). Rows past the tile's valid pixels stay zero.
  // POOL: dz of tile pixel r (stem row oh0 + r / OW, column r % OW), channels cc*8 .. +7, from the pooled
  // rows in LDS: windows (A + dr, B + ds) in maxpool_bwd2_kernel's order, rounded to bf16 as it writes dz
  auto pooled_dz = [&](const char* buf, int oh0, int r, int cc, float (&g)[8]) {
    const int ih = oh0 + r / OW, iw = r % OW;
    const int A = ih >> 1, rr = ih & 1, B = iw >> 1, sc = iw & 1;
    const int A1 = min(PH - 1, A + 1), B1 = min(PW - 1, B + 1);
    const int a = oh0 >> 1;  // pooled row of LDS row 0
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dr = q >> 1, ds = q & 1;
      if ((dr && !rr) || (ds && !sc)) continue;
      if ((dr && A1 == A) || (ds && B1 == B)) continue;
      const int po = (dr ? A1 : A) - a, pc = ds ? B1 : B;
      const uint32_t idx = (uint32_t)((dr ? 0 : rr + 1) * 3 + (ds ? 0 : sc + 1));
      const uint4 dv = *reinterpret_cast<const uint4*>(buf + (po * PW + pc) * 128 + cc * 16);
      const uint2 cw = *reinterpret_cast<const uint2*>(buf + 2 * PW * 128 + (po * PW + pc) * 64 + cc * 8);
      const uint32_t w[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = __uint_as_float(j & 1 ? (w[j >> 1] & 0xffff0000u) : (w[j >> 1] << 16));
        const uint32_t cj = ((j < 4 ? cw.x : cw.y) >> (8 * (j & 3))) & 0xffu;
        g[j] += cj == idx ? v : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = bf2f(f2bf(g[j]));
  };
  auto bn_apply_tile = [&](int t, char* buf) {
    const int n = t / nrt, oh0 = (t - n * nrt) * kGRowsOut;
    const int vrows = min(kGRowsOut, OH - oh0) * OW;
    if constexpr (POOL) {
      // every thread's rows first (the pooled data lies where the results go), then one barrier
      int tix;
      asm volatile("v_mov_b32 %0, %1" : "=v"(tix) : "v"((int)threadIdx.x));
      const int cc = tix & 7;
      constexpr int kU = (kGMaxPx + 63) / 64;
      uint4 res[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int r = (tix >> 3) + 64 * u;
        float o[8];
        if (r < vrows) {
          float g[8], xf[8];
          pooled_dz(buf, oh0, r, cc, g);
          const char* px = buf + kGBuf + r * 128 + ((cc ^ (((r >> 1) & 3) << 1)) * 16);
          ld8_bf16(reinterpret_cast<const uint16_t*>(px), xf);
          // the dz-tile path's coefficient loads and formula (bn_apply_dx: bit-identical)
          float av[8], bv[8], dv[8], mv[8];
          const float4* ct = reinterpret_cast<const float4*>(ctab + cc * 8);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float4 a4 = ct[h], b4 = ct[16 + h], d4 = ct[32 + h], m4 = ct[48 + h];
            av[4 * h] = a4.x; av[4 * h + 1] = a4.y; av[4 * h + 2] = a4.z; av[4 * h + 3] = a4.w;
            bv[4 * h] = b4.x; bv[4 * h + 1] = b4.y; bv[4 * h + 2] = b4.z; bv[4 * h + 3] = b4.w;
            dv[4 * h] = d4.x; dv[4 * h + 1] = d4.y; dv[4 * h + 2] = d4.z; dv[4 * h + 3] = d4.w;
            mv[4 * h] = m4.x; mv[4 * h + 1] = m4.y; mv[4 * h + 2] = m4.z; mv[4 * h + 3] = m4.w;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = bn_apply_dx(av[j], g[j], bv[j], xf[j], mv[j], dv[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = 0.f;
        }
        res[u].x = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
        res[u].y = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
        res[u].z = (uint32_t)f2bf(o[4]) | ((uint32_t)f2bf(o[5]) << 16);
        res[u].w = (uint32_t)f2bf(o[6]) | ((uint32_t)f2bf(o[7]) << 16);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int r = (tix >> 3) + 64 * u;
        if (r < P) *reinterpret_cast<uint4*>(buf + r * 128 + ((cc ^ (((r >> 1) & 3) << 1)) * 16)) = res[u];
      }
      return;
    }
    // one row at a time, coefficients re-read from LDS per row, and the thread index passed through
    // an opaque move so its derived addresses are not hoisted out of the tile loop: this kernel's
    // compute phase already holds 256 VGPRs, so nothing of the apply may stay live across it
    int tix;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tix) : "v"((int)threadIdx.x));
    const int cc = tix & 7;
#pragma unroll 1
    for (int u = 0; u < (kGMaxPx + 63) / 64; ++u) {
      const int r = (tix >> 3) + 64 * u;
      if (r >= P) break;
      char* pz = buf + r * 128 + ((cc ^ (((r >> 1) & 3) << 1)) * 16);
      float o[8];
      if (r < vrows) {
        float g[8], xf[8], av[8], bv[8], dv[8], mv[8];
        ld8_bf16(reinterpret_cast<const uint16_t*>(pz), g);
        ld8_bf16(reinterpret_cast<const uint16_t*>(pz + kGBuf), xf);
        const float4* ct = reinterpret_cast<const float4*>(ctab + cc * 8);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 a4 = ct[h], b4 = ct[16 + h], d4 = ct[32 + h], m4 = ct[48 + h];
          av[4 * h] = a4.x; av[4 * h + 1] = a4.y; av[4 * h + 2] = a4.z; av[4 * h + 3] = a4.w;
          bv[4 * h] = b4.x; bv[4 * h + 1] = b4.y; bv[4 * h + 2] = b4.z; bv[4 * h + 3] = b4.w;
          dv[4 * h] = d4.x; dv[4 * h + 1] = d4.y; dv[4 * h + 2] = d4.z; dv[4 * h + 3] = d4.w;
          mv[4 * h] = m4.x; mv[4 * h + 1] = m4.y; mv[4 * h + 2] = m4.z; mv[4 * h + 3] = m4.w;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = bn_apply_dx(av[j], g[j], bv[j], xf[j], mv[j], dv[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = 0.f;
      }
      st8_bf16(reinterpret_cast<uint16_t*>(pz), o);
    }
  };
  uint3 xv[kGRounds];
  bool xok[kGRounds];
  auto load_x = [&](int t) {
    const int n = t / nrt, oh0 = (t - n * nrt) * kGRowsOut;
#pragma unroll
    for (int u = 0; u < kGRounds; ++u) {
      const int i = tid + u * kGThreads;
      const int r = i / kGPairs, pp = i - r * kGPairs;
      const int ih = 2 * oh0 - 3 + r, iw = 2 * pp - 4;  // even: a pair is all in or all out of the image
      // clamped address, zeroed in store_x (the select here would wait for the load at once)
      const bool ok = i < kGItems && ih >= 0 && ih < H && iw >= 0 && iw < W;
      xv[u] = *reinterpret_cast<const uint3*>(X + (ok ? ((int64_t)(n * H + ih) * W + iw) * 3 : 0));
      xok[u] = ok;
    }
  };
  auto store_x = [&](char* win) {
#pragma unroll
    for (int u = 0; u < kGRounds; ++u) {
      const int i = tid + u * kGThreads;
      if (i >= kGItems) continue;
      const int r = i / kGPairs, pp = i - r * kGPairs;
      // (c0 c1 c2)(c0 c1 c2) -> (c0 c1 c2 0)(c0 c1 c2 0)
      const uint3 w = xok[u] ? xv[u] : make_uint3(0u, 0u, 0u);
      *reinterpret_cast<uint4*>(win + r * kGInPitch + pp * 16) =
          make_uint4(w.x, w.y & 0xffffu, (w.y >> 16) | (w.z << 16), w.z >> 16);
    }
  };

  // ---- per-lane fragment geometry: lane group g, row-in-group rsub, 8-B column piece csub
  const int g = lane >> 4, li = lane & 15, rsub = li >> 2, csub = li & 3;
  const int khalf = wid & 1, pgrp = wid >> 1;
  const int sw = (((4 * g + rsub) >> 1) & 3) << 1;  // the dY swizzle of rows 4g + rsub (+16, +32k)
  int dyo[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) dyo[cb] = (((2 * cb) ^ sw) | (csub >> 1)) * 16 + (csub & 1) * 8;

  f4 acc[4][7];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int b = 0; b < 7; ++b) acc[cb][b] = f4{0.f, 0.f, 0.f, 0.f};

  // 2 buffers. Iteration k: load tile k+1's window into registers and DMA its dY (opaque: see
  // dma16_opaque), compute tile k, write the window registers (the compiler's wait for them also
  // retires the DMA issued after them), barrier.
  if (cnt > 0) {
    load_x(t0);
    dma_dy(t0, lds);
    store_x(lds + kGDy);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int k = 0; k < cnt; ++k) {
    char* const buf = lds + (k & 1) * kBuf;
    char* const nbuf = lds + ((k + 1) & 1) * kBuf;
    if (BNA) {  // this tile's DMA landed before the last barrier; the next tile's goes to nbuf
      if (k + 1 < cnt) dma_dy(t0 + k + 1, nbuf);
      bn_apply_tile(t0 + k, buf);
      __syncthreads();
      if (k + 1 < cnt) load_x(t0 + k + 1);  // after the apply: its registers are not live across it
    } else if (PDT_STEM_WG_PROBE != 2 && k + 1 < cnt) {
      load_x(t0 + k + 1);
      dma_dy(t0 + k + 1, nbuf);
    }
    const char* win = buf + kGDy;
    // this wave's k-steps of the tile: j0 and j0 + 4 (7 k-steps over 4 pixel groups); both
    // steps' fragments are read before the first MFMA so the second batch of reads overlaps it
    const int j0 = (pgrp - (t0 + k)) & 3;
    const int nj = PDT_STEM_WG_PROBE == 1 ? 0 : (j0 < nks) + (j0 + 4 < nks);
    auto frags = [&](int u, bf16x8 (&au)[4], bf16x8 (&bu)[7]) {
      const int r0 = (j0 + 4 * u) * 32 + 4 * g + rsub, r1 = r0 + 16;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) au[cb] = tr8(buf + r0 * 128 + dyo[cb], buf + r1 * 128 + dyo[cb]);
      // window address of pixel r: row 2 (r >= OW), column 2 (r mod OW) + 1, plus this lane's piece
      const int h0 = r0 >= OW, h1 = r1 >= OW;
      const char* x0 = win + 2 * h0 * kGInPitch + (2 * (r0 - h0 * OW) + csub + 1) * 8;
      const char* x1 = win + 2 * h1 * kGInPitch + (2 * (r1 - h1 * OW) + csub + 1) * 8;
#pragma unroll
      for (int b = 0; b < 7; ++b) {
        const int kb = 7 * khalf + b;
        const int off = (kb >> 1) * kGInPitch + (kb & 1) * 32;
        bu[b] = tr8(x0 + off, x1 + off);
      }
    };
    if constexpr (BNA) {  // one k-step's fragments at a time: 44 fewer live VGPRs (no spills)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u < nj) {
          bf16x8 a[4], bx[7];
          frags(u, a, bx);
#pragma unroll
          for (int b = 0; b < 7; ++b)
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) acc[cb][b] = mfma(a[cb], bx[b], acc[cb][b]);
        }
      }
    } else {
      bf16x8 a[2][4], bx[2][7];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (u < nj) frags(u, a[u], bx[u]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u < nj) {
#pragma unroll
          for (int b = 0; b < 7; ++b)
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) acc[cb][b] = mfma(a[u][cb], bx[u][b], acc[cb][b]);  // D[co][patch k]
        }
      }
    }
    if (PDT_STEM_WG_PROBE != 2 && k + 1 < cnt) store_x(nbuf + kGDy);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile k + 1 landed everywhere; everyone is done with tile k's buffer
  }

  // ---- pixel groups 1..3 -> LDS -> group 0 adds (one patch block column per round)
  f4* red = reinterpret_cast<f4*>(lds);
#pragma unroll
  for (int b = 0; b < 7; ++b) {
    if (pgrp != 0) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) red[(((pgrp - 1) * 2 + khalf) * 4 + cb) * 64 + lane] = acc[cb][b];
    }
    __syncthreads();
    if (pgrp == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb][b] += red[((q * 2 + khalf) * 4 + cb) * 64 + lane];
    }
    __syncthreads();
  }
  if (pgrp != 0) return;
  // partial [64 co][224 k]: lane holds D[co = 16 cb + 4 g + t][k = 16 kb + li]
  float* wp = ws + (int64_t)blockIdx.x * 64 * kGK;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int b = 0; b < 7; ++b)
#pragma unroll
      for (int t = 0; t < 4; ++t) wp[(cb * 16 + 4 * g + t) * kGK + (7 * khalf + b) * 16 + li] = acc[cb][b][t];
}

// dw[co][kh][kw][ci] (bf16, the channels_last storage of [64, 3, 7, 7]) = sum of the partials in
// workgroup order (deterministic), dropping the padded tap kw = 7 and channel ci = 3. Block b
// sums columns [256 b, 256 b + 256) of the [64 x 224] partials: 4 partial subsets x 256 columns,
// loads issued 16 at a time (a thread-per-column loop over 256 partials took 62 us in the step).
__global__ __launch_bounds__(1024) void stem_wgrad_reduce_kernel(const float* __restrict__ ws, int nparts,
                                                                 uint16_t* __restrict__ dw) {
  __shared__ float sm[4][256];
  const int tid = threadIdx.x, c = tid & 255, q = tid >> 8;
  const int col = blockIdx.x * 256 + c;  // < 64 * 224 (grid = 56)
  float a = 0.f;
  for (int p0 = q; p0 < nparts; p0 += 4 * 16) {
    float t[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int p = p0 + 4 * u;
      t[u] = ws[(int64_t)(p < nparts ? p : q) * 64 * kGK + col];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) a += (p0 + 4 * u < nparts) ? t[u] : 0.f;
  }
  sm[q][c] = a;
  __syncthreads();
  if (q != 0) return;
  const float s = sm[0][c] + sm[1][c] + sm[2][c] + sm[3][c];
  const int co = col / kGK, k = col - co * kGK, kh = k >> 5, kw = (k >> 2) & 7, ci = k & 3;
  if (kw < 7 && ci < 3) dw[co * 147 + kh * 21 + kw * 3 + ci] = __builtin_bit_cast(uint16_t, (__bf16)s);
}

}  // namespace

static int stem_ncu();

extern "C" int64_t pdt_stem_conv_wprep_elems() { return kWPrepElems; }

// y[N, 64, OH, OW] (channels_last) = conv2d(x[N, 3, H, W] (channels_last), w[64, 3, 7, 7]
// (channels_last storage [64][7][7][3]), stride 2, padding 3); wp: kWPrepElems bf16 scratch.
extern "C" int pdt_stem_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* wp, uint16_t* y, int N, int H,
                                 int W, hipStream_t s) {
  if (N < 1 || H < 1 || W < 32 || W % 32 != 0) return -1;
  const int OH = (H - 1) / 2 + 1, OW = W / 2;
  static const bool attr_ok =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_conv_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_conv_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess;
  if (!attr_ok) return -2;
  const int ncu = stem_ncu();
  const int nrt = (OH + kRowsOut - 1) / kRowsOut, nct = (OW + kTW - 1) / kTW;
  const int64_t ntiles = (int64_t)N * nrt * nct;
  if (ntiles > 0x7fffffff || (int64_t)N * H > 0x7fffffff / 4) return -3;
  const int grid = (int)std::min<int64_t>(ntiles, 2 * ncu);  // 2 workgroups (61.4 KB LDS each) per CU: out of phase
  hipLaunchKernelGGL(stem_wprep_kernel, dim3((kWPrepElems + 255) / 256), dim3(256), 0, s, w, wp);
  if (OW % kTW == 0)
    hipLaunchKernelGGL(stem_conv_kernel<true>, dim3(grid), dim3(kThreads), kLds, s, x, wp, y, H, W, OH, OW, nrt, nct,
                       (int)ntiles, nullptr);
  else
    hipLaunchKernelGGL(stem_conv_kernel<false>, dim3(grid), dim3(kThreads), kLds, s, x, wp, y, H, W, OH, OW, nrt, nct,
                       (int)ntiles, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Partials written by pdt_stem_conv_fwd_stats for an [N, 3, H, W] input: 0 when it does not apply
// (it needs OW == 112, i.e. W == 224 — the ImageNet stem).
extern "C" int64_t pdt_stem_stats_parts(int N, int H, int W) {
  if (N < 1 || H < 1 || W / 2 != kTW || W % 32 != 0) return 0;
  const int OH = (H - 1) / 2 + 1;
  const int64_t ntiles = (int64_t)N * ((OH + kRowsOut - 1) / kRowsOut);
  return std::min<int64_t>(ntiles, 2 * stem_ncu()) * kRowsOut;
}

// pdt_stem_conv_fwd plus the BatchNorm statistics of y in the epilogue, so the stem's BatchNorm never
// reads y for them (that reduce pass over the 1.6 GB stem output took 320 us of a 1024-image step):
// each wave reads back the 16 x 64 block it just staged in LDS (the bf16 values stored) and keeps
// shifted sums of its channel pair over every row it owns; at the end it writes one partial.
// part (floats, P = pdt_stem_stats_parts): [P][64] sums S_p, [P][64] centred M2_p, [P] row counts n_p
// — consumed by pdt_bn_relu_maxpool_fwd_train_parts. (A first statistics epilogue with Chan merges of
// per-lane accumulators spilled; this one keeps 6 VGPRs across tiles.)
extern "C" int pdt_stem_conv_fwd_stats(const uint16_t* x, const uint16_t* w, uint16_t* wp, uint16_t* y, float* part,
                                       int N, int H, int W, hipStream_t s) {
  const int64_t P = pdt_stem_stats_parts(N, H, W);
  if (P == 0) return -1;
  static const bool attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_conv_kernel<true, true>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, kLdsStats) == hipSuccess;
  if (!attr_ok) return -2;
  const int OH = (H - 1) / 2 + 1, OW = W / 2;
  const int nrt = (OH + kRowsOut - 1) / kRowsOut, nct = 1;
  const int64_t ntiles = (int64_t)N * nrt;
  if (ntiles > 0x7fffffff || (int64_t)N * H > 0x7fffffff / 4) return -3;
  const int grid = (int)(P / kRowsOut);
  hipLaunchKernelGGL(stem_wprep_kernel, dim3((kWPrepElems + 255) / 256), dim3(256), 0, s, w, wp);
  hipLaunchKernelGGL((stem_conv_kernel<true, true>), dim3(grid), dim3(kThreads), kLdsStats, s, x, wp, y, H, W, OH, OW, nrt,
                     nct, (int)ntiles, part);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

static int stem_ncu() {
  static const int ncu = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }();
  return ncu;
}

// fp32 workspace floats for pdt_stem_conv_wgrad (one [64][224] partial per workgroup).
extern "C" int64_t pdt_stem_wgrad_ws_floats() { return (int64_t)stem_ncu() * 64 * kGK; }

namespace {
int stem_wgrad_launch(const uint16_t* x, const uint16_t* dy, const uint16_t* xb, const float* coef, const float* mean,
                      uint16_t* dw, float* ws, int N, int H, int W, hipStream_t s, const uint8_t* pcode = nullptr) {
  if (N < 1 || H < 1 || W < 32 || W % 32 != 0 || W > 2 * kTW) return -1;
  const int OH = (H - 1) / 2 + 1, OW = W / 2;
  static const bool attr_ok =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kGLds) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kGLdsB) == hipSuccess &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_wgrad_kernel<true, true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kGLdsB) == hipSuccess;
  if (!attr_ok) return -2;
  const int nrt = (OH + kGRowsOut - 1) / kGRowsOut;
  const int64_t ntiles = (int64_t)N * nrt;
  if (ntiles > 0x7fffffff || (int64_t)N * OH * OW * 64 > 0x7fffffffLL * 4) return -3;
  const int grid = (int)std::min<int64_t>(ntiles, stem_ncu());
  // (POOL: the two pooled rows of a tile, dy + codes = 2 PW x 192 B, fit the 28 KB dz-tile space)
  static_assert(2 * ((kTW + 1) / 2) * 192 <= kGDy, "pooled rows in the dz tile's space");
  if (xb && pcode)
    hipLaunchKernelGGL((stem_wgrad_kernel<true, true>), dim3(grid), dim3(kGThreads), kGLdsB, s, x, dy, ws, H, W, OH,
                       OW, nrt, (int)ntiles, xb, coef, mean, pcode);
  else if (xb)
    hipLaunchKernelGGL(stem_wgrad_kernel<true>, dim3(grid), dim3(kGThreads), kGLdsB, s, x, dy, ws, H, W, OH, OW, nrt,
                       (int)ntiles, xb, coef, mean);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<false>, dim3(grid), dim3(kGThreads), kGLds, s, x, dy, ws, H, W, OH, OW, nrt,
                       (int)ntiles, nullptr, nullptr, nullptr);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(64 * kGK / 256), dim3(1024), 0, s, ws, grid, dw);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
}  // namespace

// dw [64, 3, 7, 7] (channels_last storage [64][7][7][3], bf16) of the stem conv from x [N, 3, H, W]
// and dy [N, 64, OH, OW] (both channels_last). Requires W % 32 == 0 and W <= 224 (OW <= 112).
extern "C" int pdt_stem_conv_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H,
                                   int W, hipStream_t s) {
  return stem_wgrad_launch(x, dy, nullptr, nullptr, nullptr, dw, ws, N, H, W, s);
}

// Same, with the stem BatchNorm's backward apply fused into the dY load: dz [N, 64, OH, OW] is the
// gradient at the BN output, xb the BN input (the stem conv output), coef [3][64] = A, B, D and mean
// [64] as bn_bwd_apply_kernel takes them; the conv's dY = A dz + B (xb - mean) + D (bf16).
extern "C" int pdt_stem_conv_wgrad_bn(const uint16_t* x, const uint16_t* dz, const uint16_t* xb, const float* coef,
                                      const float* mean, uint16_t* dw, float* ws, int N, int H, int W, hipStream_t s) {
  if (!xb || !coef || !mean) return -1;
  return stem_wgrad_launch(x, dz, xb, coef, mean, dw, ws, N, H, W, s);
}

// Same from the gradient at the MAX-POOL output: dyp [N, 64, PH, PW] and the pool's winner codes
// (bn_apply_pool_kernel, 1 byte per (pooled position, channel)); the pool's input gradient dz is formed
// per tile in LDS (pdt_maxpool3s2_bwd_bn_coef with dz = null gives coef without writing it).
extern "C" int pdt_stem_conv_wgrad_bn_pool(const uint16_t* x, const uint16_t* dyp, const uint8_t* code,
                                           const uint16_t* xb, const float* coef, const float* mean, uint16_t* dw,
                                           float* ws, int N, int H, int W, hipStream_t s) {
  if (!xb || !coef || !mean || !code) return -1;
  return stem_wgrad_launch(x, dyp, xb, coef, mean, dw, ws, N, H, W, s, code);
}
