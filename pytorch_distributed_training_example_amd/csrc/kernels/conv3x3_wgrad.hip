// Weight gradient of the stride-1 / pad-1 3x3 convolution on MFMA (gfx950), NHWC bf16, fp32 accumulate:
//
//   dW[co, tap, ci] = sum_m dY[m, co] * X[pixel(m) + shift(tap), ci]      (m = (n, oh, ow), 9 taps)
//
// Not in the reference (LeNet's convs are 5x5 on cuDNN, /root/reference/cnn.py:10-16). Replaces
// MIOpen's igemm_wrw kernels on ResNet-50's 13 stride-1 3x3 convs (~8 ms/step at 1024/GPU with
// their zero-fill / cast passes, profiles/r2/steady_resnet50_b1024_ours.md) and its algorithm
// search (most of the 124 s fresh-box first step).
//
// GEMM view: M = Co, N = 9 x Ci, K = pixels. Both operands are pixel-major in NHWC (channels
// contiguous), i.e. K-strided: fragments come from LDS through the hardware transposed read
// ds_read_b64_tr_b16 (a 16-lane group reads 4 pixel rows x 16 channels and each lane receives one
// channel's 4 pixels) — no transpose pass.
//
// Structure:
//   * a workgroup owns CO_T (64 | 128) output channels x 64 input channels x all 9 taps and a
//     contiguous range of pixel tiles (split-K over pixels; fp32 partials per split, summed in a
//     fixed order by conv3x3_wgrad_reduce_kernel: deterministic);
//   * a pixel tile is R whole image rows (P = R*W ~ 112 pixels, K padded to 16 with zero dY rows);
//     its input operand is staged ONCE as the padded halo of those rows (R+2 padded rows per image
//     touched, W+2 pixels each, pad rows/columns zero) and the nine taps read shifted rows of it:
//     halo row of (pixel j, tap kh,kw) = table[j] + kh*(W+2) + kw. Every input pixel crosses
//     L2 -> LDS ~1.5x instead of 9x;
//   * waves split the block 32 (co) x 32 (ci): 9 v_mfma_f32_32x32x16_bf16 accumulators (144 VGPRs)
//     per wave; per 16-pixel k-step 2 transposed reads of dY (reused by the 9 taps) + 2 per tap of
//     X: 20 reads per 9 MFMAs (~55 % of the LDS read rate at 2 waves/SIMD);
//   * the next tile's global loads are issued into registers before the current tile's MFMAs
//     (in flight under them) and written to LDS after the compute barrier; 128-B LDS rows with an
//     XOR chunk swizzle keep the 4-row transposed reads conflict-free; 2 workgroups per CU;
//   * block -> (split, channel block) map XCD-aware: all channel blocks of one split (same pixel
//     range: shared dY / X tiles) run on one XCD's L2.
//
// Stride 2 (S = 2, ResNet-50's layer2-4 block-0 conv2; MIOpen's igemm_wrw before): output pixel
// (oh, ow) tap (kh, kw) reads padded input (2 oh + kh, 2 ow + kw). The halo stores each padded input
// row with its columns DE-INTERLEAVED (even columns, then odd ones, HALF = pad4((W_in + 2) / 2)
// each), so consecutive output pixels still read consecutive halo rows (the 4-row transposed reads
// stay conflict-free) and tap (kh, kw) is the row shift kh * 2 HALF + {0, HALF, 1}[kw]. About 4
// input pixels per output pixel are staged (vs ~1.5 at stride 1), so tiles are 2-8 output rows.
#include "../common.h"

using namespace pdt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef short s4v __attribute__((ext_vector_type(4)));

constexpr int kTileTarget = 112;  // pixels per tile (R whole rows)
// K rows (pixels, padded to 16) per tile: 128 at stride 1; 64 at stride 2, whose tiles are halo-
// limited to 2-8 output rows anyway — halving the dY prefetch registers keeps the 8-wave prefetching
// workgroup under 256 VGPRs without spilling
constexpr int kp_max(int S) { return S == 1 ? 128 : 64; }
// halo pixel rows per tile: stride 1 -> 256 (LDS 32 KB; ResNet-50: <= 240); stride 2 -> 320 (R = 2-8
// output rows on ResNet-50: a 640-row halo would need 40 prefetch VGPRs and spill heavily)
constexpr int halo_max(int S) { return S == 1 ? 256 : 320; }

// (An LDS-DMA staging variant — global_load_lds into 1 or 2 LDS buffers, source-swizzled — measured
// 5-11 % SLOWER than the register staging below on every ResNet-50 shape, e.g. 336 vs 302 us at
// 28x28x128, 493 vs 445 us at 56x56x64: the loop is bound by LDS-read latency, not by staging VGPRs.)
// W2T: the halo row pitch W2 (padded pixels per image row) as a compile-time constant (0: runtime), so
// the tap offsets kh * W2 * 128 are ds_read immediates instead of a VALU add per fragment read.
template <int CO_T_, bool PF_, int S_ = 1, int W2T_ = 0>
struct WCfg {
  static constexpr int CO_T = CO_T_, CI_T = 64, S = S_, W2T = W2T_;
  static constexpr int kHaloMax = halo_max(S), kKpMax = kp_max(S);
  static constexpr bool PF = PF_;      // register staging: next tile's loads under this tile's MFMAs
  static constexpr int kWaves = (CO_T / 32) * (CI_T / 32);
  static constexpr int kThreads = kWaves * 64;
  static constexpr int kRowY = CO_T * 2;                 // dY LDS row bytes
  static constexpr int kChY = CO_T / 8;                  // 16-B chunks per dY row
  static constexpr int kDyBytes = kKpMax * kRowY;
  static constexpr int kHaloBytes = kHaloMax * 128;
  static constexpr int kLds = kDyBytes + kHaloBytes + kKpMax * 16;  // table: int4 per pixel
  // prefetch registers (16-B pieces per thread), sized for the worst tile
  static constexpr int kPfY = kKpMax * kChY / kThreads;  // exact: writes never leave the buffers
  static constexpr int kPfX = kHaloMax * 8 / kThreads;
};

// XOR chunk swizzles: 4 consecutive rows of a transposed read land on 4 distinct 64-B bank groups.
__device__ __forceinline__ int swz128(int row, int ch) { return ch ^ (((row >> 1) & 1) << 2); }  // 8 chunks/row
__device__ __forceinline__ int swz256(int row, int ch) { return ch ^ ((row & 3) << 2); }         // 16 chunks/row
template <int ROWB>
__device__ __forceinline__ int chunk_off(int row, int ch) {
  return row * ROWB + ((ROWB == 128 ? swz128(row, ch) : swz256(row, ch)) << 4);
}

__device__ __forceinline__ s4v tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}
__device__ __forceinline__ bf16x8 cat2(s4v a, s4v b) {
  typedef short s8 __attribute__((ext_vector_type(8)));
  s8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

struct Geo {
  int N, H, W, Ci, Co, R, NH, ntiles, tiles_per_split, nsplit, nblk;  // H, W: OUTPUT (= dY) size
  int Hi, Wi;  // input size (= H, W at stride 1)
  int probe;  // diagnostics (wgrad3x3_bench): 1 = staging only, 2 = MFMA only (first tile staged)
};

template <class Cf>
__global__ __launch_bounds__(Cf::kThreads, 2) void conv3x3_wgrad_kernel(const uint16_t* __restrict__ X,
                                                                        const uint16_t* __restrict__ dY,
                                                                        float* __restrict__ ws, Geo g) {
  constexpr int CO_T = Cf::CO_T;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* const dys = lds;
  char* const hal = lds + Cf::kDyBytes;
  int4* const table = reinterpret_cast<int4*>(lds + Cf::kDyBytes + Cf::kHaloBytes);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // halo rows of one padded image row: W + 2 rounded up to a multiple of 4, so the tap offset kh*W2
  // never changes a row's chunk swizzle (it depends on row bit 1); stride 2: two de-interleaved
  // halves of HALF (a multiple of 4) rows
  constexpr int S = Cf::S;
  const int H = g.H, W = g.W, Hi = g.Hi, Wi = g.Wi;
  const int HALF = S == 1 ? 0 : ((Wi + 3) / 2 + 3) & ~3;
  const int W2r = S == 1 ? (W + 2 + 3) & ~3 : 2 * HALF, H2 = Hi + 2;
  const int W2 = Cf::W2T ? Cf::W2T : W2r;  // launch checks W2T == W2r
  const int kwo1 = S == 1 ? 1 : HALF, kwo2 = S == 1 ? 2 : 1;  // row shift of taps kw = 1, 2
  const int nblk_ci = g.Ci / 64;
  // XCD-aware: consecutive logical ids (one split's channel blocks) on one XCD
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / g.nblk, bt = L % g.nblk;
  const int co0 = (bt / nblk_ci) * CO_T, ci0 = (bt % nblk_ci) * 64;
  const int t_begin = split * g.tiles_per_split;
  const int t_end = min(g.ntiles, t_begin + g.tiles_per_split);
  const int P = g.R * W;
  const int KP = (P + 15) & ~15;

  // Staging through registers with raw buffer loads: an out-of-range offset (padding pixel, rows
  // past the tile) returns zeros in hardware, so every load is unconditional and a thread's loads
  // issue back to back (branchy guarded loads made the compiler wait on each one in turn).
  uint4 pfy[Cf::kPfY], pfx[Cf::kPfX];
  int pf_pv = 0, pf_prs = 0, pf_g0 = 0;
  constexpr uint32_t kOob = 0xfffffff0u;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(X), (short)0, (uint32_t)((int64_t)g.N * Hi * Wi * g.Ci * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(dY), (short)0, (uint32_t)((int64_t)g.NH * W * g.Co * 2), 0x00020000);

  auto load_tile = [&](int t) {
    const int g0 = t * g.R, gl = min(g0 + g.R, g.NH) - 1;
    const int pv = (gl - g0 + 1) * W;
    const int prs = (g0 / H) * H2 + S * (g0 % H);      // first halo padded row (tap kh = 0 of row g0)
    const int pre = (gl / H) * H2 + S * (gl % H) + 2;  // last halo padded row (tap kh = 2 of row gl)
    const int nh = (pre - prs + 1) * W2;
    pf_pv = pv; pf_prs = prs; pf_g0 = g0;
    const uint32_t ybase = (uint32_t)g0 * W * g.Co * 2 + co0 * 2;
#pragma unroll
    for (int i = 0; i < Cf::kPfY; ++i) {
      const int c = tid + i * Cf::kThreads, row = c / Cf::kChY, ch = c % Cf::kChY;
      const uint32_t off = row < pv ? ybase + (uint32_t)(row * g.Co + ch * 8) * 2 : kOob;
      pfy[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrs, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < Cf::kPfX; ++i) {
      const int c = tid + i * Cf::kThreads, row = c >> 3, ch = c & 7;
      const int r = row / W2, col = row - r * W2;
      const int pc = S == 1 ? col : (col < HALF ? 2 * col : 2 * (col - HALF) + 1);  // padded input column
      const int pr = prs + r, n = pr / H2, ih = pr - n * H2 - 1, iw = pc - 1;
      const bool ok = row < nh && ih >= 0 && ih < Hi && iw >= 0 && iw < Wi;
      const uint32_t off = ok ? (uint32_t)((((n * Hi + ih) * Wi + iw) * g.Ci + ci0 + ch * 8) * 2) : kOob;
      pfx[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
  };
  // table[j]: for pixel j the halo byte offsets of its tap (0, kw) rows, kw = 0, 1, 2, with the row's
  // XOR swizzle folded in (T(row) = row * 128 | (row & 2) << 5; a lane's read address is T ^ its chunk
  // and half offset): 3 XORs per pixel set and k-step instead of ~5 VALU per swizzled row address
  auto trow = [](int row) { return (row << 7) | ((row & 2) << 5); };
  auto write_table = [&]() {  // into `table` (the current buffer)
    for (int j = tid; j < KP; j += Cf::kThreads) {
      int hr = 0;  // pad pixels (dY rows are zero): any finite halo row
      if (j < pf_pv) {
        const int gg = pf_g0 + j / W, w = j % W;
        hr = ((gg / H) * H2 + S * (gg % H) - pf_prs) * W2 + w;  // tap (0, 0) of pixel j
      }
      table[j] = make_int4(trow(hr), trow(hr + kwo1), trow(hr + kwo2), 0);
    }
  };
  auto write_tile = [&]() {
#pragma unroll
    for (int i = 0; i < Cf::kPfY; ++i) {
      const int c = tid + i * Cf::kThreads, row = c / Cf::kChY, ch = c % Cf::kChY;
      *reinterpret_cast<uint4*>(dys + chunk_off<Cf::kRowY>(row, ch)) = pfy[i];
    }
#pragma unroll
    for (int i = 0; i < Cf::kPfX; ++i) {
      const int c = tid + i * Cf::kThreads, row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(hal + chunk_off<128>(row, ch)) = pfx[i];
    }
    write_table();
  };

  // wave -> 32 (co) x 32 (ci) block; lane roles of the transposed reads
  const int wco = wid >> 1, wci = wid & 1;
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int prow = 8 * (grp >> 1) + q;                       // + 4 r + 16 kk
  const int ychunk = (wco * 32 + 16 * (grp & 1) + 4 * p) >> 3;  // dY chunk of this lane's 4 columns
  const int xchunk = (wci * 32 + 16 * (grp & 1) + 4 * p) >> 3;
  const int half8 = (p & 1) * 8;                              // byte offset inside the 16-B chunk

  f16v acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

  if (Cf::PF && t_begin < t_end) {
    load_tile(t_begin);
    write_tile();
  }
  __syncthreads();
  for (int tl = t_begin; tl < t_end; ++tl) {
    const bool stage = g.probe != 2 || tl == t_begin;
    if constexpr (Cf::PF) {
      if (tl + 1 < t_end && g.probe != 2) load_tile(tl + 1);  // in flight during this tile's MFMAs
    } else if (stage) {
      load_tile(tl);
      write_tile();
      __syncthreads();
    }
    // Software-pipelined k loop: B fragments rotate through a 3-deep register ring (the reads for
    // tap t+3 are issued right after MFMA t), and the next k-step's A fragment and table entries
    // are read under this step's MFMAs, so no MFMA waits on a just-issued LDS read (the compiler
    // otherwise issues each fragment's 2 reads right before its MFMA with lgkmcnt(0)).
    const int nk = KP / 16;
    // LDS byte address of this lane's 8-byte piece of row `row`: (row, chunk) -> row*ROWB + swizzled
    // chunk*16 + half. Rows r and r+4 share the swizzle (bit 1), so the second A read is a constant
    // offset; B rows of tap (kh, kw) = (h + kw) + kh*W2 with W2 % 4 == 0: 3 swizzled bases per
    // pixel set and per k-step, the kh taps by adding kh*W2*128.
    auto addrY = [&](int row) { return chunk_off<Cf::kRowY>(row, ychunk) + half8; };
    const int xl = (xchunk << 4) | half8;  // this lane's piece of a 128-B halo row, before the row swizzle
    const int khs = W2 * 128;
    auto rdA = [&](int r) {
      const char* p = dys + addrY(r);
      return cat2(tr_read(p), tr_read(p + 4 * Cf::kRowY));
    };
    int bx0[3], bx1[3];
    auto bases = [&](int4 e0, int4 e1) {
      bx0[0] = e0.x ^ xl;
      bx1[0] = e1.x ^ xl;
      bx0[1] = e0.y ^ xl;
      bx1[1] = e1.y ^ xl;
      bx0[2] = e0.z ^ xl;
      bx1[2] = e1.z ^ xl;
    };
    auto rdB = [&](int, int, int t) {
      const int kh = t / 3, kw = t % 3;
      const int ko = Cf::W2T ? kh * Cf::W2T * 128 : kh * khs;  // immediate when the pitch is compile-time
      return cat2(tr_read(hal + bx0[kw] + ko), tr_read(hal + bx1[kw] + ko));
    };
    // cross-step pipelining: the next k-step's A fragment, table entries, swizzled bases and its
    // first three B fragments are read while this step's last MFMAs run
    int r0 = prow;
    bf16x8 a = rdA(r0);
    bases(table[r0], table[r0 + 4]);
    bf16x8 bq0 = rdB(0, 0, 0), bq1 = rdB(0, 0, 1), bq2 = rdB(0, 0, 2);
    // (sched_barrier(0) pins the written order: LLVM's scheduler otherwise sinks each read to just
    // before its MFMA, which then waits out the whole LDS latency.)
#define PDT_MF(t, bq) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq, acc[t], 0, 0, 0)
#define PDT_PIN() __builtin_amdgcn_sched_barrier(0)
    for (int kk = 0; kk < (g.probe == 1 ? 0 : nk); ++kk) {
      // next step (the last step re-reads its own rows: harmless, keeps the loop branch-free)
      const int rn = kk + 1 < nk ? r0 + 16 : r0;
      PDT_MF(0, bq0);  // D[co][ci]
      bq0 = rdB(0, 0, 3);
      PDT_PIN();
      PDT_MF(1, bq1);
      bq1 = rdB(0, 0, 4);
      PDT_PIN();
      PDT_MF(2, bq2);
      bq2 = rdB(0, 0, 5);
      const int4 h0n = table[rn], h1n = table[rn + 4];
      PDT_PIN();
      PDT_MF(3, bq0);
      bq0 = rdB(0, 0, 6);
      PDT_PIN();
      PDT_MF(4, bq1);
      bq1 = rdB(0, 0, 7);
      const bf16x8 an = rdA(rn);
      PDT_PIN();
      PDT_MF(5, bq2);
      bq2 = rdB(0, 0, 8);
      bases(h0n, h1n);
      PDT_PIN();
      PDT_MF(6, bq0);
      bq0 = rdB(0, 0, 0);
      PDT_PIN();
      PDT_MF(7, bq1);
      bq1 = rdB(0, 0, 1);
      PDT_PIN();
      PDT_MF(8, bq2);
      bq2 = rdB(0, 0, 2);
      PDT_PIN();
      a = an;
      r0 = rn;
    }
#undef PDT_MF
#undef PDT_PIN
    __syncthreads();  // every wave is done reading this tile
    if constexpr (Cf::PF) {
      if (tl + 1 < t_end && g.probe != 2) {
        write_tile();
        __syncthreads();
      }
    }
  }
  // partials ws[split][tap][co][ci]; 32x32 accumulator: lane holds ci = l%32,
  // co = 8*(v/4) + 4*(l/32) + v%4 for v = 0..15
  float* wsp = ws + (int64_t)split * 9 * g.Co * g.Ci;
  const int ci = ci0 + wci * 32 + (lane & 31);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int co = co0 + wco * 32 + 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
      wsp[((int64_t)t * g.Co + co) * g.Ci + ci] = acc[t][v];
    }
}

// dw[co][tap][ci] (bf16, the channels_last storage of [Co, Ci, 3, 3]) = sum over splits, fixed order.
// A workgroup takes 16 float4 columns; its 16 thread groups split the partials round-robin (each
// summed in order), then one fixed-order pass over the group sums: deterministic, and 16x the
// parallelism of one thread per column (layer 1: 512 splits deep, 132 us for a 147 KB result).
constexpr int kRedCols = 16, kRedGroups = 16;
__global__ __launch_bounds__(256) void conv3x3_wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                   uint16_t* __restrict__ dw, int nsplit, int Co,
                                                                   int Ci) {
  __shared__ float4 part[kRedGroups][kRedCols];
  const int64_t per4 = (int64_t)9 * Co * Ci / 4;
  const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
  const int64_t i = (int64_t)blockIdx.x * kRedCols + col;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < per4)
    for (int k = grp; k < nsplit; k += kRedGroups) {
      const float4 v = reinterpret_cast<const float4*>(ws + (int64_t)k * 9 * Co * Ci)[i];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  part[grp][col] = s;
  __syncthreads();
  if (grp == 0 && i < per4) {
    float4 t = part[0][col];
#pragma unroll
    for (int k = 1; k < kRedGroups; ++k) {
      const float4 v = part[k][col];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const int64_t e = i * 4;  // (t, co, ci..ci+3)
    const int tp = (int)(e / ((int64_t)Co * Ci)), rem = (int)(e % ((int64_t)Co * Ci));
    const int co = rem / Ci, ci = rem % Ci;
    uint16_t* o = dw + ((int64_t)co * 9 + tp) * Ci + ci;
    const uint32_t lo = (uint32_t)f2bf(t.x) | ((uint32_t)f2bf(t.y) << 16);
    const uint32_t hi = (uint32_t)f2bf(t.z) | ((uint32_t)f2bf(t.w) << 16);
    *reinterpret_cast<uint2*>(o) = make_uint2(lo, hi);
  }
}

inline int rows_per_tile(int W) {
  int R = (kTileTarget + W / 2) / W;
  return R < 1 ? 1 : R;
}

// Largest halo (padded pixel rows) of any tile: tiles start at global rows t*R, whose offsets in
// their image cycle through {t*R mod H}; a tile starting at offset o touches (o + R - 1)/H + 1 images
// and stages R real rows plus 2 pad rows per image. Stride 2 (input Hi x Wi, output H x W): padded
// input rows pr(g) = (g / H)(Hi + 2) + 2 (g % H) .. pr(last) + 2.
inline int64_t halo_rows(int R, int H, int W, int S = 1, int Hi = 0, int Wi = 0) {
  if (S == 1) {
    int imgs = 1;
    for (int t = 0, o = 0; t < H; ++t, o = (o + R) % H) {
      const int k = (o + R - 1) / H + 1;
      imgs = k > imgs ? k : imgs;
    }
    return (int64_t)(R + 2 * imgs) * ((W + 2 + 3) & ~3);
  }
  int64_t rows = 0;
  for (int t = 0, o = 0; t < H; ++t, o = (o + R) % H) {
    const int last = o + R - 1;
    const int64_t r = (int64_t)(last / H) * (Hi + 2) + 2 * (last % H) + 2 - 2 * o + 1;
    rows = r > rows ? r : rows;
  }
  return rows * 2 * (((Wi + 3) / 2 + 3) & ~3);
}

int g_probe = 0;

// H, W: output (dY) size; Hi, Wi: input size (stride S)
inline bool geo_of(int N, int H, int W, int Ci, int Co, int co_t, int target_wgs, Geo& g, int S = 1, int Hi = 0,
                   int Wi = 0) {
  if (S == 1) { Hi = H; Wi = W; }
  g.N = N; g.H = H; g.W = W; g.Ci = Ci; g.Co = Co; g.Hi = Hi; g.Wi = Wi;
  const int hmax = halo_max(S), kpmax = kp_max(S);
  g.R = rows_per_tile(W);
  // tiny images: more pad rows per tile; stride 2: also the K-row cap
  while (g.R > 1 && (halo_rows(g.R, H, W, S, Hi, Wi) > hmax || ((g.R * W + 15) & ~15) > kpmax)) --g.R;
  g.NH = N * H;
  const int P = g.R * W, KP = (P + 15) & ~15;
  if (KP > kpmax) return false;
  if (halo_rows(g.R, H, W, S, Hi, Wi) > hmax) return false;
  g.ntiles = (g.NH + g.R - 1) / g.R;
  g.nblk = (Co / co_t) * (Ci / 64);
  int ns = (target_wgs + g.nblk - 1) / g.nblk;
  if (ns > g.ntiles) ns = g.ntiles;
  if (ns < 1) ns = 1;
  g.tiles_per_split = (g.ntiles + ns - 1) / ns;
  g.probe = g_probe;
  g.nsplit = (g.ntiles + g.tiles_per_split - 1) / g.tiles_per_split;
  return true;
}

int g_target_wgs = 0;    // 0: by tile (CO_T 128: 256 = one per CU; CO_T 64: 512 = two per CU)
int g_co_tile = 0;       // 0: by shape; 64 / 128 forced (tuning)

// CO_T = 128 (Co % 128 == 0): 8 waves, next tile prefetched in registers, one workgroup (2
// waves/SIMD) per CU, half the dY staging per FLOP — fastest on ResNet-50 layers 2-4 (302 / 282 / 284
// us vs 329-341 / 305-319 / 313-324 for CO_T = 64 at batch 1024); CO_T = 64 (layer 1): 4 waves,
// 48.5 KB LDS, two workgroups per CU overlapping each other's staging.
inline int target_wgs(int co_t) { return g_target_wgs > 0 ? g_target_wgs : (co_t == 128 ? 256 : 512); }

inline int co_tile_of(int Co) {
  if (g_co_tile == 64 || (g_co_tile == 128 && Co % 128 == 0)) return g_co_tile;
  return Co % 128 == 0 ? 128 : 64;
}

template <class Cf>
int launch(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, const Geo& g, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_wgrad_kernel<Cf>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  hipLaunchKernelGGL(conv3x3_wgrad_kernel<Cf>, dim3(g.nsplit * g.nblk), dim3(Cf::kThreads), Cf::kLds, s, x, dy, ws,
                     g);
  const int64_t per4 = (int64_t)9 * g.Co * g.Ci / 4;
  hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel, dim3((unsigned)((per4 + kRedCols - 1) / kRedCols)),
                     dim3(kRedCols * kRedGroups), 0, s, ws, dw, g.nsplit, g.Co, g.Ci);
  return 0;
}

// The halo row pitch of the shape as a compile-time constant where ResNet-50 / ResNet-18 at 224 x 224
// need one (stride 1: W + 2 rounded up to 4 -> 60, 32, 16, 12; stride 2: 2 HALF -> 64, 32, 16); any other
// pitch takes the runtime-pitch instantiation.
template <int CO_T, bool PF, int S>
int launch_pitch(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, const Geo& g, hipStream_t s) {
  const int half = ((g.Wi + 3) / 2 + 3) & ~3;
  const int w2 = S == 1 ? (g.W + 2 + 3) & ~3 : 2 * half;
  switch (w2) {
    case 12: return launch<WCfg<CO_T, PF, S, 12>>(x, dy, dw, ws, g, s);
    case 16: return launch<WCfg<CO_T, PF, S, 16>>(x, dy, dw, ws, g, s);
    case 32: return launch<WCfg<CO_T, PF, S, 32>>(x, dy, dw, ws, g, s);
    case 60: return launch<WCfg<CO_T, PF, S, 60>>(x, dy, dw, ws, g, s);
    case 64: return launch<WCfg<CO_T, PF, S, 64>>(x, dy, dw, ws, g, s);
    default: return launch<WCfg<CO_T, PF, S, 0>>(x, dy, dw, ws, g, s);
  }
}

}  // namespace

extern "C" {

// fp32 workspace floats for pdt_conv3x3s1_wgrad at this shape (0: unsupported shape).
int64_t pdt_conv3x3_wgrad_ws_floats(int N, int H, int W, int Ci, int Co, int* nsplit_out) {
  Geo g;
  const int co_t = co_tile_of(Co);
  if (Ci % 64 != 0 || Co % 64 != 0 || !geo_of(N, H, W, Ci, Co, co_t, target_wgs(co_t), g)) return 0;
  if (nsplit_out) *nsplit_out = g.nsplit;
  return (int64_t)g.nsplit * 9 * Co * Ci;
}

// dw[Co,3,3,Ci] (bf16, channels_last weight storage) of the stride-1 pad-1 3x3 conv from
// x[N,H,W,Ci] and dy[N,H,W,Co] (NHWC bf16). ws: pdt_conv3x3_wgrad_ws_floats() floats.
// Returns 0, or < 0 for an unsupported shape (caller falls back).
int pdt_conv3x3s1_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H, int W, int Ci,
                        int Co, hipStream_t s) {
  if (Ci % 64 != 0 || Co % 64 != 0 || N < 1 || H < 1 || W < 1) return -1;
  if ((int64_t)N * H * W * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31) return -2;  // 32-bit buffer offsets
  Geo g;
  const int co_t = co_tile_of(Co);
  if (!geo_of(N, H, W, Ci, Co, co_t, target_wgs(co_t), g)) return -4;
  return co_t == 128 ? launch_pitch<128, true, 1>(x, dy, dw, ws, g, s) : launch_pitch<64, false, 1>(x, dy, dw, ws, g, s);
}

// Stride 2 / pad 1 (input x [N,H,W,Ci], dy [N,Ho,Wo,Co], Ho = (H-1)/2+1), Ci % 64 == 0, Co % 64 == 0.
// CO_T 128 (one 8-wave workgroup per CU, next tile prefetched in registers) unless forced to 64
// (pdt_conv3x3_wgrad_tune) or Co % 128 != 0: 4 waves, 2 workgroups per CU, synchronous staging.
inline int s2_co_tile(int Co) { return (g_co_tile == 64 || Co % 128 != 0) ? 64 : 128; }

int64_t pdt_conv3x3s2_wgrad_ws_floats(int N, int H, int W, int Ci, int Co, int* nsplit_out) {
  Geo g;
  if (Ci % 64 != 0 || Co % 64 != 0 || H < 2 || W < 2) return 0;
  const int co_t = s2_co_tile(Co);
  if (!geo_of(N, (H - 1) / 2 + 1, (W - 1) / 2 + 1, Ci, Co, co_t, target_wgs(co_t), g, 2, H, W)) return 0;
  if (nsplit_out) *nsplit_out = g.nsplit;
  return (int64_t)g.nsplit * 9 * Co * Ci;
}

int pdt_conv3x3s2_wgrad(const uint16_t* x, const uint16_t* dy, uint16_t* dw, float* ws, int N, int H, int W, int Ci,
                        int Co, hipStream_t s) {
  if (Ci % 64 != 0 || Co % 64 != 0 || N < 1 || H < 2 || W < 2) return -1;
  if ((int64_t)N * H * W * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31) return -2;  // 32-bit buffer offsets
  Geo g;
  const int co_t = s2_co_tile(Co);
  if (!geo_of(N, (H - 1) / 2 + 1, (W - 1) / 2 + 1, Ci, Co, co_t, target_wgs(co_t), g, 2, H, W)) return -4;
  return co_t == 128 ? launch_pitch<128, true, 2>(x, dy, dw, ws, g, s) : launch_pitch<64, false, 2>(x, dy, dw, ws, g, s);
}

void pdt_conv3x3_wgrad_probe(int probe) { g_probe = probe; }

// Tuning / A-B hooks (tools/convbench/wgrad3x3_bench.cpp): target workgroups (0 = by tile) and
// forced CO_T (0 = by shape).
void pdt_conv3x3_wgrad_tune(int target_wgs, int co_tile) {
  if (target_wgs >= 0) g_target_wgs = target_wgs;
  if (co_tile >= 0) g_co_tile = co_tile;
}

}  // extern "C"
