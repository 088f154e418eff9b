// Stride-2 / pad-1 3x3 convolution (forward and data gradient) as a gathered implicit GEMM on MFMA
// (gfx950), NHWC bf16, fp32 accumulate.
//
// Not in the reference (LeNet's convs are stride 1, /root/reference/cnn.py:10-16). Serves the three
// stride-2 3x3 convs of ResNet-50 (layer2-4 block 0, torchvision v1.5 puts the stride in conv2), which
// ran on MIOpen (ck grouped_conv_fwd, igemm_bwd: ~2.5 ms/step at 1024/GPU plus their fill passes,
// profiles/r3/steady_resnet50_b1024_ours.md) and kept MIOpen's solver search in the first step.
//
// One kernel, two uses — a GEMM whose A rows are gathered input pixels, one tap per k-step:
//
//   Y[pix(m), n] = sum_{u in taps, c} X[n_img, y(m)*a + dy_u, x(m)*a + dx_u, c] * Wt[n, w_u, c]
//
//   forward      : m over the N*Ho*Wo outputs, a = 2, taps (kh-1, kw-1) for the 9 (kh, kw), Wt = W
//                  [Co][9][Ci]; statistics of the consuming BatchNorm in the epilogue (tile_stats.h)
//   data gradient: the stride-2 transposed conv splits into 4 output PHASES (py, px) = parity of
//                  (ih, iw): dx[n, 2y+py, 2x+px] takes dy[n, y + (py+1-kh)/2, x + (px+1-kw)/2] from
//                  the taps whose (py+1-kh) and (px+1-kw) are even — 1, 2, 2 and 4 taps, so no MFMA
//                  ever multiplies an inserted zero. a = 1, Wt = the flipped transposed weights
//                  [Ci][9][Co] (conv3x3_flip: w_u = 8 - (kh*3+kw)); the backward reduction of the
//                  BatchNorm whose output gradient this is in the epilogue (BSTATS). The four phases run
//                  in ONE launch (block -> (tile, phase), phases interleaved so every XCD gets an even mix).
//
// Structure: the per-tap ring of conv3x3.hip (tile 256 pixels x 128 channels, 8 waves of 64x64 as
// 4x4 v_mfma_f32_16x16x32_bf16, A and B staged global -> LDS by LDS-DMA through a 3-slot ring, one
// raw s_barrier per k-step with a counted vmcnt, padding rows from a zero page, XOR-swizzled 64-B
// rows, operands swapped so a lane's accumulator holds 4 channels of one pixel, bf16 tile staged
// through LDS for 16-B row stores and the fused BatchNorm epilogues, XCD-aware tile map).
#include "../common.h"
#include "../tile_stats.h"

using namespace pdt;

namespace {

__device__ uint8_t g_s2_ones[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};  // "no ReLU mask"


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define PDT_LDS __attribute__((address_space(3)))

__device__ __attribute__((aligned(256))) uint4 g_s2_zero[16];  // zero page for padding rows (never written)

// Tile 256 pixels x BN output channels: BN = 128 (8 waves, 4 x 2) or 64 (4 waves, 4 x 1, for a GEMM N
// of 64 channels: the data gradient of a 64-input-channel conv, ResNet-18/34 layer2 block 0).
template <int BN_>
struct S2Cfg {
  static constexpr int kBM = 256, kBN = BN_, kBK = 32, kWM = 4, kWN = BN_ / 64, kSlots = 3;
  static constexpr int kWaves = kWM * kWN, kThreads = kWaves * 64;
  static constexpr int kABytes = kBM * 64, kBBytes = kBN * 64, kSlot = kABytes + kBBytes;
  static constexpr int kEpiStride = kBN * 2 + 16;
  static constexpr int kEpi = kBM * kEpiStride + tile_bn_stats_lds<kBM, kBN, kThreads>();
  static constexpr int kLds = kSlots * kSlot > kEpi ? kSlots * kSlot : kEpi;
  static constexpr int kMB = kBM / kWM / 16, kNB = kBN / kWN / 16;
  static constexpr int kALd = kBM / 16 / kWaves, kBLd = kBN / 16 / kWaves, kG = kALd + kBLd;
  static_assert(kALd * 16 * kWaves == kBM && kBLd * 16 * kWaves == kBN, "DMA split");
};
constexpr int kBM = 256, kBK = 32;

template <int G>
__device__ __forceinline__ void wait_vm() {
  static_assert(G == 3 || G == 5, "vmcnt: DMA instructions per k-step");
  if constexpr (G == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
}

struct Taps {  // one phase: n taps, input-pixel offsets (dy, dx) and weight tap index w
  int n;
  int dy[9], dx[9], w[9];
};

struct Geo {
  int N, Ho, Wo;      // GEMM row space of one phase: M = N * Ho * Wo pixels (n, y, x)
  int Hin, Win, Cin;  // gathered tensor [N, Hin, Win, Cin]; pixel of (m, u) = (y*a + dy_u, x*a + dx_u)
  int a;
  int Co;             // GEMM N = output channels; Wt rows [Co][9][Cin]
  int Hy, Wy, sy;     // output tensor [N, Hy, Wy, Co], pixel (y*sy + py, x*sy + px)
  int nph, tpp, T;    // phases, 256-row tiles per phase, partial rows (nph * tpp)
  int py[4], px[4];
  Taps ph[4];
};

__device__ __forceinline__ int chk64(int row, int p) { return p ^ (((row >> 2) & 1) << 1); }  // involution
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + (chk64(row, chunk) << 4); }

__device__ __forceinline__ f4 mfma(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (PDT_LDS void*)lds_wave_base, 16, 0, 0);
}

template <class Cf, bool STATS, bool BSTATS>
__global__ __launch_bounds__(Cf::kThreads, 4) void conv3x3g_kernel(const uint16_t* __restrict__ X,
                                                                  const uint16_t* __restrict__ Wt,
                                                                  uint16_t* __restrict__ Y, float* __restrict__ part,
                                                                  BnSrc bs, Geo g) {
  constexpr int kBN = Cf::kBN, kWM = Cf::kWM, kSlots = Cf::kSlots, kWaves = Cf::kWaves, kThreads = Cf::kThreads;
  constexpr int kABytes = Cf::kABytes, kSlot = Cf::kSlot, kEpiStride = Cf::kEpiStride, kMB = Cf::kMB;
  constexpr int kNB = Cf::kNB, kALd = Cf::kALd, kBLd = Cf::kBLd;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid % kWM, wn = wid / kWM;
  const int HW = g.Ho * g.Wo, M = g.N * HW;
  const int ntn = g.Co / kBN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mtg = tile / ntn, n0 = (tile % ntn) * kBN;
  // phases interleaved tile by tile: an XCD's contiguous range of logical tiles mixes the 1-, 2- and
  // 4-tap phases evenly, and the four phase tiles of one position read the same dY rows (shared L2)
  const int ph = mtg % g.nph, mt = mtg / g.nph;
  const int m0 = mt * kBM;
  const Taps& tp = g.ph[ph];
  const int ntap = tp.n;

  // ---- A rows this lane DMAs: row (wid*kALd + i)*16 + lane/4, source chunk pre-swizzled
  const int sub = lane >> 2, p = lane & 3;
  int aoff[kALd];
  unsigned amask[kALd];
#pragma unroll
  for (int i = 0; i < kALd; ++i) {
    const int r = (wid * kALd + i) * 16 + sub;
    const int m = m0 + r;
    unsigned mk = 0;
    aoff[i] = chk64(r, p) * 8;
    if (m < M) {
      const int n = m / HW, rem = m % HW, y = rem / g.Wo, x = rem % g.Wo;
      const int iy = y * g.a, ix = x * g.a;
      aoff[i] += ((n * g.Hin + iy) * g.Win + ix) * g.Cin;
      for (int u = 0; u < ntap; ++u) {
        const int yy = iy + tp.dy[u], xx = ix + tp.dx[u];
        if (yy >= 0 && yy < g.Hin && xx >= 0 && xx < g.Win) mk |= 1u << u;
      }
    }
    amask[i] = mk;
  }
  int boff[kBLd];
#pragma unroll
  for (int j = 0; j < kBLd; ++j) {
    const int r = (wid * kBLd + j) * 16 + sub;
    boff[j] = (n0 + r) * 9 * g.Cin + chk64(r, p) * 8;
  }
  const int S = ntap * (g.Cin / kBK);

  auto issue = [&](int s) {
    const int cc = s / ntap, u = s - cc * ntap;
    const int toff = (tp.dy[u] * g.Win + tp.dx[u]) * g.Cin + cc * kBK;
    char* slot = lds + (s % kSlots) * kSlot;
#pragma unroll
    for (int i = 0; i < kALd; ++i) {
      const uint16_t* src = ((amask[i] >> u) & 1u) ? X + (aoff[i] + toff) : reinterpret_cast<const uint16_t*>(g_s2_zero);
      dma16(src, slot + (wid * kALd + i) * 1024);
    }
    const int wo = tp.w[u] * g.Cin + cc * kBK;
#pragma unroll
    for (int j = 0; j < kBLd; ++j) dma16(Wt + (boff[j] + wo), slot + kABytes + (wid * kBLd + j) * 1024);
  };

  f4 acc[kMB][kNB];
#pragma unroll
  for (int i = 0; i < kMB; ++i)
#pragma unroll
    for (int j = 0; j < kNB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (S > 1) issue(1);
  const int lrow = lane & 15, lchk = lane >> 4;
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) wait_vm<Cf::kG>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 2 < S) issue(s + 2);  // slot (s+2)%3 was last read at step s-1: every wave is past it
    const char* As = lds + (s % kSlots) * kSlot;
    const char* Bs = As + kABytes;
    bf16x8 a[kMB], b[kNB];
#pragma unroll
    for (int i = 0; i < kMB; ++i) a[i] = *reinterpret_cast<const bf16x8*>(As + swz64(wm * 64 + i * 16 + lrow, lchk));
#pragma unroll
    for (int j = 0; j < kNB; ++j) b[j] = *reinterpret_cast<const bf16x8*>(Bs + swz64(wn * 64 + j * 16 + lrow, lchk));
#pragma unroll
    for (int i = 0; i < kMB; ++i)
#pragma unroll
      for (int j = 0; j < kNB; ++j) acc[i][j] = mfma(b[j], a[i], acc[i][j]);  // D[n][m]
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // ---- epilogue: bf16 tile [256 pixels][128] staged in LDS
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < kMB; ++i)
#pragma unroll
    for (int j = 0; j < kNB; ++j) {
      const int ml = wm * 64 + i * 16 + lrow;
      const int cl = wn * 64 + j * 16 + 4 * lchk;
      const f4 v = acc[i][j];
      uint2 pk;
      pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(lds + ml * kEpiStride + cl * 2) = pk;
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int kChunks = kBN / 8;
  RowStats8 rst;  // STATS (forward only: one phase, output rows = GEMM rows), tile_stats.h RowStats8
  float kst = 0.f;
  if constexpr (STATS) {
    rs8_init(rst, *reinterpret_cast<const uint4*>(lds + (tid % kChunks) * 16));
    if (tid < kBN) kst = __uint_as_float((uint32_t)*reinterpret_cast<const uint16_t*>(lds + tid * 2) << 16);
  }
  float bs1[8], bs2[8], bmu[8];
  if constexpr (BSTATS) {
    const int c = tid % kChunks;
    *reinterpret_cast<float4*>(bmu) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8);
    *reinterpret_cast<float4*>(bmu + 4) = *reinterpret_cast<const float4*>(bs.mean + n0 + c * 8 + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) { bs1[k] = 0.f; bs2[k] = 0.f; }
  }
  const int py = g.py[ph], px = g.px[ph];
  // rows in batches, their BN-input loads issued before the first use and branch-free (invalid rows read
  // row 0 and add nothing): per-row conditional loads waited a memory latency each (conv3x3.hip, halo
  // kernel epilogue, has the same note)
  constexpr int kRowIt = kBM * kChunks / kThreads;
  constexpr int kBt = BSTATS && kRowIt > 4 ? 4 : kRowIt;
  static_assert(kRowIt * kThreads == kBM * kChunks && kRowIt % kBt == 0, "epilogue rows");
  const uint8_t* const bm_base = bs.mask ? bs.mask : g_s2_ones;
  const int64_t bm_scale = bs.mask ? 1 : 0;
#pragma unroll 1
  for (int h = 0; h < kRowIt; h += kBt) {
    int64_t offv[kBt];
    bool okv[kBt];
    uint4 xbv[kBt];
    unsigned mkv[kBt];
#pragma unroll
    for (int it = 0; it < kBt; ++it) {
      const int idx = tid + (h + it) * kThreads, r = idx / kChunks, c = idx % kChunks;
      const int m = m0 + r, mc = m < M ? m : M - 1;
      const int n = mc / HW, rem = mc % HW, y = rem / g.Wo, x = rem % g.Wo;
      const int oy = y * g.sy + py, ox = x * g.sy + px;
      // (odd input size: the last phase row / column is outside)
      okv[it] = m < M && oy < g.Hy && ox < g.Wy;
      offv[it] = okv[it] ? ((int64_t)(n * g.Hy + oy) * g.Wy + ox) * g.Co + n0 + c * 8 : (int64_t)n0 + c * 8;
      if constexpr (BSTATS) {
        xbv[it] = *reinterpret_cast<const uint4*>(bs.x + offv[it]);
        const unsigned mk = bm_base[(offv[it] >> 3) * bm_scale];
        mkv[it] = okv[it] ? mk : 0u;
      }
    }
#pragma unroll
    for (int it = 0; it < kBt; ++it) {
      const int idx = tid + (h + it) * kThreads, r = idx / kChunks, c = idx % kChunks;
      const uint4 v = *reinterpret_cast<const uint4*>(lds + r * kEpiStride + c * 16);
      if constexpr (BSTATS) bn_bwd_accum8(v, xbv[it], mkv[it], bmu, bs1, bs2);
      if (!okv[it]) continue;
      if constexpr (STATS) rs8_add(rst, v);
      *reinterpret_cast<uint4*>(Y + offv[it]) = v;
    }
  }
  if constexpr (BSTATS)  // every wave is done reading the staged tile: its LDS holds the block sums
    bn_bwd_tile_store<kBN, kWaves>(bs1, bs2, reinterpret_cast<float*>(lds), bs.part, g.T, ph * g.tpp + mt, g.Co, n0);
  if constexpr (STATS) {
    __syncthreads();
    rs8_tile_store<kBN, kWaves>(rst, kst, reinterpret_cast<float*>(lds), part, min(kBM, M - m0), g.T, mt, g.Co, n0);
  }
}

template <class Cf, bool STATS, bool BSTATS>
int launch_cf(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, const BnSrc& bs, const Geo& g,
              hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3g_kernel<Cf, STATS, BSTATS>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, Cf::kLds) != hipSuccess)
      return -3;
    attr = true;
  }
  const int64_t grid = (int64_t)g.nph * g.tpp * (g.Co / Cf::kBN);
  hipLaunchKernelGGL((conv3x3g_kernel<Cf, STATS, BSTATS>), dim3((unsigned)grid), dim3(Cf::kThreads), Cf::kLds, s, x,
                     w, y, part, bs, g);
  return 0;
}

// the GEMM N (g.Co) picks the tile: 128 channels when it divides, else 64
template <bool STATS, bool BSTATS>
int launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, const BnSrc& bs, const Geo& g,
           hipStream_t s) {
  if (g.Co % 128 == 0 && !small_grid_narrow((int64_t)g.nph * g.tpp * (g.Co / 128)))
    return launch_cf<S2Cfg<128>, STATS, BSTATS>(x, w, y, part, bs, g, s);
  return launch_cf<S2Cfg<64>, STATS, BSTATS>(x, w, y, part, bs, g, s);
}

inline int tiles_of(int64_t M) { return (int)((M + kBM - 1) / kBM); }

// shape limits: 32-bit element offsets; the GEMM's N (output channels of this direction) tiles by 64 / 128,
// its K (gathered channels) by 64 (two kBK steps per tap)
inline int check_shape(int N, int H, int W, int Ci, int Co, int kdim, int ndim) {
  if (N < 1 || H < 2 || W < 2 || kdim % 64 != 0 || ndim % 64 != 0) return -1;
  if ((int64_t)N * H * W * (Ci > Co ? Ci : Co) >= (int64_t)1 << 31 || (int64_t)Co * 9 * Ci >= (int64_t)1 << 31)
    return -2;
  return 0;
}

}  // namespace

extern "C" {

int pdt_conv3x3s2_tile_rows() { return kBM; }

// Partial rows (T) of pdt_conv3x3s2_dgrad's BatchNorm backward partials for input size H x W.
int pdt_conv3x3s2_dgrad_tiles(int N, int H, int W) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  return 4 * tiles_of((int64_t)N * Ho * Wo);
}

// y[N,Ho,Wo,Co] = conv2d(x[N,H,W,Ci], w[Co,3,3,Ci], stride 2, padding 1), Ho = (H-1)/2+1 (NHWC bf16).
// part (or null): per-256-pixel-tile BatchNorm statistics of y, [2][ceil(N*Ho*Wo/256)][Co] fp32.
// Ci % 64 == 0, Co % 64 == 0. Returns 0, or < 0 for an unsupported shape (caller falls back).
int pdt_conv3x3s2_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, int N, int H, int W, int Ci,
                      int Co, hipStream_t s) {
  const int rc = check_shape(N, H, W, Ci, Co, Ci, Co);
  if (rc) return rc;
  Geo g{};
  g.N = N; g.Ho = (H - 1) / 2 + 1; g.Wo = (W - 1) / 2 + 1;
  g.Hin = H; g.Win = W; g.Cin = Ci; g.a = 2; g.Co = Co;
  g.Hy = g.Ho; g.Wy = g.Wo; g.sy = 1;
  g.nph = 1; g.tpp = tiles_of((int64_t)N * g.Ho * g.Wo); g.T = g.tpp;
  g.ph[0].n = 9;
  for (int u = 0; u < 9; ++u) {
    g.ph[0].dy[u] = u / 3 - 1;
    g.ph[0].dx[u] = u % 3 - 1;
    g.ph[0].w[u] = u;
  }
  return part ? launch<true, false>(x, w, y, part, BnSrc{}, g, s) : launch<false, false>(x, w, y, nullptr, BnSrc{}, g, s);
}

// dx[N,H,W,Ci] = data gradient of that conv from dy[N,Ho,Wo,Co] and the flipped transposed weights
// wf[Ci,3,3,Co] (pdt_conv3x3_flip_weights). bn_x / bn_mask / bn_mean / bn_part (all null = off): dx is
// the gradient at the output of a BatchNorm with input bn_x [N,H,W,Ci], ReLU mask bn_mask (or null)
// and mean bn_mean; bn_part [2][pdt_conv3x3s2_dgrad_tiles()][Ci] receives its backward partials.
// Ci % 64 == 0, Co % 64 == 0.
int pdt_conv3x3s2_dgrad(const uint16_t* dy, const uint16_t* wf, uint16_t* dx, const uint16_t* bn_x,
                        const uint8_t* bn_mask, const float* bn_mean, float* bn_part, int N, int H, int W, int Ci,
                        int Co, hipStream_t s) {
  const int rc = check_shape(N, H, W, Ci, Co, Co, Ci);
  if (rc) return rc;
  if (bn_part && (!bn_x || !bn_mean)) return -1;
  Geo g{};
  g.N = N; g.Ho = (H - 1) / 2 + 1; g.Wo = (W - 1) / 2 + 1;
  g.Hin = g.Ho; g.Win = g.Wo; g.Cin = Co; g.a = 1; g.Co = Ci;
  g.Hy = H; g.Wy = W; g.sy = 2;
  g.nph = 4; g.tpp = tiles_of((int64_t)N * g.Ho * g.Wo); g.T = 4 * g.tpp;
  // (kh, row offset) pairs of one parity: even output rows take kh = 1 (dy row y); odd ones kh = 0
  // (dy row y + 1) and kh = 2 (dy row y)
  const int nk[2] = {1, 2}, kk[2][2] = {{1, 1}, {0, 2}}, dd[2][2] = {{0, 0}, {1, 0}};
  for (int q = 0; q < 4; ++q) {
    const int py = q >> 1, px = q & 1;
    g.py[q] = py; g.px[q] = px;
    Taps& t = g.ph[q];
    t.n = 0;
    for (int i = 0; i < nk[py]; ++i)
      for (int j = 0; j < nk[px]; ++j) {
        const int kh = kk[py][i], kw = kk[px][j];
        t.dy[t.n] = dd[py][i];
        t.dx[t.n] = dd[px][j];
        t.w[t.n] = 8 - (kh * 3 + kw);
        ++t.n;
      }
  }
  if (bn_part)
    return launch<false, true>(dy, wf, dx, nullptr, BnSrc{bn_x, bn_mask, bn_mean, bn_part}, g, s);
  return launch<false, false>(dy, wf, dx, nullptr, BnSrc{}, g, s);
}

}  // extern "C"
