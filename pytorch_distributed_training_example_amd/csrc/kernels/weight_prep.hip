// Per-step weight transforms of every convolution, in ONE launch (ops/conv.py prepare_weights):
//
//   1x1 conv   (taps = 1): W [Co][Ci]          -> W^T [Ci][Co]          (the data-gradient GEMM's B rows)
//   3x3 conv   (taps = 9): W [Co][3][3][Ci]    -> Wf [Ci][3][3][Co],  Wf[ci][t][co] = W[co][8 - t][ci]
//                          (flipped + transposed: the data gradient as a forward conv, conv3x3.hip)
//
// Not in the reference (LeNet's three convs run on cuDNN there, /root/reference/cnn.py:10-16). ResNet-50
// ran these as 37 transpose copies + 16 flip kernels per step, each a separate launch of a few us
// (0.45 ms/step at 1024 images per GPU, 0.34 ms of a 12.8 ms step at 128 — profiles/r4). Both kinds
// are batched strided 2-D transposes: tap slice t of item i is [R = Co][C = Ci] with row stride
// taps * C at src + src_tap(t) * C, written as [C][R] with row stride taps * R at dst + t * R. One
// workgroup moves one 64 x 64 tile through LDS (coalesced 128-B reads and writes); grid.y = item.
#include "../common.h"

namespace {

constexpr int kMaxItems = 64;
constexpr int kT = 64;

struct PrepItem {
  const uint16_t* src;
  uint16_t* dst;
  int R, C, taps;
};

struct PrepBatch {
  PrepItem it[kMaxItems];
};

__global__ __launch_bounds__(256) void weight_prep_kernel(PrepBatch b) {
  __shared__ uint16_t tile[kT][kT + 8];  // +8: 16-B aligned rows, 4-bank shift per row
  const PrepItem& p = b.it[blockIdx.y];
  const int tr = (p.R + kT - 1) / kT, tc = (p.C + kT - 1) / kT;
  const int ntiles = tr * tc * p.taps;
  const int tid = threadIdx.x;
  const bool vec = (p.C % 8 == 0) && (p.R % 8 == 0);  // 16-B rows both ways (every ResNet conv)
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int tap = t / (tr * tc), rc = t % (tr * tc);
    const int r0 = (rc / tc) * kT, c0 = (rc % tc) * kT;
    const int stap = p.taps == 9 ? 8 - tap : 0;
    const uint16_t* src = p.src + (int64_t)stap * p.C;
    uint16_t* dst = p.dst + (int64_t)tap * p.R;
    const int64_t srs = (int64_t)p.taps * p.C, drs = (int64_t)p.taps * p.R;
    if (vec) {
      // read: 64 rows x 8 pieces of 8 columns (16 B), 2 pieces per thread
      for (int i = tid; i < kT * 8; i += 256) {
        const int r = i >> 3, pc = (i & 7) * 8;
        const int gr = r0 + r, gc = c0 + pc;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (gr < p.R && gc < p.C) v = *reinterpret_cast<const uint4*>(src + gr * srs + gc);
        *reinterpret_cast<uint4*>(&tile[r][pc]) = v;
      }
      __syncthreads();
      // write: 64 dst rows (columns c) x 8 pieces of 8 consecutive r, gathered from the tile
      for (int i = tid; i < kT * 8; i += 256) {
        const int c = i >> 3, pr = (i & 7) * 8;
        const int gr = r0 + pr, gc = c0 + c;
        if (gr < p.R && gc < p.C) {
          uint32_t w[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            w[k] = (uint32_t)tile[pr + 2 * k][c] | ((uint32_t)tile[pr + 2 * k + 1][c] << 16);
          *reinterpret_cast<uint4*>(dst + gc * drs + gr) = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    } else {
      for (int i = tid; i < kT * kT; i += 256) {
        const int r = i / kT, c = i % kT;
        const int gr = r0 + r, gc = c0 + c;
        tile[r][c] = (gr < p.R && gc < p.C) ? src[gr * srs + gc] : (uint16_t)0;
      }
      __syncthreads();
      for (int i = tid; i < kT * kT; i += 256) {
        const int c = i / kT, r = i % kT;
        const int gr = r0 + r, gc = c0 + c;
        if (gr < p.R && gc < p.C) dst[gc * drs + gr] = tile[r][c];
      }
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" {

int pdt_weight_prep_max_items() { return kMaxItems; }

// n items (<= pdt_weight_prep_max_items()): src[i] [R][taps][C] -> dst[i] [C][taps][R] as described above.
int pdt_weight_prep(const uint16_t* const* src, uint16_t* const* dst, const int* R, const int* C, const int* taps,
                    int n, hipStream_t s) {
  if (n < 1 || n > kMaxItems) return -1;
  PrepBatch b{};
  int most = 1;
  for (int i = 0; i < n; ++i) {
    if ((taps[i] != 1 && taps[i] != 9) || R[i] < 1 || C[i] < 1 || (int64_t)R[i] * C[i] * taps[i] >= (1ll << 31))
      return -1;
    b.it[i] = PrepItem{src[i], dst[i], R[i], C[i], taps[i]};
    const int tiles = ((R[i] + kT - 1) / kT) * ((C[i] + kT - 1) / kT) * taps[i];
    most = tiles > most ? tiles : most;
  }
  const int gx = most < 128 ? most : 128;  // tiles per item in flight; the grid strides over the rest
  hipLaunchKernelGGL(weight_prep_kernel, dim3(gx, n), dim3(256), 0, s, b);
  return 0;
}

}  // extern "C"
