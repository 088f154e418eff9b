// LeNet (the reference model) hot ops for gfx950 — SURVEY.md §2.3's per-op replacements.
//
// Reference model: /root/reference/cnn.py:9-23 —
//   UpsamplingBilinear2d(32) -> Conv2d(1,6,5) -> LeakyReLU(0.2) -> MaxPool2d(2)
//   -> Conv2d(6,16,5) -> LeakyReLU -> MaxPool2d(2) -> Conv2d(16,120,5) -> LeakyReLU
//   -> Linear(120,84) -> LeakyReLU -> Linear(84,10) -> Softmax, loss = nll_loss(probs) (train.py:48).
//
// The model is tiny (61,706 params, ~0.83 MFLOP/sample): on a 256-CU MI355X every op is latency
// bound, so the design goal is fewer, fatter kernels and fewer bytes, not MFMA tiling:
//   * lenet_stem_fwd: bilinear upsample 28->32 (align_corners) + conv1 5x5 + bias + LeakyReLU +
//     2x2 max-pool in ONE kernel, one workgroup per image, everything staged in LDS. The 32x32
//     upsampled image and the 6x28x28 pre-pool activations never touch HBM. Because LeakyReLU
//     is monotone, max(leaky(z)) == leaky(max(z)): the pool runs on raw conv outputs and only the
//     winner is activated. A 1-byte code per pooled output records the 2x2 argmax (bits 0-1) and
//     the winner's sign (bit 2) — everything backward needs (no int64 indices, no pre-pool tensor).
//   * lenet_stem_bwd: dW1/db1 straight from (dpooled, code, x): recomputes the upsampled image in
//     LDS, per-block partial sums into a slab, fixed-order finalize (deterministic). The input
//     needs no gradient (cnn.py:9 upsample of data), so conv1's dX is never formed.
//   * leaky_pool fwd/bwd: LeakyReLU + 2x2 max-pool (+ code byte) after conv2 (MIOpen); backward
//     writes the full pre-pool gradient in one pass (replaces aten's zero_ + scatter).
//   * softmax_nll_small: one wave per row for small class counts (V=10 here): log-softmax CE with
//     label smoothing, or the reference's NLL-on-probabilities (-p_y), fused with its backward
//     and with the eval metrics (sum loss, correct count accumulated on device — no per-batch
//     .item() like train.py:68-70).
#include "../common.h"

using namespace pdt;

namespace {

constexpr int kIn = 28, kUp = 32, kC1 = 6, kK = 5, kConv = 28, kPool = 14;
constexpr int kW1 = kC1 * kK * kK;  // 150 weights
constexpr int kStemPooled = kC1 * kPool * kPool;  // 1176

__device__ __forceinline__ float leaky(float z, float slope) { return z > 0.f ? z : z * slope; }

// align_corners=True bilinear 28 -> 32 of one image into LDS (torch upsample_bilinear2d semantics).
__device__ __forceinline__ void upsample_to_lds(const float* __restrict__ src, float* __restrict__ img,
                                                float* __restrict__ up) {
  for (int i = threadIdx.x; i < kIn * kIn; i += blockDim.x) img[i] = src[i];
  __syncthreads();
  const float r = (float)(kIn - 1) / (float)(kUp - 1);
  for (int i = threadIdx.x; i < kUp * kUp; i += blockDim.x) {
    const int oy = i / kUp, ox = i % kUp;
    const float sy = oy * r, sx = ox * r;
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = min(y0 + 1, kIn - 1), x1 = min(x0 + 1, kIn - 1);
    const float ly = sy - y0, lx = sx - x0;
    const float top = img[y0 * kIn + x0] * (1.f - lx) + img[y0 * kIn + x1] * lx;
    const float bot = img[y1 * kIn + x0] * (1.f - lx) + img[y1 * kIn + x1] * lx;
    up[i] = top * (1.f - ly) + bot * ly;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void lenet_stem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ b, float slope,
                                                             float* __restrict__ y, uint8_t* __restrict__ code) {
  __shared__ float img[kIn * kIn];
  __shared__ float up[kUp * kUp];
  __shared__ float sw[kW1 + kC1];
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < kW1 + kC1; i += blockDim.x) sw[i] = i < kW1 ? w[i] : b[i - kW1];
  upsample_to_lds(x + (int64_t)n * kIn * kIn, img, up);
  float* yo = y + (int64_t)n * kStemPooled;
  uint8_t* co = code + (int64_t)n * kStemPooled;
  for (int o = threadIdx.x; o < kStemPooled; o += blockDim.x) {
    const int c = o / (kPool * kPool), py = (o / kPool) % kPool, px = o % kPool;
    const float* wc = sw + c * kK * kK;
    // 2x2 window of conv outputs from a 6x6 input patch held in registers
    float patch[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int q = 0; q < 6; ++q) patch[r][q] = up[(2 * py + r) * kUp + 2 * px + q];
    float z[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1, dx = d & 1;
      float acc = sw[kW1 + c];
#pragma unroll
      for (int kh = 0; kh < kK; ++kh)
#pragma unroll
        for (int kw = 0; kw < kK; ++kw) acc = fmaf(wc[kh * kK + kw], patch[dy + kh][dx + kw], acc);
      z[d] = acc;
    }
    int am = 0;
    float zm = z[0];
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (z[d] > zm) { zm = z[d]; am = d; }  // first max wins, like aten's max_pool2d
    yo[o] = leaky(zm, slope);
    co[o] = (uint8_t)(am | (zm > 0.f ? 4 : 0));
  }
}

// Per-block partial dW1 (150) and db1 (6) over `ipb` images -> slab[blockIdx.x][156].
__global__ __launch_bounds__(256) void lenet_stem_bwd_kernel(const float* __restrict__ dy,
                                                             const uint8_t* __restrict__ code,
                                                             const float* __restrict__ x, int64_t N, int ipb,
                                                             float slope, float* __restrict__ slab) {
  __shared__ float img[kIn * kIn];
  __shared__ float up[kUp * kUp];
  __shared__ float dz[kStemPooled];
  __shared__ uint8_t pos[kStemPooled];
  const int t = threadIdx.x;
  float acc = 0.f;  // thread t < 156 owns one weight (t < 150) or one bias (150..155)
  const int c = t < kW1 ? t / (kK * kK) : t - kW1;
  const int kh = (t % (kK * kK)) / kK, kw = t % kK;
  for (int i = 0; i < ipb; ++i) {
    const int64_t n = (int64_t)blockIdx.x * ipb + i;
    if (n >= N) break;
    __syncthreads();  // previous image's LDS reads are done
    const float* dyn = dy + n * kStemPooled;
    const uint8_t* cn = code + n * kStemPooled;
    for (int o = t; o < kStemPooled; o += blockDim.x) {
      const uint8_t k = cn[o];
      dz[o] = dyn[o] * ((k & 4) ? 1.f : slope);
      pos[o] = k & 3;
    }
    upsample_to_lds(x + n * kIn * kIn, img, up);
    if (t < kW1 + kC1) {
      const float* dzc = dz + c * kPool * kPool;
      const uint8_t* pc = pos + c * kPool * kPool;
      if (t < kW1) {
        for (int p = 0; p < kPool * kPool; ++p) {
          const int py = p / kPool, px = p % kPool, a = pc[p];
          const int oy = 2 * py + (a >> 1), ox = 2 * px + (a & 1);
          acc = fmaf(dzc[p], up[(oy + kh) * kUp + ox + kw], acc);
        }
      } else {
        for (int p = 0; p < kPool * kPool; ++p) acc += dzc[p];
      }
    }
  }
  if (t < kW1 + kC1) slab[(int64_t)blockIdx.x * (kW1 + kC1) + t] = acc;
}

__global__ void slab_finalize_kernel(const float* __restrict__ slab, int nblk, int width, float* __restrict__ out_a,
                                     int na, float* __restrict__ out_b) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= width) return;
  float s = 0.f;
  for (int i = 0; i < nblk; ++i) s += slab[(int64_t)i * width + t];  // fixed order: deterministic
  if (t < na) out_a[t] = s;
  else out_b[t - na] = s;
}

// LeakyReLU + 2x2/2 max-pool over NCHW planes (floor mode). One thread per pooled output.
__global__ void leaky_pool_fwd_kernel(const float* __restrict__ x, int64_t planes, int H, int W, float slope,
                                      float* __restrict__ y, uint8_t* __restrict__ code) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = planes * Ho * Wo;
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pl = o / (Ho * Wo);
    const int r = (int)(o % (Ho * Wo)), py = r / Wo, px = r % Wo;
    const float* xp = x + pl * H * W + (2 * py) * W + 2 * px;
    const float z[4] = {xp[0], xp[1], xp[W], xp[W + 1]};
    int am = 0;
    float zm = z[0];
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (z[d] > zm) { zm = z[d]; am = d; }
    y[o] = leaky(zm, slope);
    code[o] = (uint8_t)(am | (zm > 0.f ? 4 : 0));
  }
}

// Full pre-pool gradient in one pass: each pooled output writes its 2x2 window (winner gets
// dy*leaky', the rest 0); odd trailing rows/cols (floor mode) are zeroed by the edge threads.
__global__ void leaky_pool_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ code, int64_t planes,
                                      int H, int W, float slope, float* __restrict__ dx) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = planes * Ho * Wo;
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pl = o / (Ho * Wo);
    const int r = (int)(o % (Ho * Wo)), py = r / Wo, px = r % Wo;
    const uint8_t k = code[o];
    const float g = dy[o] * ((k & 4) ? 1.f : slope);
    const int a = k & 3;
    float* dp = dx + pl * H * W + (2 * py) * W + 2 * px;
    dp[0] = a == 0 ? g : 0.f;
    dp[1] = a == 1 ? g : 0.f;
    dp[W] = a == 2 ? g : 0.f;
    dp[W + 1] = a == 3 ? g : 0.f;
    if ((W & 1) && px == Wo - 1) { dp[2] = 0.f; dp[W + 2] = 0.f; }
    if ((H & 1) && py == Ho - 1) {
      dp[2 * W] = 0.f; dp[2 * W + 1] = 0.f;
      if ((W & 1) && px == Wo - 1) dp[2 * W + 2] = 0.f;
    }
  }
}

// One wave per row, V <= 64 * kVPL classes held in registers.
// mode 0: cross-entropy with label smoothing (log-softmax NLL); mode 1: the reference's
// nll_loss on softmax probabilities, loss = -p_y (train.py:48).
// Writes per-row loss (optional), dlogits scaled by dscale (optional, fused backward: the
// gradient of the MEAN loss is produced in the same pass), and accumulates the eval metrics
// acc[0] += loss, acc[1] += (argmax == y), acc[2] += 1 (optional).
constexpr int kVPL = 16;
template <typename T>
__global__ __launch_bounds__(256) void softmax_nll_small_kernel(const T* __restrict__ logits,
                                                                const int64_t* __restrict__ target, int64_t N, int V,
                                                                int mode, float smoothing, float* __restrict__ loss,
                                                                T* __restrict__ dlogits, float dscale,
                                                                double* __restrict__ acc) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const T* x = logits + row * V;
  float v[kVPL];
  float m = -INFINITY, sum = 0.f;
  int am = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < kVPL; ++j) {
    const int i = j * 64 + lane;
    v[j] = i < V ? Elt<T>::ld(x, i) : -INFINITY;
    if (i < V) sum += v[j];
    if (v[j] > m) { m = v[j]; am = i; }
  }
  // wave argmax (first index among equal maxima, like torch.argmax)
  float wm = m;
  int wa = am;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(wm, off);
    const int oa = __shfl_xor(wa, off);
    if (om > wm || (om == wm && oa < wa)) { wm = om; wa = oa; }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < kVPL; ++j) s += (j * 64 + lane < V) ? __expf(v[j] - wm) : 0.f;
  s = wave_sum(s);
  sum = wave_sum(sum);
  const float lse = wm + __logf(s);
  const int64_t t = target[row];
  const float xt = __shfl(v[(int)(t >> 6) & (kVPL - 1)], (int)(t & 63));
  const float pt = __expf(xt - lse);
  float l;
  if (mode == 0) l = (1.f - smoothing) * (lse - xt) + smoothing * (lse - sum / (float)V);
  else l = -pt;
  if (lane == 0) {
    if (loss) loss[row] = l;
    if (acc) {
      atomicAdd(acc + 0, (double)l);
      atomicAdd(acc + 1, (double)(wa == t ? 1 : 0));
      atomicAdd(acc + 2, 1.0);
    }
  }
  if (dlogits) {
    T* dx = dlogits + row * V;
    const float sv = smoothing / (float)V;
#pragma unroll
    for (int j = 0; j < kVPL; ++j) {
      const int i = j * 64 + lane;
      if (i >= V) continue;
      const float p = __expf(v[j] - lse);
      float g;
      if (mode == 0) g = p - ((i == t ? 1.f - smoothing : 0.f) + sv);
      else g = -pt * ((i == t ? 1.f : 0.f) - p);  // d(-p_t)/dz_i = -p_t (delta_it - p_i)
      Elt<T>::st(dx, i, g * dscale);
    }
  }
}

// mean of n floats in a fixed order (one workgroup): the training loss of softmax_nll_small without a
// torch reduction launch per step.
__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ v, int64_t n, float scale,
                                                   float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1] + red[2] + red[3]) * scale;
}

}  // namespace

extern "C" {

// out[0] = scale * sum(v[0 .. n)), fixed order.
int pdt_mean_small(const float* v, int64_t n, float scale, float* out, hipStream_t s) {
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, v, n, scale, out);
  return 0;
}

int pdt_lenet_stem_fwd(const float* x, const float* w, const float* b, int64_t N, float slope, float* y,
                       uint8_t* code, hipStream_t s) {
  if (N == 0) return 0;
  hipLaunchKernelGGL(lenet_stem_fwd_kernel, dim3((unsigned)N), dim3(256), 0, s, x, w, b, slope, y, code);
  return 0;
}

int64_t pdt_lenet_stem_slab_floats(int64_t N, int ipb) { return ((N + ipb - 1) / ipb) * (kW1 + kC1); }

int pdt_lenet_stem_bwd(const float* dy, const uint8_t* code, const float* x, int64_t N, int ipb, float slope,
                       float* slab, float* dw, float* db, hipStream_t s) {
  const int nblk = (int)((N + ipb - 1) / ipb);
  if (N > 0)
    hipLaunchKernelGGL(lenet_stem_bwd_kernel, dim3(nblk), dim3(256), 0, s, dy, code, x, N, ipb, slope, slab);
  hipLaunchKernelGGL(slab_finalize_kernel, dim3(1), dim3(256), 0, s, slab, N > 0 ? nblk : 0, kW1 + kC1, dw, kW1,
                     db);
  return 0;
}

static unsigned grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 65535 ? 65535 : g));
}

int pdt_leaky_pool_fwd(const float* x, int64_t planes, int H, int W, float slope, float* y, uint8_t* code,
                       hipStream_t s) {
  const int64_t total = planes * (H / 2) * (W / 2);
  if (total == 0) return 0;
  hipLaunchKernelGGL(leaky_pool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, s, x, planes, H, W, slope, y, code);
  return 0;
}

int pdt_leaky_pool_bwd(const float* dy, const uint8_t* code, int64_t planes, int H, int W, float slope, float* dx,
                       hipStream_t s) {
  const int64_t total = planes * (H / 2) * (W / 2);
  if (total == 0) return 0;
  hipLaunchKernelGGL(leaky_pool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, s, dy, code, planes, H, W, slope,
                     dx);
  return 0;
}

int pdt_softmax_nll_small(const void* logits, int dtype, const int64_t* target, int64_t N, int V, int mode,
                          float smoothing, float* loss, void* dlogits, float dscale, double* acc, hipStream_t s) {
  if (V > 64 * kVPL) return 1;
  if (N == 0) return 0;
  const unsigned grid = (unsigned)((N + 3) / 4);
  if (dtype == 0)
    hipLaunchKernelGGL(softmax_nll_small_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)logits, target, N,
                       V, mode, smoothing, loss, (float*)dlogits, dscale, acc);
  else
    hipLaunchKernelGGL(softmax_nll_small_kernel<uint16_t>, dim3(grid), dim3(256), 0, s, (const uint16_t*)logits,
                       target, N, V, mode, smoothing, loss, (uint16_t*)dlogits, dscale, acc);
  return 0;
}

}  // extern "C"
