// The reference LeNet's layers after the stem — /root/reference/cnn.py:13-22:
//   Conv2d(6,16,5) -> LeakyReLU(0.2) -> MaxPool2d(2) -> Conv2d(16,120,5) -> LeakyReLU
//   -> flatten -> Linear(120,84) -> LeakyReLU -> Linear(84,10)            (logits; softmax + loss elsewhere)
// as ONE forward kernel and two backward kernels (fp32, like the reference), replacing 7 forward and
// ~15 backward library / aten launches (MIOpen convs, leaky_relu, max-pool, addmm, mm, sum) that each
// ran a few microseconds on a handful of CUs: at 128 images per GPU (the reference's 1024 over 8
// ranks, train.py:82) the LeNet step is launch and latency bound, so the win is fewer launches and
// no HBM round trips between layers, not matrix-core tiling.
//
//   lenet_tail_fwd : one workgroup per image. The stem's pooled output p1 [6,14,14] and conv2's
//                    weights sit in LDS; conv2 (16x10x10 outputs, 150 MACs each) -> 2x2 max-pool on the
//                    raw outputs + LeakyReLU of the winner (monotone: max(leaky z) = leaky(max z)) with a
//                    1-byte code (argmax, sign) -> conv3 as a 400-long dot per output (a wave per output,
//                    coalesced float4 weight rows) -> LeakyReLU -> fc1 -> LeakyReLU -> fc2.
//                    Saved for backward: code2, p2 [400], h3 [120], h4 [84] (activations AFTER LeakyReLU:
//                    their sign is the pre-activation's sign, all LeakyReLU backward needs).
//   lenet_tail_bwd : one workgroup per image: g4 = (fc2^T dl) * leaky'(h4), g3 = (fc1^T g4) * leaky'(h3),
//                    dp2 = w3^T g3, the pool-2 backward into dz2 [16,10,10] (LDS only), this image's conv2
//                    weight / bias gradient partial (fixed-size slab), and dp1 = conv2^T dz2 (the input
//                    gradient the stem's weight-gradient kernel consumes).
//   lenet_tail_wgrad : every remaining weight / bias gradient as a sum over the batch in index order
//                    (dW3 = sum_b g3 (x) p2, dfw1 = sum_b g4 (x) h3, dfw2 = sum_b dl (x) h4, the biases, and
//                    the conv2 slabs): deterministic, no atomics.
#include "../common.h"

using namespace pdt;

namespace {

constexpr int kC1 = 6, kP1 = 14, kC2 = 16, kO2 = 10, kP2 = 5, kK = 5;
constexpr int kIn1 = kC1 * kP1 * kP1;      // 1176
constexpr int kW2 = kC2 * kC1 * kK * kK;   // 2400
constexpr int kF3 = kC2 * kP2 * kP2;       // 400 = conv3 fan-in
constexpr int kC3 = 120, kH4 = 84, kOut = 10;
constexpr int kThreads = 256, kWaves = kThreads / 64;

__device__ __forceinline__ float leaky(float z, float s) { return z > 0.f ? z : z * s; }
__device__ __forceinline__ float dleaky(float h, float s) { return h > 0.f ? 1.f : s; }

// y[o] = b[o] + w[o, :] . x for `nout` outputs with fan-in `nin` (nin % 4 == 0): one wave per output,
// lanes reading consecutive float4 of the weight row (coalesced), wave sum. x in LDS.
__device__ __forceinline__ void wave_dots(const float* __restrict__ w, const float* __restrict__ b, const float* x,
                                          int nout, int nin, float* y, float slope) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n4 = nin / 4;
  for (int o = wid; o < nout; o += kWaves) {
    float acc = 0.f;
    for (int i = lane; i < n4; i += 64) {
      const float4 wv = reinterpret_cast<const float4*>(w + (int64_t)o * nin)[i];
      acc += wv.x * x[4 * i] + wv.y * x[4 * i + 1] + wv.z * x[4 * i + 2] + wv.w * x[4 * i + 3];
    }
    acc = wave_sum(acc);
    if (lane == 0) y[o] = leaky(acc + b[o], slope);
  }
}

struct TailW {
  const float *w2, *b2, *w3, *b3, *fw1, *fb1, *fw2, *fb2;
};

__global__ __launch_bounds__(kThreads) void lenet_tail_fwd_kernel(const float* __restrict__ p1g, TailW W, float slope,
                                                                  float* __restrict__ logits, uint8_t* __restrict__ code2,
                                                                  float* __restrict__ p2g, float* __restrict__ h3g,
                                                                  float* __restrict__ h4g) {
  __shared__ float p1[kIn1];
  __shared__ float w2[kW2];
  __shared__ float z2[kC2 * kO2 * kO2];
  __shared__ float p2[kF3];
  __shared__ float h3[kC3];
  __shared__ float h4[kH4];
  const int n = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < kIn1; i += kThreads) p1[i] = p1g[(int64_t)n * kIn1 + i];
  for (int i = t; i < kW2; i += kThreads) w2[i] = W.w2[i];
  __syncthreads();
  // conv2: output (o, y, x) = b2[o] + sum_{c,kh,kw} w2[o,c,kh,kw] p1[c, y+kh, x+kw]
  for (int q = t; q < kC2 * kO2 * kO2; q += kThreads) {
    const int o = q / (kO2 * kO2), y = (q / kO2) % kO2, x = q % kO2;
    float acc = W.b2[o];
#pragma unroll
    for (int c = 0; c < kC1; ++c)
#pragma unroll
      for (int kh = 0; kh < kK; ++kh)
#pragma unroll
        for (int kw = 0; kw < kK; ++kw)
          acc += w2[((o * kC1 + c) * kK + kh) * kK + kw] * p1[(c * kP1 + y + kh) * kP1 + x + kw];
    z2[q] = acc;
  }
  __syncthreads();
  // 2x2 max-pool of the raw conv outputs, LeakyReLU of the winner; code = argmax | (winner > 0) << 2
  for (int q = t; q < kF3; q += kThreads) {
    const int o = q / (kP2 * kP2), py = (q / kP2) % kP2, px = q % kP2;
    const float* base = z2 + (o * kO2 + 2 * py) * kO2 + 2 * px;
    float m = base[0];
    int am = 0;
    const float v1 = base[1], v2 = base[kO2], v3 = base[kO2 + 1];
    if (v1 > m) { m = v1; am = 1; }  // first maximum in scan order (aten's max_pool2d tie rule)
    if (v2 > m) { m = v2; am = 2; }
    if (v3 > m) { m = v3; am = 3; }
    const float h = leaky(m, slope);
    p2[q] = h;
    p2g[(int64_t)n * kF3 + q] = h;
    code2[(int64_t)n * kF3 + q] = (uint8_t)(am | (m > 0.f ? 4 : 0));
  }
  __syncthreads();
  wave_dots(W.w3, W.b3, p2, kC3, kF3, h3, slope);  // conv3 (5x5 over a 5x5 map = a dot of 400) + leaky
  __syncthreads();
  wave_dots(W.fw1, W.fb1, h3, kH4, kC3, h4, slope);  // fc1 + leaky
  __syncthreads();
  for (int i = t; i < kC3; i += kThreads) h3g[(int64_t)n * kC3 + i] = h3[i];
  for (int i = t; i < kH4; i += kThreads) h4g[(int64_t)n * kH4 + i] = h4[i];
  // fc2: 10 outputs of 84 (84 % 4 == 0), no activation
  {
    const int lane = t & 63, wid = t >> 6;
    for (int o = wid; o < kOut; o += kWaves) {
      float acc = 0.f;
      for (int i = lane; i < kH4 / 4; i += 64) {
        const float4 wv = reinterpret_cast<const float4*>(W.fw2 + o * kH4)[i];
        acc += wv.x * h4[4 * i] + wv.y * h4[4 * i + 1] + wv.z * h4[4 * i + 2] + wv.w * h4[4 * i + 3];
      }
      acc = wave_sum(acc);
      if (lane == 0) logits[(int64_t)n * kOut + o] = acc + W.fb2[o];
    }
  }
}

// Per-image backward. g4/g3 out (the batch-summed weight gradients are taken from them by
// lenet_tail_wgrad), the conv2 weight+bias partial of this image into slab [n][kW2 + kC2], dp1 out.
__global__ __launch_bounds__(kThreads) void lenet_tail_bwd_kernel(const float* __restrict__ dl, const float* __restrict__ p1g,
                                                                  TailW W, float slope, const uint8_t* __restrict__ code2,
                                                                  const float* __restrict__ h3g, const float* __restrict__ h4g,
                                                                  float* __restrict__ g4g, float* __restrict__ g3g,
                                                                  float* __restrict__ slab, float* __restrict__ dp1) {
  __shared__ float p1[kIn1];
  __shared__ float w2[kW2];
  __shared__ float dz2[kC2 * kO2 * kO2];
  __shared__ float dp2[kF3];
  __shared__ float g3[kC3];
  __shared__ float g4[kH4];
  __shared__ float d10[kOut];
  const int n = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < kIn1; i += kThreads) p1[i] = p1g[(int64_t)n * kIn1 + i];
  for (int i = t; i < kW2; i += kThreads) w2[i] = W.w2[i];
  for (int i = t; i < kC2 * kO2 * kO2; i += kThreads) dz2[i] = 0.f;
  if (t < kOut) d10[t] = dl[(int64_t)n * kOut + t];
  __syncthreads();
  // g4 = (fc2^T dl) * leaky'(h4)
  if (t < kH4) {
    float a = 0.f;
#pragma unroll
    for (int o = 0; o < kOut; ++o) a += W.fw2[o * kH4 + t] * d10[o];
    const float g = a * dleaky(h4g[(int64_t)n * kH4 + t], slope);
    g4[t] = g;
    g4g[(int64_t)n * kH4 + t] = g;
  }
  __syncthreads();
  // g3 = (fc1^T g4) * leaky'(h3)
  if (t < kC3) {
    float a = 0.f;
    for (int o = 0; o < kH4; ++o) a += W.fw1[o * kC3 + t] * g4[o];
    const float g = a * dleaky(h3g[(int64_t)n * kC3 + t], slope);
    g3[t] = g;
    g3g[(int64_t)n * kC3 + t] = g;
  }
  __syncthreads();
  // dp2 = w3^T g3 (threads read consecutive columns of each w3 row: coalesced)
  for (int k = t; k < kF3; k += kThreads) {
    float a = 0.f;
    for (int o = 0; o < kC3; ++o) a += W.w3[o * kF3 + k] * g3[o];
    dp2[k] = a;
  }
  __syncthreads();
  // pool-2 backward with LeakyReLU': the gradient goes to the window's argmax only (distinct
  // positions per pooled output: no write conflicts)
  for (int q = t; q < kF3; q += kThreads) {
    const int o = q / (kP2 * kP2), py = (q / kP2) % kP2, px = q % kP2;
    const unsigned c = code2[(int64_t)n * kF3 + q];
    const int am = c & 3;
    const float g = dp2[q] * ((c & 4) ? 1.f : slope);
    dz2[(o * kO2 + 2 * py + (am >> 1)) * kO2 + 2 * px + (am & 1)] = g;
  }
  __syncthreads();
  // conv2 weight / bias gradient of this image: dW2[o,c,kh,kw] = sum_{y,x} dz2[o,y,x] p1[c,y+kh,x+kw]
  float* sl = slab + (int64_t)n * (kW2 + kC2);
  for (int q = t; q < kW2; q += kThreads) {
    const int o = q / (kC1 * kK * kK), c = (q / (kK * kK)) % kC1, kh = (q / kK) % kK, kw = q % kK;
    float a = 0.f;
    for (int y = 0; y < kO2; ++y)
#pragma unroll
      for (int x = 0; x < kO2; ++x) a += dz2[(o * kO2 + y) * kO2 + x] * p1[(c * kP1 + y + kh) * kP1 + x + kw];
    sl[q] = a;
  }
  if (t < kC2) {
    float a = 0.f;
    for (int i = 0; i < kO2 * kO2; ++i) a += dz2[t * kO2 * kO2 + i];
    sl[kW2 + t] = a;
  }
  // dp1[c,y,x] = sum_{o,kh,kw} dz2[o, y-kh, x-kw] w2[o,c,kh,kw] (valid taps only)
  for (int q = t; q < kIn1; q += kThreads) {
    const int c = q / (kP1 * kP1), y = (q / kP1) % kP1, x = q % kP1;
    float a = 0.f;
    for (int o = 0; o < kC2; ++o)
#pragma unroll
      for (int kh = 0; kh < kK; ++kh) {
        const int yy = y - kh;
        if (yy < 0 || yy >= kO2) continue;
#pragma unroll
        for (int kw = 0; kw < kK; ++kw) {
          const int xx = x - kw;
          if (xx >= 0 && xx < kO2) a += dz2[(o * kO2 + yy) * kO2 + xx] * w2[((o * kC1 + c) * kK + kh) * kK + kw];
        }
      }
    dp1[(int64_t)n * kIn1 + q] = a;
  }
}

// Every batch-summed gradient, one output element per thread, batch order 0..N-1 (8 images per
// round, loads issued first). Segments of the flat index space:
//   [0, 2400) dW2 (conv2 slabs) | [.., +16) db2 | [.., +48000) dW3 = sum g3 (x) p2 | [.., +120) db3
//   | [.., +10080) dfw1 = sum g4 (x) h3 | [.., +84) dfb1 | [.., +840) dfw2 = sum dl (x) h4 | [.., +10) dfb2
struct TailG {
  float *dw2, *db2, *dw3, *db3, *dfw1, *dfb1, *dfw2, *dfb2;
};
constexpr int kSeg[9] = {0, kW2, kW2 + kC2, kW2 + kC2 + kC3 * kF3, kW2 + kC2 + kC3 * kF3 + kC3,
                         kW2 + kC2 + kC3 * kF3 + kC3 + kH4 * kC3, kW2 + kC2 + kC3 * kF3 + kC3 + kH4 * kC3 + kH4,
                         kW2 + kC2 + kC3 * kF3 + kC3 + kH4 * kC3 + kH4 + kOut * kH4,
                         kW2 + kC2 + kC3 * kF3 + kC3 + kH4 * kC3 + kH4 + kOut * kH4 + kOut};

// out = sum_b a[b*sa + ia] * (x ? x[b*sx + ix] : 1)
__device__ __forceinline__ float bsum(const float* __restrict__ a, int sa, int ia, const float* __restrict__ x, int sx,
                                      int ix, int N) {
  float s = 0.f;
  int b = 0;
  for (; b + 8 <= N; b += 8) {
    float va[8], vx[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      va[u] = a[(int64_t)(b + u) * sa + ia];
      vx[u] = x ? x[(int64_t)(b + u) * sx + ix] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += va[u] * vx[u];
  }
  for (; b < N; ++b) s += a[(int64_t)b * sa + ia] * (x ? x[(int64_t)b * sx + ix] : 1.f);
  return s;
}

__global__ __launch_bounds__(256) void lenet_tail_wgrad_kernel(const float* __restrict__ slab, const float* __restrict__ dl,
                                                               const float* __restrict__ g3, const float* __restrict__ g4,
                                                               const float* __restrict__ p2, const float* __restrict__ h3,
                                                               const float* __restrict__ h4, int N, TailG G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kSeg[8]) return;
  if (i < kSeg[1]) {
    G.dw2[i] = bsum(slab, kW2 + kC2, i, nullptr, 0, 0, N);
  } else if (i < kSeg[2]) {
    G.db2[i - kSeg[1]] = bsum(slab, kW2 + kC2, kW2 + i - kSeg[1], nullptr, 0, 0, N);
  } else if (i < kSeg[3]) {
    const int j = i - kSeg[2], o = j / kF3, k = j % kF3;
    G.dw3[j] = bsum(g3, kC3, o, p2, kF3, k, N);
  } else if (i < kSeg[4]) {
    G.db3[i - kSeg[3]] = bsum(g3, kC3, i - kSeg[3], nullptr, 0, 0, N);
  } else if (i < kSeg[5]) {
    const int j = i - kSeg[4], o = j / kC3, k = j % kC3;
    G.dfw1[j] = bsum(g4, kH4, o, h3, kC3, k, N);
  } else if (i < kSeg[6]) {
    G.dfb1[i - kSeg[5]] = bsum(g4, kH4, i - kSeg[5], nullptr, 0, 0, N);
  } else if (i < kSeg[7]) {
    const int j = i - kSeg[6], o = j / kH4, k = j % kH4;
    G.dfw2[j] = bsum(dl, kOut, o, h4, kH4, k, N);
  } else {
    G.dfb2[i - kSeg[7]] = bsum(dl, kOut, i - kSeg[7], nullptr, 0, 0, N);
  }
}

}  // namespace

extern "C" {

// Forward of the LeNet tail for N images. p1: [N,6,14,14] (the stem's pooled output); weights in
// the nn.Module layouts (w2 [16,6,5,5], w3 [120,16,5,5], fw1 [84,120], fw2 [10,84], contiguous fp32).
// Outputs: logits [N,10]; saved code2 [N,400] bytes, p2 [N,400], h3 [N,120], h4 [N,84].
int pdt_lenet_tail_fwd(const float* p1, const float* w2, const float* b2, const float* w3, const float* b3,
                       const float* fw1, const float* fb1, const float* fw2, const float* fb2, float slope, int N,
                       float* logits, uint8_t* code2, float* p2, float* h3, float* h4, hipStream_t s) {
  if (N < 1) return N == 0 ? 0 : -1;
  const TailW W{w2, b2, w3, b3, fw1, fb1, fw2, fb2};
  hipLaunchKernelGGL(lenet_tail_fwd_kernel, dim3(N), dim3(kThreads), 0, s, p1, W, slope, logits, code2, p2, h3, h4);
  return 0;
}

// Floats of the backward workspace: g4 [N,84] + g3 [N,120] + conv2 slabs [N, 2416].
int64_t pdt_lenet_tail_ws_floats(int N) { return (int64_t)N * (kH4 + kC3 + kW2 + kC2); }

// Backward from dl = d loss / d logits [N,10]: every tail parameter's gradient (same layouts as the
// weights) and dp1 [N,6,14,14], the gradient of the stem's pooled output.
int pdt_lenet_tail_bwd(const float* dl, const float* p1, const float* w2, const float* b2, const float* w3,
                       const float* b3, const float* fw1, const float* fb1, const float* fw2, const float* fb2,
                       float slope, int N, const uint8_t* code2, const float* p2, const float* h3, const float* h4,
                       float* ws, float* dp1, float* dw2, float* db2, float* dw3, float* db3, float* dfw1, float* dfb1,
                       float* dfw2, float* dfb2, hipStream_t s) {
  if (N < 1) return -1;
  const TailW W{w2, b2, w3, b3, fw1, fb1, fw2, fb2};
  float* g4 = ws;
  float* g3 = g4 + (int64_t)N * kH4;
  float* slab = g3 + (int64_t)N * kC3;
  hipLaunchKernelGGL(lenet_tail_bwd_kernel, dim3(N), dim3(kThreads), 0, s, dl, p1, W, slope, code2, h3, h4, g4, g3,
                     slab, dp1);
  const TailG G{dw2, db2, dw3, db3, dfw1, dfb1, dfw2, dfb2};
  hipLaunchKernelGGL(lenet_tail_wgrad_kernel, dim3((kSeg[8] + 255) / 256), dim3(256), 0, s, slab, dl, g3, g4, p2, h3, h4,
                     N, G);
  return 0;
}

}  // extern "C"
