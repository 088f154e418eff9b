// Fused softmax cross-entropy (forward + backward) for gfx950.
//
// Reference: the LeNet head is Softmax followed by nll_loss on the probabilities
// (/root/reference/cnn.py:23, train.py:48). The framework trains with a proper
// log-softmax cross-entropy by default (reference behaviour stays available as
// loss='nll_on_probs'); for the north-star models (1000-way ImageNet, 50304-way GPT-2
// vocabulary) the loss is one pass over the logits: one workgroup per row computes the
// online max / sum-exp, the target logit and the mean logit (label smoothing), and stores
// the row's log-sum-exp. Backward recomputes softmax from the logits and LSE and writes
// dlogits = (softmax - smoothed one-hot) * dloss in the logits' dtype.
#include "../common.h"

using namespace pdt;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                     int64_t V, float smoothing, int64_t ignore_index,
                                                     float* __restrict__ loss, float* __restrict__ lse_out) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * V;
  float m = -INFINITY, s = 0.f, sum = 0.f;
  const bool vec = std::is_same<T, uint16_t>::value && (V % 8 == 0) && ((((uintptr_t)x) & 15) == 0);
  if (vec) {
    for (int64_t i = threadIdx.x * 8; i < V; i += 256 * 8) {
      float v[8];
      ld8_bf16(reinterpret_cast<const uint16_t*>(x) + i, v);
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
      const float nm = fmaxf(m, lm);
      s *= __expf(m - nm);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s += __expf(v[j] - nm); sum += v[j]; }
      m = nm;
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float v = Elt<T>::ld(x, i);
      const float nm = fmaxf(m, v);
      s = s * __expf(m - nm) + __expf(v - nm);
      m = nm;
      sum += v;
    }
  }
  // combine (m, s) across the block
  const float bm = block_max(m, red);
  float sc = (m == -INFINITY) ? 0.f : s * __expf(m - bm);
  const float bs = block_sum(sc, red);
  const float bsum = block_sum(sum, red);
  if (threadIdx.x == 0) {
    const int64_t t = target[row];
    const float lse = bm + __logf(bs);
    lse_out[row] = lse;
    if (t == ignore_index) {
      loss[row] = 0.f;
    } else {
      const float xt = Elt<T>::ld(x, t);
      const float nll = lse - xt;
      const float smooth = lse - bsum / (float)V;
      loss[row] = (1.f - smoothing) * nll + smoothing * smooth;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                     const float* __restrict__ lse, const float* __restrict__ dloss,
                                                     float dloss_scale, int64_t V, float smoothing,
                                                     int64_t ignore_index, T* __restrict__ dlogits) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * V;
  T* dx = dlogits + row * V;
  const int64_t t = target[row];
  const float g = (t == ignore_index) ? 0.f : (dloss ? dloss[row] : 1.f) * dloss_scale;
  const float l = lse[row];
  const float sv = smoothing / (float)V;
  const bool vec = std::is_same<T, uint16_t>::value && (V % 8 == 0) && ((((uintptr_t)x) & 15) == 0) &&
                   ((((uintptr_t)dx) & 15) == 0);
  if (vec) {
    for (int64_t i = threadIdx.x * 8; i < V; i += 256 * 8) {
      float v[8];
      ld8_bf16(reinterpret_cast<const uint16_t*>(x) + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __expf(v[j] - l);
        const float y = (i + j == t ? (1.f - smoothing) : 0.f) + sv;
        v[j] = (p - y) * g;
      }
      st8_bf16(reinterpret_cast<uint16_t*>(dx) + i, v);
    }
  } else {
    for (int64_t i = threadIdx.x; i < V; i += 256) {
      const float p = __expf(Elt<T>::ld(x, i) - l);
      const float y = (i == t ? (1.f - smoothing) : 0.f) + sv;
      Elt<T>::st(dx, i, (p - y) * g);
    }
  }
}

}  // namespace

extern "C" {

int pdt_ce_fwd(const void* logits, int dtype, const int64_t* target, int64_t N, int64_t V, float smoothing,
               int64_t ignore_index, float* loss, float* lse, hipStream_t s) {
  if (N == 0) return 0;
  if (dtype == 0)
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(N), dim3(256), 0, s, (const float*)logits, target, V, smoothing,
                       ignore_index, loss, lse);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<uint16_t>, dim3(N), dim3(256), 0, s, (const uint16_t*)logits, target, V,
                       smoothing, ignore_index, loss, lse);
  return 0;
}

int pdt_ce_bwd(const void* logits, int dtype, const int64_t* target, const float* lse, const float* dloss,
               float dloss_scale, int64_t N, int64_t V, float smoothing, int64_t ignore_index, void* dlogits,
               hipStream_t s) {
  if (N == 0) return 0;
  if (dtype == 0)
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(N), dim3(256), 0, s, (const float*)logits, target, lse, dloss,
                       dloss_scale, V, smoothing, ignore_index, (float*)dlogits);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<uint16_t>, dim3(N), dim3(256), 0, s, (const uint16_t*)logits, target, lse,
                       dloss, dloss_scale, V, smoothing, ignore_index, (uint16_t*)dlogits);
  return 0;
}

}  // extern "C"
