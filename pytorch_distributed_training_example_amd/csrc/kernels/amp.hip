// AMP and gradient-buffer kernels (multi-tensor, graph-capture safe).
//
//  * pdt_amp_unscale   : g *= *inv_scale in place; *found_inf = 1 if any non-finite
//                        (one launch for all gradients instead of torch's per-dtype foreach
//                        + separate inf check).
//  * pdt_amp_update    : dynamic loss-scale update (backoff on inf, growth after N clean
//                        steps), entirely on device so no host readback per step.
//  * pdt_l2norm_sq     : sum of squares over many tensors (grad clipping), block partials
//                        + one float atomic per workgroup.
//  * pdt_clip_coef     : coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) on device.
//  * pdt_mt_scale      : x *= *scale (apply clip coefficient / averaging factor).
//  * pdt_mt_copy       : dst = src * scale with dtype conversion (bucket flatten/unflatten,
//                        fp32 <-> bf16 reduction buffers), 1/world folded in.
#include "../multi_tensor.h"

using namespace pdt;

namespace {

template <typename T>
struct UnscaleOp {
  const float* inv_scale;
  float* found_inf;
  __device__ bool enabled() const { return true; }
  __device__ void vec4(MTMeta<1>& m, int t, int64_t i) const {
    float v[4];
    Vec4<T>::ld((T*)m.ptr[0][t], i, v);
    const float s = *inv_scale;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) { bad |= !isfinite(v[k]); v[k] *= s; }
    if (bad) *found_inf = 1.f;
    Vec4<T>::st((T*)m.ptr[0][t], i, v);
  }
  __device__ void scalar(MTMeta<1>& m, int t, int64_t i) const {
    float v = Elt<T>::ld((T*)m.ptr[0][t], i);
    if (!isfinite(v)) *found_inf = 1.f;
    Elt<T>::st((T*)m.ptr[0][t], i, v * *inv_scale);
  }
  __device__ void finish(MTMeta<1>&, int) const {}
};

template <typename T>
struct ScaleOp {
  const float* scale_ptr;
  float scale;
  __device__ bool enabled() const { return true; }
  __device__ float s() const { return scale_ptr ? *scale_ptr * scale : scale; }
  __device__ void vec4(MTMeta<1>& m, int t, int64_t i) const {
    float v[4];
    Vec4<T>::ld((T*)m.ptr[0][t], i, v);
    const float k = s();
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= k;
    Vec4<T>::st((T*)m.ptr[0][t], i, v);
  }
  __device__ void scalar(MTMeta<1>& m, int t, int64_t i) const {
    Elt<T>::st((T*)m.ptr[0][t], i, Elt<T>::ld((T*)m.ptr[0][t], i) * s());
  }
  __device__ void finish(MTMeta<1>&, int) const {}
};

template <typename S, typename D>
struct CopyOp {
  const float* scale_ptr;
  float scale;
  __device__ bool enabled() const { return true; }
  __device__ float s() const { return scale_ptr ? *scale_ptr * scale : scale; }
  __device__ void vec4(MTMeta<2>& m, int t, int64_t i) const {
    float v[4];
    Vec4<S>::ld((S*)m.ptr[0][t], i, v);
    const float k = s();
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= k;
    Vec4<D>::st((D*)m.ptr[1][t], i, v);
  }
  __device__ void scalar(MTMeta<2>& m, int t, int64_t i) const {
    Elt<D>::st((D*)m.ptr[1][t], i, Elt<S>::ld((S*)m.ptr[0][t], i) * s());
  }
  __device__ void finish(MTMeta<2>&, int) const {}
};

template <typename T>
__global__ __launch_bounds__(256) void l2norm_kernel(MTMeta<1> meta, float* out) {
  __shared__ float red[4];
  const int t = mt_find(meta, blockIdx.x);
  const int64_t c = blockIdx.x - meta.chunk_start[t];
  const int64_t n = meta.numel[t];
  const int64_t start = c * PDT_MT_CHUNK;
  const int64_t end = start + PDT_MT_CHUNK < n ? start + PDT_MT_CHUNK : n;
  const T* p = (const T*)meta.ptr[0][t];
  float acc = 0.f;
  if ((((uintptr_t)p) & 15) == 0) {
    int64_t vend = start + ((end - start) & ~(int64_t)3);
    for (int64_t i = start + threadIdx.x * 4; i < vend; i += 1024) {
      float v[4];
      Vec4<T>::ld(p, i, v);
      acc += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += 256) { float v = Elt<T>::ld(p, i); acc += v * v; }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += 256) { float v = Elt<T>::ld(p, i); acc += v * v; }
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

__global__ void amp_update_kernel(float* scale, int* growth_tracker, const float* found_inf,
                                  float growth, float backoff, int interval) {
  if (*found_inf != 0.f) {
    *scale = *scale * backoff;
    *growth_tracker = 0;
  } else {
    int g = *growth_tracker + 1;
    if (g == interval) {
      float ns = *scale * growth;
      if (isfinite(ns)) *scale = ns;
      g = 0;
    }
    *growth_tracker = g;
  }
}

__global__ void clip_coef_kernel(const float* sumsq, float max_norm, float* coef, float* norm) {
  const float nrm = sqrtf(*sumsq);
  if (norm) *norm = nrm;
  const float c = max_norm / (nrm + 1e-6f);
  *coef = c < 1.f ? c : 1.f;
}

template <int NL, template <typename> class OP, typename Fill>
int dispatch1(int dt, int n, void* const* lists[NL], const int64_t* numel, Fill fill, hipStream_t s) {
  if (dt == 0) { OP<float> op; fill(op); mt_launch<NL>(n, lists, numel, op, s); return 0; }
  if (dt == 1) { OP<uint16_t> op; fill(op); mt_launch<NL>(n, lists, numel, op, s); return 0; }
  return -1;
}

}  // namespace

extern "C" {

int pdt_amp_unscale(int n, void* const* g, const int64_t* numel, int dtype, const float* inv_scale,
                    float* found_inf, hipStream_t s) {
  void* const* lists[1] = {g};
  return dispatch1<1, UnscaleOp>(dtype, n, lists, numel, [&](auto& op) {
    op.inv_scale = inv_scale;
    op.found_inf = found_inf;
  }, s);
}

int pdt_amp_update(float* scale, int* growth_tracker, const float* found_inf, float growth,
                   float backoff, int interval, hipStream_t s) {
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(1), 0, s, scale, growth_tracker, found_inf,
                     growth, backoff, interval);
  return 0;
}

int pdt_mt_scale(int n, void* const* x, const int64_t* numel, int dtype, const float* scale_ptr,
                 float scale, hipStream_t s) {
  void* const* lists[1] = {x};
  return dispatch1<1, ScaleOp>(dtype, n, lists, numel, [&](auto& op) {
    op.scale_ptr = scale_ptr;
    op.scale = scale;
  }, s);
}

int pdt_mt_copy(int n, void* const* src, void* const* dst, const int64_t* numel, int sdt, int ddt,
                const float* scale_ptr, float scale, hipStream_t s) {
  void* const* lists[2] = {src, dst};
#define PDT_COPY(ST, DT)                                    \
  {                                                         \
    CopyOp<ST, DT> op;                                      \
    op.scale_ptr = scale_ptr;                               \
    op.scale = scale;                                       \
    mt_launch<2>(n, lists, numel, op, s);                   \
    return 0;                                               \
  }
  if (sdt == 0 && ddt == 0) PDT_COPY(float, float)
  if (sdt == 0 && ddt == 1) PDT_COPY(float, uint16_t)
  if (sdt == 1 && ddt == 0) PDT_COPY(uint16_t, float)
  if (sdt == 1 && ddt == 1) PDT_COPY(uint16_t, uint16_t)
#undef PDT_COPY
  return -1;
}

int pdt_l2norm_sq(int n, void* const* x, const int64_t* numel, int dtype, float* out, hipStream_t s) {
  hipMemsetAsync(out, 0, sizeof(float), s);
  void* const* lists[1] = {x};
  mt_batches<1>(n, lists, numel, [&](const MTMeta<1>& meta, int nblocks) {
    if (dtype == 0) hipLaunchKernelGGL(l2norm_kernel<float>, dim3(nblocks), dim3(256), 0, s, meta, out);
    else hipLaunchKernelGGL(l2norm_kernel<uint16_t>, dim3(nblocks), dim3(256), 0, s, meta, out);
  });
  return 0;
}

int pdt_clip_coef(const float* sumsq, float max_norm, float* coef, float* norm, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, s, sumsq, max_norm, coef, norm);
  return 0;
}

}  // extern "C"
