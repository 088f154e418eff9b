// Fused multi-tensor optimizers for gfx950: SGD(momentum/nesterov/wd), Adam/AdamW, Adadelta.
//
// Reference: /root/reference/train.py:99 uses torch.optim.Adadelta (math at
// torch/optim/adadelta.py:386-399, ~7 _foreach_ launches/step); the north-star configs need
// SGD (ResNet-50) and AdamW (ViT/GPT-2). One kernel per ≤320×32Ki-element chunk set reads
// param, grad and states once and writes them once. Mixed precision: parameters may be an
// fp32 master copy with a bf16 model copy written in the same pass (no separate cast
// kernel), gradients fp32 or bf16 (e.g. straight out of a bf16 DDP bucket). lr, the AMP
// inverse scale, the inf flag and the Adam step come from device memory so a captured
// hipGraph replays with the current values.
#include "../multi_tensor.h"

using namespace pdt;

namespace {

struct Common {
  float lr;
  const float* lr_ptr;
  const float* inv_scale;   // optional: grads are multiplied by *inv_scale
  const float* found_inf;   // optional: skip the step when *found_inf != 0
  float wd;
  int maximize;
  __device__ __forceinline__ bool enabled() const { return !(found_inf && *found_inf != 0.f); }
  __device__ __forceinline__ float get_lr() const { return lr_ptr ? *lr_ptr : lr; }
  __device__ __forceinline__ float gscale() const {
    float s = inv_scale ? *inv_scale : 1.f;
    return maximize ? -s : s;
  }
};

// ---------------------------------------------------------------- SGD
// lists: 0 param (P), 1 grad (G), 2 momentum buf (f32, may be null), 3 model copy (bf16, may be null)
template <typename P, typename G>
struct SGDOp {
  Common c;
  float momentum, dampening;
  int nesterov, first;
  __device__ bool enabled() const { return c.enabled(); }
  __device__ __forceinline__ void step(float& p, float g, float& b, bool has_buf, float lr) const {
    if (c.wd != 0.f) g += c.wd * p;
    if (has_buf) {
      b = first ? g : momentum * b + (1.f - dampening) * g;
      g = nesterov ? g + momentum * b : b;
    }
    p -= lr * g;
  }
  __device__ void vec4(MTMeta<4>& m, int t, int64_t i) const {
    const float lr = c.get_lr(), sc = c.gscale();
    float p[4], g[4], b[4] = {0, 0, 0, 0};
    Vec4<P>::ld((P*)m.ptr[0][t], i, p);
    Vec4<G>::ld((G*)m.ptr[1][t], i, g);
    float* bp = (float*)m.ptr[2][t];
    if (bp && !first) Vec4<float>::ld(bp, i, b);
#pragma unroll
    for (int k = 0; k < 4; ++k) step(p[k], g[k] * sc, b[k], bp != nullptr, lr);
    Vec4<P>::st((P*)m.ptr[0][t], i, p);
    if (bp) Vec4<float>::st(bp, i, b);
    if (m.ptr[3][t]) Vec4<uint16_t>::st((uint16_t*)m.ptr[3][t], i, p);
  }
  __device__ void scalar(MTMeta<4>& m, int t, int64_t i) const {
    const float lr = c.get_lr(), sc = c.gscale();
    float p = Elt<P>::ld((P*)m.ptr[0][t], i), g = Elt<G>::ld((G*)m.ptr[1][t], i) * sc, b = 0.f;
    float* bp = (float*)m.ptr[2][t];
    if (bp && !first) b = bp[i];
    step(p, g, b, bp != nullptr, lr);
    Elt<P>::st((P*)m.ptr[0][t], i, p);
    if (bp) bp[i] = b;
    if (m.ptr[3][t]) Elt<uint16_t>::st((uint16_t*)m.ptr[3][t], i, p);
  }
  __device__ void finish(MTMeta<4>&, int) const {}
};

// ---------------------------------------------------------------- Adam / AdamW
// lists: 0 param, 1 grad, 2 exp_avg (f32), 3 exp_avg_sq (f32), 4 model copy (bf16, may be null)
template <typename P, typename G>
struct AdamOp {
  Common c;
  float beta1, beta2, eps;
  const float* step_ptr;  // step count AFTER increment (device)
  float step_host;
  int decoupled;          // 1 = AdamW
  __device__ bool enabled() const { return c.enabled(); }
  __device__ __forceinline__ void coef(float& lr, float& step_size, float& bc2s) const {
    lr = c.get_lr();
    const float st = step_ptr ? *step_ptr : step_host;
    const float bc1 = 1.f - powf(beta1, st);
    const float bc2 = 1.f - powf(beta2, st);
    step_size = lr / bc1;
    bc2s = sqrtf(bc2);
  }
  __device__ __forceinline__ void step(float& p, float g, float& m, float& v, float lr,
                                       float step_size, float bc2s) const {
    if (decoupled) p *= (1.f - lr * c.wd);
    else if (c.wd != 0.f) g += c.wd * p;
    m = m + (1.f - beta1) * (g - m);
    v = beta2 * v + (1.f - beta2) * g * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p -= step_size * (m / denom);
  }
  __device__ void vec4(MTMeta<5>& mm, int t, int64_t i) const {
    float lr, ss, b2;
    coef(lr, ss, b2);
    const float sc = c.gscale();
    float p[4], g[4], m[4], v[4];
    Vec4<P>::ld((P*)mm.ptr[0][t], i, p);
    Vec4<G>::ld((G*)mm.ptr[1][t], i, g);
    Vec4<float>::ld((float*)mm.ptr[2][t], i, m);
    Vec4<float>::ld((float*)mm.ptr[3][t], i, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) step(p[k], g[k] * sc, m[k], v[k], lr, ss, b2);
    Vec4<P>::st((P*)mm.ptr[0][t], i, p);
    Vec4<float>::st((float*)mm.ptr[2][t], i, m);
    Vec4<float>::st((float*)mm.ptr[3][t], i, v);
    if (mm.ptr[4][t]) Vec4<uint16_t>::st((uint16_t*)mm.ptr[4][t], i, p);
  }
  __device__ void scalar(MTMeta<5>& mm, int t, int64_t i) const {
    float lr, ss, b2;
    coef(lr, ss, b2);
    float p = Elt<P>::ld((P*)mm.ptr[0][t], i), g = Elt<G>::ld((G*)mm.ptr[1][t], i) * c.gscale();
    float* mp = (float*)mm.ptr[2][t];
    float* vp = (float*)mm.ptr[3][t];
    float m = mp[i], v = vp[i];
    step(p, g, m, v, lr, ss, b2);
    Elt<P>::st((P*)mm.ptr[0][t], i, p);
    mp[i] = m;
    vp[i] = v;
    if (mm.ptr[4][t]) Elt<uint16_t>::st((uint16_t*)mm.ptr[4][t], i, p);
  }
  __device__ void finish(MTMeta<5>&, int) const {}
};

// ---------------------------------------------------------------- Adadelta (the reference's optimizer)
// lists: 0 param, 1 grad, 2 square_avg (f32), 3 acc_delta (f32), 4 model copy (bf16, may be null)
template <typename P, typename G>
struct AdadeltaOp {
  Common c;
  float rho, eps;
  __device__ bool enabled() const { return c.enabled(); }
  __device__ __forceinline__ void step(float& p, float g, float& sa, float& ad, float lr) const {
    if (c.wd != 0.f) g += c.wd * p;
    sa = sa * rho + (1.f - rho) * g * g;
    const float std_ = sqrtf(sa + eps);
    const float delta = sqrtf(ad + eps) / std_ * g;
    ad = ad * rho + (1.f - rho) * delta * delta;
    p -= lr * delta;
  }
  __device__ void vec4(MTMeta<5>& mm, int t, int64_t i) const {
    const float lr = c.get_lr(), sc = c.gscale();
    float p[4], g[4], sa[4], ad[4];
    Vec4<P>::ld((P*)mm.ptr[0][t], i, p);
    Vec4<G>::ld((G*)mm.ptr[1][t], i, g);
    Vec4<float>::ld((float*)mm.ptr[2][t], i, sa);
    Vec4<float>::ld((float*)mm.ptr[3][t], i, ad);
#pragma unroll
    for (int k = 0; k < 4; ++k) step(p[k], g[k] * sc, sa[k], ad[k], lr);
    Vec4<P>::st((P*)mm.ptr[0][t], i, p);
    Vec4<float>::st((float*)mm.ptr[2][t], i, sa);
    Vec4<float>::st((float*)mm.ptr[3][t], i, ad);
    if (mm.ptr[4][t]) Vec4<uint16_t>::st((uint16_t*)mm.ptr[4][t], i, p);
  }
  __device__ void scalar(MTMeta<5>& mm, int t, int64_t i) const {
    const float lr = c.get_lr();
    float p = Elt<P>::ld((P*)mm.ptr[0][t], i), g = Elt<G>::ld((G*)mm.ptr[1][t], i) * c.gscale();
    float* sp = (float*)mm.ptr[2][t];
    float* ap = (float*)mm.ptr[3][t];
    float sa = sp[i], ad = ap[i];
    step(p, g, sa, ad, lr);
    Elt<P>::st((P*)mm.ptr[0][t], i, p);
    sp[i] = sa;
    ap[i] = ad;
    if (mm.ptr[4][t]) Elt<uint16_t>::st((uint16_t*)mm.ptr[4][t], i, p);
  }
  __device__ void finish(MTMeta<5>&, int) const {}
};

// dtype codes shared with the binding: 0 = fp32, 1 = bf16
template <template <typename, typename> class OP, int NL, typename Fill>
int dispatch(int pd, int gd, int n, void* const* lists[NL], const int64_t* numel, Fill fill,
             hipStream_t s) {
#define PDT_CASE(PT, GT)                  \
  {                                       \
    OP<PT, GT> op;                        \
    fill(op);                             \
    mt_launch<NL>(n, lists, numel, op, s); \
    return 0;                             \
  }
  if (pd == 0 && gd == 0) PDT_CASE(float, float)
  if (pd == 0 && gd == 1) PDT_CASE(float, uint16_t)
  if (pd == 1 && gd == 1) PDT_CASE(uint16_t, uint16_t)
  if (pd == 1 && gd == 0) PDT_CASE(uint16_t, float)
#undef PDT_CASE
  return -1;
}

}  // namespace

extern "C" {

int pdt_sgd(int n, void* const* p, void* const* g, void* const* buf, void* const* copy,
            const int64_t* numel, int p_dtype, int g_dtype, float lr, const float* lr_ptr,
            float momentum, float dampening, float wd, int nesterov, int first, int maximize,
            const float* inv_scale, const float* found_inf, hipStream_t s) {
  void* const* lists[4] = {p, g, buf, copy};
  return dispatch<SGDOp, 4>(p_dtype, g_dtype, n, lists, numel, [&](auto& op) {
    op.c = Common{lr, lr_ptr, inv_scale, found_inf, wd, maximize};
    op.momentum = momentum;
    op.dampening = dampening;
    op.nesterov = nesterov;
    op.first = first;
  }, s);
}

int pdt_adam(int n, void* const* p, void* const* g, void* const* m, void* const* v,
             void* const* copy, const int64_t* numel, int p_dtype, int g_dtype, float lr,
             const float* lr_ptr, float beta1, float beta2, float eps, float wd, int decoupled,
             const float* step_ptr, float step_host, int maximize, const float* inv_scale,
             const float* found_inf, hipStream_t s) {
  void* const* lists[5] = {p, g, m, v, copy};
  return dispatch<AdamOp, 5>(p_dtype, g_dtype, n, lists, numel, [&](auto& op) {
    op.c = Common{lr, lr_ptr, inv_scale, found_inf, wd, maximize};
    op.beta1 = beta1;
    op.beta2 = beta2;
    op.eps = eps;
    op.step_ptr = step_ptr;
    op.step_host = step_host;
    op.decoupled = decoupled;
  }, s);
}

int pdt_adadelta(int n, void* const* p, void* const* g, void* const* sa, void* const* ad,
                 void* const* copy, const int64_t* numel, int p_dtype, int g_dtype, float lr,
                 const float* lr_ptr, float rho, float eps, float wd, int maximize,
                 const float* inv_scale, const float* found_inf, hipStream_t s) {
  void* const* lists[5] = {p, g, sa, ad, copy};
  return dispatch<AdadeltaOp, 5>(p_dtype, g_dtype, n, lists, numel, [&](auto& op) {
    op.c = Common{lr, lr_ptr, inv_scale, found_inf, wd, maximize};
    op.rho = rho;
    op.eps = eps;
  }, s);
}

}  // extern "C"
