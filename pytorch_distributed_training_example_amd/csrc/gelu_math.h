// GELU and its derivative in short-latency gfx950 math, shared by the bias+GELU strip kernels
// (kernels/gelu.hip) and the fused GELU + fp8 cast kernels (kernels/fp8.hip) so both produce the
// same fp32 values bit for bit.
#pragma once

namespace pdt {

// tanh form through the logistic function: 0.5 (1 + tanh(u)) = 1 / (1 + e^(-2u)), evaluated as
// v_exp_f32 + v_rcp_f32 (a few ulp, far inside bf16) instead of ocml's tanhf: the strip kernels
// were partly VALU-bound on it (GPT-2's [8192, 4096] MLP activation: ~25 VALU ops per element).
// sigma(2u) saturates cleanly: e^(-2u) -> inf gives 0, -> 0 gives 1.
__device__ __forceinline__ float sig2u(float v) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * fmaf(k1 * v, v * v, v);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));  // e^(-2u) = 2^(-2u log2 e)
}
// erf for the exact (ViT) form, branch-free: Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 (far
// inside bf16 and the fp32 tests' 1e-5), one v_rcp_f32 + one v_exp_f32 + 5 FMAs instead of ocml's
// piecewise erff (divergent ranges per lane).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * ax * ax);  // e^(-x^2)
  return copysignf(fmaf(-p * t, e, 1.f), x);
}
__device__ __forceinline__ float gelu_f(float v, int tanh_form) {
  if (tanh_form) return v * sig2u(v);
  return 0.5f * v * (1.f + erf_fast(v * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_grad(float v, int tanh_form) {
  if (tanh_form) {  // d/dv [v s], s = sigma(2u): s + 2 v s (1 - s) u'
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float sg = sig2u(v);
    const float du = k0 * fmaf(3.f * k1 * v, v, 1.f);
    return fmaf(2.f * v * sg * (1.f - sg), du, sg);
  }
  const float cdf = 0.5f * (1.f + erf_fast(v * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.7213475204444817f * v * v);  // e^(-v^2/2)
  return cdf + v * pdf;
}

}  // namespace pdt
