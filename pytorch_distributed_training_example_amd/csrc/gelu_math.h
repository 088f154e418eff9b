// GELU and its derivative in short-latency gfx950 math, shared by the bias+GELU strip kernels
// (kernels/gelu.hip) and the fused GELU + fp8 cast kernels (kernels/fp8.hip) so both produce the
// same fp32 values bit for bit.
#pragma once

namespace pdt {

// Evaluated on PAIRS of values (two fp32 lanes per VGPR pair): the multiply / FMA chains issue as
// gfx950's packed v_pk_mul_f32 / v_pk_fma_f32 (two results per instruction; the transcendental
// v_exp_f32 / v_rcp_f32 stay per value). Per-lane IEEE results equal the scalar forms, and every
// kernel that evaluates GELU (bias+GELU strips, the fp8 GELU casts) calls these, so all of them
// produce the same bits.
typedef float gf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gf2 g2(float a) { return gf2{a, a}; }
__device__ __forceinline__ gf2 fma2(gf2 a, gf2 b, gf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ gf2 rcp2(gf2 a) { return gf2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }
__device__ __forceinline__ gf2 exp2_2(gf2 a) { return gf2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)}; }

// tanh form through the logistic function: 0.5 (1 + tanh(u)) = 1 / (1 + e^(-2u)), evaluated as
// v_exp_f32 + v_rcp_f32 (a few ulp, far inside bf16) instead of ocml's tanhf: the strip kernels
// were partly VALU-bound on it (GPT-2's [8192, 4096] MLP activation: ~25 VALU ops per element).
// sigma(2u) saturates cleanly: e^(-2u) -> inf gives 0, -> 0 gives 1.
__device__ __forceinline__ gf2 sig2u2(gf2 v) {
  const gf2 u = g2(0.7978845608028654f) * fma2(g2(0.044715f) * v, v * v, v);
  return rcp2(g2(1.f) + exp2_2(g2(-2.8853900817779268f) * u));  // e^(-2u) = 2^(-2u log2 e)
}
// erf for the exact (ViT) form, branch-free: Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 (far
// inside bf16 and the fp32 tests' 1e-5), one v_rcp_f32 + one v_exp_f32 + 5 FMAs per value instead
// of ocml's piecewise erff (divergent ranges per lane).
__device__ __forceinline__ gf2 erf_fast2(gf2 x) {
  const gf2 ax = __builtin_elementwise_abs(x);
  const gf2 t = rcp2(fma2(g2(0.3275911f), ax, g2(1.f)));
  gf2 p = fma2(g2(1.061405429f), t, g2(-1.453152027f));
  p = fma2(p, t, g2(1.421413741f));
  p = fma2(p, t, g2(-0.284496736f));
  p = fma2(p, t, g2(0.254829592f));
  const gf2 e = exp2_2(g2(-1.4426950408889634f) * ax * ax);  // e^(-x^2)
  return __builtin_elementwise_copysign(fma2(-p * t, e, g2(1.f)), x);
}
__device__ __forceinline__ gf2 gelu2(gf2 v, int tanh_form) {
  if (tanh_form) return v * sig2u2(v);
  return g2(0.5f) * v * (g2(1.f) + erf_fast2(v * g2(0.7071067811865476f)));
}
__device__ __forceinline__ gf2 gelu_grad2(gf2 v, int tanh_form) {
  if (tanh_form) {  // d/dv [v s], s = sigma(2u): s + 2 v s (1 - s) u'
    const gf2 sg = sig2u2(v);
    const gf2 du = g2(0.7978845608028654f) * fma2(g2(3.f * 0.044715f) * v, v, g2(1.f));
    return fma2(g2(2.f) * v * sg * (g2(1.f) - sg), du, sg);
  }
  const gf2 cdf = g2(0.5f) * (g2(1.f) + erf_fast2(v * g2(0.7071067811865476f)));
  const gf2 pdf = g2(0.3989422804014327f) * exp2_2(g2(-0.7213475204444817f) * v * v);  // e^(-v^2/2)
  return fma2(v, pdf, cdf);
}

}  // namespace pdt
