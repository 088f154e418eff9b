// OCP e4m3fn (gfx950 fp8) packing shared by the cast kernels (kernels/fp8.hip) and the producers
// that emit fp8 directly (kernels/layernorm.hip).
#pragma once

namespace pdt {

constexpr float kE4M3Max = 448.f;

// Striped fp8 state rows (ops/fp8.py Fp8State): [amax, scale, scale_inv, pad, 16 amax stripes 16 floats
// (64 B) apart, history...]. A row of at least kAmaxRowMin floats is striped (the C API takes the flag).
constexpr int kAmaxStripes = 16, kAmaxStripe0 = 4, kAmaxStripeStride = 16;
constexpr int kAmaxHist = kAmaxStripe0 + kAmaxStripes * kAmaxStripeStride;  // 260: history offset
constexpr int kAmaxRowMin = kAmaxHist + 1;
__device__ __forceinline__ float* amax_slot(float* row, int striped, int wg) {
  return striped ? row + kAmaxStripe0 + (wg & (kAmaxStripes - 1)) * kAmaxStripeStride : row;
}

// 4 floats -> 4 saturated e4m3 bytes (byte i = value i), round to nearest even.
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = __builtin_amdgcn_fmed3f(a, kE4M3Max, -kE4M3Max);
  b = __builtin_amdgcn_fmed3f(b, kE4M3Max, -kE4M3Max);
  c = __builtin_amdgcn_fmed3f(c, kE4M3Max, -kE4M3Max);
  d = __builtin_amdgcn_fmed3f(d, kE4M3Max, -kE4M3Max);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);  // bytes 0,1
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);        // bytes 2,3
  return (uint32_t)w;
}

// Byte j of each of 4 words -> one word (byte i from word i): a 4 x 4 byte transpose column.
__device__ __forceinline__ uint32_t byte_col(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int j) {
  const int sh = 8 * j;
  return ((w0 >> sh) & 0xffu) | (((w1 >> sh) & 0xffu) << 8) | (((w2 >> sh) & 0xffu) << 16) | ((w3 >> sh) << 24);
}

}  // namespace pdt
