// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, 64-bit ballots; wave width is hard-coded to 64.
//   * bf16 is carried as raw uint16_t in memory (vector loads of 8 B / 16 B per lane) and
//     converted with the native __bf16 cast (lowers to v_cvt_pk_bf16_f32 on gfx950, which
//     keeps NaNs NaN and rounds to nearest-even).
//   * every kernel has a C-ABI launcher `pdt_<op>(..., hipStream_t)` that is graph-capture
//     safe: no allocation, no sync, no host readback; scalars that change step to step
//     (lr, loss scale, step count) are read from device memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#define PDT_WAVE 64

#include <stdlib.h>

namespace pdt {

// Small grids (the reference's 128 images per rank at the 8-GPU point, ResNet layers 3-4): a conv whose
// wide-tile grid gives fewer than one workgroup per CU takes the half-width tile instead (twice the
// workgroups). PDT_SMALL_GRID_NARROW = the workgroup threshold (default 256 = one per CU; 0 = off),
// read once per process.
inline bool small_grid_narrow(int64_t wide_blocks) {
  static const int64_t thr = [] {
    const char* e = getenv("PDT_SMALL_GRID_NARROW");
    if (!e || !e[0]) return (int64_t)256;
    const long v = strtol(e, nullptr, 10);
    return (int64_t)(v == 1 ? 256 : (v < 0 ? 0 : v));  // "1" kept as "on" (earlier A/B scripts)
  }();
  return wide_blocks < thr;
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// Generic element load/store as float (T = float or uint16_t-as-bf16).
template <typename T> struct Elt;
template <> struct Elt<float> {
  __device__ __forceinline__ static float ld(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Elt<uint16_t> {
  __device__ __forceinline__ static float ld(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
  __device__ __forceinline__ static void st(uint16_t* p, int64_t i, float v) { p[i] = f2bf(v); }
};

// 4-wide vector load/store as float (16 B for fp32, 8 B for bf16). Caller guarantees alignment.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ __forceinline__ static void ld(const float* p, int64_t i, float (&v)[4]) {
    float4 t = *reinterpret_cast<const float4*>(p + i);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ __forceinline__ static void st(float* p, int64_t i, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<uint16_t> {
  __device__ __forceinline__ static void ld(const uint16_t* p, int64_t i, float (&v)[4]) {
    uint2 t = *reinterpret_cast<const uint2*>(p + i);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void st(uint16_t* p, int64_t i, const float (&v)[4]) {
    uint2 t;
    t.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    t.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(p + i) = t;
  }
};

// 8 x bf16 <-> 8 x float through one 16-byte access.
__device__ __forceinline__ void ld8_bf16(const uint16_t* p, float (&v)[8]) {
  uint4 t = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8_bf16(uint16_t* p, const float (&v)[8]) {
  uint4 t;
  t.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  t.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  t.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  t.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = t;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Cross-lane adds in the VALU (DPP row permutes, gfx950 v_permlane16/32_swap) instead of ds_bpermute
// (__shfl_xor goes through the LDS crossbar: ~100-cycle latency per step, serialised in a reduction
// chain). Each pairs the same lanes as v + __shfl_xor(v, SH), so results are bit-identical to the
// shuffle forms. SH = 8 has no exact VALU form and stays a shuffle.
template <int SH>
__device__ __forceinline__ float xor_add(float v) {
  static_assert(SH == 1 || SH == 2 || SH == 8 || SH == 16 || SH == 32, "xor_add: lane distance");
  if constexpr (SH == 1) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  } else if constexpr (SH == 2) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  } else if constexpr (SH == 8) {
    return v + __shfl_xor(v, 8, 64);
  } else if constexpr (SH == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
}

// Sum over the 16 lanes of each DPP row (lanes 16r .. 16r+15), in every lane of the row: the pairs of
// v += __shfl_xor(v, 1, 2, 4, 8) in that order (after the xor-1/2 steps a quad is uniform, so the
// half-row mirror pairs quad 0 with 1 as xor 4 does; after it a half-row is uniform, so the row mirror
// pairs the halves as xor 8 does): bit-identical to the shuffle chain, four VALU ops.
__device__ __forceinline__ float row16_sum(float v) {
  v = xor_add<1>(v);
  v = xor_add<2>(v);
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, true));
  return v;
}

// Block-wide sum; `red` needs blockDim.x/64 floats of LDS. Result valid in all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// XCD-aware remap of a 1-D block id (bijective for any nwg): consecutive logical tiles land
// on the same XCD (shared L2). Speed only, never correctness (MI355X_MICROARCH §dispatch).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

}  // namespace pdt

// Multi-tensor launch metadata, passed BY VALUE as a kernel argument (graph-capture safe,
// no H2D copy). Workgroup b processes chunk (b - chunk_start[t]) of tensor t, where t is the
// last tensor with chunk_start[t] <= b.
#define PDT_MT_MAX_TENSORS 36
#define PDT_MT_CHUNK 16384
#define PDT_MT_MAX_GRID (1 << 30)

template <int NL>
struct MTMeta {
  void* ptr[NL][PDT_MT_MAX_TENSORS];
  int64_t numel[PDT_MT_MAX_TENSORS];
  int chunk_start[PDT_MT_MAX_TENSORS + 1];
  int ntensors;
};
