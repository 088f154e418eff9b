// Multi-tensor apply for gfx950: one launch walks many tensors (optimizer, AMP, bucket copy).
//
// The reference's optimizer (torch.optim.Adadelta, /root/reference/train.py:99) dispatches
// ~7 _foreach_ kernels per step and its gradient averaging 10 div_ kernels
// (train.py:39). Here every such per-step elementwise pass is ONE kernel per ≤320 chunks of
// 32 Ki elements: each workgroup (256 threads = 4 waves) takes one (tensor, chunk) pair and
// streams it with 16-byte (fp32) / 8-byte (bf16) per-lane accesses when all operand pointers
// of that tensor are 16-byte aligned, scalar otherwise.
#pragma once
#include "common.h"

namespace pdt {

template <int NL>
__device__ __forceinline__ bool mt_aligned(const MTMeta<NL>& m, int t) {
  bool ok = true;
#pragma unroll
  for (int l = 0; l < NL; ++l) ok &= (((uintptr_t)m.ptr[l][t]) & 15) == 0;
  return ok;
}

template <int NL, typename Op>
__global__ __launch_bounds__(256) void mt_kernel(MTMeta<NL> meta, Op op) {
  const int t = meta.block_tensor[blockIdx.x];
  const int64_t c = meta.block_chunk[blockIdx.x];
  const int64_t n = meta.numel[t];
  const int64_t start = c * PDT_MT_CHUNK;
  const int64_t end = start + PDT_MT_CHUNK < n ? start + PDT_MT_CHUNK : n;
  if (!op.enabled()) return;
  if (mt_aligned(meta, t)) {
    int64_t vend = start + ((end - start) & ~(int64_t)3);
    for (int64_t i = start + threadIdx.x * 4; i < vend; i += (int64_t)blockDim.x * 4) op.vec4(meta, t, i);
    for (int64_t i = vend + threadIdx.x; i < end; i += blockDim.x) op.scalar(meta, t, i);
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) op.scalar(meta, t, i);
  }
  op.finish(meta, t);
}

// Host side: chunk `ntensors` tensors (operand l of tensor t at lists[l][t]) into launches.
template <int NL, typename Op>
inline void mt_launch(int ntensors, void* const* lists[NL], const int64_t* numel, const Op& op,
                      hipStream_t stream) {
  MTMeta<NL> meta;
  meta.nblocks = 0;
  int tl = 0;  // slot of the current tensor in meta
  for (int t = 0; t < ntensors; ++t) {
    const int64_t n = numel[t];
    if (n == 0) continue;
    for (int l = 0; l < NL; ++l) meta.ptr[l][tl] = lists[l] ? lists[l][t] : nullptr;
    meta.numel[tl] = n;
    const int64_t nch = (n + PDT_MT_CHUNK - 1) / PDT_MT_CHUNK;
    for (int64_t c = 0; c < nch; ++c) {
      meta.block_tensor[meta.nblocks] = (uint8_t)tl;
      meta.block_chunk[meta.nblocks] = (uint16_t)c;
      meta.nblocks++;
      const bool last_chunk = c == nch - 1;
      const bool full_blocks = meta.nblocks == PDT_MT_MAX_BLOCKS;
      const bool full_tensors = (tl + 1 == PDT_MT_MAX_TENSORS) && last_chunk;
      if (full_blocks || full_tensors) {
        hipLaunchKernelGGL((mt_kernel<NL, Op>), dim3(meta.nblocks), dim3(256), 0, stream, meta, op);
        meta.nblocks = 0;
        if (last_chunk) {
          tl = -1;  // next tensor goes to slot 0
        } else {
          for (int l = 0; l < NL; ++l) meta.ptr[l][0] = meta.ptr[l][tl];
          meta.numel[0] = n;
          tl = 0;
          // remaining chunks of this tensor keep using slot 0
        }
      }
    }
    tl++;
  }
  if (meta.nblocks > 0)
    hipLaunchKernelGGL((mt_kernel<NL, Op>), dim3(meta.nblocks), dim3(256), 0, stream, meta, op);
}

}  // namespace pdt
