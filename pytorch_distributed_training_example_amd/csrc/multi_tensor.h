// Multi-tensor apply for gfx950: one launch walks many tensors (optimizer, AMP, bucket copy).
//
// The reference's optimizer (torch.optim.Adadelta, /root/reference/train.py:99) dispatches
// ~7 _foreach_ kernels per step and its gradient averaging 10 div_ kernels
// (train.py:39). Here every such per-step elementwise pass is ONE kernel per group of up to
// 36 tensors. The launch covers every 16 Ki-element chunk of those tensors (any number of
// workgroups: the block → (tensor, chunk) map is a prefix sum over the tensors' chunk
// counts, passed by value, so the grid is as wide as the data and keeps HBM saturated).
// Each workgroup (256 threads = 4 waves) streams its chunk with 16-byte (fp32) / 8-byte
// (bf16) per-lane accesses, two vectors in flight per lane, when all operand pointers of that
// tensor are 16-byte aligned; scalar otherwise.
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

template <int NL>
__device__ __forceinline__ int mt_find(const MTMeta<NL>& m, int bid) {
  int t = 0;
  while (t + 1 < m.ntensors && m.chunk_start[t + 1] <= bid) ++t;
  return t;
}

template <int NL, typename Op>
__global__ __launch_bounds__(256) void mt_kernel(MTMeta<NL> meta, Op op) {
  if (!op.enabled()) return;
  const int t = mt_find(meta, blockIdx.x);
  const int64_t c = blockIdx.x - meta.chunk_start[t];
  const int64_t n = meta.numel[t];
  const int64_t start = c * PDT_MT_CHUNK;
  const int64_t end = start + PDT_MT_CHUNK < n ? start + PDT_MT_CHUNK : n;
  if (mt_aligned(meta, t)) {
    const int64_t vend = start + ((end - start) & ~(int64_t)3);
    int64_t i = start + threadIdx.x * 4;
    for (; i + 1024 < vend; i += 2048) {  // two independent vectors in flight per lane
      op.vec4(meta, t, i);
      op.vec4(meta, t, i + 1024);
    }
    for (; i < vend; i += 1024) op.vec4(meta, t, i);
    for (int64_t j = vend + threadIdx.x; j < end; j += blockDim.x) op.scalar(meta, t, j);
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) op.scalar(meta, t, i);
  }
  op.finish(meta, t);
}

// Host side: group `ntensors` tensors (operand l of tensor t at lists[l][t]) into launches of
// up to PDT_MT_MAX_TENSORS tensors; each launch's grid covers all their chunks.
template <int NL, typename Launch>
inline void mt_batches(int ntensors, void* const* lists[NL], const int64_t* numel, Launch&& launch) {
  MTMeta<NL> meta;
  meta.ntensors = 0;
  int nblocks = 0;
  auto flush = [&]() {
    if (meta.ntensors == 0) return;
    meta.chunk_start[meta.ntensors] = nblocks;
    launch(meta, nblocks);
    meta.ntensors = 0;
    nblocks = 0;
  };
  for (int t = 0; t < ntensors; ++t) {
    const int64_t n = numel[t];
    if (n == 0) continue;
    const int64_t nch = (n + PDT_MT_CHUNK - 1) / PDT_MT_CHUNK;
    if (meta.ntensors == PDT_MT_MAX_TENSORS || (int64_t)nblocks + nch > PDT_MT_MAX_GRID) flush();
    const int k = meta.ntensors++;
    for (int l = 0; l < NL; ++l) meta.ptr[l][k] = lists[l] ? lists[l][t] : nullptr;
    meta.numel[k] = n;
    meta.chunk_start[k] = nblocks;
    nblocks += (int)nch;
  }
  flush();
}

template <int NL, typename Op>
inline void mt_launch(int ntensors, void* const* lists[NL], const int64_t* numel, const Op& op,
                      hipStream_t stream) {
  mt_batches<NL>(ntensors, lists, numel, [&](const MTMeta<NL>& meta, int nblocks) {
    hipLaunchKernelGGL((mt_kernel<NL, Op>), dim3(nblocks), dim3(256), 0, stream, meta, op);
  });
}

}  // namespace pdt
