// GPT-2 token + position embedding, forward and DETERMINISTIC backward (SURVEY.md §2.3 "embedding
// fwd/bwd"; not in the reference, whose only model is LeNet, /root/reference/cnn.py).
//
//   forward : out[i, :] = wte[idx[i], :] + wpe[i % T, :]        one pass, fp32 add, one bf16 rounding
//             (aten: two gathers + an add kernel = 3 passes over [B*T, D])
//   backward: dwte[v, :] = sum over tokens i with idx[i] == v of dout[i, :], in increasing i
//             dwpe[t, :] = sum over b of dout[b*T + t, :], in increasing b
//
// The token gradient is a scatter with collisions (repeated tokens). An fp32 atomicAdd scatter is
// not reproducible run to run; aten's deterministic path sorts the indices. Here: a counting sort
// (histogram, exclusive scan, unordered placement by atomic slot), then ONE wave per vocabulary row
// ranks its bucket's token positions (each lane counts the smaller entries: buckets are small —
// 0.16 tokens per row on average for 8K tokens over GPT-2's 50K vocabulary) and sums the rows in
// increasing token order. Every row of dwte is written exactly once (zeros for absent tokens), so
// no separate zero-fill pass exists. Replicas and reruns produce bit-identical gradients.
//
// Token ids are range-checked in every kernel: an id < 0 or >= V never indexes memory (its output
// row is zeros, its gradient row is dropped) and sets a device error word that the host reads
// (ops/embedding.py: raised like nn.Embedding's index error), instead of out-of-bounds atomics.
#include "../common.h"

using namespace pdt;

namespace {

__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ idx, const uint16_t* __restrict__ wte,
                                                      const uint16_t* __restrict__ wpe, uint16_t* __restrict__ out,
                                                      int64_t n, int T, int D, int V, int* __restrict__ err) {
  const int per = D / 8;  // 16-B pieces per row
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n * per; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q / per;
    const int c = (int)(q % per) * 8;
    const int64_t v = idx[i];
    float a[8], b[8];
    if (v < 0 || v >= V) {  // out of range: zeros, and report (never read past the table)
      if (c == 0) atomicOr(err, 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
      st8_bf16(out + i * D + c, a);
      continue;
    }
    ld8_bf16(wte + v * D + c, a);
    ld8_bf16(wpe + (int64_t)(i % T) * D + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += b[j];
    st8_bf16(out + i * D + c, a);
  }
}

__global__ __launch_bounds__(256) void emb_hist_kernel(const int64_t* __restrict__ idx, int* __restrict__ cnt, int64_t n,
                                                       int V, int* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = idx[i];
    if (v < 0 || v >= V) {
      atomicOr(err, 1);
      continue;
    }
    atomicAdd(cnt + v, 1);
  }
}

// Exclusive scan of cnt[V] into off[V] by one 1024-thread workgroup (V ~ 50K: 49 per thread).
__global__ __launch_bounds__(1024) void emb_scan_kernel(const int* __restrict__ cnt, int* __restrict__ off, int V) {
  __shared__ int part[1024];
  const int per = (V + 1023) / 1024, lo = threadIdx.x * per, hi = min(V, lo + per);
  int s = 0;
  for (int v = lo; v < hi; ++v) s += cnt[v];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // Hillis-Steele inclusive scan of the 1024 partials
    const int add = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  int run = part[threadIdx.x] - s;
  for (int v = lo; v < hi; ++v) {
    off[v] = run;
    run += cnt[v];
  }
}

__global__ __launch_bounds__(256) void emb_place_kernel(const int64_t* __restrict__ idx, const int* __restrict__ off,
                                                        int* __restrict__ fill, int* __restrict__ pos, int64_t n, int V) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = idx[i];
    if (v < 0 || v >= V) continue;  // reported by emb_hist_kernel
    pos[off[v] + atomicAdd(fill + v, 1)] = (int)i;
  }
}

// One wave per vocabulary row: rank the bucket (token positions are distinct), then sum its rows in
// increasing token order; lane l owns columns [8 l, 8 l + 8) (+ 512 per pass) of D.
__global__ __launch_bounds__(256) void emb_bwd_rows_kernel(const uint16_t* __restrict__ dout, const int* __restrict__ cnt,
                                                           const int* __restrict__ off, int* __restrict__ pos,
                                                           int* __restrict__ sorted, uint16_t* __restrict__ dwte,
                                                           int V, int D) {
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= V) return;  // whole wave exits together (v is wave-uniform)
  const int c = cnt[v], o = off[v];
  for (int j = lane; j < c; j += 64) {  // stable order: rank = number of smaller positions
    const int e = pos[o + j];
    int r = 0;
    for (int k = 0; k < c; ++k) r += pos[o + k] < e;
    sorted[o + r] = e;
  }
  __threadfence_block();  // this wave's stores to `sorted` are visible to its own reloads
  __builtin_amdgcn_wave_barrier();
  for (int col = lane * 8; col < D; col += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < c; ++k) {
      float d[8];
      ld8_bf16(dout + (int64_t)sorted[o + k] * D + col, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d[j];
    }
    st8_bf16(dwte + (int64_t)v * D + col, acc);
  }
}

__global__ __launch_bounds__(256) void emb_bwd_pos_kernel(const uint16_t* __restrict__ dout, uint16_t* __restrict__ dwpe,
                                                          int B, int T, int D) {
  const int per = D / 8;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < (int64_t)T * per; q += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(q / per), c = (int)(q % per) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
      float d[8];
      ld8_bf16(dout + ((int64_t)b * T + t) * D + c, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d[j];
    }
    st8_bf16(dwpe + (int64_t)t * D + c, acc);
  }
}

inline int grid_of(int64_t work) {
  const int64_t g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

extern "C" {

// out[B*T, D] = wte[idx] + wpe[pos]; idx int64 [B*T], D % 8 == 0. An id outside [0, V) gives a zero
// row and sets *err (device int, never cleared here).
int pdt_embedding_fwd(const int64_t* idx, const uint16_t* wte, const uint16_t* wpe, uint16_t* out, int64_t n, int T,
                      int D, int V, int* err, hipStream_t s) {
  if (D % 8 != 0 || T < 1 || V < 1 || !err) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3(grid_of(n * D / 8)), dim3(256), 0, s, idx, wte, wpe, out, n, T, D, V, err);
  return 0;
}

// Workspace ints: cnt[V], off[V], fill[V], pos[n], sorted[n]. cnt and fill must be zero on entry.
int64_t pdt_embedding_bwd_ws_ints(int64_t n, int V) { return 3 * (int64_t)V + 2 * n; }

// dwte[V, D] (every row written), dwpe[T, D] (nullable) from dout[B*T, D]; n = B*T. Ids outside
// [0, V) contribute nothing and set *err.
int pdt_embedding_bwd(const int64_t* idx, const uint16_t* dout, uint16_t* dwte, uint16_t* dwpe, int* ws, int64_t n,
                      int B, int T, int V, int D, int* err, hipStream_t s) {
  if (D % 8 != 0 || n != (int64_t)B * T || V < 1 || !err) return -1;
  int* cnt = ws;
  int* off = cnt + V;
  int* fill = off + V;
  int* pos = fill + V;
  int* sorted = pos + n;
  hipLaunchKernelGGL(emb_hist_kernel, dim3(grid_of(n)), dim3(256), 0, s, idx, cnt, n, V, err);
  hipLaunchKernelGGL(emb_scan_kernel, dim3(1), dim3(1024), 0, s, cnt, off, V);
  hipLaunchKernelGGL(emb_place_kernel, dim3(grid_of(n)), dim3(256), 0, s, idx, off, fill, pos, n, V);
  hipLaunchKernelGGL(emb_bwd_rows_kernel, dim3((V + 3) / 4), dim3(256), 0, s, dout, cnt, off, pos, sorted, dwte, V, D);
  if (dwpe) hipLaunchKernelGGL(emb_bwd_pos_kernel, dim3(grid_of((int64_t)T * D / 8)), dim3(256), 0, s, dout, dwpe, B, T, D);
  return 0;
}

}  // extern "C"
