// Intra-node peer-to-peer all-reduce over xGMI ("custom xGMI P2P all-reduce",
// one-shot for small buckets). Not in the reference, which issues 10 tiny per-parameter NCCL
// all-reduces per step (/root/reference/train.py:34-39, 247 KB total — pure latency).
//
// Every rank owns one IPC-exported, uncached device region:
//     flags  [2 parity][MAX_BLOCKS][MAX_RANKS] uint32      (written by peers, polled locally)
//     data   [2 parity][cap bytes]                          (staging, read by peers)
// and has the other ranks' regions mapped (hipIpcOpenMemHandle; handles exchanged through the
// c10d store by parallel/p2p.py). One kernel per all-reduce, on the caller's stream:
//   1. block b copies its slice of the input into its own staging[parity] and fences (system);
//   2. block b stores `epoch` into flags[parity][b][me] of every peer (release, system scope)
//      and waits until every peer has stored `epoch` into its own flags[parity][b][*]
//      (acquire; bounded spin -> error flag instead of a hang);
//   3. block b sums slice b of all staging buffers in rank order 0..n-1 (fp32 accumulate, so
//      every rank computes bit-identical results) and writes it, times post_scale (1/world for
//      averaging), to the output.
// Reusing a parity two calls later is safe without a second barrier: a peer reads staging[p]
// for call k before it can signal call k+1, and call k+2 (the next writer of staging[p]) starts
// only after this rank saw that call-(k+1) signal (stream order on each rank).
// One-shot moves (n-1)·S bytes into each GPU over 7 xGMI links in parallel instead of a ring's
// 2(n-1)/n·S over one link; it wins below ~1 MiB where ring all-reduce is latency-bound.
#include "../common.h"

using namespace pdt;

#define PDT_P2P_MAX_RANKS 8
#define PDT_P2P_MAX_BLOCKS 128

namespace {

struct P2PPeers {
  char* data[PDT_P2P_MAX_RANKS];
  uint32_t* flags[PDT_P2P_MAX_RANKS];
};

template <typename T> struct V8;  // 8 elements <-> 8 floats through 16 B (bf16) / 32 B (fp32)
template <> struct V8<uint16_t> {
  __device__ __forceinline__ static void ld(const uint16_t* p, float (&v)[8]) { ld8_bf16(p, v); }
  __device__ __forceinline__ static void st(uint16_t* p, const float (&v)[8]) { st8_bf16(p, v); }
  __device__ __forceinline__ static void cp(const uint16_t* s, uint16_t* d) {
    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
  }
};
template <> struct V8<float> {
  __device__ __forceinline__ static void ld(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void st(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  __device__ __forceinline__ static void cp(const float* s, float* d) {
    reinterpret_cast<float4*>(d)[0] = reinterpret_cast<const float4*>(s)[0];
    reinterpret_cast<float4*>(d)[1] = reinterpret_cast<const float4*>(s)[1];
  }
};

template <typename T>
__global__ __launch_bounds__(256) void p2p_oneshot_kernel(const T* __restrict__ in, T* __restrict__ out, int64_t n,
                                                          P2PPeers peers, int rank, int world, int64_t cap,
                                                          uint32_t epoch, int parity, float post_scale,
                                                          int* __restrict__ err, int64_t spin_limit) {
  const int b = blockIdx.x;
  const int64_t n8 = n / 8;  // host guarantees n % 8 == 0
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = b * per, hi = min(n8, lo + per);
  T* mine = reinterpret_cast<T*>(peers.data[rank] + (int64_t)parity * cap);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) V8<T>::cp(in + i * 8, mine + i * 8);
  __threadfence_system();
  __syncthreads();
  const int slot = (parity * PDT_P2P_MAX_BLOCKS + b) * PDT_P2P_MAX_RANKS;
  if (threadIdx.x < world) {
    __hip_atomic_store(peers.flags[threadIdx.x] + slot + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = peers.flags[rank] + slot + threadIdx.x;
    int64_t it = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > spin_limit) {  // a peer never arrived: report instead of hanging the GPU
        atomicExch(err, 1);
        break;
      }
    }
  }
  __syncthreads();
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      float v[8];
      V8<T>::ld(reinterpret_cast<const T*>(peers.data[p] + (int64_t)parity * cap) + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= post_scale;
    V8<T>::st(out + i * 8, acc);
  }
}

}  // namespace

extern "C" {

int64_t pdt_p2p_flags_bytes() {
  return (int64_t)2 * PDT_P2P_MAX_BLOCKS * PDT_P2P_MAX_RANKS * sizeof(uint32_t);
}

// data_ptrs / flag_ptrs: `world` device pointers (own + mapped peers), flags region of each rank
// is pdt_p2p_flags_bytes() long. dtype 0 = fp32, 1 = bf16. n % 8 == 0, n * esize <= cap.
int pdt_p2p_allreduce(const void* in, void* out, int64_t n, int dtype, char* const* data_ptrs,
                      uint32_t* const* flag_ptrs, int rank, int world, int64_t cap, uint32_t epoch,
                      float post_scale, int* err, int max_blocks, hipStream_t s) {
  if (world < 1 || world > PDT_P2P_MAX_RANKS || n % 8 != 0) return -1;
  const int64_t esize = dtype == 0 ? 4 : 2;
  if (n * esize > cap) return -2;
  if (n == 0) return 0;
  P2PPeers peers{};
  for (int r = 0; r < world; ++r) {
    peers.data[r] = data_ptrs[r];
    peers.flags[r] = flag_ptrs[r];
  }
  // ~16 KiB of payload per block, at most max_blocks (<= PDT_P2P_MAX_BLOCKS) blocks
  int64_t nb = (n * esize + 16383) / 16384;
  const int64_t mb = max_blocks < PDT_P2P_MAX_BLOCKS ? max_blocks : PDT_P2P_MAX_BLOCKS;
  if (nb > mb) nb = mb;
  if (nb < 1) nb = 1;
  const int parity = (int)(epoch & 1u);
  const int64_t spin_limit = 20000000;  // ~1-2 s of polling
  if (dtype == 0)
    hipLaunchKernelGGL(p2p_oneshot_kernel<float>, dim3((unsigned)nb), dim3(256), 0, s, (const float*)in,
                       (float*)out, n, peers, rank, world, cap, epoch, parity, post_scale, err, spin_limit);
  else
    hipLaunchKernelGGL(p2p_oneshot_kernel<uint16_t>, dim3((unsigned)nb), dim3(256), 0, s, (const uint16_t*)in,
                       (uint16_t*)out, n, peers, rank, world, cap, epoch, parity, post_scale, err, spin_limit);
  return 0;
}

}  // extern "C"
