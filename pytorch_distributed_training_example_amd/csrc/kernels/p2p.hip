// Intra-node peer-to-peer all-reduce over xGMI ("custom xGMI P2P all-reduce",
// one-shot for small buckets, two-shot reduce-scatter + all-gather for mid sizes). Not in the
// reference, which issues 10 tiny per-parameter NCCL all-reduces per step
// (/root/reference/train.py:34-39, 247 KB total — pure latency).
//
// Every rank owns one IPC-exported, uncached device region:
//     flags  [4 slots][MAX_BLOCKS][MAX_RANKS] uint32   (written by peers, polled locally)
//              slots 0/1: one-shot, by epoch parity; slots 2/3: two-shot phase 1 / phase 2
//     data   [2 parity][cap] staging + [cap] two-shot result   (read by peers)
// and the other ranks' regions mapped (hipIpcOpenMemHandle; handles exchanged by parallel/p2p.py).
//
// Capture-safe: NOTHING per call comes from the host. The call counter (epoch) lives in device
// memory (`st`, private to the rank): every block reads epoch = st[0] + 1 at its start, and the
// last block to finish (done counter st[1]) stores st[0] = epoch — so a hipGraph replay of the
// same kernel node advances the epoch exactly like an eager call (a host-side epoch baked into a
// captured node would make every replay see last replay's flags and skip the barrier).
//
// Failure: a barrier wait is bounded in WALL-CLOCK time (s_memrealtime, 100 MHz), by a timeout the
// host derives from the process group's (parallel/p2p.py) — a legitimately late peer (first-step
// skew, rank-0-only host work) is waited for like an RCCL peer would be. On expiry the block sets
// st[2] = 1 (sticky until the host resets it) and writes NaN to its output slice instead of a
// partial sum, so a lost peer is never a silently wrong gradient: the DDP hook checks st[2] and NaN
// trips the AMP inf-check.
//
// One-shot (small): block b copies slice b of the input into staging[parity], fences (system
// scope), release-stores `epoch` into flags[parity][b][me] of every peer, waits for every peer's
// flag (acquire), then sums slice b of every rank's staging in rank order 0..n-1 (fp32 accumulate:
// bit-identical replicas). (n-1)·S bytes into each GPU over 7 links at once.
// Two-shot (mid sizes): rank r owns chunk r of the buffer. Phase 1: block b stages sub-slice b of
// every chunk, barrier (slot 2). Phase 2: block b reduces sub-slice b of chunk r over all ranks (rank
// order) into its result region and its output, barrier (slot 3). Phase 3: block b copies
// sub-slice b of chunk j from rank j's result. 2(n-1)/n·S bytes in per GPU, spread over all links
// (a ring moves the same bytes over ONE link).
// Reuse without extra barriers: a peer reads my staging[p] of call k before signalling call k+1,
// and my call k+2 (next writer of staging[p]) starts after I saw that signal (stream order). The
// two-shot's trailing phase-2 barrier means no peer still reads my staging or result after my call
// ends. Waits test `== epoch` on monotonically increasing values in per-kind slots, so a peer
// that is one call ahead never overwrites a flag I have not read yet.
#include "../common.h"

using namespace pdt;

#define PDT_P2P_MAX_RANKS 8
#define PDT_P2P_MAX_BLOCKS 128
#define PDT_P2P_SLOTS 4

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

// Block-wide start: epoch = st[0] + 1 (read by thread 0, shared through LDS).
__device__ __forceinline__ uint32_t read_epoch(uint32_t* st, uint32_t* sh) {
  if (threadIdx.x == 0) sh[0] = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __syncthreads();
  return sh[0];
}

// Block-wide end: the last block of the grid publishes st[0] = epoch for the next call.
__device__ __forceinline__ void finish_epoch(uint32_t* st, uint32_t epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(st + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(st + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Signal `epoch` into slot `slot` of every rank's flags for block b, then wait until every rank
// signalled this block. Returns false (and sets the sticky error word) if a peer never arrived.
__device__ __forceinline__ bool block_barrier(const P2PPeers& peers, int rank, int world, int slot_kind, int b,
                                              uint32_t epoch, uint32_t* st, uint64_t timeout_ticks, int* sh_ok) {
  const int slot = (slot_kind * PDT_P2P_MAX_BLOCKS + b) * PDT_P2P_MAX_RANKS;
  if (threadIdx.x == 0) sh_ok[0] = 1;
  __syncthreads();
  if (threadIdx.x < world) {
    __hip_atomic_store(peers.flags[threadIdx.x] + slot + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = peers.flags[rank] + slot + threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {  // a peer never arrived: report, never hang
        __hip_atomic_store(reinterpret_cast<int*>(st + 2), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_ok[0] = 0;
        break;
      }
    }
  }
  __syncthreads();
  return sh_ok[0] != 0;
}

template <typename T>
__device__ __forceinline__ void poison(T* out, int64_t lo, int64_t hi) {
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __builtin_nanf("");
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) V8<T>::st(out + i * 8, v);
}

template <typename T>
__global__ __launch_bounds__(256) void p2p_oneshot_kernel(const T* __restrict__ in, T* __restrict__ out, int64_t n,
                                                          P2PPeers peers, int rank, int world, int64_t cap,
                                                          float post_scale, uint32_t* __restrict__ st,
                                                          uint64_t timeout_ticks) {
  __shared__ uint32_t sh[2];
  const uint32_t epoch = read_epoch(st, sh);
  const int parity = (int)(epoch & 1u);
  const int b = blockIdx.x;
  const int64_t n8 = n / 8;  // host guarantees n % 8 == 0
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = b * per, hi = min(n8, lo + per);
  T* mine = reinterpret_cast<T*>(peers.data[rank] + (int64_t)parity * cap);
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) V8<T>::cp(in + i * 8, mine + i * 8);
  __threadfence_system();
  if (!block_barrier(peers, rank, world, parity, b, epoch, st, timeout_ticks, reinterpret_cast<int*>(sh + 1))) {
    poison(out, lo, hi);
  } else {
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
  finish_epoch(st, epoch);
}

// [c0, c1) vectors of chunk j (floor split of n8 vectors over world chunks), sub-slice b of nb.
__device__ __forceinline__ void sub_slice(int64_t n8, int world, int j, int b, int nb, int64_t& lo, int64_t& hi) {
  const int64_t c0 = n8 * j / world, c1 = n8 * (j + 1) / world;
  const int64_t per = (c1 - c0 + nb - 1) / nb;
  lo = min(c1, c0 + b * per);
  hi = min(c1, lo + per);
}

template <typename T>
__global__ __launch_bounds__(256) void p2p_twoshot_kernel(const T* __restrict__ in, T* __restrict__ out, int64_t n,
                                                          P2PPeers peers, int rank, int world, int64_t cap,
                                                          float post_scale, uint32_t* __restrict__ st,
                                                          uint64_t timeout_ticks) {
  __shared__ uint32_t sh[2];
  const uint32_t epoch = read_epoch(st, sh);
  const int parity = (int)(epoch & 1u);
  const int b = blockIdx.x, nb = gridDim.x;
  const int64_t n8 = n / 8;
  T* mine = reinterpret_cast<T*>(peers.data[rank] + (int64_t)parity * cap);
  // phase 1: stage sub-slice b of every chunk
  for (int j = 0; j < world; ++j) {
    int64_t lo, hi;
    sub_slice(n8, world, j, b, nb, lo, hi);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) V8<T>::cp(in + i * 8, mine + i * 8);
  }
  __threadfence_system();
  bool ok = block_barrier(peers, rank, world, 2, b, epoch, st, timeout_ticks, reinterpret_cast<int*>(sh + 1));
  // phase 2: reduce my chunk's sub-slice b over all ranks (rank order), into result + out
  int64_t mlo, mhi;
  sub_slice(n8, world, rank, b, nb, mlo, mhi);
  T* res = reinterpret_cast<T*>(peers.data[rank] + 2 * cap);
  if (ok) {
    for (int64_t i = mlo + threadIdx.x; i < mhi; i += blockDim.x) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < world; ++p) {
        float v[8];
        V8<T>::ld(reinterpret_cast<const T*>(peers.data[p] + (int64_t)parity * cap) + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= post_scale;
      V8<T>::st(res + i * 8, acc);
      V8<T>::st(out + i * 8, acc);
    }
    __threadfence_system();
    ok = block_barrier(peers, rank, world, 3, b, epoch, st, timeout_ticks, reinterpret_cast<int*>(sh + 1));
  }
  // phase 3: gather the other chunks' sub-slice b from their owners' result regions
  for (int j = 0; j < world; ++j) {
    int64_t lo, hi;
    sub_slice(n8, world, j, b, nb, lo, hi);
    if (!ok) {
      poison(out, lo, hi);
      continue;
    }
    if (j == rank) continue;
    const T* src = reinterpret_cast<const T*>(peers.data[j] + 2 * cap);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) V8<T>::cp(src + i * 8, out + i * 8);
  }
  finish_epoch(st, epoch);
}

}  // namespace

extern "C" {

int64_t pdt_p2p_flags_bytes() {
  return (int64_t)PDT_P2P_SLOTS * PDT_P2P_MAX_BLOCKS * PDT_P2P_MAX_RANKS * sizeof(uint32_t);
}

// Data region bytes per rank for a staging capacity of `cap` bytes: 2 staging parities + result.
int64_t pdt_p2p_data_bytes(int64_t cap) { return 3 * cap; }

// data_ptrs / flag_ptrs: `world` device pointers (own + mapped peers); flags regions are
// pdt_p2p_flags_bytes() long, data regions pdt_p2p_data_bytes(cap). dtype 0 = fp32, 1 = bf16.
// n % 8 == 0, n * esize <= cap. st: this rank's private device state, 3 uint32 zero-initialised
// ([0] epoch, [1] finished-block counter, [2] sticky error). algo 0 = one-shot, 1 = two-shot.
// timeout_s: how long a block waits for a peer (wall clock) before poisoning its output.
int pdt_p2p_allreduce(const void* in, void* out, int64_t n, int dtype, char* const* data_ptrs,
                      uint32_t* const* flag_ptrs, int rank, int world, int64_t cap, float post_scale,
                      uint32_t* st, int algo, int max_blocks, double timeout_s, hipStream_t s) {
  if (world < 1 || world > PDT_P2P_MAX_RANKS || n % 8 != 0 || !st) return -1;
  const int64_t esize = dtype == 0 ? 4 : 2;
  if (n * esize > cap) return -2;
  if (n == 0) return 0;
  P2PPeers peers{};
  for (int r = 0; r < world; ++r) {
    peers.data[r] = data_ptrs[r];
    peers.flags[r] = flag_ptrs[r];
  }
  const int64_t mb = max_blocks < PDT_P2P_MAX_BLOCKS ? max_blocks : PDT_P2P_MAX_BLOCKS;
  // one-shot: ~16 KiB of payload per block; two-shot: ~16 KiB of this rank's chunk per block
  int64_t nb = algo == 1 ? (n * esize / world + 16383) / 16384 : (n * esize + 16383) / 16384;
  if (nb > mb) nb = mb;
  if (nb < 1) nb = 1;
  // s_memrealtime ticks at 100 MHz; at least 1 ms, at most a day
  const double ts = timeout_s < 1e-3 ? 1e-3 : (timeout_s > 86400.0 ? 86400.0 : timeout_s);
  const uint64_t timeout_ticks = (uint64_t)(ts * 1e8);
#define PDT_P2P_LAUNCH(K, T)                                                                                 \
  hipLaunchKernelGGL(K<T>, dim3((unsigned)nb), dim3(256), 0, s, (const T*)in, (T*)out, n, peers, rank, world, \
                     cap, post_scale, st, timeout_ticks)
  if (algo == 1) {
    if (dtype == 0) PDT_P2P_LAUNCH(p2p_twoshot_kernel, float);
    else PDT_P2P_LAUNCH(p2p_twoshot_kernel, uint16_t);
  } else {
    if (dtype == 0) PDT_P2P_LAUNCH(p2p_oneshot_kernel, float);
    else PDT_P2P_LAUNCH(p2p_oneshot_kernel, uint16_t);
  }
#undef PDT_P2P_LAUNCH
  return 0;
}

}  // extern "C"
