// One-shot intra-node all-reduce over xGMI peer memory (MI355X: 8 GPUs, full mesh, 7 links/GPU).
//
// Why not RCCL for the flagship step: the 62->128->62 gradient is 64 KB, so an RCCL ring
// all-reduce (2(N-1) link hops, each a few us of protocol latency) costs tens of us against a
// ~150 us step.  On a fully connected xGMI mesh every GPU can instead READ all N-1 peer
// gradient buffers directly, in parallel over its own links: one hop, ~0.5 us of bandwidth,
// and the reduction lands inside the Adam kernel (no extra launch, graph-capturable).
//
// Protocol (per rank r, own buffer B_r = hipExtMallocWithFlags(uncached), shared via IPC):
//   header : flag (published seq, written by r, polled by peers)  @ 0
//            error word (timeouts)                                @ 64
//            seq_local, ticket (r only)                           @ 128, 132
//   data   : two slots of `cap` floats                             @ 4096
//   LL     : two slots of `cap` 8-byte words (the fused DP consumer) @ 4096 + 8 cap
// step s = seq_local + 1:
//   1. producer kernel (slab reduce / stage) writes slot[s & 1] of B_r.
//   2. consumer kernel: block 0 publishes flag_r = s (system-scope release; the producer's
//      writes are already in HBM at its kernel boundary, and the buffer is uncached);
//      every block polls flag_q >= s for all q (bounded by a wall-clock timeout), then
//      sums slot[s & 1] of B_0 .. B_{N-1} in rank order (identical bits on every rank)
//      and the last block to finish publishes seq_local = s.
// Slot reuse is safe with two slots: r overwrites slot[s & 1] in step s+2 only after its
// step-(s+1) consumer saw every flag_q >= s+1, and q publishes s+1 only after finishing its
// step-s consumer (stream order).  Flags only grow, so nothing is ever reset.
//
// LL form (the fused DP step, adam.hip adam_slab_xgmi_kernel): the consumer itself produces the slot,
// as "LL" words -- 8 bytes {float bits, sequence number s} stored with one 64-bit system-scope store --
// in a second pair of slots after the float slots.  Block j reduces its own slice j, stores its 64 LL
// words and, with no drain, no flag and no barrier, reads slice j of every peer: each reader polls the
// peer's word itself until its tag reaches s.  One round trip per exchange instead of three (slot
// stores drained, flag raised, flags polled, slots read).  The reuse argument above holds per word:
// q writes tag s + 2 into the same-parity slot only in its step-(s+2) consumer, i.e. after its
// step-(s+1) consumer read our tag-(s+1) words, which we store only after finishing step s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int XG_MAXW = 8;
constexpr int XG_HDR_BYTES = 4096;
constexpr int XG_FLAG = 0;     // int index into the header
constexpr int XG_ERROR = 16;   // byte 64
constexpr int XG_SEQ = 32;     // byte 128
constexpr int XG_TICKET = 33;  // byte 132

struct XgmiDesc {
  const float* peer_data[XG_MAXW];  // slot 0 of every rank's buffer (own included), rank order
  const int* peer_hdr[XG_MAXW];
  int* my_hdr;
  float* my_data;
  int world, rank, cap;
  long long timeout_ticks;  // wall_clock64 ticks
};

__device__ __forceinline__ int xg_next_seq(const int* hdr) {
  return __hip_atomic_load(&hdr[XG_SEQ], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
}

// slot base (own buffer) the producer of the next step writes
__device__ __forceinline__ float* xg_produce_slot(int* hdr, float* data, int cap) {
  return data + (size_t)(xg_next_seq(hdr) & 1) * cap;
}

// Every block waits until header int `idx` of every rank reached s (lane q polls rank q).
// Returns false (and raises the error word) on timeout.  Must be called by all threads.
__device__ __forceinline__ bool xg_wait_flags(const XgmiDesc& d, int s, int idx) {
  __shared__ int xg_bad;
  if (threadIdx.x == 0) xg_bad = 0;
  __syncthreads();
  if (threadIdx.x < (unsigned)d.world) {
    const int* f = &d.peer_hdr[threadIdx.x][idx];
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < s) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > d.timeout_ticks) {
        xg_bad = 1;
        __hip_atomic_store(&d.my_hdr[XG_ERROR], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale peer lines after the flags
  __syncthreads();
  return xg_bad == 0;
}

// Consumer prologue: block 0 publishes this rank's flag; every block waits for all peers.
__device__ __forceinline__ bool xg_publish_and_wait(const XgmiDesc& d, int s) {
  if (threadIdx.x == 0 && blockIdx.x == 0)
    __hip_atomic_store(&d.my_hdr[XG_FLAG], s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  return xg_wait_flags(d, s, XG_FLAG);
}

// LL words: after the two float slots of a buffer, two slots of `cap` 8-byte words (parity s & 1)
__device__ __forceinline__ const uint64_t* xg_ll(const float* data, int cap, int s) {
  return reinterpret_cast<const uint64_t*>(data + 2 * (size_t)cap) + (size_t)(s & 1) * cap;
}
__device__ __forceinline__ uint64_t xg_ll_word(float v, int s) {
  return ((uint64_t)(uint32_t)s << 32) | (uint64_t)__float_as_uint(v);
}
__device__ __forceinline__ bool xg_ll_ready(uint64_t w, int s) { return (int)(uint32_t)(w >> 32) >= s; }
// this rank's element i of step s
__device__ __forceinline__ void xg_ll_put(const XgmiDesc& d, int s, int i, float v) {
  uint64_t* w = const_cast<uint64_t*>(xg_ll(d.my_data, d.cap, s)) + i;
  __hip_atomic_store(w, xg_ll_word(v, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Element i of step s summed over all ranks in rank order (bitwise identical on every rank); `own` is
// this rank's value (not read back).  Every peer word is polled until its tag reaches s; the loads of
// all peers are in flight together.  A timeout raises the error word and *bad (an LDS flag the caller
// shares across its block: later slices then skip their waits) and returns ok = false.
__device__ __forceinline__ float xg_ll_sum(const XgmiDesc& d, int s, int i, float own, bool& ok, int* bad) {
  uint64_t w[XG_MAXW];
#pragma unroll
  for (int q = 0; q < XG_MAXW; ++q)
    w[q] = (q < d.world && q != d.rank)
               ? __hip_atomic_load(xg_ll(d.peer_data[q], d.cap, s) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
               : xg_ll_word(own, s);
  ok = *bad == 0;
  const long long t0 = wall_clock64();
  while (ok) {
    bool all = true;
#pragma unroll
    for (int q = 0; q < XG_MAXW; ++q)
      if (!xg_ll_ready(w[q], s)) {
        all = false;
        w[q] = __hip_atomic_load(xg_ll(d.peer_data[q], d.cap, s) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    if (all) break;
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > d.timeout_ticks) {
      ok = false;
      *bad = 1;
      __hip_atomic_store(&d.my_hdr[XG_ERROR], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  float acc = __uint_as_float((uint32_t)w[0]);
#pragma unroll
  for (int q = 1; q < XG_MAXW; ++q)
    if (q < d.world) acc += __uint_as_float((uint32_t)w[q]);
  return acc;
}

// Sum element i of slot (s & 1) over all ranks, rank order (bitwise identical on every rank).
__device__ __forceinline__ float xg_sum(const XgmiDesc& d, int s, int i) {
  const size_t off = (size_t)(s & 1) * d.cap + i;
  float v[XG_MAXW];
#pragma unroll
  for (int q = 0; q < XG_MAXW; ++q)
    v[q] = q < d.world ? __hip_atomic_load(d.peer_data[q] + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0.f;
  float acc = v[0];
#pragma unroll
  for (int q = 1; q < XG_MAXW; ++q)
    if (q < d.world) acc += v[q];
  return acc;
}

// Consumer epilogue: the last block to finish advances seq_local (after every block read it).
__device__ __forceinline__ void xg_finish(const XgmiDesc& d, int s) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tk = __hip_atomic_fetch_add(&d.my_hdr[XG_TICKET], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (int)gridDim.x - 1) {
      __hip_atomic_store(&d.my_hdr[XG_TICKET], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&d.my_hdr[XG_SEQ], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Buffer bytes for a capacity of `cap` floats: header, two float slots, two LL slots.
inline size_t xg_buffer_bytes(int cap) { return XG_HDR_BYTES + 2ull * cap * sizeof(float) + 2ull * cap * sizeof(uint64_t); }

// Host side (xgmi.hip): the C++ communicator object behind the opaque handle.
struct XgmiComm {
  void* own = nullptr;        // hipExtMallocWithFlags(uncached) base
  size_t bytes = 0;
  void* peers[XG_MAXW] = {};  // IPC-opened peer bases (own at [rank])
  XgmiDesc desc{};
  int device = 0;
  bool connected = false;
  bool local_proxy = false;   // em_xgmi_connect_local: peers are this process's buffers (no IPC)
  void* peer_ptrs = nullptr;  // em_xgmi_emulate_peers: device array of the peers' header / data pointers
};
