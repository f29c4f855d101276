// xGMI one-shot all-reduce: IPC buffer management + generic stage/reduce kernels.
// Protocol and memory layout: xgmi.h.  The fused-MLP step uses the Adam consumer in
// adam.hip (em_adam_xgmi); the kernels here serve any small flat fp32 all-reduce and the
// communicator self-test (parallel/xgmi.py).
//
// Reference parity: the reference has no collectives at all; this is the
// C1 gradient all-reduce for the north star's DP=8 config (BASELINE.json configs[2]).
#include "common.h"
#include "xgmi.h"

#include <cstring>
#include <new>

namespace {

constexpr int XG_BLOCK = 256;

__global__ void __launch_bounds__(XG_BLOCK)
xgmi_stage_kernel(int* __restrict__ hdr, float* __restrict__ data, int cap, const float* __restrict__ src, int n) {
  float* slot = xg_produce_slot(hdr, data, cap);
  for (int i = blockIdx.x * XG_BLOCK + threadIdx.x; i < n; i += gridDim.x * XG_BLOCK) slot[i] = src[i];
}

__global__ void __launch_bounds__(XG_BLOCK) xgmi_reduce_kernel(XgmiDesc d, float* __restrict__ out, int n, float scale) {
  const int s = xg_next_seq(d.my_hdr);
  const bool ok = xg_publish_and_wait(d, s);
  if (ok) {
    for (int i = blockIdx.x * XG_BLOCK + threadIdx.x; i < n; i += gridDim.x * XG_BLOCK) out[i] = xg_sum(d, s, i) * scale;
  }
  xg_finish(d, s);
}

// One-process proxy of the N-rank exchange (tools/xgmi_budget.py): stands in for the peers of rank
// d.rank.  After `delay_ticks` of wall clock (the peers reaching the exchange later than this rank:
// publication skew) every emulated peer's slot gets this rank's staged gradient and its flag the
// step's sequence number, as the peers' own consumers would publish them.
__global__ void __launch_bounds__(XG_BLOCK)
xgmi_emulate_peers_kernel(XgmiDesc d, int* const* __restrict__ peer_hdr, float* const* __restrict__ peer_data, int n,
                          long long delay_ticks) {
  __shared__ int s_sh;
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < delay_ticks) __builtin_amdgcn_s_sleep(2);
    s_sh = xg_next_seq(d.my_hdr);
  }
  __syncthreads();
  const int s = s_sh;
  if (n > 0) {  // optional: the peers' slots get this rank's gradient (one block: ~30 us for 7 x 64 KB,
                // so the budget runs use n = 0 and the peers' slots keep what em_xgmi_stage left there)
    const float* src = d.my_data + (size_t)(s & 1) * d.cap;
    for (int q = 0; q < d.world; ++q) {
      if (q == d.rank) continue;
      float* dst = peer_data[q] + (size_t)(s & 1) * d.cap;
      for (int i = threadIdx.x; i < n; i += XG_BLOCK) dst[i] = src[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // slot data before the flags (system scope)
    __syncthreads();
  }
  if (threadIdx.x < (unsigned)d.world && (int)threadIdx.x != d.rank)
    __hip_atomic_store(&peer_hdr[threadIdx.x][XG_FLAG], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same for the LL form (adam_slab_xgmi_kernel, xgmi.h): block j stands in for the peers' words
// of slice j (64 elements; block 0 also the elements past the last full slice: the loss).
//   copy 1: each element waits until this rank's own LL word carries tag s (its slice is published),
//           `delay_ticks` more, then copies the word into every emulated peer's slot (bit-exact sums).
//           Every wait is bounded by the communicator's timeout (the error word is raised).
//   copy 0: timing only: `delay_ticks` after the block starts, the peers' words get tag s (value 0)
//           without waiting on the consumer, so a graph replay that runs it first cannot deadlock.
//   copy 2: the peers' words get tag INT_MAX once (peers infinitely early: no consumer wait on this
//           communicator ever blocks again; the budget's lower bound).
__global__ void __launch_bounds__(64)
xgmi_emulate_block_peers_kernel(XgmiDesc d, float* const* __restrict__ peer_data, int n, int copy,
                                long long delay_ticks) {
  const int j = blockIdx.x;
  const int s = copy == 2 ? 0x7FFFFFFF : xg_next_seq(d.my_hdr);
  const int full = 64 * (int)gridDim.x;
  auto one = [&](int i) {
    uint64_t w = xg_ll_word(0.f, s);
    const long long t0 = wall_clock64();
    if (copy == 1) {
      const uint64_t* own = xg_ll(d.my_data, d.cap, s) + i;
      for (;;) {
        w = __hip_atomic_load(own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (xg_ll_ready(w, s)) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > d.timeout_ticks) {
          __hip_atomic_store(&d.my_hdr[XG_ERROR], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return;
        }
      }
    }
    const long long t1 = wall_clock64();
    while (wall_clock64() - t1 < delay_ticks) __builtin_amdgcn_s_sleep(2);
    for (int q = 0; q < d.world; ++q) {
      if (q == d.rank) continue;
      for (int par = 0; par < (copy == 2 ? 2 : 1); ++par) {  // (saturated: both parities' slots)
        // (unsigned: copy == 2 sets s = INT_MAX, and s + par must wrap to parity 0 without signed overflow)
        uint64_t* dst = const_cast<uint64_t*>(xg_ll(peer_data[q], d.cap, (int)((unsigned)s + (unsigned)par))) + i;
        __hip_atomic_store(dst, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  };
  const int i = 64 * j + (int)threadIdx.x;
  if (i < full && i < n) one(i);
  if (j == 0)
    for (int k = full + (int)threadIdx.x; k < n; k += 64) one(k);
}

// consumer blocks spin on peer flags, so keep the grid well inside one wave of residency
int grid_for(int n) {
  int nb = (n + XG_BLOCK - 1) / XG_BLOCK;
  return nb < 1 ? 1 : (nb > 256 ? 256 : nb);
}

}  // namespace

EM_API int em_xgmi_create(int cap_floats, double timeout_s, void** out) {
  if (cap_floats <= 0 || !out) return EM_ERR_ARG;
  XgmiComm* c = new (std::nothrow) XgmiComm();
  if (!c) return EM_ERR_ARG;
  hipError_t e = hipGetDevice(&c->device);
  if (e != hipSuccess) {
    delete c;
    return (int)e;
  }
  const int cap = (cap_floats + 255) & ~255;
  c->bytes = xg_buffer_bytes(cap);
  // uncached: the flag/data words are exchanged between devices inside running kernels
  e = hipExtMallocWithFlags(&c->own, c->bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(c->own, 0, c->bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (c->own) (void)hipFree(c->own);
    delete c;
    return (int)e;
  }
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  c->desc.my_hdr = reinterpret_cast<int*>(c->own);
  c->desc.my_data = reinterpret_cast<float*>(static_cast<char*>(c->own) + XG_HDR_BYTES);
  c->desc.cap = cap;
  c->desc.world = 1;
  c->desc.rank = 0;
  c->desc.timeout_ticks = (long long)(timeout_s * 1000.0 * khz);
  c->desc.peer_data[0] = c->desc.my_data;
  c->desc.peer_hdr[0] = c->desc.my_hdr;
  *out = c;
  return 0;
}

EM_API int em_xgmi_handle(void* h, uint8_t* out64) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !out64) return EM_ERR_ARG;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  hipIpcMemHandle_t mh;
  hipError_t e = hipIpcGetMemHandle(&mh, c->own);
  if (e != hipSuccess) return (int)e;
  memcpy(out64, &mh, 64);
  return 0;
}

// handles = world x 64 bytes in rank order (own entry ignored)
EM_API int em_xgmi_connect(void* h, int world, int rank, const uint8_t* handles) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !handles || world < 1 || world > XG_MAXW || rank < 0 || rank >= world || c->connected) return EM_ERR_ARG;
  for (int q = 0; q < world; ++q) {
    if (q == rank) {
      c->peers[q] = c->own;
      continue;
    }
    hipIpcMemHandle_t mh;
    memcpy(&mh, handles + 64 * q, 64);
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, mh, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      for (int k = 0; k < q; ++k)
        if (k != rank && c->peers[k]) (void)hipIpcCloseMemHandle(c->peers[k]);
      return (int)e;
    }
    c->peers[q] = p;
  }
  for (int q = 0; q < world; ++q) {
    c->desc.peer_hdr[q] = reinterpret_cast<const int*>(c->peers[q]);
    c->desc.peer_data[q] = reinterpret_cast<const float*>(static_cast<const char*>(c->peers[q]) + XG_HDR_BYTES);
  }
  c->desc.world = world;
  c->desc.rank = rank;
  c->connected = true;
  return 0;
}

EM_API int em_xgmi_set_timeout(void* h, double timeout_s) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || timeout_s <= 0) return EM_ERR_ARG;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  c->desc.timeout_ticks = (long long)(timeout_s * 1000.0 * khz);
  return 0;
}

// error word (1 = a consumer timed out waiting for a peer); synchronous read
EM_API int em_xgmi_error(void* h, int* out) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !out) return EM_ERR_ARG;
  hipError_t e = hipMemcpy(out, c->desc.my_hdr + XG_ERROR, sizeof(int), hipMemcpyDeviceToHost);
  return (int)e;
}

EM_API int em_xgmi_capacity(void* h) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  return c ? c->desc.cap : -1;
}

EM_API int em_xgmi_destroy(void* h) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c) return 0;
  (void)hipDeviceSynchronize();
  if (c->connected && !c->local_proxy)
    for (int q = 0; q < c->desc.world; ++q)
      if (q != c->desc.rank && c->peers[q]) (void)hipIpcCloseMemHandle(c->peers[q]);
  if (c->peer_ptrs) (void)hipFree(c->peer_ptrs);
  if (c->own) (void)hipFree(c->own);
  delete c;
  return 0;
}

// producer: copy n floats of a local device array into this rank's next slot
EM_API int em_xgmi_stage(void* h, const float* src, int n, hipStream_t stream) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !src || n <= 0 || n > c->desc.cap) return EM_ERR_ARG;
  hipLaunchKernelGGL(xgmi_stage_kernel, dim3(grid_for(n)), dim3(XG_BLOCK), 0, stream, c->desc.my_hdr, c->desc.my_data,
                     c->desc.cap, src, n);
  EM_CHECK_LAUNCH();
  return 0;
}

// consumer: out[i] = scale * sum_q slot_q[i]  (out may alias the staged source)
EM_API int em_xgmi_reduce(void* h, float* out, int n, float scale, hipStream_t stream) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !out || n <= 0 || n > c->desc.cap || !c->connected) return EM_ERR_ARG;
  hipLaunchKernelGGL(xgmi_reduce_kernel, dim3(grid_for(n)), dim3(XG_BLOCK), 0, stream, c->desc, out, n, scale);
  EM_CHECK_LAUNCH();
  return 0;
}

// ---- one-process proxy of an N-rank exchange (tools/xgmi_budget.py; never used for training) ----
// Connects `h` as rank `rank` of `world` whose peers are the buffers of other comms created in THIS
// process on the same device (`others[q]`, q != rank; no IPC, no peer access): the consumer kernels
// then read 7 peer slots and poll 7 flags exactly as on a node, with the peers played by
// em_xgmi_emulate_peers.
EM_API int em_xgmi_connect_local(void* h, int world, int rank, void* const* others) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !others || world < 1 || world > XG_MAXW || rank < 0 || rank >= world || c->connected) return EM_ERR_ARG;
  for (int q = 0; q < world; ++q) {
    XgmiComm* o = q == rank ? c : static_cast<XgmiComm*>(others[q]);
    if (!o || o->desc.cap != c->desc.cap) return EM_ERR_ARG;
    c->desc.peer_hdr[q] = o->desc.my_hdr;
    c->desc.peer_data[q] = o->desc.my_data;
  }
  c->desc.world = world;
  c->desc.rank = rank;
  c->local_proxy = true;  // peers are not IPC mappings: nothing to close
  c->connected = true;
  return 0;
}

namespace {
// device copies of a connect_local'ed comm's peer header / data pointers
int peer_ptr_table(XgmiComm* c) {
  if (!c->peer_ptrs) {
    if (hipMalloc(&c->peer_ptrs, 2 * XG_MAXW * sizeof(void*)) != hipSuccess) return EM_ERR_ARG;
    void* host[2 * XG_MAXW];
    for (int q = 0; q < XG_MAXW; ++q) {
      host[q] = q < c->desc.world ? (void*)c->desc.peer_hdr[q] : nullptr;
      host[XG_MAXW + q] = q < c->desc.world ? (void*)c->desc.peer_data[q] : nullptr;
    }
    if (hipMemcpy(c->peer_ptrs, host, sizeof(host), hipMemcpyHostToDevice) != hipSuccess) return EM_ERR_ARG;
  }
  return 0;
}
}  // namespace

// the emulated peers of a connect_local'ed comm publish their flags (and n floats, if n > 0) after delay_us
EM_API int em_xgmi_emulate_peers(void* h, int n, double delay_us, hipStream_t stream) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !c->local_proxy || n < 0 || n > c->desc.cap || delay_us < 0) return EM_ERR_ARG;
  if (int e = peer_ptr_table(c)) return e;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  int* const* hdr = reinterpret_cast<int* const*>(c->peer_ptrs);
  float* const* data = reinterpret_cast<float* const*>(c->peer_ptrs) + XG_MAXW;
  hipLaunchKernelGGL(xgmi_emulate_peers_kernel, dim3(1), dim3(XG_BLOCK), 0, stream, c->desc, hdr, data, n,
                     (long long)(delay_us * 1e-3 * khz));
  EM_CHECK_LAUNCH();
  return 0;
}

// LL form (the fused DP consumer, em_adam_slab_xgmi over nblocks = P / 64 slices of an n-element
// exchange): run on a side stream beside the consumer (copy 0 / 1) or once before the timed steps
// (copy 2); see xgmi_emulate_block_peers_kernel
EM_API int em_xgmi_emulate_block_peers(void* h, int nblocks, int n, int copy, double delay_us, hipStream_t stream) {
  XgmiComm* c = static_cast<XgmiComm*>(h);
  if (!c || !c->local_proxy || nblocks <= 0 || n < 0 || n > c->desc.cap || n > 64 * nblocks + 64 || copy < 0 ||
      copy > 2 || delay_us < 0)
    return EM_ERR_ARG;
  if (int e = peer_ptr_table(c)) return e;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0) khz = 100000;
  float* const* data = reinterpret_cast<float* const*>(c->peer_ptrs) + XG_MAXW;
  hipLaunchKernelGGL(xgmi_emulate_block_peers_kernel, dim3(nblocks), dim3(64), 0, stream, c->desc, data, n, copy,
                     (long long)(delay_us * 1e-3 * khz));
  EM_CHECK_LAUNCH();
  return 0;
}
