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
  c->bytes = XG_HDR_BYTES + 2ull * cap * sizeof(float);
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
  if (c->connected)
    for (int q = 0; q < c->desc.world; ++q)
      if (q != c->desc.rank && c->peers[q]) (void)hipIpcCloseMemHandle(c->peers[q]);
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
