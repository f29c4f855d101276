// K6 — fused Adam for MI355X: deterministic slab reduction + Adam + bf16 weight packing.
//
// The reference's only optimizer is inside libxgboost (Newton boosting,
// Main.java:137-138); the north star's Adam comes from the declared-but-unused
// DL4J updater (pom.xml:62-66).  One flat fp32 master buffer
// (params, m, v); each thread owns one parameter:
//   g  = grad_scale * sum_{slab} slabs[slab][p]     (fixed order -> bitwise reproducible)
//   m  = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2
//   p -= lr * (m / bc1) / (sqrt(v / bc2) + eps)      (torch.optim.Adam semantics)
// and, for the fused small MLP, writes the bf16 value of p into the LDS-ready
// weight images consumed by mlp_fused.hip (so the train kernel's prologue is a
// straight 48 KB copy).  Modes let DP insert an RCCL all-reduce between the slab
// reduction and the update.
#include "common.h"
#include "mlp_adam.h"
#include "xgmi.h"

namespace {

using mlp::P_TOTAL;
using mlp::IMG_BYTES;

// 4 threads per parameter (slab-split), 64 parameters per 256-thread block.
// Bias-correction step counter kept on the device: every block reads `step` first; the last block
// to finish (ticket) publishes step+1.  So one launch = one Adam step, with no host round-trip,
// and the whole train step can be replayed from a hipGraph.
EM_DEVICE int adam_begin(int* state) { return __hip_atomic_load(&state[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1; }
// No release fence: the parameters/moments are consumed by later launches (a kernel boundary
// publishes them); the ticket only orders the step counter, whose read in adam_begin has already
// returned (its value fed the bias correction) before this block draws its ticket.  An agent-scope
// release here is an L2 writeback per block (cdna_hip_programming.md 5, "3.9x slower").
EM_DEVICE void adam_end(int* state, int t) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tk = __hip_atomic_fetch_add(&state[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (int)gridDim.x - 1) {
      __hip_atomic_store(&state[0], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&state[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Step-counter modes (the `mode` argument's bit 2, EM_ADAM_PRE): without it every launch reads
// state[0] + 1 and the last block to draw a ticket publishes it (adam_end); with it the producer
// of this step's gradients already advanced state[0] (mlp_fused.hip advance_step), so the counter
// is read as is and no ticket is drawn.
constexpr int EM_ADAM_PRE = 4;

// torch.optim.Adam update of parameter p with gradient g (pad slots of the MLP image pinned to 0).
// w0/m0/v0 are params[p]/m[p]/v[p], loaded by the caller (the slab kernel issues those loads
// before its slab reduction so their latency overlaps it).
// bc1 / bc2: the step's bias corrections (bias_correction(beta, t)), computed by the caller where
// their latency hides (adam_slab4_kernel: while its slab loads are in flight)
EM_DEVICE void adam_apply_bc(int p, float g, float w0, float m0, float v0, float bc1, float bc2,
                             float* __restrict__ params, float* __restrict__ m, float* __restrict__ v,
                             const float* __restrict__ hp, uint8_t* __restrict__ mlp_img) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4];
  if (mlp_img && mlp::pad_slot(p)) {
    params[p] = 0.f;
    m[p] = 0.f;
    v[p] = 0.f;
    mlp::pack_one(p, 0.f, mlp_img);
  } else {
    float mm = m0, vv = v0;
    const float w = adam_math(g, w0, mm, vv, lr, b1, b2, eps, wd, bc1, bc2);
    m[p] = mm;
    v[p] = vv;
    params[p] = w;
    if (mlp_img) mlp::pack_one(p, w, mlp_img);
  }
}

EM_DEVICE void adam_apply_loaded(int p, float g, float w0, float m0, float v0, int tstep, float* __restrict__ params,
                                 float* __restrict__ m, float* __restrict__ v, const float* __restrict__ hp,
                                 uint8_t* __restrict__ mlp_img) {
  adam_apply_bc(p, g, w0, m0, v0, bias_correction(hp[1], tstep), bias_correction(hp[2], tstep), params, m, v, hp,
                mlp_img);
}

EM_DEVICE void adam_apply(int p, float g, int tstep, float* __restrict__ params, float* __restrict__ m,
                          float* __restrict__ v, const float* __restrict__ hp, uint8_t* __restrict__ mlp_img) {
  adam_apply_loaded(p, g, params[p], m[p], v[p], tstep, params, m, v, hp, mlp_img);
}

// 16 threads per parameter (slab-split, all loads issued up front), 64 parameters per 1024-thread block.
// The slab reduction is latency-bound (16 MB spread over 256 slabs): every thread keeps its 16
// loads in flight at once.
constexpr int AS_P = 64, AS_G = 16;
__global__ void __launch_bounds__(AS_P * AS_G)
adam_slab_kernel(const float* __restrict__ slabs, int nslab, int P, int stride, float grad_scale, float* __restrict__ params,
                 float* __restrict__ m, float* __restrict__ v, float* __restrict__ grad_io, const float* __restrict__ hp,
                 int* __restrict__ state, int mode, uint8_t* __restrict__ mlp_img, const float* __restrict__ loss_slabs,
                 float* __restrict__ loss_out, float loss_scale, int pre) {
  const int tstep = (mode == 1) ? 0 : pre ? state[0] : adam_begin(state);
  // hp = {lr, beta1, beta2, eps, weight_decay}; state = {step, ticket} (device ints, graph-replay safe)
  __shared__ float part[AS_G][AS_P];
  const int tx = threadIdx.x % AS_P, ty = threadIdx.x / AS_P;
  const int p = blockIdx.x * AS_P + tx;
  float g = 0.f;
  if (mode != 2) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (p < P) {
      int sl = ty;
      for (; sl + 7 * AS_G < nslab; sl += 8 * AS_G) {  // 8 independent loads in flight per thread
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += slabs[(size_t)(sl + k * AS_G) * stride + p];
      }
      for (; sl < nslab; sl += AS_G) acc[0] += slabs[(size_t)sl * stride + p];
    }
    part[ty][tx] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    if (ty == 0) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < AS_G; ++k) t += part[k][tx];
      g = t * grad_scale;
    }
  } else if (p < P) {
    g = grad_io[p];
  }
  if (blockIdx.x == 0 && loss_slabs && loss_out && threadIdx.x < 64) {
    float l = 0.f;
    for (int i = threadIdx.x; i < nslab; i += 64) l += loss_slabs[i];
    l = wave_sum(l);
    if (threadIdx.x == 0) loss_out[0] = l * loss_scale;
  }
  if (mode == 1) {
    if (ty == 0 && p < P) grad_io[p] = g;
    return;
  }
  if (ty == 0 && p < P) adam_apply(p, g, tstep, params, m, v, hp, mlp_img);
  if (!pre) adam_end(state, tstep);
}

// Vectorised slab reduction (P % 64 == 0, stride % 4 == 0): 256 threads per 64 parameters, thread
// t = (slab group g = t >> 4, quad q = t & 15) sums float4 quads of slabs g, g + 16, ... with all of
// its loads in flight (16-B loads: 4x fewer memory instructions than one float per thread), then
// thread (quad, e) adds the 16 group sums in group order.  The fixed summation order keeps the result
// bitwise reproducible; the single-GPU step (adam_slab4_kernel) and the fused xGMI DP step
// (adam_slab_xgmi_kernel) share it, so their per-rank gradients are bit-identical.
// The slabs are read once, so their loads are nontemporal: same-box A/B over 3 interleaved rounds of
// the 1M-sample step (round 5, profiles/r5/ab_headline.jsonl), 88.63 -> 87.51 us per step with
// bit-identical parameters.  32 slab groups per block (512 threads, 8 loads in flight per thread)
// measured 87.98 us and changes the summation order; it was not kept.
// (compile-time A/B knob for side builds, tools/build_variant.sh: ADAM_G slab groups per block)
#ifndef ADAM_G
#define ADAM_G 16
#endif
constexpr int A4_G = ADAM_G, A4_T = 16 * A4_G, A4_U = 256 / A4_G;
static_assert(A4_U >= 4 && A4_U * A4_G == 256, "slab groups");
EM_DEVICE f32x4 slab_ld(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p)); }
struct Slab4Out {
  float g = 0.f;                  // threads < 64: grad_scale * sum over slabs of parameter blockIdx.x * 64 + t
  float w0 = 0.f, m0 = 0.f, v0 = 0.f;  // threads < 64 (with adam): the Adam operands, loaded under the slab loads
  float bc1 = 1.f, bc2 = 1.f;     // threads < 64 (with adam): bias corrections of step tstep
};
// (slice j = parameters 64 j .. 64 j + 63; callers that loop over slices sync before the next call)
EM_DEVICE Slab4Out slab4_reduce(int j, const float* __restrict__ slabs, int nslab, int stride, float grad_scale,
                                bool adam, int tstep, const float* __restrict__ params, const float* __restrict__ m,
                                const float* __restrict__ v, const float* __restrict__ hp) {
  __shared__ f32x4 part[A4_G][16];
  Slab4Out o;
  const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
  const float* src = slabs + j * 64 + 4 * q;
  if (adam && threadIdx.x < 64) {
    const int p = j * 64 + threadIdx.x;
    o.w0 = params[p];
    o.m0 = m[p];
    o.v0 = v[p];
  }
  f32x4 acc[4] = {f32x4{}, f32x4{}, f32x4{}, f32x4{}};
  int sl = g;
  for (; sl + (A4_U - 1) * A4_G < nslab; sl += A4_U * A4_G) {
    f32x4 t[A4_U];
#pragma unroll
    for (int k = 0; k < A4_U; ++k) t[k] = slab_ld(src + (size_t)(sl + k * A4_G) * stride);
    if (sl == g && adam && threadIdx.x < 64) {  // the fp64 chain runs while the loads are in flight
      o.bc1 = bias_correction(hp[1], tstep);
      o.bc2 = bias_correction(hp[2], tstep);
    }
#pragma unroll
    for (int k = 0; k < A4_U; ++k) acc[k & 3] += t[k];
  }
  if (nslab <= g + (A4_U - 1) * A4_G && adam && threadIdx.x < 64) {  // (no full block of slabs above)
    o.bc1 = bias_correction(hp[1], tstep);
    o.bc2 = bias_correction(hp[2], tstep);
  }
  for (; sl < nslab; sl += A4_G) acc[0] += slab_ld(src + (size_t)sl * stride);
  part[g][q] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (threadIdx.x < 64) {
    const int pq = threadIdx.x >> 2, e = threadIdx.x & 3;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < A4_G; ++k) t += part[k][pq][e];
    o.g = t * grad_scale;
  }
  return o;
}

// sum of the per-workgroup loss partials (one wave)
EM_DEVICE float loss_sum(const float* __restrict__ loss_slabs, int nslab, int lane) {
  float l = 0.f;
  for (int i = lane; i < nslab; i += 64) l += loss_slabs[i];
  return wave_sum(l);
}

__global__ void __launch_bounds__(A4_T)
adam_slab4_kernel(const float* __restrict__ slabs, int nslab, int P, int stride, float grad_scale,
                  float* __restrict__ params, float* __restrict__ m, float* __restrict__ v, float* __restrict__ grad_io,
                  const float* __restrict__ hp, int* __restrict__ state, int mode, uint8_t* __restrict__ mlp_img,
                  const float* __restrict__ loss_slabs, float* __restrict__ loss_out, float loss_scale, int pre) {
  // the step counter: only wave 0 (the 64 Adam lanes) needs it.  A plain load suffices -- the previous
  // kernel boundary published it, and this launch writes it (ticket mode) only after every block's
  // ticket -- whereas 1024 waves issuing an agent-scope atomic load of one word serialise on one L2 channel.
  int tstep = 0;
  if (mode != 1 && threadIdx.x < 64) tstep = state[0] + (pre ? 0 : 1);
  const Slab4Out o = slab4_reduce(blockIdx.x, slabs, nslab, stride, grad_scale, mode != 1, tstep, params, m, v, hp);
  if (blockIdx.x == 0 && loss_slabs && loss_out && threadIdx.x >= 64 && threadIdx.x < 128) {
    const float l = loss_sum(loss_slabs, nslab, threadIdx.x - 64);
    if (threadIdx.x == 64) loss_out[0] = l * loss_scale;
  }
  if (threadIdx.x < 64) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (mode == 1) grad_io[p] = o.g;
    else adam_apply_bc(p, o.g, o.w0, o.m0, o.v0, o.bc1, o.bc2, params, m, v, hp, mlp_img);
  }
  if (mode != 1 && !pre) adam_end(state, tstep);
}

// The data-parallel step's second (and last) launch over xGMI (xgmi.h, LL form): slice j (parameters
// 64j .. 64j + 63) is reduced from this rank's slabs exactly as adam_slab4_kernel does and stored as
// LL words {value, s} into slice j of the own LL slot (slice 0 adds the loss as element P); each of
// the 64 lanes then polls the N - 1 peers' words of its parameter until they carry tag s, sums the N
// values in rank order (bit-identical on every rank) and applies Adam.  No separate slab-reduction
// launch, no drain, flag or barrier: a slice travels as soon as it is reduced, in one round trip.
// (The round-5 block-flag form -- drained slot stores, a block flag, flag polls, then slot reads --
// was three round trips: tools/xgmi_budget.py, profiles/r5/.)
// One block per slice on a node (257 blocks); ranks that share a device launch fewer blocks that loop
// over the slices, so the spinning consumer leaves CUs free for a peer's whole-CU train kernel.
__global__ void __launch_bounds__(A4_T)
adam_slab_xgmi_kernel(XgmiDesc d, const float* __restrict__ slabs, int nslab, int stride, float grad_scale,
                      float* __restrict__ params, float* __restrict__ m, float* __restrict__ v,
                      const float* __restrict__ hp, int* __restrict__ state, uint8_t* __restrict__ mlp_img,
                      const float* __restrict__ loss_slabs, float* __restrict__ loss_out, float loss_scale,
                      int P, int pre) {
  const int s = xg_next_seq(d.my_hdr);
  int tstep = 0;
  if (threadIdx.x < 64) tstep = state[0] + (pre ? 0 : 1);
  __shared__ int bad;  // a peer wait of this block timed out: later slices skip their waits
  if (threadIdx.x == 0) bad = 0;
  for (int j = blockIdx.x; j < P / 64; j += gridDim.x) {
    __syncthreads();  // (bad initialised; the previous slice's LDS partials are consumed)
    const Slab4Out o = slab4_reduce(j, slabs, nslab, stride, grad_scale, true, tstep, params, m, v, hp);
    const int p = j * 64 + threadIdx.x;
    // LL exchange (xgmi.h): store this rank's words, then poll every peer's words of the slice
    if (threadIdx.x < 64) xg_ll_put(d, s, p, o.g);
    float lsum = 0.f;
    if (j == 0 && threadIdx.x >= 64 && threadIdx.x < 128) {
      const float l = loss_sum(loss_slabs, nslab, threadIdx.x - 64);
      if (threadIdx.x == 64) {
        lsum = l * loss_scale;
        xg_ll_put(d, s, P, lsum);
      }
    }
    bool ok = true;
    if (threadIdx.x < 64) {
      const float g = xg_ll_sum(d, s, p, o.g, ok, &bad);
      if (ok) adam_apply_bc(p, g, o.w0, o.m0, o.v0, o.bc1, o.bc2, params, m, v, hp, mlp_img);
    }
    if (j == 0 && threadIdx.x == 64) {
      const float l = xg_ll_sum(d, s, P, lsum, ok, &bad);
      if (ok && loss_out) loss_out[0] = l;
    }
  }
  xg_finish(d, s);
  if (!pre) adam_end(state, tstep);
}

__global__ void mlp_pack_kernel(const float* __restrict__ params, uint8_t* __restrict__ img) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P_TOTAL) return;
  mlp::pack_one(p, mlp::pad_slot(p) ? 0.f : params[p], img);
}

// plain multi-tensor-style Adam over a flat buffer (generic path: K6 for any model).  G = float, or
// __bf16 for gradients that were all-reduced in bf16 (GemmMLPTrainer comm_dtype="bf16"): they are
// widened here and the moments / master weights stay fp32.
template <typename G>
EM_DEVICE f32x4 load_grad4(const G* g) {
  if constexpr (sizeof(G) == 4) {
    return *reinterpret_cast<const f32x4*>(g);
  } else {
    const bf16x4 b = *reinterpret_cast<const bf16x4*>(g);
    return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
  }
}
template <typename G>
__global__ void __launch_bounds__(256)
adam_flat_kernel(float* __restrict__ params, const G* __restrict__ grad, float* __restrict__ m,
                 float* __restrict__ v, int64_t n, const float* __restrict__ hp, int* __restrict__ state,
                 float grad_scale, __bf16* __restrict__ shadow) {
  const int tstep = adam_begin(state);
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4];
  const float bc1 = bias_correction(b1, tstep), bc2 = bias_correction(b2, tstep);
  // AF_U float4 groups per thread per pass, every load of the pass issued before the first update
  // (one group per pass left a single 64-B round trip in flight per thread: 4.4 TB/s on 67 M params)
  constexpr int AF_U = 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  for (; i0 + (AF_U - 1) * stride + 4 <= n; i0 += AF_U * stride) {
    f32x4 w[AF_U], g[AF_U], mm[AF_U], vv[AF_U];
#pragma unroll
    for (int u = 0; u < AF_U; ++u) {
      const int64_t i4 = i0 + u * stride;
      w[u] = *reinterpret_cast<const f32x4*>(params + i4);
      g[u] = load_grad4<G>(grad + i4);
      mm[u] = *reinterpret_cast<const f32x4*>(m + i4);
      vv[u] = *reinterpret_cast<const f32x4*>(v + i4);
    }
#pragma unroll
    for (int u = 0; u < AF_U; ++u) {
      const int64_t i4 = i0 + u * stride;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gg = g[u][k] * grad_scale + wd * w[u][k];
        mm[u][k] = b1 * mm[u][k] + (1.f - b1) * gg;
        vv[u][k] = b2 * vv[u][k] + (1.f - b2) * gg * gg;
        w[u][k] -= lr * (mm[u][k] / bc1) / (sqrtf(vv[u][k] / bc2) + eps);
      }
      *reinterpret_cast<f32x4*>(params + i4) = w[u];
      *reinterpret_cast<f32x4*>(m + i4) = mm[u];
      *reinterpret_cast<f32x4*>(v + i4) = vv[u];
      if (shadow) {
        bf16x4 sb;
        sb[0] = (__bf16)w[u][0]; sb[1] = (__bf16)w[u][1]; sb[2] = (__bf16)w[u][2]; sb[3] = (__bf16)w[u][3];
        *reinterpret_cast<bf16x4*>(shadow + i4) = sb;
      }
    }
  }
  for (int64_t i4 = i0; i4 < n; i4 += stride) {
    if (i4 + 4 <= n) {
      f32x4 w = *reinterpret_cast<const f32x4*>(params + i4);
      f32x4 g = load_grad4<G>(grad + i4);
      f32x4 mm = *reinterpret_cast<const f32x4*>(m + i4);
      f32x4 vv = *reinterpret_cast<const f32x4*>(v + i4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gg = g[k] * grad_scale + wd * w[k];
        mm[k] = b1 * mm[k] + (1.f - b1) * gg;
        vv[k] = b2 * vv[k] + (1.f - b2) * gg * gg;
        w[k] -= lr * (mm[k] / bc1) / (sqrtf(vv[k] / bc2) + eps);
      }
      *reinterpret_cast<f32x4*>(params + i4) = w;
      *reinterpret_cast<f32x4*>(m + i4) = mm;
      *reinterpret_cast<f32x4*>(v + i4) = vv;
      if (shadow) {
        bf16x4 sb;
        sb[0] = (__bf16)w[0]; sb[1] = (__bf16)w[1]; sb[2] = (__bf16)w[2]; sb[3] = (__bf16)w[3];
        *reinterpret_cast<bf16x4*>(shadow + i4) = sb;
      }
    } else {
      for (int64_t i = i4; i < n; ++i) {
        float w = params[i];
        const float gg = (float)grad[i] * grad_scale + wd * w;
        const float mm = b1 * m[i] + (1.f - b1) * gg;
        const float vv = b2 * v[i] + (1.f - b2) * gg * gg;
        m[i] = mm;
        v[i] = vv;
        w -= lr * (mm / bc1) / (sqrtf(vv / bc2) + eps);
        params[i] = w;
        if (shadow) shadow[i] = (__bf16)w;
      }
    }
  }
  adam_end(state, tstep);
}

}  // namespace

EM_API int em_adam_slab(const float* slabs, int nslab, int P, int stride, float grad_scale, float* params, float* m, float* v,
                        float* grad_io, const float* hp, int* state, int mode, void* mlp_img, const float* loss_slabs,
                        float* loss_out, float loss_scale, hipStream_t stream) {
  const int pre = (mode & EM_ADAM_PRE) ? 1 : 0;
  mode &= ~EM_ADAM_PRE;
  if (mode < 0 || mode > 2) return EM_ERR_ARG;
  if (P <= 0 || (mode != 2 && (!slabs || nslab <= 0 || stride < P)) || (mode != 0 && !grad_io)) return EM_ERR_ARG;
  if (mode != 1 && (!params || !m || !v || !hp || !state)) return EM_ERR_ARG;
  if (mlp_img && P != P_TOTAL) return EM_ERR_ARG;
  const int nb = (P + AS_P - 1) / AS_P;
  if (mode != 2 && P % 64 == 0 && stride % 4 == 0 && ((uintptr_t)slabs & 15) == 0) {
    hipLaunchKernelGGL(adam_slab4_kernel, dim3(P / 64), dim3(A4_T), 0, stream, slabs, nslab, P, stride, grad_scale,
                       params, m, v, grad_io, hp, state, mode, (uint8_t*)mlp_img, loss_slabs, loss_out, loss_scale, pre);
    EM_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(adam_slab_kernel, dim3(nb), dim3(AS_P * AS_G), 0, stream, slabs, nslab, P, stride, grad_scale, params, m, v,
                     grad_io, hp, state, mode, (uint8_t*)mlp_img, loss_slabs, loss_out, loss_scale, pre);
  EM_CHECK_LAUNCH();
  return 0;
}

// The fused DP optimizer step (adam_slab_xgmi_kernel): slab reduction into the own xGMI LL slot,
// exchange, rank-order sum and Adam in ONE launch.  Needs P % 64 == 0 and a 16-B aligned slab array; max_blocks > 0
// caps the grid (ranks sharing a device);
// loss_out (optional) receives the reduced loss; pre = the step counter was already advanced by this
// step's train kernel (EM_ADAM_PRE).
EM_API int em_adam_slab_xgmi(void* xgmi, const float* slabs, int nslab, int stride, float grad_scale, int P, float* params,
                             float* m, float* v, const float* hp, int* state, void* mlp_img, const float* loss_slabs,
                             float* loss_out, float loss_scale, int pre, int max_blocks, hipStream_t stream) {
  XgmiComm* xc = static_cast<XgmiComm*>(xgmi);
  if (!xc || !xc->connected || P <= 0 || P % 64 || xc->desc.cap < P + 1 || !slabs || nslab <= 0 || stride < P ||
      stride % 4 || ((uintptr_t)slabs & 15) || !params || !m || !v || !hp || !state || !loss_slabs)
    return EM_ERR_ARG;
  if (mlp_img && P != P_TOTAL) return EM_ERR_ARG;
  int nb = P / 64;
  // blocks loop over slices past the grid; <= 1024 blocks stay co-resident (4 per CU), so no block
  // polls a peer while this rank's own block for the same slice is still waiting to be scheduled
  if (nb > 1024) nb = 1024;
  if (max_blocks > 0 && nb > max_blocks) nb = max_blocks;
  hipLaunchKernelGGL(adam_slab_xgmi_kernel, dim3(nb), dim3(A4_T), 0, stream, xc->desc, slabs, nslab, stride, grad_scale,
                     params, m, v, hp, state, (uint8_t*)mlp_img, loss_slabs, loss_out, loss_scale, P, pre ? 1 : 0);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_mlp_fused_pack(const float* params, void* img, hipStream_t stream) {
  if (!params || !img) return EM_ERR_ARG;
  hipLaunchKernelGGL(mlp_pack_kernel, dim3((P_TOTAL + 255) / 256), dim3(256), 0, stream, params, (uint8_t*)img);
  EM_CHECK_LAUNCH();
  return 0;
}

namespace {
// Flat-Adam grid: one 256-thread block per CU at most, each striding over the vector.  Measured on the wide
// MLP's 67.7 M parameters (kernel trace, profiles/r3/adam_flat_grid.txt): a 4096-block grid 472-500 µs,
// 1024 blocks 415-436, 512 blocks 400, one block per CU (256) 352-356 (5.8 TB/s), 384 blocks 418, 128 blocks 528.
int64_t flat_grid(int64_t n) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  int64_t nb = (n / 4 + 255) / 256;
  if (nb > cus) nb = cus;
  return nb < 1 ? 1 : nb;
}
}  // namespace

EM_API int em_adam_flat(float* params, const float* grad, float* m, float* v, int64_t n, const float* hp, int* state,
                        float grad_scale, void* shadow_bf16, hipStream_t stream) {
  if (!params || !grad || !m || !v || !hp || !state || n < 0) return EM_ERR_ARG;
  if (n == 0) return 0;
  const int64_t nb = flat_grid(n);
  hipLaunchKernelGGL(adam_flat_kernel<float>, dim3((unsigned)nb), dim3(256), 0, stream, params, grad, m, v, n, hp,
                     state, grad_scale, (__bf16*)shadow_bf16);
  EM_CHECK_LAUNCH();
  return 0;
}

// the same update from a bf16 gradient (all-reduced in bf16); grad must be 8-B aligned
EM_API int em_adam_flat_bf16g(float* params, const void* grad_bf16, float* m, float* v, int64_t n, const float* hp,
                              int* state, float grad_scale, void* shadow_bf16, hipStream_t stream) {
  if (!params || !grad_bf16 || !m || !v || !hp || !state || n < 0 || ((uintptr_t)grad_bf16 & 7)) return EM_ERR_ARG;
  if (n == 0) return 0;
  const int64_t nb = flat_grid(n);
  hipLaunchKernelGGL(adam_flat_kernel<__bf16>, dim3((unsigned)nb), dim3(256), 0, stream, params,
                     (const __bf16*)grad_bf16, m, v, n, hp, state, grad_scale, (__bf16*)shadow_bf16);
  EM_CHECK_LAUNCH();
  return 0;
}

namespace {
__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ src, __bf16* __restrict__ dst,
                                                            int64_t n) {
  for (int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i4 < n; i4 += (int64_t)gridDim.x * 256 * 4) {
    if (i4 + 4 <= n) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(src + i4);
      bf16x4 b;
      b[0] = (__bf16)x[0]; b[1] = (__bf16)x[1]; b[2] = (__bf16)x[2]; b[3] = (__bf16)x[3];
      *reinterpret_cast<bf16x4*>(dst + i4) = b;
    } else {
      for (int64_t i = i4; i < n; ++i) dst[i] = (__bf16)src[i];
    }
  }
}
}  // namespace

// fp32 -> bf16 (round to nearest even) of a gradient bucket before a bf16 all-reduce
EM_API int em_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (!src || !dst || n < 0 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 7)) return EM_ERR_ARG;
  if (n == 0) return 0;
  int64_t nb = (n / 4 + 255) / 256;
  if (nb > 8192) nb = 8192;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)nb), dim3(256), 0, stream, src, (__bf16*)dst, n);
  EM_CHECK_LAUNCH();
  return 0;
}
