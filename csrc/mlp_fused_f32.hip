// K7-f32 -- fused small-MLP training step in exact fp32 for MI355X (gfx950).
//
// The same model, sample format, gradient slabs and Adam as the bf16 kernel (csrc/mlp_fused.hip), for
// the fp32 configuration ND4J runs by default (pom.xml:62-66: DL4J's default dtype).  Every product is
// a v_mfma_f32_32x32x2_f32 on fp32 operands (exact fp32 products, fp32 accumulation), so this kernel is
// matrix-bound by construction: 640 MFMAs x 64 cycles per 32-sample tile against ~1 k VALU / LDS
// instructions that issue beside them.  That changes the design against the bf16 kernel:
//   * no producer/consumer ring: one wave runs forward, loss and backward of its own tiles
//     (4 waves per workgroup, one per SIMD, one workgroup per CU); a dependent 32x32x2 f32 MFMA chain
//     runs at full rate (accumulator latency == issue), so single chains keep the pipe busy;
//   * the weight gradients dW1^T (128 x 64) and dW2 (128 x 64) stay in the wave's 256 AGPRs for the
//     whole launch; the weights are read from fp32 LDS images as MFMA operands (one dword per lane
//     per MFMA, far below the LDS rate);
//   * orientation (32x32x2: lane l supplies A[l & 31][l >> 5] and B[l >> 5][l & 31]; C lane l holds
//     column l & 31, rows 8(i >> 2) + 4(l >> 5) + (i & 3)):
//        F1  Z1[c][s]  = sum_f W1T[c][f] X[f][s]       k = f = s0 + 32h (consecutive per lane: b128 reads)
//        F2  Z2[o][s]  = sum_c W2[c][o] H[c][s] + b2   k = c = 32t + 8g + 4h + e: H is the accumulator
//                                                       register 4g + e of the lane -- no data movement
//        dH  dH[c][s]  = sum_o W2[c][o] dZ2[o][s]      k = o, dZ2 from its staged image
//        dW2 dW2[c][o] += sum_s H[c][s] dZ2[o][s]      k = samples: H / dZ2 staged in LDS [row][sample]
//        dW1 dW1T[c][f] += sum_s dZ1[c][s] X[f][s]     dZ1 staged the same way, X from the sample masks
//   * the loss is the bf16 kernel's per-tile softmax-CE / sigmoid-BCE (mlp_loss.h, same layout);
//   * the four waves' gradients meet in LDS in wave order and leave as ONE parameter-order slab per
//     workgroup (the bf16 kernel's slab format: em_adam_slab reduces them, bit-reproducible).
#include <cstdlib>

#include "common.h"
#include "mlp_adam.h"
#include "mlp_loss.h"

namespace {
using mlp::HID, mlp::OUT, mlp::P_W1, mlp::P_W2, mlp::P_B2, mlp::P_TOTAL;

constexpr int F32_NT = 256;
constexpr int F32_SLAB_STRIDE = 16640;  // == SLAB_STRIDE of csrc/mlp_fused.hip (the shared slab format)
constexpr uint64_t F32_BIAS_BIT = 1ull << 62;
// LDS (bytes).  Row paddings keep the operand reads conflict-free (see each reader).
constexpr int F32_RS1 = 68;   // W1T [128 c][68]: F1 reads 16 B at row c, column s0 + 32h
constexpr int F32_RS2 = 72;   // W2  [128 c][72]: F2 reads one dword at (c, o), c + 4 for h = 1 -> banks + 32
constexpr int F32_RST = 36;   // staged [row][36]: 32 samples + pad, 16-B reads at column j0 + 16h
constexpr int F32_W1T = 0;
constexpr int F32_W2 = F32_W1T + 128 * F32_RS1 * 4;          // 34816
constexpr int F32_B2 = F32_W2 + 128 * F32_RS2 * 4;           // 71680
constexpr int F32_YLUT = F32_B2 + 256;                       // 16 x f32x4 target nibble table
constexpr int F32_WAVE = F32_YLUT + 256;                     // per-wave staging
constexpr int F32_DZ = 0, F32_T = 64 * F32_RST * 4, F32_MASK = 2 * 64 * F32_RST * 4;
constexpr int F32_ACC = F32_MASK + 32 * 8;                   // [64 lanes] db2 + [64 lanes] loss, kept in LDS
constexpr int F32_WAVE_BYTES = F32_ACC + 2 * 64 * 4;         // 19200
constexpr int F32_LDS = F32_WAVE + 4 * F32_WAVE_BYTES;       // 148992
// end of launch: the fold image (register layout of the accumulators, conflict-free) reuses the LDS
constexpr int F32_FOLD_FLOATS = 2 * 8 * 16 * 64 + 64;         // dW1T + dW2 partials + b2
static_assert(F32_FOLD_FLOATS * 4 <= F32_LDS, "fold image must fit");

EM_DEVICE f32x16 mfma_f32(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int LOSS>
__global__ void __launch_bounds__(F32_NT, 1)
mlp_fused_train_f32_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                           const float* __restrict__ params, float* __restrict__ slabs,
                           float* __restrict__ loss_slabs, int* __restrict__ step) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (step && blockIdx.x == 0 && tid == 0) step[0] = step[0] + 1;  // em_adam_slab pre mode (as the bf16 kernel)
  // ---- weight images from the fp32 master parameters
  for (int p = tid; p < P_W2; p += F32_NT) {  // W1[f][c] -> W1T[c][f]
    const int f = p >> 7, c = p & 127;
    reinterpret_cast<float*>(smem + F32_W1T)[c * F32_RS1 + f] = params[P_W1 + p];
  }
  for (int q = tid; q < HID * OUT; q += F32_NT) {  // W2[c][o]
    const int c = q >> 6, o = q & 63;
    reinterpret_cast<float*>(smem + F32_W2)[c * F32_RS2 + o] = params[P_W2 + q];
  }
  if (tid < 64) {
    reinterpret_cast<float*>(smem + F32_B2)[tid] = params[P_B2 + tid];
    reinterpret_cast<float*>(smem + F32_YLUT)[tid] = (float)(((tid >> 2) >> (tid & 3)) & 1);
  }
  __syncthreads();

  const float* W1T = reinterpret_cast<const float*>(smem + F32_W1T);
  const float* W2 = reinterpret_cast<const float*>(smem + F32_W2);
  const float* B2 = reinterpret_cast<const float*>(smem + F32_B2);
  char* ws = smem + F32_WAVE + wave * F32_WAVE_BYTES;
  float* DZI = reinterpret_cast<float*>(ws + F32_DZ);  // [64 o][36]: dZ2 of the tile
  float* TI = reinterpret_cast<float*>(ws + F32_T);    // [64 c][36]: half of H, then half of dZ1
  uint64_t* MI = reinterpret_cast<uint64_t*>(ws + F32_MASK);
  // the lane's db2 (lane = output o) and loss sums live in LDS between tiles: as loop-carried registers
  // the allocator spilled them to scratch inside the loop
  float* ACC = reinterpret_cast<float*>(ws + F32_ACC);
  ACC[lane] = 0.f;
  ACC[64 + lane] = 0.f;

  f32x16 gw1[4][2], gw2[4][2];  // dW1T [c tile][f tile], dW2 [c tile][o tile]: the launch's accumulators
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) gw1[t][j] = gw2[t][j] = f32x16{};

  const int nwav = gridDim.x * 4, ntiles = (B + 31) / 32;
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += nwav) {
    const int s = tile * 32 + r;
    const bool valid = s < B;
    uint64_t xm = 0, tm = 0;
    if (valid) {
      const int idx = sidx ? sidx[s] : offset + s;
      xm = masks[idx] | F32_BIAS_BIT;
      tm = masks[idx + 1];
    }
    if (h == 0) MI[r] = xm;
    const uint32_t xw = h ? (uint32_t)(xm >> 32) : (uint32_t)xm;  // this lane's k half of the features

    // ---- F1: Z1[c][s] over f = s0 + 32h.  Each phase below loads the NEXT group's operands before the
    // current group's MFMAs, with sched_barriers between (left alone the scheduler hoists every LDS
    // read of a phase to its top and spills)
    f32x16 z1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) z1[t] = f32x16{};
    {
      f32x4 a[2][4];
      auto ld = [&](int buf, int s0) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          a[buf][t] = *reinterpret_cast<const f32x4*>(W1T + (32 * t + r) * F32_RS1 + s0 + 32 * h);
      };
      ld(0, 0);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8) ld((q + 1) & 1, 4 * (q + 1));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xb = (float)__builtin_amdgcn_ubfe(xw, 4 * q + e, 1);
#pragma unroll
          for (int t = 0; t < 4; ++t) z1[t] = mfma_f32(a[q & 1][t][e], xb, z1[t]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) z1[t][i] = z1[t][i] > 0.f ? z1[t][i] : 0.f;  // H (a select: fmaxf adds a canonicalize)

    // ---- F2: Z2[o][s] = b2 + sum over c = 32t + 8g + 4h + e of W2[c][o] H[c][s]
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) z2[u][i] = B2[32 * u + oo0(i) + 4 * h];
    {
      float w[2][8][2];  // group q = (t, i half): [buffer][i][u]
      auto ld = [&](int buf, int q) __attribute__((always_inline)) {
#pragma unroll
        for (int ii = 0; ii < 8; ++ii) {
          const int c = 32 * (q >> 1) + oo0(8 * (q & 1) + ii) + 4 * h;
#pragma unroll
          for (int u = 0; u < 2; ++u) w[buf][ii][u] = W2[c * F32_RS2 + 32 * u + r];
        }
      };
      ld(0, 0);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q + 1 < 8) ld((q + 1) & 1, q + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ii = 0; ii < 8; ++ii)
#pragma unroll
          for (int u = 0; u < 2; ++u) z2[u] = mfma_f32(w[q & 1][ii][u], z1[q >> 1][8 * (q & 1) + ii], z2[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // relu mask of H (one bit per H register), and H's first half [c][s] into LDS now: the softmax
    // below runs with 32 H registers live instead of 64
    uint32_t hb[2] = {0u, 0u};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) hb[t >> 1] |= (z1[t][i] > 0.f ? 1u : 0u) << (16 * (t & 1) + i);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 16; ++i) TI[(32 * tt + oo0(i) + 4 * h) * F32_RST + r] = z1[tt][i];

    // ---- loss and dZ2 (the bf16 kernel's tile loss, same accumulator layout)
    float dz[2][16];
    float lt = 0.f;
    if (LOSS == 0) {
      auto hook = [](auto&& stepf) {
#pragma unroll
        for (int j = 0; j < 8; ++j) stepf(j);
      };
      v6_softmax_split<F32_WAVE - 256, false>(smem, z2, valid ? tm : 0ull, h, dz, lt, hook);
    } else {
      bce_tile_loss<F32_WAVE - 256>(smem, z2, valid ? tm : 0ull, valid, h, dz, lt);
    }
    ACC[64 + lane] += lt;

    // ---- stage dZ2 [o][s]; db2 += its row sums (lane o sums its row in a fixed order)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) DZI[(32 * u + oo0(i) + 4 * h) * F32_RST + r] = dz[u][i];
    wave_lds_sync();
    {
      float rs = 0.f;
#pragma unroll
      for (int j0 = 0; j0 < 32; j0 += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(DZI + lane * F32_RST + j0);
        rs += (v[0] + v[1]) + (v[2] + v[3]);
      }
      ACC[lane] += rs;
    }

    // ---- dW2[c][o] += sum_s H[c][s] dZ2[o][s], K = the tile's samples (s = j + 16h per lane)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half)  // (the first half was staged before the softmax)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int i = 0; i < 16; ++i) TI[(32 * tt + oo0(i) + 4 * h) * F32_RST + r] = z1[2 + tt][i];
      wave_lds_sync();
#pragma unroll
      for (int j0 = 0; j0 < 16; j0 += 4) {
        f32x4 a[2], b[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) a[tt] = *reinterpret_cast<const f32x4*>(TI + (32 * tt + r) * F32_RST + j0 + 16 * h);
#pragma unroll
        for (int u = 0; u < 2; ++u) b[u] = *reinterpret_cast<const f32x4*>(DZI + (32 * u + r) * F32_RST + j0 + 16 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int u = 0; u < 2; ++u) gw2[2 * half + tt][u] = mfma_f32(a[tt][e], b[u][e], gw2[2 * half + tt][u]);
      }
      wave_lds_sync();
    }

    // ---- dH[c][s] = sum over o = 32u + 8g + 4h + e of W2[c][o] dZ2[o][s]; relu' -> dZ1 -> dW1T
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * half + tt;
        f32x16 dh = f32x16{};
        f32x4 a[2][4];  // group u: [buffer][g]
        auto ld = [&](int buf, int u) __attribute__((always_inline)) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
            a[buf][g] = *reinterpret_cast<const f32x4*>(W2 + (32 * t + r) * F32_RS2 + 32 * u + 8 * g + 4 * h);
        };
        ld(0, 0);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u == 0) ld(1, 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e)  // dZ2 back from its LDS image: its registers died after staging
              dh = mfma_f32(a[u][g][e], DZI[(32 * u + 8 * g + 4 * h + e) * F32_RST + r], dh);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          TI[(32 * tt + oo0(i) + 4 * h) * F32_RST + r] = ((hb[half] >> (16 * tt + i)) & 1u) ? dh[i] : 0.f;
      }
      wave_lds_sync();
      // dW1T for these c tiles: A = dZ1 [c][s], B = X [s][f] from the tile's masks
#pragma unroll
      for (int j0 = 0; j0 < 16; j0 += 4) {
        f32x4 a[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) a[tt] = *reinterpret_cast<const f32x4*>(TI + (32 * tt + r) * F32_RST + j0 + 16 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint64_t m = MI[j0 + e + 16 * h];
#pragma unroll
          for (int fb = 0; fb < 2; ++fb) {
            const float xb = (float)__builtin_amdgcn_ubfe(fb ? (uint32_t)(m >> 32) : (uint32_t)m, r, 1);
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) gw1[2 * half + tt][fb] = mfma_f32(a[tt][e], xb, gw1[2 * half + tt][fb]);
          }
        }
      }
      wave_lds_sync();
    }
  }

  // ---- fold the four waves' partials in wave order, then one parameter-order slab
  __syncthreads();  // every wave is past its last LDS read of the weight and staging images
  float* FO = reinterpret_cast<float*>(smem);  // [2 (w1, w2)][8 (t, j)][16 i][64 lane] + b2[64]
  const float gb2 = ACC[lane], loss_acc = ACC[64 + lane];
  __syncthreads();
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            float* p1 = FO + ((t * 2 + j) * 16 + i) * 64 + lane;
            float* p2 = p1 + 8 * 16 * 64;
            *p1 = w ? *p1 + gw1[t][j][i] : gw1[t][j][i];
            *p2 = w ? *p2 + gw2[t][j][i] : gw2[t][j][i];
          }
      float* pb = FO + 2 * 8 * 16 * 64 + lane;
      *pb = w ? *pb + gb2 : gb2;
      const float lw = wave_sum(loss_acc);
      if (lane == 0) FO[F32_FOLD_FLOATS + w] = lw;
    }
    __syncthreads();
  }
  float* slab = slabs + (size_t)blockIdx.x * F32_SLAB_STRIDE;
  for (int p = tid; p < P_TOTAL; p += F32_NT) {
    float v;
    if (p < P_W2) {  // W1[f][c] = dW1T[c][f]: tile (c >> 5, f >> 5), lane f & 31 + 32 h, register i
      const int f = p >> 7, c = p & 127, cc = c & 31;
      const int i = ((cc >> 3) << 2) | (cc & 3), hh = (cc >> 2) & 1;
      v = FO[(((c >> 5) * 2 + (f >> 5)) * 16 + i) * 64 + (f & 31) + 32 * hh];
    } else if (p < P_B2) {  // W2[c][o] = dW2 tile (c >> 5, o >> 5), lane o & 31 + 32 h
      const int q = p - P_W2, c = q >> 6, o = q & 63, cc = c & 31;
      const int i = ((cc >> 3) << 2) | (cc & 3), hh = (cc >> 2) & 1;
      v = FO[8 * 16 * 64 + (((c >> 5) * 2 + (o >> 5)) * 16 + i) * 64 + (o & 31) + 32 * hh];
    } else {
      v = FO[2 * 8 * 16 * 64 + (p - P_B2)];
    }
    slab[p] = v;
  }
  if (tid == 0) {
    const float* LW = FO + F32_FOLD_FLOATS;
    loss_slabs[blockIdx.x] = ((LW[0] + LW[1]) + LW[2]) + LW[3];
  }
}

}  // namespace

EM_API int em_mlp_fused_f32_lds_bytes() { return F32_LDS; }

// The exact-fp32 train kernel: same arguments and slab output as em_mlp_fused_train, with the fp32
// master parameters (P_TOTAL floats, parameter order) in place of the bf16 weight images.
EM_API int em_mlp_fused_train_f32(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                                  const float* params, float* slabs, float* loss_slabs, int nslab, int loss_kind,
                                  int* step, hipStream_t stream) {
  if (draws && !sidx && offset > 0) {
    draws += offset;
    offset = 0;
  }
  if (!draws || !params || !slabs || !loss_slabs || nslab <= 0 || B < 0 || offset < 0 ||
      B + offset + 1 > (int64_t)INT32_MAX)
    return EM_ERR_ARG;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_f32_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F32_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_f32_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F32_LDS);
    attr = true;
  }
  if (loss_kind == 0)
    hipLaunchKernelGGL(mlp_fused_train_f32_kernel<0>, dim3(nslab), dim3(F32_NT), F32_LDS, stream, draws, sidx, (int)B,
                       (int)offset, params, slabs, loss_slabs, step);
  else
    hipLaunchKernelGGL(mlp_fused_train_f32_kernel<1>, dim3(nslab), dim3(F32_NT), F32_LDS, stream, draws, sidx, (int)B,
                       (int)offset, params, slabs, loss_slabs, step);
  EM_CHECK_LAUNCH();
  return 0;
}
