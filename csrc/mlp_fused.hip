// K7 — fused persistent small-MLP training step for MI355X (gfx950).
//
// Model (BASELINE.json config 2): multi-hot 62-wide draw
// vector -> Linear(62,128) -> ReLU -> Linear(128,62) -> grouped softmax-CE
// (50 main numbers / 12 lucky stars) or sigmoid-BCE.  The reference declares
// DL4J for this (pom.xml:62-66) but never calls it; its only learner is
// XGBoost (Main.java:113-138), reproduced separately in gbdt.hip.
//
// One launch computes the forward, the loss, the backward and the per-workgroup
// weight-gradient partial sums for a whole mini-batch:
//   * 1 workgroup (4 waves) per CU, persistent over 32-sample tiles.
//   * Weights live in LDS as three bf16 images laid out so that EVERY weight
//     fragment is one conflict-free ds_read_b128 (packed by em_adam_pack).
//   * Samples are 8-byte draw rows (input draw t, target draw t+1).  The
//     multi-hot X tile is never materialised in HBM: each lane builds its MFMA
//     fragments from a 64-bit feature mask (bit 62 = constant-1 bias feature,
//     so b1 is row 62 of W1 and its gradient falls out of dW1 for free).
//   * Orientation is chosen so products chain accumulator->operand without LDS
//     (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand"):
//        F1  Z1ᵀ = W1ᵀ·Xᵀ         (samples on lanes)   -> relu -> Hᵀ (B operand)
//        F2  Z2ᵀ = W2ᵀ·Hᵀ + b2                         -> loss, dZ2ᵀ
//        R1  Z1  = X·W1           (same LDS frags as F1, operands swapped)
//        B1  dH  = dZ2·W2ᵀ        (dZ2ᵀ accumulator used as the A operand)
//        dW2 += Hᵀ·dZ2   dW1ᵀ += dZ1ᵀ·X   (K = samples: the two operands whose
//        sample axis sits on lanes go through a 4 KB wave-private LDS image and
//        come back with ds_read_b64_tr_b16; no workgroup barrier in the loop)
//   * dW accumulators (2 x 8 tiles x 16 regs = 256 regs) stay in AGPRs for the
//     whole launch; one wave per SIMD.  The 4 waves are summed through LDS at
//     the end and each workgroup writes ONE fp32 slab (deterministic; no atomics).
#include "common.h"

namespace {

constexpr int IN = 64, HID = 128, OUT = 64;
constexpr int P_W1 = 0, P_W2 = IN * HID, P_B2 = P_W2 + HID * OUT, P_TOTAL = P_B2 + OUT;  // 16448
constexpr int IMG_W1T = 0, IMG_W2P = 16384, IMG_W2Q = 32768, IMG_B2 = 49152, IMG_BYTES = 49408;

constexpr uint64_t MAIN_BITS = (1ull << 50) - 1;
constexpr uint64_t STAR_BITS = ((1ull << 12) - 1) << 50;
constexpr uint64_t BIAS_BIT = 1ull << 62;

EM_DEVICE uint64_t draw_mask(uint2 row) {
  uint64_t m = 0;
  const uint32_t w0 = row.x, w1 = row.y;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint32_t n = (k < 4) ? ((w0 >> (8 * k)) & 0xFF) : (w1 & 0xFF);
    m |= (n >= 1 && n <= 50) ? (1ull << (n - 1)) : 0ull;
  }
#pragma unroll
  for (int k = 1; k < 3; ++k) {
    uint32_t s = (w1 >> (8 * k)) & 0xFF;
    m |= (s >= 1 && s <= 12) ? (1ull << (49 + s)) : 0ull;
  }
  return m;
}

// byte offsets into the LDS weight images (see em_adam_pack for the writer)
EM_DEVICE uint32_t w1t_off(int row, int k8) { return IMG_W1T + row * 128 + ((k8 ^ ((row >> 1) & 7)) << 4); }
EM_DEVICE uint32_t w2p_off(int row, int k16) { return IMG_W2P + row * 256 + ((k16 ^ (row & 15)) << 4); }
EM_DEVICE uint32_t w2q_off(int row, int k8) { return IMG_W2Q + row * 128 + ((k8 ^ ((row >> 1) & 7)) << 4); }
// wave-private [32 samples][64 cols] bf16 image, 128-B rows, chunk ^= row&7
EM_DEVICE uint32_t img_off(uint32_t base, int row, int col) {
  return base + row * 128 + ((((col >> 3) ^ (row & 7))) << 4) + (col & 7) * 2;
}

// o(u,i,h) = 32u + (i&3) + 8(i>>2) + 4h : output index held in register i of Z2ᵀ tile u
EM_DEVICE constexpr int oo0(int i) { return (i & 3) + 8 * (i >> 2); }

template <int LOSS>  // 0 = grouped softmax CE (main 50 / stars 12), 1 = sigmoid BCE over 62
EM_DEVICE void loss_and_grad(const f32x16 (&z)[2], int h, uint64_t tmask, bool valid, float (&dz)[2][16],
                             float& loss_acc) {
  // per-slot class: 0 main, 1 star, 2 pad ; target bit per slot
  const uint32_t tm[2] = {(uint32_t)tmask >> (4 * h), (uint32_t)(tmask >> 32) >> (4 * h)};
  auto cls = [&](int u, int i) -> int {
    const int o = 32 * u + oo0(i) + 4 * h;
    return o < 50 ? 0 : (o < 62 ? 1 : 2);
  };
  if (LOSS == 0) {
    const int nm = __builtin_popcountll(tmask & MAIN_BITS), ns = __builtin_popcountll(tmask & STAR_BITS);
    const float inv_m = nm ? 1.f / (float)nm : 0.f, inv_s = ns ? 1.f / (float)ns : 0.f;
    float mx_m = -3.0e38f, mx_s = -3.0e38f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = cls(u, i);
        const float v = z[u][i];
        mx_m = (c == 0) ? fmaxf(mx_m, v) : mx_m;
        mx_s = (c == 1) ? fmaxf(mx_s, v) : mx_s;
      }
    mx_m = fmaxf(mx_m, __shfl_xor(mx_m, 32));
    mx_s = fmaxf(mx_s, __shfl_xor(mx_s, 32));
    float s_m = 0.f, s_s = 0.f, zt = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = cls(u, i);
        const float v = z[u][i];
        const float e = __expf(v - (c == 0 ? mx_m : mx_s));
        const float ee = (c == 2) ? 0.f : e;
        dz[u][i] = ee;
        s_m += (c == 0) ? ee : 0.f;
        s_s += (c == 1) ? ee : 0.f;
        const bool t = (tm[u] >> oo0(i)) & 1u;
        zt += t ? v * (c == 0 ? inv_m : inv_s) : 0.f;
      }
    s_m += __shfl_xor(s_m, 32);
    s_s += __shfl_xor(s_s, 32);
    const float r_m = nm ? 1.f / s_m : 0.f, r_s = ns ? 1.f / s_s : 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = cls(u, i);
        const bool t = (tm[u] >> oo0(i)) & 1u;
        const float pr = dz[u][i] * (c == 0 ? r_m : r_s);
        const float y = t ? (c == 0 ? inv_m : inv_s) : 0.f;
        dz[u][i] = (valid && c != 2) ? pr - y : 0.f;
      }
    float l = -zt;
    if (h == 0) l += (nm ? mx_m + __logf(s_m) : 0.f) + (ns ? mx_s + __logf(s_s) : 0.f);
    loss_acc += valid ? l : 0.f;
  } else {
    float l = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = cls(u, i);
        const float v = z[u][i];
        const float y = ((tm[u] >> oo0(i)) & 1u) ? 1.f : 0.f;
        const float en = __expf(-fabsf(v));
        const float p = v >= 0.f ? 1.f / (1.f + en) : en / (1.f + en);
        const float sp = fmaxf(v, 0.f) + __logf(1.f + en);  // softplus, stable
        const bool ok = valid && c != 2;
        dz[u][i] = ok ? (p - y) : 0.f;
        l += ok ? (sp - y * v) : 0.f;
      }
    loss_acc += l;
  }
}

EM_DEVICE bf16x8 relu_pack(const f32x16& a, int q) {
  return pack8(fmaxf(a[8 * q + 0], 0.f), fmaxf(a[8 * q + 1], 0.f), fmaxf(a[8 * q + 2], 0.f), fmaxf(a[8 * q + 3], 0.f),
               fmaxf(a[8 * q + 4], 0.f), fmaxf(a[8 * q + 5], 0.f), fmaxf(a[8 * q + 6], 0.f), fmaxf(a[8 * q + 7], 0.f));
}

// LDS layout of the train kernel (bytes):
//   [0, IMG_BYTES)                 weight images + b2 (copied from wimg)
//   per wave w at IMG_BYTES + w*WREG:  X image 4 KB | D2 image 4 KB | FRAG 8 KB
// Wave pairs (0,1) and (2,3) split the weight-gradient products: the even wave
// accumulates dW2 (A = H fragments) and the odd wave dW1ᵀ (A = dZ1 fragments)
// for BOTH tiles of the pair; each hands the other the fragments it does not
// keep through FRAG.  128 accumulator registers per wave instead of 256.
constexpr int WREG = 16384;
constexpr int TRAIN_LDS = IMG_BYTES + 4 * WREG + 4 * 64 * 4 + 64;

template <int LOSS>
__global__ void __launch_bounds__(256, 1)
mlp_fused_train_kernel(const uint8_t* __restrict__ draws, const int32_t* __restrict__ sidx, int64_t B,
                       int64_t offset, const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                       float* __restrict__ loss_slabs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const bool even = (wave & 1) == 0;

  {
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    for (int i = tid; i < IMG_BYTES / 16; i += 256) dst[i] = src[i];
  }
  __syncthreads();

  const uint32_t XB = IMG_BYTES + wave * WREG, DB = XB + 4096, FB = XB + 8192;
  const uint32_t pXB = IMG_BYTES + (wave ^ 1) * WREG, pDB = pXB + 4096, pFB = pXB + 8192;
  // the B-operand image this wave's dW product reads: D2 (even, dW2) or X (odd, dW1ᵀ)
  const uint32_t myB = even ? DB : XB, parB = even ? pDB : pXB;

  f32x16 dacc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) dacc[t][u] = f32x16{};
  float db2[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) db2[u][i] = 0.f;
  float loss_acc = 0.f;

  const int64_t ngroups = (B + 127) / 128;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;

  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t s = grp * 128 + wave * 32 + r;
    const bool valid = s < B;
    uint64_t imask = 0, tmask = 0;
    if (valid) {
      const int64_t idx = sidx ? (int64_t)sidx[s] : (offset + s);
      const uint2 rin = *reinterpret_cast<const uint2*>(draws + idx * 8);
      const uint2 rtg = *reinterpret_cast<const uint2*>(draws + (idx + 1) * 8);
      imask = draw_mask(rin) | BIAS_BIT;
      tmask = draw_mask(rtg);
    }
    bf16x8 xf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xf[q] = bits_to_bf16x8((uint32_t)(imask >> (16 * q + 8 * h)) & 0xFFu);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<bf16x8*>(smem + XB + r * 128 + ((((2 * q + h) ^ (r & 7))) << 4)) = xf[q];

    // ---- F1 (Z1ᵀ = W1ᵀ·Xᵀ) and R1 (Z1 = X·W1) per hidden tile: shared LDS fragments ----
    bf16x8 hT[4][2], hR[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = lds_frag(smem, w1t_off(32 * t + r, 2 * q + h));
      f32x16 a1 = f32x16{}, aR = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q) a1 = mfma32(w[q], xf[q], a1);
#pragma unroll
      for (int q = 0; q < 4; ++q) aR = mfma32(xf[q], w[q], aR);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        hT[t][q] = relu_pack(a1, q);
        hR[t][q] = relu_pack(aR, q);
      }
    }

    // ---- F2: Z2ᵀ = W2ᵀ·Hᵀ + b2 ----
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * u + 8 * g + 4 * h) * 4);
        z2[u][4 * g + 0] = b[0]; z2[u][4 * g + 1] = b[1]; z2[u][4 * g + 2] = b[2]; z2[u][4 * g + 3] = b[3];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          z2[u] = mfma32(lds_frag(smem, w2p_off(32 * u + r, (2 * t + q) * 2 + h)), hT[t][q], z2[u]);
    }

    // ---- loss + dZ2 (+ db2 partial sums) ----
    float dz[2][16];
    loss_and_grad<LOSS>(z2, h, tmask, valid, dz, loss_acc);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) db2[u][i] += dz[u][i];
    bf16x8 dzf[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        dzf[u][q] = pack8(dz[u][8 * q + 0], dz[u][8 * q + 1], dz[u][8 * q + 2], dz[u][8 * q + 3], dz[u][8 * q + 4],
                          dz[u][8 * q + 5], dz[u][8 * q + 6], dz[u][8 * q + 7]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x8 f = dzf[u][g >> 1];
        bf16x4 v;
        v[0] = f[4 * (g & 1) + 0]; v[1] = f[4 * (g & 1) + 1]; v[2] = f[4 * (g & 1) + 2]; v[3] = f[4 * (g & 1) + 3];
        *reinterpret_cast<bf16x4*>(smem + DB + r * 128 + ((((4 * u + g) ^ (r & 7))) << 4) + h * 8) = v;
      }

    // ---- B1: dH = dZ2·W2ᵀ, dZ1 = dH * (Z1 > 0) ----
    bf16x8 keep[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 aD = f32x16{};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          aD = mfma32(dzf[u][q], lds_frag(smem, w2q_off(32 * t + r, (2 * u + q) * 2 + h)), aD);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bf16x8 d;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = (__bf16)((float)hR[t][q][j] > 0.f ? aD[8 * q + j] : 0.f);
        // even keeps H (dW2), hands dZ1 to the odd partner; odd keeps dZ1 (dW1ᵀ), hands H
        const bf16x8 give = even ? d : hR[t][q];
        keep[t][q] = even ? hR[t][q] : d;
        *reinterpret_cast<bf16x8*>(smem + FB + ((t * 2 + q) * 64 + lane) * 16) = give;
      }
    }

    __syncthreads();  // partner's X / D2 / FRAG images are complete

    // ---- dW (K = 32 samples per tile, own tile + partner tile) ----
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int col = 32 * u + 16 * g1 + 4 * p4;
        const int r0 = 16 * q + 4 * h + q4;
        const bf16x8 bo = cat_tr(lds_tr16(smem, img_off(myB, r0, col)), lds_tr16(smem, img_off(myB, r0 + 8, col)));
        const bf16x8 bp = cat_tr(lds_tr16(smem, img_off(parB, r0, col)), lds_tr16(smem, img_off(parB, r0 + 8, col)));
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          dacc[t][u] = mfma32(keep[t][q], bo, dacc[t][u]);
          dacc[t][u] = mfma32(lds_frag(smem, pFB + ((t * 2 + q) * 64 + lane) * 16), bp, dacc[t][u]);
        }
      }

    __syncthreads();  // images are overwritten next round
  }

  // ================= epilogue: per-workgroup reduction =================
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float v = db2[u][i];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o);
      db2[u][i] = v;
    }
  const float lsum = wave_sum(loss_acc);
  float* RED = reinterpret_cast<float*>(smem);  // 2 x 32 KB (waves 0 and 1 publish)
  float* DB2S = reinterpret_cast<float*>(smem + IMG_BYTES + 4 * WREG);
  float* LOSSS = DB2S + 4 * 64;
  // (the loop ended with a barrier: LDS images are free)
  if (r == 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) DB2S[wave * 64 + 32 * u + oo0(i) + 4 * h] = db2[u][i];
  }
  if (lane == 0) LOSSS[wave] = lsum;
  if (wave < 2) {
    float* R = RED + wave * 8192;
#pragma unroll
    for (int T = 0; T < 8; ++T)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& acc = dacc[T >> 1][T & 1];
        *reinterpret_cast<f32x4*>(R + ((T * 4 + g) * 64 + lane) * 4) =
            f32x4{acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
      }
  }
  __syncthreads();
  float* slab = slabs + (size_t)blockIdx.x * P_TOTAL;
  if (wave >= 2) {
    const float* R = RED + (wave - 2) * 8192;
#pragma unroll
    for (int T = 0; T < 8; ++T) {
      const int t = T >> 1, u = T & 1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& acc = dacc[t][u];
        const f32x4 v = *reinterpret_cast<const f32x4*>(R + ((T * 4 + g) * 64 + lane) * 4) +
                        f32x4{acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
        const int c0 = 32 * t + 8 * g + 4 * h;  // hidden rows c0..c0+3
        if (wave == 2) {  // dW2[c][o], o = 32u + r
#pragma unroll
          for (int k = 0; k < 4; ++k) slab[P_W2 + (c0 + k) * OUT + 32 * u + r] = v[k];
        } else {  // dW1ᵀ tile -> W1[f][c], f = 32u + r
          *reinterpret_cast<f32x4*>(slab + P_W1 + (32 * u + r) * HID + c0) = v;
        }
      }
    }
  }
  if (tid < 64) slab[P_B2 + tid] = DB2S[tid] + DB2S[64 + tid] + DB2S[128 + tid] + DB2S[192 + tid];
  if (tid == 0) loss_slabs[blockIdx.x] = LOSSS[0] + LOSSS[1] + LOSSS[2] + LOSSS[3];
}

// Forward only: logits [B, 64] fp32 (cols 62/63 padding).  F1+F2 of the train kernel.
__global__ void __launch_bounds__(256)
mlp_fused_forward_kernel(const uint8_t* __restrict__ draws, const int32_t* __restrict__ sidx, int64_t B,
                         int64_t offset, const uint8_t* __restrict__ wimg, float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    for (int i = tid; i < IMG_BYTES / 16; i += 256) dst[i] = src[i];
  }
  __syncthreads();
  const int64_t ntiles = (B + 31) / 32;
  const int nwaves = gridDim.x * 4;
  for (int64_t tile = blockIdx.x * 4 + wave; tile < ntiles; tile += nwaves) {
    const int64_t s = tile * 32 + r;
    const bool valid = s < B;
    uint64_t imask = 0;
    if (valid) {
      const int64_t idx = sidx ? (int64_t)sidx[s] : (offset + s);
      imask = draw_mask(*reinterpret_cast<const uint2*>(draws + idx * 8)) | BIAS_BIT;
    }
    bf16x8 xf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xf[q] = bits_to_bf16x8((uint32_t)(imask >> (16 * q + 8 * h)) & 0xFFu);
    f32x16 a1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      a1[t] = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q) a1[t] = mfma32(lds_frag(smem, w1t_off(32 * t + r, 2 * q + h)), xf[q], a1[t]);
    }
    bf16x8 hT[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        hT[t][q] = pack8(fmaxf(a1[t][8 * q + 0], 0.f), fmaxf(a1[t][8 * q + 1], 0.f), fmaxf(a1[t][8 * q + 2], 0.f),
                         fmaxf(a1[t][8 * q + 3], 0.f), fmaxf(a1[t][8 * q + 4], 0.f), fmaxf(a1[t][8 * q + 5], 0.f),
                         fmaxf(a1[t][8 * q + 6], 0.f), fmaxf(a1[t][8 * q + 7], 0.f));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      f32x16 z;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * u + 8 * g + 4 * h) * 4);
        z[4 * g + 0] = b[0]; z[4 * g + 1] = b[1]; z[4 * g + 2] = b[2]; z[4 * g + 3] = b[3];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          z = mfma32(lds_frag(smem, w2p_off(32 * u + r, (2 * t + q) * 2 + h)), hT[t][q], z);
      if (valid) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = {z[4 * g + 0], z[4 * g + 1], z[4 * g + 2], z[4 * g + 3]};
          *reinterpret_cast<f32x4*>(logits + s * OUT + 32 * u + 8 * g + 4 * h) = v;
        }
      }
    }
  }
}

}  // namespace

EM_API int em_mlp_fused_param_count() { return P_TOTAL; }
EM_API int em_mlp_fused_image_bytes() { return IMG_BYTES; }
EM_API int em_mlp_fused_lds_bytes() { return TRAIN_LDS; }

// draws: [ndraws, 8] uint8; sample s = (draws[i], draws[i+1]) with i = sidx ? sidx[s] : offset+s
EM_API int em_mlp_fused_train(const uint8_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                              const void* wimg, float* slabs, float* loss_slabs, int nslab, int loss_kind,
                              hipStream_t stream) {
  if (!draws || !wimg || !slabs || !loss_slabs || nslab <= 0 || B < 0) return EM_ERR_ARG;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              TRAIN_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              TRAIN_LDS);
    attr_set = true;
  }
  if (loss_kind == 0)
    hipLaunchKernelGGL(mlp_fused_train_kernel<0>, dim3(nslab), dim3(256), TRAIN_LDS, stream, draws, sidx, B, offset,
                       (const uint8_t*)wimg, slabs, loss_slabs);
  else
    hipLaunchKernelGGL(mlp_fused_train_kernel<1>, dim3(nslab), dim3(256), TRAIN_LDS, stream, draws, sidx, B, offset,
                       (const uint8_t*)wimg, slabs, loss_slabs);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_mlp_fused_forward(const uint8_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                                const void* wimg, float* logits, int nblocks, hipStream_t stream) {
  if (!draws || !wimg || !logits || nblocks <= 0) return EM_ERR_ARG;
  hipLaunchKernelGGL(mlp_fused_forward_kernel, dim3(nblocks), dim3(256), IMG_BYTES, stream, draws, sidx, B, offset,
                     (const uint8_t*)wimg, logits);
  EM_CHECK_LAUNCH();
  return 0;
}
