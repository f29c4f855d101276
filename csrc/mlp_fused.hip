// K7 — fused persistent small-MLP training step for MI355X (gfx950).
// EM_BUILD_FLAGS: -mllvm -amdgpu-mfma-vgpr-form=1
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
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int IN = 64, HID = 128, OUT = 64;
constexpr int P_W1 = 0, P_W2 = IN * HID, P_B2 = P_W2 + HID * OUT, P_TOTAL = P_B2 + OUT;  // 16448
// gradient slabs are SLAB_STRIDE floats apart (P_TOTAL rounded to an odd multiple of 256 B so the
// cross-slab reduction in em_adam_slab does not hit the same HBM channel for every slab)
constexpr int SLAB_STRIDE = 16640;
// weight images with padded rows (144 B / 272 B: 16 consecutive rows start in distinct 16-B bank
// groups, so the 16-lane phases of ds_read_b128 are conflict-free) instead of an XOR swizzle: a
// fragment address is then one per-lane base + an immediate, not one VGPR per (row, chunk) pair
constexpr int W1T_RS = 144, W2P_RS = 272, W2Q_RS = 144;
constexpr int IMG_W1T = 0, IMG_W2P = IMG_W1T + 128 * W1T_RS, IMG_W2Q = IMG_W2P + 64 * W2P_RS,
              IMG_B2 = IMG_W2Q + 128 * W2Q_RS, IMG_BYTES = IMG_B2 + 256;  // 54528

constexpr uint64_t MAIN_BITS = (1ull << 50) - 1;
constexpr uint64_t STAR_BITS = ((1ull << 12) - 1) << 50;
constexpr uint64_t BIAS_BIT = 1ull << 62;

// Samples are read as precomputed 64-bit feature masks (bit n-1: main number n, bit 49+s: star s;
// em_rows_to_masks builds them once per dataset), so the hot loop spends no VALU on decoding rows.

// 256-entry LDS table: byte b -> 8 bf16 {0,1} (element j = bit j); an X fragment is one ds_read_b128
constexpr int LUT_BYTES = 4096;
EM_DEVICE void fill_lut(char* lut, int tid) {
  if (tid < 256) *reinterpret_cast<bf16x8*>(lut + tid * 16) = bits_to_bf16x8((uint32_t)tid);
}
EM_DEVICE bf16x8 lut_frag(const char* lut, uint64_t m, int q, int h) {
  const uint32_t w = q < 2 ? (uint32_t)m : (uint32_t)(m >> 32);
  const uint32_t byte = (w >> (16 * (q & 1) + 8 * h)) & 0xFFu;
  return *reinterpret_cast<const bf16x8*>(lut + byte * 16);
}

// byte offsets into the LDS weight images (see em_adam_pack for the writer)
EM_DEVICE uint32_t w1t_off(int row, int k8) { return IMG_W1T + row * W1T_RS + k8 * 16; }
EM_DEVICE uint32_t w2p_off(int row, int k16) { return IMG_W2P + row * W2P_RS + k16 * 16; }
EM_DEVICE uint32_t w2q_off(int row, int k8) { return IMG_W2Q + row * W2Q_RS + k8 * 16; }
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
  const uint32_t tm[2] = {(uint32_t)tmask >> (4 * h), (uint32_t)(tmask >> 32) >> (4 * h)};  // slot bits
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

typedef short s16x2 __attribute__((ext_vector_type(2)));

// NOTE (ROCm 7.2 clang): `__builtin_bit_cast(s16x2, v[k])` on an element of an ext_vector inside an
// unrolled loop is miscompiled (every k reads element 0).  These memcpy-based casts compile to the
// expected one v_pk_* per dword; tests/test_fused_mlp_gpu.py checks logits and gradients end to end.
EM_DEVICE s16x2 as_s16x2(uint32_t x) {
  s16x2 r;
  __builtin_memcpy(&r, &x, 4);
  return r;
}
EM_DEVICE uint32_t as_u32(s16x2 x) {
  uint32_t r;
  __builtin_memcpy(&r, &x, 4);
  return r;
}

// relu on packed bf16 pairs: for sign-magnitude bf16, max(x, 0) as int16 == relu (one v_pk_max_i16 per 2 values)
EM_DEVICE bf16x8 relu_pack(const f32x16& a, int q) {
  const bf16x8 p = pack8(a[8 * q + 0], a[8 * q + 1], a[8 * q + 2], a[8 * q + 3], a[8 * q + 4], a[8 * q + 5],
                         a[8 * q + 6], a[8 * q + 7]);
  u32x4 d = __builtin_bit_cast(u32x4, p);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = d[k];
    d[k] = as_u32(__builtin_elementwise_max(as_s16x2(x), (s16x2){0, 0}));
  }
  return __builtin_bit_cast(bf16x8, d);
}

// dZ1 = dH * (Z1 > 0) on packed bf16: the relu'd H fragment is 0 exactly where Z1 <= 0 and a
// positive bf16 (bits 0x0001..0x7f7f) otherwise, so min_u16(h, 1) is the 0/1 mask and a 16-bit
// integer multiply applies it (v_pk_min_u16 + v_pk_mul_lo_u16 per two values)
EM_DEVICE bf16x8 mask_by(const bf16x8 hfrag, const f32x16& a, int q) {
  const bf16x8 p = pack8(a[8 * q + 0], a[8 * q + 1], a[8 * q + 2], a[8 * q + 3], a[8 * q + 4], a[8 * q + 5],
                         a[8 * q + 6], a[8 * q + 7]);
  u32x4 d = __builtin_bit_cast(u32x4, p);
  const u32x4 hh = __builtin_bit_cast(u32x4, hfrag);
  // (inline asm: written in C the compiler re-derives a compare + select per 16-bit half)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t m;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(hh[k]), "s"(0x00010001u));
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(d[k]) : "v"(d[k]), "v"(m));
  }
  return __builtin_bit_cast(bf16x8, d);
}

// wave-private [32 samples][128 hid] bf16 image, 256-B rows, chunk ^= row&15
EM_DEVICE uint32_t himg_off(uint32_t base, int row, int col) {
  return base + row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
}

// A "samples as K" fragment (rows = lane column, k = samples in accumulator-perm order) from a
// [32 samples][C cols] image via ds_read_b64_tr_b16 (two 4-row blocks per fragment).
template <int HIMG>
EM_DEVICE bf16x8 tr_frag(const char* smem, uint32_t base, int colbase, int q, int h, int q4, int p4, int g1) {
  const int col = colbase + 16 * g1 + 4 * p4;
  const int r0 = 16 * q + 4 * h + q4;
  if (HIMG) return cat_tr(lds_tr16(smem, himg_off(base, r0, col)), lds_tr16(smem, himg_off(base, r0 + 8, col)));
  return cat_tr(lds_tr16(smem, img_off(base, r0, col)), lds_tr16(smem, img_off(base, r0 + 8, col)));
}

// LDS layout of the train kernel (bytes):
//   [0, IMG_BYTES)                      weight images + b2 (copied from wimg)
//   [IMG_BYTES, +LUT_BYTES)             byte -> bf16x8 table for X fragments
//   per wave w at WBASE + w*WREG:       X image 4 KB | D2 image 4 KB | H image 8 KB
// Every wave is independent inside the loop (no barrier): it keeps the FULL dW2 and dW1ᵀ
// accumulators (2 x 8 tiles x 16 = 256 AGPRs, pinned with inline-asm MFMAs) while all
// transient MFMAs are VGPR-form builtins.  The images are wave-private transposes:
//   X  [32 samples][64 feat]  -> B operand of dW1ᵀ = dZ1ᵀ·X   (tr reads)
//   D2 [32 samples][64 out]   -> B operand of dW2  = Hᵀ·dZ2   (tr reads)
//   H  [32 samples][128 hid]  -> A operand of dW2 and the relu mask of dZ1 (tr reads),
//                                instead of recomputing Z1 = X·W1 in the other orientation.
constexpr int WREG = 16384;
constexpr int WBASE = IMG_BYTES + LUT_BYTES;
constexpr int RED_BYTES = 2 * 65536;                       // epilogue: two 64 KB fp32 dW images
constexpr int LOOP_LDS = WBASE + 4 * WREG;
constexpr int TRAIN_LDS = (LOOP_LDS > RED_BYTES ? LOOP_LDS : RED_BYTES) + 4 * 64 * 4 + 64;

// dW accumulation MFMA with the accumulator pinned in AGPRs ("+a").  Every other MFMA is a
// VGPR-form builtin (file built with -mllvm -amdgpu-mfma-vgpr-form=1), so no AGPR<->VGPR copies
// are needed for results the VALU consumes.  The leading s_nop 1 covers a VALU write of an A/B
// operand right before the asm (hipcc does not pad hazards into inline asm).
EM_DEVICE void mfma_acc_agpr(f32x16& d, bf16x8 a, bf16x8 b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
}

// The optimizer's step counter (Adam bias correction, csrc/adam.hip) is advanced here, by one
// thread, when the caller passes it: stream order puts this launch strictly between two Adam
// launches, so Adam can read the counter with a plain load instead of drawing a grid-wide ticket
// (252 same-address device-scope atomics = 2.8 us per step, tools/dev/adam_probe.py).
EM_DEVICE void advance_step(int* step) {
  if (step && blockIdx.x == 0 && threadIdx.x == 0) step[0] = step[0] + 1;
}

template <int LOSS>
__global__ void __launch_bounds__(256, 1)
mlp_fused_train_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                       int offset, const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                       float* __restrict__ loss_slabs, int* __restrict__ step) {
  advance_step(step);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;

  {
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    for (int i = tid; i < IMG_BYTES / 16; i += 256) dst[i] = src[i];
  }
  const char* lut = smem + IMG_BYTES;
  fill_lut(smem + IMG_BYTES, tid);
  __syncthreads();

  const uint32_t XB = WBASE + wave * WREG, DB = XB + 4096, HB = XB + 8192;

  f32x16 dW2[4][2], dW1T[4][2];  // AGPR-resident for the whole launch
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      dW2[t][u] = f32x16{};
      dW1T[t][u] = f32x16{};
    }
  float db2[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) db2[u][i] = 0.f;
  float loss_acc = 0.f;

  const int ntiles = (B + 31) / 32;
  const int nwaves = gridDim.x * 4;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;

  // software prefetch of the next tile's feature masks (input draw, target draw)
  auto fetch = [&](int tile, uint64_t& mi, uint64_t& mt) {
    const int s = tile * 32 + r;
    mi = 0;
    mt = 0;
    if (tile < ntiles && s < B) {
      const int idx = sidx ? sidx[s] : (offset + s);
      mi = masks[idx];
      mt = masks[idx + 1];
    }
  };
  const int first = blockIdx.x * 4 + wave;
  uint64_t nin, ntg;
  fetch(first, nin, ntg);

  for (int tile = first; tile < ntiles; tile += nwaves) {
    const int s = tile * 32 + r;
    const bool valid = s < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(tile + nwaves, nin, ntg);

    bf16x8 xf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xf[q] = lut_frag(lut, imask, q, h);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<bf16x8*>(smem + XB + r * 128 + ((((2 * q + h) ^ (r & 7))) << 4)) = xf[q];

    // ---- F1: Z1ᵀ = W1ᵀ·Xᵀ -> relu -> Hᵀ fragments (B of F2) + H image (samples x hid) ----
    bf16x8 hT[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 a1 = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q) a1 = mfma32(lds_frag(smem, w1t_off(32 * t + r, 2 * q + h)), xf[q], a1);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        hT[t][q] = relu_pack(a1, q);
        // element j <-> hid 32t + 16q + 8(j>>2) + 4h + (j&3): two 8-byte pieces per fragment
        const u32x4 d = __builtin_bit_cast(u32x4, hT[t][q]);
        *reinterpret_cast<u32x2*>(smem + HB + r * 256 + ((((4 * t + 2 * q) ^ (r & 15))) << 4) + h * 8) =
            u32x2{d[0], d[1]};
        *reinterpret_cast<u32x2*>(smem + HB + r * 256 + ((((4 * t + 2 * q + 1) ^ (r & 15))) << 4) + h * 8) =
            u32x2{d[2], d[3]};
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
        const u32x4 f = __builtin_bit_cast(u32x4, dzf[u][g >> 1]);
        *reinterpret_cast<u32x2*>(smem + DB + r * 128 + ((((4 * u + g) ^ (r & 7))) << 4) + h * 8) =
            u32x2{f[2 * (g & 1)], f[2 * (g & 1) + 1]};
      }

    wave_lds_sync();  // X / H / D2 images complete (written by all lanes of this wave)

    // ---- B1: dH = dZ2·W2ᵀ ; dZ1 = dH * (Z1 > 0) with H fragments from the H image ----
    bf16x8 hR[4][2], dz1[4][2];
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
        hR[t][q] = tr_frag<1>(smem, HB, 32 * t, q, h, q4, p4, g1);
        dz1[t][q] = mask_by(hR[t][q], aD, q);
      }
    }

    // ---- dW2 += Hᵀ·dZ2, dW1ᵀ += dZ1ᵀ·X   (K = the tile's 32 samples) ----
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 bd = tr_frag<0>(smem, DB, 32 * u, q, h, q4, p4, g1);
        const bf16x8 bx = tr_frag<0>(smem, XB, 32 * u, q, h, q4, p4, g1);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          mfma_acc_agpr(dW2[t][u], hR[t][q], bd);
          mfma_acc_agpr(dW1T[t][u], dz1[t][q], bx);
        }
      }

    wave_lds_sync();  // images are overwritten by the next tile
  }
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");  // MFMA (asm, AGPR D) -> v_accvgpr_read hazard

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
  __syncthreads();  // all waves are done with the loop's LDS
  float* RED0 = reinterpret_cast<float*>(smem);
  float* RED1 = reinterpret_cast<float*>(smem + 65536);
  float* DB2S = reinterpret_cast<float*>(smem + (TRAIN_LDS - 4 * 64 * 4 - 64));
  float* LOSSS = DB2S + 4 * 64;
  if (r == 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) DB2S[wave * 64 + 32 * u + oo0(i) + 4 * h] = db2[u][i];
  }
  if (lane == 0) LOSSS[wave] = lsum;
  // tile T: 0..7 -> dW2[T>>1][T&1], 8..15 -> dW1ᵀ[(T-8)>>1][(T-8)&1]; layout [T][g][lane][4]
  auto region_io = [&](float* R, bool add) {
#pragma unroll
    for (int T = 0; T < 16; ++T) {
      const f32x16& acc = (T < 8) ? dW2[T >> 1][T & 1] : dW1T[(T - 8) >> 1][(T - 8) & 1];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4* p = reinterpret_cast<f32x4*>(R + ((T * 4 + g) * 64 + lane) * 4);
        f32x4 v = {acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
        if (add) v += *p;
        *p = v;
      }
    }
  };
  if (wave == 0) region_io(RED0, false);
  if (wave == 1) region_io(RED1, false);
  __syncthreads();
  if (wave == 2) region_io(RED0, true);
  if (wave == 3) region_io(RED1, true);
  __syncthreads();

  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  for (int e = tid; e < 16 * 4 * 64; e += 256) {
    const int T = e >> 8, g = (e >> 6) & 3, l = e & 63, hh = l >> 5, rr = l & 31;
    const f32x4 v = *reinterpret_cast<const f32x4*>(RED0 + e * 4) + *reinterpret_cast<const f32x4*>(RED1 + e * 4);
    const int c0 = 32 * ((T & 7) >> 1) + 8 * g + 4 * hh;  // hidden rows c0..c0+3
    const int col = 32 * (T & 1) + rr;
    if (T < 8) {  // dW2[c][o]
#pragma unroll
      for (int k = 0; k < 4; ++k) slab[P_W2 + (c0 + k) * OUT + col] = v[k];
    } else {  // dW1ᵀ tile -> W1[f][c]
      *reinterpret_cast<f32x4*>(slab + P_W1 + col * HID + c0) = v;
    }
  }
  if (tid < 64) slab[P_B2 + tid] = DB2S[tid] + DB2S[64 + tid] + DB2S[128 + tid] + DB2S[192 + tid];
  if (tid == 0) loss_slabs[blockIdx.x] = LOSSS[0] + LOSSS[1] + LOSSS[2] + LOSSS[3];
}

// ============================================================================================
// v4: hidden-split wave pairs, two waves per SIMD.
//
// v3 keeps the whole dW (256 AGPRs) in every wave, so a CU runs one wave per SIMD and the
// serial F1 -> relu -> F2 -> loss -> B1 -> mask -> dW chain of a tile leaves the matrix pipe idle
// most of the time (PMC: MFMA busy 21 %, waiting 48 %).  v4 runs 8 waves (4 pairs) per CU.  The two
// waves of a pair work on the SAME 32-sample tile and split the hidden layer: role rho owns hidden
// units [64 rho, 64 rho + 64) and output tile u = rho, so each holds half of dW2 and of dW1T
// (128 AGPRs) and does half of the MFMAs (40 per tile).  Per tile the pair exchanges through LDS:
//   (1) the partial logits of the partner's output tile (4 KB fp32),
//   (2) the per-sample softmax statistics (online-softmax merge: max and scaled sum),
//   (3) the bf16 dZ2 fragments of its output tile (for B1) + its half of the D2 image.
// Synchronisation is per pair through LDS counters (no workgroup barrier in the loop), so the two
// waves that share a SIMD belong to different pairs and fill each other's dependency stalls.
// Every spin is bounded: a broken protocol produces NaN losses, never a hung GPU.
constexpr int V4_PAIR_BYTES = 25152;  // X 4K | D2 4K | H0 4K | H1 4K | XB0 4K | XB1 4K | stats 2x256 | flags 64
constexpr int V4_PX = 0, V4_PD2 = 4096, V4_PH = 8192, V4_PXB = 16384, V4_PST = 24576, V4_PFL = 25088;
static_assert(V4_PST + 2 * 256 <= V4_PFL && V4_PFL + 64 <= V4_PAIR_BYTES, "v4 pair layout");
constexpr int V4_BASE = IMG_BYTES + LUT_BYTES;
constexpr int V4_YLUT = V4_BASE + 4 * V4_PAIR_BYTES;  // 16 x f32x4: target nibble -> 4 {0,1} floats
constexpr int V4_XLUT = V4_YLUT + 256;  // 16 x 8 B: input nibble -> 4 bf16 {0,1}
constexpr int V4_LOOP_LDS = V4_XLUT + 128;
constexpr int V4_RED = 131072;  // epilogue: two fp32 dW images [2][16384] below this offset
constexpr int V4_LDS = (V4_LOOP_LDS > V4_RED + 4096 ? V4_LOOP_LDS : V4_RED + 4096);
#ifndef V4_STAGGER
#define V4_STAGGER 0
#endif
#ifndef V4_PRIO
#define V4_PRIO 0
#endif
#ifndef V4_SLEEP
#define V4_SLEEP 0
#endif
constexpr int V4_SPIN_LIMIT = V4_SLEEP ? (1 << 22) : (1 << 24);
static_assert(V4_LDS <= 163840, "v4 LDS budget");
static_assert(IMG_BYTES == 54528 && IMG_BYTES % 16 == 0, "image size (ops/fused_mlp.py IMG_BYTES)");

EM_DEVICE void pair_signal(char* smem, uint32_t flag_off, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(reinterpret_cast<int*>(smem + flag_off), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// returns false if the partner never arrived (protocol bug): the caller poisons its loss
EM_DEVICE bool pair_wait(const char* smem, uint32_t flag_off, int target) {
  int spins = 0;
  while (__hip_atomic_load(reinterpret_cast<const int*>(smem + flag_off), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
    if (V4_SLEEP) __builtin_amdgcn_s_sleep(1);
    if (++spins > V4_SPIN_LIMIT) return false;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

// class of output o = 32 RHO + oo0(i) + 4h: 0 main, 1 star, 2 pad
template <int RHO>
EM_DEVICE int v4_cls(int i, int h) {
  const int o = 32 * RHO + oo0(i) + 4 * h;
  return o < 50 ? 0 : (o < 62 ? 1 : 2);
}

// Diagnostic phase timers (build with --define V4_STAMPS=1; tools/fused_phases.py reads them):
// s_memtime deltas summed per phase per wave, written after the dW slab into spare slab floats.
// They force an lgkmcnt drain at every mark, so they perturb what they measure (+~10 %).
#ifndef V4_MIX
#define V4_MIX 1
#endif
#ifndef V4_NODB2
#define V4_NODB2 0
#endif
#ifndef V4_STAMPS
#define V4_STAMPS 0
#endif
#ifndef V4_F1_HOIST
#define V4_F1_HOIST 0  // measured slower (130 vs 126 us/step, same box): the hoisted reads spill
#endif
struct V4Stamps {
  uint64_t last = 0;
  uint64_t acc[10] = {};
  EM_DEVICE void start() {
    if (V4_STAMPS) last = __builtin_amdgcn_s_memtime();
  }
  EM_DEVICE void mark(int k) {
    if (V4_STAMPS) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
};

// v4 pair images [32 samples][64 cols] bf16, 128-B rows.  Row r XORs its 16-B chunk index with
// fr(r) and (H, D2 only) its 8-B half with gr(r), chosen so that every access of the tile is
// conflict-free under the CDNA4 banking rules (tools/lds_conflicts.py): the per-row 8-B writes
// (16-lane groups, 32 banks) need (fr, gr) injective on rows 0-15, the partner's 8-B row reads
// (32-lane groups, 64 banks) injective on each row parity, and the transposing reads (4 rows x 64 B
// per 32-lane group) need fr's top bit to follow row bit 1.  The X image is written in whole 16-B
// chunks, so it keeps gr = 0.
EM_DEVICE uint32_t v4_fr(int r) { return ((r ^ (r >> 4)) & 1) | (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2); }
EM_DEVICE uint32_t v4_gr(int r) { return (r >> 3) & 1; }
template <bool G>
EM_DEVICE uint32_t v4_img(uint32_t base, int row, int col) {
  const uint32_t c = (uint32_t)(((col >> 3) ^ v4_fr(row)) << 4);
  return base + row * 128 + c + (G ? (((((col >> 2) & 1) ^ v4_gr(row)) << 3) + (col & 3) * 2) : (col & 7) * 2);
}
template <bool G>
EM_DEVICE bf16x8 v4_tr_frag(const char* smem, uint32_t base, int colbase, int q, int h, int q4, int p4, int g1) {
  const int col = colbase + 16 * g1 + 4 * p4;
  const int r0 = 16 * q + 4 * h + q4;
  return cat_tr(lds_tr16(smem, v4_img<G>(base, r0, col)), lds_tr16(smem, v4_img<G>(base, r0 + 8, col)));
}
// X fragments from a 16-entry nibble table (4 bf16 {0,1} per entry, 128 B): two ds_read_b64 per
// fragment; distinct entries never share a bank, unlike a 256-entry byte table
template <int LUT = V4_XLUT>
EM_DEVICE bf16x8 v4_xfrag(const char* smem, uint32_t w, int q) {
  const int sh = 16 * (q & 1);
  const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + LUT + (__builtin_amdgcn_ubfe(w, sh, 4) << 3));
  const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + LUT + (__builtin_amdgcn_ubfe(w, sh + 4, 4) << 3));
  return __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
}

template <int LOSS, int RHO>
EM_DEVICE void v4_tile(char* smem, const char* lut, uint32_t PB, int pairw, int r, int h, int lane, int q4, int p4,
                       int g1, uint64_t imask, uint64_t tmask, bool valid, int& sig, bool& ok, f32x16 (&dW2)[2][2],
                       f32x16 (&dW1T)[2][2], f32x16& db2, const bf16x8 ones, float& loss_acc, V4Stamps& st) {
  constexpr int PR = 1 - RHO;
  const uint32_t XB = PB + V4_PX, DB = PB + V4_PD2, HB = PB + V4_PH + RHO * 4096;
  const uint32_t MYX = PB + V4_PXB + RHO * 4096, PAX = PB + V4_PXB + PR * 4096;
  const uint32_t MYFL = PB + V4_PFL + RHO * 4, PAFL = PB + V4_PFL + PR * 4;
  (void)pairw;
  (void)lut;

  bf16x8 xf[4];
  const uint32_t wlo = (uint32_t)imask >> (8 * h), whi = (uint32_t)(imask >> 32) >> (8 * h);
#pragma unroll
  for (int q = 0; q < 4; ++q) xf[q] = v4_xfrag(smem, q < 2 ? wlo : whi, q);

  // ---- F1 (own hidden half) -> relu -> hT (B of F2) + own H image [32 samples][64 hid] ----
  bf16x8 hT[2][2];
  // every W1ᵀ fragment read issued before the first MFMA (V4_F1_HOIST), so the chain pays one LDS
  // latency instead of one per MFMA pair; then both hidden tiles' chains interleaved
  bf16x8 w1f[2][4];
  if (V4_F1_HOIST) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) w1f[tt][q] = lds_frag(smem, w1t_off(32 * (2 * RHO + tt) + r, 2 * q + h));
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the chain (the scheduler interleaves them)
  }
  f32x16 a1s[2] = {f32x16{}, f32x16{}};
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
      a1s[tt] = mfma32(V4_F1_HOIST ? w1f[tt][q] : lds_frag(smem, w1t_off(32 * (2 * RHO + tt) + r, 2 * q + h)), xf[q],
                       a1s[tt]);
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const f32x16& a1 = a1s[tt];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      hT[tt][q] = relu_pack(a1, q);
      const u32x4 d = __builtin_bit_cast(u32x4, hT[tt][q]);
      *reinterpret_cast<u32x2*>(smem + v4_img<true>(HB, r, 32 * tt + 16 * q + 4 * h)) = u32x2{d[0], d[1]};
      *reinterpret_cast<u32x2*>(smem + v4_img<true>(HB, r, 32 * tt + 16 * q + 8 + 4 * h)) = u32x2{d[2], d[3]};
    }
  }

  // ---- exchange (1): the H images.  Each wave computes the FULL logits of its own output tile:
  // its own hidden half from registers, the partner's half read back as B fragments from the
  // partner's H image (two ds_read_b64 each) -- no fp32 partial-sum round trip through LDS ----
  st.mark(0);
  pair_signal(smem, MYFL, ++sig);
  f32x16 z;
#pragma unroll
  for (int g = 0; g < 4; ++g) {  // b2 rides in as the accumulator init
    const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * RHO + 8 * g + 4 * h) * 4);
    z[4 * g + 0] = b[0]; z[4 * g + 1] = b[1]; z[4 * g + 2] = b[2]; z[4 * g + 3] = b[3];
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int q = 0; q < 2; ++q)
      z = mfma32(lds_frag(smem, w2p_off(32 * RHO + r, (2 * (2 * RHO + tt) + q) * 2 + h)), hT[tt][q], z);
  st.mark(1);
  ok &= pair_wait(smem, PAFL, sig);
  st.mark(2);
  const uint32_t PHB = PB + V4_PH + PR * 4096;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + v4_img<true>(PHB, r, 32 * tt + 16 * q + 4 * h));
      const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + v4_img<true>(PHB, r, 32 * tt + 16 * q + 8 + 4 * h));
      const bf16x8 pT = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
      z = mfma32(lds_frag(smem, w2p_off(32 * RHO + r, (2 * (2 * PR + tt) + q) * 2 + h)), pT, z);
    }
  if (RHO == 0) {  // the pair-shared X image [32 samples][64 feat]; the partner is past its previous tile
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<bf16x8*>(smem + v4_img<false>(XB, r, 16 * q + 8 * h)) = xf[q];
  }

  st.mark(3);
  // ---- loss on the own output tile ----
  // target bits of the lane's 16 outputs as 0/1 floats: register group g holds outputs
  // 8g + 4h .. +3 of the tile = one nibble of the target mask -> one ds_read_b128 of a 16-entry table
  const uint32_t tmh = (uint32_t)(tmask >> (32 * RHO)) >> (4 * h);
  float yb[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + V4_YLUT + (__builtin_amdgcn_ubfe(tmh, 8 * g, 4) << 4));
    yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
  }
  float dz[16];
  if (LOSS == 0) {
    // VALU-lean grouped softmax: exponentials as exp2(z·log2e − max·log2e) (one fma + v_exp each),
    // reciprocals with v_rcp, and no per-element validity select -- an invalid (padding) sample has
    // an all-zero target mask, so nm = ns = 0 zeroes its factors and hence its dZ and loss.
    constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
    const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
    const int nm = __builtin_popcount(tlo) + __builtin_popcount(thi & 0x3FFFFu);  // bits 0..49
    const int ns = __builtin_popcount(thi & 0x3FFC0000u);                          // bits 50..61
    const float inv_m = nm ? __builtin_amdgcn_rcpf((float)nm) : 0.f;
    const float inv_s = (RHO == 1 && ns) ? __builtin_amdgcn_rcpf((float)ns) : 0.f;
    float mx_m = -3.0e38f, mx_s = -3.0e38f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = v4_cls<RHO>(i, h);
      mx_m = (c == 0) ? fmaxf(mx_m, z[i]) : mx_m;
      if (RHO == 1) mx_s = (c == 1) ? fmaxf(mx_s, z[i]) : mx_s;
    }
    mx_m = xhalf_max(mx_m);
    if (RHO == 1) mx_s = xhalf_max(mx_s);
    const float nmL = -mx_m * L2E, nsL = -mx_s * L2E;
    float s_m = 0.f, s_s = 0.f, zt_m = 0.f, zt_s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = v4_cls<RHO>(i, h);
      const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(z[i], L2E, (RHO == 1 && c == 1) ? nsL : nmL));
      const float ee = (c == 2) ? 0.f : e;
      dz[i] = ee;
      // branch-free: c is a compile-time constant except for the two registers straddling 50/62
      s_m += (c == 0) ? ee : 0.f;
      zt_m = __builtin_fmaf((c == 0) ? yb[i] : 0.f, z[i], zt_m);
      if (RHO == 1) {
        s_s += (c == 1) ? ee : 0.f;
        zt_s = __builtin_fmaf((c == 1) ? yb[i] : 0.f, z[i], zt_s);
      }
    }
    s_m = xhalf_sum(s_m);
    if (RHO == 1) s_s = xhalf_sum(s_s);
    // exchange (2): online-softmax merge of the main-group statistics
    if (h == 0) *reinterpret_cast<float2*>(smem + PB + V4_PST + RHO * 256 + r * 8) = float2{mx_m, s_m};
    st.mark(4);
    pair_signal(smem, MYFL, ++sig);
    ok &= pair_wait(smem, PAFL, sig);
    st.mark(5);
    const float2 ps = *reinterpret_cast<const float2*>(smem + PB + V4_PST + PR * 256 + r * 8);
    const float M = fmaxf(mx_m, ps.x);
    const float sc_own = __builtin_amdgcn_exp2f((mx_m - M) * L2E);
    const float S = s_m * sc_own + ps.y * __builtin_amdgcn_exp2f((ps.x - M) * L2E);
    const float f_m = nm ? sc_own * __builtin_amdgcn_rcpf(S) : 0.f;
    const float f_s = (RHO == 1 && ns) ? __builtin_amdgcn_rcpf(s_s) : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = v4_cls<RHO>(i, h);
      dz[i] = (c == 2) ? 0.f : __builtin_fmaf(dz[i], c == 0 ? f_m : f_s, -yb[i] * (c == 0 ? inv_m : inv_s));
    }
    float l = -(zt_m * inv_m + zt_s * inv_s);
    if (RHO == 1 && h == 0)
      l += (nm ? M + __builtin_amdgcn_logf(S) * LN2 : 0.f) + (ns ? mx_s + __builtin_amdgcn_logf(s_s) * LN2 : 0.f);
    loss_acc += l;
  } else {
    constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = v4_cls<RHO>(i, h);
      const float v = z[i];
      const float y = yb[i];
      const float en = __builtin_amdgcn_exp2f(-fabsf(v) * L2E);  // stable sigmoid / softplus
      const float rp = __builtin_amdgcn_rcpf(1.f + en);
      const float pr = v >= 0.f ? rp : en * rp;
      const float sp = fmaxf(v, 0.f) + __builtin_amdgcn_logf(1.f + en) * LN2;
      const bool okc = valid && c != 2;
      dz[i] = okc ? (pr - y) : 0.f;
      l += okc ? (sp - y * v) : 0.f;
    }
    loss_acc += l;
    pair_signal(smem, MYFL, ++sig);  // keeps the exchange-buffer reuse below ordered
    ok &= pair_wait(smem, PAFL, sig);
  }
  bf16x8 dzf[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
    dzf[q] = pack8(dz[8 * q + 0], dz[8 * q + 1], dz[8 * q + 2], dz[8 * q + 3], dz[8 * q + 4], dz[8 * q + 5],
                   dz[8 * q + 6], dz[8 * q + 7]);
  // exchange (3): dZ2 fragments (lane-for-lane dump into our exchange buffer; the partner has read
  // its partial from it, which it did before its signal (2)) + our half of the D2 image
#pragma unroll
  for (int q = 0; q < 2; ++q) *reinterpret_cast<bf16x8*>(smem + MYX + (q * 64 + lane) * 16) = dzf[q];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32x4 f = __builtin_bit_cast(u32x4, dzf[g >> 1]);
    *reinterpret_cast<u32x2*>(smem + v4_img<true>(DB, r, 32 * RHO + 8 * g + 4 * h)) =
        u32x2{f[2 * (g & 1)], f[2 * (g & 1) + 1]};
  }
  st.mark(6);
  pair_signal(smem, MYFL, ++sig);

  // ---- work that needs only our own dZ2 half, issued before waiting for the partner's:
  // B1 over the own output tile, dW2 for the own output columns, db2 ----
  // (BCE keeps the old order: its longer loss code leaves no registers for the early accumulators)
  bf16x8 hR[2][2], dz1[2][2];
  f32x16 aD[2];
  if (LOSS == 0) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * RHO + tt;
      aD[tt] = f32x16{};
#pragma unroll
      for (int q = 0; q < 2; ++q)
        aD[tt] = mfma32(dzf[q], lds_frag(smem, w2q_off(32 * t + r, (2 * RHO + q) * 2 + h)), aD[tt]);
#pragma unroll
      for (int q = 0; q < 2; ++q) hR[tt][q] = v4_tr_frag<true>(smem, HB, 32 * tt, q, h, q4, p4, g1);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bf16x8 bd = v4_tr_frag<true>(smem, DB, 32 * RHO, q, h, q4, p4, g1);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) mfma_acc_agpr(dW2[tt][RHO], hR[tt][q], bd);
      // db2 of the own output tile on the matrix pipe: ones(32 x samples) · dZ2 (every row of the
      // accumulator is the column sum) instead of 16 VALU adds per tile
      if (!V4_NODB2) db2 = mfma32(ones, bd, db2);
    }
  }
  ok &= pair_wait(smem, PAFL, sig);
  if (LOSS != 0) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * RHO + tt;
      aD[tt] = f32x16{};
#pragma unroll
      for (int q = 0; q < 2; ++q)
        aD[tt] = mfma32(dzf[q], lds_frag(smem, w2q_off(32 * t + r, (2 * RHO + q) * 2 + h)), aD[tt]);
#pragma unroll
      for (int q = 0; q < 2; ++q) hR[tt][q] = v4_tr_frag<true>(smem, HB, 32 * tt, q, h, q4, p4, g1);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bf16x8 bd = v4_tr_frag<true>(smem, DB, 32 * RHO, q, h, q4, p4, g1);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) mfma_acc_agpr(dW2[tt][RHO], hR[tt][q], bd);
      // db2 of the own output tile on the matrix pipe: ones(32 x samples) · dZ2 (every row of the
      // accumulator is the column sum) instead of 16 VALU adds per tile
      db2 = mfma32(ones, bd, db2);
    }
  }
  st.mark(7);
  bf16x8 dzp[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) dzp[q] = *reinterpret_cast<const bf16x8*>(smem + PAX + (q * 64 + lane) * 16);

  // ---- B1 (partner's output tile): dH = dZ2·W2ᵀ for the own hidden half; dZ1 = dH * (Z1 > 0) ----
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int t = 2 * RHO + tt;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      aD[tt] = mfma32(dzp[q], lds_frag(smem, w2q_off(32 * t + r, (2 * PR + q) * 2 + h)), aD[tt]);
#pragma unroll
    for (int q = 0; q < 2; ++q) dz1[tt][q] = mask_by(hR[tt][q], aD[tt], q);
  }

  st.mark(8);
  // ---- dW2[own hid][partner out] += Hᵀ·dZ2 ; dW1ᵀ[own hid][feat] += dZ1ᵀ·X ----
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const bf16x8 bd = v4_tr_frag<true>(smem, DB, 32 * PR, q, h, q4, p4, g1);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) mfma_acc_agpr(dW2[tt][PR], hR[tt][q], bd);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bf16x8 bx = v4_tr_frag<false>(smem, XB, 32 * u, q, h, q4, p4, g1);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) mfma_acc_agpr(dW1T[tt][u], dz1[tt][q], bx);
    }
  wave_lds_sync();  // own H image is rewritten by the next tile
  st.mark(9);
}

// One role's whole persistent loop + its share of the epilogue reduction.  Instantiated per role so
// the AGPR-pinned dW accumulators never cross a role branch (a merge point would force copies).
template <int LOSS, int RHO>
EM_DEVICE void v4_body(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                       int offset, int pair, int lane, float* slab_spare, uint64_t nin, uint64_t ntg) {
  const int r = lane & 31, h = lane >> 5;
  const char* lut = smem + IMG_BYTES;
  const uint32_t PB = V4_BASE + pair * V4_PAIR_BYTES;
  f32x16 dW2[2][2], dW1T[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      dW2[t][u] = f32x16{};
      dW1T[t][u] = f32x16{};
    }
  f32x16 db2 = f32x16{};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  float loss_acc = 0.f;
  int sig = 0;
  bool ok = true;

  const int ntiles = (B + 31) / 32;
  const int npairs = gridDim.x * 4;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;
  auto fetch = [&](int tile, uint64_t& mi, uint64_t& mt) {
    const int s = tile * 32 + r;
    mi = 0;
    mt = 0;
    if (tile < ntiles && s < B) {
      const int idx = sidx ? sidx[s] : (offset + s);
      mi = masks[idx];
      mt = masks[idx + 1];
    }
  };
  V4Stamps st;
  const int first = blockIdx.x * 4 + pair;  // its masks (nin, ntg) were fetched before the prologue
  st.start();
  for (int tile = first; tile < ntiles; tile += npairs) {
    const int s = tile * 32 + r;
    const bool valid = s < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(tile + npairs, nin, ntg);
    v4_tile<LOSS, RHO>(smem, lut, PB, pair, r, h, lane, q4, p4, g1, imask, tmask, valid, sig, ok, dW2, dW1T, db2,
                       ones, loss_acc, st);
  }
  asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");  // asm MFMA (AGPR D) -> v_accvgpr_read hazard

  float lsum = wave_sum(loss_acc);
  if (!ok) lsum = __builtin_nanf("");
  if (V4_STAMPS && lane < 10) {  // phase cycles of this wave -> spare slab floats
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 10; ++k) v = (lane == k) ? st.acc[k] : v;
    slab_spare[(2 * pair + RHO) * 16 + lane] = (float)v;
  }
  __syncthreads();  // every wave is out of the loop: the loop's LDS is free
  float* RED = reinterpret_cast<float*>(smem);  // [16 tiles][4 g][64 lanes][4]: tiles 0..7 dW2, 8..15 dW1T
  float* DB2S = reinterpret_cast<float*>(smem + V4_RED);          // [4 pairs][64]
  float* LOSSS = reinterpret_cast<float*>(smem + V4_RED + 1024);  // [8]
  if (h == 0) DB2S[pair * 64 + 32 * RHO + r] = db2[0];  // accumulator column r = output 32 RHO + r
  if (lane == 0) LOSSS[2 * pair + RHO] = lsum;
  // the same number of barriers in both role instantiations (wave-uniform branch)
  // two stages: pairs 0/1 store into halves 0/1, then pairs 2/3 add theirs (fixed order, so the
  // slab is bit-reproducible); the slab writer sums the halves
  for (int stage = 0; stage < 2; ++stage) {
    if ((pair >> 1) == stage) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int which = 0; which < 2; ++which) {
            const f32x16& acc = which ? dW1T[tt][u] : dW2[tt][u];
            const int T = 8 * which + 2 * (2 * RHO + tt) + u;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              f32x4* p = reinterpret_cast<f32x4*>(RED + (pair & 1) * 16384 + ((T * 4 + g) * 64 + lane) * 4);
              f32x4 v = {acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
              if (stage) v += *p;
              *p = v;
            }
          }
    }
    __syncthreads();
  }
}

template <int LOSS>
__global__ void __launch_bounds__(512, 1)
mlp_fused_train_v4_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                          const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                          float* __restrict__ loss_slabs, int* __restrict__ step) {
  advance_step(step);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint64_t ts[4] = {};  // V4_STAMPS: 100 MHz wall-clock marks (entry, prologue done, loop done, dW folded)
  if (V4_STAMPS) ts[0] = __builtin_amdgcn_s_memrealtime();
  // wave w runs on SIMD w % 4: pairs 2/3 take their roles swapped so every SIMD hosts one role-0 and
  // one role-1 wave (role 1 owns the star group and issues ~20 % more VALU per tile)
  const int pair = wave >> 1, rho = (wave & 1) ^ (V4_MIX ? (wave >> 2) : 0);
  // the first tile's feature masks: loads issued before the prologue so their HBM latency overlaps it
  uint64_t nin = 0, ntg = 0;
  {
    const int s0 = (blockIdx.x * 4 + pair) * 32 + (lane & 31);
    if (s0 < B) {
      const int idx = sidx ? sidx[s0] : (offset + s0);
      nin = masks[idx];
      ntg = masks[idx + 1];
    }
  }
  {  // all loads of the weight image in flight before the first LDS store
    constexpr int N16 = IMG_BYTES / 16, K = (N16 + 511) / 512;
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (tid + 512 * k < N16) v[k] = src[tid + 512 * k];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (tid + 512 * k < N16) dst[tid + 512 * k] = v[k];
  }
  if (tid < 64) reinterpret_cast<float*>(smem + V4_YLUT)[tid] = (float)(((tid >> 2) >> (tid & 3)) & 1);
  if (tid < 32) {  // nibble n = tid >> 1, dword tid & 1 holds elements 2(tid&1), 2(tid&1)+1
    const uint32_t n = (uint32_t)tid >> 1, b = 2u * (tid & 1);
    reinterpret_cast<uint32_t*>(smem + V4_XLUT)[tid] = (((n >> b) & 1u) ? 0x3F80u : 0u) | (((n >> (b + 1)) & 1u) ? 0x3F800000u : 0u);
  }
  if (lane < 2) reinterpret_cast<int*>(smem + V4_BASE + pair * V4_PAIR_BYTES + V4_PFL)[lane] = 0;
  __syncthreads();
  if (V4_STAMPS) ts[1] = __builtin_amdgcn_s_memrealtime();
  // waves 4-7 share SIMDs with waves 0-3 (other pairs): start them half a tile later so the two
  // co-resident waves do not hit their MFMA and VALU phases in lockstep (MI355X_MICROARCH.md,
  // "Two waves per SIMD" item 9), and give the younger half static priority (item 4)
  if (V4_STAGGER && wave >= 4) __builtin_amdgcn_s_sleep(V4_STAGGER);  // ~64 cycles per unit
  if (V4_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);
  float* slab_spare = slabs + (size_t)blockIdx.x * SLAB_STRIDE + P_TOTAL;  // 192 spare floats per slab
  if (rho == 0)
    v4_body<LOSS, 0>(smem, masks, sidx, B, offset, pair, lane, slab_spare, nin, ntg);
  else
    v4_body<LOSS, 1>(smem, masks, sidx, B, offset, pair, lane, slab_spare, nin, ntg);
  if (V4_STAMPS) ts[2] = __builtin_amdgcn_s_memrealtime();

  const float* RED = reinterpret_cast<const float*>(smem);
  const float* DB2S = reinterpret_cast<const float*>(smem + V4_RED);
  const float* LOSSS = reinterpret_cast<const float*>(smem + V4_RED + 1024);
  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  // The slab is written in parameter order with 16-B write-through (sc1) stores: the bytes head for
  // memory while later workgroups are still in their loops, instead of sitting dirty in the XCD's L2
  // until the kernel boundary writes them back in front of the Adam launch (MI355X_MICROARCH.md,
  // "publish-large" and the "boundary" row: +B / 6 TB/s for B dirty bytes).
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(slab, 0, SLAB_STRIDE * 4, 0x00020000);
  for (int e = tid; e < 2 * 2048; e += 512) {
    f32x4 v;
    if (e < 2048) {  // W1[f][c..c+3] = dW1T tile T = 8 + 2 (c >> 5) + (f >> 5): one 16-B read per half
      const int f = e >> 5, c = (e & 31) * 4;
      const int T = 8 + 2 * (c >> 5) + (f >> 5), g = (c & 31) >> 3, l = ((c >> 2) & 1) * 32 + (f & 31);
      const int at = ((T * 4 + g) * 64 + l) * 4;
      v = *reinterpret_cast<const f32x4*>(RED + at) + *reinterpret_cast<const f32x4*>(RED + 16384 + at);
    } else {  // W2[c][o..o+3]: 4 lanes of dW2 tile T = 2 (c >> 5) + (o >> 5), register k = c & 3
      const int q = e - 2048, c = q >> 4, o = (q & 15) * 4;
      const int T = 2 * (c >> 5) + (o >> 5), g = (c & 31) >> 3, l = ((c >> 2) & 1) * 32 + (o & 31);
      const int at = ((T * 4 + g) * 64 + l) * 4 + (c & 3);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = RED[at + 4 * k] + RED[16384 + at + 4 * k];
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), srd, e * 16, 0, 16 /* sc1 */);
  }
  if (V4_STAMPS && tid == 0) {
    ts[3] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 4; ++k) slab_spare[128 + k] = __builtin_bit_cast(float, (uint32_t)ts[k]);
  }
  if (tid < 64) slab[P_B2 + tid] = DB2S[tid] + DB2S[64 + tid] + DB2S[128 + tid] + DB2S[192 + tid];
  if (tid == 0) {
    float l = 0.f;
    for (int w = 0; w < 8; ++w) l += LOSSS[w];
    loss_slabs[blockIdx.x] = l;
  }
}

// ============================================================================================
// v5: round-synchronous workgroup -- per-wave forward/backward chains, cross-wave dW GEMMs.
//
// v4's hidden-split pairs exchange H, the softmax statistics and dZ2 through LDS three times per
// tile; phase stamps showed each wave waiting on its partner ~28 % of the time, and the AGPR-resident
// full dW (128 AGPRs per wave) caps the CU at two waves per SIMD with no room to pipeline.  v5 moves
// the dW accumulation out of the per-tile chain:
//   phase A   each of the 8 waves runs ONE 32-sample tile through F1 -> relu -> F2 -> loss -> B1 ->
//             mask entirely on its own (48 MFMAs, no exchange), leaving its H image [32 x 128] and
//             its dZ2 image [32 x 64] in LDS and dZ1ᵀ (samples on the lanes) in registers;
//   barrier   then the workgroup computes dW2 = Hᵀ·dZ2 over all 8 tiles (K = 256 samples): wave w
//   phase B1  owns hidden block w >> 1 and K-half w & 1, both output blocks (16 MFMAs; db2 rides on
//             4 waves as a ones·dZ2 MFMA);
//   dump      the dZ1 image overwrites the H image, the X image overwrites dZ2;
//   phase B2  dW1ᵀ = dZ1ᵀ·X the same way (16 MFMAs).
// Each wave keeps only a quarter of a dW partial (64 registers + 16 for db2), the per-tile work has no
// waits, and phase B is a dense MFMA stream.  The two K-halves are summed in a fixed order in the
// epilogue (bit-reproducible slabs).  LDS: weights 54.5 KB + 8 tiles x 12 KB = 150 KB.
//
// Status (measured, 1x MI355X, same box): correct (tests/test_fused_mlp_gpu.py under EM_FUSED_V5=1)
// but 135 us/step vs v4's 127 us.  Phase stamps: phase A takes ~7.2 k cycles per 32-sample tile -- one
// wave's serial F1 -> F2 -> loss -> B1 chain is latency-bound, and with every wave of a group in the
// same phase the co-resident waves of a SIMD cannot hide each other's stalls; ~25 % of its VALU is LDS
// address arithmetic for the XOR-swizzled images.  v4 stays the default; v5 is opt-in (EM_FUSED_V5=1)
// for further work (shorter chains per wave, fewer swizzled addresses).
constexpr int V5_XLUT = IMG_BYTES;        // 16 x 8 B: input nibble -> 4 bf16 {0,1}
constexpr int V5_YLUT = V5_XLUT + 128;    // 16 x f32x4: target nibble -> 4 {0,1} floats
constexpr int V5_TILES = V5_YLUT + 256;   // 8 x [H image / dZ1 frags 8 KB | dZ2 image / X image 4 KB]
constexpr int V5_TILE_BYTES = 12288;
constexpr int V5_FLAGS = V5_TILES + 8 * V5_TILE_BYTES;  // [2 groups][4 waves] sync counters
#ifndef V5_STAGGER
#define V5_STAGGER 1
#endif
constexpr int V5_LOOP_LDS = V5_FLAGS + 32;
constexpr int V5_RED = 131072;  // epilogue: two fp32 dW images [2][16384] below, DB2S [8][32] + LOSSS [8] above
constexpr int V5_LDS = (V5_LOOP_LDS > V5_RED + 2048 ? V5_LOOP_LDS : V5_RED + 2048);
static_assert(V5_LDS <= 163840 && V5_TILES % 16 == 0, "v5 LDS budget");

// class of output o = 32 u + oo0(i) + 4h: 0 main, 1 star, 2 pad
EM_DEVICE int v5_cls(int u, int i, int h) {
  const int o = 32 * u + oo0(i) + 4 * h;
  return o < 50 ? 0 : (o < 62 ? 1 : 2);
}

// Loss + dZ2 of a whole 32-sample tile in ONE wave (both 32-output tiles; v5 and v6): the lane's
// 32 logits z2[u][i] (output 32u + oo0(i) + 4h of sample r; lanes r and r + 32 share the sample).
// Targets as {0,1} floats, one output tile at a time: register group g of tile u holds outputs
// 32u + 8g + 4h .. +3 = one nibble of the target mask -> one ds_read_b128 of a 16-entry table (YL).
template <int LOSS, int YL>
EM_DEVICE void full_tile_loss(const char* smem, const f32x16 (&z2)[2], uint64_t tmask, bool valid, int h,
                              float (&dz)[2][16], float& loss_acc) {
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  auto targets = [&](int u, float (&yb)[16]) {
    const uint32_t tmh = (uint32_t)(tmask >> (32 * u)) >> (4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + YL + (__builtin_amdgcn_ubfe(tmh, 8 * g, 4) << 4));
      yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
    }
  };
  if (LOSS == 0) {
    // grouped softmax (main 50 / stars 12): exp2 with the max folded into one fma, v_rcp, and no
    // validity select -- an invalid sample has an all-zero target mask, so nm = ns = 0 zero it
    const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
    const int nm = __builtin_popcount(tlo) + __builtin_popcount(thi & 0x3FFFFu);
    const int ns = __builtin_popcount(thi & 0x3FFC0000u);
    const float inv_m = nm ? __builtin_amdgcn_rcpf((float)nm) : 0.f;
    const float inv_s = ns ? __builtin_amdgcn_rcpf((float)ns) : 0.f;
    float mx_m = -3.0e38f, mx_s = -3.0e38f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = v5_cls(u, i, h);
        mx_m = (c == 0) ? fmaxf(mx_m, z2[u][i]) : mx_m;
        mx_s = (c == 1) ? fmaxf(mx_s, z2[u][i]) : mx_s;
      }
    mx_m = xhalf_max(mx_m);
    mx_s = xhalf_max(mx_s);
    const float nmL = -mx_m * L2E, nsL = -mx_s * L2E;
    float s_m = 0.f, s_s = 0.f, zt_m = 0.f, zt_s = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float yb[16];
      targets(u, yb);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = v5_cls(u, i, h);
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(z2[u][i], L2E, c == 1 ? nsL : nmL));
        const float ee = (c == 2) ? 0.f : e;
        s_m += (c == 0) ? ee : 0.f;
        s_s += (c == 1) ? ee : 0.f;
        zt_m = __builtin_fmaf((c == 0) ? yb[i] : 0.f, z2[u][i], zt_m);
        zt_s = __builtin_fmaf((c == 1) ? yb[i] : 0.f, z2[u][i], zt_s);
        dz[u][i] = ee;
      }
    }
    s_m = xhalf_sum(s_m);
    s_s = xhalf_sum(s_s);
    const float f_m = nm ? __builtin_amdgcn_rcpf(s_m) : 0.f, f_s = ns ? __builtin_amdgcn_rcpf(s_s) : 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float yb[16];
      targets(u, yb);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = v5_cls(u, i, h);
        dz[u][i] = (c == 2) ? 0.f : __builtin_fmaf(dz[u][i], c == 0 ? f_m : f_s, -yb[i] * (c == 0 ? inv_m : inv_s));
      }
    }
    float l = -(zt_m * inv_m + zt_s * inv_s);
    if (h == 0)
      l += (nm ? mx_m + __builtin_amdgcn_logf(s_m) * LN2 : 0.f) + (ns ? mx_s + __builtin_amdgcn_logf(s_s) * LN2 : 0.f);
    loss_acc += l;
  } else {
    float l = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float yb[16];
      targets(u, yb);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = v5_cls(u, i, h);
        const float v = z2[u][i], y = yb[i];
        const float en = __builtin_amdgcn_exp2f(-fabsf(v) * L2E);  // stable sigmoid / softplus
        const float rp = __builtin_amdgcn_rcpf(1.f + en);
        const float pr = v >= 0.f ? rp : en * rp;
        const float sp = fmaxf(v, 0.f) + __builtin_amdgcn_logf(1.f + en) * LN2;
        const bool okc = valid && c != 2;
        dz[u][i] = okc ? (pr - y) : 0.f;
        l += okc ? (sp - y * v) : 0.f;
      }
    }
    loss_acc += l;
  }
}

template <int LOSS>
__global__ void __launch_bounds__(512, 1)
mlp_fused_train_v5_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                          const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                          float* __restrict__ loss_slabs, int* __restrict__ step) {
  advance_step(step);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;
  const int ntiles = (B + 31) / 32;
  const int per_round = gridDim.x * 8;
  auto fetch = [&](int tile, uint64_t& mi, uint64_t& mt) {
    const int s = tile * 32 + r;
    mi = 0;
    mt = 0;
    if (tile < ntiles && s < B) {
      const int idx = sidx ? sidx[s] : (offset + s);
      mi = masks[idx];
      mt = masks[idx + 1];
    }
  };
  uint64_t nin, ntg;  // the first round's masks: in flight during the prologue
  fetch(blockIdx.x * 8 + wave, nin, ntg);
  {
    constexpr int N16 = IMG_BYTES / 16, K = (N16 + 511) / 512;
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (tid + 512 * k < N16) v[k] = src[tid + 512 * k];
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (tid + 512 * k < N16) dst[tid + 512 * k] = v[k];
  }
  if (tid < 64) reinterpret_cast<float*>(smem + V5_YLUT)[tid] = (float)(((tid >> 2) >> (tid & 3)) & 1);
  if (tid < 32) {
    const uint32_t n = (uint32_t)tid >> 1, b = 2u * (tid & 1);
    reinterpret_cast<uint32_t*>(smem + V5_XLUT)[tid] =
        (((n >> b) & 1u) ? 0x3F80u : 0u) | (((n >> (b + 1)) & 1u) ? 0x3F800000u : 0u);
  }
  if (tid < 8) reinterpret_cast<int*>(smem + V5_FLAGS)[tid] = 0;
  __syncthreads();

  const uint32_t HB = V5_TILES + wave * V5_TILE_BYTES, DB = HB + 8192;  // this wave's tile regions
  // two independent groups of 4 waves (wave w and w + 4 share a SIMD): group kh owns the tiles of
  // waves 4kh .. 4kh+3 and the K-half kh of every dW partial; wave TB = w & 3 of the group owns hidden
  // block TB.  The groups synchronise only internally (LDS counters), so one group's phase A (a
  // latency-bound chain) runs beside the other group's phase B (a dense MFMA stream) on every SIMD.
  const int TB = wave & 3, kh = wave >> 2;
  int gsig = 0;
  bool ok = true;
  const uint32_t GFL = V5_FLAGS + kh * 16;
  auto group_sync = [&]() {  // the 4 waves of this group: release own LDS writes, acquire the others'
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    int* own = static_cast<int*>(__builtin_assume_aligned(smem + GFL + TB * 4, 4));
    __hip_atomic_store(own, ++gsig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int spins = 0;
    for (;;) {
      const int* f = static_cast<const int*>(__builtin_assume_aligned(smem + GFL, 16));
      const int m0 = __hip_atomic_load(f + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int m1 = __hip_atomic_load(f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int m2 = __hip_atomic_load(f + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int m3 = __hip_atomic_load(f + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (min(min(m0, m1), min(m2, m3)) >= gsig) break;
      if (++spins > V4_SPIN_LIMIT) {  // a broken protocol poisons the loss instead of hanging the GPU
        ok = false;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  f32x16 dW2p[2], dW1p[2];  // partials (80 registers with db2a): [out block] / [feature block] of hidden block TB
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    dW2p[u] = f32x16{};
    dW1p[u] = f32x16{};
  }
  f32x16 db2a = f32x16{};
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  float loss_acc = 0.f;
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  V4Stamps st;  // V4_STAMPS builds: A, wait 1, B1, wait 2, dump, wait 3, B2, wait 4 (tools/fused_phases.py)
  if (V5_STAGGER && kh == 1 && blockIdx.x * 8 < ntiles) {
    // start group 1 once group 0 has finished its first phase A, so the two groups run opposite
    // phases (chain beside stream) instead of in lockstep; group 0 never waits for group 1
    int spins = 0;
    const int* f = static_cast<const int*>(__builtin_assume_aligned(smem + V5_FLAGS, 16));
    while (min(min(__hip_atomic_load(f + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP),
                   __hip_atomic_load(f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)),
               min(__hip_atomic_load(f + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP),
                   __hip_atomic_load(f + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) < 1) {
      if (++spins > V4_SPIN_LIMIT) {
        ok = false;
        break;
      }
    }
  }
  st.start();

  for (int base = blockIdx.x * 8; base < ntiles; base += per_round) {
    const int tile = base + wave;
    const bool valid = tile * 32 + r < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(tile + per_round, nin, ntg);

    // ================= phase A: this wave's tile, start to dZ1 =================
    const uint32_t wlo = (uint32_t)imask >> (8 * h), whi = (uint32_t)(imask >> 32) >> (8 * h);
    bf16x8 xf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xf[q] = v4_xfrag<V5_XLUT>(smem, q < 2 ? wlo : whi, q);
    // F1: Z1ᵀ = W1ᵀ·Xᵀ, two hidden tiles' chains interleaved -> relu -> Hᵀ fragments + H image
    bf16x8 hT[4][2];
#pragma unroll
    for (int tp = 0; tp < 2; ++tp) {
      f32x16 a1s[2] = {f32x16{}, f32x16{}};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          a1s[tt] = mfma32(lds_frag(smem, w1t_off(32 * (2 * tp + tt) + r, 2 * q + h)), xf[q], a1s[tt]);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * tp + tt;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          hT[t][q] = relu_pack(a1s[tt], q);
          const u32x4 d = __builtin_bit_cast(u32x4, hT[t][q]);
          *reinterpret_cast<u32x2*>(smem + HB + r * 256 + ((((4 * t + 2 * q) ^ (r & 15))) << 4) + h * 8) =
              u32x2{d[0], d[1]};
          *reinterpret_cast<u32x2*>(smem + HB + r * 256 + ((((4 * t + 2 * q + 1) ^ (r & 15))) << 4) + h * 8) =
              u32x2{d[2], d[3]};
        }
      }
    }
    // F2: Z2ᵀ = W2ᵀ·Hᵀ + b2, both output tiles' chains interleaved
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * u + 8 * g + 4 * h) * 4);
        z2[u][4 * g + 0] = b[0]; z2[u][4 * g + 1] = b[1]; z2[u][4 * g + 2] = b[2]; z2[u][4 * g + 3] = b[3];
      }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          z2[u] = mfma32(lds_frag(smem, w2p_off(32 * u + r, (2 * t + q) * 2 + h)), hT[t][q], z2[u]);

    float dz[2][16];
    full_tile_loss<LOSS, V5_YLUT>(smem, z2, tmask, valid, h, dz, loss_acc);
    bf16x8 dzf[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        dzf[u][q] = pack8(dz[u][8 * q + 0], dz[u][8 * q + 1], dz[u][8 * q + 2], dz[u][8 * q + 3], dz[u][8 * q + 4],
                          dz[u][8 * q + 5], dz[u][8 * q + 6], dz[u][8 * q + 7]);
    // dZ2 image [32 samples][64 outs] (phase B1's B operand)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x4 f = __builtin_bit_cast(u32x4, dzf[u][g >> 1]);
        *reinterpret_cast<u32x2*>(smem + DB + r * 128 + ((((4 * u + g) ^ (r & 7))) << 4) + h * 8) =
            u32x2{f[2 * (g & 1)], f[2 * (g & 1) + 1]};
      }
    // B1: dHᵀ = W2·dZ2ᵀ with the samples on the lanes (the W2Q fragments as the A operand, dZ2ᵀ
    // straight from its accumulator as B), so dHᵀ has hT's layout and dZ1ᵀ = dHᵀ * (H > 0) needs no
    // LDS round trip
    bf16x8 dz1[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 aD = f32x16{};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          aD = mfma32(lds_frag(smem, w2q_off(32 * t + r, (2 * u + q) * 2 + h)), dzf[u][q], aD);
#pragma unroll
      for (int q = 0; q < 2; ++q) dz1[t][q] = mask_by(hT[t][q], aD, q);
    }
    st.mark(0);
    group_sync();  // (1) the group's H and dZ2 images are in LDS
    st.mark(1);
    // Phase B and the dump address LDS through lane values the compiler may not hoist out of the
    // loop: hoisted, their ~30 loop-invariant addresses spill (256-VGPR budget); recomputed here they
    // cost a few VALU while the matrix pipe is the bottleneck.
    int lb = lane;
    asm volatile("" : "+v"(lb));
    const int rb = lb & 31, hb_ = lb >> 5, q4b = (lb & 15) >> 2, p4b = lb & 3, g1b = (lb >> 4) & 1;

    // ================= phase B1: dW2 partial = Hᵀ·dZ2 over this K-half's 4 tiles =================
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t hb = V5_TILES + (4 * kh + j) * V5_TILE_BYTES, db = hb + 8192;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 a = tr_frag<1>(smem, hb, 32 * TB, q, hb_, q4b, p4b, g1b);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bf16x8 bd = tr_frag<0>(smem, db, 32 * u, q, hb_, q4b, p4b, g1b);
          dW2p[u] = mfma32(a, bd, dW2p[u]);
          if (TB == u) db2a = mfma32(ones, bd, db2a);  // waves 0-3: db2 of out block TB, this K-half
        }
      }
    }
    st.mark(2);
    group_sync();  // (2) the group's H and dZ2 images are consumed
    st.mark(3);

    // dump: the dZ1 image [32 samples][128 hid] over the H image (same layout: phase B2 reads it
    // transposed like B1 reads H), the X image [32 samples][64 feat] over the dZ2 image
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x4 d = __builtin_bit_cast(u32x4, dz1[t][q]);
        *reinterpret_cast<u32x2*>(smem + HB + rb * 256 + ((((4 * t + 2 * q) ^ (rb & 15))) << 4) + hb_ * 8) =
            u32x2{d[0], d[1]};
        *reinterpret_cast<u32x2*>(smem + HB + rb * 256 + ((((4 * t + 2 * q + 1) ^ (rb & 15))) << 4) + hb_ * 8) =
            u32x2{d[2], d[3]};
      }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<bf16x8*>(smem + DB + rb * 128 + ((((2 * q + hb_) ^ (rb & 7))) << 4)) =
          v4_xfrag<V5_XLUT>(smem, q < 2 ? wlo : whi, q);
    st.mark(4);
    group_sync();  // (3)
    st.mark(5);

    // ================= phase B2: dW1ᵀ partial = dZ1ᵀ·X over this K-half's 4 tiles =================
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t hb = V5_TILES + (4 * kh + j) * V5_TILE_BYTES, xb = hb + 8192;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 a = tr_frag<1>(smem, hb, 32 * TB, q, hb_, q4b, p4b, g1b);
#pragma unroll
        for (int u = 0; u < 2; ++u) dW1p[u] = mfma32(a, tr_frag<0>(smem, xb, 32 * u, q, hb_, q4b, p4b, g1b), dW1p[u]);
      }
    }
    st.mark(6);
    group_sync();  // (4) the next round rewrites the group's tile regions
    st.mark(7);
  }
  // ================= epilogue: the two K-halves -> one slab, fixed order =================
  float lsum = wave_sum(loss_acc);
  if (!ok) lsum = __builtin_nanf("");
  __syncthreads();  // both groups are out of their loops: the tile regions are free
  float* RED = reinterpret_cast<float*>(smem);  // [kh][16 tiles][4 g][64 lanes][4]: 0..7 dW2, 8..15 dW1ᵀ
  float* DB2S = reinterpret_cast<float*>(smem + V5_RED);  // [4 waves][32]
  float* LOSSS = DB2S + 8 * 32;                           // [8]
#pragma unroll
  for (int which = 0; which < 2; ++which)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const f32x16& acc = which ? dW1p[u] : dW2p[u];
      const int T = 8 * which + 2 * TB + u;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(RED + kh * 16384 + ((T * 4 + g) * 64 + lane) * 4) =
            f32x4{acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
    }
  if (TB < 2 && h == 0) DB2S[wave * 32 + r] = db2a[0];  // accumulator column r = output 32 TB + r
  if (lane == 0) LOSSS[wave] = lsum;
  __syncthreads();
  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(slab, 0, SLAB_STRIDE * 4, 0x00020000);
  for (int e = tid; e < 2 * 2048; e += 512) {
    f32x4 v;
    if (e < 2048) {
      const int f = e >> 5, c = (e & 31) * 4;
      const int T = 8 + 2 * (c >> 5) + (f >> 5), g = (c & 31) >> 3, l = ((c >> 2) & 1) * 32 + (f & 31);
      const int at = ((T * 4 + g) * 64 + l) * 4;
      v = *reinterpret_cast<const f32x4*>(RED + at) + *reinterpret_cast<const f32x4*>(RED + 16384 + at);
    } else {
      const int q = e - 2048, c = q >> 4, o = (q & 15) * 4;
      const int T = 2 * (c >> 5) + (o >> 5), g = (c & 31) >> 3, l = ((c >> 2) & 1) * 32 + (o & 31);
      const int at = ((T * 4 + g) * 64 + l) * 4 + (c & 3);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = RED[at + 4 * k] + RED[16384 + at + 4 * k];
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), srd, e * 16, 0, 16 /* sc1 */);
  }
  if (tid < 64) {  // b2: out block u = tid >> 5 from waves u (K-half 0) and 4 + u (K-half 1)
    const int u = tid >> 5, o = tid & 31;
    slab[P_B2 + tid] = DB2S[u * 32 + o] + DB2S[(4 + u) * 32 + o];
  }
  if (tid == 0) {
    float l = 0.f;
    for (int w = 0; w < 8; ++w) l += LOSSS[w];
    loss_slabs[blockIdx.x] = l;
  }
  if (V4_STAMPS && lane < 10) {  // phase cycles of this wave -> spare slab floats (after the slab)
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < 10; ++j) v = (lane == j) ? st.acc[j] : v;
    slab[P_TOTAL + wave * 16 + lane] = (float)v;
  }
}

// ============================================================================================
// v6: producer/consumer units -- forward waves feed backward waves through a 3-slot LDS ring.
//
// v4's hidden-split pairs meet three times per 32-sample tile (H halves, softmax statistics, dZ2
// halves); V4_STAMPS phase timers show each wave spending ~27 % of the tile waiting on its partner,
// and a meeting costs its LDS round trips even when both arrive together.  v6 splits the work by
// STAGE instead of by hidden unit:
//   * a unit = 4 waves working on one tile stream: two forward waves F0/F1 (even / odd tiles of the
//     unit) and two backward waves B0/B1 (hidden halves of every tile of the unit);
//   * F runs a whole tile alone -- X -> F1 (16 MFMAs) -> relu -> F2 (16) -> full grouped softmax over
//     all 64 outputs (no statistics exchange) -> dZ2 -- and leaves the H, dZ2 and X images of the
//     tile in a ring slot (16 KB), then raises the slot's FULL counter;
//   * B_rho waits for FULL, runs B1 for its hidden half (dZ2 A fragments read back from the dZ2
//     image: the same 8-byte granules F wrote), the relu mask from the H image, then dW2 / dW1T
//     into its AGPR-resident half of dW (v4's accumulator set) and db2 of output tile rho; it raises
//     its DONE counter once its last read of the slot has returned;
//   * F waits for a slot only when the ring is full (3 slots: F writes tile k while B works on k-1,
//     k-2), so in steady state nobody waits: the only coupling is a one-way hand-off.
// Both units share the CU so that every SIMD hosts one forward and one backward wave (wave w runs
// on SIMD w % 4): the VALU-heavy loss of one beside the MFMA-heavy dW chain of the other.  Counters
// are monotonic (no ABA) and every wait is bounded: a broken protocol poisons the loss with NaN.
#ifndef V6_AGPR
#define V6_AGPR 0  // 1: B's dW accumulators pinned in AGPRs (128 V + 128 A); 0: VGPR-form (256 VGPRs for both roles)
#endif
#ifndef V6_WREG
#define V6_WREG 1  // forward waves keep their 32 weight fragments in registers (needs V6_AGPR 0)
#endif
#ifndef V6_BPRE
#define V6_BPRE 1  // backward waves issue every LDS read of a tile at once and release the slot before computing
#endif
#ifndef V6_FPRIO
#define V6_FPRIO 1  // 1: forward waves run at s_setprio 1 (they bound the pipeline; backward waves have slack)
#endif
#ifndef V6_SPLIT
#define V6_SPLIT 1  // 1: per-output-tile softmax statistics merged online (tile 0's loss beside tile 1's F2)
#endif
#ifndef V6_ILV
#define V6_ILV 1  // 1: sched_barrier fences keep tile 0's softmax steps between tile 1's F2 MFMAs
#endif
#ifndef V6_YB1
#define V6_YB1 1  // 1: the forward softmax reads the target LUT once per tile (8 KB of LDS reads fewer per tile)
#endif
#ifndef V6_DYN
#define V6_DYN 0  // 1 (measured -0.6%): forward waves claim the unit's tiles from an LDS counter instead of strictly alternating
#endif
#ifndef V6_BPRIO
#define V6_BPRIO 0  // 1 (measured -22%): backward waves raise their priority above the forward waves' for their read burst
#endif
#ifndef V6_XPRE
#define V6_XPRE 0  // 1 (measured -3.7%): the forward wave builds its next tile's X fragments at the end of the current tile
#endif
#ifndef V6_SEG
#define V6_SEG 0  // 1: forward waves share SIMDs with forward waves, backward with backward
#endif
#ifndef V6_NOFENCE
#define V6_NOFENCE 0  // 1: ring counters raised with a compiler barrier only (LDS executes a wave's ops in order)
#endif
#ifndef V6_F1P
#define V6_F1P 1  // hidden tiles whose F1 accumulator chains are interleaved (1 or 2)
#endif
#ifndef V6_UNROLL
#define V6_UNROLL 0  // 1: forward loop unrolled over the 3 ring slots (measured: more live addresses, spills)
#endif
#ifndef V6_DB2DOT
#define V6_DB2DOT 0  // 1 (measured slower): db2 column sums on v_dot2_f32_bf16 (8 VALU per tile) instead of 2 ones·dZ2 MFMAs
#endif
#ifndef V6_XMASK
#define V6_XMASK 0  // 1: a slot carries the tile's 32 input masks (256 B) instead of the 4 KB X image
#endif
#ifndef V6_RECYCLE
#define V6_RECYCLE 1  // 1: the W1ᵀ / W2ᵀ(P) images (dead once the forward waves hold their weights in
                      // registers) become each unit's 4th ring slot
#endif
// slot: H0 4K | H1 4K | D2 4K | X image 4K (V6_XMASK 0) or input masks 256 B (V6_XMASK 1: 4 slots fit)
constexpr int V6_SLOT = V6_XMASK ? 12544 : 16384;
constexpr int V6_RSLOTS = V6_XMASK ? 4 : 3;  // slots per unit in the ring area (+1 recycled image slot)
constexpr int V6_NSLOT = V6_RSLOTS + ((V6_RECYCLE && V6_WREG) ? 1 : 0);
static_assert(!V6_RECYCLE || V6_XMASK || 2 * V6_SLOT <= IMG_W2Q, "recycled slots must fit below the W2Q image");
constexpr int V6_SH = 0, V6_SD2 = 8192, V6_SX = 12288;
constexpr int V6_XLUT = IMG_BYTES;       // 16 x 8 B: input nibble -> 4 bf16 {0,1}
constexpr int V6_YLUT = V6_XLUT + 128;   // 16 x f32x4: target nibble -> 4 {0,1} floats
constexpr int V6_FLAGS = V6_YLUT + 256;  // [2 units][16 ints]: full[N] | done0[N] | done1[N] | next (V6_DYN)
constexpr int V6_RING = V6_FLAGS + 128;  // [2 units][3 slots][16 KB]
constexpr int V6_LOSSR = V6_RING + 2 * V6_RSLOTS * V6_SLOT;  // V6_DYN: [2 units][slot][64 lanes] per-tile loss
constexpr int V6_LOOP_LDS = V6_LOSSR + 2 * V6_NSLOT * 256;
// byte offset of ring slot `slot` of unit `unit`
EM_DEVICE uint32_t v6_slot(int unit, int slot) {
  return slot < V6_RSLOTS ? V6_RING + (unit * V6_RSLOTS + slot) * V6_SLOT : unit * V6_SLOT;
}
constexpr int V6_RED = 131072;  // epilogue: two fp32 dW images [2][16384] below, DB2S [2][64] + LOSSS [8] above
constexpr int V6_LDS = (V6_LOOP_LDS > V6_RED + 2048 ? V6_LOOP_LDS : V6_RED + 2048);
static_assert(V6_LDS <= 163840 && V6_RING % 16 == 0, "v6 LDS budget");
constexpr int V6_SPIN_LIMIT = 1 << 20;  // ~50 ms of polling: a legitimate wait is microseconds

// raise a ring counter.  V6_NOFENCE: the LDS pipeline executes one wave's operations in issue order,
// so a flag store issued after the wave's data writes (or reads) lands after them and no
// s_waitcnt lgkmcnt(0) is needed; the asm memory clobbers keep the compiler from moving LDS ops across it
EM_DEVICE void v6_signal(char* smem, uint32_t off, int value) {
  if (V6_NOFENCE) {
    asm volatile("" ::: "memory");
    __hip_atomic_store(reinterpret_cast<int*>(smem + off), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
  } else {
    pair_signal(smem, off, value);
  }
}

// wait until the LDS counter at off reaches target (skipped once a wait has failed: the launch then
// drains quickly and reports NaN)
EM_DEVICE void v6_wait(const char* smem, uint32_t off, int target, bool& ok) {
  if (!ok) return;
  int spins = 0;
  while (__hip_atomic_load(reinterpret_cast<const int*>(smem + off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
         target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > V6_SPIN_LIMIT) {
      ok = false;
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// stream index U of a unit (tiles U, U + nunits, ...).  V6_TMAP 1: blocks are numbered XCD-major
// (block b runs on XCD b % 8), so the 32 blocks of one XCD own 64 consecutive streams and each XCD
// reads one contiguous 16 KB run of masks per round instead of 512-B pieces 4 KB apart
#ifndef V6_TMAP
#define V6_TMAP 0
#endif
EM_DEVICE int v6_unit_id(int unit) {
  int b = blockIdx.x;
  if (V6_TMAP && (gridDim.x & 7) == 0) b = (b & 7) * (gridDim.x >> 3) + (b >> 3);
  return b * 2 + unit;
}

EM_DEVICE int v6_ntiles_of_unit(int B, int U, int nunits) {
  const int ntiles = (B + 31) / 32;
  return U < ntiles ? (ntiles - U + nunits - 1) / nunits : 0;
}

// Grouped softmax-CE of a whole tile in ONE wave (v6 forward).  The class of the lane's element i of
// output tile u (main / star / pad) is a compile-time constant except for 4 elements of tile 1 whose
// class depends on the lane half h (outputs 48-51 and 58-63 straddle the group edges), so every
// statically classified element emits only its own group's ops: a select-form "x ? v : 0" fed into
// an fma or add would have to be kept (IEEE: fma(0, inf, a) is NaN) and costs a VALU op per element
// per group.  Max / sum / target-dot reductions run as independent partial chains.
template <int YL>
EM_DEVICE void v6_softmax(const char* smem, const f32x16 (&z2)[2], uint64_t tmask, int h, float (&dz)[2][16],
                          float& loss_acc) {
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  auto targets = [&](int u, float (&yb)[16]) {
    const uint32_t tmh = (uint32_t)(tmask >> (32 * u)) >> (4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + YL + (__builtin_amdgcn_ubfe(tmh, 8 * g, 4) << 4));
      yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
    }
  };
  const bool h0 = h == 0;
  const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
  const int nm = __builtin_popcount(tlo) + __builtin_popcount(thi & 0x3FFFFu);  // bits 0..49
  const int ns = __builtin_popcount(thi & 0x3FFC0000u);                          // bits 50..61
  const float inv_m = nm ? __builtin_amdgcn_rcpf((float)nm) : 0.f;
  const float inv_s = ns ? __builtin_amdgcn_rcpf((float)ns) : 0.f;
  float mm[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f}, ms[2] = {-3.0e38f, -3.0e38f};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = v5_cls(u, i, 0), c1 = v5_cls(u, i, 1);
      const float v = z2[u][i];
      if (c0 == c1) {
        if (c0 == 0) mm[i & 3] = fmaxf(mm[i & 3], v);
        if (c0 == 1) ms[i & 1] = fmaxf(ms[i & 1], v);
      } else if (c0 == 0) {  // main (h = 0) / star (h = 1)
        mm[i & 3] = h0 ? fmaxf(mm[i & 3], v) : mm[i & 3];
        ms[i & 1] = h0 ? ms[i & 1] : fmaxf(ms[i & 1], v);
      } else {  // star (h = 0) / pad (h = 1)
        ms[i & 1] = h0 ? fmaxf(ms[i & 1], v) : ms[i & 1];
      }
    }
  const float mx_m = xhalf_max(fmaxf(fmaxf(mm[0], mm[1]), fmaxf(mm[2], mm[3])));
  const float mx_s = xhalf_max(fmaxf(ms[0], ms[1]));
  const float nmL = -mx_m * L2E, nsL = -mx_s * L2E;
  float sm[4] = {0.f, 0.f, 0.f, 0.f}, ss[2] = {0.f, 0.f}, tm[4] = {0.f, 0.f, 0.f, 0.f}, ts[2] = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float yb[16];
    targets(u, yb);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = v5_cls(u, i, 0), c1 = v5_cls(u, i, 1);
      const float v = z2[u][i];
      float e = 0.f;
      if (c0 == c1) {
        if (c0 == 0) {
          e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nmL));
          sm[i & 3] += e;
          tm[i & 3] = __builtin_fmaf(yb[i], v, tm[i & 3]);
        } else if (c0 == 1) {
          e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nsL));
          ss[i & 1] += e;
          ts[i & 1] = __builtin_fmaf(yb[i], v, ts[i & 1]);
        }
      } else if (c0 == 0) {  // main (h = 0) / star (h = 1)
        e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, h0 ? nmL : nsL));
        const float ty = yb[i] * v;
        sm[i & 3] = h0 ? sm[i & 3] + e : sm[i & 3];
        ss[i & 1] = h0 ? ss[i & 1] : ss[i & 1] + e;
        tm[i & 3] = h0 ? tm[i & 3] + ty : tm[i & 3];
        ts[i & 1] = h0 ? ts[i & 1] : ts[i & 1] + ty;
      } else {  // star (h = 0) / pad (h = 1)
        e = h0 ? __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nsL)) : 0.f;
        ss[i & 1] += e;
        ts[i & 1] = h0 ? __builtin_fmaf(yb[i], v, ts[i & 1]) : ts[i & 1];
      }
      dz[u][i] = e;
    }
  }
  const float s_m = xhalf_sum((sm[0] + sm[1]) + (sm[2] + sm[3])), s_s = xhalf_sum(ss[0] + ss[1]);
  const float f_m = nm ? __builtin_amdgcn_rcpf(s_m) : 0.f, f_s = ns ? __builtin_amdgcn_rcpf(s_s) : 0.f;
  const float ni_m = -inv_m, ni_s = -inv_s;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float yb[16];  // re-read (8 LDS loads) rather than held across the sums: keeps the forward wave spill-free
    targets(u, yb);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = v5_cls(u, i, 0), c1 = v5_cls(u, i, 1);
      if (c0 == c1) {
        if (c0 == 0) dz[u][i] = __builtin_fmaf(dz[u][i], f_m, yb[i] * ni_m);
        if (c0 == 1) dz[u][i] = __builtin_fmaf(dz[u][i], f_s, yb[i] * ni_s);
        if (c0 == 2) dz[u][i] = 0.f;
      } else if (c0 == 0) {
        dz[u][i] = __builtin_fmaf(dz[u][i], h0 ? f_m : f_s, yb[i] * (h0 ? ni_m : ni_s));
      } else {  // the pad lanes' e is 0 and their target bit (outputs 62/63) is 0
        dz[u][i] = __builtin_fmaf(dz[u][i], f_s, yb[i] * ni_s);
      }
    }
  }
  float l = -(((tm[0] + tm[1]) + (tm[2] + tm[3])) * inv_m + (ts[0] + ts[1]) * inv_s);
  if (h == 0)
    l += (nm ? mx_m + __builtin_amdgcn_logf(s_m) * LN2 : 0.f) + (ns ? mx_s + __builtin_amdgcn_logf(s_s) * LN2 : 0.f);
  loss_acc += l;
}

// v6_softmax with the main-group statistics split per output tile and merged online (flash-softmax
// style): tile 0's max / exp / sums need only Z2 tile 0, so they can run on the VALU while tile 1's
// F2 chain is still in the matrix pipe.  dZ2 of tile u carries its tile's rescale a_u = exp(m_u - M).
template <int YL, typename Hook>
EM_DEVICE void v6_softmax_split(const char* smem, const f32x16 (&z2)[2], uint64_t tmask, int h, float (&dz)[2][16],
                                float& loss_acc, Hook&& hook) {
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  auto targets = [&](int u, float (&yb)[16]) {
    const uint32_t tmh = (uint32_t)(tmask >> (32 * u)) >> (4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + YL + (__builtin_amdgcn_ubfe(tmh, 8 * g, 4) << 4));
      yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
    }
  };
  const bool h0 = h == 0;
  const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
  const int nm = __builtin_popcount(tlo) + __builtin_popcount(thi & 0x3FFFFu);  // bits 0..49
  const int ns = __builtin_popcount(thi & 0x3FFC0000u);                          // bits 50..61
  const float inv_m = nm ? __builtin_amdgcn_rcpf((float)nm) : 0.f;
  const float inv_s = ns ? __builtin_amdgcn_rcpf((float)ns) : 0.f;
  float tm[4] = {0.f, 0.f, 0.f, 0.f}, ts[2] = {0.f, 0.f};
  // ---- tile 0: outputs 0..31, all main.  step(j), j = 0..7, is issued between tile 1's F2 MFMAs by
  // the caller (hook): in-order issue lets the VALU run only between MFMAs in program order ----
  float m0 = 0.f, s0 = 0.f, nL = 0.f;
  float mm0[4], sm[4] = {0.f, 0.f, 0.f, 0.f}, yb0[16];
  auto step = [&](int j) {
    if (j == 0) {
      mm0[0] = z2[0][0]; mm0[1] = z2[0][1]; mm0[2] = z2[0][2]; mm0[3] = z2[0][3];
#pragma unroll
      for (int i = 4; i < 16; ++i) mm0[i & 3] = fmaxf(mm0[i & 3], z2[0][i]);
      targets(0, yb0);
    } else if (j == 1) {
      m0 = xhalf_max(fmaxf(fmaxf(mm0[0], mm0[1]), fmaxf(mm0[2], mm0[3])));
      nL = -m0 * L2E;
    } else if (j < 6) {
#pragma unroll
      for (int i = 4 * (j - 2); i < 4 * (j - 1); ++i) {
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(z2[0][i], L2E, nL));
        sm[i & 3] += e;
        tm[i & 3] = __builtin_fmaf(yb0[i], z2[0][i], tm[i & 3]);
        dz[0][i] = e;
      }
    } else if (j == 6) {
      s0 = xhalf_sum((sm[0] + sm[1]) + (sm[2] + sm[3]));
    }
  };
  hook(step);
  // ---- tile 1: outputs 32..63 (main 32..49, star 50..61, pad 62/63) ----
  float mm[2] = {-3.0e38f, -3.0e38f}, ms[2] = {-3.0e38f, -3.0e38f};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c0 = v5_cls(1, i, 0), c1 = v5_cls(1, i, 1);
    const float v = z2[1][i];
    if (c0 == c1) {
      if (c0 == 0) mm[i & 1] = fmaxf(mm[i & 1], v);
      if (c0 == 1) ms[i & 1] = fmaxf(ms[i & 1], v);
    } else if (c0 == 0) {  // main (h = 0) / star (h = 1)
      mm[i & 1] = h0 ? fmaxf(mm[i & 1], v) : mm[i & 1];
      ms[i & 1] = h0 ? ms[i & 1] : fmaxf(ms[i & 1], v);
    } else {  // star (h = 0) / pad (h = 1)
      ms[i & 1] = h0 ? fmaxf(ms[i & 1], v) : ms[i & 1];
    }
  }
  const float m1 = xhalf_max(fmaxf(mm[0], mm[1]));
  const float mx_s = xhalf_max(fmaxf(ms[0], ms[1]));
  const float nmL = -m1 * L2E, nsL = -mx_s * L2E;
  float s1p[2] = {0.f, 0.f}, ss[2] = {0.f, 0.f};
  float yb1[16];
  targets(1, yb1);
  {
    float (&yb)[16] = yb1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = v5_cls(1, i, 0), c1 = v5_cls(1, i, 1);
      const float v = z2[1][i];
      float e = 0.f;
      if (c0 == c1) {
        if (c0 == 0) {
          e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nmL));
          s1p[i & 1] += e;
          tm[i & 3] = __builtin_fmaf(yb[i], v, tm[i & 3]);
        } else if (c0 == 1) {
          e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nsL));
          ss[i & 1] += e;
          ts[i & 1] = __builtin_fmaf(yb[i], v, ts[i & 1]);
        }
      } else if (c0 == 0) {
        e = __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, h0 ? nmL : nsL));
        const float ty = yb[i] * v;
        s1p[i & 1] = h0 ? s1p[i & 1] + e : s1p[i & 1];
        ss[i & 1] = h0 ? ss[i & 1] : ss[i & 1] + e;
        tm[i & 3] = h0 ? tm[i & 3] + ty : tm[i & 3];
        ts[i & 1] = h0 ? ts[i & 1] : ts[i & 1] + ty;
      } else {
        e = h0 ? __builtin_amdgcn_exp2f(__builtin_fmaf(v, L2E, nsL)) : 0.f;
        ss[i & 1] += e;
        ts[i & 1] = h0 ? __builtin_fmaf(yb[i], v, ts[i & 1]) : ts[i & 1];
      }
      dz[1][i] = e;
    }
  }
  const float s1 = xhalf_sum(s1p[0] + s1p[1]), s_s = xhalf_sum(ss[0] + ss[1]);
  // ---- online merge of the main group: M = max(m0, m1), S = a0 s0 + a1 s1 ----
  const float M = fmaxf(m0, m1);
  const float a0 = __builtin_amdgcn_exp2f((m0 - M) * L2E), a1 = __builtin_amdgcn_exp2f((m1 - M) * L2E);
  const float S = __builtin_fmaf(a0, s0, a1 * s1);
  const float rS = nm ? __builtin_amdgcn_rcpf(S) : 0.f;
  const float f0 = a0 * rS, f1 = a1 * rS, f_s = ns ? __builtin_amdgcn_rcpf(s_s) : 0.f;
  const float ni_m = -inv_m, ni_s = -inv_s;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float yr[16];  // V6_YB1: the targets read once per tile (held in registers); else re-read here
    if (!V6_YB1) targets(u, yr);
    const float (&yb)[16] = V6_YB1 ? (u == 0 ? yb0 : yb1) : yr;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = v5_cls(u, i, 0), c1 = v5_cls(u, i, 1);
      const float fm = u == 0 ? f0 : f1;
      if (c0 == c1) {
        if (c0 == 0) dz[u][i] = __builtin_fmaf(dz[u][i], fm, yb[i] * ni_m);
        if (c0 == 1) dz[u][i] = __builtin_fmaf(dz[u][i], f_s, yb[i] * ni_s);
        if (c0 == 2) dz[u][i] = 0.f;
      } else if (c0 == 0) {
        dz[u][i] = __builtin_fmaf(dz[u][i], h0 ? fm : f_s, yb[i] * (h0 ? ni_m : ni_s));
      } else {  // the pad lanes' e is 0 and their target bit (outputs 62/63) is 0
        dz[u][i] = __builtin_fmaf(dz[u][i], f_s, yb[i] * ni_s);
      }
    }
  }
  float l = -(((tm[0] + tm[1]) + (tm[2] + tm[3])) * inv_m + (ts[0] + ts[1]) * inv_s);
  if (h == 0)
    l += (nm ? M + __builtin_amdgcn_logf(S) * LN2 : 0.f) + (ns ? mx_s + __builtin_amdgcn_logf(s_s) * LN2 : 0.f);
  loss_acc += l;
}

// forward wave F (0/1) of unit `unit`: tiles k = F, F + 2, ... of the unit's stream
template <int LOSS, int F>
EM_DEVICE void v6_forward(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                          int offset, int unit, int lane, float& loss_acc, bool& ok, V4Stamps& st) {
  const int r = lane & 31, h = lane >> 5;
  const int nunits = gridDim.x * 2, U = v6_unit_id(unit);
  const int K = v6_ntiles_of_unit(B, U, nunits);
  const uint32_t FL = V6_FLAGS + unit * 64;
  auto fetch = [&](int k, uint64_t& mi, uint64_t& mt) {
    const int s = (U + k * nunits) * 32 + r;
    mi = 0;
    mt = 0;
    if (k < K && s < B) {
      const int idx = sidx ? sidx[s] : (offset + s);
      mi = masks[idx];
      mt = masks[idx + 1];
    }
  };
  uint64_t nin = 0, ntg = 0;
  if (!V6_DYN) fetch(F, nin, ntg);
  // the forward wave's weight fragments (W1ᵀ 4 x 4, W2ᵀ 2 x 8: 128 VGPRs) stay in registers for the
  // whole launch: no LDS read stands between the tile's operands and its 32 MFMAs
  bf16x8 w1r[4][4], w2r[2][8];
  if (V6_WREG) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) w1r[t][q] = lds_frag(smem, w1t_off(32 * t + r, 2 * q + h));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) w2r[u][kk] = lds_frag(smem, w2p_off(32 * u + r, kk * 2 + h));
  }
  if (V6_NSLOT > V6_RSLOTS) __syncthreads();  // every forward wave holds its weights: the images are free
  st.start();
  bf16x8 xfc[4];  // V6_XPRE: X fragments of the wave's next tile
  auto xbuild = [&](int k) {
    const bool vk = (U + k * nunits) * 32 + r < B;
    const uint64_t im = vk ? (nin | BIAS_BIT) : 0ull;
    const uint32_t wlo = (uint32_t)im >> (8 * h), whi = (uint32_t)(im >> 32) >> (8 * h);
#pragma unroll
    for (int q = 0; q < 4; ++q) xfc[q] = v4_xfrag<V6_XLUT>(smem, q < 2 ? wlo : whi, q);
  };
  auto ftile = [&](int k, auto slot_c, int knext) {  // slot_c: the ring slot (compile-time when unrolled)
    const int slot = slot_c;
    const bool valid = (U + k * nunits) * 32 + r < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(knext, nin, ntg);
    const uint32_t SB = v6_slot(unit, slot);
    if (k >= V6_NSLOT) {  // the slot's previous tile (k - 3) must be consumed by both backward waves
      v6_wait(smem, FL + (V6_NSLOT + slot) * 4, k - V6_NSLOT + 1, ok);
      v6_wait(smem, FL + (2 * V6_NSLOT + slot) * 4, k - V6_NSLOT + 1, ok);
    }
    st.mark(0);

    // X fragments (B of F1) + X image [32 samples][64 feat] for dW1T.  V6_XPRE: the fragments were built
    // at the end of the previous tile (loop-carried xfc), so F1 starts without an LDS round trip
    bf16x8 xf[4];
    if (V6_XPRE) {
#pragma unroll
      for (int q = 0; q < 4; ++q) xf[q] = xfc[q];
    } else {
      const uint32_t wlo = (uint32_t)imask >> (8 * h), whi = (uint32_t)(imask >> 32) >> (8 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) xf[q] = v4_xfrag<V6_XLUT>(smem, q < 2 ? wlo : whi, q);
    }
    if (V6_XMASK) {
      if (h == 0) *reinterpret_cast<uint64_t*>(smem + SB + V6_SX + 8 * r) = imask;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(smem + v4_img<false>(SB + V6_SX, r, 16 * q + 8 * h)) = xf[q];
    }

    // F1: Z1ᵀ = W1ᵀ·Xᵀ (two hidden tiles' chains interleaved) -> relu -> Hᵀ fragments + H images
    bf16x8 hT[4][2];
    constexpr int F1P = V6_F1P;  // hidden tiles per F1 chain group (interleaved accumulator chains)
#pragma unroll
    for (int tp = 0; tp < 4 / F1P; ++tp) {
      f32x16 a1s[F1P];
#pragma unroll
      for (int tt = 0; tt < F1P; ++tt) a1s[tt] = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int tt = 0; tt < F1P; ++tt)
          a1s[tt] = mfma32(V6_WREG ? w1r[F1P * tp + tt][q] : lds_frag(smem, w1t_off(32 * (F1P * tp + tt) + r, 2 * q + h)),
                           xf[q], a1s[tt]);
#pragma unroll
      for (int tt = 0; tt < F1P; ++tt) {
        const int t = F1P * tp + tt;
        const uint32_t HB = SB + V6_SH + (t >> 1) * 4096;  // H sub-image of hidden half t >> 1
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          hT[t][q] = relu_pack(a1s[tt], q);
          const u32x4 d = __builtin_bit_cast(u32x4, hT[t][q]);
          *reinterpret_cast<u32x2*>(smem + v4_img<true>(HB, r, 32 * (t & 1) + 16 * q + 4 * h)) = u32x2{d[0], d[1]};
          *reinterpret_cast<u32x2*>(smem + v4_img<true>(HB, r, 32 * (t & 1) + 16 * q + 8 + 4 * h)) = u32x2{d[2], d[3]};
        }
      }
    }

    st.mark(1);
    // F2: Z2ᵀ = W2ᵀ·Hᵀ + b2, both output tiles' chains interleaved
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * u + 8 * g + 4 * h) * 4);
        z2[u][4 * g + 0] = b[0]; z2[u][4 * g + 1] = b[1]; z2[u][4 * g + 2] = b[2]; z2[u][4 * g + 3] = b[3];
      }
    auto f2mfma = [&](int u, int kk) {
      z2[u] = mfma32(V6_WREG ? w2r[u][kk] : lds_frag(smem, w2p_off(32 * u + r, kk * 2 + h)), hT[kk >> 1][kk & 1], z2[u]);
    };
    // tile 0's chain first; tile 1's chain is issued by the softmax hook, one MFMA per step of tile 0's
    // statistics (V6_ILV: sched_barrier fences pin that order)
    auto hook = [&](auto&& step) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f2mfma(1, j);
        if (V6_ILV) __builtin_amdgcn_sched_barrier(0);
        step(j);
        if (V6_ILV) __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (V6_SPLIT && LOSS == 0) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) f2mfma(0, kk);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int u = 0; u < 2; ++u)
            z2[u] = mfma32(V6_WREG ? w2r[u][2 * t + q] : lds_frag(smem, w2p_off(32 * u + r, (2 * t + q) * 2 + h)),
                           hT[t][q], z2[u]);
    }
    st.mark(2);

    float dz[2][16];
    float lt = 0.f;  // this lane's loss terms of the tile
    if (LOSS == 0 && V6_SPLIT)
      v6_softmax_split<V6_YLUT>(smem, z2, tmask, h, dz, lt, hook);
    else if (LOSS == 0)
      v6_softmax<V6_YLUT>(smem, z2, tmask, h, dz, lt);
    else
      full_tile_loss<LOSS, V6_YLUT>(smem, z2, tmask, valid, h, dz, lt);
    // V6_DYN: the tile's loss rides in the ring and B0 sums it in tile order (which forward wave ran a tile
    // varies from run to run; the reported loss must not)
    if (V6_DYN) reinterpret_cast<float*>(smem + V6_LOSSR)[(unit * V6_NSLOT + slot) * 64 + lane] = lt;
    else loss_acc += lt;
    st.mark(3);

    // dZ2 image [32 samples][64 outs]: 8-byte granules of 4 consecutive outputs (B reads the same
    // granules back as its B1 A fragments and through transposing reads for dW2 / db2)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x4 fq = __builtin_bit_cast(
            u32x4, pack8(dz[u][8 * q + 0], dz[u][8 * q + 1], dz[u][8 * q + 2], dz[u][8 * q + 3], dz[u][8 * q + 4],
                         dz[u][8 * q + 5], dz[u][8 * q + 6], dz[u][8 * q + 7]));
        *reinterpret_cast<u32x2*>(smem + v4_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 4 * h)) = u32x2{fq[0], fq[1]};
        *reinterpret_cast<u32x2*>(smem + v4_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 8 + 4 * h)) =
            u32x2{fq[2], fq[3]};
      }
    v6_signal(smem, FL + slot * 4, k + 1);  // FULL
    if (V6_XPRE) xbuild(knext);  // the next tile's X fragments (its masks were fetched a tile ago)
    st.mark(4);
  };
  if (V6_DYN) {
    int* next = reinterpret_cast<int*>(smem + FL + 3 * V6_NSLOT * 4);
    auto claim = [&]() {
      int v = 0;
      if (lane == 0) v = __hip_atomic_fetch_add(next, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return __builtin_amdgcn_readfirstlane(v);
    };
    int kc = claim();
    fetch(kc, nin, ntg);
    if (V6_XPRE) xbuild(kc);
    while (kc < K) {
      const int kn = claim();
      ftile(kc, kc % V6_NSLOT, kn);
      kc = kn;
    }
  } else if (V6_XPRE) {
    xbuild(F);
    for (int k = F; k < K; k += 2) ftile(k, k % V6_NSLOT, k + 2);
  } else if (V6_UNROLL && V6_NSLOT == 4) {
    // tiles k = F + 2m alternate between slots F and F + 2: unrolled so both slot bases are constants
    // folded into the LDS instructions' offsets instead of one address add per access per tile
    for (int k = F; k < K; k += 4) {
      ftile(k, std::integral_constant<int, F>{}, k + 2);
      if (k + 2 >= K) break;
      ftile(k + 2, std::integral_constant<int, F + 2>{}, k + 4);
    }
  } else if (V6_UNROLL && V6_NSLOT == 3) {
    constexpr int S0 = F % 3, S1 = (F + 2) % 3, S2 = (F + 1) % 3;  // tiles k = F + 2m visit these slots
    for (int k = F; k < K; k += 6) {
      ftile(k, std::integral_constant<int, S0>{}, k + 2);
      if (k + 2 >= K) break;
      ftile(k + 2, std::integral_constant<int, S1>{}, k + 4);
      if (k + 4 >= K) break;
      ftile(k + 4, std::integral_constant<int, S2>{}, k + 6);
    }
  } else {
    for (int k = F; k < K; k += 2) ftile(k, k % V6_NSLOT, k + 2);
  }
}

// backward wave of hidden half RHO: every tile of the unit's stream.  V6_BPRE: every LDS read of the
// tile (dZ2 A fragments, H / dZ2 / X transposes, W2ᵀ fragments: ~96 VGPRs) is issued at once right
// after FULL, the slot is released as soon as they have landed, and the 26 MFMAs then run from
// registers (B1, then dW2 + db2 while B1's results drain, the relu mask, dW1ᵀ).
template <int RHO>
EM_DEVICE void v6_backward(char* smem, int B, int unit, int lane, f32x16 (&dW2)[2][2], f32x16 (&dW1T)[2][2],
                           f32x16& db2, float& loss_acc, bool& ok, V4Stamps& st) {
  const int r = lane & 31, h = lane >> 5;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;
  const int nunits = gridDim.x * 2, U = v6_unit_id(unit);
  const int K = v6_ntiles_of_unit(B, U, nunits);
  const uint32_t FL = V6_FLAGS + unit * 64;
  const uint32_t MYDONE = FL + ((1 + RHO) * V6_NSLOT) * 4;
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  auto acc_mfma = [&](f32x16& d, bf16x8 x, bf16x8 y) {
    if (V6_AGPR) mfma_acc_agpr(d, x, y);
    else d = mfma32(x, y, d);
  };
  if (V6_NSLOT > V6_RSLOTS) __syncthreads();  // matches the forward waves' barrier (recycled images)
  st.start();
  for (int k = 0; k < K; ++k) {
    const int slot = k % V6_NSLOT;
    const uint32_t SB = v6_slot(unit, slot), D2 = SB + V6_SD2, HB = SB + V6_SH + RHO * 4096;
    v6_wait(smem, FL + slot * 4, k + 1, ok);
    st.mark(5);

    // dZ2 as B1's A operand (samples x outputs): F's own 8-byte granules, k-step (u, q)
    if (V6_DYN && RHO == 0) loss_acc += reinterpret_cast<const float*>(smem + V6_LOSSR)[(unit * V6_NSLOT + slot) * 64 + lane];
    if (V6_BPRIO) __builtin_amdgcn_s_setprio(2);
    bf16x8 dzA[2][2], hR[2][2], bd[2][2], bx[2][2], w2q[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + v4_img<true>(D2, r, 32 * u + 16 * q + 4 * h));
        const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + v4_img<true>(D2, r, 32 * u + 16 * q + 8 + 4 * h));
        dzA[u][q] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
      }
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int q = 0; q < 2; ++q) hR[tt][q] = v4_tr_frag<true>(smem, HB, 32 * tt, q, h, q4, p4, g1);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) w2q[tt][kk] = lds_frag(smem, w2q_off(32 * (2 * RHO + tt) + r, kk * 2 + h));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) bd[u][q] = v4_tr_frag<true>(smem, D2, 32 * u, q, h, q4, p4, g1);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (V6_XMASK) {
          // X[sample perm(q,h,j)][feature 32u + r] from the tile's masks: the 8 samples of the k-step are
          // two runs of 4 (16q + 4h + 0..3, 16q + 8 + 4h + 0..3), read as 4 broadcast 16-B loads
          const u32x4* MK = reinterpret_cast<const u32x4*>(smem + SB + V6_SX);
          const u32x4 mA = MK[8 * q + 2 * h], mB = MK[8 * q + 2 * h + 1], mC = MK[8 * q + 4 + 2 * h],
                      mD = MK[8 * q + 4 + 2 * h + 1];
          const uint32_t w[8] = {mA[u], mA[2 + u], mB[u], mB[2 + u], mC[u], mC[2 + u], mD[u], mD[2 + u]};
          u32x4 d;
#pragma unroll
          for (int p = 0; p < 4; ++p)
            d[p] = ((uint32_t)__builtin_amdgcn_sbfe(w[2 * p], r, 1) & 0x3F80u) |
                   ((uint32_t)__builtin_amdgcn_sbfe(w[2 * p + 1], r, 1) & 0x3F800000u);
          bx[u][q] = __builtin_bit_cast(bf16x8, d);
        } else {
          bx[u][q] = v4_tr_frag<false>(smem, SB + V6_SX, 32 * u, q, h, q4, p4, g1);
        }
      }
    if (V6_BPRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (V6_BPRE) v6_signal(smem, MYDONE + slot * 4, k + 1);  // DONE: the release waits for every read above
    st.mark(6);

    // B1: dH = dZ2·W2ᵀ for the own hidden half
    f32x16 aD[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) aD[tt] = mfma32(dzA[kk >> 1][kk & 1], w2q[tt][kk], aD[tt]);
    // dW2[own hid][out] += Hᵀ·dZ2 ; db2[out tile RHO] += ones·dZ2 (independent of B1: fills the pipe)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc_mfma(dW2[tt][u], hR[tt][q], bd[u][q]);
        if (u == RHO) {
          if (V6_DB2DOT) {  // lane (r, h): 8 samples of output 32 RHO + r; the h halves are summed at the end
            // (memcpy casts: a bit_cast of an ext_vector element in an unrolled loop reads element 0, see as_s16x2)
            bf16x2_t b2v[4];
            __builtin_memcpy(b2v, &bd[u][q], 16);
            const bf16x2_t one2 = __builtin_bit_cast(bf16x2_t, 0x3F803F80u);
#pragma unroll
            for (int e = 0; e < 4; ++e) db2[0] = __builtin_amdgcn_fdot2_f32_bf16(b2v[e], one2, db2[0], false);
          } else {
            db2 = mfma32(ones, bd[u][q], db2);
          }
        }
      }
    st.mark(7);
    // dZ1 = dH * (H > 0), then dW1ᵀ[own hid][feat] += dZ1ᵀ·X
    bf16x8 dz1[2][2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int q = 0; q < 2; ++q) dz1[tt][q] = mask_by(hR[tt][q], aD[tt], q);
    if (!V6_BPRE) v6_signal(smem, MYDONE + slot * 4, k + 1);
    st.mark(8);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc_mfma(dW1T[tt][u], dz1[tt][q], bx[u][q]);
    st.mark(9);
  }
}

// f32x4 slot of accumulator group g of tile T, lane (L, h) in the epilogue's fold image.  The dW1ᵀ tiles
// XOR the lane slot with the slab writer's lane bits (hidden tile parity, g, h): the writer's 16-lane
// groups read 16 distinct (T, g, h) at one L, which without the swizzle all land on one 16-B bank group
// (a 16-way conflict per read, ~2 us of the epilogue); the B waves' 8-lane store groups stay conflict-free.
EM_DEVICE int v6_red_slot(int T, int g, int L, int h) {
  const int sw = T >= 8 ? ((((T - 8) >> 1) & 1) << 3) | (g << 1) | h : 0;
  return (T * 4 + g) * 64 + h * 32 + (L ^ sw);
}

// one role's loop + its share of the epilogue (the same two barriers in every role instantiation)
template <int LOSS, int ROLE>  // ROLE 0/1 = forward f, 2/3 = backward rho
EM_DEVICE void v6_body(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                       int offset, int unit, int wave, int lane, float* slab_spare) {
  const int r = lane & 31, h = lane >> 5;
  bool ok = true;
  V4Stamps st;
  float* RED = reinterpret_cast<float*>(smem);  // [unit][16 tiles][4 g][64 lanes][4]: 0..7 dW2, 8..15 dW1T
  float* DB2S = reinterpret_cast<float*>(smem + V6_RED);          // [2 units][64]
  float* LOSSS = reinterpret_cast<float*>(smem + V6_RED + 512);   // [8]
  auto dump = [&]() {
    if (V4_STAMPS && lane < 10) {  // phase cycles of this wave -> spare slab floats
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 10; ++k) v = (lane == k) ? st.acc[k] : v;
      slab_spare[wave * 16 + lane] = (float)v;
    }
  };
  if (ROLE < 2) {
    float loss_acc = 0.f;
    if (V6_FPRIO) __builtin_amdgcn_s_setprio(1);
    v6_forward<LOSS, ROLE>(smem, masks, sidx, B, offset, unit, lane, loss_acc, ok, st);
    float lsum = wave_sum(loss_acc);
    if (!ok) lsum = __builtin_nanf("");
    dump();
    __syncthreads();  // every wave is out of the loop: the loop's LDS is free
    if (lane == 0) LOSSS[wave] = lsum;
    __syncthreads();
  } else {
    constexpr int RHO = ROLE - 2;
    f32x16 dW2[2][2], dW1T[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        dW2[t][u] = f32x16{};
        dW1T[t][u] = f32x16{};
      }
    f32x16 db2 = f32x16{};
    float loss_acc = 0.f;
    v6_backward<RHO>(smem, B, unit, lane, dW2, dW1T, db2, loss_acc, ok, st);
    const float lsum = wave_sum(loss_acc);
    asm volatile("s_nop 15\n\ts_nop 7" ::: "memory");  // asm MFMA (AGPR D) -> v_accvgpr_read hazard
    dump();
    __syncthreads();
    if (V6_DB2DOT) db2[0] = xhalf_sum(db2[0]);           // the two sample halves of output 32 RHO + r
    if (h == 0) DB2S[unit * 64 + 32 * RHO + r] = db2[0];  // accumulator column r = output 32 RHO + r
    if (lane == 0) LOSSS[wave] = ok ? lsum : __builtin_nanf("");
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int which = 0; which < 2; ++which) {
          const f32x16& acc = which ? dW1T[tt][u] : dW2[tt][u];
          const int T = 8 * which + 2 * (2 * RHO + tt) + u;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(RED + unit * 16384 + v6_red_slot(T, g, r, h) * 4) =
                f32x4{acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
        }
    __syncthreads();
  }
}

template <int LOSS>
__global__ void __launch_bounds__(512, 1)
mlp_fused_train_v6_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                          const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                          float* __restrict__ loss_slabs, int* __restrict__ step) {
  advance_step(step);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  {  // all loads of the weight image in flight before the first LDS store
    constexpr int N16 = IMG_BYTES / 16, KK = (N16 + 511) / 512;
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    u32x4 v[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k)
      if (tid + 512 * k < N16) v[k] = src[tid + 512 * k];
#pragma unroll
    for (int k = 0; k < KK; ++k)
      if (tid + 512 * k < N16) dst[tid + 512 * k] = v[k];
  }
  if (tid < 64) reinterpret_cast<float*>(smem + V6_YLUT)[tid] = (float)(((tid >> 2) >> (tid & 3)) & 1);
  if (tid < 32) {
    const uint32_t n = (uint32_t)tid >> 1, b = 2u * (tid & 1);
    reinterpret_cast<uint32_t*>(smem + V6_XLUT)[tid] =
        (((n >> b) & 1u) ? 0x3F80u : 0u) | (((n >> (b + 1)) & 1u) ? 0x3F800000u : 0u);
  }
  if (tid < 32) reinterpret_cast<int*>(smem + V6_FLAGS)[tid] = 0;
  __syncthreads();
  // wave w runs on SIMD w % 4.  unit 0 = waves 0-3 (F0 F1 B0 B1), unit 1 = waves 4-7 (B0 B1 F0 F1):
  // every SIMD hosts one forward and one backward wave
  uint64_t ts[4] = {};  // V4_STAMPS: 100 MHz wall-clock marks (entry, prologue done, loop done, dW folded)
  if (V4_STAMPS) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int unit = wave >> 2, wl = wave & 3;
  // V6_SEG: both units use the same map, so SIMDs 0/1 host two forward waves and SIMDs 2/3 two backward
  // waves (forward chains never share a matrix pipe with backward dW streams)
  const int role = (unit == 0 || V6_SEG) ? wl : (wl ^ 2);  // 0/1 forward f, 2/3 backward rho
  float* slab_spare = slabs + (size_t)blockIdx.x * SLAB_STRIDE + P_TOTAL;  // 192 spare floats per slab
  if (V4_STAMPS) ts[1] = __builtin_amdgcn_s_memrealtime();
  if (role == 0)
    v6_body<LOSS, 0>(smem, masks, sidx, B, offset, unit, wave, lane, slab_spare);
  else if (role == 1)
    v6_body<LOSS, 1>(smem, masks, sidx, B, offset, unit, wave, lane, slab_spare);
  else if (role == 2)
    v6_body<LOSS, 2>(smem, masks, sidx, B, offset, unit, wave, lane, slab_spare);
  else
    v6_body<LOSS, 3>(smem, masks, sidx, B, offset, unit, wave, lane, slab_spare);
  if (V4_STAMPS) ts[2] = __builtin_amdgcn_s_memrealtime();

  const float* RED = reinterpret_cast<const float*>(smem);
  const float* DB2S = reinterpret_cast<const float*>(smem + V6_RED);
  const float* LOSSS = reinterpret_cast<const float*>(smem + V6_RED + 512);
  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  // parameter-order slab with 16-B write-through (sc1) stores (see the v4 epilogue)
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(slab, 0, SLAB_STRIDE * 4, 0x00020000);
  for (int e = tid; e < 2048; e += 512) {  // W1[f][c..c+3]: one 16-B store per f32x4 of a dW1ᵀ tile
    const int f = e >> 5, c = (e & 31) * 4;
    const int T = 8 + 2 * (c >> 5) + (f >> 5), g = (c & 31) >> 3;
    const int at = v6_red_slot(T, g, f & 31, (c >> 2) & 1) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(RED + at) + *reinterpret_cast<const f32x4*>(RED + 16384 + at);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), srd, e * 16, 0, 16 /* sc1 */);
  }
  for (int q = tid; q < 2048; q += 512) {  // dW2 tiles read in slot order; W2[c + k][o] as 4 coalesced scalars
    const int T = q >> 8, g = (q >> 6) & 3, L = q & 31, hh = (q >> 5) & 1;
    const f32x4 v = *reinterpret_cast<const f32x4*>(RED + q * 4) + *reinterpret_cast<const f32x4*>(RED + 16384 + q * 4);
    const int c = 32 * (T >> 1) + 8 * g + 4 * hh, o = 32 * (T & 1) + L;
    uint32_t vb[4];  // memcpy, not a bit_cast of v[k]: see as_s16x2
    __builtin_memcpy(vb, &v, 16);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_buffer_store_b32(vb[k], srd, (P_W2 + (c + k) * OUT + o) * 4, 0, 16 /* sc1 */);
  }
  if (V4_STAMPS && tid == 0) {
    ts[3] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 4; ++k) slab_spare[128 + k] = __builtin_bit_cast(float, (uint32_t)ts[k]);
  }
  if (tid < 64) slab[P_B2 + tid] = DB2S[tid] + DB2S[64 + tid];
  if (tid == 0) {
    float l = 0.f;
    for (int w = 0; w < 8; ++w) l += LOSSS[w];
    loss_slabs[blockIdx.x] = l;
  }
}

// Forward only: logits [B, 64] fp32 (cols 62/63 padding).  F1+F2 of the train kernel.
__global__ void __launch_bounds__(256)
mlp_fused_forward_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                         int offset, const uint8_t* __restrict__ wimg, float* __restrict__ logits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  {
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    for (int i = tid; i < IMG_BYTES / 16; i += 256) dst[i] = src[i];
  }
  const char* lut = smem + IMG_BYTES;
  fill_lut(smem + IMG_BYTES, tid);
  __syncthreads();
  const int ntiles = (B + 31) / 32;
  const int nwaves = gridDim.x * 4;
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += nwaves) {
    const int s = tile * 32 + r;
    const bool valid = s < B;
    const uint64_t imask = valid ? (masks[sidx ? sidx[s] : (offset + s)] | BIAS_BIT) : 0ull;
    bf16x8 xf[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xf[q] = lut_frag(lut, imask, q, h);
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
          *reinterpret_cast<f32x4*>(logits + (int64_t)s * OUT + 32 * u + 8 * g + 4 * h) = v;
        }
      }
    }
  }
}

}  // namespace

EM_API int em_mlp_fused_param_count() { return P_TOTAL; }
EM_API int em_mlp_fused_slab_stride() { return SLAB_STRIDE; }
EM_API int em_mlp_fused_image_bytes() { return IMG_BYTES; }
EM_API int em_mlp_fused_lds_bytes() { return TRAIN_LDS; }

// Which train kernel em_mlp_fused_train launches: 6 (default: producer/consumer units), 4 (hidden-split
// pairs), 5 (round-synchronous, experimental) or 3 (one wave per SIMD).  The first call reads
// EM_FUSED_KERNEL (or the older EM_FUSED_V3 / EM_FUSED_V5 / EM_FUSED_V6 flags); em_mlp_fused_select_kernel
// overrides it at run time (tests cover every version in one process).
static int g_fused_kernel = -1;
static int fused_kernel_version() {
  if (g_fused_kernel < 0) {
    int v = 6;
    const char* e = std::getenv("EM_FUSED_KERNEL");
    const char* e3 = std::getenv("EM_FUSED_V3");
    const char* e5 = std::getenv("EM_FUSED_V5");
    const char* e6 = std::getenv("EM_FUSED_V6");
    if (e6 && e6[0] == '0') v = 4;
    if (e5 && e5[0] == '1') v = 5;
    if (e3 && e3[0] == '1') v = 3;
    if (e && (e[0] == '3' || e[0] == '4' || e[0] == '5' || e[0] == '6') && e[1] == 0) v = e[0] - '0';
    g_fused_kernel = v;
  }
  return g_fused_kernel;
}
EM_API int em_mlp_fused_select_kernel(int version) {  // returns the previous version; -1 = back to the env default
  const int prev = fused_kernel_version();
  if (version == -1 || version == 3 || version == 4 || version == 5 || version == 6) g_fused_kernel = version;
  else return EM_ERR_ARG;
  return prev;
}

// masks: [ndraws] uint64 feature masks; sample s = (masks[i], masks[i+1]) with i = sidx ? sidx[s] : offset+s
EM_API int em_mlp_fused_train(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                              const void* wimg, float* slabs, float* loss_slabs, int nslab, int loss_kind,
                              int* step, hipStream_t stream) {
  if (draws && !sidx && offset > 0) {  // sequential samples: 64-bit offsets (HBM-filling datasets) via the base
    draws += offset;
    offset = 0;
  }
  if (!draws || !wimg || !slabs || !loss_slabs || nslab <= 0 || B < 0 || offset < 0 ||
      B + offset + 1 > (int64_t)INT32_MAX)
    return EM_ERR_ARG;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              TRAIN_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              TRAIN_LDS);
    attr_set = true;
  }
  static bool attrs = false;
  if (!attrs) {
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v4_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V4_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v4_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V4_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v5_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V5_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v5_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V5_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v6_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V6_LDS);
    (void)hipFuncSetAttribute((const void*)mlp_fused_train_v6_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              V6_LDS);
    attrs = true;
  }
  const int ver = fused_kernel_version();
  const dim3 grid(nslab);
  const int Bi = (int)B, oi = (int)offset;
  const uint8_t* w = (const uint8_t*)wimg;
  if (ver == 6) {
    if (loss_kind == 0)
      hipLaunchKernelGGL(mlp_fused_train_v6_kernel<0>, grid, dim3(512), V6_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
    else
      hipLaunchKernelGGL(mlp_fused_train_v6_kernel<1>, grid, dim3(512), V6_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
  } else if (ver == 5) {
    if (loss_kind == 0)
      hipLaunchKernelGGL(mlp_fused_train_v5_kernel<0>, grid, dim3(512), V5_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
    else
      hipLaunchKernelGGL(mlp_fused_train_v5_kernel<1>, grid, dim3(512), V5_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
  } else if (ver == 4) {
    if (loss_kind == 0)
      hipLaunchKernelGGL(mlp_fused_train_v4_kernel<0>, grid, dim3(512), V4_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
    else
      hipLaunchKernelGGL(mlp_fused_train_v4_kernel<1>, grid, dim3(512), V4_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
  } else if (loss_kind == 0) {
    hipLaunchKernelGGL(mlp_fused_train_kernel<0>, grid, dim3(256), TRAIN_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
  } else {
    hipLaunchKernelGGL(mlp_fused_train_kernel<1>, grid, dim3(256), TRAIN_LDS, stream, draws, sidx, Bi, oi, w, slabs, loss_slabs, step);
  }
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_mlp_fused_forward(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                                const void* wimg, float* logits, int nblocks, hipStream_t stream) {
  if (draws && !sidx && offset > 0) {
    draws += offset;
    offset = 0;
  }
  if (!draws || !wimg || !logits || nblocks <= 0 || B < 0 || offset < 0 || B + offset > (int64_t)INT32_MAX)
    return EM_ERR_ARG;
  hipLaunchKernelGGL(mlp_fused_forward_kernel, dim3(nblocks), dim3(256), IMG_BYTES + LUT_BYTES, stream, draws, sidx,
                     (int)B, (int)offset,
                     (const uint8_t*)wimg, logits);
  EM_CHECK_LAUNCH();
  return 0;
}
