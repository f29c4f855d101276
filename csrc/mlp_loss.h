// Per-tile loss kernels shared by the fused small-MLP train kernels (csrc/mlp_fused.hip: bf16 v6,
// csrc/mlp_fused_f32.hip: exact fp32).  Both hold a 32-sample tile's logits in the 32x32 MFMA
// accumulator layout: lane (r, h) = sample r, register i of output tile u = output 32u + oo0(i) + 4h.
#pragma once
#include "common.h"
#include "mlp_adam.h"

// o(u,i,h) = 32u + (i&3) + 8(i>>2) + 4h : output index held in register i of Z2ᵀ tile u
EM_DEVICE constexpr int oo0(int i) { return (i & 3) + 8 * (i >> 2); }


// class of the output at position o = 32 u + oo0(i) + 4h: 0 main, 1 star, 2 pad.  PERM: positions are
// physical (mlp_adam.h out_phys) -- the pads count as main (their logits are PAD_B2) and no class depends
// on the lane half h.
template <bool PERM = false>
EM_DEVICE constexpr int out_cls(int u, int i, int h) {
  const int o = PERM ? mlp::out_logical(32 * u + oo0(i) + 4 * h) : 32 * u + oo0(i) + 4 * h;
  return o < 50 ? 0 : (o < 62 ? 1 : (PERM ? 0 : 2));
}
static_assert(out_cls<true>(1, 8, 0) == out_cls<true>(1, 8, 1) && out_cls<true>(1, 9, 1) == 0 &&
                  out_cls<true>(1, 10, 0) == 1 && out_cls<true>(1, 10, 1) == 1 && out_cls<true>(1, 12, 1) == 1,
              "PERM: one class per register");

// the target mask in physical output order (PERM): logical bits 52-59 -> 56-63, 60/61 -> 54/55; the pad
// bits 62/63 (-> 52/53) are zero in every target
EM_DEVICE uint64_t phys_targets(uint64_t t) {
  const uint32_t hi = (uint32_t)(t >> 32);
  const uint32_t ph = (hi & 0x000FFFFFu) | ((hi & 0x0FF00000u) << 4) | ((hi >> 6) & 0x00C00000u);
  return ((uint64_t)ph << 32) | (uint32_t)t;
}

// Sigmoid-BCE loss + dZ2 of a whole 32-sample tile in ONE wave: the lane's 32 logits z2[u][i] (output
// 32u + oo0(i) + 4h of sample r; lanes r and r + 32 share the sample).  Targets as {0,1} floats from
// a 16-entry nibble table (YL): register group g of tile u holds outputs 32u + 8g + 4h .. +3 = one
// nibble of the target mask.
template <int YL, bool PERM = false>
EM_DEVICE void bce_tile_loss(const char* smem, const f32x16 (&z2)[2], uint64_t tmask, bool valid, int h,
                             float (&dz)[2][16], float& loss_acc) {
  if (PERM) tmask = phys_targets(tmask);
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  float l = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float yb[16];
    const uint32_t tmh = (uint32_t)(tmask >> (32 * u)) >> (4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + lut_off<YL, 4>(tmh, 8 * g));
      yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = out_cls<PERM>(u, i, h);
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

// Grouped softmax-CE of a whole tile in ONE wave (v6 forward), main-group statistics split per
// output tile and merged online (flash-softmax style): tile 0's max / exp / sums need only Z2 tile
// 0, so they run on the VALU while tile 1's F2 chain is still in the matrix pipe (the caller's hook
// issues step(j) between tile 1's MFMAs; in-order issue overlaps only VALU that sits between MFMAs
// in program order).  dZ2 of tile u carries its tile's rescale a_u = exp(m_u - M).
// The class of the lane's element i of output tile u (main / star / pad) is a compile-time
// constant except for 4 elements of tile 1 whose class depends on the lane half h (outputs 48-51
// and 58-63 straddle the group edges), so every statically classified element emits only its own
// group's ops (a select-form "x ? v : 0" fed into an fma would have to be kept: fma(0, inf, a) is
// NaN).  Max / sum / target-dot reductions run as independent partial chains.
// Packed fp32 pairs: the accumulator registers (i, i + 1), i even, are an aligned VGPR pair, so the
// exp argument, the exp sums and the target dot of two outputs issue as ONE v_pk_fma_f32 / v_pk_add_f32
// (full rate on the 2-wide packed path).  Elements (i, i + 1) of a tile share their class for both h
// (out_cls), except where noted below.  38 fewer VALU per forward tile (494 -> 456); the same-box A/B
// was within noise (89.4 vs 89.5 us, profiles/r3/ab_packed_softmax.jsonl): the forward wave's tile is
// bound by its dependency chain, not by issue.
typedef float f32x2 __attribute__((ext_vector_type(2)));
EM_DEVICE f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int YL, bool PERM = false, typename Hook>
EM_DEVICE void v6_softmax_split(const char* smem, const f32x16 (&z2)[2], uint64_t tmask, int h, float (&dz)[2][16],
                                float& loss_acc, Hook&& hook) {
  if (PERM) tmask = phys_targets(tmask);
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  const f32x2 L2E2 = {L2E, L2E};
  auto targets = [&](int u, float (&yb)[16]) {
    const uint32_t tmh = (uint32_t)(tmask >> (32 * u)) >> (4 * h);
    // SDWA form (table at 256, the K7 windowed layout): byte g of sp = nibble 8g + 16, so one byte-select
    // shift per lookup gives 256 + 16 nib -- 5 VALU per word instead of 8
    constexpr bool SD = YL == 256 && PERM;
    const uint32_t sp = (tmh & 0x0F0F0F0Fu) | 0x10101010u;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint32_t off;
      if constexpr (SD) {
        off = g == 0 ? sdwa_byte_shl<0, 4>(sp) : g == 1 ? sdwa_byte_shl<1, 4>(sp) : g == 2 ? sdwa_byte_shl<2, 4>(sp)
                                                                                          : sdwa_byte_shl<3, 4>(sp);
      } else {
        off = lut_off<YL, 4>(tmh, 8 * g);
      }
      const f32x4 y4 = *reinterpret_cast<const f32x4*>(smem + off);
      yb[4 * g + 0] = y4[0]; yb[4 * g + 1] = y4[1]; yb[4 * g + 2] = y4[2]; yb[4 * g + 3] = y4[3];
    }
  };
  auto zpair = [&](int u, int i) { return f32x2{z2[u][i], z2[u][i + 1]}; };
  auto exp2 = [](f32x2 t) { return f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)}; };
  const bool h0 = h == 0;
  const uint32_t tlo = (uint32_t)tmask, thi = (uint32_t)(tmask >> 32);
  const int nm = __builtin_popcount(tlo) + __builtin_popcount(thi & 0x3FFFFu);  // bits 0..49
  const int ns = __builtin_popcount(thi & (PERM ? 0xFFFC0000u : 0x3FFC0000u));   // bits 50..61 (PERM: 50..63)
  const float inv_m = nm ? __builtin_amdgcn_rcpf((float)nm) : 0.f;
  const float inv_s = ns ? __builtin_amdgcn_rcpf((float)ns) : 0.f;
  // target dots: tm[q] holds elements with (i & 3) >> 1 == q (x: even i, y: odd i), ts by i & 1
  f32x2 tm[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}}, ts = {0.f, 0.f};
  // ---- tile 0: outputs 0..31, all main.  step(j), j = 0..7, is issued between tile 1's F2 MFMAs by
  // the caller (hook): in-order issue lets the VALU run only between MFMAs in program order ----
  float m0 = 0.f, s0 = 0.f;
  f32x2 nL2 = {0.f, 0.f};
  float mm0[4], yb0[16];
  f32x2 sm[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
  // PERM (the bf16 train kernels): max trees of v_max3_f32 without canonicalisation (raw_max3): 8
  // instructions per 16 logits instead of ~15
  const auto& z0 = z2[0];
  auto step = [&](int j) {
    if (j == 0) {
      if (PERM) {
        mm0[0] = raw_max3(raw_max3(z0[0], z0[1], z0[2]), raw_max3(z0[3], z0[4], z0[5]), raw_max3(z0[6], z0[7], z0[8]));
        mm0[1] = raw_max3(raw_max3(z0[9], z0[10], z0[11]), raw_max3(z0[12], z0[13], z0[14]), z0[15]);
      } else {
        mm0[0] = z2[0][0]; mm0[1] = z2[0][1]; mm0[2] = z2[0][2]; mm0[3] = z2[0][3];
#pragma unroll
        for (int i = 4; i < 16; ++i) mm0[i & 3] = fmaxf(mm0[i & 3], z2[0][i]);
      }
      targets(0, yb0);
    } else if (j == 1) {
      m0 = PERM ? xhalf_max_raw(raw_max(mm0[0], mm0[1]))
                : xhalf_max(fmaxf(fmaxf(mm0[0], mm0[1]), fmaxf(mm0[2], mm0[3])));
      nL2 = f32x2{-m0 * L2E, -m0 * L2E};
    } else if (j < 6) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 4 * (j - 2) + 2 * q;
        const f32x2 zz = zpair(0, i);
        const f32x2 e = exp2(pfma(zz, L2E2, nL2));
        sm[q] += e;
        tm[q] = pfma(f32x2{yb0[i], yb0[i + 1]}, zz, tm[q]);
        dz[0][i] = e.x;
        dz[0][i + 1] = e.y;
      }
    } else if (j == 6) {
      s0 = xhalf_sum((sm[0].x + sm[0].y) + (sm[1].x + sm[1].y));
    }
  };
  hook(step);
  // ---- tile 1: outputs 32..63 (main 32..49, star 50..61, pad 62/63) ----
  float mm[2] = {-3.0e38f, -3.0e38f}, ms[2] = {-3.0e38f, -3.0e38f};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c0 = out_cls<PERM>(1, i, 0), c1 = out_cls<PERM>(1, i, 1);
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
  float m1, mx_s;
  if (PERM) {  // main: registers 0-9, star: 10-15 (out_cls<true>)
    const auto& z = z2[1];
    static_assert(out_cls<PERM>(1, 9, 0) == 0 && out_cls<PERM>(1, 10, 0) == 1, "PERM tile-1 classes");
    const float a = raw_max3(raw_max3(z[0], z[1], z[2]), raw_max3(z[3], z[4], z[5]), raw_max3(z[6], z[7], z[8]));
    m1 = xhalf_max_raw(raw_max(a, z[9]));
    mx_s = xhalf_max_raw(raw_max(raw_max3(z[10], z[11], z[12]), raw_max3(z[13], z[14], z[15])));
  } else {
    m1 = xhalf_max(fmaxf(mm[0], mm[1]));
    mx_s = xhalf_max(fmaxf(ms[0], ms[1]));
  }
  const float nmL = -m1 * L2E, nsL = -mx_s * L2E;
  const f32x2 nmL2 = {nmL, nmL}, nsL2 = {nsL, nsL};
  f32x2 s1p = {0.f, 0.f}, ss = {0.f, 0.f};
  float yb1[16];
  targets(1, yb1);
  {
    float (&yb)[16] = yb1;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const int c0 = out_cls<PERM>(1, i, 0), c1 = out_cls<PERM>(1, i, 1);
      static_assert(out_cls<PERM>(1, 9, 0) == out_cls<PERM>(1, 8, 0) && out_cls<PERM>(1, 15, 1) == out_cls<PERM>(1, 14, 1) &&
                        out_cls<PERM>(1, 11, 0) == out_cls<PERM>(1, 10, 0),
                    "pair classes");
      const f32x2 zz = zpair(1, i), yy = {yb[i], yb[i + 1]};
      f32x2 e;
      if (c0 == c1 && c0 == 0) {
        e = exp2(pfma(zz, L2E2, nmL2));
        s1p += e;
        tm[(i & 3) >> 1] = pfma(yy, zz, tm[(i & 3) >> 1]);
      } else if (c0 == c1 && c0 == 1) {
        e = exp2(pfma(zz, L2E2, nsL2));
        ss += e;
        ts = pfma(yy, zz, ts);
      } else if (c0 == 0) {  // main (h = 0) / star (h = 1): outputs 48/49 | 52/53
        e = exp2(pfma(zz, L2E2, h0 ? nmL2 : nsL2));
        const f32x2 ty = yy * zz;
        s1p = h0 ? s1p + e : s1p;
        ss = h0 ? ss : ss + e;
        tm[(i & 3) >> 1] = h0 ? tm[(i & 3) >> 1] + ty : tm[(i & 3) >> 1];
        ts = h0 ? ts : ts + ty;
      } else {  // star (h = 0) / pad (h = 1): outputs 58/59 | 62/63
        const f32x2 ex = exp2(pfma(zz, L2E2, nsL2));
        e = h0 ? ex : f32x2{0.f, 0.f};
        ss += e;
        ts = h0 ? pfma(yy, zz, ts) : ts;
      }
      dz[1][i] = e.x;
      dz[1][i + 1] = e.y;
    }
  }
  const float s1 = xhalf_sum(s1p.x + s1p.y), s_s = xhalf_sum(ss.x + ss.y);
  // ---- online merge of the main group: M = max(m0, m1), S = a0 s0 + a1 s1 ----
  const float M = PERM ? raw_max(m0, m1) : fmaxf(m0, m1);
  const float a0 = __builtin_amdgcn_exp2f((m0 - M) * L2E), a1 = __builtin_amdgcn_exp2f((m1 - M) * L2E);
  const float S = __builtin_fmaf(a0, s0, a1 * s1);
  const float rS = nm ? __builtin_amdgcn_rcpf(S) : 0.f;
  const float f0 = a0 * rS, f1 = a1 * rS, f_s = ns ? __builtin_amdgcn_rcpf(s_s) : 0.f;
  const float ni_m = -inv_m, ni_s = -inv_s;
  // (written per element: the compiler pairs these into v_pk_mul_f32 + v_pk_fma_f32 by itself, and the
  // explicit f32x2 form compiled to 8 more VALU)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float (&yb)[16] = u == 0 ? yb0 : yb1;  // the targets, read once per tile
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c0 = out_cls<PERM>(u, i, 0), c1 = out_cls<PERM>(u, i, 1);
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
  float l = -(((tm[0].x + tm[0].y) + (tm[1].x + tm[1].y)) * inv_m + (ts.x + ts.y) * inv_s);
  if (h == 0)
    l += (nm ? M + __builtin_amdgcn_logf(S) * LN2 : 0.f) + (ns ? mx_s + __builtin_amdgcn_logf(s_s) * LN2 : 0.f);
  loss_acc += l;
}
