// K7 -- fused persistent small-MLP training step for MI355X (gfx950).
// EM_BUILD_FLAGS: -mllvm -amdgpu-mfma-vgpr-form=1 -mllvm -amdgpu-use-amdgpu-trackers -mllvm -amdgpu-schedule-metric-bias=0 -mllvm -amdgpu-sched-strategy=max-memory-clause
// (VGPR-form MFMAs give every wave 256 arch VGPRs; the register-pressure trackers and a latency-first
// schedule remove the default build's 2 spilled dwords: +0.35 % and +0.6 % in same-box A/Bs,
// profiles/r3/ab_sched_fused*.jsonl.  The max-memory-clause scheduling strategy (round 5): 87.1 -> 86.7 us
// per 1M-sample step over 6 interleaved rounds, bit-identical parameters; max-ilp 90.6 us, rejected --
// profiles/r5/ab_sched_strategy_headline.jsonl)
//
// Model (BASELINE.json config 2): multi-hot 62-wide draw
// vector -> Linear(62,128) -> ReLU -> Linear(128,62) -> grouped softmax-CE
// (50 main numbers / 12 lucky stars) or sigmoid-BCE.  The reference declares
// DL4J for this (pom.xml:62-66) but never calls it; its only learner is
// XGBoost (Main.java:113-138), reproduced separately in gbdt.hip.
//
// One launch computes the forward, the loss, the backward and the per-workgroup
// weight-gradient partial sums for a whole mini-batch (design: docs/DESIGN.md §2):
//   * 1 workgroup (8 waves) per CU, persistent over 32-sample tiles; two producer/consumer
//     units per workgroup (forward waves -> LDS ring -> backward waves), see "producer/consumer
//     units" below.
//   * Weights arrive as bf16 images laid out so that every weight fragment is one conflict-free
//     ds_read_b128 (packed by em_adam_pack / the Adam epilogue); the forward waves keep theirs in
//     registers for the whole launch.
//   * Samples are 8-byte draw masks (input draw t, target draw t+1).  The multi-hot X tile is
//     never materialised in HBM: each lane builds its MFMA fragments from a 64-bit feature mask
//     (bit 62 = constant-1 bias feature, so b1 is row 62 of W1 and its gradient falls out of dW1).
//   * Orientation is chosen so products chain accumulator->operand without LDS
//     (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand"):
//        F1  Z1ᵀ = W1ᵀ·Xᵀ         (samples on lanes)   -> relu -> Hᵀ (B operand)
//        F2  Z2ᵀ = W2ᵀ·Hᵀ + b2                         -> loss, dZ2ᵀ
//        B1  dH  = dZ2·W2ᵀ        (dZ2 granules read back as the A operand)
//        dW2 += Hᵀ·dZ2   dW1ᵀ += dZ1ᵀ·X   (K = samples: the operands whose sample axis sits on
//        lanes go through LDS images and come back with ds_read_b64_tr_b16)
//   * Every workgroup writes ONE fp32 gradient slab (fixed summation order: bit-reproducible).
//
// Generations v3 (one wave per SIMD), v4 (hidden-split wave pairs) and v5 (round-synchronous
// dW GEMMs) were measured slower than v6 and removed (git history: csrc/mlp_fused.hip before
// round 3; docs/DESIGN.md §6 keeps their numbers).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "mlp_adam.h"
#include "mlp_loss.h"

namespace {
using mlp::IN, mlp::HID, mlp::OUT, mlp::P_W1, mlp::P_W2, mlp::P_B2, mlp::P_TOTAL;
using mlp::W1T_RS, mlp::W2P_RS, mlp::W2Q_RS, mlp::IMG_W1T, mlp::IMG_W2P, mlp::IMG_W2Q, mlp::IMG_B2, mlp::IMG_BYTES;
// gradient slabs are SLAB_STRIDE floats apart (P_TOTAL rounded to an odd multiple of 256 B so the
// cross-slab reduction in em_adam_slab does not hit the same HBM channel for every slab)
constexpr int SLAB_STRIDE = 16640;
// weight images (mlp_adam.h): padded rows instead of an XOR swizzle, so a fragment address is one
// per-lane base + an immediate, not one VGPR per (row, chunk) pair

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
EM_DEVICE uint32_t w2q_off(int row, int k8) { return IMG_W2Q + row * W2Q_RS + (k8 ^ mlp::w2q_swz(row)) * 16; }

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
// the same on two 16x16 accumulator quads (the backward wave: k 0-3 from sample tile 0, 4-7 from sample tile 1)
template <class V4>
EM_DEVICE bf16x8 mask_by4(const bf16x8 hfrag, const V4& a0, const V4& a1) {
  const bf16x8 p = pack8(a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]);
  u32x4 d = __builtin_bit_cast(u32x4, p);
  const u32x4 hh = __builtin_bit_cast(u32x4, hfrag);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t m;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(hh[k]), "s"(0x00010001u));
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(d[k]) : "v"(d[k]), "v"(m));
  }
  return __builtin_bit_cast(bf16x8, d);
}

// ============================================================================================
// LDS protocol helpers (workgroup scope), diagnostic stamps, swizzled tile images
// ============================================================================================
EM_DEVICE void lds_signal(char* smem, uint32_t flag_off, int value) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __hip_atomic_store(reinterpret_cast<int*>(smem + flag_off), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (Round 6 measured the ring counters without the release fence's s_waitcnt lgkmcnt(0) -- LDS performs one
// wave's instructions in issue order -- at 82.6 vs 82.2 µs for the fenced form, profiles/r6/ab_v6_lds_order.jsonl;
// the compiler places the backward waves' DONE among their MFMAs either way.  The fenced lds_signal stays.)

// Diagnostic phase timers (build with --define FUSED_STAMPS=1; tools/fused_phases.py reads them):
// s_memtime deltas summed per phase per wave, written into spare slab floats.  They force an
// lgkmcnt drain at every mark, so they perturb what they measure (+~10 %).
#ifndef FUSED_STAMPS
#define FUSED_STAMPS 0
#endif
// A/B knobs (tools/build_variant.sh; profiles/r3/ab_knobs.jsonl): the ring wait's s_sleep (0 and 3 within
// noise of 1) and the forward waves' priority (0: 8 % slower, 2: same as 1)
#ifndef FUSED_SLEEP
#define FUSED_SLEEP 1
#endif
#ifndef FUSED_FPRIO
#define FUSED_FPRIO 1
#endif
// FUSED_PROBE (diagnostic side builds only: the gradients are WRONG under it; profiles/r6/k7_probes.md)
// prices moving the softmax from the forward to the backward waves before building it.  Bit 1: the
// forward wave's softmax replaced by dZ2 = Z2 / 64 (its VALU gone, F2's latency kept).  Bit 2: every
// backward tile issues FUSED_PROBE_VALU independent VALU (FMA chains + exp2, 1 in 8) on registers of
// its own between its MFMAs, about the share of a split softmax a backward wave would take.
#ifndef FUSED_PROBE
#define FUSED_PROBE 0
#endif
#ifndef FUSED_PROBE_VALU
#define FUSED_PROBE_VALU 128
#endif
struct Stamps {
  uint64_t last = 0;
  uint64_t acc[10] = {};
  EM_DEVICE void start() {
    if (FUSED_STAMPS) last = __builtin_amdgcn_s_memtime();
  }
  EM_DEVICE void mark(int k) {
    if (FUSED_STAMPS) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      acc[k] += t - last;
      last = t;
    }
  }
};

// Per-tile images [32 samples][64 cols] bf16, 128-B rows.  Row r XORs its 16-B chunk index with
// fr(r) and (H, D2 only: G) its 8-B half with gr(r), chosen so that every access of the tile is
// conflict-free under the CDNA4 banking rules (tools/lds_conflicts.py, tests/test_lds_model.py):
// the per-row 8-B writes (16-lane groups, 32 banks) need (fr, gr) injective on rows 0-15, the 8-B
// row reads (32-lane groups, 64 banks) injective on each row parity, and the transposing reads
// (4 rows x 64 B per 32-lane group) need fr's top bit to follow row bit 1.  The X image is written
// in whole 16-B chunks, so it keeps gr = 0.
EM_DEVICE uint32_t img_fr(int r) { return ((r ^ (r >> 4)) & 1) | (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2); }
EM_DEVICE uint32_t img_gr(int r) { return (r >> 3) & 1; }
template <bool G>
EM_DEVICE uint32_t tile_img(uint32_t base, int row, int col) {
  const uint32_t c = (uint32_t)(((col >> 3) ^ img_fr(row)) << 4);
  return base + row * 128 + c + (G ? (((((col >> 2) & 1) ^ img_gr(row)) << 3) + (col & 3) * 2) : (col & 7) * 2);
}
// A "samples as K" fragment (rows = lane column, k = samples in accumulator-perm order) from a tile
// image via ds_read_b64_tr_b16 (two 4-row blocks per fragment).
template <bool G>
EM_DEVICE bf16x8 tile_tr_frag(const char* smem, uint32_t base, int colbase, int q, int h, int q4, int p4, int g1) {
  const int col = colbase + 16 * g1 + 4 * p4;
  const int r0 = 16 * q + 4 * h + q4;
  return cat_tr(lds_tr16(smem, tile_img<G>(base, r0, col)), lds_tr16(smem, tile_img<G>(base, r0 + 8, col)));
}
// The 16x16x32 form (backward wave): lane column colbase + (lane & 15), k = samples σ of lane group g = lane >> 4:
// rows 16 (g >> 1) + 4 (g & 1) + 0..3, then + 8 (the same two 4-row blocks as tile_tr_frag)
template <bool G>
EM_DEVICE bf16x8 tile_tr16_frag(const char* smem, uint32_t base, int colbase, int lane) {
  const int col = colbase + 4 * (lane & 3);
  const int r0 = 16 * ((lane >> 5) & 1) + 4 * ((lane >> 4) & 1) + ((lane >> 2) & 3);
  return cat_tr(lds_tr16(smem, tile_img<G>(base, r0, col)), lds_tr16(smem, tile_img<G>(base, r0 + 8, col)));
}
// X fragments from a 16-entry nibble table (4 bf16 {0,1} per entry, 128 B): two ds_read_b64 per
// fragment; distinct entries never share a bank, unlike a 256-entry byte table
template <int LUT>
EM_DEVICE bf16x8 nib_xfrag(const char* smem, uint32_t w, int q) {
  const int sh = 16 * (q & 1);
  const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + lut_off<LUT, 3>(w, sh));
  const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + lut_off<LUT, 3>(w, sh + 4));
  return __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
}

// ============================================================================================
// v6: producer/consumer units -- forward waves feed backward waves through an LDS ring.
//
// Hidden-split wave pairs (the earlier v4) met three times per 32-sample tile (H halves, softmax
// statistics, dZ2 halves) and phase stamps showed each wave waiting on its partner ~27 % of the
// tile.  v6 splits the work by STAGE instead of by hidden unit:
//   * a unit = 4 waves working on one tile stream: two forward waves F0/F1 (even / odd tiles of the
//     unit) and two backward waves B0/B1 (hidden halves of every tile of the unit);
//   * F runs a whole tile alone -- X -> F1 (16 MFMAs) -> relu -> F2 (16) -> full grouped softmax over
//     all 64 outputs (no statistics exchange) -> dZ2 -- and leaves the H, dZ2 and X images of the
//     tile in a ring slot (16 KB), then raises the slot's FULL counter;
//   * B_rho waits for FULL, issues every LDS read of the tile at once (dZ2 A fragments from the same
//     8-byte granules F wrote, H / dZ2 / X transposes, W2ᵀ fragments), raises its DONE counter as
//     soon as they have landed, then runs B1 for its hidden half, dW2 + db2 (independent of B1: they
//     fill the matrix pipe while B1's results drain), the relu mask and dW1ᵀ from registers;
//   * F waits for a slot only when the ring is full (4 slots: the W1ᵀ / W2ᵀ images are dead once the
//     forward waves hold their weights in registers, and become each unit's 4th slot).
// Both units share the CU so that every SIMD hosts one forward and one backward wave (wave w runs
// on SIMD w % 4): the VALU-heavy loss of one beside the MFMA-heavy dW chain of the other.  Forward
// waves run at s_setprio 1 (they bound the pipeline).  Counters are monotonic LDS words (no ABA)
// and every wait is bounded: a broken protocol poisons the loss with NaN instead of hanging.
//
// Measured and rejected (docs/DESIGN.md §2; knobs removed in round 3): forward waves claiming tiles
// from an LDS counter (-0.6 %), backward waves raising priority for their read burst (-22 %), the
// next tile's X fragments built at the end of a tile (-3.7 %), forward and backward waves on
// separate SIMDs (-14 %), db2 on v_dot2 instead of 2 MFMAs (-0.6 %), input masks instead of the X
// image in a slot (-3.5 %), F1 with two interleaved hidden-tile chains (-1.3 %), the forward loop
// unrolled over the ring slots (spills), XCD-major stream numbering (-0.5 %).
//
// slot: H0 4K | H1 4K | D2 4K | X image 4K
// FUSED_SHARED: one tile stream per workgroup, 4 forward waves (tiles f, f + 4, ...) and 4 backward
// waves (hidden half rho x tile parity pi) sharing one ring; 0: two independent units of 2 + 2 waves
#ifndef FUSED_SHARED
#define FUSED_SHARED 1
#endif
#ifndef FUSED_RECYCLE
#define FUSED_RECYCLE 1
#endif
constexpr int V6_SLOT = 16384;
constexpr int V6_NSTREAM = FUSED_SHARED ? 1 : 2;  // tile streams (rings) per workgroup
constexpr int V6_NF = FUSED_SHARED ? 4 : 2;       // forward waves per stream
constexpr int V6_NBP = FUSED_SHARED ? 2 : 1;      // backward waves per hidden half (tile parities)
#ifndef V6_RSLOTS_SHARED
#define V6_RSLOTS_SHARED 6
#endif
constexpr int V6_RSLOTS = FUSED_SHARED ? V6_RSLOTS_SHARED : 3;  // slots per stream in the ring area
// + the recycled weight-image slots (the W1ᵀ / W2ᵀ images are dead once the forward waves hold their
// weights in registers)
constexpr int V6_NREC = FUSED_RECYCLE ? 2 / V6_NSTREAM : 0;
constexpr int V6_NSLOT = V6_RSLOTS + V6_NREC;
static_assert(V6_NREC == 0 || 2 * V6_SLOT <= IMG_W2Q, "recycled slots must fit below the W2Q image");
static_assert(V6_NSLOT % V6_NBP == 0, "a slot's tiles share one parity");
constexpr int V6_SH = 0, V6_SD2 = 8192, V6_SX = 12288;
// V6_WIN: the SIMD's vector issue port bounds the loop (profiles/r6/k7_probes.md: 128 extra VALU per
// backward tile cost +14 %, the forward softmax's VALU is 16 % of the step), and ~50 of the VALU per SIMD
// per tile period are slot-address adds (slot base + lane offset, the slot known only at run time).  The
// windowed layout puts each tile parity's four slots in one 64 KB window -- slot s at RING + (s & 1) * 64K
// + (s >> 1) * 16K, the ring over the dead W1ᵀ / W2ᵀ images -- and unrolls the forward loop by 2 and the
// backward loop by 4, so that within an unrolled copy the slot is a constant offset from a per-wave base:
// DS immediates instead of adds.  b2, the LUTs and the flags stay below 64K (at 0, ahead of the ring: their
// lookups keep the base in the immediate too), the W2Q image moves above the ring.
// Bit 0 unrolls the forward loop, bit 1 the backward loop (either bit selects the layout).  Same-box A/B
// (4 rounds, profiles/r6/ab_v6_win.jsonl, median µs per step): round-5 kernel 87.8; with static LDS:
// old layout 89.1, windowed + forward unrolled 87.0, + backward unrolled 86.8, both 87.1 -- at 256
// VGPRs the unrolled forward copy traded its adds for register moves.  Once the softmax's max trees
// dropped their NaN canonicalisation (common.h raw_max: v_maximum3_f32) both unrolled measured 80.8 vs
// 82.5 for the backward alone and 83.0 for the previous commit (profiles/r6/ab_v6_maxtree.jsonl).
// Default 3.
#ifndef V6_WIN
#define V6_WIN 3
#endif
// The backward wave runs on v_mfma_f32_16x16x32_bf16 (B1, dW2, dW1ᵀ, db2: 50 MFMAs of 16 cycles per tile;
// round 6 replaced 24 of 32x32x16 + 2 for db2).  K = 32 samples fits one instruction, so every operand is read
// once: the same fragment count and VGPRs as the 32x32 form.  The samples take the order σ(st, i) = 8 st +
// 16 (i >> 3) + (i & 7) as B1's rows (sample tile st) and the same order as the k index of dW2 / dW1ᵀ, i.e. the
// two-4-row transposing reads of tile_tr16_frag and conflict-free 8-B dZ2 row reads (rows {0-7, 16-23} of a tile
// have distinct img_fr per row parity).  The accumulators are 16x16 tiles; the epilogue stores each f32x4 at the
// 32x32 layout's slot, so the fold is unchanged.  db2 uses ones as A, so its k order is free.  (MI355X_MICROARCH.md
// DVFS item 7: bf16 loops on the 16x16x32 shape hold a higher clock on random data.)  Measured, same box:
// db2 alone on 16x16x32 81.95 vs 82.85 µs per step (profiles/r6/ab_v6_db2_16.jsonl), then the whole wave 79.5 vs
// 80.6 (ab_v6_b16.jsonl).  At the 4-tile backward unroll the per-slot address registers spill 14 VGPRs (2 scratch
// reloads per tile); a 2-tile unroll without spills (81.9 µs) and no unroll (82.7) measured slower than the
// spilling 4-tile loop (80.8, ab_v6_b16_unroll.jsonl).  W2 fragments held in registers for the launch instead of
// read per tile (32x32 form) spilled 100 B per lane: 94.4 vs 82.0 µs (ab_v6_sdwa_w2q.jsonl).  The 32x32 backward
// wave and those knobs are in git history (round 6).
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef f32x4v v6_db2_t[2];     // db2 of output 16-tiles 2 rho, 2 rho + 1 (every accumulator row holds the sum)
typedef f32x4v v6_acc_t[4][4];  // [hidden 16-tile of the own half][output / feature 16-tile]
static_assert(!V6_WIN || (FUSED_SHARED && V6_NSLOT == 8), "windowed layout: shared ring of 8 slots");
// windowed: b2 256 | YLUT 256 | XLUT 128 | flags 128 | ring 8 x 16K (W1ᵀ / W2ᵀ images at its start) | W2Q
constexpr int V6_IMGB = V6_WIN ? 768 : 0;                        // LDS base of the W1ᵀ / W2ᵀ images
constexpr int V6_B2B = V6_WIN ? 0 : IMG_B2;                      // b2 (forward waves)
// (the tables at 256 / 512 let mlp_loss.h / nib_xfrag take the SDWA byte-select lookup form)
constexpr int V6_XLUT = V6_WIN ? 512 : IMG_BYTES;                // 16 x 8 B: input nibble -> 4 bf16 {0,1}
constexpr int V6_YLUT = V6_WIN ? 256 : V6_XLUT + 128;            // 16 x f32x4: target nibble -> 4 {0,1} floats
constexpr int V6_FLAGS = V6_WIN ? 640 : V6_YLUT + 256;  // [streams][32 / streams ints]: full[N] | done0[N] | done1[N]
constexpr int V6_FLAG_STRIDE = 128 / V6_NSTREAM;
static_assert(3 * V6_NSLOT * 4 <= V6_FLAG_STRIDE, "flag words");
constexpr int V6_RING = V6_FLAGS + 128;  // [streams][ring slots][16 KB]
constexpr int V6_W2QB = V6_WIN ? V6_RING + 8 * V6_SLOT : IMG_W2Q;  // W2Q image base (backward waves)
constexpr int V6_LOOP_LDS = V6_WIN ? V6_W2QB + (IMG_B2 - IMG_W2Q) : V6_RING + V6_NSTREAM * V6_RSLOTS * V6_SLOT;
static_assert(!V6_WIN || (V6_RING == V6_IMGB && IMG_W2Q <= 8 * V6_SLOT), "windowed layout");
// byte offset of slot `slot` of stream `st`
EM_DEVICE uint32_t v6_slot(int st, int slot) {
  if (V6_WIN) return V6_RING + (slot & 1) * 65536 + (slot >> 1) * V6_SLOT;
  return slot < V6_RSLOTS ? V6_RING + (st * V6_RSLOTS + slot) * V6_SLOT
                          : (FUSED_SHARED ? slot - V6_RSLOTS : st) * V6_SLOT;
}
EM_DEVICE uint32_t v6_w2q_off(int row, int k8) { return V6_W2QB + row * W2Q_RS + (k8 ^ mlp::w2q_swz(row)) * 16; }
// LDS destination of byte `b` of the weight image
EM_DEVICE uint32_t v6_img_dst(uint32_t b) {
  if (!V6_WIN) return b;
  return b < (uint32_t)IMG_W2Q ? V6_IMGB + b : b < (uint32_t)IMG_B2 ? b - IMG_W2Q + V6_W2QB : b - IMG_B2 + V6_B2B;
}
constexpr int V6_RED = 131072;  // epilogue: two fp32 dW images [2][16384] below, DB2S [2][64] + LOSSS [8] above
constexpr int V6_LDS = (V6_LOOP_LDS > V6_RED + 2048 ? V6_LOOP_LDS : V6_RED + 2048);
static_assert(V6_LDS <= 163840 && V6_RING % 16 == 0, "v6 LDS budget");
static_assert(IMG_BYTES == 54528 && IMG_BYTES % 16 == 0, "image size (ops/fused_mlp.py IMG_BYTES)");
constexpr int V6_SPIN_LIMIT = 1 << 20;  // ~50 ms of polling: a legitimate wait is microseconds

// wait until the LDS counter at off reaches target (skipped once a wait has failed: the launch then
// drains quickly and reports NaN)
EM_DEVICE void v6_wait(const char* smem, uint32_t off, int target, bool& ok) {
  if (!ok) return;
  int spins = 0;
  while (__hip_atomic_load(reinterpret_cast<const int*>(smem + off), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
         target) {
    __builtin_amdgcn_s_sleep(FUSED_SLEEP);
    if (++spins > V6_SPIN_LIMIT) {
      ok = false;
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// tile stream `st` of this block: global stream U, tiles U, U + nunits, ...
EM_DEVICE int v6_unit_id(int st) { return blockIdx.x * V6_NSTREAM + st; }

EM_DEVICE int v6_ntiles_of_unit(int B, int U, int nunits) {
  const int ntiles = (B + 31) / 32;
  return U < ntiles ? (ntiles - U + nunits - 1) / nunits : 0;
}

// forward wave f of stream `unit`: tiles k = f, f + V6_NF, ... of the stream
template <int LOSS, bool SIDX>
EM_DEVICE void v6_forward(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                          int offset, int unit, int f, int lane, float& loss_acc, bool& ok, Stamps& st) {
  const int r = lane & 31, h = lane >> 5;
  const int nunits = gridDim.x * V6_NSTREAM, U = v6_unit_id(unit);
  const int K = v6_ntiles_of_unit(B, U, nunits);
  const uint32_t FL = V6_FLAGS + unit * V6_FLAG_STRIDE;
  // Branch-free prefetch of the next tile's masks: samples past the stream read sample 0 (valid when
  // K > 0) and are masked at use.  An exec-masked load here made the compiler wait vmcnt(0) right
  // after issuing it -- one HBM round trip (~900 cycles) per forward tile, round 3's "F wait slot".
  auto fetch = [&](int k, uint64_t& mi, uint64_t& mt) {
    const int s = (U + k * nunits) * 32 + r;
    const int sc = (k < K && s < B) ? s : 0;
    const int idx = SIDX ? sidx[sc] : (offset + sc);
    mi = masks[idx];
    mt = masks[idx + 1];
  };
  uint64_t nin = 0, ntg = 0;
  if (K > 0) fetch(f, nin, ntg);
  // the forward wave's weight fragments (W1ᵀ 4 x 4, W2ᵀ 2 x 8: 128 VGPRs) stay in registers for the
  // whole launch: no LDS read stands between the tile's operands and its 32 MFMAs
  bf16x8 w1r[4][4], w2r[2][8];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) w1r[t][q] = lds_frag(smem, V6_IMGB + w1t_off(32 * t + r, 2 * q + h));
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) w2r[u][kk] = lds_frag(smem, V6_IMGB + w2p_off(32 * u + r, kk * 2 + h));
  __syncthreads();  // every forward wave holds its weights: the W1ᵀ / W2ᵀ images are free (recycled slots)
  st.start();
  // (one tile as a lambda called from the loop below: written inline in the loop, the same body
  // compiles to 9 more VALU per tile -- slot addresses recomputed -- and measured 3 % slower)
  auto ftile = [&](int k, int slot, int knext, uint32_t SB) {
    const bool valid = (U + k * nunits) * 32 + r < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(knext, nin, ntg);
    if (k >= V6_NSLOT) {  // the slot's previous tile (k - 4) must be consumed by both backward waves
      v6_wait(smem, FL + (V6_NSLOT + slot) * 4, k - V6_NSLOT + 1, ok);
      v6_wait(smem, FL + (2 * V6_NSLOT + slot) * 4, k - V6_NSLOT + 1, ok);
    }
    st.mark(0);

    // X fragments (B of F1) + X image [32 samples][64 feat] for dW1ᵀ
    bf16x8 xf[4];
    {
      const uint32_t wlo = (uint32_t)imask >> (8 * h), whi = (uint32_t)(imask >> 32) >> (8 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) xf[q] = nib_xfrag<V6_XLUT>(smem, q < 2 ? wlo : whi, q);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(smem + tile_img<false>(SB + V6_SX, r, 16 * q + 8 * h)) = xf[q];

    // F1: Z1ᵀ = W1ᵀ·Xᵀ -> relu -> Hᵀ fragments + H images
    bf16x8 hT[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 a1 = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q) a1 = mfma32(w1r[t][q], xf[q], a1);
      const uint32_t HB = SB + V6_SH + (t >> 1) * 4096;  // H sub-image of hidden half t >> 1
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        hT[t][q] = relu_pack(a1, q);
        const u32x4 d = __builtin_bit_cast(u32x4, hT[t][q]);
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(HB, r, 32 * (t & 1) + 16 * q + 4 * h)) = u32x2{d[0], d[1]};
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(HB, r, 32 * (t & 1) + 16 * q + 8 + 4 * h)) = u32x2{d[2], d[3]};
      }
    }
    st.mark(1);

    // F2: Z2ᵀ = W2ᵀ·Hᵀ + b2
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + V6_B2B + (32 * u + 8 * g + 4 * h) * 4);
        z2[u][4 * g + 0] = b[0]; z2[u][4 * g + 1] = b[1]; z2[u][4 * g + 2] = b[2]; z2[u][4 * g + 3] = b[3];
      }
    auto f2mfma = [&](int u, int kk) { z2[u] = mfma32(w2r[u][kk], hT[kk >> 1][kk & 1], z2[u]); };
    // softmax: tile 0's chain first; tile 1's chain is issued by the softmax hook, one MFMA per step
    // of tile 0's statistics (sched_barrier fences pin that order)
    auto hook = [&](auto&& step) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f2mfma(1, j);
        __builtin_amdgcn_sched_barrier(0);
        step(j);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (LOSS == 0) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) f2mfma(0, kk);
    } else {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int u = 0; u < 2; ++u) f2mfma(u, kk);
    }
    st.mark(2);

    float dz[2][16];
    float lt = 0.f;  // this lane's loss terms of the tile
    if ((FUSED_PROBE & 1) && LOSS == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f2mfma(1, j);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) dz[u][i] = z2[u][i] * 0.015625f;
      lt = (float)(tmask & 1);
    } else if (LOSS == 0)
      v6_softmax_split<V6_YLUT, true>(smem, z2, tmask, h, dz, lt, hook);
    else
      bce_tile_loss<V6_YLUT, true>(smem, z2, tmask, valid, h, dz, lt);
    loss_acc += lt;
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
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 4 * h)) = u32x2{fq[0], fq[1]};
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 8 + 4 * h)) =
            u32x2{fq[2], fq[3]};
      }
    lds_signal(smem, FL + slot * 4, k + 1);  // FULL
    st.mark(4);
  };
  if (V6_WIN & 1) {  // tiles f, f + 4, ... alternate slots f and f + 4: the second is the first + 32K
    const uint32_t SB0 = v6_slot(unit, f);
    for (int k = f; k < K; k += 2 * V6_NF) {
      ftile(k, f, k + V6_NF, SB0);
      if (k + V6_NF < K) ftile(k + V6_NF, f + V6_NF, k + 2 * V6_NF, SB0 + 2 * V6_SLOT);
    }
  } else {
    for (int k = f; k < K; k += V6_NF) ftile(k, k % V6_NSLOT, k + V6_NF, v6_slot(unit, k % V6_NSLOT));
  }
}

// backward wave of hidden half RHO: every tile of the unit's stream.  Every LDS read of the tile
// (dZ2 A fragments, H / dZ2 / X transposes, W2ᵀ fragments: ~96 VGPRs) is issued at once right after
// FULL, the slot is released as soon as they have landed, and the 26 MFMAs then run from registers.
template <int RHO>
EM_DEVICE void v6_backward(char* smem, int B, int unit, int parity, int lane, v6_acc_t& dW2, v6_acc_t& dW1T,
                           v6_db2_t& db2, bool& ok, Stamps& st) {
  const int r = lane & 31, h = lane >> 5;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;
  const int nunits = gridDim.x * V6_NSTREAM, U = v6_unit_id(unit);
  const int K = v6_ntiles_of_unit(B, U, nunits);
  const uint32_t FL = V6_FLAGS + unit * V6_FLAG_STRIDE;
  const uint32_t MYDONE = FL + ((1 + RHO) * V6_NSLOT) * 4;
  const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  __syncthreads();  // matches the forward waves' barrier (recycled images)
  st.start();
  auto btile = [&](int k, int slot, uint32_t SB) {
    const uint32_t D2 = SB + V6_SD2, HB = SB + V6_SH + RHO * 4096;
    const int g = lane >> 4, gw = g ^ mlp::w2q_swz(lane & 15);
    v6_wait(smem, FL + slot * 4, k + 1, ok);
    st.mark(5);

    // dZ2 as B1's A operand: row i = sample σ(st, i) = 8 st + 16 (i >> 3) + (i & 7), k = W2Q granule 4 kk + g
    // (outputs 16 c + 4 (g & 1) + 0..3 and + 8.., c = 2 kk + (g >> 1): the granule's own order)
    bf16x8 dzA[2][2], w2q[4][2], hR[4], bd[4], bx[4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int row = 8 * s + 16 * ((lane >> 3) & 1) + (lane & 7), col = 16 * (2 * kk + (g >> 1)) + 4 * (g & 1);
        const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + tile_img<true>(D2, row, col));
        const u32x2 hi = *reinterpret_cast<const u32x2*>(smem + tile_img<true>(D2, row, col + 8));
        dzA[s][kk] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
      }
#pragma unroll
    for (int t = 0; t < 4; ++t) hR[t] = tile_tr16_frag<true>(smem, HB, 16 * t, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)  // v6_w2q_off with the swizzle taken from lane & 15 (= row & 15) once
        w2q[t][kk] = lds_frag(smem, V6_W2QB + (64 * RHO + 16 * t + (lane & 15)) * W2Q_RS + 64 * kk + 16 * gw);
#pragma unroll
    for (int u = 0; u < 4; ++u) bd[u] = tile_tr16_frag<true>(smem, D2, 16 * u, lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) bx[u] = tile_tr16_frag<false>(smem, SB + V6_SX, 16 * u, lane);
    lds_signal(smem, MYDONE + slot * 4, k + 1);  // DONE (fenced form: waits for every read above)
    st.mark(6);

    // B1: dH[sample σ][own hidden] = dZ2·W2ᵀ, two sample tiles x four hidden tiles
    f32x4v aD[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) aD[s][t] = f32x4v{};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          aD[s][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dzA[s][kk], w2q[t][kk], aD[s][t], 0, 0, 0);
    // dW2[own hid][out] += Hᵀ·dZ2 ; db2 += ones·dZ2 (independent of B1: fills the pipe)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) dW2[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hR[t], bd[u], dW2[t][u], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < 2; ++m)
      db2[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bd[2 * RHO + m], db2[m], 0, 0, 0);
    if (FUSED_PROBE & 2) {
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = (float)(lane + j) * 1e-3f + (float)k * 1e-6f;
#pragma unroll
      for (int it = 0; it < FUSED_PROBE_VALU / 8; ++it)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          a[j] = (it & 7) == 7 ? __builtin_amdgcn_exp2f(a[j]) : __builtin_fmaf(a[j], 0.999f, 0.25f);
      asm volatile("" ::"v"(a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6] + a[7]));
    }
    st.mark(7);
    // dZ1 = dH * (H > 0): lane group g's k = samples σ(0, 4g..) then σ(1, 4g..) = aD[0][t], aD[1][t]
    bf16x8 dz1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) dz1[t] = mask_by4(hR[t], aD[0][t], aD[1][t]);
    st.mark(8);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        dW1T[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dz1[t], bx[u], dW1T[t][u], 0, 0, 0);
    st.mark(9);
  };
  if (V6_WIN & 2) {  // tiles parity, parity + 2, ... cycle through slots parity + 0/2/4/6: base + 0/16/32/48K
    const uint32_t SB0 = v6_slot(unit, parity);
    for (int k = parity; k < K; k += 4 * V6_NBP) {
      btile(k, parity, SB0);
      if (k + V6_NBP < K) btile(k + V6_NBP, parity + 2, SB0 + V6_SLOT);
      if (k + 2 * V6_NBP < K) btile(k + 2 * V6_NBP, parity + 4, SB0 + 2 * V6_SLOT);
      if (k + 3 * V6_NBP < K) btile(k + 3 * V6_NBP, parity + 6, SB0 + 3 * V6_SLOT);
    }
  } else {
    for (int k = parity; k < K; k += V6_NBP) btile(k, k % V6_NSLOT, v6_slot(unit, k % V6_NSLOT));
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
// ROLE 0 = forward wave sub (its first tile), 2/3 = backward wave of hidden half rho = ROLE - 2 and
// tile parity sub
template <int LOSS, bool SIDX, int ROLE>
EM_DEVICE void v6_body(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                       int offset, int unit, int sub, int wave, int lane, float* slab_spare) {
  const int r = lane & 31, h = lane >> 5;
  bool ok = true;
  Stamps st;
  // per part (stream, or tile parity in the shared layout): [16 tiles][4 g][64 lanes][4] f32, 0..7 dW2,
  // 8..15 dW1T
  float* RED = reinterpret_cast<float*>(smem);
  float* DB2S = reinterpret_cast<float*>(smem + V6_RED);          // [2 parts][64]
  float* LOSSS = reinterpret_cast<float*>(smem + V6_RED + 512);   // [8]
  auto dump = [&]() {
    if (FUSED_STAMPS && lane < 10) {  // phase cycles of this wave -> spare slab floats
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 10; ++k) v = (lane == k) ? st.acc[k] : v;
      slab_spare[wave * 16 + lane] = (float)v;
    }
  };
  if (ROLE < 2) {
    float loss_acc = 0.f;
    __builtin_amdgcn_s_setprio(FUSED_FPRIO);  // forward waves bound the pipeline (+3 % at 1)
    v6_forward<LOSS, SIDX>(smem, masks, sidx, B, offset, unit, sub, lane, loss_acc, ok, st);
    float lsum = wave_sum(loss_acc);
    if (!ok) lsum = __builtin_nanf("");
    dump();
    __syncthreads();  // every wave is out of the loop: the loop's LDS is free
    if (lane == 0) LOSSS[wave] = lsum;
    __syncthreads();
  } else {
    constexpr int RHO = ROLE - 2;
    v6_acc_t dW2, dW1T;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        dW2[t][u] = f32x4v{};
        dW1T[t][u] = f32x4v{};
      }
    v6_db2_t db2;
    db2[0] = f32x4v{};
    db2[1] = f32x4v{};
    v6_backward<RHO>(smem, B, unit, sub, lane, dW2, dW1T, db2, ok, st);
    const int part = FUSED_SHARED ? sub : unit;
    dump();
    __syncthreads();
    if (lane < 16) {  // 16x16 accumulator column lane = output 32 RHO + 16 m + lane (every row holds the sum)
      DB2S[part * 64 + 32 * RHO + lane] = db2[0][0];
      DB2S[part * 64 + 32 * RHO + 16 + lane] = db2[1][0];
    }
    if (lane == 0) LOSSS[wave] = ok ? 0.f : __builtin_nanf("");
    // 16x16 tile (t, u), lane (j, g'): rows 16 (t & 1) + 4 g' .. + 3 of 32x32 tile (t >> 1, u >> 1), column
    // 16 (u & 1) + j -- the 32x32 layout's group 2 (t & 1) + (g' >> 1) of lane (16 (u & 1) + j, g' & 1)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int which = 0; which < 2; ++which) {
          const f32x4v& acc = which ? dW1T[t][u] : dW2[t][u];
          const int T = 8 * which + 2 * (2 * RHO + (t >> 1)) + (u >> 1), gq = lane >> 4;
          *reinterpret_cast<f32x4*>(RED + part * 16384 +
                                    v6_red_slot(T, 2 * (t & 1) + (gq >> 1), 16 * (u & 1) + (lane & 15), gq & 1) * 4) =
              f32x4{acc[0], acc[1], acc[2], acc[3]};
        }
    __syncthreads();
  }
}

// ============================================================================================
// v8: THREE waves per SIMD -- two forward waves and one backward wave on every SIMD.
//
// v6's phase stamps (profiles/r5/fused_timeline_xcc.txt) put the forward wave at the pole: per tile
// 4.5 k cycles of work + 0.7 k waiting for a slot, of which ~2.2 k is the softmax's in-order VALU
// chain, while the matrix pipe idles ~half the time.  One forward chain per SIMD cannot hide its own
// latency, and at 256 VGPRs (weights in registers, half-hidden dW accumulators) no third wave fits.
// v8 trades registers for LDS traffic so that 12 waves fit at <= 168 VGPRs:
//   * 8 forward waves (tiles f, f + 8, ... of the workgroup's stream) read their W1ᵀ / W2ᵀ fragments
//     from the LDS images for every tile (32 ds_read_b128 per tile) instead of holding them, and write
//     the tile's X / H / dZ2 images into a ring slot only at the END of the tile (X fragments and Hᵀ
//     stay in registers through F2 and the softmax), so a slot is held only from that write burst to
//     the backward waves' reads: 6 slots serve 8 producers;
//   * 4 backward waves, one per hidden QUARTER, each consume EVERY tile in order (13 MFMAs per tile:
//     B1 4, dW2 4, dW1ᵀ 4, db2 on v_dot2 instead of a 16-register MFMA accumulator): 64 dW accumulator
//     registers per wave instead of 144, and no parity copies to fold;
//   * a slot is free again when all four backward waves have read it (one LDS counter, +1 per wave).
// Waves 0-7 forward, 8-11 backward: wave w runs on SIMD w % 4, so every SIMD hosts two forward and one
// backward wave.  Gradient summation order is fixed (every backward wave walks the tiles in order), so
// slabs stay bit-reproducible run to run.  Selected at run time (EUROM_FUSED_V=8); v6 stays the default
// until a same-box A/B says otherwise.
#ifndef V8_FPRIO
#define V8_FPRIO 0
#endif
#ifndef V8_BPRIO
#define V8_BPRIO 1
#endif
// V8_DYN: 0 = static tiles f, f + 8, ... per forward wave; 1 = tiles claimed from an LDS counter one tile
// ahead (masks prefetched).  Measured equal (93.2 / 94.2 us per step); claiming at the tile start, with the
// mask loads exposed, 94.6 (removed).
#ifndef V8_DYN
#define V8_DYN 0
#endif
// FUSED_TRACE (diagnostic builds only, tools/fused_trace.py): block 0 records s_memtime per tile into
// loss_slabs[gridDim.x ...] (12 words per tile: forward start / computed / written / wave, then FULL seen
// and DONE per backward wave)
#ifndef FUSED_TRACE
#define FUSED_TRACE 0
#endif
constexpr int V8_NF = 8, V8_NB = 4, V8_THREADS = 64 * (V8_NF + V8_NB);
// Slot layouts.  v8: H 8K | D2 4K | X 4K | loss terms 256 B, 6 slots.  v9 (VER = 9): the forward waves also
// run B1 and the relu mask, and hand the backward waves dZ1 as an 8 KB image (after X), 4 slots.
template <int VER>
struct V8L {
  static constexpr int NSLOT = VER == 9 ? 4 : 6;
  static constexpr int SD1 = V6_SLOT;                          // v9: dZ1 image [32 samples][128 hidden]
  static constexpr int SLOSS = VER == 9 ? V6_SLOT + 8192 : V6_SLOT;  // the tile's per-lane loss terms
  static constexpr int SLOT = SLOSS + 256;
};
constexpr int V8_XLUT = IMG_BYTES;       // 16 x 8 B: input nibble -> 4 bf16 {0,1}
constexpr int V8_YLUT = V8_XLUT + 128;   // 16 x f32x4: target nibble -> 4 {0,1} floats
constexpr int V8_FLAGS = V8_YLUT + 256;  // FULL[8] | DONE[8] (ints)
constexpr int V8_DONE = V8_FLAGS + 32;
constexpr int V8_CLAIM = V8_FLAGS + 64;
constexpr int V8_RING = V8_FLAGS + 128;
template <int VER>
constexpr int v8_lds() { return V8_RING + V8L<VER>::NSLOT * V8L<VER>::SLOT; }
constexpr int V8_RED = 0, V8_DB2S = 65536, V8_LOSSS = V8_DB2S + 1024;  // epilogue (after the loop)
static_assert(v8_lds<8>() <= 163840 && v8_lds<9>() <= 163840 && V8_RING % 16 == 0, "v8 / v9 LDS budget");
static_assert(V8_LOSSS + 64 <= v8_lds<9>() && V8_LOSSS + 64 <= v8_lds<8>(), "epilogue area");
static_assert(V8L<8>::NSLOT <= 8, "flag words");
template <int VER>
EM_DEVICE uint32_t v8_slot(int slot) { return V8_RING + slot * V8L<VER>::SLOT; }
EM_DEVICE void v8_trace(uint32_t* tr, int k, int word, int lane) {
  if (FUSED_TRACE && tr && blockIdx.x == 0 && lane == 0) tr[k * 12 + word] = (uint32_t)__builtin_amdgcn_s_memtime();
}

// forward wave f: tiles k = f, f + V8_NF, ... of the workgroup's stream
template <int LOSS, bool SIDX, int VER>
EM_DEVICE void v8_forward(char* smem, const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                          int offset, int f, int lane, float& loss_acc, bool& ok, Stamps& st, uint32_t* tr) {
  const int r = lane & 31, h = lane >> 5;
  const int nunits = gridDim.x, U = blockIdx.x;
  const int K = v6_ntiles_of_unit(B, U, nunits);
  auto fetch = [&](int k, uint64_t& mi, uint64_t& mt) {  // branch-free prefetch (see v6_forward)
    const int s = (U + k * nunits) * 32 + r;
    const int sc = (k < K && s < B) ? s : 0;
    const int idx = SIDX ? sidx[sc] : (offset + sc);
    mi = masks[idx];
    mt = masks[idx + 1];
  };
  uint64_t nin = 0, ntg = 0;
  st.start();
  auto ftile = [&](int k, int slot, int knext) {
    const bool valid = (U + k * nunits) * 32 + r < B;
    const uint64_t imask = valid ? (nin | BIAS_BIT) : 0ull;
    const uint64_t tmask = valid ? ntg : 0ull;
    fetch(knext, nin, ntg);
    v8_trace(tr, k, 0, lane);
    if (FUSED_TRACE && tr && blockIdx.x == 0 && lane == 0) tr[k * 12 + 3] = f;

    bf16x8 xf[4];
    {
      const uint32_t wlo = (uint32_t)imask >> (8 * h), whi = (uint32_t)(imask >> 32) >> (8 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) xf[q] = nib_xfrag<V8_XLUT>(smem, q < 2 ? wlo : whi, q);
    }
    // F1: Z1ᵀ = W1ᵀ·Xᵀ (W1ᵀ fragments from the LDS image) -> relu -> Hᵀ fragments (kept in registers)
    bf16x8 hT[4][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 a1 = f32x16{};
#pragma unroll
      for (int q = 0; q < 4; ++q) a1 = mfma32(lds_frag(smem, w1t_off(32 * t + r, 2 * q + h)), xf[q], a1);
#pragma unroll
      for (int q = 0; q < 2; ++q) hT[t][q] = relu_pack(a1, q);
    }
    st.mark(1);

    // F2: Z2ᵀ = W2ᵀ·Hᵀ + b2
    f32x16 z2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + IMG_B2 + (32 * u + 8 * g + 4 * h) * 4);
        z2[u][4 * g + 0] = b[0]; z2[u][4 * g + 1] = b[1]; z2[u][4 * g + 2] = b[2]; z2[u][4 * g + 3] = b[3];
      }
    auto w2f = [&](int u, int kk) { return lds_frag(smem, w2p_off(32 * u + r, kk * 2 + h)); };
    // tile 1's chain runs inside the softmax hook (fenced by sched_barriers), so its W2ᵀ fragments are
    // read two MFMAs ahead there instead of being hoisted by the scheduler
    bf16x8 w2n[8];
    auto hook = [&](auto&& step) {
      w2n[0] = w2f(1, 0);
      w2n[1] = w2f(1, 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j + 2 < 8) w2n[j + 2] = w2f(1, j + 2);
        z2[1] = mfma32(w2n[j], hT[j >> 1][j & 1], z2[1]);
        __builtin_amdgcn_sched_barrier(0);
        step(j);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (LOSS == 0) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) z2[0] = mfma32(w2f(0, kk), hT[kk >> 1][kk & 1], z2[0]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int u = 0; u < 2; ++u) z2[u] = mfma32(w2f(u, kk), hT[kk >> 1][kk & 1], z2[u]);
    }
    st.mark(2);

    float dz[2][16];
    float lt = 0.f;
    if (LOSS == 0)
      v6_softmax_split<V8_YLUT, true>(smem, z2, tmask, h, dz, lt, hook);
    else
      bce_tile_loss<V8_YLUT, true>(smem, z2, tmask, valid, h, dz, lt);
    // dZ2ᵀ as bf16 fragments: [u][q] holds outputs 32u + acc_perm(q, h, 0..7) of sample r -- the D2 image's
    // granules, and (v9) the B operand of B1
    u32x4 dzq[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        dzq[u][q] = __builtin_bit_cast(
            u32x4, pack8(dz[u][8 * q + 0], dz[u][8 * q + 1], dz[u][8 * q + 2], dz[u][8 * q + 3], dz[u][8 * q + 4],
                         dz[u][8 * q + 5], dz[u][8 * q + 6], dz[u][8 * q + 7]));
    st.mark(3);
    // v9: B1 on the forward wave, chained from its own dZ2ᵀ fragments: dHᵀ = W2·dZ2ᵀ (W2 rows = hidden, k =
    // outputs in accumulator-perm order: the W2Q image), the relu mask from Hᵀ in the same layout, dZ1ᵀ to the
    // slot for the backward waves' dW1ᵀ
    bf16x8 dz1[4][2];
    if (VER == 9) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x16 aT = f32x16{};
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          aT = mfma32(lds_frag(smem, w2q_off(32 * t + r, kk * 2 + h)), __builtin_bit_cast(bf16x8, dzq[kk >> 1][kk & 1]),
                      aT);
#pragma unroll
        for (int q = 0; q < 2; ++q) dz1[t][q] = mask_by(hT[t][q], aT, q);
      }
    }
    v8_trace(tr, k, 1, lane);

    // the slot's previous tile (k - NSLOT) must have been read by all four backward waves
    constexpr int NSLOT = V8L<VER>::NSLOT;
    if (k >= NSLOT) v6_wait(smem, V8_DONE + slot * 4, V8_NB * (k / NSLOT), ok);
    st.mark(0);
    const uint32_t SB = v8_slot<VER>(slot);
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(smem + tile_img<false>(SB + V6_SX, r, 16 * q + 8 * h)) = xf[q];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t HB = SB + V6_SH + (t >> 1) * 4096;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x4 d = __builtin_bit_cast(u32x4, hT[t][q]);
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(HB, r, 32 * (t & 1) + 16 * q + 4 * h)) = u32x2{d[0], d[1]};
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(HB, r, 32 * (t & 1) + 16 * q + 8 + 4 * h)) = u32x2{d[2], d[3]};
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x4 fq = dzq[u][q];
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 4 * h)) = u32x2{fq[0], fq[1]};
        *reinterpret_cast<u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 8 + 4 * h)) =
            u32x2{fq[2], fq[3]};
      }
    if (VER == 9) {  // dZ1 image: the H image's layout (the backward waves read it with the same transposes)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t DB = SB + V8L<VER>::SD1 + (t >> 1) * 4096;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const u32x4 d = __builtin_bit_cast(u32x4, dz1[t][q]);
          *reinterpret_cast<u32x2*>(smem + tile_img<true>(DB, r, 32 * (t & 1) + 16 * q + 4 * h)) = u32x2{d[0], d[1]};
          *reinterpret_cast<u32x2*>(smem + tile_img<true>(DB, r, 32 * (t & 1) + 16 * q + 8 + 4 * h)) = u32x2{d[2], d[3]};
        }
      }
    }
    // the tile's loss terms travel with it: backward wave 0 sums them in tile order (bit-reproducible
    // however the tiles were distributed over the forward waves)
    reinterpret_cast<float*>(smem + SB + V8L<VER>::SLOSS)[lane] = lt;
    lds_signal(smem, V8_FLAGS + slot * 4, k + 1);  // FULL
    st.mark(4);
    v8_trace(tr, k, 2, lane);
  };
  if (V8_DYN == 0) {
    if (K > 0) fetch(f, nin, ntg);
    for (int k = f; k < K; k += V8_NF) ftile(k, k % V8L<VER>::NSLOT, k + V8_NF);
  } else {
    auto claim = [&]() {
      int t = 0;
      if (lane == 0)
        t = __hip_atomic_fetch_add(reinterpret_cast<int*>(smem + V8_CLAIM), 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
      return __builtin_amdgcn_readfirstlane(t);
    };
    int cur = claim();
    if (cur < K) fetch(cur, nin, ntg);
    while (cur < K) {
      const int nxt = claim();
      ftile(cur, cur % V8L<VER>::NSLOT, nxt);
      cur = nxt;
    }
  }
}

// backward wave of hidden quarter Q (hidden units 32Q .. 32Q + 31): every tile of the stream, in order.
// The tile's reads go out in three groups with the MFMAs that need only the earlier groups in between.
// tools/fused_trace.py puts this wave at ~1.5 k cycles per tile either way (one read burst: 0.64 k burst +
// 0.85 k MFMA issue), which bounds v8 (profiles/r6/k7_v8_runs.md).  Reading tile k + 1 under tile k's MFMAs
// (a cross-tile pipeline) needs ~25 VGPRs more than the 168 of three waves per SIMD: built, spilled 80-96 B
// per lane in the loop, removed.
// v9 (VER = 9): the forward wave already ran B1 and the mask; this wave reads dZ1ᵀ from the slot's dZ1 image
// (the same transposing reads as Hᵀ) and runs only dW2, db2 and dW1ᵀ -- 8 MFMAs, no dependency chain.
template <int Q, int VER>
EM_DEVICE void v8_backward(char* smem, int B, int lane, f32x16 (&dW2)[2], f32x16 (&dW1T)[2], float& db2,
                           float& loss_acc, bool& ok, Stamps& st, uint32_t* tr) {
  const int r = lane & 31, h = lane >> 5;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g1 = (lane >> 4) & 1;
  const int K = v6_ntiles_of_unit(B, blockIdx.x, gridDim.x);
  const uint32_t HOFF = V6_SH + (Q >> 1) * 4096;  // H sub-image holding this quarter
  constexpr int hcol = 32 * (Q & 1), du = Q >> 1, ds = Q & 1;  // db2 share: output tile du, sample half ds
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  const bf16x2v one2 = {(__bf16)1.0f, (__bf16)1.0f};
  bf16x8 w2q[4], dzA[2][2], hR[2], bd[2][2], bx[2][2];
  auto rd_dzA = [&](uint32_t SB) {  // dZ2 as B1's A operand (samples x outputs): the forward wave's granules
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) w2q[kk] = lds_frag(smem, w2q_off(32 * Q + r, kk * 2 + h));
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const u32x2 lo = *reinterpret_cast<const u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 4 * h));
        const u32x2 hi =
            *reinterpret_cast<const u32x2*>(smem + tile_img<true>(SB + V6_SD2, r, 32 * u + 16 * q + 8 + 4 * h));
        dzA[u][q] = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
      }
  };
  auto rd_bd = [&](uint32_t SB) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) bd[u][q] = tile_tr_frag<true>(smem, SB + V6_SD2, 32 * u, q, h, q4, p4, g1);
  };
  auto rd_hR = [&](uint32_t SB) {
#pragma unroll
    for (int q = 0; q < 2; ++q) hR[q] = tile_tr_frag<true>(smem, SB + HOFF, hcol, q, h, q4, p4, g1);
  };
  auto rd_bx = [&](uint32_t SB) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) bx[u][q] = tile_tr_frag<false>(smem, SB + V6_SX, 32 * u, q, h, q4, p4, g1);
    if (Q == 0) loss_acc += reinterpret_cast<const float*>(smem + SB + V8L<VER>::SLOSS)[lane];
  };
  auto release = [&](int slot, int k) {  // every read of the slot has landed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0)
      __hip_atomic_fetch_add(reinterpret_cast<int*>(smem + V8_DONE + slot * 4), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    v8_trace(tr, k, 5 + 2 * Q, lane);
  };
  auto wait_full = [&](int slot, int k) {
    v6_wait(smem, V8_FLAGS + slot * 4, k + 1, ok);
    v8_trace(tr, k, 4 + 2 * Q, lane);
  };
  auto db2_share = [&]() {  // db2[out tile du] += this lane's 8 samples of sample half ds (v_dot2 with ones)
    uint32_t b[4];  // memcpy, not a bit_cast of a vector element: see as_s16x2
    __builtin_memcpy(b, &bd[du][ds], 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x2v pr;
      __builtin_memcpy(&pr, &b[j], 4);
      db2 = __builtin_amdgcn_fdot2_f32_bf16(pr, one2, db2, false);
    }
  };
  st.start();
  if (VER == 9) {
    int slot = 0;
    for (int k = 0; k < K; ++k) {
      const uint32_t SB = v8_slot<VER>(slot);
      wait_full(slot, k);
      st.mark(5);
      bf16x8 dz1[2];
      rd_hR(SB);
      rd_bd(SB);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        dz1[q] = tile_tr_frag<true>(smem, SB + V8L<VER>::SD1 + (Q >> 1) * 4096, hcol, q, h, q4, p4, g1);
      rd_bx(SB);
      release(slot, k);
      slot = slot + 1 == V8L<VER>::NSLOT ? 0 : slot + 1;
      st.mark(6);
#pragma unroll
      for (int u = 0; u < 2; ++u)  // dW2[own hid][out] += Hᵀ·dZ2
#pragma unroll
        for (int q = 0; q < 2; ++q) dW2[u] = mfma32(hR[q], bd[u][q], dW2[u]);
      db2_share();
#pragma unroll
      for (int u = 0; u < 2; ++u)  // dW1ᵀ[own hid][feat] += dZ1ᵀ·X
#pragma unroll
        for (int q = 0; q < 2; ++q) dW1T[u] = mfma32(dz1[q], bx[u][q], dW1T[u]);
      st.mark(9);
    }
    return;
  }
  {  // staged reads inside the tile: each group's read latency runs under the MFMAs before it
    int slot = 0;
    for (int k = 0; k < K; ++k) {
      const uint32_t SB = v8_slot<VER>(slot);
      wait_full(slot, k);
      st.mark(5);
      rd_dzA(SB);  // (+ the W2ᵀ fragments)
      __builtin_amdgcn_sched_barrier(0);
      rd_hR(SB);
      rd_bd(SB);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 aD = f32x16{};  // B1: dH = dZ2·W2ᵀ for the own hidden quarter
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) aD = mfma32(dzA[kk >> 1][kk & 1], w2q[kk], aD);
      __builtin_amdgcn_sched_barrier(0);
      rd_bx(SB);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u)  // dW2[own hid][out] += Hᵀ·dZ2 (independent of B1)
#pragma unroll
        for (int q = 0; q < 2; ++q) dW2[u] = mfma32(hR[q], bd[u][q], dW2[u]);
      db2_share();
      __builtin_amdgcn_sched_barrier(0);
      release(slot, k);
      slot = slot + 1 == V8L<VER>::NSLOT ? 0 : slot + 1;
      st.mark(6);
      bf16x8 dz1[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) dz1[q] = mask_by(hR[q], aD, q);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int q = 0; q < 2; ++q) dW1T[u] = mfma32(dz1[q], bx[u][q], dW1T[u]);
      st.mark(9);
    }
  }
}

template <int LOSS, bool SIDX, int VER>
__device__ __forceinline__ void train_v8(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                                         int offset, const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                                         float* __restrict__ loss_slabs, int* __restrict__ step) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t ts[4] = {};
  if (FUSED_STAMPS) ts[0] = __builtin_amdgcn_s_memrealtime();
  if (step && blockIdx.x == 0 && threadIdx.x == 0) step[0] = step[0] + 1;  // see train_v6
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  {
    constexpr int N16 = IMG_BYTES / 16, KK = (N16 + V8_THREADS - 1) / V8_THREADS;
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4* dst = reinterpret_cast<u32x4*>(smem);
    u32x4 v[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) v[k] = src[min(tid + V8_THREADS * k, N16 - 1)];  // branch-free loads
#pragma unroll
    for (int k = 0; k < KK; ++k)
      if (tid + V8_THREADS * k < N16) dst[tid + V8_THREADS * k] = v[k];
  }
  if (tid < 64) reinterpret_cast<float*>(smem + V8_YLUT)[tid] = (float)(((tid >> 2) >> (tid & 3)) & 1);
  if (tid < 32) {
    const uint32_t n = (uint32_t)tid >> 1, b = 2u * (tid & 1);
    reinterpret_cast<uint32_t*>(smem + V8_XLUT)[tid] =
        (((n >> b) & 1u) ? 0x3F80u : 0u) | (((n >> (b + 1)) & 1u) ? 0x3F800000u : 0u);
  }
  if (tid < 32) reinterpret_cast<int*>(smem + V8_FLAGS)[tid] = 0;  // FULL, DONE, CLAIM
  __syncthreads();
  float* slab_spare = slabs + (size_t)blockIdx.x * SLAB_STRIDE + P_TOTAL;  // 192 spare floats per slab
  if (FUSED_STAMPS) ts[1] = __builtin_amdgcn_s_memrealtime();
  uint32_t* tr = FUSED_TRACE ? reinterpret_cast<uint32_t*>(loss_slabs + gridDim.x) : nullptr;
  float* RED = reinterpret_cast<float*>(smem + V8_RED);
  float* DB2S = reinterpret_cast<float*>(smem + V8_DB2S);
  float* LOSSS = reinterpret_cast<float*>(smem + V8_LOSSS);
  bool ok = true;
  Stamps st;
  auto dump = [&]() {
    if (FUSED_STAMPS && lane < 10) {
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 10; ++k) v = (lane == k) ? st.acc[k] : v;
      slab_spare[wave * 16 + lane] = (float)v;
    }
  };
  if (wave < V8_NF) {
    float loss_acc = 0.f;  // (unused: the loss terms go to backward wave 0 with their tile)
    __builtin_amdgcn_s_setprio(V8_FPRIO);
    v8_forward<LOSS, SIDX, VER>(smem, masks, sidx, B, offset, wave, lane, loss_acc, ok, st, tr);
    dump();
    __syncthreads();  // every wave is out of the loop: the loop's LDS is free
    if (lane == 0) LOSSS[wave] = ok ? 0.f : __builtin_nanf("");
    __syncthreads();
  } else {
    const int Q = wave - V8_NF;
    __builtin_amdgcn_s_setprio(V8_BPRIO);
    f32x16 dW2[2] = {f32x16{}, f32x16{}}, dW1T[2] = {f32x16{}, f32x16{}};
    float db2 = 0.f, loss_acc = 0.f;
    // (Q as a template argument: the db2 share bd[Q >> 1][Q & 1] indexed at run time went to scratch)
    if (Q == 0)
      v8_backward<0, VER>(smem, B, lane, dW2, dW1T, db2, loss_acc, ok, st, tr);
    else if (Q == 1)
      v8_backward<1, VER>(smem, B, lane, dW2, dW1T, db2, loss_acc, ok, st, tr);
    else if (Q == 2)
      v8_backward<2, VER>(smem, B, lane, dW2, dW1T, db2, loss_acc, ok, st, tr);
    else
      v8_backward<3, VER>(smem, B, lane, dW2, dW1T, db2, loss_acc, ok, st, tr);
    float lsum = wave_sum(loss_acc);
    if (!ok) lsum = __builtin_nanf("");
    dump();
    __syncthreads();
    DB2S[Q * 64 + lane] = db2;
    if (lane == 0) LOSSS[wave] = lsum;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const f32x16& acc = which ? dW1T[u] : dW2[u];
        const int T = 8 * which + 2 * Q + u;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(RED + v6_red_slot(T, g, lane & 31, lane >> 5) * 4) =
              f32x4{acc[4 * g + 0], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
      }
    __syncthreads();
  }
  if (FUSED_STAMPS) ts[2] = __builtin_amdgcn_s_memrealtime();

  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc(slab, 0, SLAB_STRIDE * 4, 0x00020000);
  for (int e = tid; e < 2048; e += V8_THREADS) {  // W1[f][c..c+3] (see train_v6)
    const int f = e >> 5, c = (e & 31) * 4;
    const int T = 8 + 2 * (c >> 5) + (f >> 5), g = (c & 31) >> 3;
    const f32x4 v = *reinterpret_cast<const f32x4*>(RED + v6_red_slot(T, g, f & 31, (c >> 2) & 1) * 4);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), srd, e * 16, 0, 16 /* sc1 */);
  }
  for (int q = tid; q < 2048; q += V8_THREADS) {  // W2[c + k][o]
    const int T = q >> 8, g = (q >> 6) & 3, L = q & 31, hh = (q >> 5) & 1;
    const f32x4 v = *reinterpret_cast<const f32x4*>(RED + q * 4);
    const int c = 32 * (T >> 1) + 8 * g + 4 * hh, o = mlp::out_logical(32 * (T & 1) + L);  // physical -> logical
    uint32_t vb[4];
    __builtin_memcpy(vb, &v, 16);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_buffer_store_b32(vb[k], srd, (P_W2 + (c + k) * OUT + o) * 4, 0, 16 /* sc1 */);
  }
  if (tid < 64) {  // b2[32u + L]: quarters 2u, 2u + 1 (sample halves) x lane halves, fixed order
    const int u = tid >> 5, L = tid & 31;
    const float v = (DB2S[(2 * u) * 64 + L] + DB2S[(2 * u) * 64 + 32 + L]) +
                    (DB2S[(2 * u + 1) * 64 + L] + DB2S[(2 * u + 1) * 64 + 32 + L]);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), srd, (P_B2 + mlp::out_logical(tid)) * 4, 0,
                                          16 /* sc1 */);
  }
  if (tid == 0) {
    float l = 0.f;
    for (int w = 0; w < V8_NF + V8_NB; ++w) l += LOSSS[w];
    __hip_atomic_store(loss_slabs + blockIdx.x, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (FUSED_STAMPS && tid == 0) {  // wave 0's spare stamp lanes 10..14
    ts[3] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 4; ++k) slab_spare[10 + k] = __builtin_bit_cast(float, (uint32_t)ts[k]);
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    slab_spare[14] = __builtin_bit_cast(float, xcc & 15u);
  }
}

template <int LOSS, bool SIDX, int VER>
__global__ void __launch_bounds__(V8_THREADS, 1)
mlp_fused_train_v8_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                          const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                          float* __restrict__ loss_slabs, int* __restrict__ step) {
  train_v8<LOSS, SIDX, VER>(masks, sidx, B, offset, wimg, slabs, loss_slabs, step);
}

// Slabs only: em_adam_slab reduces them (or the DP paths all-reduce them first).  A one-launch form
// with the slab reduction and Adam inside this kernel was measured 4.3 us per step slower (round 3,
// docs/DESIGN.md §6b) and removed in round 4.
template <int LOSS, bool SIDX>
__device__ __forceinline__ void train_v6(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B,
                                         int offset, const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                                         float* __restrict__ loss_slabs, int* __restrict__ step) {
  // static, not dynamic, LDS: the base is then a link-time-free constant 0, so a data-dependent LUT
  // address folds its table offset into the DS immediate instead of paying a v_add of the LDS base
  __shared__ __attribute__((aligned(16))) char smem[V6_LDS];
  uint64_t ts[4] = {};  // FUSED_STAMPS: 100 MHz wall-clock marks (entry, prologue done, loop done, slab written)
  if (FUSED_STAMPS) ts[0] = __builtin_amdgcn_s_memrealtime();
  if (step && blockIdx.x == 0 && threadIdx.x == 0) {
    // the optimizer's step counter (em_adam_slab pre mode): stream order puts this launch strictly
    // between two Adam launches, so one plain store here saves Adam a grid-wide ticket
    step[0] = step[0] + 1;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  {  // all loads of the weight image in flight before the first LDS store
    constexpr int N16 = IMG_BYTES / 16, KK = (N16 + 511) / 512;
    const u32x4* src = reinterpret_cast<const u32x4*>(wimg);
    u32x4 v[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k)
      if (tid + 512 * k < N16) v[k] = src[tid + 512 * k];
#pragma unroll
    for (int k = 0; k < KK; ++k)
      if (tid + 512 * k < N16) *reinterpret_cast<u32x4*>(smem + v6_img_dst(16u * (tid + 512 * k))) = v[k];
  }
  if (tid < 64) {
    const float bit = (float)(((tid >> 2) >> (tid & 3)) & 1);
    reinterpret_cast<float*>(smem + V6_YLUT)[tid] = bit;
  }
  if (tid < 32) {
    const uint32_t n = (uint32_t)tid >> 1, b = 2u * (tid & 1);
    reinterpret_cast<uint32_t*>(smem + V6_XLUT)[tid] =
        (((n >> b) & 1u) ? 0x3F80u : 0u) | (((n >> (b + 1)) & 1u) ? 0x3F800000u : 0u);
  }
  if (tid < 32) reinterpret_cast<int*>(smem + V6_FLAGS)[tid] = 0;
  __syncthreads();
  // wave w runs on SIMD w % 4, and every SIMD hosts one forward and one backward wave.
  //   shared ring: waves 0-3 forward (first tile w), waves 4-7 backward (rho = (w >> 1) & 1, parity w & 1)
  //   two units: unit 0 = waves 0-3 (F0 F1 B0 B1), unit 1 = waves 4-7 (B0 B1 F0 F1) (pairing F and B of
  //   the same unit on a SIMD measured 1.5 % slower)
  int unit = 0, role, sub;
  if (FUSED_SHARED) {
    role = wave < 4 ? 0 : 2 + ((wave >> 1) & 1);
    sub = wave < 4 ? wave : (wave & 1);
  } else {
    unit = wave >> 2;
    const int r0 = unit == 0 ? (wave & 3) : ((wave & 3) ^ 2);  // 0/1 forward f, 2/3 backward rho
    role = r0 < 2 ? 0 : r0;
    sub = r0 < 2 ? r0 : 0;
  }
  float* slab_spare = slabs + (size_t)blockIdx.x * SLAB_STRIDE + P_TOTAL;  // 192 spare floats per slab
  if (FUSED_STAMPS) ts[1] = __builtin_amdgcn_s_memrealtime();
  if (role == 0)
    v6_body<LOSS, SIDX, 0>(smem, masks, sidx, B, offset, unit, sub, wave, lane, slab_spare);
  else if (role == 2)
    v6_body<LOSS, SIDX, 2>(smem, masks, sidx, B, offset, unit, sub, wave, lane, slab_spare);
  else
    v6_body<LOSS, SIDX, 3>(smem, masks, sidx, B, offset, unit, sub, wave, lane, slab_spare);
  if (FUSED_STAMPS) ts[2] = __builtin_amdgcn_s_memrealtime();

  const float* RED = reinterpret_cast<const float*>(smem);
  const float* DB2S = reinterpret_cast<const float*>(smem + V6_RED);
  const float* LOSSS = reinterpret_cast<const float*>(smem + V6_RED + 512);
  float* slab = slabs + (size_t)blockIdx.x * SLAB_STRIDE;
  // parameter-order slab with write-through (sc1) stores: 16 B for W1, 4 B for W2 / b2
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
    const int c = 32 * (T >> 1) + 8 * g + 4 * hh, o = mlp::out_logical(32 * (T & 1) + L);  // physical -> logical
    uint32_t vb[4];  // memcpy, not a bit_cast of v[k]: see as_s16x2
    __builtin_memcpy(vb, &v, 16);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_buffer_store_b32(vb[k], srd, (P_W2 + (c + k) * OUT + o) * 4, 0, 16 /* sc1 */);
  }
  if (tid < 64)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, DB2S[tid] + DB2S[64 + tid]), srd,
                                          (P_B2 + mlp::out_logical(tid)) * 4, 0, 16 /* sc1 */);
  if (tid == 0) {
    float l = 0.f;
    for (int w = 0; w < 8; ++w) l += LOSSS[w];
    __hip_atomic_store(loss_slabs + blockIdx.x, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (FUSED_STAMPS && tid == 0) {
    ts[3] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int k = 0; k < 4; ++k) slab_spare[128 + k] = __builtin_bit_cast(float, (uint32_t)ts[k]);
    uint32_t xcc;  // which XCD ran this block (HIP promises no placement: recorded, never relied on)
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    slab_spare[132] = __builtin_bit_cast(float, xcc & 15u);
  }
}

// SIDX: samples addressed through sidx (shuffled epochs) instead of offset + s
template <int LOSS, bool SIDX>
__global__ void __launch_bounds__(512, 1)
mlp_fused_train_v6_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int B, int offset,
                          const uint8_t* __restrict__ wimg, float* __restrict__ slabs,
                          float* __restrict__ loss_slabs, int* __restrict__ step) {
  train_v6<LOSS, SIDX>(masks, sidx, B, offset, wimg, slabs, loss_slabs, step);
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
        for (int g = 0; g < 4; ++g) {  // physical nibble n -> logical (mlp_adam.h out_phys): 13 -> 15 rotated
          const int n = 8 * u + 2 * g + h, ln = n <= 12 ? n : n == 13 ? 15 : n - 1;
          // (the pads 62 / 63 read 0, as the parameters say: PAD_B2 exists for the train kernels' softmax only)
          const f32x4 v = n == 13 ? f32x4{z[4 * g + 2], z[4 * g + 3], 0.f, 0.f}
                                  : f32x4{z[4 * g + 0], z[4 * g + 1], z[4 * g + 2], z[4 * g + 3]};
          *reinterpret_cast<f32x4*>(logits + (int64_t)s * OUT + 4 * ln) = v;
        }
      }
    }
  }
}

}  // namespace

EM_API int em_mlp_fused_param_count() { return P_TOTAL; }
EM_API int em_mlp_fused_slab_stride() { return SLAB_STRIDE; }
EM_API int em_mlp_fused_image_bytes() { return IMG_BYTES; }
EM_API int em_mlp_fused_lds_bytes() { return V6_LDS; }

namespace {
template <int LOSS>
void set_lds_attr() {
  // (v6 uses static LDS: nothing to raise)
  (void)hipFuncSetAttribute((const void*)mlp_fused_train_v8_kernel<LOSS, false, 8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, v8_lds<8>());
  (void)hipFuncSetAttribute((const void*)mlp_fused_train_v8_kernel<LOSS, true, 8>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, v8_lds<8>());
  (void)hipFuncSetAttribute((const void*)mlp_fused_train_v8_kernel<LOSS, false, 9>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, v8_lds<9>());
  (void)hipFuncSetAttribute((const void*)mlp_fused_train_v8_kernel<LOSS, true, 9>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, v8_lds<9>());
}
// train kernel generation: EUROM_FUSED_V=8 / 9 selects v8 / v9 (read once per process)
int fused_variant() {
  static const int v = [] {
    const char* e = std::getenv("EUROM_FUSED_V");
    const int x = e ? std::atoi(e) : 6;
    return (x == 8 || x == 9) ? x : 6;
  }();
  return v;
}
int check_train_args(const uint64_t*& draws, const int32_t* sidx, int64_t B, int64_t& offset, const void* wimg,
                     float* slabs, float* loss_slabs, int nslab) {
  if (draws && !sidx && offset > 0) {  // sequential samples: 64-bit offsets (HBM-filling datasets) via the base
    draws += offset;
    offset = 0;
  }
  if (!draws || !wimg || !slabs || !loss_slabs || nslab <= 0 || B < 0 || offset < 0 ||
      B + offset + 1 > (int64_t)INT32_MAX)
    return EM_ERR_ARG;
  static bool attrs = false;
  if (!attrs) {
    set_lds_attr<0>();
    set_lds_attr<1>();
    attrs = true;
  }
  return 0;
}
}  // namespace

// masks: [ndraws] uint64 feature masks; sample s = (masks[i], masks[i+1]) with i = sidx ? sidx[s] : offset+s.
// Writes one gradient slab per workgroup (em_adam_slab reduces them); `step` (optional) is advanced
// by one for em_adam_slab's pre mode.
EM_API int em_mlp_fused_train(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset,
                              const void* wimg, float* slabs, float* loss_slabs, int nslab, int loss_kind,
                              int* step, hipStream_t stream) {
  if (int e = check_train_args(draws, sidx, B, offset, wimg, slabs, loss_slabs, nslab)) return e;
  const int Bi = (int)B, oi = (int)offset;
  const uint8_t* w = (const uint8_t*)wimg;
  const int ver = fused_variant();
  const bool v8 = ver != 6;
  const int lds = ver == 9 ? v8_lds<9>() : ver == 8 ? v8_lds<8>() : 0;  // v6: static LDS
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nslab), dim3(v8 ? V8_THREADS : 512), lds, stream, draws, sidx, Bi, oi, w, slabs,
                       loss_slabs, step);
  };
  if (ver == 9) {
    if (loss_kind == 0)
      sidx ? go(mlp_fused_train_v8_kernel<0, true, 9>) : go(mlp_fused_train_v8_kernel<0, false, 9>);
    else
      sidx ? go(mlp_fused_train_v8_kernel<1, true, 9>) : go(mlp_fused_train_v8_kernel<1, false, 9>);
  } else if (v8) {
    if (loss_kind == 0)
      sidx ? go(mlp_fused_train_v8_kernel<0, true, 8>) : go(mlp_fused_train_v8_kernel<0, false, 8>);
    else
      sidx ? go(mlp_fused_train_v8_kernel<1, true, 8>) : go(mlp_fused_train_v8_kernel<1, false, 8>);
  } else if (loss_kind == 0) {
    sidx ? go(mlp_fused_train_v6_kernel<0, true>) : go(mlp_fused_train_v6_kernel<0, false>);
  } else {
    sidx ? go(mlp_fused_train_v6_kernel<1, true>) : go(mlp_fused_train_v6_kernel<1, false>);
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
                     (int)B, (int)offset, (const uint8_t*)wimg, logits);
  EM_CHECK_LAUNCH();
  return 0;
}
