// Shared between csrc/adam.hip (K6, the standalone fused Adam launches) and csrc/mlp_fused.hip (K7's
// in-launch Adam epilogue): the flat parameter layout of the 62->128->62 MLP, the LDS-ready bf16
// weight images the train kernel reads, and torch.optim.Adam's update.  The reference's only
// optimizer is libxgboost's Newton boosting (Main.java:137-138); Adam comes from the declared but
// unused DL4J updater (pom.xml:62-66).
#pragma once
#include "common.h"

namespace mlp {

constexpr int IN = 64, HID = 128, OUT = 64;
constexpr int P_W1 = 0, P_W2 = IN * HID, P_B2 = P_W2 + HID * OUT, P_TOTAL = P_B2 + OUT;  // 16448
// weight images with padded rows (144 B / 272 B: 16 consecutive rows start in distinct 16-B bank
// groups, so the 16-lane phases of ds_read_b128 are conflict-free)
constexpr int W1T_RS = 144, W2P_RS = 272, W2Q_RS = 144;
constexpr int IMG_W1T = 0, IMG_W2P = IMG_W1T + 128 * W1T_RS, IMG_W2Q = IMG_W2P + 64 * W2P_RS,
              IMG_B2 = IMG_W2Q + 128 * W2Q_RS, IMG_BYTES = IMG_B2 + 256;  // 54528

// Physical output order of the weight images (W2P rows, W2Q k index, b2): the train kernels hold a
// 32-sample tile's logits with output 32u + 8g + 4h + (i & 3) in register i = 4g + (i & 3) of lane half
// h, so lane halves h = 0 / 1 share a register for physical nibbles 2m / 2m + 1.  Logical nibbles 13, 14
// (stars 52-59) move to physical 14, 15 and logical nibble 15 (stars 60, 61, pads 62, 63) to physical
// 13, rotated by two: every register then has ONE class (main / star) in both lane halves -- main 0-51
// incl. the pads, which carry b2 = PAD_B2 in the image (exp underflows to 0, never the max, target 0)
// -- and the softmax drops its lane-half selects (csrc/mlp_loss.h SOFTMAX_PERM).  Targets are permuted
// the same way per sample (phys_targets_hi).  Nibble-granular, so f32x4 logit stores stay aligned.
EM_DEVICE constexpr int out_phys(int o) {
  return o < 52 ? o : o < 60 ? o + 4 : o < 62 ? o - 6 : o - 10;
}
EM_DEVICE constexpr int out_logical(int p) {
  return p < 52 ? p : p < 54 ? p + 10 : p < 56 ? p + 6 : p - 4;
}
static_assert(out_logical(out_phys(52)) == 52 && out_logical(out_phys(61)) == 61 && out_logical(out_phys(62)) == 62 &&
                  out_phys(60) == 54 && out_phys(62) == 52 && out_phys(59) == 63,
              "output permutation");
constexpr float PAD_B2 = -1.0e30f;  // image value of the pad logits' bias

// W2Q granule swizzle: rows with (row & 15) in 4..11 swap granules k8 ^ 1.  K7's 16x16x32 backward wave
// (mlp_fused.hip v6_backward) reads granule 4 kk + g in lane group g = lane >> 4 from row (lane & 15); the
// ds_read_b128 lane groups {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} then mix rows 4-11 of one granule
// with rows 0-3 / 12-15 of its neighbour, and at 144-B rows (9 16-B units) those collide on a bank unless
// the neighbour granules of rows 4-11 trade places (tools/lds_conflicts.py, tests/test_lds_model.py).
EM_DEVICE constexpr int w2q_swz(int row) { return ((row + 4) >> 3) & 1; }

// true for padding slots that must stay exactly zero (W1 row 63, W2 cols 62/63, b2[62/63])
EM_DEVICE bool pad_slot(int p) {
  if (p < P_W2) return (p >> 7) == 63;
  if (p < P_B2) return ((p - P_W2) & 63) >= 62;
  return (p - P_B2) >= 62;
}

// write parameter p (value val) into the bf16 weight images (fp32 for b2)
EM_DEVICE void pack_one(int p, float val, uint8_t* img) {
  const uint16_t b = f2bf_bits(val);
  if (p < P_W2) {  // W1[f][c] -> W1T image row c, feature f
    const int f = p >> 7, c = p & 127;
    const uint32_t off = IMG_W1T + c * W1T_RS + (f >> 3) * 16 + (f & 7) * 2;
    *reinterpret_cast<uint16_t*>(img + off) = b;
  } else if (p < P_B2) {  // W2[c][o], o at its physical position
    const int q = p - P_W2, c = q >> 6, o = out_phys(q & 63);
    {  // W2P: row o, hid c = 32t + perm(s,h,j)
      const int t = c >> 5, cc = c & 31, s = cc >> 4, a = (cc >> 3) & 1, hh = (cc >> 2) & 1, bb = cc & 3;
      const int j = 4 * a + bb, k16 = (2 * t + s) * 2 + hh;
      *reinterpret_cast<uint16_t*>(img + IMG_W2P + o * W2P_RS + k16 * 16 + j * 2) = b;
    }
    {  // W2Q: row c, out o = 32u + perm(s,h,j)
      const int u = o >> 5, oo = o & 31, s = oo >> 4, a = (oo >> 3) & 1, hh = (oo >> 2) & 1, bb = oo & 3;
      const int j = 4 * a + bb, k8 = (2 * u + s) * 2 + hh;
      *reinterpret_cast<uint16_t*>(img + IMG_W2Q + c * W2Q_RS + (k8 ^ w2q_swz(c)) * 16 + j * 2) = b;
    }
  } else {
    const int o = p - P_B2;
    *reinterpret_cast<float*>(img + IMG_B2 + out_phys(o) * 4) = o >= 62 ? PAD_B2 : val;
  }
}

}  // namespace mlp

// 1 - beta^t, as torch.optim.Adam computes it (Python float64 math, rounded once): beta^t by binary
// exponentiation in fp64 (<= 2 log2(t) multiplies, a few ulp), so the early steps' corrections are
// exact to fp32 rounding instead of losing ~1e-4 to the cancellation of a native exp2/log2 form.
EM_DEVICE float bias_correction(float beta, int t) {
  double b = (double)beta, r = 1.0;
  for (unsigned e = (unsigned)(t > 0 ? t : 0); e; e >>= 1) {
    if (e & 1u) r *= b;
    b *= b;
  }
  return (float)(1.0 - r);
}

// torch.optim.Adam (L2 weight decay folded into g) for one parameter: returns the new value and
// updates the moments in place
EM_DEVICE float adam_math(float g, float w, float& m, float& v, float lr, float b1, float b2, float eps, float wd,
                          float bc1, float bc2) {
  g += wd * w;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  return w - lr * (m / bc1) / (sqrtf(v / bc2) + eps);
}
