// Shared CDNA4 (gfx950) helpers for euromillioner_amd native kernels.
//
// Everything here is written for wave64 / MFMA 32x32x16 bf16 on MI355X.  No
// CUDA shims, no dual paths.  Fragment-layout facts used across the kernels
// (cdna_hip_programming.md §3, verified by the A=I / asymmetric-B tests in
// tests/test_native_numerics.py):
//   A operand (32x32x16): lane l, r=l&31, h=l>>5 holds A[row r][k=8h+j], j=0..7
//   B operand           : lane l holds B[k=8h+j][col r]
//   C/D                 : col = l&31, row = (reg&3) + 8*(reg>>2) + 4*h
//   accumulator-as-operand: regs 8s..8s+7 of a 32x32 f32 tile, cvt to bf16, are
//   the k-step-s fragment with element j <-> tile row perm(s,h,j) below.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define EM_LDS __attribute__((address_space(3)))

#define EM_DEVICE __device__ __forceinline__

// k-row of a chained accumulator fragment (see header comment).
EM_DEVICE constexpr int acc_perm(int s, int h, int j) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

EM_DEVICE f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

EM_DEVICE uint16_t f2bf_bits(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) at -O3
  return __builtin_bit_cast(uint16_t, b);
}

EM_DEVICE float bf2f(__bf16 b) { return (float)b; }

EM_DEVICE float bf16_bits_to_f32(uint16_t u) { return __builtin_bit_cast(float, ((uint32_t)u) << 16); }

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// 2 f32 -> packed bf16 pair: ONE v_cvt_pk_bf16_f32 (element-wise (__bf16) casts compile to two
// single-lane converts plus a v_perm_b32 on ROCm 7.2)
EM_DEVICE uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// 8 f32 -> bf16x8 fragment (4 v_cvt_pk_bf16_f32)
EM_DEVICE bf16x8 pack8(float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7) {
  const u32x4 d = {pack2(a0, a1), pack2(a2, a3), pack2(a4, a5), pack2(a6, a7)};
  return __builtin_bit_cast(bf16x8, d);
}

// Expand 8 mask bits into 8 bf16 {0,1} values (element j = bit j).
EM_DEVICE bf16x8 bits_to_bf16x8(uint32_t b) {
  u32x4 d;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t lo = (b >> (2 * q)) & 1u, hi = (b >> (2 * q + 1)) & 1u;
    d[q] = lo * 0x3F80u | hi * 0x3F800000u;
  }
  return __builtin_bit_cast(bf16x8, d);
}

// LDS: ds_read_b128 of a bf16 fragment at byte offset
EM_DEVICE bf16x8 lds_frag(const char* lds_base, uint32_t byte_off) {
  return *reinterpret_cast<const bf16x8*>(lds_base + byte_off);
}

// Byte offset of entry `nib` (0..15, bits 4+ of `word >> sh` ignored) of a 16-entry LDS table at LUT with
// 2^SH-byte entries: shift + mask, the base in the DS instruction's 16-bit immediate when the table sits
// below 64K and the LDS base is a compile-time constant (static __shared__); otherwise a third VALU adds it
template <int LUT, int SH>
EM_DEVICE uint32_t lut_off(uint32_t word, int sh) {
  return (uint32_t)LUT + (__builtin_amdgcn_ubfe(word, sh, 4) << SH);
}

// Byte BYTE of v, shifted left by SH, in ONE VALU (SDWA source select): the byte-per-entry form of a
// table lookup when the byte already holds (entry + table_base >> SH).  The operand is a plain VALU
// result (no MFMA hazard for the recognizer to miss), so inline asm is safe here.
template <int BYTE, int SH>
EM_DEVICE uint32_t sdwa_byte_shl(uint32_t v) {
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%3"
      : "=v"(r)
      : "v"(v), "i"(SH), "i"(BYTE));
  return r;
}

// ds_read_b64_tr_b16: 4 rows x 16 cols block per 16-lane group, column-major to lanes
EM_DEVICE s16x4 lds_tr16(const char* lds_base, uint32_t byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((EM_LDS s16x4*)(lds_base + byte_off));
}

EM_DEVICE bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// Wave-local LDS ordering (writes by some lanes, reads by other lanes of the SAME wave).
EM_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Combine lanes l and l ^ 32 (the two k-halves that share an MFMA 32x32 accumulator column) with one
// v_permlane32_swap (VALU) instead of a ds_bpermute LDS round trip.  With vdst = src = v the swap
// leaves r[0] = v[l & 31] and r[1] = v[(l & 31) + 32] in every lane, so both halves compute the same
// expression in the same operand order: bitwise-identical results.
EM_DEVICE float xhalf_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
EM_DEVICE float xhalf_max(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

// max without the NaN canonicalisation the compiler puts in front of fmaxf (IEEE maxNum) on operands it
// cannot prove canonical (a v_max_f32 x, x each, e.g. after a permlane or a phi): IEEE-754-2019 maximum
// (NaN-propagating), which gfx950 runs as v_maximum3_f32 with no canonicalisation.  (An inline-asm
// v_max3_f32 was tried first: the hazard recognizer does not see asm operands, so it read MFMA results
// before they were written -- caught by tests/test_xgmi_proxy_gpu.py's bit-identity check.)
EM_DEVICE float raw_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
EM_DEVICE float raw_max3(float a, float b, float c) { return raw_max(raw_max(a, b), c); }
EM_DEVICE float xhalf_max_raw(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return raw_max(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

EM_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

EM_DEVICE double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

EM_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5 T1).
EM_DEVICE int xcd_remap(int bid, int nwg) {
  const int nxcd = 8;
  int q = nwg / nxcd, r = nwg % nxcd, xcd = bid % nxcd;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / nxcd;
}

// Error codes returned by C-ABI launchers (0 = ok, >0 = hipError_t, <0 = ours)
#define EM_ERR_ARG (-1)
#define EM_CHECK_LAUNCH()                       \
  do {                                          \
    hipError_t _e = hipGetLastError();          \
    if (_e != hipSuccess) return (int)_e;       \
  } while (0)

#define EM_API extern "C" __attribute__((visibility("default")))
