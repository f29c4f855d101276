// HBM-resident synthetic draw datasets: draws generated on the GPU directly as 8-byte feature masks.
//
// This replaces the reference's acquisition stage, an HTTP scrape of the results table
// (Main.java:37-67), for the north star's "288 GB of HBM per GPU" data sizes.
// The host generator is one sequential splitmix64 stream, so it cannot fill HBM in reasonable time.
// Here the sequence is cut into independent segments, and one thread generates each segment.
// The specification, including the RNG call order, is euromillioner_amd/data/device_gen.py
// (generate_masks_py); this kernel reproduces it bit for bit (tests/test_device_gen_gpu.py).
//
// Mask layout (as em_rows_to_masks): bit n-1 = main number n (1..50), bit 49+s = star s (1..12).
// Each thread keeps 16 masks (one 128-B line) in registers and stores them as eight 16-B pieces
// back to back.  A wave's 64 lines are then completed within eight store instructions, so the L2
// merges them into whole-line writes.  Generation runs at close to HBM write bandwidth.
#include "common.h"

namespace {

constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull, SEG_SALT = 0xD1B54A32D192ED03ull;
constexpr uint64_t MAIN_BITS = (1ull << 50) - 1;

EM_DEVICE uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct SplitMix {
  uint64_t s;
  EM_DEVICE uint64_t next() {
    s += GOLDEN;
    return mix64(s);
  }
  EM_DEVICE uint32_t range(uint32_t k) { return (uint32_t)(((next() >> 32) * (uint64_t)k) >> 32); }
};

EM_DEVICE uint64_t gen_one(SplitMix& g, uint64_t prev, bool planted, uint32_t thr, const uint8_t* P) {
  uint64_t mask = 0;
  if (planted) {
    uint64_t b = prev & MAIN_BITS;  // previous mains, ascending
    while (b) {
      const int k = __builtin_ctzll(b);
      b &= b - 1;
      if ((uint32_t)(g.next() >> 40) < thr) mask |= 1ull << (P[k] - 1);
    }
  }
  while (__builtin_popcountll(mask & MAIN_BITS) < 5) mask |= 1ull << g.range(50);
  if (planted) {
    uint64_t b = prev >> 50;  // previous stars, ascending
    while (b) {
      const int k = __builtin_ctzll(b);
      b &= b - 1;
      if ((uint32_t)(g.next() >> 40) < thr) mask |= 1ull << (49 + P[50 + k]);
    }
  }
  while (__builtin_popcountll(mask >> 50) < 2) mask |= 1ull << (50 + g.range(12));
  return mask;
}

constexpr int GEN_T = 256, GEN_LINE = 16;  // masks per 128-B line

__global__ void __launch_bounds__(GEN_T)
gen_masks_kernel(uint64_t seed, uint32_t thr, int64_t n, int64_t seg_len, int64_t nseg, int64_t seg0,
                 const int32_t* __restrict__ perm, uint64_t* __restrict__ out) {
  __shared__ uint8_t P[64];
  if (threadIdx.x < 62) P[threadIdx.x] = (uint8_t)perm[threadIdx.x];
  __syncthreads();
  const int64_t seg = (int64_t)blockIdx.x * GEN_T + threadIdx.x;
  if (seg >= nseg) return;
  // global segment index seg0 + seg: a shard of one long sequence starts at draw seg0 * seg_len
  SplitMix g{mix64(seed ^ ((uint64_t)(seg0 + seg + 1) * SEG_SALT))};
  const int64_t t0 = seg * seg_len, t1 = (t0 + seg_len < n) ? t0 + seg_len : n;
  uint64_t prev = 0;
  bool first = true;
  for (int64_t t = t0; t < t1; t += GEN_LINE) {
    uint64_t buf[GEN_LINE];
#pragma unroll
    for (int j = 0; j < GEN_LINE; ++j) {
      if (t + j < t1) {
        prev = gen_one(g, prev, !first && thr != 0, thr, P);
        first = false;
      }
      buf[j] = prev;
    }
    if (t + GEN_LINE <= t1) {
      u32x4* dst = reinterpret_cast<u32x4*>(out + t);
#pragma unroll
      for (int j = 0; j < GEN_LINE / 2; ++j)
        dst[j] = u32x4{(uint32_t)buf[2 * j], (uint32_t)(buf[2 * j] >> 32), (uint32_t)buf[2 * j + 1],
                       (uint32_t)(buf[2 * j + 1] >> 32)};
    } else {
      for (int j = 0; j < GEN_LINE && t + j < t1; ++j) out[t + j] = buf[j];
    }
  }
}

}  // namespace

// masks[n] (int64, 16-B aligned) <- draws [seg0 * seg_len, seg0 * seg_len + n) of the segmented synthetic
// sequence (seg0 > 0: a rank's shard of one sequence); seg_len must be a multiple of 16
EM_API int em_gen_masks_at(uint64_t seed, uint32_t planted_thr, int64_t n, int64_t seg_len, int64_t seg0,
                           const int32_t* perm, uint64_t* out, hipStream_t stream) {
  if (n <= 0 || seg_len <= 0 || seg_len % GEN_LINE || seg0 < 0 || !perm || !out || ((uintptr_t)out & 15))
    return EM_ERR_ARG;
  if (planted_thr > (1u << 24)) return EM_ERR_ARG;
  const int64_t nseg = (n + seg_len - 1) / seg_len;
  const int64_t nb = (nseg + GEN_T - 1) / GEN_T;
  if (nb > 0x7FFFFFFF) return EM_ERR_ARG;
  hipLaunchKernelGGL(gen_masks_kernel, dim3((unsigned)nb), dim3(GEN_T), 0, stream, seed, planted_thr, n, seg_len,
                     nseg, seg0, perm, out);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_gen_masks(uint64_t seed, uint32_t planted_thr, int64_t n, int64_t seg_len, const int32_t* perm,
                        uint64_t* out, hipStream_t stream) {
  return em_gen_masks_at(seed, planted_thr, n, seg_len, 0, perm, out, stream);
}
