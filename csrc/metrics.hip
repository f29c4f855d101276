// K13 metric reductions + K14 multi-hot encoder for 62-wide draw vectors.
//
// The reference prints only `checkPredicts` (exact equality of two prediction
// arrays, Main.java:143,150-162) and logs XGBoost's per-round logloss
// (Main.java:124,128-134).  The README's "0.9+" (README.md:5) needs a defined
// metric, so we compute, per validation sample and in one pass over the logits:
//   loss            the training loss (grouped softmax-CE or BCE)
//   acc             element-wise accuracy of the structured prediction
//                   (top-5 main numbers + top-2 stars set to 1)
//   acc_thr         element-wise accuracy of p >= 0.5 per output
//   hits_main/star  |top-5 ∩ target main|, |top-2 ∩ target stars|
//   exact           the whole 62-vector predicted exactly
//   trivial         element-wise accuracy of the all-zero prediction (0.887 floor)
// Samples are read as 64-bit feature masks (see em_rows_to_masks).
// Partial sums per 256-sample block -> [nblocks][8] (summed on the host side in fp64).
#include "common.h"

namespace {

constexpr uint64_t MAIN_BITS = (1ull << 50) - 1;
constexpr uint64_t STAR_BITS = ((1ull << 12) - 1) << 50;

EM_DEVICE uint64_t draw_mask8(const uint8_t* row) {
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t n = row[k];
    m |= (n >= 1 && n <= 50) ? (1ull << (n - 1)) : 0ull;
  }
#pragma unroll
  for (int k = 5; k < 7; ++k) {
    const uint32_t s = row[k];
    m |= (s >= 1 && s <= 12) ? (1ull << (49 + s)) : 0ull;
  }
  return m;
}

template <int K>
EM_DEVICE uint64_t topk_mask(const float* z, int lo, int hi) {
  float bv[K];
  int bi[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { bv[k] = -3.0e38f; bi[k] = lo; }
  for (int o = lo; o < hi; ++o) {
    float v = z[o];
    int id = o;
#pragma unroll
    for (int k = 0; k < K; ++k) {  // insertion (stable: earlier index wins ties)
      const bool sw = v > bv[k];
      const float tv = bv[k];
      const int ti = bi[k];
      bv[k] = sw ? v : tv;
      bi[k] = sw ? id : ti;
      v = sw ? tv : v;
      id = sw ? ti : id;
    }
  }
  uint64_t m = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) m |= 1ull << bi[k];
  return m;
}

__global__ void __launch_bounds__(256)
draw_metrics_kernel(const float* __restrict__ logits, int ld, const uint64_t* __restrict__ masks,
                    const int32_t* __restrict__ sidx, int64_t B, int64_t offset, int loss_kind,
                    float* __restrict__ partials) {
  __shared__ float red[4][8];
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (s < B) {
    const int64_t idx = sidx ? (int64_t)sidx[s] : offset + s;
    const uint64_t tm = masks[idx + 1] & (MAIN_BITS | STAR_BITS);
    float z[64];
    const f32x4* zr = reinterpret_cast<const f32x4*>(logits + s * ld);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const f32x4 v = zr[k];
      z[4 * k] = v[0]; z[4 * k + 1] = v[1]; z[4 * k + 2] = v[2]; z[4 * k + 3] = v[3];
    }
    const int nm = __builtin_popcountll(tm & MAIN_BITS), ns = __builtin_popcountll(tm & STAR_BITS);
    uint64_t thr = 0;
    float loss = 0.f;
    if (loss_kind == 0) {
      float mm = -3.0e38f, ms = -3.0e38f;
      for (int o = 0; o < 50; ++o) mm = fmaxf(mm, z[o]);
      for (int o = 50; o < 62; ++o) ms = fmaxf(ms, z[o]);
      float sm = 0.f, ss = 0.f;
      for (int o = 0; o < 50; ++o) sm += __expf(z[o] - mm);
      for (int o = 50; o < 62; ++o) ss += __expf(z[o] - ms);
      const float lsm = mm + __logf(sm), lss = ms + __logf(ss);
      for (int o = 0; o < 62; ++o) {
        const float lp = z[o] - (o < 50 ? lsm : lss);
        if (lp >= -0.69314718f) thr |= 1ull << o;
        if ((tm >> o) & 1ull) loss -= lp / (float)(o < 50 ? nm : ns);
      }
    } else {
      for (int o = 0; o < 62; ++o) {
        const float v = z[o];
        const float y = ((tm >> o) & 1ull) ? 1.f : 0.f;
        if (v >= 0.f) thr |= 1ull << o;
        loss += (fmaxf(v, 0.f) + __logf(1.f + __expf(-fabsf(v))) - y * v) * (1.f / 62.f);
      }
    }
    const uint64_t pred = topk_mask<5>(z, 0, 50) | topk_mask<2>(z, 50, 62);
    const int hm = __builtin_popcountll(pred & tm & MAIN_BITS), hs = __builtin_popcountll(pred & tm & STAR_BITS);
    const int mism = __builtin_popcountll(pred ^ tm), mism_thr = __builtin_popcountll(thr ^ tm);
    st[0] = loss;
    st[1] = (62.f - mism) / 62.f;
    st[2] = (62.f - mism_thr) / 62.f;
    st[3] = (float)hm;
    st[4] = (float)hs;
    st[5] = mism == 0 ? 1.f : 0.f;
    st[6] = (62.f - (float)(nm + ns)) / 62.f;
    st[7] = 1.f;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float v = wave_sum(st[k]);
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int k = threadIdx.x;
    partials[blockIdx.x * 8 + k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  }
}

// draw rows [n][8] -> 64-bit feature masks (the on-device sample format of every draw kernel)
__global__ void rows_to_masks_kernel(const uint8_t* __restrict__ rows, int64_t n, uint64_t* __restrict__ masks) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) masks[i] = draw_mask8(rows + i * 8);
}

// K14: feature masks -> multi-hot bf16 [B][64] (optional constant-1 bias feature at 62)
template <typename T>
__global__ void onehot_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int64_t B,
                              int64_t offset, int which, int with_bias, T* __restrict__ out) {
  // one thread per (sample, 8-feature chunk): 16-byte (bf16) / 2x16-byte (fp32) stores
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * 8) return;
  const int64_t s = e >> 3;
  const int c = (int)(e & 7);
  const int64_t idx = (sidx ? (int64_t)sidx[s] : offset + s) + which;
  uint64_t m = masks[idx] & (MAIN_BITS | STAR_BITS);
  if (with_bias) m |= 1ull << 62;
  const uint32_t b = (uint32_t)(m >> (8 * c)) & 0xFFu;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<bf16x8*>(out + s * 64 + c * 8) = bits_to_bf16x8(b);
  } else {
    f32x4* o = reinterpret_cast<f32x4*>(out + s * 64 + c * 8);
    o[0] = f32x4{(float)(b & 1u), (float)((b >> 1) & 1u), (float)((b >> 2) & 1u), (float)((b >> 3) & 1u)};
    o[1] = f32x4{(float)((b >> 4) & 1u), (float)((b >> 5) & 1u), (float)((b >> 6) & 1u), (float)((b >> 7) & 1u)};
  }
}

// K14 with a lag window (data.lags > 1): row s = [onehot(masks[i]) | onehot(masks[i+1]) | ... |
// onehot(masks[i+lags-1])] with i = sidx ? sidx[s] : offset + s, each block 64 wide (62 live + 2 pad),
// row stride 64 * lags.  The matching target is masks[i + lags] (the trainer passes masks + lags - 1 to
// the loss/metric kernels, whose target is their masks[i + 1]).  This is the multi-hot lag window of
// data/draws.lag_features, built on the device from 8-byte masks.
template <typename T>
__global__ void onehot_lags_kernel(const uint64_t* __restrict__ masks, const int32_t* __restrict__ sidx, int64_t B,
                                   int64_t offset, int lags, T* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (sample, block, 8-feature chunk)
  const int64_t per = (int64_t)lags * 8;
  if (e >= B * per) return;
  const int64_t s = e / per;
  const int r = (int)(e - s * per), k = r >> 3, c = r & 7;
  const int64_t idx = (sidx ? (int64_t)sidx[s] : offset + s) + k;
  const uint32_t b = (uint32_t)((masks[idx] & (MAIN_BITS | STAR_BITS)) >> (8 * c)) & 0xFFu;
  T* o = out + s * 64 * lags + 64 * k + 8 * c;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<bf16x8*>(o) = bits_to_bf16x8(b);
  } else {
    f32x4* q = reinterpret_cast<f32x4*>(o);
    q[0] = f32x4{(float)(b & 1u), (float)((b >> 1) & 1u), (float)((b >> 2) & 1u), (float)((b >> 3) & 1u)};
    q[1] = f32x4{(float)((b >> 4) & 1u), (float)((b >> 5) & 1u), (float)((b >> 6) & 1u), (float)((b >> 7) & 1u)};
  }
}

// K10: loss + dL/dlogits for the GEMM-path MLPs.  16 lanes per sample, lane q = outputs 4q..4q+3
// (one 16-B load of the logit row per lane: a wave reads 4 whole rows), group statistics as
// 16-lane butterfly reductions, grid-stride over 4-sample wave groups.  Outputs 62/63 are padding
// (dz = 0).  dz is written already scaled by grad_scale (1/global_batch) as the next GEMM's operand
// type; partials[w] = the loss of samples 4w..4w+3 summed in sample order.
EM_DEVICE float g16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
  return v;
}
EM_DEVICE float g16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 16));
  return v;
}

template <typename T>  // dz element type: __bf16 (bf16 GEMM path) or float (fp32 path)
__global__ void __launch_bounds__(256)
loss_grad_kernel(const float* __restrict__ logits, int ld, const uint64_t* __restrict__ masks,
                 const int32_t* __restrict__ sidx, int64_t B, int64_t offset, int loss_kind, float grad_scale,
                 T* __restrict__ dz, int ldz, float* __restrict__ partials, float* __restrict__ colpart) {
  // colpart (optional): this block's column sums of the written dz (as T-rounded values) ->
  // colpart[blockIdx.x][64], fixed order (lane's samples in loop order, then the 4 sample slots of a
  // wave, then the block's 4 waves): the last layer's bias gradient without another pass over dz
  const int lane = threadIdx.x & 63, q = lane & 15, sub = lane >> 4;
  const int64_t ngroups = (B + 3) / 4;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; gw < ngroups;
       gw += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t s = gw * 4 + sub;
    const bool ok = s < B;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    uint64_t tm = 0;
    if (ok) {
      const int64_t idx = sidx ? (int64_t)sidx[s] : offset + s;
      tm = masks[idx + 1] & (MAIN_BITS | STAR_BITS);
      if ((ld & 3) == 0) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(logits + s * ld + 4 * q);
        z[0] = v[0]; z[1] = v[1]; z[2] = v[2]; z[3] = v[3];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) z[k] = 4 * q + k < 62 ? logits[s * ld + 4 * q + k] : 0.f;
      }
    }
    float y[4], g[4];
    bool live[4], mn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = 4 * q + k;
      live[k] = o < 62;
      mn[k] = o < 50;
      y[k] = live[k] ? (float)((tm >> o) & 1ull) : 0.f;
      if (!live[k]) z[k] = 0.f;
    }
    float loss = 0.f;
    if (loss_kind == 0) {
      float am = -INFINITY, as = -INFINITY;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (mn[k]) am = fmaxf(am, z[k]);
        else if (live[k]) as = fmaxf(as, z[k]);
      }
      const float mx_m = g16_max(am), mx_s = g16_max(as);
      float e[4], sm = 0.f, ss = 0.f, ym = 0.f, ys = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        e[k] = live[k] ? __expf(z[k] - (mn[k] ? mx_m : mx_s)) : 0.f;
        if (mn[k]) {
          sm += e[k];
          ym += y[k];
        } else {
          ss += e[k];
          ys += y[k];
        }
      }
      const float se_m = g16_sum(sm), se_s = g16_sum(ss), sy_m = g16_sum(ym), sy_s = g16_sum(ys);
      const float inv_m = 1.f / fmaxf(sy_m, 1.f), inv_s = 1.f / fmaxf(sy_s, 1.f);
      const float lse_m = mx_m + __logf(se_m), lse_s = mx_s + __logf(se_s);
      float l = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float se = mn[k] ? se_m : se_s, sy = mn[k] ? sy_m : sy_s, inv = mn[k] ? inv_m : inv_s;
        g[k] = live[k] ? (e[k] / se * sy - y[k]) * inv : 0.f;
        l += live[k] ? -y[k] * (z[k] - (mn[k] ? lse_m : lse_s)) * inv : 0.f;
      }
      loss = g16_sum(l);
    } else {
      float l = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float sg = 1.f / (1.f + __expf(-z[k]));
        g[k] = live[k] ? (sg - y[k]) * (1.f / 62.f) : 0.f;
        l += live[k] ? fmaxf(z[k], 0.f) - z[k] * y[k] + __logf(1.f + __expf(-fabsf(z[k]))) : 0.f;
      }
      loss = g16_sum(l) * (1.f / 62.f);
    }
    if (ok) {
      T d4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        d4[k] = (T)(g[k] * grad_scale);
        cs[k] += (float)d4[k];
      }
      T* d = dz + s * ldz + 4 * q;
      if ((ldz & 3) == 0) {  // one 16-B (fp32) / 8-B (bf16) store per lane
        if constexpr (sizeof(T) == 4) {
          f32x4 v;
          __builtin_memcpy(&v, d4, 16);
          *reinterpret_cast<f32x4*>(d) = v;
        } else {
          uint64_t v;
          __builtin_memcpy(&v, d4, 8);
          *reinterpret_cast<uint64_t*>(d) = v;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = d4[k];
      }
    }
    // the wave's 4 sample losses in sample order (a sample past B contributes +0)
    const float l0 = __shfl(loss, 0), l1 = __shfl(loss, 16), l2 = __shfl(loss, 32), l3 = __shfl(loss, 48);
    const int64_t s0 = gw * 4;
    if (lane == 0)
      partials[gw] = ((l0 + (s0 + 1 < B ? l1 : 0.f)) + (s0 + 2 < B ? l2 : 0.f)) + (s0 + 3 < B ? l3 : 0.f);
  }
  if (colpart) {
    __shared__ float red[4][64];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = cs[k];
      v += __shfl_xor(v, 16);  // the wave's 4 sample slots (sub) of output 4q + k
      v += __shfl_xor(v, 32);
      if (sub == 0) red[w][4 * q + k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 64)
      colpart[(int64_t)blockIdx.x * 64 + threadIdx.x] =
          ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  }
}

}  // namespace

EM_API int em_draw_metrics(const float* logits, int ld, const uint64_t* draws, const int32_t* sidx, int64_t B,
                           int64_t offset, int loss_kind, float* partials, hipStream_t stream) {
  if (!logits || !draws || !partials || ld < 64 || (ld & 3) || B < 0) return EM_ERR_ARG;
  if (B == 0) return 0;
  const int64_t nb = (B + 255) / 256;
  hipLaunchKernelGGL(draw_metrics_kernel, dim3((unsigned)nb), dim3(256), 0, stream, logits, ld, draws, sidx, B,
                     offset, loss_kind, partials);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_rows_to_masks(const uint8_t* rows, int64_t n, uint64_t* masks, hipStream_t stream) {
  if (!rows || !masks || n < 0) return EM_ERR_ARG;
  if (n == 0) return 0;
  hipLaunchKernelGGL(rows_to_masks_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, rows, n, masks);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_onehot_encode(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset, int which,
                            int with_bias, void* out, hipStream_t stream) {
  if (!draws || !out || B < 0) return EM_ERR_ARG;
  if (B == 0) return 0;
  const int64_t n = B * 8;
  hipLaunchKernelGGL(onehot_kernel<__bf16>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, draws, sidx, B,
                     offset, which, with_bias, (__bf16*)out);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_onehot_encode_f32(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset, int which,
                                int with_bias, float* out, hipStream_t stream) {
  if (!draws || !out || B < 0) return EM_ERR_ARG;
  if (B == 0) return 0;
  const int64_t n = B * 8;
  hipLaunchKernelGGL(onehot_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, draws, sidx, B,
                     offset, which, with_bias, out);
  EM_CHECK_LAUNCH();
  return 0;
}

namespace {
// 16 samples per 256-thread block; at most 4096 blocks (16 per CU), grid-stride beyond
// (em_loss_grad_blocks: the colpart row count)
unsigned loss_grad_blocks(int64_t B) {
  const int64_t nb = (B + 15) / 16;
  return (unsigned)(nb < 4096 ? nb : 4096);
}
}  // namespace

EM_API int em_loss_grad_blocks(int64_t B) { return B > 0 ? (int)loss_grad_blocks(B) : 0; }

EM_API int em_loss_grad(const float* logits, int ld, const uint64_t* masks, const int32_t* sidx, int64_t B,
                        int64_t offset, int loss_kind, float grad_scale, void* dz, int ldz, float* partials,
                        float* colpart, hipStream_t stream) {
  if (!logits || !masks || !dz || !partials || ld < 62 || ldz < 64 || B < 0 || loss_kind < 0 || loss_kind > 1)
    return EM_ERR_ARG;
  if (B == 0) return 0;
  hipLaunchKernelGGL(loss_grad_kernel<__bf16>, dim3(loss_grad_blocks(B)), dim3(256), 0, stream, logits, ld, masks,
                     sidx, B, offset, loss_kind, grad_scale, (__bf16*)dz, ldz, partials, colpart);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_loss_grad_f32(const float* logits, int ld, const uint64_t* masks, const int32_t* sidx, int64_t B,
                            int64_t offset, int loss_kind, float grad_scale, float* dz, int ldz, float* partials,
                            float* colpart, hipStream_t stream) {
  if (!logits || !masks || !dz || !partials || ld < 62 || ldz < 64 || B < 0 || loss_kind < 0 || loss_kind > 1)
    return EM_ERR_ARG;
  if (B == 0) return 0;
  hipLaunchKernelGGL(loss_grad_kernel<float>, dim3(loss_grad_blocks(B)), dim3(256), 0, stream, logits, ld, masks,
                     sidx, B, offset, loss_kind, grad_scale, dz, ldz, partials, colpart);
  EM_CHECK_LAUNCH();
  return 0;
}

// lag-window multi-hot [B][64 * lags] (bf16 if fp32 == 0, else fp32)
EM_API int em_onehot_lags(const uint64_t* draws, const int32_t* sidx, int64_t B, int64_t offset, int lags, int fp32,
                          void* out, hipStream_t stream) {
  if (!draws || !out || B < 0 || lags < 1 || lags > 64) return EM_ERR_ARG;
  if (B == 0) return 0;
  const int64_t n = B * lags * 8;
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (fp32)
    hipLaunchKernelGGL(onehot_lags_kernel<float>, dim3(nb), dim3(256), 0, stream, draws, sidx, B, offset, lags,
                       (float*)out);
  else
    hipLaunchKernelGGL(onehot_lags_kernel<__bf16>, dim3(nb), dim3(256), 0, stream, draws, sidx, B, offset, lags,
                       (__bf16*)out);
  EM_CHECK_LAUNCH();
  return 0;
}
