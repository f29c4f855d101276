// XGBoost-semantics gbtree engine for MI355X (the reference's learner, Main.java:113-141).
//
// Device-resident training: the C++ driver em_gbdt_fit runs every boosting round
// and level on the GPU without host round-trips (XGBoost4J crosses JNI twice per
// round).  T boosters (tasks) train in lock-step, one tree each per
// round.  Kernels:
//   K12 gbdt_grad       g, h per (task, row) for reg:logistic / reg:squarederror
//   K8  gbdt_hist       per-(chunk, task, feature-tile) histograms; each thread owns
//                       one feature's bins in LDS -> no atomics, bitwise deterministic
//   K9  gbdt_split      one wave per (task, node): fixed-order chunk reduction,
//                       64-lane prefix scan over bins, XGBoost loss_chg, arg-max
//                       (lower feature, then lower bin wins ties)
//   K10 gbdt_partition  row -> child node
//       gbdt_finalize   TreePruner (gamma, bottom-up) + leaf = -G/(H+lambda)*eta
//   K12 gbdt_update     margin += leaf(row)
//   K11 gbdt_predict    ensemble traversal over binned rows
//   K13 gbdt_metric     logloss / rmse / error partial sums -> per-round history
// Node numbering is heap order (children 2i+1, 2i+2); status 0 unused / 1 split / 2 leaf.
#include "common.h"

namespace {

constexpr float KRT_EPS = 1e-6f;
enum { OBJ_LOGISTIC = 0, OBJ_SQERR = 1, OBJ_SOFTMAX = 2 };
enum { MET_LOGLOSS = 0, MET_RMSE = 1, MET_ERROR = 2, MET_MLOGLOSS = 3, MET_MERROR = 4 };

// multi:softprob over the T class margins of row r ([T][n] layout), sequential class order
EM_DEVICE float softmax_p(const float* __restrict__ margin, int T, int n, int r, int t) {
  float mx = margin[r];
  for (int k = 1; k < T; ++k) mx = fmaxf(mx, margin[(int64_t)k * n + r]);
  float s = 0.f;
  for (int k = 0; k < T; ++k) s += expf(margin[(int64_t)k * n + r] - mx);
  return expf(margin[(int64_t)t * n + r] - mx) / s;
}

EM_DEVICE uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

// per-round tree reset: status/feature/bin/gain cleared, every task's root opened (status 2)
__global__ void gbdt_round_init(int8_t* __restrict__ st, int16_t* __restrict__ fe, uint8_t* __restrict__ sb,
                                float* __restrict__ gn, int total, int NN) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    st[i] = (i % NN) == 0 ? 2 : 0;
    fe[i] = -1;
    sb[i] = 0;
    gn[i] = 0.f;
  }
}

__global__ void gbdt_init_margin(float* __restrict__ margin, int64_t total, float base) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    margin[i] = base;
}

// margin/g/h/node: [T][n]; Y: [n][T]
__global__ void gbdt_grad(const float* __restrict__ margin, const float* __restrict__ Y, float* __restrict__ g,
                          float* __restrict__ h, int16_t* __restrict__ node, int T, int n, int obj, float subsample,
                          uint32_t seed, int round) {
  const int64_t total = (int64_t)T * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const float m = margin[i], y = Y[(int64_t)r * T + t];
    float gg, hh;
    if (obj == OBJ_LOGISTIC) {
      const float p = 1.f / (1.f + expf(-m));
      gg = p - y;
      hh = fmaxf(p * (1.f - p), 1e-16f);
    } else if (obj == OBJ_SOFTMAX) {  // XGBoost SoftmaxMultiClassObj: g = p - y, h = max(2p(1-p), eps)
      const float p = softmax_p(margin, T, n, r, t);
      gg = p - y;
      hh = fmaxf(2.f * p * (1.f - p), 1e-16f);
    } else {
      gg = m - y;
      hh = 1.f;
    }
    if (subsample < 1.f) {
      const float u = (hash3(seed, (uint32_t)round * 131071u + t, r) >> 8) * (1.f / 16777216.f);
      if (u >= subsample) gg = hh = 0.f;
    }
    g[i] = gg;
    h[i] = hh;
    node[i] = 0;
  }
}

// grid (nchunks, T, nftiles); block = FT threads (one per feature of the tile, padded to 64)
// partial: [nchunks][T][nodesL][F][NB][2]
__global__ void gbdt_hist(const uint8_t* __restrict__ bins, const float* __restrict__ g, const float* __restrict__ h,
                          const int16_t* __restrict__ node, double* __restrict__ partial, int T, int n, int F, int NB,
                          int level, int chunk, int FT) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* hist = reinterpret_cast<double*>(smem);  // sums in double, like XGBoost's GradStats
  const int nodesL = 1 << level, first = nodesL - 1;
  const int c = blockIdx.x, t = blockIdx.y, f0 = blockIdx.z * FT;
  const int fl = threadIdx.x, f = f0 + fl;
  const int per = nodesL * NB * 2;
  const bool active = fl < FT && f < F;
  if (active)
    for (int i = 0; i < per; ++i) hist[fl * per + i] = 0.0;
  const int r0 = c * chunk, r1 = min(n, r0 + chunk);
  // the chunk's per-row (node, g, h) are shared by every feature thread: stage them in LDS once
  // (coalesced), after the per-thread histograms (chunk <= 1024 rows -> 12 KB)
  float* sg = reinterpret_cast<float*>(smem + (size_t)FT * per * sizeof(double));
  float* sh = sg + chunk;
  int16_t* sn = reinterpret_cast<int16_t*>(sh + chunk);
  const int64_t base = (int64_t)t * n;
  for (int r = r0 + (int)threadIdx.x; r < r1; r += blockDim.x) {
    sg[r - r0] = g[base + r];
    sh[r - r0] = h[base + r];
    sn[r - r0] = (int16_t)(node[base + r] - first);
  }
  __syncthreads();
  if (active) {
    double* my = hist + fl * per;
    int r = r0;
    // 8 rows per step: the 8 bin loads are issued before any update (memory-level parallelism);
    // the updates stay in row order, so the sums are bitwise those of the plain loop
    for (; r + 8 <= r1; r += 8) {
      int b[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) b[u] = bins[(int64_t)(r + u) * F + f];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int nd = sn[r + u - r0];
        if (nd < 0 || nd >= nodesL) continue;
        double* e = my + (nd * NB + b[u]) * 2;
        e[0] += (double)sg[r + u - r0];
        e[1] += (double)sh[r + u - r0];
      }
    }
    for (; r < r1; ++r) {
      const int nd = sn[r - r0];
      if (nd < 0 || nd >= nodesL) continue;
      const int b = bins[(int64_t)r * F + f];
      double* e = my + (nd * NB + b) * 2;
      e[0] += (double)sg[r - r0];
      e[1] += (double)sh[r - r0];
    }
  }
  __syncthreads();
  if (active) {
    double* out = partial + ((int64_t)c * T + t) * (int64_t)nodesL * F * NB * 2;
    for (int nd = 0; nd < nodesL; ++nd)
      for (int b = 0; b < NB; ++b) {
        const double* e = hist + fl * per + (nd * NB + b) * 2;
        double* o = out + (((int64_t)nd * F + f) * NB + b) * 2;
        o[0] = e[0];
        o[1] = e[1];
      }
  }
}

// one 64-thread block per (task, node of this level)
// G/H: [T][NN] node totals (in: this level's nodes; out: their children)
__global__ void gbdt_split(const double* __restrict__ partial, int nchunks, int T, int F, int NB, int level, int NN,
                           double* __restrict__ G, double* __restrict__ H, int8_t* __restrict__ status,
                           int16_t* __restrict__ feat, uint8_t* __restrict__ sbin, float* __restrict__ gain, double lam,
                           double mcw) {
  const int nodesL = 1 << level, first = nodesL - 1;
  const int t = blockIdx.x / nodesL, nd = blockIdx.x % nodesL, i = first + nd;
  const int lane = threadIdx.x;
  int8_t* st = status + (int64_t)t * NN;
  if (st[i] != 2) return;
  const int64_t tstride = (int64_t)nodesL * F * NB * 2;
  // node totals: the root sums feature 0 over all bins; other nodes were set by the parent split
  double Gn, Hn;
  if (level == 0) {
    double sg = 0.0, sh = 0.0;
    for (int b = lane; b < NB; b += 64)
      for (int c = 0; c < nchunks; ++c) {
        const double* e = partial + ((int64_t)c * T + t) * tstride + ((int64_t)0 * NB + b) * 2;
        sg += e[0];
        sh += e[1];
      }
    Gn = wave_sum_d(sg);
    Hn = wave_sum_d(sh);
    if (lane == 0) {
      G[(int64_t)t * NN] = Gn;
      H[(int64_t)t * NN] = Hn;
    }
  } else {
    Gn = G[(int64_t)t * NN + i];
    Hn = H[(int64_t)t * NN + i];
  }
  const double root = Gn * Gn / (Hn + lam);
  double best = -INFINITY, bGL = 0.0, bHL = 0.0;
  int bf = -1, bb = 0;
  for (int f = 0; f < F; ++f) {
    double carry_g = 0.0, carry_h = 0.0;
    for (int b0 = 0; b0 < NB; b0 += 64) {
      const int b = b0 + lane;
      double hg = 0.0, hh = 0.0;
      if (b < NB)
        for (int c = 0; c < nchunks; ++c) {
          const double* e = partial + ((int64_t)c * T + t) * tstride + (((int64_t)nd * F + f) * NB + b) * 2;
          hg += e[0];
          hh += e[1];
        }
      // inclusive prefix scan across the wave
      double sg = hg, sh = hh;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double ug = __shfl_up(sg, o), uh = __shfl_up(sh, o);
        if (lane >= o) {
          sg += ug;
          sh += uh;
        }
      }
      const double GL = carry_g + sg, HL = carry_h + sh;
      const double GR = Gn - GL, HR = Hn - HL;
      double gn = -INFINITY;
      if (b < NB - 1 && HL >= mcw && HR >= mcw) gn = GL * GL / (HL + lam) + GR * GR / (HR + lam) - root;
      // wave arg-max: larger gain wins; ties -> lower bin (lane)
      double bv = gn;
      int bl = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o);
        const int ol = __shfl_xor(bl, o);
        if (ov > bv || (ov == bv && ol < bl)) {
          bv = ov;
          bl = ol;
        }
      }
      const double wGL = __shfl(GL, bl), wHL = __shfl(HL, bl);
      if (bv > best) {  // strict: earlier (feature, bin) wins ties
        best = bv;
        bf = f;
        bb = b0 + bl;
        bGL = wGL;
        bHL = wHL;
      }
      carry_g = __shfl(GL, 63);
      carry_h = __shfl(HL, 63);
    }
  }
  if (lane == 0) {
    if (bf >= 0 && best > KRT_EPS) {
      st[i] = 1;
      feat[(int64_t)t * NN + i] = (int16_t)bf;
      sbin[(int64_t)t * NN + i] = (uint8_t)bb;
      gain[(int64_t)t * NN + i] = (float)best;
      const int l = 2 * i + 1, r = 2 * i + 2;
      st[l] = 2;
      st[r] = 2;
      G[(int64_t)t * NN + l] = bGL;
      H[(int64_t)t * NN + l] = bHL;
      G[(int64_t)t * NN + r] = Gn - bGL;
      H[(int64_t)t * NN + r] = Hn - bHL;
    }
  }
}

__global__ void gbdt_partition(const uint8_t* __restrict__ bins, int16_t* __restrict__ node, int T, int n, int F,
                               int NN, const int8_t* __restrict__ status, const int16_t* __restrict__ feat,
                               const uint8_t* __restrict__ sbin, int level) {
  const int first = (1 << level) - 1, last = (1 << (level + 1)) - 1;
  const int64_t total = (int64_t)T * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const int nd = node[i];
    if (nd < first || nd >= last) continue;
    const int64_t k = (int64_t)t * NN + nd;
    if (status[k] != 1) continue;
    const int b = bins[(int64_t)r * F + feat[k]];
    node[i] = (int16_t)(2 * nd + 1 + (b > sbin[k] ? 1 : 0));
  }
}

// one thread per task: prune (gamma) bottom-up, leaf values, cover
__global__ void gbdt_finalize(int T, int NN, int max_depth, int8_t* __restrict__ status, int16_t* __restrict__ feat,
                              const float* __restrict__ gain, const double* __restrict__ G, const double* __restrict__ H,
                              float* __restrict__ leaf, float* __restrict__ cover, double lam, float gamma, double eta) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  int8_t* st = status + (int64_t)t * NN;
  const int64_t o = (int64_t)t * NN;
  for (int i = (1 << max_depth) - 2; i >= 0; --i) {
    if (st[i] == 1 && st[2 * i + 1] == 2 && st[2 * i + 2] == 2 && gain[o + i] < gamma) {
      st[i] = 2;
      st[2 * i + 1] = 0;
      st[2 * i + 2] = 0;
      feat[o + i] = -1;
    }
  }
  for (int i = 0; i < NN; ++i) {
    leaf[o + i] = st[i] == 2 ? (float)(-G[o + i] / (H[o + i] + lam) * eta) : 0.f;
    cover[o + i] = st[i] ? (float)H[o + i] : 0.f;
  }
}

EM_DEVICE int leaf_ancestor(const int8_t* st, int nd) {
  while (nd > 0 && st[nd] != 2) nd = (nd - 1) >> 1;
  return nd;
}

__global__ void gbdt_update(float* __restrict__ margin, const int16_t* __restrict__ node, int T, int n, int NN,
                            const int8_t* __restrict__ status, const float* __restrict__ leaf) {
  const int64_t total = (int64_t)T * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / n);
    const int8_t* st = status + (int64_t)t * NN;
    margin[i] += leaf[(int64_t)t * NN + leaf_ancestor(st, node[i])];
  }
}

// K11: margin[t][r] += sum over trees k in [k0, k1) (task of tree k = k % T) — traversal on bins
__global__ void gbdt_predict(const uint8_t* __restrict__ bins, float* __restrict__ margin, int T, int n, int F, int NN,
                             int k0, int k1, const int8_t* __restrict__ status, const int16_t* __restrict__ feat,
                             const uint8_t* __restrict__ sbin, const float* __restrict__ leaf) {
  const int64_t total = (int64_t)T * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const uint8_t* row = bins + (int64_t)r * F;
    float acc = 0.f;
    for (int k = k0 + ((t - k0 % T) % T + T) % T; k < k1; k += T) {
      const int64_t o = (int64_t)k * NN;
      int nd = 0;
      while (status[o + nd] == 1) nd = 2 * nd + 1 + (row[feat[o + nd]] > sbin[o + nd] ? 1 : 0);
      acc += leaf[o + nd];
    }
    margin[i] += acc;
  }
}

// K13: partial sums per block of the metric over (task,row); Y [n][T], margin [T][n]
__global__ void __launch_bounds__(256)
gbdt_metric(const float* __restrict__ margin, const float* __restrict__ Y, int T, int n, int obj, int metric,
            double* __restrict__ partial) {
  const bool rowwise = metric >= MET_MLOGLOSS;  // multi-class metrics: one term per row
  const int64_t total = rowwise ? (int64_t)n : (int64_t)T * n;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    if (rowwise) {
      const int r = (int)i;
      int lab = 0, am = 0;
      for (int k = 0; k < T; ++k) {
        if (Y[(int64_t)r * T + k] > 0.5f) lab = k;
        if (margin[(int64_t)k * n + r] > margin[(int64_t)am * n + r]) am = k;
      }
      if (metric == MET_MLOGLOSS) {
        const double p = (double)softmax_p(margin, T, n, r, lab);
        acc += -log(fmax(p, 1e-16));
      } else {
        acc += (am != lab) ? 1.0 : 0.0;
      }
      continue;
    }
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const float m = margin[i], y = Y[(int64_t)r * T + t];
    const float p = obj == OBJ_LOGISTIC ? 1.f / (1.f + expf(-m)) : m;
    double v;
    if (metric == MET_LOGLOSS) {
      const double pc = fmin(fmax((double)p, 1e-16), 1.0 - 1e-16);
      v = -(y * log(pc) + (1.0 - y) * log(1.0 - pc));
    } else if (metric == MET_RMSE) {
      v = (double)(p - y) * (double)(p - y);
    } else {
      v = ((p > 0.5f ? 1.f : 0.f) != y) ? 1.0 : 0.0;
    }
    acc += v;
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void gbdt_metric_final(const double* __restrict__ partial, int nb, int64_t count, int metric,
                                  float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) s += partial[i];
  double v = s / (double)(count > 0 ? count : 1);
  if (metric == MET_RMSE) v = sqrt(v);
  out[0] = (float)v;
}

// DP path: fold the per-chunk partial histograms into chunk 0 (fixed order), ready for an all-reduce
__global__ void gbdt_chunk_reduce(double* __restrict__ partial, int nchunks, int64_t S) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < S; e += (int64_t)gridDim.x * blockDim.x) {
    double acc = 0.0;
    for (int c = 0; c < nchunks; ++c) acc += partial[(int64_t)c * S + e];
    partial[e] = acc;
  }
}

__global__ void gbdt_metric_sum(const double* __restrict__ partial, int nb, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) s += partial[i];
  out[0] = s;
}

inline int grid_for(int64_t total, int bs = 256) {
  int64_t g = (total + bs - 1) / bs;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

// ------------------------------------------------------------------ C ABI
struct EmGbdtEval {
  const uint8_t* bins;  // [n][F]
  const float* Y;       // [n][T]
  float* margin;        // [T][n] (initialised by the driver)
  int n;
};

// Trains rounds [r0, r1).  Tree arrays hold ALL rounds: [R*T][NN] (tree k = round*T + task).
// scratch: g, h [T][n]; node int16 [T][n]; partial (see gbdt_hist); G, H [T][NN]; mpart double[4096]
// hist_out: float [R][1 + n_evals] (metric of train + each eval set after each round)
EM_API int em_gbdt_fit(const uint8_t* bins, const float* Y, int n, int F, int NB, int T, float* margin,
                       const EmGbdtEval* evals, int n_evals, int r0, int r1, int max_depth, int obj, int metric,
                       float eta, float lam, float gamma, float mcw, float subsample, uint32_t seed, float* g, float* h,
                       int16_t* node, double* partial, int64_t partial_doubles, double* Gs, double* Hs, double* mpart,
                       int8_t* status, int16_t* feat, uint8_t* sbin, float* leaf, float* gainv, float* cover,
                       float* hist_out, hipStream_t stream) {
  if (!bins || !Y || !margin || n <= 0 || F <= 0 || NB < 1 || NB > 256 || T <= 0 || max_depth < 1 ||
      max_depth > 12 || r0 < 0 || r1 < r0)
    return EM_ERR_ARG;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int chunk = 1024;
  const int nchunks = (n + chunk - 1) / chunk;
  const int64_t TN = (int64_t)T * n;
  for (int round = r0; round < r1; ++round) {
    int8_t* st = status + (int64_t)round * T * NN;
    int16_t* fe = feat + (int64_t)round * T * NN;
    uint8_t* sb = sbin + (int64_t)round * T * NN;
    float* lf = leaf + (int64_t)round * T * NN;
    float* gn = gainv + (int64_t)round * T * NN;
    float* cv = cover + (int64_t)round * T * NN;
    hipLaunchKernelGGL(gbdt_round_init, dim3(grid_for((int64_t)T * NN)), dim3(256), 0, stream, st, fe, sb, gn, T * NN,
                       NN);
    hipLaunchKernelGGL(gbdt_grad, dim3(grid_for(TN)), dim3(256), 0, stream, margin, Y, g, h, node, T, n, obj, subsample,
                       seed, round);
    for (int level = 0; level < max_depth; ++level) {
      const int nodesL = 1 << level;
      // feature tile so that FT * nodesL * NB * 2 floats fit in 64 KB of LDS
      int FT = (int)((65536 - 10240) / ((int64_t)nodesL * NB * 2 * 8));  // + 10 KB row staging <= 64 KB
      if (FT > F) FT = F;
      if (FT > 256) FT = 256;
      if (FT < 1) return EM_ERR_ARG;  // nodesL * NB too large for one thread's LDS slice
      const int64_t need = (int64_t)nchunks * T * nodesL * F * NB * 2;
      if (need > partial_doubles) return EM_ERR_ARG;
      const int nft = (F + FT - 1) / FT;
      const int threads = ((FT + 63) / 64) * 64;
      const size_t lds = (size_t)FT * nodesL * NB * 2 * sizeof(double) + (size_t)chunk * 10;
      hipLaunchKernelGGL(gbdt_hist, dim3(nchunks, T, nft), dim3(threads), lds, stream, bins, g, h, node, partial, T, n,
                         F, NB, level, chunk, FT);
      hipLaunchKernelGGL(gbdt_split, dim3(T * nodesL), dim3(64), 0, stream, partial, nchunks, T, F, NB, level, NN, Gs,
                         Hs, st, fe, sb, gn, (double)lam, (double)mcw);
      hipLaunchKernelGGL(gbdt_partition, dim3(grid_for(TN)), dim3(256), 0, stream, bins, node, T, n, F, NN, st, fe, sb,
                         level);
    }
    hipLaunchKernelGGL(gbdt_finalize, dim3((T + 63) / 64), dim3(64), 0, stream, T, NN, max_depth, st, fe, gn, Gs, Hs,
                       lf, cv, (double)lam, gamma, (double)eta);
    hipLaunchKernelGGL(gbdt_update, dim3(grid_for(TN)), dim3(256), 0, stream, margin, node, T, n, NN, st, lf);
    // metrics (train + evals)
    const int mb_train = grid_for(TN);
    hipLaunchKernelGGL(gbdt_metric, dim3(mb_train), dim3(256), 0, stream, margin, Y, T, n, obj, metric, mpart);
    hipLaunchKernelGGL(gbdt_metric_final, dim3(1), dim3(1), 0, stream, mpart, mb_train,
                       metric >= MET_MLOGLOSS ? (int64_t)n : TN, metric, hist_out + (int64_t)round * (1 + n_evals));
    for (int e = 0; e < n_evals; ++e) {
      const int64_t TE = (int64_t)T * evals[e].n;
      const int64_t k0 = (int64_t)round * T;
      hipLaunchKernelGGL(gbdt_predict, dim3(grid_for(TE)), dim3(256), 0, stream, evals[e].bins, evals[e].margin, T,
                         evals[e].n, F, NN, (int)k0, (int)(k0 + T), status, feat, sbin, leaf);
      const int mb = grid_for(TE);
      hipLaunchKernelGGL(gbdt_metric, dim3(mb), dim3(256), 0, stream, evals[e].margin, evals[e].Y, T, evals[e].n, obj,
                         metric, mpart);
      hipLaunchKernelGGL(gbdt_metric_final, dim3(1), dim3(1), 0, stream, mpart, mb,
                         metric >= MET_MLOGLOSS ? (int64_t)evals[e].n : TE, metric,
                         hist_out + (int64_t)round * (1 + n_evals) + 1 + e);
    }
    EM_CHECK_LAUNCH();
  }
  return 0;
}

EM_API int em_gbdt_init_margin(float* margin, int64_t total, float base, hipStream_t stream) {
  if (!margin || total < 0) return EM_ERR_ARG;
  hipLaunchKernelGGL(gbdt_init_margin, dim3(grid_for(total)), dim3(256), 0, stream, margin, total, base);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_gbdt_predict(const uint8_t* bins, float* margin, int T, int n, int F, int max_depth, int k0, int k1,
                           const int8_t* status, const int16_t* feat, const uint8_t* sbin, const float* leaf,
                           hipStream_t stream) {
  if (!bins || !margin || T <= 0 || n < 0 || max_depth < 1) return EM_ERR_ARG;
  if (n == 0) return 0;
  const int NN = (1 << (max_depth + 1)) - 1;
  hipLaunchKernelGGL(gbdt_predict, dim3(grid_for((int64_t)T * n)), dim3(256), 0, stream, bins, margin, T, n, F, NN, k0,
                     k1, status, feat, sbin, leaf);
  EM_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- data-parallel (C4) primitives
// The single-call driver above runs whole rounds on the stream; under data parallelism the host
// interleaves these per-level steps with an all-reduce of the folded histogram (and of the metric
// sums), so every rank takes identical split decisions on its own row shard.
EM_API int em_gbdt_dp_round_begin(int round, int T, int n, int max_depth, const float* margin, const float* Y, float* g,
                                  float* h, int16_t* node, int obj, float subsample, uint32_t seed, int8_t* status,
                                  int16_t* feat, uint8_t* sbin, float* gainv, hipStream_t stream) {
  if (!margin || !Y || !g || !h || !node || !status || T <= 0 || n <= 0 || max_depth < 1 || max_depth > 12)
    return EM_ERR_ARG;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int64_t TN = (int64_t)T * n;
  hipLaunchKernelGGL(gbdt_round_init, dim3(grid_for((int64_t)T * NN)), dim3(256), 0, stream, status, feat, sbin, gainv,
                     T * NN, NN);
  hipLaunchKernelGGL(gbdt_grad, dim3(grid_for(TN)), dim3(256), 0, stream, margin, Y, g, h, node, T, n, obj, subsample,
                     seed, round);
  EM_CHECK_LAUNCH();
  return 0;
}

// histogram of one level folded into partial[0 : T*2^level*F*NB*2]; returns that length in *len_out
EM_API int em_gbdt_dp_level_hist(int level, const uint8_t* bins, const float* g, const float* h, const int16_t* node,
                                 int T, int n, int F, int NB, double* partial, int64_t partial_doubles,
                                 int64_t* len_out, hipStream_t stream) {
  if (!bins || !g || !h || !node || !partial || !len_out || level < 0 || level > 11) return EM_ERR_ARG;
  const int chunk = 1024;
  const int nchunks = (n + chunk - 1) / chunk;
  const int nodesL = 1 << level;
  int FT = (int)((65536 - 10240) / ((int64_t)nodesL * NB * 2 * 8));  // + 10 KB row staging <= 64 KB
  if (FT > F) FT = F;
  if (FT > 256) FT = 256;
  if (FT < 1) return EM_ERR_ARG;
  const int64_t S = (int64_t)T * nodesL * F * NB * 2;
  if (S * nchunks > partial_doubles) return EM_ERR_ARG;
  const int nft = (F + FT - 1) / FT;
  const int threads = ((FT + 63) / 64) * 64;
  const size_t lds = (size_t)FT * nodesL * NB * 2 * sizeof(double) + (size_t)chunk * 10;
  hipLaunchKernelGGL(gbdt_hist, dim3(nchunks, T, nft), dim3(threads), lds, stream, bins, g, h, node, partial, T, n, F,
                     NB, level, chunk, FT);
  if (nchunks > 1)
    hipLaunchKernelGGL(gbdt_chunk_reduce, dim3(grid_for(S)), dim3(256), 0, stream, partial, nchunks, S);
  EM_CHECK_LAUNCH();
  *len_out = S;
  return 0;
}

EM_API int em_gbdt_dp_level_split(int level, const uint8_t* bins, const double* hist, int T, int n, int F, int NB,
                                  int max_depth, int16_t* node, double* Gs, double* Hs, int8_t* status, int16_t* feat,
                                  uint8_t* sbin, float* gainv, float lam, float mcw, hipStream_t stream) {
  if (!bins || !hist || !node || !Gs || !Hs || !status || level < 0 || level >= max_depth) return EM_ERR_ARG;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int nodesL = 1 << level;
  const int64_t TN = (int64_t)T * n;
  hipLaunchKernelGGL(gbdt_split, dim3(T * nodesL), dim3(64), 0, stream, hist, 1, T, F, NB, level, NN, Gs, Hs, status,
                     feat, sbin, gainv, (double)lam, (double)mcw);
  hipLaunchKernelGGL(gbdt_partition, dim3(grid_for(TN)), dim3(256), 0, stream, bins, node, T, n, F, NN, status, feat,
                     sbin, level);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_gbdt_dp_round_end(int T, int n, int max_depth, float* margin, const int16_t* node, int8_t* status,
                                int16_t* feat, float* gainv, double* Gs, double* Hs, float* leaf, float* cover,
                                float lam, float gamma, float eta, hipStream_t stream) {
  if (!margin || !node || !status || !leaf || T <= 0 || n <= 0) return EM_ERR_ARG;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int64_t TN = (int64_t)T * n;
  hipLaunchKernelGGL(gbdt_finalize, dim3((T + 63) / 64), dim3(64), 0, stream, T, NN, max_depth, status, feat, gainv,
                     Gs, Hs, leaf, cover, (double)lam, gamma, (double)eta);
  hipLaunchKernelGGL(gbdt_update, dim3(grid_for(TN)), dim3(256), 0, stream, margin, node, T, n, NN, status, leaf);
  EM_CHECK_LAUNCH();
  return 0;
}

// sum (not mean) of the per-element metric term over [T][n] margins -> out[0] (double)
EM_API int em_gbdt_metric_sum(const float* margin, const float* Y, int T, int n, int obj, int metric, double* mpart,
                              double* out, hipStream_t stream) {
  if (!margin || !Y || !mpart || !out || T <= 0 || n < 0) return EM_ERR_ARG;
  const int64_t TN = (int64_t)T * n;
  const int mb = grid_for(TN);
  if (n > 0) {
    hipLaunchKernelGGL(gbdt_metric, dim3(mb), dim3(256), 0, stream, margin, Y, T, n, obj, metric, mpart);
    hipLaunchKernelGGL(gbdt_metric_sum, dim3(1), dim3(1), 0, stream, mpart, mb, out);
  } else {
    hipLaunchKernelGGL(gbdt_metric_sum, dim3(1), dim3(1), 0, stream, mpart, 0, out);
  }
  EM_CHECK_LAUNCH();
  return 0;
}
