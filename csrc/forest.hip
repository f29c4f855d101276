// K8/K9/K10/K11 for the random forest: 100 multi-output trees over binary
// (one-hot / multi-hot) features, built level-wise for all trees at once on one MI355X.
//
// The reference only declares Spark MLlib's RandomForest (pom.xml:56-61, README.md:6) and never
// calls it.  Semantics implemented here (Spark-like, multi-output):
//   * bootstrap by Poisson(1) row weights per (tree, row) (Spark's subsampling scheme),
//     drawn from a counter-based hash so host oracle and device agree bit-for-bit;
//   * per-node random feature subset of k features (Spark featureSubsetStrategy);
//   * impurity = sum over the 62 binary outputs of the weighted variance (== Gini / 2), so
//     gain(f) = SL2/nL + SR2/nR - S2/n with integer sums S (exact: weights and labels are
//     integers, gains are evaluated in double from exact integers => the numpy oracle
//     (euromillioner_amd/models/forest.py) reproduces every split exactly);
//   * leaves hold the weighted mean 62-vector (per-output probabilities).
//
// Per level (one C++ driver loop on the stream, em_rf_fit):
//   rf_hist_split  one workgroup per (tree, node): LDS integer histogram hist[f][j] = sum of
//                  w * x_f * y_j over the node's rows (set bits only: <= 7 x 7 LDS atomics per
//                  row for one-hot draws), node totals, then a split scan (one wavefront per
//                  candidate feature, lane j = output j) and the node record;
//   rf_partition   stable-free ballot partition of the node's row list into its children.
// Trees are complete binary arrays: node i has children 2i+1 (x_f = 0) and 2i+2 (x_f = 1).
#include <cstdint>

#include "common.h"

namespace {

constexpr int RF_MAXF = 256;  // features (4 x 64-bit words)
constexpr int RF_NT = 256;

__host__ __device__ inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__host__ __device__ inline uint64_t hash3(uint64_t seed, uint64_t a, uint64_t b) { return mix64(mix64(seed ^ mix64(a)) ^ b); }

// Poisson(1) inverse CDF on a 53-bit uniform (literals shared with models/forest.py)
__device__ inline int poisson1(uint64_t h) {
  const double u = (double)(h >> 11) * 0x1.0p-53;
  const double cdf[9] = {0.36787944117144233, 0.7357588823428847, 0.9196986029286058, 0.9810118431238463,
                         0.9963401531726563, 0.9994058151824183, 0.999916758850712, 0.9999897508033253,
                         0.999998874797402};
  int w = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) w += u >= cdf[k] ? 1 : 0;
  return w;
}

__device__ inline int row_weight(int bootstrap, uint64_t seed, int tree, int64_t row) {
  return bootstrap ? poisson1(hash3(seed, 0x100000000ull + (uint64_t)tree, (uint64_t)row)) : 1;
}

__device__ inline int xbit(const uint64_t* __restrict__ X, int W, int64_t row, int f) {
  return (int)((X[row * W + (f >> 6)] >> (f & 63)) & 1ull);
}

// root row lists: rows with non-zero bootstrap weight, compacted per tree (one block per tree)
__global__ void rf_init_rows(int64_t N, int T, int bootstrap, uint64_t seed, int t_off, int32_t* __restrict__ rows,
                             int32_t* __restrict__ seg, int nodes) {
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ int wcnt[4];
  __shared__ int base;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  int32_t* out = rows + (int64_t)t * N;
  for (int64_t c = 0; c < N; c += RF_NT) {
    const int64_t r = c + threadIdx.x;
    const bool keep = r < N && row_weight(bootstrap, seed, t + t_off, r) > 0;
    const uint64_t bal = __ballot(keep);
    const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
    if (lane == 0) wcnt[wv] = __builtin_popcountll(bal);
    __syncthreads();
    int off = base;
    for (int i = 0; i < wv; ++i) off += wcnt[i];
    if (keep) out[off + pre] = (int32_t)r;
    __syncthreads();
    if (threadIdx.x == 0) base += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
  int32_t* s = seg + (int64_t)t * nodes * 2;
  for (int i = 1 + threadIdx.x; i < nodes; i += RF_NT) {  // everything below the root starts absent
    s[2 * i] = 0;
    s[2 * i + 1] = -1;
  }
  if (threadIdx.x == 0) {
    s[0] = 0;
    s[1] = base;
  }
}

struct RfParams {
  const uint64_t* X;
  const uint64_t* Y;
  int64_t N;
  int W, F, T, max_depth, k_feat, min_leaf, bootstrap, t_off, nodes;
  uint64_t seed;
  int32_t* seg;   // [T][nodes][2] (start, count; count -1 = node absent)
  int16_t* feat;  // [T][nodes]  -1 leaf, -2 absent, else split feature
  float* value;   // [T][nodes][64]
  double* gain;   // [T][nodes]
  float* cover;   // [T][nodes] weighted count
};

__global__ void __launch_bounds__(RF_NT) rf_hist_split(RfParams p, const int32_t* __restrict__ rows, int level) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* hist = lds;                       // [F][64]
  uint32_t* cnt = hist + p.F * 64;            // [F]
  uint32_t* S = cnt + p.F;                    // [4 waves][64]
  __shared__ uint32_t nw[4];
  __shared__ int cand[RF_MAXF];
  __shared__ double bgain[4];
  __shared__ int bfeat[4];
  const int t = blockIdx.y;
  const int node = (1 << level) - 1 + blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  const int start = sg[0], count = sg[1];
  int16_t* fo = p.feat + (int64_t)t * p.nodes + node;
  if (count < 0) {  // absent node (below a leaf)
    if (tid == 0) *fo = -2;
    return;
  }
  for (int i = tid; i < p.F * 64 + p.F + 4 * 64; i += RF_NT) lds[i] = 0u;
  __syncthreads();
  const int32_t* rl = rows + (int64_t)t * p.N + start;
  uint32_t my_n = 0;
  for (int i = tid; i < count; i += RF_NT) {
    const int64_t r = rl[i];
    const uint32_t w = (uint32_t)row_weight(p.bootstrap, p.seed, t + p.t_off, r);
    if (!w) continue;
    my_n += w;
    const uint64_t y = p.Y[r] & ((1ull << 62) - 1);
    uint64_t yy = y;
    while (yy) {
      const int j = __builtin_ctzll(yy);
      yy &= yy - 1;
      atomicAdd(&S[wv * 64 + j], w);
    }
    for (int wd = 0; wd < p.W; ++wd) {
      uint64_t xx = p.X[r * p.W + wd];
      while (xx) {
        const int f = wd * 64 + __builtin_ctzll(xx);
        xx &= xx - 1;
        if (f >= p.F) break;
        atomicAdd(&cnt[f], w);
        uint64_t y2 = y;
        while (y2) {
          const int j = __builtin_ctzll(y2);
          y2 &= y2 - 1;
          atomicAdd(&hist[f * 64 + j], w);
        }
      }
    }
  }
  // weighted node size
  uint32_t nsum = my_n;
  for (int o = 32; o > 0; o >>= 1) nsum += __shfl_xor(nsum, o);
  if (lane == 0) nw[wv] = nsum;
  // candidate features (partial Fisher-Yates on a hashed stream), by one thread
  if (tid == 0) {
    for (int i = 0; i < p.F; ++i) cand[i] = i;
    for (int i = 0; i < p.k_feat && i < p.F; ++i) {
      const uint64_t h = hash3(p.seed ^ 0x5EEDF00Dull, ((uint64_t)(t + p.t_off) << 32) | (uint64_t)node, (uint64_t)i);
      const int j = i + (int)(h % (uint64_t)(p.F - i));
      const int tmp = cand[i];
      cand[i] = cand[j];
      cand[j] = tmp;
    }
  }
  __syncthreads();
  const uint32_t n = nw[0] + nw[1] + nw[2] + nw[3];
  // node record: weighted mean of the outputs (leaf value / diagnostics)
  const uint32_t Sj = lane < 62 ? S[lane] + S[64 + lane] + S[128 + lane] + S[192 + lane] : 0u;
  if (wv == 0) {
    float* vo = p.value + ((int64_t)t * p.nodes + node) * 64;
    vo[lane] = (n > 0 && lane < 62) ? (float)((double)Sj / (double)n) : 0.f;
  }
  if (tid == 0) p.cover[(int64_t)t * p.nodes + node] = (float)n;
  const bool can_split = level < p.max_depth && n >= (uint32_t)(2 * p.min_leaf) && n > 0;
  double best = 0.0;
  int bf = -1;
  if (can_split) {
    // S2 = sum_j S_j^2 (exact integer)
    uint64_t s2 = (uint64_t)Sj * Sj;
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const int kk = p.k_feat < p.F ? p.k_feat : p.F;
    for (int c = wv; c < kk; c += 4) {
      const int f = cand[c];
      const uint32_t nR = cnt[f], nL = n - nR;
      const uint32_t SR = lane < 62 ? hist[f * 64 + lane] : 0u;
      const uint32_t SL = Sj - SR;
      uint64_t aL = (uint64_t)SL * SL, aR = (uint64_t)SR * SR;
      for (int o = 32; o > 0; o >>= 1) {
        aL += __shfl_xor(aL, o);
        aR += __shfl_xor(aR, o);
      }
      if (nL < (uint32_t)p.min_leaf || nR < (uint32_t)p.min_leaf || nL == 0 || nR == 0) continue;
      const double g = (double)aL / (double)nL + (double)aR / (double)nR - (double)s2 / (double)n;
      if (g > best || (g == best && bf >= 0 && f < bf)) {
        best = g;
        bf = f;
      }
    }
    if (lane == 0) {
      bgain[wv] = best;
      bfeat[wv] = bf;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int f = -1;
    double g = 0.0;
    if (can_split) {
      for (int i = 0; i < 4; ++i) {
        if (bfeat[i] < 0) continue;
        if (f < 0 || bgain[i] > g || (bgain[i] == g && bfeat[i] < f)) {
          g = bgain[i];
          f = bfeat[i];
        }
      }
      // a split must reduce impurity by more than rounding noise
      if (f >= 0 && !(g > 1e-9 * (1.0 + g))) f = -1;
    }
    *fo = (int16_t)f;
    p.gain[(int64_t)t * p.nodes + node] = f >= 0 ? g : 0.0;
  }
}

// children row lists: left (x_f = 0) fills from the segment start, right from its end
__global__ void __launch_bounds__(RF_NT) rf_partition(RfParams p, const int32_t* __restrict__ rin,
                                                      int32_t* __restrict__ rout, int level) {
  const int t = blockIdx.y;
  const int node = (1 << level) - 1 + blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  const int start = sg[0], count = sg[1];
  const int f = p.feat[(int64_t)t * p.nodes + node];
  const bool has_children = 2 * node + 2 < p.nodes;
  if (f < 0 || count < 0) {
    if (threadIdx.x == 0 && has_children) {
      int32_t* c = p.seg + ((int64_t)t * p.nodes + 2 * node + 1) * 2;
      c[0] = 0; c[1] = -1; c[2] = 0; c[3] = -1;
    }
    return;
  }
  __shared__ int lc[4], rc[4];
  __shared__ int lbase, rbase;
  if (threadIdx.x == 0) {
    lbase = 0;
    rbase = 0;
  }
  __syncthreads();
  const int32_t* ri = rin + (int64_t)t * p.N + start;
  int32_t* ro = rout + (int64_t)t * p.N + start;
  for (int c = 0; c < count; c += RF_NT) {
    const int i = c + threadIdx.x;
    const bool live = i < count;
    const int32_t r = live ? ri[i] : 0;
    const bool right = live && xbit(p.X, p.W, r, f);
    const bool left = live && !right;
    const uint64_t bl = __ballot(left), br = __ballot(right);
    const int pl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0));
    const int pr = __builtin_amdgcn_mbcnt_hi((uint32_t)(br >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)br, 0));
    if (lane == 0) {
      lc[wv] = __builtin_popcountll(bl);
      rc[wv] = __builtin_popcountll(br);
    }
    __syncthreads();
    int lo = lbase, roff = rbase;
    for (int k = 0; k < wv; ++k) {
      lo += lc[k];
      roff += rc[k];
    }
    if (left) ro[lo + pl] = r;
    if (right) ro[count - 1 - (roff + pr)] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
      lbase += lc[0] + lc[1] + lc[2] + lc[3];
      rbase += rc[0] + rc[1] + rc[2] + rc[3];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && has_children) {
    int32_t* ch = p.seg + ((int64_t)t * p.nodes + 2 * node + 1) * 2;
    ch[0] = start;
    ch[1] = lbase;
    ch[2] = start + lbase;
    ch[3] = rbase;
  }
}

// mean of leaf vectors over trees: one wavefront per row, lane j = output j
__global__ void rf_predict(const uint64_t* __restrict__ X, int W, int64_t N, const int16_t* __restrict__ feat,
                           const float* __restrict__ value, int T, int nodes, int out_logit, float* __restrict__ out,
                           int ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= N) return;
  float acc = 0.f;
  for (int t = 0; t < T; ++t) {
    const int16_t* ft = feat + (int64_t)t * nodes;
    int nd = 0;
    int f = ft[0];
    while (f >= 0) {
      nd = 2 * nd + 1 + xbit(X, W, r, f);
      f = ft[nd];
    }
    acc += value[((int64_t)t * nodes + nd) * 64 + lane];
  }
  float pr = T > 0 ? acc / (float)T : 0.f;
  if (out_logit) {
    const float pc = fminf(fmaxf(pr, 1e-7f), 1.f - 1e-7f);
    pr = lane < 62 ? __logf(pc / (1.f - pc)) : -30.f;
  } else if (lane >= 62) {
    pr = 0.f;
  }
  out[r * ldo + lane] = pr;
}

}  // namespace

EM_API int em_rf_nodes(int max_depth) { return (1 << (max_depth + 1)) - 1; }

EM_API int em_rf_lds_bytes(int F) { return (F * 64 + F + 4 * 64) * 4; }

// Native level-wise driver: all T trees advance one level per (hist_split, partition) pair.
EM_API int em_rf_fit(const uint64_t* X, int W, const uint64_t* Y, int64_t N, int F, int T, int max_depth, int k_feat,
                     int min_leaf, int bootstrap, uint64_t seed, int t_off, int32_t* rows_a, int32_t* rows_b,
                     int32_t* seg, int16_t* feat, float* value, double* gain, float* cover, hipStream_t stream) {
  if (!X || !Y || !rows_a || !rows_b || !seg || !feat || !value || !gain || !cover) return EM_ERR_ARG;
  if (W < 1 || F < 1 || F > RF_MAXF || F > 64 * W || T < 1 || max_depth < 0 || max_depth > 14 || k_feat < 1 ||
      min_leaf < 1 || N < 1 || N >= (1ll << 31))
    return EM_ERR_ARG;
  const int nodes = (1 << (max_depth + 1)) - 1;
  const int lds = em_rf_lds_bytes(F);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rf_hist_split, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 4096);
    attr = true;
  }
  RfParams p{X, Y, N, W, F, T, max_depth, k_feat, min_leaf, bootstrap, t_off, nodes, seed, seg, feat, value, gain, cover};
  hipLaunchKernelGGL(rf_init_rows, dim3(T), dim3(RF_NT), 0, stream, N, T, bootstrap, seed, t_off, rows_a, seg, nodes);
  EM_CHECK_LAUNCH();
  int32_t* rin = rows_a;
  int32_t* rout = rows_b;
  for (int level = 0; level <= max_depth; ++level) {
    const dim3 grid(1u << level, (unsigned)T);
    hipLaunchKernelGGL(rf_hist_split, grid, dim3(RF_NT), lds, stream, p, rin, level);
    EM_CHECK_LAUNCH();
    if (level == max_depth) break;
    hipLaunchKernelGGL(rf_partition, grid, dim3(RF_NT), 0, stream, p, rin, rout, level);
    EM_CHECK_LAUNCH();
    int32_t* tmp = rin;
    rin = rout;
    rout = tmp;
  }
  return 0;
}

EM_API int em_rf_predict(const uint64_t* X, int W, int64_t N, const int16_t* feat, const float* value, int T,
                         int max_depth, int out_logit, float* out, int ldo, hipStream_t stream) {
  if (!X || !feat || !value || !out || W < 1 || N < 0 || T < 0 || ldo < 64 || max_depth < 0 || max_depth > 14)
    return EM_ERR_ARG;
  if (N == 0) return 0;
  const int nodes = (1 << (max_depth + 1)) - 1;
  hipLaunchKernelGGL(rf_predict, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, stream, X, W, N, feat, value, T, nodes,
                     out_logit, out, ldo);
  EM_CHECK_LAUNCH();
  return 0;
}
