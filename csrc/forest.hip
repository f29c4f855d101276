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
#include <cstdlib>
#include <type_traits>

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
// u = m * 2^-53 with m = h >> 11 < 2^53, so u >= cdf[k] <=> m >= cdf[k] * 2^53, an exact integer for
// every cdf[k] below: the same weights from 9 integer compares (no fp64 conversion or compares)
__device__ inline int poisson1(uint64_t h) {
  const uint64_t m = h >> 11;
  const uint64_t th[9] = {0xbc5ab1b16779cull,  0x178b56362cef38ull, 0x1d6e2bc3b82b06ull,
                          0x1f6472f2e6944bull, 0x1fe204beb22e9cull, 0x1ffb21e77480acull,
                          0x1fff516e3f8e59ull, 0x1fffea81812296ull, 0x1ffffda3e9551eull};
  int w = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) w += m >= th[k] ? 1 : 0;
  return w;
}

__device__ inline int row_weight(int bootstrap, uint64_t seed, int tree, int64_t row) {
  return bootstrap ? poisson1(hash3(seed, 0x100000000ull + (uint64_t)tree, (uint64_t)row)) : 1;
}

// Row-list entries carry the row's bootstrap weight (1..9, computed once in rf_init_rows) in bits
// 27..30 when N < 2^27, so the per-level kernels skip the hash + Poisson inverse CDF per row.
constexpr int RF_WSHIFT = 27;
constexpr int32_t RF_RMASK = (1 << RF_WSHIFT) - 1;
__device__ inline bool rf_packed(int64_t N) { return N <= RF_RMASK; }

__device__ inline int xbit(const uint64_t* __restrict__ X, int W, int64_t row, int f) {
  return (int)((X[row * W + (f >> 6)] >> (f & 63)) & 1ull);
}

// Row lists come in two forms.  Index form (int32, any W): the row id, with the bootstrap weight in
// bits 27..30 when N < 2^27; every level gathers X[r] and Y[r] at random.  Record form (W == 1,
// N < 2^27): the row's data itself, 16 B = {x | w_hi << 62, y | w_lo << 62} (x, y: 62 feature / output
// bits, w: 4-bit bootstrap weight), so each level streams its nodes' rows contiguously and the
// partition moves records instead of indices (MI355X: the deep levels were bound by the 8-B random
// gathers -- 4.4 ms of a 4.5 ms level at 64 nodes per tree -- not by the histogram arithmetic).
constexpr uint64_t RF_M62 = (1ull << 62) - 1;
struct RfRec {
  uint64_t x, y;
};
EM_DEVICE RfRec rf_make_rec(uint64_t x, uint64_t y, uint32_t w) {
  return RfRec{(x & RF_M62) | ((uint64_t)(w >> 2) << 62), (y & RF_M62) | ((uint64_t)(w & 3u) << 62)};
}
EM_DEVICE uint32_t rf_rec_w(const RfRec& r) { return (uint32_t)((r.x >> 62) << 2 | (r.y >> 62)); }

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
  int16_t* cand;  // [T][2^max_depth][k] candidate features of the current level's nodes
  uint32_t* acc;  // [T][2^max_depth][rec] per-node integer sums of the current level (see rec_words)
  int32_t* lrc;   // [T][2^max_depth][2] partition counters (left, right) of the current level
  const int32_t* yover;  // fused driver: 0 = every row has <= 7 outputs (position-form records), else 1
};

// per-node record of integer sums: S[64] (sum of w*y_j), n (sum of w), 3 pad, cnt[kp] (sum of w*x_f
// per candidate), hist[k][64] (sum of w*x_f*y_j) -- exact, so block partials merge with atomics in
// any order and the split decision is independent of row order and of the block count
__host__ __device__ inline int rec_words(int k) { return 68 + ((k + 3) & ~3) + 64 * k; }
// The fused partition's LDS image of a child's cnt / hist words, replicated by lane so the lanes of one
// atomic mostly hit distinct words: cnt [RF_REP_CNT][kp + 1] (lane & 15), hist [RF_REP_HIST][k * 64 + 16]
// (lane & 3; the +16 pad moves a replica's output j to another bank).  Summed at the merge.
#ifndef RF_REP_CNT
#define RF_REP_CNT 16
#endif
#ifndef RF_REP_HIST
#define RF_REP_HIST 4
#endif
__host__ __device__ inline int rf_rep_cnt_stride(int k) { return ((k + 3) & ~3) + 1; }
__host__ __device__ inline int rf_rep_hist_stride(int k) { return 64 * k + 16; }
__host__ __device__ inline int rf_chl_words(int k) {
  return RF_REP_CNT * rf_rep_cnt_stride(k) + RF_REP_HIST * rf_rep_hist_stride(k);
}

// A row's output bits, extracted once per row: the first 8 positions (-1 = none) + the rest (rows with
// more than 8 set outputs; a drawn row has 7).  Every candidate bit of the row then adds to its output
// words with 8 branch-free atomics (an absent position adds 0 to pad word 63: exact integers) instead
// of a divergent bit-walk loop per candidate -- the loop's ~13 instructions per output were the
// histogram's cost, not the atomics.
#ifndef RF_YBITS
#define RF_YBITS 1
#endif
// RF_CNT62: the fused partition counts a candidate's rows (cnt) as output word 62 of its histogram row
// (no output uses it), so a drawn row's 7 outputs + its count are exactly the 8 unrolled atomics
#ifndef RF_CNT62
#define RF_CNT62 1
#endif
struct RfYBits {
  int j[8];
  uint64_t rest;
};
EM_DEVICE RfYBits rf_ybits(uint64_t y) {
  RfYBits b;
  uint64_t yy = y;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    b.j[q] = yy ? (int)__builtin_ctzll(yy) : -1;
    yy &= yy - 1;
  }
  b.rest = yy;
  return b;
}
EM_DEVICE void rf_add_ybits(uint32_t* __restrict__ row, const RfYBits& b, uint32_t w) {
#pragma unroll
  for (int q = 0; q < 8; ++q) atomicAdd(&row[b.j[q] & 63], b.j[q] >= 0 ? w : 0u);
  for (uint64_t r = b.rest; r; r &= r - 1) atomicAdd(&row[__builtin_ctzll(r)], w);
}

// Position-form records (the fused driver, when no row has more than 7 outputs -- a draw has 5 + 2):
// the y word holds the row's output positions instead of its output mask, extracted once by
// rf_init_rows -- p0..p4 in bits 0..29, p5, p6 in bits 32..43 (6 bits each, absent = 63: the pad
// word), w_lo in bits 62..63 as before.  Every level's histogram then reads the positions with 7 bit-field
// extracts instead of re-extracting them from the mask (~11 VALU per output per row per level: the
// partition was VALU-issue bound).  rf_ycheck decides the form on the device (no host sync).
constexpr int RF_NPOS = 7;
struct RfPos {
  uint32_t o[RF_NPOS];  // output positions (63 = none)
};
EM_DEVICE RfPos rf_pos_extract(uint64_t y) {  // y: the output mask (bits 0..61)
  RfPos p;
  uint64_t yy = y | (1ull << 63);  // sentinel: an exhausted mask yields 63
#pragma unroll
  for (int q = 0; q < RF_NPOS; ++q) {
    p.o[q] = (uint32_t)__builtin_ctzll(yy);
    yy = (yy & (yy - 1)) | (1ull << 63);
  }
  return p;
}
EM_DEVICE uint64_t rf_pos_pack(const RfPos& p) {
  const uint32_t lo = p.o[0] | p.o[1] << 6 | p.o[2] << 12 | p.o[3] << 18 | p.o[4] << 24;
  const uint32_t hi = p.o[5] | p.o[6] << 6;
  return (uint64_t)lo | (uint64_t)hi << 32;
}
EM_DEVICE RfPos rf_pos_unpack(uint64_t yw) {
  const uint32_t lo = (uint32_t)yw, hi = (uint32_t)(yw >> 32);
  RfPos p;
#pragma unroll
  for (int q = 0; q < 5; ++q) p.o[q] = (lo >> (6 * q)) & 63u;
  p.o[5] = hi & 63u;
  p.o[6] = (hi >> 6) & 63u;
  return p;
}
// a candidate bit's histogram row: the 7 outputs + the row count as output word 62 (RF_CNT62 layout)
EM_DEVICE void rf_add_pos(uint32_t* __restrict__ row, const RfPos& p, uint32_t w) {
#pragma unroll
  for (int q = 0; q < RF_NPOS; ++q) atomicAdd(&row[p.o[q]], w);
  atomicAdd(&row[62], w);
}
static_assert(RF_YBITS && RF_CNT62, "position-form records assume the count-as-word-62 layout");

__global__ void __launch_bounds__(256) rf_ycheck(const uint64_t* __restrict__ Y, int64_t N, int32_t* __restrict__ over) {
  int o = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x)
    o |= __builtin_popcountll(Y[i] & RF_M62) > RF_NPOS ? 1 : 0;
  if (__ballot(o) && (threadIdx.x & 63) == 0) atomicOr(over, 1);
}
// Root row lists: rows with non-zero bootstrap weight, compacted per tree by (blocks x tree)
// workgroups; each 256-row chunk reserves its output range with one atomic (row order inside a list
// is irrelevant: every sum is an exact integer).  Root count -> lrc[t][0][0].
// ROOTH (record rows, the fused driver): the root's histogram record (S, n, candidate cnt / hist) is
// accumulated while the rows are listed -- the root histogram pass re-read every record (700 MB at
// 700 k rows x 100 trees) -- in an LDS image per block, added to the zeroed root record at the end.
EM_DEVICE void rf_node_cands_wave(const RfParams& p, int t, int node, int16_t* __restrict__ co);
#ifndef RF_INIT_RR
#define RF_INIT_RR 4
#endif
// RF_INIT_REP: the position-form root sums go to lane-replicated LDS images (S by lane & 15, the
// candidate histograms by lane & 3) summed at the merge: a wave's q-th smallest outputs crowd a few
// words (the smallest drawn number), and same-word atomics serialise
#ifndef RF_INIT_REP
#define RF_INIT_REP 1
#endif
#ifndef RF_IREP_S
#define RF_IREP_S 16
#endif
#ifndef RF_IREP_H
#define RF_IREP_H 4
#endif
__host__ __device__ inline int rf_init_lds_words(int k) {
  return ((rec_words(k) + 3) & ~3) + (RF_INIT_REP ? RF_IREP_S * 64 + RF_IREP_H * rf_rep_hist_stride(k) : 0);
}
template <bool REC, bool ROOTH = false>
__global__ void __launch_bounds__(RF_NT) rf_init_rows(RfParams p, void* __restrict__ rows_v) {
  // chunks of RR x RF_NT rows: every thread hashes RR rows (all hashes / loads in flight), one count
  // exchange and one atomic reservation per chunk; the count arrays are double-buffered, so a chunk
  // costs two barriers (was three per RF_NT rows)
  constexpr int RR = RF_INIT_RR;
  const int t = blockIdx.y, B = gridDim.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ int wcnt[2][RR][4];
  __shared__ int base[2];
  extern __shared__ __attribute__((aligned(16))) uint32_t rlds[];  // ROOTH: [rec] image
  __shared__ int8_t rslot[64];
  __shared__ uint64_t rmask;
  __shared__ int16_t rco[RF_MAXF];
  const int k = p.k_feat, rec = rec_words(k), kp = (k + 3) & ~3;
  const bool pos = ROOTH && p.yover && *p.yover == 0;
  uint32_t my_n = 0;
  uint32_t* Sr = rlds + ((rec + 3) & ~3);  // RF_INIT_REP images: S [16][64], candidate hist [4][hst]
  uint32_t* Hr = Sr + RF_IREP_S * 64;
  const int hst = rf_rep_hist_stride(k);
  if constexpr (ROOTH) {
    for (int i = threadIdx.x; i < rf_init_lds_words(k); i += blockDim.x) rlds[i] = 0u;
    if (threadIdx.x < 64) rslot[threadIdx.x] = -1;
    if (wv == 0) rf_node_cands_wave(p, t, 0, rco);
    __syncthreads();
    if (blockIdx.x == 0 && p.max_depth > 0)  // the root's candidates for rf_split (rf_level_begin draws none)
      for (int i = threadIdx.x; i < (k < p.F ? k : p.F); i += blockDim.x) p.cand[(int64_t)t * k + i] = rco[i];
    if (threadIdx.x == 0) {
      uint64_t m = 0;
      const int kk = k < p.F ? k : p.F;
      for (int i = 0; i < kk; ++i) {
        rslot[rco[i]] = (int8_t)i;
        m |= 1ull << rco[i];
      }
      rmask = p.max_depth > 0 ? m : 0ull;
    }
    __syncthreads();
  }
  int32_t* out = static_cast<int32_t*>(rows_v) + (int64_t)t * p.N;
  RfRec* outr = static_cast<RfRec*>(rows_v) + (int64_t)t * p.N;
  const int64_t r0 = p.N * blockIdx.x / B, r1 = p.N * (blockIdx.x + 1) / B;
  int par = 0;
  for (int64_t c = r0; c < r1; c += RR * RF_NT, par ^= 1) {
    int w[RR], pre[RR];
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      const int64_t r = c + k * RF_NT + threadIdx.x;
      w[k] = r < r1 ? row_weight(p.bootstrap, p.seed, t + p.t_off, r) : 0;
    }
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      const uint64_t bal = __ballot(w[k] > 0);
      pre[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
      if (lane == 0) wcnt[par][k][wv] = __builtin_popcountll(bal);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
#pragma unroll
      for (int k = 0; k < RR; ++k) tot += wcnt[par][k][0] + wcnt[par][k][1] + wcnt[par][k][2] + wcnt[par][k][3];
      base[par] = atomicAdd(&p.lrc[(int64_t)t * 2], tot);
    }
    __syncthreads();
    int off = base[par];
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      int o = off;
      for (int i = 0; i < wv; ++i) o += wcnt[par][k][i];
      if (w[k] > 0) {
        const int64_t r = c + k * RF_NT + threadIdx.x;
        if constexpr (REC) {
          const uint64_t xv = p.X[r], yv = p.Y[r];
          const uint32_t wk = (uint32_t)w[k];
          if (ROOTH && pos) {  // position form: the outputs extracted once, for the record and the root sums
            const RfPos ps = rf_pos_extract(yv & RF_M62);
            RfRec e = rf_make_rec(xv, 0ull, wk);
            e.y |= rf_pos_pack(ps);
            outr[o + pre[k]] = e;
            my_n += wk;
            uint32_t* srow = RF_INIT_REP ? Sr + (lane & (RF_IREP_S - 1)) * 64 : rlds;
            uint32_t* hrow = RF_INIT_REP ? Hr + (lane & (RF_IREP_H - 1)) * hst : rlds + 68 + kp;
#pragma unroll
            for (int q = 0; q < RF_NPOS; ++q) atomicAdd(&srow[ps.o[q]], wk);  // S (none: pad word 63)
            for (uint64_t xx = xv & RF_M62 & rmask; xx; xx &= xx - 1)
              rf_add_pos(hrow + rslot[__builtin_ctzll(xx)] * 64, ps, wk);
          } else {
            outr[o + pre[k]] = rf_make_rec(xv, yv, wk);
          }
          if (ROOTH && !pos) {
            const uint64_t y = yv & RF_M62;
            my_n += wk;
            for (uint64_t yy = y; yy; yy &= yy - 1) atomicAdd(&rlds[__builtin_ctzll(yy)], wk);
            uint64_t xx = xv & RF_M62 & rmask;
            if (xx) {  // candidate bits: outputs once, the count as output word 62 (as rf_hist)
              const RfYBits yb = rf_ybits(y | (1ull << 62));
              while (xx) {
                const int sl = rslot[__builtin_ctzll(xx)];
                xx &= xx - 1;
                rf_add_ybits(rlds + 68 + kp + sl * 64, yb, wk);
              }
            }
          }
        } else {
          out[o + pre[k]] = rf_packed(p.N) ? (int32_t)(r | ((int64_t)w[k] << RF_WSHIFT)) : (int32_t)r;
        }
      }
      off += wcnt[par][k][0] + wcnt[par][k][1] + wcnt[par][k][2] + wcnt[par][k][3];
    }
  }
  if constexpr (ROOTH) {
    for (int o = 32; o > 0; o >>= 1) my_n += __shfl_xor(my_n, o);
    if (lane == 0) atomicAdd(&rlds[64], my_n);
    __syncthreads();
    uint32_t* dst = p.acc + (int64_t)t * rec;  // the root record of tree t (zeroed by the driver)
    for (int i = threadIdx.x; i < rec; i += blockDim.x) {
      uint32_t v = 0;
      if (RF_INIT_REP && pos) {  // sum the replicas
        if (i < 62) {
          for (int q = 0; q < RF_IREP_S; ++q) v += Sr[q * 64 + i];
        } else if (i == 64) {
          v = rlds[64];
        } else if (i >= 68 && i < 68 + kp) {
          if (i - 68 < k)
            for (int q = 0; q < RF_IREP_H; ++q) v += Hr[q * hst + (i - 68) * 64 + 62];
        } else if (i >= 68 + kp && ((i - 68 - kp) & 63) < 62) {
          for (int q = 0; q < RF_IREP_H; ++q) v += Hr[q * hst + (i - 68 - kp)];
        }
      } else if (i < 68) v = (i & ~1) == 62 ? 0u : rlds[i];  // (S words 62 / 63: pads)
      else if (i < 68 + kp) v = i - 68 < k ? rlds[68 + kp + (i - 68) * 64 + 62] : 0u;
      else v = ((i - 68 - kp) & 63) < 62 ? rlds[i] : 0u;
      if (v) atomicAdd(&dst[i], v);
    }
  }
}

// the node's candidate features: partial Fisher-Yates on a hashed stream, as the oracle
EM_DEVICE void rf_node_cands(const RfParams& p, int t, int node, int16_t* __restrict__ co) {
  int arr[RF_MAXF];
  for (int i = 0; i < p.F; ++i) arr[i] = i;
  const int kk = p.k_feat < p.F ? p.k_feat : p.F;
  for (int i = 0; i < kk; ++i) {
    const uint64_t h = hash3(p.seed ^ 0x5EEDF00Dull, ((uint64_t)(t + p.t_off) << 32) | (uint64_t)node, (uint64_t)i);
    const int j = i + (int)(h % (uint64_t)(p.F - i));
    const int tmp = arr[i];
    arr[i] = arr[j];
    arr[j] = tmp;
    co[i] = (int16_t)arr[i];
  }
}

// rf_node_cands by one whole wave (all 64 lanes call it): the identity array lives in registers,
// element e in lane e & 63, register e >> 6 (F <= 256), so the partial Fisher-Yates needs no
// private array (rf_node_cands' int[256] is scratch memory).  Same hash stream and swaps.
EM_DEVICE void rf_node_cands_wave(const RfParams& p, int t, int node, int16_t* __restrict__ co) {
  const int lane = threadIdx.x & 63;
  int v[RF_MAXF / 64];
#pragma unroll
  for (int q = 0; q < RF_MAXF / 64; ++q) v[q] = lane + 64 * q;
  auto get = [&](int e) {  // arr[e] (e uniform)
    const int q = e >> 6;
    const int src = q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
    return __shfl(src, e & 63);
  };
  auto put = [&](int e, int val) {  // arr[e] = val (e uniform)
    if (lane == (e & 63)) {
      const int q = e >> 6;
      if (q == 0) v[0] = val;
      else if (q == 1) v[1] = val;
      else if (q == 2) v[2] = val;
      else v[3] = val;
    }
  };
  const int kk = p.k_feat < p.F ? p.k_feat : p.F;
  for (int i = 0; i < kk; ++i) {
    const uint64_t h = hash3(p.seed ^ 0x5EEDF00Dull, ((uint64_t)(t + p.t_off) << 32) | (uint64_t)node, (uint64_t)i);
    const int j = i + (int)(h % (uint64_t)(p.F - i));
    const int ai = get(i), aj = get(j);
    put(i, aj);
    put(j, ai);
    if (lane == 0) co[i] = (int16_t)aj;
  }
}

// One thread per (tree, node of this level): child segments from the parent's partition counters,
// then the node's candidate features (partial Fisher-Yates on a hashed stream, as the oracle).
__global__ void rf_level_prep(RfParams p, int level) {
  const int nodesL = 1 << level, first = nodesL - 1;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)p.T * nodesL) return;
  const int t = (int)(gid / nodesL), nd = (int)(gid - (int64_t)t * nodesL), node = first + nd;
  int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  int start = 0, count = -1;
  if (level == 0) {
    count = p.lrc[(int64_t)t * 2];
  } else {
    const int parent = (node - 1) >> 1, pnd = parent - ((nodesL >> 1) - 1);
    const int32_t* ps = p.seg + ((int64_t)t * p.nodes + parent) * 2;
    if (ps[1] >= 0 && p.feat[(int64_t)t * p.nodes + parent] >= 0) {
      const int lc = p.lrc[((int64_t)t * (nodesL >> 1) + pnd) * 2];
      const bool left = ((node - 1) & 1) == 0;
      start = left ? ps[0] : ps[0] + lc;
      count = left ? lc : ps[1] - lc;
    }
  }
  sg[0] = start;
  sg[1] = count;
  if (count < 0 || level >= p.max_depth) return;
  rf_node_cands(p, t, node, p.cand + ((int64_t)t * nodesL + nd) * p.k_feat);
}

// Level work lists.  Deep levels are very unbalanced (a one-hot split sends ~90 % of a node's rows to
// the x = 0 child, so at level 6 one node of each tree holds about half of its rows), and sizing the
// blocks per node from the AVERAGE node left one workgroup grinding through a 200k-row node while the
// rest of the GPU idled.  rf_worklist gives every (tree, node) of the level ceil(count / RF_CHUNK)
// blocks (exclusive prefix in wl[]); the level kernels run a 1-D grid and map block g to its
// (tree, node, slice) by binary search.
constexpr int RF_CHUNK = 8192;
// the root level's nodes hold every kept row of their tree: their partition blocks all merge into the
// same two child records with global atomics, so fewer, longer blocks there (RF_CHUNK0 rows)
#ifndef RF_CHUNK0
#define RF_CHUNK0 32768
#endif
#ifndef RF_CHUNK1
#define RF_CHUNK1 8192
#endif
static_assert(RF_CHUNK0 >= RF_CHUNK && RF_CHUNK1 >= RF_CHUNK, "the launch bound assumes RF_CHUNK is the smallest");
__host__ __device__ inline int rf_chunk(int level) { return level == 0 ? RF_CHUNK0 : (level == 1 ? RF_CHUNK1 : RF_CHUNK); }
struct RfWork {
  int t, nd, j, nb;
};
EM_DEVICE bool rf_work(const int32_t* __restrict__ wl, int nitems, int nodesL, RfWork& w) {
  const int g = blockIdx.x;
  if (g >= wl[nitems]) return false;
  int lo = 0, hi = nitems;  // last i with wl[i] <= g (then g < wl[i + 1])
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (wl[mid] <= g) lo = mid;
    else hi = mid;
  }
  w = RfWork{lo / nodesL, lo % nodesL, g - wl[lo], wl[lo + 1] - wl[lo]};
  return true;
}

__global__ void __launch_bounds__(1024) rf_worklist(RfParams p, int level, int32_t* __restrict__ wl) {
  const int nodesL = 1 << level, first = nodesL - 1, n = p.T * nodesL;
  __shared__ int part[1024];
  const int per = (n + 1023) / 1024, a = threadIdx.x * per, b = min(n, a + per);
  auto blocks = [&](int i) {
    const int t = i / nodesL, nd = i - t * nodesL;
    const int cnt = p.seg[((int64_t)t * p.nodes + first + nd) * 2 + 1];
    return cnt < 0 ? 0 : max(1, (cnt + rf_chunk(level) - 1) / rf_chunk(level));
  };
  int sum = 0;
  for (int i = a; i < b; ++i) sum += blocks(i);
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = part[threadIdx.x] - sum;
  for (int i = a; i < b; ++i) {
    wl[i] = run;
    run += blocks(i);
  }
  if (threadIdx.x == 1023) wl[n] = part[1023];
}

// partition blocks of a node with `count` rows at `level` (rf_worklist's rule)
EM_DEVICE int rf_blocks(int count, int level) {
  return count < 0 ? 0 : max(1, (count + rf_chunk(level) - 1) / rf_chunk(level));
}
constexpr int RF_BEGIN_LDS = 16384;  // rf_level_begin keeps per-node block counts in LDS up to this many nodes
// The fused driver's level start in ONE workgroup: rf_level_prep's child segments (no candidates:
// the root's come with rf_init_rows, deeper levels' from the parent's rf_split), then -- after every
// segment is written and every parent counter read -- this level's partition counters zeroed (and, at
// the root, the root records), then rf_worklist's scan.  Replaces 2 kernels and 1-2 memsets per level.
__global__ void __launch_bounds__(1024) rf_level_begin(RfParams p, int level, int32_t* __restrict__ wl,
                                                       int zero_root) {
  const int nodesL = 1 << level, first = nodesL - 1, n = p.T * nodesL;
  __shared__ uint16_t nblk[RF_BEGIN_LDS];
  // items in batches of 8 per thread: the batch's parent loads are all issued before its stores
  constexpr int PB = 8;
  for (int g0 = 0; g0 < n; g0 += PB * 1024) {
    int ps0[PB], ps1[PB], pf[PB], lc[PB];
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int gid = g0 + u * 1024 + (int)threadIdx.x;
      ps0[u] = 0;
      ps1[u] = -1;
      pf[u] = -1;
      lc[u] = 0;
      if (gid >= n) continue;
      const int t = gid / nodesL, nd = gid - t * nodesL, node = first + nd;
      if (level == 0) {
        lc[u] = p.lrc[(int64_t)t * 2];
      } else {
        const int parent = (node - 1) >> 1, pnd = parent - ((nodesL >> 1) - 1);
        ps0[u] = p.seg[((int64_t)t * p.nodes + parent) * 2];
        ps1[u] = p.seg[((int64_t)t * p.nodes + parent) * 2 + 1];
        pf[u] = p.feat[(int64_t)t * p.nodes + parent];
        lc[u] = p.lrc[((int64_t)t * (nodesL >> 1) + pnd) * 2];
      }
    }
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int gid = g0 + u * 1024 + (int)threadIdx.x;
      if (gid >= n) continue;
      const int t = gid / nodesL, nd = gid - t * nodesL, node = first + nd;
      int start = 0, count = -1;
      if (level == 0) {
        count = lc[u];
      } else if (ps1[u] >= 0 && pf[u] >= 0) {
        const bool left = ((node - 1) & 1) == 0;
        start = left ? ps0[u] : ps0[u] + lc[u];
        count = left ? lc[u] : ps1[u] - lc[u];
      }
      int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
      sg[0] = start;
      sg[1] = count;
      if (gid < RF_BEGIN_LDS) nblk[gid] = (uint16_t)rf_blocks(count, level);
    }
  }
  __syncthreads();  // segments written, the parents' counters read
  for (int i = threadIdx.x; i < 2 * n; i += 1024) p.lrc[i] = 0;
  if (level == 0 && zero_root)
    for (int i = threadIdx.x; i < n * rec_words(p.k_feat); i += 1024) p.acc[i] = 0u;
  __shared__ int part[1024];
  const int per = (n + 1023) / 1024, a = threadIdx.x * per, b = min(n, a + per);
  auto blocks = [&](int i) {  // (counts from LDS: each global re-read costs ~1 us, in series per thread)
    if (n <= RF_BEGIN_LDS) return (int)nblk[i];
    const int t = i / nodesL, nd = i - t * nodesL;
    return rf_blocks(p.seg[((int64_t)t * p.nodes + first + nd) * 2 + 1], level);
  };
  int sum = 0;
  for (int i = a; i < b; ++i) sum += blocks(i);
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = part[threadIdx.x] - sum;
  for (int i = a; i < b; ++i) {
    wl[i] = run;
    run += blocks(i);
  }
  if (threadIdx.x == 1023) wl[n] = part[1023];
}

// K8: (blocks x nodes x trees) workgroups; block b of a node sums its slice of the node's row list
// into LDS (integer atomics on set bits only: y bits for S, candidate x bits for cnt/hist), then
// merges into the node record (plain stores when one block owns the node, else global atomics).
// DERIVE (levels >= 1): the node totals S / n are not accumulated here -- rf_child_totals already
// wrote them from the parent's record (right child = the parent's histogram of its split feature,
// left = parent - right, exact integers), so a row costs its candidate bits' atomics only.
template <bool REC, bool DERIVE>
__global__ void __launch_bounds__(RF_NT) rf_hist(RfParams p, const void* __restrict__ rows_v, int level,
                                                 const int32_t* __restrict__ wl) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int nodesL = 1 << level, first = nodesL - 1;
  RfWork wk;
  if (!rf_work(wl, p.T * nodesL, nodesL, wk)) return;
  const int t = wk.t, nd = wk.nd, B = wk.nb;
  const int node = first + nd;
  const int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  const int start = sg[0], count = sg[1];
  if (count < 0) return;
  const int k = p.k_feat, rec = rec_words(k), kp = (k + 3) & ~3;
  uint32_t* S = lds;                // [64]
  uint32_t* nn = lds + 64;          // [1] (+3 pad)
  uint32_t* cnt = lds + 68;         // [kp]
  uint32_t* hist = cnt + kp;        // [k][64]
  __shared__ int16_t slot[RF_MAXF];
  __shared__ uint64_t cmask[RF_MAXF / 64];
  const bool split = level < p.max_depth;
  for (int i = threadIdx.x; i < rec; i += blockDim.x) lds[i] = 0u;
  for (int i = threadIdx.x; i < p.F; i += blockDim.x) slot[i] = -1;
  if (threadIdx.x < RF_MAXF / 64) cmask[threadIdx.x] = 0ull;
  __syncthreads();
  const int kk = k < p.F ? k : p.F;
  if (split && threadIdx.x == 0) {
    const int16_t* co = p.cand + ((int64_t)t * nodesL + nd) * k;
    for (int i = 0; i < kk; ++i) {
      slot[co[i]] = (int16_t)i;
      cmask[co[i] >> 6] |= 1ull << (co[i] & 63);
    }
  }
  __syncthreads();
  const int32_t* rl = static_cast<const int32_t*>(rows_v) + (int64_t)t * p.N + start;
  const RfRec* rr = static_cast<const RfRec*>(rows_v) + (int64_t)t * p.N + start;
  const int i0 = (int)((int64_t)count * wk.j / B), i1 = (int)((int64_t)count * (wk.j + 1) / B);
  uint32_t my_n = 0;
  const bool packed = rf_packed(p.N);
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    int64_t r = 0;
    uint32_t w;
    uint64_t y, xr = 0;
    if constexpr (REC) {
      const RfRec e = rr[i];
      w = rf_rec_w(e);
      y = e.y & RF_M62;
      xr = e.x & RF_M62;
    } else {
      const int32_t e = rl[i];
      r = packed ? (e & RF_RMASK) : e;
      w = packed ? (uint32_t)e >> RF_WSHIFT : (uint32_t)row_weight(p.bootstrap, p.seed, t + p.t_off, r);
      y = p.Y[r] & RF_M62;
    }
    if (!DERIVE) {  // (every row: the uniform 7-output walk is already branch-coherent)
      my_n += w;
      uint64_t yy = y;
      while (yy) {
        atomicAdd(&S[__builtin_ctzll(yy)], w);
        yy &= yy - 1;
      }
    }
    if (!split) continue;
    for (int wd = 0; wd < p.W; ++wd) {
      uint64_t xx = (REC ? xr : p.X[r * p.W + wd]) & cmask[wd];
      if (RF_YBITS && xx) {  // candidate rows: outputs extracted once, the count as output word 62
        const RfYBits yb = rf_ybits(y | (1ull << 62));
        while (xx) {
          const int sl = slot[wd * 64 + __builtin_ctzll(xx)];
          xx &= xx - 1;
          rf_add_ybits(hist + sl * 64, yb, w);
        }
      }
      while (!RF_YBITS && xx) {
        const int sl = slot[wd * 64 + __builtin_ctzll(xx)];
        xx &= xx - 1;
        atomicAdd(&cnt[sl], w);
        {
          uint64_t y2 = y;
          while (y2) {
            atomicAdd(&hist[sl * 64 + __builtin_ctzll(y2)], w);
            y2 &= y2 - 1;
          }
        }
      }
    }
  }
  if (!DERIVE) {
    for (int o = 32; o > 0; o >>= 1) my_n += __shfl_xor(my_n, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(nn, my_n);
  }
  __syncthreads();
  uint32_t* dst = p.acc + ((int64_t)t * nodesL + nd) * rec;
  const int used = split ? rec : 68;
  const int lo = DERIVE ? 68 : 0;  // S / n (words 0..67) already hold the derived totals
  auto word = [&](int i) -> uint32_t {  // RF_YBITS: cnt[c] was counted in hist[c][62]
    if (!RF_YBITS || i < 68) return lds[i];
    if (i < 68 + kp) return i - 68 < k ? lds[68 + kp + (i - 68) * 64 + 62] : 0u;
    return ((i - 68 - kp) & 63) < 62 ? lds[i] : 0u;
  };
  if (B == 1) {
    for (int i = lo + threadIdx.x; i < used; i += blockDim.x) dst[i] = word(i);
  } else {
    for (int i = lo + threadIdx.x; i < used; i += blockDim.x) {
      const uint32_t v = word(i);
      if (v) atomicAdd(&dst[i], v);
    }
  }
}

// Level >= 1 node totals from the parent's record (DERIVE histograms): the parent's rf_split left the
// winning candidate slot c in its record word 65; node index 2i+1 (even nd) is the x_f = 0 child.
// One wavefront per (tree, node); lane j < 64 writes S[j], lane 0 also n.
__global__ void __launch_bounds__(64) rf_child_totals(RfParams p, const uint32_t* __restrict__ prev, int level) {
  const int nodesL = 1 << level, first = nodesL - 1;
  const int t = blockIdx.y, nd = blockIdx.x, node = first + nd;
  const int lane = threadIdx.x;
  if (p.seg[((int64_t)t * p.nodes + node) * 2 + 1] < 0) return;  // under an unsplit parent: no record
  const int k = p.k_feat, rec = rec_words(k), kp = (k + 3) & ~3;
  const uint32_t* P = prev + ((int64_t)t * (nodesL >> 1) + (nd >> 1)) * rec;
  const int c = (int)P[65];
  const bool right = nd & 1;
  const uint32_t sr = P[68 + kp + c * 64 + lane], nr = P[68 + c];
  uint32_t* dst = p.acc + ((int64_t)t * nodesL + nd) * rec;
  dst[lane] = right ? sr : P[lane] - sr;
  if (lane == 0) dst[64] = right ? nr : P[64] - nr;
}

// K9: one wavefront per (tree, node): node record (weighted mean outputs, cover) and the split scan
// over the candidates (lane j = output j): gain = SL2/nL + SR2/nR - S2/n from exact integers.
// child_acc (the fused driver, derived totals): a node that splits also writes its two children's
// records for level + 1 -- node totals S / n (right = the histogram of the split candidate, left =
// parent - right: rf_child_totals' arithmetic), every other word zeroed for the partition's histogram
// atomics -- and, with child_cand, draws the children's candidate features (rf_node_cands).
// (launched with 128 threads when child_cand is set: the second wave draws the children's candidates
// -- they depend on (seed, tree, node) only -- while the first runs the split scan)
__global__ void __launch_bounds__(128) rf_split(RfParams p, int level, uint32_t* __restrict__ child_acc,
                                                int16_t* __restrict__ child_cand) {
  const int nodesL = 1 << level, first = nodesL - 1;
  const int t = blockIdx.y, nd = blockIdx.x, node = first + nd;
  const int lane = threadIdx.x & 63;
  const int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  int16_t* fo = p.feat + (int64_t)t * p.nodes + node;
  if (sg[1] < 0) {
    if (threadIdx.x == 0) *fo = -2;
    return;
  }
  if (threadIdx.x >= 64) {  // wave 1: the children's candidates (unused if this node ends as a leaf)
    for (int sd = 0; sd < 2; ++sd)
      rf_node_cands_wave(p, t, 2 * node + 1 + sd, child_cand + ((int64_t)t * (2 * nodesL) + 2 * nd + sd) * p.k_feat);
    return;
  }
  const int k = p.k_feat, rec = rec_words(k), kp = (k + 3) & ~3;
  uint32_t* A = p.acc + ((int64_t)t * nodesL + nd) * rec;
  const uint32_t n = A[64];
  const uint32_t Sj = lane < 62 ? A[lane] : 0u;
  float* vo = p.value + ((int64_t)t * p.nodes + node) * 64;
  vo[lane] = (n > 0 && lane < 62) ? (float)((double)Sj / (double)n) : 0.f;
  if (lane == 0) p.cover[(int64_t)t * p.nodes + node] = (float)n;
  const bool can_split = level < p.max_depth && n >= (uint32_t)(2 * p.min_leaf) && n > 0;
  double best = 0.0;
  int bf = -1, bc = -1;
  if (can_split) {
    uint64_t s2 = (uint64_t)Sj * Sj;
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
    const int kk = k < p.F ? k : p.F;
    const int16_t* co = p.cand + ((int64_t)t * nodesL + nd) * k;
    // candidates in batches of 8 whose record words are all loaded first: one global round trip per
    // batch instead of one per candidate (the serial loads were ~12 us of every level's split)
    for (int c0 = 0; c0 < kk; c0 += 8) {
      int fb[8];
      uint32_t nRb[8], SRb[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u < kk ? c0 + u : kk - 1;
        fb[u] = co[c];
        nRb[u] = A[68 + c];
        SRb[u] = lane < 62 ? A[68 + kp + c * 64 + lane] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u;
        if (c >= kk) break;
        const int f = fb[u];
        const uint32_t nR = nRb[u], nL = n - nR;
        const uint32_t SR = SRb[u];
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
          bc = c;
        }
      }
    }
    // a split must reduce impurity by more than rounding noise
    if (bf >= 0 && !(best > 1e-9 * (1.0 + best))) bf = -1;
  }
  if (lane == 0) {
    *fo = (int16_t)bf;
    p.gain[(int64_t)t * p.nodes + node] = bf >= 0 ? best : 0.0;
    A[65] = bf >= 0 ? (uint32_t)bc : 0u;  // candidate slot of the split (rf_child_totals)
  }
  if (bf < 0 || !child_acc) return;
  const uint32_t sr = A[68 + kp + bc * 64 + lane], nr = A[68 + bc];
  if (level + 1 == p.max_depth) {
    // the children are leaves of the last level: their outputs straight from the derived totals (what
    // rf_split of that level would compute from the records written below), so the fused driver needs
    // no last partition, level start or split
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const uint32_t cs = sd ? sr : A[lane] - sr, cn = sd ? nr : n - nr;
      const int64_t c = (int64_t)t * p.nodes + 2 * node + 1 + sd;
      p.value[c * 64 + lane] = (cn > 0 && lane < 62) ? (float)((double)cs / (double)cn) : 0.f;
      if (lane == 0) {
        p.cover[c] = (float)cn;
        p.feat[c] = -1;
        p.gain[c] = 0.0;
      }
    }
    return;
  }
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {  // sd 0: x_f = 0 child (2 node + 1), 1: x_f = 1 child
    uint32_t* dst = child_acc + ((int64_t)t * (2 * nodesL) + 2 * nd + sd) * rec;
    dst[lane] = sd ? sr : A[lane] - sr;
    // words 68.. are the partition's: it stores them when one block owns this node (rf_worklist:
    // ceil(count / RF_CHUNK) blocks) and adds into zeroed words otherwise
    const int hi = (sg[1] + rf_chunk(level) - 1) / rf_chunk(level) > 1 ? rec : 68;
    for (int i = 64 + lane; i < hi; i += 64) dst[i] = i == 64 ? (sd ? nr : n - nr) : 0u;
  }
}

// K10: children row lists, (blocks x nodes x trees) workgroups: left rows (x_f = 0) fill the parent
// segment from its start, right rows from its end; every 256-row chunk reserves its ranges with one
// atomic per side on the node's counters (lrc), which rf_level_prep turns into the child segments.
// HIST (record rows, derived node totals): while a record moves to its child, its candidate bits are
// also added to that child's histogram (cnt / hist words of the child's record in acc_next, LDS partials
// merged by integer atomics), so level + 1 needs no histogram pass over its rows.
#ifndef RF_PART_RR
#define RF_PART_RR 4
#endif
template <bool REC, bool HIST>
__global__ void __launch_bounds__(RF_NT) rf_partition(RfParams p, const void* __restrict__ rin_v,
                                                      void* __restrict__ rout_v, int level,
                                                      const int32_t* __restrict__ wl, uint32_t* __restrict__ acc_next,
                                                      const int16_t* __restrict__ cand_next) {
  using E = typename std::conditional<REC, RfRec, int32_t>::type;
  const E* rin = static_cast<const E*>(rin_v);
  E* rout = static_cast<E*>(rout_v);
  const int nodesL = 1 << level, first = nodesL - 1;
  RfWork wk;
  if (!rf_work(wl, p.T * nodesL, nodesL, wk)) return;
  const int t = wk.t, nd = wk.nd, B = wk.nb, node = first + nd;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const int32_t* sg = p.seg + ((int64_t)t * p.nodes + node) * 2;
  const int start = sg[0], count = sg[1];
  const int f = p.feat[(int64_t)t * p.nodes + node];
  if (f < 0 || count < 0) return;
  extern __shared__ __attribute__((aligned(16))) uint32_t chl[];  // HIST: [2 children][rec]
  __shared__ int8_t cslot[2][64];
  __shared__ uint64_t cmk[2];
  const int kf = p.k_feat, rec = rec_words(kf), kp = (kf + 3) & ~3;
  const int chw = rf_chl_words(kf), cst = rf_rep_cnt_stride(kf), hst = rf_rep_hist_stride(kf);
  const int lane_c = (threadIdx.x & 63) % RF_REP_CNT, lane_h = (threadIdx.x & 63) % RF_REP_HIST;
  const bool pos = HIST && REC && p.yover && *p.yover == 0;
  if (HIST) {
    for (int i = threadIdx.x; i < 2 * chw; i += blockDim.x) chl[i] = 0u;
    if (threadIdx.x < 2) {
      const int s = threadIdx.x;
      const int16_t* co = cand_next + ((int64_t)t * (2 * nodesL) + 2 * nd + s) * kf;
      uint64_t m = 0;
      const int kk = kf < p.F ? kf : p.F;
      for (int i = 0; i < kk; ++i) {
        cslot[s][co[i]] = (int8_t)i;
        m |= 1ull << co[i];
      }
      cmk[s] = m;
    }
    __syncthreads();
  }
  // chunks of RR x blockDim rows: RR ballots per wave (row k of the thread = c + k*blockDim + tid), one
  // LDS count exchange and one atomic reservation per side per chunk (instead of per blockDim rows);
  // the small count arrays are double-buffered so a chunk needs two barriers
  constexpr int RR = RF_PART_RR;
  __shared__ int lc[2][RR][4], rc[2][RR][4];
  __shared__ int lbase[2], rbase[2];
  int32_t* ctr = p.lrc + ((int64_t)t * nodesL + nd) * 2;
  const E* ri = rin + (int64_t)t * p.N + start;
  E* ro = rout + (int64_t)t * p.N + start;
  const int i0 = (int)((int64_t)count * wk.j / B), i1 = (int)((int64_t)count * (wk.j + 1) / B);
  int buf = 0;
  for (int c = i0; c < i1; c += RR * blockDim.x, buf ^= 1) {
    E r[RR];
    bool right[RR], left[RR], have[RR];
#pragma unroll
    for (int k = 0; k < RR; ++k) {  // the RR row loads, then the RR feature-bit loads, all in flight
      const int i = c + k * blockDim.x + threadIdx.x;
      have[k] = i < i1;
      if (have[k]) r[k] = ri[i];
    }
    int pl[RR], pr[RR];
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      if constexpr (REC) right[k] = have[k] && ((r[k].x >> f) & 1ull);
      else right[k] = have[k] && xbit(p.X, p.W, r[k] & (rf_packed(p.N) ? RF_RMASK : 0x7FFFFFFF), f);
      left[k] = have[k] && !right[k];
      const uint64_t bl = __ballot(left[k]), br = __ballot(right[k]);
      pl[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0));
      pr[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(br >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)br, 0));
      if (lane == 0) {
        lc[buf][k][wv] = __builtin_popcountll(bl);
        rc[buf][k][wv] = __builtin_popcountll(br);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tl = 0, tr = 0;
      for (int k = 0; k < RR; ++k)
        for (int q = 0; q < nwv; ++q) {
          tl += lc[buf][k][q];
          tr += rc[buf][k][q];
        }
      lbase[buf] = atomicAdd(&ctr[0], tl);
      rbase[buf] = atomicAdd(&ctr[1], tr);
    }
    __syncthreads();
    int lo = lbase[buf], roff = rbase[buf];
#pragma unroll
    for (int k = 0; k < RR; ++k) {  // offsets in (k, wave, lane) order
      int l = lo, rr = roff;
      for (int q = 0; q < wv; ++q) {
        l += lc[buf][k][q];
        rr += rc[buf][k][q];
      }
      if (left[k]) ro[l + pl[k]] = r[k];
      if (right[k]) ro[count - 1 - (rr + pr[k])] = r[k];
      for (int q = 0; q < nwv; ++q) {
        lo += lc[buf][k][q];
        roff += rc[buf][k][q];
      }
    }
    if constexpr (HIST && REC) {
#pragma unroll
      for (int k2 = 0; k2 < RR; ++k2) {
        if (!have[k2]) continue;
        const int sd = right[k2] ? 1 : 0;
        const uint32_t w = rf_rec_w(r[k2]);
        const uint64_t y = r[k2].y & RF_M62;
        uint64_t xx = r[k2].x & RF_M62 & cmk[sd];
        uint32_t* cnt = chl + sd * chw + lane_c * cst;
        uint32_t* hist = chl + sd * chw + RF_REP_CNT * cst + lane_h * hst;
        if (pos) {  // position-form record: the outputs are 7 bit fields
          if (xx) {
            const RfPos ps = rf_pos_unpack(r[k2].y);
            for (; xx; xx &= xx - 1) rf_add_pos(hist + cslot[sd][__builtin_ctzll(xx)] * 64, ps, w);
          }
          continue;
        }
        if (RF_YBITS && xx) {
          const RfYBits yb = rf_ybits(RF_CNT62 ? (y | (1ull << 62)) : y);
          while (xx) {
            const int sl = cslot[sd][__builtin_ctzll(xx)];
            xx &= xx - 1;
            if (!RF_CNT62) atomicAdd(&cnt[sl], w);
            rf_add_ybits(hist + sl * 64, yb, w);
          }
        }
        while (!RF_YBITS && xx) {
          const int sl = cslot[sd][__builtin_ctzll(xx)];
          xx &= xx - 1;
          atomicAdd(&cnt[sl], w);
          uint64_t y2 = y;
          while (y2) {
            atomicAdd(&hist[sl * 64 + __builtin_ctzll(y2)], w);
            y2 &= y2 - 1;
          }
        }
      }
    }
  }
  if constexpr (HIST) {
    __syncthreads();
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      uint32_t* dst = acc_next + ((int64_t)t * (2 * nodesL) + 2 * nd + sd) * rec;
      const uint32_t* src = chl + sd * chw;
      for (int i = 68 + threadIdx.x; i < rec; i += blockDim.x) {
        uint32_t v = 0;
        if (i < 68 + kp) {  // cnt[sl]: its replicas (RF_CNT62: word 62 of the slot's histogram row)
          if (RF_YBITS && RF_CNT62) {
            if (i - 68 < kf)
              for (int q = 0; q < RF_REP_HIST; ++q) v += src[RF_REP_CNT * cst + q * hst + (i - 68) * 64 + 62];
          } else {
            for (int q = 0; q < RF_REP_CNT; ++q) v += src[q * cst + (i - 68)];
          }
        } else if (!(RF_YBITS && RF_CNT62) || ((i - 68 - kp) & 63) < 62) {  // hist[sl][j]: its replicas
          const int o = i - 68 - kp;
          for (int q = 0; q < RF_REP_HIST; ++q) v += src[RF_REP_CNT * cst + q * hst + o];
        }
        if (B == 1)  // the node's only block: plain stores (rf_split did not zero these words)
          dst[i] = v;
        else if (v)
          atomicAdd(&dst[i], v);
      }
    }
  }
}

// K11: mean leaf vector over trees, one wavefront per row.  The traversals run lane-parallel
// (lane l walks tree t0 + l: 8 dependent loads per 64 trees instead of per tree), then lane j
// (= output j) gathers the 64 trees' leaf values through wave shuffles of the leaf indices.
// NOTE (ROCm 7.2): holding the row's feature words in registers and picking one with a per-lane
// select chain + 64-bit shift produced wrong bits for ~3 % of rows on gfx950; reading the bit
// through xbit() (an L1-resident load) is exact -- tests/test_forest.py checks the deep-tree case.
__global__ void __launch_bounds__(256) rf_predict(const uint64_t* __restrict__ X, int W, int64_t N,
                                                  const int16_t* __restrict__ feat, const float* __restrict__ value,
                                                  int T, int nodes, int out_logit, float* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= N) return;
  float acc = 0.f;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    int nd = 0;
    if (t < T) {
      const int16_t* ft = feat + (int64_t)t * nodes;
      int f = ft[0];
      while (f >= 0) {
        nd = 2 * nd + 1 + xbit(X, W, r, f);
        f = ft[nd];
      }
    }
    const int cnt = T - t0 < 64 ? T - t0 : 64;
    const float* vb = value + (int64_t)t0 * nodes * 64 + lane;
    for (int k = 0; k < cnt; ++k) {
      const int ndk = __shfl(nd, k);
      acc += vb[((int64_t)k * nodes + ndk) * 64];
    }
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

// K11, tree-streamed form (W == 1, max_depth <= 8: at most 256 leaves per tree).  Predict was bound by
// the leaf gathers: N x T x 256 B (7.7 GB for 300 k rows x 100 trees) read from L2 / MALL, one 256-B
// leaf vector per (row, tree).  Here each workgroup owns a block of rows for the whole launch and
// streams the trees through LDS instead: per tree one 1-KB node table (features, leaves encoded as
// -(slot + 1)) and the tree's compacted leaf vectors (nleaf x 256 B), double-buffered by LDS-DMA
// (buffer_load ... lds) while the previous tree is applied.  A lane owns one row: it walks the tree in
// LDS and adds its leaf's 16 float4 chunks into 64 accumulator registers per 64-row group.  The chunk
// order is rotated by the lane (step c reads chunk (lane + c) & 15), so the 16 lanes of a ds_read_b128
// phase always hit 16 different bank groups whatever leaves they read, and register set c of lane l
// holds output chunk (l + c) & 15 (un-rotated by the store addresses).  Every output still sums its
// trees in tree order, so the result is bit-identical to rf_predict.
constexpr int RFP_TREE = 1024 + 256 * 256;  // bytes per prepared tree: node table + 256 leaf vectors

// one workgroup per tree: node table with leaves encoded, leaf vectors compacted in level order;
// word 511 of the node table (a padding slot: nodes <= 511) holds the leaf count.  The feature row is
// staged into LDS by all 512 threads first (the level walk is then LDS-only), and the leaf vectors are
// copied as float4s in batches of 4 independent loads per thread (a per-node loop of dependent
// load -> store round trips made this kernel cost milliseconds).
constexpr int RFP_PREP_THREADS = 512;
__global__ void __launch_bounds__(RFP_PREP_THREADS) rf_predict_prepare(const int16_t* __restrict__ feat,
                                                                       const float* __restrict__ value, int nodes,
                                                                       int depth, uint8_t* __restrict__ prep) {
  __shared__ int16_t ft[512];
  __shared__ uint8_t reach[512];
  __shared__ int16_t slot_of[512];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  int16_t* enc = reinterpret_cast<int16_t*>(prep + (int64_t)t * RFP_TREE);
  f32x4* vals = reinterpret_cast<f32x4*>(prep + (int64_t)t * RFP_TREE + 1024);
  for (int n = tid; n < nodes; n += RFP_PREP_THREADS) ft[n] = feat[(int64_t)t * nodes + n];
  __syncthreads();
  if (tid < 64) {
    int base = 0;
    for (int d = 0; d <= depth; ++d) {  // level order: a node's parent is decided before it
      const int n0 = (1 << d) - 1, n1 = (2 << d) - 1;
      for (int c0 = n0; c0 < n1; c0 += 64) {
        const int n = c0 + lane;
        bool live = false, leaf = false;
        int f = -1;
        if (n < n1) {
          f = ft[n];
          live = n == 0 || (reach[(n - 1) >> 1] && ft[(n - 1) >> 1] >= 0);
          leaf = live && (f < 0 || d == depth);
        }
        const uint64_t m = __ballot(leaf);
        const int slot = base + __popcll(m & ((1ull << lane) - 1));
        if (n < n1) {
          reach[n] = live;
          slot_of[n] = leaf ? (int16_t)slot : (int16_t)-1;
          enc[n] = leaf ? (int16_t)(-(slot + 1)) : (live ? (int16_t)f : (int16_t)-1);
        }
        base += __popcll(m);
        __builtin_amdgcn_wave_barrier();  // (one wave: LDS writes above are visible to its next chunk)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      }
    }
    if (lane == 0) enc[511] = (int16_t)base;
  }
  __syncthreads();
  const f32x4* src = reinterpret_cast<const f32x4*>(value + (int64_t)t * nodes * 64);
  const int total = nodes * 16;  // float4s
  constexpr int U = 4;
  for (int i0 = tid; i0 < total; i0 += U * RFP_PREP_THREADS) {
    f32x4 v[U];
    int dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * RFP_PREP_THREADS;
      const int sl = i < total ? slot_of[i >> 4] : -1;
      dst[u] = sl >= 0 ? sl * 16 + (i & 15) : -1;
      if (dst[u] >= 0) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (dst[u] >= 0) vals[dst[u]] = v[u];
  }
}

// RFP_WAVES waves per workgroup, at most 2 x 64 rows per wave: 3 waves per SIMD hide the walk's
// dependent LDS reads, and 64 accumulators per row fit the 168 VGPRs a wave gets (a 3-group form at
// 2 waves per SIMD needed 192 accumulators and spilled 576 B per lane to scratch: 2.27 ms for 300 k
// rows x 100 trees, round 5)
constexpr int RFP_WAVES = 12;
template <int G>
__global__ void __launch_bounds__(RFP_WAVES * 64) rf_predict_lds(const uint64_t* __restrict__ X, int64_t N,
                                                      const uint8_t* __restrict__ prep, int T, int rows_per_wave,
                                                      int64_t rows_per_block, int out_logit, float* __restrict__ out,
                                                      int ldo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t rw0 = (int64_t)blockIdx.x * rows_per_block + (int64_t)wave * rows_per_wave;
  const int64_t rend = rw0 + rows_per_wave < N ? rw0 + rows_per_wave : N;
  uint32_t xlo[G], xhi[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t r = rw0 + 64 * g + lane;
    const uint64_t x = r < rend ? X[r] : 0ull;
    xlo[g] = (uint32_t)x;
    xhi[g] = (uint32_t)(x >> 32);
  }
  f32x4 acc[G][16];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[g][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)prep, 0, 0x7FFFFFFF, 0x00020000);
  // tree t's node table + leaf vectors -> LDS buffer t & 1: 1 + nleaf / 4 pieces of 1 KB, over the waves
  // (all 65 pieces whatever the tree's leaf count: reading the count first put one dependent global load
  // in front of every tree's DMA)
  auto stage = [&](int t) {
    char* dst = smem + (t & 1) * RFP_TREE;
    for (int pc = wave; pc < RFP_TREE / 1024; pc += RFP_WAVES)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (EM_LDS void*)(dst + pc * 1024), 16, (uint32_t)lane * 16,
                                               (uint32_t)t * RFP_TREE + (uint32_t)pc * 1024, 0, 0);
  };
  if (T > 0) stage(0);
  const uint32_t rot = (uint32_t)lane << 4;
  for (int t = 0; t < T; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tree t have landed
    __syncthreads();                                   // every wave's; and tree t - 1's buffer is free
    if (t + 1 < T) stage(t + 1);
    const char* buf = smem + (t & 1) * RFP_TREE;
    const int16_t* enc = reinterpret_cast<const int16_t*>(buf);
    // the G row groups walk the tree together: their dependent node reads are independent of each
    // other, so each step has G reads in flight instead of one
    int nd[G], f[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      nd[g] = 0;
      f[g] = rw0 + 64 * g < rend ? (int)enc[0] : -1;  // (wave-uniform: groups past the wave's rows stay out)
    }
    for (;;) {
      bool more = false;
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (f[g] >= 0) {
          const uint32_t w = f[g] < 32 ? xlo[g] : xhi[g];
          nd[g] = 2 * nd[g] + 1 + (int)((w >> (f[g] & 31)) & 1u);
          f[g] = enc[nd[g]];
          more |= f[g] >= 0;
        }
      if (!__builtin_amdgcn_ballot_w64(more)) break;
    }
    // leaf chunks: lane l reads chunk (l + c) & 15 at step c from base A = leaf + ((l & 15) << 4), or
    // A - 256 once the rotation wraps: one select per step and the step's 16 c in the instruction's
    // immediate offset.  4 steps at a time for every group together (the groups' reads in flight at
    // once), each batch's adds done before the next batch's reads issue (register budget).
    uint32_t A[G];
#pragma unroll
    for (int g = 0; g < G; ++g) A[g] = 1024u + (uint32_t)(-f[g] - 1) * 256u + (rot & 0xF0u);
#pragma unroll
    for (int c0 = 0; c0 < 16; c0 += 4) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (rw0 + 64 * g >= rend) break;  // (wave-uniform)
#pragma unroll
        for (int c = c0; c < c0 + 4; ++c) {
          const uint32_t base = ((lane & 15) + c >= 16) ? A[g] - 256u : A[g];
          acc[g][c] += *reinterpret_cast<const f32x4*>(buf + base + 16u * c);
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g)
        asm volatile("" : "+v"(acc[g][c0]), "+v"(acc[g][c0 + 1]), "+v"(acc[g][c0 + 2]), "+v"(acc[g][c0 + 3]));
    }
  }
  const float invT = 1.f / (float)(T > 0 ? T : 1);
  (void)invT;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t r = rw0 + 64 * g + lane;
    if (r >= rend) continue;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int k = (lane + c) & 15;  // output chunk held in register set c
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = 4 * k + e;
        float pr = T > 0 ? acc[g][c][e] / (float)T : 0.f;
        if (out_logit) {
          const float pc = fminf(fmaxf(pr, 1e-7f), 1.f - 1e-7f);
          pr = o < 62 ? __logf(pc / (1.f - pc)) : -30.f;
        } else if (o >= 62) {
          pr = 0.f;
        }
        v[e] = pr;
      }
      *reinterpret_cast<f32x4*>(out + r * ldo + 4 * k) = v;
    }
  }
}

}  // namespace

EM_API int em_rf_nodes(int max_depth) { return (1 << (max_depth + 1)) - 1; }

// bytes per row of the rows_a / rows_b scratch em_rf_fit expects: 16 (record form: one feature word with
// bits 62/63 free for the weight) or 4 (index form)
EM_API int em_rf_row_bytes(int W, int F, int64_t N) { return (W == 1 && F <= 62 && N <= (int64_t)RF_RMASK) ? 16 : 4; }

// per-level launch shape: blocks per node from the average node size (>= 4096 rows per block)
static void rf_shape(int64_t N, int level, int& B, int& nt) {
  const int64_t avg = N / (1ll << level);
  int64_t b = avg / 4096;
  B = (int)(b < 1 ? 1 : (b > 64 ? 64 : b));
  nt = avg >= 2048 ? RF_NT : 64;
}

EM_API int64_t em_rf_acc_words(int T, int max_depth, int k_feat) {
  if (T < 1 || max_depth < 0 || max_depth > 14 || k_feat < 1 || k_feat > RF_MAXF) return -1;
  // two levels' records (rf_child_totals) + a second candidate buffer (the fused partition fills the
  // next level's candidates while the current level's are still in use)
  // (+1: the fused driver's rf_ycheck flag, the last word)
  return 2 * (int64_t)T * (1ll << max_depth) * rec_words(k_feat) + ((int64_t)T * (1ll << max_depth) * k_feat + 1) / 2 + 1;
}

// Native level-wise driver: all T trees advance one level per (prep, hist, split, partition) round.
// scratch: cand int16 [T][2^D][k], acc uint32 [em_rf_acc_words], lrc int32 [T][2^D][2]
EM_API int em_rf_fit(const uint64_t* X, int W, const uint64_t* Y, int64_t N, int F, int T, int max_depth, int k_feat,
                     int min_leaf, int bootstrap, uint64_t seed, int t_off, void* rows_a, void* rows_b,
                     int32_t* seg, int16_t* feat, float* value, double* gain, float* cover, int16_t* cand,
                     uint32_t* acc, int32_t* lrc, int32_t* wl, hipStream_t stream) {
  if (!X || !Y || !rows_a || !rows_b || !seg || !feat || !value || !gain || !cover || !cand || !acc || !lrc || !wl)
    return EM_ERR_ARG;
  if (W < 1 || F < 1 || F > RF_MAXF || F > 64 * W || T < 1 || max_depth < 0 || max_depth > 14 || k_feat < 1 ||
      k_feat > RF_MAXF || min_leaf < 1 || N < 1 || N >= (1ll << 31))
    return EM_ERR_ARG;
  const int nodes = (1 << (max_depth + 1)) - 1;
  const int rec = rec_words(k_feat);
  const size_t lds = (size_t)rec * 4;
  if (lds > 160 * 1024 - 8192) return EM_ERR_ARG;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rf_hist<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 8192);
    (void)hipFuncSetAttribute((const void*)rf_hist<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 8192);
    (void)hipFuncSetAttribute((const void*)rf_hist<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 8192);
    (void)hipFuncSetAttribute((const void*)rf_hist<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 8192);
    (void)hipFuncSetAttribute((const void*)rf_partition<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 8192);
    attr = true;
  }
  // record-form row lists for one-word features (rows_a/rows_b hold 16 B per row: em_rf_row_bytes).
  // Variants measured slower and removed in round 5 (docs/DESIGN.md §2 keeps their numbers): the
  // matrix-core histogram (rf_hist_mfma: 7.0 vs 6.2 ms), node totals accumulated at every level instead
  // of derived from the parent (8.45 vs 6.67 ms), a separate histogram pass at every level (6.0 vs
  // 4.8-5.2 ms).
  const bool rec_rows = em_rf_row_bytes(W, F, N) == 16;
  uint32_t* accs[2] = {acc, acc + (int64_t)T * (1ll << max_depth) * rec};
  int16_t* cands[2] = {cand, reinterpret_cast<int16_t*>(acc + 2 * (int64_t)T * (1ll << max_depth) * rec)};
  // (the fused partition's replicated child images must fit the LDS: k <= ~70 candidates)
  const bool fuse = rec_rows && (size_t)2 * rf_chl_words(k_feat) * 4 <= 160 * 1024 - 8192 &&
                    (size_t)rf_init_lds_words(k_feat) * 4 <= 160 * 1024 - 8192;
  int32_t* yover = reinterpret_cast<int32_t*>(acc) + em_rf_acc_words(T, max_depth, k_feat) - 1;
  RfParams p{X, Y, N, W, F, T, max_depth, k_feat, min_leaf, bootstrap, t_off, nodes, seed, seg, feat, value, gain,
             cover, cand, accs[0], lrc, fuse ? yover : nullptr};
  (void)hipMemsetAsync(lrc, 0, (size_t)T * 2 * sizeof(int32_t), stream);
  {
    int B, nt;
    rf_shape(N, 0, B, nt);
    if (fuse) {  // the root records are accumulated by the listing pass
      (void)hipMemsetAsync(accs[0], 0, (size_t)T * rec * sizeof(uint32_t), stream);
      (void)hipMemsetAsync(yover, 0, sizeof(int32_t), stream);  // record form decided on the device
      const int64_t yb = (N + 255) / 256;
      hipLaunchKernelGGL(rf_ycheck, dim3((unsigned)(yb < 1024 ? yb : 1024)), dim3(256), 0, stream, Y, N, yover);
      static bool ra = false;
      if (!ra) {
        (void)hipFuncSetAttribute((const void*)rf_init_rows<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024 - 8192);
        ra = true;
      }
      hipLaunchKernelGGL((rf_init_rows<true, true>), dim3(B, T), dim3(RF_NT), (size_t)rf_init_lds_words(k_feat) * 4,
                         stream, p, (void*)rows_a);
    } else if (rec_rows)
      hipLaunchKernelGGL(rf_init_rows<true>, dim3(B, T), dim3(RF_NT), 0, stream, p, (void*)rows_a);
    else
      hipLaunchKernelGGL(rf_init_rows<false>, dim3(B, T), dim3(RF_NT), 0, stream, p, (void*)rows_a);
  }
  EM_CHECK_LAUNCH();
  void* rin = rows_a;
  void* rout = rows_b;
  const int64_t kept = bootstrap ? (N * 632) / 1000 : N;  // expected rows per tree (Poisson(1): 1 - 1/e)
  if (fuse) {
    // per level: rf_level_begin (segments, counters, work list), rf_split (also the children's totals,
    // zeroed records and candidates), the partition (also the children's histograms while a next
    // level still splits) -- 3 launches per level; the root's record came with the row lists
    for (int level = 0; level <= max_depth; ++level) {
      const int nodesL = 1 << level;
      int B, nt;
      rf_shape(kept, level, B, nt);
      (void)B;
      const int64_t tn = (int64_t)T * nodesL;
      p.acc = accs[level & 1];
      p.cand = cands[level & 1];
      hipLaunchKernelGGL(rf_level_begin, dim3(1), dim3(1024), 0, stream, p, level, wl, 0);
      const int64_t gmax = (int64_t)T * ((N + RF_CHUNK - 1) / RF_CHUNK + 1) + tn;
      const unsigned G = (unsigned)(gmax < 0x7FFFFFFF ? gmax : 0x7FFFFFFF);
      uint32_t* an = level < max_depth ? accs[(level + 1) & 1] : nullptr;
      int16_t* cn = level + 1 < max_depth ? cands[(level + 1) & 1] : nullptr;
      hipLaunchKernelGGL(rf_split, dim3(nodesL, T), dim3(cn ? 128 : 64), 0, stream, p, level, an, cn);
      EM_CHECK_LAUNCH();
      // rf_split of the level before the last wrote the last level's leaves (their rows are never read)
      if (level + 1 >= max_depth) break;
      hipLaunchKernelGGL((rf_partition<true, true>), dim3(G), dim3(nt), (size_t)2 * rf_chl_words(k_feat) * 4, stream,
                         p, (const void*)rin, rout,
                         level, (const int32_t*)wl, an, (const int16_t*)cn);
      EM_CHECK_LAUNCH();
      void* tmp = rin;
      rin = rout;
      rout = tmp;
    }
    return 0;
  }
  for (int level = 0; level <= max_depth; ++level) {
    const int nodesL = 1 << level;
    int B, nt;
    rf_shape(kept, level, B, nt);
    const int64_t tn = (int64_t)T * nodesL;
    p.acc = accs[level & 1];  // this level's node records and candidate lists (double-buffered)
    p.cand = cands[level & 1];
    hipLaunchKernelGGL(rf_level_prep, dim3((unsigned)((tn + 127) / 128)), dim3(128), 0, stream, p, level);
    hipLaunchKernelGGL(rf_worklist, dim3(1), dim3(1024), 0, stream, p, level, wl);
    // grid: an upper bound of the work list (the kernels exit past wl[tn])
    const int64_t gmax = (int64_t)T * ((N + RF_CHUNK - 1) / RF_CHUNK + 1) + tn;  // kept rows per tree <= N
    const unsigned G = (unsigned)(gmax < 0x7FFFFFFF ? gmax : 0x7FFFFFFF);
    (void)B;
    (void)hipMemsetAsync(p.acc, 0, (size_t)tn * rec * sizeof(uint32_t), stream);
    const bool dl = level > 0;  // node totals derived from the parent's histogram below the root
    if (dl) hipLaunchKernelGGL(rf_child_totals, dim3(nodesL, T), dim3(64), 0, stream, p, accs[(level - 1) & 1], level);
    if (dl && level == max_depth)
      ;  // the last level needs node totals only: all derived
    else if (rec_rows && dl)
      hipLaunchKernelGGL((rf_hist<true, true>), dim3(G), dim3(nt), lds, stream, p, (const void*)rin, level, (const int32_t*)wl);
    else if (rec_rows)
      hipLaunchKernelGGL((rf_hist<true, false>), dim3(G), dim3(nt), lds, stream, p, (const void*)rin, level, (const int32_t*)wl);
    else if (dl)
      hipLaunchKernelGGL((rf_hist<false, true>), dim3(G), dim3(nt), lds, stream, p, (const void*)rin, level, (const int32_t*)wl);
    else
      hipLaunchKernelGGL((rf_hist<false, false>), dim3(G), dim3(nt), lds, stream, p, (const void*)rin, level, (const int32_t*)wl);
    hipLaunchKernelGGL(rf_split, dim3(nodesL, T), dim3(64), 0, stream, p, level, (uint32_t*)nullptr,
                       (int16_t*)nullptr);
    EM_CHECK_LAUNCH();
    if (level == max_depth) break;
    (void)hipMemsetAsync(lrc, 0, (size_t)tn * 2 * sizeof(int32_t), stream);
    if (rec_rows) {
      hipLaunchKernelGGL((rf_partition<true, false>), dim3(G), dim3(nt), 0, stream, p, (const void*)rin, rout, level,
                         (const int32_t*)wl, (uint32_t*)nullptr, (const int16_t*)nullptr);
    } else {
      hipLaunchKernelGGL((rf_partition<false, false>), dim3(G), dim3(nt), 0, stream, p, (const void*)rin, rout, level,
                         (const int32_t*)wl, (uint32_t*)nullptr, (const int16_t*)nullptr);
    }
    EM_CHECK_LAUNCH();
    void* tmp = rin;
    rin = rout;
    rout = tmp;
  }
  return 0;
}

// scratch bytes em_rf_predict's tree-streamed path needs (0: that path does not apply)
EM_API int64_t em_rf_predict_scratch(int W, int T, int max_depth) {
  // rf_predict_lds addresses tree t at the 32-bit buffer offset t * RFP_TREE: forests whose images would
  // pass 2^31 bytes (~32 k trees) take the one-wave-per-row kernel instead of reading out of range
  if (W != 1 || max_depth > 8 || T <= 0 || (int64_t)T * RFP_TREE >= (int64_t(1) << 31)) return 0;
  return (int64_t)T * RFP_TREE;
}

// prep: em_rf_predict_scratch(W, T, max_depth) bytes (16-B aligned), or null for the one-wave-per-row path
EM_API int em_rf_predict(const uint64_t* X, int W, int64_t N, const int16_t* feat, const float* value, int T,
                         int max_depth, int out_logit, float* out, int ldo, void* prep, hipStream_t stream) {
  if (!X || !feat || !value || !out || W < 1 || N < 0 || T < 0 || ldo < 64 || max_depth < 0 || max_depth > 14)
    return EM_ERR_ARG;
  if (N == 0) return 0;
  const int nodes = (1 << (max_depth + 1)) - 1;
  if (prep && em_rf_predict_scratch(W, T, max_depth) > 0 && ((uintptr_t)prep & 15) == 0 && (ldo & 3) == 0 &&
      ((uintptr_t)out & 15) == 0) {
    hipLaunchKernelGGL(rf_predict_prepare, dim3(T), dim3(RFP_PREP_THREADS), 0, stream, feat, value, nodes, max_depth, (uint8_t*)prep);
    EM_CHECK_LAUNCH();
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
      (void)hipFuncSetAttribute((const void*)rf_predict_lds<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * RFP_TREE);
      (void)hipFuncSetAttribute((const void*)rf_predict_lds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * RFP_TREE);
    }
    // one workgroup per CU (the LDS double buffer), rows spread evenly; at most 2 x 64 rows per wave
    constexpr int NW = RFP_WAVES;
    int64_t grid = (N + 64 * NW - 1) / (64 * NW);
    if (grid > cus) grid = cus;
    int64_t rpw = ((N + grid - 1) / grid + NW - 1) / NW;
    if (rpw > 128) {
      rpw = 128;
      grid = (N + NW * rpw - 1) / (NW * rpw);
    }
    const int G = (int)((rpw + 63) / 64);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NW * 64), 2 * RFP_TREE, stream, X, N, (const uint8_t*)prep,
                         T, (int)rpw, NW * rpw, out_logit, out, ldo);
    };
    if (G == 1) go(rf_predict_lds<1>);
    else go(rf_predict_lds<2>);
    EM_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(rf_predict, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, stream, X, W, N, feat, value, T, nodes,
                     out_logit, out, ldo);
  EM_CHECK_LAUNCH();
  return 0;
}
