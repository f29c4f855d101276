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
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

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

// (Round 4's hipGraph-replayed rounds, which offset every per-round array by a device round counter,
// measured slower than the eager stream -- 0.056 vs 0.049 s on the reference fit -- and were removed
// in round 5 together with that counter; docs/DESIGN.md §6c keeps the numbers.)

// GBDT_STAMPS=1 builds (tools/build_variant.sh): block 0's wall clock at phase boundaries of the round
// kernels, slot = kernel base + phase (em_gbdt_stamps copies them out); compiled out otherwise
#ifndef GBDT_STAMPS
#define GBDT_STAMPS 0
#endif
#if GBDT_STAMPS
__device__ unsigned long long g_stamp[512];  // [0, 256): 100 MHz wall clock, [256, 512): shader clock
#define GSTAMP(slot) \
  do { \
    if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) { \
      g_stamp[(slot) & 255] = wall_clock64(); \
      g_stamp[256 + ((slot) & 255)] = __builtin_amdgcn_s_memtime(); \
    } \
  } while (0)
#else
#define GSTAMP(slot) \
  do { \
  } while (0)
#endif

EM_DEVICE void round_init_elem(int i, int8_t* st, int16_t* fe, uint8_t* sb, float* gn, int NN) {
  st[i] = (i % NN) == 0 ? 2 : 0;
  fe[i] = -1;
  sb[i] = 0;
  gn[i] = 0.f;
}

// per-round tree reset: status/feature/bin/gain cleared, every task's root opened (status 2)
__global__ void gbdt_round_init(int8_t* __restrict__ st, int16_t* __restrict__ fe, uint8_t* __restrict__ sb,
                                float* __restrict__ gn, int total, int NN) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x)
    round_init_elem(i, st, fe, sb, gn, NN);
}

__global__ void gbdt_init_margin(float* __restrict__ margin, int64_t total, float base) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    margin[i] = base;
}

// g / h of one (task t, row r) element of round `round` from its margin m and label y (per-task
// objectives; the row subsample's hash drops the element)
EM_DEVICE void grad_of(float m, float y, int obj, float subsample, uint32_t seed, int round, int t, int r, float& gg,
                       float& hh) {
  if (obj == OBJ_LOGISTIC) {
    const float p = 1.f / (1.f + expf(-m));
    gg = p - y;
    hh = fmaxf(p * (1.f - p), 1e-16f);
  } else {
    gg = m - y;
    hh = 1.f;
  }
  if (subsample < 1.f) {
    const float u = (hash3(seed, (uint32_t)round * 131071u + t, r) >> 8) * (1.f / 16777216.f);
    if (u >= subsample) gg = hh = 0.f;
  }
}

// margin/g/h/node: [T][n]; Y: [n][T]
EM_DEVICE void grad_elem(int64_t i, const float* __restrict__ margin, const float* __restrict__ Y,
                         float* __restrict__ g, float* __restrict__ h, int16_t* __restrict__ node, int T, int n,
                         int obj, float subsample, uint32_t seed, int round) {
  const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
  const float m = margin[i], y = Y[(int64_t)r * T + t];
  float gg, hh;
  if (obj == OBJ_SOFTMAX) {  // XGBoost SoftmaxMultiClassObj: g = p - y, h = max(2p(1-p), eps)
    const float p = softmax_p(margin, T, n, r, t);
    gg = p - y;
    hh = fmaxf(2.f * p * (1.f - p), 1e-16f);
    if (subsample < 1.f) {
      const float u = (hash3(seed, (uint32_t)round * 131071u + t, r) >> 8) * (1.f / 16777216.f);
      if (u >= subsample) gg = hh = 0.f;
    }
  } else {
    grad_of(m, y, obj, subsample, seed, round, t, r, gg, hh);
  }
  g[i] = gg;
  h[i] = hh;
  node[i] = 0;
}

__global__ void gbdt_grad(const float* __restrict__ margin, const float* __restrict__ Y, float* __restrict__ g,
                          float* __restrict__ h, int16_t* __restrict__ node, int T, int n, int obj, float subsample,
                          uint32_t seed, int round) {
  const int64_t total = (int64_t)T * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    grad_elem(i, margin, Y, g, h, node, T, n, obj, subsample, seed, round);
}

// round_init + grad in one launch (independent element spaces; the reference-size fit is launch-bound)
__global__ void gbdt_round_start(int8_t* __restrict__ st, int16_t* __restrict__ fe, uint8_t* __restrict__ sb,
                                 float* __restrict__ gn, int TNN, int NN, const float* __restrict__ margin,
                                 const float* __restrict__ Y, float* __restrict__ g, float* __restrict__ h,
                                 int16_t* __restrict__ node, int T, int n, int obj, float subsample, uint32_t seed,
                                 int round) {
  const int64_t total = (int64_t)T * n;
  const int64_t all = total > TNN ? total : TNN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < all; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < TNN) round_init_elem((int)i, st, fe, sb, gn, NN);
    if (i < total) grad_elem(i, margin, Y, g, h, node, T, n, obj, subsample, seed, round);
  }
}

EM_DEVICE int leaf_ancestor(const int8_t* st, int nd);
EM_DEVICE double metric_term(float m, float y, int obj, int metric);

// eval sets handled by trailing blocks of the update launch (or, see HistUpdate, by extra blocks of the
// next round's level-0 histogram pass)
struct EvalSets {
  const uint8_t* bins[4];
  float* margin[4];
  const float* Y[4];
  int n[4];
  int mb[4];
  int count = 0;
  int64_t pstride = 4096;  // doubles between the sets' partial regions
};

// The level-0 histogram pass of round r doing the rows' part of round r - 1's update (exact fused form,
// per-task objectives, one block per (chunk, task)): a block stages its rows' (g, h) by computing them --
// the margin plus the leaf of round r - 1's tree (its last partition applied here), the metric term of
// round r - 1, round r's g / h -- and writes margin, g, h and the reset node ids for the later levels;
// extra blocks (z >= nz) predict round r - 1's trees on the eval sets.  The update launch of every
// round but the last is gone; the arithmetic per element is the update's, so trees and margins are
// bit-identical to the separate launches (the metric's per-block partial sums are grouped by chunk).
struct HistUpdate {
  int on = 0;     // compute the rows' g / h (round `round`) and initialise round `round`'s tree arrays
  int apply = 0;  // first apply round - 1's tree (margins, metric partials, eval sets)
  int round = 0, obj = 0, metric = 0, NN = 0, plevel = 0, nz = 1;
  float subsample = 1.f;
  uint32_t seed = 0;
  float* margin = nullptr;
  const float* Y = nullptr;
  float* g = nullptr;
  float* h = nullptr;
  int16_t* node = nullptr;
  int8_t* st = nullptr;  // round `round`'s tree arrays (task-major [T][NN])
  int16_t* fe = nullptr;
  uint8_t* sb = nullptr;
  float* gn = nullptr;
  const int8_t* pst = nullptr;  // round - 1's
  const int16_t* pfe = nullptr;
  const uint8_t* psb = nullptr;
  const float* plf = nullptr;
  const int16_t* pnode = nullptr;  // the rows' nodes before round - 1's last partition
  double* mpart = nullptr;         // round - 1's deferred partials: train [T * chunks], eval set s at (1 + s) * mstride
  int64_t mstride = 0;
  EvalSets evs;
};

// fixed-order block sum (<= 1024 threads; thread 0 gets the result): a butterfly per wave, then the
// waves in order.  (128 B of static LDS: the histogram kernels' dynamic LDS may take all the rest)
EM_DEVICE double block_sum_waves(double acc) {
  __shared__ double wsum[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  double tot = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < ((int)blockDim.x + 63) >> 6; ++w) tot += wsum[w];
  return tot;
}

struct SplitFinal {
  int* tctr = nullptr;  // [T] zeroed arrival counters (left zeroed)
  float* leaf = nullptr;
  float* cover = nullptr;
  float gamma = 0.f;
  double eta = 0.0;
  int max_depth = 0;
};
EM_DEVICE void prune_task(int8_t* st, int16_t* fe, const float* gn, int max_depth, float gamma);
template <typename A, bool COH, int NPRE = 32>
EM_DEVICE void split_body(int vb, char* smem, const A* __restrict__ hist, int nchunks, int64_t cstride,
                          const int* __restrict__ foff, int T, int F, int C, int level, int NN, double* __restrict__ G,
                          double* __restrict__ H, int8_t* __restrict__ status, int16_t* __restrict__ feat,
                          uint8_t* __restrict__ sbin, float* __restrict__ gain, double lam, double mcw, double qinv,
                          SplitFinal fin, int oneshot, int pscan, const int4* __restrict__ cellinfo);

// The level-0 histogram pass splitting its task's root itself (exact fused rounds, with HistUpdate): every
// chunk block stores its partials write-through (agent-scope), drains them, and adds to the task's
// counter; the last-arriving block reads them back with agent-scope loads and runs the split (gbdt_split's
// body) -- the "write-through stores + vmcnt(0) + relaxed arrival" hand-off of the fused finalize.  The
// round's tree arrays are initialised with write-through stores too (a plain store could sit in another
// XCD's L2 and be written back over the split's results).  One launch less per round.
struct HistSplit {
  int on = 0;
  int* ctr = nullptr;  // [T] arrival counters (left zeroed)
  double* G = nullptr;
  double* H = nullptr;
  double lam = 0.0, mcw = 0.0;
  SplitFinal fin;
  int oneshot = 0, pscan = 0, NN = 0;
  int64_t cstride = 0;
  const int4* cellinfo = nullptr;
};

// The previous level's split run by the leading blocks of a histogram pass (levels >= 2 of the exact fused
// round): z-planes 0 .. nz - 1 are split blocks (node zb * gridDim.x + x of task y), the
// remaining planes the histogram.  Split blocks come first in dispatch order; each runs gbdt_split's body
// (its stores are write-through), drains them and adds 1 to its task's counter.  A histogram block of task
// t polls that counter (one lane, agent-scope loads, bounded) until the task's nodes are all decided, then
// reads the split arrays with agent-scope loads -- the "write-through stores + vmcnt(0) + relaxed arrival"
// hand-off of HistSplit.  A task's next level starts when its own splits finish instead of at a launch
// boundary; no block waits on another task.  The levels' chunk partials alternate between two buffer halves,
// so this level's histogram never overwrites what the split blocks still read.  Counters are cumulative
// over the fit (want = the running total); a timed-out poll raises err[0] (em_gbdt_fused_error).
struct HistPre {
  int on = 0, nz = 0, nodes = 0, level = 0, nchunks = 0, oneshot = 0, pscan = 0, NN = 0;
  int want = 0;
  int* ctr = nullptr;  // [T] cumulative arrivals
  int* err = nullptr;  // set when a poll timed out (em_gbdt_fused_error)
  const double* hist = nullptr;
  int64_t cstride = 0;
  double* G = nullptr;
  double* H = nullptr;
  int8_t* st = nullptr;
  int16_t* fe = nullptr;
  uint8_t* sb = nullptr;
  float* gn = nullptr;
  double lam = 0.0, mcw = 0.0;
  const int4* cellinfo = nullptr;
};
constexpr int64_t PRE_SPIN_LIMIT = 1ll << 24;  // ~1 s of polling at s_sleep 1: a legitimate wait is microseconds

// ---------------------------------------------------------------- K8 histogram (compact cells)
// Cells: feature f owns bins [foff[f], foff[f+1]) of a compact axis of C = foff[F] cells (a one-hot
// lag feature has 2 cells, "day" 31 ...), so a (task, node) histogram of the reference features is
// ~200 cells (3 KB of double pairs) instead of F x max_bins.
// Work split: block = (row chunk, task, tile); tile = FT features x NTn nodes; thread (p, fl) owns
// feature f0 + fl for the p-th contiguous sub-range of each staged piece of the chunk's rows.
// Two forms, chosen per fit by the host (models/gbdt.py quant_bits):
//  * exact (fp64, gbdt_hist): no atomics -- every thread accumulates its private LDS copy in row
//    order, the P copies are folded in p order and the chunks by gbdt_chunk_reduce in chunk order,
//    so two features that induce the same partition of the rows get bit-identical sums (exact gain
//    ties keep breaking towards the lower feature).  Per row a thread does one 16-B LDS
//    read-modify-write; that serial chain bounds the kernel (1.17 ms per level at 183k rows x 62
//    tasks, profiles/README.md).
//  * fixed point (gbdt_hist_q): g and h are quantised per row to int64 (q = rint(x * 2^s), s chosen
//    so that any sum over the n rows stays below 2^61) and accumulated with non-returning LDS
//    integer atomics into ONE shared copy: integer addition is exact and order-free, so the sums
//    are deterministic without the per-thread copies or the serial chain, and the numpy oracle
//    reproduces them exactly (models/gbdt.py _quant_hist).
constexpr int HIST_MAX_CHUNK = 1024;             // rows staged in LDS per piece
constexpr int64_t HIST_PARTIAL_CAP = 1ll << 27;  // 8-byte words of per-chunk partials (1 GiB) per level
constexpr int HIST_LDS_BUDGET = 36 * 1024;       // per-block histogram copies (+ staged rows)
// exact form: up to 8 private copies in a 512-thread block (round 5, with 256-row chunks; round 4 had
// measured 512-thread blocks slower with 64-row chunks, where they only added blocks' LDS)
// (side-build knobs: GBDT_HIST_THREADS / GBDT_HIST_PMAX / GBDT_HIST_LDS_KB)
#ifndef GBDT_HIST_THREADS
#define GBDT_HIST_THREADS 512
#endif
#ifndef GBDT_HIST_PMAX
#define GBDT_HIST_PMAX 8
#endif
#ifndef GBDT_HIST_LDS_KB
#define GBDT_HIST_LDS_KB 72
#endif
constexpr int HIST_EXACT_LDS_BUDGET = GBDT_HIST_LDS_KB * 1024;
constexpr int HIST_EXACT_THREADS = GBDT_HIST_THREADS;
// partial loads in flight per thread of the split inside the level-0 histogram pass (see GBDT_SPLIT_NPRE):
// 4 x 512 threads cover a root's 1488 doubles; 4 instead of 16 takes the histogram kernel from 126 to 69
// VGPRs, +3.1 % trees/s (profiles/r5/gbdt_hist_regs_ab.txt)
#ifndef GBDT_HSPLIT_NPRE
#define GBDT_HSPLIT_NPRE 4
#endif
// gbdt_hist's dynamic LDS ceiling: 160 KB less 2 KB for its static LDS (block_sum_waves, two split_body
// instantiations: 1200 B); setting the attribute to the full 160 KB fails once the kernel has any static
// LDS (and leaves hipErrorInvalidValue as the last error, which the next launch check reports)
constexpr int GBDT_HIST_MAX_DYN = 158 * 1024;
constexpr int HIST_QBIN_LDS = 16 * 1024;         // fixed point: staged bin bytes per piece
// rows per histogram chunk at least HIST_MIN_CHUNK (compile-time A/B knob for side builds,
// tools/build_variant.sh -DHIST_MIN_CHUNK=...; the split folds one partial per chunk).  Round 5 on the
// reference fit (trees/s, same box, profiles/r5/gbdt_chunk_ab.txt, gbdt_threads_ab.txt): 256-thread
// blocks with up to 4 row phases, 64-row chunks 689 k -> 128-row chunks 733 k; 512-thread blocks with
// up to 8 phases (72 KB of private copies) and 256-row chunks 765 k (128-row: 737 k): half the blocks
// per level, and each thread's serial update chain stays at ~37 rows.
#ifndef HIST_MIN_CHUNK
#define HIST_MIN_CHUNK 256
#endif

__global__ void __launch_bounds__(HIST_EXACT_THREADS)
gbdt_hist(const uint8_t* __restrict__ bins, const float* __restrict__ g, const float* __restrict__ h,
          const int16_t* __restrict__ node, const int* __restrict__ foff, double* __restrict__ partial, int T, int n,
          int F, int C, int level, int chunk, int FT, int NTn, int P, int ldsC, int piece, int stage_rows,
          int16_t* __restrict__ node_out, const int8_t* __restrict__ pst, const int16_t* __restrict__ pfe,
          const uint8_t* __restrict__ psb, int NN, HistUpdate hu, HistSplit hsp, HistPre pre) {
  // stage_rows > 0: each piece's bin rows are staged in LDS with 16-B loads (one round trip instead of
  // one per 8 rows of byte loads); the host sets it when a piece's rows fit (stage_rows * F <= 16 KB).
  // node_out != nullptr (level >= 1): the rows' nodes are the previous level's partition, applied here
  // (gbdt_partition's rule on the round's split arrays pst / pfe / psb, staged in LDS), and the
  // (chunk, task)'s first tile block writes them to node_out for the next level -- one launch less per level
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nodesL = 1 << level, first = nodesL - 1;
  GSTAMP(64 + 16 * level);
  const int c = blockIdx.x, t = blockIdx.y;
  if (pre.on && (int)blockIdx.z < pre.nz) {  // a split block of the previous level (see HistPre)
    const int nd = (int)blockIdx.z * (int)gridDim.x + c;
    if (nd < pre.nodes) {
      split_body<double, false, GBDT_HSPLIT_NPRE>(t * pre.nodes + nd, smem, pre.hist, pre.nchunks, pre.cstride, foff, T,
                                                  F, C, pre.level, pre.NN, pre.G, pre.H, pre.st, pre.fe, pre.sb,
                                                  pre.gn, pre.lam, pre.mcw, 0.0, SplitFinal(), pre.oneshot, pre.pscan,
                                                  pre.cellinfo);
      if (threadIdx.x == 0) {  // (thread 0 made every store of the split, all write-through)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(pre.ctr + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  const int zb = (int)blockIdx.z - (pre.on ? pre.nz : 0);  // this block's plane of the histogram pass
  if (pre.on) {  // the task's previous-level nodes must all be decided before their partition is applied
    if (threadIdx.x == 0) {  // (the other threads load the split arrays after the barrier below)
      int64_t spins = 0;
      while (__hip_atomic_load(pre.ctr + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < pre.want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > PRE_SPIN_LIMIT) {
          __hip_atomic_fetch_or(pre.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
  }
  if (hu.apply && zb >= hu.nz) {  // eval set es: round - 1's tree of task t on a chunk of its rows
    // (the set's fields picked with selects: a dynamic index into the by-value argument arrays would
    // copy them to scratch memory for every block of the launch)
    const int es = zb - hu.nz;
    auto pick = [es](auto a0, auto a1, auto a2, auto a3) { return es == 0 ? a0 : es == 1 ? a1 : es == 2 ? a2 : a3; };
    const uint8_t* ebins = pick(hu.evs.bins[0], hu.evs.bins[1], hu.evs.bins[2], hu.evs.bins[3]);
    float* emargin = pick(hu.evs.margin[0], hu.evs.margin[1], hu.evs.margin[2], hu.evs.margin[3]);
    const float* eY = pick(hu.evs.Y[0], hu.evs.Y[1], hu.evs.Y[2], hu.evs.Y[3]);
    const int ne = pick(hu.evs.n[0], hu.evs.n[1], hu.evs.n[2], hu.evs.n[3]), per = (ne + (int)gridDim.x - 1) / (int)gridDim.x;
    const int eb = c * per, ee = min(ne, eb + per);
    const int64_t o = (int64_t)t * hu.NN;
    double acc = 0.0;
    for (int r = eb + (int)threadIdx.x; r < ee; r += blockDim.x) {
      const uint8_t* row = ebins + (int64_t)r * F;
      int nd = 0;
      while (hu.pst[o + nd] == 1) nd = 2 * nd + 1 + (row[hu.pfe[o + nd]] > hu.psb[o + nd] ? 1 : 0);
      const int64_t i = (int64_t)t * ne + r;
      const float m = emargin[i] + hu.plf[o + nd];
      emargin[i] = m;
      acc += metric_term(m, eY[(int64_t)r * T + t], hu.obj, hu.metric);
    }
    const double bs = block_sum_waves(acc);
    if (threadIdx.x == 0) hu.mpart[(1 + es) * hu.mstride + (int64_t)t * gridDim.x + c] = bs;
    return;
  }
  double macc = 0.0;  // (hu.apply) round - 1's metric terms of this thread's rows
  const int nft = (F + FT - 1) / FT;
  const int ft = zb % nft, nt = zb / nft;
  const int f0 = ft * FT, f1 = min(F, f0 + FT), n0 = nt * NTn;
  const int c0 = foff[f0], c1 = foff[f1], Ct = c1 - c0;
  double* hist = reinterpret_cast<double*>(smem);  // [P][NTn][ldsC][2]
  const int per = NTn * ldsC * 2;
  for (int i = threadIdx.x; i < P * per; i += blockDim.x) hist[i] = 0.0;  // (ordered by the loop's first barrier)
  float* sg = reinterpret_cast<float*>(smem + (size_t)P * per * sizeof(double));
  float* sh = sg + piece;
  int16_t* sn = reinterpret_cast<int16_t*>(sh + piece);
  // the previous level's split arrays of this task (nodes pf .. first - 1): int32 {status | sbin << 8 | feat << 16}
  int32_t* ptree = reinterpret_cast<int32_t*>(smem + (((size_t)P * per * 8 + (size_t)piece * 10 + 15) & ~(size_t)15));
  const int pf = (first - 1) >> 1, npn = node_out ? first - pf : 0;
  u32x4* sbw = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(ptree) + (((size_t)npn * 4 + 15) & ~(size_t)15));
  if (npn) {
    const int64_t k0 = (int64_t)t * NN + pf;
    for (int i = threadIdx.x; i < npn; i += blockDim.x) {
      if (pre.on) {  // written in this launch by the split blocks (write-through): agent-scope loads
        const int8_t a = __hip_atomic_load(pst + k0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint8_t b = __hip_atomic_load(psb + k0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int16_t e = __hip_atomic_load(pfe + k0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ptree[i] = (int32_t)(uint8_t)a | ((int32_t)b << 8) | ((int32_t)e << 16);
      } else {
        ptree[i] = (int32_t)(uint8_t)pst[k0 + i] | ((int32_t)psb[k0 + i] << 8) | ((int32_t)pfe[k0 + i] << 16);
      }
    }
  }
  const int64_t base = (int64_t)t * n;
  const int nth = f1 - f0;
  const int p = threadIdx.x / nth, fl = threadIdx.x - p * nth;
  const int f = f0 + (p < P ? fl : 0);
  double* my = hist + (size_t)(p < P ? p : 0) * per + (foff[f] - c0) * 2;
  const int64_t nbytes = (int64_t)n * F;
  // the block's rows [c*chunk, +chunk) in staged pieces of <= piece rows: per piece the rows'
  // (node, g, h) go to LDS once, shared by every feature thread, then thread (p, fl) adds the p-th
  // contiguous part of the piece to its copy in row order
  const int rb = c * chunk, re = min(n, rb + chunk);
  for (int r0 = rb; r0 < re; r0 += piece) {
    const int r1 = min(re, r0 + piece);
    __syncthreads();  // the previous piece's staging is consumed
    // the piece's bin rows: bytes [r0 F, r1 F) as 16-B words (range-checked buffer loads; a word running
    // past the array's end is assembled bytewise), row r's byte f at rowb[(r - r0) F + f]
    const uint8_t* rowb = bins + (int64_t)r0 * F;
    if (stage_rows) {
      const int64_t w0 = ((int64_t)r0 * F) >> 4;
      const int boff = (int)(((int64_t)r0 * F) & 15);
      const int nw = (int)((((int64_t)r1 * F + 15) >> 4) - w0);
      const int64_t left = nbytes - w0 * 16;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(bins + w0 * 16), 0, (int)(left < 0x7FFFFFF0 ? left : 0x7FFFFFF0), 0x00020000);
      const bool tail = (w0 + nw) * 16 > nbytes;
      for (int i = threadIdx.x; i < nw - (tail ? 1 : 0); i += blockDim.x)
        sbw[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, 0));
      if (tail && threadIdx.x == 0) {
        uint8_t* wb = reinterpret_cast<uint8_t*>(sbw + nw - 1);
        for (int k = 0; k < 16; ++k) {
          const int64_t q = (w0 + nw - 1) * 16 + k;
          wb[k] = q < nbytes ? bins[q] : 0;
        }
      }
      rowb = reinterpret_cast<const uint8_t*>(sbw) + boff;
    }
    for (int r = r0 + (int)threadIdx.x; r < r1; r += blockDim.x) {
      if (hu.on) {  // (level 0, one tile per (chunk, task): this thread is the row's only writer)
        const int64_t i = base + r;
        const float y = hu.Y[(int64_t)r * T + t];
        float m = hu.margin[i];
        if (hu.apply) {  // round - 1's last partition and leaf (gbdt_update_metric's arithmetic)
          const int64_t o = (int64_t)t * hu.NN;
          const int ppf = (1 << hu.plevel) - 1, ppl = 2 * ppf + 1;
          int nd = hu.pnode[i];
          if (nd >= ppf && nd < ppl && hu.pst[o + nd] == 1)
            nd = 2 * nd + 1 + (bins[(int64_t)r * F + hu.pfe[o + nd]] > hu.psb[o + nd] ? 1 : 0);
          m = m + hu.plf[o + leaf_ancestor(hu.pst + o, nd)];
          hu.margin[i] = m;
          macc += metric_term(m, y, hu.obj, hu.metric);
        }
        float gg, hh;
        grad_of(m, y, hu.obj, hu.subsample, hu.seed, hu.round, t, r, gg, hh);
        hu.g[i] = gg;
        hu.h[i] = hh;
        hu.node[i] = 0;
        sg[r - r0] = gg;
        sh[r - r0] = hh;
        sn[r - r0] = 0;  // every row at the root
        continue;
      }
      sg[r - r0] = g[base + r];
      sh[r - r0] = h[base + r];
      const int nd = node[base + r];
      sn[r - r0] = (int16_t)(npn ? nd : nd - first - n0);  // tile-relative node (outside -> skipped)
    }
    __syncthreads();
    GSTAMP(64 + 16 * level + 1);
    if (npn) {  // the previous level's partition on the staged rows
      for (int r = r0 + (int)threadIdx.x; r < r1; r += blockDim.x) {
        int nd = sn[r - r0];
        if (nd >= pf && nd < first) {
          const int32_t e = ptree[nd - pf];
          if ((e & 0xFF) == 1) nd = 2 * nd + 1 + ((int)rowb[(int64_t)(r - r0) * F + (e >> 16)] > ((e >> 8) & 0xFF) ? 1 : 0);
        }
        if (zb == 0) node_out[base + r] = (int16_t)nd;
        sn[r - r0] = (int16_t)(nd - first - n0);
      }
      __syncthreads();
      GSTAMP(64 + 16 * level + 2);
    }
    if (p < P) {
      const int len = r1 - r0, sub = (len + P - 1) / P;
      const int a0 = min(len, p * sub), a1 = min(len, a0 + sub);
      const uint8_t* col = rowb + f;
      int r = a0;
      // 8 rows' inputs first, then their 8 updates in row order (sums bitwise = the plain loop)
      for (; r + 8 <= a1; r += 8) {
        int b[8], nd[8];
        float gv[8], hv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          b[u] = col[(int64_t)(r + u) * F];
          nd[u] = sn[r + u];
          gv[u] = sg[r + u];
          hv[u] = sh[r + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if ((unsigned)nd[u] >= (unsigned)NTn) continue;
          double* e = my + (nd[u] * ldsC + b[u]) * 2;
          e[0] += (double)gv[u];
          e[1] += (double)hv[u];
        }
      }
      for (; r < a1; ++r) {
        const int nd = sn[r];
        if ((unsigned)nd >= (unsigned)NTn) continue;
        double* e = my + (nd * ldsC + col[(int64_t)r * F]) * 2;
        e[0] += (double)sg[r];
        e[1] += (double)sh[r];
      }
    }
  }
  __syncthreads();
  GSTAMP(64 + 16 * level + 3);
  // fold the P copies (p order) and write this chunk's cells: partial [nchunks][T][nodesL][C][2]
  double* out = partial + ((int64_t)c * T + t) * (int64_t)nodesL * C * 2;
  const int nn = min(NTn, nodesL - n0);
  for (int i = threadIdx.x; i < nn * Ct; i += blockDim.x) {
    const int nd = i / Ct, cc = i - nd * Ct;
    double sgv = 0.0, shv = 0.0;
    for (int q = 0; q < P; ++q) {
      const double* e = hist + (size_t)q * per + (nd * ldsC + cc) * 2;
      sgv += e[0];
      shv += e[1];
    }
    double* o = out + ((int64_t)(n0 + nd) * C + c0 + cc) * 2;
    if (hsp.on) {  // (write-through: read back by this task's last-arriving block)
      __hip_atomic_store(o, sgv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 1, shv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      o[0] = sgv;
      o[1] = shv;
    }
  }
  if (hu.apply) {
    const double bs = block_sum_waves(macc);
    if (threadIdx.x == 0) hu.mpart[(int64_t)t * gridDim.x + c] = bs;
  }
  if (hu.on && c == 0) {  // round `round`'s tree arrays of task t
    for (int k = threadIdx.x; k < hu.NN; k += blockDim.x) {
      const int e = t * hu.NN + k;
      if (hsp.on) {
        __hip_atomic_store(hu.st + e, (int8_t)(k == 0 ? 2 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hu.fe + e, (int16_t)-1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hu.sb + e, (uint8_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hu.gn + e, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        round_init_elem(e, hu.st, hu.fe, hu.sb, hu.gn, hu.NN);
      }
    }
  }
  if (hsp.on) {
    __shared__ int lastblk;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's write-through stores have completed
    __syncthreads();                                   // ... and every thread's
    if (threadIdx.x == 0)
      lastblk = __hip_atomic_fetch_add(hsp.ctr + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    if (lastblk) {
      if (threadIdx.x == 0) __hip_atomic_store(hsp.ctr + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      split_body<double, true, GBDT_HSPLIT_NPRE>(t, smem, partial, gridDim.x, hsp.cstride, foff, T, F, C, 0, hsp.NN, hsp.G, hsp.H,
                               hu.st, hu.fe, hu.sb, hu.gn, hsp.lam, hsp.mcw, 0.0, hsp.fin, hsp.oneshot, hsp.pscan,
                               hsp.cellinfo);
    }
  }
  GSTAMP(64 + 16 * level + 4);
}

// fixed-point value of x * 2^s (x a float, |x * 2^s| < 2^62): the product is exact (power-of-two
// scale), rint rounds half to even like numpy's np.rint, and the int64 conversion of an integral
// double is exact
EM_DEVICE long long quantise(float x, double scale) { return (long long)__builtin_rint((double)x * scale); }
// hessians: a positive h never rounds to 0 (the 1e-16 floor of a saturated row would at s < 53, and a
// node of such rows would then have H = 0 exactly where the exact form keeps H > 0: with
// min_child_weight = lambda = 0 its gain and leaf divide by zero).  models/gbdt.py _quantise_h agrees.
EM_DEVICE long long quantise_h(float x, double scale) {
  const long long q = quantise(x, scale);
  return (x > 0.f && q < 1) ? 1 : q;
}

// LDS layout of the fixed-point form: two planes (g sums, then h sums) of 8-byte cells, so a lane's
// atomic touches one 8-byte word, and one pad cell after every feature's bins: with the compact
// layout a one-hot feature's cells sit 2 words apart, lanes f and f + 16 of a wave share a bank pair
// and every atomic is replayed 4-8 times; the pad makes the per-feature stride 3 words (odd).
// Cell (feature f, bin b) of tile node nd: plane[nd * ldsW + (foff[f] - c0) + (f - f0) + b]; the
// node's row total sits in its last cell, plane[nd * ldsW + ldsW - 1].
// Bin 0 is never accumulated: each p-phase has one extra "total" lane that adds every row of the
// node, and bin 0 of a feature is written out as total - (its other bins), exact in integers.  For
// the multi-hot draw features (a number is drawn in ~7 of 62 columns) that removes ~90 % of the
// atomics' active lanes.
__global__ void __launch_bounds__(256)
gbdt_hist_q(const uint8_t* __restrict__ bins, const float* __restrict__ g, const float* __restrict__ h,
            const int16_t* __restrict__ node, const int* __restrict__ foff, const int* __restrict__ fmap,
            const int* __restrict__ gfoff, long long* __restrict__ partial, int T, int n, int F, int Fs, int C,
            int level, int chunk, int FT, int NTn, int P, int ldsW, int piece, double qscale) {
  // features: the Fs features of a sub-problem (foff: their compact cells; fmap: sub -> row column,
  // null = identity; gfoff: the full problem's cells, where the output goes); F = bytes per bin row.
  // (4 replicas of the cells for the phases of a wave measured 2.5x slower on the calendar
  // sub-problem: lanes of one atomic on the same word are cheap, and the footprint forced node tiles)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nodesL = 1 << level, first = nodesL - 1;
  const int c = blockIdx.x, t = blockIdx.y;
  const int nft = (Fs + FT - 1) / FT;
  const int ft = blockIdx.z % nft, nt = blockIdx.z / nft;
  const int f0 = ft * FT, f1 = min(Fs, f0 + FT), n0 = nt * NTn;
  const int c0 = foff[f0], c1 = foff[f1], Ct = c1 - c0;
  long long* hist = reinterpret_cast<long long*>(smem);  // [2 planes][NTn][ldsW], shared by all P phases
  const int per = NTn * ldsW;
  for (int i = threadIdx.x; i < 2 * per; i += blockDim.x) hist[i] = 0;
  long long* sq = hist + 2 * per;  // staged rows: (qg, qh) pairs, the tile-relative node ids, the bin rows
  int16_t* sn = reinterpret_cast<int16_t*>(sq + 2 * piece);
  u32x4* sbw = reinterpret_cast<u32x4*>(smem + (((size_t)(2 * per + 2 * piece) * 8 + (size_t)piece * 2 + 15) & ~15));
  const int64_t nbytes = (int64_t)n * F;
  const int64_t base = (int64_t)t * n;
  const int nth = f1 - f0 + 1;  // the tile's features + the total lane
  const int p = threadIdx.x / nth, fl = threadIdx.x - p * nth;
  const bool tot = fl == nth - 1;
  const int f = f0 + ((p < P && !tot) ? fl : 0);
  long long* my = hist + (tot ? ldsW - 2 : (foff[f] - c0) + (f - f0));  // total lane: "bin 1" = the last cell
  const int rb = c * chunk, re = min(n, rb + chunk);
  for (int r0 = rb; r0 < re; r0 += piece) {
    const int r1 = min(re, r0 + piece);
    __syncthreads();  // the previous piece's staging is consumed (first pass: the zeroing is done)
    // the piece's bin rows: 16-B words covering bytes [r0 F, r1 F), all loads in flight at once
    // (range-checked buffer loads: words past the end of the array read as 0)
    const int64_t w0 = ((int64_t)r0 * F) >> 4;
    const int boff = (int)(((int64_t)r0 * F) & 15);
    const int nw = (int)((((int64_t)r1 * F + 15) >> 4) - w0);
    {
      const int64_t left = nbytes - w0 * 16;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(bins + w0 * 16), 0, (int)(left < 0x7FFFFFF0 ? left : 0x7FFFFFF0), 0x00020000);
      // a word running past the array's end would read as 0 in full: that one is assembled bytewise
      const bool tail = (w0 + nw) * 16 > nbytes;
      for (int i = threadIdx.x; i < nw - (tail ? 1 : 0); i += blockDim.x)
        sbw[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, 0));
      if (tail && threadIdx.x == 0) {
        uint8_t* wb = reinterpret_cast<uint8_t*>(sbw + nw - 1);
        for (int k = 0; k < 16; ++k) {
          const int64_t q = (w0 + nw - 1) * 16 + k;
          wb[k] = q < nbytes ? bins[q] : 0;
        }
      }
    }
    for (int r = r0 + (int)threadIdx.x; r < r1; r += blockDim.x) {
      sq[2 * (r - r0)] = quantise(g[base + r], qscale);
      sq[2 * (r - r0) + 1] = quantise_h(h[base + r], qscale);
      sn[r - r0] = (int16_t)(node[base + r] - first - n0);
    }
    __syncthreads();
    if (p < P) {
      const int len = r1 - r0;
      const uint8_t* col = reinterpret_cast<const uint8_t*>(sbw) + boff + (fmap ? fmap[f] : f);  // row r: col[r F]
      int r = p;  // phases interleave rows, so the P waves of a row read neighbouring bin bytes
      for (; r + 7 * P < len; r += 8 * P) {
        int b[8], nd[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          b[u] = tot ? 1 : col[(r + u * P) * F];
          nd[u] = sn[r + u * P];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if ((unsigned)nd[u] >= (unsigned)NTn || b[u] == 0) continue;
          long long* e = my + nd[u] * ldsW + b[u];
          const long long qg = sq[2 * (r + u * P)], qh = sq[2 * (r + u * P) + 1];
          __hip_atomic_fetch_add(e, qg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(e + per, qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      for (; r < len; r += P) {
        const int nd = sn[r];
        const int bb = tot ? 1 : col[r * F];
        if ((unsigned)nd >= (unsigned)NTn || bb == 0) continue;
        long long* e = my + nd * ldsW + bb;
        __hip_atomic_fetch_add(e, sq[2 * r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(e + per, sq[2 * r + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __syncthreads();
  long long* out = partial + ((int64_t)c * T + t) * (int64_t)nodesL * C * 2;
  const int nn = min(NTn, nodesL - n0);
  for (int i = threadIdx.x; i < nn * Ct; i += blockDim.x) {
    const int nd = i / Ct, cc = i - nd * Ct;
    int fi = f0;  // the feature of compact cell c0 + cc (its pad cells precede it)
    while (foff[fi + 1] <= c0 + cc) ++fi;
    auto cell = [&](int k, int plane) { return hist[plane * per + nd * ldsW + k]; };
    const int k0 = cc + (fi - f0);
    long long vg = cell(k0, 0), vh = cell(k0, 1);
    if (c0 + cc == foff[fi]) {  // bin 0: the node's total minus the feature's other bins
      vg = cell(ldsW - 1, 0);
      vh = cell(ldsW - 1, 1);
      for (int k = 1; k < foff[fi + 1] - foff[fi]; ++k) {
        vg -= cell(k0 + k, 0);
        vh -= cell(k0 + k, 1);
      }
    }
    const int fo = fmap ? fmap[fi] : fi;
    long long* o = out + ((int64_t)(n0 + nd) * C + gfoff[fo] + (c0 + cc - foff[fi])) * 2;
    o[0] = vg;
    o[1] = vh;
  }
}

// One-hot (2-bin) features of the fixed-point form, one ROW per lane: a row's set bits (bmask, packed
// once per fit by gbdt_pack_bits) are walked with find-first-set, so every atomic instruction carries
// one live (row, feature) pair per lane instead of the ~7 of 64 of the lane-per-feature form.  LDS per
// tile node: [bin-1 cell of each one-hot feature j | the node total], two planes (g, h).  Bin 0 goes
// out as total - bin 1 (exact in integers).  Same chunks and partial layout as gbdt_hist_q.
__global__ void gbdt_pack_bits(const uint8_t* __restrict__ bins, int n, int F, const int* __restrict__ bfeat, int nb,
                               int WB, uint64_t* __restrict__ bmask) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)n * WB;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / WB;
    const int w = (int)(i - r * WB);
    uint64_t m = 0;
    for (int j = 0; j < 64 && w * 64 + j < nb; ++j) m |= (uint64_t)(bins[r * F + bfeat[w * 64 + j]] != 0) << j;
    bmask[i] = m;
  }
}

constexpr int QB_ROWS = 4;  // rows per thread in flight
constexpr int QB_REP = 4;   // replicas of the one-hot cells and the total (lane & 3)
constexpr int QB_MPRE = 4;  // multi-bin features whose bin bytes are loaded with the row's other inputs
// The other (multi-bin) features ride along: per row one byte load and one atomic pair each, into
// cells of their own (no replicas; consecutive rows mostly share a calendar bin, i.e. a word, and
// lanes of one atomic on the same word are cheap).
// LDS per tile node: [QB_REP x ((nb + 1) | 1) one-hot + total words][Cm multi-bin cells], two planes.
__global__ void __launch_bounds__(256)
gbdt_hist_qb(const uint64_t* __restrict__ bmask, int WB, const int* __restrict__ bcell, int nb,
             const uint8_t* __restrict__ bins, int F, const int* __restrict__ fmap, const int* __restrict__ foffm,
             const int* __restrict__ gfoff, int Fm, const float* __restrict__ g, const float* __restrict__ h,
             const int16_t* __restrict__ node, long long* __restrict__ partial, int T, int n, int C, int level,
             int chunk, int NTn, double qscale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nodesL = 1 << level, first = nodesL - 1;
  const int c = blockIdx.x, t = blockIdx.y, n0 = blockIdx.z * NTn;
  const int W = (nb + 1) | 1;  // one replica: bin-1 cell of each one-hot feature, the total (odd word count)
  const int Cm = Fm ? foffm[Fm] : 0;
  const int NW = QB_REP * W + Cm;  // words per node
  const int per = NTn * NW;
  long long* hist = reinterpret_cast<long long*>(smem);
  for (int i = threadIdx.x; i < 2 * per; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)t * n;
  const int rep = threadIdx.x & (QB_REP - 1);
  // lane-dependent start bit: at the k-th set bit, lanes of one wave sit on different features (the
  // k-th smallest drawn number is otherwise the same few cells for every row of the wave)
  const int rot = (int)((threadIdx.x * 37u) & 63u);
  const int rb = c * chunk, re = min(n, rb + chunk);
  for (int r0 = rb + (int)threadIdx.x; r0 < re; r0 += QB_ROWS * blockDim.x) {
    int nd[QB_ROWS], mb[QB_ROWS][QB_MPRE];
    float gv[QB_ROWS], hv[QB_ROWS];
    uint64_t m0[QB_ROWS];
#pragma unroll
    for (int u = 0; u < QB_ROWS; ++u) {  // every load of the thread's rows in flight
      const int r = r0 + u * blockDim.x;
      const bool ok = r < re;
      nd[u] = ok ? node[base + r] - first - n0 : -1;
      gv[u] = ok ? g[base + r] : 0.f;
      hv[u] = ok ? h[base + r] : 0.f;
      m0[u] = ok ? bmask[(int64_t)r * WB] : 0ull;
#pragma unroll
      for (int k = 0; k < QB_MPRE; ++k) mb[u][k] = (ok && k < Fm) ? bins[(int64_t)r * F + fmap[k]] : 0;
    }
#pragma unroll
    for (int u = 0; u < QB_ROWS; ++u) {
      if ((unsigned)nd[u] >= (unsigned)NTn) continue;
      const long long qg = quantise(gv[u], qscale), qh = quantise_h(hv[u], qscale);
      long long* pn = hist + nd[u] * NW;
      long long* pl = pn + rep * W;
      __hip_atomic_fetch_add(pl + nb, qg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(pl + nb + per, qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const int r = r0 + u * blockDim.x;
      for (int k = 0; k < Fm; ++k) {  // multi-bin features: their own cells, bin 0 derived at the end
        const int b = k < QB_MPRE ? mb[u][k] : bins[(int64_t)r * F + fmap[k]];
        if (b == 0) continue;
        long long* e = pn + QB_REP * W + foffm[k] + b;
        __hip_atomic_fetch_add(e, qg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(e + per, qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      for (int w = 0; w < WB; ++w) {
        const uint64_t mw = w == 0 ? m0[u] : bmask[(int64_t)r * WB + w];
        uint64_t m = rot ? (mw >> rot) | (mw << (64 - rot)) : mw;  // rotate right by rot
        while (m) {
          const int j = w * 64 + ((__builtin_ctzll(m) + rot) & 63);
          m &= m - 1;
          __hip_atomic_fetch_add(pl + j, qg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(pl + j + per, qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  __syncthreads();
  long long* out = partial + ((int64_t)c * T + t) * (int64_t)nodesL * C * 2;
  const int nn = min(NTn, nodesL - n0);
  auto total = [&](int nd, int plane) {
    long long v = 0;
#pragma unroll
    for (int q = 0; q < QB_REP; ++q) v += hist[plane * per + nd * NW + q * W + nb];
    return v;
  };
  for (int i = threadIdx.x; i < nn * nb; i += blockDim.x) {  // one-hot features: bin 0 = total - bin 1
    const int nd = i / nb, j = i - nd * nb;
    long long g1 = 0, h1 = 0;
#pragma unroll
    for (int q = 0; q < QB_REP; ++q) {
      g1 += hist[nd * NW + q * W + j];
      h1 += hist[per + nd * NW + q * W + j];
    }
    long long* o = out + ((int64_t)(n0 + nd) * C + bcell[j]) * 2;  // bcell = the feature's bin-0 cell
    o[0] = total(nd, 0) - g1;
    o[1] = total(nd, 1) - h1;
    o[2] = g1;
    o[3] = h1;
  }
  for (int i = threadIdx.x; i < nn * Cm; i += blockDim.x) {  // multi-bin features
    const int nd = i / Cm, cc = i - nd * Cm;
    int k = 0;
    while (foffm[k + 1] <= cc) ++k;
    const long long* e = hist + nd * NW + QB_REP * W;
    long long vg = e[cc], vh = e[per + cc];
    if (cc == foffm[k]) {  // bin 0: the node's total minus the feature's other bins
      vg = total(nd, 0);
      vh = total(nd, 1);
      for (int q = foffm[k] + 1; q < foffm[k + 1]; ++q) {
        vg -= e[q];
        vh -= e[per + q];
      }
    }
    long long* o = out + ((int64_t)(n0 + nd) * C + gfoff[fmap[k]] + (cc - foffm[k])) * 2;
    o[0] = vg;
    o[1] = vh;
  }
}

// fold the per-chunk histograms into chunk 0 in chunk order (single-GPU and DP paths alike)
template <typename A>
__global__ void gbdt_chunk_reduce(A* __restrict__ partial, int nchunks, int64_t S) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < S; e += (int64_t)gridDim.x * blockDim.x) {
    A acc = partial[e];
    for (int c = 1; c < nchunks; ++c) acc += partial[(int64_t)c * S + e];
    partial[e] = acc;
  }
}

// ---------------------------------------------------------------- K9 split scan
// one block (64..256 threads) per (task, node of this level).  hist: [T][nodesL][C][2] (folded).
// Thread <-> feature: a sequential left-sum over the feature's bins (bin order), XGBoost loss_chg
// at every candidate "bin <= b", first maximum kept; then a block arg-max where the larger gain
// wins and equal gains go to the lower feature == numpy's first argmax in (feature, bin) order.
// A = double (exact form) or long long (fixed point, value = q * qinv): the fixed-point form keeps
// the left sums and the node totals (feature 0's cells, every level) in integers and converts each
// to double once, so GR = (Gn - GL) is exact as well.
// Finalize (tf != nullptr, the last level): each (task, node) block arrives on the task's counter after
// its decision (release); the task's last block (acquire) runs gbdt_finalize's prune and leaves for the
// task and re-arms the counter -- one launch less per round.
constexpr int SPLIT_FINAL_MAX_DEPTH = 8;
constexpr int SPLIT_DIRECT_MAX_BINS = 32;  // direct candidate form up to this many bins per feature
constexpr int EM_GBDT_SEPARATE = 1;  // em_gbdt_fit launch_flags: the separate launches instead of the fused round
constexpr int EM_GBDT_PRESPLIT = 2;  // em_gbdt_fit launch_flags: splits inside the next level's histogram pass
constexpr int SPLIT_ONESHOT_LDS = 48 * 1024;  // chunk partials staged at once up to this many bytes (+ the
                                              // finalize's <= 12 KB: within the default 64 KB)  // the fused finalize stages NN <= 511 nodes (23 B each) in LDS

// One node's split (block vb = task * nodesL + node of the level), shared by the split launch and the
// level-0 histogram pass that splits its task's root itself (COH: the chunk partials and the node's
// status come from other workgroups of the same launch -- agent-scope loads, see HistSplit).
template <typename A, bool COH, int NPRE>
EM_DEVICE void split_body(int vb, char* smem, const A* __restrict__ hist, int nchunks, int64_t cstride,
                          const int* __restrict__ foff, int T, int F, int C, int level, int NN, double* __restrict__ G,
                          double* __restrict__ H, int8_t* __restrict__ status, int16_t* __restrict__ feat,
                          uint8_t* __restrict__ sbin, float* __restrict__ gain, double lam, double mcw, double qinv,
                          SplitFinal fin, int oneshot, int pscan, const int4* __restrict__ cellinfo) {
  constexpr bool Q = std::is_same<A, long long>::value;
  auto ldp = [](const A* p) -> A {
    if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
  };
  const int nodesL = 1 << level, first = nodesL - 1;
  const int t = vb / nodesL, nd = vb % nodesL, i = first + nd;
  GSTAMP(16 * level);
  int8_t* st = status + (int64_t)t * NN;
  // the thread's feature cells and feature 0's, loaded before the partials (one round trip for all)
  const int fa0 = foff[0], fb0 = foff[1];
  const int myca = (int)threadIdx.x < F ? foff[threadIdx.x] : 0, mycb = (int)threadIdx.x < F ? foff[threadIdx.x + 1] : 0;
  // direct candidate form (cellinfo != null, every feature <= SPLIT_DIRECT_MAX_BINS bins): this thread's
  // cell's {feature, first cell, end cell}, loaded with the rest
  const int4 myci = cellinfo && (int)threadIdx.x < C ? cellinfo[threadIdx.x] : int4{0, 0, 0, 0};
  // the first batch of the one-shot partial loads goes out with the node's status load (one round trip
  // instead of status first, then partials; a closed node's partials are read and dropped)
  const A* hs0 = hist + ((int64_t)t * nodesL + nd) * C * 2;
  const bool one = nchunks > 1 && oneshot;
  const int tot = nchunks * 2 * C;
  // below the root (exact form) the node's totals come from the parent's split: loaded with the rest
  double pGn = 0.0, pHn = 0.0;
  if (!Q && level > 0 && threadIdx.x == 0) {
    pGn = G[(int64_t)t * NN + i];
    pHn = H[(int64_t)t * NN + i];
  }
  A pre[NPRE];
  if (one) {
#pragma unroll
    for (int u = 0; u < NPRE; ++u) {
      const int idx = (int)threadIdx.x + u * (int)blockDim.x, c = idx / (2 * C), e = idx - c * 2 * C;
      pre[u] = idx < tot ? ldp(hs0 + (int64_t)c * cstride + e) : A(0);
    }
  }
  int8_t sti;
  if constexpr (COH)
    sti = __hip_atomic_load(st + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    sti = st[i];
  if (sti == 2) {  // block-uniform: an open node
    const A* hs = hs0;
    if (one) {
      // every chunk's cells staged at once (32 loads per thread in flight: one round trip, where the
      // per-element chunk loop took 2-3), then folded in chunk order (== gbdt_chunk_reduce)
      A* stg = reinterpret_cast<A*>(smem);
      for (int b0 = threadIdx.x; b0 < tot; b0 += NPRE * blockDim.x) {
        A v[NPRE];
#pragma unroll
        for (int u = 0; u < NPRE; ++u) {
          const int idx = b0 + u * blockDim.x, c = idx / (2 * C), e = idx - c * 2 * C;
          v[u] = b0 == (int)threadIdx.x ? pre[u] : (idx < tot ? ldp(hs + (int64_t)c * cstride + e) : A(0));
        }
#pragma unroll
        for (int u = 0; u < NPRE; ++u) {
          const int idx = b0 + u * blockDim.x;
          if (idx < tot) stg[idx] = v[u];
        }
      }
      __syncthreads();
      for (int e = threadIdx.x; e < 2 * C; e += blockDim.x) {
        A acc = stg[e];
        for (int c = 1; c < nchunks; ++c) acc += stg[c * 2 * C + e];
        stg[e] = acc;
      }
      __syncthreads();
      GSTAMP(16 * level + 1);
      hs = stg;
    } else if (nchunks > 1) {  // per-chunk partials: fold this node's cells into LDS in chunk order (== gbdt_chunk_reduce)
      A* fold = reinterpret_cast<A*>(smem);
      for (int e = threadIdx.x; e < 2 * C; e += blockDim.x) {
        A acc = hs[e];
        int c = 1;
        for (; c + 8 <= nchunks; c += 8) {  // 8 independent loads in flight, added in chunk order
          A v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = hs[(int64_t)(c + u) * cstride + e];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; c < nchunks; ++c) acc += hs[(int64_t)c * cstride + e];
        fold[e] = acc;
      }
      __syncthreads();
      hs = fold;
    }
    auto val = [=](A x) -> double {
      if constexpr (Q)
        return (double)x * qinv;
      else
        return x;
    };
    __shared__ A sGn[2];
    __shared__ double rv[16];  // (per wave: <= 1024 threads)
    __shared__ int rf[16], rb[16];
    __shared__ A rgl[16], rhl[16];
    if (threadIdx.x == 0) {
      A Gn, Hn;
      if (Q || level == 0) {  // node totals: feature 0's cells in bin order
        Gn = 0;
        Hn = 0;
        for (int c = fa0; c < fb0; ++c) {
          Gn += hs[2 * c];
          Hn += hs[2 * c + 1];
        }
        if (level == 0) {
          __hip_atomic_store(G + (int64_t)t * NN, val(Gn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(H + (int64_t)t * NN, val(Hn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        Gn = pGn;
        Hn = pHn;
      }
      sGn[0] = Gn;
      sGn[1] = Hn;
    }
    __syncthreads();
    GSTAMP(16 * level + 2);
    const A Gna = sGn[0], Hna = sGn[1];
    const double Gn = val(Gna), Hn = val(Hna);
    const double root = Gn * Gn / (Hn + lam);
    double best = -INFINITY;
    A bGL = 0, bHL = 0;
    int bf = 0x7fffffff, bb = 0;
    auto cand = [&](int f, int b, A GLa, A HLa) {  // candidate "bin <= b" of feature f
      const double GL = val(GLa), HL = val(HLa);
      const double GR = val(Gna - GLa), HR = val(Hna - HLa);
      if (HL >= mcw && HR >= mcw) {
        const double gn = GL * GL / (HL + lam) + GR * GR / (HR + lam) - root;
        if (gn > best) {  // strict: candidates come in ascending (feature, bin) order per thread
          best = gn;
          bf = f;
          bb = b;
          bGL = GLa;
          bHL = HLa;
        }
      }
    };
    if (cellinfo && nchunks > 1) {  // (the folded cells are in LDS)
      // direct form: thread c sums its feature's cells up to c in bin order -- the very sums of the
      // sequential scan below, so bitwise the same candidates -- and evaluates candidate c at once: no
      // per-feature chain over a many-bin feature, no LDS pass, no barrier (round 5: the two-pass scan
      // took ~2 us of the split's ~8.5, profiles/r5/gbdt_split_stamps.jsonl)
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const int4 ci = c == (int)threadIdx.x ? myci : cellinfo[c];
        if (c >= ci.z - 1) continue;  // the last bin is never a candidate (nothing to its right)
        A GLa = 0, HLa = 0;
#pragma unroll 8
        for (int k = ci.y; k <= c; ++k) {
          GLa += hs[2 * k];
          HLa += hs[2 * k + 1];
        }
        cand(ci.x, c - ci.y, GLa, HLa);
      }
    } else if (pscan) {
      // two passes: thread f writes its feature's left sums in bin order (the same sequential sums),
      // then thread c evaluates candidate cell c -- the divisions of a 31-bin feature no longer
      // run one after another on one lane
      char* sa = smem + (nchunks > 1 ? (((oneshot ? nchunks : 1) * 2 * C * (int)sizeof(A) + 15) & ~15) : 0);
      A* cGL = reinterpret_cast<A*>(sa);
      A* cHL = cGL + C;
      int16_t* cfe = reinterpret_cast<int16_t*>(cHL + C);  // feature of a candidate cell, -1: a last bin
      int16_t* cbn = cfe + C;                              // its bin
      for (int f = threadIdx.x; f < F; f += blockDim.x) {
        const int ca = f == (int)threadIdx.x ? myca : foff[f], cb = f == (int)threadIdx.x ? mycb : foff[f + 1];
        A GLa = 0, HLa = 0;
        int c = ca;
        for (; c + 8 <= cb - 1; c += 8) {  // 8 cells' loads in flight, then their left sums in bin order
          A vg[8], vh[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            vg[u] = hs[2 * (c + u)];
            vh[u] = hs[2 * (c + u) + 1];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            GLa += vg[u];
            HLa += vh[u];
            cGL[c + u] = GLa;
            cHL[c + u] = HLa;
            cfe[c + u] = (int16_t)f;
            cbn[c + u] = (int16_t)(c + u - ca);
          }
        }
        for (; c < cb - 1; ++c) {
          GLa += hs[2 * c];
          HLa += hs[2 * c + 1];
          cGL[c] = GLa;
          cHL[c] = HLa;
          cfe[c] = (int16_t)f;
          cbn[c] = (int16_t)(c - ca);
        }
        cfe[cb - 1] = -1;
      }
      __syncthreads();
      GSTAMP(16 * level + 6);
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const int f = cfe[c];
        if (f >= 0) cand(f, cbn[c], cGL[c], cHL[c]);
      }
      GSTAMP(16 * level + 7);
    } else {
      for (int f = threadIdx.x; f < F; f += blockDim.x) {
        const int ca = f == (int)threadIdx.x ? myca : foff[f], cb = f == (int)threadIdx.x ? mycb : foff[f + 1];
        A GLa = 0, HLa = 0;
        for (int c = ca; c < cb - 1; ++c) {  // the last bin is never a candidate (nothing to its right)
          GLa += hs[2 * c];
          HLa += hs[2 * c + 1];
          cand(f, c - ca, GLa, HLa);
        }
      }
    }
    // block arg-max: larger gain, then lower feature (a thread's features ascend with its loop)
    // (the butterfly carries the owner lane of the best candidate, not its two sums: (gain, feature,
    // bin) order every candidate uniquely, so the winner's sums are fetched once afterwards)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int bl = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(best, o);
      const int of = __shfl_xor(bf, o), ob = __shfl_xor(bb, o), ol = __shfl_xor(bl, o);
      if (ov > best || (ov == best && (of < bf || (of == bf && ob < bb)))) {
        best = ov;
        bf = of;
        bb = ob;
        bl = ol;
      }
    }
    bGL = __shfl(bGL, bl);
    bHL = __shfl(bHL, bl);
    if (lane == 0) {
      rv[w] = best;
      rf[w] = bf;
      rb[w] = bb;
      rgl[w] = bGL;
      rhl[w] = bHL;
    }
    __syncthreads();
    GSTAMP(16 * level + 3);
    if (threadIdx.x == 0) {
      const int nw = (blockDim.x + 63) >> 6;
      for (int k = 1; k < nw; ++k)
        if (rv[k] > best || (rv[k] == best && (rf[k] < bf || (rf[k] == bf && rb[k] < bb)))) {
          best = rv[k];
          bf = rf[k];
          bb = rb[k];
          bGL = rgl[k];
          bHL = rhl[k];
        }
      if (bf < F && best > KRT_EPS) {
        // write-through (agent-scope) stores: the fused finalize's last block reads them back without
        // an acq_rel arrival, which would write back every arriving block's L2
        auto wt = [](auto* ptr, auto v) { __hip_atomic_store(ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        wt(st + i, (int8_t)1);
        wt(feat + (int64_t)t * NN + i, (int16_t)bf);
        wt(sbin + (int64_t)t * NN + i, (uint8_t)bb);
        wt(gain + (int64_t)t * NN + i, (float)best);
        const int l = 2 * i + 1, r = 2 * i + 2;
        wt(st + l, (int8_t)2);
        wt(st + r, (int8_t)2);
        wt(G + (int64_t)t * NN + l, val(bGL));
        wt(H + (int64_t)t * NN + l, val(bHL));
        wt(G + (int64_t)t * NN + r, val(Gna - bGL));
        wt(H + (int64_t)t * NN + r, val(Hna - bHL));
      }
    }
  }
  GSTAMP(16 * level + 4);
  if (!fin.tctr) return;
  __shared__ int last;
  // Memory-model note: there is no release/acquire pair here.  The hand-off is the gfx950
  // "write-through stores + drained vmcnt + relaxed arrival" form (MI355X_MICROARCH.md, Workgroup
  // dispatch / inter-workgroup visibility, "Valid forms" table row 1): ONE lane made every store of the
  // handed-off bytes as an agent-scope (sc1, write-through) store, waited vmcnt(0) (inline asm, so the
  // compiler cannot drop or move it), then added to the per-task counter; the last adder's block reads
  // them back with agent-scope (sc1, L1-bypassing) loads after a workgroup barrier.  That ordering is a
  // property of gfx9 cache hardware measured on MI355X, not of the HIP memory model: on any other
  // target this must become an agent-scope release add / acquire fence.  The guards are
  // tests/test_gbdt.py (fused vs separate launches, bit-identical) and the separate-launch path.
  if (threadIdx.x == 0) {  // (this block's write-through stores have completed before its arrival)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(fin.tctr + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nodesL - 1;
  }
  __syncthreads();
  if (!last) return;  // block-uniform
  // the task's tree staged in LDS (after the fold area), pruned by one thread, leaves by all
  char* fa = smem + (nchunks > 1 ? (((oneshot ? nchunks : 1) * 2 * C * (int)sizeof(A) + 15) & ~15) : 0) +
             (pscan ? ((C * (2 * (int)sizeof(A) + 4) + 15) & ~15) : 0);
  double* sG = reinterpret_cast<double*>(fa);
  double* sH = sG + NN;
  float* sgn = reinterpret_cast<float*>(sH + NN);
  int16_t* sfe = reinterpret_cast<int16_t*>(sgn + NN);
  int8_t* sst = reinterpret_cast<int8_t*>(sfe + NN);
  const int64_t o = (int64_t)t * NN;
  for (int k = threadIdx.x; k < NN; k += blockDim.x) {  // (agent-scope loads: the siblings' stores)
    sst[k] = __hip_atomic_load(st + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sfe[k] = __hip_atomic_load(feat + o + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sgn[k] = __hip_atomic_load(gain + o + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sG[k] = __hip_atomic_load(G + o + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sH[k] = __hip_atomic_load(H + o + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    fin.tctr[t] = 0;  // re-armed for the next round (the kernel boundary orders it)
    prune_task(sst, sfe, sgn, fin.max_depth, fin.gamma);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NN; k += blockDim.x) {
    st[k] = sst[k];
    feat[o + k] = sfe[k];
    fin.leaf[o + k] = sst[k] == 2 ? (float)(-sG[k] / (sH[k] + lam) * fin.eta) : 0.f;
    fin.cover[o + k] = sst[k] ? (float)sH[k] : 0.f;
  }
  GSTAMP(16 * level + 5);
}

// Partial loads kept in flight per thread by the split launch's one-shot prefetch: 1488 doubles per node at
// the reference depth-2 level; 8 x 256 threads cover them in one round trip, 4 in two (larger nodes loop).
// 8 instead of 32 takes the kernel from 256 VGPRs (+ AGPRs) to 66: reference fit +4.7 % trees/s, same box
// (16: +2.4 %); 4 another +1.2 % (profiles/r5/gbdt_hist_regs_ab.txt).  (side-build knob)
#ifndef GBDT_SPLIT_NPRE
#define GBDT_SPLIT_NPRE 4
#endif
template <typename A>
__global__ void __launch_bounds__(256)
gbdt_split(const A* __restrict__ hist, int nchunks, int64_t cstride, const int* __restrict__ foff, int T, int F,
           int C, int level, int NN, double* __restrict__ G, double* __restrict__ H, int8_t* __restrict__ status,
           int16_t* __restrict__ feat, uint8_t* __restrict__ sbin, float* __restrict__ gain, double lam, double mcw,
           double qinv, SplitFinal fin, int oneshot, int pscan, const int4* __restrict__ cellinfo) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  split_body<A, false, GBDT_SPLIT_NPRE>(blockIdx.x, smem, hist, nchunks, cstride, foff, T, F, C, level, NN, G, H, status, feat, sbin,
                       gain, lam, mcw, qinv, fin, oneshot, pscan, cellinfo);
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
  const int64_t o = (int64_t)t * NN;
  int8_t* st = status + o;
  prune_task(st, feat + o, gain + o, max_depth, gamma);
  for (int i = 0; i < NN; ++i) {
    leaf[o + i] = st[i] == 2 ? (float)(-G[o + i] / (H[o + i] + lam) * eta) : 0.f;
    cover[o + i] = st[i] ? (float)H[o + i] : 0.f;
  }
}

// TreePruner: a split whose children are both leaves and whose gain is below gamma becomes a leaf
// (bottom-up over the internal slots; arrays at the task's base)
EM_DEVICE void prune_task(int8_t* st, int16_t* fe, const float* gn, int max_depth, float gamma) {
  for (int i = (1 << max_depth) - 2; i >= 0; --i) {
    if (st[i] == 1 && st[2 * i + 1] == 2 && st[2 * i + 2] == 2 && gn[i] < gamma) {
      st[i] = 2;
      st[2 * i + 1] = 0;
      st[2 * i + 2] = 0;
      fe[i] = -1;
    }
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

// per-element term of the elementwise metrics (logloss / rmse / error) of one (task, row) margin
EM_DEVICE double metric_term(float m, float y, int obj, int metric) {
  const float p = obj == OBJ_LOGISTIC ? 1.f / (1.f + expf(-m)) : m;
  if (metric == MET_LOGLOSS) {
    const double pc = fmin(fmax((double)p, 1e-16), 1.0 - 1e-16);
    return -(y * log(pc) + (1.0 - y) * log(1.0 - pc));
  }
  if (metric == MET_RMSE) return (double)(p - y) * (double)(p - y);
  return ((p > 0.5f ? 1.f : 0.f) != y) ? 1.0 : 0.0;
}

// fixed-order tree sum over the 256 threads of a block (thread 0 gets the result)
EM_DEVICE double block_tree_sum(double acc) {
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  return red[0];
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
    acc += metric_term(margin[i], Y[(int64_t)r * T + t], obj, metric);
  }
  const double bs = block_tree_sum(acc);
  if (threadIdx.x == 0) partial[blockIdx.x] = bs;
}

// fixed-order block reduction of the per-block metric partials (256 threads: strided sequential
// sums, then a tree) -- deterministic, and ~50x faster than one thread walking 4096 doubles
EM_DEVICE double block_sum_partials(const double* __restrict__ partial, int nb) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  return red[0];
}

__global__ void __launch_bounds__(256)
gbdt_metric_final(const double* __restrict__ partial, int nb, int64_t count, int metric, float* __restrict__ out) {
  const double s = block_sum_partials(partial, nb);
  if (threadIdx.x == 0) {
    double v = s / (double)(count > 0 ? count : 1);
    if (metric == MET_RMSE) v = sqrt(v);
    out[0] = (float)v;
  }
}

// The last-arriving block of a fused metric launch: every block stores its partial write-through (sc1)
// and drains it before its single arrival add; the block whose add completes the count sums the
// partials (sc1 loads) exactly as gbdt_metric_final does, writes the mean and re-arms the counter.
// (b, nb: this block's index among the nb blocks of its metric set; a fused launch runs several sets)
// ctr == nullptr: deferred form -- the block only stores its partial (the kernel boundary publishes it)
// and gbdt_metric_rounds reduces every round's partials after the last round, in the same order: the
// metric is history, not an input of the next round, so its reduction leaves each round's critical path.
EM_DEVICE void metric_arrive_final(double bs, double* __restrict__ partial, int* __restrict__ ctr, int64_t count,
                                   int metric, float* __restrict__ out, int b, int nb) {
  __shared__ int last;
  if (!ctr) {
    if (threadIdx.x == 0) partial[b] = bs;
    return;
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + b, bs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
  }
  __syncthreads();
  if (!last) return;
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256)
    s += __hip_atomic_load(partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double v = red[0] / (double)(count > 0 ? count : 1);
    if (metric == MET_RMSE) v = sqrt(v);
    out[0] = (float)v;
    __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The next round's start inside the current round's update (eager driver): its tree arrays reset and,
// from each element's freshly updated margin, its g / h with every row back at the root
// (gbdt_round_start's work for per-task objectives) -- one launch less per round.
EM_DEVICE void predict_metric_body(const uint8_t* __restrict__ bins, float* __restrict__ margin, int T, int n, int F,
                                   int NN, int k0, int k1, const int8_t* __restrict__ status,
                                   const int16_t* __restrict__ feat, const uint8_t* __restrict__ sbin,
                                   const float* __restrict__ leaf, const float* __restrict__ Y, int obj, int metric,
                                   double* __restrict__ partial, int* __restrict__ ctr, float* __restrict__ out,
                                   int b, int nb);
// eval sets handled by the update launch's trailing blocks (eager rounds): set s gets mb blocks, its own
// partial region (partial + (1 + s) * 4096) and arrival counter (ctr + 1 + s)
struct NextRound {
  int round = -1;  // < 0: none
  float* g = nullptr;
  float* h = nullptr;
  int16_t* node = nullptr;  // the next round's level-0 node buffer
  int8_t* st = nullptr;     // the next round's tree arrays (host-offset)
  int16_t* fe = nullptr;
  uint8_t* sb = nullptr;
  float* gn = nullptr;
  float subsample = 1.f;
  uint32_t seed = 0;
};

// gbdt_update + gbdt_metric + gbdt_metric_final (elementwise metrics) in one launch: same grid, same
// elements per thread, same partial and final sums -> bit-identical to the three launches.
// plevel >= 0: the rows' nodes are before the last level's partition, applied here (gbdt_partition's
// rule: a node of level plevel that still splits after pruning sends the row to a child; a pruned one
// is a leaf, where the partition-then-ancestor walk of the separate launches ends as well).
__global__ void __launch_bounds__(256)
gbdt_update_metric(float* __restrict__ margin, const int16_t* __restrict__ node, int T, int n, int NN,
                   const int8_t* __restrict__ status, const float* __restrict__ leaf,
                   const float* __restrict__ Y, int obj, int metric, double* __restrict__ partial, int* __restrict__ ctr,
                   float* __restrict__ out, const uint8_t* __restrict__ bins,
                   int F, int plevel, const int16_t* __restrict__ feat, const uint8_t* __restrict__ sbin,
                   NextRound nx, int nbu, EvalSets evs) {
  if ((int)blockIdx.x >= nbu) {  // an eval set's prediction + metric
    int b = (int)blockIdx.x - nbu, s = 0;
    while (s < evs.count - 1 && b >= evs.mb[s]) b -= evs.mb[s++];
    // (status / feat / sbin / leaf are this round's arrays: its trees are 0 .. T - 1 of them)
    predict_metric_body(evs.bins[s], evs.margin[s], T, evs.n[s], F, NN, 0, T, status, feat, sbin, leaf, evs.Y[s], obj,
                        metric, partial + (int64_t)(1 + s) * evs.pstride, ctr ? ctr + 1 + s : nullptr, out + 1 + s, b,
                        evs.mb[s]);
    return;
  }
  const int64_t total = (int64_t)T * n;
  const int pf = plevel >= 0 ? (1 << plevel) - 1 : 0, pl = plevel >= 0 ? 2 * pf + 1 : 0;
  GSTAMP(128);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)nbu * blockDim.x) {
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const int8_t* st = status + (int64_t)t * NN;
    int nd = node[i];
    if (nd >= pf && nd < pl && st[nd] == 1) {
      const int64_t k = (int64_t)t * NN + nd;
      nd = 2 * nd + 1 + (bins[(int64_t)r * F + feat[k]] > sbin[k] ? 1 : 0);
    }
    const float m = margin[i] + leaf[(int64_t)t * NN + leaf_ancestor(st, nd)];
    margin[i] = m;
    acc += metric_term(m, Y[(int64_t)r * T + t], obj, metric);
    if (nx.round >= 0) grad_elem(i, margin, Y, nx.g, nx.h, nx.node, T, n, obj, nx.subsample, nx.seed, nx.round);
  }
  if (nx.round >= 0)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)T * NN;
         i += (int64_t)nbu * blockDim.x)
      round_init_elem((int)i, nx.st, nx.fe, nx.sb, nx.gn, NN);
  GSTAMP(129);
  metric_arrive_final(block_tree_sum(acc), partial, ctr, total, metric, out, blockIdx.x, nbu);
  GSTAMP(130);
}

// gbdt_predict (one round's trees) + gbdt_metric + gbdt_metric_final of an eval set in one launch
EM_DEVICE void predict_metric_body(const uint8_t* __restrict__ bins, float* __restrict__ margin, int T, int n, int F,
                                   int NN, int k0, int k1, const int8_t* __restrict__ status,
                                   const int16_t* __restrict__ feat, const uint8_t* __restrict__ sbin,
                                   const float* __restrict__ leaf, const float* __restrict__ Y, int obj, int metric,
                                   double* __restrict__ partial, int* __restrict__ ctr, float* __restrict__ out,
                                   int b, int nb) {
  const int64_t total = (int64_t)T * n;
  double acc = 0.0;
  for (int64_t i = (int64_t)b * blockDim.x + threadIdx.x; i < total; i += (int64_t)nb * blockDim.x) {
    const int t = (int)(i / n), r = (int)(i - (int64_t)t * n);
    const uint8_t* row = bins + (int64_t)r * F;
    float tacc = 0.f;
    for (int k = k0 + ((t - k0 % T) % T + T) % T; k < k1; k += T) {
      const int64_t o = (int64_t)k * NN;
      int nd = 0;
      while (status[o + nd] == 1) nd = 2 * nd + 1 + (row[feat[o + nd]] > sbin[o + nd] ? 1 : 0);
      tacc += leaf[o + nd];
    }
    const float m = margin[i] + tacc;
    margin[i] = m;
    acc += metric_term(m, Y[(int64_t)r * T + t], obj, metric);
  }
  metric_arrive_final(block_tree_sum(acc), partial, ctr, total, metric, out, b, nb);
}
__global__ void __launch_bounds__(256)
gbdt_predict_metric(const uint8_t* __restrict__ bins, float* __restrict__ margin, int T, int n, int F, int NN, int k0,
                    int k1, const int8_t* __restrict__ status, const int16_t* __restrict__ feat,
                    const uint8_t* __restrict__ sbin, const float* __restrict__ leaf,
                    const float* __restrict__ Y, int obj, int metric, double* __restrict__ partial,
                    int* __restrict__ ctr, float* __restrict__ out) {
  predict_metric_body(bins, margin, T, n, F, NN, k0, k1, status, feat, sbin, leaf, Y, obj, metric, partial, ctr,
                      out, blockIdx.x, gridDim.x);
}

// the deferred metrics of `rounds` rounds x `sets` sets: block (r, s) reduces partials
// [(r * sets + s) * stride, + nb[s]) as metric_arrive_final's last block would, into out[r * sets + s]
struct MetricRounds {
  int nb[5];
  int64_t count[5];
};
__global__ void __launch_bounds__(256)
gbdt_metric_rounds(const double* __restrict__ partial, int64_t stride, int sets, MetricRounds mr, int metric,
                   float* __restrict__ out) {
  const int r = blockIdx.x / sets, s = blockIdx.x % sets;
  const double sum = block_sum_partials(partial + ((int64_t)r * sets + s) * stride, mr.nb[s]);
  if (threadIdx.x == 0) {
    double v = sum / (double)(mr.count[s] > 0 ? mr.count[s] : 1);
    if (metric == MET_RMSE) v = sqrt(v);
    out[(int64_t)r * sets + s] = (float)v;
  }
}

__global__ void __launch_bounds__(256)
gbdt_metric_sum(const double* __restrict__ partial, int nb, double* __restrict__ out) {
  const double s = block_sum_partials(partial, nb);
  if (threadIdx.x == 0) out[0] = s;
}

inline int grid_for(int64_t total, int bs = 256) {
  int64_t g = (total + bs - 1) / bs;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

// ------------------------------------------------------------------ host-side histogram plan
namespace {
struct HistPlan {
  int chunk, nchunks, FT, NTn, P, ldsC, nft, ntn, threads, piece;
  size_t lds;
};

// Tile plan of one level: widest feature tile (then fewest node tiles) whose histogram copies fit
// the LDS budget (P private copies in the exact form, one shared copy in the fixed-point form); P
// (row phases, 1..4) fills a 256-thread block when F is small.  Chunks are sized so a level launches
// ~4096 blocks (all 256 CUs busy even for the reference's ~930 rows).
bool plan_hist(int level, int n, int T, int F, const int* foff, bool quant, HistPlan& pl, int row_bytes = 0) {
  // F features with cells foff[0..F]; row_bytes = bytes per bin row (0: F; a feature sub-problem's rows
  // are the full rows)
  const int nodesL = 1 << level;
  const int RB = row_bytes > 0 ? row_bytes : F;
  for (int NTn = nodesL; NTn >= 1; NTn >>= 1) {
    for (int FT = F < (quant ? 255 : 256) ? F : (quant ? 255 : 256);; FT = (FT + 1) / 2) {
      int maxC = 0;
      for (int f0 = 0; f0 < F; f0 += FT) {
        const int f1 = f0 + FT < F ? f0 + FT : F;
        maxC = foff[f1] - foff[f0] > maxC ? foff[f1] - foff[f0] : maxC;
      }
      const int lanes = FT + (quant ? 1 : 0);  // fixed point: + the total lane per phase
      const int W = maxC + (quant ? FT + 1 : 0);  // fixed point: + a pad cell per feature + the total cell
      // row phases: the exact form keeps P private copies (<= 8 in a 512-thread block: each copy's serial
      // read-modify-write chain is a P-th of the chunk), the fixed-point form one shared copy, so a
      // few-feature tile fills its 256-thread block with phases
      int P = (quant ? 256 : HIST_EXACT_THREADS) / lanes;
      const int Pmax = quant ? 64 : GBDT_HIST_PMAX;
      P = P > Pmax ? Pmax : (P < 1 ? 1 : P);
      for (; P >= 1; --P)
        if ((int64_t)(quant ? 1 : P) * NTn * W * 16 <= (quant ? HIST_LDS_BUDGET : HIST_EXACT_LDS_BUDGET)) break;
      if (P >= 1) {
        pl.FT = FT;
        pl.NTn = NTn;
        pl.P = P;
        pl.ldsC = W;
        pl.nft = (F + FT - 1) / FT;
        pl.ntn = nodesL / NTn;
        pl.threads = ((lanes * P + 63) / 64) * 64;
        // chunks: ~4096 blocks per level, >= 64 rows each, and the per-chunk partials within the cap
        const int64_t per_chunk = (int64_t)T * pl.nft * pl.ntn;
        const int64_t S = (int64_t)T * nodesL * foff[F] * 2;
        if (S > HIST_PARTIAL_CAP) return false;
        int64_t want = (4096 + per_chunk - 1) / per_chunk;
        const int64_t cap = HIST_PARTIAL_CAP / S;
        want = want > cap ? cap : want;
        int64_t chunk = (n + want - 1) / want;
        chunk = chunk < HIST_MIN_CHUNK ? HIST_MIN_CHUNK : chunk;
        pl.chunk = (int)chunk;
        pl.nchunks = (int)((n + chunk - 1) / chunk);
        // staged rows: (g, h) floats + node id (exact); (qg, qh) int64 + node id + the piece's bin
        // rows (fixed point: ~16 KB of bins per piece, fetched with 16-B loads)
        pl.piece = quant ? ((HIST_QBIN_LDS / RB) & ~15) : HIST_MAX_CHUNK;
        if (pl.piece > HIST_MAX_CHUNK) pl.piece = HIST_MAX_CHUNK;
        if (pl.piece < 16) pl.piece = 16;
        // exact form: no staging beyond the chunk (a 64-row chunk staged 1024 rows' worth of LDS, which
        // cut the blocks per CU from 4 to 3 at depth 2 of the reference fit: two rounds of blocks)
        if (!quant && pl.piece > pl.chunk) pl.piece = (pl.chunk + 15) & ~15;
        pl.lds = (size_t)(quant ? 1 : P) * NTn * pl.ldsC * 16 + (size_t)pl.piece * (quant ? 18 : 10) + 4 +
                 (quant ? ((size_t)pl.piece * RB + 32 + 15) / 16 * 16 : 0);
        return true;
      }
      if (FT == 1) break;
    }
  }
  return false;
}

int64_t partial_need(int level, int n, int T, int F, const int* foff) {
  HistPlan pl;  // the fixed-point plan never has more chunks (same tiles or wider)
  if (!plan_hist(level, n, T, F, foff, false, pl)) return -1;
  HistPlan pq;
  if (!plan_hist(level, n, T, F, foff, true, pq)) return -1;
  const int64_t nch = pl.nchunks > pq.nchunks ? pl.nchunks : pq.nchunks;
  return nch * T * (1 << level) * foff[F] * 2;
}

// K8 for one level: per-chunk histograms, then folded into partial[0 : T*nodesL*C*2] (8-byte words:
// doubles, or int64 when qscale != 0)
// fold = false leaves the per-chunk partials for gbdt_split to fold (small chunk counts); *nchunks_out
// = the number of partial copies left in `partial` (1 after a fold)
constexpr int SPLIT_FOLD_MAX_CHUNKS = 32, SPLIT_FOLD_MAX_LDS = 32 * 1024;
// Fixed-point sparse form (em_gbdt_fit, quant_bits > 0, >= 8 one-hot features): one-hot features on
// gbdt_hist_qb (row per lane over the packed bit masks), the others on gbdt_hist_q over their feature
// sub-problem; both write their own cells of the same per-chunk partials.
struct QuantAux {
  int nb = 0, WB = 0;                 // one-hot features, 64-bit words per row mask
  const int* bcell_d = nullptr;       // [nb] bin-0 cell of each one-hot feature (bin 1 follows)
  const uint64_t* bmask_d = nullptr;  // [n][WB]
  int Fm = 0;                         // the other features
  std::vector<int> foffm_h;           // [Fm + 1] their compact cells
  const int* foffm_d = nullptr;
  const int* fmap_d = nullptr;        // [Fm] sub-feature -> bin-row column
};

struct HistPartition {  // the previous level's partition fused into the exact-form histogram (gbdt_hist)
  int16_t* node_out = nullptr;
  const int8_t* st = nullptr;
  const int16_t* fe = nullptr;
  const uint8_t* sb = nullptr;
  int NN = 0;
};
int launch_level_hist(int level, const uint8_t* bins, const float* g, const float* h, const int16_t* node, int T,
                      int n, int F, const int* foff_h, const int* foff_d, double* partial, int64_t partial_doubles,
                      bool fold, double qscale, int* nchunks_out, hipStream_t stream, const QuantAux* qa = nullptr,
                      const HistPartition& hp = HistPartition(), const HistUpdate* hu = nullptr,
                      const HistSplit* hsp = nullptr, size_t min_lds = 0, const HistPre* pre = nullptr) {
  const bool quant = qscale != 0.0;
  const int C = foff_h[F];
  const int nodesL = 1 << level;
  const int64_t S = (int64_t)T * nodesL * C * 2;
  long long* qpart = reinterpret_cast<long long*>(partial);
  int nchunks = 0;
  if (quant && qa && qa->nb > 0) {
    int NTb = nodesL;
    const int NWb = QB_REP * ((qa->nb + 1) | 1) + qa->foffm_h[qa->Fm];  // words per node
    while (NTb > 1 && (int64_t)2 * NTb * NWb * 8 > HIST_LDS_BUDGET) NTb >>= 1;
    const int64_t per_chunk = (int64_t)T * (nodesL / NTb);  // ~4096 blocks per level
    const int64_t want = (4096 + per_chunk - 1) / per_chunk;
    int64_t chunk = (n + want - 1) / want;
    const int64_t maxch = partial_doubles / S;  // chunks that fit the partial buffer
    if (maxch < 1) return EM_ERR_ARG;
    if ((n + chunk - 1) / chunk > maxch) chunk = (n + maxch - 1) / maxch;
    if (chunk < 64) chunk = 64;
    nchunks = (int)((n + chunk - 1) / chunk);
    hipLaunchKernelGGL(gbdt_hist_qb, dim3(nchunks, T, nodesL / NTb), dim3(256), (size_t)2 * NTb * NWb * 8, stream,
                       qa->bmask_d, qa->WB, qa->bcell_d, qa->nb, bins, F, qa->fmap_d, qa->foffm_d, foff_d, qa->Fm, g,
                       h, node, qpart, T, n, C, level, (int)chunk, NTb, qscale);
  } else {
    HistPlan pl;
    if (!plan_hist(level, n, T, F, foff_h, quant, pl)) return EM_ERR_ARG;
    if ((int64_t)pl.nchunks * S > partial_doubles) return EM_ERR_ARG;
    nchunks = pl.nchunks;
    // (hu: level 0 with one tile per (chunk, task); eval sets on extra z planes)
    if (hu && (quant || level != 0 || pl.nft * pl.ntn != 1)) return EM_ERR_ARG;
    if (pre && (quant || hu || hsp)) return EM_ERR_ARG;
    HistPre pr = pre ? *pre : HistPre();
    if (pre) pr.nz = (pr.nodes + pl.nchunks - 1) / pl.nchunks;  // split planes in front of the histogram's
    const dim3 grid(pl.nchunks, T, pr.nz + pl.nft * pl.ntn + (hu && hu->apply ? hu->evs.count : 0));
    if (quant)
      hipLaunchKernelGGL(gbdt_hist_q, grid, dim3(pl.threads), pl.lds, stream, bins, g, h, node, foff_d,
                         (const int*)nullptr, foff_d, qpart, T, n, F, F, C, level, pl.chunk, pl.FT, pl.NTn, pl.P,
                         pl.ldsC, pl.piece, qscale);
    else
    {
      // exact form: the previous level's split arrays (partition fused in) and, when a piece's bin rows
      // fit 16 KB, the rows themselves are staged in LDS after the (g, h, node) staging
      const int srows = pl.piece < pl.chunk ? pl.piece : pl.chunk;
      const int npn = hp.node_out ? (1 << level) - (1 << (level - 1)) : 0;
      size_t lds = ((pl.lds + 15) & ~(size_t)15) + (((size_t)npn * 4 + 15) & ~(size_t)15);
      const size_t sbytes = (((size_t)srows * F + 32 + 15) & ~(size_t)15);
      const int stage = ((int64_t)srows * F <= 16 * 1024 && lds + sbytes <= GBDT_HIST_MAX_DYN) ? srows : 0;
      if (stage) lds += sbytes;
      if (lds < min_lds) lds = min_lds;  // (the fused root split reuses the histogram's LDS)
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)gbdt_hist, hipFuncAttributeMaxDynamicSharedMemorySize, GBDT_HIST_MAX_DYN);
        attr = true;
      }
      hipLaunchKernelGGL(gbdt_hist, grid, dim3(pl.threads), lds, stream, bins, g, h, node, foff_d, partial, T, n, F,
                         C, level, pl.chunk, pl.FT, pl.NTn, pl.P, pl.ldsC, pl.piece, stage, hp.node_out, hp.st, hp.fe,
                         hp.sb, hp.NN, hu ? *hu : HistUpdate(), hsp ? *hsp : HistSplit(), pr);
    }
  }
  const bool split_folds = !fold && nchunks <= SPLIT_FOLD_MAX_CHUNKS && (int64_t)C * 16 <= SPLIT_FOLD_MAX_LDS;
  if (nchunks > 1 && !split_folds) {
    if (quant)
      hipLaunchKernelGGL(gbdt_chunk_reduce<long long>, dim3(grid_for(S)), dim3(256), 0, stream, qpart, nchunks, S);
    else
      hipLaunchKernelGGL(gbdt_chunk_reduce<double>, dim3(grid_for(S)), dim3(256), 0, stream, partial, nchunks, S);
  }
  *nchunks_out = split_folds ? nchunks : 1;
  EM_CHECK_LAUNCH();
  return 0;
}

bool valid_foff(const int* foff, int F) {
  if (!foff || foff[0] != 0) return false;
  for (int f = 0; f < F; ++f)
    if (foff[f + 1] - foff[f] < 1 || foff[f + 1] - foff[f] > 256) return false;
  return true;
}

// [T] zeroed device ints (grown on demand; left zeroed by every use): gbdt_split's per-task arrival
// counters of the fused finalize
int* task_counters(int T) {
  static int* ctr = nullptr;
  static int cap = 0, dev = -1;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  if (!ctr || dev != d || T > cap) {
    if (ctr && dev == d) {
      (void)hipDeviceSynchronize();
      (void)hipFree(ctr);
    }
    ctr = nullptr;
    int* p = nullptr;
    const int want = T > 1024 ? T : 1024;
    if (hipMalloc(&p, (size_t)want * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, (size_t)want * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
    ctr = p;
    cap = want;
    dev = d;
  }
  return ctr;
}
// one zeroed device int per process (per device in use): the fused metric launches' arrival counter
int* metric_counter() {
  static int* ctr = nullptr;
  static int dev = -1;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  if (!ctr || dev != d) {
    int* p = nullptr;
    if (hipMalloc(&p, 64) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
    ctr = p;
    dev = d;
  }
  return ctr;
}
// one zeroed device int per process (per device in use): raised by a histogram block whose HistPre poll timed
// out (the fit's trees are then invalid); read and cleared by em_gbdt_fused_error
int* fused_error_word() {
  static int* w = nullptr;
  static int dev = -1;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  if (!w || dev != d) {
    int* p = nullptr;
    if (hipMalloc(&p, 64) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
    w = p;
    dev = d;
  }
  return w;
}
}  // namespace

// ------------------------------------------------------------------ C ABI
struct EmGbdtEval {
  const uint8_t* bins;  // [n][F]
  const float* Y;       // [n][T]
  float* margin;        // [T][n] (initialised by the driver)
  int n;
};

// doubles of histogram scratch the driver needs (max over the levels of a depth-D tree); -1 = unsupported
EM_API int64_t em_gbdt_partial_doubles(int n, int T, int F, const int* foff, int max_depth) {
  if (n <= 0 || T <= 0 || F <= 0 || max_depth < 1 || max_depth > 12 || !valid_foff(foff, F)) return -1;
  int64_t need = 0;
  for (int l = 0; l < max_depth; ++l) {
    const int64_t v = partial_need(l, n, T, F, foff);
    if (v < 0) return -1;
    need = v > need ? v : need;
  }
  // two halves (consecutive levels' partials, em_gbdt_fit's HistPre levels) while that stays small
  return need <= (int64_t(1) << 24) ? 2 * need : need;
}

// Trains rounds [r0, r1).  Tree arrays hold ALL rounds: [R*T][NN] (tree k = round*T + task).
// foff_h / foff_d: feature -> first compact histogram cell, [F+1] (host copy for the plan, device copy
// for the kernels); feature f has foff[f+1]-foff[f] bins.
// scratch: g, h [T][n]; node, node2 int16 [T][n]; partial (em_gbdt_partial_doubles); G, H [T][NN]; mpart double[5 * 4096]
// hist_out: float [R][1 + n_evals] (metric of train + each eval set after each round)
EM_API int em_gbdt_fit(const uint8_t* bins, const float* Y, int n, int F, const int* foff_h, const int* foff_d, int T,
                       float* margin, const EmGbdtEval* evals, int n_evals, int r0, int r1, int max_depth, int obj,
                       int metric, float eta, float lam, float gamma, float mcw, float subsample, uint32_t seed,
                       float* g, float* h, int16_t* node, int16_t* node2, double* partial, int64_t partial_doubles,
                       double* Gs, double* Hs, double* mpart, int8_t* status, int16_t* feat, uint8_t* sbin,
                       float* leaf, float* gainv, float* cover, float* hist_out, int quant_bits, int launch_flags,
                       hipStream_t stream) {
  if (!bins || !Y || !margin || n <= 0 || F <= 0 || !valid_foff(foff_h, F) || !foff_d || T <= 0 || max_depth < 1 ||
      max_depth > 12 || r0 < 0 || r1 < r0 || quant_bits < 0 || quant_bits > 61)
    return EM_ERR_ARG;
  // fixed-point histograms (quant_bits = s > 0): the caller guarantees |g|, |h| <= 1 and n < 2^(61-s),
  // so every per-cell and per-node sum of q = rint(x * 2^s) stays below 2^61 in magnitude
  if (quant_bits && (obj == OBJ_SQERR || (int64_t)n >= (1ll << (61 - quant_bits)))) return EM_ERR_ARG;
  const double qscale = quant_bits ? ldexp(1.0, quant_bits) : 0.0, qinv = quant_bits ? ldexp(1.0, -quant_bits) : 0.0;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int C = foff_h[F];
  const int64_t TN = (int64_t)T * n;
  int* mctr = metric_counter();  // arrival counter of the fused metric launches (re-armed by each)
  if (!mctr) return EM_ERR_ARG;
  // fixed point with >= 8 one-hot features: the sparse form (QuantAux)
  QuantAux qa;
  void* qmem = nullptr;
  if (quant_bits) {
    std::vector<int> bcell, bfeat, fmap;
    qa.foffm_h.push_back(0);
    for (int f = 0; f < F; ++f) {
      const int nbins = foff_h[f + 1] - foff_h[f];
      if (nbins == 2) {
        bcell.push_back(foff_h[f]);
        bfeat.push_back(f);
      } else {
        fmap.push_back(f);
        qa.foffm_h.push_back(qa.foffm_h.back() + nbins);
      }
    }
    // sparse form only when one node's cells fit the LDS budget (many continuous features: dense form)
    if (bcell.size() >= 8 && (int64_t)16 * (QB_REP * (((int)bcell.size() + 1) | 1) + qa.foffm_h.back()) <=
                                 HIST_LDS_BUDGET) {
      qa.nb = (int)bcell.size();
      qa.WB = (qa.nb + 63) / 64;
      qa.Fm = (int)fmap.size();
      const size_t ints = 2 * (size_t)qa.nb + (size_t)qa.Fm + (size_t)qa.Fm + 1;
      const size_t mask_off = (ints * 4 + 15) / 16 * 16;
      if (hipError_t e = hipMalloc(&qmem, mask_off + (size_t)n * qa.WB * 8)) return (int)e;
      std::vector<int> hostv;
      hostv.insert(hostv.end(), bcell.begin(), bcell.end());
      hostv.insert(hostv.end(), bfeat.begin(), bfeat.end());
      hostv.insert(hostv.end(), fmap.begin(), fmap.end());
      hostv.insert(hostv.end(), qa.foffm_h.begin(), qa.foffm_h.end());
      int* dv = static_cast<int*>(qmem);
      (void)hipMemcpyAsync(dv, hostv.data(), hostv.size() * 4, hipMemcpyHostToDevice, stream);
      qa.bcell_d = dv;
      qa.fmap_d = dv + 2 * qa.nb;
      qa.foffm_d = dv + 2 * qa.nb + qa.Fm;
      qa.bmask_d = reinterpret_cast<const uint64_t*>(static_cast<char*>(qmem) + mask_off);
      hipLaunchKernelGGL(gbdt_pack_bits, dim3(grid_for((int64_t)n * qa.WB)), dim3(256), 0, stream, bins, n, F,
                         dv + qa.nb, qa.nb, qa.WB, const_cast<uint64_t*>(qa.bmask_d));
    }
  }
  struct Free {  // the scratch outlives every launch of this call: freed after the stream drains
    void* p;
    hipStream_t s;
    ~Free() {
      if (p) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(p);
      }
    }
  } qfree{qmem, stream};
  // direct split candidates (gbdt_split): cell -> {feature, its first cell, its end cell} when no feature
  // has more than SPLIT_DIRECT_MAX_BINS bins (the reference's calendar features: 31); stream-ordered
  // allocation, freed after the last round's launches
  int4* cellinfo_d = nullptr;
  {
    int maxb = 0;
    for (int f = 0; f < F; ++f) maxb = foff_h[f + 1] - foff_h[f] > maxb ? foff_h[f + 1] - foff_h[f] : maxb;
    if (maxb <= SPLIT_DIRECT_MAX_BINS && C > 0) {
      std::vector<int4> ci((size_t)C);
      for (int f = 0; f < F; ++f)
        for (int c = foff_h[f]; c < foff_h[f + 1]; ++c) ci[c] = int4{f, foff_h[f], foff_h[f + 1], 0};
      if (hipMallocAsync(reinterpret_cast<void**>(&cellinfo_d), ci.size() * sizeof(int4), stream) != hipSuccess ||
          hipMemcpyAsync(cellinfo_d, ci.data(), ci.size() * sizeof(int4), hipMemcpyHostToDevice, stream) != hipSuccess)
        return EM_ERR_ARG;
    }
  }
  struct FreeAsync {
    void* p;
    hipStream_t s;
    ~FreeAsync() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } cfree{cellinfo_d, stream};
  // Exact-form fits with an elementwise metric run the fused round: the previous level's partition
  // inside each histogram pass (double-buffered nodes), the prune / leaves in the last level's split
  // (last-arriving block per task), the last partition in the update, and -- per-task objectives --
  // the next round's start in the update too: 7 launches per depth-3 round instead of 13.
  // Bit-identical to the separate launches (same arithmetic on the same values).
  // launch_flags & EM_GBDT_SEPARATE: the separate launches (the bit-identity tests; quantised fits and
  // multi-class metrics always take them)
  int* tctr = nullptr;
  const bool fuse = !(launch_flags & EM_GBDT_SEPARATE) && !quant_bits && metric < MET_MLOGLOSS &&
                    max_depth <= SPLIT_FINAL_MAX_DEPTH && node2 && (tctr = task_counters(2 * T)) != nullptr;
  // deferred metrics (metric_arrive_final with ctr == nullptr): every round's per-block partials of the
  // train and eval sets, reduced by gbdt_metric_rounds after the last round
  const int sets = 1 + n_evals;
  const bool deferred = metric < MET_MLOGLOSS && n_evals <= 4;
  int64_t mstride = grid_for(TN);
  for (int e = 0; e < n_evals; ++e)
    mstride = grid_for((int64_t)T * evals[e].n) > mstride ? grid_for((int64_t)T * evals[e].n) : mstride;
  // update-in-histogram rounds (HistUpdate): the level-0 histogram pass of round r does round r - 1's
  // update; one update launch for the call's last round
  HistPlan p0;
  const bool hist_update = fuse && obj != OBJ_SOFTMAX && deferred && plan_hist(0, n, T, F, foff_h, false, p0) &&
                           p0.nft * p0.ntn == 1 && p0.nchunks * (int64_t)T <= (int64_t)1 << 20;
  const int nch0 = hist_update ? p0.nchunks : 0;
  if (hist_update && (int64_t)T * nch0 > mstride) mstride = (int64_t)T * nch0;
  double* mround = nullptr;
  if (deferred && hipMallocAsync(reinterpret_cast<void**>(&mround), (size_t)(r1 - r0) * sets * mstride * sizeof(double),
                                 stream) != hipSuccess)
    return EM_ERR_ARG;
  FreeAsync mfree{mround, stream};
  // EM_GBDT_PRESPLIT=1: levels >= 1 of the exact fused round run level L's split in the leading blocks of
  // level L + 1's histogram pass (HistPre) when the partial buffer holds two levels' partials (double-
  // buffered halves).  Bit-identical trees; measured equal on the reference fit (849-855 k vs 844-853 k
  // trees/s, 3 interleaved rounds, profiles/r6/gbdt_presplit_ab.txt): the launch boundary it removes is
  // paid back as the in-launch hand-off, so the split launches stay the default
  int64_t pneed = 0;
  for (int l = 0; l < max_depth; ++l) {
    const int64_t v = partial_need(l, n, T, F, foff_h);
    pneed = v > pneed ? v : pneed;
  }
  static const bool presplit_env = [] {
    const char* e = std::getenv("EM_GBDT_PRESPLIT");
    return e && e[0] == '1';
  }();
  const bool presplit = (presplit_env || (launch_flags & EM_GBDT_PRESPLIT)) && fuse && max_depth >= 3 && pneed > 0 &&
                        partial_doubles >= 2 * pneed;
  const int64_t half = presplit ? (partial_doubles / 2) & ~(int64_t)1 : partial_doubles;
  int* sctr = nullptr;  // [T] cumulative split arrivals of this fit
  if (presplit) {
    if (hipMallocAsync(reinterpret_cast<void**>(&sctr), (size_t)T * sizeof(int), stream) != hipSuccess ||
        hipMemsetAsync(sctr, 0, (size_t)T * sizeof(int), stream) != hipSuccess)
      return EM_ERR_ARG;
  }
  FreeAsync sfree{sctr, stream};
  int* perr = presplit ? fused_error_word() : nullptr;
  if (presplit && !perr) return EM_ERR_ARG;
  int pre_cum = 0;  // arrivals per task so far
  // one round's kernel sequence (the arrays of `round` addressed from the host)
  auto enqueue_round = [&](int round, hipStream_t s) -> int {
    const int64_t ro = (int64_t)round * T * NN;
    int8_t* st = status + ro;
    int16_t* fe = feat + ro;
    uint8_t* sb = sbin + ro;
    float* lf = leaf + ro;
    float* gn = gainv + ro;
    float* cv = cover + ro;
    const bool next_in_update = fuse && obj != OBJ_SOFTMAX && !hist_update;  // round + 1 started by this update
    int16_t* nb[2] = {node, fuse ? node2 : node};
    HistPre pending;  // the previous level's split, deferred into this level's histogram pass
    size_t pending_lds = 0;
    if (!hist_update && (!next_in_update || round == r0))
      hipLaunchKernelGGL(gbdt_round_start, dim3(grid_for(TN > (int64_t)T * NN ? TN : (int64_t)T * NN)), dim3(256), 0,
                         s, st, fe, sb, gn, T * NN, NN, margin, Y, g, h, node, T, n, obj, subsample, seed, round);
    for (int level = 0; level < max_depth; ++level) {
      const int nodesL = 1 << level;
      int nch = 1;
      HistPartition hp;
      const int16_t* nin = node;
      if (fuse && level >= 1) {
        nin = nb[(level - 1) & 1];
        hp.node_out = nb[level & 1];
        hp.st = st;
        hp.fe = fe;
        hp.sb = sb;
        hp.NN = NN;
      }
      HistUpdate hu;
      if (hist_update && level == 0) {
        hu.on = 1;
        hu.apply = round > r0;
        hu.round = round;
        hu.obj = obj;
        hu.metric = metric;
        hu.NN = NN;
        hu.plevel = max_depth - 1;
        hu.nz = 1;
        hu.subsample = subsample;
        hu.seed = seed;
        hu.margin = margin;
        hu.Y = Y;
        hu.g = g;
        hu.h = h;
        hu.node = node;
        hu.st = st;
        hu.fe = fe;
        hu.sb = sb;
        hu.gn = gn;
        if (hu.apply) {  // round - 1's tree, node ids and metric partials
          const int64_t rp = ro - (int64_t)T * NN;
          hu.pst = status + rp;
          hu.pfe = feat + rp;
          hu.psb = sbin + rp;
          hu.plf = leaf + rp;
          hu.pnode = nb[(max_depth - 1) & 1];
          hu.mpart = mround + (int64_t)(round - 1 - r0) * sets * mstride;
          hu.mstride = mstride;
          for (int e = 0; e < n_evals; ++e) {
            hu.evs.bins[e] = evals[e].bins;
            hu.evs.margin[e] = evals[e].margin;
            hu.evs.Y[e] = evals[e].Y;
            hu.evs.n[e] = evals[e].n;
          }
          hu.evs.count = n_evals;
        }
      }
      // the root split inside the level-0 pass (HistSplit: its task's last-arriving chunk block)
      HistSplit hsp;
      size_t hsp_lds = 0;
      const bool fsplit = hist_update && level == 0 && nch0 > 1 && nch0 <= SPLIT_FOLD_MAX_CHUNKS &&
                          (int64_t)C * 16 <= SPLIT_FOLD_MAX_LDS && (int64_t)nch0 * C * 16 <= SPLIT_ONESHOT_LDS;
      if (fsplit) {
        hsp.on = 1;
        hsp.ctr = tctr + T;
        hsp.G = Gs;
        hsp.H = Hs;
        hsp.lam = (double)lam;
        hsp.mcw = (double)mcw;
        hsp.NN = NN;
        hsp.cstride = (int64_t)T * C * 2;
        hsp.oneshot = 1;
        hsp.cellinfo = cellinfo_d;
        size_t sl = ((size_t)nch0 * C * 16 + 15) & ~(size_t)15;
        const size_t sb_ = ((size_t)C * 20 + 15) & ~(size_t)15;
        hsp.pscan = sl + sb_ + (size_t)NN * 24 <= 60 * 1024;
        if (hsp.pscan) sl += sb_;
        if (max_depth == 1) {
          hsp.fin.tctr = tctr;
          hsp.fin.leaf = lf;
          hsp.fin.cover = cv;
          hsp.fin.gamma = gamma;
          hsp.fin.eta = (double)eta;
          hsp.fin.max_depth = max_depth;
          sl += (size_t)NN * 24;
        }
        hsp_lds = sl;
      }
      double* lpart = presplit ? partial + (level & 1) * half : partial;  // this level's partials
      HistPre* prep = nullptr;
      if (pending.on) {
        pre_cum += pending.nodes;
        pending.want = pre_cum;
        prep = &pending;
      }
      const int rc = launch_level_hist(level, bins, g, h, nin, T, n, F, foff_h, foff_d, lpart, half,
                                       false, qscale, &nch, s, qa.nb ? &qa : nullptr, hp,
                                       hist_update && level == 0 ? &hu : nullptr, fsplit ? &hsp : nullptr,
                                       prep ? pending_lds : hsp_lds, prep);
      pending = HistPre();
      if (rc) return rc;
      if (fsplit) continue;  // (split done by the pass itself)
      const int sth = (F >= 256 || nch > 1) ? 256 : ((F + 63) / 64) * 64;
      const int64_t cstride = (int64_t)T * nodesL * C * 2;
      const int oneshot = nch > 1 && (int64_t)nch * C * 16 <= SPLIT_ONESHOT_LDS;
      size_t slds = nch > 1 ? (((size_t)(oneshot ? nch : 1) * C * 16 + 15) & ~(size_t)15) : 0;
      const size_t scan_b = ((size_t)C * 20 + 15) & ~(size_t)15;
      const int pscan = slds + scan_b + (size_t)NN * 24 <= 60 * 1024;  // (+ the finalize area: < 64 KB)
      if (pscan) slds += scan_b;
      SplitFinal fin;
      if (fuse && level == max_depth - 1) {
        fin.tctr = tctr;
        fin.leaf = lf;
        fin.cover = cv;
        fin.gamma = gamma;
        fin.eta = (double)eta;
        fin.max_depth = max_depth;
        slds += (size_t)NN * 24;
      }
      if (presplit && level >= 1 && level + 1 < max_depth) {  // runs in the next level's histogram pass
        pending.on = 1;
        pending.nodes = nodesL;
        pending.level = level;
        pending.nchunks = nch;
        pending.oneshot = oneshot;
        pending.pscan = pscan;
        pending.NN = NN;
        pending.ctr = sctr;
        pending.err = perr;
        pending.hist = lpart;
        pending.cstride = cstride;
        pending.G = Gs;
        pending.H = Hs;
        pending.st = st;
        pending.fe = fe;
        pending.sb = sb;
        pending.gn = gn;
        pending.lam = (double)lam;
        pending.mcw = (double)mcw;
        pending.cellinfo = cellinfo_d;
        pending_lds = slds;
        continue;
      }
      if (quant_bits)
        hipLaunchKernelGGL(gbdt_split<long long>, dim3(T * nodesL), dim3(sth), slds, s,
                           reinterpret_cast<const long long*>(lpart), nch, cstride, foff_d, T, F, C, level, NN, Gs,
                           Hs, st, fe, sb, gn, (double)lam, (double)mcw, qinv, fin, oneshot, pscan, cellinfo_d);
      else
        hipLaunchKernelGGL(gbdt_split<double>, dim3(T * nodesL), dim3(sth), slds, s, lpart, nch, cstride,
                           foff_d, T, F, C, level, NN, Gs, Hs, st, fe, sb, gn, (double)lam, (double)mcw, 0.0, fin,
                           oneshot, pscan, cellinfo_d);
      if (!fuse)
        hipLaunchKernelGGL(gbdt_partition, dim3(grid_for(TN)), dim3(256), 0, s, bins, node, T, n, F, NN, st, fe, sb,
                           level);
    }
    if (!fuse)
      hipLaunchKernelGGL(gbdt_finalize, dim3((T + 63) / 64), dim3(64), 0, s, T, NN, max_depth, st, fe, gn, Gs, Hs, lf,
                         cv, (double)lam, gamma, (double)eta);
    if (hist_update && round < r1 - 1) {  // this round's update runs in the next round's level-0 pass
      EM_CHECK_LAUNCH();
      return 0;
    }
    // metrics (train + evals) into hist_out[round].  Elementwise metrics: the leaf update / eval
    // prediction, the metric partials and the final sum are one launch each (last-arriving block)
    const int hs = 1 + n_evals;
    float* ho = hist_out + (int64_t)round * hs;
    const int mb_train = grid_for(TN);
    const bool fused_metric = metric < MET_MLOGLOSS;
    if (fused_metric) {
      NextRound nx;
      if (next_in_update && round + 1 < r1) {
        const int64_t rn = ro + (int64_t)T * NN;
        nx.round = round + 1;
        nx.g = g;
        nx.h = h;
        nx.node = node;
        nx.st = st + (int64_t)T * NN;
        nx.fe = fe + (int64_t)T * NN;
        nx.sb = sb + (int64_t)T * NN;
        nx.gn = gainv + rn;
        nx.subsample = subsample;
        nx.seed = seed;
      }
      // the eval sets' predictions ride in the same launch (trailing blocks)
      EvalSets evs;
      int grid = mb_train;
      if (n_evals <= 4) {
        for (int e = 0; e < n_evals; ++e) {
          evs.bins[e] = evals[e].bins;
          evs.margin[e] = evals[e].margin;
          evs.Y[e] = evals[e].Y;
          evs.n[e] = evals[e].n;
          evs.mb[e] = grid_for((int64_t)T * evals[e].n);
          grid += evs.mb[e];
        }
        evs.count = n_evals;
        if (deferred) evs.pstride = mstride;
      }
      double* mp = deferred ? mround + (int64_t)(round - r0) * sets * mstride : mpart;
      hipLaunchKernelGGL(gbdt_update_metric, dim3(grid), dim3(256), 0, s, margin,
                         fuse ? nb[(max_depth - 1) & 1] : node, T, n, NN, st, lf, Y, obj, metric, mp,
                         deferred ? nullptr : mctr, ho,
                         bins, F, fuse ? max_depth - 1 : -1, fe, sb, nx, mb_train, evs);
      if (evs.count == n_evals) {
        EM_CHECK_LAUNCH();
        return 0;
      }
    } else {
      hipLaunchKernelGGL(gbdt_update, dim3(grid_for(TN)), dim3(256), 0, s, margin, node, T, n, NN, st, lf);
      hipLaunchKernelGGL(gbdt_metric, dim3(mb_train), dim3(256), 0, s, margin, Y, T, n, obj, metric, mpart);
      hipLaunchKernelGGL(gbdt_metric_final, dim3(1), dim3(256), 0, s, mpart, mb_train,
                         metric >= MET_MLOGLOSS ? (int64_t)n : TN, metric, ho);
    }
    for (int e = 0; e < n_evals; ++e) {
      const int64_t TE = (int64_t)T * evals[e].n;
      const int k0 = round * T;
      const int mb = grid_for(TE);
      if (fused_metric) {
        hipLaunchKernelGGL(gbdt_predict_metric, dim3(mb), dim3(256), 0, s, evals[e].bins, evals[e].margin, T,
                           evals[e].n, F, NN, k0, k0 + T, status, feat, sbin, leaf, evals[e].Y, obj, metric, mpart,
                           mctr, ho + 1 + e);
        continue;
      }
      hipLaunchKernelGGL(gbdt_predict, dim3(grid_for(TE)), dim3(256), 0, s, evals[e].bins, evals[e].margin, T,
                         evals[e].n, F, NN, k0, k0 + T, status, feat, sbin, leaf);
      hipLaunchKernelGGL(gbdt_metric, dim3(mb), dim3(256), 0, s, evals[e].margin, evals[e].Y, T, evals[e].n, obj,
                         metric, mpart);
      hipLaunchKernelGGL(gbdt_metric_final, dim3(1), dim3(256), 0, s, mpart, mb,
                         metric >= MET_MLOGLOSS ? (int64_t)evals[e].n : TE, metric, ho + 1 + e);
    }
    EM_CHECK_LAUNCH();
    return 0;
  };
  for (int round = r0; round < r1; ++round)
    if (int rc = enqueue_round(round, stream)) return rc;
  if (deferred) {
    MetricRounds mr{};
    mr.count[0] = TN;
    for (int e = 0; e < n_evals; ++e) mr.count[1 + e] = (int64_t)T * evals[e].n;
    const int first = hist_update ? r1 - 1 : r0;  // rounds [r0, first): partials of the level-0 passes
    if (first > r0) {
      for (int k = 0; k < sets; ++k) mr.nb[k] = T * nch0;
      hipLaunchKernelGGL(gbdt_metric_rounds, dim3((first - r0) * sets), dim3(256), 0, stream, mround, mstride, sets,
                         mr, metric, hist_out + (int64_t)r0 * sets);
    }
    mr.nb[0] = grid_for(TN);
    for (int e = 0; e < n_evals; ++e) mr.nb[1 + e] = grid_for((int64_t)T * evals[e].n);
    hipLaunchKernelGGL(gbdt_metric_rounds, dim3((r1 - first) * sets), dim3(256), 0, stream,
                       mround + (int64_t)(first - r0) * sets * mstride, mstride, sets, mr, metric,
                       hist_out + (int64_t)first * sets);
    EM_CHECK_LAUNCH();
  }
  return 0;
}

// 1 if a fused-level poll timed out since the last call (the trees of that fit are invalid), else 0;
// synchronises the device and clears the word
EM_API int em_gbdt_fused_error() {
  int* w = fused_error_word();
  if (!w) return -1;
  int v = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&v, w, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (v) (void)hipMemset(w, 0, sizeof(int));
  return v;
}

// GBDT_STAMPS builds: the 256 phase stamps (100 MHz ticks) and the matching 256 shader-clock counts
// to host memory (512 values); -1 in other builds
EM_API int em_gbdt_stamps(unsigned long long* out) {
#if GBDT_STAMPS
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(g_stamp));
#else
  (void)out;
  return -1;
#endif
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

// histogram of one level folded into partial[0 : T*2^level*C*2]; returns that length in *len_out
EM_API int em_gbdt_dp_level_hist(int level, const uint8_t* bins, const float* g, const float* h, const int16_t* node,
                                 int T, int n, int F, const int* foff_h, const int* foff_d, double* partial,
                                 int64_t partial_doubles, int64_t* len_out, hipStream_t stream) {
  if (!bins || !g || !h || !node || !partial || !len_out || level < 0 || level > 11 || !valid_foff(foff_h, F) ||
      !foff_d)
    return EM_ERR_ARG;
  int nch = 1;
  const int rc = launch_level_hist(level, bins, g, h, node, T, n, F, foff_h, foff_d, partial, partial_doubles, true,
                                   0.0, &nch, stream);
  if (rc) return rc;
  EM_CHECK_LAUNCH();
  *len_out = (int64_t)T * (1 << level) * foff_h[F] * 2;
  return 0;
}

EM_API int em_gbdt_dp_level_split(int level, const uint8_t* bins, const double* hist, int T, int n, int F,
                                  const int* foff_d, int C, int max_depth, int16_t* node, double* Gs, double* Hs,
                                  int8_t* status, int16_t* feat, uint8_t* sbin, float* gainv, float lam, float mcw,
                                  hipStream_t stream) {
  if (!bins || !hist || !node || !Gs || !Hs || !status || !foff_d || C < F || level < 0 || level >= max_depth)
    return EM_ERR_ARG;
  const int NN = (1 << (max_depth + 1)) - 1;
  const int nodesL = 1 << level;
  const int64_t TN = (int64_t)T * n;
  const int sth = F >= 256 ? 256 : ((F + 63) / 64) * 64;
  hipLaunchKernelGGL(gbdt_split<double>, dim3(T * nodesL), dim3(sth), 0, stream, hist, 1, (int64_t)0, foff_d, T, F, C,
                     level, NN, Gs, Hs, status, feat, sbin, gainv, (double)lam, (double)mcw, 0.0, SplitFinal(), 0, 0,
                     (const int4*)nullptr);
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
    hipLaunchKernelGGL(gbdt_metric_sum, dim3(1), dim3(256), 0, stream, mpart, mb, out);
  } else {
    hipLaunchKernelGGL(gbdt_metric_sum, dim3(1), dim3(256), 0, stream, mpart, 0, out);
  }
  EM_CHECK_LAUNCH();
  return 0;
}
