// K1/K2/K3 — bf16 MFMA GEMM with fused epilogues for the generic MLP layers (MI355X / gfx950).
//
// The declared-but-unused DL4J/ND4J dense layers (pom.xml:62-66) become one templated
// kernel:  C[m][n] = epi( alpha * sum_k A[m][k] * B[k][n] )
//   A[m][k] at A + m*lda + k   (A_KC = 1, K-contiguous)   or A + k*lda + m (A_KC = 0)
//   B[k][n] at B + n*ldb + k   (B_KC = 1, K-contiguous)   or B + k*ldb + n (B_KC = 0)
//   epi: + bias[n], activation (none/relu/sigmoid/tanh), * act'(Y[m][n]) (activation backward
//        from the saved layer output Y: relu Y>0, sigmoid Y(1-Y), tanh 1-Y^2),
//        + beta * C_old (fp32 accumulate), store fp32 or bf16.
// Uses: forward  Y = act(X W^T + b)            A=X (KC), B=W[N][K] (KC)
//       dgrad    dZ_prev = (dZ W) * act'(Y_prev) A=dZ (KC), B=W (NC), Y=Y_prev
//       wgrad    dW = dZ^T X  (fp32)            A=dZ (MC), B=X (NC)
//
// Tiling: 128x128 output tile per 256-thread workgroup (2x2 waves of 64x64, each 2x2 MFMA
// 32x32x16 tiles, 64 accumulator registers), BK = 64, two LDS stages (64 KB).  Global ->
// register -> LDS staging with the next K tile's loads issued before the current tile's
// MFMAs (write-after-barrier, cdna_hip_programming.md §5.5 T14).  K-contiguous tiles are
// stored [rows][64] with a 16-byte-chunk XOR swizzle (chunk ^ row&7: conflict-free
// ds_read_b128 fragment reads); MN-contiguous tiles are stored [64 k][128] (256-B rows,
// chunk ^ k&15) and read as MFMA fragments with ds_read_b64_tr_b16.  Block ids are
// remapped so neighbouring tiles share an XCD's L2 (§5.5 T1, bijective form).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KB per operand per stage
constexpr int LDS_BYTES = 2 * 2 * TILE_BYTES;

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

EM_DEVICE uint32_t kc_off(int row, int chunk) { return row * 128 + (((chunk ^ (row & 7))) << 4); }     // [128][64]
EM_DEVICE uint32_t mc_off(int krow, int chunk) { return krow * 256 + (((chunk ^ (krow & 15))) << 4); }  // [64][128]

// load one 128x64 (KC) or 64x128 (MC) bf16 tile piece: 4 x 16 B per thread, zero-filled out of range
template <int KC>
EM_DEVICE void load_tile(const __bf16* __restrict__ P, int64_t ld, int r0, int k0, int R, int K, int tid,
                         u32x4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + i * NT;  // 1024 chunks of 16 B
    int row, kk;
    if (KC) {  // tile rows = r (128), 8 chunks of 8 k each
      row = r0 + (c >> 3);
      kk = k0 + (c & 7) * 8;
    } else {  // tile rows = k (64), 16 chunks of 8 rows(m/n) each
      kk = k0 + (c >> 4);
      row = r0 + (c & 15) * 8;
    }
    u32x4 v = {0u, 0u, 0u, 0u};
    if (KC) {
      if (row < R && kk + 8 <= K) {
        v = *reinterpret_cast<const u32x4*>(P + (int64_t)row * ld + kk);
      } else if (row < R && kk < K) {
        __bf16 tmp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tmp[e] = (kk + e < K) ? P[(int64_t)row * ld + kk + e] : (__bf16)0.f;
        v = *reinterpret_cast<const u32x4*>(tmp);
      }
    } else {
      if (kk < K && row + 8 <= R) {
        v = *reinterpret_cast<const u32x4*>(P + (int64_t)kk * ld + row);
      } else if (kk < K && row < R) {
        __bf16 tmp[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) tmp[e] = (row + e < R) ? P[(int64_t)kk * ld + row + e] : (__bf16)0.f;
        v = *reinterpret_cast<const u32x4*>(tmp);
      }
    }
    reg[i] = v;
  }
}

template <int KC>
EM_DEVICE void store_tile(char* lds, int tid, const u32x4 (&reg)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + i * NT;
    const uint32_t off = KC ? kc_off(c >> 3, c & 7) : mc_off(c >> 4, c & 15);
    *reinterpret_cast<u32x4*>(lds + off) = reg[i];
  }
}

// fragment for k-step s: lane's row/col index `rc` (0..127 within the tile), elements k = 16s+8h+j
template <int KC>
EM_DEVICE bf16x8 frag(const char* lds, int rc, int s, int lane) {
  const int h = lane >> 5;
  if (KC) return *reinterpret_cast<const bf16x8*>(lds + kc_off(rc, 2 * s + h));
  // MC: transposed read of 4 k-rows x 16 cols per 16-lane group
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int cbase = rc - i16;  // first column of the group's 16
  const int col = cbase + 4 * p4;
  const int kr = 16 * s + 8 * h + q4;
  const uint32_t o0 = mc_off(kr, col >> 3) + (col & 7) * 2;
  const uint32_t o1 = mc_off(kr + 4, col >> 3) + (col & 7) * 2;
  return cat_tr(lds_tr16(lds, o0), lds_tr16(lds, o1));
}

EM_DEVICE float apply_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

template <int A_KC, int B_KC>
__global__ void __launch_bounds__(NT, 2)
gemm_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb, void* __restrict__ C,
            int64_t ldc, int c_bf16, int M, int N, int K, const float* __restrict__ bias, int act,
            const __bf16* __restrict__ mask, int64_t ldm, int dact, float alpha, float beta, int kstep,
            int64_t c_split) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (gridDim.y > 1) {  // split-K: slice blockIdx.y of the reduction into its own fp32/bf16 partial output
    const int k0 = blockIdx.y * kstep;
    A += A_KC ? (int64_t)k0 : (int64_t)k0 * lda;
    B += B_KC ? (int64_t)k0 : (int64_t)k0 * ldb;
    K = min(kstep, K - k0);
    C = reinterpret_cast<char*>(C) + (int64_t)blockIdx.y * c_split * (c_bf16 ? 2 : 4);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = (K + BK - 1) / BK;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  u32x4 ra[4], rb[4];
  load_tile<A_KC>(A, lda, m0, 0, M, K, tid, ra);
  load_tile<B_KC>(B, ldb, n0, 0, N, K, tid, rb);
  store_tile<A_KC>(smem, tid, ra);
  store_tile<B_KC>(smem + TILE_BYTES, tid, rb);
  __syncthreads();

  const int r = lane & 31;
  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    const char* la = smem + cur * 2 * TILE_BYTES;
    const char* lb = la + TILE_BYTES;
    const bool more = kt + 1 < ktiles;
    if (more) {  // issue next tile's global loads before this tile's MFMAs
      load_tile<A_KC>(A, lda, m0, (kt + 1) * BK, M, K, tid, ra);
      load_tile<B_KC>(B, ldb, n0, (kt + 1) * BK, N, K, tid, rb);
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const bf16x8 a0 = frag<A_KC>(la, wm * 64 + r, s, lane);
      const bf16x8 a1 = frag<A_KC>(la, wm * 64 + 32 + r, s, lane);
      const bf16x8 b0 = frag<B_KC>(lb, wn * 64 + r, s, lane);
      const bf16x8 b1 = frag<B_KC>(lb, wn * 64 + 32 + r, s, lane);
      acc[0][0] = mfma32(a0, b0, acc[0][0]);
      acc[0][1] = mfma32(a0, b1, acc[0][1]);
      acc[1][0] = mfma32(a1, b0, acc[1][0]);
      acc[1][1] = mfma32(a1, b1, acc[1][1]);
    }
    if (more) {
      char* na = smem + (cur ^ 1) * 2 * TILE_BYTES;
      store_tile<A_KC>(na, tid, ra);  // the other stage was last read before the previous barrier
      store_tile<B_KC>(na + TILE_BYTES, tid, rb);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + 32 * j + r;
    if (col >= N) continue;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int row = m0 + wm * 64 + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (row >= M) continue;
        float x = alpha * acc[i][j][v] + bv;
        x = apply_act(x, act);
        if (mask) {
          const float y = (float)mask[(int64_t)row * ldm + col];
          x *= dact == ACT_RELU ? (y > 0.f ? 1.f : 0.f) : dact == ACT_SIGMOID ? y * (1.f - y) : 1.f - y * y;
        }
        if (c_bf16) {
          reinterpret_cast<__bf16*>(C)[(int64_t)row * ldc + col] = (__bf16)x;
        } else {
          float* cp = reinterpret_cast<float*>(C) + (int64_t)row * ldc + col;
          *cp = beta != 0.f ? x + beta * *cp : x;
        }
      }
    }
  }
}

// ============================================================================================
// 256x256 NT GEMM (both operands K-contiguous): the large-shape path (wide MLP hidden layers).
// 8 waves as 2(M) x 4(N), each 128x64 = 4x2 MFMA 32x32x16 tiles (128 accumulator registers);
// BK = 64; per K-tile each wave issues 4+4 global_load_lds_dwordx4 (1 KiB each, 8 rows) into
// the other LDS stage while it reads fragments and runs 32 MFMAs on the current one.  The LDS
// image is lane-linear per instruction (glds writes base + lane*16), so the bank swizzle is
// applied to the per-lane SOURCE address (cdna_hip_programming.md rule 21): logical chunk c of
// row r sits at physical chunk c ^ ((r >> 1) & 7) of its 128-B row -- 16 distinct 16-B slots
// for every ds_read_b128 lane group of the 32x32x16 operand read (MI355X_MICROARCH.md LDS table).
constexpr int G_BM = 256, G_BN = 256, G_BK = 64, G_NT = 512;
constexpr int G_TILE = G_BM * G_BK * 2;  // 32 KB per operand per stage
constexpr int G_LOOP_LDS = 2 * 2 * G_TILE;  // 128 KB: 2 stages x (A, B)
constexpr int G_EPI_LDS = 8 * (64 * 80 + 32 * 144);  // epilogue: per-wave transposed 64x32 tile + 32x64 Y block
constexpr int G_LDS = G_LOOP_LDS > G_EPI_LDS ? G_LOOP_LDS : G_EPI_LDS;

EM_DEVICE uint32_t g_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// (XCD-contiguous) block id -> output tile, grouped GM tile-rows at a time: the ~32 blocks an XCD
// runs at once form a GM x (32/GM) super-tile, so each A panel slice is shared by 32/GM blocks and
// each B panel slice by GM blocks in that XCD's L2 (GM = 8: ~12 GB of panel traffic per 65536 x 8192
// x 8192 GEMM instead of ~33 GB with whole tile-rows, whose 32 distinct B panels miss L2).
// GM: tile-rows per group.  Measured (tools/gpurun_gemm_gm.sh, TF/s at GM = 1 / 2 / 4 / 8): without a
// C^T output 4 is best (65536x8192x8192 forward 1353 / 1384 / 1413 / 1366, NT dgrad 1270 / 1311 /
// 1341 / 1324); with C^T 8 is (forward+C^T 1256 / 1287 / 1314 / 1329).

template <int HAS_CT>
EM_DEVICE void g_tile(int bid, int tiles_m, int tiles_n, int& m0, int& n0) {
  constexpr int GM = HAS_CT ? 8 : 4;
  const int per = GM * tiles_n;
  const int grp = bid / per, first = grp * GM;
  const int gm = tiles_m - first < GM ? tiles_m - first : GM;
  const int in = bid - grp * per;
  m0 = (first + in % gm) * G_BM;
  n0 = (in / gm) * G_BN;
}

// One operand's K-tile piece for this wave: 4 x buffer_load_dwordx4 ... lds (1 KiB each).
// The descriptor covers the block's 256-row panel; the per-lane part is one 32-bit voffset per
// row-group parity (the swizzle depends on (row >> 1) & 7), everything else is scalar.
//
// MN-contiguous operands (MN = 1: element (row r, k) at P + k * ld + r -- the natural layout of a
// wgrad's dZ and X and of a dgrad's W, so no transposed copies): the 64 x 256 K-tile is stored as 8
// sub-units of 32 rows, sub-unit s = [64 k][64 B] at s * 4 KiB; 1-KiB piece `grp` = sub-unit grp >> 2,
// k-rows 16 (grp & 3) .. + 15 (4 lanes x 16 B per k-row, one 64-B global segment each), so a piece
// sits at grp * 1 KiB exactly like the K-contiguous image and the staging schedule is unchanged.
// The 32-B half h of k-row k is stored at half h ^ ((k >> 3) & 1): the ds_read_b64_tr_b16 fragment
// reads (16 lanes = 4 k-rows x 32 B, 4 groups 8 k-rows apart) then cover 8 distinct 32-B bank slots
// per half-wave.
struct GPanel {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff[2];  // per-lane byte offsets for even / odd 8-row groups (MN: both the same)
  uint32_t row_bytes;
};

template <int MN>
EM_DEVICE GPanel g_panel(const __bf16* P, int64_t ld, int r0, int lane) {
  GPanel g;
  const __bf16* base = MN ? P + r0 : P + (int64_t)r0 * ld;
  g.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFFF, 0x00020000);
  if (MN) {
    const int lr = lane >> 2;                                 // k-row within the 16-row piece
    const int c = (lane & 3) ^ (((lr >> 3) & 1) << 1);       // stored 16-B chunk -> source chunk
    g.voff[0] = g.voff[1] = (uint32_t)((lr * ld + 8 * c) * 2);
  } else {
    const int lr = lane >> 3;  // row within the 8-row group
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int c = (lane & 7) ^ ((4 * par + (lane >> 4)) & 7);  // (row >> 1) & 7 with row = 8g + lr
      g.voff[par] = (uint32_t)((lr * ld + 8 * c) * 2);
    }
  }
  g.row_bytes = (uint32_t)(ld * 2);
  return g;
}

// scalar source offset of 1-KiB piece `grp` of the K-tile at k0
template <int MN>
EM_DEVICE uint32_t g_soff(const GPanel& g, int grp, int k0) {
  if (MN) return (uint32_t)(k0 + 16 * (grp & 3)) * g.row_bytes + (uint32_t)(grp >> 2) * 64;
  return (uint32_t)(grp * 8) * g.row_bytes + (uint32_t)k0 * 2;
}

// (mn is a compile-time constant at every call site; the staging helpers are plain functions because
// the host pass of a template rejects the LDS-pointer builtin)
EM_DEVICE void g_stage(const GPanel& g, int k0, char* lds_tile, int wave, bool mn) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int grp = wave * 4 + i;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(g.rsrc, (EM_LDS void*)(lds_tile + grp * 1024), 16, g.voff[i & 1],
                                             mn ? g_soff<1>(g, grp, k0) : g_soff<0>(g, grp, k0), 0, 0);
  }
}

// 16x16x32 operand fragment of rows row0 .. row0 + 15 (row0 % 16 == 0), k-step ks of the K-tile image:
// lane l gets row row0 + (l & 15), k = 32 ks + 8 (l >> 4) + 0..7
template <int MN>
EM_DEVICE bf16x8 g_frag(const char* l, int row0, int ks, int lane) {
  const int r16 = lane & 15, c4 = lane >> 4;
  if (!MN) return *reinterpret_cast<const bf16x8*>(l + g_off(row0 + r16, 4 * ks + c4));
  // transposed reads: lane (q4, p4) of a 16-lane group addresses k-row kr + q4, rows row0 + 4 p4 .. + 3
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const uint32_t o = (uint32_t)((row0 >> 5) * 4096 + (32 * ks + 8 * c4 + q4) * 64 +
                                ((((row0 >> 4) & 1) ^ (c4 & 1)) << 5) + 8 * p4);
  return cat_tr(lds_tr16(l, o), lds_tr16(l, o + 256));  // k-rows + 0..3, + 4..7
}

template <int FN>
EM_DEVICE float g_fn(float v) {
  if (FN == ACT_RELU) return fmaxf(v, 0.f);
  if (FN == ACT_SIGMOID) return 1.f / (1.f + __expf(-v));
  if (FN == ACT_TANH) return tanhf(v);
  return v;
}
template <int FN>
EM_DEVICE float g_dfn(float y) {  // activation derivative from the saved output y
  if (FN == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (FN == ACT_SIGMOID) return y * (1.f - y);
  return 1.f - y * y;
}

// ReLU activity bits, uint32 [M / 32][N]: bit (m & 31) of word (m >> 5) * N + n is output[m][n] > 0.
// A forward epilogue with relu writes them next to its bf16 output; the relu dgrad of the layer above
// reads one dword per lane and 32-row block instead of staging the 32 x 64 bf16 activation block.
// Per 32-row block the lane of the 32x32 accumulator layout (column lc, rows 8g + 4h + e) holds bits
// 8g + 4h + e; the 16x16 layout's lane (column lc, rows 16tm + 4(lane >> 4) + e) holds 16tm + 4(lane >> 4) + e.
EM_DEVICE uint32_t or_xhalf(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (uint32_t)r[0] | (uint32_t)r[1];
}
EM_DEVICE uint32_t or_rows16(uint32_t v) {  // OR over the four 16-lane rows (same lane & 15)
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return or_xhalf((uint32_t)a[0] | (uint32_t)a[1]);
}
EM_DEVICE float bit_mul(uint32_t w, int b, float v) { return ((w >> b) & 1u) ? v : v * 0.f; }

// ============================================================================================
// 256x256 NT GEMM, ping-pong schedule (the large-shape path).  The K loop is structured so
// that the two waves sharing each SIMD alternate roles (cdna_hip_programming.md §5 "256² 8-phase
// template", MI355X_MICROARCH.md "Two waves per SIMD"):
//   * G0 = waves 0-3 (A rows 0-127), G1 = waves 4-7 (A rows 128-255); G1 starts one barrier late,
//     so in every barrier interval ("slot") one group runs MFMAs while the other reads fragments
//     and issues staging -> matrix work beside memory work on every SIMD.
//   * a phase = one 64x32 quadrant of the wave's 128x64 tile over one K-tile (8 MFMA 32x32x16);
//     quadrants qn-major: (qm, qn) = (0,0) (1,0) (0,1) (1,1), the B fragments of (0,qn) are reused
//     by (1,qn) (40 instead of 48 ds_read_b128 per wave per K-tile).
//   * LDS holds 2 K-tiles (64 KB each: A 32 KB | B 32 KB).  A K-tile is staged as 8 units of 64 rows
//     (8 KB: 2 buffer_load...lds per thread of ONE group): A0..A3 = A rows 64u.., and B units by
//     the quadrant half they feed: B(lo, p) = rows {(2p+b)*64 + 0..31}, B(hi, p) = {(2p+b)*64 + 32..63}.
//   * one unit per slot; unit of K-tile kt issued in slot 8kt + o: B(lo,0) -12, B(lo,1) -11, A0 -10,
//     A2 -9, A1 -8, A3 -7, B(hi,0) -6, B(hi,1) -5 (residue r = slot & 7 picks the unit).
//     Each load segment issues its unit then waits vmcnt(6): the unit its group issued 3 load
//     segments (6 slots) earlier has landed, and becomes readable after the barrier that follows.
//   Hazards (slot numbers relative to 8kt; G0 reads phase g in slot 2g-1, G1 in slot 2g):
//     RAW: unit issued at o is readable from o+7 <= its first read (B lo -1, A0 -1, A2 0, A1 1,
//          A3 2, B hi 3).
//     WAR: the same unit of K-tile kt-2 was last read at (B lo 2, A0 3, A2 4, A1 5, A3 6, B hi 4)-16;
//          each reader retires its reads (lgkmcnt(0)) before the barrier that ends its next slot,
//          so a restage 2 slots after the last read is safe: every o above is >= last + 2 - 16.
// (MN operands: piece grp = sub-unit grp >> 2, so a 64-row unit is sub-units 2u, 2u + 1 and the B
// halves B(lo / hi, p) are the sub-units 2 (2p + b) + hsel -- the same 1-KiB slots as the KC image)
__device__ __forceinline__ void pp_stage_unit(const GPanel& g, int k0, char* lds_op, int first_grp, bool split_b,
                                               int hsel, int pair, int wi, bool mn) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = 2 * wi + i;  // this wave's row-group of the unit's 8
    const int grp = split_b ? (2 * pair + (j >> 2)) * 8 + hsel * 4 + (j & 3) : first_grp + j;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(g.rsrc, (EM_LDS void*)(lds_op + grp * 1024), 16, g.voff[grp & 1],
                                             mn ? g_soff<1>(g, grp, k0) : g_soff<0>(g, grp, k0), 0, 0);
  }
}

// issue the unit scheduled for slot s (wave-uniform); false when it belongs past the last K-tile
template <int AMN, int BMN>
__device__ __forceinline__ bool pp_stage_slot(const GPanel& pa, const GPanel& pb, char* smem, int s, int ktiles,
                                               int wi) {
  const int r = s & 7, w = s >> 3;  // arithmetic shift: s = -1 -> w = -1, r = 7
  const int kt = w + (r < 4 ? 1 : 2);
  if (kt >= ktiles) return false;
  char* buf = smem + (kt & 1) * 2 * G_TILE;
  const int k0 = kt * G_BK;
  switch (r) {
    case 0: pp_stage_unit(pa, k0, buf, 8, false, 0, 0, wi, AMN); break;            // A1
    case 1: pp_stage_unit(pa, k0, buf, 24, false, 0, 0, wi, AMN); break;           // A3
    case 2: pp_stage_unit(pb, k0, buf + G_TILE, 0, true, 1, 0, wi, BMN); break;    // B(hi,0)
    case 3: pp_stage_unit(pb, k0, buf + G_TILE, 0, true, 1, 1, wi, BMN); break;    // B(hi,1)
    case 4: pp_stage_unit(pb, k0, buf + G_TILE, 0, true, 0, 0, wi, BMN); break;    // B(lo,0)
    case 5: pp_stage_unit(pb, k0, buf + G_TILE, 0, true, 0, 1, wi, BMN); break;    // B(lo,1)
    case 6: pp_stage_unit(pa, k0, buf, 0, false, 0, 0, wi, AMN); break;            // A0
    default: pp_stage_unit(pa, k0, buf, 16, false, 0, 0, wi, AMN); break;          // A2
  }
  return true;
}

// --------------------------------------------------------------------------------------------
// The same ping-pong K loop on v_mfma_f32_16x16x32_bf16 (16 cycles, 16x16 output per instruction).
// Same LDS image, staging units, slot schedule and quadrant order; per phase a wave runs
// 4 (rows) x 2 (cols) x 2 (k-steps of 32) = 16 MFMAs instead of 8 of the 32x32x16 form.  The
// 16x16x32 shape sustains a higher clock under load for the same cycles per FLOP
// (MI355X_MICROARCH.md, matrix-core notes), which is where its gain comes from.
// Fragment reads: lane l takes row (l & 15) of a 16-row block and the 16-B chunk 4*ks + (l >> 4)
// of the 128-B row; with the (row >> 1) & 7 chunk swizzle each 16-lane group of a ds_read_b128
// hits 16 distinct 16-B slots (conflict-free, as for the 32-row reads).
// Accumulators acc[mb][nb] (mb = 16-row block 0..7 of the wave's 128 rows, nb = 16-col block 0..3):
// lane l holds rows 4*(l >> 4) + e, column l & 15.
EM_DEVICE f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// OUT_BF16: 1 -> bf16 C (optionally + transposed C^T when HAS_CT), 0 -> fp32 C (+ beta * C_old)
// FN: activation (DACT = 0, applied to alpha*acc + bias) or activation' (DACT = 1, multiplies
// alpha*acc by act'(mask[m][n]))
// G_CROW = 1: bf16 C rows leave through a row image, 8 lanes per 128-B row (see gemm_k64_kernel)
#ifndef G_CROW
#define G_CROW 1
#endif
// g_epilogue for the 16x16 accumulator layout: per 32-row block i the lane's values land in the
// same transposed per-wave LDS tile T[64 cols][32 rows] (4 consecutive rows = one 8-B write), so
// everything after the tile is shared with the 32x32 form.
// acc[mb][nb0 + nb] (nb = 0..3) is the wave's 128 x 64 block at rows rowbase.., cols colw..
template <int OUT_BF16, int FN, int DACT, int HAS_CT, int NBT>
EM_DEVICE void g_epilogue16(f32x4 (&acc)[8][NBT], int nb0, char* smem, int wave, int lane, int rowbase, int colw,
                            void* __restrict__ C, int64_t ldc, __bf16* __restrict__ CT, int64_t ldct,
                            const float* __restrict__ bias, const __bf16* __restrict__ mask, int64_t ldm, float alpha,
                            float beta, float* __restrict__ colpart, int N, uint32_t* __restrict__ bits) {
  constexpr int TS = 80;
  constexpr int YS = 144;
  constexpr int WEPI = 64 * TS + 32 * YS;
  char* tb = smem + wave * WEPI;
  char* yb = tb + 64 * TS;
  const int c16 = lane & 15, r4 = 4 * (lane >> 4);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};  // column sums of the epilogue values over the wave's 128 rows (colpart)
  constexpr bool WBITS = !DACT && FN == ACT_RELU && OUT_BF16;
  // a relu dgrad's activity words for all four 32-row blocks, loaded at once (one round trip instead of
  // one per block between the stores)
  uint32_t bpre[4][4];
  if (DACT && bits) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) bpre[i][nb] = bits[(int64_t)((rowbase >> 5) + i) * N + colw + 16 * nb + c16];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rowb = rowbase + 32 * i;
    uint32_t bw[4] = {0u, 0u, 0u, 0u};  // per 16-column group nb (see g_epilogue)
    if (DACT && bits) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) bw[nb] = bpre[i][nb];
    } else if (DACT) {
      const __bf16* ysrc = mask + (int64_t)rowb * ldm + colw;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int q = lane + 64 * t;
        const int row = q >> 3, ch = q & 7;
        *reinterpret_cast<u32x4*>(yb + row * YS + ch * 16) =
            *reinterpret_cast<const u32x4*>(ysrc + (int64_t)row * ldm + ch * 8);
      }
      wave_lds_sync();
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int lc = 16 * nb + c16;
      const float bv = (!DACT && bias) ? bias[colw + lc] : 0.f;
#pragma unroll
      for (int tm = 0; tm < 2; ++tm) {
        const f32x4& a = acc[2 * i + tm][nb0 + nb];
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lr = 16 * tm + r4 + e;
          float v = alpha * a[e];
          if (DACT) {
            v = bits ? bit_mul(bw[nb], lr, v) : v * g_dfn<FN>((float)*reinterpret_cast<const __bf16*>(yb + lr * YS + lc * 2));
          } else {
            v = g_fn<FN>(v + bv);
            if (WBITS) bw[nb] |= (v > 0.f ? 1u : 0u) << (16 * tm + e);
          }
          x[e] = v;
          cs[nb] += v;
          if (!OUT_BF16) {
            float* cp = reinterpret_cast<float*>(C) + (int64_t)(rowb + lr) * ldc + colw + lc;
            *cp = beta != 0.f ? v + beta * *cp : v;
          }
        }
        if (OUT_BF16) {
          u32x2 pk = {pack2(x[0], x[1]), pack2(x[2], x[3])};
          *reinterpret_cast<u32x2*>(tb + lc * TS + (16 * tm + r4) * 2) = pk;
        }
      }
    }
    if (WBITS && bits) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const uint32_t w = or_rows16(bw[nb] << r4);
        if (lane < 16) bits[(int64_t)(rowb >> 5) * N + colw + 16 * nb + c16] = w;
      }
    }
    if (OUT_BF16) {
      wave_lds_sync();
      const int gg = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int cb = 8 * (gg >> 1) + 16 * it;
        const int r0 = 16 * (gg & 1), row = r0 + i16;
        const s16x4 lo = lds_tr16(tb, (uint32_t)((cb + q4) * TS + (r0 + 4 * p4) * 2));
        const s16x4 hi = lds_tr16(tb, (uint32_t)((cb + 4 + q4) * TS + (r0 + 4 * p4) * 2));
        const bf16x8 v8 = cat_tr(lo, hi);
        if (G_CROW)  // row image [32 rows][128 B] in the (consumed) Y block, chunk c of a row at c ^ (row & 7)
          *reinterpret_cast<bf16x8*>(yb + row * 128 + (((cb >> 3) ^ (row & 7)) << 4)) = v8;
        else
          *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(C) + (int64_t)(rowb + row) * ldc + colw + cb) = v8;
      }
      if (G_CROW) {  // 8 lanes per 128-B row segment: each store covers 8 whole lines (as gemm_k64_kernel)
        wave_lds_sync();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = lane + 64 * k, row = q >> 3, ch = q & 7;
          *reinterpret_cast<u32x4*>(reinterpret_cast<__bf16*>(C) + (int64_t)(rowb + row) * ldc + colw + ch * 8) =
              *reinterpret_cast<const u32x4*>(yb + row * 128 + ((ch ^ (row & 7)) << 4));
        }
      }
      if (HAS_CT) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int q = lane + 64 * k;
          const int col = q >> 2, part = q & 3;
          *reinterpret_cast<u32x4*>(CT + (int64_t)(colw + col) * ldct + rowb + part * 8) =
              *reinterpret_cast<const u32x4*>(tb + col * TS + part * 16);
        }
      }
    }
    wave_lds_sync();
  }
  if (colpart) {  // bias gradient partials: the four 16-lane row groups hold the same columns
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      float t = cs[nb];
      t += __shfl_xor(t, 16);
      t += __shfl_xor(t, 32);
      if (lane < 16) colpart[(int64_t)(rowbase >> 7) * N + colw + 16 * nb + c16] = t;
    }
  }
}

// Diagnostic segment timers for the pp16 kernel (diagnostic build only: --define G_STAMPS=1; read
// with em_gemm_stamps / tools/gemm_stamps.py).  Per wave, s_memtime deltas summed over the main loop:
// [0] load segment: fragment reads + LDS-DMA issue (the stamp's lgkmcnt(0) also drains the reads)
// [1] load segment: counted vmcnt wait  [2] load segment: closing barrier
// [3] MFMA segment: lgkmcnt wait  [4] MFMA issue  [5] MFMA segment: closing barrier
// [6] prologue (kernel start -> loop)  [7] epilogue (loop end -> kernel end)
#ifndef G_STAMPS
#define G_STAMPS 0
#endif
#if G_STAMPS
constexpr int G_STAMP_BLOCKS = 4096;
__device__ uint64_t g_gstamps[G_STAMP_BLOCKS * 8 * 8];
#define G_MARK(t)                                                                 \
  do {                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");   \
    __builtin_amdgcn_sched_barrier(0);                                            \
  } while (0)
#else
#define G_MARK(t) (void)0
#endif

// The fragment reads are spread evenly over the four load segments of a K-tile (at most 8
// ds_read_b128 per wave instead of 12, 8, 4, 0): phase 3's segment reads the NEXT K-tile's A(qm 0)
// half into fa[0] (free during phase 3, which runs on fa[1] x B(qn 1)), so phase 0 reads only
// B(qn 0).  In phase 0 the loading group's 12 reads + the LDS-DMA unit filled the LDS array for the
// whole 256-cycle MFMA slot of the other group.  Hazards, with the unchanged staging schedule:
// A0 / A2 of K-tile kt+1 are issued in slots 8kt-2 / 8kt-1 (-10 / -9 relative to 8(kt+1)), so they are
// readable from 8kt+5 / 8kt+6 -- exactly the slots in which G0 / G1 read phase 3 of kt; their last read
// now sits 3 slots earlier than before, so the WAR distance to the restage only grows.
// AMN / BMN: operand MN-contiguous (see GPanel); 0 = K-contiguous
template <int OUT_BF16, int FN, int DACT, int HAS_CT, int AMN, int BMN>
__global__ void __launch_bounds__(G_NT, 1)
gemm256_pp16_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
                    void* __restrict__ C, int64_t ldc, __bf16* __restrict__ CT, int64_t ldct, int M, int N, int K,
                    const float* __restrict__ bias, const __bf16* __restrict__ mask, int64_t ldm, float alpha,
                    float beta, float* __restrict__ colpart, uint32_t* __restrict__ bits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t st_acc[8] = {}, st_t0 = 0, st_a = 0, st_b = 0;
  (void)st_acc;
  (void)st_t0;
  (void)st_a;
  (void)st_b;
  G_MARK(st_t0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_n = N / G_BN;
  const int nwg = (M / G_BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  int m0, n0;
  g_tile<HAS_CT>(bid, M / G_BM, tiles_n, m0, n0);
  const int ktiles = K / G_BK;
  const int nph = 4 * ktiles;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int wi = wave_s & 3;
  const bool g1 = wave_s >= 4;
  const GPanel pa = g_panel<AMN>(A, lda, m0, lane), pb = g_panel<BMN>(B, ldb, n0, lane);
  g_stage(pa, 0, smem, wave_s, AMN);
  g_stage(pb, 0, smem + G_TILE, wave_s, BMN);
  // (issuing every unit 2 slots ahead of its schedule with vmcnt(8) -- a staging "lead" -- measured
  // mixed, +-1.5 %, and was removed in round 5; docs/DESIGN.md §6)
  if (g1) {
    const bool a = pp_stage_slot<AMN, BMN>(pa, pb, smem, -4, ktiles, wi);
    const bool b = pp_stage_slot<AMN, BMN>(pa, pb, smem, -2, ktiles, wi);
    if (a && b) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (pp_stage_slot<AMN, BMN>(pa, pb, smem, -3, ktiles, wi)) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  // fragment registers: both A halves (qm) stay resident across their two quadrants, so a K-tile
  // reads A once and B once (24 ds_read_b128 per wave instead of 40): phase 0 reads A(qm 0) + B(qn 0),
  // phase 1 A(qm 1), phase 2 B(qn 1), phase 3 nothing.  Reads only move earlier than in the 32x32
  // schedule (first reads unchanged), so the staging slots' RAW / WAR analysis above still holds.
  bf16x8 fa[2][4][2], fb[2][2];
  auto load_seg = [&](int g, int slot) {
    if (g < nph) {
      const int kt = g >> 2, q = g & 3;
      const char* la = smem + (kt & 1) * 2 * G_TILE;
      const char* lb = la + G_TILE;
      if (q == 0 || q == 2) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fb[jj][ks] = g_frag<BMN>(lb, wn * 64 + (q >> 1) * 32 + 16 * jj, ks, lane);
      }
      const bool rd_a = q == 1 || (q == 0 && kt == 0) || (q == 3 && kt + 1 < ktiles);
      if (rd_a) {
        const int qa = q & 1;  // q == 3 reads qm 0 of the next K-tile
        const char* lsrc = q == 3 ? smem + ((kt + 1) & 1) * 2 * G_TILE : la;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fa[qa ^ (q == 3)][ii][ks] = g_frag<AMN>(lsrc, wm * 128 + (qa ^ (q == 3)) * 64 + 16 * ii, ks, lane);
      }
    }
    const bool staged = pp_stage_slot<AMN, BMN>(pa, pb, smem, slot, ktiles, wi);
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[0] += t - st_a;
      st_a = t;
    }
    if (!staged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[1] += t - st_a;
      st_a = t;
    }
    __builtin_amdgcn_s_barrier();
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[2] += t - st_a;
      st_a = t;
    }
  };
  auto mfma_seg = [&](int q) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[3] += t - st_a;
      st_a = t;
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x4& c = acc[4 * (q & 1) + ii][2 * (q >> 1) + jj];
          c = mfma16(fa[q & 1][ii][ks], fb[jj][ks], c);
        }
    __builtin_amdgcn_s_setprio(0);
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[4] += t - st_a;
      st_a = t;
    }
    __builtin_amdgcn_s_barrier();
    if (G_STAMPS) {
      uint64_t t;
      G_MARK(t);
      st_acc[5] += t - st_a;
      st_a = t;
    }
  };
  if (G_STAMPS) {
    G_MARK(st_a);
    st_acc[6] = st_a - st_t0;
  }

  if (!g1) {
    load_seg(0, -1);
    for (int kt = 0; kt < ktiles; ++kt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int g = 4 * kt + q;
        mfma_seg(q);
        load_seg(g + 1, 2 * g + 1);
      }
    }
  } else {
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < ktiles; ++kt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int g = 4 * kt + q;
        load_seg(g, 2 * g);
        mfma_seg(q);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (G_STAMPS) G_MARK(st_b);
  g_epilogue16<OUT_BF16, FN, DACT, HAS_CT, 4>(acc, 0, smem, wave, lane, m0 + wm * 128, n0 + wn * 64, C, ldc, CT,
                                              ldct, bias, mask, ldm, alpha, beta, colpart, N, bits);
#if G_STAMPS
  {
    uint64_t t;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    G_MARK(t);
    st_acc[7] = t - st_b;
    if (lane == 0 && blockIdx.x < G_STAMP_BLOCKS)
      for (int k = 0; k < 8; ++k) g_gstamps[((size_t)blockIdx.x * 8 + wave) * 8 + k] = st_acc[k];
  }
#endif
}

template <int OUT_BF16, int FN, int DACT, int HAS_CT, int AMN = 0, int BMN = 0>
int g_launch(dim3 grid, hipStream_t st, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, void* C,
             int64_t ldc, __bf16* CT, int64_t ldct, int M, int N, int K, const float* bias, const __bf16* mask,
             int64_t ldm, float alpha, float beta, float* colpart, uint32_t* bits) {
  // (the 32x32x16 ping-pong kernel, the non-ping-pong 256 kernel and the unbalanced fragment-read
  // schedule were measured slower and removed in round 5; docs/DESIGN.md §2 and §6 keep their numbers)
  static bool attr = false;
  auto kern = gemm256_pp16_kernel<OUT_BF16, FN, DACT, HAS_CT, AMN, BMN>;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, G_LDS);
    attr = true;
  }
  hipLaunchKernelGGL(kern, grid, dim3(G_NT), G_LDS, st, A, lda, B, ldb, C, ldc, CT, ldct, M, N, K, bias, mask, ldm,
                     alpha, beta, colpart, bits);
  return 0;
}

// runtime (layout, out, act/dact, ct) -> one of 20 instantiations.  Layouts besides NT (a_kc = b_kc = 1):
// wgrad dW = dZ^T X from the natural [batch][features] tensors (both operands MN: fp32 out, no
// activation) and dgrad (dZ W) * act' from the natural weight (B MN: bf16 out, act' or none, no C^T).
// Whether a layout is taken is decided by g_layout_ok.
int g_dispatch(dim3 grid, hipStream_t st, int a_kc, int b_kc, const __bf16* A, int64_t lda, const __bf16* B,
               int64_t ldb, void* C, int64_t ldc, int c_bf16, __bf16* CT, int64_t ldct, int M, int N, int K,
               const float* bias, int act, const __bf16* mask, int64_t ldm, int dact, float alpha, float beta,
               float* colpart, uint32_t* bits) {
#define EM_GL(OB, FN, DA, CTV, AM, BM)                                                                              \
  return g_launch<OB, FN, DA, CTV, AM, BM>(grid, st, A, lda, B, ldb, C, ldc, CT, ldct, M, N, K, bias, mask, ldm, alpha, \
                                           beta, colpart, bits)
#define EM_G(OB, FN, DA, CTV) EM_GL(OB, FN, DA, CTV, 0, 0)
  if (!a_kc && !b_kc) {
    if (c_bf16 || act != ACT_NONE || mask || dact || CT || bits) return EM_ERR_ARG;
    EM_GL(0, ACT_NONE, 0, 0, 1, 1);
  }
  if (!b_kc) {
    if (!a_kc || !c_bf16 || act != ACT_NONE || CT) return EM_ERR_ARG;
    switch (dact) {
      case 0: EM_GL(1, ACT_NONE, 0, 0, 0, 1);
      case ACT_RELU: EM_GL(1, ACT_RELU, 1, 0, 0, 1);
      case ACT_SIGMOID: EM_GL(1, ACT_SIGMOID, 1, 0, 0, 1);
      case ACT_TANH: EM_GL(1, ACT_TANH, 1, 0, 0, 1);
      default: return EM_ERR_ARG;
    }
  }
  if (!a_kc) return EM_ERR_ARG;
  if (!c_bf16) {
    if (act != ACT_NONE || mask || dact || CT || bits) return EM_ERR_ARG;
    EM_G(0, ACT_NONE, 0, 0);
  }
  const bool ct = CT != nullptr;
  if (mask || dact) {
    if (act != ACT_NONE) return EM_ERR_ARG;
    switch (dact) {
      case ACT_RELU: if (ct) EM_G(1, ACT_RELU, 1, 1); else EM_G(1, ACT_RELU, 1, 0);
      case ACT_SIGMOID: if (ct) EM_G(1, ACT_SIGMOID, 1, 1); else EM_G(1, ACT_SIGMOID, 1, 0);
      case ACT_TANH: if (ct) EM_G(1, ACT_TANH, 1, 1); else EM_G(1, ACT_TANH, 1, 0);
      default: return EM_ERR_ARG;
    }
  }
  switch (act) {
    case ACT_NONE: if (ct) EM_G(1, ACT_NONE, 0, 1); else EM_G(1, ACT_NONE, 0, 0);
    case ACT_RELU: if (ct) EM_G(1, ACT_RELU, 0, 1); else EM_G(1, ACT_RELU, 0, 0);
    case ACT_SIGMOID: if (ct) EM_G(1, ACT_SIGMOID, 0, 1); else EM_G(1, ACT_SIGMOID, 0, 0);
    case ACT_TANH: if (ct) EM_G(1, ACT_TANH, 0, 1); else EM_G(1, ACT_TANH, 0, 0);
    default: return EM_ERR_ARG;
  }
#undef EM_G
#undef EM_GL
}

// The 256-tile kernel's layouts (see g_dispatch); MN operands need 32-bit buffer offsets over all of K
bool g_layout_ok(int a_kc, int b_kc, int c_bf16, int act, const void* mask, int dact, const void* ct,
                 const void* bits, int64_t lda, int64_t ldb, int K) {
  if (a_kc && b_kc) return true;
  if ((!a_kc && (int64_t)K * lda * 2 >= (1ll << 31)) || (!b_kc && (int64_t)K * ldb * 2 >= (1ll << 31))) return false;
  if (!a_kc && !b_kc) return !c_bf16 && act == ACT_NONE && !mask && !dact && !ct && !bits;
  if (!b_kc) return c_bf16 && act == ACT_NONE && !ct;
  return false;
}

// bf16 transpose: dst[c][r] = src[r][c]; 64x64 tiles through LDS, 16-B global accesses
__global__ void __launch_bounds__(256) transpose_kernel(const __bf16* __restrict__ src, int64_t lds_, int R, int Cc,
                                                        __bf16* __restrict__ dst, int64_t ldd) {
  __shared__ __bf16 tile[64][72];
  const int tiles_c = (Cc + 63) / 64;
  const int r0 = (blockIdx.x / tiles_c) * 64, c0 = (blockIdx.x % tiles_c) * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + it * 256;  // 512 chunks of 8 elements
    const int rr = q >> 3, cc = (q & 7) * 8;
    const int gr = r0 + rr, gc = c0 + cc;
    if (gr < R && gc + 8 <= Cc) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(src + (int64_t)gr * lds_ + gc);
      const __bf16* e = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[rr][cc + k] = e[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[rr][cc + k] = (gr < R && gc + k < Cc) ? src[(int64_t)gr * lds_ + gc + k] : (__bf16)0.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = tid + it * 256;
    const int cc = q >> 3, rr = (q & 7) * 8;  // output row = source col
    const int gc = c0 + cc, gr = r0 + rr;
    if (gc >= Cc) continue;
    __bf16 e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = tile[rr + k][cc];
    if (gr + 8 <= R) {
      *reinterpret_cast<u32x4*>(dst + (int64_t)gc * ldd + gr) = *reinterpret_cast<const u32x4*>(e);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (gr + k < R) dst[(int64_t)gc * ldd + gr + k] = e[k];
    }
  }
}

// ============================================================================================
// Skinny-K GEMM (K = 64 or 128): the wide MLP's first-layer forward (X[B,64] W0ᵀ) and last-layer
// dgrad (dZ[B,64] W2) write a [B, 8192] bf16 output plus its transposed copy, with almost no
// arithmetic (2 GB written per 8 MFLOP-ish tile work).  On the 256-tile ping-pong kernel (1 block /
// CU, 226 VGPRs, epilogue serialized per wave) they ran at 2.9-3.4 TB/s.  This kernel is built for
// the store stream instead: 128 x 128 tiles, 4 waves (2 x 2, 64 x 64 each, 16 MFMAs), <= 128 VGPRs
// and 36 KB of LDS (68 KB with a staged act' mask) so 4 workgroups share a CU and hide each other's
// epilogue latencies.
//   * the whole K of the tile is staged once (register staging, XOR-swizzled [128][64] images);
//   * epilogue per wave: act'(mask) via ds_read_b64_tr_b16 of a staged 64 x 64 mask block (4 rows of
//     one column per read = the accumulator layout), bf16 values into a [col][row] image T, then C
//     rows (128 B per row: two transposed reads per 16 B) and C^T rows (128 B straight from T);
//   * optional column sums (fused bias gradient, same [M / 128][N] partial format as the 256 path).
constexpr int K64_BM = 128, K64_BN = 128, K64_NT = 256;
constexpr int K64_TS = 144;                          // bytes per T row: 64 bf16 + 16 pad
constexpr int K64_WEPI = 64 * K64_TS;                // 9216 B per wave
constexpr int K64_LDS = 4 * K64_WEPI + 4 * 8 * 1024;  // T images + staged 64 x 64 mask blocks (8 KB / wave)
static_assert(K64_LDS >= 2 * K64_BM * 64 * 2 && 4 * K64_WEPI >= 2 * K64_BM * 64 * 2, "operand tiles must fit");

// The C rows go out row-contiguous: the transposed reads of T (held in 32 VGPRs) become a row image built in
// place of T once T's reads and the C^T stores are issued, and 8 lanes store one 128-B row segment (a store
// instruction covers 8 whole lines instead of 16 B of 64 lines).  Without a staged act' mask a block then needs
// 36 KB of LDS: 4 workgroups per CU to overlap each other's load and epilogue phases (round 5; the row image
// in a separate 8 KB-per-wave block, 68 KB and 2 workgroups per CU, measured 16-21 % slower:
// profiles/r5/k64_inplace_rowimage_ab.txt; the direct 16-B-per-line form slower still, docs/DESIGN.md §6).
constexpr int K64_LDS_SLIM = 4 * K64_WEPI;
template <int FN, int DACT, int HAS_CT>
__global__ void __launch_bounds__(K64_NT, 4)
gemm_k64_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B, int64_t ldb,
                __bf16* __restrict__ C, int64_t ldc, __bf16* __restrict__ CT, int64_t ldct, int M, int N, int K,
                const float* __restrict__ bias, const __bf16* __restrict__ mask, int64_t ldm, float alpha,
                float* __restrict__ colpart, uint32_t* __restrict__ bits) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / K64_BN;
  const int bid = xcd_remap(blockIdx.x, (M / K64_BM) * tiles_n);
  const int m0 = (bid / tiles_n) * K64_BM, n0 = (bid % tiles_n) * K64_BN;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  // the dgrad's ReLU activity words are loaded before the operands: with K = 64 the MFMA phase is one
  // K tile, and loaded at the epilogue their round trip sat between the MFMAs and the stores (dgrad
  // 615 -> 559 us on the wide MLP)
  uint32_t bw[2][2] = {{0u, 0u}, {0u, 0u}};  // ReLU activity words [32-row block i][column half j] (g_epilogue)
  auto load_bits = [&]() {
    const int rb = m0 + wm * 64, cw = n0 + wn * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) bw[i][j] = bits[(int64_t)((rb >> 5) + i) * N + cw + 32 * j + r];
  };
  if (DACT && bits) load_bits();
  for (int k0 = 0; k0 < K; k0 += 64) {
    u32x4 rs[4];  // one staging set for both operands (keeps the kernel at <= 128 VGPRs, 4 blocks / CU)
    if (k0) __syncthreads();  // the previous K tile's fragments are read
    load_tile<1>(A, lda, m0, k0, M, K, tid, rs);
    store_tile<1>(smem, tid, rs);
    load_tile<1>(B, ldb, n0, k0, N, K, tid, rs);
    store_tile<1>(smem + K64_BM * 128, tid, rs);
    __syncthreads();
    const char* la = smem;
    const char* lb = smem + K64_BM * 128;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 a0 = frag<1>(la, wm * 64 + r, s, lane), a1 = frag<1>(la, wm * 64 + 32 + r, s, lane);
      const bf16x8 b0 = frag<1>(lb, wn * 64 + r, s, lane), b1 = frag<1>(lb, wn * 64 + 32 + r, s, lane);
      acc[0][0] = mfma32(a0, b0, acc[0][0]);
      acc[0][1] = mfma32(a0, b1, acc[0][1]);
      acc[1][0] = mfma32(a1, b0, acc[1][0]);
      acc[1][1] = mfma32(a1, b1, acc[1][1]);
    }
  }
  __syncthreads();  // operand tiles dead: the LDS becomes the epilogue images

  char* tb = smem + wave * K64_WEPI;
  char* yb = smem + 4 * K64_WEPI + wave * 8192;  // [64 rows][64 cols] bf16, 128-B rows, 16-B chunk ^= row & 7
  const int rowb = m0 + wm * 64, colw = n0 + wn * 64;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, gq = lane >> 4;
  constexpr bool WBITS = !DACT && FN == ACT_RELU;
  if (DACT && !bits) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {  // 512 chunks of 16 B: rows q >> 3, chunk q & 7
      const int q = lane + 64 * t, row = q >> 3, ch = q & 7;
      *reinterpret_cast<u32x4*>(yb + row * 128 + ((ch ^ (row & 7)) << 4)) =
          *reinterpret_cast<const u32x4*>(mask + (int64_t)(rowb + row) * ldm + colw + ch * 8);
    }
    wave_lds_sync();
  }
  float cs[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int lc = 32 * j + r;
    const float bv = (!DACT && bias) ? bias[colw + lc] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int lr = 32 * i + 8 * g + 4 * h;  // the lane's 4 consecutive rows lr .. lr + 3, column lc
        float y[4] = {0.f, 0.f, 0.f, 0.f};
        if (DACT && !bits) {  // transposed read: lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3
          const int rr = 32 * i + 8 * g + 4 * (gq >> 1) + q4, cc = 32 * j + 16 * (gq & 1) + 4 * p4;
          const s16x4 m4 = lds_tr16(yb, (uint32_t)(rr * 128 + (((cc >> 3) ^ (rr & 7)) << 4) + (cc & 7) * 2));
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = bf16_bits_to_f32((uint16_t)m4[e]);
        }
        float x[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = alpha * acc[i][j][4 * g + e];
          if (DACT) {
            v = bits ? bit_mul(bw[i][j], 8 * g + 4 * h + e, v) : v * g_dfn<FN>(y[e]);
          } else {
            v = g_fn<FN>(v + bv);
            if (WBITS) bw[i][j] |= (v > 0.f ? 1u : 0u) << (8 * g + e);
          }
          x[e] = v;
          cs[j] += v;
        }
        *reinterpret_cast<u32x2*>(tb + lc * K64_TS + lr * 2) = u32x2{pack2(x[0], x[1]), pack2(x[2], x[3])};
      }
  }
  if (WBITS && bits) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t w = or_xhalf(bw[i][j] << (4 * h));
        if (h == 0) bits[(int64_t)((rowb >> 5) + i) * N + colw + 32 * j + r] = w;
      }
  }
  wave_lds_sync();
  {
    bf16x8 rv[8];  // C rows: per iteration a 16-lane group reads 16 rows x 8 columns (one 16-B piece per lane)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int cb = 8 * it, r0 = 16 * gq;
      rv[it] = cat_tr(lds_tr16(tb, (uint32_t)((cb + q4) * K64_TS + (r0 + 4 * p4) * 2)),
                      lds_tr16(tb, (uint32_t)((cb + 4 + q4) * K64_TS + (r0 + 4 * p4) * 2)));
    }
    if (HAS_CT) {  // C^T row = one column of the block: 64 rows = 128 B straight from T (before T is reused)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = lane + 64 * k, col = q >> 3, part = q & 7;
        *reinterpret_cast<u32x4*>(CT + (int64_t)(colw + col) * ldct + rowb + part * 8) =
            *reinterpret_cast<const u32x4*>(tb + col * K64_TS + part * 16);
      }
    }
    wave_lds_sync();  // T consumed: the row image [64 rows][128 B] (8 KB of T's 9 KB) takes its place
    const int row = 16 * gq + i16;
#pragma unroll
    for (int it = 0; it < 8; ++it) *reinterpret_cast<bf16x8*>(tb + row * 128 + ((it ^ (row & 7)) << 4)) = rv[it];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = lane + 64 * k, rr = q >> 3, ch = q & 7;
      *reinterpret_cast<u32x4*>(C + (int64_t)(rowb + rr) * ldc + colw + ch * 8) =
          *reinterpret_cast<const u32x4*>(tb + rr * 128 + ((ch ^ (rr & 7)) << 4));
    }
  }
  if (colpart) {  // bias-gradient partials, row (m0 >> 7) of [M / 128][N]: the two wm waves add via LDS
#pragma unroll
    for (int j = 0; j < 2; ++j) cs[j] = xhalf_sum(cs[j]);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [2 wn][64 cols] of the wm = 1 waves
    if (wm == 1 && h == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) red[wn * 64 + 32 * j + r] = cs[j];
    }
    __syncthreads();
    if (wm == 0 && h == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        colpart[(int64_t)(m0 >> 7) * N + colw + 32 * j + r] = cs[j] + red[wn * 64 + 32 * j + r];
    }
  }
}

template <int FN, int DACT, int HAS_CT>
int k64_launch(hipStream_t st, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, __bf16* C, int64_t ldc,
               __bf16* CT, int64_t ldct, int M, int N, int K, const float* bias, const __bf16* mask, int64_t ldm,
               float alpha, float* colpart, uint32_t* bits) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_k64_kernel<FN, DACT, HAS_CT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, K64_LDS);
    attr = true;
  }
  const int lds = (DACT && !bits) ? K64_LDS : K64_LDS_SLIM;  // (the staged act' mask needs its 32 KB)
  hipLaunchKernelGGL((gemm_k64_kernel<FN, DACT, HAS_CT>), dim3((M / K64_BM) * (N / K64_BN)), dim3(K64_NT), lds, st,
                     A, lda, B, ldb, C, ldc, CT, ldct, M, N, K, bias, mask, ldm, alpha, colpart, bits);
  return 0;
}

// runtime (act / dact, ct) -> instantiation; bf16 output only
int k64_dispatch(hipStream_t st, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, __bf16* C, int64_t ldc,
                 __bf16* CT, int64_t ldct, int M, int N, int K, const float* bias, int act, const __bf16* mask,
                 int64_t ldm, int dact, float alpha, float* colpart, uint32_t* bits) {
#define EM_K(FN, DA, CTV) \
  return k64_launch<FN, DA, CTV>(st, A, lda, B, ldb, C, ldc, CT, ldct, M, N, K, bias, mask, ldm, alpha, colpart, bits)
  const bool ct = CT != nullptr;
  if (mask || dact) {
    if (act != ACT_NONE) return EM_ERR_ARG;
    switch (dact) {
      case ACT_RELU: if (ct) EM_K(ACT_RELU, 1, 1); else EM_K(ACT_RELU, 1, 0);
      case ACT_SIGMOID: if (ct) EM_K(ACT_SIGMOID, 1, 1); else EM_K(ACT_SIGMOID, 1, 0);
      case ACT_TANH: if (ct) EM_K(ACT_TANH, 1, 1); else EM_K(ACT_TANH, 1, 0);
      default: return EM_ERR_ARG;
    }
  }
  switch (act) {
    case ACT_NONE: if (ct) EM_K(ACT_NONE, 0, 1); else EM_K(ACT_NONE, 0, 0);
    case ACT_RELU: if (ct) EM_K(ACT_RELU, 0, 1); else EM_K(ACT_RELU, 0, 0);
    case ACT_SIGMOID: if (ct) EM_K(ACT_SIGMOID, 0, 1); else EM_K(ACT_SIGMOID, 0, 0);
    case ACT_TANH: if (ct) EM_K(ACT_TANH, 0, 1); else EM_K(ACT_TANH, 0, 0);
    default: return EM_ERR_ARG;
  }
#undef EM_K
}

// column sums of a bf16 [M][N] matrix (bias gradients), deterministic two-pass:
// pass 1: block (column group of 512, row chunk of CS_ROWS) -> fp32 partial [chunk][N]
// pass 2: fixed-order sum over chunks (+ optional accumulate / scale)
constexpr int CS_ROWS = 512;
__global__ void __launch_bounds__(256) colsum_partial_kernel(const __bf16* __restrict__ X, int64_t ldx, int M, int N,
                                                             float* __restrict__ part) {
  __shared__ float red[4][512];
  const int cg = threadIdx.x & 63, rp = threadIdx.x >> 6;  // 64 column groups of 8 x 4 row phases
  const int c0 = blockIdx.x * 512 + cg * 8;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(M, r0 + CS_ROWS);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 + 8 <= N) {
    for (int rr = r0 + rp; rr < r1; rr += 4) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(X + (int64_t)rr * ldx + c0);
      const __bf16* e = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += (float)e[k];
    }
  } else if (c0 < N) {
    for (int rr = r0 + rp; rr < r1; rr += 4)
      for (int k = 0; k < 8 && c0 + k < N; ++k) acc[k] += (float)X[(int64_t)rr * ldx + c0 + k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rp][cg * 8 + k] = acc[k];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int col = blockIdx.x * 512 + c;
    if (col < N) part[(int64_t)blockIdx.y * N + col] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  }
}

// Fixed-order sum of fp32 partial rows [chunks][N] -> out[N] (+ accumulate, * scale): 64 columns x 16
// chunk groups per 1024-thread block; group g sums chunks g, g + 16, ... with 8 loads in flight, then
// the 16 group sums are added in group order (bit-reproducible, and one round of loads deep instead
// of a serial walk over the chunks).  Used for the colsum partials and for the GEMM epilogue's fused
// bias-gradient partials (em_gemm_bf16_cs).
constexpr int CR_COLS = 64, CR_G = 16;
__global__ void __launch_bounds__(CR_COLS * CR_G) colsum_final_kernel(const float* __restrict__ part, int chunks, int N,
                                                                      float* __restrict__ out, int accumulate,
                                                                      float scale) {
  __shared__ float red[CR_G][CR_COLS];
  const int c = threadIdx.x % CR_COLS, g = threadIdx.x / CR_COLS;
  const int col = blockIdx.x * CR_COLS + c;
  float s = 0.f;
  if (col < N) {
    int k = g;
    for (; k + 7 * CR_G < chunks; k += 8 * CR_G) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(k + u * CR_G) * N + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < chunks; k += CR_G) s += part[(int64_t)k * N + col];
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    float t = red[0][c];
#pragma unroll
    for (int q = 1; q < CR_G; ++q) t += red[q][c];
    t *= scale;
    out[col] = accumulate ? out[col] + t : t;
  }
}

// row sums of a bf16 [R][C] matrix (bias gradients from a transposed dZ copy): one wavefront per row
__global__ void __launch_bounds__(256) rowsum_kernel(const __bf16* __restrict__ X, int64_t ldx, int R, int Cc,
                                                     float* __restrict__ out, int accumulate, float scale) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const __bf16* xr = X + (int64_t)row * ldx;
  float s = 0.f;
  int c = lane * 8;
  for (; c + 8 <= Cc; c += 512) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(xr + c);
    const __bf16* e = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += (float)e[k];
  }
  for (int k = c; k < Cc && k < c + 8; ++k) s += (float)xr[k];
  s = wave_sum(s) * scale;
  if (lane == 0) out[row] = accumulate ? out[row] + s : s;
}

// ============================================================================================
// Skinny weight gradient: C = alpha * P^T Q (+ beta C) with P [K][J <= 64] and Q [K][W] both
// row-major over the batch K (the wide MLP's first and last layers: 64 x 8192 over 65536 rows).
// The 128x128 any-layout kernel wastes half its MFMAs on the 64-wide side and hides its global
// latency poorly; this path reads the W-wide operand exactly once, streaming it through a 3-stage
// buffer_load...lds ring.  Block = (256-column tile of Q, K-slice); 4 waves, each a 64 x 64 output
// (2 x 2 MFMA 32x32x16 tiles); fragments via ds_read_b64_tr_b16 from [64 k][128 col] images
// (frag<0>, the MC layout of the any-layout kernel).  Each K-slice writes an fp32 partial; a
// fixed-order reduce sums the slices (deterministic) and writes C or C^T.
constexpr int SK_WT = 256, SK_STAGES = 3;
constexpr int SK_IMG = 64 * 256;             // one [64 k][128 col] bf16 image, 16 KB
constexpr int SK_STAGE = 3 * SK_IMG;         // P image (64 of its 128 columns used) + 2 Q images
constexpr int SK_LDS = SK_STAGES * SK_STAGE;  // 144 KB

struct SkPanel {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff[4];
  uint32_t row_bytes;
};
// one buffer_load...lds writes 1 KB = 4 image rows lane-linearly (row 4g + (L >> 4), physical
// 16-B chunk L & 15); the mc_off swizzle (chunk ^ (k & 15)) is applied to the source chunk, so
// the per-lane offset depends on g mod 4
EM_DEVICE SkPanel sk_panel(const __bf16* base, int64_t ld, int64_t bytes, int lane) {
  SkPanel p;
  p.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(bytes < 0x7FFFFFFF ? bytes : 0x7FFFFFFF),
                                             0x00020000);
  const int lr = lane >> 4, pc = lane & 15;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int c = pc ^ ((4 * g4 + lr) & 15);
    p.voff[g4] = (uint32_t)((lr * ld + 8 * c) * 2);
  }
  p.row_bytes = (uint32_t)(ld * 2);
  return p;
}
// this wave's 4 of the image's 16 row groups; k0 relative to the panel base, col0 in elements
EM_DEVICE void sk_stage_img(const SkPanel& p, int k0, int col0, char* img, int wave) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = wave * 4 + i;
    const uint32_t soff = (uint32_t)(k0 + 4 * g) * p.row_bytes + (uint32_t)col0 * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(p.rsrc, (EM_LDS void*)(img + g * 1024), 16, p.voff[g & 3], soff, 0, 0);
  }
}

__global__ void __launch_bounds__(256, 1)
wgrad_skinny_kernel(const __bf16* __restrict__ P, int64_t ldp, const __bf16* __restrict__ Q, int64_t ldq, int K,
                    int W, int kstep, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w0 = blockIdx.x * SK_WT, s = blockIdx.y;
  const int kb = s * kstep, ke = min(K, kb + kstep);
  const int T = (ke - kb) / 64;
  const SkPanel pp = sk_panel(P + (int64_t)kb * ldp, ldp, ((int64_t)(K - kb) * ldp) * 2, lane);
  const SkPanel pq = sk_panel(Q + (int64_t)kb * ldq + w0, ldq, ((int64_t)(K - kb) * ldq - w0) * 2, lane);
  auto stage = [&](int t) {
    char* st = smem + (t % SK_STAGES) * SK_STAGE;
    sk_stage_img(pp, t * 64, 0, st, wave);
    sk_stage_img(pq, t * 64, 0, st + SK_IMG, wave);
    sk_stage_img(pq, t * 64, 128, st + 2 * SK_IMG, wave);
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  if (T > 0) stage(0);
  if (T > 1) {
    stage(1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // tile 0 landed, tile 1 in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const int r = lane & 31;
  const int qimg = SK_IMG * (1 + (wave >> 1)), qc = (wave & 1) * 64;
  for (int t = 0; t < T; ++t) {
    // the slot of tile t-1 is free: every wave consumed its fragments before the last barrier
    if (t + 2 < T) stage(t + 2);
    const char* st = smem + (t % SK_STAGES) * SK_STAGE;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 a0 = frag<0>(st, r, ks, lane), a1 = frag<0>(st, 32 + r, ks, lane);
      const bf16x8 b0 = frag<0>(st + qimg, qc + r, ks, lane), b1 = frag<0>(st + qimg, qc + 32 + r, ks, lane);
      acc[0][0] = mfma32(a0, b0, acc[0][0]);
      acc[0][1] = mfma32(a0, b1, acc[0][1]);
      acc[1][0] = mfma32(a1, b0, acc[1][0]);
      acc[1][1] = mfma32(a1, b1, acc[1][1]);
    }
    if (t + 2 < T) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");  // tile t+1 landed
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // fp32 partial of this K-slice: part[s][j][w] (j = P column 0..63)
  const int h = lane >> 5;
  float* ps = part + (int64_t)s * 64 * W;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int wt = 0; wt < 2; ++wt)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int j = 32 * jt + (v & 3) + 8 * (v >> 2) + 4 * h;
        const int w = w0 + (wave >> 1) * 128 + qc + 32 * wt + r;
        ps[(int64_t)j * W + w] = acc[jt][wt][v];
      }
}

// fixed-order sum over the K-slices; C [J][W] (trans = 0) or C^T [W][J] (trans = 1)
__global__ void __launch_bounds__(256)
wgrad_skinny_reduce_kernel(const float* __restrict__ part, int S, int J, int W, float* __restrict__ C, int64_t ldc,
                           int trans, float alpha, float beta) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)J * W) return;
  const int j = (int)(e / W), w = (int)(e - (int64_t)j * W);
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += part[((int64_t)s * 64 + j) * W + w];
  acc *= alpha;
  float* o = trans ? C + (int64_t)w * ldc + j : C + (int64_t)j * ldc + w;
  *o = beta != 0.f ? acc + beta * *o : acc;
}

}  // namespace

static int gemm_impl(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                     int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                     int64_t ldm, int dact, float alpha, float beta, void* ct, int64_t ldct, int splits, int kstep,
                     int64_t c_split, hipStream_t stream, float* colpart = nullptr, uint32_t* bits = nullptr);

EM_API int em_gemm_bf16(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                        int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                        int64_t ldm, int dact, float alpha, float beta, void* ct, int64_t ldct, hipStream_t stream) {
  return gemm_impl(A, lda, a_kc, B, ldb, b_kc, C, ldc, c_bf16, M, N, K, bias, act, mask, ldm, dact, alpha, beta, ct,
                   ldct, 1, K, 0, stream);
}

// The same GEMM on the 256-tile path with the epilogue's column sums (K3 bias gradient, fused): colpart
// receives fp32 [M / 128][N] partials -- row p = sum over output rows 128p .. 128p + 127 of the final
// epilogue values (after act' for dgrad), before the bf16 rounding.  em_colpart_reduce sums them.
EM_API int em_gemm_bf16_cs(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                           int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                           int64_t ldm, int dact, float alpha, float beta, void* ct, int64_t ldct, float* colpart,
                           hipStream_t stream) {
  if (!colpart || ((uintptr_t)colpart & 3)) return EM_ERR_ARG;
  return gemm_impl(A, lda, a_kc, B, ldb, b_kc, C, ldc, c_bf16, M, N, K, bias, act, mask, ldm, dact, alpha, beta, ct,
                   ldct, 1, K, 0, stream, colpart);
}

// The general form: optional column partials (as em_gemm_bf16_cs) and ReLU activity bits (uint32
// [M / 32][N], bit m & 31 of word (m >> 5) * N + n = output[m][n] > 0): written when act is relu,
// read in place of the saved activation when dact is relu and mask is null (64x less traffic than
// the bf16 activation).
EM_API int em_gemm_bf16_ex(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                           int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                           int64_t ldm, int dact, float alpha, float beta, void* ct, int64_t ldct, float* colpart,
                           uint32_t* bits, hipStream_t stream) {
  if ((uintptr_t)colpart & 3) return EM_ERR_ARG;
  return gemm_impl(A, lda, a_kc, B, ldb, b_kc, C, ldc, c_bf16, M, N, K, bias, act, mask, ldm, dact, alpha, beta, ct,
                   ldct, 1, K, 0, stream, colpart, bits);
}

// Split-K on the any-layout kernel: `splits` slices of `kstep` (multiple of 64) along K, slice s writing
// C + s * c_split (elements).  For small outputs with a huge reduction (64 x 8192 over a 64k batch).
EM_API int em_gemm_bf16_splitk(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                               int64_t ldc, int c_bf16, int M, int N, int K, float alpha, int splits, int kstep,
                               int64_t c_split, hipStream_t stream) {
  if (splits < 1 || splits > 65535 || kstep <= 0 || (kstep & 63) || (int64_t)splits * kstep < K || c_split < 0)
    return EM_ERR_ARG;
  return gemm_impl(A, lda, a_kc, B, ldb, b_kc, C, ldc, c_bf16, M, N, K, nullptr, 0, nullptr, 0, 0, alpha, 0.f,
                   nullptr, 0, splits, kstep, c_split, stream);
}

static int gemm_impl(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                     int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                     int64_t ldm, int dact, float alpha, float beta, void* ct, int64_t ldct, int splits, int kstep,
                     int64_t c_split, hipStream_t stream, float* colpart, uint32_t* bits) {
  if (!A || !B || !C || M < 0 || N < 0 || K < 0 || act < 0 || act > 3) return EM_ERR_ARG;
  if (mask && (dact < 1 || dact > 3)) return EM_ERR_ARG;
  // ReLU activity bits (see relu_bits_*): written by a bf16 forward with act relu, read instead of the
  // saved activation by a relu dgrad; 256-tile / skinny-K paths only, M a multiple of 32
  if (bits) {
    const bool wr = act == ACT_RELU && !mask && dact == 0, rd = act == ACT_NONE && !mask && dact == ACT_RELU;
    if (!(wr || rd) || !c_bf16 || (M & 31) || ((uintptr_t)bits & 3)) return EM_ERR_ARG;
  } else if (dact && !mask) {
    return EM_ERR_ARG;
  }
  if (M == 0 || N == 0) return 0;
  // 16-byte vector loads need 8-element-aligned leading dimensions and base pointers
  if ((lda & 7) || (ldb & 7) || (((uintptr_t)A) & 15) || (((uintptr_t)B) & 15)) return EM_ERR_ARG;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr = true;
  }
  const bool big = splits == 1 && (M % G_BM) == 0 && (N % G_BN) == 0 && (K % G_BK) == 0 && K > 0 &&
                   (((uintptr_t)A | (uintptr_t)B) & 15) == 0 &&
                   (c_bf16 || (act == ACT_NONE && !mask)) &&  // fp32 + act / act' epilogues: any-layout kernel
                   g_layout_ok(a_kc, b_kc, c_bf16, act, mask, dact, ct, bits, lda, ldb, K);
  // skinny K (64 / 128) with a bf16 output: the store-stream kernel (see gemm_k64_kernel)
  if (big && a_kc && b_kc && c_bf16 && (K == 64 || K == 128) && beta == 0.f) {
    const int rc = k64_dispatch(stream, (const __bf16*)A, lda, (const __bf16*)B, ldb, (__bf16*)C, ldc, (__bf16*)ct,
                                ldct, M, N, K, bias, act, (const __bf16*)mask, ldm, dact, alpha, colpart, bits);
    if (rc) return rc;
    EM_CHECK_LAUNCH();
    return 0;
  }
  if (big) {
    const int rc = g_dispatch(dim3((M / G_BM) * (N / G_BN)), stream, a_kc, b_kc, (const __bf16*)A, lda,
                              (const __bf16*)B, ldb, C, ldc, c_bf16, (__bf16*)ct, ldct, M, N, K, bias, act, (const __bf16*)mask, ldm, dact, alpha,
                              beta, colpart, bits);
    if (rc) return rc;
    EM_CHECK_LAUNCH();
    return 0;
  }
  if (ct || colpart || bits) return EM_ERR_ARG;  // transposed copy / column partials / bits: 256 path only
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  const __bf16* mk = (const __bf16*)mask;
#define EM_GEMM_LAUNCH(AK, BKC)                                                                                        \
  hipLaunchKernelGGL((gemm_kernel<AK, BKC>), dim3(grid, splits), dim3(NT), LDS_BYTES, stream, a, lda, b, ldb, C, ldc,   \
                     c_bf16, M, N, K, bias, act, mk, ldm, dact, alpha, beta, kstep, c_split)
  if (a_kc && b_kc) EM_GEMM_LAUNCH(1, 1);
  else if (a_kc && !b_kc) EM_GEMM_LAUNCH(1, 0);
  else if (!a_kc && !b_kc) EM_GEMM_LAUNCH(0, 0);
  else EM_GEMM_LAUNCH(0, 1);
#undef EM_GEMM_LAUNCH
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_transpose_bf16(const void* src, int64_t ld_src, int R, int Cc, void* dst, int64_t ld_dst,
                             hipStream_t stream) {
  if (!src || !dst || R < 0 || Cc < 0) return EM_ERR_ARG;
  if ((ld_src & 7) || (ld_dst & 7) || (((uintptr_t)src | (uintptr_t)dst) & 15)) return EM_ERR_ARG;
  if (R == 0 || Cc == 0) return 0;
  const int64_t grid = (int64_t)((R + 63) / 64) * ((Cc + 63) / 64);
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)grid), dim3(256), 0, stream, (const __bf16*)src, ld_src, R, Cc,
                     (__bf16*)dst, ld_dst);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_colsum_ws_floats(int M, int N) { return ((M + CS_ROWS - 1) / CS_ROWS) * N; }

EM_API int em_colsum_bf16(const void* X, int64_t ldx, int M, int N, float* out, int accumulate, float scale, float* ws,
                          hipStream_t stream) {
  if (!X || !out || !ws || M < 0 || N < 0 || (ldx & 7) || (((uintptr_t)X) & 15)) return EM_ERR_ARG;
  if (N == 0) return 0;
  const int chunks = M > 0 ? (M + CS_ROWS - 1) / CS_ROWS : 0;
  if (chunks > 0) {
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 511) / 512, chunks), dim3(256), 0, stream, (const __bf16*)X,
                       ldx, M, N, ws);
    EM_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + CR_COLS - 1) / CR_COLS), dim3(CR_COLS * CR_G), 0, stream, ws,
                     chunks, N, out, accumulate, scale);
  EM_CHECK_LAUNCH();
  return 0;
}

// out[n] (+)= scale * sum_p part[p][n], fixed order (the em_gemm_bf16_cs bias-gradient partials)
EM_API int em_colpart_reduce(const float* part, int nparts, int N, float* out, int accumulate, float scale,
                             hipStream_t stream) {
  if (!part || !out || nparts < 0 || N < 0) return EM_ERR_ARG;
  if (N == 0) return 0;
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + CR_COLS - 1) / CR_COLS), dim3(CR_COLS * CR_G), 0, stream, part,
                     nparts, N, out, accumulate, scale);
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_rowsum_bf16(const void* X, int64_t ldx, int R, int Cc, float* out, int accumulate, float scale,
                          hipStream_t stream) {
  if (!X || !out || R < 0 || Cc < 0 || (ldx & 7) || (((uintptr_t)X) & 15)) return EM_ERR_ARG;
  if (R == 0) return 0;
  hipLaunchKernelGGL(rowsum_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, (const __bf16*)X, ldx, R, Cc, out,
                     accumulate, scale);
  EM_CHECK_LAUNCH();
  return 0;
}

// C = alpha * P^T Q (+ beta C): P bf16 [K][J <= 64] (ldp), Q bf16 [K][W] (ldq, W % 256 == 0), K % 64 == 0;
// part: fp32 workspace of splits * 64 * W floats; trans = 1 writes C^T [W][J] (ldc) instead of C [J][W].
EM_API int em_wgrad_skinny(const void* P, int64_t ldp, const void* Q, int64_t ldq, int K, int J, int W, float* C,
                           int64_t ldc, int trans, float alpha, float beta, float* part, int splits, int kstep,
                           hipStream_t stream) {
  if (!P || !Q || !C || !part || K <= 0 || (K & 63) || J < 1 || J > 64 || W <= 0 || (W % SK_WT) || splits < 1 ||
      kstep <= 0 || (kstep & 63) || (int64_t)splits * kstep < K || (int64_t)(splits - 1) * kstep >= K)
    return EM_ERR_ARG;
  if ((ldp & 7) || (ldq & 7) || ldp < J || ldq < W || ldc < (trans ? J : W) ||
      (((uintptr_t)P | (uintptr_t)Q) & 15))
    return EM_ERR_ARG;
  if ((int64_t)kstep * ldq * 2 >= (1ll << 31) || (int64_t)kstep * ldp * 2 >= (1ll << 31)) return EM_ERR_ARG;  // 32-bit offsets
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_skinny_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, SK_LDS);
    attr = true;
  }
  hipLaunchKernelGGL(wgrad_skinny_kernel, dim3(W / SK_WT, splits), dim3(256), SK_LDS, stream, (const __bf16*)P, ldp,
                     (const __bf16*)Q, ldq, K, W, kstep, part);
  EM_CHECK_LAUNCH();
  const int64_t n = (int64_t)J * W;
  hipLaunchKernelGGL(wgrad_skinny_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, part, splits,
                     J, W, C, ldc, trans, alpha, beta);
  EM_CHECK_LAUNCH();
  return 0;
}

// Segment timers of the last pp16 launches (diagnostic build, G_STAMPS=1): u64 [G_STAMP_BLOCKS][8 waves][8]
EM_API int em_gemm_stamps(void* host_out, int64_t bytes) {
#if G_STAMPS
  const int64_t have = (int64_t)sizeof(uint64_t) * G_STAMP_BLOCKS * 8 * 8;
  if (!host_out || bytes <= 0) return EM_ERR_ARG;
  const hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_gstamps), bytes < have ? bytes : have, 0,
                                           hipMemcpyDeviceToHost);
  return e == hipSuccess ? 0 : (int)e;
#else
  (void)host_out;
  (void)bytes;
  return EM_ERR_ARG;  // not a G_STAMPS build
#endif
}
