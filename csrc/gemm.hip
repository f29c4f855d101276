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
            const __bf16* __restrict__ mask, int64_t ldm, int dact, float alpha, float beta) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
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

// column sums of a bf16 [M][N] matrix into fp32 out[N] (+= if accumulate): bias gradients
__global__ void colsum_kernel(const __bf16* __restrict__ X, int64_t ldx, int M, int N, float* __restrict__ out,
                              int accumulate, float scale) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;  // 4 row partitions
  __shared__ float red[4][64];
  float s = 0.f;
  if (col < N)
    for (int m = part; m < M; m += 4) s += (float)X[(int64_t)m * ldx + col];
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && col < N) {
    const float t = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x])) * scale;
    out[col] = accumulate ? out[col] + t : t;
  }
}

}  // namespace

EM_API int em_gemm_bf16(const void* A, int64_t lda, int a_kc, const void* B, int64_t ldb, int b_kc, void* C,
                        int64_t ldc, int c_bf16, int M, int N, int K, const float* bias, int act, const void* mask,
                        int64_t ldm, int dact, float alpha, float beta, hipStream_t stream) {
  if (!A || !B || !C || M < 0 || N < 0 || K < 0 || act < 0 || act > 3) return EM_ERR_ARG;
  if (mask && (dact < 1 || dact > 3)) return EM_ERR_ARG;
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
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  const __bf16* mk = (const __bf16*)mask;
#define EM_GEMM_LAUNCH(AK, BKC)                                                                                        \
  hipLaunchKernelGGL((gemm_kernel<AK, BKC>), dim3(grid), dim3(NT), LDS_BYTES, stream, a, lda, b, ldb, C, ldc, c_bf16, M, \
                     N, K, bias, act, mk, ldm, dact, alpha, beta)
  if (a_kc && b_kc) EM_GEMM_LAUNCH(1, 1);
  else if (a_kc && !b_kc) EM_GEMM_LAUNCH(1, 0);
  else if (!a_kc && !b_kc) EM_GEMM_LAUNCH(0, 0);
  else EM_GEMM_LAUNCH(0, 1);
#undef EM_GEMM_LAUNCH
  EM_CHECK_LAUNCH();
  return 0;
}

EM_API int em_colsum_bf16(const void* X, int64_t ldx, int M, int N, float* out, int accumulate, float scale,
                          hipStream_t stream) {
  if (!X || !out || M < 0 || N < 0) return EM_ERR_ARG;
  if (N == 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(256), 0, stream, (const __bf16*)X, ldx, M, N, out,
                     accumulate, scale);
  EM_CHECK_LAUNCH();
  return 0;
}
