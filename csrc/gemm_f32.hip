// K1/K2/K3 fp32 variant — exact-fp32 MFMA GEMM for the `--dtype fp32` MLP path (MI355X / gfx950).
//
// SURVEY.md §2.7 K1 asks for "an f32-MFMA variant for the fp32 config" next to the bf16 kernels
// in gemm.hip (the reference's declared DL4J/ND4J dense layers, pom.xml:62-66, default to fp32).
// CDNA4 has no TF32/xf32 shortcut: v_mfma_f32_32x32x2_f32 multiplies exact fp32 inputs, two k
// per instruction, into the same 32x32 accumulator layout as the bf16 MFMAs.
//
//   C[m][n] = epi( alpha * sum_k A[m][k] * B[k][n] )      (fp32 in, fp32 accumulate, fp32 out)
//   A[m][k] at A + m*lda + k (A_KC = 1) or A + k*lda + m (A_KC = 0); B[k][n] likewise with B_KC
//   epi: + bias[n], activation, or * act'(Y[m][n]) from the saved fp32 layer output Y, + beta*C_old
//
// Tiling: 128x128 output tile per 256-thread workgroup (2x2 waves of 64x64 = 2x2 MFMA 32x32
// blocks, 64 accumulator registers), BK = 16, two LDS stages.  Both operands are staged k-major
// ([16 k][128 + 4] floats): an MFMA operand is then one ds_read_b32 per lane whose 32-lane group
// reads 32 consecutive floats of one k row -- conflict-free, no swizzle.  Global loads are 16 B
// (four consecutive k for K-contiguous operands, four consecutive rows otherwise).  Split-K over
// gridDim.y writes slice s of the K range to C + s*c_split (summed by the caller) so the wgrad of
// a small layer over a large batch still fills the chip.  Block ids are XCD-remapped like gemm.hip.
#include "common.h"

namespace {

constexpr int FBM = 128, FBN = 128, FBK = 16, FNT = 256;
constexpr int FROW = FBM + 4;                      // floats per staged k row (pad keeps 16-B alignment)
constexpr int FTILE = FBK * FROW * 4;              // bytes per operand per stage
constexpr int F_LDS = 2 * 2 * FTILE;

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3 };

EM_DEVICE f32x16 mfma32_f32(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

EM_DEVICE float f_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}
EM_DEVICE float f_dact(float y, int act) {  // derivative expressed through the saved output y
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

// 128 rows x 16 k of one operand: 512 float4 pieces, 2 per thread, zero-filled out of range
template <int KC>
EM_DEVICE void f_load(const float* __restrict__ P, int64_t ld, int r0, int k0, int k1, int R, int tid, f32x4 (&v)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + i * FNT;
    int row, kk;
    if (KC) {  // 128 rows x 4 pieces of 4 k
      row = r0 + (c >> 2);
      kk = k0 + (c & 3) * 4;
    } else {  // 16 k rows x 32 pieces of 4 rows
      kk = k0 + (c >> 5);
      row = r0 + (c & 31) * 4;
    }
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (KC) {
      if (row < R) {
        if (kk + 4 <= k1 && ((reinterpret_cast<uintptr_t>(P + (int64_t)row * ld + kk) & 15) == 0)) {
          x = *reinterpret_cast<const f32x4*>(P + (int64_t)row * ld + kk);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = (kk + e < k1) ? P[(int64_t)row * ld + kk + e] : 0.f;
        }
      }
    } else {
      if (kk < k1) {
        if (row + 4 <= R && ((reinterpret_cast<uintptr_t>(P + (int64_t)kk * ld + row) & 15) == 0)) {
          x = *reinterpret_cast<const f32x4*>(P + (int64_t)kk * ld + row);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = (row + e < R) ? P[(int64_t)kk * ld + row + e] : 0.f;
        }
      }
    }
    v[i] = x;
  }
}

template <int KC>
EM_DEVICE void f_store(char* lds, int tid, const f32x4 (&v)[2]) {
  float* t = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + i * FNT;
    if (KC) {  // four k rows of one tile row
      const int row = c >> 2, k = (c & 3) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) t[(k + e) * FROW + row] = v[i][e];
    } else {
      *reinterpret_cast<f32x4*>(t + (c >> 5) * FROW + (c & 31) * 4) = v[i];
    }
  }
}

EM_DEVICE int f_xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int A_KC, int B_KC>
__global__ void __launch_bounds__(FNT, 2)
gemm_f32_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                float* __restrict__ C, int64_t ldc, int M, int N, int K, const float* __restrict__ bias, int act,
                const float* __restrict__ Y, int64_t ldy, int dact, float alpha, float beta, int kstep,
                int64_t c_split, float* __restrict__ colpart) {
  // colpart (optional, no split-K): column sums of this tile's 128 output rows (the stored values)
  // -> colpart[m0 / 128][n], fixed order: a lane's 32 rows, the two lane halves, then wm 0 + wm 1
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (N + FBN - 1) / FBN, tiles_m = (M + FBM - 1) / FBM;
  const int bid = f_xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * FBM, n0 = (bid % tiles_n) * FBN;
  const int kb = blockIdx.y * kstep, ke = min(K, kb + kstep);
  C += (int64_t)blockIdx.y * c_split;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int nk = (ke - kb + FBK - 1) / FBK;
  f32x4 ra[2], rb[2];
  if (nk > 0) {
    f_load<A_KC>(A, lda, m0, kb, ke, M, tid, ra);
    f_load<B_KC>(B, ldb, n0, kb, ke, N, tid, rb);
    f_store<A_KC>(smem, tid, ra);
    f_store<B_KC>(smem + FTILE, tid, rb);
  }
  __syncthreads();
  const int r = lane & 31, h = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    const float* la = reinterpret_cast<const float*>(smem + (t & 1) * 2 * FTILE);
    const float* lb = la + FTILE / 4;
    const bool more = t + 1 < nk;
    if (more) {  // next tile's global loads in flight during this tile's MFMAs
      f_load<A_KC>(A, lda, m0, kb + (t + 1) * FBK, ke, M, tid, ra);
      f_load<B_KC>(B, ldb, n0, kb + (t + 1) * FBK, ke, N, tid, rb);
    }
#pragma unroll
    for (int s = 0; s < FBK / 2; ++s) {
      const int k = 2 * s + h;
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = la[k * FROW + wm * 64 + 32 * i + r];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = lb[k * FROW + wn * 64 + 32 * j + r];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32_f32(a[i], b[j], acc[i][j]);
    }
    if (more) {  // the other stage was last read in iteration t-1, before this iteration's barrier
      char* nx = smem + ((t + 1) & 1) * 2 * FTILE;
      f_store<A_KC>(nx, tid, ra);
      f_store<B_KC>(nx + FTILE, tid, rb);
    }
    __syncthreads();
  }

  // epilogue: accumulator register g of block (i, j) = row 8*(g>>2) + 4h + (g&3), column r
  float cs[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + 32 * j + r;
      if (col >= N) continue;
      const float bv = (bias && !dact) ? bias[col] : 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = m0 + wm * 64 + 32 * i + 8 * (g >> 2) + 4 * h + (g & 3);
        if (row >= M) continue;
        float v = alpha * acc[i][j][g];
        if (dact) {
          v *= f_dact(Y[(int64_t)row * ldy + col], act);
        } else {
          v = f_act(v + bv, act);
        }
        float* cp = C + (int64_t)row * ldc + col;
        v = beta != 0.f ? v + beta * *cp : v;
        *cp = v;
        cs[j] += v;
      }
    }
  if (colpart) {  // block-uniform
    float* red = reinterpret_cast<float*>(smem);  // [2 wm][128 cols]; the K loop ended on a barrier
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float v = cs[j] + __shfl_xor(cs[j], 32);
      if (h == 0) red[wm * 128 + wn * 64 + 32 * j + r] = v;
    }
    __syncthreads();
    if (tid < 128 && n0 + tid < N) colpart[(int64_t)(m0 / FBM) * N + n0 + tid] = red[tid] + red[128 + tid];
  }
}

template <int A_KC, int B_KC>
void f_launch(dim3 grid, hipStream_t st, const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
              int64_t ldc, int M, int N, int K, const float* bias, int act, const float* Y, int64_t ldy, int dact,
              float alpha, float beta, int kstep, int64_t c_split, float* colpart) {
  hipLaunchKernelGGL((gemm_f32_kernel<A_KC, B_KC>), grid, dim3(FNT), F_LDS, st, A, lda, B, ldb, C, ldc, M, N, K, bias,
                     act, Y, ldy, dact, alpha, beta, kstep, c_split, colpart);
}

}  // namespace

// fp32 GEMM (see header).  splits > 1: slice s covers k in [s*kstep, (s+1)*kstep) and writes
// C + s*c_split (bias/activation must then be applied by the caller after summing; beta per slice).
EM_API int em_gemm_f32(const float* A, int64_t lda, int a_kc, const float* B, int64_t ldb, int b_kc, float* C,
                       int64_t ldc, int M, int N, int K, const float* bias, int act, const float* Y, int64_t ldy,
                       int dact, float alpha, float beta, int splits, int kstep, int64_t c_split,
                       float* colpart, hipStream_t stream) {
  // colpart: [ceil(M / 128)][N] fp32 column sums of C per 128-row tile (bias gradient partials)
  if (!A || !B || !C || M < 0 || N < 0 || K < 0 || act < 0 || act > 3 || (dact && !Y) || splits < 1 ||
      (colpart && splits > 1))
    return EM_ERR_ARG;
  if (M == 0 || N == 0) return 0;
  if (splits > 1 && (kstep <= 0 || (int64_t)kstep * splits < K || c_split < (int64_t)M * ldc || bias || act))
    return EM_ERR_ARG;
  if (splits == 1) {
    kstep = K > 0 ? K : 1;
    c_split = 0;
  }
  const int tiles = ((M + FBM - 1) / FBM) * ((N + FBN - 1) / FBN);
  const dim3 grid((unsigned)tiles, (unsigned)splits);
  if (a_kc && b_kc)
    f_launch<1, 1>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, bias, act, Y, ldy, dact, alpha, beta, kstep, c_split,
                   colpart);
  else if (a_kc)
    f_launch<1, 0>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, bias, act, Y, ldy, dact, alpha, beta, kstep, c_split,
                   colpart);
  else if (b_kc)
    f_launch<0, 1>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, bias, act, Y, ldy, dact, alpha, beta, kstep, c_split,
                   colpart);
  else
    f_launch<0, 0>(grid, stream, A, lda, B, ldb, C, ldc, M, N, K, bias, act, Y, ldy, dact, alpha, beta, kstep, c_split,
                   colpart);
  EM_CHECK_LAUNCH();
  return 0;
}
