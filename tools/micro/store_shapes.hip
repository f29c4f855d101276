// Store-shape micro-benchmark (round 5): chip-wide bf16 write rate of a [R][8192] row-major output when each
// 16-B-per-lane wave store instruction covers SEG contiguous bytes of 1024 / SEG rows (SEG = 128: 8 rows x
// 128 B, the GEMM epilogues' row-image form; 256: 4 x 256 B; 512; 1024: one row).  Each workgroup writes a
// 128 x 128 bf16 tile (32 KB) like the skinny-K GEMM, 4 waves, grid = tiles.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/store_shapes.hip -o /tmp/store_shapes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int SEG>
__global__ void __launch_bounds__(256) store_tile_kernel(uint16_t* __restrict__ C, int64_t ldc, int tiles_n, int tcols) {
  const int bid = blockIdx.x, m0 = (bid / tiles_n) * 128, n0 = (bid % tiles_n) * tcols;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int LPR = SEG / 16;         // lanes per row segment
  constexpr int RPI = 64 / LPR;         // rows per instruction
  const int rows_per_wave = 128 * tcols * 2 / SEG / 4;  // row segments per wave
  u32x4 v = {(uint32_t)lane, (uint32_t)bid, 7u, 9u};
  for (int s = lane / LPR; s < rows_per_wave; s += RPI) {
    // segment s of this wave: (row, column block)
    const int segs_per_row = tcols * 2 / SEG;
    const int seg = wave * rows_per_wave + s;
    const int row = seg / segs_per_row, cb = seg % segs_per_row;
    *reinterpret_cast<u32x4*>(C + (int64_t)(m0 + row) * ldc + n0 + cb * (SEG / 2) + (lane % LPR) * 8) = v;
  }
}

template <int SEG>
float run(uint16_t* C, int R, int N, int tcols, int iters) {
  const int tiles = (R / 128) * (N / tcols);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_tile_kernel<SEG>, dim3(tiles), dim3(256), 0, 0, C, N, N / tcols, tcols);
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(store_tile_kernel<SEG>, dim3(tiles), dim3(256), 0, 0, C, N, N / tcols, tcols);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  const int R = 65536, N = 8192, iters = 20;
  uint16_t* C = nullptr;
  if (hipMalloc(&C, (size_t)R * N * 2) != hipSuccess) return 1;
  const double gb = (double)R * N * 2 / 1e9;
  for (int tcols : {128, 256}) {
    float t128 = run<128>(C, R, N, tcols, iters), t256 = run<256>(C, R, N, tcols, iters);
    float t512 = tcols >= 256 ? run<512>(C, R, N, tcols, iters) : 0.f;
    printf("{\"tile_cols\": %d, \"seg128_tbps\": %.2f, \"seg256_tbps\": %.2f, \"seg512_tbps\": %.2f}\n", tcols,
           gb / t128, gb / t256, t512 > 0 ? gb / t512 : 0.0);
  }
  hipFree(C);
  return 0;
}
