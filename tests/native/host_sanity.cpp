// Host-code sanitizer driver: links the C++ host sources directly (no Python, no
// LD_PRELOAD) so they can be built with -fsanitize=address,undefined or -fsanitize=thread and
// exercised: synthetic draw generation and the multithreaded CSV loader.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
int emh_generate_draws(uint64_t seed, int64_t n, double planted, const int32_t* star_max, uint8_t* out,
                       int32_t* perm_out);
int64_t emh_csv_shape(const char* path, int skip_header, int64_t* ncols_out);
int emh_csv_load(const char* path, int skip_header, int64_t nrows, int64_t ncols, float* out, int nthreads);
}

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "host_sanity.csv";
  const int64_t n = 20000;
  std::vector<int32_t> star_max(n, 12);
  std::vector<uint8_t> draws(n * 8);
  std::vector<int32_t> perm(62);
  if (emh_generate_draws(42, n, 0.7, star_max.data(), draws.data(), perm.data()) != 0) return fail("generate");
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* r = &draws[i * 8];
    for (int k = 0; k < 5; ++k)
      if (r[k] < 1 || r[k] > 50) return fail("main range");
    for (int k = 5; k < 7; ++k)
      if (r[k] < 1 || r[k] > 12) return fail("star range");
  }
  FILE* f = std::fopen(path, "w");
  if (!f) return fail("open");
  std::fprintf(f, "a,b,c,d,e,f,g\n");
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* r = &draws[i * 8];
    std::fprintf(f, "%d,%d,%d,%d,%d,%d,%d%s\n", r[0], r[1], r[2], r[3], r[4], r[5], r[6], (i % 7 == 0) ? "," : "");
  }
  std::fprintf(f, "x,1,2,3,4,5,6\n");  // non-numeric field -> NaN
  std::fclose(f);
  int64_t ncols = 0;
  const int64_t rows = emh_csv_shape(path, 1, &ncols);
  if (rows != n + 1 || ncols != 7) return fail("shape");
  std::vector<float> out(rows * ncols);
  if (emh_csv_load(path, 1, rows, ncols, out.data(), 8) != 0) return fail("load");
  for (int64_t i = 0; i < n; ++i)
    for (int k = 0; k < 7; ++k)
      if (out[i * 7 + k] != (float)draws[i * 8 + k]) return fail("value");
  if (!std::isnan(out[n * 7])) return fail("nan");
  std::remove(path);
  std::puts("host_sanity ok");
  return 0;
}
