// Host-side synthetic Euromillions draw generator (SURVEY.md §2.4 N1, §0.3 domain facts).
//
// Replaces the reference's HTTP scrape of portalseven.com (Main.java:37-58) when no
// CSV is given.  Rules: 5 distinct main numbers 1..50, 2 distinct stars 1..S(t)
// (S = 9 / 11 / 12 by era, supplied per draw by the caller from the draw dates).
// Optional planted structure (a seeded Markov chain), so that "0.9+" accuracy is a
// property of learnable data, not an artefact:  each number of draw t+1 is, with
// probability `planted`, the image pi(n) of the corresponding number n of draw t
// under a fixed seeded permutation pi (separately for mains and stars); the rest
// are uniform.  planted = 0 gives iid draws (no model can beat chance).
//
// The PRNG is splitmix64 and every random call happens in a fixed order, so the
// pure-Python twin in euromillioner_amd/data/synthetic.py produces identical draws
// (tested bit-for-bit); this C++ version exists for the 10^7-10^9-draw HBM-filling
// datasets.
#include <algorithm>
#include <cstdint>
#include <cstring>

namespace {

struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t uint(uint32_t n) { return (uint32_t)(next() % n); }
  double u01() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

void shuffle_perm(SplitMix64& g, int* a, int n) {
  for (int i = 0; i < n; ++i) a[i] = i + 1;
  for (int i = n - 1; i >= 1; --i) {
    const int j = (int)g.uint((uint32_t)(i + 1));
    std::swap(a[i], a[j]);
  }
}

inline bool has(const uint8_t* v, int cnt, int c) {
  for (int i = 0; i < cnt; ++i)
    if (v[i] == c) return true;
  return false;
}

}  // namespace

extern "C" {

// out: [n][8] uint8 = 5 sorted mains, 2 sorted stars, 0 pad.  perm_out (optional): [62] = pi_main[1..50], pi_star[1..12]
int emh_generate_draws(uint64_t seed, int64_t n, double planted, const int32_t* star_max, uint8_t* out,
                       int32_t* perm_out) {
  if (n < 0 || !out || planted < 0.0 || planted > 1.0) return -1;
  SplitMix64 g{seed};
  int pim[50], pis[12];
  shuffle_perm(g, pim, 50);
  shuffle_perm(g, pis, 12);
  if (perm_out) {
    for (int i = 0; i < 50; ++i) perm_out[i] = pim[i];
    for (int i = 0; i < 12; ++i) perm_out[50 + i] = pis[i];
  }
  uint8_t pm[5] = {0}, ps[2] = {0};
  for (int64_t t = 0; t < n; ++t) {
    const int smax = star_max ? star_max[t] : 12;
    if (smax < 2 || smax > 12) return -2;
    uint8_t m[5], s[2];
    int cm = 0, cs = 0;
    if (t > 0 && planted > 0.0) {
      for (int k = 0; k < 5; ++k) {
        const double u = g.u01();
        if (u < planted) {
          const int c = pim[pm[k] - 1];
          if (!has(m, cm, c)) m[cm++] = (uint8_t)c;
        }
      }
    }
    while (cm < 5) {
      const int c = 1 + (int)g.uint(50);
      if (!has(m, cm, c)) m[cm++] = (uint8_t)c;
    }
    if (t > 0 && planted > 0.0) {
      for (int k = 0; k < 2; ++k) {
        const double u = g.u01();
        if (u < planted) {
          const int c = pis[ps[k] - 1];
          if (c <= smax && !has(s, cs, c)) s[cs++] = (uint8_t)c;
        }
      }
    }
    while (cs < 2) {
      const int c = 1 + (int)g.uint((uint32_t)smax);
      if (!has(s, cs, c)) s[cs++] = (uint8_t)c;
    }
    std::sort(m, m + 5);
    std::sort(s, s + 2);
    uint8_t* o = out + t * 8;
    std::memcpy(o, m, 5);
    o[5] = s[0];
    o[6] = s[1];
    o[7] = 0;
    std::memcpy(pm, m, 5);
    std::memcpy(ps, s, 2);
  }
  return 0;
}

}  // extern "C"
