// X1 equivalent: multithreaded numeric CSV loader.
//
// The reference hands its temp CSVs to dmlc-core through
// `new DMatrix(path + "?format=csv&label_column=0")` (Main.java:110-111).  This
// loader reads a numeric CSV into a dense row-major float32 matrix:
//   * optional header line (the reference wrote one but dmlc would have parsed it
//     as data, defect D-c; here it is skipped explicitly),
//   * fields split on ',' with surrounding blanks ignored, a trailing empty field
//     (the reference's ", " record terminator) dropped,
//   * non-numeric fields become NaN, short rows are NaN-padded,
//   * rows are parsed in parallel (std::thread over line ranges).
// Label-column extraction happens in Python on the returned matrix.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

bool read_file(const char* path, std::string& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(sz > 0 ? (size_t)sz : 0);
  const size_t got = sz > 0 ? std::fread(&buf[0], 1, (size_t)sz, f) : 0;
  std::fclose(f);
  buf.resize(got);
  return true;
}

// line [b, e) -> fields (count only if out == nullptr)
int64_t parse_line(const char* b, const char* e, float* out, int64_t ncols) {
  int64_t col = 0;
  const char* p = b;
  while (p <= e) {
    const char* q = p;
    while (q < e && *q != ',') ++q;
    const char* fb = p;
    const char* fe = q;
    while (fb < fe && (*fb == ' ' || *fb == '\t' || *fb == '\r' || *fb == '"')) ++fb;
    while (fe > fb && (fe[-1] == ' ' || fe[-1] == '\t' || fe[-1] == '\r' || fe[-1] == '"')) --fe;
    const bool last = (q >= e);
    if (!(last && fb == fe && col > 0)) {  // drop a trailing empty field
      if (out && col < ncols) {
        char tmp[64];
        const size_t len = (size_t)(fe - fb) < sizeof(tmp) - 1 ? (size_t)(fe - fb) : sizeof(tmp) - 1;
        std::memcpy(tmp, fb, len);
        tmp[len] = 0;
        char* endp = nullptr;
        errno = 0;
        const float v = std::strtof(tmp, &endp);
        out[col] = (len == 0 || endp == tmp || *endp != 0) ? NAN : v;
      }
      ++col;
    }
    if (last) break;
    p = q + 1;
  }
  if (out)
    for (int64_t c = col; c < ncols; ++c) out[c] = NAN;
  return col;
}

void line_index(const std::string& buf, int skip_header, std::vector<std::pair<size_t, size_t>>& lines) {
  size_t i = 0, n = buf.size();
  bool first = true;
  while (i < n) {
    size_t j = buf.find('\n', i);
    if (j == std::string::npos) j = n;
    size_t e = j;
    if (e > i && buf[e - 1] == '\r') --e;
    bool blank = true;
    for (size_t k = i; k < e; ++k)
      if (buf[k] != ' ' && buf[k] != '\t' && buf[k] != ',') { blank = false; break; }
    if (!blank) {
      if (first && skip_header) {
        first = false;
      } else {
        lines.emplace_back(i, e);
        first = false;
      }
    }
    i = j + 1;
  }
}

}  // namespace

extern "C" {

// returns number of data rows (or <0 on error); *ncols_out = max field count
int64_t emh_csv_shape(const char* path, int skip_header, int64_t* ncols_out) {
  std::string buf;
  if (!read_file(path, buf)) return -1;
  std::vector<std::pair<size_t, size_t>> lines;
  line_index(buf, skip_header, lines);
  int64_t mc = 0;
  for (auto& l : lines) {
    const int64_t c = parse_line(buf.data() + l.first, buf.data() + l.second, nullptr, 0);
    if (c > mc) mc = c;
  }
  if (ncols_out) *ncols_out = mc;
  return (int64_t)lines.size();
}

int emh_csv_load(const char* path, int skip_header, int64_t nrows, int64_t ncols, float* out, int nthreads) {
  std::string buf;
  if (!read_file(path, buf)) return -1;
  std::vector<std::pair<size_t, size_t>> lines;
  line_index(buf, skip_header, lines);
  if ((int64_t)lines.size() != nrows) return -2;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  std::vector<std::thread> th;
  const int64_t per = (nrows + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t a = t * per, b = std::min<int64_t>(nrows, a + per);
    if (a >= b) break;
    th.emplace_back([&, a, b]() {
      for (int64_t r = a; r < b; ++r)
        parse_line(buf.data() + lines[r].first, buf.data() + lines[r].second, out + r * ncols, ncols);
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

}  // extern "C"
