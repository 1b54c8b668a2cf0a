// Sanitizer driver for the native log writer (dps_log.cpp + dps_error.cpp),
// built by `make -C distributed-pathsim_amd/csrc asan` with
// -fsanitize=address,undefined and run by tests/test_sanitizers.py.
// Checks: dps_format_float round-trips (strtod of the text gives the same
// bits) on special values and random bit patterns; dps_write_topk_log writes
// the expected number of lines for multi-part, multi-thread runs with empty
// slots (-1), and rejects bad arguments.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "dpathsim.h"

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/dps_log_asan.log";
  char buf[64];
  const double specials[] = {0.0, -0.0, 1.0, 0.1, 1e16, 1e-4, 9.999e-5, 123456789012345678.0,
                             5e-324, 1.7976931348623157e308, 2.0 / 3.0, INFINITY, -INFINITY};
  for (double v : specials) {
    if (dps_format_float(v, buf, sizeof(buf)) != DPS_OK) return fail("format special");
    if (std::isfinite(v) && std::strtod(buf, nullptr) != v) return fail(buf);
  }
  if (dps_format_float(NAN, buf, sizeof(buf)) != DPS_OK || std::strcmp(buf, "nan") != 0)
    return fail("nan");
  if (dps_format_float(0.1, buf, 3) == DPS_OK) return fail("tiny buffer accepted");
  std::mt19937_64 rng(7);
  for (int i = 0; i < 200000; ++i) {
    uint64_t bits = rng();
    double v;
    std::memcpy(&v, &bits, 8);
    if (!std::isfinite(v)) continue;
    if (dps_format_float(v, buf, sizeof(buf)) != DPS_OK) return fail("format random");
    double back = std::strtod(buf, nullptr);
    if (std::memcmp(&back, &v, 8) != 0) return fail(buf);
  }
  // all-pairs writer: n_authors authors, rows [row_begin, row_begin + n_rows)
  const int64_t na = 10000, row_begin = 37, n_rows = 9000;
  const int32_t k = 3;
  std::vector<int32_t> idx(n_rows * k);
  std::vector<int64_t> cnt(n_rows * k), g(na);
  std::vector<double> sc(n_rows * k);
  int64_t ranked = 0;
  for (int64_t r = 0; r < n_rows; ++r)
    for (int s = 0; s < k; ++s) {
      const bool empty = (r % 7 == 0 && s == k - 1);
      idx[r * k + s] = empty ? -1 : static_cast<int32_t>((r * 31 + s * 7) % na);
      cnt[r * k + s] = r + s;
      sc[r * k + s] = 1.0 / (1 + r + s);
      ranked += !empty;
    }
  for (int64_t a = 0; a < na; ++a) g[a] = a * 3;
  std::string ids, labels;
  std::vector<int64_t> id_off(na + 1, 0), lab_off(na + 1, 0);
  for (int64_t a = 0; a < na; ++a) {
    ids += "author_" + std::to_string(a);
    labels += "Author Name " + std::to_string(a);
    id_off[a + 1] = ids.size();
    lab_off[a + 1] = labels.size();
  }
  for (int threads : {1, 4}) {
    int rc = dps_write_topk_log(path, 0, row_begin, n_rows, k, idx.data(), cnt.data(), sc.data(),
                                g.data(), ids.data(), id_off.data(), labels.data(),
                                lab_off.data(), 0.25, 1.5, threads);
    if (rc != DPS_OK) return fail(dps_last_error());
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail("reopen");
    int64_t lines = 0;
    int ch;
    while ((ch = std::fgetc(f)) != EOF) lines += ch == '\n';
    std::fclose(f);
    if (lines != n_rows + 5 * ranked + 1) return fail("line count");
  }
  if (dps_write_topk_log(path, 0, -1, 1, k, idx.data(), cnt.data(), sc.data(), g.data(),
                         ids.data(), id_off.data(), labels.data(), lab_off.data(), 0, 0, 1) ==
      DPS_OK)
    return fail("negative row_begin accepted");
  if (dps_write_topk_log(path, 0, 0, 1, k, nullptr, cnt.data(), sc.data(), g.data(), ids.data(),
                         id_off.data(), labels.data(), lab_off.data(), 0, 0, 1) == DPS_OK)
    return fail("null array accepted");
  std::printf("log asan ok\n");
  return 0;
}
