// High-volume writer of the reference's run-log format for all-pairs top-k
// results (format of DPathSim_APVPA.py:32-67).
//
// Host code only (no device work).  Per source row x the block is
//   Source author global walk: {g[x]}
// followed, for every ranked target y (idx >= 0) in rank order, by
//   Pairwise authors walk {id[y]}: {M}
//   Target author global walk: {g[y]}
//   Sim score {label[x]} - {label[y]}: {score}
//   ***Stage done in: {stage_seconds}
//   ---
// and optionally one closing "***Overall done in: {overall_seconds}".  Floats
// are printed exactly as Python's str()/repr() prints them (shortest digits
// that round-trip, fixed notation for 1e-4 <= |v| < 1e16, else d.ddde+XX with
// at least two exponent digits, ".0" on integral values): the shortest digits
// come from std::to_chars, the layout follows CPython's float_repr rules.
// Rows are formatted in parallel into per-thread buffers and written in order.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "dps_host.hpp"

namespace dps {
namespace {

void put_i64(std::string& out, int64_t v) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof(buf), v);
  out.append(buf, r.ptr);
}

}  // namespace

// Python repr() of a double (CPython float_repr_style 'short', repr mode).
void format_py_float(std::string& out, double v) {
  if (std::isnan(v)) { out += "nan"; return; }
  if (std::isinf(v)) { out += v < 0 ? "-inf" : "inf"; return; }
  if (v == 0.0) { out += std::signbit(v) ? "-0.0" : "0.0"; return; }
  char buf[64];
  // shortest round-trip digits in scientific form: [-]d[.ddd]e(+|-)XX
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  const char* p = buf;
  const char* end = r.ptr;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[32];
  int nd = 0;
  const char* q = p;
  for (; q < end && *q != 'e'; ++q)
    if (*q != '.') digits[nd++] = *q;
  int exp10 = 0;
  std::from_chars(q + 1 + (q[1] == '+' ? 1 : 0), end, exp10);
  while (nd > 1 && digits[nd - 1] == '0') --nd;   // to_chars is already shortest
  const int decpt = exp10 + 1;                     // value = 0.d1d2... * 10^decpt
  if (neg) out += '-';
  if (decpt <= -4 || decpt > 16) {
    out += digits[0];
    if (nd > 1) { out += '.'; out.append(digits + 1, nd - 1); }
    out += 'e';
    const int e = decpt - 1;
    out += e < 0 ? '-' : '+';
    const int ae = e < 0 ? -e : e;
    if (ae < 10) out += '0';
    put_i64(out, ae);
  } else if (decpt <= 0) {
    out += "0.";
    out.append(static_cast<size_t>(-decpt), '0');
    out.append(digits, nd);
  } else if (decpt >= nd) {
    out.append(digits, nd);
    out.append(static_cast<size_t>(decpt - nd), '0');
    out += ".0";
  } else {
    out.append(digits, decpt);
    out += '.';
    out.append(digits + decpt, nd - decpt);
  }
}

}  // namespace dps

using namespace dps;

extern "C" {

int dps_format_float(double v, char* out, size_t cap) {
  std::string s;
  format_py_float(s, v);
  DPS_REQUIRE(out && cap > s.size(), DPS_ERR_INVALID, "output buffer too small");
  std::memcpy(out, s.data(), s.size());
  out[s.size()] = '\0';
  return DPS_OK;
}

int dps_write_topk_log(const char* path, int append, int64_t row_begin, int64_t n_rows, int32_t k,
                       const int32_t* idx_host, const int64_t* cnt_host, const double* score_host,
                       const int64_t* g_host, const char* id_blob, const int64_t* id_off,
                       const char* label_blob, const int64_t* label_off, double stage_seconds,
                       double overall_seconds, int n_threads) {
  DPS_REQUIRE(path && n_rows >= 0 && k >= 1 && row_begin >= 0, DPS_ERR_INVALID,
              "bad arguments to dps_write_topk_log");
  DPS_REQUIRE(n_rows == 0 || (idx_host && cnt_host && score_host && g_host && id_blob && id_off &&
                              label_blob && label_off),
              DPS_ERR_INVALID, "null host array");
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  DPS_REQUIRE(f, DPS_ERR_INVALID, "cannot open %s", path);
  std::string stage;
  format_py_float(stage, stage_seconds);
  const int T = std::max(1, n_threads > 0 ? n_threads
                                           : static_cast<int>(std::thread::hardware_concurrency()));
  constexpr int64_t kRowsPerPart = 4096;
  int64_t done = 0;
  bool ok = true;
  while (done < n_rows && ok) {
    // one round: T parts of kRowsPerPart rows each, formatted in parallel
    const int64_t round_rows = std::min<int64_t>(n_rows - done, kRowsPerPart * T);
    const int parts = static_cast<int>((round_rows + kRowsPerPart - 1) / kRowsPerPart);
    std::vector<std::string> buf(parts);
    auto work = [&](int part) {
      std::string& o = buf[part];
      const int64_t r0 = done + part * kRowsPerPart;
      const int64_t r1 = std::min(done + round_rows, r0 + kRowsPerPart);
      o.reserve(static_cast<size_t>(r1 - r0) * (64 + static_cast<size_t>(k) * 200));
      for (int64_t r = r0; r < r1; ++r) {
        const int64_t x = row_begin + r;
        o += "Source author global walk: ";
        put_i64(o, g_host[x]);
        o += '\n';
        for (int32_t s = 0; s < k; ++s) {
          const int64_t e = r * k + s;
          const int32_t y = idx_host[e];
          if (y < 0) continue;
          o += "Pairwise authors walk ";
          o.append(id_blob + id_off[y], static_cast<size_t>(id_off[y + 1] - id_off[y]));
          o += ": ";
          put_i64(o, cnt_host[e]);
          o += "\nTarget author global walk: ";
          put_i64(o, g_host[y]);
          o += "\nSim score ";
          o.append(label_blob + label_off[x], static_cast<size_t>(label_off[x + 1] - label_off[x]));
          o += " - ";
          o.append(label_blob + label_off[y], static_cast<size_t>(label_off[y + 1] - label_off[y]));
          o += ": ";
          format_py_float(o, score_host[e]);
          o += "\n***Stage done in: ";
          o += stage;
          o += "\n---\n";
        }
      }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < parts; ++i) th.emplace_back(work, i);
    work(0);
    for (auto& t : th) t.join();
    for (auto& b : buf)
      if (std::fwrite(b.data(), 1, b.size(), f) != b.size()) ok = false;
    done += round_rows;
  }
  if (ok && overall_seconds >= 0.0) {
    std::string o = "***Overall done in: ";
    format_py_float(o, overall_seconds);
    o += '\n';
    if (std::fwrite(o.data(), 1, o.size(), f) != o.size()) ok = false;
  }
  if (std::fclose(f) != 0) ok = false;
  DPS_REQUIRE(ok, DPS_ERR_INVALID, "write to %s failed", path);
  return DPS_OK;
}

}  // extern "C"
