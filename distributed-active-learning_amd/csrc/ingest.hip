// Pool ingest: the reference's on-disk text format parsed natively into a
// (pinned) host buffer that the Python side uploads to HBM asynchronously.
//
// Reference: final_thesis/uncertainty_sampling.py:37-42 and
// density_weighting.py:45-53,59-65 read whitespace-separated rows with the
// label last through sc.textFile, map each row to
//   LabeledPoint(0 if int(_[-1]) == -1 else 1, np.array(_[:-1]).astype(float))
// (features parsed as fp64) and optionally keep the first n_samples rows
// (``sc.parallelize(data.take(n_samples))``).  Here: features are parsed as
// fp64 (strtod, correctly rounded) and narrowed to fp32 -- the same bits as
// ``np.array(fields, dtype=np.float64).astype(np.float32)`` -- and labels with
// the reference's -1 -> 0 / else -> 1 map (or kept as is for 0/1 files).
// Blank lines are skipped (str.split() of an empty line yields no fields).
//
// Host code only (no kernels): a byte range is split at line starts into one
// segment per thread; each thread counts its rows, the counts are prefix-summed
// and each thread parses its rows into their final positions.
#include <locale.h>

#include <cerrno>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// Start of the line containing position p (or p itself if it starts a line).
size_t line_start(const char* t, size_t len, size_t p) {
  if (p >= len) return len;
  while (p > 0 && t[p - 1] != '\n') --p;
  return p;
}

// Number of whitespace-separated fields in [a, b).
int64_t count_fields(const char* t, size_t a, size_t b) {
  int64_t f = 0;
  size_t i = a;
  while (i < b) {
    while (i < b && is_space(t[i])) ++i;
    if (i >= b) break;
    ++f;
    while (i < b && !is_space(t[i])) ++i;
  }
  return f;
}

size_t line_end(const char* t, size_t len, size_t p) {
  while (p < len && t[p] != '\n') ++p;
  return p;
}

int64_t count_rows(const char* t, size_t a, size_t b) {
  int64_t r = 0;
  size_t i = a;
  while (i < b) {
    const size_t e = line_end(t, b, i);
    if (count_fields(t, i, e) > 0) ++r;
    i = e + 1;
  }
  return r;
}

// The "C" numeric locale, created once: the reference parses with Python's
// float(), which ignores LC_NUMERIC ('.' is the only decimal point).
locale_t c_numeric_locale() {
  static locale_t loc = newlocale(LC_NUMERIC_MASK, "C", static_cast<locale_t>(0));
  return loc;
}

// Copy token [a, b) into a NUL-terminated buffer without its PEP 515
// digit-group underscores, as Python's float() / int() read them ("1_000.5" =
// 1000.5): an underscore must sit between two digits, anything else rejects
// the token, and so does a NUL byte (not a field delimiter; float('1\x00')
// raises).  Tokens that do not fit the caller's stack buffer go to ``big``
// (float() takes any length: a 200-digit field is inf after the fp32 narrowing).
const char* copy_token(const char* t, size_t a, size_t b, char* buf, size_t cap, std::string& big) {
  const size_t n = b - a;
  if (n == 0) return nullptr;
  char* dst = buf;
  if (n >= cap) {
    big.assign(n + 1, '\0');
    dst = &big[0];
  }
  size_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    const char c = t[a + i];
    if (c == 0) return nullptr;  // an embedded NUL would end strtod early: float() rejects the token
    if (c == '_') {
      const bool ok = i > 0 && i + 1 < n && is_digit(t[a + i - 1]) && is_digit(t[a + i + 1]);
      if (!ok) return nullptr;
      continue;
    }
    dst[m++] = c;
  }
  dst[m] = 0;
  return dst;
}

// Parse one field [a, b) as fp64 (the token must be consumed entirely).
// Python's float() accepts decimal literals with digit-group underscores,
// inf/infinity/nan (any case, with a sign); strtod also takes hex floats
// ("0x1p3") and "nan(chars)", which float() rejects -- such tokens are
// rejected here too.  Fields are whitespace-delimited, so a token never
// carries the surrounding whitespace float() would strip.
bool parse_double(const char* t, size_t a, size_t b, double& v) {
  char buf[128];
  std::string big;
  for (size_t i = a; i < b; ++i)
    if (t[i] == 'x' || t[i] == 'X' || t[i] == '(') return false;
  const char* s = copy_token(t, a, b, buf, sizeof(buf), big);
  if (!s) return false;
  const locale_t loc = c_numeric_locale();
  if (!loc) return false;
  char* end = nullptr;
  errno = 0;
  v = strtod_l(s, &end, loc);
  return end != s && *end == 0;
}

// An integer field as Python's int() reads it (sign, digits, underscores).
// Out of the int64 range: ``huge`` is set and v is unusable (int() still
// reads it, so the reference map -- -1 or not -- can be applied).
bool parse_int(const char* t, size_t a, size_t b, long long& v, bool& huge) {
  char buf[64];
  std::string big;
  const char* s = copy_token(t, a, b, buf, sizeof(buf), big);
  if (!s) return false;
  char* end = nullptr;
  errno = 0;
  v = std::strtoll(s, &end, 10);
  huge = errno == ERANGE;
  return end != s && *end == 0 && (errno == 0 || huge);
}

// Parse the rows of [a, b) into x[row0..], labels[row0..]; stops after
// max_rows rows.  Returns DAL_OK or an error code.
int parse_range(const char* t, size_t a, size_t b, int64_t row0, int64_t max_rows, int64_t cols, int label_map,
                float* x, int64_t* labels) {
  int64_t r = row0;
  size_t i = a;
  while (i < b && r < max_rows) {
    const size_t e = line_end(t, b, i);
    size_t p = i;
    int64_t f = 0;
    bool any = false;
    while (p < e) {
      while (p < e && is_space(t[p])) ++p;
      if (p >= e) break;
      size_t q = p;
      while (q < e && !is_space(t[q])) ++q;
      if (!any) any = true;
      if (f >= cols) return DAL_ERR_SHAPE;
      if (f < cols - 1) {
        double v;
        if (!parse_double(t, p, q, v)) return DAL_ERR_ARG;
        x[r * (cols - 1) + f] = static_cast<float>(v);
      } else {
        long long lab;
        bool huge = false;
        if (!parse_int(t, p, q, lab, huge)) return DAL_ERR_ARG;
        if (huge && label_map != 0) return DAL_ERR_ARG;  // an as-is label must fit int64
        labels[r] = label_map == 0 ? (!huge && lab == -1 ? 0 : 1) : lab;
      }
      ++f;
      p = q;
    }
    if (any) {
      if (f != cols) return DAL_ERR_SHAPE;
      ++r;
    }
    i = e + 1;
  }
  return DAL_OK;
}

}  // namespace

// Shape of a text byte range: rows (non-blank lines, at most max_rows if
// max_rows >= 0) and fields per row (of the first non-blank line; features =
// fields - 1).
extern "C" int dal_text_shape(const char* text, size_t len, int64_t max_rows, int64_t* rows, int64_t* cols) {
  if (!text || !rows || !cols) return DAL_ERR_ARG;
  int64_t r = 0, c = 0;
  size_t i = 0;
  while (i < len && (max_rows < 0 || r < max_rows)) {
    const size_t e = line_end(text, len, i);
    const int64_t f = count_fields(text, i, e);
    if (f > 0) {
      if (c == 0) c = f;
      ++r;
    }
    i = e + 1;
  }
  *rows = r;
  *cols = c;
  return DAL_OK;
}

// Parse the first ``rows`` non-blank rows of a text byte range into x
// [rows][cols - 1] fp32 and labels [rows] (label_map 0: the reference's
// ``0 if int(l) == -1 else 1``; 1: the integer label as is), with up to
// n_threads host threads.  Errors: DAL_ERR_SHAPE (a row with a different field
// count), DAL_ERR_ARG (a field that is not a number / a non-integer label).
extern "C" int dal_parse_labeled_text(const char* text, size_t len, int64_t rows, int64_t cols, int label_map,
                                      float* x, int64_t* labels, int n_threads) {
  if (!text || !x || !labels || (label_map != 0 && label_map != 1)) return DAL_ERR_ARG;
  if (rows < 0 || cols < 2) return DAL_ERR_SHAPE;
  if (rows == 0) return DAL_OK;
  int nt = n_threads < 1 ? 1 : (n_threads > 64 ? 64 : n_threads);
  if (len < static_cast<size_t>(nt) * 4096) nt = 1;
  std::vector<size_t> seg(nt + 1);
  seg[0] = 0;
  seg[nt] = len;
  for (int s = 1; s < nt; ++s) {
    const size_t p = line_start(text, len, len / nt * s);
    seg[s] = p < seg[s - 1] ? seg[s - 1] : p;
  }
  std::vector<int64_t> cnt(nt, 0);
  {
    std::vector<std::thread> th;
    for (int s = 0; s < nt; ++s)
      th.emplace_back([&, s] { cnt[s] = count_rows(text, seg[s], seg[s + 1]); });
    for (auto& t : th) t.join();
  }
  std::vector<int64_t> first(nt, 0);
  for (int s = 1; s < nt; ++s) first[s] = first[s - 1] + cnt[s - 1];
  if (first[nt - 1] + cnt[nt - 1] < rows) return DAL_ERR_SHAPE;
  std::vector<int> rc(nt, DAL_OK);
  {
    std::vector<std::thread> th;
    for (int s = 0; s < nt; ++s) {
      if (first[s] >= rows) break;
      th.emplace_back([&, s] { rc[s] = parse_range(text, seg[s], seg[s + 1], first[s], rows, cols, label_map, x, labels); });
    }
    for (auto& t : th) t.join();
  }
  for (int s = 0; s < nt; ++s)
    if (rc[s] != DAL_OK) return rc[s];
  return DAL_OK;
}
