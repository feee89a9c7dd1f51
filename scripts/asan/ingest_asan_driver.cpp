// Host AddressSanitizer / UBSan driver of the pool-ingest parser
// (csrc/ingest.hip: dal_text_shape + dal_parse_labeled_text), SURVEY §5.
//
// The Python loader (dal/ingest.py _load) cannot run under ASan (python is not
// instrumented), so this driver repeats its host logic in C++ against an
// instrumented build of the parser: the file is read into a heap buffer of
// EXACTLY its size (ASan's redzone right behind the last byte: any read past a
// chunk or the file end is reported), cut into ~chunk_bytes ranges at line
// starts, shaped per chunk, then parsed per chunk with n_threads threads.
//
//   ingest_asan_driver FILE MAX_ROWS LABEL_MAP N_THREADS CHUNK_BYTES OUT_X OUT_Y
//
// Prints "rc=<status> rows=<r> cols=<c>"; rc 100 = the loader's own
// ValueErrors (rows of different field counts across chunks, no rows, fewer
// than two fields).  OUT_X: fp32 [rows][cols-1], OUT_Y: int64 [rows].
// Reference: final_thesis/uncertainty_sampling.py:37-42,
// density_weighting.py:45-53,59-65.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "dal.h"

int main(int argc, char** argv) {
  if (argc != 8) {
    std::fprintf(stderr, "usage: %s FILE MAX_ROWS LABEL_MAP N_THREADS CHUNK_BYTES OUT_X OUT_Y\n", argv[0]);
    return 2;
  }
  const int64_t max_rows = std::strtoll(argv[2], nullptr, 10);
  const int label_map = std::atoi(argv[3]);
  const int n_threads = std::atoi(argv[4]);
  const size_t chunk = static_cast<size_t>(std::strtoull(argv[5], nullptr, 10));
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::fseek(f, 0, SEEK_END);
  const long size = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (size <= 0) {
    std::printf("rc=100 rows=0 cols=0\n");
    return 0;
  }
  char* buf = static_cast<char*>(std::malloc(static_cast<size_t>(size)));  // exact size: no terminator
  if (std::fread(buf, 1, static_cast<size_t>(size), f) != static_cast<size_t>(size)) return 2;
  std::fclose(f);
  const size_t n = static_cast<size_t>(size);

  struct Piece {
    size_t a, b;
    int64_t r0, r;
  };
  std::vector<Piece> plan;
  int64_t total = 0, cols = -1;
  int rc = 0;
  for (size_t a = 0; a < n;) {  // dal/ingest.py _chunks: ranges end after a newline
    size_t b = a + chunk < n ? a + chunk : n;
    if (b < n) {
      const void* nl = std::memchr(buf + b, '\n', n - b);
      b = nl ? static_cast<size_t>(static_cast<const char*>(nl) - buf) + 1 : n;
    }
    if (max_rows >= 0 && total >= max_rows) break;
    int64_t r = 0, c = 0;
    rc = dal_text_shape(buf + a, b - a, max_rows < 0 ? -1 : max_rows - total, &r, &c);
    if (rc) break;
    if (r > 0) {
      if (cols < 0) cols = c;
      else if (c != cols) {
        rc = 100;
        break;
      }
      plan.push_back({a, b, total, r});
      total += r;
    }
    a = b;
  }
  if (!rc && (plan.empty() || cols < 2)) rc = 100;
  std::vector<float> x;
  std::vector<int64_t> y;
  if (!rc) {
    const int64_t d = cols - 1;
    x.resize(static_cast<size_t>(total * d));
    y.resize(static_cast<size_t>(total));
    for (const Piece& p : plan) {
      rc = dal_parse_labeled_text(buf + p.a, p.b - p.a, p.r, cols, label_map, x.data() + p.r0 * d,
                                  y.data() + p.r0, n_threads);
      if (rc) break;
    }
  }
  std::free(buf);
  std::printf("rc=%d rows=%lld cols=%lld\n", rc, static_cast<long long>(rc ? 0 : total),
              static_cast<long long>(cols));
  if (!rc) {
    FILE* fx = std::fopen(argv[6], "wb");
    FILE* fy = std::fopen(argv[7], "wb");
    if (!fx || !fy) return 2;
    std::fwrite(x.data(), sizeof(float), x.size(), fx);
    std::fwrite(y.data(), sizeof(int64_t), y.size(), fy);
    std::fclose(fx);
    std::fclose(fy);
  }
  return 0;
}
