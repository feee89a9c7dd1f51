// Shared device helpers for libdal (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dal.h"

#define DAL_RETURN_IF_LAUNCH_FAILED()                 \
  do {                                                \
    if (hipGetLastError() != hipSuccess) return DAL_ERR_HIP; \
  } while (0)

namespace dal {

constexpr int kWave = 64;

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

inline hipStream_t as_stream(dal_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Order-preserving map of an fp64 score to a uint64 key, smaller = better.
// -0.0 and +0.0 share a key (the reference compares them equal); NaN sorts
// after every number (DAL_KEY_NAN) in either direction.
__device__ __forceinline__ uint64_t score_key(double s, int order) {
  if (s != s) return DAL_KEY_NAN;
  if (s == 0.0) s = 0.0;  // -0.0 -> +0.0
  const uint64_t b = static_cast<uint64_t>(__double_as_longlong(s));
  const uint64_t u = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  return order == DAL_DESCENDING ? ~u : u;
}

// The half-width of a score's uncertainty interval for the density path:
// |lut[v]| * err_d, and the interval's pessimistic / optimistic ends.
__device__ __forceinline__ double pessimistic(double s, double e, int order) {
  return order == DAL_DESCENDING ? __dadd_rn(s, -e) : __dadd_rn(s, e);
}
__device__ __forceinline__ double optimistic(double s, double e, int order) {
  return order == DAL_DESCENDING ? __dadd_rn(s, e) : __dadd_rn(s, -e);
}

// fp32 -> int64 fixed point (scale 2^32), round to nearest even.  Exact
// integer accumulation afterwards makes the density independent of the
// order in which partial sums arrive.
__device__ __forceinline__ long long to_fixed(float v) {
  return static_cast<long long>(__builtin_rint(static_cast<double>(v) * DAL_FIXED_SCALE));
}

__device__ __forceinline__ double from_fixed(long long a) {
  return static_cast<double>(a) * (1.0 / DAL_FIXED_SCALE);
}

}  // namespace dal
