// Gram operand preparation: every pool row L2-normalised (canonical fp64
// norm) and its fp32 unit row written at scale 2^12 as two fp16 terms,
//   H = fp16_rn(2^12 u),   L = fp16_rn(2^12 u - H)   (the difference is exact),
// so 2^12 u = H + L + e with |e| <= 2^-22 |2^12 u|; every product of two terms
// is exact in fp32 and lands in units of 2^-24.  Layout [n_pad][d_pad / KS]
// [KS H | KS L] with KS = split_ks(d_pad) (gram_sym.hip reads it).
//
// Reference: final_thesis/density_weighting.py:66 (``_/np.linalg.norm(_)``),
// cosine_similarity.py:28, similarity.py:28.

#include <stdlib.h>

#include "common.hpp"

namespace dal {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// fp32 unit rows -> two-term fp16 split, layout [n_pad][d_pad/KS][hi KS | lo KS].
// One thread per 8 features (one 16-B slot of hi and of lo).
__global__ __launch_bounds__(256) void split_f16_kernel(const float* __restrict__ u, int64_t n_pad,
                                                        int d_pad, int64_t ld, int ks,
                                                        uint16_t* __restrict__ out) {
  const int groups = d_pad / 8;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n_pad * groups) return;
  const int64_t row = t / groups;
  const int f0 = static_cast<int>(t % groups) * 8;
  const float4 v0 = *reinterpret_cast<const float4*>(u + row * ld + f0);
  const float4 v1 = *reinterpret_cast<const float4*>(u + row * ld + f0 + 4);
  const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  f16x8 h, l;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float sv = v[e] * 4096.0f;                 // exact
    const _Float16 he = static_cast<_Float16>(sv);
    const float r = sv - static_cast<float>(he);     // exact
    h[e] = he;
    l[e] = static_cast<_Float16>(r);
  }
  uint16_t* dst = out + row * (2 * static_cast<int64_t>(d_pad)) + (f0 / ks) * (2 * ks) + (f0 % ks);
  *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, h);
  *reinterpret_cast<uint4*>(dst + ks) = __builtin_bit_cast(uint4, l);
}

// Fused row L2-normalisation + split: x -> (norm64, H, L) without the fp32 unit
// rows in HBM (dal_normalize_rows + dal_split_f16 in one pass, same bits).
// Block = 64 rows: wave 0 forms the canonical sequential fp64 norms from an
// LDS tile; then every thread converts 8-feature groups (fp64 divide, fp32
// round, two-term split at scale 2^12) and writes one 16-B H and one 16-B L.
constexpr int kNsRows = 64;
__global__ __launch_bounds__(256) void normalize_split_kernel(
    const float* __restrict__ x, int64_t n, int d, int64_t ldx, const uint8_t* __restrict__ flags,
    int64_t n_pad, int d_pad, int ks, uint16_t* __restrict__ out, double* __restrict__ norm64,
    int32_t* __restrict__ status, long long* __restrict__ acc_zero) {
  __shared__ float tile[kNsRows][65];
  __shared__ double rnorm[kNsRows];
  const int tid = threadIdx.x;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kNsRows;
  // the density accumulator of these rows starts at zero (no separate fill)
  if (acc_zero && tid < kNsRows && row0 + tid < n_pad) acc_zero[row0 + tid] = 0;
  double n2 = 0.0;
  for (int c0 = 0; c0 < d; c0 += 64) {
    // 16 independent loads per thread, all in flight before the LDS writes
    float v[kNsRows * 64 / 256];
#pragma unroll
    for (int j = 0; j < kNsRows * 64 / 256; ++j) {
      const int e = tid + 256 * j, r = e / 64, c = e % 64;
      const int64_t row = row0 + r;
      v[j] = (row < n && c0 + c < d) ? x[row * ldx + c0 + c] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < kNsRows * 64 / 256; ++j) {
      const int e = tid + 256 * j;
      tile[e / 64][e % 64] = v[j];
    }
    __syncthreads();
    if (tid < kNsRows) {
      const int cmax = min(64, d - c0);
      for (int c = 0; c < cmax; ++c) {
        const double v = static_cast<double>(tile[tid][c]);
        n2 = n2 + v * v;  // -ffp-contract=off: mul then add (canonical order)
      }
    }
    if (c0 + 64 < d) __syncthreads();
  }
  if (tid < kNsRows) {
    const int64_t row = row0 + tid;
    const double nr = __builtin_sqrt(n2);
    if (row < n) {
      if (!(n2 > 0.0)) atomicOr(status, DAL_FLAG_ZERO_NORM);
      norm64[row] = nr;
    }
    rnorm[tid] = nr;
  }
  __syncthreads();
  const int groups = d_pad / 8;
  const bool from_tile = d <= 64;  // the tile still holds every feature
  for (int item = tid; item < kNsRows * groups; item += 256) {
    const int r = item / groups, f0 = (item % groups) * 8;
    const int64_t row = row0 + r;
    if (row >= n_pad) break;
    const bool live = row < n && !(flags && (flags[row] & DAL_ROW_EXCLUDED)) && rnorm[r] > 0.0;
    const double nr = rnorm[r];
    f16x8 h, l;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = f0 + e;
      float v = 0.0f;
      if (live && f < d) {
        const float xv = from_tile ? tile[r][f] : x[row * ldx + f];
        v = static_cast<float>(static_cast<double>(xv) / nr);
      }
      const float sv = v * 4096.0f;  // exact
      const _Float16 he = static_cast<_Float16>(sv);
      h[e] = he;
      l[e] = static_cast<_Float16>(sv - static_cast<float>(he));
    }
    uint16_t* dst = out + row * (2 * static_cast<int64_t>(d_pad)) + (f0 / ks) * (2 * ks) + (f0 % ks);
    *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, h);
    *reinterpret_cast<uint4*>(dst + ks) = __builtin_bit_cast(uint4, l);
  }
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" int64_t dal_split_f16_halves(int64_t n_pad, int64_t d_pad) { return n_pad * 2 * d_pad; }

extern "C" int dal_split_f16(const float* u, int64_t n_pad, int64_t d_pad, int64_t ld, uint16_t* out,
                             dal_stream_t stream) {
  if (!u || !out) return DAL_ERR_ARG;
  if (n_pad <= 0 || n_pad % DAL_ROW_GRANULE) return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad) || ld < d_pad || (ld % 4)) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(out)) & 15) return DAL_ERR_SHAPE;
  const int64_t threads = n_pad * (d_pad / 8);
  hipLaunchKernelGGL(split_f16_kernel, dim3(static_cast<unsigned>(ceil_div(threads, 256))), dim3(256), 0,
                     as_stream(stream), u, n_pad, static_cast<int>(d_pad), ld, split_ks(d_pad), out);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_canon_colsum_partials(const float* x, int64_t n, int64_t d, int64_t ldx, const double* norm64,
                                         const uint8_t* row_flags, double* partials, dal_stream_t stream);

extern "C" int dal_prep_split(const float* x, int64_t n, int64_t d, int64_t ldx, const uint8_t* row_flags,
                              int64_t n_pad, int64_t d_pad, uint16_t* out, double* norm64, double* partials,
                              int64_t* acc_zero, int32_t* dev_status, dal_stream_t stream) {
  if (!x || !out || (!norm64 && n) || !dev_status) return DAL_ERR_ARG;
  if (n < 0 || d < 1 || ldx < d || n_pad < n || n_pad % DAL_ROW_GRANULE || d > (1 << 20)) return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad) || d_pad < d) return DAL_ERR_SHAPE;
  if (reinterpret_cast<uintptr_t>(out) & 15) return DAL_ERR_SHAPE;
  // two launches: a single-chunk-per-block fused form measured slower (65 us
  // vs 21 + 29 us at 100k x 64: too few blocks for the sequential chains)
  hipLaunchKernelGGL(normalize_split_kernel, dim3(static_cast<unsigned>(ceil_div(n_pad, kNsRows))), dim3(256), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ldx, row_flags, n_pad, static_cast<int>(d_pad),
                     split_ks(d_pad), out, norm64, dev_status, reinterpret_cast<long long*>(acc_zero));
  DAL_RETURN_IF_LAUNCH_FAILED();
  if (partials && n > 0) return dal_canon_colsum_partials(x, n, d, ldx, norm64, row_flags, partials, stream);
  return DAL_OK;
}

