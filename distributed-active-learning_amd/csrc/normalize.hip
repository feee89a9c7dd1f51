// Row L2 normalisation and the canonical fp64 column sum.
//
// Reference: final_thesis/density_weighting.py:66 (``_/np.linalg.norm(_)``),
// cosine_similarity.py:28, similarity.py:28; exclusion of L0 as column j:
// density_weighting.py:95-100.
//
// HBM-bound O(N*D) passes.  The fp64 arithmetic here is the canonical
// definition the selected set is bit-exact to, so the library is built with
// -ffp-contract=off: every multiply and add rounds separately, in the order
// the oracle uses (sequential over features / rows).
#include <cstdlib>

#include <algorithm>

#include "common.hpp"

namespace dal {
namespace {

constexpr int kNormRows = 64;    // rows per block (one per lane of wave 0)
constexpr int kNormCols = 64;    // feature columns staged per step
constexpr int kNormThreads = 256;

// One block normalises 64 rows.  Pass 1 stages 64x64 tiles through LDS with
// coalesced loads so that lane r can sum row r sequentially over features
// (canonical order); pass 2 writes the fp32 unit rows (coalesced) and the
// zero padding.
__global__ __launch_bounds__(kNormThreads) void normalize_rows_kernel(
    const float* __restrict__ x, int64_t n, int d, int64_t ldx, const uint8_t* __restrict__ flags,
    int64_t n_pad, int d_pad, float* __restrict__ u, double* __restrict__ norm64,
    int32_t* __restrict__ status) {
  __shared__ float tile[kNormRows][kNormCols + 1];
  __shared__ double rnorm[kNormRows];
  const int tid = threadIdx.x;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kNormRows;
  double n2 = 0.0;
  for (int c0 = 0; c0 < d; c0 += kNormCols) {
    // coalesced load: 256 threads = 4 rows x 64 columns per step
    for (int e = tid; e < kNormRows * kNormCols; e += kNormThreads) {
      const int r = e / kNormCols, c = e % kNormCols;
      const int64_t row = row0 + r;
      float v = 0.0f;
      if (row < n && c0 + c < d) v = x[row * ldx + c0 + c];
      tile[r][c] = v;
    }
    __syncthreads();
    if (tid < kNormRows) {
      const int cmax = min(kNormCols, d - c0);
      for (int c = 0; c < cmax; ++c) {
        const double v = static_cast<double>(tile[tid][c]);
        n2 = n2 + v * v;  // -ffp-contract=off: mul then add
      }
    }
    __syncthreads();
  }
  if (tid < kNormRows) {
    const int64_t row = row0 + tid;
    double nr = __builtin_sqrt(n2);
    if (row < n) {
      if (!(n2 > 0.0)) atomicOr(status, DAL_FLAG_ZERO_NORM);
      if (norm64) norm64[row] = nr;
    }
    rnorm[tid] = nr;
  }
  __syncthreads();
  for (int r = tid / kWave; r < kNormRows; r += kNormThreads / kWave) {
    const int64_t row = row0 + r;
    if (row >= n_pad) break;
    const bool live = row < n && !(flags && (flags[row] & DAL_ROW_EXCLUDED));
    const double nr = rnorm[r];
    float* urow = u + row * d_pad;
    for (int c = tid % kWave; c < d_pad; c += kWave) {
      float v = 0.0f;
      if (live && c < d && nr > 0.0) v = static_cast<float>(static_cast<double>(x[row * ldx + c]) / nr);
      urow[c] = v;
    }
  }
}

// partials[c][f] = sum_{r in chunk c, not excluded} x_rf / norm64[r]
// (sequential over the chunk's rows).  Two kernels, the same bits:
//  * many chunks (config 4): one wave per (chunk, 64 features), lane =
//    feature, so every row's features are one coalesced load; the chunk goes
//    in batches of kColBatch rows, lane j of a batch also loading row j's norm
//    and flag, broadcast to the wave for the in-order divisions and adds;
//  * few chunks (configs 2, 3): a block per (chunk, 8 features), all 256
//    threads forming the quotients into an fp64 LDS tile, then 8 lanes adding
//    the 256 rows in order -- more waves for the same work (the wave kernel:
//    100k x 64 43 -> 109 us, 284,807 x 30 55 -> 125 us for the whole prep).
// The block kernel alone: 1.72 ms at config 4, the wave kernel 1.49 ms (fp64
// VALU bound: ~21 instructions per row and wave; the 2 GB are fetched once).
// Markstein's reciprocal division (3 fp64 operations per element in place of
// the division sequence) measured no faster in either kernel and is not used.
constexpr int kColBatch = 32;
#ifndef DAL_COLSUM_WAVE_MIN
#define DAL_COLSUM_WAVE_MIN 8192  // waves (chunks x 64-feature groups) from which the wave kernel runs
#endif

__global__ __launch_bounds__(256) void canon_colsum_wave_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                int64_t ldx, const double* __restrict__ norm64,
                                                                const uint8_t* __restrict__ flags,
                                                                double* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int fgroups = (d + 63) / 64;
  const int64_t c = wave / fgroups;
  const int f = static_cast<int>(wave % fgroups) * 64 + lane;
  const int64_t chunks = (n + DAL_CANON_CHUNK - 1) / DAL_CANON_CHUNK;
  if (c >= chunks) return;  // (whole waves)
  const bool lf = f < d;
  // Excluded / padding rows contribute +0.0: the running sum starts at +0.0
  // and can never become -0.0, so adding +0.0 is bit-identical to skipping.
  double acc = 0.0;
#pragma unroll 1
  for (int64_t rb = c * DAL_CANON_CHUNK; rb < (c + 1) * DAL_CANON_CHUNK; rb += kColBatch) {
    float xv[kColBatch];
#pragma unroll
    for (int j = 0; j < kColBatch; ++j) xv[j] = (lf && rb + j < n) ? x[(rb + j) * ldx + f] : 0.0f;
    const int64_t rl = rb + lane;
    const bool in = lane < kColBatch && rl < n;
    const double nl = in ? norm64[rl] : 1.0;
    const uint64_t nb = __builtin_bit_cast(uint64_t, nl);
    const uint64_t live = __ballot(in && !(flags && (flags[rl] & DAL_ROW_EXCLUDED)));
    const int nlo = static_cast<int>(static_cast<uint32_t>(nb)), nhi = static_cast<int>(static_cast<uint32_t>(nb >> 32));
#pragma unroll
    for (int j = 0; j < kColBatch; ++j) {
      const double nj = __builtin_bit_cast(
          double, static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(nlo, j))) |
                      (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(nhi, j))) << 32));
      const double u = ((live >> j) & 1) ? static_cast<double>(xv[j]) / nj : 0.0;
      acc = acc + u;
    }
  }
  if (lf) partials[c * d + f] = acc;
}

constexpr int kColFeat = 8;  // features per block of the few-chunks kernel
__global__ __launch_bounds__(256) void canon_colsum_block_kernel(const float* __restrict__ x, int64_t n, int d,
                                                                 int64_t ldx, const double* __restrict__ norm64,
                                                                 const uint8_t* __restrict__ flags,
                                                                 double* __restrict__ partials) {
  __shared__ double u[DAL_CANON_CHUNK][kColFeat];
  __shared__ double sn[DAL_CANON_CHUNK];
  __shared__ uint8_t sl[DAL_CANON_CHUNK];
  const int tid = threadIdx.x;
  const int fl = tid % kColFeat, rs = tid / kColFeat;
  const int64_t c = blockIdx.x;
  const int f = blockIdx.y * kColFeat + fl;
  constexpr int kRowsPerPass = 256 / kColFeat;
  constexpr int kPer = DAL_CANON_CHUNK / kRowsPerPass;
  // every thread: one row's norm and liveness; its kPer features
  // loaded meanwhile (all in flight)
  static_assert(DAL_CANON_CHUNK == 256, "one row per thread");
  {
    const int64_t r = c * DAL_CANON_CHUNK + tid;
    const double nr = r < n ? norm64[r] : 1.0;
    sn[tid] = nr;
    sl[tid] = r < n && !(flags && (flags[r] & DAL_ROW_EXCLUDED));
  }
  float xv[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t r = c * DAL_CANON_CHUNK + rs + k * kRowsPerPass;
    xv[k] = (r < n && f < d) ? x[r * ldx + f] : 0.0f;
  }
  __syncthreads();
  // Excluded / padding rows contribute +0.0: the running sum starts at +0.0
  // and can never become -0.0, so adding +0.0 is bit-identical to skipping.
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int rl = rs + k * kRowsPerPass;
    u[rl][fl] = (sl[rl] && f < d) ? static_cast<double>(xv[k]) / sn[rl] : 0.0;
  }
  __syncthreads();
  if (tid >= kColFeat || f >= d) return;
  double acc = 0.0;
#pragma unroll 32
  for (int rl = 0; rl < DAL_CANON_CHUNK; ++rl) acc = acc + u[rl][tid];
  partials[c * d + f] = acc;
}

// Separable canonical density for every row: d_i = sum_f (x_if / norm64[i]) *
// s_f, sequential over f (the same fp64 operation order as the re-rank and the
// oracle, so every bit matches); NaN for excluded rows.  64 rows per block:
// tiles of 64 features staged through LDS with coalesced loads, lane r owns row r.
__global__ __launch_bounds__(256) void density_separable_kernel(
    const float* __restrict__ x, int64_t n, int d, int64_t ldx, const double* __restrict__ norm64,
    const double* __restrict__ colsum, const uint8_t* __restrict__ flags, double* __restrict__ dens) {
  __shared__ float tile[64][65];
  __shared__ double sv[64];
  const int tid = threadIdx.x;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * 64;
  const int64_t row = row0 + tid;
  const double nr = (tid < 64 && row < n) ? norm64[row] : 1.0;
  double acc = 0.0;
  for (int c0 = 0; c0 < d; c0 += 64) {
    for (int e = tid; e < 64 * 64; e += 256) {
      const int r = e / 64, c = e % 64;
      const int64_t rr = row0 + r;
      tile[r][c] = (rr < n && c0 + c < d) ? x[rr * ldx + c0 + c] : 0.0f;
    }
    if (tid < 64) sv[tid] = c0 + tid < d ? colsum[c0 + tid] : 0.0;
    __syncthreads();
    if (tid < 64) {
      const int cmax = min(64, d - c0);
      for (int c = 0; c < cmax; ++c) acc = acc + (static_cast<double>(tile[tid][c]) / nr) * sv[c];
    }
    __syncthreads();
  }
  if (tid < 64 && row < n) {
    if (flags && (flags[row] & DAL_ROW_EXCLUDED)) acc = __builtin_nan("");
    dens[row] = acc;
  }
}

// s[f] = sum_c partials[c][f], sequential over c; loads batched 32 deep.
constexpr int kRedFeat = 32;     // features per reduce block
constexpr int kRedTile = 512;    // chunks staged in LDS per pass (128 KiB)
__global__ __launch_bounds__(256) void canon_colsum_reduce_kernel(const double* __restrict__ partials,
                                                                  int64_t n_chunks, int d,
                                                                  double* __restrict__ s) {
  // all 256 threads stage a tile of partials in LDS (many loads in flight),
  // then kRedFeat lanes add the chunks in order
  __shared__ double t[kRedTile][kRedFeat];
  const int tid = threadIdx.x;
  const int f0 = blockIdx.x * kRedFeat;
  double acc = 0.0;
  for (int64_t c0 = 0; c0 < n_chunks; c0 += kRedTile) {
    const int m = static_cast<int>(n_chunks - c0 < kRedTile ? n_chunks - c0 : kRedTile);
    // staging: batches of 16 independent loads per thread (latency overlapped)
    for (int e0 = 0; e0 < m * kRedFeat; e0 += 256 * 16) {
      double v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int e = e0 + j * 256 + tid;
        const int ci = e / kRedFeat, fl = e % kRedFeat;
        v[j] = (e < m * kRedFeat && f0 + fl < d) ? partials[(c0 + ci) * d + f0 + fl] : 0.0;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int e = e0 + j * 256 + tid;
        if (e < m * kRedFeat) t[e / kRedFeat][e % kRedFeat] = v[j];
      }
    }
    __syncthreads();
    if (tid < kRedFeat) {
      int ci = 0;
      for (; ci + 8 <= m; ci += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc = acc + t[ci + i][tid];
      }
      for (; ci < m; ++ci) acc = acc + t[ci][tid];
    }
    __syncthreads();
  }
  if (tid < kRedFeat && f0 + tid < d) s[f0 + tid] = acc;
}

__global__ __launch_bounds__(256) void mark_rows_kernel(const int64_t* __restrict__ idx, int64_t count,
                                                        int64_t row_base, int64_t n, unsigned bits,
                                                        uint8_t* __restrict__ flags) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= count) return;
  const int64_t r = idx[t] - row_base;
  if (r >= 0 && r < n) flags[r] |= static_cast<uint8_t>(bits);  // duplicates write the same value
}

// The same marking, grid-stride over a bounded grid, counting the indices that
// fall inside the shard (one atomic per block: the same-address atomics bound
// it -- 8192 256-thread blocks measured 100 us at 8M indices, 2048 40 us, 512
// 47 us -- so the blocks are 1,024 threads, at most 512 of them).
constexpr int kMarkThreads = 1024;
__global__ __launch_bounds__(kMarkThreads) void mark_rows_count_kernel(const int64_t* __restrict__ idx, int64_t count,
                                                              int64_t row_base, int64_t n, unsigned bits,
                                                              uint8_t* __restrict__ flags,
                                                              int32_t* __restrict__ in_range) {
  int c = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kMarkThreads;
  // 4 index loads in flight per thread before the flag writes
  for (int64_t t0 = static_cast<int64_t>(blockIdx.x) * kMarkThreads + threadIdx.x; t0 < count; t0 += 4 * stride) {
    int64_t r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t t = t0 + j * stride;
      r[j] = t < count ? idx[t] - row_base : -1;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (r[j] >= 0 && r[j] < n) {
        flags[r[j]] |= static_cast<uint8_t>(bits);
        ++c;
      }
    }
  }
  __shared__ int part[kMarkThreads / 64];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int b = 0;
    for (int w = 0; w < kMarkThreads / 64; ++w) b += part[w];
    if (b) atomicAdd(in_range, b);
  }
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" int dal_mark_rows_count(const int64_t* idx, int64_t count, int64_t row_base, int64_t n, int bits,
                                   uint8_t* flags, int32_t* in_range, dal_stream_t stream) {
  if ((!idx && count) || !flags || !in_range) return DAL_ERR_ARG;
  if (count < 0 || n < 0 || count > INT32_MAX) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  if (hipMemsetAsync(in_range, 0, sizeof(int32_t), st) != hipSuccess) return DAL_ERR_HIP;
  if (count == 0) return DAL_OK;
  const int64_t blocks = std::min<int64_t>(ceil_div(count, kMarkThreads), 512);
  hipLaunchKernelGGL(mark_rows_count_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kMarkThreads), 0, st, idx, count,
                     row_base, n, static_cast<unsigned>(bits), flags, in_range);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_mark_rows(const int64_t* idx, int64_t count, int64_t row_base, int64_t n, int bits,
                             uint8_t* flags, dal_stream_t stream) {
  if ((!idx && count) || !flags) return DAL_ERR_ARG;
  if (count < 0 || n < 0) return DAL_ERR_SHAPE;
  if (count == 0) return DAL_OK;
  hipLaunchKernelGGL(mark_rows_kernel, dim3(static_cast<unsigned>(ceil_div(count, 256))), dim3(256), 0,
                     as_stream(stream), idx, count, row_base, n, static_cast<unsigned>(bits), flags);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int64_t dal_pad_rows(int64_t n) { return round_up(n < 1 ? 1 : n, DAL_ROW_GRANULE); }

extern "C" int64_t dal_pad_features(int64_t d) {
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  if (d <= 128) return 128;
  return round_up(d, 256);
}

extern "C" int dal_normalize_rows(const float* x, int64_t n, int64_t d, int64_t ldx,
                                  const uint8_t* row_flags, int64_t n_pad, int64_t d_pad, float* u,
                                  double* norm64, int32_t* dev_status, dal_stream_t stream) {
  if (!x || !u || !dev_status) return DAL_ERR_ARG;
  if (n < 0 || d < 1 || ldx < d || n_pad < n || d_pad < d || d > (1 << 20)) return DAL_ERR_SHAPE;
  if (n_pad == 0) return DAL_OK;
  const int64_t blocks = ceil_div(n_pad, kNormRows);
  hipLaunchKernelGGL(normalize_rows_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kNormThreads), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ldx, row_flags, n_pad,
                     static_cast<int>(d_pad), u, norm64, dev_status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_canon_colsum_partials(const float* x, int64_t n, int64_t d, int64_t ldx,
                                         const double* norm64, const uint8_t* row_flags,
                                         double* partials, dal_stream_t stream) {
  if (!x || !norm64 || !partials) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ldx < d) return DAL_ERR_SHAPE;
  const int64_t chunks = ceil_div(n, DAL_CANON_CHUNK), waves = chunks * ceil_div(d, 64);
  if (waves >= DAL_COLSUM_WAVE_MIN) {
    hipLaunchKernelGGL(canon_colsum_wave_kernel, dim3(static_cast<unsigned>(ceil_div(waves, 4))), dim3(256), 0,
                       as_stream(stream), x, n, static_cast<int>(d), ldx, norm64, row_flags, partials);
  } else {
    hipLaunchKernelGGL(canon_colsum_block_kernel,
                       dim3(static_cast<unsigned>(chunks), static_cast<unsigned>(ceil_div(d, kColFeat))), dim3(256), 0,
                       as_stream(stream), x, n, static_cast<int>(d), ldx, norm64, row_flags, partials);
  }
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_density_separable(const float* x, int64_t n, int64_t d, int64_t ldx, const double* norm64,
                                     const double* colsum, const uint8_t* row_flags, double* density,
                                     dal_stream_t stream) {
  if (!x || !norm64 || !colsum || !density) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ldx < d) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(density_separable_kernel, dim3(static_cast<unsigned>(ceil_div(n, 64))), dim3(256), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ldx, norm64, colsum, row_flags, density);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_canon_colsum_reduce(const double* partials, int64_t n_chunks, int64_t d,
                                       double* colsum, dal_stream_t stream) {
  if (!partials || !colsum) return DAL_ERR_ARG;
  if (n_chunks < 1 || d < 1) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(canon_colsum_reduce_kernel, dim3(static_cast<unsigned>(ceil_div(d, kRedFeat))),
                     dim3(256), 0, as_stream(stream), partials, n_chunks, static_cast<int>(d),
                     colsum);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
