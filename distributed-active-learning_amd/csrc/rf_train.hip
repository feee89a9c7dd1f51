// Random-forest training on the GPU.
//
// Reference: the per-iteration model fit
//   RandomForest.trainClassifier(train, numClasses=2, categoricalFeaturesInfo={},
//                                numTrees=T, featureSubsetStrategy="auto",
//                                impurity='gini', maxDepth=4, maxBins=32)
//   final_thesis/uncertainty_sampling.py:71-76, density_weighting.py:119-124
// whose arithmetic is Apache Spark 2.1.0 MLlib (not vendored).  Restated for
// continuous features and binary labels (oracle/rf_oracle.py holds the CPU
// restatement with the algorithm's steps):
//   * candidate thresholds per feature: findSplitsForContinuousFeature
//     (distinct sorted values; all of them if few, else the stride rule);
//   * bins: #{thresholds < x} (Arrays.binarySearch), split k: bin <= k left;
//   * level-wise growth: weighted class histograms per (node, feature, bin),
//     Gini gain in fp64 in MLlib's operation order, first maximum over the
//     node's features (subset order) and splits (index order), leaf when
//     gain <= 0 or at maxDepth, children preset as leaves when pure.
// The bootstrap weights (Poisson counts) and per-node feature subsets come in
// from the caller (MLlib draws them from JVM RNGs that cannot be reproduced),
// so the result is deterministic and comparable with the oracle bit for bit.
//
// MI355X design: the training set of an AL iteration is the labeled window
// (10..~10^4 rows) -- small, so the work is latency- not bandwidth-bound and
// the design minimises launches: one block per feature sorts its sample in
// LDS (bitonic) and emits the thresholds with block-wide first-index
// searches; per level ONE histogram kernel (route rows from the previous
// level's decision + integer LDS atomics, flushed once per block: weights are
// integers, so the histograms are exact and order-free) and ONE split kernel
// (a wave per node: per-slot prefix sums in LDS, every (feature, split) gain
// in fp64, lexicographic first-max wave reduction).
#include <algorithm>
#include <cfloat>
#include <climits>

#include "common.hpp"

namespace dal {
namespace {

constexpr int kSortThreads = 1024;
constexpr uint8_t kAbsent = 0, kOpen = 1, kLeaf = 2;

__device__ __forceinline__ double gini2(int64_t c0, int64_t c1) {
  const double total = static_cast<double>(c0) + static_cast<double>(c1);
  if (total == 0.0) return 0.0;
  double imp = 1.0;
  const double f0 = static_cast<double>(c0) / total;
  imp -= f0 * f0;
  const double f1 = static_cast<double>(c1) / total;
  imp -= f1 * f1;
  return imp;
}

// calculateImpurityStats (MLlib 2.1): -DBL_MAX marks an invalid split.
__device__ __forceinline__ double split_gain(int64_t l0, int64_t l1, int64_t r0, int64_t r1, double parent_imp,
                                             int min_instances, double min_gain, double* li_out,
                                             double* ri_out) {
  const int64_t lc = l0 + l1, rc = r0 + r1;
  if (lc < min_instances || rc < min_instances) return -DBL_MAX;
  const int64_t tc = lc + rc;
  const double li = gini2(l0, l1), ri = gini2(r0, r1);
  const double lw = static_cast<double>(lc) / static_cast<double>(tc);
  const double rw = static_cast<double>(rc) / static_cast<double>(tc);
  const double gain = parent_imp - lw * li - rw * ri;
  if (gain < min_gain) return -DBL_MAX;
  *li_out = li;
  *ri_out = ri;
  return gain;
}

__device__ __forceinline__ int block_min_int(int v, int* red) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int m = INT_MAX;
    for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) m = min(m, red[i]);
    red[0] = m;
  }
  __syncthreads();
  const int r = red[0];
  __syncthreads();
  return r;
}

// One block per feature: sort the sample column, find the distinct values and
// their cumulative counts, emit the thresholds (findSplitsForContinuousFeature).
__global__ __launch_bounds__(kSortThreads) void rf_find_splits_kernel(
    const float* __restrict__ x, int64_t n, int d, int64_t ldx, const int64_t* __restrict__ sample_rows,
    int n_s, int pow2, int num_splits, float* __restrict__ thresholds, int32_t* __restrict__ n_splits,
    int32_t* dev_status) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s = reinterpret_cast<float*>(smem);                  // [pow2] sorted sample
  int* pos = reinterpret_cast<int*>(smem + pow2 * 4);         // [n_s] first position of distinct j
  int* red = pos + n_s;                                       // [32] scan / reduction scratch
  const int f = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < pow2; i += kSortThreads) {
    float v = __builtin_inff();
    if (i < n_s) {
      const int64_t r = sample_rows ? sample_rows[i] : i;
      v = x[r * ldx + f];
    }
    s[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= pow2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < pow2; i += kSortThreads) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float a = s[i], b = s[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            s[i] = b;
            s[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // distinct heads: each thread owns a contiguous chunk, block exclusive scan
  const int chunk = (n_s + kSortThreads - 1) / kSortThreads;
  const int i0 = min(tid * chunk, n_s), i1 = min(i0 + chunk, n_s);
  int cnt = 0;
  for (int i = i0; i < i1; ++i) cnt += (i == 0 || s[i] != s[i - 1]);
  // wave-inclusive scan, then across the 16 waves
  int incl = cnt;
  const int lane = tid & 63, w = tid >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) red[w] = incl;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int q = 0; q < kSortThreads / 64; ++q) {
      const int c = red[q];
      red[q] = run;
      run += c;
    }
    red[kSortThreads / 64] = run;
  }
  __syncthreads();
  int j = red[w] + incl - cnt;
  const int n_distinct = red[kSortThreads / 64];
  for (int i = i0; i < i1; ++i)
    if (i == 0 || s[i] != s[i - 1]) pos[j++] = i;
  __syncthreads();
  float* out = thresholds + static_cast<int64_t>(f) * DAL_RF_MAX_SPLITS;
  if (n_distinct <= num_splits) {
    for (int q = tid; q < n_distinct; q += kSortThreads) out[q] = s[pos[q]];
    if (tid == 0) n_splits[f] = n_distinct;
    return;
  }
  // stride rule: the next threshold is uniq[j-1] for the first j >= start with
  // |cum[j-1] - target| < |cum[j] - target|; cum[j] = values <= uniq[j]
  const double stride = static_cast<double>(n_s) / static_cast<double>(num_splits + 1);
  double target = stride;
  int start = 1, emitted = 0;
  const int cap = min(num_splits + 1, DAL_RF_MAX_SPLITS);
  while (true) {
    int found = INT_MAX;
    for (int q = start + tid; q < n_distinct; q += kSortThreads) {
      const int prev = pos[q];                                  // cum[q-1]
      const int cur = q + 1 < n_distinct ? pos[q + 1] : n_s;    // cum[q]
      if (fabs(static_cast<double>(prev) - target) < fabs(static_cast<double>(cur) - target)) {
        found = q;
        break;
      }
    }
    found = block_min_int(found, red);
    if (found == INT_MAX) break;
    if (emitted == cap) {
      if (tid == 0) atomicOr(dev_status, DAL_FLAG_RF_SPLITS);
      break;
    }
    if (tid == 0) out[emitted] = s[pos[found - 1]];
    ++emitted;
    target += stride;
    start = found + 1;
  }
  if (tid == 0) n_splits[f] = emitted;
}

// bins[i][f] = #{thresholds_f < x[i][f]} (lower bound; an equal threshold
// gives its own index, as Arrays.binarySearch does).
__global__ void rf_bin_kernel(const float* __restrict__ x, int64_t n, int d, int64_t ldx,
                              const float* __restrict__ thresholds, const int32_t* __restrict__ n_splits,
                              uint8_t* __restrict__ bins) {
  const int64_t total = n * d;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t i = e / d;
    const int f = static_cast<int>(e - i * d);
    const float v = x[i * ldx + f];
    const float* t = thresholds + static_cast<int64_t>(f) * DAL_RF_MAX_SPLITS;
    int lo = 0, hi = n_splits[f];
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    bins[e] = static_cast<uint8_t>(lo);
  }
}

struct RfArgs {
  const uint8_t* bins;     // [n][d]
  const uint8_t* labels;   // [n]
  const int32_t* weights;  // [T][n]
  const int32_t* subsets;  // [T][n_inner][m]
  const float* thresholds;
  const int32_t* n_splits;
  int64_t n;
  int d, m, T, max_depth, hb, kmax;
  int min_instances;
  double min_gain;
  int32_t* node;       // [T][n] heap index at the previous level (-1 settled)
  uint8_t* status;     // [T][n_all]
  int32_t* split_f;    // [T][n_inner]
  int32_t* split_b;    // [T][n_inner]
  int32_t* hist;       // [T][2^l][m][hb][2] for the current level
  int32_t* cls;        // [T][2^l][2]
  int32_t* out_inner;  // [T][n_inner][2]
  uint8_t* out_leaf;   // [T][n_leaf]
};

// Route every (tree, row) of positive weight from level l-1 to level l, and
// accumulate the class counts of every live node and the (feature, bin, class)
// histograms of the open ones.
__global__ __launch_bounds__(256) void rf_hist_kernel(RfArgs A, int level, int rows_per_block, bool lds_hist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = blockIdx.y;
  const int nodes = 1 << level;
  const int first = nodes - 1;
  const int n_inner = (1 << A.max_depth) - 1;
  const int n_all = 2 * n_inner + 1;
  int* cls_s = reinterpret_cast<int*>(smem);
  int* hist_s = cls_s + 2 * nodes;
  const int hist_n = lds_hist ? nodes * A.m * A.hb * 2 : 0;
  for (int e = threadIdx.x; e < 2 * nodes + hist_n; e += blockDim.x) cls_s[e] = 0;
  __syncthreads();
  int32_t* ghist = A.hist + static_cast<int64_t>(t) * nodes * A.m * A.hb * 2;
  const uint8_t* st = A.status + static_cast<int64_t>(t) * n_all;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(A.n, r0 + rows_per_block);
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    const int w = A.weights[static_cast<int64_t>(t) * A.n + i];
    if (w <= 0) continue;
    int32_t* nd = A.node + static_cast<int64_t>(t) * A.n + i;
    int h = 0;
    if (level > 0) {
      const int hp = *nd;
      if (hp < 0) continue;
      const int f = A.split_f[static_cast<int64_t>(t) * n_inner + hp];
      if (f < 0) {  // the row's node became a leaf
        *nd = -1;
        continue;
      }
      const int b = A.bins[i * A.d + f];
      h = 2 * hp + 1 + (b > A.split_b[static_cast<int64_t>(t) * n_inner + hp] ? 1 : 0);
    }
    *nd = h;
    const int local = h - first;
    const int y = A.labels[i] ? 1 : 0;
    atomicAdd(&cls_s[2 * local + y], w);
    if (st[h] != kOpen) continue;
    const int32_t* sub = A.subsets + (static_cast<int64_t>(t) * n_inner + h) * A.m;
    for (int s = 0; s < A.m; ++s) {
      const int b = A.bins[i * A.d + sub[s]];
      const int64_t o = ((static_cast<int64_t>(local) * A.m + s) * A.hb + b) * 2 + y;
      if (lds_hist) atomicAdd(&hist_s[o], w);
      else atomicAdd(&ghist[o], w);
    }
  }
  __syncthreads();
  int32_t* gcls = A.cls + static_cast<int64_t>(t) * nodes * 2;
  for (int e = threadIdx.x; e < 2 * nodes; e += blockDim.x)
    if (cls_s[e]) atomicAdd(&gcls[e], cls_s[e]);
  for (int e = threadIdx.x; e < hist_n; e += blockDim.x)
    if (hist_s[e]) atomicAdd(&ghist[e], hist_s[e]);
}

__device__ __forceinline__ void fill_leaf(const RfArgs& A, int t, int h, int level, int64_t c0, int64_t c1) {
  const int n_inner = (1 << A.max_depth) - 1;
  const int span = 1 << (A.max_depth - level);
  const int first_leaf = (h + 1) * span - 1 - n_inner;
  const uint8_t cls = c1 > c0 ? 1 : 0;  // indexOfLargestArrayElement: first maximum
  uint8_t* out = A.out_leaf + static_cast<int64_t>(t) * (n_inner + 1) + first_leaf;
  for (int q = 0; q < span; ++q) out[q] = cls;
}

// One wave per node of the level: leaf class or best split.
__global__ __launch_bounds__(64) void rf_split_kernel(RfArgs A, int level) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* cum = reinterpret_cast<int*>(smem);  // [m][hb][2] prefix sums over bins
  const int t = blockIdx.y, local = blockIdx.x;
  const int nodes = 1 << level, h = nodes - 1 + local;
  const int n_inner = (1 << A.max_depth) - 1;
  const int n_all = 2 * n_inner + 1;
  uint8_t* st = A.status + static_cast<int64_t>(t) * n_all;
  const uint8_t s_h = st[h];
  if (s_h == kAbsent) return;
  const int lane = threadIdx.x;
  const int32_t* gc = A.cls + (static_cast<int64_t>(t) * nodes + local) * 2;
  const int64_t c0 = gc[0], c1 = gc[1];
  if (s_h == kLeaf || level == A.max_depth) {
    if (lane == 0) {
      fill_leaf(A, t, h, level, c0, c1);
      if (h < n_inner) A.split_f[static_cast<int64_t>(t) * n_inner + h] = -1;
    }
    return;
  }
  const int32_t* gh = A.hist + (static_cast<int64_t>(t) * nodes + local) * A.m * A.hb * 2;
  const int32_t* sub = A.subsets + (static_cast<int64_t>(t) * n_inner + h) * A.m;
  for (int s = lane; s < A.m; s += 64) {
    const int nb = A.n_splits[sub[s]] + 1;
    int a0 = 0, a1 = 0;
    for (int b = 0; b < nb; ++b) {
      a0 += gh[(s * A.hb + b) * 2];
      a1 += gh[(s * A.hb + b) * 2 + 1];
      cum[(s * A.hb + b) * 2] = a0;
      cum[(s * A.hb + b) * 2 + 1] = a1;
    }
  }
  __syncthreads();
  const double parent_imp = gini2(c0, c1);
  double best = -DBL_MAX;
  int best_p = INT_MAX;
  const int pairs = A.m * A.kmax;
  for (int p = lane; p < pairs; p += 64) {
    const int s = p / A.kmax, k = p - s * A.kmax;
    if (k >= A.n_splits[sub[s]]) continue;
    const int64_t l0 = cum[(s * A.hb + k) * 2], l1 = cum[(s * A.hb + k) * 2 + 1];
    double li, ri;
    const double g = split_gain(l0, l1, c0 - l0, c1 - l1, parent_imp, A.min_instances, A.min_gain, &li, &ri);
    if (g > best) {  // strict: a lane visits p in increasing order
      best = g;
      best_p = p;
    }
  }
  // lexicographic first maximum over (gain desc, pair index asc)
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best, o);
    const int op = __shfl_xor(best_p, o);
    if (og > best || (og == best && op < best_p)) {
      best = og;
      best_p = op;
    }
  }
  if (lane != 0) return;
  if (!(best > 0.0)) {  // gain <= 0 or no valid split: leaf
    fill_leaf(A, t, h, level, c0, c1);
    A.split_f[static_cast<int64_t>(t) * n_inner + h] = -1;
    return;
  }
  const int s = best_p / A.kmax, k = best_p - s * A.kmax;
  const int f = sub[s];
  const int64_t l0 = cum[(s * A.hb + k) * 2], l1 = cum[(s * A.hb + k) * 2 + 1];
  double li = 0.0, ri = 0.0;
  split_gain(l0, l1, c0 - l0, c1 - l1, parent_imp, A.min_instances, A.min_gain, &li, &ri);
  A.split_f[static_cast<int64_t>(t) * n_inner + h] = f;
  A.split_b[static_cast<int64_t>(t) * n_inner + h] = k;
  const bool child_leaf = level + 1 == A.max_depth;
  st[2 * h + 1] = (child_leaf || li == 0.0) ? kLeaf : kOpen;
  st[2 * h + 2] = (child_leaf || ri == 0.0) ? kLeaf : kOpen;
}

// Heap arrays of dal_forest_score: (feature, fp32 threshold bits) per inner
// node; absent / leaf positions become always-left (0, +inf) padding.
__global__ void rf_finalize_kernel(RfArgs A) {
  const int n_inner = (1 << A.max_depth) - 1;
  const int64_t total = static_cast<int64_t>(A.T) * n_inner;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int t = static_cast<int>(e / n_inner), h = static_cast<int>(e - static_cast<int64_t>(t) * n_inner);
    const uint8_t s = A.status[static_cast<int64_t>(t) * (2 * n_inner + 1) + h];
    const int f = s == kAbsent ? -1 : A.split_f[e];
    int2 out = make_int2(0, __float_as_int(__builtin_inff()));
    if (f >= 0) out = make_int2(f, __float_as_int(A.thresholds[static_cast<int64_t>(f) * DAL_RF_MAX_SPLITS +
                                                                A.split_b[e]]));
    reinterpret_cast<int2*>(A.out_inner)[e] = out;
  }
}

__global__ void rf_init_status_kernel(uint8_t* status, int T, int64_t n_all) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < T) status[static_cast<int64_t>(t) * n_all] = kOpen;
}

struct RfLayout {
  size_t bins, node, status, split_f, split_b, hist, cls, total;
};

RfLayout rf_layout(int64_t n, int64_t d, int64_t T, int max_depth, int64_t m, int64_t hb) {
  RfLayout L{};
  const int64_t n_inner = (int64_t{1} << max_depth) - 1;
  const int64_t split_nodes = int64_t{1} << (max_depth - 1);  // deepest level that is split
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += static_cast<size_t>(round_up(static_cast<int64_t>(bytes), 256));
    return at;
  };
  L.bins = take(static_cast<size_t>(n * d));
  L.node = take(static_cast<size_t>(T * n * 4));
  L.status = take(static_cast<size_t>(T * (2 * n_inner + 1)));
  L.split_f = take(static_cast<size_t>(T * n_inner * 4));
  L.split_b = take(static_cast<size_t>(T * n_inner * 4));
  L.hist = take(static_cast<size_t>(T * split_nodes * m * hb * 2 * 4));
  L.cls = take(static_cast<size_t>(T * (n_inner + 1) * 2 * 4));
  L.total = o;
  return L;
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" int dal_rf_find_splits(const float* x, int64_t n, int64_t d, int64_t ldx, const int64_t* sample_rows,
                                  int64_t n_sample, int32_t num_splits, float* thresholds, int32_t* n_splits,
                                  int32_t* dev_status, dal_stream_t stream) {
  if (!x || !thresholds || !n_splits || !dev_status) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ldx < d || n_sample < 1 || n_sample > DAL_RF_MAX_SPLIT_SAMPLE) return DAL_ERR_SHAPE;
  if (!sample_rows && n_sample > n) return DAL_ERR_SHAPE;
  if (num_splits < 0 || num_splits >= DAL_RF_MAX_SPLITS) return DAL_ERR_SHAPE;
  int pow2 = 1;
  while (pow2 < n_sample) pow2 <<= 1;
  const size_t smem = static_cast<size_t>(pow2) * 4 + static_cast<size_t>(n_sample) * 4 + 32 * 4;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(rf_find_splits_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem)) != hipSuccess)
    return DAL_ERR_HIP;
  hipLaunchKernelGGL(rf_find_splits_kernel, dim3(static_cast<unsigned>(d)), dim3(kSortThreads), smem,
                     as_stream(stream), x, n, static_cast<int>(d), ldx, sample_rows, static_cast<int>(n_sample),
                     pow2, num_splits, thresholds, n_splits, dev_status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" size_t dal_rf_train_workspace_bytes(int64_t n, int64_t d, int32_t n_trees, int32_t max_depth, int32_t m,
                                               int32_t num_splits) {
  if (n < 1 || d < 1 || n_trees < 1 || max_depth < 1 || max_depth > DAL_RF_MAX_DEPTH || m < 1 || num_splits < 0)
    return 0;
  return rf_layout(n, d, n_trees, max_depth, m, num_splits + 2).total;
}

extern "C" int dal_rf_train(const float* x, int64_t n, int64_t d, int64_t ldx, const uint8_t* labels,
                            const float* thresholds, const int32_t* n_splits, int32_t num_splits,
                            const int32_t* weights, const int32_t* feature_subsets, int32_t m, int32_t n_trees,
                            int32_t max_depth, int32_t min_instances, double min_info_gain, int32_t* out_inner,
                            uint8_t* out_leaf, void* ws, size_t ws_bytes, dal_stream_t stream) {
  if (!x || !labels || !thresholds || !n_splits || !weights || !feature_subsets || !out_inner || !out_leaf || !ws)
    return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ldx < d || n_trees < 1 || m < 1 || m > d) return DAL_ERR_SHAPE;
  if (max_depth < 1 || max_depth > DAL_RF_MAX_DEPTH) return DAL_ERR_UNSUPPORTED;
  if (num_splits < 0 || num_splits >= DAL_RF_MAX_SPLITS) return DAL_ERR_SHAPE;
  const int hb = num_splits + 2;  // find_splits emits at most num_splits + 1 thresholds
  // the split kernel keeps one node's whole (slot, bin, class) histogram in LDS
  if (static_cast<int64_t>(m) * hb * 2 * 4 > DAL_RF_SPLIT_LDS_BYTES) return DAL_ERR_UNSUPPORTED;
  const RfLayout L = rf_layout(n, d, n_trees, max_depth, m, hb);
  if (ws_bytes < L.total || reinterpret_cast<uintptr_t>(ws) % 256) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  unsigned char* w = static_cast<unsigned char*>(ws);
  RfArgs A{};
  A.bins = w + L.bins;
  A.labels = labels;
  A.weights = weights;
  A.subsets = feature_subsets;
  A.thresholds = thresholds;
  A.n_splits = n_splits;
  A.n = n;
  A.d = static_cast<int>(d);
  A.m = m;
  A.T = n_trees;
  A.max_depth = max_depth;
  A.hb = hb;
  A.kmax = num_splits + 1;
  A.min_instances = min_instances;
  A.min_gain = min_info_gain;
  A.node = reinterpret_cast<int32_t*>(w + L.node);
  A.status = w + L.status;
  A.split_f = reinterpret_cast<int32_t*>(w + L.split_f);
  A.split_b = reinterpret_cast<int32_t*>(w + L.split_b);
  A.hist = reinterpret_cast<int32_t*>(w + L.hist);
  A.cls = reinterpret_cast<int32_t*>(w + L.cls);
  A.out_inner = out_inner;
  A.out_leaf = out_leaf;
  const int64_t n_inner = (int64_t{1} << max_depth) - 1;

  hipLaunchKernelGGL(rf_bin_kernel, dim3(static_cast<unsigned>(std::min<int64_t>(ceil_div(n * d, 256), 4096))),
                     dim3(256), 0, st, x, n, static_cast<int>(d), ldx, thresholds, n_splits,
                     const_cast<uint8_t*>(A.bins));
  DAL_RETURN_IF_LAUNCH_FAILED();
  // root open, everything else absent
  if (hipMemsetAsync(A.status, 0, static_cast<size_t>(n_trees) * (2 * n_inner + 1), st) != hipSuccess)
    return DAL_ERR_HIP;
  hipLaunchKernelGGL(rf_init_status_kernel, dim3(static_cast<unsigned>(ceil_div(n_trees, 256))), dim3(256), 0, st,
                     A.status, n_trees, 2 * n_inner + 1);
  DAL_RETURN_IF_LAUNCH_FAILED();
  const int rows_per_block = 1024;
  const dim3 hgrid(static_cast<unsigned>(ceil_div(n, rows_per_block)), static_cast<unsigned>(n_trees));
  for (int level = 0; level <= max_depth; ++level) {
    const int64_t nodes = int64_t{1} << level;
    const bool open_level = level < max_depth;
    const int64_t hist_ints = open_level ? nodes * m * hb * 2 : 0;
    if (hipMemsetAsync(A.cls, 0, static_cast<size_t>(n_trees * nodes * 2 * 4), st) != hipSuccess) return DAL_ERR_HIP;
    if (open_level &&
        hipMemsetAsync(A.hist, 0, static_cast<size_t>(n_trees * hist_ints * 4), st) != hipSuccess)
      return DAL_ERR_HIP;
    const bool lds_hist = (2 * nodes + hist_ints) * 4 <= 64 * 1024;
    const size_t hsmem = static_cast<size_t>(2 * nodes + (lds_hist ? hist_ints : 0)) * 4;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(rf_hist_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(hsmem)) != hipSuccess)
      return DAL_ERR_HIP;
    hipLaunchKernelGGL(rf_hist_kernel, hgrid, dim3(256), hsmem, st, A, level, rows_per_block, lds_hist);
    DAL_RETURN_IF_LAUNCH_FAILED();
    const size_t ssmem = open_level ? static_cast<size_t>(m) * hb * 2 * 4 : 16;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(rf_split_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ssmem)) != hipSuccess)
      return DAL_ERR_HIP;
    hipLaunchKernelGGL(rf_split_kernel, dim3(static_cast<unsigned>(nodes), static_cast<unsigned>(n_trees)),
                       dim3(64), ssmem, st, A, level);
    DAL_RETURN_IF_LAUNCH_FAILED();
  }
  hipLaunchKernelGGL(rf_finalize_kernel,
                     dim3(static_cast<unsigned>(std::min<int64_t>(ceil_div(n_trees * n_inner, 256), 4096))),
                     dim3(256), 0, st, A);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
