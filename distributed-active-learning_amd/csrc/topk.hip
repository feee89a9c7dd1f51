// Top-k selection: sortBy(score).take(k) with a deterministic tie rule, and
// the density-weighted selection with its exact fp64 re-rank.
//
// Reference: final_thesis/uncertainty_sampling.py:106,109 (ascending
// sortBy + take(window_size)); density_weighting.py:168,172 (descending);
// lal_direct_mllib_implementation/classes/active_learner.py:203 (k = 1).
// Spark breaks ties by partition order (nondeterministic); the canonical rule
// here is (key, then lower global row index), with NaN last and -0 == +0
// (score_key in common.hpp).
//
// Pipeline (all device-side, no host round trip):
//   6 x radix_hist   exact k-th smallest key, 11-bit digits MSB first; every
//                    block re-derives the running (prefix, remaining-k) state
//                    from the previous pass's 2048-bin histogram.
//   count/scan/write ordered compaction: every key < K*, plus the first
//                    (in row order) keys == K* -- stable, so ties go to the
//                    lower index.
//   sort             one 1024-thread block, bitonic on (key, index) in LDS.
// HBM-bound: each pass reads 8 B/row.
//
// Fast level 1 of the interval selections (dal_dw_select / dal_dw_step /
// dal_maxcos_select with level1_passes > 0; cap <= DAL_SORT_CAP_PAYLOAD):
//   row-group minima  the pool is cut into <= kMaxGroups row groups and each
//                     group's minimum pessimistic and optimistic keys are
//                     kept (written by dal_dw_step's score kernel itself, or by
//                     one group_min_kernel pass);
//   summary_select    every block derives tau = the k-th smallest group
//                     minimum (a block radix select over <= 4096 keys); any k
//                     keys of the pool bound the k-th smallest key K from above,
//                     so tau >= K.  Only groups whose optimistic minimum is
//                     <= tau are scanned; every row whose OPTIMISTIC key is
//                     <= tau joins the candidates (with the density-weighted
//                     selections, its canonical fp64 score is computed in
//                     place) and the block that finishes last sorts them.
// {optimistic <= tau} contains {optimistic <= K}, the exact path's candidate
// set, so the selection is the same.  When the top-k rows lie in distinct
// groups (k << groups) tau is within a few ranks of K, so the candidates are
// about the rows whose score interval reaches the k-th score.  More than cap
// candidates raises DAL_FLAG_SAMPLE_MISS (the caller re-runs with
// level1_passes = 0).
#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include "common.hpp"

namespace dal {
namespace {

constexpr int kRadixThreads = 256;
constexpr int kCompactRows = 1024;  // rows per compaction block (4 per thread)
constexpr int kSortThreads = 1024;

// Radix digits: 11 bits MSB first -> 6 passes over the 64-bit key (the last
// pass covers the low 9 bits).  8-bit digits needed 8 dependent launches; each
// pass costs about one launch on small pools, so fewer passes is the win.
constexpr int kDigitBits = 11;
constexpr int kPasses = (64 + kDigitBits - 1) / kDigitBits;  // 6
constexpr int kBins = 1 << kDigitBits;                       // 2048
constexpr int kBinsPerThread = kBins / kRadixThreads;        // 8

__host__ __device__ constexpr int digit_shift(int p) {
  return 64 - kDigitBits * (p + 1) > 0 ? 64 - kDigitBits * (p + 1) : 0;
}
__host__ __device__ constexpr int digit_bins(int p) {
  return 1 << (64 - kDigitBits * p - digit_shift(p));
}

// Agent-scope relaxed loads / stores (global_load / global_store ... sc1):
// the hand-off from the blocks of summary_select_kernel to the one that
// arrives last (candidates, their count) is written and read only this way,
// so no release / acquire fence is needed (MI355X_MICROARCH.md, "Valid
// forms": sc1 stores or agent atomics, vmcnt(0) + a workgroup barrier before
// one lane's arrival, sc1 loads after it).
template <class T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(ld_sc1(reinterpret_cast<const long long*>(p)));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  st_sc1(reinterpret_cast<long long*>(p), __double_as_longlong(v));
}

// summary_select_kernel's blocks, each owning a candidate region (<= 32 row
// groups per block: the candidate scoring spreads over up to 128 CUs)
constexpr int kMaxRegions = 128;

struct TopkHdr {
  // fast level 1 (summary_select_kernel): candidate count, the blocks'
  // arrival counter and tau -- the words a fast-path call needs zero
  unsigned int cand_count, arrive;
  unsigned long long kstar;
  // exact path
  unsigned long long kfinal, total_lt, total_eq;
  unsigned int overflow, pad0;
  unsigned long long prefix[kPasses + 1];
  unsigned long long krem[kPasses + 1];
  uint32_t hist[kPasses][kBins];
  // fast level 1: candidates found by each summary_select block (its region)
  unsigned int reg_count[kMaxRegions];
};

struct TopkLayout {
  size_t hdr, blk, off, ckey, cidx, cpay, total;
  int64_t nb, cap;
};

TopkLayout topk_layout(int64_t n, int64_t cap) {
  TopkLayout L;
  L.nb = ceil_div(n < 1 ? 1 : n, kCompactRows);
  L.cap = cap;
  size_t o = 0;
  L.hdr = o;
  o += round_up(sizeof(TopkHdr), 256);
  L.blk = o;
  o += round_up(L.nb * 2 * sizeof(uint32_t), 256);
  L.off = o;
  o += round_up(L.nb * 2 * sizeof(uint32_t), 256);
  L.ckey = o;
  o += round_up(cap * 8, 256);
  L.cidx = o;
  o += round_up(cap * 8, 256);
  L.cpay = o;
  o += round_up(cap * 8, 256);
  L.total = o;
  return L;
}

// ---------------------------------------------------------------- radix ----
// Resolve the digit of pass p from its histogram: the first bucket whose
// inclusive count reaches the remaining k.  256 threads x 8 consecutive
// buckets; a block scan of the per-thread totals locates the crossing.
__device__ void resolve_digit(const TopkHdr* h, int p, unsigned long long& prefix,
                              unsigned long long& krem, uint32_t* sh) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const unsigned long long kr = h->krem[p];
  const int nb = digit_bins(p);
  uint32_t c[kBinsPerThread];
  uint32_t tot = 0;
#pragma unroll
  for (int j = 0; j < kBinsPerThread; ++j) {
    const int b = tid * kBinsPerThread + j;
    c[j] = b < nb ? h->hist[p][b] : 0u;
    tot += c[j];
  }
  uint32_t x = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  __shared__ unsigned long long s_pre, s_krem;
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t excl = x - tot;
  for (int i = 0; i < w; ++i) excl += sh[i];
  if (excl < kr && excl + tot >= kr) {
    uint32_t run = excl;
#pragma unroll
    for (int j = 0; j < kBinsPerThread; ++j) {
      if (run < kr && run + c[j] >= kr) {
        s_pre = h->prefix[p] |
                (static_cast<unsigned long long>(tid * kBinsPerThread + j) << digit_shift(p));
        s_krem = kr - run;
      }
      run += c[j];
    }
  }
  __syncthreads();
  prefix = s_pre;
  krem = s_krem;
  __syncthreads();
}

__global__ __launch_bounds__(kRadixThreads) void radix_hist_kernel(const uint64_t* __restrict__ keys,
                                                                   int64_t n, int64_t k, int pass,
                                                                   TopkHdr* __restrict__ h) {
  __shared__ uint32_t hist[kBins];
  __shared__ uint32_t scan[kRadixThreads / 64];
  const int tid = threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kRadixThreads;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kRadixThreads + tid;
  // the first kPre keys of the thread are loaded before the previous pass is
  // resolved: the key fetch and the histogram read overlap (on small pools
  // these are all the keys, and each pass is latency-bound)
  constexpr int kPre = 8;
  unsigned long long pre[kPre];
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    const int64_t i = i0 + j * stride;
    pre[j] = i < n ? keys[i] : 0ull;
  }
  unsigned long long prefix = 0, krem = static_cast<unsigned long long>(k);
  if (pass > 0) resolve_digit(h, pass - 1, prefix, krem, scan);
  if (blockIdx.x == 0 && tid == 0) {
    h->prefix[pass] = prefix;
    h->krem[pass] = krem;
  }
#pragma unroll
  for (int j = 0; j < kBinsPerThread; ++j) hist[j * kRadixThreads + tid] = 0;
  __syncthreads();
  const int shift = digit_shift(pass);
  const unsigned long long dmask = static_cast<unsigned long long>(digit_bins(pass) - 1);
  const unsigned long long hmask = pass == 0 ? 0ull : (~0ull << (64 - kDigitBits * pass));
  // scores cluster (DW keys share their sign/exponent digit, LC keys take
  // T+1 values): the wave's most common bin -- the first valid lane's -- is
  // counted with ONE atomic, the other lanes add theirs (no 64-way LDS
  // same-address serialisation on the heavy bin)
  const int lane = tid & 63;
  auto count = [&](bool valid, unsigned bin) {
    const unsigned long long vm = __ballot(valid);
    if (!vm) return;
    const int first = __ffsll(static_cast<long long>(vm)) - 1;
    const unsigned b0 = __shfl(bin, first);
    const unsigned long long m0 = __ballot(valid && bin == b0);
    if (lane == first) atomicAdd(&hist[b0], static_cast<unsigned>(__popcll(m0)));
    if (valid && bin != b0) atomicAdd(&hist[bin], 1u);
  };
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    const unsigned long long key = pre[j];
    count(i0 + j * stride < n && (key & hmask) == prefix, static_cast<unsigned>((key >> shift) & dmask));
  }
  // the rest in batches of kPre keys, each batch's loads in flight together
  // (wave-uniform trip count: the ballots see every lane)
  for (int64_t i0b = i0 - tid + kPre * stride; i0b < n; i0b += kPre * stride) {
    unsigned long long kb[kPre];
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int64_t i = i0b + j * stride + tid;
      kb[j] = i < n ? keys[i] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int64_t i = i0b + j * stride + tid;
      count(i < n && (kb[j] & hmask) == prefix, static_cast<unsigned>((kb[j] >> shift) & dmask));
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kBinsPerThread; ++j) {
    const int b = j * kRadixThreads + tid;
    const uint32_t v = hist[b];
    if (v) atomicAdd(&h->hist[pass][b], v);
  }
}

// ----------------------------------------------------------- compaction ---
// Predicates per row: lt (take unconditionally) / eq (take the first eq_take
// in row order).  EXACT: on the key itself.  INTERVAL: on the optimistic end
// of the row's density-score interval (dal_dw_select).
struct IntervalArgs {
  const uint64_t* keys_hi;  // optimistic key of each row's score interval
};

template <bool INTERVAL>
__device__ __forceinline__ void predicate(const uint64_t* keys, const IntervalArgs& I, int64_t i,
                                          unsigned long long K, bool& lt, bool& eq) {
  const unsigned long long lo = keys[i];
  if (!INTERVAL) {
    lt = lo < K;
    eq = lo == K;
    return;
  }
  // K = k-th smallest pessimistic key.  A row can reach the canonical top-k
  // only if its optimistic key is <= K; rows whose interval is a point
  // (exact score) and equal to K are ties resolved by index.
  const unsigned long long hi = I.keys_hi[i];
  const bool exact = hi == lo;
  lt = hi < K || (hi == K && !exact);
  eq = hi == K && exact;
}

__device__ __forceinline__ void final_threshold(TopkHdr* h, unsigned long long& K,
                                                unsigned long long& krem, uint32_t* scan) {
  resolve_digit(h, kPasses - 1, K, krem, scan);
}

template <bool INTERVAL>
__global__ __launch_bounds__(kRadixThreads) void compact_count_kernel(const uint64_t* __restrict__ keys,
                                                                      IntervalArgs I, int64_t n,
                                                                      TopkHdr* __restrict__ h,
                                                                      uint32_t* __restrict__ blk) {
  __shared__ uint32_t scan[256];
  __shared__ uint32_t red[2][4];
  unsigned long long K, krem;
  final_threshold(h, K, krem, scan);
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) {
    h->kstar = K;
    h->kfinal = krem;
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kCompactRows;
  uint32_t lt_c = 0, eq_c = 0;
  for (int j = 0; j < 4; ++j) {
    const int64_t i = r0 + tid * 4 + j;
    if (i >= n) break;
    bool lt, eq;
    predicate<INTERVAL>(keys, I, i, K, lt, eq);
    lt_c += lt;
    eq_c += eq;
  }
  for (int o = 32; o > 0; o >>= 1) {
    lt_c += __shfl_xor(lt_c, o);
    eq_c += __shfl_xor(eq_c, o);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = lt_c;
    red[1][tid >> 6] = eq_c;
  }
  __syncthreads();
  if (tid == 0) {
    blk[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    blk[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// exclusive scan of the per-block (lt, eq) counts; one 1024-thread block.
__global__ __launch_bounds__(1024) void compact_scan_kernel(const uint32_t* __restrict__ blk,
                                                            uint32_t* __restrict__ off, int64_t nb,
                                                            TopkHdr* __restrict__ h) {
  __shared__ uint32_t s[2][1024];
  const int tid = threadIdx.x;
  uint32_t carry_lt = 0, carry_eq = 0;
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t b = base + tid;
    const uint32_t vl = b < nb ? blk[2 * b] : 0, ve = b < nb ? blk[2 * b + 1] : 0;
    s[0][tid] = vl;
    s[1][tid] = ve;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const uint32_t yl = tid >= o ? s[0][tid - o] : 0, ye = tid >= o ? s[1][tid - o] : 0;
      __syncthreads();
      s[0][tid] += yl;
      s[1][tid] += ye;
      __syncthreads();
    }
    if (b < nb) {
      off[2 * b] = carry_lt + s[0][tid] - vl;
      off[2 * b + 1] = carry_eq + s[1][tid] - ve;
    }
    carry_lt += s[0][1023];
    carry_eq += s[1][1023];
    __syncthreads();
  }
  if (tid == 0) {
    h->total_lt = carry_lt;
    h->total_eq = carry_eq;
  }
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (int i = 0; i < kRadixThreads / 64; ++i) {
    if (i < w) before += sh[i];
    total += sh[i];
  }
  __syncthreads();
  return x - v + before;
}

// EXACT:    every key < K, then the first (k - #lt) keys == K in row order.
// INTERVAL: candidates = lt rows plus eq rows whose global eq rank is < k,
//           written as ONE stream in row order (position = #candidates before
//           the row), so ties among candidates later resolve by row index.
template <bool INTERVAL>
__global__ __launch_bounds__(kRadixThreads) void compact_write_kernel(
    const uint64_t* __restrict__ keys, IntervalArgs I, int64_t n, int64_t idx_base, int64_t k,
    TopkHdr* __restrict__ h, const uint32_t* __restrict__ off, uint64_t* __restrict__ ckey,
    int64_t* __restrict__ cidx, int64_t cap, int32_t* __restrict__ status) {
  __shared__ uint32_t sh[3][4];
  const int tid = threadIdx.x;
  const unsigned long long K = h->kstar;
  const uint64_t eq_take = INTERVAL ? static_cast<uint64_t>(k) : h->kfinal;
  const uint64_t total_lt = h->total_lt;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kCompactRows;
  bool lt[4], eq[4];
  uint32_t lc = 0, ec = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = r0 + tid * 4 + j;
    lt[j] = eq[j] = false;
    if (i < n) predicate<INTERVAL>(keys, I, i, K, lt[j], eq[j]);
    lc += lt[j];
    ec += eq[j];
  }
  uint32_t tl, te;
  const uint32_t lt_off = off[2 * blockIdx.x], eq_off = off[2 * blockIdx.x + 1];
  uint32_t pl = block_excl_scan(lc, sh[0], tl) + lt_off;
  uint32_t pe = block_excl_scan(ec, sh[1], te) + eq_off;
  bool ovf = false;
  if (!INTERVAL) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = r0 + tid * 4 + j;
      int64_t pos = -1;
      if (lt[j]) pos = pl++;
      else if (eq[j]) {
        if (pe < eq_take) pos = static_cast<int64_t>(total_lt + pe);
        ++pe;
      }
      if (pos >= 0) {
        if (pos < cap) {
          ckey[pos] = keys[i];
          cidx[pos] = idx_base + i;
        } else {
          ovf = true;
        }
      }
    }
  } else {
    bool cand[4];
    uint32_t cc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cand[j] = lt[j] || (eq[j] && pe < eq_take);
      if (eq[j]) ++pe;
      cc += cand[j];
    }
    uint32_t tc;
    const uint64_t before = lt_off + (eq_off < eq_take ? eq_off : eq_take);
    uint64_t pc = block_excl_scan(cc, sh[2], tc) + before;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!cand[j]) continue;
      const int64_t pos = static_cast<int64_t>(pc++);
      if (pos < cap) cidx[pos] = idx_base + r0 + tid * 4 + j;
      else ovf = true;
    }
  }
  if (ovf) {
    atomicOr(&h->overflow, 1u);
    if (status) atomicOr(status, DAL_FLAG_CAND_OVERFLOW);
  }
  if (blockIdx.x == 0 && tid == 0) {
    const uint64_t take_eq = h->total_eq < eq_take ? h->total_eq : eq_take;
    const uint64_t cnt = total_lt + take_eq;
    h->cand_count = static_cast<unsigned>(cnt < static_cast<uint64_t>(cap) ? cnt : cap);
  }
}

// ------------------------------------------------------------- re-rank ----
// Canonical fp64 density-weighted score of a row (bit-identical to
// oracle.density_canonical: x/norm, then sequential mul+add over features;
// the library is compiled with -ffp-contract=off).
struct DwRerank {
  const float* x;
  int d;
  int64_t ldx;
  const double* norm64;
  const double* colsum;
  const double* lut;
  const int32_t* votes;
  const uint8_t* flags;
  double beta;
  // a plan step (ForestStepHooks): flags = base_flags | (stamp == step ?
  // CANDIDATE : 0), derived here for the candidates instead of stored per row
  const uint8_t* base_flags = nullptr;
  const uint8_t* stamp = nullptr;
  const uint32_t* step_id = nullptr;
};

__device__ __forceinline__ uint8_t rerank_flag(const DwRerank& R, int64_t i) {
  if (R.base_flags)
    return static_cast<uint8_t>(R.base_flags[i] | (R.stamp[i] == static_cast<uint8_t>(*R.step_id) ? DAL_ROW_CANDIDATE : 0));
  return R.flags ? R.flags[i] : DAL_ROW_CANDIDATE;
}

// The canonical score of local row i, computed by a whole wave (every lane
// calls it with the same row): lane f forms the rounded product
// (x_f / norm) * s_f -- the loads and divisions of 256 features in flight
// together (one memory round trip per 256 features: a round trip per
// 64-feature chunk made a d = 256 row cost ~13 us) -- and the sequential sum
// over f takes the products in order (the oracle's operations in the
// oracle's order) from the wave's 64-double LDS slot `tr`: each chunk's
// products are written there and read back as broadcasts, two per
// ds_read_b128 (two v_readlane per product before).  false (NONE key, NaN
// payload) when the row is not an unlabeled candidate (a shard with < k
// candidates).
__device__ __forceinline__ double readlane_f64(double v, int l) {  // l wave-uniform
  const long long b = __double_as_longlong(v);
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(b >> 32), l));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

// d^beta for beta != 1 (the reference declares beta, density_weighting.py:33;
// 1 in every call): out of line, so its constants do not crowd the callers'
// scalar registers.
__device__ __attribute__((noinline)) double density_pow_canon(double d, double beta) { return pow(d, beta); }

__device__ __forceinline__ bool dw_canonical_score_wave(const DwRerank& R, int64_t i, double& s, double* tr,
                                                        double lut_lane = 0.0, int n_lut = 0) {
  constexpr int kC = 4;  // 64-feature chunks per round: every chunk's loads and divisions in flight together
  const int lane = threadIdx.x & 63;
  const uint8_t fl = rerank_flag(R, i);
  const double nr = R.norm64[i];
  const int v = R.votes[i];
  const float* xr = R.x + i * R.ldx;
  double acc = 0.0;
  for (int f0 = 0; f0 < R.d; f0 += 64 * kC) {
    double p[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const int f = f0 + 64 * c + lane;
      p[c] = f < R.d ? (static_cast<double>(xr[f]) / nr) * R.colsum[f] : 0.0;
    }
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const int rest = __builtin_amdgcn_readfirstlane(R.d - f0 - 64 * c);
      if (rest <= 0) break;
      // the previous chunk's reads are issued before this write (LDS
      // operations of one wave complete in order)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      tr[lane] = p[c];
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (rest >= 64) {
        // 16 products' broadcast reads ahead of their adds: only the add
        // chain is serial
        const double2* tr2 = reinterpret_cast<const double2*>(tr);
#pragma unroll
        for (int q0 = 0; q0 < 32; q0 += 8) {
          double2 t[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) t[j] = tr2[q0 + j];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc = acc + t[j].x;
            acc = acc + t[j].y;
          }
        }
      } else {
        for (int q = 0; q < rest; ++q) acc = acc + tr[q];
      }
    }
  }
  if (!(fl & DAL_ROW_CANDIDATE)) {
    s = __builtin_nan("");
    return false;
  }
  if (fl & DAL_ROW_EXCLUDED) acc = __builtin_nan("");
  // n_lut > 0: lane l holds lut[l] (T < 64), no dependent load on the vote
  const double e = v < n_lut ? readlane_f64(lut_lane, v) : R.lut[v];
  s = e * (R.beta == 1.0 ? acc : density_pow_canon(acc, R.beta));
  return true;
}

// The same canonical score computed by one lane alone (sequential over f,
// the row's features fetched 64 at a time); e = lut[vote] passed in when the
// LUT is held in lanes (n_lut > 0).  For waves with many candidates, where
// one wave-wide pass per candidate would serialise them.
template <int kChunk = 64>
__device__ __forceinline__ bool dw_canonical_score_lane(const DwRerank& R, int64_t i, double& s, double e_in,
                                                        int n_lut) {
  const uint8_t fl = rerank_flag(R, i);
  if (!(fl & DAL_ROW_CANDIDATE)) {
    s = __builtin_nan("");
    return false;
  }
  const double nr = R.norm64[i];
  const float* xr = R.x + i * R.ldx;
  double acc = 0.0;
  int f0 = 0;
  for (; f0 + kChunk <= R.d; f0 += kChunk) {
    float xv[kChunk];
#pragma unroll
    for (int q = 0; q < kChunk; ++q) xv[q] = xr[f0 + q];
#pragma unroll
    for (int q = 0; q < kChunk; ++q) {
      const double u = static_cast<double>(xv[q]) / nr;
      acc = acc + u * R.colsum[f0 + q];
    }
  }
  for (int f = f0; f < R.d; ++f) {
    const double u = static_cast<double>(xr[f]) / nr;
    acc = acc + u * R.colsum[f];
  }
  if (fl & DAL_ROW_EXCLUDED) acc = __builtin_nan("");
  const double e = n_lut ? e_in : R.lut[R.votes[i]];
  s = e * (R.beta == 1.0 ? acc : density_pow_canon(acc, R.beta));
  return true;
}

// Prefetch of a candidate row's re-rank inputs into L2 (and the TLB) by
// LDS-DMA loads whose landing slots nobody reads: every 64-B piece of x's row,
// norm64, the vote and the row flags (or the plan's base flags and stamp).
// One lane per row; a wave issues its lanes' loads together (64-bit
// addresses, no VGPR results: nothing waits for them).
__device__ __forceinline__ void lds_dma_dword(const void* p, unsigned* slots) {
  typedef __attribute__((address_space(3))) unsigned lds_u32;
  const unsigned dst = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_u32*)slots)));
  const unsigned long long a = reinterpret_cast<uintptr_t>(p) & ~3ull;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(a), "s"(dst)
      : "memory");
}
__device__ __forceinline__ void prefetch_row(const DwRerank& R, int64_t i, unsigned* slots) {
  const char* xr = reinterpret_cast<const char*>(R.x + i * R.ldx);
  const int bytes = R.d * 4;
  for (int b = 0; b < bytes; b += 64) lds_dma_dword(xr + b, slots);  // (d uniform: every lane the same count)
  lds_dma_dword(R.norm64 + i, slots);
  lds_dma_dword(R.votes + i, slots);
  if (R.base_flags) {
    lds_dma_dword(R.base_flags + i, slots);
    lds_dma_dword(R.stamp + i, slots);
  } else if (R.flags) {
    lds_dma_dword(R.flags + i, slots);
  }
}

// Re-rank target of summary_select_kernel's density-weighted form.
struct AppendRerank {
  DwRerank R;
  uint64_t* ckey;
  double* cpay;
};

// One wave per candidate slot (dw_canonical_score_wave).
__global__ __launch_bounds__(256) void rerank_kernel(const TopkHdr* __restrict__ h, int64_t idx_base, DwRerank R,
                                                     uint64_t* __restrict__ ckey,
                                                     const int64_t* __restrict__ cidx,
                                                     double* __restrict__ cpay, int64_t cap,
                                                     bool cap_miss, int32_t* __restrict__ status) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const bool lead = (threadIdx.x & 63) == 0;
  if (cap_miss && c == 0 && lead && h->cand_count > cap)
    atomicOr(status, DAL_FLAG_SAMPLE_MISS);  // fast level 1 over capacity: the caller re-runs exactly
  if (c >= cap) return;
  if (c >= h->cand_count) {
    if (lead) ckey[c] = DAL_KEY_NONE;
    return;
  }
  __shared__ __attribute__((aligned(16))) double s_tr[4][64];
  double s;
  const bool ok = dw_canonical_score_wave(R, cidx[c] - idx_base, s, s_tr[threadIdx.x >> 6]);
  if (lead) {
    cpay[c] = s;
    ckey[c] = ok ? score_key(s, DAL_DESCENDING) : DAL_KEY_NONE;
  }
}

// Canonical fp64 max-cosine of each candidate: one wave per candidate, lanes
// over labeled rows; cos = sequential sum over features of u_if * u_lf with
// u_i = x_i / ||x_i|| (sequential norm, no FMA) and u_l precomputed the same
// way; max keeps the first (lowest l) maximum.
__device__ __forceinline__ float bf16f(uint16_t b) { return __uint_as_float(static_cast<unsigned>(b) << 16); }

// Canonical fp64 max-cosine of the candidates (oracle: max_cosine_canonical):
// u_i = x_i / sqrt(sum_f x_if^2) (sequential), cos_il = sum_f u_if * ulab_lf
// (sequential in f, no FMA), max over l, ties -> lowest l.  A block takes
// kRrC candidates: their unit rows are computed once into LDS, then each
// lane carries kRrC x kRrJ independent fp32 accumulators over labeled rows
// l = lane + 64 * (wave + 4 j) (+ 1024 per outer pass), reading the
// feature-major table ulabT[f * m + l] coalesced.  Only the rows whose fp32
// dot lies within 2 B of the candidate's fp32 maximum get the canonical fp64
// sum (round 6: every row's fp64 sum before, 1.5 M sequential 128-step chains
// per config-5 call).
#ifndef DAL_RR_CANDS
#define DAL_RR_CANDS 4  // candidates per block (8 measured 92 vs 77 us at config 5 with fp64 dots: fewer blocks)
#endif
constexpr int kRrC = DAL_RR_CANDS;
constexpr int kRrJ = 4;
__global__ __launch_bounds__(256) void rerank_maxcos_kernel(const TopkHdr* __restrict__ h, int64_t idx_base,
                                                            const uint16_t* __restrict__ pool, int d,
                                                            int64_t ld, const double* __restrict__ ulabT,
                                                            int64_t m, uint64_t* __restrict__ ckey,
                                                            const int64_t* __restrict__ cidx,
                                                            double* __restrict__ cpay, int64_t cap,
                                                            bool cap_miss, int32_t* __restrict__ status) {
  __shared__ double su[256][kRrC];  // [f][candidate]
  __shared__ float sf[256][kRrC];
  __shared__ float s_m32[4][kRrC];
  __shared__ __attribute__((aligned(16))) double s_tr[4][64];
  __shared__ double rb[4][kRrC];
  __shared__ long long ra[4][kRrC];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * kRrC;
  const int64_t count = h->cand_count;
  if (cap_miss && c0 == 0 && tid == 0 && h->cand_count > cap)
    atomicOr(status, DAL_FLAG_SAMPLE_MISS);  // fast level 1 over capacity: the caller re-runs exactly
  if (c0 >= count) {
    if (tid < kRrC && c0 + tid < cap) ckey[c0 + tid] = DAL_KEY_NONE;
    return;
  }
  // wave w builds candidate c0 + w's canonical unit row (every lane runs the
  // same sequential norm; lanes then divide their features)
  for (int q = wave; q < kRrC; q += 4) {
    const int64_t c = c0 + q;
    if (c < count) {
      const uint16_t* xr = pool + (cidx[c] - idx_base) * ld;
      const double nr = __builtin_sqrt(row_sq_norm_bf16(xr, d));  // sequential in f, vector loads
      for (int f = lane; f < d; f += 64) su[f][q] = static_cast<double>(bf16f(xr[f])) / nr;
    } else {
      for (int f = lane; f < d; f += 64) su[f][q] = 0.0;
    }
  }
  __syncthreads();
  // fp32 copies of the unit rows: every (candidate, labeled row) dot first in
  // fp32 (FMA chains), then the canonical fp64 sum only for the labeled rows
  // within 2 B of the candidate's fp32 maximum.  |fp32 dot - canonical| <= B
  // for unit rows at d <= 256 (d 2^-24 for the chain, 2^-23 for the operands'
  // rounding to fp32, < 1e-13 for the canonical fp64 sum: B = 2^-16 holds
  // with a 2x margin), so every row reaching the canonical maximum is among
  // them and the (value, lowest row) result is the full scan's.
  for (int e = tid; e < d * kRrC; e += 256) sf[e / kRrC][e % kRrC] = static_cast<float>(su[e / kRrC][e % kRrC]);
  __syncthreads();
  const bool one = m <= 256 * kRrJ;  // one chunk of labeled rows: the fp32 dots stay in registers
  float a[kRrC][kRrJ];
  int64_t l[kRrJ];
  bool ok[kRrJ];
  auto chunk = [&](int64_t lb) {
#pragma unroll
    for (int j = 0; j < kRrJ; ++j) {
      l[j] = lb + lane + 64 * (wave + 4 * j);
      ok[j] = l[j] < m;
      if (!ok[j]) l[j] = m - 1;
    }
#pragma unroll
    for (int q = 0; q < kRrC; ++q)
#pragma unroll
      for (int j = 0; j < kRrJ; ++j) a[q][j] = 0.f;
#pragma unroll 4
    for (int f = 0; f < d; ++f) {
      float ul[kRrJ];
#pragma unroll
      for (int j = 0; j < kRrJ; ++j) ul[j] = static_cast<float>(ulabT[static_cast<int64_t>(f) * m + l[j]]);
#pragma unroll
      for (int q = 0; q < kRrC; ++q) {
        const float uq = sf[f][q];
#pragma unroll
        for (int j = 0; j < kRrJ; ++j) a[q][j] = __builtin_fmaf(uq, ul[j], a[q][j]);
      }
    }
  };
  float m32[kRrC];
#pragma unroll
  for (int q = 0; q < kRrC; ++q) m32[q] = -__builtin_inff();
  for (int64_t lb = 0; lb < m; lb += 256 * kRrJ) {
    chunk(lb);
#pragma unroll
    for (int j = 0; j < kRrJ; ++j)
#pragma unroll
      for (int q = 0; q < kRrC; ++q)
        if (ok[j]) m32[q] = __builtin_fmaxf(m32[q], a[q][j]);
  }
#pragma unroll
  for (int q = 0; q < kRrC; ++q) {
    for (int o = 32; o > 0; o >>= 1) m32[q] = __builtin_fmaxf(m32[q], __shfl_xor(m32[q], o));
    if (lane == 0) s_m32[wave][q] = m32[q];
  }
  __syncthreads();
  constexpr float kNear = 0x1p-15f;  // 2 B
  float thr[kRrC];
#pragma unroll
  for (int q = 0; q < kRrC; ++q)  // (a slot past the candidates -- zero unit row -- takes no pair)
    thr[q] = c0 + q < count ? __builtin_fmaxf(__builtin_fmaxf(s_m32[0][q], s_m32[1][q]),
                                              __builtin_fmaxf(s_m32[2][q], s_m32[3][q])) - kNear
                            : __builtin_inff();
  double best[kRrC];
  long long arg[kRrC];
#pragma unroll
  for (int q = 0; q < kRrC; ++q) {
    best[q] = -__builtin_inf();
    arg[q] = 0x7FFFFFFFFFFFFFFFll;
  }
  // a near (candidate, labeled row) pair: its canonical sum by the whole
  // wave -- lane f's rounded products u_if * u_lf with every load in flight,
  // then the sequential sum over f through the wave's LDS slot (the products'
  // rounding and the adds' order are the canonical ones)
  auto canon_dot = [&](int q, int64_t lr) -> double {
    double p[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 64 * c + lane;
      p[c] = f < d ? su[f][q] * ulabT[static_cast<int64_t>(f) * m + lr] : 0.0;
    }
    double acc = 0.0;
    double* tr = s_tr[wave];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int rest = __builtin_amdgcn_readfirstlane(d - 64 * c);
      if (rest <= 0) break;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      tr[lane] = p[c];
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int cnt = rest < 64 ? rest : 64;
      for (int f = 0; f < cnt; ++f) acc = acc + tr[f];
    }
    return acc;
  };
  for (int64_t lb = 0; lb < m; lb += 256 * kRrJ) {
    if (!one) chunk(lb);  // (one chunk: its dots are still in a)
#pragma unroll
    for (int j = 0; j < kRrJ; ++j) {
#pragma unroll
      for (int q = 0; q < kRrC; ++q) {
        unsigned long long near = __ballot(ok[j] && a[q][j] >= thr[q]);
        while (near) {  // (wave-uniform)
          const int src = __ffsll(static_cast<long long>(near)) - 1;
          near &= near - 1;
          const int64_t lr = static_cast<int64_t>(__shfl(l[j], src));
          const double acc = canon_dot(q, lr);
          if (acc > best[q] || (acc == best[q] && lr < arg[q])) {  // (wave-uniform)
            best[q] = acc;
            arg[q] = lr;
          }
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kRrC; ++q) {
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(best[q], o);
      const long long oa = __shfl_xor(arg[q], o);
      if (ob > best[q] || (ob == best[q] && oa < arg[q])) {
        best[q] = ob;
        arg[q] = oa;
      }
    }
    if (lane == 0) {
      rb[wave][q] = best[q];
      ra[wave][q] = arg[q];
    }
  }
  __syncthreads();
  if (tid < kRrC) {
    const int64_t c = c0 + tid;
    double b = rb[0][tid];
    long long a = ra[0][tid];
    for (int w = 1; w < 4; ++w) {
      if (rb[w][tid] > b || (rb[w][tid] == b && ra[w][tid] < a)) {
        b = rb[w][tid];
        a = ra[w][tid];
      }
    }
    if (c < count) {
      cpay[c] = b;
      ckey[c] = score_key(b, DAL_ASCENDING);
    } else if (c < cap) {
      ckey[c] = DAL_KEY_NONE;
    }
  }
}

__global__ __launch_bounds__(256) void gather_selected_kernel(const int64_t* __restrict__ pos,
                                                              const uint64_t* __restrict__ pkeys, int64_t k,
                                                              const int64_t* __restrict__ cidx,
                                                              const double* __restrict__ cpay,
                                                              int64_t* __restrict__ out_idx,
                                                              double* __restrict__ out_scores,
                                                              uint64_t* __restrict__ out_keys) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= k) return;
  const int64_t p = pos[t];
  out_idx[t] = cidx[p];
  out_scores[t] = cpay[p];
  if (out_keys) out_keys[t] = pkeys[t];
}

// ---------------------------------------------------------------- sort ----
// Fast-level-1 tail (summary_select_kernel): the candidate capacity check
// (more than cap candidates -> DAL_FLAG_SAMPLE_MISS: the caller re-runs with
// the exact level 1), and the words the next call needs zero -- the level-1
// counters and, when the score kernel folded its group minima with atomics,
// the minima -- cleared once every thread has read them, so a replayed
// hipGraph starts clean without a memset launch.
// Plan publishing (dal_dw_plan_run): out_slot points at two host-mapped
// words holding the device addresses the selected indices and scores are
// also written to (fresh tensors per step; NULL: none), status_mirror at a
// host-mapped copy of the status word written last -- the host reads both
// after its stream sync, with no copy launches after the graph.
struct SortTail {
  int64_t cap = 0;
  bool cap_miss = false;
  // candidates in n_reg regions of reg_stride entries (summary_select_kernel:
  // one per block, reg_count[r] each) instead of one list of cand_count
  int n_reg = 0;
  int64_t reg_stride = 0;
  const unsigned int* reg_count = nullptr;
  int64_t reg_uniform = 0;  // > 0: every region holds this many (no reg_count)
  // > 0: a region holding at most this many entries is sorted by (key, index)
  // (summary_select_kernel ranks its own candidates); when every region is,
  // the tail merges them instead of sorting
  int64_t sorted_max = 0;
  int32_t* status = nullptr;
  uint32_t* clear = nullptr;
  int64_t clear_words = 0;
  uint32_t* clear2 = nullptr;
  int64_t clear2_words = 0;
  int64_t* const* out_slot = nullptr;
  int32_t* status_mirror = nullptr;
};

__device__ __forceinline__ int64_t* load_out_slot(int64_t* const* slot, int which) {
  return slot ? __hip_atomic_load(const_cast<int64_t**>(slot) + which, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
              : nullptr;
}

__device__ __forceinline__ void publish_status(int32_t* status, int32_t* mirror) {
  const int32_t v = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(mirror, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Exact-level-1 plans: the same publishing as a separate one-block launch.
__global__ __launch_bounds__(256) void publish_kernel(const int64_t* __restrict__ out_idx,
                                                      const double* __restrict__ out_scores, int64_t k,
                                                      int64_t* const* out_slot, int32_t* status,
                                                      int32_t* status_mirror) {
  int64_t* const di = load_out_slot(out_slot, 0);
  double* const ds = reinterpret_cast<double*>(load_out_slot(out_slot, 1));
  for (int64_t i = threadIdx.x; i < k; i += 256) {
    if (di) di[i] = out_idx[i];
    if (ds) ds[i] = out_scores[i];
  }
  if (status_mirror) {
    __syncthreads();
    if (threadIdx.x == 0) publish_status(status, status_mirror);
  }
}

// Block radix select for sort_kernel: m (<= 4 * kSortThreads) keys, k-th
// smallest.  Digits of 8 bits MSB first over the keys that still match the
// resolved prefix; stops as soon as the k-th key's bucket holds <= kSelSmall
// keys.  Then the keys below the prefix (all in the top k) and the keys in
// the bucket are compacted (any order) into sk/si/sp[0..m_out).  Returns
// false (nothing written) when the bucket never shrinks that far (many equal
// keys): the caller sorts everything.  Block-uniform.
// Logical candidate e -> its slot: identity for one list, else region r with
// pre[r] <= e < pre[r + 1] (pre: LDS prefix sums of the region counts; empty
// regions repeat a value, the last such r is the one holding e).
struct RegionMap {
  int n = 0;
  int64_t stride = 0;
  const unsigned int* pre = nullptr;
  __device__ int64_t operator()(int64_t e) const {
    if (n == 0) return e;
    int lo = 0, hi = n - 1;  // the last r with pre[r] <= e (binary search: <= 5 LDS reads)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    return lo * stride + (e - pre[lo]);
  }
};

constexpr int64_t kSelMin = 1024;    // below this the full bitonic is cheap
#ifndef DAL_RANK_MAX
#define DAL_RANK_MAX 512
#endif
constexpr int64_t kRankMax = DAL_RANK_MAX;  // at most this many: rank selection, no sorting network
// wave min / max / count reductions of the selection's critical path by DPP
// (common.hpp) instead of ds_bpermute shuffles
#ifndef DAL_K3_DPP
#define DAL_K3_DPP 1
#endif

constexpr int64_t kSelMaxK = 1536;   // k + kSelSmall must fit the sort arrays
constexpr int kSelSmall = 512;

__device__ bool select_compact(const uint64_t* __restrict__ keys, const int64_t* __restrict__ idx,
                               const double* __restrict__ pay, const RegionMap& M, int64_t m, int64_t k,
                               unsigned long long* sk, long long* si, double* sp, int64_t& m_out) {
  __shared__ unsigned int hist[256];
  __shared__ unsigned long long s_prefix;
  __shared__ unsigned int s_krem, s_neq, s_count;
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int kPer = DAL_SORT_CAP_PAYLOAD / kSortThreads;  // 4
  // the indices and payloads are loaded with the keys (the compaction below
  // then needs no second coherent round trip)
  unsigned long long key[kPer];
  long long iv[kPer];
  double pv[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t e = tid + static_cast<int64_t>(j) * kSortThreads;
    key[j] = 0ull;
    iv[j] = 0;
    pv[j] = 0.0;
    if (e < m) {
      const int64_t q = M(e);
      key[j] = ld_sc1(keys + q);
      iv[j] = ld_sc1(idx + q);
      pv[j] = ld_sc1(pay + q);
    }
  }
  // the digits start below the keys' common high bits (for density-weighted
  // keys the sign and most of the exponent: the first 8-bit pass over them
  // put every key in one bin)
  __shared__ unsigned long long s_mn[kSortThreads / 64], s_mx[kSortThreads / 64];
  unsigned long long mn = ~0ull, mx = 0ull;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (tid + static_cast<int64_t>(j) * kSortThreads < m) {
      mn = key[j] < mn ? key[j] : mn;
      mx = key[j] > mx ? key[j] : mx;
    }
  }
#if DAL_K3_DPP
  mn = wave_min_u64_dpp(mn);
  mx = wave_max_u64_dpp(mx);
#else
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
#endif
  if (lane == 0) {
    s_mn[tid >> 6] = mn;
    s_mx[tid >> 6] = mx;
  }
  // the radix histogram is zeroed here and then by the scanning wave as it
  // reads each pass's bins: two barriers per pass instead of four
  if (tid < 256) hist[tid] = 0u;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kSortThreads / 64; ++q) {
    mn = s_mn[q] < mn ? s_mn[q] : mn;
    mx = s_mx[q] > mx ? s_mx[q] : mx;
  }
  int top = 64 - __clzll(static_cast<long long>(mn ^ mx));  // bits [0, top) still to resolve (0: all equal)
  unsigned long long mask = top == 64 ? 0ull : ~((1ull << top) - 1ull);
  unsigned long long prefix = mn & mask;
  unsigned int krem = static_cast<unsigned int>(k), neq = static_cast<unsigned int>(m);
  while (neq > static_cast<unsigned int>(kSelSmall) && top > 0) {  // (block-uniform)
    const int width = top < 8 ? top : 8, shift = top - width;
    const unsigned long long dmask = (1ull << width) - 1ull;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool valid = tid + j * kSortThreads < m && (key[j] & mask) == prefix;
      const unsigned bin = static_cast<unsigned>((key[j] >> shift) & dmask);
      // the wave's most common bin (the first valid lane's) with one atomic
      const unsigned long long vm = __ballot(valid);
      if (vm) {
        const int first = __ffsll(static_cast<long long>(vm)) - 1;
        const unsigned b0 = __shfl(bin, first);
        const unsigned long long m0 = __ballot(valid && bin == b0);
        if (lane == first) atomicAdd(&hist[b0], static_cast<unsigned>(__popcll(m0)));
        if (valid && bin != b0) atomicAdd(&hist[bin], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {  // one wave: 4 bins per lane (read, then zeroed for the next pass), inclusive scan, locate krem
      unsigned c[4], tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c[q] = hist[lane * 4 + q];
        hist[lane * 4 + q] = 0u;
        tot += c[q];
      }
      unsigned x = tot;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      unsigned run = x - tot;
      if (run < krem && run + tot >= krem) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (run < krem && run + c[q] >= krem) {
            s_prefix = prefix | (static_cast<unsigned long long>(lane * 4 + q) << shift);
            s_krem = krem - run;
            s_neq = c[q];
          }
          run += c[q];
        }
      }
    }
    __syncthreads();
    prefix = s_prefix;
    krem = s_krem;
    neq = s_neq;
    mask |= dmask << shift;
    top = shift;
  }
  if (neq > static_cast<unsigned int>(kSelSmall)) return false;
  // the k - krem keys below the prefix and the neq keys in its bucket
  if (tid == 0) s_count = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t e = tid + static_cast<int64_t>(j) * kSortThreads;
    const bool take = e < m && (key[j] & mask) <= prefix;
    const unsigned long long tm = __ballot(take);
    if (!tm) continue;
    unsigned base = 0;
    if (lane == 0) base = atomicAdd(&s_count, static_cast<unsigned>(__popcll(tm)));
    base = __shfl(base, 0);
    if (take) {
      const unsigned p = base + static_cast<unsigned>(__popcll(tm & ((1ull << lane) - 1ull)));
      sk[p] = key[j];
      si[p] = iv[j];
      sp[p] = pv[j];
    }
  }
  __syncthreads();
  m_out = s_count;
  return true;
}

// The sort tail as a block-level device function (kSortThreads threads): the
// The rank selection's lanes per element stop doubling once FILL x lanes x m
// would exceed the block (2: at most half the threads busy).
#ifndef DAL_K3_RANK_FILL
#define DAL_K3_RANK_FILL 2
#endif
// body of sort_kernel, also run by the last block of summary_select_kernel.
template <bool PAY>
__device__ void sort_tail_body(const uint64_t* __restrict__ keys, const int64_t* __restrict__ idx,
                               const double* __restrict__ pay, const TopkHdr* __restrict__ h, int64_t n_static,
                               int64_t k, uint64_t* __restrict__ out_keys, int64_t* __restrict__ out_idx,
                               double* __restrict__ out_pay, const SortTail& tail) {
  constexpr int CAP = PAY ? DAL_SORT_CAP_PAYLOAD : DAL_SORT_CAP;
  __shared__ unsigned long long sk[CAP];
  __shared__ long long si[CAP];
  __shared__ double sp[PAY ? CAP : 1];
  __shared__ int64_t* s_dest[2];
  const int tid = threadIdx.x;
  if (tid < 2) s_dest[tid] = load_out_slot(tail.out_slot, tid);  // host round trips, overlapping the sort
  __shared__ unsigned int s_pre[kMaxRegions + 1];
  __shared__ int s_runs_sorted, s_run_max;
  RegionMap M;
  int64_t m;
  // the first kSpecSlots entries of every region, loaded with the region
  // counts instead of after their scan (one coherent round trip fewer for the
  // rank selection of short lists: config 4, k = 100 holds <= 4 per region)
  constexpr int kSpecSlots = kSortThreads / kMaxRegions;  // 8
  const int spec_r = tid / kSpecSlots, spec_s = tid % kSpecSlots;
  const bool spec = PAY && tail.n_reg > 0 && spec_r < tail.n_reg && spec_s < tail.reg_stride;
  unsigned long long spec_k = 0;
  long long spec_i = 0;
  double spec_p = 0.0;
  if (spec) {
    const int64_t q = static_cast<int64_t>(spec_r) * tail.reg_stride + spec_s;
    spec_k = ld_sc1(keys + q);
    spec_i = ld_sc1(idx + q);
    if (PAY) spec_p = ld_sc1(pay + q);
  }
  if (tail.n_reg) {
    if (tid < 64) {
      // wave 0: the counts' loads in parallel, two regions per lane, and a
      // shuffle scan of the clamped counts (one thread summing 128 regions
      // serially cost ~4 us); a region over capacity makes the total a miss
      // while the offsets stay monotonic (every gather below stays inside its
      // region; the selection is then discarded by the host)
      const int r = 2 * tid;
      const unsigned long long stride = static_cast<unsigned long long>(tail.reg_stride);
      unsigned long long c0 = 0, c1 = 0;
      if (r < tail.n_reg) c0 = tail.reg_uniform ? tail.reg_uniform : ld_sc1(tail.reg_count + r);
      if (r + 1 < tail.n_reg) c1 = tail.reg_uniform ? tail.reg_uniform : ld_sc1(tail.reg_count + r + 1);
      const bool over = c0 > stride || c1 > stride;
      const unsigned long long smax = static_cast<unsigned long long>(tail.sorted_max);
      const bool unsorted = c0 > smax || c1 > smax;
      c0 = c0 < stride ? c0 : stride;
      c1 = c1 < stride ? c1 : stride;
      unsigned long long x = c0 + c1;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o);
        if (tid >= o) x += y;
      }
      const unsigned long long ex = x - c0 - c1;
      if (r < tail.n_reg) s_pre[r] = static_cast<unsigned>(ex);
      if (r + 1 < tail.n_reg) s_pre[r + 1] = static_cast<unsigned>(ex + c0);
      const bool miss = __ballot(over) != 0 || x > 0xFFFFFFFFull;
      const bool all_sorted = smax > 0 && __ballot(unsorted) == 0;
      unsigned long long cm = c0 > c1 ? c0 : c1;  // the longest region
#if DAL_K3_DPP
      cm = wave_max_u64_dpp(cm);
#else
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(cm, o);
        cm = y > cm ? y : cm;
      }
#endif
      if (tid == 63) {
        s_run_max = static_cast<int>(cm);
        s_pre[tail.n_reg] = miss ? 0xFFFFFFFFu : static_cast<unsigned>(x);
        s_runs_sorted = all_sorted && !miss;
      }
    }
    __syncthreads();
    M = RegionMap{tail.n_reg, tail.reg_stride, s_pre};
    m = s_pre[tail.n_reg];
  } else {
    m = !h ? n_static : static_cast<int64_t>(ld_sc1(&h->cand_count));
  }
  if (tail.cap_miss && tid == 0 && m > tail.cap) atomicOr(tail.status, DAL_FLAG_SAMPLE_MISS);
  if (tail.cap && m > tail.cap) m = tail.cap;
  if (m > CAP) m = CAP;
  // Sorted regions are merged when the rank selection is too long (m >
  // kRankMax) and the radix pre-selection would not shorten the sort much
  // (k + kSelSmall >= m: config 4 at k = 1,000, m = 1,261: bitonic 31 us,
  // merge 19 us); short lists keep the rank selection (k = 100, m = 135: 5 us
  // vs 8 us for the merge's seven levels) and long lists with a small k the
  // pre-selection (config 3: m = 1,700, k = 100).
  if constexpr (PAY) if (tail.n_reg > 1 && s_runs_sorted && static_cast<int64_t>(s_pre[tail.n_reg]) == m && m > kRankMax &&
      (m <= kSelMin || k + kSelSmall >= m) && m <= CAP / 2) {  // (every run whole: no capacity clamp above)
    // every region is a sorted run (summary_select_kernel ranked its own
    // candidates): a tree of pairwise merges, ceil(log2 regions) levels --
    // an entry's place in the merged pair is its offset in its own run plus
    // the count below it in the partner run (a binary search; ties between
    // runs, impossible for distinct indices, go to the left run).  The two
    // halves of the arrays alternate as source and destination.  Measured at
    // config 4, k = 1,000 (123 runs, m = 1,261): 19 us; 4- and 8-way groups
    // with their searches advanced together (branch-free, every probe's reads
    // issued at once) 41-45 us -- the probes' LDS reads, not their latency,
    // bound it.
    constexpr int H = CAP / 2;
    static_assert(H <= 2 * kSortThreads, "two entries per thread");
    __shared__ unsigned int s_bd2[kMaxRegions + 1];
    __shared__ unsigned char s_rid[2][H];  // each entry's run at the current level (< kMaxRegions)
    for (int i = tid; i < m; i += kSortThreads) {
      const int64_t q = M(i);
      sk[i] = ld_sc1(keys + q);
      si[i] = ld_sc1(idx + q);
      if (PAY) sp[i] = ld_sc1(pay + q);
      s_rid[0][i] = static_cast<unsigned char>(q / tail.reg_stride);
    }
    __syncthreads();
    if (tail.clear) {  // every thread read the header above
      for (int64_t w = tid; w < tail.clear_words; w += kSortThreads) tail.clear[w] = 0u;
      for (int64_t w = tid; w < tail.clear2_words; w += kSortThreads) tail.clear2[w] = 0u;
    }
    const int mm = static_cast<int>(m);
    const unsigned int* bd = s_pre;
    unsigned int* nbd = s_bd2;
    int nr = tail.n_reg, src = 0, run_max = s_run_max;
    while (nr > 1) {  // (block-uniform)
      int steps = 0;  // probes that settle a search over any run of this level
      while ((1 << steps) <= run_max) ++steps;
      const unsigned long long* ks = sk + src * H;
      const long long* is = si + src * H;
      const double* ps = sp + (PAY ? src * H : 0);
      unsigned long long* kd = sk + (src ^ 1) * H;
      long long* id = si + (src ^ 1) * H;
      double* pd = sp + (PAY ? (src ^ 1) * H : 0);
      // a thread's two entries (tid, tid + 1024) searched together: their
      // probes' reads in flight at once
      int e[2], a[2], lo[2], hi[2], base[2], pos[2];
      bool left[2];
      unsigned long long ke[2];
      long long ie[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        e[u] = tid + u * kSortThreads;
        const bool live = e[u] < mm;
        a[u] = live ? s_rid[src][e[u]] : 0;
        ke[u] = live ? ks[e[u]] : 0ull;
        ie[u] = live ? is[e[u]] : 0ll;
        const int r0 = a[u] & ~1;
        pos[u] = e[u];
        lo[u] = hi[u] = base[u] = 0;
        left[u] = a[u] == r0;
        if (live && r0 + 1 < nr) {
          const int lo0 = static_cast<int>(bd[r0]), mid0 = static_cast<int>(bd[r0 + 1]);
          const int hi0 = static_cast<int>(bd[r0 + 2]);
          lo[u] = base[u] = left[u] ? mid0 : lo0;  // the partner run
          hi[u] = left[u] ? hi0 : mid0;
          pos[u] = left[u] ? e[u] : lo0 + (e[u] - mid0);
        }
      }
      for (int s = 0; s < steps; ++s) {
        unsigned long long km[2];
        int mid[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          mid[u] = lo[u] < hi[u] ? (lo[u] + hi[u]) >> 1 : 0;
          km[u] = ks[mid[u]];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bool open = lo[u] < hi[u];
          // the index only on equal keys (LDS bandwidth bounds the probes)
          bool below = km[u] < ke[u];
          if (km[u] == ke[u]) {
            const long long im = is[mid[u]];
            below = left[u] ? im < ie[u] : im <= ie[u];
          }
          lo[u] = open && below ? mid[u] + 1 : lo[u];
          hi[u] = open && !below ? mid[u] : hi[u];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (e[u] < mm) {
          const int p = pos[u] + (lo[u] - base[u]);
          kd[p] = ke[u];
          id[p] = ie[u];
          if (PAY) pd[p] = ps[e[u]];
          s_rid[src ^ 1][p] = static_cast<unsigned char>(a[u] >> 1);
        }
      }
      const int nn = (nr + 1) >> 1;
      for (int j = tid; j <= nn; j += kSortThreads) nbd[j] = j < nn ? bd[2 * j] : bd[nr];
      __syncthreads();
      const unsigned int* t0 = bd;
      bd = nbd;
      nbd = const_cast<unsigned int*>(t0);
      nr = nn;
      src ^= 1;
      run_max = 2 * run_max < mm ? 2 * run_max : mm;
    }
    const unsigned long long* ks = sk + src * H;
    const long long* is = si + src * H;
    const double* ps = sp + (PAY ? src * H : 0);
    int64_t* const di = s_dest[0];  // written before the first barrier
    double* const ds = reinterpret_cast<double*>(s_dest[1]);
    const int64_t kk = k < m ? k : m;
    for (int i = tid; i < kk; i += kSortThreads) {
      if (out_keys) out_keys[i] = ks[i];
      out_idx[i] = is[i];
      if (PAY && out_pay) out_pay[i] = ps[i];
      if (di) di[i] = is[i];
      if (PAY && ds) ds[i] = ps[i];
    }
    if (PAY && h) {
      for (int64_t i = kk + tid; i < k; i += kSortThreads) {
        if (out_keys) out_keys[i] = DAL_KEY_NONE;
        out_idx[i] = -1;
        if (out_pay) out_pay[i] = __builtin_nan("");
        if (di) di[i] = -1;
        if (ds) ds[i] = __builtin_nan("");
      }
    }
    if (tail.status_mirror) {
      __syncthreads();
      if (tid == 0) publish_status(tail.status, tail.status_mirror);
    }
    return;
  }
  // Long lists (config 3: ~1,750 candidates, k = 100): a block radix select of
  // the k-th key first (8-bit digits, keys in registers), then only the keys
  // below its bucket plus the bucket itself (<= kSelSmall) are kept -- the
  // full bitonic over 4,096 keys is LDS-bound (~95 us).  Same result: every
  // key of the top k lies in the kept subset, which the rank selection below
  // orders when it is short (config 3: 168 kept; the bitonic over them took
  // 8.6 us) and the bitonic network otherwise.
  bool loaded = false;
  if (PAY && (h || tail.n_reg) && m > kSelMin && k <= kSelMaxK && k < m)
    loaded = select_compact(keys, idx, pay, M, m, k, sk, si, sp, m);
  if (m <= kRankMax) {
    // short lists (the common case: ~100-300 candidates): rank selection.
    // Every element's rank -- the count of smaller (key, index, position)
    // triples, read as LDS broadcasts -- is its output position: two
    // barriers instead of the bitonic network's log^2 m stages.  tpe lanes of
    // one wave share an element (each counts every tpe-th pair, a butterfly
    // adds them): m / tpe dependent LDS reads per lane instead of m (one
    // lane per element: ~10 us at m = 110).
    if (!loaded) {  // (block-uniform)
      // whole regions (no capacity clamp): the speculative entries, then the
      // slots past them of the longer regions
      const bool whole = PAY && tail.n_reg > 0 && static_cast<int64_t>(s_pre[tail.n_reg]) == m;
      if (whole) {
        if (spec && spec_s < static_cast<int>(s_pre[spec_r + 1] - s_pre[spec_r])) {
          const unsigned p = s_pre[spec_r] + static_cast<unsigned>(spec_s);
          sk[p] = spec_k;
          si[p] = spec_i;
          if (PAY) sp[p] = spec_p;
        }
      }
      if (!whole || s_run_max > kSpecSlots) {  // (block-uniform)
        for (int i = tid; i < m; i += kSortThreads) {
          const int64_t q = M(i);
          if (whole && q % tail.reg_stride < kSpecSlots) continue;
          sk[i] = ld_sc1(keys + q);
          si[i] = ld_sc1(idx + q);
          if (PAY) sp[i] = ld_sc1(pay + q);
        }
      }
      __syncthreads();
    }
    if (tail.clear) {  // every thread read the header above
      for (int64_t w = tid; w < tail.clear_words; w += kSortThreads) tail.clear[w] = 0u;
      for (int64_t w = tid; w < tail.clear2_words; w += kSortThreads) tail.clear2[w] = 0u;
    }
    int64_t* const di = s_dest[0];
    double* const ds = reinterpret_cast<double*>(s_dest[1]);
    const int64_t kk = k < m ? k : m;
    int tpe = 1;  // lanes per element: a power of two <= 64, tpe * m <= kSortThreads
    while (tpe < 64 && DAL_K3_RANK_FILL * tpe * m <= kSortThreads) tpe <<= 1;
    const int part = tid & (tpe - 1);
    for (int e0 = 0; e0 < m; e0 += kSortThreads / tpe) {  // block-uniform
      const int e = e0 + tid / tpe;
      const bool live = e < m;
      const unsigned long long ke = live ? sk[e] : 0ull;
      const long long ie = live ? si[e] : 0ll;
      // keys only (one 8-B read and two compares per pair); an element whose
      // key occurs more than once (equal scores, the merge's NONE padding)
      // is recounted on (key, index, position)
      int r = 0, eq = 0;
      if (live) {
#pragma unroll 4
        for (int j = part; j < m; j += tpe) {
          const unsigned long long kj = sk[j];
          r += kj < ke;
          eq += kj == ke;
        }
      }
      for (int o = 1; o < tpe; o <<= 1) {
        r += __shfl_xor(r, o);
        eq += __shfl_xor(eq, o);
      }
      if (__ballot(live && eq > 1)) {  // (wave-uniform; rare)
        const bool again = live && eq > 1;  // (the same for an element's tpe lanes)
        int rr = 0;
        if (again) {
          for (int j = part; j < m; j += tpe) {
            const unsigned long long kj = sk[j];
            const long long ij = si[j];
            // equal pairs (the merge's padding: NONE key, index -1) rank by position
            rr += kj < ke || (kj == ke && (ij < ie || (ij == ie && j < e)));
          }
        }
        for (int o = 1; o < tpe; o <<= 1) rr += __shfl_xor(rr, o);
        if (again) r = rr;
      }
      if (live && part == 0 && r < kk) {
        if (out_keys) out_keys[r] = ke;
        out_idx[r] = ie;
        if (PAY && out_pay) out_pay[r] = sp[e];
        if (di) di[r] = ie;
        if (PAY && ds) ds[r] = sp[e];
      }
    }
    if (PAY && h) {
      for (int64_t i = kk + tid; i < k; i += kSortThreads) {
        if (out_keys) out_keys[i] = DAL_KEY_NONE;
        out_idx[i] = -1;
        if (out_pay) out_pay[i] = __builtin_nan("");
        if (di) di[i] = -1;
        if (ds) ds[i] = __builtin_nan("");
      }
    }
    if (tail.status_mirror) {
      __syncthreads();
      if (tid == 0) publish_status(tail.status, tail.status_mirror);
    }
    return;
  }
  int mp = 2;
  while (mp < m) mp <<= 1;
  for (int i = tid; i < mp; i += kSortThreads) {
    if (loaded) {
      if (i >= m) {
        sk[i] = ~0ull;
        si[i] = 0x7FFFFFFFFFFFFFFFll;
        if (PAY) sp[i] = 0.0;
      }
    } else if (i < m) {
      const int64_t q = M(i);
      sk[i] = ld_sc1(keys + q);
      si[i] = ld_sc1(idx + q);
      if (PAY) sp[i] = ld_sc1(pay + q);
    } else {
      sk[i] = ~0ull;
      si[i] = 0x7FFFFFFFFFFFFFFFll;
      if (PAY) sp[i] = 0.0;
    }
  }
  __syncthreads();
  for (int size = 2; size <= mp; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (mp >> 1); t += kSortThreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long ka = sk[lo], kb = sk[hi];
        const long long ia = si[lo], ib = si[hi];
        const bool a_gt_b = ka > kb || (ka == kb && ia > ib);
        if (a_gt_b == up) {
          sk[lo] = kb;
          sk[hi] = ka;
          si[lo] = ib;
          si[hi] = ia;
          if (PAY) {
            const double t0 = sp[lo];
            sp[lo] = sp[hi];
            sp[hi] = t0;
          }
        }
      }
      __syncthreads();
    }
  }
  if (tail.clear) {  // every thread read the header before the first barrier above
    for (int64_t w = tid; w < tail.clear_words; w += kSortThreads) tail.clear[w] = 0u;
    for (int64_t w = tid; w < tail.clear2_words; w += kSortThreads) tail.clear2[w] = 0u;
  }
  int64_t* const di = s_dest[0];  // written before the first barrier
  double* const ds = reinterpret_cast<double*>(s_dest[1]);
  const int64_t kk = k < m ? k : m;
  for (int i = tid; i < kk; i += kSortThreads) {
    if (out_keys) out_keys[i] = sk[i];
    out_idx[i] = si[i];
    if (PAY && out_pay) out_pay[i] = sp[i];
    if (di) di[i] = si[i];
    if (PAY && ds) ds[i] = sp[i];
  }
  // candidate lists (h != null) shorter than k -- a shard with fewer than k
  // unlabeled rows under the sampled level 1 -- are padded with the NONE key
  if (PAY && h) {
    for (int64_t i = kk + tid; i < k; i += kSortThreads) {
      if (out_keys) out_keys[i] = DAL_KEY_NONE;
      out_idx[i] = -1;
      if (out_pay) out_pay[i] = __builtin_nan("");
      if (di) di[i] = -1;
      if (ds) ds[i] = __builtin_nan("");
    }
  }
  if (tail.status_mirror) {  // last: every status writer of the step has finished
    __syncthreads();
    if (tid == 0) publish_status(tail.status, tail.status_mirror);
  }
}

template <bool PAY>
__global__ __launch_bounds__(kSortThreads) void sort_kernel(const uint64_t* __restrict__ keys,
                                                            const int64_t* __restrict__ idx,
                                                            const double* __restrict__ pay,
                                                            const TopkHdr* __restrict__ h,
                                                            int64_t n_static, int64_t k,
                                                            uint64_t* __restrict__ out_keys,
                                                            int64_t* __restrict__ out_idx,
                                                            double* __restrict__ out_pay, SortTail tail) {
  sort_tail_body<PAY>(keys, idx, pay, h, n_static, k, out_keys, out_idx, out_pay, tail);
}

// ------------------------------------- fast level 1 (row-group minima) ----
constexpr int kMaxGroups = 4096;             // row groups of the fast level 1
constexpr int kSumThreads = kSortThreads;    // 1024: the last block runs the sort tail

// ginv[g] = ~(minimum pessimistic key of group g), ginv[ng + g] = ~(minimum
// optimistic key): inverted so that a zeroed buffer reads DAL_KEY_NONE and an
// atomic max folds a minimum.  Group g = rows [g * group_rows, ...).
struct GroupSummary {
  const uint64_t* ginv;
  int64_t ng;
  int64_t group_rows;
};

// tau = the k-th smallest of the groups' minimum pessimistic keys (NONE when
// fewer than k groups hold a key): k group minima are k keys of the pool, so
// at least k keys are <= tau, i.e. tau >= K.  Block radix select over the
// keys' differing low bits (the common high bits of the minimum and maximum
// -- for DW keys the sign and most of the exponent -- are skipped; up to 4
// keys per thread in registers, 8-bit digits) until the k-th key's bucket
// holds <= 64 keys; tau is that bucket's upper edge.  Every block computes it
// (no grid sync).
#ifndef DAL_TAU_BUCKET
#define DAL_TAU_BUCKET 64  // radix passes stop once the k-th key's bucket holds at most this many minima (256 / 1024: neutral)
#endif
struct NoHook {
  __device__ void operator()() const {}
};
// after_load: called by every thread once the minima are in registers (their
// loads waited for), before the radix passes -- the select kernel issues its
// prefetches there, to land while tau is computed.
template <class Hook = NoHook>
__device__ unsigned long long group_threshold(const GroupSummary& S, int64_t k, const Hook& after_load = Hook{}) {
  constexpr int PER = kMaxGroups / kSumThreads;
  constexpr int W = kSumThreads / 64;
  __shared__ unsigned int hist[256];
  __shared__ unsigned long long s_prefix, s_mn[W], s_mx[W];
  __shared__ unsigned int s_krem, s_cnt, s_nv[W];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (k > S.ng) return DAL_KEY_NONE;
  unsigned long long key[PER];
  bool val[PER];
  unsigned long long mn = DAL_KEY_NONE, mx = 0;
  unsigned nv = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int64_t g = tid + static_cast<int64_t>(j) * kSumThreads;
    key[j] = g < S.ng ? ~S.ginv[g] : DAL_KEY_NONE;
    val[j] = key[j] != DAL_KEY_NONE;
    if (val[j]) {
      mn = key[j] < mn ? key[j] : mn;
      mx = key[j] > mx ? key[j] : mx;
      ++nv;
    }
  }
#if DAL_K3_DPP
  mn = wave_min_u64_dpp(mn);
  mx = wave_max_u64_dpp(mx);
  nv = wave_sum_u32_dpp(nv);
#else
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    nv += __shfl_xor(nv, o);
  }
#endif
  if (lane == 0) {
    s_mn[w] = mn;
    s_mx[w] = mx;
    s_nv[w] = nv;
  }
  // the radix histogram is zeroed here (this barrier orders it before the
  // first pass) and then by the scanning wave as it reads each pass's bins:
  // two barriers per pass instead of three
  if (tid < 256) hist[tid] = 0u;
  after_load();
  __syncthreads();
  nv = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    mn = s_mn[q] < mn ? s_mn[q] : mn;
    mx = s_mx[q] > mx ? s_mx[q] : mx;
    nv += s_nv[q];
  }
  if (nv < k) return DAL_KEY_NONE;  // (block-uniform)
  if (mn == mx) return mn;
  int top = 64 - __clzll(static_cast<long long>(mn ^ mx));  // bits [0, top) still to resolve
  unsigned long long mask = top == 64 ? 0ull : ~((1ull << top) - 1ull);
  unsigned long long prefix = mn & mask;
  unsigned int krem = static_cast<unsigned int>(k), cnt = nv;
  while (cnt > DAL_TAU_BUCKET && top > 0) {
    const int width = top < 8 ? top : 8, shift = top - width;
    const unsigned dmask = (1u << width) - 1u;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const bool valid = val[j] && (key[j] & mask) == prefix;
      const unsigned bin = static_cast<unsigned>(key[j] >> shift) & dmask;
      const unsigned long long vm = __ballot(valid);
      if (vm) {  // the wave's most common bin (the first valid lane's) with one atomic
        const int first = __ffsll(static_cast<long long>(vm)) - 1;
        const unsigned b0 = __shfl(bin, first);
        const unsigned long long m0 = __ballot(valid && bin == b0);
        if (lane == first) atomicAdd(&hist[b0], static_cast<unsigned>(__popcll(m0)));
        if (valid && bin != b0) atomicAdd(&hist[bin], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {  // one wave: 4 bins per lane (read, then zeroed for the next pass), inclusive scan, locate krem
      unsigned c[4], tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c[q] = hist[lane * 4 + q];
        hist[lane * 4 + q] = 0u;
        tot += c[q];
      }
      unsigned x = tot;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      unsigned run = x - tot;
      if (run < krem && run + tot >= krem) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (run < krem && run + c[q] >= krem) {
            s_prefix = prefix | (static_cast<unsigned long long>(lane * 4 + q) << shift);
            s_krem = krem - run;
            s_cnt = c[q];
          }
          run += c[q];
        }
      }
    }
    __syncthreads();
    prefix = s_prefix;
    krem = s_krem;
    cnt = s_cnt;
    mask |= static_cast<unsigned long long>(dmask) << shift;
    top = shift;
  }
  // the upper edge of the k-th key's bucket: >= the k-th group minimum, and at
  // most the bucket's <= 64 keys above it (ranking them exactly -- a gather
  // and two more barriers -- cost more than the few extra candidates)
  return prefix | (top >= 64 ? ~0ull : ((1ull << top) - 1ull));
}

// Group minima of the keys (the standalone selections; dal_dw_step's score
// kernel writes them itself on pools of >= 2k blocks): groups of >= 64 rows
// take one wave each (8 x 64 keys in flight); smaller groups (a power of two
// of rows) are lane segments of a wave: one coalesced key per lane and a
// butterfly over each segment.  Block 0 also zeroes the fast-path header words.
__global__ __launch_bounds__(256) void group_min_kernel(const uint64_t* __restrict__ keys_lo,
                                                        const uint64_t* __restrict__ keys_hi, int64_t n,
                                                        int64_t group_rows, int64_t ng, uint64_t* __restrict__ ginv,
                                                        uint32_t* __restrict__ zero, int64_t zero_words) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (blockIdx.x == 0 && zero)
    for (int64_t w = tid; w < zero_words; w += 256) zero[w] = 0u;
  unsigned long long lo = DAL_KEY_NONE, hi = DAL_KEY_NONE;
  if (group_rows < 64) {  // segments of group_rows lanes
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid;
    if (i < n) {
      lo = keys_lo[i];
      hi = pack_hint(keys_hi[i], i % group_rows);
    }
    for (int o = 1; o < group_rows; o <<= 1) {
      const unsigned long long a = __shfl_xor(lo, o), c = __shfl_xor(hi, o);
      lo = a < lo ? a : lo;
      hi = c < hi ? c : hi;
    }
    const int64_t g = i / group_rows;
    if ((lane & (group_rows - 1)) == 0 && g < ng) {
      ginv[g] = ~lo;
      ginv[ng + g] = ~hi;
    }
    return;
  }
  const int64_t g = static_cast<int64_t>(blockIdx.x) * 4 + (tid >> 6);  // a wave per group
  if (g >= ng) return;
  const int64_t r0 = g * group_rows;
  const int64_t r1 = r0 + group_rows < n ? r0 + group_rows : n;
  constexpr int kIlp = 8;
  for (int64_t b = r0; b < r1; b += kIlp * 64) {
    unsigned long long a[kIlp], c[kIlp];
#pragma unroll
    for (int j = 0; j < kIlp; ++j) {
      const int64_t i = b + j * 64 + lane;
      a[j] = i < r1 ? keys_lo[i] : DAL_KEY_NONE;
      c[j] = i < r1 ? keys_hi[i] : DAL_KEY_NONE;
    }
#pragma unroll
    for (int j = 0; j < kIlp; ++j) {
      const unsigned long long cj = pack_hint(c[j], b + j * 64 + lane - r0);
      lo = a[j] < lo ? a[j] : lo;
      hi = cj < hi ? cj : hi;
    }
  }
#if DAL_K3_DPP
  lo = wave_min_u64_dpp(lo);
  hi = wave_min_u64_dpp(hi);
#else
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(lo, o), c = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = c < hi ? c : hi;
  }
#endif
  if (lane == 0) {
    ginv[g] = ~lo;
    ginv[ng + g] = ~hi;
  }
}

// The fast level 1 over the group minima (see the top of the file).  Block b
// owns groups [b * per, (b + 1) * per): those whose optimistic minimum is
// <= tau are listed in LDS and scanned by the block's waves (a group's rows,
// 8 x 64 keys in flight per wave); each 64-row slice with candidates reserves
// its slots with one atomic.  DW: the candidates are listed in LDS, then
// scored by all of the block's waves (canonical fp64: <= one per wave by the
// whole wave, more by one lane each), and the block that arrives last sorts
// the candidates (sort_tail_body: capacity check, selection, header clear).
// !DW: indices only (a separate re-rank follows).
// candidates per wave scored by whole waves (one after another) before the
// lane form takes over: at d = 256 a whole-wave score costs ~4.4 us with four
// waves per SIMD, a wave's lane pass ~17 us whatever it holds
constexpr int kWaveScoreMax = 3;
// a block whose list holds at most this many ranks them and writes its region
// sorted (SortTail::sorted_max): the last block then merges instead of sorting
constexpr int kLocalSort = 256;
// features per load round of a lane-scored candidate (all of a round's loads
// in flight before its divisions: 8 left a d = 256 row 32 dependent HBM round
// trips, ~86 us for a block holding a few dozen candidates)
#ifndef DAL_K3_LANE_CHUNK
#define DAL_K3_LANE_CHUNK 64
#endif

template <bool DW>
__global__ __launch_bounds__(kSumThreads) void summary_select_kernel(
    const uint64_t* __restrict__ keys_hi, int64_t n, int64_t k, int64_t idx_base, GroupSummary S,
    TopkHdr* __restrict__ h, int64_t* __restrict__ cidx, int64_t cap, AppendRerank AR, int n_lut,
    uint64_t* __restrict__ out_keys, int64_t* __restrict__ out_idx, double* __restrict__ out_scores, SortTail tail) {
  constexpr int W = kSumThreads / 64;
  __shared__ int s_hits[kMaxGroups / 32];  // per <= 128 groups (summary_grid)
  __shared__ unsigned s_nh, s_nc, s_last;
  // DW: the block's candidate rows, listed by the scan and scored after it;
  // a short list's (key, index, score) staged for its rank sort
  __shared__ int s_cand[DW ? DAL_SORT_CAP_PAYLOAD : 1];
  __shared__ unsigned long long s_lk[DW ? kLocalSort : 1];
  __shared__ long long s_li[DW ? kLocalSort : 1];
  __shared__ double s_lp[DW ? kLocalSort : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t per = ceil_div(S.ng, static_cast<int64_t>(gridDim.x));
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * per;
  const int64_t g1 = g0 + per < S.ng ? g0 + per : S.ng;
  // this block's groups' optimistic minima (<= 128: one per thread), loaded
  // with tau's inputs; DW: each one's hinted row (its offset in the group,
  // pack_hint) is prefetched while tau is computed -- the candidates are
  // nearly always those rows, and their canonical re-rank then reads them
  // from L2 (the warm plan's score kernel never touches the row-major pool)
  const unsigned long long my_m = tid < g1 - g0 ? ~S.ginv[S.ng + g0 + tid] : DAL_KEY_NONE;
  __shared__ __attribute__((aligned(16))) unsigned s_pf[DW ? 64 : 1];  // the prefetch DMA's landing slots (never read)
  auto prefetch = [&]() {
    if constexpr (DW) {
      const int64_t off = static_cast<int64_t>(my_m & kHintMask);
      const int64_t row = (g0 + tid) * S.group_rows + off;
      if (my_m != DAL_KEY_NONE && off < S.group_rows && row < n) prefetch_row(AR.R, row, s_pf);
    }
  };
  const unsigned long long tau = group_threshold(S, k, prefetch);
  if (blockIdx.x == 0 && tid == 0) h->kstar = tau;
  if (tid == 0) {
    s_nh = 0u;
    s_nc = 0u;
  }
  __syncthreads();
  if ((my_m & ~kHintMask) <= tau && my_m != DAL_KEY_NONE)  // (masked: the exact minimum <= tau implies it)
    s_hits[atomicAdd(&s_nh, 1u)] = static_cast<int>(g0 + tid);
  __syncthreads();
  const int nh = static_cast<int>(s_nh);
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  // DW: the list holds at most this many (the region's capacity)
  const int64_t kept = DW ? (cap < DAL_SORT_CAP_PAYLOAD ? cap : DAL_SORT_CAP_PAYLOAD) : cap;
  constexpr int kIlp = 8;
  for (int q = w; q < nh; q += W) {
    const int64_t r0 = static_cast<int64_t>(s_hits[q]) * S.group_rows;
    const int64_t r1 = r0 + S.group_rows < n ? r0 + S.group_rows : n;
    for (int64_t b = r0; b < r1; b += kIlp * 64) {
      unsigned long long hk[kIlp];
#pragma unroll
      for (int j = 0; j < kIlp; ++j) {
        const int64_t i = b + j * 64 + lane;
        hk[j] = i < r1 ? keys_hi[i] : DAL_KEY_NONE;
      }
      unsigned cbits = 0;  // bit j: this lane's row of slice j is a candidate
#pragma unroll
      for (int j = 0; j < kIlp; ++j) cbits |= (hk[j] <= tau && hk[j] != DAL_KEY_NONE ? 1u : 0u) << j;
      if (!__ballot(cbits != 0)) continue;
#pragma unroll 1
      for (int j = 0; j < kIlp; ++j) {
        const int64_t i = b + j * 64 + lane;
        const bool cand = (cbits >> j) & 1u;
        const unsigned long long cm = __ballot(cand);
        if (!cm) continue;
        if constexpr (DW) {
          // slots in this block's list (an LDS counter: same-address device
          // atomics from ~100 waves serialised at ~0.1 us each)
          unsigned base = 0;
          if (lane == 0) base = atomicAdd(&s_nc, static_cast<unsigned>(__popcll(cm)));
          const int64_t p = static_cast<int64_t>(__shfl(base, 0)) + __popcll(cm & lt_mask);
          if (cand && p < kept) s_cand[p] = static_cast<int>(i);
        } else {
          unsigned base = 0;
          if (lane == 0) base = atomicAdd(&h->cand_count, static_cast<unsigned>(__popcll(cm)));
          const int64_t p = static_cast<int64_t>(__shfl(base, 0)) + __popcll(cm & lt_mask);
          if (cand && p < cap) cidx[p] = idx_base + i;
        }
      }
    }
  }
  if constexpr (!DW) return;
  // Score the listed candidates (canonical fp64, density_weighting.py:148,
  // 157-167), spread over the block's waves whichever waves found them: up to
  // kWaveScoreMax per wave, each by the whole wave (its features' loads and divisions in
  // flight together, the oracle's sequential sum through the lanes); more, by
  // one lane each in as few waves as hold them: a wave's lane pass is fp64
  // division-bound and costs the same for 1 candidate as for 64 (dealing 40
  // candidates round-robin put every wave, four per SIMD, through it: ~60 us).
  __syncthreads();
  const int nc = static_cast<int>(s_nc < kept ? s_nc : kept);
  const double lut_lane = lane < n_lut ? AR.R.lut[lane] : 0.0;
  const int64_t reg0 = static_cast<int64_t>(blockIdx.x) * cap;
  // a short list is staged in LDS and written to the region sorted by (key,
  // index) -- each entry at its rank -- so the last block merges the regions
  const bool local = nc <= kLocalSort;  // (block-uniform)
  auto put = [&](int c, int64_t i, double sc, bool ok) {
    const unsigned long long key = ok ? score_key(sc, DAL_DESCENDING) : DAL_KEY_NONE;
    if (local) {
      s_lk[c] = key;
      s_li[c] = idx_base + i;
      s_lp[c] = sc;
    } else {
      st_sc1(cidx + reg0 + c, static_cast<int64_t>(idx_base + i));
      st_sc1(AR.cpay + reg0 + c, sc);
      st_sc1(AR.ckey + reg0 + c, static_cast<uint64_t>(key));
    }
  };
  // Every listed row is < n by construction (the scan writes slot p < kept
  // only, nc <= kept is read after the barrier above).  The row is still
  // checked before it forms an address (x + i * ldx, norm64, votes, flags): a
  // slot read before its write -- the round-4 work-in-progress aperture
  // violation ("Aperture violation") -- then costs a
  // DAL_FLAG_SAMPLE_MISS (exact re-run) instead of a wild load.
  auto row_ok = [&](int64_t i) { return static_cast<uint64_t>(i) < static_cast<uint64_t>(n); };
  if (nc <= kWaveScoreMax * W) {  // (block-uniform)
    __shared__ __attribute__((aligned(16))) double s_tr[DW ? W : 1][64];
    for (int c = w; c < nc; c += W) {  // (wave-uniform)
      const int64_t i = s_cand[c];
      double sc = __builtin_nan("");
      bool ok = false;
      if (row_ok(i)) ok = dw_canonical_score_wave(AR.R, i, sc, s_tr[DW ? w : 0], lut_lane, n_lut);
      else if (lane == 0) atomicOr(tail.status, DAL_FLAG_SAMPLE_MISS);
      if (lane == 0) put(c, i, sc, ok);
    }
  } else {
    for (int c0 = 0; c0 < nc; c0 += kSumThreads) {  // (block-uniform trip count)
      const int c = c0 + tid;  // packed: as few waves as hold them, waves 0-3 on four SIMDs
      const int64_t i = c < nc ? s_cand[c] : 0;
      const bool live = c < nc && row_ok(i);
      if (c < nc && !live) atomicOr(tail.status, DAL_FLAG_SAMPLE_MISS);
      const int v = live ? AR.R.votes[i] : 0;
      const double e = n_lut ? __shfl(lut_lane, v) : 0.0;  // (every lane takes part)
      if (live) {
        double sc;
        const bool ok = dw_canonical_score_lane<DAL_K3_LANE_CHUNK>(AR.R, i, sc, e, n_lut);
        put(c, i, sc, ok);
      } else if (c < nc) {
        put(c, i, __builtin_nan(""), false);
      }
    }
  }
  __syncthreads();
  if (local) {
    for (int c = tid; c < nc; c += kSumThreads) {
      const unsigned long long kc = s_lk[c];
      const long long ic = s_li[c];
      int r = 0;
      for (int j = 0; j < nc; ++j) {
        const unsigned long long kj = s_lk[j];
        const long long ij = s_li[j];
        r += kj < kc || (kj == kc && ij < ic);
      }
      st_sc1(cidx + reg0 + r, static_cast<int64_t>(ic));
      st_sc1(AR.cpay + reg0 + r, s_lp[c]);
      st_sc1(AR.ckey + reg0 + r, static_cast<uint64_t>(kc));
    }
  }
  // this block's count, then the last block to arrive sorts the candidates
  if (tid == 0) st_sc1(&h->reg_count[blockIdx.x], s_nc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(&h->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == gridDim.x - 1;  // the returned value: every other block's stores are complete
  }
  __syncthreads();
  if (!s_last) return;
  sort_tail_body<true>(AR.ckey, cidx, AR.cpay, h, int64_t{0}, k, out_keys, out_idx, out_scores, tail);
}

// Zero the header with a kernel rather than hipMemsetAsync: the select is
// replayed inside hipGraphs (engine.WarmStepGraph), where a captured memset
// node did not clear the header on every replay (observed on gfx950 / ROCm 7).
__global__ __launch_bounds__(256) void zero_words_kernel(uint32_t* __restrict__ p, int64_t words) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < words;
       i += static_cast<int64_t>(gridDim.x) * 256)
    p[i] = 0u;
}

constexpr int64_t kHdrWords = sizeof(TopkHdr) / 4;
static_assert(sizeof(TopkHdr) % 4 == 0, "header is whole words");
constexpr int64_t kFastHdrWords = offsetof(TopkHdr, kfinal) / 4;  // cand_count, arrive, kstar

void zero_words(uint32_t* p, int64_t words, hipStream_t st) {
  hipLaunchKernelGGL(zero_words_kernel, dim3(static_cast<unsigned>(ceil_div(words, 256 * 4))), dim3(256), 0, st, p,
                     words);
}

void zero_header(TopkHdr* h, hipStream_t st) { zero_words(reinterpret_cast<uint32_t*>(h), kHdrWords, st); }

// Row groups of the fast level 1: whole blocks of `unit` rows, at most
// kMaxGroups groups.
GroupSummary make_groups(const uint64_t* ginv, int64_t n, int64_t unit) {
  const int64_t units = ceil_div(n, unit);
  const int64_t per = ceil_div(units, kMaxGroups);
  return GroupSummary{ginv, ceil_div(units, per), per * unit};
}

// The group layout of launch_group_min: at most kMaxGroups groups; groups
// below a wave are a power of two of rows (lane segments).
GroupSummary group_min_layout(const uint64_t* ginv, int64_t n) {
  int64_t rows = ceil_div(n, kMaxGroups), unit = 1;
  while (unit < rows && unit < 64) unit <<= 1;
  return make_groups(ginv, n, unit);
}

// The minima of both keys over kMaxGroups (or n) groups, by group_min_kernel
// (which also zeroes `zero_words` words at `zero`).
GroupSummary launch_group_min(const uint64_t* keys_lo, const uint64_t* keys_hi, int64_t n, uint64_t* ginv,
                              uint32_t* zero, int64_t zero_words, hipStream_t st) {
  const GroupSummary S = group_min_layout(ginv, n);
  const int64_t blocks = S.group_rows < 64 ? ceil_div(n, 256) : ceil_div(S.ng, 4);
  hipLaunchKernelGGL(group_min_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, keys_lo, keys_hi, n,
                     S.group_rows, S.ng, ginv, zero, zero_words);
  return S;
}

// summary_select_kernel's grid: <= 32 groups per block (each block derives
// tau itself; 128 blocks x 32 = kMaxGroups), so a block's hits fit its list
// and its candidates' canonical scores (fp64 divisions: VALU-bound when a CU
// holds many) spread over up to 128 CUs -- 32 blocks of 128 groups left
// config 4 at k = 1,000 ~2.5 candidates per wave on a quarter of the CUs.
#ifndef DAL_K3_GROUPS_PER_BLOCK
#define DAL_K3_GROUPS_PER_BLOCK 32
#endif
static_assert(kMaxGroups / DAL_K3_GROUPS_PER_BLOCK <= kMaxRegions, "regions");
int summary_grid(int64_t ng) {
  int64_t g = ceil_div(ng, DAL_K3_GROUPS_PER_BLOCK);
  if (g > kMaxRegions) g = kMaxRegions;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}
// The LDS lists of summary_select_kernel hold a block's groups (s_hits:
// kMaxGroups / 32) and its regions' counts (kMaxRegions): a grid / group
// summary outside them is rejected on the host before the launch.
bool summary_shape_ok(const GroupSummary& S, int G, int64_t cap) {
  if (S.ng < 1 || S.ng > kMaxGroups || S.group_rows < 1 || G < 1 || G > kMaxRegions) return false;
  if (ceil_div(S.ng, static_cast<int64_t>(G)) > kMaxGroups / 32) return false;
  return cap >= 1 && cap <= DAL_SORT_CAP_PAYLOAD;
}

// Radix passes 0 .. passes-1 (zero: clear the header first).
int run_radix(const uint64_t* keys, int64_t n, int64_t k, TopkHdr* h, hipStream_t st, int passes = kPasses,
              bool zero = true) {
  if (zero) zero_header(h, st);
  // each block flushes up to 2048 bins with global atomics: beyond ~256
  // blocks the flush, not the key stream, sets a pass's time (2M keys: 977
  // blocks -> 2M atomics)
  int64_t blocks = ceil_div(n, kRadixThreads * 8);
  if (blocks > 256) blocks = 256;
  if (blocks < 1) blocks = 1;
  for (int p = 0; p < passes; ++p) {
    hipLaunchKernelGGL(radix_hist_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kRadixThreads), 0,
                       st, keys, n, k, p, h);
  }
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

template <bool INTERVAL>
int run_compact(const uint64_t* keys, const IntervalArgs& I, int64_t n, int64_t idx_base, int64_t k,
                void* ws, const TopkLayout& L, int32_t* status, hipStream_t st) {
  char* base = static_cast<char*>(ws);
  TopkHdr* h = reinterpret_cast<TopkHdr*>(base + L.hdr);
  uint32_t* blk = reinterpret_cast<uint32_t*>(base + L.blk);
  uint32_t* off = reinterpret_cast<uint32_t*>(base + L.off);
  const dim3 g(static_cast<unsigned>(L.nb));
  hipLaunchKernelGGL(compact_count_kernel<INTERVAL>, g, dim3(kRadixThreads), 0, st, keys, I, n, h, blk);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, blk, off, L.nb, h);
  hipLaunchKernelGGL(compact_write_kernel<INTERVAL>, g, dim3(kRadixThreads), 0, st, keys, I, n,
                     idx_base, k, h, off, reinterpret_cast<uint64_t*>(base + L.ckey),
                     reinterpret_cast<int64_t*>(base + L.cidx), L.cap, status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" size_t dal_topk_workspace_bytes(int64_t n, int64_t k) {
  return topk_layout(n, k < 1 ? 1 : k).total;
}

extern "C" int dal_topk(const uint64_t* keys, int64_t n, int64_t k, int64_t idx_base, void* ws,
                        size_t ws_bytes, int64_t* out_idx, uint64_t* out_keys, dal_stream_t stream) {
  if (!keys || !ws || !out_idx) return DAL_ERR_ARG;
  if (n < 1 || k < 1 || k > n) return DAL_ERR_SHAPE;
  if (k > DAL_SORT_CAP) return DAL_ERR_CAPACITY;
  const TopkLayout L = topk_layout(n, k);
  if (ws_bytes < L.total || (reinterpret_cast<uintptr_t>(ws) & 255)) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  TopkHdr* h = reinterpret_cast<TopkHdr*>(static_cast<char*>(ws) + L.hdr);
  int rc = run_radix(keys, n, k, h, st);
  if (rc) return rc;
  rc = run_compact<false>(keys, IntervalArgs{nullptr}, n, idx_base, k, ws, L, nullptr, st);
  if (rc) return rc;
  char* base = static_cast<char*>(ws);
  hipLaunchKernelGGL(sort_kernel<false>, dim3(1), dim3(kSortThreads), 0, st,
                     reinterpret_cast<const uint64_t*>(base + L.ckey),
                     reinterpret_cast<const int64_t*>(base + L.cidx), nullptr, h, int64_t{0}, k,
                     out_keys, out_idx, nullptr, SortTail{});
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// Two-level workspace: level 1 selects candidates from n rows (capacity cap),
// level 2 is an exact top-k over the cap canonical candidate keys; then the
// selected positions and the fast level 1's group minima ([2][kMaxGroups]).
struct RerankWs {
  TopkLayout L1, L2;
  size_t l2, pos, gmin, reg, total;
};
constexpr int kMaxSumBlocks = kMaxRegions;  // summary_select_kernel blocks (candidate regions)

static RerankWs rerank_ws(int64_t n, int64_t k, int64_t cap) {
  RerankWs W;
  W.L1 = topk_layout(n, cap);
  W.L2 = topk_layout(cap, k);
  W.l2 = W.L1.total;
  W.pos = W.l2 + W.L2.total;
  W.gmin = W.pos + round_up(k * 8, 256);
  // per-block candidate regions of the fast level 1: keys | indices | scores
  W.reg = W.gmin + round_up(2 * kMaxGroups * 8, 256);
  W.total = W.reg + 3 * round_up(kMaxSumBlocks * cap * 8, 256);
  return W;
}

static size_t rerank_ws_bytes(int64_t n, int64_t k, int64_t cap) { return rerank_ws(n, k, cap).total; }

// Candidate arguments shared by the level-1 checks of the three selections.
static int check_rerank_args(int64_t n, int64_t k, int64_t cap, int passes, void* ws, size_t ws_bytes) {
  if (n < 1 || k < 1 || k > n || cap < k) return DAL_ERR_SHAPE;
  if (passes < 0 || passes >= kPasses || (passes > 0 && cap > DAL_SORT_CAP_PAYLOAD)) return DAL_ERR_ARG;
  if (k > DAL_SORT_CAP) return DAL_ERR_CAPACITY;
  if (ws_bytes < rerank_ws_bytes(n, k, cap) || (reinterpret_cast<uintptr_t>(ws) & 255)) return DAL_ERR_SHAPE;
  return DAL_OK;
}

// The density-weighted fast level 1 writes its candidates into per-block
// regions of the workspace (keys | indices | scores, cap each).
struct DwRegions {
  uint64_t* keys;
  int64_t* idx;
  double* pay;
};

static DwRegions dw_regions(void* ws, const RerankWs& W, int64_t cap) {
  char* r = static_cast<char*>(ws) + W.reg;
  const size_t part = round_up(kMaxSumBlocks * cap * 8, 256);
  return DwRegions{reinterpret_cast<uint64_t*>(r), reinterpret_cast<int64_t*>(r + part),
                   reinterpret_cast<double*>(r + 2 * part)};
}

static void set_regions(SortTail& tail, TopkHdr* h, int64_t cap, int blocks) {
  tail.n_reg = blocks;
  tail.reg_stride = cap;
  tail.sorted_max = kLocalSort;
  tail.reg_count = h->reg_count;
}

// The standalone fast level 1: group minima (one pass over both keys; block 0
// zeroes the level-1 counters) and the summary select.
template <bool DW>
static int launch_fast_level1(const uint64_t* keys_lo, const uint64_t* keys_hi, int64_t n, int64_t k,
                              int64_t idx_base, int64_t cap, void* ws, const AppendRerank& AR, int32_t* status,
                              int64_t* out_idx, double* out_scores, uint64_t* out_keys, hipStream_t st) {
  const RerankWs W = rerank_ws(n, k, cap);
  char* base = static_cast<char*>(ws);
  TopkHdr* h1 = reinterpret_cast<TopkHdr*>(base + W.L1.hdr);
  uint64_t* gmin = reinterpret_cast<uint64_t*>(base + W.gmin);
  const GroupSummary S = launch_group_min(keys_lo, keys_hi, n, gmin, reinterpret_cast<uint32_t*>(h1),
                                         kFastHdrWords, st);
  SortTail tail;
  tail.cap = cap;
  tail.cap_miss = true;
  tail.status = status;
  tail.clear = reinterpret_cast<uint32_t*>(h1);
  tail.clear_words = kFastHdrWords;
  const int G = summary_grid(S.ng);
  if (!summary_shape_ok(S, G, cap)) return DAL_ERR_SHAPE;
  AppendRerank A = AR;
  int64_t* cidx = reinterpret_cast<int64_t*>(base + W.L1.cidx);
  if (DW) {  // candidates in per-block regions, gathered by the last block
    const DwRegions Rg = dw_regions(ws, W, cap);
    A.ckey = Rg.keys;
    A.cpay = Rg.pay;
    cidx = Rg.idx;
    set_regions(tail, h1, cap, G);
  }
  hipLaunchKernelGGL(summary_select_kernel<DW>, dim3(static_cast<unsigned>(G)), dim3(kSumThreads), 0, st, keys_hi, n,
                     k, idx_base, S, h1, cidx, cap, A, 0, out_keys, out_idx, out_scores, tail);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// Exact level 1 (radix select of K + interval compaction) or the fast level 1
// (group minima, indices only), then `rerank` (canonical keys of every slot),
// then the exact top-k of the candidates.
template <class Rerank>
static int select_with_rerank(const uint64_t* keys_lo, const uint64_t* keys_hi, int64_t n, int64_t k,
                              int64_t idx_base, int64_t cap, int passes, void* ws, size_t ws_bytes,
                              Rerank rerank, int64_t* out_idx, double* out_scores, uint64_t* out_keys,
                              int32_t* dev_status, hipStream_t st) {
  int rc = check_rerank_args(n, k, cap, passes, ws, ws_bytes);
  if (rc) return rc;
  const RerankWs W = rerank_ws(n, k, cap);
  char* base = static_cast<char*>(ws);
  char* base2 = base + W.l2;
  int64_t* pos = reinterpret_cast<int64_t*>(base + W.pos);
  TopkHdr* h1 = reinterpret_cast<TopkHdr*>(base + W.L1.hdr);
  TopkHdr* h2 = reinterpret_cast<TopkHdr*>(base2 + W.L2.hdr);
  uint64_t* ckey = reinterpret_cast<uint64_t*>(base + W.L1.ckey);
  int64_t* cidx = reinterpret_cast<int64_t*>(base + W.L1.cidx);
  double* cpay = reinterpret_cast<double*>(base + W.L1.cpay);
  if (passes > 0) {
    rc = launch_fast_level1<false>(keys_lo, keys_hi, n, k, idx_base, cap, ws, AppendRerank{}, dev_status, nullptr,
                                   nullptr, nullptr, st);
    if (rc) return rc;
  } else {
    rc = run_radix(keys_lo, n, k, h1, st);
    if (rc) return rc;
    rc = run_compact<true>(keys_lo, IntervalArgs{keys_hi}, n, idx_base, k, ws, W.L1, dev_status, st);
    if (rc) return rc;
  }
  // canonical keys for every slot (NONE past the count); with the fast level
  // 1 the re-rank also checks the candidate capacity
  rerank(h1, ckey, cidx, cpay, cap, passes > 0);
  if (cap <= DAL_SORT_CAP_PAYLOAD) {
    // level 2 fits one block: sort the cand_count candidates by canonical key
    // (then row) with their scores, take k
    hipLaunchKernelGGL(sort_kernel<true>, dim3(1), dim3(kSortThreads), 0, st, ckey, cidx, cpay, h1, int64_t{0},
                       k, out_keys, out_idx, out_scores, SortTail{});
    DAL_RETURN_IF_LAUNCH_FAILED();
    return DAL_OK;
  }
  rc = run_radix(ckey, cap, k, h2, st);
  if (rc) return rc;
  rc = run_compact<false>(ckey, IntervalArgs{nullptr}, cap, 0, k, base2, W.L2, nullptr, st);
  if (rc) return rc;
  uint64_t* pkeys = reinterpret_cast<uint64_t*>(base2 + W.L2.ckey);
  hipLaunchKernelGGL(sort_kernel<false>, dim3(1), dim3(kSortThreads), 0, st, pkeys,
                     reinterpret_cast<const int64_t*>(base2 + W.L2.cidx), nullptr, h2, int64_t{0}, k, pkeys,
                     pos, nullptr, SortTail{});
  hipLaunchKernelGGL(gather_selected_kernel, dim3(static_cast<unsigned>(ceil_div(k, 256))), dim3(256), 0, st,
                     pos, pkeys, k, cidx, cpay, out_idx, out_scores, out_keys);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" size_t dal_dw_select_workspace_bytes(int64_t n, int64_t k, int64_t cap) {
  return rerank_ws_bytes(n, k, cap);
}

extern "C" int dal_dw_select(const uint64_t* keys_lo, const uint64_t* keys_hi, const int32_t* votes,
                             const uint8_t* row_flags, int64_t n, int64_t k, int64_t idx_base,
                             const double* lut, double beta, const float* x, int64_t d, int64_t ldx,
                             const double* norm64, const double* colsum, int64_t cap, int32_t level1_passes,
                             void* ws, size_t ws_bytes, int64_t* out_idx, double* out_scores,
                             uint64_t* out_keys, int32_t* dev_status, dal_event_t colsum_ready,
                             dal_stream_t stream) {
  if (!keys_lo || !keys_hi || !votes || !lut || !x || !norm64 || !colsum || !ws || !out_idx ||
      !out_scores || !dev_status)
    return DAL_ERR_ARG;
  if (d < 1 || ldx < d) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  const DwRerank R{x, static_cast<int>(d), ldx, norm64, colsum, lut, votes, row_flags, beta};
  if (level1_passes > 0) {
    // fast level 1: group minima + ONE launch (tau, append with the in-place
    // canonical re-rank, last-block sort)
    const int rc = check_rerank_args(n, k, cap, level1_passes, ws, ws_bytes);
    if (rc) return rc;
    if (colsum_ready && hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(colsum_ready), 0) != hipSuccess)
      return DAL_ERR_HIP;
    const RerankWs W = rerank_ws(n, k, cap);
    char* base = static_cast<char*>(ws);
    // (the LUT size is not an argument of dal_dw_select: no lane-held LUT)
    return launch_fast_level1<true>(keys_lo, keys_hi, n, k, idx_base, cap, ws,
                                    AppendRerank{R, reinterpret_cast<uint64_t*>(base + W.L1.ckey),
                                                 reinterpret_cast<double*>(base + W.L1.cpay)},
                                    dev_status, out_idx, out_scores, out_keys, st);
  }
  bool wait_failed = false;
  auto rerank = [&](TopkHdr* h, uint64_t* ckey, int64_t* cidx, double* cpay, int64_t cp, bool cap_miss) {
    // the only consumer of colsum: join its producer stream here, not before the call
    if (colsum_ready && hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(colsum_ready), 0) != hipSuccess)
      wait_failed = true;
    hipLaunchKernelGGL(rerank_kernel, dim3(static_cast<unsigned>(ceil_div(cp, 4))), dim3(256), 0, st, h,
                       idx_base, R, ckey, cidx, cpay, cp, cap_miss, dev_status);
  };
  const int rc = select_with_rerank(keys_lo, keys_hi, n, k, idx_base, cap, 0, ws, ws_bytes, rerank,
                                    out_idx, out_scores, out_keys, dev_status, st);
  return rc ? rc : (wait_failed ? DAL_ERR_HIP : DAL_OK);
}

extern "C" size_t dal_dw_step_workspace_bytes(int64_t n, int64_t k, int64_t cap) {
  return rerank_ws_bytes(n, k, cap);
}

// One density-weighted iteration: dal_forest_score (DAL_DENSITY_FIXED,
// DAL_DESCENDING, interval keys) + dal_dw_select in one call.  With the fast
// level 1 (level1_passes > 0, cap <= DAL_SORT_CAP_PAYLOAD) the score kernel
// also folds each block's minimum keys into the row groups, so the selection
// is ONE more launch (summary_select_kernel: tau, the append with the
// in-place canonical re-rank, the last-block sort with the capacity check and
// the clears) -- no zeroing launch with DAL_STEP_WS_CLEAN, no status memset
// with DAL_STEP_RESET_STATUS.  Same bits as the two calls.
namespace dal {

int dw_step_impl(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                 const int32_t* inner,
                 const uint8_t* leaf,
                 int32_t n_trees, int32_t depth, const double* lut, const int64_t* density_fixed, double density_err,
                 const uint8_t* row_flags, double beta, int64_t idx_base, const double* norm64, const double* colsum,
                 int64_t k, int64_t cap, int32_t level1_passes, uint32_t step_flags, void* ws, size_t ws_bytes,
                 int32_t* votes, double* scores, uint64_t* keys_lo, uint64_t* keys_hi, int64_t* out_idx,
                 double* out_scores, uint64_t* out_keys, int32_t* dev_status, dal_event_t colsum_ready,
                 dal_stream_t stream, int64_t* const* out_slot, int32_t* status_mirror,
                 const ForestStepHooks* plan_hooks) {
  if (!x || !inner || !leaf || !lut || !density_fixed || !norm64 || !colsum || !ws || !votes || !scores ||
      !keys_lo || !keys_hi || !out_idx || !out_scores || !dev_status)
    return DAL_ERR_ARG;
  if (step_flags & ~static_cast<uint32_t>(DAL_STEP_RESET_STATUS | DAL_STEP_WS_CLEAN | DAL_STEP_KEEP_GROUPS |
                                         DAL_STEP_SELECT_ONLY))
    return DAL_ERR_ARG;
  if (d < 1 || ldx < d) return DAL_ERR_SHAPE;
  int rc = check_rerank_args(n, k, cap, level1_passes, ws, ws_bytes);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  const bool clean = step_flags & DAL_STEP_WS_CLEAN;
  const bool keep = step_flags & DAL_STEP_KEEP_GROUPS;
  const bool select_only = step_flags & DAL_STEP_SELECT_ONLY;
  // the selection launch alone re-reads the keys and group minima a previous
  // call left (KEEP_GROUPS): fast level 1, clean header, status owned by the caller
  if (select_only && (level1_passes == 0 || !clean || (step_flags & DAL_STEP_RESET_STATUS))) return DAL_ERR_ARG;
  if (keep && level1_passes == 0) return DAL_ERR_ARG;
  ForestStepHooks hooks;
  if (plan_hooks) hooks = *plan_hooks;
  if (step_flags & DAL_STEP_RESET_STATUS) hooks.status_reset = dev_status;
  const RerankWs W = rerank_ws(n, k, cap);
  char* base = static_cast<char*>(ws);
  TopkHdr* h1 = reinterpret_cast<TopkHdr*>(base + W.L1.hdr);
  if (level1_passes == 0) {  // exact level 1: the two calls as they are
    rc = forest_score_launch(x, xb, fprep, n, d, ldx, inner, leaf, n_trees, depth, lut, density_fixed, DAL_DENSITY_FIXED,
                             density_err, row_flags, beta, DAL_DESCENDING, votes, scores, keys_lo, keys_hi, hooks,
                             st);
    if (rc) return rc;
    rc = dal_dw_select(keys_lo, keys_hi, votes, row_flags, n, k, idx_base, lut, beta, x, d, ldx, norm64, colsum,
                       cap, 0, ws, ws_bytes, out_idx, out_scores, out_keys, dev_status, colsum_ready, stream);
    if (rc) return rc;
    if (clean) zero_header(h1, st);  // keep the contract: the header is left zero
    if (out_slot || status_mirror)
      hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(256), 0, st, out_idx, out_scores, k, out_slot, dev_status,
                         status_mirror);
    DAL_RETURN_IF_LAUNCH_FAILED();
    return DAL_OK;
  }
  // the score kernel's blocks are the row groups when there are >= 2k of them
  // (tau then lies within a few ranks of K); smaller pools take one
  // group_min_kernel pass over finer groups after the score kernel
  uint64_t* gmin = reinterpret_cast<uint64_t*>(base + W.gmin);
  const int rows_per_block = forest_rows_per_block(x, xb, d, ldx, n_trees, depth);
  GroupSummary S = make_groups(gmin, n, rows_per_block);
  const bool in_score = S.ng >= 2 * k;
  if (in_score) {
    hooks.gmin = gmin;
    hooks.group_blocks = static_cast<int>(S.group_rows / rows_per_block);
    hooks.n_groups = S.ng;
  }
  const bool folded = in_score && hooks.group_blocks > 1;  // atomic max: the buffer starts (and is left) zero
  hooks.write_flags = false;  // the re-rank below derives its candidates' flags from the stamps
  if (!clean) {
    zero_words(reinterpret_cast<uint32_t*>(h1), kFastHdrWords, st);
    if (folded) zero_words(reinterpret_cast<uint32_t*>(gmin), 2 * S.ng * 2, st);
  }
  if (!select_only) {
    rc = forest_score_launch(x, xb, fprep, n, d, ldx, inner, leaf, n_trees, depth, lut, density_fixed, DAL_DENSITY_FIXED,
                             density_err, row_flags, beta, DAL_DESCENDING, votes, scores, keys_lo, keys_hi, hooks,
                             st);
    if (rc) return rc;
    if (!in_score) S = launch_group_min(keys_lo, keys_hi, n, gmin, nullptr, 0, st);
  } else if (!in_score) {
    S = group_min_layout(gmin, n);  // the minima the previous call's group_min_kernel wrote
  }
  if (colsum_ready && hipStreamWaitEvent(st, reinterpret_cast<hipEvent_t>(colsum_ready), 0) != hipSuccess)
    return DAL_ERR_HIP;
  const DwRerank R{x, static_cast<int>(d), ldx, norm64, colsum, lut, votes, row_flags, beta,
                   hooks.base_flags, hooks.stamp, hooks.step_id};
  const int n_lut = n_trees < 64 ? n_trees + 1 : 0;  // LUT held in lanes when it fits a wave
  SortTail tail;
  tail.cap = cap;
  tail.cap_miss = true;
  tail.status = dev_status;
  tail.clear = reinterpret_cast<uint32_t*>(h1);
  tail.clear_words = kFastHdrWords;
  if (folded && !keep) {
    tail.clear2 = reinterpret_cast<uint32_t*>(gmin);
    tail.clear2_words = 2 * S.ng * 2;
  }
  tail.out_slot = out_slot;
  tail.status_mirror = status_mirror;
  const int G = summary_grid(S.ng);
  if (!summary_shape_ok(S, G, cap)) return DAL_ERR_SHAPE;
  const DwRegions Rg = dw_regions(ws, W, cap);
  set_regions(tail, h1, cap, G);
  hipLaunchKernelGGL(summary_select_kernel<true>, dim3(static_cast<unsigned>(G)), dim3(kSumThreads), 0, st, keys_hi,
                     n, k, idx_base, S, h1, Rg.idx, cap, AppendRerank{R, Rg.keys, Rg.pay},
                     n_lut, out_keys, out_idx, out_scores, tail);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

}  // namespace dal

extern "C" int dal_dw_step(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                           const int32_t* inner,
                           const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                           const int64_t* density_fixed, double density_err, const uint8_t* row_flags, double beta,
                           int64_t idx_base, const double* norm64, const double* colsum, int64_t k, int64_t cap,
                           int32_t level1_passes, uint32_t step_flags, void* ws, size_t ws_bytes, int32_t* votes,
                           double* scores, uint64_t* keys_lo, uint64_t* keys_hi, int64_t* out_idx,
                           double* out_scores, uint64_t* out_keys, int32_t* dev_status, dal_event_t colsum_ready,
                           dal_stream_t stream) {
  return dw_step_impl(x, xb, fprep, n, d, ldx, inner, leaf, n_trees, depth, lut, density_fixed, density_err, row_flags,
                      beta,
                      idx_base, norm64, colsum, k, cap, level1_passes, step_flags, ws, ws_bytes, votes, scores,
                      keys_lo, keys_hi, out_idx, out_scores, out_keys, dev_status, colsum_ready, stream, nullptr,
                      nullptr, nullptr);
}

extern "C" size_t dal_maxcos_select_workspace_bytes(int64_t n, int64_t k, int64_t cap) {
  return rerank_ws_bytes(n, k, cap);
}

extern "C" int dal_maxcos_select(const uint64_t* keys_lo, const uint64_t* keys_hi, int64_t n, int64_t k,
                                 int64_t idx_base, const uint16_t* pool, int64_t d, int64_t ld,
                                 const double* ulab, int64_t m, int64_t cap, int32_t level1_passes, void* ws,
                                 size_t ws_bytes,
                                 int64_t* out_idx, double* out_scores, uint64_t* out_keys,
                                 int32_t* dev_status, dal_stream_t stream) {
  if (!keys_lo || !keys_hi || !pool || !ulab || !ws || !out_idx || !out_scores || !dev_status)
    return DAL_ERR_ARG;
  if (d < 1 || d > 256 || ld < d || m < 1) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  auto rerank = [&](TopkHdr* h, uint64_t* ckey, int64_t* cidx, double* cpay, int64_t cp, bool cap_miss) {
    hipLaunchKernelGGL(rerank_maxcos_kernel, dim3(static_cast<unsigned>(ceil_div(cp, kRrC))), dim3(256), 0, st,
                       h, idx_base, pool, static_cast<int>(d), ld, ulab, m, ckey, cidx, cpay, cp, cap_miss,
                       dev_status);
  };
  return select_with_rerank(keys_lo, keys_hi, n, k, idx_base, cap, level1_passes, ws, ws_bytes, rerank, out_idx,
                            out_scores, out_keys, dev_status, st);
}

// Interval keys of fp32 values: lo/hi = keys of the pessimistic/optimistic
// ends of [v - err, v + err] for ``order``; DAL_KEY_NONE for non-candidates.
// Four rows per thread: one 16-B value load, one 4-B flag load and 16-B key
// stores (vec4: v, flags, lo and hi 16-B aligned; the last rows one by one).
__device__ __forceinline__ void interval_key_row(float v, bool cand, double err, int order, uint64_t& lo,
                                                 uint64_t& hi) {
  const double s = static_cast<double>(v);
  lo = cand ? score_key(pessimistic(s, err, order), order) : DAL_KEY_NONE;
  hi = cand ? score_key(optimistic(s, err, order), order) : DAL_KEY_NONE;
}
__global__ __launch_bounds__(256) void interval_keys_f32_kernel(const float* __restrict__ v, int64_t n,
                                                                double err, const uint8_t* __restrict__ flags,
                                                                int order, uint64_t* __restrict__ lo,
                                                                uint64_t* __restrict__ hi, bool vec4) {
  const int64_t i0 = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i0 >= n) return;
  if (vec4 && i0 + 4 <= n) {
    const float4 x = *reinterpret_cast<const float4*>(v + i0);
    const unsigned fw = flags ? *reinterpret_cast<const unsigned*>(flags + i0) : ~0u;
    const float xv[4] = {x.x, x.y, x.z, x.w};
    uint64_t l[4], h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) interval_key_row(xv[j], (fw >> (8 * j)) & DAL_ROW_CANDIDATE, err, order, l[j], h[j]);
    reinterpret_cast<ulonglong2*>(lo + i0)[0] = make_ulonglong2(l[0], l[1]);
    reinterpret_cast<ulonglong2*>(lo + i0)[1] = make_ulonglong2(l[2], l[3]);
    reinterpret_cast<ulonglong2*>(hi + i0)[0] = make_ulonglong2(h[0], h[1]);
    reinterpret_cast<ulonglong2*>(hi + i0)[1] = make_ulonglong2(h[2], h[3]);
    return;
  }
  for (int64_t i = i0; i < i0 + 4 && i < n; ++i) {
    const bool cand = flags ? (flags[i] & DAL_ROW_CANDIDATE) : true;
    interval_key_row(v[i], cand, err, order, lo[i], hi[i]);
  }
}

extern "C" int dal_interval_keys_f32(const float* values, int64_t n, double err, const uint8_t* row_flags,
                                     int order, uint64_t* keys_lo, uint64_t* keys_hi, dal_stream_t stream) {
  if (!values || !keys_lo || !keys_hi) return DAL_ERR_ARG;
  if (order != DAL_ASCENDING && order != DAL_DESCENDING) return DAL_ERR_ARG;
  if (n < 1 || !(err > 0.0)) return DAL_ERR_SHAPE;
  const bool vec4 = reinterpret_cast<uintptr_t>(values) % 16 == 0 && reinterpret_cast<uintptr_t>(keys_lo) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(keys_hi) % 16 == 0 &&
                    (!row_flags || reinterpret_cast<uintptr_t>(row_flags) % 4 == 0);
  hipLaunchKernelGGL(interval_keys_f32_kernel, dim3(static_cast<unsigned>(ceil_div(n, 1024))), dim3(256), 0,
                     as_stream(stream), values, n, err, row_flags, order, keys_lo, keys_hi, vec4);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// ---- multi-GPU merge over the packed all-gather --------------------------
// packed [n_ranks][width] int64: keys [k] | global indices [k] | fp64 score
// bits [k] (| status word): one all-gather's output, read in place.
namespace dal {
namespace {
__global__ __launch_bounds__(256) void merge_unpack_kernel(const int64_t* __restrict__ packed, int64_t n_ranks,
                                                           int64_t width, int64_t k, uint64_t* __restrict__ keys,
                                                           int64_t* __restrict__ pos,
                                                           int32_t* __restrict__ status_or) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (status_or && t == 0) {
    int32_t s = 0;
    for (int64_t r = 0; r < n_ranks; ++r) s |= static_cast<int32_t>(packed[r * width + 3 * k]);
    *status_or = s;
  }
  if (t >= n_ranks * k) return;
  const int64_t r = t / k, i = t - r * k;
  keys[t] = static_cast<uint64_t>(packed[r * width + i]);
  pos[t] = t;  // rank-major: lists are sorted per rank and ranks hold ascending rows
}

__global__ __launch_bounds__(256) void merge_gather_kernel(const int64_t* __restrict__ packed, int64_t width,
                                                           int64_t k, const int64_t* __restrict__ best,
                                                           int64_t* __restrict__ out_idx,
                                                           double* __restrict__ out_scores) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (j >= k) return;
  const int64_t p = best[j], r = p / k, i = p - r * k;
  out_idx[j] = packed[r * width + k + i];
  out_scores[j] = __builtin_bit_cast(double, packed[r * width + 2 * k + i]);
}
}  // namespace
}  // namespace dal

namespace dal {
namespace {
// The merge in ONE launch when the P x k candidates fit the payload sort:
// the packed rows are P regions of the sort tail (keys | indices | score
// bits at offsets 0, k, 2k of a row), ordered by (key, global index) --
// the same order as (key, rank-major position): ranks hold ascending row
// ranges and each rank's list is sorted by (key, index); padding keys sort
// last -- and the status words are OR-ed by thread 0.
__global__ __launch_bounds__(kSortThreads) void merge_rows_kernel(const int64_t* __restrict__ packed, int64_t n_ranks,
                                                                  int64_t width, int64_t k,
                                                                  int64_t* __restrict__ out_idx,
                                                                  double* __restrict__ out_scores,
                                                                  uint64_t* __restrict__ out_keys,
                                                                  int32_t* __restrict__ status_or) {
  if (status_or && threadIdx.x == 0) {
    int32_t s = 0;
    for (int64_t r = 0; r < n_ranks; ++r) s |= static_cast<int32_t>(packed[r * width + 3 * k]);
    *status_or = s;
  }
  SortTail tail;
  tail.n_reg = static_cast<int>(n_ranks);
  tail.reg_stride = width;
  tail.reg_uniform = k;
  sort_tail_body<true>(reinterpret_cast<const uint64_t*>(packed), packed + k,
                       reinterpret_cast<const double*>(packed + 2 * k), nullptr, int64_t{0}, k, out_keys, out_idx,
                       out_scores, tail);
}
}  // namespace
}  // namespace dal

extern "C" size_t dal_topk_merge_workspace_bytes(int64_t n_ranks, int64_t k) {
  if (n_ranks < 1 || k < 1) return 0;
  if (n_ranks * k <= DAL_SORT_CAP_PAYLOAD && n_ranks <= 32) return 0;  // the one-launch merge
  return static_cast<size_t>(n_ranks * k) * 16 + static_cast<size_t>(k) * 16;
}

extern "C" int dal_topk_merge(const int64_t* packed, int64_t n_ranks, int64_t width, int64_t k, void* ws,
                              size_t ws_bytes, int64_t* out_idx, double* out_scores, uint64_t* out_keys,
                              int32_t* status_or, dal_stream_t stream) {
  if (!packed || !out_idx || !out_scores) return DAL_ERR_ARG;
  if (n_ranks < 1 || k < 1 || width < 3 * k + (status_or ? 1 : 0)) return DAL_ERR_SHAPE;
  const int64_t n = n_ranks * k;
  if (n > DAL_SORT_CAP) return DAL_ERR_CAPACITY;
  hipStream_t st = as_stream(stream);
  if (n <= DAL_SORT_CAP_PAYLOAD && n_ranks <= 32) {  // one launch, no workspace
    hipLaunchKernelGGL(merge_rows_kernel, dim3(1), dim3(kSortThreads), 0, st, packed, n_ranks, width, k, out_idx,
                       out_scores, out_keys, status_or);
    DAL_RETURN_IF_LAUNCH_FAILED();
    return DAL_OK;
  }
  if (!ws) return DAL_ERR_ARG;
  if (ws_bytes < dal_topk_merge_workspace_bytes(n_ranks, k)) return DAL_ERR_CAPACITY;
  uint64_t* keys = static_cast<uint64_t*>(ws);
  int64_t* pos = reinterpret_cast<int64_t*>(keys + n);
  uint64_t* ws_keys = reinterpret_cast<uint64_t*>(pos + n);
  int64_t* best = reinterpret_cast<int64_t*>(ws_keys + k);
  if (!out_keys) out_keys = ws_keys;
  hipLaunchKernelGGL(merge_unpack_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, st, packed,
                     n_ranks, width, k, keys, pos, status_or);
  hipLaunchKernelGGL(sort_kernel<false>, dim3(1), dim3(kSortThreads), 0, st, keys, pos, nullptr, nullptr, n, k,
                     out_keys, best, nullptr, SortTail{});
  hipLaunchKernelGGL(merge_gather_kernel, dim3(static_cast<unsigned>(ceil_div(k, 256))), dim3(256), 0, st, packed,
                     width, k, best, out_idx, out_scores);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_sort_pairs(const uint64_t* keys, const int64_t* idx, const double* payload, int64_t n,
                              int64_t k, uint64_t* out_keys, int64_t* out_idx, double* out_payload,
                              dal_stream_t stream) {
  if (!keys || !idx || !out_idx) return DAL_ERR_ARG;
  if (n < 1 || k < 1) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  if (payload) {
    if (n > DAL_SORT_CAP_PAYLOAD) return DAL_ERR_CAPACITY;
    hipLaunchKernelGGL(sort_kernel<true>, dim3(1), dim3(kSortThreads), 0, st, keys, idx, payload,
                       nullptr, n, k, out_keys, out_idx, out_payload, SortTail{});
  } else {
    if (n > DAL_SORT_CAP) return DAL_ERR_CAPACITY;
    hipLaunchKernelGGL(sort_kernel<false>, dim3(1), dim3(kSortThreads), 0, st, keys, idx, nullptr,
                       nullptr, n, k, out_keys, out_idx, nullptr, SortTail{});
  }
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
