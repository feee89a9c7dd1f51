// Random-forest hard votes fused with the uncertainty / density-weighted score.
//
// Reference:
//   per-tree predict   final_thesis/uncertainty_sampling.py:88-93,
//                      density_weighting.py:136-141 (T Spark jobs of
//                      DecisionTreeModel(tree).predict; MLlib 2.1 Node.predict:
//                      continuous split x[f] <= threshold -> left)
//   vote sum           uncertainty_sampling.py:96-97 (groupByKey().mapValues(sum))
//   LC score           uncertainty_sampling.py:98   abs(0.5 - (1 - v/T))
//   DW entropy         density_weighting.py:148     -(1-v/T) log2(1-v/T)
//   density product    density_weighting.py:166-167 e * d
// The per-row positional re-key of uncertainty_sampling.py:100-104 is not
// needed: row i's score stays in slot i (the aligned semantics of
// lal_direct_mllib_implementation/classes/active_learner.py:160-183).
//
// MI355X design: HBM-bound streaming kernel.  A block stages R pool rows into
// LDS with coalesced loads (row stride d+1 floats: the per-lane feature
// gathers of the traversal hit distinct banks), the forest (complete-heap SoA,
// 8 B per inner node) is LDS-resident when it fits, and TPR = 256/R threads
// share a row, each walking every TPR-th tree with 4 independent traversals in
// flight (ILP over trees).  Votes are integers; the score comes from an fp64
// look-up table indexed by v, so US scores are exact fp64 and identical to the
// reference's Python float arithmetic.
#include "common.hpp"

namespace dal {
namespace {

#ifndef DAL_FOREST_THREADS
#define DAL_FOREST_THREADS 256
#endif
constexpr int kForestThreads = DAL_FOREST_THREADS;
#ifndef DAL_FOREST_ILP
#define DAL_FOREST_ILP 4
#endif
constexpr int kTreeIlp = DAL_FOREST_ILP;  // independent tree walks in flight per lane
#ifndef DAL_FOREST_BLOCKED_ILP
#define DAL_FOREST_BLOCKED_ILP 4  // ... in the blocked kernel
#endif

struct ForestArgs {
  const float* x;
  int64_t n;
  int d;
  int64_t ldx;
  const int2* inner;
  const uint8_t* leaf;
  int n_trees;
  int depth;
  const double* lut;
  const void* density;
  int dkind;  // 0 none (uncertainty), 1 int64 fixed point (GEMM), 2 exact fp64
  double derr;
  const uint8_t* flags;
  double beta;
  int order;
  int32_t* votes;
  double* scores;
  uint64_t* keys;
  uint64_t* keys_hi;
  ForestStepHooks hooks;  // dal_dw_step only (common.hpp)
};


// beta != 1 calls out of line: inlined, pow's registers counted against every
// score kernel's occupancy although beta == 1 in the common case, where no
// call is made (the blocked kernel 101 -> 74 VGPRs, 4 -> 6 waves per SIMD).
__device__ __attribute__((noinline)) double density_pow_general(double d, double beta) { return pow(d, beta); }
__device__ __forceinline__ double density_pow(double d, double beta) {
  return beta == 1.0 ? d : density_pow_general(d, beta);
}

// |d^beta - d'^beta| bound for |d - d'| <= derr.
__device__ __attribute__((noinline)) double density_pow_err_general(double d, double derr, double beta) {
  const double p = pow(fabs(d), beta);
  const double hi = pow(fabs(d) + derr, beta);
  const double lo = pow(fmax(fabs(d) - derr, 0.0), beta);
  return fmax(fabs(hi - p), fabs(p - lo)) * (1.0 + 1e-12) + fabs(p) * 1e-14;
}
__device__ __forceinline__ double density_pow_err(double d, double derr, double beta) {
  return beta == 1.0 ? derr : density_pow_err_general(d, derr, beta);
}

// A row's flags: row_flags[row], or (warm-step plan) the pool's base flags
// with DAL_ROW_CANDIDATE from this step's mark stamp.
__device__ __forceinline__ uint8_t row_flag(const ForestArgs& A, int64_t row) {
  if (!A.hooks.base_flags) return A.flags[row];
  const bool cand = A.hooks.stamp[row] == static_cast<uint8_t>(*A.hooks.step_id);
  return static_cast<uint8_t>(A.hooks.base_flags[row] | (cand ? DAL_ROW_CANDIDATE : 0));
}

constexpr int kForestWaves = kForestThreads / 64;

// A tile's group fold left for the persistent kernel's thread 0: the tile's
// per-wave minimum keys sit in wmin[slot] (LDS, written by each wave's lane 0
// at the end of its traversal -- no block barrier inside the tile); slot =
// the block's iteration parity, so the next tile's waves write the other one
// while thread 0 reads this one.
struct GroupFold {
  int64_t tile = -1;  // -1: nothing pending
  int slot = 0;       // this block's next free wmin slot / the pending tile's
};

// thread 0, after the next tile's DMA wait: reduce the pending tile's wave
// minima and atomic-max them into its row group (the atomics then complete
// during that tile's traversal: up to 16 blocks hit a group's two words at
// once, and a contended atomic in flight would hold the next DMA wait)
template <int NW = kForestWaves>
__device__ __forceinline__ void issue_fold(const ForestArgs& A, GroupFold& f,
                                           const unsigned long long (*wmin)[2][NW]) {
  if (f.tile < 0) return;
  const unsigned long long(&m)[2][NW] = wmin[f.slot ^ 1];
  unsigned long long lo = m[0][0], hi = m[1][0];
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    lo = m[0][w] < lo ? m[0][w] : lo;
    hi = m[1][w] < hi ? m[1][w] : hi;
  }
  unsigned long long* lo_g = reinterpret_cast<unsigned long long*>(A.hooks.gmin) +
                             static_cast<uint32_t>(f.tile) / static_cast<uint32_t>(A.hooks.group_blocks);
  if (lo != DAL_KEY_NONE) atomicMax(lo_g, ~lo);
  if (hi != DAL_KEY_NONE) atomicMax(lo_g + A.hooks.n_groups, ~hi);
  f.tile = -1;
}

// The minimum of a u64 over the wave, on every lane: a prefix minimum by DPP
// row shifts (1, 2, 4, 8) and row broadcasts (15, 31) -- lane 63 ends with the
// total -- instead of six 64-bit ds_bpermute exchanges (two LDS round trips
// each, on the rows' epilogue wave of every tile).  Out-of-row sources and
// rows outside the mask read the identity (~0).
#ifndef DAL_FOREST_DPP_MIN
#define DAL_FOREST_DPP_MIN 1
#endif
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned long long dpp_min_step(unsigned long long v) {
  const int lo = __builtin_amdgcn_update_dpp(-1, static_cast<int>(v), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(-1, static_cast<int>(v >> 32), CTRL, ROWS, 0xf, false);
  const unsigned long long t =
      (static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) | static_cast<unsigned>(lo);
  return t < v ? t : v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  v = dpp_min_step<0x111, 0xf>(v);  // row_shr:1
  v = dpp_min_step<0x112, 0xf>(v);  // row_shr:2
  v = dpp_min_step<0x114, 0xf>(v);  // row_shr:4
  v = dpp_min_step<0x118, 0xf>(v);  // row_shr:8: lane 15 of each row holds the row's minimum
  v = dpp_min_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v = dpp_min_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3: lane 63 holds the total
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), 63));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

// Votes, score and keys of tile `tile` (R rows from LDS or global memory),
// and the tile's minimum keys folded into its row group (hooks.gmin).  With
// several blocks per group in the persistent kernel (wmin non-null) the
// fold is left pending (GroupFold, issue_fold).
// WROWS (the blocked feature-major path): wave w holds rows (w / tpr) * 64 +
// lane and walks trees w % tpr, + tpr, ...; the waves' partial votes of a row
// are summed through LDS.
// Byte-addressed walks of M trees (t, t + tpr, ...) at once for one row
// (score_tile BYTEA): node h of tree t sits at LDS byte tb + 8 h, so its
// child 2h + 1 (x <= thr) or 2h + 2 sits at 2a + (8 - tb) or 2a + (16 - tb)
// -- a select and a shift-add per level; the leaf byte at (a >> 3) + lbase +
// t * n_leaf - n_inner - tb / 8.  Returns the M trees' summed votes.
struct ByteWalk {
  unsigned fbase, lbase, xb;  // LDS byte addresses: nodes, leaves, this row's x
  int tpr, n_inner, n_leaf, depth;
};
template <int M>
__device__ __forceinline__ int walk_group(const ByteWalk& W, int t) {
  typedef __attribute__((address_space(3))) const float lds_float;
  typedef __attribute__((address_space(3))) const uint8_t lds_u8;
  typedef __attribute__((address_space(3))) const unsigned long long lds_u64;
  unsigned a[M], kl[M], kr[M], lo[M];
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const int tj = t + j * W.tpr;
    const unsigned tb = W.fbase + static_cast<unsigned>(8 * tj * W.n_inner);
    a[j] = tb;
    kl[j] = 8u - tb;
    kr[j] = 16u - tb;
    lo[j] = W.lbase + static_cast<unsigned>(tj * W.n_leaf - W.n_inner) - (tb >> 3);
    // opaque to the optimiser and held in vector registers, so the step stays
    // select + shift-add instead of shift, subtract, select, add
    asm volatile("" : "+v"(kl[j]), "+v"(kr[j]));
  }
  for (int lvl = 0; lvl < W.depth; ++lvl) {
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const unsigned long long nd = *(lds_u64*)static_cast<uintptr_t>(a[j]);  // {feature run offset, thr}
      const float xv = *(lds_float*)static_cast<uintptr_t>(W.xb + static_cast<unsigned>(nd));
      a[j] = 2u * a[j] + (xv <= __uint_as_float(static_cast<unsigned>(nd >> 32)) ? kl[j] : kr[j]);
    }
  }
  int v = 0;
#pragma unroll
  for (int j = 0; j < M; ++j) v += *(lds_u8*)static_cast<uintptr_t>((a[j] >> 3) + lo[j]);
  return v;
}
// the last rem (< ILP) trees of a wave as one group (rem wave-uniform)
template <int M>
__device__ __forceinline__ int walk_tail(const ByteWalk& W, int t, int rem) {
  if constexpr (M == 0) {
    return 0;
  } else {
    return rem == M ? walk_group<M>(W, t) : walk_tail<M - 1>(W, t, rem);
  }
}

// BYTEA (the prepared blocked path: LDS nodes whose feature is the BYTE
// offset slot * 256 of its run): walk_group -- 4 VALU per node visit (x
// address, compare, select, shift-add) against 5, the tree index
// wave-uniform (scalar), and a wave's last trees walked together.
template <bool X_LDS, bool WROWS = false, int NW = kForestWaves, int ILP = kTreeIlp, bool BYTEA = false>
__device__ __forceinline__ void score_tile(const ForestArgs& A, const float* xs, int xstride, int64_t tile, int R,
                                           int tpr, const int2* inner, const uint8_t* leaf, bool pre,
                                           uint8_t fl_pre, long long dens_pre, GroupFold& fold,
                                           unsigned long long (*wmin)[2][NW], const double* lut_s = nullptr) {
  static_assert(!BYTEA || (WROWS && X_LDS), "byte-addressed walks: the blocked kernel's LDS tiles only");
  constexpr int NT = NW * 64;  // threads of the block
  const int n_inner = (1 << A.depth) - 1;
  const int n_leaf = 1 << A.depth;
  const int tid = threadIdx.x;
  const int64_t row0 = tile * R;
  constexpr bool wr = WROWS;  // rows by wave lanes, trees by waves
  const int r = wr ? (tid >> 6) / tpr * 64 + (tid & 63) : tid / tpr;
  const int sub = wr ? (tid >> 6) % tpr : tid - r * tpr;
  const int64_t row = row0 + r;
  const bool live = r < R && row < A.n;

  const float* xrow = X_LDS ? xs + r * xstride : A.x + (live ? row : 0) * A.ldx;

  int v = 0;
  if constexpr (BYTEA) {
    typedef __attribute__((address_space(3))) const int2 lds_int2;
    typedef __attribute__((address_space(3))) const float lds_float;
    typedef __attribute__((address_space(3))) const uint8_t lds_u8;
    const ByteWalk W{static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_int2*)inner)),
                     static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_u8*)leaf)),
                     static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_float*)xrow)), tpr, n_inner, n_leaf,
                     A.depth};
    if (live) {
      // groups of ILP trees, then the wave's last trees as ONE group of their
      // count (T = 10 over 4 waves: 3 or 2 walks in flight, not one at a time)
      for (int t = __builtin_amdgcn_readfirstlane(sub); t < A.n_trees; t += ILP * tpr) {  // (wave-uniform)
        const int rem = (A.n_trees - t + tpr - 1) / tpr;
        v += rem >= ILP ? walk_group<ILP>(W, t) : walk_tail<ILP - 1>(W, t, rem);
      }
    }
  } else if (live) {
    int t = sub;
    for (; t + (ILP - 1) * tpr < A.n_trees; t += ILP * tpr) {
      int h[ILP];
#pragma unroll
      for (int j = 0; j < ILP; ++j) h[j] = 0;
      for (int lvl = 0; lvl < A.depth; ++lvl) {
#pragma unroll
        for (int j = 0; j < ILP; ++j) {
          const int2 nd = inner[(t + j * tpr) * n_inner + h[j]];
          const float xv = xrow[nd.x];
          h[j] = 2 * h[j] + (xv <= __int_as_float(nd.y) ? 1 : 2);
        }
      }
#pragma unroll
      for (int j = 0; j < ILP; ++j) v += leaf[(t + j * tpr) * n_leaf + (h[j] - n_inner)];
    }
    for (; t < A.n_trees; t += tpr) {
      int h = 0;
      for (int lvl = 0; lvl < A.depth; ++lvl) {
        const int2 nd = inner[t * n_inner + h];
        h = 2 * h + (xrow[nd.x] <= __int_as_float(nd.y) ? 1 : 2);
      }
      v += leaf[t * n_leaf + (h - n_inner)];
    }
  }
  if constexpr (wr) {  // a row's tree phases are in different waves (partial votes < 256: T <= 1020 here)
    __shared__ uint8_t s_vote[NT];
    s_vote[sub * R + r] = static_cast<uint8_t>(v);
    __syncthreads();
    if (sub == 0)
      for (int q = 1; q < tpr; ++q) v += s_vote[q * R + r];
  } else {  // a row's TPR threads are consecutive lanes
    for (int o = 1; o < tpr; o <<= 1) v += __shfl_xor(v, o);
  }
  unsigned long long klo = DAL_KEY_NONE, khi = DAL_KEY_NONE;
  if (live && sub == 0) {
    const uint8_t fl = pre ? fl_pre : A.flags ? row_flag(A, row) : DAL_ROW_CANDIDATE;
    if (A.hooks.base_flags && A.hooks.write_flags) const_cast<uint8_t*>(A.flags)[row] = fl;  // for later kernels
    const double e = lut_s ? lut_s[v] : A.lut[v];  // (lut_s: the LUT in LDS, no dependent global load)
    double s, err = 0.0;
    if (A.dkind) {
      const long long draw = pre ? dens_pre : static_cast<const long long*>(A.density)[row];
      double d = A.dkind == 1 ? from_fixed(draw) : __builtin_bit_cast(double, draw);
      if (fl & DAL_ROW_EXCLUDED) d = __builtin_nan("");
      s = e * density_pow(d, A.beta);
      if (A.dkind == 1 && e == e && e != 0.0 && d == d) {
        err = fabs(e) * density_pow_err(d, A.derr, A.beta);
        // keep the interval ends distinct from s after rounding
        err = fmax(err, fabs(s) * 4.5e-16);
      }
    } else {
      s = e;
    }
    A.votes[row] = v;
    A.scores[row] = s;
    if (fl & DAL_ROW_CANDIDATE) {
      klo = score_key(pessimistic(s, err, A.order), A.order);
      khi = score_key(optimistic(s, err, A.order), A.order);
    }
    A.keys[row] = klo;
    if (A.keys_hi) A.keys_hi[row] = khi;
  }
  if (!A.hooks.gmin) return;  // kernel-uniform
  // the optimistic key carries the row's offset in its group (the select's prefetch hint)
  khi = pack_hint(khi, static_cast<long long>(tile % A.hooks.group_blocks) * R + r);
  // the block's minimum keys -> its row group (the top-k's fast level 1);
  // with rows on wave lanes (wr) only the row leaders' wave (sub 0) holds keys
  if (!wr || sub == 0) {  // (wave-uniform)
#if DAL_FOREST_DPP_MIN
    klo = wave_min_u64(klo);
    khi = wave_min_u64(khi);
#else
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long a = __shfl_xor(klo, o), b = __shfl_xor(khi, o);
      klo = a < klo ? a : klo;
      khi = b < khi ? b : khi;
    }
#endif
  }
  if (wmin && A.hooks.group_blocks > 1) {  // kernel-uniform
    if ((tid & 63) == 0) {
      wmin[fold.slot][0][tid >> 6] = klo;
      wmin[fold.slot][1][tid >> 6] = khi;
    }
    fold.tile = tile;
    fold.slot ^= 1;  // issue_fold reads slot ^ 1: this tile's
    return;
  }
  __shared__ unsigned long long s_min[2][NW];
  if ((tid & 63) == 0) {
    s_min[0][tid >> 6] = klo;
    s_min[1][tid >> 6] = khi;
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      klo = s_min[0][w] < klo ? s_min[0][w] : klo;
      khi = s_min[1][w] < khi ? s_min[1][w] : khi;
    }
    const int64_t g = tile / A.hooks.group_blocks;
    unsigned long long* lo_g = reinterpret_cast<unsigned long long*>(A.hooks.gmin) + g;
    unsigned long long* hi_g = lo_g + A.hooks.n_groups;
    if (A.hooks.group_blocks == 1) {
      *lo_g = ~klo;
      *hi_g = ~khi;
    } else {
      if (klo != DAL_KEY_NONE) atomicMax(lo_g, ~klo);
      if (khi != DAL_KEY_NONE) atomicMax(hi_g, ~khi);
    }
  }
}

// One block per tile (grid = tiles), or PERSIST (LDS-DMA staging only; grid
// = the blocks resident at once, walking tiles blockIdx.x, + gridDim.x, ...):
// the forest is copied into LDS once per block instead of once per tile
// (T = 100: 13.6 KB per 32-row tile).  PERSIST is its own instantiation: the
// vec4 staging path's registers would cost it occupancy (147 VGPRs, 3 waves
// per SIMD, against 65 / 7 without the loop).  Each tile: the leaders'
// epilogue inputs and the rows are loaded together, then scored (score_tile).
template <bool X_LDS, bool F_LDS, bool PERSIST>
__global__ __launch_bounds__(kForestThreads) void forest_score_kernel(ForestArgs A, int R, int tpr,
                                                                      int x_floats, bool vec4, bool pad4,
                                                                      bool pre, bool dma, int64_t n_tiles) {
  static_assert(!PERSIST || X_LDS, "the persistent form stages rows by LDS-DMA");
  if (PERSIST) {
    dma = true;
    vec4 = false;
    pad4 = true;
  }
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xs = reinterpret_cast<float*>(smem);
  if (A.hooks.status_reset && blockIdx.x == 0 && threadIdx.x == 0) *A.hooks.status_reset = 0;
  const int n_inner = (1 << A.depth) - 1;
  const int n_leaf = 1 << A.depth;
  const int2* inner = A.inner;
  const uint8_t* leaf = A.leaf;
  const int tid = threadIdx.x;
  if (F_LDS) {
    int2* fs = reinterpret_cast<int2*>(smem + static_cast<size_t>(x_floats) * 4);
    uint8_t* ls = reinterpret_cast<uint8_t*>(fs + A.n_trees * n_inner);
    for (int e = tid; e < A.n_trees * n_inner; e += kForestThreads) fs[e] = A.inner[e];
    for (int e = tid; e < A.n_trees * n_leaf; e += kForestThreads) ls[e] = A.leaf[e];
    inner = fs;
    leaf = ls;
  }
  // row stride in LDS: d + 1 words for scalar staging; with 16-B staging
  // d + 4 (rows stay 16-B aligned, one ds_write_b128 per load, consecutive
  // lanes on consecutive banks; rows of a wave start 4 banks apart)
  const int xstride = A.d + (pad4 ? 4 : 1);
  const int r = tid / tpr;  // (the row / tree-phase mapping of score_tile)
  const int sub = tid - r * tpr;
  GroupFold fold;  // the previous tile's group fold, not yet issued (persistent kernel)
  __shared__ unsigned long long wmin[2][2][kForestWaves];
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {  // block-uniform
    const int64_t row0 = tile * R;
    const int64_t row = row0 + r;
    const bool live = r < R && row < A.n;
    // the row leader's epilogue inputs are loaded with the tile (one HBM
    // latency per tile instead of two)
    uint8_t fl_pre = DAL_ROW_CANDIDATE;
    long long dens_pre = 0;
    if (pre && live && sub == 0) {
      if (A.flags) fl_pre = row_flag(A, row);
      if (A.dkind) dens_pre = static_cast<const long long*>(A.density)[row];
    }
    if (X_LDS) {
      const int rows_here = static_cast<int>(min(static_cast<int64_t>(R), A.n - row0));
      if (dma) {
        // LDS-DMA staging (d % 4 == 0, 16-B-aligned padded rows): one
        // global_load_lds_dwordx4 per 1 KiB of a row (the last piece with only
        // the lanes it needs), lane l's 16 B landing at M0 + 16 l; no VGPRs and
        // no LDS write instructions (2M x 256: 535 -> 433 us)
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        const int row_bytes = A.d * 4;
        for (int rr = wave; rr < rows_here; rr += kForestThreads / 64) {
          const float* src = A.x + (row0 + rr) * A.ldx;
          for (int p = 0; p * 1024 < row_bytes; ++p) {
            typedef __attribute__((address_space(3))) float lds_float;
            const unsigned dst = __builtin_amdgcn_readfirstlane(
                static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_float*)(xs + rr * xstride + p * 256))));
            const unsigned voff = static_cast<unsigned>(p * 1024 + lane * 16);
            if (static_cast<int>(voff) < row_bytes) {
              unsigned keep;
              asm volatile(
                  "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                  "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
                  : "=&s"(keep)
                  : "v"(voff), "s"(dst), "s"(src)
                  : "memory");
            }
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (vec4) {
        // 16-B loads, kStageBatch per thread issued before any LDS write (the
        // block's whole tile in flight: this kernel is an HBM stream)
        constexpr int kStageBatch = 8;
        const int q = A.d >> 2, total = rows_here * q;
        for (int e0 = 0; e0 < total; e0 += kForestThreads * kStageBatch) {
          typedef float v4f __attribute__((ext_vector_type(4)));
          v4f v[kStageBatch];
  #pragma unroll
          for (int j = 0; j < kStageBatch; ++j) {
            const int e = e0 + j * kForestThreads + tid;
            if (e < total) {
              const int r = e / q, c = e - r * q;
              v[j] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(A.x + (row0 + r) * A.ldx) + c);
            }
          }
  #pragma unroll
          for (int j = 0; j < kStageBatch; ++j) {
            const int e = e0 + j * kForestThreads + tid;
            if (e < total) {
              const int r = e / q, c = e - r * q;
              float* dst = xs + r * xstride + 4 * c;
              if (pad4) {
                *reinterpret_cast<v4f*>(dst) = v[j];
              } else {
                dst[0] = v[j].x;
                dst[1] = v[j].y;
                dst[2] = v[j].z;
                dst[3] = v[j].w;
              }
            }
          }
        }
      } else {
        for (int e = tid; e < rows_here * A.d; e += kForestThreads) {
          const int r = e / A.d, c = e - r * A.d;
          xs[r * xstride + c] = A.x[(row0 + r) * A.ldx + c];
        }
      }
    }
    __syncthreads();
    if (PERSIST && tid == 0) issue_fold(A, fold, wmin);  // after this tile's DMA wait
    score_tile<X_LDS>(A, xs, xstride, tile, R, tpr, inner, leaf, pre, fl_pre, dens_pre, fold,
                      PERSIST ? wmin : nullptr);
    if (!PERSIST) break;
    __syncthreads();  // every wave done with the tile before the next one is staged
  }
  if (PERSIST && tid == 0) issue_fold(A, fold, wmin);  // the last tile's (its waves passed the loop barrier)
}

// ---------------------------------------------- blocked feature-major path --
// dal_pool_blocked: the pool as tiles of kBlk rows, feature-major inside a
// tile: xb[(tile * d + f) * kBlk + r] = x[tile * kBlk + r][f] (rows past n are
// zero).  A tile's feature f is one contiguous 256-B run, so a kernel that
// needs only some features of a tile reads only those runs.
constexpr int kBlk = 64;

__global__ __launch_bounds__(256) void pool_blocked_kernel(const float* __restrict__ x, int64_t n, int d,
                                                           int64_t ldx, float* __restrict__ xb) {
  __shared__ float t[kBlk][kBlk + 1];
  const int64_t tile = blockIdx.x;
  const int tid = threadIdx.x;
  for (int f0 = 0; f0 < d; f0 += kBlk) {
    for (int e = tid; e < kBlk * kBlk; e += 256) {  // row-major reads (coalesced along f)
      const int r = e / kBlk, c = e % kBlk;
      const int64_t row = tile * kBlk + r;
      t[r][c] = row < n && f0 + c < d ? x[row * ldx + f0 + c] : 0.0f;
    }
    __syncthreads();
    for (int e = tid; e < kBlk * kBlk; e += 256) {  // feature-major writes (coalesced along r)
      const int c = e / kBlk, r = e % kBlk;
      if (f0 + c < d) xb[(tile * d + f0 + c) * kBlk + r] = t[r][c];
    }
    __syncthreads();
  }
}

// Forest votes + score over the blocked copy, reading only the features the
// forest tests.  Each block (persistent grid) first lists the forest's
// distinct features (a bitmap over d, prefix popcounts) and rewrites every
// LDS node's feature as its slot in that list (times kBlk); a 64-row tile is
// then staged by LDS-DMA as the listed features' 256-B runs only (four runs
// per global_load_lds_dwordx4: lane l loads 16 B of run 4i + l / 16), and
// scored with the rows on the lanes of every wave and the trees dealt over
// the waves (x of row r, slot s at xs[s * kBlk + r]: a wave's 64 lanes read
// 64 consecutive words of a run whatever slot each lane's tree asks for --
// no bank conflicts).  Bytes per row: 4 F_used + the epilogue's, against
// 4 d for the row-major tile (config 4, T = 10: ~113 of 256 features).
// PREP (ABI v10): the forest was prepared once per (forest, d) by
// dal_forest_prepare -- feature list, remapped nodes and leaves in the LDS
// layout below -- and every block copies that blob instead of building it
// (the per-block bitmap, popcounts and remap are gone).

// The prepared forest (dal_forest_prepare): a 16-B header {fu, bad, nn,
// fu_max} then the payload [nodes int2 nn (feature -> byte offset slot * kBlk * 4 of its
// run in the LDS tile) | leaves u8
// round4(T * 2^depth) | feature list u16 round2(fu_max)], zero-padded to 16 B:
// the blocked kernel's LDS layout from its forest region on.
struct BlockedPrepLayout {
  int64_t nodes, leaves, used, payload, total;
};
__host__ __device__ inline BlockedPrepLayout blocked_prep_layout(int64_t n_trees, int32_t depth, int64_t fu_max) {
  BlockedPrepLayout L;
  L.nodes = n_trees * ((int64_t{1} << depth) - 1) * 8;
  L.leaves = round_up(n_trees << depth, 4);
  L.used = round_up(fu_max, 2) * 2;
  L.payload = round_up(L.nodes + L.leaves + L.used, 16);
  L.total = 16 + L.payload;
  return L;
}

// The prepared forest's tree walks by LDS byte address (score_tile BYTEA; 1)
// or by heap index like the unprepared kernel (0).  The prepared node format
// follows: a byte offset of the feature's run, or its float index.
#ifndef DAL_FOREST_BYTEA
#define DAL_FOREST_BYTEA 1
#endif
constexpr bool kByteWalk = DAL_FOREST_BYTEA != 0;

template <int NW, bool PREP>
__global__ __launch_bounds__(NW * 64) void forest_blocked_kernel(ForestArgs A, const float* __restrict__ xb,
                                                                 const unsigned char* __restrict__ prep,
                                                                 int fu_max, int64_t n_tiles) {
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int tpr = NW;  // one tree phase per wave, 64 rows per tile
  const int n_inner = (1 << A.depth) - 1, n_leaf = 1 << A.depth;
  const int nn = A.n_trees * n_inner, nw = (A.d + 31) >> 5;
  float* xs = reinterpret_cast<float*>(smem);
  int2* fs = reinterpret_cast<int2*>(smem + static_cast<size_t>(fu_max) * kBlk * 4);
  uint8_t* ls = reinterpret_cast<uint8_t*>(fs + nn);
  uint16_t* used = reinterpret_cast<uint16_t*>(ls + round_up(static_cast<int64_t>(A.n_trees) * n_leaf, 4));
  unsigned* bits = reinterpret_cast<unsigned*>(used + round_up(fu_max, 2));
  int* pre = reinterpret_cast<int*>(bits + nw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (A.hooks.status_reset && blockIdx.x == 0 && tid == 0) *A.hooks.status_reset = 0;
  // the score LUT (T + 1 doubles) in LDS after the forest region: the rows'
  // epilogue looks the vote up there instead of a dependent global load
  double* lut_s = reinterpret_cast<double*>(
      (reinterpret_cast<uintptr_t>(PREP ? reinterpret_cast<unsigned char*>(fs) +
                                              blocked_prep_layout(A.n_trees, A.depth, fu_max).payload
                                        : reinterpret_cast<unsigned char*>(pre + nw)) +
       7) & ~static_cast<uintptr_t>(7));
  for (int i = tid; i <= A.n_trees; i += NT) lut_s[i] = A.lut[i];  // (read after the setup's barrier)
  int fu;
  if constexpr (PREP) {
    // the prepared payload -> LDS, 16 B per thread, kPrepBatch loads in flight
    constexpr int kPrepBatch = 4;
    const int n16 = static_cast<int>(blocked_prep_layout(A.n_trees, A.depth, fu_max).payload >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(prep + 16);
    uint4* dst = reinterpret_cast<uint4*>(fs);
    for (int e0 = tid; e0 < n16; e0 += kPrepBatch * NT) {
      uint4 q[kPrepBatch];
#pragma unroll
      for (int j = 0; j < kPrepBatch; ++j) q[j] = e0 + j * NT < n16 ? src[e0 + j * NT] : uint4{};
#pragma unroll
      for (int j = 0; j < kPrepBatch; ++j)
        if (e0 + j * NT < n16) dst[e0 + j * NT] = q[j];
    }
    fu = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(prep));
    __syncthreads();
  } else {
  for (int w = tid; w < nw; w += NT) bits[w] = 0u;
  // the forest's leaves and nodes, kSetupBatch loads per thread in flight at
  // once (a load-then-use loop waits one memory latency per element)
  constexpr int kSetupBatch = 8;
  for (int e0 = tid; e0 < A.n_trees * n_leaf; e0 += kSetupBatch * NT) {
    uint8_t b[kSetupBatch];
#pragma unroll
    for (int j = 0; j < kSetupBatch; ++j) b[j] = e0 + j * NT < A.n_trees * n_leaf ? A.leaf[e0 + j * NT] : 0;
#pragma unroll
    for (int j = 0; j < kSetupBatch; ++j)
      if (e0 + j * NT < A.n_trees * n_leaf) ls[e0 + j * NT] = b[j];
  }
  __syncthreads();
  // d <= 64 and many nodes: the bitmap's words OR-reduced per wave, one
  // atomic each (same-word LDS atomics serialise: 1,500 at config 3, 42.5 ->
  // 39.0 us; with 150 nodes (T = 10) the reduction cost more than it saved)
  const bool wave_or = nw <= 2 && nn >= 2 * NT;  // (block-uniform)
  unsigned m0 = 0u, m1 = 0u;
  for (int e0 = tid; e0 < nn; e0 += kSetupBatch * NT) {
    int2 q[kSetupBatch];
#pragma unroll
    for (int j = 0; j < kSetupBatch; ++j) q[j] = e0 + j * NT < nn ? A.inner[e0 + j * NT] : int2{0, 0};
#pragma unroll
    for (int j = 0; j < kSetupBatch; ++j) {
      const int e = e0 + j * NT;
      if (e >= nn) break;
      q[j].x = q[j].x < 0 ? 0 : q[j].x >= A.d ? A.d - 1 : q[j].x;  // (a valid forest tests features < d)
      fs[e] = q[j];
      if (wave_or) {
        m0 |= q[j].x < 32 ? 1u << q[j].x : 0u;
        m1 |= q[j].x >= 32 ? 1u << (q[j].x - 32) : 0u;
      } else {
        atomicOr(&bits[q[j].x >> 5], 1u << (q[j].x & 31));
      }
    }
  }
  if (wave_or) {
    for (int o = 32; o > 0; o >>= 1) {
      m0 |= __shfl_xor(m0, o);
      m1 |= __shfl_xor(m1, o);
    }
    if (lane == 0) {
      if (m0) atomicOr(&bits[0], m0);
      if (m1) atomicOr(&bits[1], m1);
    }
  }
  __syncthreads();
  for (int w = tid; w < nw; w += NT) {
    int c = 0;
    for (int j = 0; j < w; ++j) c += __popc(bits[j]);
    pre[w] = c;
  }
  __syncthreads();
  auto slot = [&](int f) { return pre[f >> 5] + __popc(bits[f >> 5] & ((1u << (f & 31)) - 1u)); };
  for (int f = tid; f < A.d; f += NT)
    if ((bits[f >> 5] >> (f & 31)) & 1u) used[slot(f)] = static_cast<uint16_t>(f);  // d <= 2^16 here
  for (int e = tid; e < nn; e += NT) fs[e].x = slot(fs[e].x) * kBlk;
  fu = pre[nw - 1] + __popc(bits[nw - 1]);  // <= fu_max
  __syncthreads();
  }
  const int n_ins = (fu + 3) >> 2;  // DMA instructions per tile (4 runs each)
  typedef __attribute__((address_space(3))) float lds_float;
  GroupFold fold;
  __shared__ unsigned long long wmin[2][2][NW];
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {  // block-uniform
    const int64_t row = tile * kBlk + lane;
    const bool lead = wave == 0 && row < A.n;  // the rows' epilogue: wave 0
    uint8_t fl_pre = DAL_ROW_CANDIDATE;
    long long dens_pre = 0;
    if (lead) {
      if (A.flags) fl_pre = row_flag(A, row);
      if (A.dkind) dens_pre = static_cast<const long long*>(A.density)[row];
    }
    const char* src = reinterpret_cast<const char*>(xb + tile * A.d * kBlk);
    for (int i = wave; i < n_ins; i += NW) {
      const int sl = 4 * i + (lane >> 4);
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_float*)(xs + 4 * i * kBlk))));
      if (sl < fu) {
        const unsigned voff = static_cast<unsigned>(used[sl]) * (kBlk * 4u) + static_cast<unsigned>(lane & 15) * 16u;
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(dst), "s"(src)
            : "memory");
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) issue_fold<NW>(A, fold, wmin);  // after this tile's DMA wait
    score_tile<true, true, NW, DAL_FOREST_BLOCKED_ILP, PREP && kByteWalk>(A, xs, 1, tile, kBlk, tpr, fs, ls, true,
                                                                          fl_pre, dens_pre, fold, wmin, lut_s);
    __syncthreads();  // every wave done with the tile before the next one is staged
  }
  if (tid == 0) issue_fold<NW>(A, fold, wmin);
}

// dal_forest_prepare: one block builds the prepared forest (the blocked
// kernel's per-block setup, done once): the distinct features (bitmap,
// prefix popcounts), every node's feature as its run's byte offset slot * kBlk * 4,
// the leaves, the
// feature list.  A feature outside [0, d) is clamped as the unprepared kernel
// does and counted in the header's ``bad`` word.
constexpr int kPrepThreads = 1024;
__global__ __launch_bounds__(kPrepThreads) void forest_prepare_kernel(const int2* __restrict__ inner,
                                                                     const uint8_t* __restrict__ leaf, int n_trees,
                                                                     int depth, int d, int fu_max,
                                                                     unsigned char* __restrict__ prep) {
  extern __shared__ unsigned pbits[];  // [nw] bitmap | [nw] prefix counts
  const int n_inner = (1 << depth) - 1, n_leaf = 1 << depth;
  const int nn = n_trees * n_inner, nw = (d + 31) >> 5, tid = threadIdx.x;
  int* ppre = reinterpret_cast<int*>(pbits + nw);
  __shared__ int s_bad;
  if (tid == 0) s_bad = 0;
  for (int w = tid; w < nw; w += kPrepThreads) pbits[w] = 0u;
  __syncthreads();
  int bad = 0;
  for (int e = tid; e < nn; e += kPrepThreads) {
    const int f = inner[e].x;
    bad += f < 0 || f >= d;
    const int fc = f < 0 ? 0 : f >= d ? d - 1 : f;
    atomicOr(&pbits[fc >> 5], 1u << (fc & 31));
  }
  if (bad) atomicAdd(&s_bad, bad);
  __syncthreads();
  for (int w = tid; w < nw; w += kPrepThreads) {
    int c = 0;
    for (int j = 0; j < w; ++j) c += __popc(pbits[j]);
    ppre[w] = c;
  }
  __syncthreads();
  auto slot = [&](int f) { return ppre[f >> 5] + __popc(pbits[f >> 5] & ((1u << (f & 31)) - 1u)); };
  const BlockedPrepLayout L = blocked_prep_layout(n_trees, depth, fu_max);
  unsigned char* pay = prep + 16;
  int2* nodes = reinterpret_cast<int2*>(pay);
  uint8_t* leaves = pay + L.nodes;
  uint16_t* used = reinterpret_cast<uint16_t*>(pay + L.nodes + L.leaves);
  for (int e = tid; e < nn; e += kPrepThreads) {
    int2 q = inner[e];
    q.x = slot(q.x < 0 ? 0 : q.x >= d ? d - 1 : q.x) * kBlk * (kByteWalk ? 4 : 1);  // the run's byte (float) offset
    nodes[e] = q;
  }
  for (int64_t e = tid; e < L.leaves; e += kPrepThreads) leaves[e] = e < int64_t{n_trees} * n_leaf ? leaf[e] : 0;
  const int fu = ppre[nw - 1] + __popc(pbits[nw - 1]);
  for (int sl = tid; sl < static_cast<int>(L.used / 2); sl += kPrepThreads) used[sl] = 0;
  __syncthreads();  // (the padding zeros before the list entries over them)
  for (int f = tid; f < d; f += kPrepThreads)
    if ((pbits[f >> 5] >> (f & 31)) & 1u) used[slot(f)] = static_cast<uint16_t>(f);
  for (int64_t b = L.nodes + L.leaves + L.used + tid; b < L.payload; b += kPrepThreads) pay[b] = 0;
  if (tid == 0) {
    int* hdr = reinterpret_cast<int*>(prep);
    hdr[0] = fu;
    hdr[1] = s_bad;
    hdr[2] = nn;
    hdr[3] = fu_max;
  }
}

}  // namespace
}  // namespace dal

namespace dal {

namespace {
// The blocked path's LDS bound on the forest's distinct features, or 0 when
// the path does not apply.  The node count bounds the distinct features; a
// tile holds that many 256-B runs (<= 256: config 4 at T = 10 stages <= 150,
// four blocks per CU; at T = 100 all 256, two), plus the forest, the feature
// list and the bitmap, within 96 KiB.  The blocked kernel beat the row-major
// one in every shape measured, whole rows included (same process, bits
// identical: 2M x 256 x 100 501 -> 468 us, 1M x 128 x 100 193 -> 155 us,
// 100k x 64 x 10 12.7 -> 9.6 us, config 3 43.4 -> 41.9 us): conflict-free
// gathers, LDS-DMA staging and a persistent grid for every width.
// Waves per block of the blocked kernel (the trees are dealt over them): 4,
// or 8 when a block's LDS lets at most two blocks onto a CU (a 256-run tile
// and a 100-tree forest): 2M x 256 x 100 469.7 -> 437.4 us, while 8 waves
// where four-wave blocks fit three or more per CU were slower (config 4 at
// T = 10 206 -> 234 us, config 3 41.8 -> 45.0 us).
#ifndef DAL_FOREST_BLOCKED_PER_CU
#define DAL_FOREST_BLOCKED_PER_CU 5
#endif
constexpr int kBlockedWaves = 4;
constexpr int kBlockedWavesWide = 8;
#ifndef DAL_FOREST_BLOCKED_MAX_RUNS
#define DAL_FOREST_BLOCKED_MAX_RUNS 256
#endif
// the score LUT after the forest region (8-B aligned: up to 7 bytes of slack)
size_t blocked_lut_bytes(int32_t n_trees) { return static_cast<size_t>(n_trees + 1) * 8 + 8; }
size_t blocked_smem(int fu_max, int64_t d, int32_t n_trees, int32_t depth) {
  const int64_t nn = static_cast<int64_t>(n_trees) * ((int64_t{1} << depth) - 1);
  return static_cast<size_t>(fu_max) * kBlk * 4 + static_cast<size_t>(nn) * 8 +
         static_cast<size_t>(round_up(static_cast<int64_t>(n_trees) << depth, 4)) +
         static_cast<size_t>(round_up(fu_max, 2)) * 2 + static_cast<size_t>((d + 31) / 32) * 8 +
         blocked_lut_bytes(n_trees);
}
int blocked_fu_max(int64_t d, int32_t n_trees, int32_t depth) {
  const int64_t nodes = static_cast<int64_t>(n_trees) * ((int64_t{1} << depth) - 1);
  const int64_t fu = nodes < d ? nodes : d;
  // (16-bit feature list; a wave's partial vote fits the 8-bit LDS slot)
  if (fu > DAL_FOREST_BLOCKED_MAX_RUNS || d > 65536 || n_trees > 255 * kBlockedWaves) return 0;  // (either form)
  return blocked_smem(static_cast<int>(fu), d, n_trees, depth) <= 96 * 1024 ? static_cast<int>(fu) : 0;
}

struct ForestTiling {
  int R;        // rows per block
  bool x_lds;   // pool rows staged in LDS
  bool dma;     // ... by LDS-DMA (wide rows)
};

ForestTiling forest_tiling(const float* x, int64_t d, int64_t ldx, int32_t n_trees) {
  // rows per block: stage up to ~16 KiB of pool rows in LDS.  Small tiles keep
  // more blocks (and their loads) resident per CU: at 2M x 256 a 16 KiB tile
  // runs 0.52 ms vs 0.60 (32 KiB) / 0.85 (96 KiB) / 0.75 (8 KiB); neutral at
  // 100k x 64 and 284,807 x 30
  ForestTiling T{256, true, false};
  // LDS-DMA staging for wide rows (d % 4 == 0, ldx % 4 == 0, 16-B-aligned
  // pool; narrow rows leave most lanes of each DMA instruction idle: 2M x 32 x
  // 100: 264 -> 290 us, 100k x 64: 18.4 -> 19.8) holds no registers: 32 KiB
  // tiles there (2M x 256: 441 -> 411 us; 64 KiB 1248)
  T.dma = d >= 128 && d % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0;
  const int64_t tile_cap = T.dma ? 33280 : 16640 * (kForestThreads / 256);
  while (T.R > 16 && static_cast<int64_t>(T.R) * (d + 1) * 4 > tile_cap) T.R >>= 1;
  // wide rows: 16 rows may exceed the preferred tile; LDS staging up to 64 KiB
  if (static_cast<int64_t>(T.R) * (d + 1) * 4 > 65536) {
    T.x_lds = false;
    T.dma = false;
    T.R = 256;
  }
  // many trees (config 3: T = 100): spread a row's trees over more lanes --
  // the traversal's dependent LDS round trips, not HBM, bound that case
#ifndef DAL_FOREST_TPR
#define DAL_FOREST_TPR 2
#endif
  const int tpr_min = n_trees >= 64 ? DAL_FOREST_TPR : 1;  // config 3: 60.7 -> 51.8 us (4: 53.5, 8: 60.9)
  if (T.x_lds) {
    while (T.R > 1 && kForestThreads / T.R < tpr_min) T.R >>= 1;
  }
  return T;
}
}  // namespace

int forest_rows_per_block(const float* x, const float* xb, int64_t d, int64_t ldx, int32_t n_trees,
                          int32_t depth) {
  if (xb && blocked_fu_max(d, n_trees, depth)) return kBlk;
  return forest_tiling(x, d, ldx, n_trees).R;
}

int forest_score_launch(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                        const int32_t* inner, const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                        const void* density, int density_kind, double density_err, const uint8_t* row_flags,
                        double beta, int order, int32_t* votes, double* scores, uint64_t* keys,
                        uint64_t* keys_hi, const ForestStepHooks& hooks_in, hipStream_t st) {
  if (!x || !inner || !leaf || !lut || !votes || !scores || !keys) return DAL_ERR_ARG;
  if (fprep && reinterpret_cast<uintptr_t>(fprep) % 16 != 0) return DAL_ERR_ARG;
  if (order != DAL_ASCENDING && order != DAL_DESCENDING) return DAL_ERR_ARG;
  if (density_kind < 0 || density_kind > 2 || (density_kind && !density)) return DAL_ERR_ARG;
  if (n < 0 || d < 1 || ldx < d || n_trees < 1) return DAL_ERR_SHAPE;
  if (depth < 1 || depth > DAL_MAX_TREE_DEPTH) return DAL_ERR_UNSUPPORTED;
  if (xb && reinterpret_cast<uintptr_t>(xb) % 16 != 0) return DAL_ERR_ARG;
  if (n == 0) return DAL_OK;
  if (const int fu_max = xb ? blocked_fu_max(d, n_trees, depth) : 0) {
    const int64_t tiles = ceil_div(n, kBlk);
    if (hooks_in.gmin &&
        (hooks_in.group_blocks < 1 || ceil_div(tiles, hooks_in.group_blocks) != hooks_in.n_groups))
      return DAL_ERR_ARG;
    ForestArgs A{x, n, static_cast<int>(d), ldx, reinterpret_cast<const int2*>(inner), leaf, n_trees,
                 depth, lut, density_kind ? density : nullptr, density_kind, density_err, row_flags, beta,
                 order, votes, scores, keys, keys_hi, hooks_in};
    const bool pr = fprep != nullptr;
    // prepared: the forest region holds the payload only (no bitmap / prefix counts)
    const size_t smem = pr ? static_cast<size_t>(fu_max) * kBlk * 4 +
                                 static_cast<size_t>(blocked_prep_layout(n_trees, depth, fu_max).payload) +
                                 blocked_lut_bytes(n_trees)
                           : blocked_smem(fu_max, d, n_trees, depth);
    const bool wide = smem > (160u << 10) / 3;  // at most two blocks per CU by LDS: 8-wave blocks
    const int nw = wide ? kBlockedWavesWide : kBlockedWaves;
    const void* fn = wide ? (pr ? reinterpret_cast<const void*>(forest_blocked_kernel<kBlockedWavesWide, true>)
                                : reinterpret_cast<const void*>(forest_blocked_kernel<kBlockedWavesWide, false>))
                          : (pr ? reinterpret_cast<const void*>(forest_blocked_kernel<kBlockedWaves, true>)
                                : reinterpret_cast<const void*>(forest_blocked_kernel<kBlockedWaves, false>));
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1 ||
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem)) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nw * 64, smem) != hipSuccess)
      return DAL_ERR_HIP;
    // at most DAL_FOREST_BLOCKED_PER_CU blocks per CU: every block stages the
    // forest once, so more, shorter-lived blocks pay that setup more often
    // (config 3 at 6 blocks per CU 37.0 us, at 5 35.5, at 4 -- the VGPR limit
    // before pow went out of line -- 37.8)
    if (per_cu > DAL_FOREST_BLOCKED_PER_CU) per_cu = DAL_FOREST_BLOCKED_PER_CU;
    if (per_cu < 1) per_cu = 1;
    const int64_t grid = tiles < static_cast<int64_t>(cus) * per_cu ? tiles : static_cast<int64_t>(cus) * per_cu;
    const unsigned char* pb = static_cast<const unsigned char*>(fprep);
#define DAL_BLOCKED_LAUNCH(W, P)                                                                          \
  hipLaunchKernelGGL((forest_blocked_kernel<W, P>), dim3(static_cast<unsigned>(grid)), dim3(nw * 64), smem, st, A, \
                     xb, pb, fu_max, tiles)
    if (wide && pr) DAL_BLOCKED_LAUNCH(kBlockedWavesWide, true);
    else if (wide) DAL_BLOCKED_LAUNCH(kBlockedWavesWide, false);
    else if (pr) DAL_BLOCKED_LAUNCH(kBlockedWaves, true);
    else DAL_BLOCKED_LAUNCH(kBlockedWaves, false);
#undef DAL_BLOCKED_LAUNCH
    DAL_RETURN_IF_LAUNCH_FAILED();
    return DAL_OK;
  }
  const ForestTiling T = forest_tiling(x, d, ldx, n_trees);
  const int R = T.R, tpr = kForestThreads / R;
  const int64_t blocks = ceil_div(n, R);
  if (hooks_in.gmin &&
      (hooks_in.group_blocks < 1 || ceil_div(blocks, hooks_in.group_blocks) != hooks_in.n_groups))
    return DAL_ERR_ARG;
  ForestArgs A{x, n, static_cast<int>(d), ldx, reinterpret_cast<const int2*>(inner), leaf, n_trees,
               depth, lut, density_kind ? density : nullptr, density_kind, density_err, row_flags, beta,
               order, votes, scores, keys, keys_hi, hooks_in};
  // 16-B staging writes into rows padded to d + 4 words (conflict-free), and
  // the row leader's flag and density loaded with the tile
  const bool vec4 = (d % 4 == 0) && (ldx % 4 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0);
  const bool pad4 = vec4, pre = true;
  const int x_floats = T.x_lds ? R * static_cast<int>(d + (pad4 ? 4 : 1)) : 0;
  const int64_t n_inner = (int64_t{1} << depth) - 1, n_leaf = int64_t{1} << depth;
  const int64_t f_bytes = n_trees * (n_inner * 8 + n_leaf);
  // forest nodes from LDS whenever they fit (from global memory measured
  // slower at every shape: 2M x 256 521 -> 566 us, config 3 46.6 -> 89.8 us)
  const bool f_lds = f_bytes <= 65536;
  const int xf = static_cast<int>(round_up(x_floats, 4));  // forest region 16-B aligned
  size_t smem = static_cast<size_t>(xf) * 4 + (f_lds ? static_cast<size_t>(f_bytes) : 0);
  if (smem == 0) smem = 16;
  // LDS-DMA tiles: a persistent grid of exactly the blocks resident at once
  // (registers, LDS, waves: the occupancy query -- a grid past it would start
  // its extra blocks only when others END) (2M x 256: 430 -> 404 us at
  // T = 10, 677 -> 486 us at T = 100: the forest is copied once per block,
  // not once per 32-row tile)
  int64_t persist_grid = 0;
  if (T.dma) {
    int dev = 0, cus = 0, per_cu = 0;
    const void* fn = f_lds ? reinterpret_cast<const void*>(forest_score_kernel<true, true, true>)
                           : reinterpret_cast<const void*>(forest_score_kernel<true, false, true>);
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1 ||
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem)) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kForestThreads, smem) != hipSuccess)
      return DAL_ERR_HIP;
    if (per_cu < 1) per_cu = 1;
    persist_grid = blocks < static_cast<int64_t>(cus) * per_cu ? blocks : static_cast<int64_t>(cus) * per_cu;
  }
#define DAL_FOREST_LAUNCH(XL, FL, PS, G)                                                                  \
  do {                                                                                                    \
    if (!(PS) && hipFuncSetAttribute(reinterpret_cast<const void*>(forest_score_kernel<XL, FL, PS>),      \
                                     hipFuncAttributeMaxDynamicSharedMemorySize,                          \
                                     static_cast<int>(smem)) != hipSuccess)                               \
      return DAL_ERR_HIP;                                                                                 \
    hipLaunchKernelGGL((forest_score_kernel<XL, FL, PS>), dim3(static_cast<unsigned>(G)),                 \
                       dim3(kForestThreads), smem, st, A, R, tpr, xf, vec4, pad4, pre, T.dma, blocks);    \
  } while (0)
  if (T.dma && f_lds) DAL_FOREST_LAUNCH(true, true, true, persist_grid);
  else if (T.dma) DAL_FOREST_LAUNCH(true, false, true, persist_grid);
  else if (T.x_lds && f_lds) DAL_FOREST_LAUNCH(true, true, false, blocks);
  else if (T.x_lds) DAL_FOREST_LAUNCH(true, false, false, blocks);
  else if (f_lds) DAL_FOREST_LAUNCH(false, true, false, blocks);
  else DAL_FOREST_LAUNCH(false, false, false, blocks);
#undef DAL_FOREST_LAUNCH
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

}  // namespace dal

using namespace dal;

extern "C" int dal_forest_score(const float* x, int64_t n, int64_t d, int64_t ldx, const int32_t* inner,
                                const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                                const void* density, int density_kind, double density_err,
                                const uint8_t* row_flags,
                                double beta, int order, int32_t* votes, double* scores, uint64_t* keys,
                                uint64_t* keys_hi, dal_stream_t stream) {
  return forest_score_launch(x, nullptr, nullptr, n, d, ldx, inner, leaf, n_trees, depth, lut, density, density_kind,
                             density_err, row_flags, beta, order, votes, scores, keys, keys_hi, ForestStepHooks{},
                             as_stream(stream));
}

extern "C" int dal_forest_blocked_rows(int64_t d, int32_t n_trees, int32_t depth) {
  if (d < 1 || n_trees < 1 || depth < 1 || depth > DAL_MAX_TREE_DEPTH) return 0;
  return blocked_fu_max(d, n_trees, depth) ? kBlk : 0;
}

extern "C" int64_t dal_pool_blocked_floats(int64_t n, int64_t d) {
  return n < 0 || d < 1 ? -1 : ceil_div(n, kBlk) * kBlk * d;
}

extern "C" int dal_pool_blocked(const float* x, int64_t n, int64_t d, int64_t ldx, float* xb, dal_stream_t stream) {
  if (!x || !xb) return DAL_ERR_ARG;
  if (n < 0 || d < 1 || ldx < d || d > (int64_t{1} << 24)) return DAL_ERR_SHAPE;
  if (n == 0) return DAL_OK;
  hipLaunchKernelGGL(pool_blocked_kernel, dim3(static_cast<unsigned>(ceil_div(n, kBlk))), dim3(256), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ldx, xb);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" size_t dal_forest_prep_bytes(int64_t d, int32_t n_trees, int32_t depth) {
  if (d < 1 || n_trees < 1 || depth < 1 || depth > DAL_MAX_TREE_DEPTH) return 0;
  const int fu_max = blocked_fu_max(d, n_trees, depth);
  return fu_max ? static_cast<size_t>(blocked_prep_layout(n_trees, depth, fu_max).total) : 0;
}

extern "C" int dal_forest_prepare(const int32_t* inner, const uint8_t* leaf, int32_t n_trees, int32_t depth,
                                  int64_t d, void* prep, size_t prep_bytes, dal_stream_t stream) {
  if (!inner || !leaf || !prep || reinterpret_cast<uintptr_t>(prep) % 16 != 0) return DAL_ERR_ARG;
  if (d < 1 || n_trees < 1) return DAL_ERR_SHAPE;
  if (depth < 1 || depth > DAL_MAX_TREE_DEPTH) return DAL_ERR_UNSUPPORTED;
  const int fu_max = blocked_fu_max(d, n_trees, depth);
  if (!fu_max) return DAL_ERR_UNSUPPORTED;  // the blocked path does not apply (dal_forest_blocked_rows == 0)
  if (prep_bytes < static_cast<size_t>(blocked_prep_layout(n_trees, depth, fu_max).total)) return DAL_ERR_SHAPE;
  const size_t smem = static_cast<size_t>((d + 31) / 32) * 8;
  hipLaunchKernelGGL(forest_prepare_kernel, dim3(1), dim3(kPrepThreads), smem, as_stream(stream),
                     reinterpret_cast<const int2*>(inner), leaf, n_trees, depth, static_cast<int>(d), fu_max,
                     static_cast<unsigned char*>(prep));
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_forest_score_blocked(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d,
                                        int64_t ldx, const int32_t* inner, const uint8_t* leaf, int32_t n_trees,
                                        int32_t depth, const double* lut, const void* density, int density_kind,
                                        double density_err, const uint8_t* row_flags, double beta, int order,
                                        int32_t* votes, double* scores, uint64_t* keys, uint64_t* keys_hi,
                                        dal_stream_t stream) {
  return forest_score_launch(x, xb, fprep, n, d, ldx, inner, leaf, n_trees, depth, lut, density, density_kind,
                             density_err, row_flags, beta, order, votes, scores, keys, keys_hi, ForestStepHooks{},
                             as_stream(stream));
}
