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

// Features per slice of the split Gram operand (gram_sym.hip): 128 when
// d_pad % 128 == 0, 32 for d_pad == 32, else 64.
int split_ks(int64_t d_pad);

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

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) { return __uint_as_float(static_cast<unsigned>(b) << 16); }

// sum_f x_f^2 of one bf16 row in fp64, sequential in f (the canonical order);
// 16-B aligned rows with d % 8 == 0 are read 64 features at a time (8
// independent loads in flight instead of d dependent-latency scalar loads).
__device__ __forceinline__ double row_sq_norm_bf16(const uint16_t* __restrict__ xr, int d) {
  double s = 0.0;
  if ((reinterpret_cast<uintptr_t>(xr) & 15) == 0 && (d & 7) == 0) {
    for (int f0 = 0; f0 < d; f0 += 64) {
      uint4 q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        q[j] = f0 + 8 * j < d ? *reinterpret_cast<const uint4*>(xr + f0 + 8 * j) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (f0 + 8 * j >= d) break;
        const uint32_t w[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {  // little endian: feature 2e in the low half
          const double lo = bf16_bits_to_f32(static_cast<uint16_t>(w[e] & 0xFFFFu));
          const double hi = bf16_bits_to_f32(static_cast<uint16_t>(w[e] >> 16));
          s = s + lo * lo;
          s = s + hi * hi;
        }
      }
    }
    return s;
  }
  for (int f = 0; f < d; ++f) {
    const double v = bf16_bits_to_f32(xr[f]);
    s = s + v * v;
  }
  return s;
}

// Row-group minima of the optimistic keys carry a row hint in their low
// kHintBits bits: (key & ~kHintMask) | (row offset in the group), so the
// select kernel can prefetch each group's best row before tau is known (its
// canonical re-rank then reads that row from L2).  The selection tests the
// masked key (m & ~kHintMask) <= tau: implied by the exact minimum <= tau, so
// the candidate set stays a superset; the offset is capped below the mask so
// a packed key never reads DAL_KEY_NONE.
constexpr int kHintBits = 24;
constexpr unsigned long long kHintMask = (1ull << kHintBits) - 1ull;
__device__ __forceinline__ unsigned long long pack_hint(unsigned long long key, long long off) {
  if (key == DAL_KEY_NONE) return key;
  const unsigned long long o = off < static_cast<long long>(kHintMask) ? static_cast<unsigned long long>(off)
                                                                        : kHintMask - 1ull;
  return (key & ~kHintMask) | o;
}

// Wave reductions by DPP, the result on every lane: a prefix by row shifts
// (1, 2, 4, 8) and row broadcasts (15, 31) leaves the total in lane 63, read
// back as a scalar.  Sources outside the row (shifts) or rows outside the mask
// (broadcasts) read the identity.  Six dependent VALU steps instead of six
// ds_bpermute exchanges (two per 64-bit value) through the LDS pipe.
template <int CTRL, int ROWS, class Op>
__device__ __forceinline__ unsigned long long dpp_step_u64(unsigned long long v, unsigned long long id, Op op) {
  const int lo = __builtin_amdgcn_update_dpp(static_cast<int>(id), static_cast<int>(v), CTRL, ROWS, 0xf, false);
  const int hi =
      __builtin_amdgcn_update_dpp(static_cast<int>(id >> 32), static_cast<int>(v >> 32), CTRL, ROWS, 0xf, false);
  return op(v, (static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) | static_cast<unsigned>(lo));
}
template <class Op>
__device__ __forceinline__ unsigned long long wave_reduce_u64(unsigned long long v, unsigned long long id, Op op) {
  v = dpp_step_u64<0x111, 0xf>(v, id, op);  // row_shr:1
  v = dpp_step_u64<0x112, 0xf>(v, id, op);  // row_shr:2
  v = dpp_step_u64<0x114, 0xf>(v, id, op);  // row_shr:4
  v = dpp_step_u64<0x118, 0xf>(v, id, op);  // row_shr:8
  v = dpp_step_u64<0x142, 0xa>(v, id, op);  // row_bcast:15
  v = dpp_step_u64<0x143, 0xc>(v, id, op);  // row_bcast:31
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), 63));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}
__device__ __forceinline__ unsigned long long wave_min_u64_dpp(unsigned long long v) {
  return wave_reduce_u64(v, ~0ull, [](unsigned long long a, unsigned long long b) { return b < a ? b : a; });
}
__device__ __forceinline__ unsigned long long wave_max_u64_dpp(unsigned long long v) {
  return wave_reduce_u64(v, 0ull, [](unsigned long long a, unsigned long long b) { return b > a ? b : a; });
}
__device__ __forceinline__ unsigned wave_sum_u32_dpp(unsigned v) {
  return static_cast<unsigned>(
      wave_reduce_u64(v, 0ull, [](unsigned long long a, unsigned long long b) { return a + b; }));
}

// Internal hooks of dal_dw_step into dal_forest_score's kernel (forest.hip):
//   status_reset (nullable) is zeroed by the first thread, before any later
//                kernel of the step can raise a flag (a replayed step starts clean);
//   base_flags   (nullable; the warm-step plan) the row flags are built here:
//                base_flags[r] | (stamp[r] == (uint8_t)*step_id ? DAL_ROW_CANDIDATE : 0)
//                (8-bit stamps: the plan cycles its step ids through 1..255 and
//                clears the stamps when they wrap),
//                written to row_flags for the step's later kernels -- the
//                unlabeled rows were stamped by the plan's mark kernel, so no
//                per-step copy of the base flags;
//   gmin         (nullable; the fast level 1 of the top-k, topk.hip) block b
//                folds the minimum (pessimistic, optimistic) keys of its rows
//                into group g = b / group_blocks: gmin[g] / gmin[n_groups + g]
//                (the optimistic one with its row hint, pack_hint),
//                stored inverted (~key, so a zero word reads DAL_KEY_NONE) --
//                a plain store when group_blocks == 1, else an atomic max on a
//                buffer the top-k leaves zero.
struct ForestStepHooks {
  int32_t* status_reset = nullptr;
  const uint8_t* base_flags = nullptr;
  const uint8_t* stamp = nullptr;
  const uint32_t* step_id = nullptr;
  uint64_t* gmin = nullptr;
  int group_blocks = 1;
  int64_t n_groups = 0;
  // base_flags set: also write the step's flags to row_flags for later
  // kernels (the exact level 1 reads them); the fast level 1's re-rank derives
  // its candidates' flags from the stamps itself (2M byte stores: 20 us)
  bool write_flags = true;
};

// Rows per block of dal_forest_score's kernel for this shape (the row
// groups of ForestStepHooks::gmin are whole blocks).
// xb: the pool's blocked feature-major copy (dal_pool_blocked) or null; the
// blocked path (64-row tiles) runs when the forest is small enough.
int forest_rows_per_block(const float* x, const float* xb, int64_t d, int64_t ldx, int32_t n_trees,
                          int32_t depth);

// fprep: the forest prepared by dal_forest_prepare for this d (nullable; with
// xb only): the blocked kernel's blocks copy it instead of building it.
int forest_score_launch(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                        const int32_t* inner, const uint8_t* leaf, int32_t n_trees, int32_t depth, const double* lut,
                        const void* density, int density_kind, double density_err, const uint8_t* row_flags,
                        double beta, int order, int32_t* votes, double* scores, uint64_t* keys,
                        uint64_t* keys_hi, const ForestStepHooks& hooks, hipStream_t st);

// dal_dw_step with the plan's publishing hooks (topk.hip, SortTail): the
// selection is also written to *out_slot (a host-mapped word holding a device
// address; nullable) and the final status word to *status_mirror (host-mapped).
int dw_step_impl(const float* x, const float* xb, const void* fprep, int64_t n, int64_t d, int64_t ldx,
                 const int32_t* inner,
                 const uint8_t* leaf,
                 int32_t n_trees, int32_t depth, const double* lut, const int64_t* density_fixed, double density_err,
                 const uint8_t* row_flags, double beta, int64_t idx_base, const double* norm64, const double* colsum,
                 int64_t k, int64_t cap, int32_t level1_passes, uint32_t step_flags, void* ws, size_t ws_bytes,
                 int32_t* votes, double* scores, uint64_t* keys_lo, uint64_t* keys_hi, int64_t* out_idx,
                 double* out_scores, uint64_t* out_keys, int32_t* dev_status, dal_event_t colsum_ready,
                 dal_stream_t stream, int64_t* const* out_slot, int32_t* status_mirror,
                 const ForestStepHooks* plan_hooks);

}  // namespace dal
