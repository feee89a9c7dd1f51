// Max-cosine to a labeled set on bf16 MFMA (SURVEY §8(a) a12 at scale).
//
// Reference: final_thesis/similarity.py:26-43 normalises the pool (:28),
// transposes it so points become columns (:34-37) and calls
// RowMatrix.columnSimilarities() (:38), the exact cosine of every pair.  The
// batch-mode diversity restatement of BASELINE config 5 keeps, per pool row,
//   m_i = max_{l in L} cos(x_i, x_l)
// and selects the k rows least similar to the labeled set.
//
// MI355X design: v_mfma_f32_16x16x32_bf16 (fp32 accumulate; bf16 x bf16
// products are exact in fp32).  A block = 4 waves x 64 pool rows held as A
// fragments in VGPRs (loaded once from HBM: the pool is streamed exactly
// once); the labeled rows stream through a 2-stage LDS ring by LDS-DMA
// (source-address XOR swizzle -> conflict-free ds_read_b128).  Each 16x16
// output tile is scaled by 1/||x_l|| (per lane = per column) and max-reduced
// into a running per-lane maximum (one v_max3 per two products); a recursive-
// halving max over the 16 column lanes and the row's 1/||x_i|| (the diagonal
// of the resident fragments' own Gram, four MFMAs per row tile) finish the
// row.  The similarity matrix is never stored.
//
// The kernel is bound by vector ISSUE, not by the matrix pipe: an MFMA holds
// its SIMD's issue for 8 cycles (of 16 for this shape) and each product costs
// 1.5 VALU in the epilogue, so what paid was taking VALU out (fp64 norms ->
// MFMA norms) and putting more waves beside it (three per SIMD: 16 KiB
// stages, 152 VGPRs at d = 128).
// Measured at 8M x 128, m = 1024 (scripts/maxcos_ab.py, same process): the
// previous 32x32x16 kernel (two waves per SIMD, fp64 norms) 1.97 ms; this one
// 1.57 ms (53 % of the dense bf16 peak); with the arg-max 9.30 -> 3.14 ms.
#include <type_traits>

#include "common.hpp"

namespace dal {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define AS3 __attribute__((address_space(3)))

constexpr int kMcRows = 256;     // pool rows per block (64 per wave)
constexpr int kMaxLab = 4096;    // labeled rows whose 1/||x|| fit the LDS table

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<unsigned>(b) << 16);
}

// Lane layout: A/B fragments hold row/column li = lane & 15, k = 8 (lane >> 4)
// .. +7 of a 32-wide k-step; the 16x16 output holds column li, rows
// 4 (lane >> 4) + i.  The running maximum keeps 4 x 4 values per lane.
//
// ARG: also the arg-max (labeled-row position l) of every pool row.  Each lane
// keeps, per accumulator slot, its best value b1 (first l on equal values: l
// grows along a lane's columns and only a strictly larger value replaces b1),
// that value's l, and the runner-up b2; a butterfly over the 16 column lanes
// merges the triples.  When the scaled top two are more than 2 x the error
// bound apart the fp32 arg-max is the canonical one (|m_gpu - m_canon| <= err
// per entry); otherwise the row gets -1 - l and dal_maxcos_argmax_resolve
// recomputes it in canonical fp64.

template <int DK, int STAGE_ = 32768>
struct McCfg {
  static constexpr int STAGE = STAGE_;
  static constexpr int F4 = STAGE / 16;
  static constexpr int ROWB = DK * 2;
  static constexpr int SLOTS = ROWB / 16;
  static constexpr int SR = STAGE / ROWB;   // labeled rows per stage
  static constexpr int NCT = SR / 16;       // 16-column tiles per stage (even)
  static constexpr int NKS = DK / 32;
  static constexpr int RT = 4;              // 16-row tiles per wave
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = STAGE / (4 * 1024);
  static_assert(NCT % 2 == 0, "column tiles go in pairs");
};

// UNIT (dal_max_cosine_unit, no arg-max): the labeled operand is the fp16
// table 2^15 x_l / ||x_l|| (dal_unit_rows_f16) and every pool row is scaled by
// the power of two 2^s that puts its largest |x_if| in [2^15, 2^16) and
// converted to fp16 in registers (exact for the bf16 significand; only
// entries below 2^-29 of the row maximum lose bits).  The per-column scaling
// leaves the epilogue -- one v_max3 per two products -- which is what held
// this kernel's clock down; the operand rounding widens the bound to
// dal_maxcos_unit_error_bound (about 2^-11 on the cosine).
template <bool UNIT>
__device__ __forceinline__ f32x4 mc_mfma(const uint4& a, const uint4& b, const f32x4& c) {
  if constexpr (UNIT)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
}

template <int DK, bool ARG, int OCC, bool UNIT = false>
__global__ __launch_bounds__(256, OCC) void maxcos_kernel(
    const uint16_t* __restrict__ pool, int64_t n, const uint16_t* __restrict__ lab, int64_t m_pad,
    const float* __restrict__ inv_lab, const float* __restrict__ inv_pool, float* __restrict__ out,
    int32_t* __restrict__ out_arg, double gap, int32_t* __restrict__ status) {
  using C = McCfg<DK, OCC == 3 ? 16384 : 32768>;
  extern __shared__ __attribute__((aligned(16))) float4 mc_dyn[];
  float4* lds = mc_dyn;
  float* invl = reinterpret_cast<float*>(mc_dyn + 2 * C::F4);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * 256 + wave * 64;
  const int n_stages = static_cast<int>(m_pad / C::SR);

  if constexpr (!UNIT)
    for (int i = tid; i < m_pad; i += 256) invl[i] = inv_lab[i];

  unsigned voff[C::PIECES];
#pragma unroll
  for (int q = 0; q < C::PIECES; ++q) {
    const int p = (wave * C::PIECES + q) * 64 + lane;
    const int row = p / C::SLOTS;
    const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
    voff[q] = static_cast<unsigned>(row * C::ROWB + slot * 16);
  }
  const unsigned dst0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + wave * C::PIECES * 64))));
  auto issue = [&](int buf, int stage) {
    const char* sbase = reinterpret_cast<const char*>(lab) + static_cast<int64_t>(stage) * C::STAGE;
#pragma unroll
    for (int q = 0; q < C::PIECES; ++q) {
      const unsigned dst = dst0 + static_cast<unsigned>(buf * C::STAGE + q * 1024);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff[q]), "s"(dst), "s"(sbase)
          : "memory");
    }
  };
  issue(0, 0);

  uint4 a[C::RT][C::NKS];
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt) {
    int64_t row = row0 + rt * 16 + li;
    row = row < n ? row : n - 1;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) a[rt][s] = *reinterpret_cast<const uint4*>(pool + row * DK + 32 * s + 8 * lq);
  }
  if constexpr (UNIT) {
    // row r of tile rt lives on lanes li = r of the four lane groups: the
    // largest |bits| of the row (bf16 magnitudes order as their bit patterns)
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
      u16x2 mm = {0, 0};
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const unsigned w[4] = {a[rt][s].x, a[rt][s].y, a[rt][s].z, a[rt][s].w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          mm = __builtin_elementwise_max(mm, __builtin_bit_cast(u16x2, w[e] & 0x7FFF7FFFu));
      }
      unsigned mr = mm.x > mm.y ? mm.x : mm.y;
      mr = max(mr, static_cast<unsigned>(__shfl_xor(static_cast<int>(mr), 16)));
      mr = max(mr, static_cast<unsigned>(__shfl_xor(static_cast<int>(mr), 32)));
      // 2^s puts the row maximum in [2^15, 2^16); exponent-0 rows (zero or
      // bf16-subnormal) stay unscaled and end as zero-norm rows
      const int ex = static_cast<int>(mr >> 7);
      const int sc = ex ? 142 - ex : 0;
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        unsigned w[4] = {a[rt][s].x, a[rt][s].y, a[rt][s].z, a[rt][s].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = __builtin_ldexpf(__uint_as_float(w[e] << 16), sc);
          const float hi = __builtin_ldexpf(__uint_as_float(w[e] & 0xFFFF0000u), sc);
          w[e] = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(lo, hi));
        }
        a[rt][s] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }

  // 1/||x_i|| from the resident fragments: ||x_i||^2 is the diagonal of the
  // tile's own Gram A A^T (an A fragment is also the B fragment of the same
  // rows), NKS MFMAs per row tile instead of d fp64 conversions and FMAs per
  // row -- this kernel is vector-issue-bound, not MFMA-bound.  Exact products,
  // fp32 sums: the norm's error is part of dal_maxcos_error_bound.  Diagonal
  // (r, r) sits on lane r + 16 (r >> 2), element r & 3.
  float inv_row[C::RT];
  {
    const int src = li + 16 * (li >> 2);
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
      f32x4 g = {};
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) g = mc_mfma<UNIT>(a[rt][s], a[rt][s], g);
      const int j = li & 3;
      const float mine = j == 0 ? g[0] : j == 1 ? g[1] : j == 2 ? g[2] : g[3];
      const float n2 = __shfl(mine, src);
      inv_row[rt] = static_cast<float>(1.0 / __builtin_sqrt(static_cast<double>(n2)));
    }
  }

  float mx[C::RT][4];
  float sb[ARG ? C::RT : 1][4];
  int ag[ARG ? C::RT : 1][4];
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) mx[rt][i] = -__builtin_inff();
  if constexpr (ARG) {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sb[rt][i] = -__builtin_inff();
        ag[rt][i] = 0x7FFFFFFF;
      }
  }
  auto upd = [](float& b1, float& b2, int& a, float v, int l) {
    if (v > b1) {
      b2 = b1;
      b1 = v;
      a = l;
    } else {
      b2 = fmaxf(b2, v);
    }
  };
  const f32x4 zero = {};
  int boff[C::NKS];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) boff[s] = li * C::SLOTS + ((4 * s + lq) ^ (li & C::SWZ));

  // column tile ct: its B fragments were read during tile ct - 1's MFMAs
  // (two register sets: the LDS latency never waits in front of a tile);
  // accumulators alternate between (c, e) and the scaled running max takes a
  // pair of tiles at once.  A scheduling fence per tile keeps the compiler
  // from hoisting a whole stage's B reads (registers decide the occupancy).
  f32x4 acc[2][C::RT];
  auto load_b = [&](const float4* B, int ct, uint4 (&bb)[C::NKS]) {
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) bb[s] = __builtin_bit_cast(uint4, B[ct * 16 * C::SLOTS + boff[s]]);
  };
  auto mfma_ct = [&](const uint4 (&bb)[C::NKS], f32x4 (&c)[C::RT]) {
#pragma unroll
    for (int s = 0; s < C::NKS; ++s)
#pragma unroll
      for (int rt = 0; rt < C::RT; ++rt) c[rt] = mc_mfma<UNIT>(a[rt][s], bb[s], s == 0 ? zero : c[rt]);
  };
  // d = 256: two register sets of 8 k-steps' B do not fit beside the A
  // fragments (spills); a pair of tiles reads its B as it goes
  constexpr bool kPrefetch = DK <= 128;
  auto mfma_pair = [&](const float4* B, int ct, f32x4 (&c)[2][C::RT]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const uint4 b = __builtin_bit_cast(uint4, B[(ct + h) * 16 * C::SLOTS + boff[s]]);
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) c[h][rt] = mc_mfma<UNIT>(a[rt][s], b, s == 0 ? zero : c[h][rt]);
      }
    }
  };
  auto epi_pair = [&](int col, const f32x4 (&c)[2][C::RT]) {
    if constexpr (UNIT) {
#pragma unroll
      for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx[rt][i] = fmaxf(fmaxf(mx[rt][i], c[0][rt][i]), c[1][rt][i]);
      return;
    }
    const float ila = invl[col + li], ilb = invl[col + 16 + li];
    if constexpr (ARG) {
#pragma unroll
      for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          upd(mx[rt][i], sb[rt][i], ag[rt][i], c[0][rt][i] * ila, col + li);
          upd(mx[rt][i], sb[rt][i], ag[rt][i], c[1][rt][i] * ilb, col + 16 + li);
        }
    } else {
#pragma unroll
      for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) mx[rt][i] = fmaxf(fmaxf(mx[rt][i], c[0][rt][i] * ila), c[1][rt][i] * ilb);
    }
  };
  // materialise a stage's maxima at its end: otherwise the compiler sinks the
  // epilogue past the next barrier and keeps every accumulator alive (spills)
  auto pin = [&]() {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        asm volatile("" : "+v"(mx[rt][i]));
        if constexpr (ARG) asm volatile("" : "+v"(sb[rt][i]), "+v"(ag[rt][i]));
      }
  };
  auto stage_body = [&](auto bufc, int st) {
    constexpr int buf = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 1 < n_stages) issue(buf ^ 1, st + 1);
    const float4* B = lds + buf * C::F4;
    if constexpr (kPrefetch) {
      uint4 bb[2][C::NKS];
      load_b(B, 0, bb[0]);
#pragma unroll
      for (int ct = 0; ct < C::NCT; ++ct) {
        __builtin_amdgcn_sched_barrier(0);
        if (ct + 1 < C::NCT) load_b(B, ct + 1, bb[(ct + 1) & 1]);
        mfma_ct(bb[ct & 1], acc[ct & 1]);
        if (ct & 1) epi_pair(st * C::SR + (ct - 1) * 16, acc);
      }
    } else {
#pragma unroll
      for (int p = 0; p < C::NCT / 2; ++p) {
        __builtin_amdgcn_sched_barrier(0);
        mfma_pair(B, 2 * p, acc);
        epi_pair(st * C::SR + 2 * p * 16, acc);
      }
    }
    pin();
  };
  // the label granule (65536 / (2d) rows) is two 32 KiB stages: n_stages is even
  for (int st = 0; st < n_stages; st += 2) {
    stage_body(std::integral_constant<int, 0>{}, st);
    stage_body(std::integral_constant<int, 1>{}, st + 1);
  }
  // slot j = 4 rt + i holds row 16 rt + 4 lq + i; lane li finishes slot j = li
  const int rl = 16 * (li >> 2) + 4 * lq + (li & 3);
  const int64_t row = row0 + rl;
  // inv_row[rt] of row 16 rt + r lives on the lanes with li = r
  float iv_reg = 0.0f;
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt) {
    const float t = __shfl(inv_row[rt], rl & 15);
    if ((li >> 2) == rt) iv_reg = t;
  }
  if constexpr (ARG) {
    float b1[16], b2[16];
    int av[16];
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        b1[4 * rt + i] = mx[rt][i];
        b2[4 * rt + i] = sb[rt][i];
        av[4 * rt + i] = ag[rt][i];
      }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float ob1 = __shfl_xor(b1[j], o), ob2 = __shfl_xor(b2[j], o);
        const int oa = __shfl_xor(av[j], o);
        if (ob1 > b1[j] || (ob1 == b1[j] && oa < av[j])) {
          b2[j] = fmaxf(b1[j], ob2);
          b1[j] = ob1;
          av[j] = oa;
        } else {
          b2[j] = fmaxf(b2[j], ob1);
        }
      }
    }
    float v1 = b1[0], v2 = b2[0];
    int va = av[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      if (li == j) {
        v1 = b1[j];
        v2 = b2[j];
        va = av[j];
      }
    }
    if (row < n) {
      const float iv = inv_pool ? inv_pool[row] : iv_reg;
      if (!(iv < __builtin_inff())) atomicOr(status, DAL_FLAG_ZERO_NORM);
      const float m1 = v1 * iv, m2 = v2 * iv;
      out[row] = m1;
      const bool certain = static_cast<double>(m1) - static_cast<double>(m2) > gap;
      out_arg[row] = certain ? va : -1 - va;
    }
    return;
  }
  float v[16];
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) v[4 * rt + i] = mx[rt][i];
#pragma unroll
  for (int step = 0; step < 4; ++step) {
    const int m = 8 >> step;
    const unsigned upm = (li & m) ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < m; ++j) {
      const unsigned lo = __float_as_uint(v[j]), hi = __float_as_uint(v[j + m]);
      const float send = __uint_as_float((lo & upm) | (hi & ~upm));
      const float keep = __uint_as_float((hi & upm) | (lo & ~upm));
      v[j] = fmaxf(keep, __shfl_xor(send, m));
    }
  }
  if (row < n) {
    const float iv = inv_pool ? inv_pool[row] : iv_reg;
    if (!(iv < __builtin_inff())) atomicOr(status, DAL_FLAG_ZERO_NORM);
    // UNIT: the labeled operand carries 2^15 (an exact power-of-two rescale)
    out[row] = UNIT ? (v[0] * iv) * 0x1p-15f : v[0] * iv;
  }
}

// 1/||x|| (fp32) of bf16 rows, ||x||^2 summed in fp64; zero rows flag status.
// Rows in [n, n_pad) get NaN (padding of the labeled table).
__global__ __launch_bounds__(256) void inv_norms_bf16_kernel(const uint16_t* __restrict__ x, int64_t n,
                                                             int64_t n_pad, int d, int64_t ld,
                                                             float* __restrict__ inv,
                                                             int32_t* __restrict__ status) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n_pad) return;
  if (i >= n) {
    inv[i] = __builtin_nanf("");
    return;
  }
  const double s = row_sq_norm_bf16(x + i * ld, d);
  if (!(s > 0.0)) atomicOr(status, DAL_FLAG_ZERO_NORM);
  inv[i] = static_cast<float>(1.0 / __builtin_sqrt(s));
}

// Canonical fp64 unit rows of a bf16 table (sequential norm, then divide),
// stored row-major u[i * d + f] or feature-major u[f * n + i].
__global__ __launch_bounds__(64) void canon_unit_rows_bf16_kernel(const uint16_t* __restrict__ x, int64_t n,
                                                                  int d, int64_t ld, int feature_major,
                                                                  double* __restrict__ u) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const double nr = __builtin_sqrt(row_sq_norm_bf16(x + i * ld, d));
  for (int f = threadIdx.x; f < d; f += 64) {
    const double v = static_cast<double>(bf16_to_f32(x[i * ld + f])) / nr;
    u[feature_major ? f * n + i : i * d + f] = v;
  }
}

// The UNIT kernel's labeled operand: fp16(2^15 x_l / ||x_l||) with the
// canonical fp64 norm (sequential, as the re-rank's), one rounding fp64 ->
// fp16 (round to nearest even); padding rows [m, m_pad) repeat row 0 (a
// duplicate never changes a maximum).  Zero-norm rows flag status.
__global__ __launch_bounds__(64) void unit_rows_f16_kernel(const uint16_t* __restrict__ x, int64_t m, int d,
                                                            int64_t ld, _Float16* __restrict__ out,
                                                            int32_t* __restrict__ status) {
  const int64_t i = blockIdx.x;
  const int64_t src = i < m ? i : 0;
  const double nr = __builtin_sqrt(row_sq_norm_bf16(x + src * ld, d));
  if (i < m && !(nr > 0.0) && threadIdx.x == 0) atomicOr(status, DAL_FLAG_ZERO_NORM);
  for (int f = threadIdx.x; f < d; f += 64)
    out[i * d + f] = static_cast<_Float16>(static_cast<double>(bf16_to_f32(x[src * ld + f])) / nr * 32768.0);
}

// Canonical fp64 arg-max of the rows dal_max_cosine marked ambiguous
// (out_arg < 0): u_i = x_i / sqrt(sum_f x_if^2) (sequential), cos_il =
// sum_f u_if * ulab[f][l] (sequential in f, no FMA), max over l, first l on
// ties (oracle max_cosine_canonical).  One block per 256 rows; a block walks
// its ambiguous rows one at a time with the 256 lanes over labeled rows.
__global__ __launch_bounds__(256) void maxcos_argmax_resolve_kernel(const uint16_t* __restrict__ pool, int64_t n,
                                                                    int d, int64_t ld,
                                                                    const double* __restrict__ ulabT, int64_t m,
                                                                    int32_t* __restrict__ out_arg) {
  __shared__ int list[256];
  __shared__ int count;
  __shared__ double su[256];
  __shared__ double s_nr;
  __shared__ double rb[4];
  __shared__ int ra[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid;
  if (tid == 0) count = 0;
  __syncthreads();
  if (i < n && out_arg[i] < 0) list[atomicAdd(&count, 1)] = tid;
  __syncthreads();
  const int cnt = count;
  for (int q = 0; q < cnt; ++q) {
    const int64_t row = static_cast<int64_t>(blockIdx.x) * 256 + list[q];
    const uint16_t* xr = pool + row * ld;
    if (tid == 0) s_nr = __builtin_sqrt(row_sq_norm_bf16(xr, d));
    __syncthreads();
    if (tid < d) su[tid] = static_cast<double>(bf16_to_f32(xr[tid])) / s_nr;
    __syncthreads();
    double best = -__builtin_inf();
    int arg = 0x7FFFFFFF;
    for (int64_t l = tid; l < m; l += 256) {
      double acc = 0.0;
      for (int f = 0; f < d; ++f) acc = acc + su[f] * ulabT[static_cast<int64_t>(f) * m + l];
      if (acc > best) {  // l grows per lane: strict > keeps the first
        best = acc;
        arg = static_cast<int>(l);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(best, o);
      const int oa = __shfl_xor(arg, o);
      if (ob > best || (ob == best && oa < arg)) {
        best = ob;
        arg = oa;
      }
    }
    if (lane == 0) {
      rb[wave] = best;
      ra[wave] = arg;
    }
    __syncthreads();
    if (tid == 0) {
      double b = rb[0];
      int a = ra[0];
      for (int w = 1; w < 4; ++w) {
        if (rb[w] > b || (rb[w] == b && ra[w] < a)) {
          b = rb[w];
          a = ra[w];
        }
      }
      out_arg[row] = a;
    }
    __syncthreads();
  }
}

template <int DK, bool ARG, int OCC, bool UNIT = false>
int launch_maxcos_t(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, const float* inv_lab,
                      const float* inv_pool, float* out, int32_t* out_arg, double gap, int32_t* status,
                      hipStream_t st) {
  const int64_t blocks = ceil_div(n, kMcRows);
  const size_t shm = 2 * McCfg<DK, OCC == 3 ? 16384 : 32768>::STAGE + (UNIT ? 0 : static_cast<size_t>(m_pad) * 4);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(maxcos_kernel<DK, ARG, OCC, UNIT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)) != hipSuccess)
    return DAL_ERR_HIP;
  hipLaunchKernelGGL((maxcos_kernel<DK, ARG, OCC, UNIT>), dim3(static_cast<unsigned>(blocks)), dim3(256), shm, st, pool, n,
                     lab, m_pad, inv_lab, inv_pool, out, out_arg, gap, status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

template <int DK>
int launch_maxcos_unit(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, float* out,
                       int32_t* status, hipStream_t st) {
  constexpr int OCC = DK <= 128 ? 3 : 2;
  return launch_maxcos_t<DK, false, OCC, true>(pool, n, lab, m_pad, nullptr, nullptr, out, nullptr, 0.0, status, st);
}

template <int DK>
int launch_maxcos(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, const float* inv_lab,
                  const float* inv_pool, float* out, int32_t* out_arg, double gap, int32_t* status, hipStream_t st) {
  // three waves per SIMD where the registers allow it (16 KiB stages so three
  // blocks' rings fit the LDS): d <= 128, or d = 64 with the arg-max state
  constexpr int OCC = DK <= 128 ? 3 : 2, OCC_ARG = DK <= 64 ? 3 : 2;
  if (out_arg)
    return launch_maxcos_t<DK, true, OCC_ARG>(pool, n, lab, m_pad, inv_lab, inv_pool, out, out_arg, gap, status, st);
  return launch_maxcos_t<DK, false, OCC>(pool, n, lab, m_pad, inv_lab, inv_pool, out, nullptr, 0.0, status, st);
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" int64_t dal_maxcos_label_rows_granule(int64_t d) { return 65536 / (2 * d); }

extern "C" int dal_inv_norms_bf16(const uint16_t* x, int64_t n, int64_t n_pad, int64_t d, int64_t ld,
                                  float* inv, int32_t* dev_status, dal_stream_t stream) {
  if (!x || !inv || !dev_status) return DAL_ERR_ARG;
  if (n < 1 || n_pad < n || d < 1 || ld < d) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(inv_norms_bf16_kernel, dim3(static_cast<unsigned>(ceil_div(n_pad, 256))), dim3(256), 0,
                     as_stream(stream), x, n, n_pad, static_cast<int>(d), ld, inv, dev_status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" int dal_canon_unit_rows_bf16(const uint16_t* x, int64_t n, int64_t d, int64_t ld,
                                        int feature_major, double* u, dal_stream_t stream) {
  if (!x || !u) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ld < d) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(canon_unit_rows_bf16_kernel, dim3(static_cast<unsigned>(n)), dim3(64), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ld, feature_major, u);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// Relative to ||x_i|| ||x_l|| (Cauchy-Schwarz; the cosine is <= 1): the
// d-term dot product of exact bf16 products, summed in fp32 in any order with
// up to 2u per add, 2 (d - 1) u; the fp32 scalings by 1/||x_l|| (an fp32
// rounding of the fp64 value) and by 1/||x_i|| with their two products, 4u;
// the in-kernel ||x_i||^2 (the same kind of d-term fp32 sum, 2 (d - 1) u,
// halved by the square root) plus the fp64 -> fp32 rounding of 1/||x_i||,
// (d - 1) u + u.  Total < (3d + 6) u.
extern "C" double dal_maxcos_error_bound(int64_t d) {
  const double u = 1.0 / 16777216.0;
  const double k = 3.0 * static_cast<double>(d) + 6.0;
  return k * u / (1.0 - k * u) * 1.01 + 1e-12;
}

extern "C" int dal_unit_rows_f16(const uint16_t* x, int64_t m, int64_t m_pad, int64_t d, int64_t ld,
                                 uint16_t* out, int32_t* dev_status, dal_stream_t stream) {
  if (!x || !out || !dev_status) return DAL_ERR_ARG;
  if (m < 1 || m_pad < m || d < 1 || ld < d) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(unit_rows_f16_kernel, dim3(static_cast<unsigned>(m_pad)), dim3(64), 0, as_stream(stream), x, m,
                     static_cast<int>(d), ld, reinterpret_cast<_Float16*>(out), dev_status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// dal_max_cosine_unit, relative to the cosine scale (Cauchy-Schwarz on the
// scaled rows x~ = 2^s x, max |x~_f| in [2^15, 2^16), and y' = the fp16 table
// 2^15 y / ||y||):
//  * y' rounding: one fp64 -> fp16 rounding of an fp64 quotient, relative
//    u16 + 2u per entry (u16 = 2^-11), or at most 2^-14 absolute where y'_f is
//    fp16-subnormal or flushed: (u16 + 2u) + 2^-29 sqrt(d);
//  * x~ conversion: exact for entries in the fp16 normal range (a bf16
//    significand fits), at most 2^-14 absolute below it, i.e. 2^-29 of
//    ||x~|| >= 2^15 per entry; moving both the dot and the norm,
//    |cos(a, y) - cos(b, y)| <= 2 ||a - b|| / ||b||: 2^-28 sqrt(d);
//  * fp32 arithmetic of exact fp16 products (the dal_maxcos_error_bound
//    terms: d-term dot, in-kernel norm, two scalings): (3d + 6) u, times
//    ||y'|| / 2^15 <= 1 + 2^-10.
extern "C" double dal_maxcos_unit_error_bound(int64_t d) {
  const double u = 1.0 / 16777216.0, u16 = 1.0 / 2048.0;
  const double rd = __builtin_sqrt(static_cast<double>(d));
  const double b = (u16 + 2.0 * u) + 3.0 * 0x1p-29 * rd + (3.0 * static_cast<double>(d) + 6.0) * u * (1.0 + 0x1p-10);
  return b * 1.01 + 1e-12;
}

extern "C" int dal_max_cosine_unit(const uint16_t* pool, int64_t n, int64_t d, const uint16_t* lab_unit,
                                   int64_t m_pad, float* out_max, int32_t* dev_status, dal_stream_t stream) {
  if (!pool || !lab_unit || !out_max || !dev_status) return DAL_ERR_ARG;
  if (n < 1 || (d != 64 && d != 128 && d != 256)) return DAL_ERR_SHAPE;
  if (m_pad < 1 || m_pad % dal_maxcos_label_rows_granule(d) || m_pad > kMaxLab) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(pool) | reinterpret_cast<uintptr_t>(lab_unit)) & 15) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  if (d == 64) return launch_maxcos_unit<64>(pool, n, lab_unit, m_pad, out_max, dev_status, st);
  if (d == 128) return launch_maxcos_unit<128>(pool, n, lab_unit, m_pad, out_max, dev_status, st);
  return launch_maxcos_unit<256>(pool, n, lab_unit, m_pad, out_max, dev_status, st);
}

extern "C" int dal_max_cosine(const uint16_t* pool, int64_t n, int64_t d, const uint16_t* lab, int64_t m_pad,
                              const float* inv_lab, const float* inv_pool, float* out_max, int32_t* out_arg,
                              int32_t* dev_status, dal_stream_t stream) {
  if (!pool || !lab || !inv_lab || !out_max || !dev_status) return DAL_ERR_ARG;
  if (n < 1 || (d != 64 && d != 128 && d != 256)) return DAL_ERR_SHAPE;
  if (m_pad < 1 || m_pad % dal_maxcos_label_rows_granule(d) || m_pad > kMaxLab) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(pool) | reinterpret_cast<uintptr_t>(lab)) & 15) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  // two entries within err of their canonical values are ordered canonically
  // when their fp32 values differ by more than 2 err (+ slack for the fp32
  // row scaling, which is monotone)
  const double gap = 2.0 * dal_maxcos_error_bound(d) * (1.0 + 1e-6) + 1e-30;
  if (d == 64) return launch_maxcos<64>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, out_arg, gap, dev_status, st);
  if (d == 128)
    return launch_maxcos<128>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, out_arg, gap, dev_status, st);
  return launch_maxcos<256>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, out_arg, gap, dev_status, st);
}

extern "C" int dal_maxcos_argmax_resolve(const uint16_t* pool, int64_t n, int64_t d, int64_t ld, const double* ulab,
                                         int64_t m, int32_t* out_arg, dal_stream_t stream) {
  if (!pool || !ulab || !out_arg) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || d > 256 || ld < d || m < 1 || m > 0x7FFFFFFF) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(maxcos_argmax_resolve_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0,
                     as_stream(stream), pool, n, static_cast<int>(d), ld, ulab, m, out_arg);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
