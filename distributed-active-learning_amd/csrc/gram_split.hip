// Fused cosine Gram row-sum on fp16 MFMA with a two-term split of every
// fp32 unit row (three products per feature pair): the fp32-accurate density
// at the fp16 matrix-core rate.
//
// Reference: final_thesis/density_weighting.py:67-75 (U.multiply(UT) through
// IndexedRowMatrix/BlockMatrix), :95-100 (drop i,j in L0) and :157-161
// (groupByKey + sum per row); cosine_similarity.py:29-45 is the same product.
//
// Split.  Every normalised fp32 component u (|u| <= 1) is scaled by 2^12
// (exact) and written as two fp16 terms at that same scale:
//   H = fp16_rn(2^12 u),   L = fp16_rn(2^12 u - H)   (the difference is exact in fp32)
// so 2^12 u = H + L + e with |e| <= 2^-22 |2^12 u| (+2^-25 absolute when L is
// subnormal).  Then
//   2^24 u_i.u_j = H_i.H_j + H_i.L_j + L_i.H_j + O(3 * 2^-22 |2^12 u_i||2^12 u_j|)
// with every fp16 x fp16 product exact in fp32 and all three products in the
// SAME units (2^-24), so they can share one fp32 accumulator.  Three
// v_mfma_f32_16x16x32_f16 per 32 features replace sixteen
// v_mfma_f32_16x16x4_f32: 48 vs 512 SIMD cycles, ~10x the fp32-MFMA rate at
// equal accuracy class.  This kernel keeps two accumulators per row tile: M
// (H.H, the large term) and X (the cross terms, ~2^-11 of M).
//
// Exactness of the row sums is kept from gram.hip: per 256-column fold group
// each lane's partial v = M + X (units 2^-24) is rounded to a multiple of 2^-32
// and added into an fp64 register (integer arithmetic below 2^53); units end
// in int64 atomics.  Fold groups sit at fixed column positions (multiples of
// 256), so the density is bit-identical for any grid, unit split, column
// split or GPU count (shards are multiples of 512 rows).
//
// MI355X design
//  * 4 waves x 64 rows per block, A fragments (h and l) register-resident for
//    a 64- (or 32-) feature K-slice; two blocks per CU (two waves per SIMD,
//    256 VGPRs each): one wave's fold / DMA issue runs under the partner's
//    MFMAs.  B (column) stages of 32 KiB in a 2-deep LDS ring per block,
//    filled by global_load_lds_dwordx4 (1-KiB pieces, source-side XOR
//    swizzle -> conflict-free ds_read_b128 of the hi and lo fragments).
//  * Stages go in pairs (buffer 0 then 1) so the fold-group position of a
//    stage is a compile-time constant: no runtime accumulator selects.
//  * Persistent grid of 2 blocks per CU over (row block, column chunk) units
//    in equal contiguous ranges.

#include <stdlib.h>

#include <type_traits>
#include <utility>
#include <vector>

#include "common.hpp"

namespace dal {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define AS3 __attribute__((address_space(3)))

constexpr int kSpThreads = 256;    // 4 waves
constexpr int kSpRows = 256;       // rows per block (64 per wave = 2 MFMA row tiles)
constexpr int kSpStage = 32768;    // bytes per LDS stage
constexpr int kSpFoldCols = 256;   // columns per exact fold group

template <int KS, int MT>
struct SpCfg {
  static constexpr int ROWB = KS * 4;                   // bytes per column row: KS hi + KS lo halves
  static constexpr int SLOTS = ROWB / 16;               // 16-B slots per column row
  static constexpr int HI = KS / 8;                     // slots of the hi part
  static constexpr int SC = kSpStage / ROWB;            // columns per stage
  static constexpr int FS = kSpFoldCols / SC;           // stages per fold group (1 or 2)
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = kSpStage / (4 * 1024);  // 1-KiB DMA pieces per wave per stage
  static constexpr int F4 = kSpStage / 16;
  // MFMA geometry: MT x MT output tiles (32: v_mfma_f32_32x32x16_f16,
  // 16: v_mfma_f32_16x16x32_f16)
  static constexpr int RT = 64 / MT;                    // row tiles per wave
  static constexpr int LG = 64 / MT;                    // lane groups (K sub-blocks of 8)
  static constexpr int KSTEP = 8 * LG;                  // features per MFMA
  static constexpr int NKS = KS / KSTEP;                // k-steps per slice
  static constexpr int NCT = SC / MT;                   // column tiles per stage
  static constexpr int NV = MT * MT / 64;               // accumulator values per lane
  static_assert(FS == 1 || FS == 2, "a stage pair must hold whole fold groups");
  static_assert(NKS >= 1, "slice narrower than one k-step");
};

template <int MT>
struct SpAcc;
template <>
struct SpAcc<32> {
  typedef float type __attribute__((ext_vector_type(16)));
  static __device__ __forceinline__ type mfma(f16x8 a, f16x8 b, type c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  // row (within the tile) of accumulator value r of lane group q
  static __device__ __forceinline__ int row(int r, int q) { return (r & 3) + 8 * (r >> 2) + 4 * q; }
};
template <>
struct SpAcc<16> {
  typedef float type __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ type mfma(f16x8 a, f16x8 b, type c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int r, int q) { return 4 * q + r; }
};

// a partial in units of 2^-24 -> exact fp64 integer in units of 2^-32
__device__ __forceinline__ double fold_fixed24(float v) {
  return static_cast<double>(__builtin_rintf(v * 256.0f));
}

template <int KS, int MT>
__global__ __launch_bounds__(kSpThreads, 2) void gram_split_kernel(
    const uint16_t* __restrict__ urows, const uint16_t* __restrict__ ucols, int64_t ldh,
    int slice_off, int64_t n_pairs, int chunk_pairs, int64_t n_chunks, int64_t n_row_blocks,
    int sync_sweep, unsigned long long* __restrict__ acc_out) {
  using C = SpCfg<KS, MT>;
  using A = SpAcc<MT>;
  using acc_t = typename A::type;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * C::F4];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane % MT, lq = lane / MT;

  // Work units = (row block, column chunk).  sync_sweep: units in chunk-major
  // order dealt round-robin (block g takes g, g+G, ...), so at any moment every
  // block of every XCD reads the same one or two column chunks in lockstep and
  // each B stage is fetched into an XCD's L2 about once; the A fragments are
  // reloaded per unit.  Otherwise: equal contiguous ranges of row-major units
  // (A reloaded only when a range crosses into the next row block).
  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t n_units = n_row_blocks * n_chunks;
  const int64_t u_begin = sync_sweep ? g : (g * n_units) / G;
  const int64_t u_end = sync_sweep ? n_units : ((g + 1) * n_units) / G;
  const int64_t u_step = sync_sweep ? G : 1;
  if (u_begin >= u_end) return;
  auto unit_rb = [&](int64_t u) { return sync_sweep ? u % n_row_blocks : u / n_chunks; };
  auto unit_pair0 = [&](int64_t u) { return (sync_sweep ? u / n_row_blocks : u % n_chunks) * chunk_pairs; };

  // per-piece source offsets (stage-relative, swizzled) and the wave's LDS base
  unsigned voff[C::PIECES];
#pragma unroll
  for (int q = 0; q < C::PIECES; ++q) {
    const int p = (wave * C::PIECES + q) * 64 + lane;
    const int row = p / C::SLOTS;
    const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
    voff[q] = static_cast<unsigned>(row * ldh * 2 + slot * 16);
  }
  const unsigned dst0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + wave * C::PIECES * 64))));
  // Inline asm so the compiler does not track the DMA on vmcnt (we wait for
  // it ourselves before the barrier that publishes the stage).
  auto issue = [&](int buf, int64_t stage) {
    const uint16_t* sbase = ucols + stage * C::SC * ldh + slice_off;
#pragma unroll
    for (int q = 0; q < C::PIECES; ++q) {
      const unsigned dst = dst0 + static_cast<unsigned>(buf * kSpStage + q * 1024);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff[q]), "s"(dst), "s"(sbase)
          : "memory");
    }
  };

  int64_t unit = u_begin;
  int64_t rb = unit_rb(unit);
  int64_t pr = unit_pair0(unit);
  int64_t pr_end = pr + chunk_pairs < n_pairs ? pr + chunk_pairs : n_pairs;

  // resident A fragments: rows rb*256 + wave*64 + rt*MT + li, features of
  // k-step c and lane group lq = slot c*LG + lq of the hi / lo halves
  f16x8 ah[C::RT][C::NKS], al[C::RT][C::NKS];
  auto load_a = [&](int64_t rbk) {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
      const int64_t row = rbk * kSpRows + wave * 64 + rt * MT + li;
      const uint16_t* src = urows + row * ldh + slice_off;
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        ah[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + (c * C::LG + lq) * 8));
        al[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + KS + (c * C::LG + lq) * 8));
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): A (and any in-flight DMA) landed
  };

  // B-fragment LDS offsets (float4 units) per k-step; column tiles add ct*MT*SLOTS
  int boh[C::NKS], bol[C::NKS];
#pragma unroll
  for (int c = 0; c < C::NKS; ++c) {
    boh[c] = li * C::SLOTS + ((c * C::LG + lq) ^ (li & C::SWZ));
    bol[c] = li * C::SLOTS + ((C::HI + c * C::LG + lq) ^ (li & C::SWZ));
  }

  acc_t m[C::RT], x[C::RT];
  double facc[C::RT][C::NV];
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
    for (int r = 0; r < C::NV; ++r) facc[rt][r] = 0.0;
  const acc_t zero = {};

  auto compute = [&](auto firstc, const float4* B) {
    constexpr bool FIRST = decltype(firstc)::value;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        const f16x8 bh = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + boh[c]]);
        const f16x8 bl = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + bol[c]]);
        const bool z = FIRST && ct == 0 && c == 0;
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) m[rt] = A::mfma(ah[rt][c], bh, z ? zero : m[rt]);
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) x[rt] = A::mfma(ah[rt][c], bl, z ? zero : x[rt]);
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) x[rt] = A::mfma(al[rt][c], bh, x[rt]);
      }
    }
  };
  auto fold = [&]() {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int r = 0; r < C::NV; ++r) facc[rt][r] += fold_fixed24(m[rt][r] + x[rt][r]);
  };

  auto finish_unit = [&]() {
    // exact (integer-valued) fp64 butterfly over the MT column lanes of each group
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
      for (int r = 0; r < C::NV; ++r) {
        double v = facc[rt][r];
#pragma unroll
        for (int sh = 1; sh < MT; sh <<= 1) v += __shfl_xor(v, sh);
        facc[rt][r] = v;
      }
    }
    // lane (li, lq) publishes value li = (rt, r): the wave's 64 rows, one atomic
    double mine = 0.0;
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
      for (int r = 0; r < C::NV; ++r) {
        if (rt * C::NV + r == li) mine = facc[rt][r];
        facc[rt][r] = 0.0;
      }
    }
    const int rt = li / C::NV, r = li % C::NV;
    const int64_t row = rb * kSpRows + wave * 64 + rt * MT + A::row(r, lq);
    atomicAdd(acc_out + row, static_cast<unsigned long long>(static_cast<long long>(mine)));
  };

  issue(0, 2 * pr);
  load_a(rb);
  const float4* B0 = lds;
  const float4* B1 = lds + C::F4;

  while (true) {
    const bool last_of_unit = (pr + 1 == pr_end);
    int64_t n_unit = unit, n_pr = pr + 1;
    if (last_of_unit) {
      n_unit = unit + u_step;
      n_pr = unit_pair0(n_unit);
    }
    const bool has_next = n_unit < u_end;

    // stage 2*pr on buffer 0 (its DMA was issued one stage ago)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    issue(1, 2 * pr + 1);
    compute(std::integral_constant<bool, true>{}, B0);
    if constexpr (C::FS == 1) fold();

    // stage 2*pr+1 on buffer 1
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (has_next) issue(0, 2 * n_pr);
    compute(std::integral_constant<bool, C::FS == 1>{}, B1);
    fold();
    if (last_of_unit) finish_unit();

    if (!has_next) break;
    if (last_of_unit) {
      unit = n_unit;
      const int64_t nrb = unit_rb(unit);
      if (nrb != rb) {
        rb = nrb;
        load_a(rb);
      }
      pr_end = n_pr + chunk_pairs < n_pairs ? n_pr + chunk_pairs : n_pairs;
    }
    pr = n_pr;
  }
}

// ---------------------------------------------------------------------------
// Symmetric (SYRK-style) variant on 256-row blocks (DAL_GRAM_SYM=1; the
// default is the 512-row gram_sym2_kernel below): S = U U^T is symmetric, so
// each unordered pair of 256-row blocks {I, J} is multiplied ONCE and yields
// both the row sums of S_IJ (-> rows of I) and its column sums (-> rows of J):
// half the MFMAs.  Orientation rule, a function of the global block indices
// only (so the bits do not depend on the GPU count): row block I takes column
// block J when J == I (diagonal: row sums only), J > I and I+J even, J < I and
// I+J odd.  Every row block then takes ~nb/2 column blocks, so work is
// balanced across row blocks, units and row-sharded GPUs.  Column block = fold
// group = one pair of 128-column stages.  Epilogue SG 2 (default): the row
// sums ride in two MFMA accumulator chains (even / odd column tiles) and a
// tile's column sums are the growth of its chain's lane total; SG 1: per-tile
// fresh accumulators, row sums added on the VALU.  Column partials are rounded
// to multiples of 2^-32 and added into an LDS fp64 column accumulator (exact,
// order-free); after the pair the 256 column sums go to global int64 atomics.
// The LDS column accumulator is double-buffered so its flush (at the next
// pair's first barrier) never races the next pair's adds.
template <int KS, int MT>
struct SymCfg {
  static constexpr int ROWB = KS * 4;
  static constexpr int SLOTS = ROWB / 16;
  static constexpr int HI = KS / 8;
  static constexpr int SC = 128;                        // columns per stage (two per column block)
  static constexpr int STAGE = SC * ROWB;               // 32 KiB (KS 64) or 16 KiB (KS 32)
  static constexpr int F4 = STAGE / 16;
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = STAGE / (4 * 1024);
  static constexpr int RT = 64 / MT;
  static constexpr int LG = 64 / MT;
  static constexpr int KSTEP = 8 * LG;
  static constexpr int NKS = KS / KSTEP;
  static constexpr int NCT = SC / MT;
  static constexpr int NV = MT * MT / 64;
  static_assert(NKS >= 1 && PIECES >= 1, "bad slice");
};

template <int KS, int MT, int SG>
__global__ __launch_bounds__(kSpThreads, 2) void gram_sym_kernel(
    const uint16_t* __restrict__ urows, int row_block0, int n_rb,
    const uint16_t* __restrict__ ucols, int col_block0, int j_lo, int j_hi,
    int nb_active, int64_t ldh, int slice_off, int chunk_blocks, int n_chunks,
    unsigned long long* __restrict__ acc_out) {
  using C = SymCfg<KS, MT>;
  using A = SpAcc<MT>;
  using acc_t = typename A::type;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * C::F4];
  __shared__ double colacc[2][256];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane % MT, lq = lane / MT;
  const int G = gridDim.x, g = blockIdx.x;
  const int n_units = n_rb * n_chunks;

  colacc[0][tid] = 0.0;
  colacc[1][tid] = 0.0;

  // unit u (chunk-major, dealt round-robin): row block I, column blocks [c_lo, c_hi)
  // (32-bit block bookkeeping: keeps the persistent loop's scalar state small)
  auto unit_I = [&](int u) { return row_block0 + u % n_rb; };
  auto unit_clo = [&](int u) { return j_lo + (u / n_rb) * chunk_blocks; };
  auto unit_chi = [&](int u) {
    const int e = j_lo + (u / n_rb + 1) * chunk_blocks;
    return e < j_hi ? e : j_hi;
  };
  auto first_J = [&](int I, int lo, int hi) -> int {
    if (I >= nb_active) return -1;
    int J = lo;
    if (J < I) {
      if (((I + J) & 1) == 0) ++J;  // J < I needs I+J odd (J may become I)
    } else if (J > I) {
      if ((I + J) & 1) ++J;         // J > I needs I+J even
    }
    return J < hi ? J : -1;
  };
  auto next_J = [&](int I, int J, int hi) -> int {
    const int n = (J == I - 1) ? I : J + 2;
    return n < hi ? n : -1;
  };
  // next unit (from u, stepping by G) that has at least one column block
  auto seek = [&](int u, int& J) {
    while (u < n_units) {
      J = first_J(unit_I(u), unit_clo(u), unit_chi(u));
      if (J >= 0) break;
      u += G;
    }
    return u;
  };

  unsigned voff[C::PIECES];
#pragma unroll
  for (int q = 0; q < C::PIECES; ++q) {
    const int p = (wave * C::PIECES + q) * 64 + lane;
    const int row = p / C::SLOTS;
    const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
    voff[q] = static_cast<unsigned>(row * ldh * 2 + slot * 16);
  }
  const unsigned dst0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + wave * C::PIECES * 64))));
  // stage h (0/1) of global column block J
  auto issue = [&](int buf, int J, int h) {
    const uint16_t* sbase =
        ucols + (static_cast<int64_t>(J - col_block0) * 256 + h * C::SC) * ldh + slice_off;
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

  // A single accumulator per tile carries H_i.H_j + H_i.L_j + L_i.H_j (all in
  // units of 2^-24), so the epilogue needs no combine step.
  f16x8 ah[C::RT][C::NKS], al[C::RT][C::NKS];
  auto load_a = [&](int I) {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
      const int64_t row = static_cast<int64_t>(I - row_block0) * kSpRows + wave * 64 + rt * MT + li;
      const uint16_t* src = urows + row * ldh + slice_off;
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        ah[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + (c * C::LG + lq) * 8));
        al[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + KS + (c * C::LG + lq) * 8));
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
  };
  constexpr float kFold = 0x1p8f;  // tile sums (units of 2^-24) -> multiples of 2^-32

  int boh[C::NKS], bol[C::NKS];
#pragma unroll
  for (int c = 0; c < C::NKS; ++c) {
    boh[c] = li * C::SLOTS + ((c * C::LG + lq) ^ (li & C::SWZ));
    bol[c] = li * C::SLOTS + ((C::HI + c * C::LG + lq) ^ (li & C::SWZ));
  }

  // row accumulators as float pairs: the epilogue adds run as v_pk_add_f32
  // (two lanes' worth per issue), half the VALU issue under the MFMAs
  f32x2 racc[C::RT][C::NV / 2];
  double facc[C::RT][C::NV];
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
    for (int r = 0; r < C::NV / 2; ++r) racc[rt][r] = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int r = 0; r < C::NV; ++r) facc[rt][r] = 0.0;
  }

  // one 128-column stage: per 16-column tile, a fresh accumulator per row tile
  // -> row sums (racc) and the tile's column sums (-> LDS fp64, exact).
  // Software-pipelined: tile ct's MFMAs are issued beside tile ct-1's epilogue
  // (two accumulator sets) and tile ct+1's B fragments are read from LDS during
  // tile ct.  The column-sum add is branch-free (scaled by 0 on the diagonal
  // pair), so each tile is one scheduling region; SG interleaves it explicitly
  // (one MFMA, then a B read or one epilogue VALU op, ...) instead of leaving
  // the epilogue as a VALU burst between MFMA bursts.
  auto compute = [&](const float4* B, float cmul, double* cacc) {
    acc_t m[2][C::RT];
    f16x8 bh[2][C::NKS], bl[2][C::NKS];
    auto load_b = [&](int sb, int ct) {
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        bh[sb][c] = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + boh[c]]);
        bl[sb][c] = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + bol[c]]);
      }
    };
    load_b(0, 0);
#pragma unroll
    for (int ct = 0; ct <= C::NCT; ++ct) {
      if (ct + 1 < C::NCT) load_b((ct + 1) & 1, ct + 1);
      if (ct < C::NCT) {
        const int st = ct & 1;
        const acc_t zero = {};
#pragma unroll
        for (int c = 0; c < C::NKS; ++c) {
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) m[st][rt] = A::mfma(ah[rt][c], bh[st][c], c == 0 ? zero : m[st][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) m[st][rt] = A::mfma(ah[rt][c], bl[st][c], m[st][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) m[st][rt] = A::mfma(al[rt][c], bh[st][c], m[st][rt]);
        }
      }
      if (ct > 0) {
        const int pt = (ct - 1) & 1;
        f32x2 cp2 = {0.0f, 0.0f};
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
          for (int r = 0; r < C::NV / 2; ++r) {
            const f32x2 t = {m[pt][rt][2 * r], m[pt][rt][2 * r + 1]};
            racc[rt][r] += t;
            cp2 += t;
          }
        }
        const float cp = cp2.x + cp2.y;
        atomicAdd(cacc + (ct - 1) * MT + li, static_cast<double>(__builtin_rintf(cp * cmul)));
      }
      {
        constexpr int NM = 3 * C::NKS * C::RT;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          if (i < 2 * C::NKS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read (next tile's B)
          else __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);                   // VALU (epilogue)
        }
      }
      // pin the row accumulators here: otherwise LLVM sinks the adds to the
      // fold and keeps every tile's values live (hundreds of spilled VGPRs)
#pragma unroll
      for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
        for (int r = 0; r < C::NV / 2; ++r) asm volatile("" : "+v"(racc[rt][r]));
    }
  };
  // SG 2 ("chained"): the row sums ride in the MFMA accumulators.  Two
  // accumulator chains per row tile (even / odd column tiles) run through the
  // whole 256-column pair, so the MFMAs themselves add each tile into the row
  // sums (no per-element VALU add).  A tile's column sums are the growth of its
  // chain's lane total: T = sum of the lane's 16 values after the tile, minus T
  // before it (same column lane, the previous tile of that chain) -- one add
  // per element instead of two.  The epilogue of tile ct-1 (other chain) runs
  // beside tile ct's MFMAs and the B reads of tile ct+1.
  acc_t mc[2][C::RT];
  float tprev[2];
  auto compute_chained = [&](const float4* B, float cmul, double* cacc, bool first_stage) {
    f16x8 bh[2][C::NKS], bl[2][C::NKS];
    auto load_b = [&](int sb, int ct) {
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        bh[sb][c] = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + boh[c]]);
        bl[sb][c] = __builtin_bit_cast(f16x8, B[ct * MT * C::SLOTS + bol[c]]);
      }
    };
    load_b(0, 0);
#pragma unroll
    for (int ct = 0; ct <= C::NCT; ++ct) {
      // the next tile's B reads go out first and are fenced there, so their
      // latency hides under this tile's MFMAs (left alone, the scheduler
      // sinks them to their use and each tile starts with an LDS wait)
      if (ct + 1 < C::NCT) load_b((ct + 1) & 1, ct + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (ct < C::NCT) {
        const int ch = ct & 1;
        const bool fresh = first_stage && ct < 2;  // first tile of the chain in this pair
#pragma unroll
        for (int c = 0; c < C::NKS; ++c) {
          const acc_t zero = {};
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt)
            mc[ch][rt] = A::mfma(ah[rt][c], bh[ch][c], (c == 0 && fresh) ? zero : mc[ch][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) mc[ch][rt] = A::mfma(ah[rt][c], bl[ch][c], mc[ch][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) mc[ch][rt] = A::mfma(al[rt][c], bh[ch][c], mc[ch][rt]);
        }
      }
      if (ct > 0) {
        const int ch = (ct - 1) & 1;
        float t0 = mc[ch][0][0], t1 = mc[ch][0][1];  // two short chains (latency), fixed order
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
          for (int r = rt == 0 ? 2 : 0; r < C::NV; r += 2) {
            t0 += mc[ch][rt][r];
            t1 += mc[ch][rt][r + 1];
          }
        }
        const float T = t0 + t1;
        const float cp = (first_stage && ct - 1 < 2) ? T : T - tprev[ch];
        tprev[ch] = T;
        atomicAdd(cacc + (ct - 1) * MT + li, static_cast<double>(__builtin_rintf(cp * cmul)));
      }
      constexpr int NM = 3 * C::NKS * C::RT;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // VALU (previous tile's epilogue)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto fold_chains = [&]() {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int r = 0; r < C::NV; ++r)
        facc[rt][r] += static_cast<double>(__builtin_rintf((mc[0][rt][r] + mc[1][rt][r]) * kFold));
  };

  auto fold_rows = [&]() {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int r = 0; r < C::NV; ++r) {
        facc[rt][r] += static_cast<double>(__builtin_rintf(racc[rt][r / 2][r % 2] * kFold));
        racc[rt][r / 2][r % 2] = 0.0f;
      }
  };
  auto finish_unit = [&](int I) {
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
      for (int r = 0; r < C::NV; ++r) {
        double v = facc[rt][r];
#pragma unroll
        for (int sh = 1; sh < MT; sh <<= 1) v += __shfl_xor(v, sh);
        facc[rt][r] = v;
      }
    }
    double mine = 0.0;
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
      for (int r = 0; r < C::NV; ++r) {
        if (rt * C::NV + r == li) mine = facc[rt][r];
        facc[rt][r] = 0.0;
      }
    }
    const int rt = li / C::NV, r = li % C::NV;
    const int64_t row = static_cast<int64_t>(I) * kSpRows + wave * 64 + rt * MT + A::row(r, lq);
    atomicAdd(acc_out + row, static_cast<unsigned long long>(static_cast<long long>(mine)));
  };
  auto flush_cols = [&](int buf, int J) {
    const double v = colacc[buf][tid];
    if (v != 0.0)
      atomicAdd(acc_out + static_cast<int64_t>(J) * 256 + tid,
                static_cast<unsigned long long>(static_cast<long long>(v)));
    colacc[buf][tid] = 0.0;
  };

  int J = -1;
  int unit = seek(g, J);
  if (unit >= n_units) return;
  int I = unit_I(unit), c_hi = unit_chi(unit);
  issue(0, J, 0);
  load_a(I);
  const float4* B0 = lds;
  const float4* B1 = lds + C::F4;
  int cb = 0;             // colacc buffer of the current pair
  int flushJ = -1;        // column block whose sums wait in colacc[cb ^ 1]

  while (true) {
    int nJ = next_J(I, J, c_hi), n_unit = unit;
    if (nJ < 0) n_unit = seek(unit + G, nJ);
    const bool has_next = n_unit < n_units;
    const bool last_of_unit = n_unit != unit;
    const bool cols_too = J != I;

    const float cmul = cols_too ? kFold : 0.0f;  // diagonal pair: row sums only

    // lgkmcnt(0): the previous pair's LDS column adds (no-return ds_add_f64)
    // must land before another wave's flush reads them.  hipcc emits no LDS
    // wait at this loop-top barrier (measured: a lost tile partial, rarely)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (flushJ >= 0) flush_cols(cb ^ 1, flushJ);
    issue(1, J, 1);
    if constexpr (SG == 2) compute_chained(B0, cmul, &colacc[cb][0], true);
    else compute(B0, cmul, &colacc[cb][0]);

    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (has_next) issue(0, nJ, 0);
    if constexpr (SG == 2) {
      compute_chained(B1, cmul, &colacc[cb][C::SC], false);
      fold_chains();
    } else {
      compute(B1, cmul, &colacc[cb][C::SC]);
      fold_rows();
    }
    flushJ = cols_too ? J : -1;
    cb ^= 1;
    if (last_of_unit) finish_unit(I);

    if (!has_next) break;
    if (last_of_unit) {
      unit = n_unit;
      I = unit_I(unit);
      c_hi = unit_chi(unit);
      load_a(I);
    }
    J = nJ;
  }
  __syncthreads();
  if (flushJ >= 0) flush_cols(cb ^ 1, flushJ);
}

// ---------------------------------------------------------------------------
// Symmetric kernel on 512-row super blocks (SYM2, the default).  Same per-tile
// arithmetic as gram_sym_kernel (three products in one accumulator, row sums
// chained in the MFMA accumulators, column sums from the growth of the chain's
// lane total), but each wave owns 128 rows (8 row tiles): every B fragment
// read from LDS feeds twice the MFMAs, every LDS-DMA'd stage serves 512 rows,
// and the per-pair column flush is spread over twice the rows.  Orientation on
// super blocks (512 rows = the row granule, so shard-independent): super block
// P takes super block Q when Q == P (diagonal: row sums only, all columns),
// Q > P and P+Q even, Q < P and P+Q odd.  Work is scheduled in 512 x 256 pairs
// (P, J), J a 256-column block of super block Q = J/2: two 128-column stages,
// then the chains are folded (256 columns: the chain lengths, and so the error
// bound, of gram_sym_kernel) into an LDS fp64 row accumulator of exact
// integers, flushed to the int64 output per unit; the pair's 256 column sums
// are flushed per pair.  The half-super-block granularity keeps small launches
// (a GPU's own shard) balanced; a skip range [skip_lo, skip_hi) of J lets one
// launch cover every column but an already processed shard.
// timing-only ablations of gram_sym2_kernel (results WRONG when != 0; built
// into build/ablN by scripts/build_ablations.sh, never into the product library)
#ifndef DAL_SYM2_ABL
#define DAL_SYM2_ABL 0
#endif
// Column sums of a pair (P, J) from ONE row per block: 1^T (U_P U_J^T) =
// sigma_P U_J^T with sigma_P = sum of P's 512 operand rows, formed once per
// row unit from the resident A fragments.  For each 16-column tile one wave
// (round robin) issues 3 NKS extra MFMAs with sigma_P as the A operand (all
// 16 A rows equal, so any output row is the column sum) and stores one value
// per column: +3 % MFMAs instead of a per-element VALU add and four same-
// address LDS atomics per column per wave (those cost 7-12 %).
#ifndef DAL_SYM2_SIGMA
#define DAL_SYM2_SIGMA 1  // 1: at KS = 32 (measured faster there only), 2: always, 0: never (A/B builds)
#endif

// One step of a reduce-scatter over the 16 lanes of a DPP row: lanes whose
// select bit is clear keep v[k] (k < H) summed with their partner's, lanes
// whose bit is set keep v[k + H]; CTRL is a DPP permutation pairing each lane
// with a lane of the opposite bit (row_mirror, row_half_mirror, quad swaps).
template <int H, int CTRL, int N = 32>
__device__ __forceinline__ void row_reduce_scatter_step(float (&v)[N], bool hi) {
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float keep = hi ? v[k + H] : v[k];
    const float send = hi ? v[k] : v[k + H];
    v[k] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), CTRL,
                                                                        0xF, 0xF, false));
  }
}

// Reduce-scatter of N values over the 16 lanes of a DPP row (N = 16: lane li
// ends with the 16-lane sum of value li; N = 8: of value li & 7).
template <int N>
__device__ __forceinline__ void row_sum_scatter(float (&v)[N], int li) {
  if constexpr (N == 16) {
    row_reduce_scatter_step<8, 0x140, 16>(v, li & 8);
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k)
      v[k] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[k]), 0x140, 0xF,
                                                                   0xF, false));
  }
  row_reduce_scatter_step<4, 0x141, N>(v, li & 4);
  row_reduce_scatter_step<2, 0x4E, N>(v, li & 2);
  row_reduce_scatter_step<1, 0xB1, N>(v, li & 1);
}

// Lane id recomputed at the point of use (asm volatile: never hoisted out of
// a loop or merged with another use), so that lane-derived addresses are
// rematerialised instead of living in -- and spilling from -- VGPRs across
// the whole pair loop (a spill reload's vmcnt wait also drains the stage DMA).
#ifndef DAL_SYM2_FRESH
#define DAL_SYM2_FRESH 1  // 0: timing-only A/B build (plain lane id, spills)
#endif
__device__ __forceinline__ unsigned fresh_lane() {
  if constexpr (!DAL_SYM2_FRESH) return threadIdx.x & 63;
  unsigned v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return v;
}

template <int KS>
struct Sym2Cfg {
  static constexpr int MT = 16;
  static constexpr int ROWB = KS * 4;                 // bytes per column row (H + L)
  static constexpr int SLOTS = ROWB / 16;
  static constexpr int HI = KS / 8;
  static constexpr int STAGE = 32768;                 // bytes per LDS stage
  static constexpr int SC = STAGE / ROWB;             // columns per stage: 128 (KS 64) or 256 (KS 32)
  static constexpr int SPP = 256 / SC;                // stages per 512 x 256 pair: 2 or 1
  static constexpr int F4 = STAGE / 16;
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = STAGE / (4 * 1024);   // 1-KiB DMA pieces per wave per stage
  static constexpr int RT = 8;                        // 16-row tiles per wave (128 rows)
  static constexpr int LG = 4;
  static constexpr int NKS = KS / 32;                 // k-steps of v_mfma_f32_16x16x32_f16
  static constexpr int NCT = SC / MT;                 // column tiles per stage
  static constexpr int NV = 4;                        // accumulator values per lane
  static constexpr int SB = 512;                      // super block
  static_assert(NKS >= 1 && PIECES >= 1 && (SPP == 1 || SPP == 2), "bad slice");
};

template <int KS>
__global__ __launch_bounds__(kSpThreads, 2) void gram_sym2_kernel(
    const uint16_t* __restrict__ urows, int srow0, int n_srb,
    const uint16_t* __restrict__ ucols, int jcol0, int j_lo, int j_hi, int skip_lo, int skip_hi,
    int ns_active, int64_t ldh, int slice_off, int chunk_j, int n_chunks,
    unsigned long long* __restrict__ acc_out, int a_nt, int contig) {
  using C = Sym2Cfg<KS>;
  constexpr bool SIG = DAL_SYM2_SIGMA == 2 || (DAL_SYM2_SIGMA == 1 && KS == 32);
  using A = SpAcc<16>;
  using acc_t = A::type;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * C::F4];
  __shared__ double colacc[2][256];
  __shared__ double rowacc[C::SB];
  // sigma_P: per-wave partial sums, then the split row (H' | L', fp16 at 2^-6
  // of the operand's scale) read as an A fragment (every lane of a DPP row
  // reads the same 16 B: broadcast)
  __shared__ float sig_part[SIG ? 4 : 1][SIG ? KS : 1];
  __shared__ f16x8 sig_row[SIG ? 2 * C::HI : 1];

  const int tid = threadIdx.x;
  const int wave = DAL_SYM2_FRESH ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6, lane = tid & 63;
  const int li = lane & 15, lq = lane >> 4;
  const int G = gridDim.x, g = blockIdx.x;
  colacc[0][tid] = 0.0;
  colacc[1][tid] = 0.0;
  rowacc[tid] = 0.0;
  rowacc[tid + 256] = 0.0;

  // Work = the pairs (P, J) over row super blocks P and 256-column blocks J in
  // [j_lo, j_hi) minus [skip_lo, skip_hi), as segments (P, raw column range
  // [rlo, rhi)) walked by a raw column cursor r (J = jmap(r)):
  //  contig: block g owns the g-th 1/G of the P-major raw grid (P, r) -- an
  //          equal share of pairs (the orientation takes every other pair of
  //          column blocks along a row) in at most a few segments, so the A
  //          fragments are loaded once or twice per block;
  //  chunk:  unit u = (P = u % n_srb, column chunk u / n_srb), dealt round-robin
  //          (all blocks sweep the same column chunks together: L2 reuse of
  //          the column stages, at one A load per unit).
  const int sk_lo = skip_lo > j_lo ? skip_lo : j_lo, sk_hi = skip_hi < j_hi ? skip_hi : j_hi;
  const int skl = contig && sk_hi > sk_lo ? sk_hi - sk_lo : 0;  // chunk mode skips through takes()
  const int nje = j_hi - j_lo - skl;
  const int nre0 = ns_active - srow0, nre = nre0 < n_srb ? (nre0 > 0 ? nre0 : 0) : n_srb;
  const int64_t raw = static_cast<int64_t>(nre) * nje;
  const int64_t ka = raw * g / G, kb = raw * (g + 1) / G;
  const int n_seg = contig ? (kb > ka ? static_cast<int>((kb - 1) / nje - ka / nje) + 1 : 0) : n_srb * n_chunks;
  const int seg_step = contig ? 1 : G;
  auto seg_P = [&](int u) {
    return contig ? srow0 + static_cast<int>(ka / nje) + u : srow0 + u % n_srb;
  };
  auto seg_rlo = [&](int u) {
    return contig ? (u == 0 ? static_cast<int>(ka % nje) : 0) : (u / n_srb) * chunk_j;
  };
  auto seg_rhi = [&](int u) {
    if (contig) return u == n_seg - 1 ? static_cast<int>((kb - 1) % nje) + 1 : nje;
    const int e = (u / n_srb + 1) * chunk_j;
    return e < nje ? e : nje;
  };
  auto jmap = [&](int r) { return j_lo + r + (j_lo + r >= sk_lo ? skl : 0); };
  auto takes = [&](int P, int J) -> bool {  // orientation on super blocks, minus the skip range
    const int Q = J >> 1;
    if (J >= skip_lo && J < skip_hi) return false;
    return Q == P || (Q > P && ((P + Q) & 1) == 0) || (Q < P && ((P + Q) & 1));
  };
  // first raw column >= r (below rhi) whose pair segment row P takes, or -1
  auto first_r = [&](int P, int r, int rhi) -> int {
    if (P >= ns_active) return -1;
    while (r < rhi && !takes(P, jmap(r))) ++r;
    return r < rhi ? r : -1;
  };
  auto seek = [&](int u, int& r) {
    while (u < n_seg) {
      r = first_r(seg_P(u), seg_rlo(u), seg_rhi(u));
      if (r >= 0) break;
      u += seg_step;
    }
    return u;
  };

  // per-piece source offsets are recomputed at each issue (registers are the
  // scarce resource here, VALU issue is not)
  auto voff = [&](int q) {
    const int p = (wave * C::PIECES + q) * 64 + static_cast<int>(fresh_lane());
    const int row = p / C::SLOTS;
    const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
    return static_cast<unsigned>(row * ldh * 2 + slot * 16);
  };
  const unsigned dst0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + wave * C::PIECES * 64))));
  // stage h (0/1) of 256-column block J into buffer buf
  auto issue = [&](int buf, int J, int h) {
    if constexpr (DAL_SYM2_ABL == 4) return;
    const uint16_t* sbase =
        ucols + (static_cast<int64_t>(J - jcol0) * 256 + h * C::SC) * ldh + slice_off;
#pragma unroll
    for (int q = 0; q < C::PIECES; ++q) {
      const unsigned dst = dst0 + static_cast<unsigned>(buf * C::STAGE + q * 1024);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff(q)), "s"(dst), "s"(sbase)
          : "memory");
    }
  };

  f16x8 ah[C::RT][C::NKS], al[C::RT][C::NKS];
  auto load_a = [&](int P) {
    // uniform 64-bit base + 32-bit per-lane offsets (no per-tile 64-bit addresses)
    const uint16_t* pb = urows + static_cast<int64_t>(P - srow0) * C::SB * ldh + slice_off;
    const unsigned fl = fresh_lane();
    const unsigned lrow = static_cast<unsigned>((wave * 128 + (fl & 15)) * ldh + (fl >> 4) * 8);
    const unsigned tstep = static_cast<unsigned>(16 * ldh);
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        const unsigned o = lrow + rt * tstep + c * C::LG * 8;
        if (a_nt) {  // read once per unit: keep the column stages resident in L2
          ah[rt][c] = __builtin_nontemporal_load(reinterpret_cast<const f16x8*>(pb + o));
          al[rt][c] = __builtin_nontemporal_load(reinterpret_cast<const f16x8*>(pb + o + KS));
        } else {
          ah[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(pb + o));
          al[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(pb + o + KS));
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if constexpr (SIG) {
      // this wave's 128 rows summed per feature: in lane order over the row
      // tiles (H then L of each), then over the 16 lanes of the DPP row
      constexpr int V = C::NKS * 8;
      float sp[V];
#pragma unroll
      for (int c = 0; c < C::NKS; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = 0.0f;
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) {
            t += static_cast<float>(ah[rt][c][e]);
            t += static_cast<float>(al[rt][c][e]);
          }
          sp[c * 8 + e] = t;
        }
      const int fl = static_cast<int>(fresh_lane()), fli = fl & 15, flq = fl >> 4;
      row_sum_scatter<V>(sp, fli);
      if (fli < V) sig_part[wave][(fli >> 3) * 32 + flq * 8 + (fli & 7)] = sp[0];
    }
  };
  // after a block_sync that follows load_a: sigma_P = the four waves' partials
  // (fixed order), scaled by 2^-6 (exact) and split into two fp16 terms
  auto build_sigma = [&]() {
    if constexpr (SIG) {
      if (tid < KS) {
        const float sg = ((sig_part[0][tid] + sig_part[1][tid]) + sig_part[2][tid]) + sig_part[3][tid];
        const float s6 = sg * 0x1p-6f;
        const _Float16 h = static_cast<_Float16>(s6);
        const _Float16 l = static_cast<_Float16>(s6 - static_cast<float>(h));
        reinterpret_cast<_Float16*>(sig_row)[tid] = h;
        reinterpret_cast<_Float16*>(sig_row)[KS + tid] = l;
      }
    }
  };
  constexpr float kFold = 0x1p8f;  // units of 2^-24 -> multiples of 2^-32

  int boh[C::NKS], bol[C::NKS];
#pragma unroll
  for (int c = 0; c < C::NKS; ++c) {
    boh[c] = li * C::SLOTS + ((c * C::LG + lq) ^ (li & C::SWZ));
    bol[c] = li * C::SLOTS + ((C::HI + c * C::LG + lq) ^ (li & C::SWZ));
  }

  // row-sum chains: two (even / odd column tiles, whose growth gives the
  // column sums) or, with sigma, one per row tile
  constexpr int NCH = SIG ? 1 : 2;
  acc_t mc[NCH][C::RT];
  float tprev[2];
  f16x8 sgh[SIG ? C::NKS : 1], sgl[SIG ? C::NKS : 1];  // sigma_P fragments
  // one 128-column stage; fresh = first stage after a fold (chains restart)
  // (LDS operands are addressed by index, never through generic pointers:
  // 64-bit flat addresses would cost registers this kernel does not have)
  auto compute = [&](int buf, float cmul, int cbuf, int col0, bool fresh_stage) {
    // one register set of B fragments: k-step c of tile ct+1 is read as soon as
    // tile ct's MFMAs of k-step c are issued (24 MFMAs of latency cover)
    f16x8 bh[C::NKS], bl[C::NKS];
    auto load_b = [&](int c, int ct) {
      bh[c] = __builtin_bit_cast(f16x8, lds[buf * C::F4 + ct * 16 * C::SLOTS + boh[c]]);
      bl[c] = __builtin_bit_cast(f16x8, lds[buf * C::F4 + ct * 16 * C::SLOTS + bol[c]]);
    };
#pragma unroll
    for (int c = 0; c < C::NKS; ++c) load_b(c, 0);
#pragma unroll
    for (int ct = 0; ct <= C::NCT; ++ct) {
      __builtin_amdgcn_sched_barrier(0);
      if (ct < C::NCT) {
        const int ch = ct % NCH;
        const bool fresh = fresh_stage && ct < NCH;
        // column tile ct's sums: this wave's turn (wave-uniform branch)
        const bool sig = SIG && (ct & 3) == wave && DAL_SYM2_ABL != 8;
        acc_t sg = {};
#pragma unroll
        for (int c = 0; c < C::NKS; ++c) {
          const acc_t zero = {};
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt)
            mc[ch][rt] = A::mfma(ah[rt][c], bh[c], (c == 0 && fresh) ? zero : mc[ch][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) mc[ch][rt] = A::mfma(ah[rt][c], bl[c], mc[ch][rt]);
#pragma unroll
          for (int rt = 0; rt < C::RT; ++rt) mc[ch][rt] = A::mfma(al[rt][c], bh[c], mc[ch][rt]);
          if (sig) {
            sg = A::mfma(sgh[c], bh[c], sg);
            sg = A::mfma(sgh[c], bl[c], sg);
            sg = A::mfma(sgl[c], bh[c], sg);
          }
          if (ct + 1 < C::NCT) load_b(c, ct + 1);
        }
        // every output row of the sigma tile is the column sum (units 2^-18)
        if (sig && lq == 0) colacc[cbuf][col0 + ct * 16 + li] = static_cast<double>(__builtin_rintf(sg[0] * cmul * 64.0f));
      }
      if (!SIG && ct > 0 && DAL_SYM2_ABL != 6) {
        const int ch = (ct - 1) & 1;
        float t0 = mc[ch % NCH][0][0], t1 = mc[ch % NCH][0][1];
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) {
#pragma unroll
          for (int r = rt == 0 ? 2 : 0; r < C::NV; r += 2) {
            t0 += mc[ch % NCH][rt][r];
            t1 += mc[ch % NCH][rt][r + 1];
          }
        }
        const float T = t0 + t1;
        const float cp = (fresh_stage && ct - 1 < 2) ? T : T - tprev[ch];
        tprev[ch] = T;
        if constexpr (DAL_SYM2_ABL != 2)
          atomicAdd(&colacc[cbuf][col0 + (ct - 1) * 16 + li], static_cast<double>(__builtin_rintf(cp * cmul)));
      }
      {
        constexpr int NM = 3 * C::RT;  // MFMAs per k-step
#pragma unroll
        for (int c = 0; c < C::NKS; ++c) {
#pragma unroll
          for (int i = 0; i < NM; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            if constexpr (!SIG)
              __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // VALU (previous tile's epilogue)
          }
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);    // next tile's B, k-step c
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // chains -> LDS row accumulator (exact integer fp64 adds).  The 16 column
  // lanes of a DPP row hold partials of the same 32 rows; a 4-step
  // reduce-scatter (fixed pairing, so a fixed order per row) leaves each lane 2
  // fully summed rows, added by all 64 lanes at distinct LDS addresses (16
  // lanes adding to one LDS address serialise; a full per-row DPP reduction
  // followed by one lane's 32 adds measured 5 % slower at 100k x 64).
  auto fold_rows = [&]() {
    if constexpr (DAL_SYM2_ABL == 1) return;
    float v[32];
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int q = 0; q < C::NV; ++q) v[rt * 4 + q] = NCH == 1 ? mc[0][rt][q] : mc[0][rt][q] + mc[NCH - 1][rt][q];
    row_reduce_scatter_step<16, 0x140>(v, li & 8);  // row_mirror: lane i <-> 15 - i
    row_reduce_scatter_step<8, 0x141>(v, li & 4);   // row_half_mirror: i <-> i ^ 7
    row_reduce_scatter_step<4, 0x4E>(v, li & 2);    // quad_perm [2,3,0,1]: i <-> i ^ 2
    row_reduce_scatter_step<2, 0xB1>(v, li & 1);    // quad_perm [1,0,3,2]: i <-> i ^ 1
    // v[k] = original index k + 2 b0 + 4 b1 + 8 b2 + 16 b3 (b = bits of li) = rt * 4 + q
    const int rt = ((li >> 1) & 1) | (((li >> 2) & 1) << 1) | (((li >> 3) & 1) << 2);
    const int row = wave * 128 + rt * 16 + 4 * lq + 2 * (li & 1);
    atomicAdd(&rowacc[row], static_cast<double>(__builtin_rintf(v[0] * kFold)));
    atomicAdd(&rowacc[row + 1], static_cast<double>(__builtin_rintf(v[1] * kFold)));
  };
  auto flush_one = [&](double& slot, int64_t out_row) {
    const double v = slot;
    if (v != 0.0) atomicAdd(acc_out + out_row, static_cast<unsigned long long>(static_cast<long long>(v)));
    slot = 0.0;
  };
  auto flush_cols = [&](int cbuf, int Jf) {
    if constexpr (DAL_SYM2_ABL == 7) {  // no global column flush
      colacc[cbuf][tid] = 0.0;
      return;
    }
    flush_one(colacc[cbuf][tid], static_cast<int64_t>(Jf) * 256 + tid);
  };
  auto flush_rows = [&](int Pf) {
    flush_one(rowacc[tid], static_cast<int64_t>(Pf) * C::SB + tid);
    flush_one(rowacc[tid + 256], static_cast<int64_t>(Pf) * C::SB + tid + 256);
  };
  // lgkmcnt(0) with every barrier: LDS adds (no-return) must land before
  // another wave's flush reads them (hipcc may omit this wait at a loop barrier)
  auto block_sync = [&]() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (DAL_SYM2_ABL != 3) __syncthreads();
  };

  int r = -1;
  int unit = seek(contig ? 0 : g, r);
  if (unit >= n_seg) return;
  int P = seg_P(unit), rhi_u = seg_rhi(unit);
  int J = jmap(r);
  issue(0, J, 0);
  load_a(P);
  bool sig_fresh = true;  // sigma_P must be rebuilt (A fragments reloaded)
  int cb = 0;        // colacc buffer of the current pair
  int buf = 0;       // LDS stage of the pair's first stage (alternates per pair when SPP == 1)
  int flushJ = -1;   // column block whose sums wait in colacc[cb ^ 1]
  int flushP = -1;   // row super block whose sums wait in rowacc

  while (true) {
    int nr = first_r(P, r + 1, rhi_u), n_unit = unit;
    if (nr < 0) n_unit = seek(unit + seg_step, nr);
    const bool has_next = n_unit < n_seg;
    const int nP = has_next ? seg_P(n_unit) : -1;
    const bool new_rows = nP != P;     // the next pair needs other A rows
    const int nJ = has_next ? jmap(nr) : -1;
    const bool diag = (J >> 1) == P;
    const float cmul = diag ? 0.0f : kFold;  // diagonal super block: row sums only

    block_sync();
    if (flushJ >= 0) flush_cols(cb ^ 1, flushJ);
    if (flushP >= 0) flush_rows(flushP);
    flushP = -1;
    if (SIG && sig_fresh) {
      build_sigma();
      block_sync();
      sig_fresh = false;
#pragma unroll
      for (int c = 0; c < (SIG ? C::NKS : 0); ++c) {
        const int flq = static_cast<int>(fresh_lane()) >> 4;
        sgh[c] = sig_row[c * C::LG + flq];
        sgl[c] = sig_row[C::HI + c * C::LG + flq];
      }
    }
    if constexpr (C::SPP == 2) {  // KS 64: two 128-column stages
      issue(1, J, 1);
      compute(0, cmul, cb, 0, true);
      // one chain: fold per 128-column stage (chain length = two chains per pair)
      if constexpr (NCH == 1) fold_rows();
      block_sync();
      if (has_next) issue(0, nJ, 0);
      compute(1, cmul, cb, 128, NCH == 1);
    } else {                      // KS 32: one 256-column stage, buffers alternate per pair
      if (has_next) issue(buf ^ 1, nJ, 0);
      compute(buf, cmul, cb, 0, true);
      buf ^= 1;
    }
    fold_rows();

    flushJ = diag ? -1 : J;
    cb ^= 1;
    if (new_rows) flushP = P;
    if (!has_next) break;
    unit = n_unit;
    rhi_u = seg_rhi(unit);
    if (new_rows) {
      P = nP;
      if constexpr (DAL_SYM2_ABL != 5) load_a(P);
      sig_fresh = true;
    }
    r = nr;
    J = nJ;
  }
  block_sync();
  if (flushJ >= 0) flush_cols(cb ^ 1, flushJ);
  if (flushP >= 0) flush_rows(flushP);
}

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

int device_cus_split() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  return cus;
}

// Round-robin (sync_sweep) makespan of n_chunks column chunks: blocks take
// units g, g+G, ... of the chunk-major list; returns total / (G * makespan).
double sweep_efficiency(int64_t n_row_blocks, int64_t n_pairs, int64_t chunks, int64_t G) {
  const int64_t cs = ceil_div(n_pairs, chunks);
  const int64_t nc = ceil_div(n_pairs, cs);
  const int64_t n_units = n_row_blocks * nc;
  int64_t makespan = 0;
  // per-block load depends only on which chunks its units fall in; blocks
  // 0..G-1 differ by at most one unit, so check the heaviest candidates
  for (int64_t g = 0; g < G && g < n_units; ++g) {
    int64_t load = 0;
    for (int64_t u = g; u < n_units; u += G) {
      const int64_t c = u / n_row_blocks;
      load += (c == nc - 1) ? n_pairs - c * cs : cs;
    }
    makespan = load > makespan ? load : makespan;
  }
  return makespan ? static_cast<double>(n_row_blocks * n_pairs) / (static_cast<double>(G) * makespan) : 0.0;
}

template <int KS, int MT>
int launch_split(const uint16_t* rows, int64_t n_rows_pad, const uint16_t* cols, int64_t n_cols_pad,
                 int64_t ldh, int slice_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  using C = SpCfg<KS, MT>;
  const int64_t n_row_blocks = n_rows_pad / kSpRows;
  const int64_t n_pairs = n_cols_pad / (2 * C::SC);
  const int G0 = grid_blocks > 0 ? grid_blocks : 2 * device_cus_split();
  const char* env = getenv("DAL_GRAM_SCHED");
  const int sync_sweep = env ? atoi(env) : 1;
  int64_t cs;
  if (sync_sweep) {
    // fewest chunks (fewest A reloads) whose round-robin makespan is within 3% of ideal
    int64_t best_c = 1;
    double best_e = 0.0;
    for (int64_t c = 1; c <= 64 && c <= n_pairs; ++c) {
      const double e = sweep_efficiency(n_row_blocks, n_pairs, c, G0);
      if (e > best_e + 1e-9) {
        best_e = e;
        best_c = c;
      }
      if (e >= 0.97) {
        best_c = c;
        break;
      }
    }
    cs = ceil_div(n_pairs, best_c);
  } else {
    // ~32 units per block: short tails, long enough units to amortise the butterfly
    cs = (n_pairs * n_row_blocks) / (static_cast<int64_t>(G0) * 32);
    cs = cs < 1 ? 1 : (cs > 32 ? 32 : cs);
    if (cs > n_pairs) cs = n_pairs;
  }
  const int64_t n_chunks = ceil_div(n_pairs, cs);
  const int64_t n_units = n_row_blocks * n_chunks;
  const int64_t G = n_units < G0 ? n_units : G0;
  hipLaunchKernelGGL((gram_split_kernel<KS, MT>), dim3(static_cast<unsigned>(G)), dim3(kSpThreads), 0, stream,
                     rows, cols, ldh, slice_off, n_pairs, static_cast<int>(cs), n_chunks, n_row_blocks,
                     sync_sweep, reinterpret_cast<unsigned long long*>(acc));
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// Number of column blocks J in [lo, hi) that row block I takes under the
// symmetric orientation rule (J == I; J > I with I+J even; J < I with I+J odd).
inline int64_t sym_pairs(int64_t I, int64_t lo, int64_t hi) {
  auto same_parity = [](int64_t a, int64_t b, int64_t p) -> int64_t {  // #J in [a, b) with J % 2 == p
    if (b <= a) return 0;
    return (b - p + 1) / 2 - (a - p + 1) / 2;
  };
  int64_t n = (lo <= I && I < hi) ? 1 : 0;
  n += same_parity(lo > I + 1 ? lo : I + 1, hi, I & 1);
  n += same_parity(lo, hi < I ? hi : I, (I & 1) ^ 1);
  return n;
}

// Column-chunk count for the symmetric kernels' round-robin units: unit u =
// (row block row0 + u % n_rb, chunk u / n_rb), dealt to block u % G.  Picks,
// among chunk counts giving >= min_units_per_block units per block, the one
// whose most loaded block has the fewest pairs (exact count; cached per shape).
inline int64_t sym_chunks(int64_t row0, int64_t n_rb, int64_t lo, int64_t hi, int64_t n_active, int64_t G0,
                          int min_units_per_block) {
  struct Entry {
    int64_t k[7];
    int64_t nc;
  };
  static thread_local Entry cache[8] = {};
  static thread_local int cache_next = 0;
  if (const char* e = getenv("DAL_GRAM_NC")) {  // timing knob: force the chunk count
    const int64_t f = atoll(e);
    if (f > 0) return f < hi - lo ? f : hi - lo;
  }
  const int64_t key[7] = {row0, n_rb, lo, hi, n_active, G0, min_units_per_block};
  for (const Entry& e : cache) {
    bool hit = e.nc > 0;
    for (int i = 0; i < 7 && hit; ++i) hit = e.k[i] == key[i];
    if (hit) return e.nc;
  }
  const int64_t nj = hi - lo;
  int64_t nc0 = 1;
  while (nc0 < nj && n_rb * nc0 < static_cast<int64_t>(min_units_per_block) * G0) ++nc0;
  int64_t best_nc = nc0, best_max = -1;
  std::vector<int64_t> load;
  int64_t tried = 0;
  for (int64_t c = nc0; c <= nj && tried < 24; ++c) {
    const int64_t cb = ceil_div(nj, c), ncc = ceil_div(nj, cb);
    if (c > nc0 && cb == ceil_div(nj, c - 1)) continue;  // same partition as c - 1
    ++tried;
    const int64_t units = n_rb * ncc, G = units < G0 ? units : G0;
    load.assign(static_cast<size_t>(G), 0);
    for (int64_t u = 0; u < units; ++u) {
      const int64_t I = row0 + u % n_rb;
      if (I >= n_active) continue;
      const int64_t clo = lo + (u / n_rb) * cb, chi = clo + cb < hi ? clo + cb : hi;
      load[static_cast<size_t>(u % G)] += sym_pairs(I, clo, chi);
    }
    int64_t mx = 0;
    for (int64_t v : load) mx = v > mx ? v : mx;
    if (best_max < 0 || mx < best_max) {
      best_max = mx;
      best_nc = ncc;
    }
  }
  Entry& e = cache[cache_next];
  cache_next = (cache_next + 1) % 8;
  for (int i = 0; i < 7; ++i) e.k[i] = key[i];
  e.nc = best_nc;
  return best_nc;
}

template <int KS, int MT, int SG>
int launch_sym(const uint16_t* rows, int64_t row_block0, int64_t n_rb, const uint16_t* cols,
               int64_t col_block0, int64_t j_lo, int64_t j_hi, int64_t nb_active, int64_t ldh,
               int slice_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  const int G0 = grid_blocks > 0 ? grid_blocks : 2 * device_cus_split();
  const int64_t nj = j_hi - j_lo;
  const int64_t nc = sym_chunks(row_block0, n_rb, j_lo, j_hi, nb_active, G0, 4);
  const int64_t cbk = ceil_div(nj, nc);
  const int64_t n_chunks = ceil_div(nj, cbk);
  const int64_t n_units = n_rb * n_chunks;
  const int64_t G = n_units < G0 ? n_units : G0;
  hipLaunchKernelGGL((gram_sym_kernel<KS, MT, SG>), dim3(static_cast<unsigned>(G)), dim3(kSpThreads), 0, stream,
                     rows, static_cast<int>(row_block0), static_cast<int>(n_rb), cols,
                     static_cast<int>(col_block0), static_cast<int>(j_lo), static_cast<int>(j_hi),
                     static_cast<int>(nb_active), ldh, slice_off, static_cast<int>(cbk),
                     static_cast<int>(n_chunks), reinterpret_cast<unsigned long long*>(acc));
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

// Pairs (P, J) the super-block kernel processes for row super block P over
// 256-column blocks [a, b) minus [skip_lo, skip_hi): J is taken when its super
// block Q = J / 2 is (Q == P, Q > P with P+Q even, Q < P with P+Q odd).  O(1).
inline int64_t sym2_pairs_range(int64_t P, int64_t a, int64_t b) {
  if (b <= a) return 0;
  auto takes = [P](int64_t Q) { return Q == P || (Q > P && ((P + Q) & 1) == 0) || (Q < P && ((P + Q) & 1)); };
  const int64_t qa = a >> 1, qb = (b - 1) >> 1;  // super blocks touched (inclusive)
  int64_t n = 2 * sym_pairs(P, qa, qb + 1);
  if ((a & 1) && takes(qa)) --n;        // only the upper half of qa lies in [a, b)
  if (!((b - 1) & 1) && takes(qb)) --n; // only the lower half of qb lies in [a, b)
  return n;
}
inline int64_t sym2_pairs(int64_t P, int64_t a, int64_t b, int64_t skip_lo, int64_t skip_hi) {
  const int64_t sa = a > skip_lo ? a : skip_lo, sb = b < skip_hi ? b : skip_hi;
  return sym2_pairs_range(P, a, b) - sym2_pairs_range(P, sa, sb);
}

// Column-chunk count for the super-block kernel's units (P, chunk of J),
// dealt round-robin: the fewest chunks, at least kSym2MinChunks, whose most
// loaded block has at most 8 % more pairs than the best balance found (exact
// pair counts; cached per shape).  Fewer chunks = fewer A-fragment loads and
// row flushes per block; more chunks = a smaller column working set swept by
// every block together (MALL hits): at 2M x 256 16-32 chunks beat the 1 the
// balance rule alone picks by 3.9 % (500k x 256: 1.7 %, 4M x 64: 0.9 %;
// scripts/gram_knob_ab.py).  Chunk mode only runs for operands > 40 MB.
constexpr int64_t kSym2MinChunks = 16;
inline int64_t sym2_chunks(int64_t srow0, int64_t n_srb, int64_t lo, int64_t hi, int64_t skip_lo, int64_t skip_hi,
                           int64_t ns_active, int64_t G0) {
  if (const char* e = getenv("DAL_GRAM_NC")) {  // timing knob: force the chunk count
    const int64_t f = atoll(e);
    if (f > 0) return f < hi - lo ? f : hi - lo;
  }
  int64_t min_nc = kSym2MinChunks;
  if (const char* e = getenv("DAL_GRAM_NC_MIN")) min_nc = atoll(e);  // A/B knob (1 = balance rule only)
  struct Entry {
    int64_t k[9];
    int64_t nc;
  };
  static thread_local Entry cache[8] = {};
  static thread_local int cache_next = 0;
  const int64_t key[9] = {srow0, n_srb, lo, hi, skip_lo, skip_hi, ns_active, G0, min_nc};
  for (const Entry& e : cache) {
    bool hit = e.nc > 0;
    for (int i = 0; i < 9 && hit; ++i) hit = e.k[i] == key[i];
    if (hit) return e.nc;
  }
  const int64_t nj = hi - lo;
  int64_t best_max = -1;
  std::vector<int64_t> load;
  std::vector<std::pair<int64_t, int64_t>> cand;  // (chunk count, max pairs per block)
  int tried = 0;
  for (int64_t c = 1; c <= nj && tried < 32; ++c) {
    const int64_t cb = ceil_div(nj, c), ncc = ceil_div(nj, cb);
    if (c > 1 && cb == ceil_div(nj, c - 1)) continue;  // same partition as c - 1
    ++tried;
    const int64_t units = n_srb * ncc, G = units < G0 ? units : G0;
    load.assign(static_cast<size_t>(G), 0);
    for (int64_t u = 0; u < units; ++u) {
      const int64_t P = srow0 + u % n_srb;
      if (P >= ns_active) continue;
      const int64_t clo = lo + (u / n_srb) * cb, chi = clo + cb < hi ? clo + cb : hi;
      load[static_cast<size_t>(u % G)] += sym2_pairs(P, clo, chi, skip_lo, skip_hi);
    }
    int64_t mx = 0;
    for (int64_t v : load) mx = v > mx ? v : mx;
    cand.emplace_back(ncc, mx);
    if (best_max < 0 || mx < best_max) best_max = mx;
  }
  int64_t best_nc = -1;
  for (int pass = 0; pass < 2 && best_nc < 0; ++pass)  // at least min_nc chunks if balanced, else any
    for (const auto& c : cand)
      if ((pass || c.first >= min_nc) && c.second * 100 <= best_max * 108) {
        best_nc = c.first;
        break;
      }
  if (best_nc < 0) best_nc = cand.back().first;
  Entry& e = cache[cache_next];
  cache_next = (cache_next + 1) % 8;
  for (int i = 0; i < 9; ++i) e.k[i] = key[i];
  e.nc = best_nc;
  return best_nc;
}

template <int KS>
int launch_sym2(const uint16_t* rows, int64_t srow0, int64_t n_srb, const uint16_t* cols, int64_t jcol0,
                int64_t j_lo, int64_t j_hi, int64_t skip_lo, int64_t skip_hi, int64_t ns_active, int64_t ldh,
                int slice_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  const int G0 = grid_blocks > 0 ? grid_blocks : 2 * device_cus_split();
  const int64_t nj = j_hi - j_lo;
  // scheduling: contiguous equal shares of the pair grid per block when the
  // column operand is small (<= 32 MB: 100k x 64 = 25.6 MB is 2-5 % faster),
  // else round-robin column-chunk units, whose blocks sweep the same column
  // stages together (with the 16-chunk floor: 284,807 x 30 = 36.5 MB 2.7 %,
  // 200k x 64 = 51 MB 3 %, 500k x 256 6 % faster than contiguous).  Exact
  // integer accumulation: the schedule never changes the bits.
  // DAL_GRAM_CONTIG=0/1 forces one (A/B knob).
  const char* cenv = getenv("DAL_GRAM_CONTIG");
  const int contig = cenv ? atoi(cenv) != 0 : nj * 256 * ldh * 2 <= (int64_t{32} << 20);
  int64_t cbk = nj, n_chunks = 1, G;
  if (contig) {
    const int64_t sl = skip_lo > j_lo ? skip_lo : j_lo, sh = skip_hi < j_hi ? skip_hi : j_hi;
    const int64_t nre = ns_active - srow0 < n_srb ? ns_active - srow0 : n_srb;
    const int64_t raw = (nre > 0 ? nre : 0) * (nj - (sh > sl ? sh - sl : 0));
    if (raw <= 0) return DAL_OK;
    G = raw < G0 ? raw : G0;
  } else {
    const int64_t nc = sym2_chunks(srow0, n_srb, j_lo, j_hi, skip_lo, skip_hi, ns_active, G0);
    cbk = ceil_div(nj, nc);
    n_chunks = ceil_div(nj, cbk);
    const int64_t n_units = n_srb * n_chunks;
    G = n_units < G0 ? n_units : G0;
  }
  hipLaunchKernelGGL((gram_sym2_kernel<KS>), dim3(static_cast<unsigned>(G)), dim3(kSpThreads), 0, stream,
                     rows, static_cast<int>(srow0), static_cast<int>(n_srb), cols, static_cast<int>(jcol0),
                     static_cast<int>(j_lo), static_cast<int>(j_hi), static_cast<int>(skip_lo),
                     static_cast<int>(skip_hi), static_cast<int>(ns_active), ldh, slice_off,
                     static_cast<int>(cbk), static_cast<int>(n_chunks), reinterpret_cast<unsigned long long*>(acc),
                     getenv("DAL_GRAM_ANT") ? atoi(getenv("DAL_GRAM_ANT")) : 1, contig);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

inline int split_ks(int64_t d_pad) { return d_pad == 32 ? 32 : 64; }

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" double dal_density_error_bound_split(int64_t n_cols) {
  // Per entry, with u = 2^-23 (a conservative unit roundoff for the MFMA's
  // internal fp32 accumulation, counted as sequential adds) and at most 1088
  // additions per fold chain (256 columns / MT column lanes x KS products):
  //   main chain    gamma_1088 * sum_d |h_i h_j|,  |h| <= (1 + 2^-11) |u|
  //   cross chain   gamma_2176 * 2^-10 * sum_d |u_i u_j|  (~2.4e-7)
  //   split         3.01 * 2^-22 * sum_d |u_i u_j| (+2^-37 per feature, subnormal halves)
  //   combine fma   2^-24,  fold rounding 2^-33 per fold (<= 1e-10 per column)
  // and sum_d |u_i u_j| <= 1 (Cauchy-Schwarz on unit rows).
  const double u = 1.0 / 8388608.0;  // 2^-23
  const double gamma = 1088.0 * u / (1.0 - 1088.0 * u);
  const double s = 1.0 / 4194304.0;  // 2^-22
  return (gamma * (1.0 + 1.0 / 512.0) + 5.0 * s + 1e-10) * static_cast<double>(n_cols) + 1e-9;
}

extern "C" double dal_density_error_bound_sym(int64_t n_cols) {
  // dal_gram_rowsum_sym (chained epilogue; also covers the per-tile one).  With
  // u = 2^-23 (conservative for the MFMA's internal fp32 adds), products exact
  // (f16 x f16), and c = 1 + 2^-8 >= sum_d |h_i h_j| + |h_i l_j| + |l_i h_j| over
  // sum_d |u_i u_j| <= 1 (Cauchy-Schwarz on unit rows), per density entry:
  //   row side   two chains of <= 8 tiles x 192 products, joined by one add
  //              (+4 adds of the cross-lane row sum in the 512-row kernel):
  //              gamma_1541 * c per column
  //   column side  a tile's column partial is T_k - T_{k-1}, T = sum of the
  //              lane's 16 chain values (k <= 8 tiles into the chain):
  //              (8 gamma_192 + 15 gamma_15 + u) * c per row; or (sigma form,
  //              KS 32: one chain of 16 tiles x 96 products per row, so the
  //              same row side) <sigma_P, u_j> from sigma_P summed in fp32
  //              (<= 22 adds) and split in two fp16 terms, one MFMA chain of
  //              96 products: (gamma_22 + gamma_96 + 3 * 2^-22) * c per row
  //   split + fp32 unit rows  5 * 2^-22;  fixed-point roundings <= 2^-33 each
  // Every column j of a row's density lies on exactly one side of its pair.
  const double u = 1.0 / 8388608.0;  // 2^-23
  auto gamma = [u](double n) { return n * u / (1.0 - n * u); };
  const double row = gamma(1541.0);
  const double col = 8.0 * gamma(192.0) + 15.0 * gamma(15.0) + u;
  const double c = 1.0 + 1.0 / 256.0;
  const double s = 1.0 / 4194304.0;  // 2^-22
  return ((row > col ? row : col) * c + 5.0 * s + 1e-10) * static_cast<double>(n_cols) + 1e-9;
}

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

extern "C" int dal_gram_rowsum_split(const uint16_t* rows, int64_t n_rows_pad, const uint16_t* cols,
                                     int64_t n_cols_pad, int64_t d_pad, int64_t* acc, int grid_blocks,
                                     dal_stream_t stream) {
  if (!rows || !cols || !acc) return DAL_ERR_ARG;
  if (n_rows_pad <= 0 || n_rows_pad % kSpRows || n_cols_pad <= 0 || n_cols_pad % DAL_ROW_GRANULE)
    return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad)) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(cols)) & 15) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  const int ks = split_ks(d_pad);
  const int64_t ldh = 2 * d_pad;
  const char* env = getenv("DAL_GRAM_MT");
  const int mt = env ? atoi(env) : 16;
  for (int64_t off = 0; off < d_pad; off += ks) {
    const int so = static_cast<int>(2 * off);  // halves: slice s starts at s * 2 * KS
    int rc;
    if (mt == 16)
      rc = ks == 32 ? launch_split<32, 16>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st)
                    : launch_split<64, 16>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st);
    else
      rc = ks == 32 ? launch_split<32, 32>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st)
                    : launch_split<64, 32>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st);
    if (rc != DAL_OK) return rc;
  }
  return DAL_OK;
}

extern "C" int dal_gram_rowsum_sym_skip(const uint16_t* rows, int64_t row_block0, int64_t n_row_blocks,
                                        const uint16_t* cols, int64_t col_block0, int64_t j_lo, int64_t j_hi,
                                        int64_t skip_lo, int64_t skip_hi, int64_t nb_active, int64_t d_pad,
                                        int64_t* acc, int grid_blocks, dal_stream_t stream) {
  if (!rows || !cols || !acc) return DAL_ERR_ARG;
  if (row_block0 < 0 || n_row_blocks <= 0 || col_block0 < 0 || nb_active <= 0) return DAL_ERR_SHAPE;
  if (j_lo < col_block0 || j_hi < j_lo || j_hi > nb_active || skip_hi < skip_lo) return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad)) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(cols)) & 15) return DAL_ERR_SHAPE;
  if (j_hi == j_lo || row_block0 >= nb_active) return DAL_OK;
  hipStream_t st = as_stream(stream);
  const int ks = split_ks(d_pad);
  const int64_t ldh = 2 * d_pad;
  // kernel: 512-row super blocks (default; half the LDS bytes, DMA and
  // column flushes per MFMA -- measured 0-4 % faster from 100k to 500k rows) or
  // the 256-row-block kernel (A/B knob DAL_GRAM_SYM=1).  Fixed per build, so
  // every GPU count runs the same kernel and produces the same bits.
  const char* kenv = getenv("DAL_GRAM_SYM");
  const int kind = kenv && atoi(kenv) == 1 ? 1 : 2;
  if (kind == 2) {
    // super-block rows: the row blocks (and nb_active) must be even (shards are 512-row multiples)
    if ((row_block0 | n_row_blocks | nb_active) & 1) return DAL_ERR_SHAPE;
    for (int64_t off = 0; off < d_pad; off += ks) {
      const int so = static_cast<int>(2 * off);
      const int rc = ks == 32 ? launch_sym2<32>(rows, row_block0 / 2, n_row_blocks / 2, cols, col_block0, j_lo, j_hi,
                                                skip_lo, skip_hi, nb_active / 2, ldh, so, acc, grid_blocks, st)
                              : launch_sym2<64>(rows, row_block0 / 2, n_row_blocks / 2, cols, col_block0, j_lo, j_hi,
                                                skip_lo, skip_hi, nb_active / 2, ldh, so, acc, grid_blocks, st);
      if (rc != DAL_OK) return rc;
    }
    return DAL_OK;
  }
  if (skip_hi > skip_lo && skip_hi > j_lo && skip_lo < j_hi) {  // 256-row kernel: the two sides separately
    int rc = DAL_OK;
    if (skip_lo > j_lo)
      rc = dal_gram_rowsum_sym_skip(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, skip_lo, 0, 0,
                                    nb_active, d_pad, acc, grid_blocks, stream);
    if (rc == DAL_OK && skip_hi < j_hi)
      rc = dal_gram_rowsum_sym_skip(rows, row_block0, n_row_blocks, cols, col_block0, skip_hi, j_hi, 0, 0,
                                    nb_active, d_pad, acc, grid_blocks, stream);
    return rc;
  }
  for (int64_t off = 0; off < d_pad; off += ks) {
    const int so = static_cast<int>(2 * off);
    // epilogue variant (A/B knob): 2 = chained accumulators (default), 1 = per-tile
    const char* env = getenv("DAL_GRAM_SG");
    const int sg = env ? atoi(env) : 2;
    int rc;
    if (sg == 1)
      rc = ks == 32 ? launch_sym<32, 16, 1>(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, j_hi,
                                            nb_active, ldh, so, acc, grid_blocks, st)
                    : launch_sym<64, 16, 1>(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, j_hi,
                                            nb_active, ldh, so, acc, grid_blocks, st);
    else
      rc = ks == 32 ? launch_sym<32, 16, 2>(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, j_hi,
                                            nb_active, ldh, so, acc, grid_blocks, st)
                    : launch_sym<64, 16, 2>(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, j_hi,
                                            nb_active, ldh, so, acc, grid_blocks, st);
    if (rc != DAL_OK) return rc;
  }
  return DAL_OK;
}

extern "C" int dal_gram_rowsum_sym(const uint16_t* rows, int64_t row_block0, int64_t n_row_blocks,
                                   const uint16_t* cols, int64_t col_block0, int64_t j_lo, int64_t j_hi,
                                   int64_t nb_active, int64_t d_pad, int64_t* acc, int grid_blocks,
                                   dal_stream_t stream) {
  return dal_gram_rowsum_sym_skip(rows, row_block0, n_row_blocks, cols, col_block0, j_lo, j_hi, 0, 0, nb_active,
                                  d_pad, acc, grid_blocks, stream);
}
