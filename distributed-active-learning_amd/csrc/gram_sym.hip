// Symmetric, compensated cosine Gram row-sum: the density d_i = sum_{j not in
// E} <u_i, u_j> of every pool row on fp16 MFMA at fp32-class accuracy, with S
// never stored.
//
// Reference: final_thesis/density_weighting.py:67-75 (U.multiply(UT) through
// IndexedRowMatrix/BlockMatrix), :95-100 (drop i,j in L0) and :157-161
// (groupByKey + sum per row); cosine_similarity.py:29-45 is the same product.
//
// Operand (dal_prep_split): every fp32 unit row at scale 2^12 as two fp16
// terms, H = fp16(2^12 u), L = fp16(2^12 u - H); u~ = H + L carries 2^12 u to
// 2^-22 relative, every product of two terms is exact in fp32 and lands in
// units of 2^-24.  Layout [n_pad][d_pad / KS][KS H | KS L].
//
// Symmetry.  Rows are grouped in 512-row super blocks.  Each unordered pair
// {P, Q} is multiplied once: P takes Q iff Q == P (diagonal), Q > P with P+Q
// even, or Q < P with P+Q odd (global indices, so the bits do not depend on
// the sharding).  The taker's rows are the A operand (register resident), Q's
// the B operand (LDS-staged); the kernel keeps the tile's ROW sums (-> P's
// rows).  The tile's column sums (-> Q's rows) are linear in P's rows,
// sum_{i in P} <H_i, u~_j> = <sigma^H_P, u~_j>, so they are added in closed
// form with the residual below (round 5; before, as sigma_P MFMAs and int64
// column flushes per pair).
//
// Compensation and column sums.  The A side holds H only: the MFMAs form
// T_ij = <H_i, u~_j> (two products per feature pair, H.H and H.L).  For a row
// r of super block B, dal_gram_sym_residual adds in closed form
//   row role (B takes Q):          sum_Q <L_r, sigma~_Q>   = <L_r, R_B>
//   column role (P takes B, P!=B): sum_P <u~_r, sigma~_P>  = <u~_r, C_B>
// (the column role: the pair's column sums <sigma^H_P, u~_r> plus the
// remainder <sigma^L_P, u~_r>) with sigma~_Q the sum of u~ over Q's rows
// (exact int64 in units of 2^-24) and R_B, C_B its sums over B's partners
// (parity-class prefix sums).  d_i is then sum_j <u~_i, u~_j> with nothing
// dropped; the MFMA work per algorithmic product is 2 fp16 products on half
// the pairs, and each row's density is written only by its own rows' launches
// (no cross-GPU sum).
//
// Exactness of the row sums (as the earlier kernels): chains are folded to
// multiples of 2^-32 and added as integers (LDS fp64 below 2^53, int64
// atomics); the residual is an fp64 dot in a fixed order rounded to 2^-32.
// The density bits are identical for any grid, column split or GPU count.
//
// MI355X design: block = 4 waves x 128 rows (one super block; at KS 128 with
// the round-robin schedule 8 waves, two super blocks P and P + 2 sharing each
// B stage), A fragments (8 row tiles x KS features of H) in registers; B
// stages in a 2-deep LDS ring filled by global_load_lds_dwordx4 (source-side
// XOR swizzle -> conflict-free ds_read_b128).  One accumulator chain per 16-row
// tile carries its row sums through the MFMAs and is folded to the LDS row
// accumulator every FOLD columns.  KS = 128 for d_pad % 128 == 0 (the H-only A
// side frees the registers the L fragments held), else 64, or 32.
#include <stdlib.h>

#include <utility>
#include <vector>

#include "common.hpp"

namespace dal {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define AS3 __attribute__((address_space(3)))

constexpr int kSB = 512;       // super block rows

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// One step of a reduce-scatter over the 16 lanes of a DPP row: lanes whose
// select bit is clear keep v[k] (k < H) summed with their partner's, lanes
// whose bit is set keep v[k + H]; CTRL is a DPP permutation pairing each lane
// with a lane of the opposite bit (row_mirror, row_half_mirror, quad swaps).
template <int H, int CTRL, int N = 32>
__device__ __forceinline__ void rs_step(float (&v)[N], bool hi) {
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
  if constexpr (N >= 16) {
    rs_step<N / 2, 0x140, N>(v, li & 8);
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k)
      v[k] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[k]), 0x140, 0xF,
                                                                   0xF, false));
  }
  rs_step<N >= 16 ? 4 : N / 2, 0x141, N>(v, li & 4);
  rs_step<N >= 16 ? 2 : N / 4, 0x4E, N>(v, li & 2);
  rs_step<N >= 16 ? 1 : N / 8, 0xB1, N>(v, li & 1);
}

// Lane id recomputed at the point of use (asm volatile: never hoisted out of
// a loop), so lane-derived addresses are rematerialised instead of occupying
// VGPRs across the pair loop (a spill reload's vmcnt wait would drain the DMA).
__device__ __forceinline__ unsigned fresh_lane() {
  unsigned v;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
  return v;
}

#ifndef DAL_GRAM_PRIO8
#define DAL_GRAM_PRIO8 1  // 8-wave kernel: s_setprio 1 for waves 4-7 (> 0) or 0-3 (< 0)
#endif
#ifndef DAL_GRAM_KS64_OCC
#define DAL_GRAM_KS64_OCC 4  // KS 64: 4-wave blocks per CU (3: 16 KiB stages, 100k x 64 -3.2 % vs 2; row sums only, 128 VGPRs: 4 blocks on 8 KiB stages 100k x 64 -0.7 %, 200k x 64 -0.5 % vs 3)
#endif
#ifndef DAL_GRAM_NCH128
// row-sum chains per row tile at KS 128 (240 VGPRs, no spill; KS <= 64 keep 1).
// Two chains fold every 256 columns (once per pair) at the chain length one
// chain has folding every 128: the same density bound, half the folds
// (2M x 256 1190.7 -> 1173.4 ms, 1M x 128 -2.6 %, 200k x 256 -1.8 %; one
// chain with the 256-column fold -- a bound twice as wide -- 1169.7 ms)
#define DAL_GRAM_NCH128 2
#endif
#ifndef DAL_GRAM_FOLD64
#define DAL_GRAM_FOLD64 256  // columns per row fold at KS <= 64
#endif
#ifndef DAL_GRAM_FOLD128
#define DAL_GRAM_FOLD128 256  // columns per row fold at KS 128 (<= 256: a fold never spans two pairs)
#endif
#ifndef DAL_GRAM_STAGE8
#define DAL_GRAM_STAGE8 32768  // bytes per LDS stage of the 8-wave kernel (65536: 2M x 256 1149.6 -> 1378.3 ms)
#endif
#ifndef DAL_GRAM_CHAIN_MAX
#define DAL_GRAM_CHAIN_MAX 2048  // the longest row chain dal_density_error_bound_sym_d charges
#endif
#ifndef DAL_GRAM_W8_KS64
#define DAL_GRAM_W8_KS64 0  // KS 64 in the 8-wave two-super-block form (round robin schedule only)
#endif
#ifndef DAL_GRAM_W8_OCC64
#define DAL_GRAM_W8_OCC64 1  // 8-wave KS-64 blocks per CU (128 VGPRs, 72 KiB of LDS: two fit)
#endif
#ifndef DAL_GRAM_KS32_OCC
#define DAL_GRAM_KS32_OCC 5  // KS 32: 4-wave blocks per CU (3: 16 KiB stages; >= 4: 8 KiB stages. Config 3: 2 -> 3 -> 4 blocks 3.944 -> 3.827 -> 3.745 ms; row sums only (94 VGPRs): 4 -> 5 blocks 3.430 -> 3.391 ms)
#endif
template <int KS, int W = 4>
struct Cfg {
  static constexpr int WAVES = W;                   // 4: one super block per block; 8: two (P, P + 2)
  static constexpr int HALVES = W / 4;              // super blocks per block
  static constexpr int NT = 64 * W;                 // threads
  static constexpr int ROWB = KS * 4;               // bytes per operand row of a slice (H + L)
  static constexpr int SLOTS = ROWB / 16;           // 16-B slots per row
  static constexpr int HI = KS / 8;                 // slots of the H part
  // three 4-wave blocks per CU at KS 64 (OCC3): 16 KiB stages so three fit the LDS
  static constexpr int OCC = W == 8 ? (KS == 64 ? DAL_GRAM_W8_OCC64 : 1)
                                    : KS == 32 ? DAL_GRAM_KS32_OCC : KS == 64 ? DAL_GRAM_KS64_OCC : 2;
  static constexpr int STAGE = W == 8 ? DAL_GRAM_STAGE8 : OCC >= 4 ? 8192 : OCC == 3 ? 16384 : 32768;  // bytes per LDS stage
  static constexpr int SC = STAGE / ROWB;           // columns per stage: 64 / 128 / 256
  static constexpr int SPP = 256 / SC;              // stages per 512 x 256 pair: 4 / 2 / 1
  static constexpr int FOLD = KS == 128 ? DAL_GRAM_FOLD128 : DAL_GRAM_FOLD64;  // columns per row fold
  static constexpr int SPF = FOLD / SC;             // stages per fold group
  static constexpr int F4 = STAGE / 16;
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = STAGE / (W * 1024);  // 1-KiB DMA pieces per wave per stage
  static constexpr int RT = 8;                      // 16-row tiles per wave (128 rows)
  static constexpr int LG = 4;
  static constexpr int NKS = KS / 32;               // k-steps of v_mfma_f32_16x16x32_f16
  static constexpr int NCT = SC / 16;               // column tiles per stage
  // row-sum chains per row tile (column tiles dealt round-robin; 2 halve the
  // chain length -- a tighter density bound -- for 32 more VGPRs)
  static constexpr int NCH = KS == 128 ? DAL_GRAM_NCH128 : 1;
  // products summed by one row-chain element between two folds (the FOLD
  // columns' tiles over NCH chains, 2 KS products per tile): the length
  // dal_density_error_bound_sym_d charges the row side with
  static constexpr int CHAIN = FOLD / 16 / NCH * 2 * KS;
  static_assert(SPF >= 1 && SPP % SPF == 0 && PIECES >= 1 && NKS >= 1, "bad slice");
  static_assert(W == 4 || (W == 8 && KS >= 64), "two super blocks per block: KS >= 64 only");
  static_assert(CHAIN <= DAL_GRAM_CHAIN_MAX, "row chain longer than the density bound's worst case");
};
// the 8-wave form folds like the 4-wave one (one bound per KS)
static_assert(Cfg<128, 8>::CHAIN == Cfg<128, 4>::CHAIN, "block forms must share the chain length");

// Row sums of the taken pairs (the column sums of every pair are added in
// closed form by dal_gram_sym_residual, see the header): for each pair (P,
// J) the taker's rows accumulate <H_i, u~_j> over J's 256 columns.
template <int KS, int W>
__global__ __launch_bounds__(64 * W, (Cfg<KS, W>::OCC)) void gram_csym_kernel(
    const uint16_t* __restrict__ urows, int srow0, int n_srb,
    const uint16_t* __restrict__ ucols, int jcol0, int j_lo, int j_hi, int skip_lo, int skip_hi,
    int ns_active, int64_t ldh, int slice_off, int chunk_j, int n_chunks,
    unsigned long long* __restrict__ acc_out, int contig) {
  using C = Cfg<KS, W>;
  constexpr int HV = C::HALVES;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * C::F4];
  __shared__ double rowacc[HV * kSB];

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int half = wave >> 2, wave4 = wave & 3;  // the block's super block of this wave, wave within it
  // 8-wave block: the two waves of a SIMD (w, w + 4) run the same program in
  // lockstep; a static priority for one half settles their VALU arbitration
  // once instead of by age at every segment (MI355X_MICROARCH.md, two waves per
  // SIMD): waves 4-7 at priority 1, 2M x 256 1266.9 -> 1262.3 ms (waves 0-3:
  // 1265.0; deferring waves 4-7's last column epilogue of each stage into the
  // next one, a stagger, 1274.5)
  if constexpr (W == 8 && DAL_GRAM_PRIO8 != 0) {
    if (DAL_GRAM_PRIO8 > 0 ? half == 1 : half == 0) __builtin_amdgcn_s_setprio(1);
  }
  const int li = lane & 15, lq = lane >> 4;
  const int G = gridDim.x, g = blockIdx.x;
  for (int e = tid; e < HV * kSB; e += C::NT) rowacc[e] = 0.0;

  // Work = the pairs (P, J) over row super blocks P and 256-column blocks J in
  // [j_lo, j_hi) minus [skip_lo, skip_hi), as segments (row unit, raw column
  // range [rlo, rhi)) walked by a raw column cursor r (J = jmap(r)).  A row
  // unit is one super block (W = 4) or two of the same parity, P and P + 2
  // (W = 8: they take the same column blocks but near the diagonal, so one
  // B stage feeds both; a half whose super block does not take J idles):
  //  contig: block g owns the g-th 1/G of the unit-major raw grid (W = 4 only);
  //  chunk:  unit u = (row unit u % n_ru, column chunk u / n_ru), dealt round-robin
  //          (all blocks sweep the same column chunks together: L2 / MALL reuse).
  const int n_ru = HV == 1 ? n_srb : 2 * ((n_srb + 3) / 4);
  auto rowP = [&](int ru, int h) { return HV == 1 ? srow0 + ru : srow0 + 4 * (ru >> 1) + (ru & 1) + 2 * h; };
  auto live = [&](int P) { return P < srow0 + n_srb && P < ns_active; };
  const int sk_lo = skip_lo > j_lo ? skip_lo : j_lo, sk_hi = skip_hi < j_hi ? skip_hi : j_hi;
  const int skl = contig && sk_hi > sk_lo ? sk_hi - sk_lo : 0;  // chunk mode skips through takes()
  const int nje = j_hi - j_lo - skl;
  const int nre0 = ns_active - srow0, nre = nre0 < n_srb ? (nre0 > 0 ? nre0 : 0) : n_srb;
  const int64_t raw = static_cast<int64_t>(nre) * nje;
  const int64_t ka = raw * g / G, kb = raw * (g + 1) / G;
  const int n_seg = contig ? (kb > ka ? static_cast<int>((kb - 1) / nje - ka / nje) + 1 : 0) : n_ru * n_chunks;
  const int seg_step = contig ? 1 : G;
  auto seg_ru = [&](int u) { return contig ? static_cast<int>(ka / nje) + u : u % n_ru; };
  auto seg_rlo = [&](int u) { return contig ? (u == 0 ? static_cast<int>(ka % nje) : 0) : (u / n_ru) * chunk_j; };
  auto seg_rhi = [&](int u) {
    if (contig) return u == n_seg - 1 ? static_cast<int>((kb - 1) % nje) + 1 : nje;
    const int e = (u / n_ru + 1) * chunk_j;
    return e < nje ? e : nje;
  };
  auto jmap = [&](int r) { return j_lo + r + (j_lo + r >= sk_lo ? skl : 0); };
  auto takes = [&](int P, int J) -> bool {
    const int Q = J >> 1;
    if (J >= skip_lo && J < skip_hi) return false;
    return Q == P || (Q > P && ((P + Q) & 1) == 0) || (Q < P && ((P + Q) & 1));
  };
  // the unit's super block h takes J (and exists)
  auto takes_h = [&](int ru, int h, int J) { return live(rowP(ru, h)) && takes(rowP(ru, h), J); };
  auto takes_u = [&](int ru, int J) { return takes_h(ru, 0, J) || (HV == 2 && takes_h(ru, HV - 1, J)); };
  auto first_r = [&](int ru, int r, int rhi) -> int {
    if constexpr (HV == 1) {
      const int P = srow0 + ru;
      if (P >= ns_active) return -1;
      while (r < rhi && !takes(P, jmap(r))) ++r;
    } else {
      if (!live(rowP(ru, 0))) return -1;
      while (r < rhi && !takes_u(ru, jmap(r))) ++r;
    }
    return r < rhi ? r : -1;
  };
  auto seek = [&](int u, int& r) {
    while (u < n_seg) {
      r = first_r(seg_ru(u), seg_rlo(u), seg_rhi(u));
      if (r >= 0) break;
      u += seg_step;
    }
    return u;
  };

  // DMA source offsets.  Piece q of wave w covers stage rows
  // Wr + q * RPP + lane / SLOTS (Wr = w * PIECES * RPP, RPP = 64 / SLOTS rows
  // per piece), slot (lane % SLOTS) ^ (row & SWZ).  Wr (a multiple of
  // PIECES * RPP), q * RPP and lane / SLOTS occupy disjoint bits, so row & SWZ
  // = ((Wr + lane / SLOTS) & SWZ) ^ ((q * RPP) & SWZ): the offset is a per-lane
  // value XOR a per-piece constant (bits 4.. of the byte offset, below the row
  // part) plus the piece's row offset.
  constexpr int RPP = 64 / C::SLOTS;
  const unsigned rowbytes = static_cast<unsigned>(ldh * 2);
  const unsigned dst0 = __builtin_amdgcn_readfirstlane(
      static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + wave * C::PIECES * 64))));
  // stage h of 256-column block J into LDS buffer buf.  Inline asm so the
  // compiler does not track the DMA on vmcnt (block_sync waits for it).
  auto issue = [&](int buf, int J, int h) {
    const char* sbase = reinterpret_cast<const char*>(
        ucols + (static_cast<int64_t>(J - jcol0) * 256 + h * C::SC) * ldh + slice_off);
    const unsigned fl = fresh_lane();
    const unsigned lrow = fl / C::SLOTS + static_cast<unsigned>(wave * C::PIECES * RPP);
    const unsigned vlane = lrow * rowbytes + (((fl % C::SLOTS) ^ (lrow & C::SWZ)) << 4);
#pragma unroll
    for (int q = 0; q < C::PIECES; ++q) {
      const unsigned dst = dst0 + static_cast<unsigned>(buf * C::STAGE + q * 1024);
      const unsigned voff = (vlane ^ (static_cast<unsigned>((q * RPP) & C::SWZ) << 4)) +
                            static_cast<unsigned>(q * RPP) * rowbytes;
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff), "s"(dst), "s"(sbase)
          : "memory");
    }
  };

  // resident A fragments: H of rows P*512 + wave4*128 + rt*16 + (lane & 15)
  // (P = this wave's super block of the unit), features of k-step c and lane
  // group lq
  f16x8 ah[C::RT][C::NKS];
  auto load_a = [&](int ru) {
    const int P = rowP(ru, half);
    if (HV > 1 && !live(P)) return;  // (this half idles for the unit)
    const uint16_t* pb = urows + static_cast<int64_t>(P - srow0) * kSB * ldh + slice_off;
    const unsigned fl = fresh_lane();
    const unsigned lrow = static_cast<unsigned>((wave4 * 128 + (fl & 15)) * ldh + (fl >> 4) * 8);
    const unsigned tstep = static_cast<unsigned>(16 * ldh);
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int c = 0; c < C::NKS; ++c)  // read once per unit: keep the column stages resident in L2
        ah[rt][c] = __builtin_nontemporal_load(reinterpret_cast<const f16x8*>(pb + lrow + rt * tstep + c * C::LG * 8));
  };
  constexpr float kFold = 0x1p8f;  // units of 2^-24 -> multiples of 2^-32

  // B-fragment LDS offsets (float4 units): slot (k + lq) ^ (li & SWZ) of
  // column row li, k = c*LG (+ HI for the L half) a multiple of 4; the XOR
  // splits into a lane part (low 2 bits) and a k part (k ^ (li & SWZ & ~3)),
  // so two registers cover every k-step and half
  const int b_base = li * C::SLOTS + (lq ^ (li & 3));
  const int b_swz = li & C::SWZ & ~3;
  auto b_off = [&](int c, bool lo_half) { return b_base + ((c * C::LG + (lo_half ? C::HI : 0)) ^ b_swz); };

  f32x4 mc[C::NCH][C::RT];
  // one stage of SC columns; fresh = first stage of a fold group (the chains
  // restart).  B fragments go through two register sets: k-step i+1's are
  // read while k-step i's 16 MFMAs issue.
  auto compute = [&](int buf, bool fresh_stage) {
    f16x8 bh[2], bl[2];
    auto load_b = [&](int set, int c, int ct) {
      bh[set] = __builtin_bit_cast(f16x8, lds[buf * C::F4 + ct * 16 * C::SLOTS + b_off(c, false)]);
      bl[set] = __builtin_bit_cast(f16x8, lds[buf * C::F4 + ct * 16 * C::SLOTS + b_off(c, true)]);
    };
    load_b(0, 0, 0);
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      __builtin_amdgcn_sched_barrier(0);
      const bool fresh = fresh_stage && ct < C::NCH;
      const int ch = ct % C::NCH;
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        const int i = ct * C::NKS + c, cur = i & 1;
        if (c + 1 < C::NKS)
          load_b(cur ^ 1, c + 1, ct);
        else if (ct + 1 < C::NCT)
          load_b(cur ^ 1, 0, ct + 1);
        const f32x4 zero = {};
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt)
          mc[ch][rt] = mfma16(ah[rt][c], bh[cur], (c == 0 && fresh) ? zero : mc[ch][rt]);
#pragma unroll
        for (int rt = 0; rt < C::RT; ++rt) mc[ch][rt] = mfma16(ah[rt][c], bl[cur], mc[ch][rt]);
      }
      constexpr int NM = 2 * C::RT;  // MFMAs per k-step
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // next k-step's B
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);  // MFMA
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // chains -> LDS row accumulator (exact integer fp64 adds).  A 4-step DPP
  // reduce-scatter over the 16 column lanes leaves each lane 2 fully summed
  // rows, added by all 64 lanes at distinct LDS addresses.
  auto fold_rows = [&]() {
    float v[32];
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[rt * 4 + q] = C::NCH == 1 ? mc[0][rt][q] : mc[0][rt][q] + mc[C::NCH - 1][rt][q];
    rs_step<16, 0x140>(v, li & 8);  // row_mirror: lane i <-> 15 - i
    rs_step<8, 0x141>(v, li & 4);   // row_half_mirror: i <-> i ^ 7
    rs_step<4, 0x4E>(v, li & 2);    // quad_perm [2,3,0,1]
    rs_step<2, 0xB1>(v, li & 1);    // quad_perm [1,0,3,2]
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
  auto flush_rows = [&](int ru) {  // rowacc[h * 512 + r] -> row r of the unit's super block h
    for (int e = tid; e < HV * kSB; e += C::NT) {
      const int P = rowP(ru, e / kSB);
      if (live(P)) flush_one(rowacc[e], static_cast<int64_t>(P) * kSB + e % kSB);
    }
  };
  // every barrier waits for this wave's LDS adds and DMA first (hipcc may
  // omit the lgkmcnt wait at a loop-top barrier after no-return LDS adds)
  auto block_sync = [&]() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  };
  auto stage_sync = [&]() { block_sync(); };

  int r = -1;
  int unit = seek(contig ? 0 : g, r);
  if (unit >= n_seg) return;
  int ru = seg_ru(unit), rhi_u = seg_rhi(unit);
  int J = jmap(r);
  issue(0, J, 0);
  load_a(ru);
  int buf = 0;       // LDS stage buffer of the next stage to compute
  int flushRU = -1;  // row unit whose sums wait in rowacc

  while (true) {
    int nr = first_r(ru, r + 1, rhi_u), n_unit = unit;
    if (nr < 0) n_unit = seek(unit + seg_step, nr);
    const bool has_next = n_unit < n_seg;
    const int nru = has_next ? seg_ru(n_unit) : -1;
    const bool new_rows = nru != ru;
    const int nJ = has_next ? jmap(nr) : -1;
    // this wave's super block takes J?  (a half whose super block does not idles)
    const bool act = HV == 1 || takes_h(ru, half, J);

#pragma unroll
    for (int s = 0; s < C::SPP; ++s) {
      stage_sync();
      if (s == 0 && flushRU >= 0) {
        flush_rows(flushRU);
        flushRU = -1;
      }
      if (s + 1 < C::SPP) {
        issue(buf ^ 1, J, s + 1);
      } else if (has_next) {
        issue(buf ^ 1, nJ, 0);
      }
      if (act) {  // (wave-uniform)
        compute(buf, s % C::SPF == 0);
        if (s % C::SPF == C::SPF - 1) fold_rows();
      }
      buf ^= 1;
    }

    if (new_rows) flushRU = ru;
    if (!has_next) break;
    unit = n_unit;
    rhi_u = seg_rhi(unit);
    if (new_rows) {
      ru = nru;
      load_a(ru);
    }
    r = nr;
    J = nJ;
  }
  block_sync();
  if (flushRU >= 0) flush_rows(flushRU);
}
// ---------------------------------------------------------------------------
// Residual of the compensation (see the header).  Three launches:
//  1. per super block Q: sigma~_Q and sigma^L_Q, exact int64 in units of 2^-24
//     (every H and L is a multiple of 2^-24 below 2^13);
//  2. per feature: exclusive prefix sums over super blocks of each parity
//     class and their totals, giving R_B and C_B for every requested B (for
//     d_pad <= 64 and few super blocks the launch-3 blocks form their own R_B,
//     C_B from sigma~ instead: one launch less, 21 us at configs 2 and 3);
//  3. per row r of the requested super blocks: acc[r] += rint(2^8 *
//     (<L_r, R_B> + <u~_r, C_B>)) with the dots in fp64 in a fixed order.

// One block per (super block, group of 256 16-byte chunk columns): the
// super block's 512 operand rows are 512 x CPR 16-byte chunks (CPR = ldh / 8
// per row: the H and L halves of every slice); thread t always reads chunk
// column t % CPR (8 H or 8 L halves of one slice) of rows t / CPR, + 256 /
// CPR, ... -- independent 16-B loads, 8 in flight -- summed exactly in int64,
// then reduced over the threads of the same column in LDS.
__global__ __launch_bounds__(256) void csym_sigma_kernel(const uint16_t* __restrict__ ops, int64_t ldh, int ks,
                                                         int d_pad, long long* __restrict__ sig_u) {
  __shared__ long long red[256][9];  // [thread][8 halves] (+1: bank spread)
  const int Q = blockIdx.x;
  const int cpr = static_cast<int>(ldh / 8);      // chunks per row
  const int cols = cpr < 256 ? cpr : 256;          // chunk columns of this block
  const int col = blockIdx.y * 256 + threadIdx.x % cols;
  const int rstep = 256 / cols;                    // rows advanced per round
  const int r0 = threadIdx.x / cols;
  // this block's rows of the super block: [rb, re) (gridDim.z row slices)
  const int rb = kSB * static_cast<int>(blockIdx.z) / static_cast<int>(gridDim.z);
  const int re = kSB * (static_cast<int>(blockIdx.z) + 1) / static_cast<int>(gridDim.z);
  // Summed in fp64, exactly: every term is a multiple of 2^-24 below 2^13 and
  // a thread adds at most kSB of them (< 2^22), so every partial sum has at
  // most 46 significant bits; converted to int64 units once at the end.
  double acc[8] = {};
  if (col < cpr && r0 < rstep) {
    const uint4* base = reinterpret_cast<const uint4*>(ops + static_cast<int64_t>(Q) * kSB * ldh) + col;
    for (int r = rb + r0; r < re; r += 8 * rstep) {
      uint4 q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = r + j * rstep < re ? base[static_cast<int64_t>(r + j * rstep) * cpr] : uint4{};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w[4] = {q[j].x, q[j].y, q[j].z, q[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += static_cast<double>(
              static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(w[e] & 0xFFFFu))));
          acc[2 * e + 1] += static_cast<double>(
              static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(w[e] >> 16))));
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = static_cast<long long>(acc[e] * 16777216.0);
  __syncthreads();
  // thread t < cols finishes chunk column t: sum over the rstep row phases
  if (threadIdx.x < cols && col < cpr) {
    long long v[8] = {};
    for (int p = 0; p < rstep; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += red[p * cols + threadIdx.x][e];
    // chunk column -> (slice, half, first feature): the row is [slice][H KS | L KS]
    const int hpc = ks / 8;                        // chunks per half of a slice
    const int slice = col / (2 * hpc), within = col % (2 * hpc);
    const int f0 = slice * ks + (within % hpc) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t o = static_cast<int64_t>(Q) * d_pad + f0 + e;
      atomicAdd(reinterpret_cast<unsigned long long*>(sig_u + o), static_cast<unsigned long long>(v[e]));
    }
  }
}

// block = 8 waves; lane = one of 64 features (blockIdx.x * 64 + lane), wave w
// owns super blocks [w*ns/8, (w+1)*ns/8).  R_B, C_B written as fp64 for B in
// [b0, b1).
#ifndef DAL_CSYM_SCAN_WAVES
#define DAL_CSYM_SCAN_WAVES 16
#endif
constexpr int kScanWaves = DAL_CSYM_SCAN_WAVES;  // super-block ranges per feature (one wave each)
constexpr int kScanBatch = 16;                   // sigma~ loads in flight per thread
#ifndef DAL_CSYM_FUSED_MAX
#define DAL_CSYM_FUSED_MAX 65536  // super blocks x d_pad up to which the residual blocks skip the scan
#endif
__global__ __launch_bounds__(64 * kScanWaves) void csym_scan_kernel(const long long* __restrict__ sig_u, int ns,
                                                                    int d_pad, int b0, int b1,
                                                                    double* __restrict__ rb, double* __restrict__ cb) {
  constexpr int kW = kScanWaves;
  __shared__ long long part[kW][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + lane;
  const bool live = f < d_pad;
  const int q0 = static_cast<int>(static_cast<int64_t>(ns) * w / kW);
  const int q1 = static_cast<int>(static_cast<int64_t>(ns) * (w + 1) / kW);
  // u~ sums per parity class of the super block (even, odd); named
  // registers, not arrays indexed by q & 1 (those would live in scratch)
  // loads in batches of kScanBatch, all in flight before the adds (a wave walks
  // ns / kW super blocks: 244 at config 4)
  long long ue = 0, uo = 0;
  if (live) {
    for (int qb = q0; qb < q1; qb += kScanBatch) {
      long long v[kScanBatch];
#pragma unroll
      for (int j = 0; j < kScanBatch; ++j)
        v[j] = qb + j < q1 ? sig_u[static_cast<int64_t>(qb + j) * d_pad + f] : 0;
#pragma unroll
      for (int j = 0; j < kScanBatch; ++j) {
        const bool odd = (qb + j) & 1;
        ue += odd ? 0 : v[j];
        uo += odd ? v[j] : 0;
      }
    }
  }
  part[w][0][lane] = ue;
  part[w][1][lane] = uo;
  __syncthreads();
  // exclusive prefix over the earlier waves' ranges, and the totals
  long long eue = 0, euo = 0, tue = 0, tuo = 0;
  for (int v = 0; v < kW; ++v) {
    const long long a0 = part[v][0][lane], a1 = part[v][1][lane];
    if (v < w) {
      eue += a0;
      euo += a1;
    }
    tue += a0;
    tuo += a1;
  }
  if (!live) return;
  for (int qb = q0; qb < q1; qb += kScanBatch) {
    long long v[kScanBatch];
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j)
      v[j] = qb + j < q1 ? sig_u[static_cast<int64_t>(qb + j) * d_pad + f] : 0;
#pragma unroll
    for (int j = 0; j < kScanBatch; ++j) {
      const int q = qb + j;
      // e* = exclusive prefix (super blocks < q) per class; b = q's class
      const bool odd = q & 1;
      if (q < q1 && q >= b0 && q < b1) {
        // R_B = sum_{Q >= B, same class} + sum_{Q < B, other class} of sigma~
        // (the super blocks B takes); C_B = sum_{P < B, same class} + sum_{P >
        // B, other class} of sigma~ (the other super blocks that take B: their
        // pairs' column sums for B's rows)
        const long long R = odd ? (tuo - euo + eue) : (tue - eue + euo);
        const long long Cc = odd ? (euo + tue - eue) : (eue + tuo - euo);
        rb[static_cast<int64_t>(q - b0) * d_pad + f] = static_cast<double>(R);
        cb[static_cast<int64_t>(q - b0) * d_pad + f] = static_cast<double>(Cc);
      }
      eue += odd ? 0 : v[j];
      euo += odd ? v[j] : 0;
    }
  }
}

// One thread per row: a block's 256 rows lie in one super block B, whose R_B
// and C_B are staged in LDS once; each thread sums its row's features in
// order, t = t + l_f R_f, t = t + (h_f + l_f) C_f for f = 0, 1, ... (fp64, no
// FMA) -- a fixed order, so the bits are the same on every GPU count.  rows:
// the operand of the requested super blocks.  The rows reach the threads
// through LDS, kResFeat features at a time: the block reads each row's H and L
// runs of those features with coalesced 16-B loads (consecutive threads,
// consecutive chunks of one row), so every fetched line is used at once.
// (Round 5 before: each thread read its own row 16 B at a time, 64 rows one
// ldh apart per wave instruction -- the lines left L2 before their other
// chunks were read, 2.2 ms for config 4's 2 GB operand.  Round 4: one wave per
// row, lanes over features and a butterfly -- 2-byte loads.)
constexpr int kResRows = 256;
constexpr int kResFeat = 32;                 // features per LDS stage (divides every KS)
constexpr int kResQ = kResFeat / 4;          // 16-B chunks per row per stage: H kResFeat/8, L kResFeat/8
constexpr int kResLd = kResQ + 1;            // LDS row stride in 16-B chunks (+1: the threads' rows spread over the banks)
// kMode kResFused (d_pad 32 or 64, few super blocks): no scan launch -- every
// block forms its own R_B and C_B from sigma~ (256 / d_pad thread groups over
// the super blocks, exact int64 sums reduced in LDS; the same integers as the
// scan's).  kResStaged: the scan's R_B, C_B staged in LDS (16 d_pad bytes).
// kResGlobal (d_pad > kResLdsMaxFeat, where they would not fit beside the
// tile): read in place from the scan's output, uniform addresses.
constexpr int kResStaged = 0, kResFused = 1, kResGlobal = 2;
constexpr int kResLdsMaxFeat = 1024;  // 16 KiB of R_B | C_B + the 36 KiB tile: within 64 KiB per block
template <int kMode>
__global__ __launch_bounds__(kResRows) void csym_residual_kernel(const uint16_t* __restrict__ rows, int64_t ldh, int ks,
                                                                 int d_pad, int b0, int n_rows,
                                                                 const double* __restrict__ rb,
                                                                 const double* __restrict__ cb,
                                                                 const long long* __restrict__ sig_u, int ns,
                                                                 long long* __restrict__ acc) {
  extern __shared__ double rc[];  // [d_pad] R_B | [d_pad] C_B
  __shared__ uint4 tile[kResRows * kResLd];
  const int tid = threadIdx.x;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kResRows;  // (a multiple of 256: one super block)
  const int64_t B = r0 / kSB;                                       // relative to b0
  if constexpr (kMode == kResFused) {
    // feature pairs (16-B loads of sigma~): 256 / (d_pad / 2) thread groups
    // over the super blocks -- 8 (d_pad 64) or 16 (d_pad 32)
    __shared__ long long red[8][kResRows];
    const int qB = b0 + static_cast<int>(B);  // this block's super block
    const int hp = d_pad / 2, G = kResRows / hp, fp = tid % hp, grp = tid / hp;
    long long pe[2] = {}, po[2] = {}, te[2] = {}, to[2] = {};  // per class: sums over super blocks < qB, and totals
    const longlong2* su2 = reinterpret_cast<const longlong2*>(sig_u);
    for (int qb = grp; qb < ns; qb += kScanBatch * G) {
      longlong2 v[kScanBatch];
#pragma unroll
      for (int j = 0; j < kScanBatch; ++j) {
        const int q = qb + j * G;
        v[j] = q < ns ? su2[static_cast<int64_t>(q) * hp + fp] : longlong2{0, 0};
      }
#pragma unroll
      for (int j = 0; j < kScanBatch; ++j) {
        const int q = qb + j * G;
        const bool odd = q & 1, before = q < qB;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const long long x = c ? v[j].y : v[j].x;
          te[c] += odd ? 0 : x;
          to[c] += odd ? x : 0;
          pe[c] += before && !odd ? x : 0;
          po[c] += before && odd ? x : 0;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      red[4 * c][tid] = pe[c];
      red[4 * c + 1][tid] = po[c];
      red[4 * c + 2][tid] = te[c];
      red[4 * c + 3][tid] = to[c];
    }
    __syncthreads();
    if (tid < hp) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        long long eue = 0, euo = 0, tue = 0, tuo = 0;
        for (int g = 0; g < G; ++g) {
          eue += red[4 * c][g * hp + tid];
          euo += red[4 * c + 1][g * hp + tid];
          tue += red[4 * c + 2][g * hp + tid];
          tuo += red[4 * c + 3][g * hp + tid];
        }
        const bool odd = qB & 1;  // R_B, C_B as in csym_scan_kernel
        const int f = 2 * tid + c;
        rc[f] = static_cast<double>(odd ? (tuo - euo + eue) : (tue - eue + euo));
        rc[d_pad + f] = static_cast<double>(odd ? (euo + tue - eue) : (eue + tuo - euo));
      }
    }
  } else if constexpr (kMode == kResStaged) {
    for (int f = tid; f < d_pad; f += kResRows) {
      rc[f] = rb[B * d_pad + f];
      rc[d_pad + f] = cb[B * d_pad + f];
    }
  }
  const double* __restrict__ Rv = kMode == kResGlobal ? rb + B * d_pad : rc;
  const double* __restrict__ Cv = kMode == kResGlobal ? cb + B * d_pad : rc + d_pad;
  const int live_rows = n_rows - r0 < kResRows ? static_cast<int>(n_rows - r0) : kResRows;
  const uint16_t* blk = rows + r0 * ldh;
  double t = 0.0;
  for (int f0 = 0; f0 < d_pad; f0 += kResFeat) {
    // the stage's H run starts at halves (f0 / ks) * 2 ks + f0 % ks, its L run ks later
    const int64_t hoff = static_cast<int64_t>(f0 / ks) * 2 * ks + f0 % ks;
    uint4 q[kResQ];
#pragma unroll
    for (int j = 0; j < kResQ; ++j) {
      const int e = tid + kResRows * j;
      const int r = e / kResQ, c = e % kResQ;  // row of the block, chunk of the stage (H first, then L)
      const int64_t off = r * ldh + hoff + (c < kResQ / 2 ? c * 8 : ks + (c - kResQ / 2) * 8);
      q[j] = r < live_rows ? *reinterpret_cast<const uint4*>(blk + off) : uint4{};
    }
    if (f0) __syncthreads();  // the previous stage's tile is consumed
#pragma unroll
    for (int j = 0; j < kResQ; ++j) {
      const int e = tid + kResRows * j;
      tile[(e / kResQ) * kResLd + e % kResQ] = q[j];
    }
    __syncthreads();
    if (tid < live_rows) {
#pragma unroll
      for (int c = 0; c < kResQ / 2; ++c) {
        const uint4 hq = tile[tid * kResLd + c], lq = tile[tid * kResLd + kResQ / 2 + c];
        const uint32_t hw[4] = {hq.x, hq.y, hq.z, hq.w}, lw[4] = {lq.x, lq.y, lq.z, lq.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int f = f0 + c * 8 + e;
          const uint16_t hb = static_cast<uint16_t>(e & 1 ? hw[e >> 1] >> 16 : hw[e >> 1] & 0xFFFFu);
          const uint16_t lb = static_cast<uint16_t>(e & 1 ? lw[e >> 1] >> 16 : lw[e >> 1] & 0xFFFFu);
          const double h = static_cast<double>(static_cast<float>(__builtin_bit_cast(_Float16, hb)));
          const double l = static_cast<double>(static_cast<float>(__builtin_bit_cast(_Float16, lb)));
          t = t + l * Rv[f];
          t = t + (h + l) * Cv[f];
        }
      }
    }
  }
  // R, C in units of 2^-24 x (split units); value = t * 2^-24 * 2^-24 ... in
  // fixed point (2^32): t * 2^-24 (operand units^2 = 2^24 x value) * 2^8
  if (tid < live_rows && t != 0.0)
    acc[static_cast<int64_t>(b0) * kSB + r0 + tid] += static_cast<long long>(__builtin_rint(t * 0x1p-16));
}

// ---------------------------------------------------------------------------
int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
  return cus;
}

// Number of column blocks J in [lo, hi) that super block I takes (O(1)).
inline int64_t sb_pairs(int64_t I, int64_t lo, int64_t hi) {
  auto same_parity = [](int64_t a, int64_t b, int64_t p) -> int64_t {
    if (b <= a) return 0;
    return (b - p + 1) / 2 - (a - p + 1) / 2;
  };
  int64_t n = (lo <= I && I < hi) ? 1 : 0;
  n += same_parity(lo > I + 1 ? lo : I + 1, hi, I & 1);
  n += same_parity(lo, hi < I ? hi : I, (I & 1) ^ 1);
  return n;
}

// Pairs (P, J) for row super block P over 256-column blocks [a, b).
inline int64_t pairs_range(int64_t P, int64_t a, int64_t b) {
  if (b <= a) return 0;
  auto takes = [P](int64_t Q) { return Q == P || (Q > P && ((P + Q) & 1) == 0) || (Q < P && ((P + Q) & 1)); };
  const int64_t qa = a >> 1, qb = (b - 1) >> 1;
  int64_t n = 2 * sb_pairs(P, qa, qb + 1);
  if ((a & 1) && takes(qa)) --n;
  if (!((b - 1) & 1) && takes(qb)) --n;
  return n;
}
inline int64_t pairs_skip(int64_t P, int64_t a, int64_t b, int64_t skip_lo, int64_t skip_hi) {
  const int64_t sa = a > skip_lo ? a : skip_lo, sb = b < skip_hi ? b : skip_hi;
  return pairs_range(P, a, b) - pairs_range(P, sa, sb);
}

// Column-chunk count for the round-robin units: the fewest chunks, at least
// min_chunks, whose most loaded block has at most 8 % more pairs than the best
// balance found (exact pair counts; cached per shape).  More chunks = a
// smaller column working set swept by every block together (MALL hits; 2M x
// 256: 16 chunks 3.9 % faster than 1; 4 and 8: 0.6 % slower), fewer = fewer A
// loads and row flushes.  KS 64 with a column operand of <= DAL_GRAM_SMALL_MB
// (in L2 + MALL whole) takes >= 2 chunks instead of the contiguous schedule:
// 100k x 64 (25.6 MB) 1.6-4.7 % faster in two of three same-process runs
// (+0.7 % in the third), the clock 1.83 -> 1.88-1.92 GHz; at KS 32 and 128 the
// same change lost (60k x 32 +7.4 %, 20k x 256 +4.3 %; round 6,
// profiles/r06/pmc/clock_ab_chunk_counts.txt).
#ifndef DAL_GRAM_MIN_CHUNKS
#define DAL_GRAM_MIN_CHUNKS 16
#endif
#ifndef DAL_GRAM_SMALL_MB
#define DAL_GRAM_SMALL_MB 32
#endif
#ifndef DAL_GRAM_MIN_CHUNKS_SMALL
#define DAL_GRAM_MIN_CHUNKS_SMALL 2
#endif
// hv = super blocks per row unit (gram_csym_kernel W / 4); a two-super-block
// unit costs the pairs of the busier one (they take the same column blocks but
// near the diagonal).
int64_t choose_chunks(int64_t srow0, int64_t n_srb, int64_t lo, int64_t hi, int64_t skip_lo, int64_t skip_hi,
                      int64_t ns_active, int64_t G0, int hv, int64_t kMinChunks) {
  struct Entry {
    int64_t k[10];
    int64_t nc;
  };
  static thread_local Entry cache[8] = {};
  static thread_local int cache_next = 0;
  const int64_t key[10] = {srow0, n_srb, lo, hi, skip_lo, skip_hi, ns_active, G0, hv, kMinChunks};
  for (const Entry& e : cache) {
    bool hit = e.nc > 0;
    for (int i = 0; i < 10 && hit; ++i) hit = e.k[i] == key[i];
    if (hit) return e.nc;
  }
  const int64_t n_ru = hv == 1 ? n_srb : 2 * ceil_div(n_srb, 4);
  auto rowP = [&](int64_t ru, int h) { return hv == 1 ? srow0 + ru : srow0 + 4 * (ru >> 1) + (ru & 1) + 2 * h; };
  const int64_t nj = hi - lo;
  int64_t best_max = -1;
  std::vector<int64_t> load;
  std::vector<std::pair<int64_t, int64_t>> cand;
  int tried = 0;
  // chunk counts from 1 up (from kMinChunks when it is above 16 and the columns allow)
  for (int64_t c = kMinChunks > 16 && nj >= kMinChunks ? kMinChunks : 1; c <= nj && tried < 32; ++c) {
    const int64_t cbk = ceil_div(nj, c), ncc = ceil_div(nj, cbk);
    if (c > 1 && cbk == ceil_div(nj, c - 1)) continue;
    ++tried;
    const int64_t units = n_ru * ncc, G = units < G0 ? units : G0;
    load.assign(static_cast<size_t>(G), 0);
    for (int64_t u = 0; u < units; ++u) {
      const int64_t clo = lo + (u / n_ru) * cbk, chi = clo + cbk < hi ? clo + cbk : hi;
      int64_t w = 0;
      for (int h = 0; h < hv; ++h) {
        const int64_t P = rowP(u % n_ru, h);
        if (P >= ns_active || P >= srow0 + n_srb) continue;
        const int64_t pw = pairs_skip(P, clo, chi, skip_lo, skip_hi);
        w = pw > w ? pw : w;
      }
      load[static_cast<size_t>(u % G)] += w;
    }
    int64_t mx = 0;
    for (int64_t v : load) mx = v > mx ? v : mx;
    cand.emplace_back(ncc, mx);
    if (best_max < 0 || mx < best_max) best_max = mx;
  }
  int64_t best_nc = -1;
  for (int pass = 0; pass < 2 && best_nc < 0; ++pass)
    for (const auto& c : cand)
      if ((pass || c.first >= kMinChunks) && c.second * 100 <= best_max * 108) {
        best_nc = c.first;
        break;
      }
  if (best_nc < 0) best_nc = cand.back().first;
  Entry& e = cache[cache_next];
  cache_next = (cache_next + 1) % 8;
  for (int i = 0; i < 10; ++i) e.k[i] = key[i];
  e.nc = best_nc;
  return best_nc;
}

// Two super blocks per block (8 waves, one block per CU: each B stage feeds
// 1,024 rows, half the L2 -> LDS bytes per flop of the 4-wave form) for the
// round-robin schedule at KS 128.
#ifndef DAL_GRAM_WAVES8
#define DAL_GRAM_WAVES8 1
#endif

template <int KS, int W>
int launch_csym_w(const uint16_t* rows, int64_t srow0, int64_t n_srb, const uint16_t* cols, int64_t jcol0,
                  int64_t j_lo, int64_t j_hi, int64_t skip_lo, int64_t skip_hi, int64_t ns_active, int64_t ldh,
                  int slice_off, int64_t* acc, int grid_blocks, int contig, int64_t min_chunks,
                  hipStream_t stream) {
  // grid_blocks counts 4-wave blocks (two per CU); 8-wave blocks are one per CU
  constexpr int kOcc = Cfg<KS, W>::OCC;
  const int G0r = W == 4 ? (grid_blocks > 0 ? grid_blocks * kOcc / 2 : kOcc * device_cus())
                         : (grid_blocks > 0 ? grid_blocks : 2 * device_cus()) * 4 / W * kOcc;
  const int G0 = G0r > 0 ? G0r : 1;  // (a one-block grid in the 8-wave form)
  const int64_t nj = j_hi - j_lo;
  int64_t cbk = nj, n_chunks = 1, G;
  if (contig) {
    const int64_t sl = skip_lo > j_lo ? skip_lo : j_lo, sh = skip_hi < j_hi ? skip_hi : j_hi;
    const int64_t nre = ns_active - srow0 < n_srb ? ns_active - srow0 : n_srb;
    const int64_t raw = (nre > 0 ? nre : 0) * (nj - (sh > sl ? sh - sl : 0));
    if (raw <= 0) return DAL_OK;
    G = raw < G0 ? raw : G0;
  } else {
    const int64_t nc = choose_chunks(srow0, n_srb, j_lo, j_hi, skip_lo, skip_hi, ns_active, G0, W / 4, min_chunks);
    cbk = ceil_div(nj, nc);
    n_chunks = ceil_div(nj, cbk);
    const int64_t n_units = (W == 4 ? n_srb : 2 * ceil_div(n_srb, 4)) * n_chunks;
    G = n_units < G0 ? n_units : G0;
  }
  hipLaunchKernelGGL((gram_csym_kernel<KS, W>), dim3(static_cast<unsigned>(G)), dim3(64 * W), 0, stream, rows,
                     static_cast<int>(srow0), static_cast<int>(n_srb), cols, static_cast<int>(jcol0),
                     static_cast<int>(j_lo), static_cast<int>(j_hi), static_cast<int>(skip_lo),
                     static_cast<int>(skip_hi), static_cast<int>(ns_active), ldh, slice_off, static_cast<int>(cbk),
                     static_cast<int>(n_chunks), reinterpret_cast<unsigned long long*>(acc), contig);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

#ifndef DAL_GRAM_CONTIG_MB
#define DAL_GRAM_CONTIG_MB 32  // column operands up to this size take the contiguous schedule (KS 32, 128)
#endif
#ifndef DAL_GRAM_KS64_CHUNKED
#define DAL_GRAM_KS64_CHUNKED 1  // ... KS 64 takes >= DAL_GRAM_MIN_CHUNKS_SMALL column chunks instead
#endif
template <int KS>
int launch_csym(const uint16_t* rows, int64_t srow0, int64_t n_srb, const uint16_t* cols, int64_t jcol0,
                int64_t j_lo, int64_t j_hi, int64_t skip_lo, int64_t skip_hi, int64_t ns_active, int64_t ldh,
                int slice_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  // contiguous equal shares of the pair grid per block for a small column
  // operand (<= 32 MB at KS 32 / 128), else round-robin column chunks whose
  // blocks sweep the same column stages together (a small KS-64 operand in as
  // few as two chunks).  Exact integer accumulation: the schedule never
  // changes the bits.
  const int64_t col_bytes = (j_hi - j_lo) * 256 * ldh * 2;
  const bool small = col_bytes <= (int64_t{DAL_GRAM_SMALL_MB} << 20);
  const int contig = col_bytes <= (int64_t{DAL_GRAM_CONTIG_MB} << 20) && !(KS == 64 && DAL_GRAM_KS64_CHUNKED);
  const int64_t min_chunks = small ? DAL_GRAM_MIN_CHUNKS_SMALL : DAL_GRAM_MIN_CHUNKS;
  if constexpr ((KS == 128 && DAL_GRAM_WAVES8) || (KS == 64 && DAL_GRAM_W8_KS64))
    if (!contig)
      return launch_csym_w<KS, 8>(rows, srow0, n_srb, cols, jcol0, j_lo, j_hi, skip_lo, skip_hi, ns_active, ldh,
                                  slice_off, acc, grid_blocks, contig, min_chunks, stream);
  return launch_csym_w<KS, 4>(rows, srow0, n_srb, cols, jcol0, j_lo, j_hi, skip_lo, skip_hi, ns_active, ldh,
                              slice_off, acc, grid_blocks, contig, min_chunks, stream);
}

struct ResidualLayout {
  size_t sig_u, rb, cb, total;
};
ResidualLayout residual_layout(int64_t ns_active, int64_t n_srb, int64_t d_pad) {
  ResidualLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  L.sig_u = take(static_cast<size_t>(ns_active * d_pad) * 8);
  L.rb = take(static_cast<size_t>(n_srb * d_pad) * 8);
  L.cb = take(static_cast<size_t>(n_srb * d_pad) * 8);
  L.total = o;
  return L;
}

}  // namespace

int split_ks(int64_t d_pad) { return d_pad == 32 ? 32 : (d_pad % 128 == 0 ? 128 : 64); }

}  // namespace dal

using namespace dal;

namespace {
// Row-side chain length of the kernel that runs d_pad (split_ks), 0 = the
// longest over every KS.
int row_chain_products(int64_t d_pad) {
  if (d_pad <= 0) {
    int m = Cfg<32, 4>::CHAIN;
    m = Cfg<64, 4>::CHAIN > m ? Cfg<64, 4>::CHAIN : m;
    return Cfg<128, 4>::CHAIN > m ? Cfg<128, 4>::CHAIN : m;
  }
  const int ks = split_ks(d_pad);
  return ks == 32 ? Cfg<32, 4>::CHAIN : ks == 64 ? Cfg<64, 4>::CHAIN : Cfg<128, 4>::CHAIN;
}
}  // namespace

extern "C" double dal_density_error_bound_sym_d(int64_t n_cols, int64_t d_pad) {
  // dal_gram_rowsum_sym + dal_gram_sym_residual against the canonical fp64
  // density, per density entry (one column j of row i), u = 2^-23 (a
  // conservative unit roundoff for the MFMA's internal fp32 adds, counted as
  // sequential adds), products exact (f16 x f16), c = 1 + 2^-8 >= sum_d |h_i
  // h_j| + |h_i l_j| over sum_d |u_i u_j| <= 1 (Cauchy-Schwarz on unit rows):
  //   row side   (the MFMA row sums of the taken pairs) NCH chains per row
  //              tile between folds: Cfg<KS>::CHAIN products each (FOLD / 16 /
  //              NCH tiles x 2 KS: 1,024 at KS 32, 2,048 at KS 64 and 128), the
  //              add combining the two chains (KS 128) and 4 cross-lane adds:
  //              gamma_(CHAIN + 5) * c
  //   column side  none: every taken pair's column sums are the closed form
  //              <u~_i, C_B> of dal_gram_sym_residual (exact int64 sums, an
  //              fp64 dot), as is the row side's remainder <L_i, R_B>: below
  //              2^-40 per column together
  //   split + fp32 unit rows  5 * 2^-22;  fixed-point roundings <= 2^-33 each
  const double u = 1.0 / 8388608.0;  // 2^-23
  auto gamma = [u](double n) { return n * u / (1.0 - n * u); };
  const double s = 1.0 / 4194304.0;  // 2^-22
  const double row = gamma(static_cast<double>(row_chain_products(d_pad)) + 5.0);
  const double c = 1.0 + 1.0 / 256.0;
  return (row * c + 5.0 * s + 1e-10) * static_cast<double>(n_cols) + 1e-9;
}

// Feature-width-free form (ABI v5): the bound of the longest row chain of any
// KS, valid for every pool.
extern "C" double dal_density_error_bound_sym(int64_t n_cols) { return dal_density_error_bound_sym_d(n_cols, 0); }

extern "C" int dal_gram_rowsum_sym_skip(const uint16_t* rows, int64_t row_block0, int64_t n_row_blocks,
                                        const uint16_t* cols, int64_t col_block0, int64_t j_lo, int64_t j_hi,
                                        int64_t skip_lo, int64_t skip_hi, int64_t nb_active, int64_t d_pad,
                                        int64_t* acc, int grid_blocks, dal_stream_t stream) {
  if (!rows || !cols || !acc) return DAL_ERR_ARG;
  if (row_block0 < 0 || n_row_blocks <= 0 || col_block0 < 0 || nb_active <= 0) return DAL_ERR_SHAPE;
  if (j_lo < col_block0 || j_hi < j_lo || j_hi > nb_active || skip_hi < skip_lo) return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad)) return DAL_ERR_SHAPE;
  if ((row_block0 | n_row_blocks | nb_active) & 1) return DAL_ERR_SHAPE;  // whole 512-row super blocks
  if ((reinterpret_cast<uintptr_t>(rows) | reinterpret_cast<uintptr_t>(cols)) & 15) return DAL_ERR_SHAPE;
  if (j_hi == j_lo || row_block0 >= nb_active) return DAL_OK;
  hipStream_t st = as_stream(stream);
  const int ks = split_ks(d_pad);
  const int64_t ldh = 2 * d_pad;
  for (int64_t off = 0; off < d_pad; off += ks) {
    const int so = static_cast<int>(2 * off);  // halves: slice s starts at s * 2 * KS
    const int64_t s0 = row_block0 / 2, ns = n_row_blocks / 2, na = nb_active / 2;
    int rc;
    if (ks == 32)
      rc = launch_csym<32>(rows, s0, ns, cols, col_block0, j_lo, j_hi, skip_lo, skip_hi, na, ldh, so, acc,
                           grid_blocks, st);
    else if (ks == 64)
      rc = launch_csym<64>(rows, s0, ns, cols, col_block0, j_lo, j_hi, skip_lo, skip_hi, na, ldh, so, acc,
                           grid_blocks, st);
    else
      rc = launch_csym<128>(rows, s0, ns, cols, col_block0, j_lo, j_hi, skip_lo, skip_hi, na, ldh, so, acc,
                            grid_blocks, st);
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

extern "C" size_t dal_gram_sym_residual_workspace_bytes(int64_t nb_active, int64_t n_row_blocks, int64_t d_pad) {
  if (nb_active <= 0 || n_row_blocks <= 0 || d_pad <= 0) return 0;
  return residual_layout(nb_active / 2, n_row_blocks / 2, d_pad).total;
}

extern "C" int dal_gram_sym_residual(const uint16_t* ops, int64_t nb_active, int64_t row_block0, int64_t n_row_blocks,
                                     int64_t d_pad, int64_t* acc, void* ws, size_t ws_bytes, dal_stream_t stream) {
  if (!ops || !acc || !ws) return DAL_ERR_ARG;
  if (nb_active <= 0 || row_block0 < 0 || n_row_blocks <= 0 || ((row_block0 | n_row_blocks | nb_active) & 1))
    return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad) || (reinterpret_cast<uintptr_t>(ops) & 15) ||
      (reinterpret_cast<uintptr_t>(ws) & 255))
    return DAL_ERR_SHAPE;
  const int64_t na = nb_active / 2, s0 = row_block0 / 2;
  int64_t ns = n_row_blocks / 2;
  if (s0 >= na) return DAL_OK;
  if (s0 + ns > na) ns = na - s0;  // padding super blocks past the pool hold no rows
  const ResidualLayout L = residual_layout(na, n_row_blocks / 2, d_pad);
  if (ws_bytes < L.total) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  unsigned char* w = static_cast<unsigned char*>(ws);
  long long* sig_u = reinterpret_cast<long long*>(w + L.sig_u);
  double* rb = reinterpret_cast<double*>(w + L.rb);
  double* cb = reinterpret_cast<double*>(w + L.cb);
  const int ks = split_ks(d_pad);
  const int64_t ldh = 2 * d_pad;
  if (hipMemsetAsync(sig_u, 0, static_cast<size_t>(na * d_pad) * 8, st) != hipSuccess) return DAL_ERR_HIP;
  // rows of a super block over 4 blocks (more loads in flight: 196 super blocks at config 2)
  hipLaunchKernelGGL(csym_sigma_kernel,
                     dim3(static_cast<unsigned>(na), static_cast<unsigned>(ceil_div(ldh / 8, 256)), 4), dim3(256), 0,
                     st, ops, ldh, ks, static_cast<int>(d_pad), sig_u);
  DAL_RETURN_IF_LAUNCH_FAILED();
  const int64_t n_rows = ns * kSB;
  const dim3 grid(static_cast<unsigned>(ceil_div(n_rows, kResRows)));
  const size_t smem = static_cast<size_t>(2 * d_pad) * 8;
  const uint16_t* rows = ops + s0 * kSB * ldh;
  if (d_pad <= 64 && na * d_pad <= DAL_CSYM_FUSED_MAX) {  // the blocks form R_B, C_B themselves
    hipLaunchKernelGGL(csym_residual_kernel<kResFused>, grid, dim3(kResRows), smem, st, rows, ldh, ks,
                       static_cast<int>(d_pad), static_cast<int>(s0), static_cast<int>(n_rows), rb, cb, sig_u,
                       static_cast<int>(na), reinterpret_cast<long long*>(acc));
  } else {
    hipLaunchKernelGGL(csym_scan_kernel, dim3(static_cast<unsigned>(ceil_div(d_pad, 64))), dim3(64 * kScanWaves), 0,
                       st, sig_u, static_cast<int>(na), static_cast<int>(d_pad), static_cast<int>(s0),
                       static_cast<int>(s0 + ns), rb, cb);
    DAL_RETURN_IF_LAUNCH_FAILED();
    if (d_pad <= kResLdsMaxFeat) {
      hipLaunchKernelGGL(csym_residual_kernel<kResStaged>, grid, dim3(kResRows), smem, st, rows, ldh, ks,
                         static_cast<int>(d_pad), static_cast<int>(s0), static_cast<int>(n_rows), rb, cb, sig_u,
                         static_cast<int>(na), reinterpret_cast<long long*>(acc));
    } else {  // wide pools: R_B, C_B read in place (they would not fit in LDS beside the tile)
      hipLaunchKernelGGL(csym_residual_kernel<kResGlobal>, grid, dim3(kResRows), 0, st, rows, ldh, ks,
                         static_cast<int>(d_pad), static_cast<int>(s0), static_cast<int>(n_rows), rb, cb, sig_u,
                         static_cast<int>(na), reinterpret_cast<long long*>(acc));
    }
  }
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
