// Max-cosine to a labeled set on bf16 MFMA (SURVEY §8(a) a12 at scale).
//
// Reference: final_thesis/similarity.py:26-43 normalises the pool (:28),
// transposes it so points become columns (:34-37) and calls
// RowMatrix.columnSimilarities() (:38), the exact cosine of every pair.  The
// batch-mode diversity restatement of BASELINE config 5 keeps, per pool row,
//   m_i = max_{l in L} cos(x_i, x_l)
// and selects the k rows least similar to the labeled set.
//
// MI355X design: v_mfma_f32_32x32x16_bf16 (fp32 accumulate; bf16 x bf16
// products are exact in fp32).  A block = 4 waves x 64 pool rows held as A
// fragments in VGPRs (loaded once from HBM: the pool is streamed exactly
// once); the labeled rows stream through a 2-stage LDS ring by LDS-DMA
// (source-address XOR swizzle -> conflict-free ds_read_b128, SQ_LDS_BANK_
// CONFLICT = 0).  Each 32x32 output tile is scaled by 1/||x_l|| (per lane =
// per column) and max-reduced into a running per-lane maximum; a recursive-
// halving max over the 32 column lanes and the row's 1/||x_i|| (computed
// in-kernel from the resident fragments) finish the row.  The similarity
// matrix is never stored.
//
// Measured at 8M x 128, m = 1024 (scripts/maxcos_ab.py, bit-identical
// outputs): one wave per SIMD with 64 KiB stages 2.78 ms (30% of dense bf16
// peak; exposed per-block A fetch, 5-step butterfly reduction); two waves per
// SIMD 2.04 ms; + v_max3 pairs, hoisted DMA offsets, halving reduction
// 1.80 ms; + immediate-offset B reads 1.75 ms (48%, MFMA busy 61% at the
// 1.89 GHz the chip holds under this load).
#include <type_traits>

#include <stdlib.h>

#include "common.hpp"

namespace dal {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define AS3 __attribute__((address_space(3)))

constexpr int kMcThreads = 256;
constexpr int kMcRows = 256;     // pool rows per block (64 per wave)
constexpr int kMaxLab = 4096;    // labeled rows whose 1/||x|| fit the LDS table

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<unsigned>(b) << 16);
}

// Two waves per SIMD (OCC = 2: 32 KiB stages, 1/||x_l|| table in dynamic LDS
// so two blocks fit a CU): one wave's A-fragment fetch, norm and epilogue VALU
// run under the other wave's MFMAs.  Column tiles in pairs so the running max
// takes one v_max3 per two products; branch-free A loads (rows clamped to
// n-1, never stored); the stage-0 DMA is issued before the A fetch so both are
// in flight together; d = 128 unrolls the stage loop twice so every B-fragment
// address is a per-lane base plus an immediate.
template <int DK, int OCC, int NW = 4>
struct Mc2Cfg {
  static constexpr int STAGE = (OCC == 2 || NW == 8) ? 32768 : 65536;
  static constexpr int F4 = STAGE / 16;
  static constexpr int ROWB = DK * 2;
  static constexpr int SLOTS = ROWB / 16;
  static constexpr int SR = STAGE / ROWB;
  static constexpr int NCT = SR / 32;
  static constexpr int NKS = DK / 16;
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = STAGE / (NW * 1024);  // 1 KiB LDS-DMA pieces per wave per stage
};

// NW = waves per block (64 pool rows each).  NW = 8 (one 512-thread block per
// CU, still two waves per SIMD, half the DMA issue per MFMA) measured 12 %
// slower than NW = 4 at 8M x 128 (barriers over 8 waves), so NW = 4 is used.
//
// ARG: also the arg-max (labeled-row position l) of every pool row.  Each lane
// keeps, per accumulator slot, its best value b1 (first l on equal values: l
// grows along a lane's columns and only a strictly larger value replaces b1),
// that value's l, and the runner-up b2; a butterfly over the 32 column lanes
// merges the triples.  When the scaled top two are more than 2 x the error
// bound apart the fp32 arg-max is the canonical one (|m_gpu - m_canon| <= err
// per entry); otherwise the row gets -1 - l and dal_maxcos_argmax_resolve
// recomputes it in canonical fp64.
template <int DK, int OCC, int NW, bool ARG = false>
__global__ __launch_bounds__(64 * NW, OCC) void maxcos2_kernel(
    const uint16_t* __restrict__ pool, int64_t n, const uint16_t* __restrict__ lab, int64_t m_pad,
    const float* __restrict__ inv_lab, const float* __restrict__ inv_pool, float* __restrict__ out,
    int32_t* __restrict__ out_arg, double gap, int32_t* __restrict__ status) {
  using C = Mc2Cfg<DK, OCC, NW>;
  extern __shared__ __attribute__((aligned(16))) float4 mc_dyn[];
  float4* lds = mc_dyn;
  float* invl = reinterpret_cast<float*>(mc_dyn + 2 * C::F4);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * (64 * NW) + wave * 64;
  const int n_stages = static_cast<int>(m_pad / C::SR);

  for (int i = tid; i < m_pad; i += 64 * NW) invl[i] = inv_lab[i];

  // per-piece source offsets (swizzled) and the wave's LDS base, computed once
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
  // stage 0 first: the compiler's own waits for the (younger) A loads then
  // also cover it, which is conservative and correct
  issue(0, 0);

  bf16x8 a[2][C::NKS];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    int64_t row = row0 + rt * 32 + li;
    row = row < n ? row : n - 1;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s)
      a[rt][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pool + row * DK + 16 * s + 8 * lh));
  }

  // 1/||x_i||: fp64 sum of squares of the register-resident fragments; v*v is
  // exact in fp64, so fma(v, v, s) == s + v*v (dal_inv_norms_bf16's value)
  float inv_row[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    double s2 = 0.0;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double v = static_cast<double>(static_cast<float>(a[rt][s][e]));
        s2 = __builtin_fma(v, v, s2);
      }
    }
    s2 = s2 + __shfl_xor(s2, 32);
    inv_row[rt] = static_cast<float>(1.0 / __builtin_sqrt(s2));
  }

  float mx0[16], mx1[16];
  float sb0[ARG ? 16 : 1], sb1[ARG ? 16 : 1];  // runner-up values (ARG)
  int ag0[ARG ? 16 : 1], ag1[ARG ? 16 : 1];    // arg of mx (ARG)
#pragma unroll
  for (int r = 0; r < 16; ++r) mx0[r] = mx1[r] = -__builtin_inff();
  if constexpr (ARG) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sb0[r] = sb1[r] = -__builtin_inff();
      ag0[r] = ag1[r] = 0x7FFFFFFF;
    }
  }
  // (b1, l, b2) <- v at column l; NaN (padding) never replaces b1 or b2
  auto upd = [](float& b1, float& b2, int& a, float v, int l) {
    if (v > b1) {
      b2 = b1;
      b1 = v;
      a = l;
    } else {
      b2 = fmaxf(b2, v);
    }
  };
  const f32x16 zero = {};

  // per-lane LDS offsets of the B fragment of each k-step (float4 units);
  // column-tile and ring-buffer offsets are compile-time immediates
  int boff[C::NKS];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) boff[s] = li * C::SLOTS + ((2 * s + lh) ^ (li & C::SWZ));

  auto stage_body = [&](auto bufc, int st) {
    constexpr int buf = decltype(bufc)::value;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 1 < n_stages) issue(buf ^ 1, st + 1);
    const float4* B = lds + buf * C::F4;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ct += 2) {
      f32x16 c0, c1, d0, d1;
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, B[ct * 32 * C::SLOTS + boff[s]]);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][s], b, s == 0 ? zero : c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][s], b, s == 0 ? zero : c1, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, B[(ct + 1) * 32 * C::SLOTS + boff[s]]);
        d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][s], b, s == 0 ? zero : d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][s], b, s == 0 ? zero : d1, 0, 0, 0);
      }
      // padded labeled rows carry NaN -> ignored by fmaxf
      const float ila = invl[st * C::SR + ct * 32 + li], ilb = invl[st * C::SR + ct * 32 + 32 + li];
      if constexpr (ARG) {
        const int la = st * C::SR + ct * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          upd(mx0[r], sb0[r], ag0[r], c0[r] * ila, la);
          upd(mx0[r], sb0[r], ag0[r], d0[r] * ilb, la + 32);
          upd(mx1[r], sb1[r], ag1[r], c1[r] * ila, la);
          upd(mx1[r], sb1[r], ag1[r], d1[r] * ilb, la + 32);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          mx0[r] = fmaxf(fmaxf(mx0[r], c0[r] * ila), d0[r] * ilb);  // one v_max3
          mx1[r] = fmaxf(fmaxf(mx1[r], c1[r] * ila), d1[r] * ilb);
        }
      }
    }
  };
  auto stage_body_rt = [&](int st) {
    const int buf = st & 1;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 1 < n_stages) issue(buf ^ 1, st + 1);
    const float4* B = lds + buf * C::F4;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ct += 2) {
      f32x16 c0, c1, d0, d1;
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, B[ct * 32 * C::SLOTS + boff[s]]);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][s], b, s == 0 ? zero : c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][s], b, s == 0 ? zero : c1, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, B[(ct + 1) * 32 * C::SLOTS + boff[s]]);
        d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][s], b, s == 0 ? zero : d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][s], b, s == 0 ? zero : d1, 0, 0, 0);
      }
      // padded labeled rows carry NaN -> ignored by fmaxf
      const float ila = invl[st * C::SR + ct * 32 + li], ilb = invl[st * C::SR + ct * 32 + 32 + li];
      if constexpr (ARG) {
        const int la = st * C::SR + ct * 32 + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          upd(mx0[r], sb0[r], ag0[r], c0[r] * ila, la);
          upd(mx0[r], sb0[r], ag0[r], d0[r] * ilb, la + 32);
          upd(mx1[r], sb1[r], ag1[r], c1[r] * ila, la);
          upd(mx1[r], sb1[r], ag1[r], d1[r] * ilb, la + 32);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          mx0[r] = fmaxf(fmaxf(mx0[r], c0[r] * ila), d0[r] * ilb);  // one v_max3
          mx1[r] = fmaxf(fmaxf(mx1[r], c1[r] * ila), d1[r] * ilb);
        }
      }
    }
  };
  if constexpr (DK == 128 && (OCC == 2 || NW == 8)) {
    // the label granule (65536 / (2d) rows) is two 32 KiB stages: n_stages is even
    if ((n_stages & 1) == 0) {
      for (int st = 0; st < n_stages; st += 2) {
        stage_body(std::integral_constant<int, 0>{}, st);
        stage_body(std::integral_constant<int, 1>{}, st + 1);
      }
    } else {
      for (int st = 0; st < n_stages; ++st) stage_body_rt(st);
    }
  } else {
    // d = 64 unrolled twice exceeds the 256-register budget: keep one body
    for (int st = 0; st < n_stages; ++st) stage_body_rt(st);
  }
  if constexpr (ARG) {
    // butterfly over the 32 column lanes, every slot j: merge (b1, l, b2)
    float b1[32], b2[32];
    int ag[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      b1[r] = mx0[r];
      b1[16 + r] = mx1[r];
      b2[r] = sb0[r];
      b2[16 + r] = sb1[r];
      ag[r] = ag0[r];
      ag[16 + r] = ag1[r];
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float ob1 = __shfl_xor(b1[j], o), ob2 = __shfl_xor(b2[j], o);
        const int oa = __shfl_xor(ag[j], o);
        if (ob1 > b1[j] || (ob1 == b1[j] && oa < ag[j])) {
          b2[j] = fmaxf(b1[j], ob2);
          b1[j] = ob1;
          ag[j] = oa;
        } else {
          b2[j] = fmaxf(b2[j], ob1);
        }
      }
    }
    // lane li finishes slot j = li: row tile li>>4, accumulator element li&15
    float v1 = b1[0], v2 = b2[0];
    int va = ag[0];
#pragma unroll
    for (int j = 1; j < 32; ++j) {
      if (li == j) {
        v1 = b1[j];
        v2 = b2[j];
        va = ag[j];
      }
    }
    const int r = li & 15;
    const int rl = (li >> 4) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    const float inv0 = __shfl(inv_row[0], rl & 31), inv1 = __shfl(inv_row[1], rl & 31);
    const int64_t row = row0 + rl;
    if (row < n) {
      const float iv = inv_pool ? inv_pool[row] : ((rl >> 5) ? inv1 : inv0);
      if (!(iv < __builtin_inff())) atomicOr(status, DAL_FLAG_ZERO_NORM);
      const float m1 = v1 * iv, m2 = v2 * iv;
      out[row] = m1;
      const bool certain = static_cast<double>(m1) - static_cast<double>(m2) > gap;
      out_arg[row] = certain ? va : -1 - va;
    }
    return;
  }
  // max over the 32 column lanes by recursive halving: at mask m a lane keeps
  // the half of its 2m values selected by (li & m) and folds in the partner's
  // copy of that half (31 shuffles).  Lane li ends with value j = li, i.e.
  // row tile li>>4, accumulator element r = li&15.
  float v[32];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    v[r] = mx0[r];
    v[16 + r] = mx1[r];
  }
#pragma unroll
  for (int step = 0; step < 5; ++step) {
    const int m = 16 >> step;
    // bit-mask selects (a ternary on array elements becomes dynamic indexing)
    const unsigned upm = (li & m) ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int j = 0; j < m; ++j) {
      const unsigned lo = __float_as_uint(v[j]), hi = __float_as_uint(v[j + m]);
      const float send = __uint_as_float((lo & upm) | (hi & ~upm));
      const float keep = __uint_as_float((hi & upm) | (lo & ~upm));
      v[j] = fmaxf(keep, __shfl_xor(send, m));
    }
  }
  const float mine = v[0];
  const int r = li & 15;
  const int rl = (li >> 4) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
  const float inv0 = __shfl(inv_row[0], rl & 31), inv1 = __shfl(inv_row[1], rl & 31);
  const int64_t row = row0 + rl;
  if (row < n) {
    const float iv = inv_pool ? inv_pool[row] : ((rl >> 5) ? inv1 : inv0);
    if (!(iv < __builtin_inff())) atomicOr(status, DAL_FLAG_ZERO_NORM);
    out[row] = mine * iv;
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
  double s = 0.0;
  for (int f = 0; f < d; ++f) {
    const double v = bf16_to_f32(x[i * ld + f]);
    s = s + v * v;
  }
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
  double s = 0.0;
  for (int f = 0; f < d; ++f) {
    const double v = bf16_to_f32(x[i * ld + f]);
    s = s + v * v;
  }
  const double nr = __builtin_sqrt(s);
  for (int f = threadIdx.x; f < d; f += 64) {
    const double v = static_cast<double>(bf16_to_f32(x[i * ld + f])) / nr;
    u[feature_major ? f * n + i : i * d + f] = v;
  }
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
    if (tid == 0) {
      double n2 = 0.0;
      for (int f = 0; f < d; ++f) {
        const double v = bf16_to_f32(xr[f]);
        n2 = n2 + v * v;
      }
      s_nr = __builtin_sqrt(n2);
    }
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

template <int DK, bool ARG>
int launch_maxcos_t(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, const float* inv_lab,
                    const float* inv_pool, float* out, int32_t* out_arg, double gap, int32_t* status,
                    hipStream_t st) {
  const int64_t blocks = ceil_div(n, kMcRows);
  constexpr int OCC = DK <= 128 ? 2 : 1;
  const size_t shm = 2 * Mc2Cfg<DK, OCC>::STAGE + static_cast<size_t>(m_pad) * 4;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(maxcos2_kernel<DK, OCC, 4, ARG>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(shm)) != hipSuccess)
    return DAL_ERR_HIP;
  hipLaunchKernelGGL((maxcos2_kernel<DK, OCC, 4, ARG>), dim3(static_cast<unsigned>(blocks)), dim3(kMcThreads), shm,
                     st, pool, n, lab, m_pad, inv_lab, inv_pool, out, out_arg, gap, status);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

template <int DK>
int launch_maxcos(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, const float* inv_lab,
                  const float* inv_pool, float* out, int32_t* out_arg, double gap, int32_t* status, hipStream_t st) {
  if (out_arg) return launch_maxcos_t<DK, true>(pool, n, lab, m_pad, inv_lab, inv_pool, out, out_arg, gap, status, st);
  return launch_maxcos_t<DK, false>(pool, n, lab, m_pad, inv_lab, inv_pool, out, nullptr, 0.0, status, st);
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

extern "C" double dal_maxcos_error_bound(int64_t d) {
  const double u = 1.0 / 16777216.0;
  const double k = 2.0 * static_cast<double>(d) + 4.0;
  return k * u / (1.0 - k * u) * 1.01 + 1e-12;
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
