// Fused cosine Gram row-sum on fp16 MFMA with a two-term split of every
// fp32 unit row (three products per feature pair): the fp32-accurate density
// at the fp16 matrix-core rate.
//
// Reference: final_thesis/density_weighting.py:67-75 (U.multiply(UT) through
// IndexedRowMatrix/BlockMatrix), :95-100 (drop i,j in L0) and :157-161
// (groupByKey + sum per row); cosine_similarity.py:29-45 is the same product.
//
// Split.  Every normalised fp32 component u (|u| <= 1) is written as
//   h = fp16_rn(u),   l = fp16_rn((u - h) * 2^12)     (u - h is exact in fp32)
// so u = h + l*2^-12 + e with |e| <= 2^-22 |u| (+2^-37 absolute when h or l
// is subnormal).  Then
//   u_i.u_j = h_i.h_j + 2^-12 (h_i.l_j + l_i.h_j) + O(3 * 2^-22 |u_i||u_j|)
// and fp16 x fp16 products are exact in fp32.  Three v_mfma_f32_32x32x16_f16
// per 16 features replace eight v_mfma_f32_32x32x2_f32 per 16 features:
// 96 vs 512 SIMD cycles, 5.3x the fp32-MFMA rate at equal accuracy class.
// Two accumulators per row tile: M (h.h, the large term) and X (the cross
// terms, scaled by 2^12, ~2^-10 of M), so M's fp32 chain carries 512
// products per fold exactly like the fp32 kernel's.
//
// Exactness of the row sums is kept from gram.hip: per 256-column fold group
// each lane's partial v = fma(X, 2^-12, M) is rounded to a multiple of 2^-32
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

#include <type_traits>

#include "common.hpp"

namespace dal {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
#define AS3 __attribute__((address_space(3)))

constexpr int kSpThreads = 256;    // 4 waves
constexpr int kSpRows = 256;       // rows per block (64 per wave = 2 MFMA row tiles)
constexpr int kSpStage = 32768;    // bytes per LDS stage
constexpr int kSpFoldCols = 256;   // columns per exact fold group

template <int KS>
struct SpCfg {
  static constexpr int ROWB = KS * 4;                   // bytes per column row: KS hi + KS lo halves
  static constexpr int SLOTS = ROWB / 16;               // 16-B slots per column row
  static constexpr int HI = KS / 8;                     // slots of the hi part
  static constexpr int SC = kSpStage / ROWB;            // columns per stage
  static constexpr int NCT = SC / 32;                   // MFMA column tiles per stage
  static constexpr int NKS = KS / 16;                   // MFMA k-steps per slice
  static constexpr int FS = kSpFoldCols / SC;           // stages per fold group (1 or 2)
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
  static constexpr int PIECES = kSpStage / (4 * 1024);  // 1-KiB DMA pieces per wave per stage
  static constexpr int F4 = kSpStage / 16;
  static_assert(FS == 1 || FS == 2, "a stage pair must hold whole fold groups");
};

__device__ __forceinline__ double fold_fixed(float v) {
  return static_cast<double>(__builtin_rintf(v * 4294967296.0f));
}

template <int KS>
__global__ __launch_bounds__(kSpThreads, 2) void gram_split_kernel(
    const uint16_t* __restrict__ urows, const uint16_t* __restrict__ ucols, int64_t ldh,
    int slice_off, int64_t n_pairs, int chunk_pairs, int64_t n_chunks, int64_t n_units,
    unsigned long long* __restrict__ acc_out) {
  using C = SpCfg<KS>;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * C::F4];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;

  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t u_begin = (g * n_units) / G, u_end = ((g + 1) * n_units) / G;
  if (u_begin >= u_end) return;

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
  int64_t rb = unit / n_chunks;
  int64_t pr = (unit % n_chunks) * chunk_pairs;
  int64_t pr_end = pr + chunk_pairs < n_pairs ? pr + chunk_pairs : n_pairs;

  f16x8 ah[2][C::NKS], al[2][C::NKS];
  auto load_a = [&](int64_t rbk) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int64_t row = rbk * kSpRows + wave * 64 + rt * 32 + li;
      const uint16_t* src = urows + row * ldh + slice_off;
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        ah[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + (2 * c + lh) * 8));
        al[rt][c] = __builtin_bit_cast(f16x8, *reinterpret_cast<const uint4*>(src + KS + (2 * c + lh) * 8));
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): A (and any in-flight DMA) landed
  };

  // B-fragment LDS offsets (float4 units) per k-step; column tiles add ct*32*SLOTS
  int boh[C::NKS], bol[C::NKS];
#pragma unroll
  for (int c = 0; c < C::NKS; ++c) {
    boh[c] = li * C::SLOTS + ((2 * c + lh) ^ (li & C::SWZ));
    bol[c] = li * C::SLOTS + ((C::HI + 2 * c + lh) ^ (li & C::SWZ));
  }

  f32x16 m0, m1, x0, x1;
  double facc[2][16];
#pragma unroll
  for (int r = 0; r < 16; ++r) facc[0][r] = facc[1][r] = 0.0;
  const f32x16 zero = {};

  auto compute = [&](auto firstc, const float4* B) {
    constexpr bool FIRST = decltype(firstc)::value;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
#pragma unroll
      for (int c = 0; c < C::NKS; ++c) {
        const f16x8 bh = __builtin_bit_cast(f16x8, B[ct * 32 * C::SLOTS + boh[c]]);
        const f16x8 bl = __builtin_bit_cast(f16x8, B[ct * 32 * C::SLOTS + bol[c]]);
        const bool z = FIRST && ct == 0 && c == 0;
        m0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[0][c], bh, z ? zero : m0, 0, 0, 0);
        m1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[1][c], bh, z ? zero : m1, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[0][c], bl, z ? zero : x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[1][c], bl, z ? zero : x1, 0, 0, 0);
        x0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[0][c], bh, x0, 0, 0, 0);
        x1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[1][c], bh, x1, 0, 0, 0);
      }
    }
  };
  auto fold = [&]() {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      facc[0][r] += fold_fixed(__builtin_fmaf(x0[r], 0x1p-12f, m0[r]));
      facc[1][r] += fold_fixed(__builtin_fmaf(x1[r], 0x1p-12f, m1[r]));
    }
  };

  auto finish_unit = [&]() {
    // exact (integer-valued) fp64 butterfly over the 32 column lanes of each half
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        double v = facc[rt][r];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 16);
        facc[rt][r] = v;
      }
    }
    double mine = 0.0;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (rt * 16 + r == li) mine = facc[rt][r];
        facc[rt][r] = 0.0;
      }
    }
    const int r = li & 15;
    const int64_t row = rb * kSpRows + wave * 64 + (li >> 4) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
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
      n_unit = unit + 1;
      n_pr = (n_unit % n_chunks) * chunk_pairs;
    }
    const bool has_next = n_unit < u_end;

    // stage 2*pr on buffer 0 (its DMA was issued one stage ago)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    issue(1, 2 * pr + 1);
    compute(std::integral_constant<bool, true>{}, B0);
    if constexpr (C::FS == 1) fold();

    // stage 2*pr+1 on buffer 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (has_next) issue(0, 2 * n_pr);
    compute(std::integral_constant<bool, C::FS == 1>{}, B1);
    fold();
    if (last_of_unit) finish_unit();

    if (!has_next) break;
    if (last_of_unit) {
      unit = n_unit;
      const int64_t nrb = unit / n_chunks;
      if (nrb != rb) {
        rb = nrb;
        load_a(rb);
      }
      pr_end = n_pr + chunk_pairs < n_pairs ? n_pr + chunk_pairs : n_pairs;
    }
    pr = n_pr;
  }
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
    const _Float16 he = static_cast<_Float16>(v[e]);
    const float r = v[e] - static_cast<float>(he);  // exact
    h[e] = he;
    l[e] = static_cast<_Float16>(r * 4096.0f);
  }
  uint16_t* dst = out + row * (2 * static_cast<int64_t>(d_pad)) + (f0 / ks) * (2 * ks) + (f0 % ks);
  *reinterpret_cast<uint4*>(dst) = __builtin_bit_cast(uint4, h);
  *reinterpret_cast<uint4*>(dst + ks) = __builtin_bit_cast(uint4, l);
}

int device_cus_split() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  return cus;
}

template <int KS>
int launch_split(const uint16_t* rows, int64_t n_rows_pad, const uint16_t* cols, int64_t n_cols_pad,
                 int64_t ldh, int slice_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  using C = SpCfg<KS>;
  const int64_t n_row_blocks = n_rows_pad / kSpRows;
  const int64_t n_pairs = n_cols_pad / (2 * C::SC);
  const int G0 = grid_blocks > 0 ? grid_blocks : 2 * device_cus_split();
  // ~32 units per block: short tails, long enough units to amortise the butterfly
  int64_t cs = (n_pairs * n_row_blocks) / (static_cast<int64_t>(G0) * 32);
  cs = cs < 1 ? 1 : (cs > 32 ? 32 : cs);
  if (cs > n_pairs) cs = n_pairs;
  const int64_t n_chunks = ceil_div(n_pairs, cs);
  const int64_t n_units = n_row_blocks * n_chunks;
  const int64_t G = n_units < G0 ? n_units : G0;
  hipLaunchKernelGGL(gram_split_kernel<KS>, dim3(static_cast<unsigned>(G)), dim3(kSpThreads), 0, stream,
                     rows, cols, ldh, slice_off, n_pairs, static_cast<int>(cs), n_chunks, n_units,
                     reinterpret_cast<unsigned long long*>(acc));
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

inline int split_ks(int64_t d_pad) { return d_pad == 32 ? 32 : 64; }

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" double dal_density_error_bound_split(int64_t n_cols) {
  // Per entry, with u = 2^-23 (a conservative unit roundoff for the MFMA's
  // internal fp32 accumulation) and chains of at most 1040 additions per fold:
  //   accumulation  gamma_1040 * sum_d |h_i h_j| (+ the 2^-10-smaller cross chain)
  //   split         3 * 2^-22 * sum_d |u_i u_j|  (+2^-37 per feature, subnormal halves)
  //   combine fma   2^-24,  fold rounding  2^-33 per 8 columns
  // and sum_d |u_i u_j| <= 1 (Cauchy-Schwarz on unit rows).
  const double u = 1.0 / 8388608.0;  // 2^-23
  const double gamma = 1040.0 * u / (1.0 - 1040.0 * u);
  const double s = 1.0 / 4194304.0;  // 2^-22
  return (gamma + 4.0 * s + 1e-12) * static_cast<double>(n_cols) + 1e-9;
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
  for (int64_t off = 0; off < d_pad; off += ks) {
    const int so = static_cast<int>(2 * off);  // halves: slice s starts at s * 2 * KS
    const int rc = ks == 32 ? launch_split<32>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st)
                            : launch_split<64>(rows, n_rows_pad, cols, n_cols_pad, ldh, so, acc, grid_blocks, st);
    if (rc != DAL_OK) return rc;
  }
  return DAL_OK;
}
