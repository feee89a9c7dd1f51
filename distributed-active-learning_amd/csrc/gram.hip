// Fused cosine Gram row-sum (information density) on fp32 MFMA.
//
// Reference: final_thesis/density_weighting.py:67-75 (U.multiply(UT) through
// IndexedRowMatrix/BlockMatrix, materialising N^2 MatrixEntry records),
// :95-100 (drop i,j in L0) and :157-161 (groupByKey + sum per row);
// cosine_similarity.py:29-45 is the same product as a standalone script.
//
// MI355X design
//  * d_i = sum_j <u_i, u_j> is computed as a tiled GEMM U_rows . U_cols^T whose
//    output tile is never stored: the MFMA accumulator itself carries the row
//    sum across column tiles (acc += S_tile), so the "epilogue" is free.
//  * v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 157 TF/GPU dense).  A block
//    = 4 waves x 64 rows; each wave keeps its 64 rows' A fragments resident in
//    VGPRs for the whole sweep (KS floats/lane) and streams B (column) tiles
//    from a 2 x 64 KiB LDS ring filled by global_load_lds_dwordx4 (one 1-KiB
//    wave-instruction per 64 x 16 B), XOR-swizzled on the SOURCE address so the
//    ds_read_b128 B-fragment reads are bank-conflict free.
//  * Every stage (512 fp32 fmas per accumulator element) each fp32 accumulator
//    is folded as an integer multiple of 2^-32 (v_rndne_f32 of v*2^32) into an
//    fp64 register; integer-valued fp64 adds below 2^53 are exact, and units
//    end in int64 atomics, so per-row totals are bit-identical for any grid,
//    unit split, column split or GPU count (fold groups = fixed column stages).
//  * Persistent grid (one 256-thread block per CU): the (row-block, column-
//    chunk) work units are dealt in equal contiguous ranges, so every CU gets
//    the same number of MFMAs; a row block's A fragments are reloaded only when
//    a block's range crosses into the next row block.  Each unit ends with a
//    32-lane butterfly and ONE 64-lane int64 atomic add per wave.
//  * Feature order inside an MFMA step is permuted (lane half h takes features
//    8c+4h+m for step (c,m)) so each lane's B operand for 4 MFMAs is one
//    16-byte LDS read; A uses the same permutation, so sum_d is unchanged.
//    B reads run one step (8 MFMAs) ahead through a 2-deep register ring.
//  * Measured alternatives (scripts/gram_ab.py, same-process A/B, MI355X):
//    interleaving the fold with the next stage's MFMAs (dual accumulator sets)
//    -3%; interleaving the next stage's DMA issue with the MFMAs -1%; a
//    barrier-free variant streaming B per wave from L2 without LDS -6..-18%.

#include "common.hpp"

namespace dal {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))

constexpr int kGramThreads = 256;   // 4 waves
constexpr int kGramRows = 256;      // rows per block tile (64 per wave)
constexpr int kStageF4 = 4096;      // 64 KiB of fp32 per LDS stage

template <int KS>
struct GramCfg {
  static constexpr int SC = 16384 / KS;   // columns per stage
  static constexpr int SLOTS = KS / 4;    // 16-B slots per column row
  static constexpr int NCT = SC / 32;     // 32-column MFMA tiles per stage
  static constexpr int NKC = KS / 8;      // 8-feature chunks (4 MFMA k-steps each)
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
};

// Exact fold of an fp32 stage partial: v * 2^32 rounded to an integer in
// fp32 (|v| <= 16, so the product is exact and the rounded value is an
// integer < 2^37), accumulated in fp64.  Integer-valued fp64 sums below 2^53
// are exact, so the per-row totals do not depend on the order or grouping of
// the folds (grid, unit split, column split, GPU count).
__device__ __forceinline__ double fold_fixed(float v) {
  return static_cast<double>(__builtin_rintf(v * 4294967296.0f));
}

template <int KS>
__global__ __launch_bounds__(kGramThreads, 1) void gram_rowsum_kernel(
    const float* __restrict__ urows, const float* __restrict__ ucols, int64_t ld, int ks_off,
    int64_t n_stages, int chunk_stages, int64_t n_chunks, int64_t n_units,
    unsigned long long* __restrict__ acc_out) {
  using C = GramCfg<KS>;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * kStageF4];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;

  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t u_begin = (g * n_units) / G, u_end = ((g + 1) * n_units) / G;
  if (u_begin >= u_end) return;

  int64_t unit = u_begin;
  int64_t rb = unit / n_chunks;
  int64_t s = (unit % n_chunks) * chunk_stages;
  int64_t s_end = s + chunk_stages < n_stages ? s + chunk_stages : n_stages;

  // ---- staging: 16 LDS-DMA pieces per wave = 64 KiB per stage ----
  // Inline asm so hipcc does not track the DMA on vmcnt (a tracked
  // global_load_lds makes it wait vmcnt(0) before the next ds_read, which
  // would serialise the prefetch with the MFMAs); we wait for it ourselves
  // at the top of the next iteration.  M0 is written and restored inside the
  // statement (hipcc reserves M0).  Scalar stage base + 32-bit lane offset.
  auto issue_piece = [&](int buf, const float* sbase, int q) {
    const int base = (wave * 16 + q) * 64;
    const int p = base + lane;
    const int row = p / C::SLOTS;
    const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
    const unsigned voff = static_cast<unsigned>((row * ld + slot * 4) * 4);
    const unsigned dst = __builtin_amdgcn_readfirstlane(
        static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + buf * kStageF4 + base))));
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(dst), "s"(sbase)
        : "memory");
  };
  auto stage_base = [&](int64_t stage) { return ucols + stage * C::SC * ld + ks_off; };

  // ---- resident A fragments: rows rb*256 + wave*64 + rt*32 + li ----
  float4 a[2][C::NKC];
  auto load_a = [&](int64_t rbk) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int64_t row = rbk * kGramRows + wave * 64 + rt * 32 + li;
      const float* src = urows + row * ld + ks_off + lh * 4;
#pragma unroll
      for (int c = 0; c < C::NKC; ++c) a[rt][c] = *reinterpret_cast<const float4*>(src + 8 * c);
    }
    // vmcnt(0) expcnt(7) lgkmcnt(15): the compiler now knows A has landed and
    // will not re-wait (which would also drain the in-flight stage DMA).
    __builtin_amdgcn_s_waitcnt(0x0F70);
  };

  f32x16 acc0 = {}, acc1 = {};
  double facc[2][16];
#pragma unroll
  for (int r = 0; r < 16; ++r) facc[0][r] = facc[1][r] = 0.0;
  const f32x16 zero = {};

  // One stage: 512 MFMAs per wave over the 64-KiB LDS stage `sbuf`; the next
  // stage's DMA is in flight underneath.
  auto stage = [&](int sbuf, bool pf, const float* pf_base) {
    if (pf) {  // next stage's 16 DMA pieces up front (measured: beats interleaving)
#pragma unroll
      for (int q = 0; q < 16; ++q) issue_piece(sbuf ^ 1, pf_base, q);
    }
    const float4* B = lds + sbuf * kStageF4;
    constexpr int NSTEP = C::NCT * C::NKC;  // 8 MFMAs per step
    auto bload = [&](int j) {
      const int ct = j / C::NKC, c = j % C::NKC;
      const int rowj = ct * 32 + li;
      return B[rowj * C::SLOTS + ((2 * c + lh) ^ (rowj & C::SWZ))];
    };
    float4 ring[2];
    ring[0] = bload(0);
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
      if (j + 1 < NSTEP) ring[(j + 1) & 1] = bload(j + 1);
      const float4 b = ring[j & 1];
      const int c = j % C::NKC;
      const bool first = (j == 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][c].x, b.x, first ? zero : acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][c].x, b.x, first ? zero : acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][c].y, b.y, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][c].y, b.y, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][c].z, b.z, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][c].z, b.z, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][c].w, b.w, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][c].w, b.w, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      facc[0][r] += fold_fixed(acc0[r]);
      facc[1][r] += fold_fixed(acc1[r]);
    }
  };

  auto finish_unit = [&]() {
    // exact (integer-valued) fp64 butterfly over the 32 column lanes of each
    // half; row = (r&3) + 8(r>>2) + 4h
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
    // lane li of half h publishes value (rt = li>>4, r = li&15): 64 rows, one atomic
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
    const int64_t row = rb * kGramRows + wave * 64 + (li >> 4) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    atomicAdd(acc_out + row, static_cast<unsigned long long>(static_cast<long long>(mine)));
  };

  load_a(rb);
  {
    const float* b0 = stage_base(s);
#pragma unroll
    for (int q = 0; q < 16; ++q) issue_piece(0, b0, q);
  }
  int buf = 0;

  while (true) {
    // next (unit, stage) of this block's flat range
    const bool last_of_unit = (s + 1 == s_end);
    int64_t n_unit = unit, n_s = s + 1;
    if (last_of_unit) {
      n_unit = unit + 1;
      n_s = (n_unit % n_chunks) * chunk_stages;
    }
    const bool has_next = n_unit < u_end;

    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // this wave's DMA for `buf` landed
    __syncthreads();  // ... for every wave; everyone finished reading buf^1
    stage(buf, has_next, stage_base(n_s));
    if (last_of_unit) finish_unit();

    if (!has_next) break;
    if (last_of_unit) {
      unit = n_unit;
      const int64_t nrb = unit / n_chunks;
      if (nrb != rb) {
        rb = nrb;
        load_a(rb);
      }
      s_end = n_s + chunk_stages < n_stages ? n_s + chunk_stages : n_stages;
    }
    s = n_s;
    buf ^= 1;
  }
}

// Small-N entry dump (cosine_similarity.py:42-45): one wave per 32x32 output
// tile, operands straight from global (L2-resident at the sizes this serves).
__global__ __launch_bounds__(64) void gram_entries_kernel(const float* __restrict__ u, int64_t n_pad,
                                                          int d_pad, int64_t ld, float* __restrict__ out) {
  const int lane = threadIdx.x, li = lane & 31, lh = lane >> 5;
  const int64_t i0 = static_cast<int64_t>(blockIdx.y) * 32, j0 = static_cast<int64_t>(blockIdx.x) * 32;
  const float* ai = u + (i0 + li) * ld;
  const float* bj = u + (j0 + li) * ld;
  f32x16 acc = {};
  for (int k = 0; k < d_pad; k += 2)
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ai[k + lh], bj[k + lh], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t row = i0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    out[row * n_pad + j0 + li] = acc[r];
  }
}

int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  return cus;
}

template <int KS>
int launch_gram(const float* u_rows, int64_t n_rows_pad, const float* u_cols, int64_t n_cols_pad,
                int64_t ld, int ks_off, int64_t* acc, int grid_blocks, hipStream_t stream) {
  using C = GramCfg<KS>;
  const int64_t n_row_blocks = n_rows_pad / kGramRows;
  const int64_t n_stages = n_cols_pad / C::SC;
  const int G0 = grid_blocks > 0 ? grid_blocks : device_cus();
  // ~64 units per block: small enough tails, large enough units.
  int64_t cs = (n_stages * n_row_blocks) / (static_cast<int64_t>(G0) * 64);
  cs = cs < 2 ? 2 : (cs > 64 ? 64 : cs);
  if (cs > n_stages) cs = n_stages;
  const int64_t n_chunks = ceil_div(n_stages, cs);
  const int64_t n_units = n_row_blocks * n_chunks;
  const int64_t G = n_units < G0 ? n_units : G0;
  hipLaunchKernelGGL(gram_rowsum_kernel<KS>, dim3(static_cast<unsigned>(G)), dim3(kGramThreads), 0,
                     stream, u_rows, u_cols, ld, ks_off, n_stages, static_cast<int>(cs), n_chunks, n_units,
                     reinterpret_cast<unsigned long long*>(acc));
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

}  // namespace
}  // namespace dal

using namespace dal;

extern "C" double dal_density_error_bound(int64_t n_cols) {
  // |d_gemm - d_canonical| <= (gamma_512 + 2^-22 + 1e-12) * sum_j sum_d |u_id u_jd|
  //                        <= that * n_cols   (Cauchy-Schwarz on unit rows).
  const double u = 1.0 / 16777216.0;  // 2^-24
  const double gamma = 512.0 * u / (1.0 - 512.0 * u);
  return (gamma + 4.0 * u + 1e-12) * static_cast<double>(n_cols) + 1e-9;
}

extern "C" int dal_gram_rowsum(const float* u_rows, int64_t n_rows_pad, const float* u_cols,
                               int64_t n_cols_pad, int64_t d_pad, int64_t ld, int64_t* acc,
                               int grid_blocks, dal_stream_t stream) {
  if (!u_rows || !u_cols || !acc) return DAL_ERR_ARG;
  if (n_rows_pad <= 0 || n_rows_pad % kGramRows || n_cols_pad <= 0 || n_cols_pad % DAL_ROW_GRANULE)
    return DAL_ERR_SHAPE;
  if (d_pad != dal_pad_features(d_pad) || ld < d_pad || (ld % 4)) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(u_rows) | reinterpret_cast<uintptr_t>(u_cols)) & 15)
    return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  const int ks = d_pad == 32 ? 32 : (d_pad == 64 ? 64 : 128);
  for (int64_t off = 0; off < d_pad; off += ks) {
    int rc;
    if (ks == 32)
      rc = launch_gram<32>(u_rows, n_rows_pad, u_cols, n_cols_pad, ld, 0, acc, grid_blocks, st);
    else if (ks == 64)
      rc = launch_gram<64>(u_rows, n_rows_pad, u_cols, n_cols_pad, ld, 0, acc, grid_blocks, st);
    else  // K-slices of 128 features: A stays register-resident (128 floats/lane)
      rc = launch_gram<128>(u_rows, n_rows_pad, u_cols, n_cols_pad, ld, static_cast<int>(off), acc,
                            grid_blocks, st);
    if (rc != DAL_OK) return rc;
  }
  return DAL_OK;
}

extern "C" int dal_gram_entries(const float* u, int64_t n_pad, int64_t d_pad, int64_t ld, float* out,
                                dal_stream_t stream) {
  if (!u || !out) return DAL_ERR_ARG;
  if (n_pad <= 0 || n_pad % 32 || d_pad <= 0 || d_pad % 2 || ld < d_pad) return DAL_ERR_SHAPE;
  if (n_pad > 65535 * 32) return DAL_ERR_SHAPE;
  const unsigned t = static_cast<unsigned>(n_pad / 32);
  hipLaunchKernelGGL(gram_entries_kernel, dim3(t, t), dim3(64), 0, as_stream(stream), u, n_pad,
                     static_cast<int>(d_pad), ld, out);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}
