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
// once); the labeled rows stream through a 2 x 64 KiB LDS ring by LDS-DMA
// (source-address XOR swizzle -> conflict-free ds_read_b128).  Each 32x32
// output tile is scaled by 1/||x_l|| (per lane = per column) and max-reduced
// into a running per-lane maximum; a 32-lane butterfly max and the row's
// 1/||x_i|| finish the row.  The similarity matrix is never stored.
#include "common.hpp"

namespace dal {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
#define AS3 __attribute__((address_space(3)))

constexpr int kMcThreads = 256;
constexpr int kMcRows = 256;     // pool rows per block (64 per wave)
constexpr int kStageF4 = 4096;   // 64 KiB per LDS stage
constexpr int kMaxLab = 4096;    // labeled rows whose 1/||x|| fit the LDS table

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<unsigned>(b) << 16);
}

template <int DK>
struct McCfg {
  static constexpr int ROWB = DK * 2;          // bytes per row
  static constexpr int SLOTS = ROWB / 16;      // 16-B slots per row
  static constexpr int SR = 65536 / ROWB;      // labeled rows per stage
  static constexpr int NCT = SR / 32;          // 32-row column tiles per stage
  static constexpr int NKS = DK / 16;          // k-steps of 16 features
  static constexpr int SWZ = (SLOTS < 16 ? SLOTS : 16) - 1;
};

template <int DK>
__global__ __launch_bounds__(kMcThreads, 1) void maxcos_kernel(
    const uint16_t* __restrict__ pool, int64_t n, const uint16_t* __restrict__ lab, int64_t m_pad,
    const float* __restrict__ inv_lab, const float* __restrict__ inv_pool, float* __restrict__ out) {
  using C = McCfg<DK>;
  __shared__ __attribute__((aligned(16))) float4 lds[2 * kStageF4];
  __shared__ float invl[kMaxLab];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kMcRows + wave * 64;
  const int n_stages = static_cast<int>(m_pad / C::SR);

  for (int i = tid; i < m_pad; i += kMcThreads) invl[i] = inv_lab[i];

  auto issue = [&](int buf, int stage) {
    const char* sbase = reinterpret_cast<const char*>(lab) + static_cast<int64_t>(stage) * 65536;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int base = (wave * 16 + q) * 64;
      const int p = base + lane;
      const int row = p / C::SLOTS;
      const int slot = (p % C::SLOTS) ^ (row & C::SWZ);
      const unsigned voff = static_cast<unsigned>(row * C::ROWB + slot * 16);
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          static_cast<unsigned>(reinterpret_cast<uintptr_t>((AS3 float4*)(lds + buf * kStageF4 + base))));
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff), "s"(dst), "s"(sbase)
          : "memory");
    }
  };

  // A fragments: lane (li, lh) holds features 16s + 8lh .. +7 of its two rows
  bf16x8 a[2][C::NKS];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int64_t row = row0 + rt * 32 + li;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < n) v = *reinterpret_cast<const uint4*>(pool + row * DK + 16 * s + 8 * lh);
      a[rt][s] = __builtin_bit_cast(bf16x8, v);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // A landed; keep hipcc from re-waiting under the DMA

  float mx0[16], mx1[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) mx0[r] = mx1[r] = -__builtin_inff();
  const f32x16 zero = {};

  issue(0, 0);
  for (int st = 0; st < n_stages; ++st) {
    const int buf = st & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (st + 1 < n_stages) issue(buf ^ 1, st + 1);
    const float4* B = lds + buf * kStageF4;
#pragma unroll
    for (int ct = 0; ct < C::NCT; ++ct) {
      const int rowj = ct * 32 + li;
      f32x16 c0, c1;
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const bf16x8 b = __builtin_bit_cast(bf16x8, B[rowj * C::SLOTS + ((2 * s + lh) ^ (rowj & C::SWZ))]);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][s], b, s == 0 ? zero : c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][s], b, s == 0 ? zero : c1, 0, 0, 0);
      }
      // column j = lane's labeled row; padded rows carry NaN -> ignored by fmaxf
      const float il = invl[st * C::SR + rowj];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        mx0[r] = fmaxf(mx0[r], c0[r] * il);
        mx1[r] = fmaxf(mx1[r], c1[r] * il);
      }
    }
  }
  // max over the 32 column lanes of each half; row = (r&3) + 8(r>>2) + 4h
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      mx0[r] = fmaxf(mx0[r], __shfl_xor(mx0[r], o));
      mx1[r] = fmaxf(mx1[r], __shfl_xor(mx1[r], o));
    }
  }
  float mine = 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r == (li & 15)) mine = (li >> 4) ? mx1[r] : mx0[r];
  }
  const int r = li & 15;
  const int64_t row = row0 + (li >> 4) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
  if (row < n) out[row] = mine * inv_pool[row];
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

// Canonical fp64 unit rows of a bf16 table (sequential norm, then divide).
__global__ __launch_bounds__(64) void canon_unit_rows_bf16_kernel(const uint16_t* __restrict__ x, int64_t n,
                                                                  int d, int64_t ld,
                                                                  double* __restrict__ u) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int f = 0; f < d; ++f) {
    const double v = bf16_to_f32(x[i * ld + f]);
    s = s + v * v;
  }
  const double nr = __builtin_sqrt(s);
  for (int f = threadIdx.x; f < d; f += 64) u[i * d + f] = static_cast<double>(bf16_to_f32(x[i * ld + f])) / nr;
}

template <int DK>
int launch_maxcos(const uint16_t* pool, int64_t n, const uint16_t* lab, int64_t m_pad, const float* inv_lab,
                  const float* inv_pool, float* out, hipStream_t st) {
  const int64_t blocks = ceil_div(n, kMcRows);
  hipLaunchKernelGGL(maxcos_kernel<DK>, dim3(static_cast<unsigned>(blocks)), dim3(kMcThreads), 0, st, pool,
                     n, lab, m_pad, inv_lab, inv_pool, out);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
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

extern "C" int dal_canon_unit_rows_bf16(const uint16_t* x, int64_t n, int64_t d, int64_t ld, double* u,
                                        dal_stream_t stream) {
  if (!x || !u) return DAL_ERR_ARG;
  if (n < 1 || d < 1 || ld < d) return DAL_ERR_SHAPE;
  hipLaunchKernelGGL(canon_unit_rows_bf16_kernel, dim3(static_cast<unsigned>(n)), dim3(64), 0,
                     as_stream(stream), x, n, static_cast<int>(d), ld, u);
  DAL_RETURN_IF_LAUNCH_FAILED();
  return DAL_OK;
}

extern "C" double dal_maxcos_error_bound(int64_t d) {
  const double u = 1.0 / 16777216.0;
  const double k = 2.0 * static_cast<double>(d) + 4.0;
  return k * u / (1.0 - k * u) * 1.01 + 1e-12;
}

extern "C" int dal_max_cosine(const uint16_t* pool, int64_t n, int64_t d, const uint16_t* lab, int64_t m_pad,
                              const float* inv_lab, const float* inv_pool, float* out_max,
                              dal_stream_t stream) {
  if (!pool || !lab || !inv_lab || !inv_pool || !out_max) return DAL_ERR_ARG;
  if (n < 1 || (d != 64 && d != 128 && d != 256)) return DAL_ERR_SHAPE;
  if (m_pad < 1 || m_pad % dal_maxcos_label_rows_granule(d) || m_pad > kMaxLab) return DAL_ERR_SHAPE;
  if ((reinterpret_cast<uintptr_t>(pool) | reinterpret_cast<uintptr_t>(lab)) & 15) return DAL_ERR_SHAPE;
  hipStream_t st = as_stream(stream);
  if (d == 64) return launch_maxcos<64>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, st);
  if (d == 128) return launch_maxcos<128>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, st);
  return launch_maxcos<256>(pool, n, lab, m_pad, inv_lab, inv_pool, out_max, st);
}
