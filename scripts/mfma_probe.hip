// Numerics probe of v_mfma_f32_16x16x32_f16 (the density Gram's MFMA):
// how the 32 products of one output element and the accumulator C are added.
// One wave computes D = A * B + C for one 16x16x32 tile; the host picks A, B,
// C per case (fp16 bit patterns, fp32 C) and reads D.  Layout (the Gram
// kernel's): lane l holds A row (l & 15), k = 8 * (l >> 4) .. +7 and B column
// (l & 15), the same k range; D[4 * (l >> 4) + r][l & 15] in register r.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/mfma_probe.hip -o scripts/libmfma_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe_kernel(const uint16_t* a, const uint16_t* b, const float* c, float* d) {
  const int l = threadIdx.x;
  f16x8 av, bv;
  for (int e = 0; e < 8; ++e) {
    av[e] = __builtin_bit_cast(_Float16, a[(l & 15) * 32 + 8 * (l >> 4) + e]);
    bv[e] = __builtin_bit_cast(_Float16, b[(l & 15) * 32 + 8 * (l >> 4) + e]);
  }
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c[(4 * (l >> 4) + r) * 16 + (l & 15)];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

// a: [16 rows][32 k] fp16 bits, b: [16 cols][32 k] fp16 bits, c/d: [16][16] fp32
extern "C" int mfma_probe(const uint16_t* a_h, const uint16_t* b_h, const float* c_h, float* d_h) {
  uint16_t *a, *b;
  float *c, *d;
  if (hipMalloc(&a, 1024) || hipMalloc(&b, 1024) || hipMalloc(&c, 1024) || hipMalloc(&d, 1024)) return 1;
  hipMemcpy(a, a_h, 1024, hipMemcpyHostToDevice);
  hipMemcpy(b, b_h, 1024, hipMemcpyHostToDevice);
  hipMemcpy(c, c_h, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, a, b, c, d);
  const int rc = hipMemcpy(d_h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess;
  hipFree(a);
  hipFree(b);
  hipFree(c);
  hipFree(d);
  return rc;
}
