// fp32 as three bf16 pieces: the split and the six-product MFMA step shared
// by the bf16x6 kernels (attention_f32x.hip, gemm_f32x.hip).
//
// x = x0 + x1 + x2 exactly (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x -
// x0 - x1): 3 x 8 mantissa bits hold all 24 of an fp32), and a product a.b
// is the sum of the six piece products of order >= 2^-16 |a.b|; a bf16 x bf16
// product is exact in fp32 and v_mfma_f32_32x32x16_bf16 accumulates in
// fp32, so the only error beyond fp32 accumulation is the dropped
// a1b2 + a2b1 + a2b2 (<= ~2^-23 |a.b|, one fp32 rounding of the product).
#pragma once
#include "common.h"

namespace nos {

// x (2 lanes of a pair) -> three bf16 pieces, exactly: each residual of an
// fp32 minus its bf16 rounding has <= 16 significant bits, so the
// subtractions are exact.  The subtractions are scalar v_sub_f32 (the files
// are built with -fno-slp-vectorize): a v_pk_add_f32 beside the MFMAs costs
// more issue cycles than its two halves (x6 attention 3-5 % faster,
// profiles/r03_x6_scalar_split_ab.json)
__device__ __forceinline__ void split2(f32x2_t x, bf16x2_t& p0, bf16x2_t& p1, bf16x2_t& p2) {
  p0 = __builtin_convertvector(x, bf16x2_t);
  const float r1x = x.x - (float)p0.x, r1y = x.y - (float)p0.y;
  p1 = __builtin_convertvector(f32x2_t{r1x, r1y}, bf16x2_t);
  const float r2x = r1x - (float)p1.x, r2y = r1y - (float)p1.y;
  p2 = __builtin_convertvector(f32x2_t{r2x, r2y}, bf16x2_t);
}

__device__ __forceinline__ void split8(const float* x, bf16x8_t& p0, bf16x8_t& p1, bf16x8_t& p2) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    bf16x2_t a, b, c;
    split2(f32x2_t{x[j], x[j + 1]}, a, b, c);
    p0[j] = a.x; p0[j + 1] = a.y;
    p1[j] = b.x; p1[j + 1] = b.y;
    p2[j] = c.x; p2[j + 1] = c.y;
  }
}

// acc += sum of the six piece products of a (A operand) and b (B operand),
// smallest terms first
__device__ __forceinline__ f32x16_t mma6(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], f32x16_t acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

}  // namespace nos
