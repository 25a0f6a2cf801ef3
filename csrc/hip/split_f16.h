// fp32 as two fp16 pieces on a power-of-two scale: the split and the
// three-product MFMA step of the fp16x3 ("h3") kernels (attention_f32x.hip).
//
// x' = x * 2^E (E chosen per row / head so |x'| < 2^14) = h + l with
// h = f16(x') and l = f16(x' - h), both round-to-nearest: h keeps 11
// significant bits and |x' - h| <= 2^-11 |x'|; x' - h is exact in fp32 and l
// keeps 11 of its bits, so |x' - h - l| <= 2^-22 |x'| (~2^-24 on average):
// 22 of an fp32's 24 bits.  A product a.b is then
//   ah.bh + ah.bl + al.bh   (dropped: al.bl <= 2^-22 |a.b|)
// -- three fp16 MFMAs (products exact in fp32, fp32 accumulation) where the
// exact bf16 split (split_bf16.h) needs six.  In a dot product of 16+ terms
// the fp32 accumulation's rounding dominates these operand errors: against
// fp64 the h3 kernels stay within the exact-f32 kernels' error
// (tests/test_split_f16_numerics.py, tests/test_attention_h3_gpu.py).
// The price is range: fp16 holds 2^-14 .. 65504, so the scale puts the
// largest |x'| of a row (or the proven bound of a head's values) just under
// 2^14; a piece below 2^-14 is subnormal with an absolute error <= 2^-25,
// i.e. <= 2^-38 of the row's largest element.
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

namespace nos {

// x (2 lanes of a pair, already scaled) -> hi / lo fp16 pieces.  The lo
// pair is two mixed-precision FMAs, f16(x - 1.0 * hi) with hi read as fp16
// (v_fma_mixlo_f16 / v_fma_mixhi_f16: one rounding of the exact difference,
// the same value as converting x - (float)hi), instead of two fp16 -> fp32
// conversions, two subtractions and a pack.
__device__ __forceinline__ void split2h(f32x2_t x, f16x2_t& hi, f16x2_t& lo) {
  hi = __builtin_convertvector(x, f16x2_t);
  const unsigned hb = __builtin_bit_cast(unsigned, hi);
  unsigned lb;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lb)
      : "v"(x.x), "v"(hb), "v"(x.y));
  lo = __builtin_bit_cast(f16x2_t, lb);
}

// acc += a.b as the three piece products, smallest first (a: A operand)
__device__ __forceinline__ f32x16_t mma3h(const f16x8_t (&a)[2], const f16x8_t (&b)[2], f32x16_t acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

// 2^e as a float for |e| <= 126 (exact power of two)
__device__ __forceinline__ float pow2i(int e) { return __int_as_float((e + 127) << 23); }

// exponent of the scale that puts |v| <= vmax just under 2^14: vmax * 2^e < 2^14
// (clamped to +-126 so 2^e and 2^-e are normal floats; vmax == 0 -> 0)
__device__ __forceinline__ int h3_scale_exp(float vmax) {
  if (!(vmax > 0.f)) return 0;
  int e;
  frexpf(vmax, &e);  // vmax = f 2^e, f in [0.5, 1): vmax < 2^e
  e = 14 - e;
  return e < -126 ? -126 : (e > 126 ? 126 : e);
}

}  // namespace nos
