"""Variant: the bf16x6 kernels' fp32 -> three-bf16 split and the x6
attention's softmax as scalar f32 ops (no v_pk_add_f32 beside the MFMAs).
Build with -fno-slp-vectorize for gemm_f32x.hip and attention_f32x.hip:
  python tools/build_variant.py x6scalar tools/patches/x6_scalar_split.py \\
      gemm_f32x.hip=-fno-slp-vectorize attention_f32x.hip=-fno-slp-vectorize"""
import sys
from pathlib import Path

src = Path(sys.argv[1])
p = src / "split_bf16.h"
s = p.read_text()
old = """  p0 = __builtin_convertvector(x, bf16x2_t);
  const f32x2_t r1 = x - __builtin_convertvector(p0, f32x2_t);
  p1 = __builtin_convertvector(r1, bf16x2_t);
  const f32x2_t r2 = r1 - __builtin_convertvector(p1, f32x2_t);
  p2 = __builtin_convertvector(r2, bf16x2_t);"""
new = """  p0 = __builtin_convertvector(x, bf16x2_t);
  const float r1x = x.x - (float)p0.x, r1y = x.y - (float)p0.y;
  p1 = __builtin_convertvector(f32x2_t{r1x, r1y}, bf16x2_t);
  const float r2x = r1x - (float)p1.x, r2y = r1y - (float)p1.y;
  p2 = __builtin_convertvector(f32x2_t{r2x, r2y}, bf16x2_t);"""
assert old in s
p.write_text(s.replace(old, new))
p = src / "attention_f32x.hip"
s = p.read_text()
old = """      f32x2_t ps2 = {0.f, 0.f};
      const f32x2_t nm2 = {-m, -m};
#pragma unroll
      for (int j2 = 0; j2 < 8; ++j2) {
        f32x2_t x = f32x2_t{s[2 * j2], s[2 * j2 + 1]} + nm2;
        x.x = __builtin_amdgcn_exp2f(x.x);
        x.y = __builtin_amdgcn_exp2f(x.y);
        ps2 += x;
        bf16x2_t a, bb, cc;
        nos::split2(x, a, bb, cc);"""
new = """      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j2 = 0; j2 < 8; ++j2) {
        const float x0 = __builtin_amdgcn_exp2f(s[2 * j2] - m);
        const float x1 = __builtin_amdgcn_exp2f(s[2 * j2 + 1] - m);
        ls[(2 * j2) & 3] += x0;
        ls[(2 * j2 + 1) & 3] += x1;
        const f32x2_t x = {x0, x1};
        bf16x2_t a, bb, cc;
        nos::split2(x, a, bb, cc);"""
assert old in s
s = s.replace(old, new)
old = """      l += ps2.x + ps2.y;"""
assert old in s
p.write_text(s.replace(old, """      l += (ls[0] + ls[1]) + (ls[2] + ls[3]);"""))
