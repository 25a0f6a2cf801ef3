# variant: skip the per-tile row max.  p = exp2(s*c - m) against the current
# reference max; a lane whose 32 p's sum above 2^THR (so some score may exceed
# m + THR, or a score overflowed) sends the wave to the rare path, which recomputes
# S (8 MFMAs from the K tile still in LDS), takes the exact max, rescales and
# redoes the exponentials.  Two partial sums; loop unrolled by 2 so the LDS ring
# slot folds into the immediate offsets.
import sys
p = sys.argv[1] + "/attention.hip" if len(sys.argv) > 1 else "/root/repo/csrc/hip/attention.hip"
s = open(p).read()
a = s.index("      f32x16_t sacc[2];\n#pragma unroll\n      for (int kb = 0; kb < 2; ++kb) {")
b = s.index("      bf16x8_t pf[2][2];")
body = '''      f32x16_t sacc[2];
      auto qk = [&]() {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[kb][i] = 0.f;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(kl + koff[ks] + kb * 32 * 128);
            sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], sacc[kb], 0, 0, 0);
          }
        }
        if ((t + 1) * KVBLK > Skv) {
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int kv = t * KVBLK + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
              if (kv >= Skv) sacc[kb][i] = -INFINITY;
            }
        }
      };
      auto expsum = [&](float& s0, float& s1) {
        s0 = 0.f;
        s1 = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[0][i], c, -m));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[1][i], c, -m));
          sacc[0][i] = p0;
          sacc[1][i] = p1;
          s0 += p0;
          s1 += p1;
        }
      };
      qk();
      float ps0, ps1;
      bool redo = it == 0;
      if (!redo) {
        expsum(ps0, ps1);
        // every p <= sum of the lane's p's: a sum within 2^THR bounds them all
        redo = !__all(ps0 + ps1 <= RESCALE_LIM);
      }
      if (redo) {
        qk();
        float mt = sacc[0][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mt = fmaxf(mt, sacc[0][i]);
#pragma unroll
        for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sacc[1][i]);
        const float mrel = fmaf(xor32_max(mt), c, -m);
        const float delta = it == 0 ? mrel : fmaxf(mrel, 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        m += delta;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          oacc[0][i] *= alpha;
          oacc[1][i] *= alpha;
        }
        expsum(ps0, ps1);
      }
      l += ps0 + ps1;

'''
s = s[:a] + body + s[b:]
s = s.replace("constexpr float RESCALE_THR = 8.f;          // log2 units",
              "constexpr float RESCALE_THR = 8.f;          // log2 units\nconstexpr float RESCALE_LIM = 256.f;        // 2^RESCALE_THR")
s = s.replace("  for (int it = 0; it < niters; ++it) {\n    const int buf = it & 1;",
              "#pragma unroll 2\n  for (int it = 0; it < niters; ++it) {\n    const int buf = it & 1;")
open(p, "w").write(s)
