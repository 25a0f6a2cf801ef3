# variant: per 32-key half: softmax(kb) overlaps QK MFMAs of kb+1 and PV(kb) overlaps softmax(kb+1)
# MEASURED (r01, graph-timed, S=3401 H=6): 40.98 us vs 39.10 us for the base kernel -> not adopted.
import sys
p = sys.argv[1] + "/attention.hip" if len(sys.argv) > 1 else "/root/repo/csrc/hip/attention.hip"
s = open(p).read()
a = s.index("      if ((t + 1) * KVBLK > Skv) {")
b = s.index("    __syncthreads();  // next stage landed (vmcnt(0)); everyone done with `buf`")
new = '''      if ((t + 1) * KVBLK > Skv) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kv = t * KVBLK + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (kv >= Skv) sacc[kb][i] = -INFINITY;
          }
      }
      // per 32-key half: softmax(half 0) runs while the QK^T MFMAs of half 1
      // are in flight, PV(half 0) while softmax(half 1) runs.  The deferred
      // rescale works per half (the first half of a group's first tile sets
      // the reference max; half 0 always has a valid key).
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        float mt = sacc[kb][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mt = fmaxf(mt, sacc[kb][i]);
        const float mrel = fmaf(xor32_max(mt), c, -m);  // half max - m (log2 units)
        const bool first = it == 0 && kb == 0;
        if (first || !__all(mrel <= RESCALE_THR)) {
          const float delta = first ? mrel : fmaxf(mrel, 0.f);
          const float alpha = __builtin_amdgcn_exp2f(-delta);
          m += delta;
          l *= alpha;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            oacc[0][i] *= alpha;
            oacc[1][i] *= alpha;
          }
        }
        float psum = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kb][i], c, -m));
          sacc[kb][i] = p;
          psum += p;
        }
        l += psum;
        bf16x8_t pf[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[s2][j] = (__bf16)sacc[kb][8 * s2 + j];
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const unsigned char* base = vl + voff[db] + (kb * 32 + s2 * 16) * 128;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + 8 * 128));
            const s16x8_t a16 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a16), pf[s2],
                                                               oacc[db], 0, 0, 0);
          }
      }
    }
'''
s = s[:a] + new + s[b:]
open(p, "w").write(s)
