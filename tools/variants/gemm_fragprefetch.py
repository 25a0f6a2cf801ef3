# variant: read every fragment of the k-tile (16 x ds_read_b128) before the 16 MFMAs
import sys
p = sys.argv[1] + "/gemm.hip"
s = open(p).read()
old = s[s.index("#pragma unroll\n      for (int ks = 0; ks < BK / 16; ++ks) {\n        bf16x8_t af[2], bf[NB];"):s.index("      __syncthreads();  // next tile landed; everyone done with `cur`")]
new = '''      bf16x8_t af[BK / 16][2], bf[BK / 16][NB];
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int row = wm * 64 + mi * 32 + r;
          af[ks][mi] = *reinterpret_cast<const bf16x8_t*>(ta + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < NB; ++ni) {
          const int row = wn * WN + ni * 32 + r;
          bf[ks][ni] = *reinterpret_cast<const bf16x8_t*>(tb + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
      }
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks][mi], bf[ks][ni], acc[mi][ni], 0, 0, 0);
'''
s = s.replace(old, new)
open(p, "w").write(s)
