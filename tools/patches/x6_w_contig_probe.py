"""TIMING PROBE ONLY (wrong results): the x6 GEMM's W-plane DMA reads one
contiguous 1 KiB block per wave instruction (as a pre-tiled weight layout
would) instead of 16 rows x 64 B at the row stride; the LDS images and all
math are unchanged.  Tells whether the W pieces' line count limits the
GEMM before implementing the tiled layout.
  python tools/build_variant.py wcontig tools/patches/x6_w_contig_probe.py \\
      gemm_f32x.hip=-fno-slp-vectorize attention_f32x.hip=-fno-slp-vectorize"""
import sys
from pathlib import Path

p = Path(sys.argv[1]) / "gemm_f32x.hip"
s = p.read_text()
old = """      glds16(Wp + plane * wplane + (long long)gn * ldw + k0 + (((lane % WCH) ^ L::wswz(row)) << 3),
             dst + TA + plane * TWP + rb * WROW);"""
new = """      (void)gn;
      const long long blk = (long long)(min(n0 + rb, N - WRPI) / WRPI) * (K / BK) + k0 / BK;
      glds16(Wp + plane * wplane + blk * (WRPI * BK) + lane * 8, dst + TA + plane * TWP + rb * WROW);"""
assert old in s
p.write_text(s.replace(old, new))
