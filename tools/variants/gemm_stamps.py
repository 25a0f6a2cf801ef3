"""Diagnostic variant: s_memtime stamps in the register-epilogue GEMM.

Per workgroup (first tile only), lane 0 of wave 0 records: kernel entry,
prologue landed, K-loop done, LN statistics done, epilogue done, plus
s_memrealtime at entry / exit (100 MHz) to convert cycles to time.  Read back
with nos_dbg_read().  The stamps go to a buffer of their own (never to an
output).  Build: python tools/build_variant.py stamps tools/variants/gemm_stamps.py
"""
import sys

p = sys.argv[1] + "/gemm.hip"
s = open(p).read()
a = s.find("void gemm_bf16_rk_kernel(")
assert a > 0
head, body = s[:a], s[a:]
rep = [
    ("  const bool vec_ok = ((ldc | ldr) & 7) == 0;\n",
     "  const bool vec_ok = ((ldc | ldr) & 7) == 0;\n"
     "  const unsigned long long T0 = __builtin_amdgcn_s_memtime(), R0 = __builtin_amdgcn_s_memrealtime();\n"
     "  unsigned long long T1 = 0, T2 = 0, T3 = 0;\n"),
    ("      s_p2[tid] = LN ? c2[n] : ((epi & EPI_BIAS) ? nos::bf16_to_f32(bias[n]) : 0.f);\n    }\n    __syncthreads();\n",
     "      s_p2[tid] = LN ? c2[n] : ((epi & EPI_BIAS) ? nos::bf16_to_f32(bias[n]) : 0.f);\n    }\n    __syncthreads();\n"
     "    T1 = __builtin_amdgcn_s_memtime();\n"),
    ("    if constexpr (LN) {\n      const float sh_lo",
     "    T2 = __builtin_amdgcn_s_memtime();\n    if constexpr (LN) {\n      const float sh_lo"),
    ("    epilogue_rows<LN, BN, RESID>(",
     "    T3 = __builtin_amdgcn_s_memtime();\n    epilogue_rows<LN, BN, RESID>("),
    ("    // LDS (stages, stats, params) is rewritten by the next persistent tile; a\n",
     "    if (tid == 0 && tile == (int)blockIdx.x && blockIdx.x < 4096) {\n"
     "      const unsigned long long T4 = __builtin_amdgcn_s_memtime(), R4 = __builtin_amdgcn_s_memrealtime();\n"
     "      unsigned long long* d = g_dbg + blockIdx.x * 8;\n"
     "      d[0] = T0; d[1] = T1; d[2] = T2; d[3] = T3; d[4] = T4; d[5] = R0; d[6] = R4;\n"
     "      unsigned xcc; asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc)); d[7] = xcc;\n"
     "    }\n"
     "    // LDS (stages, stats, params) is rewritten by the next persistent tile; a\n"),
]
for old, new in rep:
    assert old in body, old
    body = body.replace(old, new, 1)
s = head + body
s = s.replace("namespace {\n", "namespace {\n__device__ unsigned long long g_dbg[4096 * 8];\n", 1)
s += """
NOS_API int nos_dbg_read(void* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbg), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
"""
open(p, "w").write(s)
