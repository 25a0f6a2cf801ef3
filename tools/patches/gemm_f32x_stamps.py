"""Stamp patch for tools/build_variant.py: s_memtime phase stamps in the x6
fp32 GEMM (prologue / wait+barrier / DMA issue / compute / epilogue), summed
per wave into a device array of their own; read by tools/gemm_stamps.py.
The stamps serialise the stream (lgkmcnt waits): read the split, not the time."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "gemm_f32x.hip"
s = p.read_text()
def rep(a, b):
    global s
    assert a in s, a
    s = s.replace(a, b, 1)
rep("namespace {\n\nconstexpr int NT = 256;", "__device__ unsigned long long g_st[8];\nnamespace {\n\nconstexpr int NT = 256;")
rep("  for (int tt = chunk.first; tt < chunk.end; tt += chunk.step) {",
    "  unsigned long long st_w = 0, st_d = 0, st_c = 0, st_e = 0, st_p = 0, t_prev = __builtin_readcyclecounter(), t_now;\n"
    "#define STAMP(acc) do { t_now = __builtin_readcyclecounter(); acc += t_now - t_prev; t_prev = t_now; } while (0)\n"
    "  for (int tt = chunk.first; tt < chunk.end; tt += chunk.step) {")
rep("  for (int kt = 0; kt < nk; ++kt) {\n", "  STAMP(st_p);\n  for (int kt = 0; kt < nk; ++kt) {\n")
rep("    __builtin_amdgcn_s_barrier();\n", "    __builtin_amdgcn_s_barrier();\n    STAMP(st_w);\n")
rep("    if (kt > 0 && kt + S - 1 < nk) stage((kt + S - 1) * BK, smem + (S == 2 ? slot ^ 1 : (kt + S - 1) % S) * STAGE);\n",
    "    if (kt > 0 && kt + S - 1 < nk) stage((kt + S - 1) * BK, smem + (S == 2 ? slot ^ 1 : (kt + S - 1) % S) * STAGE);\n    STAMP(st_d);\n")
rep("    }\n  }\n  __syncthreads();  // every wave is done with the ring", "    }\n    STAMP(st_c);\n  }\n  __syncthreads();  // every wave is done with the ring")
rep("  }  // tiles\n", "  STAMP(st_e);\n  }  // tiles\n  if ((threadIdx.x & 63) == 0) {\n    atomicAdd(&g_st[0], st_p); atomicAdd(&g_st[1], st_w); atomicAdd(&g_st[2], st_d);\n    atomicAdd(&g_st[3], st_c); atomicAdd(&g_st[4], st_e); atomicAdd(&g_st[5], 1ull);\n  }\n")
s += '''
NOS_API int nos_gemm_f32x6_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_st), sizeof(unsigned long long) * 8, 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return (int)e;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_st), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return (int)e;
}
'''
p.write_text(s)
