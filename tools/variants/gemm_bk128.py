"""Variant: the register-epilogue GEMM with BK = 128 (256-byte rows, chunk
swizzle c ^ (row & 15), 2 stages = 128 KiB LDS, one workgroup per CU) for
K % 128 == 0; other K keep the BK-64 kernel."""
import sys

p = sys.argv[1] + "/gemm.hip"
s = open(p).read()
a = s.find("template <bool LN, int BN, bool RESID>\n__global__ __launch_bounds__(NT, 2) void gemm_bf16_rk_kernel(")
b = s.find("int g_epi_impl = 1;")
assert a > 0 and b > a
k = s[a:b]
k = k.replace("gemm_bf16_rk_kernel(", "gemm_bf16_k128_kernel(")
k = k.replace("__launch_bounds__(NT, 2)", "__launch_bounds__(NT, 1)")
k = k.replace("  constexpr int STAGE_BYTES = CF::STAGE_BYTES;", "  constexpr int STAGE_BYTES = (BM + BN) * 256;")
k = k.replace("const int nk = K / BK;", "const int nk = K / 128;")
k = k.replace("stage_tile<BM>(A, lda, m0, M, 0, smem, wid, lane);", "stage_tile128<BM>(A, lda, m0, M, 0, smem, wid, lane);")
k = k.replace("stage_tile<BN>(W, ldw, n0, N, 0, smem + TILE_A_BYTES, wid, lane);",
              "stage_tile128<BN>(W, ldw, n0, N, 0, smem + BM * 256, wid, lane);")
k = k.replace("stage_tile<BM>(A, lda, m0, M, (kt + 1) * BK, nxt, wid, lane);",
              "stage_tile128<BM>(A, lda, m0, M, (kt + 1) * 128, nxt, wid, lane);")
k = k.replace("stage_tile<BN>(W, ldw, n0, N, (kt + 1) * BK, nxt + TILE_A_BYTES, wid, lane);",
              "stage_tile128<BN>(W, ldw, n0, N, (kt + 1) * 128, nxt + BM * 256, wid, lane);")
k = k.replace("const unsigned char* tb = cur + TILE_A_BYTES;", "const unsigned char* tb = cur + BM * 256;")
k = k.replace("""        for (int c = 0; c < 4; ++c) {
          const int lc = shalf * 4 + c;
          const s16x8_t v = *reinterpret_cast<const s16x8_t*>(ta + srow * 128 + ((lc ^ swz(srow)) << 4));""",
              """        for (int c = 0; c < 8; ++c) {
          const int lc = shalf * 8 + c;
          const s16x8_t v = *reinterpret_cast<const s16x8_t*>(ta + srow * 256 + ((lc ^ (srow & 15)) << 4));""")
k = k.replace("for (int ks = 0; ks < BK / 16; ++ks) {", "for (int ks = 0; ks < 128 / 16; ++ks) {")
k = k.replace("ta + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4)", "ta + row * 256 + (((2 * ks + hh) ^ (row & 15)) << 4)")
k = k.replace("tb + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4)", "tb + row * 256 + (((2 * ks + hh) ^ (row & 15)) << 4)")
assert "swz(" not in k and "TILE_A_BYTES" not in k and " BK" not in k, k
helper = '''
template <int ROWS>
__device__ __forceinline__ void stage_tile128(const unsigned short* __restrict__ src, int ld, int row0,
                                              int nrows, int k0, unsigned char* tile, int wid, int lane) {
  constexpr int PER_WAVE = ROWS / 16;  // 4 rows of 256 B per wave-instruction
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int R0 = (wid * PER_WAVE + i) * 4;
    const int row = R0 + (lane >> 4);
    const int lc = (lane & 15) ^ (row & 15);
    int grow = row0 + row;
    grow = grow < nrows ? grow : nrows - 1;
    glds16(src + (long long)grow * ld + k0 + lc * 8, tile + R0 * 256);
  }
}

'''
s = s[:b] + helper + k + "\n" + s[b:]
s = s.replace("""    if (g_epi_impl == 1)                                                                                    \\
      hipLaunchKernelGGL((gemm_bf16_rk_kernel<LNV, BNV, RV>), dim3(nwg), dim3(NT), rk_lds_bytes<BNV>(),     \\
                         stream, NOS_GEMM_ARGS);                                                            \\""",
              """    if (g_epi_impl == 1 && (K % 128) == 0)                                                                  \\
      hipLaunchKernelGGL((gemm_bf16_k128_kernel<LNV, BNV, RV>), dim3(nwg), dim3(NT),                        \\
                         2 * (BM + BNV) * 256 + (2 * BM + 2 * BNV) * 4, stream, NOS_GEMM_ARGS);             \\
    else if (g_epi_impl == 1)                                                                               \\
      hipLaunchKernelGGL((gemm_bf16_rk_kernel<LNV, BNV, RV>), dim3(nwg), dim3(NT), rk_lds_bytes<BNV>(),     \\
                         stream, NOS_GEMM_ARGS);                                                            \\""")
assert "gemm_bf16_k128_kernel<LNV" in s
open(p, "w").write(s)
