// bf16 GEMM with fused epilogue for gfx950:  C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ R)
//
// This is the "linear layer" of the tenant models (W in nn.Linear [out, in]
// layout) and the body of the gpuagent's MFMA probe (probe_mfma_bf16 runs it
// persistently on a CU-masked stream to price a slice).
//
// CDNA4 design:
//  * 256-thread workgroup (4 waves as 2x2), output tile 128x128, each wave
//    64x64 = 2x2 blocks of v_mfma_f32_32x32x16_bf16, BK = 64;
//  * both operands are K-contiguous, so both are staged the same way: direct
//    global->LDS DMA (global_load_lds_dwordx4, 1 KiB = 8 rows per wave
//    instruction) into a lane-linear image; the XOR swizzle that makes the
//    ds_read_b128 fragment reads conflict-free is applied to the per-lane
//    SOURCE address (linear destination + inverse-swizzled source + swizzled
//    read);
//  * two LDS buffers (64 KiB): tile k+1 is in flight while tile k is consumed;
//  * optional persistent mode (grid smaller than the tile count) with an
//    XCD-aware tile order so neighbouring tiles share an XCD's L2;
//  * epilogue fuses bias, exact-erf GELU and a residual add, bf16 out.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;
constexpr int TILE_A_BYTES = BM * BK * 2;  // 16 KiB
constexpr int TILE_B_BYTES = BN * BK * 2;  // 16 KiB
constexpr int STAGE_BYTES = TILE_A_BYTES + TILE_B_BYTES;

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8 };

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Stage a [128 rows][64 k] bf16 tile: 16 wave-instructions, 4 per wave.
__device__ __forceinline__ void stage_tile(const unsigned short* __restrict__ src, int ld,
                                           int row0, int nrows, int k0,
                                           unsigned char* tile, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int R = (wid * 4 + i) * 8;
    const int row = R + (lane >> 3);
    const int pc = lane & 7;
    const int lc = pc ^ swz(row);
    int grow = row0 + row;
    grow = grow < nrows ? grow : nrows - 1;
    glds16(src + (long long)grow * ld + k0 + lc * 8, tile + R * 128);
  }
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}

__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(
    const unsigned short* __restrict__ A, int lda, const unsigned short* __restrict__ W, int ldw,
    const unsigned short* __restrict__ bias, const unsigned short* __restrict__ R, int ldr,
    unsigned short* __restrict__ C, int ldc, int M, int N, int K, int epi, int tiles_m,
    int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / BK;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // XCD-aware order: consecutive tiles (same W panel) share an XCD
    const int tt = (gridDim.x >= ntiles) ? nos::xcd_remap(tile, ntiles) : tile;
    const int tn = tt / tiles_m;  // column-panel major: tiles of one W panel adjacent
    const int tm = tt - tn * tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

    f32x16_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    stage_tile(A, lda, m0, M, 0, smem, wid, lane);
    stage_tile(W, ldw, n0, N, 0, smem + TILE_A_BYTES, wid, lane);
    __syncthreads();  // drains the DMA (vmcnt(0)) and publishes the tile

    for (int kt = 0; kt < nk; ++kt) {
      unsigned char* cur = smem + (kt & 1) * STAGE_BYTES;
      if (kt + 1 < nk) {
        unsigned char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
        stage_tile(A, lda, m0, M, (kt + 1) * BK, nxt, wid, lane);
        stage_tile(W, ldw, n0, N, (kt + 1) * BK, nxt + TILE_A_BYTES, wid, lane);
      }
      const unsigned char* ta = cur;
      const unsigned char* tb = cur + TILE_A_BYTES;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8_t af[2], bf[2];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int row = wm * 64 + mi * 32 + r;
          af[mi] = *reinterpret_cast<const bf16x8_t*>(ta + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const int row = wn * 64 + ni * 32 + r;
          bf[ni] = *reinterpret_cast<const bf16x8_t*>(tb + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
      }
      __syncthreads();  // next tile landed; everyone done with `cur`
    }

    // ---- fused epilogue
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int n = n0 + wn * 64 + ni * 32 + r;
      if (n >= N) continue;
      const float bv = (epi & EPI_BIAS) ? nos::bf16_to_f32(bias[n]) : 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = m0 + wm * 64 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (m >= M) continue;
          float x = acc[mi][ni][i] + bv;
          if (epi & EPI_GELU) x = gelu_erf(x);
          if (epi & EPI_RELU) x = fmaxf(x, 0.f);
          if (epi & EPI_RESID) x += nos::bf16_to_f32(R[(long long)m * ldr + n]);
          C[(long long)m * ldc + n] = nos::f32_to_bf16(x);
        }
    }
  }
}

}  // namespace

// C = act(A . W^T + bias) (+ R).  A [M,K] (row stride lda), W [N,K] (ldw),
// R/C [M,N] (ldr/ldc), all bf16.  K must be a multiple of 64 and every row
// start 16-byte aligned.  max_wg > 0 caps the grid (persistent mode).
NOS_API int nos_gemm_bf16(const void* A, int lda, const void* W, int ldw, const void* bias,
                          const void* R, int ldr, void* C, int ldc, int M, int N, int K, int epi,
                          int max_wg, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && !R) return (int)hipErrorInvalidValue;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  int nwg = tiles_m * tiles_n;
  if (max_wg > 0 && nwg > max_wg) nwg = max_wg;
  hipLaunchKernelGGL(gemm_bf16_kernel, dim3(nwg), dim3(NT), 2 * STAGE_BYTES, stream,
                     (const unsigned short*)A, lda, (const unsigned short*)W, ldw,
                     (const unsigned short*)bias, (const unsigned short*)R, ldr,
                     (unsigned short*)C, ldc, M, N, K, epi, tiles_m, tiles_n);
  return (int)hipGetLastError();
}
