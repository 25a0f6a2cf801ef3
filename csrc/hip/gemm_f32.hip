// Exact-fp32 GEMM with fused LayerNorm / bias / GELU / ReLU / residual for the
// fp32 YOLOS pods (the reference demo's precision):
//
//   plain:     C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ R)
//   LN-fused:  C[M,N] = act(LayerNorm(A) . W^T + bias), via the folded form
//              rstd * (A . (W*gamma)^T - mu * c1) + c2 (see gemm.hip; K == hidden)
//
// gfx950 has an exact f32-input MFMA (v_mfma_f32_32x32x2_f32, fmaf-chain
// numerics, 64 FLOP/clk/SIMD) and no xf32: fp32 GEMMs are matrix-pipe bound
// at 1/16 of bf16, so the design is about keeping that pipe busy:
//
//  * 4 waves (2 x 2) per workgroup, tile BM x BN (128x128, 64x128 or 64x64,
//    chosen per shape by the tile policy), each wave (BM/2) x (BN/2) as 32x32
//    MFMA blocks, BK = 32 fp32 per stage;
//  * both operands are K-contiguous and staged the same way: LDS-DMA
//    (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per wave instruction)
//    into a 2-deep ring (a 3-deep ring measured slower: the extra LDS costs a
//    workgroup per CU), the 16-byte chunks of row r XOR-swizzled by r & 7 on
//    the SOURCE address so the fragment reads (ds_read_b128) are conflict-free;
//  * MFMA k mapping k = kk + 16h (h = lane >> 5): a lane's A / W fragment for
//    a whole stage is 64 contiguous bytes of its row (4 x ds_read_b128);
//  * epilogue in registers: accumulator register i of lane (c, h) is output
//    row (i&3) + 8(i>>2) + 4h, column c -- 32 lanes store 128 contiguous bytes
//    per register; LayerNorm row statistics are accumulated from the A tiles
//    already in LDS (no second pass over A).
#include "common.h"

namespace {

constexpr int BK = 32;              // fp32 per stage row chunk = 128 B
constexpr int NT = 256;
constexpr int ROWB = BK * 4;        // 128 B per staged row
enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8 };

__device__ __forceinline__ int swz(int row) { return row & 7; }

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// [ROWS][32 k] fp32 tile: ROWS/8 wave-instructions spread over the 4 waves
template <int ROWS>
__device__ __forceinline__ void stage_tile(const float* __restrict__ src, int ld, int row0, int nrows, int k0,
                                           unsigned char* tile, int wid, int lane) {
  constexpr int PIECES = ROWS / 8;
#pragma unroll
  for (int p = wid; p < PIECES; p += 4) {
    const int R = p * 8;
    const int row = R + (lane >> 3);
    const int lc = (lane & 7) ^ swz(row);
    int grow = row0 + row;
    grow = grow < nrows ? grow : nrows - 1;
    glds16(src + (long long)grow * ld + k0 + lc * 4, tile + R * ROWB);
  }
}

__device__ __forceinline__ float erf_fast(float x) {  // Abramowitz-Stegun 7.1.26, |err| <= 1.5e-7
  const float ax = fabsf(x);
  const float t = 1.f / fmaf(0.3275911f, ax, 1.f);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float r = fmaf(-p * t, expf(-ax * ax), 1.f);
  return copysignf(r, x);
}

// PERSIST: the slice-sized-grid instantiation (a chunk of tiles per
// workgroup); the one-tile instantiation compiles the loop away and keeps the
// register budget of a plain tile kernel
template <bool LN, int BM, int BN, bool PERSIST>
__global__ __launch_bounds__(NT, 2) void gemm_f32_kernel(
    const float* __restrict__ A, int lda, const float* __restrict__ W, int ldw, const float* __restrict__ bias,
    const float* __restrict__ c1, const float* __restrict__ c2, const float* __restrict__ R, int ldr,
    float* __restrict__ C, int ldc, int M, int N, int K, int epi, float eps, int tiles_m, int tiles_n) {
  constexpr int TA = BM * ROWB, TB = BN * ROWB, STAGE = TA + TB;
  constexpr int MI = BM / 64, NI = BN / 64;  // 32x32 blocks per wave (waves are 2 x 2)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + 2 * STAGE);
  float* s_rstd = s_mu + BM;

  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int c = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / BK;
  // one tile per workgroup, or -- with a slice-sized grid -- a chunk of tiles
  // per workgroup (nos::xcd_chunk); tiles of one A panel share an XCD's L2
  nos::XcdChunk chunk;
  if constexpr (PERSIST) {
    chunk = nos::xcd_chunk(blockIdx.x, gridDim.x, ntiles);
  } else {
    chunk.first = nos::xcd_remap(blockIdx.x, ntiles);
    chunk.end = chunk.first + 1;
    chunk.step = 1;
  }
  for (int tt = chunk.first; tt < chunk.end; tt += chunk.step) {
  if (PERSIST && tt != chunk.first) __syncthreads();  // the previous tile's ring and LN statistics are free
  const int tm = tt / tiles_n, tn = tt - tm * tiles_n;  // row-major
  const int m0 = tm * BM, n0 = tn * BN;

  f32x16_t acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // LN statistics: BM rows, NT / BM threads per row, each 32 / (NT/BM) floats per stage
  constexpr int TPR = NT / BM;           // 2 (BM 128) or 4 (BM 64)
  constexpr int FPT = BK / TPR;          // floats per thread per stage: 16 or 8
  const int srow = tid / TPR, spart = tid % TPR;
  float sshift = 0.f, ssum = 0.f, ssq = 0.f;

  stage_tile<BM>(A, lda, m0, M, 0, smem, wid, lane);
  stage_tile<BN>(W, ldw, n0, N, 0, smem + TA, wid, lane);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* cur = smem + (kt & 1) * STAGE;
    if (kt + 1 < nk) {  // the other buffer was released by the barrier that ended step kt-1
      unsigned char* nxt = smem + ((kt + 1) & 1) * STAGE;
      stage_tile<BM>(A, lda, m0, M, (kt + 1) * BK, nxt, wid, lane);
      stage_tile<BN>(W, ldw, n0, N, (kt + 1) * BK, nxt + TA, wid, lane);
    }
    const unsigned char* ta = cur;
    const unsigned char* tb = cur + TA;
    if constexpr (LN) {
#pragma unroll
      for (int q = 0; q < FPT / 4; ++q) {
        const int lc = spart * (FPT / 4) + q;
        const float4 v = *reinterpret_cast<const float4*>(ta + srow * ROWB + ((lc ^ swz(srow)) << 4));
        if (kt == 0 && q == 0) sshift = v.x;
        const float d0 = v.x - sshift, d1 = v.y - sshift, d2 = v.z - sshift, d3 = v.w - sshift;
        ssum += (d0 + d1) + (d2 + d3);
        ssq = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, ssq))));
      }
    }
    float af[MI][16], bf[NI][16];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * (BM / 2) + i * 32 + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(ta + row * ROWB + (((4 * h + q) ^ swz(row)) << 4));
        af[i][4 * q + 0] = v.x;
        af[i][4 * q + 1] = v.y;
        af[i][4 * q + 2] = v.z;
        af[i][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int row = wn * (BN / 2) + j * 32 + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(tb + row * ROWB + (((4 * h + q) ^ swz(row)) << 4));
        bf[j][4 * q + 0] = v.x;
        bf[j][4 * q + 1] = v.y;
        bf[j][4 * q + 2] = v.z;
        bf[j][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][kk], bf[j][kk], acc[i][j], 0, 0, 0);
    __syncthreads();  // next stage landed (vmcnt(0)); every wave is done with this one
  }

  if constexpr (LN) {
    // combine the TPR partial (shifted) sums of a row; shifts differ per thread
    const float kpart = (float)(K / TPR);
    float mu_part = sshift + ssum / kpart;                     // this part's mean
    float m2_part = ssq - ssum * ssum / kpart;                 // this part's sum of squared deviations
    float mean = mu_part, m2 = m2_part, cnt = kpart;
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) {                        // Chan's parallel combination
      const float om = __shfl_xor(mean, o, 64), om2 = __shfl_xor(m2, o, 64), oc = __shfl_xor(cnt, o, 64);
      const float tot = cnt + oc, dl = om - mean;
      mean = mean + dl * (oc / tot);
      m2 = m2 + om2 + dl * dl * (cnt * oc / tot);
      cnt = tot;
    }
    if (spart == 0) {
      s_mu[srow] = mean;
      s_rstd[srow] = rsqrtf(fmaxf(m2 / (float)K, 0.f) + eps);
    }
    __syncthreads();
  }

  // epilogue: register i of lane (c, h) = row (i&3) + 8(i>>2) + 4h of the block, column c
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 32 + c;
    const int nc = n < N ? n : N - 1;
    const float p1 = LN ? c1[nc] : 0.f;
    const float p2 = LN ? c2[nc] : ((epi & EPI_BIAS) ? bias[nc] : 0.f);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int m = m0 + rl;
        float v = acc[i][j][r];
        if constexpr (LN) v = fmaf(s_rstd[rl], v - s_mu[rl] * p1, p2);
        else v += p2;
        if (epi & EPI_GELU) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
        if (epi & EPI_RELU) v = fmaxf(v, 0.f);
        if (m < M && n < N) {
          if (epi & EPI_RESID) v += R[(long long)m * ldr + n];
          C[(long long)m * ldc + n] = v;
        }
      }
    }
  }
  }  // tiles
}

template <bool LN, int BM, int BN>
int launch_t(const float* A, int lda, const float* W, int ldw, const float* bias, const float* c1, const float* c2,
             const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi, float eps, hipStream_t st) {
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const long long ntiles = (long long)tiles_m * tiles_n;
  if (ntiles > (1LL << 30)) return (int)hipErrorInvalidValue;
  const size_t lds = 2 * (size_t)(BM + BN) * ROWB + 2 * BM * sizeof(float);
  const int grid = nos_grid_for((const void*)gemm_f32_kernel<LN, BM, BN, true>, NT, lds, ntiles);
  if (grid < ntiles)
    hipLaunchKernelGGL((gemm_f32_kernel<LN, BM, BN, true>), dim3((unsigned)grid), dim3(NT), lds, st, A, lda, W, ldw,
                       bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, tiles_m, tiles_n);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<LN, BM, BN, false>), dim3((unsigned)ntiles), dim3(NT), lds, st, A, lda, W,
                       ldw, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, tiles_m, tiles_n);
  return (int)hipGetLastError();
}

// Tile policy (nos_gemm_f32_set_policy):
//  * 0 = throughput: the most MFMA-efficient tile that fits the shape --
//    other pods fill the CUs a small grid leaves idle;
//  * 1 = latency (default): the tile minimising
//    rounds x per-tile time, with workgroups per CU {2, 3, 4} and relative
//    per-FLOP efficiency {1.0, 0.9, 0.75} for 128x128 / 64x128 / 64x64;
//  * 2 = small: always 64x64 (33 KB of LDS, <= 64 VGPRs: the most room for
//    co-running pods' workgroups on a CU).
int g_policy = 1;

int pick_tile(int M, int N) {
  if (g_policy == 2) return 2;
  if (g_policy == 0) {
    if (M >= 128 && N >= 128) return 0;
    if (N >= 128) return 1;
    return 2;
  }
  const int bm[3] = {128, 64, 64}, bn[3] = {128, 128, 64}, per_cu[3] = {2, 3, 4};
  const double eff[3] = {1.0, 0.9, 0.75};
  const long long cus = nos_effective_cus();  // a CU-mask slice plans for its own CUs
  int best = 2;
  double best_cost = 1e300;
  for (int c = 0; c < 3; ++c) {
    const long long tiles = (long long)((M + bm[c] - 1) / bm[c]) * ((N + bn[c] - 1) / bn[c]);
    const long long slots = cus * per_cu[c];
    const long long rounds = (tiles + slots - 1) / slots;
    const double cost = (double)rounds * bm[c] * bn[c] / eff[c];
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

int launch(const float* A, int lda, const float* W, int ldw, const float* bias, const float* c1, const float* c2,
           const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi, float eps, bool ln,
           hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 4) || (ldw % 4) || lda < K || ldw < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)W) & 15) return (int)hipErrorInvalidValue;
  if (!ln && (epi & EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if (ln && (!c1 || !c2)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && (!R || ldr < N)) return (int)hipErrorInvalidValue;
  const int cfg = pick_tile(M, N);
#define NOS_F32_LAUNCH(LNV, BMV, BNV) \
  launch_t<LNV, BMV, BNV>(A, lda, W, ldw, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, st)
  if (ln) {
    if (cfg == 0) return NOS_F32_LAUNCH(true, 128, 128);
    if (cfg == 1) return NOS_F32_LAUNCH(true, 64, 128);
    return NOS_F32_LAUNCH(true, 64, 64);
  }
  if (cfg == 0) return NOS_F32_LAUNCH(false, 128, 128);
  if (cfg == 1) return NOS_F32_LAUNCH(false, 64, 128);
  return NOS_F32_LAUNCH(false, 64, 64);
#undef NOS_F32_LAUNCH
}

}  // namespace

// The tile the policy picks for an M x N output (0: 128x128, 1: 64x128,
// 2: 64x64) -- shared with the bf16x6 split GEMM (gemm_f32x.hip).
NOS_API int nos_gemm_f32_pick_tile(int M, int N) { return pick_tile(M, N); }

NOS_API int nos_gemm_f32_set_policy(int policy) {
  if (policy < 0 || policy > 2) return (int)hipErrorInvalidValue;
  g_policy = policy;
  return 0;
}

// C = act(A . W^T + bias) (+ R), fp32; A [M,K] (lda), W [N,K] (ldw), R/C [M,N].
// K % 32 == 0, A/W rows 16-byte aligned.
NOS_API int nos_gemm_f32(const float* A, int lda, const float* W, int ldw, const float* bias, const float* R,
                         int ldr, float* C, int ldc, int M, int N, int K, int epi, hipStream_t stream) {
  return launch(A, lda, W, ldw, bias, nullptr, nullptr, R, ldr, C, ldc, M, N, K, epi, 0.f, false, stream);
}

// C = act(LayerNorm(A) . W^T + bias) with W' = W * gamma, c1 = rowsum(W'),
// c2 = W . beta + bias (fp32, ops.fold_layernorm); K is the LayerNorm width.
NOS_API int nos_gemm_ln_f32(const float* A, int lda, const float* Wg, int ldw, const float* c1, const float* c2,
                            float* C, int ldc, int M, int N, int K, int epi, float eps, hipStream_t stream) {
  return launch(A, lda, Wg, ldw, nullptr, c1, c2, nullptr, 0, C, ldc, M, N, K, epi & ~(EPI_BIAS | EPI_RESID), eps,
                true, stream);
}
