// bf16 GEMM with fused prologue / epilogue for gfx950:
//
//   plain:   C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ R)
//   LN-fused C[M,N] = act(LayerNorm(A)[M,K] . W[N,K]^T + bias)            (K == hidden)
//
// This is every linear layer of the tenant models (W in nn.Linear [out, in]
// layout) and the body of the gpuagent's MFMA probe (probe_gemm runs it
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
//    read, cdna_hip_programming.md rule 21);
//  * two LDS buffers: tile k+1 is in flight while tile k is consumed;
//  * LayerNorm fusion without a normalised copy of A: with W' = W * gamma
//    (per-k column scale, precomputed), c1[n] = sum_k W'[n,k],
//    c2[n] = sum_k W[n,k] beta[k] + bias[n]:
//        LN(x) . W^T + bias = rstd * (x . W'^T - mu * c1) + c2
//    so the MFMA main loop runs on the raw residual stream; per-row mean /
//    variance are accumulated from the A tiles already staged in LDS (the
//    K loop covers the whole row because K == hidden);
//  * register epilogue: swapped MFMA operands + v_permlane32_swap give each
//    lane 8 consecutive columns of one row; bias / LN correction / GELU /
//    residual are applied in registers and stored as 16-byte row chunks;
//  * optional persistent mode (grid smaller than the tile count) and an
//    XCD-aware tile order so tiles sharing the larger operand panel share an
//    XCD's L2.
#include "common.h"

namespace {

constexpr int BM = 128, BK = 64;
constexpr int NT = 256;
constexpr int TILE_A_BYTES = BM * BK * 2;  // 16 KiB

// BN (128 or 64) is a template parameter: N = 384 projections have only 81
// 128x128 tiles for 256 CUs, 162 with 128x64 tiles.
template <int BN>
struct Cfg {
  static constexpr int TILE_B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = TILE_A_BYTES + TILE_B_BYTES;
  static constexpr int WN = BN / 2;                    // wave tile: 64 x WN (2x2 waves)
  static constexpr int NB = WN / 32;                   // 32-column MFMA blocks per wave
};

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8 };
// Tile policy (process-wide, nos_gemm_set_policy):
//  * 0 = throughput (default): always 128x128 tiles -- fewest bytes per FLOP;
//    what fractional pods sharing a GPU want (measured: 8 co-running YOLOS
//    pods lose ~4 % aggregate throughput with narrow tiles);
//  * 1 = latency: when a GEMM has fewer 128x128 tiles than NARROW_TILES, use
//    128x64 tiles to occupy twice the CUs (single tenant: N = 384 projections
//    -24 %, FC2 -23 % kernel time);
//  * 2 = narrow: always 128x64 (A/B only).
constexpr int NARROW_TILES = 200;
int g_tile_policy = 0;
// persistent grid: 0 = one workgroup per tile, n > 0 = at most n workgroups
// per CU, each running several tiles with the next tile's loads in flight
// during the current epilogue (nos_gemm_set_persistent)
int g_persist = 0;

int num_cus() {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Stage a [ROWS][64 k] bf16 tile: ROWS/8 wave-instructions, ROWS/32 per wave.
template <int ROWS>
__device__ __forceinline__ void stage_tile(const unsigned short* __restrict__ src, int ld, int row0,
                                           int nrows, int k0, unsigned char* tile, int wid, int lane) {
  constexpr int PER_WAVE = ROWS / 32;
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int R = (wid * PER_WAVE + i) * 8;
    const int row = R + (lane >> 3);
    const int pc = lane & 7;
    const int lc = pc ^ swz(row);
    int grow = row0 + row;
    grow = grow < nrows ? grow : nrows - 1;
    glds16(src + (long long)grow * ld + k0 + lc * 8, tile + R * 128);
  }
}

// erf(x) for GELU: Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7, far below
// bf16 output precision) -- one exp + one rcp instead of the libm erff.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  const float r = fmaf(-p * t, e, 1.f);
  return copysignf(r, x);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }

// the same GELU on a register pair: the polynomial runs as packed-f32 FMAs
// (v_pk_fma_f32 / v_pk_mul_f32, two columns per VALU op); rcp and exp stay
// per element on the transcendental unit
__device__ __forceinline__ f32x2_t gelu_erf2(f32x2_t x) {
  const f32x2_t z = x * 0.70710678118654752f;
  const f32x2_t az = {fabsf(z[0]), fabsf(z[1])};
  const f32x2_t d = az * 0.3275911f + 1.f;
  const f32x2_t t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2_t p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const f32x2_t q = az * az * -1.4426950408889634f;
  const f32x2_t e = {__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])};
  const f32x2_t r = 1.f - p * t * e;  // erf(|z|)
  const f32x2_t er = {copysignf(r[0], z[0]), copysignf(r[1], z[1])};
  const f32x2_t hx = x * 0.5f;
  return hx * er + hx;
}

// ---------------------------------------------------------------------------
// Register epilogue.  The MFMA operands are swapped (D = W_frag . A_frag), so
// each 32x32 accumulator block holds C^T: lane (r, hh) owns output ROW r and
// columns 8j + 4hh + {0..3}.  One v_permlane32_swap per register pair turns
// that into 8 consecutive columns per lane, so bias / LayerNorm correction /
// activation / residual run on registers and the tile leaves as 16-byte row
// stores -- no fp32 LDS tile (the round-1 LDS-tile epilogue measured slower
// and was removed).  acc holds C^T blocks
// (MFMA operands swapped): lane (r, hh) owns row r, columns 8j + 4hh + {0..3}
// of each 32x32 block; a v_permlane32_swap per register pair gives each lane
// 8 consecutive columns of its row, stored as one 16-byte chunk.
template <bool LN, int BN, bool RESID, int MI = 2>
__device__ __forceinline__ void epilogue_rows(const f32x16_t (&acc)[MI][Cfg<BN>::NB], const float* s_mu,
                                              const float* s_rstd, const float* s_p1, const float* s_p2,
                                              const unsigned short* __restrict__ R, int ldr,
                                              unsigned short* __restrict__ C, int ldc, int M, int N, int m0,
                                              int n0, int epi, bool vec_ok, int wm, int wn, int r, int hh) {
  constexpr int WN = Cfg<BN>::WN, NB = Cfg<BN>::NB;
  // residual rows: all 16-byte loads issued up front (clamped addresses, no
  // per-element branches) so their latencies overlap instead of one round
  // trip per chunk
  s16x8_t rpre[MI][NB][2];
  if constexpr (RESID) {
    if (vec_ok && N >= 8) {
      const int nmax = ((N - 8) >> 3) << 3;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int m = min(m0 + wm * (32 * MI) + mi * 32 + r, M - 1);
#pragma unroll
        for (int ni = 0; ni < NB; ++ni)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const int n = min(n0 + wn * WN + ni * 32 + 16 * pr + 8 * hh, nmax);
            rpre[mi][ni][pr] = *reinterpret_cast<const s16x8_t*>(R + (long long)m * ldr + n);
          }
      }
    }
  }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int rl = wm * (32 * MI) + mi * 32 + r;
      const int m = m0 + rl;
      float mu = 0.f, rs = 1.f;
      if constexpr (LN) {
        mu = s_mu[rl];
        rs = s_rstd[rl];
      }
#pragma unroll
      for (int ni = 0; ni < NB; ++ni) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          // registers 8pr+e (cols 16pr + 4hh + e) and 8pr+4+e (cols 16pr + 8 + 4hh + e)
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[mi][ni][8 * pr + e]),
                                                             __float_as_uint(acc[mi][ni][8 * pr + 4 + e]),
                                                             false, false);
            v[e] = __uint_as_float(sw[0]);
            v[4 + e] = __uint_as_float(sw[1]);
          }
          // now: 8 consecutive columns cl .. cl+7 of row rl
          const int cl = wn * WN + ni * 32 + 16 * pr + 8 * hh;
          const int n = n0 + cl;
          const float4 p1a = *reinterpret_cast<const float4*>(s_p1 + cl);
          const float4 p1b = *reinterpret_cast<const float4*>(s_p1 + cl + 4);
          const float4 p2a = *reinterpret_cast<const float4*>(s_p2 + cl);
          const float4 p2b = *reinterpret_cast<const float4*>(s_p2 + cl + 4);
          const float p1[8] = {p1a.x, p1a.y, p1a.z, p1a.w, p1b.x, p1b.y, p1b.z, p1b.w};
          const float p2[8] = {p2a.x, p2a.y, p2a.z, p2a.w, p2b.x, p2b.y, p2b.z, p2b.w};
          // LN correction / bias and activation on column pairs (packed f32)
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            f32x2_t w = {v[e], v[e + 1]};
            const f32x2_t q1 = {p1[e], p1[e + 1]}, q2 = {p2[e], p2[e + 1]};
            if (LN)
              w = (w - q1 * mu) * rs + q2;
            else
              w = w + q2;
            if (epi & EPI_GELU) w = gelu_erf2(w);
            v[e] = w[0];
            v[e + 1] = w[1];
          }
          if (epi & EPI_RELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (m >= M || n >= N) continue;
          if (n + 8 <= N && vec_ok) {
            if constexpr (RESID) {
              const s16x8_t rv = rpre[mi][ni][pr];
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += nos::bf16_to_f32((unsigned short)rv[e]);
            }
            s16x8_t o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (short)nos::f32_to_bf16(v[e]);
            *reinterpret_cast<s16x8_t*>(C + (long long)m * ldc + n) = o;
          } else {
            for (int e = 0; e < 8 && n + e < N; ++e) {
              float x = v[e];
              if (RESID) x += nos::bf16_to_f32(R[(long long)m * ldr + n + e]);
              C[(long long)m * ldc + n + e] = nos::f32_to_bf16(x);
            }
          }
        }
      }
    }
}

template <bool LN, int BN, bool RESID>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_rk_kernel(
    const unsigned short* __restrict__ A, int lda, const unsigned short* __restrict__ W, int ldw,
    const unsigned short* __restrict__ bias, const float* __restrict__ c1, const float* __restrict__ c2,
    const unsigned short* __restrict__ R, int ldr, unsigned short* __restrict__ C, int ldc, int M, int N,
    int K, int epi, float eps, int tiles_m, int tiles_n) {
  using CF = Cfg<BN>;
  constexpr int STAGE_BYTES = CF::STAGE_BYTES;
  constexpr int WN = CF::WN, NB = CF::NB;
  constexpr int STATS_OFF = 2 * STAGE_BYTES;
  constexpr int LOADS_PER_STAGE = BM / 32 + BN / 32;  // global_load_lds per wave per stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + STATS_OFF);
  float* s_rstd = s_mu + BM;
  float* s_par = s_rstd + BM;  // [2 tile parities][p1 BN | p2 BN]
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / BK;
  const bool vec_ok = ((ldc | ldr) & 7) == 0;

  // Tile order.  The dispatcher deals workgroup b to XCD b % 8; every XCD
  // owns one contiguous chunk of the tile range (tiles sharing an A row panel
  // share its L2) and its workgroups walk that chunk with a stride of the
  // XCD's workgroup count.  With one workgroup per tile this is xcd_remap;
  // with a smaller (persistent) grid each workgroup runs several tiles and
  // issues the next tile's first two K-steps before the current epilogue, so
  // their latency hides under the epilogue's math and stores.
  const int G = gridDim.x, xcd = blockIdx.x % 8, j = blockIdx.x / 8;
  const int wgs_x = G / 8 + (xcd < G % 8 ? 1 : 0);
  const int t_lo = xcd * (ntiles / 8) + min(xcd, ntiles % 8);
  const int t_cnt = ntiles / 8 + (xcd < ntiles % 8 ? 1 : 0);
  if (j >= t_cnt) return;

  auto coords = [&](int t, int& m0, int& n0) {
    int tm, tn;
    if (tiles_m >= tiles_n) {
      tm = t / tiles_n;
      tn = t - tm * tiles_n;
    } else {
      tn = t / tiles_m;
      tm = t - tn * tiles_m;
    }
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // per-column epilogue parameters: (c1, c2) for the LN-fused form, (0, bias)
  // otherwise; double-buffered by tile parity (a slower wave may still be in
  // the previous tile's epilogue)
  auto params = [&](int n0, int par) {
    if (tid < BN) {
      const int n = min(n0 + tid, N - 1);
      s_par[par * 2 * BN + tid] = LN ? c1[n] : 0.f;
      s_par[par * 2 * BN + BN + tid] = LN ? c2[n] : ((epi & EPI_BIAS) ? nos::bf16_to_f32(bias[n]) : 0.f);
    }
  };
  // the first two K-steps of a tile into the two ring buffers
  auto prologue = [&](int m0, int n0) {
    stage_tile<BM>(A, lda, m0, M, 0, smem, wid, lane);
    stage_tile<BN>(W, ldw, n0, N, 0, smem + TILE_A_BYTES, wid, lane);
    if (nk > 1) {
      stage_tile<BM>(A, lda, m0, M, BK, smem + STAGE_BYTES, wid, lane);
      stage_tile<BN>(W, ldw, n0, N, BK, smem + STAGE_BYTES + TILE_A_BYTES, wid, lane);
    }
  };

  int tile = t_lo + j, m0, n0, par = 0;
  coords(tile, m0, n0);
  // params are loaded before any LDS-DMA is in flight, so waiting for them
  // drains nothing; step 1's loads overlap step 0's wait
  params(n0, 0);
  prologue(m0, n0);
  if (nk > 1)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(LOADS_PER_STAGE) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // step 0 landed for every wave; params visible

  for (int it = 1;; ++it) {
    f32x16_t acc[2][NB];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    const int srow = tid >> 1, shalf = tid & 1;
    float sshift = 0.f, ssum = 0.f, ssq = 0.f;

    for (int kt = 0; kt < nk; ++kt) {
      unsigned char* cur = smem + (kt & 1) * STAGE_BYTES;
      if (kt > 0) {
        __syncthreads();  // step kt landed (vmcnt(0)); everyone done with step kt-1's buffer
        if (kt + 1 < nk) {
          unsigned char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
          stage_tile<BM>(A, lda, m0, M, (kt + 1) * BK, nxt, wid, lane);
          stage_tile<BN>(W, ldw, n0, N, (kt + 1) * BK, nxt + TILE_A_BYTES, wid, lane);
        }
      }
      const unsigned char* ta = cur;
      const unsigned char* tb = cur + TILE_A_BYTES;
      if constexpr (LN) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int lc = shalf * 4 + c;
          const s16x8_t v = *reinterpret_cast<const s16x8_t*>(ta + srow * 128 + ((lc ^ swz(srow)) << 4));
          if (kt == 0 && c == 0) sshift = nos::bf16_to_f32((unsigned short)v[0]);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = nos::bf16_to_f32((unsigned short)v[e]) - sshift;
            ssum += d;
            ssq = fmaf(d, d, ssq);
          }
        }
      }
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8_t af[2], bf[NB];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int row = wm * 64 + mi * 32 + r;
          af[mi] = *reinterpret_cast<const bf16x8_t*>(ta + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < NB; ++ni) {
          const int row = wn * WN + ni * 32 + r;
          bf[ni] = *reinterpret_cast<const bf16x8_t*>(tb + row * 128 + (((2 * ks + hh) ^ swz(row)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NB; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[ni], af[mi], acc[mi][ni], 0, 0, 0);
      }
    }

    const int k_next = j + it * wgs_x;
    const bool more = k_next < t_cnt;
    int m1 = 0, n1 = 0;
    if (more) {
      coords(t_lo + k_next, m1, n1);
      __syncthreads();  // every wave is done reading the ring: the next tile may overwrite it
      prologue(m1, n1);
    }

    if constexpr (LN) {
      const float sh_lo = __shfl(sshift, lane & ~1, 64);
      const float dlt = sshift - sh_lo;
      const float kh = (float)(K / 2);
      float s2 = ssum + dlt * kh;
      float q2 = ssq + 2.f * dlt * ssum + dlt * dlt * kh;
      s2 += __shfl_xor(s2, 1, 64);
      q2 += __shfl_xor(q2, 1, 64);
      if (shalf == 0) {
        const float mean_d = s2 / (float)K;
        const float var = fmaxf(q2 / (float)K - mean_d * mean_d, 0.f);
        s_mu[srow] = sh_lo + mean_d;
        s_rstd[srow] = rsqrtf(var + eps);
      }
      __syncthreads();
    }

    const float* s_p1 = s_par + par * 2 * BN;
    epilogue_rows<LN, BN, RESID>(acc, s_mu, s_rstd, s_p1, s_p1 + BN, R, ldr, C, ldc, M, N, m0, n0, epi, vec_ok,
                                 wm, wn, r, hh);
    // a workgroup's last tile ends without a barrier (it would drain the stores)
    if (!more) break;
    par ^= 1;
    params(n1, par);
    m0 = m1;
    n0 = n1;
    // the next tile's steps 0/1 were issued before the epilogue; its stores and
    // residual loads share vmcnt, so wait for everything (step 0 has long landed)
    // and make the parameters (and, for LN, the consumed s_mu) safe to reuse
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

template <int BNV>
constexpr int rk_lds_bytes() { return 2 * Cfg<BNV>::STAGE_BYTES + (2 * BM + 4 * BNV) * 4; }

int launch(const void* A, int lda, const void* W, int ldw, const void* bias, const float* c1,
           const float* c2, const void* R, int ldr, void* C, int ldc, int M, int N, int K, int epi,
           float eps, int max_wg, bool ln, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8)) return (int)hipErrorInvalidValue;
  if (!ln && (epi & EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if (ln && (!c1 || !c2)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && !R) return (int)hipErrorInvalidValue;
  const int tiles_m = (M + BM - 1) / BM;
  // fewer 128-wide tiles than CUs (e.g. N = 384 projections): halve the N tile
  const bool narrow = g_tile_policy == 2 || (g_tile_policy == 1 && tiles_m * ((N + 127) / 128) < NARROW_TILES);
  const int bn = narrow ? 64 : 128;
  const int tiles_n = (N + bn - 1) / bn;
  int nwg = tiles_m * tiles_n;
  if (max_wg <= 0 && g_persist > 0) max_wg = g_persist * num_cus();
  if (max_wg > 0 && nwg > max_wg) nwg = max_wg;
  auto Ap = (const unsigned short*)A;
  auto Wp = (const unsigned short*)W;
  auto Bp = (const unsigned short*)bias;
  auto Rp = (const unsigned short*)R;
  auto Cp = (unsigned short*)C;
#define NOS_GEMM_ARGS                                                                                     \
  Ap, lda, Wp, ldw, Bp, c1, c2, Rp, ldr, Cp, ldc, M, N, K, epi, eps, tiles_m, tiles_n
#define NOS_GEMM_LAUNCH(LNV, BNV, RV)                                                                      \
  hipLaunchKernelGGL((gemm_bf16_rk_kernel<LNV, BNV, RV>), dim3(nwg), dim3(NT), rk_lds_bytes<BNV>(), stream,  \
                     NOS_GEMM_ARGS)
  const bool resid = (epi & EPI_RESID) != 0;
  if (ln) {
    if (narrow) NOS_GEMM_LAUNCH(true, 64, false); else NOS_GEMM_LAUNCH(true, 128, false);
  } else if (resid) {
    if (narrow) NOS_GEMM_LAUNCH(false, 64, true); else NOS_GEMM_LAUNCH(false, 128, true);
  } else {
    if (narrow) NOS_GEMM_LAUNCH(false, 64, false); else NOS_GEMM_LAUNCH(false, 128, false);
  }
#undef NOS_GEMM_ARGS
#undef NOS_GEMM_LAUNCH
  return (int)hipGetLastError();
}

}  // namespace

// C = act(A . W^T + bias) (+ R).  A [M,K] (row stride lda), W [N,K] (ldw),
// R/C [M,N] (ldr/ldc), all bf16.  K must be a multiple of 64 and every row
// start 16-byte aligned.  max_wg > 0 caps the grid (persistent mode).
NOS_API int nos_gemm_set_policy(int policy) {
  if (policy < 0 || policy > 2) return (int)hipErrorInvalidValue;
  g_tile_policy = policy;
  return 0;
}

NOS_API int nos_gemm_set_persistent(int wgs_per_cu) {
  if (wgs_per_cu < 0 || wgs_per_cu > 8) return (int)hipErrorInvalidValue;
  g_persist = wgs_per_cu;
  return 0;
}

NOS_API int nos_gemm_bf16(const void* A, int lda, const void* W, int ldw, const void* bias, const void* R,
                          int ldr, void* C, int ldc, int M, int N, int K, int epi, int max_wg,
                          hipStream_t stream) {
  return launch(A, lda, W, ldw, bias, nullptr, nullptr, R, ldr, C, ldc, M, N, K, epi, 0.f, max_wg, false,
                stream);
}

// C = act(LayerNorm(A) . W^T + bias) with W' = W * gamma (bf16 [N,K]),
// c1 = rowsum(W') and c2 = W . beta + bias (fp32 [N]) precomputed by the
// caller; K is the LayerNorm width.
NOS_API int nos_gemm_ln_bf16(const void* A, int lda, const void* Wg, int ldw, const float* c1,
                             const float* c2, void* C, int ldc, int M, int N, int K, int epi, float eps,
                             int max_wg, hipStream_t stream) {
  return launch(A, lda, Wg, ldw, nullptr, c1, c2, nullptr, 0, C, ldc, M, N, K, epi & ~(EPI_BIAS | EPI_RESID),
                eps, max_wg, true, stream);
}
