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
//    64x64 = 2x2 blocks of v_mfma_f32_32x32x16_bf16, BK = 64; 128x64 for
//    small-N GEMMs, 256x256 / 8 waves (128x64 wave tiles) for long-K GEMMs
//    that fill the chip (the Cfg template below);
//  * both operands are K-contiguous, so both are staged the same way: direct
//    global->LDS DMA (global_load_lds_dwordx4, 1 KiB = 8 rows per wave
//    instruction) into a lane-linear image; the XOR swizzle that makes the
//    ds_read_b128 fragment reads conflict-free is applied to the per-lane
//    SOURCE address (linear destination + inverse-swizzled source + swizzled
//    read, cdna_hip_programming.md rule 21);
//  * two LDS buffers: tile k+1 is in flight while tile k is consumed (a
//    4-deep ring of BK = 32 slices measured slower: twice the barriers);
//  * LayerNorm fusion without a normalised copy of A: with W' = W * gamma
//    (per-k column scale, precomputed), c1[n] = sum_k W'[n,k],
//    c2[n] = sum_k W[n,k] beta[k] + bias[n]:
//        LN(x) . W^T + bias = rstd * (x . W'^T - mu * c1) + c2
//    so the MFMA main loop runs on the raw residual stream; per-row mean /
//    variance are accumulated from the A tiles already staged in LDS (the
//    K loop covers the whole row because K == hidden);
//  * register epilogue: swapped MFMA operands + v_permlane32_swap give each
//    lane 8 consecutive columns of one row; bias / LN correction / GELU /
//    residual are applied in registers (packed-f32 pairs) and stored as
//    16-byte row chunks;
//  * optional persistent mode (grid smaller than the tile count) and an
//    XCD-aware tile order so tiles sharing the larger operand panel share an
//    XCD's L2.
#include "common.h"
#include "gemm_tiles.h"

namespace {

// LDS image of a [rows][BK] bf16 K-slice: RB-byte rows of CPR 16-byte chunks,
// RPI rows per 1 KiB wave-instruction.  Chunk c of row r sits at chunk
// c ^ swz(r): the 16 lanes of every ds_read_b128 lane group (rows r..r+31 of
// one chunk) then hit 16 distinct 4-bank groups.
template <int BK>
struct Lay {
  static constexpr int RB = 2 * BK, CPR = BK / 8, RPI = 64 / CPR;
  static constexpr int SH = RB == 128 ? 1 : 2;  // rows per 256-byte bank wrap: 2 or 4
  __device__ static __forceinline__ int swz(int row) { return (row >> SH) & (CPR - 1); }
};

// Workgroup tile BM x BN over WGM x WGN waves (wave tile WM x WN, MI x NB
// blocks of 32x32), K-slices of BK in an S-deep LDS-DMA ring.  128x128 / 4
// waves is the base; 128x64 doubles the tile count for small N; 256x256 / 8
// waves (128x64 wave tiles) halves the L2->LDS bytes per FLOP of the base
// tile (a 128x128 tile at the MFMA peak would need the whole L2 bandwidth)
// and reads 0.75 instead of 1 LDS fragment per MFMA.
template <int BM_, int BN_, int WGM_, int WGN_, int BK_ = 64, int S_ = 2>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, BK = BK_, S = S_;
  using L = Lay<BK>;
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  static constexpr int MI = WM / 32, NB = WN / 32;
  static constexpr int TILE_A_BYTES = BM * L::RB;
  static constexpr int TILE_B_BYTES = BN * L::RB;
  static constexpr int STAGE_BYTES = TILE_A_BYTES + TILE_B_BYTES;
  static constexpr int LOADS_PER_STAGE = (BM + BN) / (L::RPI * NW);  // global_load_lds per wave per stage
  static constexpr int MINB = NT >= 512 ? 1 : 2;
  static constexpr int LDS = S * STAGE_BYTES + (2 * BM + 4 * BN) * 4;
  static_assert(NT == 2 * BM, "LayerNorm row statistics: two threads per row");
  static_assert(BM % (L::RPI * NW) == 0 && BN % (L::RPI * NW) == 0, "staging: whole wave-instructions per wave");
  static_assert(S >= 2 && S <= 4 && (S - 1) * LOADS_PER_STAGE < 64, "ring depth / vmcnt range");
};
using CfgBase = Cfg<128, 128, 2, 2>;
using CfgNarrow = Cfg<128, 64, 2, 2>;
using CfgBig = Cfg<256, 256, 2, 4>;
using CfgWide = Cfg<256, 192, 4, 2>;  // N = 384 in two tiles, 256-row panels: one round on 256 CUs

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8 };
// Tile policy (process-wide, nos_gemm_set_policy), see pick_tile():
//  * 0 = throughput (default): least padded work over 128x128 / 256x192 /
//    256x256 tiles -- what fractional pods sharing a GPU want (8 co-running
//    YOLOS pods lose ~4 % aggregate throughput with 128x64 tiles);
//  * 1 = latency: fewest rounds of tiles over the CUs, 128x64 included
//    (single tenant: N = 384 projections at batch 1 -24 %, FC2 -23 %);
//  * 2 / 3 / 4 = always 128x64 / 256x256 / 256x192 (A/B only).
int g_tile_policy = 0;
// persistent grid: 0 = one workgroup per tile, n > 0 = at most n workgroups
// per CU, each running several tiles with the next tile's loads in flight
// during the current epilogue (nos_gemm_set_persistent)
int g_persist = 0;

int num_cus() { return nos_effective_cus(); }  // a CU-slice tenant plans for its budget

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Stage a [ROWS][BK] bf16 K-slice: ROWS/RPI wave-instructions, spread over NW waves.
template <int ROWS, int NW, int BK>
__device__ __forceinline__ void stage_tile(const unsigned short* __restrict__ src, int ld, int row0,
                                           int nrows, int k0, unsigned char* tile, int wid, int lane) {
  using L = Lay<BK>;
  constexpr int PER_WAVE = ROWS / (L::RPI * NW);
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int R = (wid * PER_WAVE + i) * L::RPI;
    const int row = R + lane / L::CPR;
    const int pc = lane % L::CPR;
    const int lc = pc ^ L::swz(row);
    int grow = row0 + row;
    grow = grow < nrows ? grow : nrows - 1;
    glds16(src + (long long)grow * ld + k0 + lc * 8, tile + R * L::RB);
  }
}

// s_waitcnt vmcnt(n * LPS) for a runtime n in [0, 3]: the immediate must be a constant
template <int LPS>
__device__ __forceinline__ void wait_stages(int n) {
  if (n <= 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
  else if (n == 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LPS) : "memory");
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
template <bool LN, class CF, bool RESID>
__device__ __forceinline__ void epilogue_rows(const f32x16_t (&acc)[CF::MI][CF::NB], const float* s_mu,
                                              const float* s_rstd, const float* s_p1, const float* s_p2,
                                              const unsigned short* __restrict__ R, int ldr,
                                              unsigned short* __restrict__ C, int ldc, int M, int N, int m0,
                                              int n0, int epi, bool vec_ok, int wm, int wn, int r, int hh) {
  constexpr int WN = CF::WN, NB = CF::NB, MI = CF::MI, WM = CF::WM;
  // residual rows: the 16-byte loads of row group mi+1 are issued before
  // group mi is finished (clamped addresses, no per-element branches), so
  // their latency overlaps the epilogue math; two groups live at a time keep
  // the 8-wave tiles (MI = 4) from spilling
  const bool rvec = RESID && vec_ok && N >= 8;
  const int nmax = N >= 8 ? ((N - 8) >> 3) << 3 : 0;
  // prefetch depth: the 256x256 tile (8 waves, MI = 4) keeps ONE group of
  // residual rows live (issued at the start of its own group) -- two spilled
  // 4 VGPRs / 20 B of scratch there
  constexpr int RPD = (CF::NW > 4 && MI >= 4) ? 1 : 2;
  s16x8_t rpre[RPD][NB][2];
  auto rload = [&](int mi) {
    const int m = min(m0 + wm * WM + mi * 32 + r, M - 1);
#pragma unroll
    for (int ni = 0; ni < NB; ++ni)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int n = min(n0 + wn * WN + ni * 32 + 16 * pr + 8 * hh, nmax);
        rpre[mi % RPD][ni][pr] = *reinterpret_cast<const s16x8_t*>(R + (long long)m * ldr + n);
      }
  };
  if (rvec) rload(0);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      if (RPD == 1 && rvec && mi > 0) rload(mi);
      if (RPD == 2 && rvec && mi + 1 < MI) rload(mi + 1);
      const int rl = wm * WM + mi * 32 + r;
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
          // LN correction / bias and activation on column pairs (packed f32);
          // the per-column parameters come from LDS a pair at a time (few live
          // registers next to the 8-wave tiles' accumulators)
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            f32x2_t w = {v[e], v[e + 1]};
            const f32x2_t q1 = *reinterpret_cast<const f32x2_t*>(s_p1 + cl + e);
            const f32x2_t q2 = *reinterpret_cast<const f32x2_t*>(s_p2 + cl + e);
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
              const s16x8_t rv = rpre[mi % RPD][ni][pr];
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

template <bool LN, class CF, bool RESID>
__global__ __launch_bounds__(CF::NT, CF::MINB) void gemm_bf16_rk_kernel(
    const unsigned short* __restrict__ A, int lda, const unsigned short* __restrict__ W, int ldw,
    const unsigned short* __restrict__ bias, const float* __restrict__ c1, const float* __restrict__ c2,
    const unsigned short* __restrict__ R, int ldr, unsigned short* __restrict__ C, int ldc, int M, int N,
    int K, int epi, float eps, int tiles_m, int tiles_n) {
  using L = typename CF::L;
  constexpr int BM = CF::BM, BN = CF::BN, NW = CF::NW, WGN = CF::WGN, BK = CF::BK, S = CF::S;
  constexpr int STAGE_BYTES = CF::STAGE_BYTES, TILE_A_BYTES = CF::TILE_A_BYTES;
  constexpr int WM = CF::WM, WN = CF::WN, MI = CF::MI, NB = CF::NB;
  constexpr int STATS_OFF = S * STAGE_BYTES;
  constexpr int LPS = CF::LOADS_PER_STAGE;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s_mu = reinterpret_cast<float*>(smem + STATS_OFF);
  float* s_rstd = s_mu + BM;
  float* s_par = s_rstd + BM;  // [2 tile parities][p1 BN | p2 BN]
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = wid / WGN, wn = wid - wm * WGN;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / BK;
  const bool vec_ok = ((ldc | ldr) & 7) == 0;

  // Tile order.  The dispatcher deals workgroup b to XCD b % 8; every XCD
  // owns one contiguous chunk of the tile range (tiles sharing an A row panel
  // share its L2) and its workgroups walk that chunk with a stride of the
  // XCD's workgroup count.  With one workgroup per tile this is xcd_remap;
  // with a smaller (persistent) grid each workgroup runs several tiles and
  // issues the next tile's first K-slices before the current epilogue, so
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
  // the staging lane index is re-derived per tile through an opaque copy:
  // hoisted to kernel entry, the lane-constant staging offsets of the 8-wave
  // LN tiles stayed live around the tile loop and spilled (10 VGPRs)
  int lane_st = lane;
  auto stage = [&](int m0, int n0, int kt) {
    unsigned char* buf = smem + (kt % S) * STAGE_BYTES;
    stage_tile<BM, NW, BK>(A, lda, m0, M, kt * BK, buf, wid, lane_st);
    stage_tile<BN, NW, BK>(W, ldw, n0, N, kt * BK, buf + TILE_A_BYTES, wid, lane_st);
  };
  // the first S K-slices of a tile (the whole ring is free)
  auto prologue = [&](int m0, int n0) {
#pragma unroll
    for (int q = 0; q < S; ++q)
      if (q < nk) stage(m0, n0, q);
  };

  int tile = t_lo + j, m0, n0, par = 0;
  coords(tile, m0, n0);
  // params are loaded before any LDS-DMA is in flight, so waiting for them
  // drains nothing
  params(n0, 0);
  prologue(m0, n0);

  for (int it = 1;; ++it) {
    asm volatile("" : "+v"(lane_st));
    f32x16_t acc[MI][NB];
#pragma unroll
    for (int a = 0; a < MI; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

    const int srow = tid >> 1, shalf = tid & 1;
    float sshift = 0.f, ssum = 0.f, ssq = 0.f;

    for (int kt = 0; kt < nk; ++kt) {
      // slice kt landed (the newer slices issued so far may stay in flight:
      // S-1 of them after the prologue, S-2 later) and every wave is done
      // with slice kt-1, whose buffer slice kt+S-1 reuses
      wait_stages<LPS>(min(kt == 0 ? S - 1 : S - 2, nk - 1 - kt));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt > 0 && kt + S - 1 < nk) stage(m0, n0, kt + S - 1);
      const unsigned char* ta = smem + (kt % S) * STAGE_BYTES;
      const unsigned char* tb = ta + TILE_A_BYTES;
      if constexpr (LN) {
        // one 16-byte chunk live at a time: the 8-wave tiles hold 128
        // accumulator registers and would spill with all chunks in flight
        constexpr int LN_UNROLL = CF::NW > 4 ? 1 : L::CPR / 2;
#pragma unroll LN_UNROLL
        for (int c = 0; c < L::CPR / 2; ++c) {
          const int lc = shalf * (L::CPR / 2) + c;
          const s16x8_t v = *reinterpret_cast<const s16x8_t*>(ta + srow * L::RB + ((lc ^ L::swz(srow)) << 4));
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
        bf16x8_t af[MI], bf[NB];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const int row = wm * WM + mi * 32 + r;
          af[mi] = *reinterpret_cast<const bf16x8_t*>(ta + row * L::RB + (((2 * ks + hh) ^ L::swz(row)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < NB; ++ni) {
          const int row = wn * WN + ni * 32 + r;
          bf[ni] = *reinterpret_cast<const bf16x8_t*>(tb + row * L::RB + (((2 * ks + hh) ^ L::swz(row)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
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
      // each thread saw half of its row's chunks: combine the two shifted sums
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
    epilogue_rows<LN, CF, RESID>(acc, s_mu, s_rstd, s_p1, s_p1 + BN, R, ldr, C, ldc, M, N, m0, n0, epi, vec_ok,
                                 wm, wn, r, hh);
    // a workgroup's last tile ends without a barrier (it would drain the stores)
    if (!more) break;
    par ^= 1;
    params(n1, par);
    m0 = m1;
    n0 = n1;
    // the next tile's first slices were issued before the epilogue; its
    // stores and residual loads share vmcnt, so drain everything here (the
    // slices have long landed) -- the K loop's first barrier then publishes
    // the parameters
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <bool LNV, class CF, bool RV>
void launch_cfg(int nwg, hipStream_t stream, const unsigned short* A, int lda, const unsigned short* W, int ldw,
                const unsigned short* bias, const float* c1, const float* c2, const unsigned short* R, int ldr,
                unsigned short* C, int ldc, int M, int N, int K, int epi, float eps, int tiles_m, int tiles_n) {
  if (nwg == tiles_m * tiles_n)  // no explicit cap: a CU-slice tenant's budget (nos_set_cu_budget) applies
    nwg = nos_grid_for((const void*)gemm_bf16_rk_kernel<LNV, CF, RV>, CF::NT, CF::LDS, nwg);
  hipLaunchKernelGGL((gemm_bf16_rk_kernel<LNV, CF, RV>), dim3(nwg), dim3(CF::NT), CF::LDS, stream, A, lda, W, ldw,
                     bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, tiles_m, tiles_n);
}

template <class CF>
int launch_tile(const void* A, int lda, const void* W, int ldw, const void* bias, const float* c1, const float* c2,
                const void* R, int ldr, void* C, int ldc, int M, int N, int K, int epi, float eps, int max_wg,
                bool ln, hipStream_t stream) {
  const int tiles_m = (M + CF::BM - 1) / CF::BM;
  const int tiles_n = (N + CF::BN - 1) / CF::BN;
  int nwg = tiles_m * tiles_n;
  if (max_wg <= 0 && g_persist > 0) max_wg = g_persist * num_cus();
  if (max_wg > 0 && nwg > max_wg) nwg = max_wg;
  auto Ap = (const unsigned short*)A;
  auto Wp = (const unsigned short*)W;
  auto Bp = (const unsigned short*)bias;
  auto Rp = (const unsigned short*)R;
  auto Cp = (unsigned short*)C;
  if (ln)
    launch_cfg<true, CF, false>(nwg, stream, Ap, lda, Wp, ldw, Bp, c1, c2, Rp, ldr, Cp, ldc, M, N, K, epi, eps,
                                tiles_m, tiles_n);
  else if (epi & EPI_RESID)
    launch_cfg<false, CF, true>(nwg, stream, Ap, lda, Wp, ldw, Bp, c1, c2, Rp, ldr, Cp, ldc, M, N, K, epi, eps,
                                tiles_m, tiles_n);
  else
    launch_cfg<false, CF, false>(nwg, stream, Ap, lda, Wp, ldw, Bp, c1, c2, Rp, ldr, Cp, ldc, M, N, K, epi, eps,
                                 tiles_m, tiles_n);
  return (int)hipGetLastError();
}

int launch(const void* A, int lda, const void* W, int ldw, const void* bias, const float* c1,
           const float* c2, const void* R, int ldr, void* C, int ldc, int M, int N, int K, int epi,
           float eps, int max_wg, bool ln, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % 64) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8)) return (int)hipErrorInvalidValue;
  if (!ln && (epi & EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if (ln && (!c1 || !c2)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && !R) return (int)hipErrorInvalidValue;
#define NOS_GEMM_ARGS A, lda, W, ldw, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, max_wg, ln, stream
  using namespace nos_gemm;
  switch (pick_tile(M, N, g_tile_policy, num_cus())) {
    case T_NARROW: return launch_tile<CfgNarrow>(NOS_GEMM_ARGS);
    case T_WIDE: return launch_tile<CfgWide>(NOS_GEMM_ARGS);
    case T_BIG: return launch_tile<CfgBig>(NOS_GEMM_ARGS);
    default: return launch_tile<CfgBase>(NOS_GEMM_ARGS);
  }
#undef NOS_GEMM_ARGS
}

}  // namespace

// C = act(A . W^T + bias) (+ R).  A [M,K] (row stride lda), W [N,K] (ldw),
// R/C [M,N] (ldr/ldc), all bf16.  K must be a multiple of 64 and every row
// start 16-byte aligned.  max_wg > 0 caps the grid (persistent mode).
NOS_API int nos_gemm_set_policy(int policy) {
  if (policy < 0 || policy > 4) return (int)hipErrorInvalidValue;
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
