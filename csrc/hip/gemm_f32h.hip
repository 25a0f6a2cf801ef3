// fp32 GEMM on the fp16x3 split (split_f16.h): both operands arrive as two
// fp16 planes on power-of-two scales, and each 16-deep step of a 32x32 block
// is three v_mfma_f32_32x32x16_f16 (hi.hi + hi.lo + lo.hi) -- half the
// matrix-pipe work of the bf16x6 GEMM (gemm_f32x.hip) and no split in the K
// loop at all:
//
//   C[M,N] = act(rinv[m] * csc[n] * (A'[m,:] . W'[n,:]) + bias[n]) (+ R)
//
//  * A' = the rows of A split by nos_split_rows_h3 (below): per row, a scale
//    2^e_m that puts max|a| just under 2^14 (or, LayerNorm mode, the rows
//    normalised first and scaled by the sqrt(K) bound of a normalised row),
//    written as hi / lo planes [2][M][K]; rinv[m] = 2^-e_m;
//  * W' = the weight's rows on their own scales 2^f_n, split once per
//    weight by the host (ops.split_f32_weight_h3); csc[n] = 2^-f_n;
//  * 4 waves per workgroup (2 x 2, or 4 x 1: 32-row strips), 128 x 128
//    tiles, BK = 32 per stage in a 2-deep LDS ring filled by LDS-DMA
//    (global_load_lds_dwordx4; every plane as rows of 64 B, 16-byte chunks
//    XOR-swizzled by (row >> 2) & 3 -- conflict-free fragment reads);
//  * the fragments of step s+1 are read from LDS while step s's MFMAs run
//    (two register sets in ping-pong, one stage boundary per two steps);
//  * epilogue: scales, bias, GELU / ReLU, residual, and optionally the K / V
//    columns of a fused QKV projection as the attention's fp16 planes
//    (KvOut: attention_f32x.hip's h3 kernel reads them).
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "split_f16.h"

namespace {

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8, EPI_BIAS_ROW = 16, EPI_RESID_PRE = 32,
             EPI_WIDE = 128 };
// EPI_WIDE (set by the host, stripped on entry): interior tiles written as
// fp16 planes go through LDS and leave as 16-byte row stores (8 per plane
// row chunk) instead of one 2-byte store per element and plane
template <int E>
using EpiC = std::integral_constant<int, E>;
// EPI_RESID adds R after the activation (transformer residuals); EPI_RESID_PRE
// before it (ResNet: relu(conv + bn + identity))

// batched GEMMs (nos_gemm_f32h3_batched): per-batch element strides of every
// operand (0 = shared by the whole batch, e.g. a conv weight); the tile index
// runs over nb x tiles_m x tiles_n, one batch's tiles adjacent (one XCD's L2)
struct Batch {
  int nb = 1;
  long long a = 0, rinv = 0, w = 0, csc = 0, c = 0, r = 0, bias = 0;  // bias: grouped convs' per-group rows
};

constexpr int BK = 32;  // K granule of the API (K % 32 == 0); stages are BKT = 32 or 16 deep

// 16-byte chunk swizzle of a plane row of CH chunks (BKT 32: 64 B rows, 4
// chunks; BKT 16: 32 B rows, 2 chunks): 16 consecutive lanes reading the same
// logical chunk of 16 consecutive rows hit 16 distinct 16-byte slots
template <int CH>
__device__ __forceinline__ int swz(int row) { return CH == 4 ? ((row >> 2) & 3) : ((row >> 3) & 1); }

// s_waitcnt vmcnt(n * LPS) for a runtime n in [0, 3]
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

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

// Abramowitz-Stegun 7.1.26, |err| <= 1.5e-7, on the hardware reciprocal and
// exp2 (v_rcp_f32 / v_exp_f32, ~1 ulp each): an IEEE division and expf's
// range reduction cost ~15 more VALU per element, and fc1's GELU epilogue is
// the largest VALU block of the h3 GEMMs
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);  // exp(-x^2); 0 past |x| ~ 10
  const float r = fmaf(-p * t, e, 1.f);
  return copysignf(r, x);
}

// the K / V columns (>= qcols) of a fused QKV projection as the h3
// attention's planes kvs[b][s][K hi, K lo, V hi, V lo][hd], each head on
// kvsc[0 / 1][head]; rows per batch S, padded to skvp
struct KvOut {
  unsigned short* kvs = nullptr;
  const float* kvsc = nullptr;
  int qcols = 0, hd = 0, S = 0, skvp = 0;
};

// the output as the NEXT h3 GEMM's A planes ([2][M][ldp], plane stride
// pplane) on the static scale sc (the host's bound of this output: fc1's
// GELU rows feeding fc2), instead of fp32 C
struct PlaneOut {
  unsigned short* p = nullptr;
  long long pplane = 0;
  int ldp = 0;
  float sc = 1.f;
};

// LayerNorm hand-off between a pre-LN residual GEMM and the LN-GEMM after it
// (no nos_split_rows_h3 pass, no fp16 planes of the activation):
//  * MODE 2 (producer): the epilogue also writes each row's statistics over
//    the tile's columns, (mean, M2 = sum (x - mean)^2), to sout[m][tn]
//    (spart = tiles_n parts of BN columns): the fp32 tile goes through LDS,
//    two threads per row, two-pass in registers, Chan's merge of the halves;
//  * MODE 1 (consumer): A is the fp32 rows X themselves; a workgroup merges
//    each of its rows' part statistics (Chan), and every stage's A tile is
//    loaded into registers, normalised ((x - mean) rstd 2^eln, the sqrt(K)
//    bound's scale) and split into the h3 planes in LDS -- what the split
//    pass did, one K-slice at a time, under the previous stage's MFMAs.
struct LnIo {
  const float* x = nullptr;     // MODE 1: A rows (fp32, row stride ldx)
  const float2* sin = nullptr;  // MODE 1: part statistics [M][nparts], parts of pw columns
  float2* sout = nullptr;       // MODE 2: [M][spart]
  int ldx = 0, nparts = 0, pw = 0, spart = 0;
  float eps = 0.f, sc = 1.f;    // MODE 1: LayerNorm eps, 2^eln
};

// Chan et al.'s pairwise update of (count, mean, M2) with a part (nb, mb, m2b)
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float mb, float m2b) {
  const float tot = n + nb;
  if (!(nb > 0.f)) return;
  const float d = mb - mean, f = nb / tot;
  mean = fmaf(d, f, mean);
  m2 += m2b + d * d * n * f;
  n = tot;
}

// BKT: K depth of an LDS stage (32: two 16-deep MFMA steps, or 16: one);
// RS: stages in the ring (RS - 1 of them in flight ahead of the one computed)
// BATCHED: the tile index spans nb batch elements (Batch strides); false: one
// GEMM, no per-tile batch offsets (fewer live SGPRs in the hot path)
// MODE: 0 A as planes (LDS-DMA); 1 A = LayerNorm(X) (LnIo); 2 row statistics out
template <int BM, int BN, int WGM, int WGN, bool PERSIST, int BKT = 32, int RS = 2, int MODE = 0,
          bool BATCHED = false>
__global__ __launch_bounds__(64 * WGM * WGN, WGM * WGN > 4 ? 1 : 2) void gemm_h3_kernel(
    const _Float16* __restrict__ Ap, int lda, long long aplane, const float* __restrict__ rinv, float rconst,
    const _Float16* __restrict__ Wp, int ldw, long long wplane, const float* __restrict__ csc,
    const float* __restrict__ bias, const float* __restrict__ R, int ldr0, float* __restrict__ C, int ldc0, int M,
    int N, int K, int epi, int tiles_m, int tiles_n, KvOut kv, PlaneOut po, Batch bt, LnIo ln) {
  constexpr int NW = WGM * WGN, MI = BM / (32 * WGM), NI = BN / (32 * WGN);
  static_assert((NW == 4 || NW == 8) && MI >= 1 && NI >= 1, "4 or 8 waves");
  constexpr int ROWB = BKT * 2, CH = ROWB / 16, RPP = 1024 / ROWB, NSTEP = BKT / 16;
  static_assert((BKT == 32 || BKT == 16) && RS >= 2 && RS <= 4, "stage shape");
  constexpr int TA = 2 * BM * ROWB, STAGE = TA + 2 * BN * ROWB;
  constexpr int APW = TA / 1024 / NW, WPW = 2 * BN * ROWB / 1024 / NW;  // 1 KiB DMA pieces per wave
  static_assert(APW * NW * 1024 == TA && WPW * NW * 1024 == 2 * BN * ROWB, "equal DMA count per wave");
  constexpr int LPS = APW + WPW;
  static_assert((RS - 2) * LPS < 64, "vmcnt range");
  static_assert(MODE == 0 || (BM == 128 && BKT == 32 && !BATCHED &&
                              (((BN == 128 || BN == 64) && NW == 4 && (RS == 2 || (MODE == 2 && RS == 3))) ||
                               (MODE == 1 && BN == 256 && NW == 8 && RS == 2))),
                "the LayerNorm hand-off runs 128 x 128 or 128 x 64 2 x 2 tiles (the producer also on a 3-deep ring); "
                "the LN-in-A-load also 128 x 256 with 2 x 4 waves");
  static_assert(MODE != 2 || BM * BN * 4 <= RS * STAGE, "the statistics tile fits the ring");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int c0 = lane & 31, h0 = lane >> 5;
  const int wm = wid / WGN, wn = wid % WGN;
  const bool wide = (epi & EPI_WIDE) != 0;
  epi &= ~EPI_WIDE;
  const int ntiles1 = tiles_m * tiles_n, ntiles = BATCHED ? ntiles1 * bt.nb : ntiles1;
  const int nk = K / BKT;
  nos::XcdChunk chunk;
  if constexpr (PERSIST) {
    chunk = nos::xcd_chunk(blockIdx.x, gridDim.x, ntiles);
  } else {
    chunk.first = nos::xcd_remap(blockIdx.x, ntiles);
    chunk.end = chunk.first + 1;
    chunk.step = 1;
  }
  for (int tt = chunk.first; tt < chunk.end; tt += chunk.step) {
    if (PERSIST && tt != chunk.first) __syncthreads();
    const int bb = BATCHED ? tt / ntiles1 : 0, t1 = BATCHED ? tt - bb * ntiles1 : tt;
    const int tm = t1 / tiles_n, tn = t1 - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    // this tile's batch element (wave-uniform scalar offsets)
    const _Float16* __restrict__ Ab = BATCHED ? Ap + bb * bt.a : Ap;
    const _Float16* __restrict__ Wb = BATCHED ? Wp + bb * bt.w : Wp;
    const float* __restrict__ rinvb = BATCHED && rinv != nullptr ? rinv + bb * bt.rinv : rinv;
    const float* __restrict__ cscb = BATCHED ? csc + bb * bt.csc : csc;
    float* __restrict__ Cb = BATCHED && C != nullptr ? C + bb * bt.c : C;
    const float* __restrict__ Rb = BATCHED && R != nullptr ? R + bb * bt.r : R;
    const float* __restrict__ biasb = BATCHED && bias != nullptr ? bias + bb * bt.bias : bias;

    // a 1 KiB piece = RPP rows x ROWB bytes of one plane; lane L: row L / CH, chunk L % CH
    auto stage_a = [&](int k0, unsigned char* dst) {
#pragma unroll
      for (int i = 0; i < APW; ++i) {
        const int p = wid * APW + i;
        const int plane = p / (BM / RPP), rb = (p % (BM / RPP)) * RPP;
        const int row = rb + lane / CH;
        int g = m0 + row;
        g = g < M ? g : M - 1;
        glds16(Ab + plane * aplane + (long long)g * lda + k0 + (((lane % CH) ^ swz<CH>(row)) << 3),
               dst + plane * BM * ROWB + rb * ROWB);
      }
    };
    auto stage_w = [&](int k0, unsigned char* dst) {
#pragma unroll
      for (int i = 0; i < WPW; ++i) {
        const int p = wid * WPW + i;
        const int plane = p / (BN / RPP), rb = (p % (BN / RPP)) * RPP;
        const int row = rb + lane / CH;
        int g = n0 + row;
        g = g < N ? g : N - 1;
        glds16(Wb + plane * wplane + (long long)g * ldw + k0 + (((lane % CH) ^ swz<CH>(row)) << 3),
               dst + TA + plane * BN * ROWB + rb * ROWB);
      }
    };
    auto stage = [&](int k0, unsigned char* dst) {
      stage_a(k0, dst);
      stage_w(k0, dst);
    };

    f32x16_t acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    struct Frag {
      f16x8_t a[MI][2], w[NI][2];
    };
    // fragments of 16-deep step s (0 / 1) of the stage at base
    auto load = [&](const unsigned char* base, int s, Frag& f) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * (BM / WGM) + i * 32 + c0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
          f.a[i][p] = *reinterpret_cast<const f16x8_t*>(base + p * BM * ROWB + row * ROWB +
                                                        (((NSTEP * s + h0) ^ swz<CH>(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wn * (BN / WGN) + j * 32 + c0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
          f.w[j][p] = *reinterpret_cast<const f16x8_t*>(base + TA + p * BN * ROWB + row * ROWB +
                                                        (((NSTEP * s + h0) ^ swz<CH>(row)) << 4));
      }
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = nos::mma3h(f.a[i], f.w[j], acc[i][j]);
    };

    if constexpr (MODE == 1) {
    // A = LayerNorm(X): thread t owns rows t/4 and 64 + t/4 of the tile and the
    // 8-deep k chunk t%4 of each stage (one 16-byte piece per plane and row)
    constexpr int AR = BM * 4 / (64 * NW);   // rows per thread: 2 with 4 waves, 1 with 8
    constexpr int RSTEP = 64 * NW / 4;       // rows between a thread's rows
    const int q = tid & 3;
    float mul[AR], add[AR];
    const float* xr[AR];
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      int g = m0 + (tid >> 2) + RSTEP * i;
      g = g < M ? g : M - 1;
      xr[i] = ln.x + (long long)g * ln.ldx + q * 8;
      const float2* st = ln.sin + (long long)g * ln.nparts;
      float n = 0.f, mean = 0.f, m2 = 0.f;
      for (int p = 0; p < ln.nparts; ++p) {
        const float2 v = st[p];
        const int nb = min(ln.pw, K - p * ln.pw);
        chan_merge(n, mean, m2, (float)nb, v.x, v.y);
      }
      mul[i] = rsqrtf(m2 / (float)K + ln.eps) * ln.sc;
      add[i] = -mean * mul[i];
    }
    float4 xa[AR][2];
    auto aload = [&](int k0) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        xa[i][0] = *reinterpret_cast<const float4*>(xr[i] + k0);
        xa[i][1] = *reinterpret_cast<const float4*>(xr[i] + k0 + 4);
      }
    };
    auto awrite = [&](unsigned char* dst) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int row = (tid >> 2) + RSTEP * i;
        const float4 u = xa[i][0], w = xa[i][1];
        f16x2_t h0, l0, h1, l1, h2, l2, h3, l3;
        nos::split2h(f32x2_t{fmaf(u.x, mul[i], add[i]), fmaf(u.y, mul[i], add[i])}, h0, l0);
        nos::split2h(f32x2_t{fmaf(u.z, mul[i], add[i]), fmaf(u.w, mul[i], add[i])}, h1, l1);
        nos::split2h(f32x2_t{fmaf(w.x, mul[i], add[i]), fmaf(w.y, mul[i], add[i])}, h2, l2);
        nos::split2h(f32x2_t{fmaf(w.z, mul[i], add[i]), fmaf(w.w, mul[i], add[i])}, h3, l3);
        const int off = row * ROWB + ((q ^ swz<CH>(row)) << 4);
        *reinterpret_cast<f16x8_t*>(dst + off) = f16x8_t{h0.x, h0.y, h1.x, h1.y, h2.x, h2.y, h3.x, h3.y};
        *reinterpret_cast<f16x8_t*>(dst + BM * ROWB + off) = f16x8_t{l0.x, l0.y, l1.x, l1.y, l2.x, l2.y, l3.x, l3.y};
      }
    };
    aload(0);
    stage_w(0, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    awrite(smem);
    if (nk > 1) {
      aload(BKT);
      stage_w(BKT, smem + STAGE);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    Frag fa, fb;
    load(smem, 0, fa);
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* cur = smem + (kt & 1) * STAGE;
      load(cur, 1, fb);
      mma(fa);
      __builtin_amdgcn_sched_barrier(0);
      // stage kt+1's A rows (registers) landed: normalised and split into the
      // buffer every wave finished reading last iteration, under fa's MFMAs
      if (kt + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        awrite(smem + ((kt + 1) & 1) * STAGE);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(fb);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) {
        // the barrier (stage kt+1 complete, stage kt read by every wave) waits under fb's MFMAs
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) {
          aload((kt + 2) * BKT);
          stage_w((kt + 2) * BKT, smem + (kt & 1) * STAGE);
        }
        load(smem + ((kt + 1) & 1) * STAGE, 0, fa);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    } else if constexpr (BKT == 32 && RS == 2) {
    stage(0, smem);
    if (nk > 1) stage(BKT, smem + STAGE);
    if (nk > 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");  // stage 0 landed, stage 1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    Frag fa, fb;
    load(smem, 0, fa);
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* cur = smem + (kt & 1) * STAGE;
      load(cur, 1, fb);  // step 1 read under step 0's MFMAs
      mma(fa);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) {
        // stage kt+1 landed (the only DMA in flight); every wave has read stage kt
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) stage((kt + 2) * BKT, smem + (kt & 1) * STAGE);
        load(smem + ((kt + 1) & 1) * STAGE, 0, fa);  // next stage's step 0 under step 1's MFMAs
      }
      mma(fb);
      __builtin_amdgcn_sched_barrier(0);
    }
    } else {
    // deep ring: RS - 1 stages in flight ahead of the one computed
#pragma unroll
    for (int q = 0; q < RS - 1; ++q)
      if (q < nk) stage(q * BKT, smem + q * STAGE);
    for (int kt = 0; kt < nk; ++kt) {
      // stage kt landed (later ones may stay in flight); every wave is done
      // with stage kt - 1, whose buffer stage kt + RS - 1 reuses
      wait_stages<LPS>(min(RS - 2, nk - 1 - kt));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + RS - 1 < nk) stage((kt + RS - 1) * BKT, smem + ((kt + RS - 1) % RS) * STAGE);
      const unsigned char* cur = smem + (kt % RS) * STAGE;
      Frag f0;
      load(cur, 0, f0);
      if constexpr (NSTEP == 2) {
        Frag f1;
        load(cur, 1, f1);
        mma(f0);
        mma(f1);
      } else {
        mma(f0);
      }
    }
    }
    __syncthreads();  // every wave is done with the ring (the next tile's prologue)

    // epilogue: register r of lane (c, h) = row (r&3) + 8(r>>2) + 4h of the block, column c.
    // Persistent loops: the lane coordinates are re-materialised per tile (opaque
    // copies), so the compiler cannot hoist the epilogue's 16 MI NI per-lane
    // offsets out of the tile loop and keep them live across the K loop (that
    // hoisting spilled the PERSIST variants: 200+ VGPRs to scratch)
    int c = c0, h = h0, ldc = ldc0, ldr = ldr0;
    asm volatile("" : "+v"(c), "+v"(h));
    asm volatile("" : "+s"(ldc), "+s"(ldr));
    float rsv[MI][16], rbv[MI][16];  // row scales; row bias (conv: per output channel)
    if (rinvb != nullptr) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          rsv[i][r] = rinvb[m < M ? m : M - 1];
        }
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) rsv[i][r] = rconst;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        rbv[i][r] = (BATCHED && (epi & EPI_BIAS_ROW)) ? biasb[m < M ? m : M - 1] : 0.f;
      }
    // the interior epilogues, instantiated per flag combination (EpiC<E>): with
    // runtime flags the compiler kept a branch per element and flag (hundreds
    // of basic blocks); E < 0 is the generic runtime-flag form.  true: done
    auto epilogue = [&](auto ec) -> bool {
      constexpr int E = decltype(ec)::value;
      auto has = [&](int f) -> bool {
        if constexpr (E < 0) return (epi & f) != 0;
        else return (E & f) != 0;
      };
      if constexpr (MODE == 2) {
        // (without sout: only the epilogue, plain fp32 C through LDS)
        // the tile goes to C through LDS: act(acc scale + bias) in the MFMA
        // layout into T (row stride BN), then threads 2r, 2r+1 take the two
        // 64-column halves of row r (16-byte chunks in a per-lane rotation:
        // conflict-free), add the residual, store C as float4 and reduce the
        // row's (mean, M2) over the valid columns; Chan's merge of the halves
        float* const T = reinterpret_cast<float*>(smem);
  #pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cl = wn * (BN / WGN) + j * 32 + c;
          const int nc = n0 + cl < N ? n0 + cl : N - 1;
          const float cs = cscb[nc];
          const float p2 = has(EPI_BIAS) ? biasb[nc] : 0.f;
  #pragma unroll
          for (int i = 0; i < MI; ++i) {
  #pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              float v = fmaf(acc[i][j][r], rsv[i][r] * cs, p2);
              if (has(EPI_GELU)) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
              if (has(EPI_RELU)) v = fmaxf(v, 0.f);
              T[rl * BN + cl] = v;
            }
          }
        }
        __syncthreads();
        const int rr = tid >> 1, hf = tid & 1, m = m0 + rr;
        const int nv = m < M ? max(0, min(BN / 2, N - n0 - hf * (BN / 2))) : 0;
        const float* tr = T + rr * BN + hf * (BN / 2);
        const long long col0 = n0 + hf * (BN / 2);
        constexpr int HV = BN / 8;  // float4s per row half
        float4 v[HV];
        // sout == nullptr: the plain LDS epilogue (no statistics); a whole row
        // half (every tile of N % BN == 0) without per-chunk tests
        const bool want = ln.sout != nullptr;
        float sum = 0.f;
        auto pass1 = [&](auto wholec) {
          constexpr bool W = decltype(wholec)::value;
  #pragma unroll
          for (int u = 0; u < HV; ++u) {
            const int k = ((u + tid) & (HV - 1)) * 4;
            v[u] = *reinterpret_cast<const float4*>(tr + k);
            if (W || k < nv) {
              if (has(EPI_RESID)) {
                const float4 q = *reinterpret_cast<const float4*>(Rb + (long long)m * ldr + col0 + k);
                v[u].x += q.x;
                v[u].y += q.y;
                v[u].z += q.z;
                v[u].w += q.w;
              }
              *reinterpret_cast<float4*>(Cb + (long long)m * ldc + col0 + k) = v[u];
              if (want) sum += (v[u].x + v[u].y) + (v[u].z + v[u].w);
            }
          }
        };
        if (nv == BN / 2) pass1(std::true_type{});
        else pass1(std::false_type{});
        if (want) {
          const float mean = nv > 0 ? sum / (float)nv : 0.f;
          float m2 = 0.f;
  #pragma unroll
          for (int u = 0; u < HV; ++u) {
            const int k = ((u + tid) & (HV - 1)) * 4;
            if (k < nv) {
              const float d0 = v[u].x - mean, d1 = v[u].y - mean, d2 = v[u].z - mean, d3 = v[u].w - mean;
              m2 = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, m2))));
            }
          }
          float n = (float)nv, mu = mean;
          const float on = __shfl_xor(n, 1, 64), omu = __shfl_xor(mu, 1, 64), om2 = __shfl_xor(m2, 1, 64);
          if (hf == 0 && n + on > 0.f) {
            chan_merge(n, mu, m2, on, omu, om2);
            ln.sout[(long long)m * ln.spart + tn] = float2{mu, m2};
          }
        }
        return true;
      }
      // interior tile stored as fp32 C (the common case): tile-local 32-bit
      // offsets from wave-uniform base pointers (saddr stores, no 64-bit
      // address math per element) and no bounds tests
      const bool full = m0 + BM <= M && n0 + BN <= N;
      // interior tile of the next GEMM's A planes (fc1 -> fc2) or of the K / V
      // planes of a one-sequence QKV projection (a 128-column tile never
      // straddles Q / K / V: hd % 128 == 0 is checked by the host): the same
      // tile-relative 32-bit offsets, two fp16 stores per element
      if (full && !(has(EPI_RESID) || has(EPI_RESID_PRE)) &&
          (po.p != nullptr || (kv.kvs != nullptr && kv.S == M && n0 >= kv.qcols && kv.hd % BN == 0))) {
        unsigned short* hi;
        long long lo_off;
        int ld;
        int t = 0;
        if (po.p != nullptr) {
          hi = po.p + (long long)m0 * po.ldp + n0;
          lo_off = po.pplane;
          ld = po.ldp;
        } else {
          t = (n0 - kv.qcols) >= kv.hd;
          hi = kv.kvs + ((long long)m0 * 4 + 2 * t) * kv.hd + (n0 - kv.qcols - t * kv.hd);
          lo_off = kv.hd;
          ld = 4 * kv.hd;
        }
        // wide: the tile's two planes in LDS (the ring is free: every wave passed the
        // K loop's last barrier), 16-byte chunks XOR-swizzled by row, then each
        // thread stores whole 16-byte row chunks of both planes
        constexpr bool WIDE_FITS = 4 * BM * BN <= RS * STAGE && !BATCHED && (BN == 128 || BN == 64);
        constexpr int SWM = BN / 8 - 1;  // 16-byte chunk swizzle mask of a tile row
        unsigned short* const T = reinterpret_cast<unsigned short*>(smem);
  #pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cl = wn * (BN / WGN) + j * 32 + c;
          const float cs = cscb[n0 + cl];
          const float p2 = has(EPI_BIAS) ? biasb[n0 + cl] : 0.f;
          const float osc = po.p != nullptr ? po.sc : kv.kvsc[t * (kv.hd >> 6) + ((n0 - kv.qcols - t * kv.hd + cl) >> 6)];
  #pragma unroll
          for (int i = 0; i < MI; ++i) {
  #pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              float v = fmaf(acc[i][j][r], rsv[i][r] * cs, p2 + rbv[i][r]);
              if (has(EPI_GELU)) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
              if (has(EPI_RELU)) v = fmaxf(v, 0.f);
              const float x = v * osc;
              const _Float16 h0 = (_Float16)x;
              const _Float16 h1 = (_Float16)(x - (float)h0);
              if (WIDE_FITS && wide) {
                const int sl = rl * BN + ((((cl >> 3) ^ (rl & SWM)) << 3) | (cl & 7));
                T[sl] = __builtin_bit_cast(unsigned short, h0);
                T[BM * BN + sl] = __builtin_bit_cast(unsigned short, h1);
              } else {
                const unsigned off = (unsigned)(rl * ld + cl);
                hi[off] = __builtin_bit_cast(unsigned short, h0);
                hi[lo_off + off] = __builtin_bit_cast(unsigned short, h1);
              }
            }
          }
        }
        if (WIDE_FITS && wide) {
          __syncthreads();
          constexpr int CPR = BN / 8;                     // 16-byte chunks per tile row
          constexpr int NCH = 2 * BM * CPR;               // both planes
  #pragma unroll
          for (int q = 0; q < NCH / (64 * NW); ++q) {
            const int id = tid + q * 64 * NW;
            const int pl = id / (BM * CPR), rem = id - pl * (BM * CPR);
            const int row = rem / CPR, ch = rem - row * CPR;
            const uint4 v = *reinterpret_cast<const uint4*>(T + pl * BM * BN + row * BN + ((ch ^ (row & SWM)) << 3));
            *reinterpret_cast<uint4*>(hi + pl * lo_off + (long long)row * ld + ch * 8) = v;
          }
        }
        return true;
      }
      const bool interior = full && po.p == nullptr && (kv.kvs == nullptr || n0 + BN <= kv.qcols);  // Q columns too
      if (interior) {
        float* Ct = Cb + (long long)m0 * ldc + n0;
        const float* Rt = has(EPI_RESID) || (BATCHED && has(EPI_RESID_PRE)) ? Rb + (long long)m0 * ldr + n0 : nullptr;
  #pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cl = wn * (BN / WGN) + j * 32 + c;
          const float cs = cscb[n0 + cl];
          const float p2 = has(EPI_BIAS) ? biasb[n0 + cl] : 0.f;
  #pragma unroll
          for (int i = 0; i < MI; ++i) {
  #pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              float v = fmaf(acc[i][j][r], rsv[i][r] * cs, p2 + rbv[i][r]);
              if (BATCHED && has(EPI_RESID_PRE)) v += Rt[(unsigned)(rl * ldr + cl)];
              if (has(EPI_GELU)) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
              if (has(EPI_RELU)) v = fmaxf(v, 0.f);
              if (has(EPI_RESID)) v += Rt[(unsigned)(rl * ldr + cl)];
              Ct[(unsigned)(rl * ldc + cl)] = v;
            }
          }
        }
        return true;
      }
      return false;
    };
    // interior tiles specialised for the flag sets each mode meets; boundary
    // tiles (and any other flag set) take the runtime-flag path below
    bool done = false;
    if constexpr (MODE == 1) {
      if (epi == EPI_BIAS) done = epilogue(EpiC<EPI_BIAS>{});
      else if (epi == (EPI_BIAS | EPI_GELU)) done = epilogue(EpiC<EPI_BIAS | EPI_GELU>{});
      else done = epilogue(EpiC<-1>{});
    } else if constexpr (MODE == 2) {
      if (epi == (EPI_BIAS | EPI_RESID)) done = epilogue(EpiC<EPI_BIAS | EPI_RESID>{});
      else if (epi == EPI_BIAS) done = epilogue(EpiC<EPI_BIAS>{});
      else done = epilogue(EpiC<-1>{});
    } else if constexpr (BATCHED) {
      done = epilogue(EpiC<-1>{});
    } else {
      switch (epi) {
        case EPI_BIAS: done = epilogue(EpiC<EPI_BIAS>{}); break;
        case EPI_BIAS | EPI_GELU: done = epilogue(EpiC<EPI_BIAS | EPI_GELU>{}); break;
        case EPI_BIAS | EPI_RESID: done = epilogue(EpiC<EPI_BIAS | EPI_RESID>{}); break;
        default: done = epilogue(EpiC<-1>{}); break;
      }
    }
    if (done) continue;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wn * (BN / WGN) + j * 32 + c;
      const int nc = n < N ? n : N - 1;
      const float cs = cscb[nc];
      const float p2 = (epi & EPI_BIAS) ? biasb[nc] : 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          float v = fmaf(acc[i][j][r], rsv[i][r] * cs, p2 + rbv[i][r]);
          if (BATCHED && (epi & EPI_RESID_PRE) && m < M && n < N) v += Rb[(long long)m * ldr + n];
          if ((epi & EPI_GELU)) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
          if ((epi & EPI_RELU)) v = fmaxf(v, 0.f);
          if (m < M && n < N) {
            if ((epi & EPI_RESID)) v += Rb[(long long)m * ldr + n];
            if (kv.kvs != nullptr && n >= kv.qcols) {
              const int t = (n - kv.qcols) >= kv.hd;  // 0: K, 1: V
              const int col = n - kv.qcols - t * kv.hd;
              const int b = kv.S == M ? 0 : m / kv.S;
              const long long row = (long long)b * kv.skvp + (m - b * kv.S);
              const float x = v * kv.kvsc[t * (kv.hd >> 6) + (col >> 6)];
              const _Float16 h0 = (_Float16)x;
              const _Float16 h1 = (_Float16)(x - (float)h0);
              unsigned short* dst = kv.kvs + (row * 4 + 2 * t) * kv.hd + col;
              dst[0] = __builtin_bit_cast(unsigned short, h0);
              dst[kv.hd] = __builtin_bit_cast(unsigned short, h1);
            } else if (po.p != nullptr) {
              const float x = v * po.sc;
              const _Float16 h0 = (_Float16)x;
              const _Float16 h1 = (_Float16)(x - (float)h0);
              po.p[(long long)m * po.ldp + n] = __builtin_bit_cast(unsigned short, h0);
              po.p[po.pplane + (long long)m * po.ldp + n] = __builtin_bit_cast(unsigned short, h1);
            } else {
              Cb[(long long)m * ldc + n] = v;
            }
          }
        }
      }
    }
  }  // tiles
}

// LDS-staged 16-byte plane stores (EPI_WIDE) for the interior tiles of GEMMs
// that write fp16 planes (fc1 -> fc2, the QKV projection's K / V);
// NOS_AMD_H3_WIDE_PLANES=0 keeps the 2-byte stores (A/B runs)
bool g_wide_planes = [] {
  const char* e = getenv("NOS_AMD_H3_WIDE_PLANES");
  return e == nullptr || atoi(e) != 0;
}();

// the plane destinations of EPI_WIDE take 16-byte stores at every tile's rows
bool wide_planes_ok(const KvOut& kv, const PlaneOut& po) {
  if (!g_wide_planes) return false;
  if (po.p != nullptr)
    return !(((uintptr_t)po.p) & 15) && !(po.ldp % 8) && !(po.pplane % 8);
  if (kv.kvs != nullptr) return !(((uintptr_t)kv.kvs) & 15) && !(kv.hd % 8) && !(kv.qcols % 8);
  return false;
}

template <int BM, int BN, int WGM, int WGN, int BKT = 32, int RS = 2, bool BATCHED = false, int MODE = 0>
int launch_t(const _Float16* Ap, int lda, long long aplane, const float* rinv, float rconst, const _Float16* Wp,
             int ldw, long long wplane, const float* csc, const float* bias, const float* R, int ldr, float* C, int ldc,
             int M, int N, int K, int epi, KvOut kv, PlaneOut po, Batch bt, hipStream_t st, LnIo ln = LnIo{}) {
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const long long ntiles = (long long)tiles_m * tiles_n * bt.nb;
  if (ntiles > (1LL << 30)) return (int)hipErrorInvalidValue;
  const size_t lds = RS * (size_t)(2 * BM * BKT * 2 + 2 * BN * BKT * 2);
  constexpr int NT = 64 * WGM * WGN;
  if (!BATCHED && wide_planes_ok(kv, po)) epi |= EPI_WIDE;
  // batched GEMMs always launch one workgroup per tile: their persistent
  // form (a CU slice's capped grid) needs 21 more VGPRs than 256 and spilled
  // to scratch; the CU mask bounds where the tiles run either way
  if constexpr (!BATCHED) {
    const int grid =
        nos_grid_for((const void*)gemm_h3_kernel<BM, BN, WGM, WGN, true, BKT, RS, MODE, BATCHED>, NT, lds, ntiles);
    if (grid < ntiles) {
      hipLaunchKernelGGL((gemm_h3_kernel<BM, BN, WGM, WGN, true, BKT, RS, MODE, BATCHED>), dim3((unsigned)grid),
                         dim3(NT), lds, st, Ap, lda, aplane, rinv, rconst, Wp, ldw, wplane, csc, bias, R, ldr, C, ldc,
                         M, N, K, epi, tiles_m, tiles_n, kv, po, bt, ln);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_h3_kernel<BM, BN, WGM, WGN, false, BKT, RS, MODE, BATCHED>), dim3((unsigned)ntiles),
                     dim3(NT), lds, st, Ap, lda, aplane, rinv, rconst, Wp, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N,
                     K, epi, tiles_m, tiles_n, kv, po, bt, ln);
  return (int)hipGetLastError();
}

// nos_gemm_f32h3_set_layout: 0: 128x128, 4 x 1 waves; 1: 128x128, 2 x 2;
// 2: 256x128, 4 x 2 (8 waves); 3: 128x128 4 x 1, 3-deep ring of BK-32
// stages (96 KiB); 4 / 5: 128x128 4 x 1 / 2 x 2, 4-deep ring of BK-16 stages.
// Default 2 x 2: 64 x 64 per wave reads 8 KiB of fragments per 12 MFMAs
// (4 x 1: 10 KiB); 28-tenant fleet 679.9 / 679.8 vs 679.0 / 676.2 inf/s,
// the deeper rings 605-635 (profiles/r04_h3_layout_ab.json)
int g_layout = 1;
// plain fp32-C GEMMs (no KV / plane output, N % 4 == 0, aligned C / R) through
// the LDS epilogue of MODE 2 (float4 stores and residual loads along rows)
bool g_lds_epi = true;  // 28-tenant fleet 801 vs 799 inf/s, batch-1 residual GEMMs 15-18 % faster
// LDS ring depth of the LDS-epilogue / row-statistics (MODE 2) GEMMs: 2 (64 KiB, two
// workgroups per CU) or 3 (96 KiB, one workgroup per CU, stage k+2 in flight under k):
// 28-tenant fleet 792 (3) vs 802 (2) inf/s, profiles/r06_packed_epilogue_rejected.json
int g_hot_ring = 2;
// tile width of the row-statistics producers and LDS-epilogue GEMMs (the
// residual GEMMs of a transformer): 128, or 64 (48 KiB ring: three workgroups
// per CU); the statistics parts are this many columns wide
int g_hot_bn = 128;
// LN-in-A-load GEMMs that write the next GEMM's planes (fc1 -> fc2) on 128 x 256
// tiles with 8 waves: half the per-workgroup A normalise-and-split work per MFMA
bool g_lna_wide = false;

// ------------------------------------------------------------ row split
// LPR lanes per row (64: a wave; 32: a half-wave, two rows per wave), the
// whole row in registers (F4 float4s per lane: K <= 4 LPR F4): one read of
// the row, its scale (max |a|, or in LayerNorm mode the mean / variance and
// the host's sqrt(K) bound of a normalised row), then its hi / lo planes.
// F4 = 0: rows longer than 4096, re-read per pass.
template <int F4, int LPR = 64>
__global__ __launch_bounds__(256) void split_rows_h3_kernel(const float* __restrict__ A, int lda,
                                                            _Float16* __restrict__ P, int ldp, long long pplane,
                                                            float* __restrict__ rinv, int M, int K, int ln,
                                                            float eps, int eln) {
  typedef __attribute__((ext_vector_type(4))) _Float16 f16x4_t;
  constexpr int RPB = 256 / LPR;  // rows per block
  const int row = blockIdx.x * RPB + (int)(threadIdx.x / LPR);
  const int lane = threadIdx.x % LPR;
  if (row >= M) return;  // whole half-waves: LPR-lane reductions never mix a live and a retired row
  const float* a = A + (long long)row * lda;
  constexpr int NR = F4 > 0 ? F4 : 1;
  float4 v[NR];
  auto get = [&](int i, int k) -> float4 {  // chunk i of this lane (k = its first column)
    if constexpr (F4 > 0) return v[i];
    return *reinterpret_cast<const float4*>(a + k);
  };
  const int nchunk = F4 > 0 ? F4 : (K + 4 * LPR - 1) / (4 * LPR);
  if constexpr (F4 > 0) {
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int k = (lane + LPR * i) * 4;
      v[i] = k < K ? *reinterpret_cast<const float4*>(a + k) : float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float mu = 0.f, rs = 1.f;
  int e;
  if (ln == 2) {  // RMSNorm: x / sqrt(mean(x^2) + eps) (gamma folded into the weight)
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < nchunk; ++i) {
      const int k = (lane + LPR * i) * 4;
      if (k < K) {
        const float4 x = get(i, k);
        q = fmaf(x.x, x.x, fmaf(x.y, x.y, fmaf(x.z, x.z, fmaf(x.w, x.w, q))));
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    rs = rsqrtf(q / (float)K + eps);
    e = eln;  // |x^| <= sqrt(K) for an RMS-normalised row too
  } else if (ln) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < nchunk; ++i) {
      const int k = (lane + LPR * i) * 4;
      if (k < K) {
        const float4 x = get(i, k);
        s += (x.x + x.y) + (x.z + x.w);
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    mu = s / (float)K;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < nchunk; ++i) {
      const int k = (lane + LPR * i) * 4;
      if (k < K) {
        const float4 x = get(i, k);
        const float d0 = x.x - mu, d1 = x.y - mu, d2 = x.z - mu, d3 = x.w - mu;
        q = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, q))));
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    rs = rsqrtf(q / (float)K + eps);
    e = eln;  // |x^| <= sqrt(K): the host's exponent for it
  } else {
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < nchunk; ++i) {
      const int k = (lane + LPR * i) * 4;
      if (k < K) {
        const float4 x = get(i, k);
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))));
      }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    e = nos::h3_scale_exp(mx);
  }
  const float sc = nos::pow2i(e);
  const float mul = rs * sc, add = -mu * mul;
  _Float16* ph = P + (long long)row * ldp;
  _Float16* pl = ph + pplane;
#pragma unroll
  for (int i = 0; i < nchunk; ++i) {
    const int k = (lane + LPR * i) * 4;
    if (k < K) {
      const float4 x = get(i, k);
      f16x2_t h01, l01, h23, l23;
      nos::split2h(f32x2_t{fmaf(x.x, mul, add), fmaf(x.y, mul, add)}, h01, l01);
      nos::split2h(f32x2_t{fmaf(x.z, mul, add), fmaf(x.w, mul, add)}, h23, l23);
      *reinterpret_cast<f16x4_t*>(ph + k) = f16x4_t{h01.x, h01.y, h23.x, h23.y};
      *reinterpret_cast<f16x4_t*>(pl + k) = f16x4_t{l01.x, l01.y, l23.x, l23.y};
    }
  }
  if (lane == 0) rinv[row] = nos::pow2i(-e);
}

// Column split (the transposed operand of a GEMM, training backward): the
// COLUMNS of fp32 X [M, K] (row stride ldx, batch stride bsx) become the rows
// of hi / lo fp16 planes [2][nb * K][ldp] (row b * K + k = column k of batch
// b, zero-padded from M to Mp = ldp's used length), each on its own
// power-of-two scale, rinv[b * K + k] = 2^-e: what transposing X into a
// contiguous copy and splitting its rows gave, without the strided copy.
// Pass 1: per column and row chunk, max |x| (coalesced along the rows).
constexpr int COLS_NCH = 32;  // row chunks of the column maxima
__global__ __launch_bounds__(256) void col_absmax_kernel(const float* __restrict__ X, int ldx, long long bsx, int M,
                                                         int K, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + tx, c = blockIdx.y, b = blockIdx.z;
  const int rpc = (M + COLS_NCH - 1) / COLS_NCH, m0 = c * rpc, m1 = min(M, m0 + rpc);
  const float* x = X + (long long)b * bsx;
  float mx = 0.f;
  if (k < K)
    for (int m = m0 + ty; m < m1; m += 4) mx = fmaxf(mx, fabsf(x[(long long)m * ldx + k]));
  red[ty][tx] = mx;
  __syncthreads();
  if (ty == 0 && k < K)
    part[((long long)b * COLS_NCH + c) * K + k] = fmaxf(fmaxf(red[0][tx], red[1][tx]), fmaxf(red[2][tx], red[3][tx]));
}

// Pass 2: a 64 x 64 tile of X through LDS; thread (k, q) writes 16
// consecutive row-elements of output row k as two 16-byte chunks per plane
__global__ __launch_bounds__(256) void split_cols_h3_kernel(const float* __restrict__ X, int ldx, long long bsx, int M,
                                                            int K, int Mp, const float* __restrict__ part,
                                                            _Float16* __restrict__ P, int ldp, long long pplane,
                                                            float* __restrict__ rinv) {
  __shared__ float tile[64][65];
  const int t = threadIdx.x, k0 = blockIdx.x * 64, m0 = blockIdx.y * 64, b = blockIdx.z;
  const float* x = X + (long long)b * bsx;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int e = t + 256 * i, r = e >> 6, cc = e & 63;
    const int m = m0 + r, k = k0 + cc;
    tile[r][cc] = (m < M && k < K) ? x[(long long)m * ldx + k] : 0.f;
  }
  __syncthreads();
  const int kk = t >> 2, q = t & 3, k = k0 + kk;
  if (k >= K || m0 + q * 16 >= Mp) return;
  float mx = 0.f;
#pragma unroll 8
  for (int c = 0; c < COLS_NCH; ++c) mx = fmaxf(mx, part[((long long)b * COLS_NCH + c) * K + k]);
  const int e = nos::h3_scale_exp(mx);
  const float sc = nos::pow2i(e);
  f16x2_t h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
    nos::split2h(f32x2_t{tile[q * 16 + 2 * j][kk] * sc, tile[q * 16 + 2 * j + 1][kk] * sc}, h[j], l[j]);
  _Float16* ph = P + ((long long)b * K + k) * ldp + m0 + q * 16;
  *reinterpret_cast<f16x8_t*>(ph) = f16x8_t{h[0].x, h[0].y, h[1].x, h[1].y, h[2].x, h[2].y, h[3].x, h[3].y};
  *reinterpret_cast<f16x8_t*>(ph + 8) = f16x8_t{h[4].x, h[4].y, h[5].x, h[5].y, h[6].x, h[6].y, h[7].x, h[7].y};
  *reinterpret_cast<f16x8_t*>(ph + pplane) = f16x8_t{l[0].x, l[0].y, l[1].x, l[1].y, l[2].x, l[2].y, l[3].x, l[3].y};
  *reinterpret_cast<f16x8_t*>(ph + pplane + 8) =
      f16x8_t{l[4].x, l[4].y, l[5].x, l[5].y, l[6].x, l[6].y, l[7].x, l[7].y};
  if (blockIdx.y == 0 && q == 0) rinv[(long long)b * K + k] = nos::pow2i(-e);
}

// per-row (mean, M2) of fp32 rows over all K columns (one statistics part): a
// half-wave per row, the row read twice (the second pass from cache)
__global__ __launch_bounds__(256) void row_stats_kernel(const float* __restrict__ X, int ldx, float2* __restrict__ out,
                                                        int M, int K) {
  const int row = blockIdx.x * 8 + (int)(threadIdx.x >> 5), lane = threadIdx.x & 31;
  if (row >= M) return;  // whole half-waves
  const float* x = X + (long long)row * ldx;
  float s = 0.f;
  for (int k = lane * 4; k < K; k += 128) {
    const float4 v = *reinterpret_cast<const float4*>(x + k);
    s += (v.x + v.y) + (v.z + v.w);
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mu = s / (float)K;
  float q = 0.f;
  for (int k = lane * 4; k < K; k += 128) {
    const float4 v = *reinterpret_cast<const float4*>(x + k);
    const float d0 = v.x - mu, d1 = v.y - mu, d2 = v.z - mu, d3 = v.w - mu;
    q = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, q))));
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  if (lane == 0) out[row] = float2{mu, q};
}

}  // namespace

// (mean, M2) of every fp32 row of X [M, K] (row stride ldx) into stats [M]
// (float2): the statistics input of nos_gemm_f32h3_lna (nparts 1, pw K) when
// the producer of X is not an h3 GEMM.  K % 4 == 0, rows 16-byte aligned.
NOS_API int nos_row_stats(const float* X, int ldx, void* stats, int M, int K, hipStream_t stream) {
  if (M <= 0 || K <= 0 || (K % 4) || (ldx % 4) || ldx < K || !X || !stats || (((uintptr_t)X) & 15) ||
      (((uintptr_t)stats) & 7))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(row_stats_kernel, dim3((unsigned)((M + 7) / 8)), dim3(256), 0, stream, X, ldx,
                     static_cast<float2*>(stats), M, K);
  return (int)hipGetLastError();
}

NOS_API int nos_gemm_f32h3_set_lds_epilogue(int on) {
  g_lds_epi = on != 0;
  return 0;
}

NOS_API int nos_gemm_f32h3_set_layout(int layout) {
  if (layout < 0 || layout > 7) return (int)hipErrorInvalidValue;
  g_layout = layout;
  return 0;
}

NOS_API int nos_gemm_f32h3_set_hot_bn(int bn) {
  if (bn != 128 && bn != 64) return (int)hipErrorInvalidValue;
  g_hot_bn = bn;
  return 0;
}

NOS_API int nos_gemm_f32h3_hot_bn() { return g_hot_bn; }

NOS_API int nos_gemm_f32h3_set_lna_wide(int on) {
  g_lna_wide = on != 0;
  return 0;
}

NOS_API int nos_gemm_f32h3_set_hot_ring(int rs) {
  if (rs != 2 && rs != 3) return (int)hipErrorInvalidValue;
  g_hot_ring = rs;
  return 0;
}

// Split the rows of fp32 A [M, K] (lda) into hi / lo fp16 planes P (row
// stride ldp, plane stride pplane elements) on per-row power-of-two scales,
// rinv[m] = 1 / scale.  ln != 0: the rows are LayerNorm-normalised first
// (no gamma / beta: those are folded into the weight and bias) and scaled by
// 2^eln (the host's bound for |x^| <= sqrt(K)); ln == 2: RMSNorm-normalised
// (x / sqrt(mean(x^2) + eps), same bound).  K % 4 == 0, rows 16-byte aligned.
NOS_API int nos_split_rows_h3(const float* A, int lda, void* P, int ldp, long long pplane, float* rinv, int M, int K,
                              int ln, float eps, int eln, hipStream_t stream) {
  if (M <= 0 || K <= 0 || (K % 4) || (lda % 4) || (ldp % 4) || ldp < K || pplane < (long long)M * ldp)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)A) | ((uintptr_t)P)) & 15) return (int)hipErrorInvalidValue;
  if (eln < -126 || eln > 126 || ln < 0 || ln > 2) return (int)hipErrorInvalidValue;
  auto* p = static_cast<_Float16*>(P);
  const dim3 grid((unsigned)((M + 3) / 4)), blk(256);
  if (K <= 512) {  // a half-wave per row: every lane busy at K = 384, one fewer reduction step
    const dim3 g2((unsigned)((M + 7) / 8));
    hipLaunchKernelGGL((split_rows_h3_kernel<4, 32>), g2, blk, 0, stream, A, lda, p, ldp, pplane, rinv, M, K, ln, eps,
                       eln);
  } else if (K <= 1024)
    hipLaunchKernelGGL(split_rows_h3_kernel<4>, grid, blk, 0, stream, A, lda, p, ldp, pplane, rinv, M, K, ln, eps, eln);
  else if (K <= 2048)
    hipLaunchKernelGGL(split_rows_h3_kernel<8>, grid, blk, 0, stream, A, lda, p, ldp, pplane, rinv, M, K, ln, eps, eln);
  else if (K <= 4096)
    hipLaunchKernelGGL(split_rows_h3_kernel<16>, grid, blk, 0, stream, A, lda, p, ldp, pplane, rinv, M, K, ln, eps,
                       eln);
  else
    hipLaunchKernelGGL(split_rows_h3_kernel<0>, grid, blk, 0, stream, A, lda, p, ldp, pplane, rinv, M, K, ln, eps, eln);
  return (int)hipGetLastError();
}

// The columns of fp32 X [nb][M, K] (row stride ldx, batch stride bsx; 16-byte
// aligned not required) as h3 plane rows: P [2][nb * K][ldp] (plane stride
// pplane elements), row b * K + k = column k of batch b over Mp = ceil32(M)
// elements (zeros past M), rinv [nb * K]; work: COLS_NCH * nb * K floats.
NOS_API int nos_split_cols_h3(const float* X, int ldx, long long bsx, int M, int K, int nb, void* P, int ldp,
                              long long pplane, float* rinv, float* work, hipStream_t stream) {
  const int Mp = (M + 31) / 32 * 32;
  if (M <= 0 || K <= 0 || nb <= 0 || ldx < K || (nb > 1 && bsx < (long long)(M - 1) * ldx + K) || ldp < Mp ||
      (ldp % 8) || pplane < (long long)nb * K * ldp || !X || !P || !rinv || !work || nb > 65535 ||
      (long long)(M + 63) / 64 > 65535)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)P) & 15) || (pplane % 8)) return (int)hipErrorInvalidValue;
  const unsigned gk = (unsigned)((K + 63) / 64);
  hipLaunchKernelGGL(col_absmax_kernel, dim3(gk, COLS_NCH, (unsigned)nb), dim3(256), 0, stream, X, ldx, bsx, M, K,
                     work);
  hipLaunchKernelGGL(split_cols_h3_kernel, dim3(gk, (unsigned)((Mp + 63) / 64), (unsigned)nb), dim3(256), 0, stream, X,
                     ldx, bsx, M, K, Mp, work, static_cast<_Float16*>(P), ldp, pplane, rinv);
  return (int)hipGetLastError();
}

namespace {

// batched: the BATCHED instantiation (batch strides, per-row bias, residual
// before the activation -- kept out of the one-GEMM kernels' registers)
int run_h3(const void* Ap, int lda, long long aplane, const float* rinv, float rconst, const void* Wp, int ldw,
           long long wplane, const float* csc, const float* bias, const float* R, int ldr, float* C, int ldc, int M,
           int N, int K, int epi, KvOut kv, PlaneOut po, Batch bt, hipStream_t stream, bool batched = false) {
  const auto* a = static_cast<const _Float16*>(Ap);
  const auto* w = static_cast<const _Float16*>(Wp);
  if (batched)  // batched GEMMs (convs, matmuls) on the default 128x128, 2 x 2 layout
    return launch_t<128, 128, 2, 2, 32, 2, true>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C,
                                                 ldc, M, N, K, epi, kv, po, bt, stream);
  if (g_layout == 3)
    return launch_t<128, 128, 4, 1, 32, 3>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M,
                                           N, K, epi, kv, po, bt, stream);
  if (g_layout == 4)
    return launch_t<128, 128, 4, 1, 16, 4>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M,
                                           N, K, epi, kv, po, bt, stream);
  if (g_layout == 5)
    return launch_t<128, 128, 2, 2, 16, 4>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M,
                                           N, K, epi, kv, po, bt, stream);
  if (g_layout == 7)  // 128 x 64 tiles (48 KiB ring: three workgroups per CU)
    return launch_t<128, 64, 2, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K,
                                   epi, kv, po, bt, stream);
  if (g_layout == 6)
    return launch_t<128, 128, 2, 2, 32, 3>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M,
                                           N, K, epi, kv, po, bt, stream);
  if (g_layout == 2)
    return launch_t<256, 128, 4, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K,
                                    epi, kv, po, bt, stream);
  if (g_layout == 1) {
    if (g_lds_epi && kv.kvs == nullptr && po.p == nullptr && C != nullptr && !(N % 4) && !(ldc % 4) &&
        !(((uintptr_t)C) & 15) && (!(epi & EPI_RESID) || (!(ldr % 4) && !(((uintptr_t)R) & 15)))) {
      if (g_hot_bn == 64)
        return launch_t<128, 64, 2, 2, 32, 2, false, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R,
                                                        ldr, C, ldc, M, N, K, epi, kv, po, bt, stream);
      if (g_hot_ring == 3)
        return launch_t<128, 128, 2, 2, 32, 3, false, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R,
                                                         ldr, C, ldc, M, N, K, epi, kv, po, bt, stream);
      return launch_t<128, 128, 2, 2, 32, 2, false, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr,
                                                       C, ldc, M, N, K, epi, kv, po, bt, stream);
    }
    return launch_t<128, 128, 2, 2>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K,
                                    epi, kv, po, bt, stream);
  }
  return launch_t<128, 128, 4, 1>(a, lda, aplane, rinv, rconst, w, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K,
                                  epi, kv, po, bt, stream);
}

}  // namespace

// C = act(rinv[m] csc[n] (A' . W'^T) + bias) (+ R) on the fp16 planes of A
// (nos_split_rows_h3, or a producer's plane output; rinv == nullptr: every
// row's inverse scale is rconst) and W ([2][N][K], ldw, plane stride wplane;
// row scales csc).  kvs != nullptr: a fused QKV projection (N = 3 hd) whose
// K / V columns go to the h3 attention's planes (S rows per batch padded to
// skvp, per-head scales kvsc [2][hd / 64]); Q to C.  P != nullptr: the
// output as the next h3 GEMM's A planes ([2][M][ldp], plane stride pplane)
// on the scale psc, instead of C.  K % 32 == 0.
NOS_API int nos_gemm_f32h3(const void* Ap, int lda, long long aplane, const float* rinv, float rconst,
                           const void* Wp, int ldw, long long wplane, const float* csc, const float* bias,
                           const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi, void* kvs, int S,
                           int skvp, const float* kvsc, void* P, int ldp, long long pplane, float psc,
                           hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8) || lda < K || ldw < K || aplane < (long long)M * lda || wplane < (long long)N * ldw)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)Ap) | ((uintptr_t)Wp)) & 15) return (int)hipErrorInvalidValue;
  if ((!rinv && !(rconst > 0.f)) || !csc || ((epi & EPI_BIAS) && !bias) || ((epi & EPI_RESID) && (!R || ldr < N)))
    return (int)hipErrorInvalidValue;
  if (((epi & EPI_BIAS_ROW) && ((epi & EPI_BIAS) || !bias)) || (epi & EPI_RESID_PRE)) return (int)hipErrorInvalidValue;
  KvOut kv;
  PlaneOut po;
  if (kvs != nullptr) {
    if (!kvsc || N % 3 || (N / 3) % 64 || S <= 0 || M % S || skvp < S || (((uintptr_t)kvs) & 15) || P)
      return (int)hipErrorInvalidValue;
    kv.kvs = static_cast<unsigned short*>(kvs);
    kv.kvsc = kvsc;
    kv.hd = N / 3;
    kv.qcols = kv.hd;
    kv.S = S;
    kv.skvp = skvp;
  }
  if (P != nullptr) {
    if (ldp < N || pplane < (long long)M * ldp || !(psc > 0.f)) return (int)hipErrorInvalidValue;
    po.p = static_cast<unsigned short*>(P);
    po.ldp = ldp;
    po.pplane = pplane;
    po.sc = psc;
  } else if (ldc < (kvs != nullptr ? N / 3 : N)) {
    return (int)hipErrorInvalidValue;
  }
  return run_h3(Ap, lda, aplane, rinv, rconst, Wp, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K, epi, kv, po,
                Batch{}, stream);
}

// nb independent GEMMs C_b = act(rinv_b[m] csc_b[n] (A'_b . W'_b^T) + bias) (+ R_b),
// operand b at base + b * stride (elements; a stride of 0 shares the operand
// across the batch: a conv's weight, a broadcast matmul side).  The planes of
// A_b are [2][M][lda] with plane stride aplane (likewise W_b); C_b / R_b are
// [M][ldc] / [M][ldr].  EPI_BIAS: bias per column n; EPI_BIAS_ROW: per row m
// (a conv computed as W . patches^T, NCHW out), batch element b's bias at
// bias + b * sbias (a grouped conv's groups).  One launch, the tiles of all
// batch elements in one grid.  K % 32 == 0.
NOS_API int nos_gemm_f32h3_batched(const void* Ap, int lda, long long aplane, long long sa, const float* rinv,
                                   long long srinv, float rconst, const void* Wp, int ldw, long long wplane,
                                   long long sw, const float* csc, long long scsc, const float* bias, long long sbias,
                                   const float* R, int ldr, long long sr, float* C, int ldc, long long sc, int M, int N,
                                   int K, int nb, int epi, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || nb <= 0 || (K % BK) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8) || lda < K || ldw < K || aplane < (long long)M * lda || wplane < (long long)N * ldw)
    return (int)hipErrorInvalidValue;
  if (sa < 0 || sw < 0 || srinv < 0 || scsc < 0 || sr < 0 || sc < 0 || sbias < 0 || (sa % 8) || (sw % 8))
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)Ap) | ((uintptr_t)Wp)) & 15) return (int)hipErrorInvalidValue;
  if ((!rinv && !(rconst > 0.f)) || !csc || !C || ldc < N) return (int)hipErrorInvalidValue;
  if ((epi & (EPI_BIAS | EPI_BIAS_ROW)) == (EPI_BIAS | EPI_BIAS_ROW) || ((epi & (EPI_BIAS | EPI_BIAS_ROW)) && !bias) ||
      ((epi & (EPI_RESID | EPI_RESID_PRE)) && (!R || ldr < N)) || (epi & EPI_RESID && epi & EPI_RESID_PRE))
    return (int)hipErrorInvalidValue;
  if (nb > 1 && sc < (long long)(M - 1) * ldc + N) return (int)hipErrorInvalidValue;  // outputs never overlap
  Batch bt;
  bt.nb = nb;
  bt.a = sa;
  bt.rinv = srinv;
  bt.w = sw;
  bt.csc = scsc;
  bt.c = sc;
  bt.r = sr;
  bt.bias = sbias;
  return run_h3(Ap, lda, aplane, rinv, rconst, Wp, ldw, wplane, csc, bias, R, ldr, C, ldc, M, N, K, epi, KvOut{},
                PlaneOut{}, bt, stream, true);
}

// nos_gemm_f32h3's plain contract (fp32 C, no KV / plane outputs; N % 4 == 0,
// C / R rows 16-byte aligned) plus the row statistics of the finished C for
// the LayerNorm of the next GEMM:
// stats[m][tn] = (mean, sum of squared deviations) of C[m, BN tn .. BN tn + BN - 1]
// (the valid columns), ceil(N / BN) parts per row (BN = nos_gemm_f32h3_hot_bn()) -- nos_gemm_f32h3_lna's input.
NOS_API int nos_gemm_f32h3_stats(const void* Ap, int lda, long long aplane, const float* rinv, float rconst,
                                 const void* Wp, int ldw, long long wplane, const float* csc, const float* bias,
                                 const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi, void* stats,
                                 hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0 || !C || ldc < N || !stats || (N % 4) || (ldc % 4) ||
      (((uintptr_t)C) & 15))
    return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && ((ldr % 4) || (((uintptr_t)R) & 15))) return (int)hipErrorInvalidValue;
  if ((lda % 8) || (ldw % 8) || lda < K || ldw < K || aplane < (long long)M * lda || wplane < (long long)N * ldw)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)Ap) | ((uintptr_t)Wp)) & 15 || (((uintptr_t)stats) & 7)) return (int)hipErrorInvalidValue;
  if ((!rinv && !(rconst > 0.f)) || !csc || ((epi & EPI_BIAS) && !bias) || ((epi & EPI_RESID) && (!R || ldr < N)) ||
      (epi & (EPI_BIAS_ROW | EPI_RESID_PRE)))
    return (int)hipErrorInvalidValue;
  LnIo ln;
  ln.sout = static_cast<float2*>(stats);
  ln.spart = (N + g_hot_bn - 1) / g_hot_bn;
  if (g_hot_bn == 64)
    return launch_t<128, 64, 2, 2, 32, 2, false, 2>(static_cast<const _Float16*>(Ap), lda, aplane, rinv, rconst,
                                                    static_cast<const _Float16*>(Wp), ldw, wplane, csc, bias, R, ldr,
                                                    C, ldc, M, N, K, epi, KvOut{}, PlaneOut{}, Batch{}, stream, ln);
  if (g_hot_ring == 3)
    return launch_t<128, 128, 2, 2, 32, 3, false, 2>(static_cast<const _Float16*>(Ap), lda, aplane, rinv, rconst,
                                                     static_cast<const _Float16*>(Wp), ldw, wplane, csc, bias, R, ldr,
                                                     C, ldc, M, N, K, epi, KvOut{}, PlaneOut{}, Batch{}, stream, ln);
  return launch_t<128, 128, 2, 2, 32, 2, false, 2>(static_cast<const _Float16*>(Ap), lda, aplane, rinv, rconst,
                                                   static_cast<const _Float16*>(Wp), ldw, wplane, csc, bias, R, ldr,
                                                   C, ldc, M, N, K, epi, KvOut{}, PlaneOut{}, Batch{}, stream, ln);
}

// C = act(2^-eln csc[n] (LN(X)' . W'^T) + bias) with LN(X)' = (X - mean) rstd
// 2^eln split into h3 planes inside the GEMM (no nos_split_rows_h3 pass): X
// fp32 [M, K] (row stride ldx, 16-byte aligned rows), its row statistics
// stats [M][nparts] = (mean, M2) over parts of pw columns (nos_gemm_f32h3_stats:
// pw 128; nos_row_stats: one part of K), rstd = 1 / sqrt(M2 / K + eps);
// LayerNorm's gamma / beta folded into W and bias.  The KV / plane outputs of
// nos_gemm_f32h3.  K % 32 == 0.
NOS_API int nos_gemm_f32h3_lna(const float* X, int ldx, const void* stats, int nparts, int pw, float eps, int eln,
                               const void* Wp, int ldw, long long wplane, const float* csc, const float* bias,
                               const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi, void* kvs,
                               int S, int skvp, const float* kvsc, void* P, int ldp, long long pplane, float psc,
                               hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % BK) != 0 || !X || (ldx % 4) || ldx < K || !stats || nparts <= 0 || pw <= 0 ||
      (long long)nparts * pw < K || (long long)(nparts - 1) * pw >= K)
    return (int)hipErrorInvalidValue;
  if ((ldw % 8) || ldw < K || wplane < (long long)N * ldw || (((uintptr_t)Wp) & 15) || (((uintptr_t)X) & 15) ||
      (((uintptr_t)stats) & 7))
    return (int)hipErrorInvalidValue;
  if (!csc || ((epi & EPI_BIAS) && !bias) || ((epi & EPI_RESID) && (!R || ldr < N)) ||
      (epi & (EPI_BIAS_ROW | EPI_RESID_PRE)) || !(eps >= 0.f) || eln < -126 || eln > 126)
    return (int)hipErrorInvalidValue;
  KvOut kv;
  PlaneOut po;
  if (kvs != nullptr) {
    if (!kvsc || N % 3 || (N / 3) % 64 || S <= 0 || M % S || skvp < S || (((uintptr_t)kvs) & 15) || P)
      return (int)hipErrorInvalidValue;
    kv.kvs = static_cast<unsigned short*>(kvs);
    kv.kvsc = kvsc;
    kv.hd = N / 3;
    kv.qcols = kv.hd;
    kv.S = S;
    kv.skvp = skvp;
  }
  if (P != nullptr) {
    if (ldp < N || pplane < (long long)M * ldp || !(psc > 0.f)) return (int)hipErrorInvalidValue;
    po.p = static_cast<unsigned short*>(P);
    po.ldp = ldp;
    po.pplane = pplane;
    po.sc = psc;
  } else if (!C || ldc < (kvs != nullptr ? N / 3 : N)) {
    return (int)hipErrorInvalidValue;
  }
  LnIo ln;
  ln.x = X;
  ln.ldx = ldx;
  ln.sin = static_cast<const float2*>(stats);
  ln.nparts = nparts;
  ln.pw = pw;
  ln.eps = eps;
  ln.sc = ldexpf(1.f, eln);
  // 128 x 128 (or 128 x 256 for plane outputs, g_lna_wide): the LN-in-A-load normalises and
  // splits its A tile per workgroup, so 128 x 64 tiles doubled that VALU work (fleet 760 vs
  // 800 inf/s, profiles/r06_hot_bn_ab.json)
  if (g_lna_wide && P != nullptr)
    return launch_t<128, 256, 2, 4, 32, 2, false, 1>(nullptr, K, (long long)M * K, nullptr, ldexpf(1.f, -eln),
                                                     static_cast<const _Float16*>(Wp), ldw, wplane, csc, bias, R, ldr,
                                                     C, ldc, M, N, K, epi, kv, po, Batch{}, stream, ln);
  return launch_t<128, 128, 2, 2, 32, 2, false, 1>(nullptr, K, (long long)M * K, nullptr, ldexpf(1.f, -eln),
                                                   static_cast<const _Float16*>(Wp), ldw, wplane, csc, bias, R, ldr,
                                                   C, ldc, M, N, K, epi, kv, po, Batch{}, stream, ln);
}
