// fp32 GEMM with fused LayerNorm / bias / GELU / ReLU / residual on the bf16
// matrix pipes (bf16x6 split, split_bf16.h): the contract and epilogues of
// the exact-f32 MFMA GEMM (gemm_f32.hip), 2.7x less matrix-pipe time per
// FLOP at the same accuracy (tests/test_kernels_gpu.py checks both against
// fp64).
//
//   plain:     C[M,N] = act(A[M,K] . W[N,K]^T + bias) (+ R)
//   LN-fused:  C[M,N] = act(rstd * (A . W'^T - mu * c1) + c2)  (folded LayerNorm)
//
// Design:
//  * W is a weight: it arrives PRE-SPLIT as three bf16 planes [3][N][K]
//    (ops.split_f32_weight, once per weight); A (activations) is fp32;
//  * 4 waves (2 x 2) per workgroup, tiles 128x128 / 64x128 / 64x64 chosen by
//    the fp32 GEMM's tile policy (nos_gemm_f32_pick_tile), each wave (BM/2) x
//    (BN/2) as 32x32 blocks, BK = 32 per stage = two 16-deep MFMA steps;
//  * LDS-DMA (global_load_lds_dwordx4) into an S-deep ring: the A tile as
//    fp32 rows of 128 B (chunks XOR-swizzled by row & 7), the three W planes
//    as rows of 64 B (chunks swizzled by (row >> 2) & 3) -- both conflict-free
//    for the fragment reads; one raw s_barrier per stage behind a COUNTED
//    vmcnt (S-2 later stages may stay in flight across it);
//  * a wave splits its A fragments in registers (the K-contiguous 8 floats
//    of a 16-deep step are exactly one bf16x8 operand) and issues six
//    v_mfma_f32_32x32x16_bf16 per 32x32 block and step;
//  * epilogue and LayerNorm statistics as in gemm_f32.hip.
#include "common.h"
#include "split_bf16.h"

namespace {

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8 };

// LDS images of one K stage of BK (32 or 64): the fp32 A rows (AROW bytes,
// ACH 16-byte chunks) and the bf16 W plane rows (WROW bytes, WCH chunks),
// chunks XOR-swizzled so 16 consecutive lanes reading the same logical chunk
// of 16 consecutive rows hit 16 distinct 16-byte bank slots
template <int BK_>
struct Lay {
  static constexpr int BK = BK_, AROW = BK * 4, WROW = BK * 2, ACH = AROW / 16, WCH = WROW / 16;
  __device__ static int aswz(int row) { return BK == 32 ? (row & 7) : (row & 15); }
  __device__ static int wswz(int row) { return BK == 32 ? ((row >> 2) & 3) : ((row >> 1) & 7); }
};

// LDS-DMA of 16 bytes per lane (lane L -> lds_wave_base + 16 L), issued as
// inline asm: the compiler then does not know the instruction writes LDS and
// inserts no vmcnt(0) before the next ds_read (hipcc assumes every ds_read may
// alias an in-flight LDS-DMA, which drained the NEXT stage's loads before the
// CURRENT stage's fragment reads -- a full L2/HBM round trip per K step).
// The explicit counted waits (wait_stages) + barrier provide the ordering.
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  // m0 is an operand ("{m0}"), so the compiler writes it and knows it is live
  // (a clobbered m0 is undefined behaviour: m0 is a reserved register); the
  // s_nop is the SALU-write-m0 -> LDS-DMA wait state the compiler cannot see
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
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

// s_waitcnt vmcnt(n * LPS) for a runtime n in [0, 3] (the immediate must be a constant)
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


// Optional second output of the fused-LN QKV projection: columns >= qcols (K
// then V, hd = H * 64 each) are written as the six bf16 planes the bf16x6
// attention reads (attention_f32x.hip: kvs[b][s][plane][hd], rows padded to
// skvp per batch), exactly the split its streaming kernel would make, so the
// fp32 K/V never go to memory; the Q columns go to C as usual.
// With kvsc (the fp16x3 attention, attention_f32x.hip): four fp16 planes per
// token instead (K hi, K lo, V hi, V lo: kvs[b][s][plane][hd], split_f16.h),
// each head's K / V on the power-of-two scale kvsc[0 / 1][head].
struct KvOut {
  unsigned short* kvs = nullptr;
  int qcols = 0, hd = 0, S = 0, skvp = 0;
  const float* kvsc = nullptr;
};

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}

// WGM x WGN waves per workgroup (4 or 8); NT threads.  PIPE: software-
// pipelined K loop (2-deep ring only, see below)
template <bool LN, int BM, int BN, bool PERSIST, int RS, int BK, int WGM = 2, int WGN = 2, bool PIPE = false>
__global__ __launch_bounds__(64 * WGM * WGN, WGM * WGN > 4 ? 1 : 2) void gemm_f32x6_kernel(
    const float* __restrict__ A, int lda, const unsigned short* __restrict__ Wp, int ldw, long long wplane,
    const float* __restrict__ bias, const float* __restrict__ c1, const float* __restrict__ c2,
    const float* __restrict__ R, int ldr, float* __restrict__ C, int ldc, int M, int N, int K, int epi, float eps,
    int tiles_m, int tiles_n, KvOut kv) {
  // waves WGM x WGN over the tile, each (BM/WGM) x (BN/WGN) as 32x32 blocks;
  // WGM x 1 makes every wave split ONE A block for all its W blocks
  constexpr int NW = WGM * WGN, NT = 64 * NW, MI = BM / (32 * WGM), NI = BN / (32 * WGN);
  static_assert(MI >= 1 && NI >= 1 && (NW == 4 || NW == 8), "wave layout");
  using L = Lay<BK>;
  constexpr int AROW = L::AROW, WROW = L::WROW, ACH = L::ACH, WCH = L::WCH;
  constexpr int TA = BM * AROW, TWP = BN * WROW, STAGE = TA + 3 * TWP;
  constexpr int APW = BM * AROW / 1024 / NW, WPW = 3 * BN * WROW / 1024 / NW;  // DMA pieces per wave
  static_assert((BM * AROW / 1024) % NW == 0 && (3 * BN * WROW / 1024) % NW == 0, "equal DMA count per wave");
  static_assert(NT % BM == 0 && BK % (4 * (NT / BM)) == 0, "LayerNorm statistics: whole float4s per thread");
  constexpr int S = RS, LPS = APW + WPW;
  static_assert(S >= 2 && S <= 4 && (S - 1) * LPS < 64, "ring depth / vmcnt range");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // the LayerNorm statistics overlay the ring: written after the K loop's
  // last barrier, read in the epilogue, before the next tile's prologue
  float* s_mu = reinterpret_cast<float*>(smem);
  float* s_rstd = s_mu + BM;

  const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int c = lane & 31, h = lane >> 5;
  const int wm = wid / WGN, wn = wid % WGN;
  const int ntiles = tiles_m * tiles_n;
  const int nk = K / BK;
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
  const int tm = tt / tiles_n, tn = tt - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // A: BM rows x 128 B = BM/8 wave instructions; W: 3 planes x BN rows x 64 B
  // = 3*BN/16 wave instructions; all spread over the 4 waves
  auto stage = [&](int k0, unsigned char* dst) {
    constexpr int ARPI = 1024 / AROW, WRPI = 1024 / WROW;  // rows per DMA instruction
#pragma unroll
    for (int i = 0; i < APW; ++i) {  // A pieces of this wave (unconditional: no branch per piece)
      const int p = wid * APW + i;
      const int row = p * ARPI + lane / ACH;
      int grow = m0 + row;
      grow = grow < M ? grow : M - 1;
      glds16(A + (long long)grow * lda + k0 + (((lane % ACH) ^ L::aswz(row)) << 2), dst + p * 1024);
    }
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int p = wid * WPW + i;
      const int plane = p / (BN / WRPI), rb = (p % (BN / WRPI)) * WRPI;
      const int row = rb + lane / WCH;
      int gn = n0 + row;
      gn = gn < N ? gn : N - 1;
      glds16(Wp + plane * wplane + (long long)gn * ldw + k0 + (((lane % WCH) ^ L::wswz(row)) << 3),
             dst + TA + plane * TWP + rb * WROW);
    }
  };

  f32x16_t acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int TPR = NT / BM;           // LN statistics: threads per row
  constexpr int FPT = BK / TPR;          // floats per thread per stage
  const int srow = tid / TPR, spart = tid % TPR;
  float sshift = 0.f, ssum = 0.f, ssq = 0.f;

#pragma unroll
  for (int q = 0; q < S; ++q)
    if (q < nk) stage(q * BK, smem + q * STAGE);

  // LayerNorm statistics of this thread's share of one stage's A rows
  auto ln_stats = [&](const unsigned char* ta, int kt) {
    if constexpr (LN) {
#pragma unroll
      for (int q = 0; q < FPT / 4; ++q) {
        const int lc = spart * (FPT / 4) + q;
        const float4 v = *reinterpret_cast<const float4*>(ta + srow * AROW + ((lc ^ L::aswz(srow)) << 4));
        if (kt == 0 && q == 0) sshift = v.x;
        const float d0 = v.x - sshift, d1 = v.y - sshift, d2 = v.z - sshift, d3 = v.w - sshift;
        ssum += (d0 + d1) + (d2 + d3);
        ssq = fmaf(d0, d0, fmaf(d1, d1, fmaf(d2, d2, fmaf(d3, d3, ssq))));
      }
    }
  };

  if constexpr (PIPE) {
    // Software-pipelined K loop.  The fragments of MFMA step s+1 (the fp32 A
    // rows and the three W planes) are read from LDS, and A is split into
    // its three bf16 pieces, WHILE the 6*MI*NI MFMAs of step s run: the
    // reads and the ~46 VALU ops of a split fill the MFMAs' issue gaps
    // (an MFMA holds the wave's vector issue for 8 of its 32 cycles) instead
    // of a split phase with no MFMA and LDS waits right before each MFMA.
    // The stage boundary sits before the LAST step's MFMAs: every wave has
    // read that step (lgkmcnt(0)), so the barrier frees the buffer for the
    // DMA of stage kt+2 and publishes stage kt+1, whose first step is then
    // read and split under the last step's MFMAs.  The accumulation order is
    // the unpipelined loop's: results are bit-identical.
    static_assert(RS == 2 && BK == 32, "the pipelined K loop runs a 2-deep ring of 2-step stages");
    struct Raw {
      float4 x0[MI], x1[MI];
      bf16x8_t w[NI][3];
    };
    auto load_raw = [&](const unsigned char* base, int s, Raw& r) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * (BM / WGM) + i * 32 + c;
        r.x0[i] = *reinterpret_cast<const float4*>(base + row * AROW + (((4 * s + 2 * h) ^ L::aswz(row)) << 4));
        r.x1[i] = *reinterpret_cast<const float4*>(base + row * AROW + (((4 * s + 2 * h + 1) ^ L::aswz(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wn * (BN / WGN) + j * 32 + c;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          r.w[j][p] = *reinterpret_cast<const bf16x8_t*>(base + TA + p * TWP + row * WROW +
                                                          (((2 * s + h) ^ L::wswz(row)) << 4));
      }
    };
    auto split_raw = [&](const Raw& r, bf16x8_t (&af)[MI][3]) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const float x[8] = {r.x0[i].x, r.x0[i].y, r.x0[i].z, r.x0[i].w, r.x1[i].x, r.x1[i].y, r.x1[i].z, r.x1[i].w};
        nos::split8(x, af[i][0], af[i][1], af[i][2]);
      }
    };
    // one quarter of a split8: elements 2k, 2k+1 of row block i
    auto split_unit = [&](const Raw& r, bf16x8_t (&af)[MI][3], int i, int k) {
      const float4 v = k < 2 ? r.x0[i] : r.x1[i];
      const f32x2_t x = (k & 1) ? f32x2_t{v.z, v.w} : f32x2_t{v.x, v.y};
      bf16x2_t a, b, cc;
      nos::split2(x, a, b, cc);
      af[i][0][2 * k] = a.x; af[i][0][2 * k + 1] = a.y;
      af[i][1][2 * k] = b.x; af[i][1][2 * k + 1] = b.y;
      af[i][2][2 * k] = cc.x; af[i][2][2 * k + 1] = cc.y;
      // pin the pieces here: without it LLVM sinks the split into the next
      // block (past the stage barrier), where its only users are
      asm volatile("" : "+v"(af[i][0]), "+v"(af[i][1]), "+v"(af[i][2]));
    };
    // One MFMA step (6*MI*NI MFMAs on af/r) with the NEXT step's fragments
    // read from `nb` (step ns) and split underneath, in MI*NI chunks fenced by
    // sched_barrier: chunk q = the six MFMAs of block q, plus (chunk 0) the A
    // reads, (every MI-th chunk) one W block's three plane reads, and from
    // chunk 1 on a quarter of a row block's split -- the split's A reads
    // land during chunk 0's MFMAs, the W reads are used one step later.
    auto step = [&](const bf16x8_t (&af)[MI][3], const Raw& r, const unsigned char* nb, int ns, Raw& rn,
                    bf16x8_t (&afn)[MI][3], bool stats, int skt) {
      constexpr int NB = MI * NI, NSP = 4 * MI;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int bi = q / NI, bj = q % NI;
        acc[bi][bj] = nos::mma6(af[bi], r.w[bj], acc[bi][bj]);
        if (q == 0) {
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int row = wm * (BM / WGM) + i * 32 + c;
            rn.x0[i] = *reinterpret_cast<const float4*>(nb + row * AROW + (((4 * ns + 2 * h) ^ L::aswz(row)) << 4));
            rn.x1[i] =
                *reinterpret_cast<const float4*>(nb + row * AROW + (((4 * ns + 2 * h + 1) ^ L::aswz(row)) << 4));
          }
        }
        if (q % MI == 0) {
          const int j = q / MI;
          const int row = wn * (BN / WGN) + j * 32 + c;
#pragma unroll
          for (int p = 0; p < 3; ++p)
            rn.w[j][p] = *reinterpret_cast<const bf16x8_t*>(nb + TA + p * TWP + row * WROW +
                                                             (((2 * ns + h) ^ L::wswz(row)) << 4));
        }
#pragma unroll
        for (int u = 0; u < NSP; ++u)
          if (NB > 1 && 1 + u * (NB - 1) / NSP == q) split_unit(rn, afn, u / 4, u % 4);
        if (stats && q == NB - 1) ln_stats(nb, skt);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (NB == 1) {
#pragma unroll
        for (int u = 0; u < NSP; ++u) split_unit(rn, afn, u / 4, u % 4);
      }
    };

    wait_stages<LPS>(nk > 1 ? 1 : 0);  // stage 0 landed (stage 1 may stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // two fragment sets in ping-pong (A: step 0 of a stage, B: step 1), so
    // nothing is copied between registers across the loop
    Raw ra, rb;
    bf16x8_t afa[MI][3], afb[MI][3];
    load_raw(smem, 0, ra);
    ln_stats(smem, 0);
    split_raw(ra, afa);
    for (int kt = 0; kt + 1 < nk; ++kt) {
      const unsigned char* base = smem + (kt & 1) * STAGE;
      step(afa, ra, base, 1, rb, afb, false, 0);  // step 1 of stage kt read under step 0's MFMAs
      // stage boundary: stage kt+1 landed (the only DMA in flight), every
      // wave has read all of stage kt (step 1 is in rb)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) stage((kt + 2) * BK, smem + (kt & 1) * STAGE);
      // step 0 of stage kt+1 (and its LayerNorm statistics) under step 1's MFMAs
      step(afb, rb, smem + ((kt + 1) & 1) * STAGE, 0, ra, afa, true, kt + 1);
    }
    step(afa, ra, smem + ((nk - 1) & 1) * STAGE, 1, rb, afb, false, 0);  // the last stage
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = nos::mma6(afb[i], rb.w[j], acc[i][j]);
  } else {
  for (int kt = 0; kt < nk; ++kt) {
    // slice kt landed (the newer slices issued so far stay in flight: S-1 of
    // them after the prologue, S-2 later) and every wave is done with slice
    // kt-1, whose buffer slice kt+S-1 reuses
    wait_stages<LPS>(min(kt == 0 ? S - 1 : S - 2, nk - 1 - kt));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int slot = S == 2 ? (kt & 1) : kt % S;
    if (kt > 0 && kt + S - 1 < nk) stage((kt + S - 1) * BK, smem + (S == 2 ? slot ^ 1 : (kt + S - 1) % S) * STAGE);
    const unsigned char* cur = smem + slot * STAGE;
    const unsigned char* ta = cur;
    const unsigned char* tw = cur + TA;
    ln_stats(ta, kt);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {  // 16-deep MFMA steps: lane holds k = 16s + 8h .. +7
      bf16x8_t af[MI][3], wf[NI][3];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * (BM / WGM) + i * 32 + c;
        const float4 x0 = *reinterpret_cast<const float4*>(ta + row * AROW + (((4 * s + 2 * h) ^ L::aswz(row)) << 4));
        const float4 x1 =
            *reinterpret_cast<const float4*>(ta + row * AROW + (((4 * s + 2 * h + 1) ^ L::aswz(row)) << 4));
        const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        nos::split8(x, af[i][0], af[i][1], af[i][2]);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wn * (BN / WGN) + j * 32 + c;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          wf[j][p] =
              *reinterpret_cast<const bf16x8_t*>(tw + p * TWP + row * WROW + (((2 * s + h) ^ L::wswz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = nos::mma6(af[i], wf[j], acc[i][j]);
    }
  }
  }  // !PIPE
  __syncthreads();  // every wave is done with the ring (the next tile's prologue, the LN statistics)

  if constexpr (LN) {
    const float kpart = (float)(K / TPR);
    float mean = sshift + ssum / kpart, m2 = ssq - ssum * ssum / kpart, cnt = kpart;
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) {  // Chan's parallel combination of the shifted partial sums
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
    const int n = n0 + wn * (BN / WGN) + j * 32 + c;
    const int nc = n < N ? n : N - 1;
    const float p1 = LN ? c1[nc] : 0.f;
    const float p2 = LN ? c2[nc] : ((epi & EPI_BIAS) ? bias[nc] : 0.f);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * (BM / WGM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int m = m0 + rl;
        float v = acc[i][j][r];
        if constexpr (LN) v = fmaf(s_rstd[rl], v - s_mu[rl] * p1, p2);
        else v += p2;
        if (epi & EPI_GELU) v = 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f));
        if (epi & EPI_RELU) v = fmaxf(v, 0.f);
        if (m < M && n < N) {
          if (epi & EPI_RESID) v += R[(long long)m * ldr + n];
          if (kv.kvs != nullptr && n >= kv.qcols) {
            const int t = (n - kv.qcols) >= kv.hd;  // 0: K, 1: V
            const int col = n - kv.qcols - t * kv.hd;
            const int b = kv.S == M ? 0 : m / kv.S;
            const long long row = (long long)b * kv.skvp + (m - b * kv.S);
            if (kv.kvsc != nullptr) {
              const float x = v * kv.kvsc[t * (kv.hd >> 6) + (col >> 6)];
              const _Float16 h0 = (_Float16)x;
              const _Float16 h1 = (_Float16)(x - (float)h0);
              unsigned short* dst = kv.kvs + (row * 4 + 2 * t) * kv.hd + col;
              dst[0] = __builtin_bit_cast(unsigned short, h0);
              dst[kv.hd] = __builtin_bit_cast(unsigned short, h1);
              continue;
            }
            unsigned short* dst = kv.kvs + (row * 6 + 3 * t) * kv.hd + col;
            const __bf16 p0 = (__bf16)v;
            const float r1 = v - (float)p0;
            const __bf16 p1 = (__bf16)r1;
            dst[0] = __builtin_bit_cast(unsigned short, p0);
            dst[kv.hd] = __builtin_bit_cast(unsigned short, p1);
            dst[2 * kv.hd] = bf16_bits(r1 - (float)p1);
          } else {
            C[(long long)m * ldc + n] = v;
          }
        }
      }
    }
  }
  }  // tiles
}

int g_pipe = 1;  // software-pipelined K loop on 2-deep rings (nos_gemm_f32x6_set_pipeline)

template <bool LN, int BM, int BN, int RS, int BK, int WGM, int WGN, bool PIPE>
int launch_p(const float* A, int lda, const unsigned short* Wp, int ldw, long long wplane, const float* bias,
             const float* c1, const float* c2, const float* R, int ldr, float* C, int ldc, int M, int N, int K,
             int epi, float eps, hipStream_t st, KvOut kv);

template <bool LN, int BM, int BN, int RS, int BK, int WGM = 2, int WGN = 2>
int launch_t(const float* A, int lda, const unsigned short* Wp, int ldw, long long wplane, const float* bias,
             const float* c1, const float* c2, const float* R, int ldr, float* C, int ldc, int M, int N, int K,
             int epi, float eps, hipStream_t st, KvOut kv) {
  if constexpr (RS == 2 && BK == 32) {
    if (g_pipe) return launch_p<LN, BM, BN, RS, BK, WGM, WGN, true>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr,
                                                                    C, ldc, M, N, K, epi, eps, st, kv);
  }
  return launch_p<LN, BM, BN, RS, BK, WGM, WGN, false>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N,
                                                       K, epi, eps, st, kv);
}

template <bool LN, int BM, int BN, int RS, int BK, int WGM, int WGN, bool PIPE>
int launch_p(const float* A, int lda, const unsigned short* Wp, int ldw, long long wplane, const float* bias,
             const float* c1, const float* c2, const float* R, int ldr, float* C, int ldc, int M, int N, int K,
             int epi, float eps, hipStream_t st, KvOut kv) {
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const long long ntiles = (long long)tiles_m * tiles_n;
  if (ntiles > (1LL << 30)) return (int)hipErrorInvalidValue;
  const size_t ring = RS * (size_t)(BM * Lay<BK>::AROW + 3 * BN * Lay<BK>::WROW);
  const size_t lds = ring > 2 * BM * sizeof(float) ? ring : 2 * BM * sizeof(float);
  constexpr int NT = 64 * WGM * WGN;
  const int grid =
      nos_grid_for((const void*)gemm_f32x6_kernel<LN, BM, BN, true, RS, BK, WGM, WGN, PIPE>, NT, lds, ntiles);
  if (grid < ntiles)
    hipLaunchKernelGGL((gemm_f32x6_kernel<LN, BM, BN, true, RS, BK, WGM, WGN, PIPE>), dim3((unsigned)grid), dim3(NT),
                       lds, st, A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, tiles_m,
                       tiles_n, kv);
  else
    hipLaunchKernelGGL((gemm_f32x6_kernel<LN, BM, BN, false, RS, BK, WGM, WGN, PIPE>), dim3((unsigned)ntiles),
                       dim3(NT), lds, st, A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps,
                       tiles_m, tiles_n, kv);
  return (int)hipGetLastError();
}

}  // namespace

NOS_API int nos_gemm_f32_pick_tile(int M, int N);

namespace {

// K-stage config (nos_gemm_f32x6_set_stage): 0 = BK 32 in a 2-deep ring,
// 1 = BK 32, 3-deep (64x64 / 64x128 tiles), 2 = BK 64, 2-deep (K % 64 == 0)
int g_stage = 0;
// tile override (nos_gemm_f32x6_set_tile): -1 = the fp32 GEMM's tile policy,
// 0 / 1 / 2 = 128x128 / 64x128 / 64x64 (2 x 2 waves), 3 = 128x64 (4 x 1 waves),
// 4 = 128x64 where N >= 1024, the policy's tile elsewhere, 5 = 128x128 (4 x 1
// waves), 6 = 128x128 where N >= 1024, 128x64 elsewhere (4 x 1 waves),
// 7 = 256x128 (8 x 1 waves)
int g_tile = -1;

int launch(const float* A, int lda, const unsigned short* Wp, int ldw, long long wplane, const float* bias,
           const float* c1, const float* c2, const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi,
           float eps, bool ln, hipStream_t st, KvOut kv = KvOut()) {
  if (M <= 0 || N <= 0 || K <= 0 || (K % 32) != 0) return (int)hipErrorInvalidValue;
  if ((lda % 4) || (ldw % 8) || (wplane % 8) || lda < K || ldw < K || ldc < N || wplane < (long long)N * ldw)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)Wp) & 15) return (int)hipErrorInvalidValue;
  if (!ln && (epi & EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if (ln && (!c1 || !c2)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_RESID) && (!R || ldr < N)) return (int)hipErrorInvalidValue;
  int cfg = g_tile >= 0 && g_tile != 4 && g_tile != 6 ? g_tile : nos_gemm_f32_pick_tile(M, N);
  if (g_tile == 4 && N >= 1024) cfg = 3;  // 128x64 (4 x 1 waves) for the wide projections only
  if (g_tile == 6) cfg = N >= 1024 ? 5 : 3;  // 128x128 / 128x64, 4 x 1 waves
  const int stg = (g_stage == 2 && K % 64 != 0) ? 0 : g_stage;
#define NOS_F32X_LAUNCH(LNV, BMV, BNV, RSV, BKV) \
  launch_t<LNV, BMV, BNV, RSV, BKV>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, eps, st, kv)
#define NOS_F32X_TILES(LNV)                                                                        \
  if (cfg == 0) return NOS_F32X_LAUNCH(LNV, 128, 128, 2, 32);                                     \
  if (cfg == 3)                                                                                    \
    return launch_t<LNV, 128, 64, 2, 32, 4, 1>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K, epi, \
                                            eps, st, kv);                                              \
  if (cfg == 7)                                                                                    \
    return launch_t<LNV, 256, 128, 2, 32, 8, 1>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K,  \
                                                epi, eps, st, kv);                                     \
  if (cfg == 5)                                                                                    \
    return launch_t<LNV, 128, 128, 2, 32, 4, 1>(A, lda, Wp, ldw, wplane, bias, c1, c2, R, ldr, C, ldc, M, N, K,    \
                                             epi, eps, st, kv);                                        \
  if (cfg == 1) {                                                                                  \
    if (stg == 1) return NOS_F32X_LAUNCH(LNV, 64, 128, 3, 32);                                    \
    if (stg == 2) return NOS_F32X_LAUNCH(LNV, 64, 128, 2, 64);                                    \
    return NOS_F32X_LAUNCH(LNV, 64, 128, 2, 32);                                                   \
  }                                                                                                \
  if (stg == 1) return NOS_F32X_LAUNCH(LNV, 64, 64, 3, 32);                                       \
  if (stg == 2) return NOS_F32X_LAUNCH(LNV, 64, 64, 2, 64);                                       \
  return NOS_F32X_LAUNCH(LNV, 64, 64, 2, 32);
  if (ln) {
    NOS_F32X_TILES(true)
  }
  NOS_F32X_TILES(false)
#undef NOS_F32X_TILES
#undef NOS_F32X_LAUNCH
}

}  // namespace

NOS_API int nos_gemm_f32x6_set_tile(int tile) {
  if (tile < -1 || tile > 7) return (int)hipErrorInvalidValue;
  g_tile = tile;
  return 0;
}

// 1 (default): software-pipelined K loop on the 2-deep-ring configs; 0: the
// unpipelined loop (A/B; the results are bit-identical)
NOS_API int nos_gemm_f32x6_set_pipeline(int on) {
  if (on < 0 || on > 1) return (int)hipErrorInvalidValue;
  g_pipe = on;
  return 0;
}

NOS_API int nos_gemm_f32x6_set_stage(int cfg) {
  if (cfg < 0 || cfg > 2) return (int)hipErrorInvalidValue;
  g_stage = cfg;
  return 0;
}

// C = act(A . W^T + bias) (+ R), fp32 A [M,K] (lda), W as three bf16 planes
// Wp + p * wplane, each [N,K] (ldw); K % 32 == 0, rows 16-byte aligned.
NOS_API int nos_gemm_f32x6(const float* A, int lda, const void* Wp, int ldw, long long wplane, const float* bias,
                           const float* R, int ldr, float* C, int ldc, int M, int N, int K, int epi,
                           hipStream_t stream) {
  return launch(A, lda, static_cast<const unsigned short*>(Wp), ldw, wplane, bias, nullptr, nullptr, R, ldr, C, ldc,
                M, N, K, epi, 0.f, false, stream);
}

// C = act(LayerNorm(A) . W^T + bias) in the folded form (ops.fold_layernorm),
// W' = W * gamma as three bf16 planes; K is the LayerNorm width.
NOS_API int nos_gemm_ln_f32x6(const float* A, int lda, const void* Wp, int ldw, long long wplane, const float* c1,
                              const float* c2, float* C, int ldc, int M, int N, int K, int epi, float eps,
                              hipStream_t stream) {
  return launch(A, lda, static_cast<const unsigned short*>(Wp), ldw, wplane, nullptr, c1, c2, nullptr, 0, C, ldc, M,
                N, K, epi & ~(EPI_BIAS | EPI_RESID), eps, true, stream);
}

// The fused-LN QKV projection whose K / V columns (N = 3 * hd) are written as
// the bf16x6 attention's planes at kvs (nos_attn_f32x6_workspace layout,
// S rows per batch padded to skvp); Q goes to C[:, :hd].  The attention then
// runs from the planes (nos_attn_fwd_f32x6_presplit_d64): no fp32 K/V store,
// no streaming split.
namespace {

int qkv_planes(const float* A, int lda, const void* Wp, int ldw, long long wplane, const float* c1, const float* c2,
               float* C, int ldc, int M, int N, int K, int epi, float eps, void* kvs, int S, int skvp,
               const float* kvsc, hipStream_t stream) {
  if (kvs == nullptr || N % 3 != 0 || S <= 0 || M % S != 0 || skvp < S || (((uintptr_t)kvs) & 15))
    return (int)hipErrorInvalidValue;
  if (kvsc != nullptr && (N / 3) % 64 != 0) return (int)hipErrorInvalidValue;
  KvOut kv;
  kv.kvsc = kvsc;
  kv.kvs = static_cast<unsigned short*>(kvs);
  kv.hd = N / 3;
  kv.qcols = kv.hd;
  kv.S = S;
  kv.skvp = skvp;
  return launch(A, lda, static_cast<const unsigned short*>(Wp), ldw, wplane, nullptr, c1, c2, nullptr, 0, C, ldc, M,
                N, K, epi & ~(EPI_BIAS | EPI_RESID), eps, true, stream, kv);
}

}  // namespace

NOS_API int nos_gemm_ln_f32x6_qkv(const float* A, int lda, const void* Wp, int ldw, long long wplane,
                                  const float* c1, const float* c2, float* C, int ldc, int M, int N, int K, int epi,
                                  float eps, void* kvs, int S, int skvp, hipStream_t stream) {
  return qkv_planes(A, lda, Wp, ldw, wplane, c1, c2, C, ldc, M, N, K, epi, eps, kvs, S, skvp, nullptr, stream);
}

// The same projection writing the fp16x3 attention's four planes per token,
// each head's K / V on the power-of-two scale kvsc[0 / 1][head]
// (nos_attn_fwd_f32h3_presplit_d64).
NOS_API int nos_gemm_ln_f32x6_qkv_h3(const float* A, int lda, const void* Wp, int ldw, long long wplane,
                                     const float* c1, const float* c2, float* C, int ldc, int M, int N, int K,
                                     int epi, float eps, void* kvs, int S, int skvp, const float* kvsc,
                                     hipStream_t stream) {
  if (kvsc == nullptr) return (int)hipErrorInvalidValue;
  return qkv_planes(A, lda, Wp, ldw, wplane, c1, c2, C, ldc, M, N, K, epi, eps, kvs, S, skvp, kvsc, stream);
}
