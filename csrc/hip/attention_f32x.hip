// fp32 self-attention (head_dim 64, non-causal) on the bf16 matrix pipes:
// every fp32 operand is split into three bf16 pieces x = x0 + x1 + x2
// (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1): 3 x 8 mantissa
// bits hold all 24 of an fp32, so the split is exact), and every product
// a.b is the sum of the six piece products whose order is <= 2^-16 |a.b|:
//   a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0.
// A bf16 x bf16 product is exact in fp32 and v_mfma_f32_32x32x16_bf16
// accumulates in fp32, so the only error beyond fp32 accumulation is the
// dropped a1b2 + a2b1 + a2b2 (<= ~2^-23 |a.b|, the size of one fp32 rounding
// of the product).  Six bf16 MFMAs (32 cycles each) replace eight
// v_mfma_f32_32x32x2_f32 (64 cycles each) per 16-deep step: 2.7x less
// matrix-pipe time than the exact-f32 MFMA (attention_f32.hip) at the same
// accuracy (tests/test_kernels_gpu.py checks both against fp64).
//
// Design (CDNA4; the bf16 kernel's structure, attention.hip):
//  * K and V are split ONCE per call by a streaming kernel into six bf16
//    planes per token (K0 K1 K2 V0 V1 V2, every head's 64 dims contiguous)
//    instead of once per workgroup that reads them (27 q-blocks per head);
//  * one workgroup = 4 waves x 32 query rows of one (batch, head); 32-key
//    tiles of the six planes (4 KiB each) arrive by LDS-DMA
//    (global_load_lds_dwordx4, swizzle applied to the source address) into a
//    2-deep ring: no staging registers, no VALU, one barrier per tile;
//  * swapped QK^T (S^T = K . Q^T): Q's three pieces (pre-scaled by
//    scale * log2 e) stay in registers as the B operand; K pieces are read
//    with ds_read_b128 from XOR-swizzled images;
//  * the S^T accumulator (query on the lane, 16 keys in registers) gives the
//    row max / sum lane-locally plus one v_permlane32_swap; P = exp2(S - m)
//    is split into three pieces in registers and used directly as the B
//    operand of O^T = V^T . P^T, whose V^T pieces come from the transposing
//    LDS read ds_read_b64_tr_b16 (no LDS round trip for P);
//  * deferred rescale (P <= 2^8) and XCD-aware (batch, head, q-block) order
//    as in attention_f32.hip; PERSIST: slice-sized grid (nos::xcd_chunk).
#include <type_traits>

#include "common.h"
#include "split_bf16.h"
#include "split_f16.h"

namespace {

constexpr int D = 64;
constexpr int W = 4;                    // waves per workgroup
constexpr int NT = 64 * W;
constexpr int QBLK = 32 * W;            // query rows per workgroup
constexpr int KVB = 32;                 // keys per tile
constexpr int IMG = KVB * D * 2;        // one bf16 piece image: 4 KiB
constexpr int STAGE = 6 * IMG;          // K0 K1 K2 V0 V1 V2
constexpr int LDS_BYTES = 2 * STAGE;    // 48 KiB ring
constexpr float RESCALE_THR = 8.f;      // log2 units

__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int vswz(int row) { return ((row >> 1) & 1) << 2; }

__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// LDS-DMA of 16 bytes per lane issued as inline asm: with the builtin, hipcc
// assumes every ds_read may alias an in-flight LDS-DMA and inserts
// s_waitcnt vmcnt(0) before the first LDS read after the issue -- draining
// the NEXT tile's loads before the CURRENT tile's math (seen in the ISA: one
// L2/HBM round trip per tile).  The ring is ordered by the explicit
// vmcnt(0) + barrier that ends each tile (dma_wait_publish).
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  // m0 is an operand ("{m0}"), so the compiler writes it and knows it is live
  // (a clobbered m0 is undefined behaviour: m0 is a reserved register); the
  // s_nop is the SALU-write-m0 -> LDS-DMA wait state the compiler cannot see
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

// LDS-DMA from a wave-uniform tile base (SGPR pair) plus a per-lane 32-bit byte
// offset: the steady-state tiles need no 64-bit VALU address arithmetic
__device__ __forceinline__ void glds16_s(const void* sbase, unsigned voff, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(lds) : "memory");
}

// every DMA this wave issued has landed, then the workgroup barrier publishes them
__device__ __forceinline__ void dma_wait_publish() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// the same with the newest N DMAs left in flight (a deeper ring): a counted
// vmcnt and a raw barrier -- __syncthreads() would drain them (vmcnt(0))
template <int N>
__device__ __forceinline__ void dma_wait_publish_keep(bool keep) {
  if (keep)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <bool PERSIST>
__global__ __launch_bounds__(NT, 3) void attn_fwd_f32x6_d64_kernel(
    const float* __restrict__ q, const unsigned short* __restrict__ kvs, float* __restrict__ o, int B, int H, int Sq,
    int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float c, int nqb, int nsplit,
    float* __restrict__ part) {
  const int ldh = H * D;  // elements per plane row
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = B * H * nqb * nsplit;
  nos::XcdChunk chunk;
  if constexpr (PERSIST) {
    chunk = nos::xcd_chunk(blockIdx.x, gridDim.x, nwg);
  } else {
    chunk.first = nos::xcd_remap(blockIdx.x, nwg);
    chunk.end = chunk.first + 1;
    chunk.step = 1;
  }

  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int r = lane & 31;
  const int hh = lane >> 5;

  // hoisted per-lane LDS read offsets (relative to a piece image)
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = r * 128 + (((2 * ks + hh) ^ kswz(r)) << 4);
  const int g16 = (lane >> 4) & 1;
  const int tq = (lane & 15) >> 2;
  const int tp = lane & 3;
  const int vlb = (tq >> 1) & 1;
  int voff[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
    voff[db] = (4 * hh + tq) * 128 + (((4 * (db ^ vlb)) + 2 * g16 + (tp >> 1)) << 4) + 8 * (tp & 1);

  const int ntiles = (Skv + KVB - 1) / KVB;
  const int skvp = ntiles * KVB;
  int soff[6];  // staging: per-lane element offset of instruction i within a tile
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int p = wid * 6 + i;
    const int plane = p >> 2;
    const int row = (p & 3) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (plane < 3 ? kswz(row) : vswz(row));
    soff[i] = (row * 6 + plane) * ldh + lc * 8;
  }

  for (int w = chunk.first; w < chunk.end; w += chunk.step) {
    if (PERSIST && w != chunk.first) __syncthreads();  // the previous item is done with the ring
    // item = (batch, head, q-block, key split), the splits of a q-block and
    // the q-blocks of a head adjacent (one XCD's L2)
    const int sp = w % nsplit;
    const int wq = w / nsplit;
    const int b = wq / (H * nqb);
    const int rem = wq - b * (H * nqb);
    const int hd = rem / nqb;
    const int qb = rem - hd * nqb;
    const long long boff = (long long)b * bs_in + hd * D;
    const int tps = (ntiles + nsplit - 1) / nsplit;  // key tiles per split (the host keeps every split non-empty)
    const int t0 = sp * tps, t1 = min(ntiles, t0 + tps);

    // ---- Q pieces (B operand): lane holds Q[row r][d = 16ks + 8hh .. +7] * c
    const int qrow = qb * QBLK + wid * 32 + r;
    bf16x8_t qf[4][3];
    {
      const float* qp = q + boff + (long long)min(qrow, Sq - 1) * ld_in + 8 * hh;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float4 x0 = *reinterpret_cast<const float4*>(qp + 16 * ks);
        const float4 x1 = *reinterpret_cast<const float4*>(qp + 16 * ks + 4);
        const float x[8] = {x0.x * c, x0.y * c, x0.z * c, x0.w * c, x1.x * c, x1.y * c, x1.z * c, x1.w * c};
        nos::split8(x, qf[ks][0], qf[ks][1], qf[ks][2]);
      }
      // Q in registers before the first DMA (see glds16: the compiler cannot
      // count the asm DMA, so a Q load sunk into the key loop would make it
      // wait with vmcnt(n) counts that drain the in-flight tiles)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(qf[ks][p]));
    }

    // ---- LDS-DMA staging: per tile 6 planes x 32 rows x 128 B = 24 wave
    // instructions, 6 per wave.  Instruction p: plane p / 4, rows (p % 4) * 8
    // + lane / 8, physical chunk lane % 8 = logical chunk ^ swizzle.
    // The planes are padded to whole tiles with zeros: a tile's address is a
    // wave-uniform base plus the hoisted per-lane offsets.
    // The tail tile's rows past Skv re-read the last key's planes (finite
    // values; the -inf mask makes their P exactly 0), so the padding rows of
    // the planes are never read and need no zeroing (no memset per call).
    const unsigned short* pb = kvs + (long long)b * skvp * (6 * ldh) + hd * D;
    auto stage_piece = [&](int t, int buf, int i) {
      const int p = wid * 6 + i;
      long long off = (long long)t * (KVB * 6) * ldh + soff[i];
      if ((t + 1) * KVB > Skv) {
        const int over = t * KVB + (p & 3) * 8 + (lane >> 3) - (Skv - 1);
        if (over > 0) off -= (long long)over * 6 * ldh;
      }
      glds16(pb + off, smem + buf * STAGE + (p >> 2) * IMG + (p & 3) * 8 * 128);
    };
#pragma unroll
    for (int i = 0; i < 6; ++i) stage_piece(t0, 0, i);

    f32x16_t oacc[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[0][i] = 0.f;
      oacc[1][i] = 0.f;
    }
    float m = 0.f, l = 0.f;  // reference max (log2 units), this lane-half's partial row sum

    dma_wait_publish();  // tile 0 landed and is visible

    for (int t = t0; t < t1; ++t) {
      const int buf = (t - t0) & 1;
      const bool more = t + 1 < t1;
      // the next tile's 6 DMA pieces, into the buffer released by the barrier
      // ending t-1; they stay in flight through this tile's math
      if (more) {
#pragma unroll
        for (int i = 0; i < 6; ++i) stage_piece(t + 1, buf ^ 1, i);
      }
      const unsigned char* kl = smem + buf * STAGE;
      const unsigned char* vl = kl + 3 * IMG;

      f32x16_t s;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8_t a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8_t*>(kl + p * IMG + koff[ks]);
        s = nos::mma6(a, qf[ks], s);
      }
      if ((t + 1) * KVB > Skv) {  // tail tile: keys past Skv never contribute
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (t * KVB + (i & 3) + 8 * (i >> 2) + 4 * hh >= Skv) s[i] = -INFINITY;
      }
      float mt = s[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mt = fmaxf(mt, s[i]);
      const float mrel = xor32_max(mt) - m;
      if (t == t0 || !__all(mrel <= RESCALE_THR)) {  // the first tile sets the reference max
        const float delta = t == t0 ? mrel : fmaxf(mrel, 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        m += delta;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          oacc[0][i] *= alpha;
          oacc[1][i] *= alpha;
        }
      }
      // P = exp2(S - m), split into three pieces: pf[s2][piece] covers the
      // 16 keys of registers 8*s2 .. 8*s2+7
      bf16x8_t pf[2][3];
      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j2 = 0; j2 < 8; ++j2) {
        const float x0 = __builtin_amdgcn_exp2f(s[2 * j2] - m);
        const float x1 = __builtin_amdgcn_exp2f(s[2 * j2 + 1] - m);
        ls[(2 * j2) & 3] += x0;
        ls[(2 * j2 + 1) & 3] += x1;
        const f32x2_t x = {x0, x1};
        bf16x2_t a, bb, cc;
        nos::split2(x, a, bb, cc);
        const int s2 = j2 >> 2, e = 2 * (j2 & 3);
        pf[s2][0][e] = a.x; pf[s2][0][e + 1] = a.y;
        pf[s2][1][e] = bb.x; pf[s2][1][e + 1] = bb.y;
        pf[s2][2][e] = cc.x; pf[s2][2][e + 1] = cc.y;
      }
      l += (ls[0] + ls[1]) + (ls[2] + ls[3]);
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8_t a[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const unsigned char* base = vl + p * IMG + voff[db] + s2 * 16 * 128;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + 8 * 128));
            const s16x8_t a16 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            a[p] = __builtin_bit_cast(bf16x8_t, a16);
          }
          oacc[db] = nos::mma6(a, pf[s2], oacc[db]);
        }
      dma_wait_publish();  // next tile landed; every wave is done with `buf`
    }

    const float lt = xor32_sum(l);
    if (nsplit > 1) {  // unnormalised partial (O, m, l) of this key range: nos_attn_f32x6 merges them
      if (qrow < Sq) {
        const long long row = ((long long)sp * B + b) * Sq + qrow;
        float* op = part + row * ldh + hd * D;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(op + 32 * db + 8 * g + 4 * hh) =
                float4{oacc[db][4 * g + 0], oacc[db][4 * g + 1], oacc[db][4 * g + 2], oacc[db][4 * g + 3]};
        if (hh == 0) {
          float* ml = part + (long long)nsplit * B * Sq * ldh + (row * H + hd) * 2;
          ml[0] = m;
          ml[1] = lt;
        }
      }
      continue;
    }
    const float inv = 1.f / lt;
    if (qrow < Sq) {
      float* op = o + (long long)b * bs_out + (long long)qrow * ld_out + hd * D;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4 y;
          y.x = oacc[db][4 * g + 0] * inv;
          y.y = oacc[db][4 * g + 1] * inv;
          y.z = oacc[db][4 * g + 2] * inv;
          y.w = oacc[db][4 * g + 3] * inv;
          *reinterpret_cast<float4*>(op + 32 * db + 8 * g + 4 * hh) = y;
        }
    }
  }  // items
}

// ---------------------------------------------------------------- fp16x3
// The same attention on two fp16 pieces per operand (split_f16.h: three
// fp16 MFMAs per product instead of six bf16 ones, same per-product error
// bound).  K and V arrive as four fp16 planes per token (K hi, K lo, V hi,
// V lo), written by the fused-LN QKV projection's epilogue on per-head
// power-of-two scales kvsc[0][h] / kvsc[1][h] that the host derives from the
// weights (LN output has L2 norm <= sqrt(K), so |k_j| <= sqrt(K)|W_j| + |b_j|
// bounds every key and value of a head before anything runs).  Q is split
// here on a per-query-row scale (the row is lane-local: lane r and r + 32
// hold its two halves), and that scale and the head's key scale fold into
// the one FMA that already turns a score into exp2 units; P <= 2^8 (deferred
// rescale) needs no scale; the value scale is divided out with 1/l.
constexpr int H3_STAGE = 4 * IMG;            // K hi, K lo, V hi, V lo
constexpr int H3_RING = 2;  // stages; 3 (two tiles in flight) measured slower: 138 VGPRs, 802 vs 818 inf/s
constexpr int H3_LDS_BYTES = H3_RING * H3_STAGE;  // 48 KiB
constexpr int H3_WG_PER_CU = 4;  // 4-wave workgroups (HW = 4); HW = 8: 2 (134 VGPRs, 3 waves / SIMD; forcing
                                 // 4 waves / SIMD -- 128 VGPRs, one spill -- fleet 797-799 vs 823-824 inf/s)

// HW waves per workgroup (4 or 8) x 32 query rows; the 16 DMA pieces of a
// key tile are spread over the waves (16 / HW each)
template <bool PERSIST, int HW>
__global__ __launch_bounds__(64 * HW, HW == 8 ? 2 : H3_WG_PER_CU) void attn_fwd_f32h3_d64_kernel(
    const float* __restrict__ q, const _Float16* __restrict__ kvs, float* __restrict__ o, int B, int H, int Sq,
    int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float c, const float* __restrict__ kvsc,
    int nqb, int nsplit, float* __restrict__ part, _Float16* __restrict__ op, long long opl, float osc) {
  const int ldh = H * D;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = B * H * nqb * nsplit;
  nos::XcdChunk chunk;
  if constexpr (PERSIST) {
    chunk = nos::xcd_chunk(blockIdx.x, gridDim.x, nwg);
  } else {
    chunk.first = nos::xcd_remap(blockIdx.x, nwg);
    chunk.end = chunk.first + 1;
    chunk.step = 1;
  }

  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int r = lane & 31;
  const int hh = lane >> 5;

  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = r * 128 + (((2 * ks + hh) ^ kswz(r)) << 4);
  const int g16 = (lane >> 4) & 1;
  const int tq = (lane & 15) >> 2;
  const int tp = lane & 3;
  const int vlb = (tq >> 1) & 1;
  int voff[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
    voff[db] = (4 * hh + tq) * 128 + (((4 * (db ^ vlb)) + 2 * g16 + (tp >> 1)) << 4) + 8 * (tp & 1);

  const int ntiles = (Skv + KVB - 1) / KVB;
  const int skvp = ntiles * KVB;
  constexpr int PPW = 16 / HW, HQBLK = 32 * HW;
  int soff[PPW];  // staging: per-lane element offset of instruction i within a tile
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wid * PPW + i;
    const int plane = p >> 2;
    const int row = (p & 3) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (plane < 2 ? kswz(row) : vswz(row));
    soff[i] = (row * 4 + plane) * ldh + lc * 8;
  }

  for (int w = chunk.first; w < chunk.end; w += chunk.step) {
    if (PERSIST && w != chunk.first) __syncthreads();
    const int sp = w % nsplit;
    const int wq = w / nsplit;
    const int b = wq / (H * nqb);
    const int rem = wq - b * (H * nqb);
    const int hd = rem / nqb;
    const int qb = rem - hd * nqb;
    const long long boff = (long long)b * bs_in + hd * D;
    const int tps = (ntiles + nsplit - 1) / nsplit;
    const int t0 = sp * tps, t1 = min(ntiles, t0 + tps);
    const float ksc = kvsc[hd], vinv = 1.f / kvsc[H + hd];  // powers of two

    // ---- Q pieces (B operand) on this query row's scale: lane holds
    // Q[row r][d = 16ks + 8hh .. +7] * c * 2^e
    const int qrow = qb * HQBLK + wid * 32 + r;
    const bool live = qb * HQBLK + wid * 32 < Sq;  // wave-uniform
    f16x8_t qf[4][2];
    float fs;  // s' -> exp2 units: 2^-e / ksc
    {
      const float* qp = q + boff + (long long)min(qrow, Sq - 1) * ld_in + 8 * hh;
      float x[4][8];
      float mx = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float4 x0 = *reinterpret_cast<const float4*>(qp + 16 * ks);
        const float4 x1 = *reinterpret_cast<const float4*>(qp + 16 * ks + 4);
        x[ks][0] = x0.x; x[ks][1] = x0.y; x[ks][2] = x0.z; x[ks][3] = x0.w;
        x[ks][4] = x1.x; x[ks][5] = x1.y; x[ks][6] = x1.z; x[ks][7] = x1.w;
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(x[ks][j]));
      }
      const int e = nos::h3_scale_exp(xor32_max(mx) * c);
      const float qm = c * nos::pow2i(e);
      fs = nos::pow2i(-e) / ksc;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          f16x2_t hi, lo;
          nos::split2h(f32x2_t{x[ks][j] * qm, x[ks][j + 1] * qm}, hi, lo);
          qf[ks][0][j] = hi.x; qf[ks][0][j + 1] = hi.y;
          qf[ks][1][j] = lo.x; qf[ks][1][j + 1] = lo.y;
        }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int p = 0; p < 2; ++p) asm volatile("" : "+v"(qf[ks][p]));
    }

    const _Float16* pb = kvs + (long long)b * skvp * (4 * ldh) + hd * D;
    auto stage_piece = [&](int t, int buf, int i) {
      const int p = wid * PPW + i;
      long long off = (long long)t * (KVB * 4) * ldh + soff[i];
      if ((t + 1) * KVB > Skv) {  // tail tile: rows past Skv re-read the last key
        const int over = t * KVB + (p & 3) * 8 + (lane >> 3) - (Skv - 1);
        if (over > 0) off -= (long long)over * 4 * ldh;
      }
      glds16(pb + off, smem + buf * H3_STAGE + (p >> 2) * IMG + (p & 3) * 8 * 128);
    };
    // full tiles: uniform base + the per-lane byte offsets (2 * soff)
    auto stage_full = [&](int t, int buf, int i) {
      const int p = wid * PPW + i;
      glds16_s(pb + (long long)t * (KVB * 4) * ldh, (unsigned)soff[i] * 2u,
               smem + buf * H3_STAGE + (p >> 2) * IMG + (p & 3) * 8 * 128);
    };
    // tile u into ring slot `slot` (full tiles from a uniform base)
    auto stage_tile = [&](int u, int slot) {
      if ((u + 1) * KVB <= Skv) {
#pragma unroll
        for (int i = 0; i < PPW; ++i) stage_full(u, slot, i);
      } else {
#pragma unroll
        for (int i = 0; i < PPW; ++i) stage_piece(u, slot, i);
      }
    };
    // the first H3_RING - 1 tiles in flight; tile t0 landed and published
#pragma unroll
    for (int i = 0; i < PPW; ++i) stage_piece(t0, 0, i);
#pragma unroll
    for (int q = 1; q < H3_RING - 1; ++q)
      if (t0 + q < t1) stage_tile(t0 + q, q);

    f32x16_t oacc[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[0][i] = 0.f;
      oacc[1][i] = 0.f;
    }
    float m = 0.f, l = 0.f;

    static_assert(H3_RING == 2 || H3_RING == 3, "ring depth");
    dma_wait_publish_keep<PPW>(H3_RING == 3 && t0 + 1 < t1);

    // the tile body; MASKED: the tail tile (keys past Skv masked).  Peeled out of
    // the main loop -- if-converted into it, the mask cost 48 VALU per tile
    auto tile = [&](int t, auto masked) {
      constexpr bool MASKED = decltype(masked)::value;
      const int buf = (t - t0) % H3_RING;
      // tile t + H3_RING - 1 into the slot tile t - 1 left (every wave passed
      // the barrier that ended tile t - 1)
      if (t + H3_RING - 1 < t1) stage_tile(t + H3_RING - 1, (t - t0 + H3_RING - 1) % H3_RING);
      // at the end: tile t + 1 landed (the ring's newer tile may stay in flight)
      const bool keep = H3_RING == 3 && t + 2 < t1;
      // a wave whose 32 query rows all lie past Sq (the last query block of a
      // head, a query range) only stages and keeps the barriers
      if (!live) {
        dma_wait_publish_keep<PPW>(keep);
        return;
      }
      const unsigned char* kl = smem + buf * H3_STAGE;
      const unsigned char* vl = kl + 2 * IMG;

      f32x16_t s;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        f16x8_t a[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) a[p] = *reinterpret_cast<const f16x8_t*>(kl + p * IMG + koff[ks]);
        s = nos::mma3h(a, qf[ks], s);
      }
      if constexpr (MASKED) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (t * KVB + (i & 3) + 8 * (i >> 2) + 4 * hh >= Skv) s[i] = -INFINITY;
      }
      float mt = s[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mt = fmaxf(mt, s[i]);
      const float mrel = xor32_max(mt) * fs - m;
      if (t == t0 || !__all(mrel <= RESCALE_THR)) {
        const float delta = t == t0 ? mrel : fmaxf(mrel, 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        m += delta;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          oacc[0][i] *= alpha;
          oacc[1][i] *= alpha;
        }
      }
      // packed: score -> exp2 units as v_pk_fma_f32 on key pairs, the row sum as
      // v_pk_add_f32 into two pair accumulators -- the same four partial sums in
      // the same order as four scalar ones (bit-identical), half the instructions
      f16x8_t pf[2][2];
      f32x2_t ls2[2] = {f32x2_t{0.f, 0.f}, f32x2_t{0.f, 0.f}};
      const f32x2_t fs2 = {fs, fs}, nm2 = {-m, -m};
#pragma unroll
      for (int j2 = 0; j2 < 8; ++j2) {
        const f32x2_t e2 = __builtin_elementwise_fma(f32x2_t{s[2 * j2], s[2 * j2 + 1]}, fs2, nm2);
        const f32x2_t x = {__builtin_amdgcn_exp2f(e2.x), __builtin_amdgcn_exp2f(e2.y)};
        ls2[j2 & 1] += x;
        f16x2_t hi, lo;
        nos::split2h(x, hi, lo);
        const int s2 = j2 >> 2, e = 2 * (j2 & 3);
        pf[s2][0][e] = hi.x; pf[s2][0][e + 1] = hi.y;
        pf[s2][1][e] = lo.x; pf[s2][1][e + 1] = lo.y;
      }
      l += (ls2[0].x + ls2[0].y) + (ls2[1].x + ls2[1].y);
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          f16x8_t a[2];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const unsigned char* base = vl + p * IMG + voff[db] + s2 * 16 * 128;
            const s16x4_t lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base));
            const s16x4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + 8 * 128));
            const s16x8_t a16 = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            a[p] = __builtin_bit_cast(f16x8_t, a16);
          }
          oacc[db] = nos::mma3h(a, pf[s2], oacc[db]);
        }
      dma_wait_publish_keep<PPW>(keep);
    };
    const int tm = (Skv % KVB) ? max(t0, min(t1, ntiles - 1)) : t1;  // the tail tile, if any, is the last
    for (int t = t0; t < tm; ++t) tile(t, std::false_type{});
    for (int t = tm; t < t1; ++t) tile(t, std::true_type{});

    const float lt = xor32_sum(l);
    if (nsplit > 1) {  // unnormalised partial (O, m, l), O on the unit scale
      if (qrow < Sq) {
        const long long row = ((long long)sp * B + b) * Sq + qrow;
        float* op = part + row * ldh + hd * D;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(op + 32 * db + 8 * g + 4 * hh) =
                float4{oacc[db][4 * g + 0] * vinv, oacc[db][4 * g + 1] * vinv, oacc[db][4 * g + 2] * vinv,
                       oacc[db][4 * g + 3] * vinv};
        if (hh == 0) {
          float* ml = part + (long long)nsplit * B * Sq * ldh + (row * H + hd) * 2;
          ml[0] = m;
          ml[1] = lt;
        }
      }
      continue;
    }
    const float inv = vinv / lt;
    if (qrow < Sq) {
      const long long ob = (long long)b * bs_out + (long long)qrow * ld_out + hd * D;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4 y;
          y.x = oacc[db][4 * g + 0] * inv;
          y.y = oacc[db][4 * g + 1] * inv;
          y.z = oacc[db][4 * g + 2] * inv;
          y.w = oacc[db][4 * g + 3] * inv;
          const int d = 32 * db + 8 * g + 4 * hh;
          if (op != nullptr) {  // the proj GEMM's A planes on the static scale osc
            f16x2_t h01, l01, h23, l23;
            nos::split2h(f32x2_t{y.x * osc, y.y * osc}, h01, l01);
            nos::split2h(f32x2_t{y.z * osc, y.w * osc}, h23, l23);
            typedef __attribute__((ext_vector_type(4))) _Float16 f16x4_t;
            *reinterpret_cast<f16x4_t*>(op + ob + d) = f16x4_t{h01.x, h01.y, h23.x, h23.y};
            *reinterpret_cast<f16x4_t*>(op + opl + ob + d) = f16x4_t{l01.x, l01.y, l23.x, l23.y};
          } else {
            *reinterpret_cast<float4*>(o + ob + d) = y;
          }
        }
    }
  }  // items
}

// K and V rows of the fused projection -> six bf16 planes per token:
// kvs[b][s][plane][H*64], plane = 3 * (0 K, 1 V) + piece, s < Skvp (rows
// past Skv are written as zeros, though the attention never reads them).
// One thread: 8 dims of one (token, tensor, head).
__global__ __launch_bounds__(256) void split_kv_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                       unsigned short* __restrict__ kvs, int S, int Sp, int H,
                                                       int ld_in, long long bs_in, int n8) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const int per_tok = 16 * H;                 // 8-dim chunks of K and V per token
  const int tok = i / per_tok;
  const int rem = i - tok * per_tok;
  const int is_v = rem >= 8 * H;
  const int ch = rem - is_v * 8 * H;          // chunk within the H*64 row
  const int b = tok / Sp, s = tok - b * Sp;
  bf16x8_t p[3];
  if (s < S) {
    const float* src = (is_v ? v : k) + b * bs_in + (long long)s * ld_in + ch * 8;
    const float4 x0 = reinterpret_cast<const float4*>(src)[0];
    const float4 x1 = reinterpret_cast<const float4*>(src)[1];
    const float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    nos::split8(x, p[0], p[1], p[2]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) p[0][j] = p[1][j] = p[2][j] = (__bf16)0.f;
  }
  unsigned short* dst = kvs + ((long long)tok * 6 + 3 * is_v) * (H * D) + ch * 8;
#pragma unroll
  for (int j = 0; j < 3; ++j) *reinterpret_cast<bf16x8_t*>(dst + j * H * D) = p[j];
}

int launch(const float* q, const unsigned short* kvs, float* o, int B, int H, int Sq, int Skv, int ld_in,
           long long bs_in, int ld_out, long long bs_out, float c, int nqb, int nsplit, float* part,
           hipStream_t stream) {
  const long long nwg = (long long)B * H * nqb * nsplit;
  const int grid = nos_grid_for((const void*)attn_fwd_f32x6_d64_kernel<true>, NT, LDS_BYTES, nwg);
  if (grid < nwg)
    hipLaunchKernelGGL((attn_fwd_f32x6_d64_kernel<true>), dim3((unsigned)grid), dim3(NT), LDS_BYTES, stream,
                       q, kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, nqb, nsplit, part);
  else
    hipLaunchKernelGGL((attn_fwd_f32x6_d64_kernel<false>), dim3((unsigned)nwg), dim3(NT), LDS_BYTES, stream,
                       q, kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, nqb, nsplit, part);
  return (int)hipGetLastError();
}

int g_kvsplit = 0;  // 0 = auto (nos_attn_f32x6_set_kvsplit)
constexpr int MAX_SPLIT = 4;
constexpr int WG_PER_CU = 3;  // the kernel's launch bound

// Key splits: when one split per q-block leaves resident-workgroup slots of
// the (budgeted) CUs empty -- one YOLOS image is 162 q-blocks for 768 slots --
// split the keys so the grid fills them, at most MAX_SPLIT ways and never so
// finely that a split has no tile.
int pick_split(long long nwg1, int ntiles, int wg_per_cu = WG_PER_CU) {
  int n = g_kvsplit;
  if (n == 0) {
    const long long slots = (long long)wg_per_cu * nos_effective_cus();
    n = nwg1 >= slots ? 1 : (int)(slots / nwg1);
  }
  n = n < 1 ? 1 : (n > MAX_SPLIT ? MAX_SPLIT : n);
  while (n > 1 && (long long)(n - 1) * ((ntiles + n - 1) / n) >= ntiles) --n;  // the last split non-empty
  return n;
}

// KV-split merge: per (batch, row, head) and 4 dims, O = sum_i O_i 2^(m_i - M) /
// sum_i l_i 2^(m_i - M), M = max_i m_i (m in log2 units, O_i unnormalised)
__global__ __launch_bounds__(256) void merge_splits_kernel(const float* __restrict__ part, float* __restrict__ o,
                                                           int B, int H, int Sq, int nsplit, int ld_out,
                                                           long long bs_out, long long n4,
                                                           _Float16* __restrict__ op = nullptr, long long opl = 0,
                                                           float osc = 1.f) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int ldh = H * D;
  const long long row = i / (ldh / 4);               // b * Sq + s
  const int col = (int)(i - row * (ldh / 4)) * 4;    // hd * 64 + d
  const int hd = col / D;
  const long long per_split = (long long)B * Sq;
  const float* ml = part + (long long)nsplit * per_split * ldh;
  float mx = -INFINITY;
  for (int sp = 0; sp < nsplit; ++sp) mx = fmaxf(mx, ml[((sp * per_split + row) * H + hd) * 2]);
  float L = 0.f;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < nsplit; ++sp) {
    const long long r = sp * per_split + row;
    const float a = __builtin_amdgcn_exp2f(ml[(r * H + hd) * 2] - mx);
    L = fmaf(ml[(r * H + hd) * 2 + 1], a, L);
    const float4 v = *reinterpret_cast<const float4*>(part + r * ldh + col);
    acc.x = fmaf(v.x, a, acc.x);
    acc.y = fmaf(v.y, a, acc.y);
    acc.z = fmaf(v.z, a, acc.z);
    acc.w = fmaf(v.w, a, acc.w);
  }
  const float inv = 1.f / L;
  const long long b = row / Sq, s = row - b * Sq;
  const float4 y = float4{acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
  if (op != nullptr) {
    f16x2_t h01, l01, h23, l23;
    nos::split2h(f32x2_t{y.x * osc, y.y * osc}, h01, l01);
    nos::split2h(f32x2_t{y.z * osc, y.w * osc}, h23, l23);
    typedef __attribute__((ext_vector_type(4))) _Float16 f16x4_t;
    *reinterpret_cast<f16x4_t*>(op + b * bs_out + s * ld_out + col) = f16x4_t{h01.x, h01.y, h23.x, h23.y};
    *reinterpret_cast<f16x4_t*>(op + opl + b * bs_out + s * ld_out + col) = f16x4_t{l01.x, l01.y, l23.x, l23.y};
    return;
  }
  *reinterpret_cast<float4*>(o + b * bs_out + s * ld_out + col) = y;
}

}  // namespace


// Workspace bytes of nos_attn_fwd_f32x6_d64 (the split K/V planes).
NOS_API int nos_attn_f32x6_set_kvsplit(int n) {
  if (n < 0 || n > MAX_SPLIT) return (int)hipErrorInvalidValue;
  g_kvsplit = n;
  return 0;
}

// Workspace bytes of nos_attn_fwd_f32x6_d64: the split K/V planes, then room
// for MAX_SPLIT partial (O, m, l) per query row and head.
NOS_API long long nos_attn_f32x6_workspace(int B, int H, int Sq, int Skv) {
  const long long skvp = (Skv + KVB - 1) / KVB * KVB;
  const long long planes = ((long long)B * skvp * 6 * H * D * 2 + 15) / 16 * 16;
  return planes + (long long)MAX_SPLIT * B * Sq * H * (D + 2) * 4;
}

// The exact-fp32 kernel's contract (attention_f32.hip: nos_attn_fwd_f32_d64)
// plus a workspace of nos_attn_f32x6_workspace() bytes (16-byte aligned).
namespace {

// shared argument checks of the two entries; 0 = ok
int check_args(const void* q, const void* o, const void* ws, long long ws_bytes, int B, int H, int Sq, int Skv,
               int ld_in, long long bs_in, int ld_out, long long bs_out) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Skv <= 0) return (int)hipErrorInvalidValue;
  if (ld_in < H * D || ld_out < H * D || (ld_in & 3) || (ld_out & 3) || (bs_in & 3) || (bs_out & 3))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)q | (uintptr_t)o | (uintptr_t)ws) & 15) return (int)hipErrorInvalidValue;
  if (ws == nullptr || ws_bytes < nos_attn_f32x6_workspace(B, H, Sq, Skv)) return (int)hipErrorInvalidValue;
  const long long skvp = (Skv + KVB - 1) / KVB * KVB;
  if ((long long)B * H * ((Sq + QBLK - 1) / QBLK) > (1LL << 28) || (long long)B * skvp * 2 * H * 8 > INT_MAX ||
      skvp * 6 * H * D > INT_MAX)
    return (int)hipErrorInvalidValue;
  return 0;
}

// the attention proper, from the six planes at the start of ws
int run_from_planes(const float* q, float* o, int B, int H, int Sq, int Skv, int ld_in, long long bs_in, int ld_out,
                    long long bs_out, float scale, void* ws, hipStream_t stream) {
  const float c = scale * 1.4426950408889634f;
  const int nqb = (Sq + QBLK - 1) / QBLK;
  const long long nwg = (long long)B * H * nqb;
  const int skvp = (Skv + KVB - 1) / KVB * KVB;
  const int nsplit = pick_split(nwg, skvp / KVB);
  auto* kvs = static_cast<unsigned short*>(ws);
  float* part = reinterpret_cast<float*>(static_cast<unsigned char*>(ws) +
                                         ((long long)B * skvp * 6 * H * D * 2 + 15) / 16 * 16);
  const int rc = launch(q, kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, nqb, nsplit, part, stream);
  if (rc != 0 || nsplit == 1) return rc;
  const long long n4 = (long long)B * Sq * H * (D / 4);
  hipLaunchKernelGGL(merge_splits_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, part, o, B, H, Sq,
                     nsplit, ld_out, bs_out, n4);
  return (int)hipGetLastError();
}

}  // namespace

NOS_API int nos_attn_fwd_f32x6_d64(const float* q, const float* k, const float* v, float* o, int B, int H, int Sq,
                                   int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float scale,
                                   void* ws, long long ws_bytes, hipStream_t stream) {
  if (int rc = check_args(q, o, ws, ws_bytes, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out)) return rc;
  if (((uintptr_t)k | (uintptr_t)v) & 15) return (int)hipErrorInvalidValue;
  const int skvp = (Skv + KVB - 1) / KVB * KVB;
  const long long n8 = (long long)B * skvp * 2 * H * 8;
  hipLaunchKernelGGL(split_kv_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, stream, k, v,
                     static_cast<unsigned short*>(ws), Skv, skvp, H, ld_in, bs_in, (int)n8);
  return run_from_planes(q, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, scale, ws, stream);
}

// The same attention when the K/V planes are already at the start of ws
// (written by the QKV projection's epilogue, nos_gemm_ln_f32x6_qkv).  The
// padding rows of the planes are never read (the kernel's tail tile re-reads
// the last key), so nothing is zeroed: no memset node per call.
NOS_API int nos_attn_fwd_f32x6_presplit_d64(const float* q, float* o, int B, int H, int Sq, int Skv, int ld_in,
                                            long long bs_in, int ld_out, long long bs_out, float scale, void* ws,
                                            long long ws_bytes, hipStream_t stream) {
  if (int rc = check_args(q, o, ws, ws_bytes, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out)) return rc;
  return run_from_planes(q, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, scale, ws, stream);
}

namespace {

// nos_attn_f32h3_set_waves; 8: the 28-tenant fleet 756 vs 743 inf/s over
// 4 rounds (profiles/r04_h3_attn_waves_ab.json)
int g_h3_waves = 8;

template <int HW>
int launch_h3(const float* q, const _Float16* kvs, float* o, int B, int H, int Sq, int Skv, int ld_in,
              long long bs_in, int ld_out, long long bs_out, float c, const float* kvsc, int nqb, int nsplit,
              float* part, _Float16* op, long long opl, float osc, hipStream_t stream) {
  const long long nwg = (long long)B * H * nqb * nsplit;
  const int grid = nos_grid_for((const void*)attn_fwd_f32h3_d64_kernel<true, HW>, 64 * HW, H3_LDS_BYTES, nwg);
  if (grid < nwg)
    hipLaunchKernelGGL((attn_fwd_f32h3_d64_kernel<true, HW>), dim3((unsigned)grid), dim3(64 * HW), H3_LDS_BYTES,
                       stream, q,
                       kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, kvsc, nqb, nsplit, part, op, opl, osc);
  else
    hipLaunchKernelGGL((attn_fwd_f32h3_d64_kernel<false, HW>), dim3((unsigned)nwg), dim3(64 * HW), H3_LDS_BYTES,
                       stream, q,
                       kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, kvsc, nqb, nsplit, part, op, opl, osc);
  return (int)hipGetLastError();
}

}  // namespace

// fp16x3 attention from the four fp16 planes per token that the QKV
// projection's epilogue wrote at the start of ws (nos_gemm_ln_f32x6_qkv_h3)
// on the per-head scales kvsc [2][H] (K, then V; powers of two).  Same
// contract and workspace as nos_attn_fwd_f32x6_presplit_d64.
//
// oplanes != nullptr: the output goes, instead of o, to the next h3 GEMM's A
// planes (hi at oplanes, lo at oplanes + opl elements, same row / batch
// strides as o) on the static scale osc (the host's bound of |O|: every O
// row is a convex combination of V rows); o is then only checked for shape.
NOS_API int nos_attn_fwd_f32h3_presplit_d64(const float* q, float* o, int B, int H, int Sq, int Skv, int ld_in,
                                            long long bs_in, int ld_out, long long bs_out, float scale,
                                            const float* kvsc, void* ws, long long ws_bytes, void* oplanes,
                                            long long opl, float osc, hipStream_t stream) {
  if (int rc = check_args(q, o, ws, ws_bytes, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out)) return rc;
  if (kvsc == nullptr) return (int)hipErrorInvalidValue;
  auto* op = static_cast<_Float16*>(oplanes);
  if (op != nullptr && ((((uintptr_t)op) & 7) || opl < (long long)B * bs_out || !(osc > 0.f)))
    return (int)hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  const int hw = g_h3_waves;
  const int nqb = (Sq + 32 * hw - 1) / (32 * hw);
  const long long nwg = (long long)B * H * nqb;
  const int skvp = (Skv + KVB - 1) / KVB * KVB;
  const int nsplit = pick_split(nwg, skvp / KVB, hw == 8 ? 2 : H3_WG_PER_CU);
  auto* kvs = static_cast<const _Float16*>(ws);
  float* part = reinterpret_cast<float*>(static_cast<unsigned char*>(ws) +
                                         ((long long)B * skvp * 6 * H * D * 2 + 15) / 16 * 16);
  const int rc = hw == 8 ? launch_h3<8>(q, kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, kvsc, nqb, nsplit,
                                        part, op, opl, osc, stream)
                         : launch_h3<4>(q, kvs, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, kvsc, nqb, nsplit,
                                        part, op, opl, osc, stream);
  if (rc != 0 || nsplit == 1) return rc;
  const long long n4 = (long long)B * Sq * H * (D / 4);
  hipLaunchKernelGGL(merge_splits_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, part, o, B, H, Sq,
                     nsplit, ld_out, bs_out, n4, op, opl, osc);
  return (int)hipGetLastError();
}

// h3 attention workgroup size: 8 waves (default: 256 query rows, 2
// workgroups per CU: each key tile is loaded once for twice the queries) or
// 4 (128 rows, 4 per CU).  The results are bit-identical.
NOS_API int nos_attn_f32h3_set_waves(int waves) {
  if (waves != 4 && waves != 8) return (int)hipErrorInvalidValue;
  g_h3_waves = waves;
  return 0;
}
