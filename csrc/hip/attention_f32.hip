// Fused multi-head self-attention forward in exact fp32 (head_dim 64, non-causal)
// for the fp32 YOLOS tenant pods -- the precision of the reference demo's
// HF model (demos/gpu-sharing-comparison/client/main.py:19-20).
//
// gfx950 has an exact f32-input MFMA (v_mfma_f32_32x32x2_f32: fmaf-chain
// numerics, 64 FLOP/clk/SIMD = 1/16 of bf16) but no xf32, so fp32 attention
// is matrix-pipe bound; the design keeps that pipe fed and everything else
// off it:
//
//  * one workgroup = W waves x 32 query rows of one (batch, head); K/V tiles
//    of KVB keys are staged ONCE per workgroup into LDS by LDS-DMA
//    (global_load_lds_dwordx4: no staging registers) into a 2-deep ring, one
//    barrier per tile; the W waves share every byte (W x less L2 traffic than
//    per-wave loads);
//  * "swapped" QK^T: S^T = K . Q^T with the head dim split as d = 32h + kk
//    (h = lane >> 5, kk = MFMA step): a lane's K operand is 128 contiguous
//    bytes of its key row (8 x ds_read_b128 from an XOR-swizzled image,
//    conflict-free) and its Q half-row (pre-scaled by scale*log2 e) stays in
//    32 registers for the whole kernel;
//  * S^T's accumulator has the query on the lane and 16 keys per 32-key tile
//    in registers: row max / sum are lane-local plus one v_permlane32_swap,
//    and O's per-query rescale is a per-lane scalar;
//  * the accumulator registers ARE the B operand of O^T = V^T . P^T
//    (register r of lane-half h is key (r&3) + 8(r>>2) + 4h), so V^T's A
//    operand is gathered in that key order with ds_read_b32 from a V image
//    whose 16-byte chunks are XOR-swizzled by key bit 2 (the two lane halves
//    then hit disjoint banks) -- no LDS round trip for P, no transpose;
//  * deferred rescale: the running max only moves when a row's tile max
//    exceeds it by more than 8 (log2 units), so O and l are rescaled rarely;
//  * XCD-aware workgroup order: the q-blocks of one head share an XCD's L2.
#include "common.h"

namespace {

constexpr int D = 64;
constexpr int ROW_BYTES = D * 4;      // 256 B = 16 chunks of 16 B
constexpr float RESCALE_THR = 8.f;    // log2 units

__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ int kswz(int row) { return row & 15; }
__device__ __forceinline__ int vswz(int row) { return ((row >> 2) & 1) << 3; }

// LDS-DMA as inline asm + explicit vmcnt(0) before the publishing barrier:
// with the builtin, hipcc drained the next stage's DMA before this stage's
// LDS reads (attention.hip: glds16)
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  // m0 is an operand ("{m0}"), so the compiler writes it and knows it is live
  // (a clobbered m0 is undefined behaviour: m0 is a reserved register); the
  // s_nop is the SALU-write-m0 -> LDS-DMA wait state the compiler cannot see
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

__device__ __forceinline__ void dma_wait_publish() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// G = 2: two groups of W waves walk interleaved key tiles of the same
// (batch, head, q-block) and merge (m, l, O) through LDS at the end -- two
// waves per SIMD from ONE workgroup, so a single pod (162 q-blocks for 256
// CUs) still overlaps one wave's softmax with the other's MFMAs.
// OCC: workgroups per CU the register budget must allow; PERSIST: the
// slice-sized-grid instantiation (a chunk of items per workgroup)
template <int W, int KVB, int G, int OCC = 1, bool PERSIST = false>
__global__ __launch_bounds__(64 * W * G, OCC) void attn_fwd_f32_d64_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, float* __restrict__ o,
    int B, int H, int Sq, int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float c, int nqb) {
  constexpr int QBLK = 32 * W;
  constexpr int TILE = KVB * ROW_BYTES;          // bytes of K (or V) per stage
  constexpr int STAGE = 2 * TILE;
  constexpr int PIECES = STAGE / 1024;           // 1 KiB per wave-wide LDS-DMA, per group
  constexpr int PER_WAVE = PIECES / W;
  constexpr int RING = G * STAGE;                // one stage of every group
  constexpr int NT32 = KVB / 32;                 // 32-key S^T tiles per stage
  static_assert(PIECES % W == 0, "stage pieces must split evenly over the waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = B * H * nqb;
  // one (batch, head, q-block) per workgroup, or a chunk of them with a
  // slice-sized grid (nos::xcd_chunk); the q-blocks of a head share an XCD
  nos::XcdChunk chunk;
  if constexpr (PERSIST) {
    chunk = nos::xcd_chunk(blockIdx.x, gridDim.x, nwg);
  } else {
    chunk.first = nos::xcd_remap(blockIdx.x, nwg);
    chunk.end = chunk.first + 1;
    chunk.step = 1;
  }
  for (int wg = chunk.first; wg < chunk.end; wg += chunk.step) {
  if (PERSIST && wg != chunk.first) __syncthreads();  // the previous item's ring / merge buffer is free
  const int b = wg / (H * nqb);
  const int rem = wg - b * (H * nqb);
  const int hd = rem / nqb;
  const int qb = rem - hd * nqb;

  const int tid = threadIdx.x;
  const int wall = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wall / W;                      // wave group (key tiles grp, grp + G, ...)
  const int wid = wall - grp * W;                // wave within the group: its 32 query rows
  const int lane = tid & 63;
  const int h = lane >> 5, col = lane & 31;

  const long long boff = (long long)b * bs_in + hd * D;
  const float* kb_ptr = k + boff;
  const float* vb_ptr = v + boff;

  float qf[32];
  {
    const int qr = min(qb * QBLK + wid * 32 + col, Sq - 1);
    const float4* qp = reinterpret_cast<const float4*>(q + boff + (long long)qr * ld_in + 32 * h);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 x = qp[u];
      qf[4 * u + 0] = x.x * c;
      qf[4 * u + 1] = x.y * c;
      qf[4 * u + 2] = x.z * c;
      qf[4 * u + 3] = x.w * c;
    }
    // Q in registers before the first (asm) DMA: see attention_f32x.hip
#pragma unroll
    for (int u = 0; u < 32; ++u) asm volatile("" : "+v"(qf[u]));
  }

  // piece p: tensor p / (PIECES/2) (K, V), 4 rows from (p % (PIECES/2)) * 4;
  // lane L writes row R + L/16, physical chunk L%16 = logical chunk ^ swizzle
  // every group stages its own tile (G * it + grp) into its slot of the ring
  auto stage = [&](int it, int buf) {
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int p = wid * PER_WAVE + i;
      const int is_v = p / (PIECES / 2);
      const int R = (p % (PIECES / 2)) * 4;
      const int row = R + (lane >> 4);
      const int pc = lane & 15;
      const int lc = pc ^ (is_v ? vswz(row) : kswz(row));
      int kv = (G * it + grp) * KVB + row;
      kv = kv < Skv ? kv : Skv - 1;
      const float* src = (is_v ? vb_ptr : kb_ptr) + (long long)kv * ld_in + lc * 4;
      glds16(src, smem + buf * RING + grp * STAGE + is_v * TILE + R * ROW_BYTES);
    }
  };

  const int ntiles = (Skv + KVB - 1) / KVB;
  const int niters = (ntiles + G - 1) / G;
  stage(0, 0);

  int koff[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) koff[u] = col * ROW_BYTES + (((8 * h + u) ^ kswz(col)) << 4);
  int voff[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) voff[dt] = 4 * h * ROW_BYTES + (((8 * dt + (col >> 2)) ^ (8 * h)) << 4) + (col & 3) * 4;

  f32x16_t oacc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    oacc[0][i] = 0.f;
    oacc[1][i] = 0.f;
  }
  float m = 0.f, l = 0.f;  // reference max (log2 units), this lane-half's partial row sum

  dma_wait_publish();  // stage 0 landed and is visible

  for (int it = 0; it < niters; ++it) {
    const int buf = it & 1;
    if (it + 1 < niters) stage(it + 1, buf ^ 1);  // that buffer was released by the barrier ending it-1
    const int tile = G * it + grp;                 // this group's key tile
    if (tile < ntiles) {
      const unsigned char* kl = smem + buf * RING + grp * STAGE;
      const unsigned char* vl = kl + TILE;

      f32x16_t s[NT32];
#pragma unroll
      for (int t = 0; t < NT32; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[t][i] = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float4 kx = *reinterpret_cast<const float4*>(kl + t * 32 * ROW_BYTES + koff[u]);
          s[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.x, qf[4 * u + 0], s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.y, qf[4 * u + 1], s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.z, qf[4 * u + 2], s[t], 0, 0, 0);
          s[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(kx.w, qf[4 * u + 3], s[t], 0, 0, 0);
        }
      }
      if ((tile + 1) * KVB > Skv) {  // tail tile: keys past Skv never contribute
#pragma unroll
        for (int t = 0; t < NT32; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (tile * KVB + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h >= Skv) s[t][i] = -INFINITY;
      }
      float mt = s[0][0];
#pragma unroll
      for (int t = 0; t < NT32; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[t][i]);
      const float mrel = xor32_max(mt) - m;
      if (it == 0 || !__all(mrel <= RESCALE_THR)) {  // the group's first tile sets the reference max
        const float delta = it == 0 ? mrel : fmaxf(mrel, 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        m += delta;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          oacc[0][i] *= alpha;
          oacc[1][i] *= alpha;
        }
      }
      float ps = 0.f;
#pragma unroll
      for (int t = 0; t < NT32; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          s[t][i] = __builtin_amdgcn_exp2f(s[t][i] - m);
          ps += s[t][i];
        }
      l += ps;
      // O^T[d][i] += V^T[d][j] P^T[j][i]; step (t, r) sums keys 32t + {key(r,0), key(r,1)}
#pragma unroll
      for (int t = 0; t < NT32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int roff = (32 * t + (r & 3) + 8 * (r >> 2)) * ROW_BYTES;
          const float v0 = *reinterpret_cast<const float*>(vl + roff + voff[0]);
          const float v1 = *reinterpret_cast<const float*>(vl + roff + voff[1]);
          oacc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0, s[t][r], oacc[0], 0, 0, 0);
          oacc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1, s[t][r], oacc[1], 0, 0, 0);
        }
    }
    dma_wait_publish();  // next stage landed; every wave is done with this buffer
  }

  float a0 = 1.f;
  if constexpr (G == 2) {
    // merge: group 1 hands (O, m, l) of every lane to group 0 through LDS (the ring is free now)
    float* xch = reinterpret_cast<float*>(smem) + wid * (34 * 64);
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        xch[i * 64 + lane] = oacc[0][i];
        xch[(16 + i) * 64 + lane] = oacc[1][i];
      }
      xch[32 * 64 + lane] = m;
      xch[33 * 64 + lane] = l;
    }
    __syncthreads();
    if (grp == 1) continue;  // group 0 finishes the item; both meet at the next item's barrier
    const bool g1 = ntiles > 1;  // group 1 saw no tile when the sequence has one: its m means nothing
    const float m1 = xch[32 * 64 + lane], l1 = xch[33 * 64 + lane];
    const float mf = g1 ? fmaxf(m, m1) : m;
    a0 = __builtin_amdgcn_exp2f(m - mf);
    const float a1 = g1 ? __builtin_amdgcn_exp2f(m1 - mf) : 0.f;
    l = l * a0 + l1 * a1;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[0][i] = oacc[0][i] * a0 + xch[i * 64 + lane] * a1;
      oacc[1][i] = oacc[1][i] * a0 + xch[(16 + i) * 64 + lane] * a1;
    }
  }

  const float inv = 1.f / xor32_sum(l);
  const int qi = qb * QBLK + wid * 32 + col;
  if (qi < Sq) {
    float* op = o + (long long)b * bs_out + (long long)qi * ld_out + hd * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 y;
        y.x = oacc[dt][4 * g + 0] * inv;
        y.y = oacc[dt][4 * g + 1] * inv;
        y.z = oacc[dt][4 * g + 2] * inv;
        y.w = oacc[dt][4 * g + 3] * inv;
        *reinterpret_cast<float4*>(op + 32 * dt + 8 * g + 4 * h) = y;
      }
  }
  }  // items
}

template <int W, int KVB, int G, int OCC = 1>
int launch(const float* q, const float* k, const float* v, float* o, int B, int H, int Sq, int Skv, int ld_in,
           long long bs_in, int ld_out, long long bs_out, float c, hipStream_t stream) {
  const int nqb = (Sq + 32 * W - 1) / (32 * W);
  const long long nwg = (long long)B * H * nqb;
  if (nwg > (1LL << 30)) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)G * 2 * 2 * KVB * ROW_BYTES;
  const int grid = nos_grid_for((const void*)attn_fwd_f32_d64_kernel<W, KVB, G, OCC, true>, 64 * W * G, lds, nwg);
  if (grid < nwg)
    hipLaunchKernelGGL((attn_fwd_f32_d64_kernel<W, KVB, G, OCC, true>), dim3((unsigned)grid), dim3(64 * W * G), lds,
                       stream, q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, nqb);
  else
    hipLaunchKernelGGL((attn_fwd_f32_d64_kernel<W, KVB, G, OCC, false>), dim3((unsigned)nwg), dim3(64 * W * G), lds,
                       stream, q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, nqb);
  return (int)hipGetLastError();
}

// 0 auto, 1: 4 waves x 64-key tiles, 2: the same with 2 wave groups (split keys),
// 3: 4 waves x 32-key tiles (half the LDS: more co-resident workgroups),
// 4: 2 waves x 64-key tiles (64-query blocks), 5: 8 waves x 64-key tiles,
// 6: variant 3 register-capped for 3 workgroups per CU (127 VGPRs, no
//    AGPRs, no scratch: 4 waves per SIMD; the same cap on variant 1 spills),
// 7: two wave groups on 32-key tiles (64 KB LDS ring),
// (the bf16x6 split kernel, attention_f32x.hip, takes a workspace: its own entry)
int g_variant = 0;

}  // namespace

NOS_API int nos_attn_f32_set_variant(int variant) {
  if (variant < 0 || variant > 7) return (int)hipErrorInvalidValue;
  g_variant = variant;
  return 0;
}

// q/k/v: row r of batch b at base + b*bs_in + r*ld_in (+ head*64), fp32, 16-byte
// aligned rows; o: [B, Sq, H*64] rows at b*bs_out + r*ld_out.
NOS_API int nos_attn_fwd_f32_d64(const float* q, const float* k, const float* v, float* o, int B, int H, int Sq,
                                 int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float scale,
                                 hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Skv <= 0) return (int)hipErrorInvalidValue;
  if (ld_in < H * D || ld_out < H * D || (ld_in & 3) || (ld_out & 3) || (bs_in & 3) || (bs_out & 3))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) return (int)hipErrorInvalidValue;
  const float c = scale * 1.4426950408889634f;
  // auto: 2 wave groups when the grid leaves CUs without a workgroup (one pod
  // at B=1: 162 workgroups, 240 vs 269 us), else 32-key tiles at 4 waves per
  // SIMD (B=8: 1298 vs 1357 us for 64-key tiles at 2;
  // profiles/r02_attention_f32.json, r02_attention_f32_tilings.json)
  const long long nwg = (long long)B * H * ((Sq + 127) / 128);
  const int var = g_variant != 0 ? g_variant : nwg <= nos_effective_cus() ? 2 : 6;
  if (var == 1) return launch<4, 64, 1>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  if (var == 3) return launch<4, 32, 1>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  if (var == 4) return launch<2, 64, 1>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  if (var == 5) return launch<8, 64, 1>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  if (var == 6) return launch<4, 32, 1, 3>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  if (var == 7) return launch<4, 32, 2>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
  return launch<4, 64, 2>(q, k, v, o, B, H, Sq, Skv, ld_in, bs_in, ld_out, bs_out, c, stream);
}
