// Fused multi-head self-attention forward in exact fp32 (head_dim 64, non-causal)
// for the fp32 YOLOS tenant pods -- the precision of the reference demo's
// HF model (demos/gpu-sharing-comparison/client/main.py:19-20).
//
// gfx950 has an exact f32-input MFMA (v_mfma_f32_32x32x2_f32: fmaf-chain
// numerics, 64 FLOP/clk/SIMD) but no xf32, so fp32 attention is MFMA-bound at
// 1/16 of the bf16 rate; the design keeps the matrix pipe fed and everything
// else off it:
//
//  * one wave = 32 query rows of one (batch, head); waves are independent (no
//    LDS, no barriers), four per workgroup; the grid is XCD-remapped so the
//    q-blocks of one head share an XCD's L2 (K/V of one head = 1.7 MB fp32);
//  * "swapped" QK^T: S^T = K . Q^T with the head dim split as d = 32*h + kk
//    (h = lane >> 5, kk = MFMA step), so each lane loads 128 contiguous bytes
//    of its K row and keeps its Q half-row (pre-scaled by scale*log2 e) in 32
//    registers for the whole kernel;
//  * S^T's accumulator has the query on the lane and 16 of the 32 keys in
//    registers: row max / sum are lane-local plus one v_permlane32_swap, and
//    O's per-query rescale is a per-lane scalar;
//  * the accumulator registers ARE the B operand of O^T = V^T . P^T (register
//    r of lane-half h is key (r&3) + 8(r>>2) + 4h, so V^T's A operand is
//    gathered in that key order) -- no LDS round trip, no transpose;
//  * the next key block's K and V are loaded into a second register set while
//    the current one is multiplied (software-pipelined global loads).
#include "common.h"

namespace {

constexpr int D = 64;
constexpr int WAVES = 4;
constexpr int NT = 64 * WAVES;

__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct KV {
  float k[32];      // K[j0 + (lane&31)][32h + kk]
  float v[2][16];   // V[j0 + key(r, h)][32t + (lane&31)]
};

__device__ __forceinline__ void load_kv(KV& kv, const float* __restrict__ kbase, const float* __restrict__ vbase,
                                        int j0, int Skv, int ld, int lane) {
  const int h = lane >> 5, c = lane & 31;
  const int jr = min(j0 + c, Skv - 1);
  const float4* kp = reinterpret_cast<const float4*>(kbase + (long long)jr * ld + 32 * h);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float4 x = kp[u];
    kv.k[4 * u + 0] = x.x;
    kv.k[4 * u + 1] = x.y;
    kv.k[4 * u + 2] = x.z;
    kv.k[4 * u + 3] = x.w;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = min(j0 + (r & 3) + 8 * (r >> 2) + 4 * h, Skv - 1);
    const float* vp = vbase + (long long)j * ld + c;
    kv.v[0][r] = vp[0];
    kv.v[1][r] = vp[32];
  }
}

__global__ __launch_bounds__(NT, 2) void attn_fwd_f32_d64_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, float* __restrict__ o,
    int B, int H, int Sq, int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float c, int nqb) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int item = nos::xcd_remap(blockIdx.x, gridDim.x) * WAVES + wave;
  if (item >= B * H * nqb) return;  // whole wave leaves; nothing below synchronises across waves
  const int qb = item % nqb;
  const int bh = item / nqb;
  const int hh = bh % H, b = bh / H;
  const int h = lane >> 5, col = lane & 31;
  const int q0 = qb * 32;

  const long long boff = (long long)b * bs_in + hh * D;
  const float* kbase = k + boff;
  const float* vbase = v + boff;

  float qf[32];
  {
    const int qr = min(q0 + col, Sq - 1);
    const float4* qp = reinterpret_cast<const float4*>(q + boff + (long long)qr * ld_in + 32 * h);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 x = qp[u];
      qf[4 * u + 0] = x.x * c;
      qf[4 * u + 1] = x.y * c;
      qf[4 * u + 2] = x.z * c;
      qf[4 * u + 3] = x.w * c;
    }
  }

  f32x16_t acc_o[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc_o[0][r] = 0.f;
    acc_o[1][r] = 0.f;
  }
  float m_run = -INFINITY;
  float l_run = 0.f;  // this lane-half's partial row sum (halves merged at the end)

  const int nkb = (Skv + 31) / 32;
  KV cur, nxt;
  load_kv(cur, kbase, vbase, 0, Skv, ld_in, lane);
  for (int kb = 0; kb < nkb; ++kb) {
    const int j0 = kb * 32;
    if (kb + 1 < nkb) load_kv(nxt, kbase, vbase, j0 + 32, Skv, ld_in, lane);

    // S^T[j][i] (log2 units): lane holds query i = col, keys key(r, h)
    f32x16_t s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) s = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.k[kk], qf[kk], s, 0, 0, 0);

    if (j0 + 32 > Skv) {  // tail block: keys past Skv never contribute
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (j0 + (r & 3) + 8 * (r >> 2) + 4 * h >= Skv) s[r] = -INFINITY;
    }
    float mb = s[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mb = fmaxf(mb, s[r]);
    mb = xor32_max(mb);
    const float m_new = fmaxf(m_run, mb);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 0 on the first block
    m_run = m_new;
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = __builtin_amdgcn_exp2f(s[r] - m_new);
      ls += s[r];
    }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc_o[0][r] *= alpha;
      acc_o[1][r] *= alpha;
    }
    // O^T[d][i] += V^T[d][j] P^T[j][i]; step r sums keys {key(r,0), key(r,1)}
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc_o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.v[0][r], s[r], acc_o[0], 0, 0, 0);
      acc_o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.v[1][r], s[r], acc_o[1], 0, 0, 0);
    }
    if (kb + 1 < nkb) cur = nxt;
  }

  const float inv = 1.f / xor32_sum(l_run);
  const int qi = q0 + col;
  if (qi < Sq) {
    float* op = o + (long long)b * bs_out + (long long)qi * ld_out + hh * D;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 y;
        y.x = acc_o[t][4 * g + 0] * inv;
        y.y = acc_o[t][4 * g + 1] * inv;
        y.z = acc_o[t][4 * g + 2] * inv;
        y.w = acc_o[t][4 * g + 3] * inv;
        *reinterpret_cast<float4*>(op + 32 * t + 8 * g + 4 * h) = y;
      }
  }
}

}  // namespace

// q/k/v: row r of batch b at base + b*bs_in + r*ld_in (+ head*64), fp32, 16-byte
// aligned rows; o: [B, Sq, H*64] rows at b*bs_out + r*ld_out.
NOS_API int nos_attn_fwd_f32_d64(const float* q, const float* k, const float* v, float* o, int B, int H, int Sq,
                                 int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float scale,
                                 hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Skv <= 0) return (int)hipErrorInvalidValue;
  if (ld_in < H * D || ld_out < H * D || (ld_in & 3) || (ld_out & 3) || (bs_in & 3) || (bs_out & 3))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15) return (int)hipErrorInvalidValue;
  const int nqb = (Sq + 31) / 32;
  const long long items = (long long)B * H * nqb;
  if (items > (1LL << 30)) return (int)hipErrorInvalidValue;
  const int grid = (int)((items + WAVES - 1) / WAVES);
  const float c = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(attn_fwd_f32_d64_kernel, dim3(grid), dim3(NT), 0, stream, q, k, v, o, B, H, Sq, Skv, ld_in,
                     bs_in, ld_out, bs_out, c, nqb);
  return (int)hipGetLastError();
}
