// Stateful decoding on the pod server (nos_amd/podserver/program/, ops
// kv_write / rotary_at / sdpa_cache / pos_add / pos_set / argmax) and the
// skinny GEMMs a decode step is made of.  A tenant's K / V cache and its
// position counter live in device memory across requests; every kernel here
// reads the positions ON THE DEVICE, so one captured HIP graph serves every
// step of a generation, and every index a position produces is bounds-checked
// against the buffers (a replay never faults on a bad counter: rows past the
// cache are dropped, table rows clamp).
//
//  * nos_kv_write -- cache[b, pos[b] + s] = x[b, s] (optionally rotated at
//    that position first: the K projection's rotary fused into the write);
//  * nos_rotary_pos -- rotate_half rotary at positions pos[b] + s;
//  * nos_attn_decode -- flash-decoding: query rows at positions pos[b] + i
//    attend the cached keys 0 .. pos[b] + i.  The cache is HBM-bound (per key
//    2 x D loads for G x Sq x 2 D FLOPs, ~2 FLOP/B at Sq = 1): the kernel runs
//    at the cache's own precision with fp32 FMAs on the VALU -- exact for an
//    fp32 cache, more precise than the h3 pipes -- and spends its effort on
//    bandwidth: one workgroup per (sequence, K/V head, 128-key split), every
//    query head of the group (grouped-query) served from one read of the
//    split's keys and values, staged through LDS with 16-byte loads;
//    nos_attn_decode_combine merges the splits (log-sum-exp);
//  * nos_pos_update -- pos += n / pos = n;
//  * nos_argmax -- greedy next tokens, one wave per row;
//  * nos_gemv -- y = act(r x W^T + b) + R for M <= 8 rows (a decode step's
//    every GEMM): weight-streaming, each wave two output columns, lanes over
//    K with 16-byte weight loads, x rows in LDS (optionally RMS-normalised in
//    the prologue: RMSNorm folded into the GEMM, gamma in W), exact fp32 math.
#include <float.h>
#include <math.h>

#include "common.h"

namespace {

enum : int { EPI_BIAS = 1, EPI_GELU = 2, EPI_RESID = 4, EPI_RELU = 8, EPI_SILU = 64, EPI_GLU = 256 };
// EPI_GLU (GEMV): W = [gate; up] (2 Nh rows), y [M, Nh] = silu(x . gate_n) * (x . up_n) -- SwiGLU
// in the merged gate-up GEMV's epilogue, each wave's two columns being n and n + Nh

__device__ __forceinline__ float ldf(const void* p, long long i, int bf) {
  return bf ? nos::bf16_to_f32(static_cast<const unsigned short*>(p)[i]) : static_cast<const float*>(p)[i];
}

__device__ __forceinline__ void stf(void* p, long long i, float v, int bf) {
  if (bf)
    static_cast<unsigned short*>(p)[i] = nos::f32_to_bf16(v);
  else
    static_cast<float*>(p)[i] = v;
}

// 4 consecutive elements (16-byte fp32 or 8-byte bf16 load) as floats
__device__ __forceinline__ float4 ld4(const void* p, long long i, int bf) {
  if (bf) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(p) + i);
    return float4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                  __uint_as_float(u.y & 0xffff0000u)};
  }
  return *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
}

// the same 4 elements split into the load and the conversion: a batch of loads stays in
// flight whatever the dtype (ld4's bf16 path converts inside its branch, so each of its
// loads waited for its data before the next one issued)
__device__ __forceinline__ uint4 ld4raw(const void* p, long long i, int bf) {
  if (bf) {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(p) + i);
    return uint4{u.x, u.y, 0u, 0u};
  }
  return *reinterpret_cast<const uint4*>(static_cast<const float*>(p) + i);
}

__device__ __forceinline__ float4 cvt4(uint4 r, int bf) {
  if (bf)
    return float4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
                  __uint_as_float(r.y & 0xffff0000u)};
  return float4{__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z), __uint_as_float(r.w)};
}

// ------------------------------------------------------------------ kv_write / rotary at device positions
// one thread per (b, s, h, d < D/2) pair (d, d + D/2): the rotate_half pair
// a fused rotary needs; without tables it just copies both elements
// one K / V pair per launch: blockIdx.y 0 = (x, cache) with the rotary tables
// (K), 1 = (x2, cache2) plain (V; x2 == nullptr: a single write)
struct KvPair {
  const void* x2;
  int ldx2;
  long long bsx2;
  void* cache2;
};

__global__ __launch_bounds__(256) void kv_write_kernel(const void* __restrict__ x, int xbf, int ldx, long long bsx,
                                                       void* __restrict__ cache, int cbf, const int* __restrict__ pos,
                                                       const float* __restrict__ cs, const float* __restrict__ sn,
                                                       int R, int B, int S, int H, int D, int L, KvPair v2) {
  if (blockIdx.y == 1) {  // the V half: its own rows, no rotation
    x = v2.x2;
    ldx = v2.ldx2;
    bsx = v2.bsx2;
    cache = v2.cache2;
    cs = sn = nullptr;
  }
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int hd = D / 2;
  if (i >= (long long)B * S * H * hd) return;
  const int d = (int)(i % hd);
  long long r = i / hd;
  const int h = (int)(r % H);
  r /= H;
  const int s = (int)(r % S), b = (int)(r / S);
  const int p = pos[b] + s;
  if (p < 0 || p >= L) return;  // past the cache: dropped (the server reports the overflow)
  const long long xo = b * bsx + (long long)s * ldx + (long long)h * D;
  float x0 = ldf(x, xo + d, xbf), x1 = ldf(x, xo + d + hd, xbf);
  if (cs != nullptr) {
    const long long t = (long long)min(p, R - 1) * D;
    const float y0 = fmaf(x0, cs[t + d], -x1 * sn[t + d]);
    const float y1 = fmaf(x1, cs[t + d + hd], x0 * sn[t + d + hd]);
    x0 = y0;
    x1 = y1;
  }
  const long long co = (((long long)b * L + p) * H + h) * D;
  stf(cache, co + d, x0, cbf);
  stf(cache, co + d + hd, x1, cbf);
}

__global__ __launch_bounds__(256) void rotary_pos_kernel(const void* __restrict__ x, int ldx, long long bsx,
                                                         void* __restrict__ y, const int* __restrict__ pos,
                                                         const float* __restrict__ cs, const float* __restrict__ sn,
                                                         int R, int B, int S, int H, int D, int bf) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int hd = D / 2;
  if (i >= (long long)B * S * H * hd) return;
  const int d = (int)(i % hd);
  long long r = i / hd;
  const int h = (int)(r % H);
  r /= H;
  const int s = (int)(r % S), b = (int)(r / S);
  const int p = min(max(pos[b] + s, 0), R - 1);
  const long long xo = b * bsx + (long long)s * ldx + (long long)h * D;
  const float x0 = ldf(x, xo + d, bf), x1 = ldf(x, xo + d + hd, bf);
  const long long t = (long long)p * D;
  const long long yo = (((long long)b * S + s) * H + h) * D;
  stf(y, yo + d, fmaf(x0, cs[t + d], -x1 * sn[t + d]), bf);
  stf(y, yo + d + hd, fmaf(x1, cs[t + d + hd], x0 * sn[t + d + hd]), bf);
}

// ------------------------------------------------------------------ decode attention
constexpr int KC = 128;      // keys per split (one workgroup)
constexpr int MAXR = 32;     // query rows (G x Sq) per launch

// workgroup (b, kvh, split): rows r = qi * G + g (query token qi of Sq, query
// head kvh * G + g); q rows scaled (and rotated) into LDS, the split's keys
// into LDS, scores -> per-row max / sum -> probabilities in LDS, the split's
// values into LDS, P V; the partial (acc[D], m, l) of every row to ws
// the step's own K / V rows (written into the caches by this kernel instead of a
// kv_write launch): token t of batch b at k + b * bsk + t * ldk + h * D (V alike),
// cache row pos[b] + t; n = 0: none (the caches already hold them)
struct Fresh {
  const void* k = nullptr;
  const void* v = nullptr;
  void* kc = nullptr;
  void* vc = nullptr;
  long long bsk = 0, bsv = 0;
  int ldk = 0, ldv = 0, bf = 0, n = 0;
};

// row r of group bk = (b, kvh): out[b, q0 + qi, h, d] = sum_s e^(m_s - M) acc_s / sum_s
// e^(m_s - M) l_s over the NS splits' partials (splits with l = 0 skipped)
template <int D>
__device__ __forceinline__ void decode_combine_row(const float* __restrict__ ws, void* __restrict__ o, int obf,
                                                   int bk, int r, int d, int NS, int G, int R, int H, int Hkv,
                                                   int Sq_total, int q0) {
  const int kvh = bk % Hkv, b = bk / Hkv;
  const int qi = r / G, h = kvh * G + r % G;
  float M = -INFINITY;
  for (int s = 0; s < NS; ++s) {
    const float* p = ws + ((long long)(bk * NS + s) * R + r) * (D + 2);
    if (p[D + 1] > 0.f) M = fmaxf(M, p[D]);
  }
  float num = 0.f, den = 0.f;
  for (int s = 0; s < NS; ++s) {
    const float* p = ws + ((long long)(bk * NS + s) * R + r) * (D + 2);
    if (p[D + 1] > 0.f) {
      const float w = __expf(p[D] - M);
      num = fmaf(w, p[d], num);
      den = fmaf(w, p[D + 1], den);
    }
  }
  const long long oo = (((long long)b * Sq_total + q0 + qi) * H + h) * D + d;
  stf(o, oo, den > 0.f ? num / den : 0.f, obf);
}

// the combine launch folded into the decode launch (sync != null): each workgroup
// publishes its partial (device-scope fence: the splits run on different XCDs, each
// with its own L2), counts itself in on its group's counter, and the group's last
// workgroup combines the NS partials and zeroes the counter for the next launch.
// No workgroup waits on another, so the grid drains whatever the order.
template <int D>
__device__ __forceinline__ void decode_combine_last(const float* __restrict__ ws, int* __restrict__ sync,
                                                    void* __restrict__ o, int obf, int bk, int NS, int G, int R,
                                                    int H, int Hkv, int Sq_total, int q0, int tid) {
  if (sync == nullptr) return;
  __shared__ int last;
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(&sync[bk], 1) == NS - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int e = tid; e < R * D; e += 256) decode_combine_row<D>(ws, o, obf, bk, e / D, e % D, NS, G, R, H, Hkv, Sq_total, q0);
  if (tid == 0) atomicExch(&sync[bk], 0);
}

template <int D, int CBF>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const void* __restrict__ q, int qbf, int ldq, long long bsq, const void* __restrict__ kc,
    const void* __restrict__ vc, int /*cbf = CBF*/, const int* __restrict__ pos, const float* __restrict__ cs,
    const float* __restrict__ sn, int Rtab, float* __restrict__ ws, int B, int H, int Hkv, int Sq, int q0, int L,
    int NS, float scale, Fresh fr, int* __restrict__ sync, void* __restrict__ o, int obf, int Sq_total) {
  constexpr int cbf = CBF;   // the cache dtype fixed at compile time: no per-load dtype branch
  constexpr int DP = D + 4;  // padded LDS row (16-byte reads of consecutive rows hit distinct banks)
  __shared__ __attribute__((aligned(16))) float qs[MAXR * D];
  __shared__ __attribute__((aligned(16))) float kv[KC * DP];
  __shared__ float sc[MAXR * KC];
  __shared__ float mrow[MAXR], lrow[MAXR];
  const int G = H / Hkv, R = G * Sq;
  const int split = blockIdx.x % NS, bk = blockIdx.x / NS;
  const int kvh = bk % Hkv, b = bk / Hkv;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p0 = pos[b] + q0;                              // position of query row qi = 0 of this launch
  const int kend = min(p0 + Sq, L);                        // keys 0 .. kend - 1 are visible to some row
  const int k0 = split * KC, nk = min(KC, kend - k0);
  float* const out = ws + (long long)blockIdx.x * R * (D + 2);
  const long long cstride = (long long)Hkv * D;  // cache row (token) stride
  // the first launch of a step writes the step's fresh K (rotated) / V rows that fall in
  // this split's key range into the caches -- every split, empty or not, so a later
  // launch (query rows q0 > 0) and the next step read them from the cache
  const bool fresh = fr.n > 0 && q0 == 0 && pos[b] >= 0;
  auto fresh_row = [&](int t, int d, bool isk, float& x0, float& x1) {
    const void* src = isk ? fr.k : fr.v;
    const long long o = (long long)b * (isk ? fr.bsk : fr.bsv) + (long long)t * (isk ? fr.ldk : fr.ldv) +
                        (long long)kvh * D;
    x0 = ldf(src, o + d, fr.bf);
    x1 = ldf(src, o + d + D / 2, fr.bf);
    if (isk && cs != nullptr) {
      const long long tt = (long long)min(pos[b] + t, Rtab - 1) * D;
      const float y0 = fmaf(x0, cs[tt + d], -x1 * sn[tt + d]);
      const float y1 = fmaf(x1, cs[tt + d + D / 2], x0 * sn[tt + d + D / 2]);
      x0 = y0;
      x1 = y1;
    }
  };
  // the split's K and V rows are loaded into registers first, every load of both in flight
  // at once; the fresh-row stores, the q staging and the scores overlap their latency (a
  // fresh row's stale cache value is replaced by the overlay below)
  const long long cbase = ((long long)b * L + k0) * cstride + (long long)kvh * D;
  constexpr int PER = KC * (D / 4) / 256;
  static_assert(PER * 256 == KC * (D / 4), "whole float4 pieces per thread");
  uint4 kr[PER], vr[PER];
  const bool live = nk > 0 && p0 >= 0;
  if (live) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + 256 * u, j = e / (D / 4), d4 = (e % (D / 4)) * 4;
      kr[u] = j < nk ? ld4raw(kc, cbase + j * cstride + d4, cbf) : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + 256 * u, j = e / (D / 4), d4 = (e % (D / 4)) * 4;
      vr[u] = j < nk ? ld4raw(vc, cbase + j * cstride + d4, cbf) : uint4{0u, 0u, 0u, 0u};
    }
  }
  if (fresh) {
    for (int e = tid; e < 2 * fr.n * (D / 2); e += 256) {
      const int isv = e >= fr.n * (D / 2), ee = isv ? e - fr.n * (D / 2) : e;
      const int t = ee / (D / 2), d = ee % (D / 2), jabs = pos[b] + t;
      if (jabs < k0 || jabs >= k0 + KC || jabs >= L) continue;
      float x0, x1;
      fresh_row(t, d, !isv, x0, x1);
      void* cache = isv ? fr.vc : fr.kc;
      const long long co = ((long long)b * L + jabs) * cstride + (long long)kvh * D;
      stf(cache, co + d, x0, cbf);
      stf(cache, co + d + D / 2, x1, cbf);
    }
  }
  // the fresh rows this split attends come from the registers' source, not the cache
  // (its stores above may still be in flight): staged over the cache's rows
  auto overlay = [&](bool isk) {
    if (!fresh) return;
    __syncthreads();
    for (int e = tid; e < fr.n * (D / 2); e += 256) {
      const int t = e / (D / 2), d = e % (D / 2), j = pos[b] + t - k0;
      if (j < 0 || j >= nk) continue;
      float x0, x1;
      fresh_row(t, d, isk, x0, x1);
      kv[j * (D + 4) + d] = x0;
      kv[j * (D + 4) + d + D / 2] = x1;
    }
  };
  if (!live) {  // an empty split (or a bad counter): l = 0, skipped by the combine
    for (int r = tid; r < R; r += 256) {
      out[r * (D + 2) + D] = -INFINITY;
      out[r * (D + 2) + D + 1] = 0.f;
    }
    decode_combine_last<D>(ws, sync, o, obf, bk, NS, G, R, H, Hkv, Sq_total, q0, tid);
    return;
  }
  // q rows -> LDS, times the softmax scale (rotated at their positions first)
  for (int e = tid; e < R * (D / 2); e += 256) {
    const int r = e / (D / 2), d = e % (D / 2);
    const int qi = r / G, g = r % G, h = kvh * G + g;
    const long long qo = b * bsq + (long long)(q0 + qi) * ldq + (long long)h * D;
    float x0 = ldf(q, qo + d, qbf), x1 = ldf(q, qo + d + D / 2, qbf);
    if (cs != nullptr) {
      const long long t = (long long)min(max(p0 + qi, 0), Rtab - 1) * D;
      const float y0 = fmaf(x0, cs[t + d], -x1 * sn[t + d]);
      const float y1 = fmaf(x1, cs[t + d + D / 2], x0 * sn[t + d + D / 2]);
      x0 = y0;
      x1 = y1;
    }
    qs[r * D + d] = x0 * scale;
    qs[r * D + d + D / 2] = x1 * scale;
  }
  // the split's rows -> LDS from the registers loaded at the start (rows past nk zero)
  auto stage = [&](const uint4 (&v)[PER]) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int e = tid + 256 * u, j = e / (D / 4), d4 = (e % (D / 4)) * 4;
      *reinterpret_cast<float4*>(&kv[j * DP + d4]) = cvt4(v[u], cbf);
    }
  };
  stage(kr);
  overlay(true);
  __syncthreads();
  // scores: thread -> key j, rows of one parity
  {
    const int j = tid & (KC - 1), rh = tid >> 7;
    const int jabs = k0 + j;
    // two partial dot products per row (even / odd float4s of d): at decode's few
    // rows (G x 1) one chain of D dependent FMAs per row was latency-bound
    float acc[MAXR / 2], acc2[MAXR / 2];
#pragma unroll
    for (int i = 0; i < MAXR / 2; ++i) acc[i] = acc2[i] = 0.f;
    for (int d4 = 0; d4 < D; d4 += 8) {
      const float4 kk = *reinterpret_cast<const float4*>(&kv[j * DP + d4]);
      const float4 k2 = *reinterpret_cast<const float4*>(&kv[j * DP + d4 + 4]);
#pragma unroll
      for (int i = 0; i < MAXR / 2; ++i) {
        const int r = rh + 2 * i;
        if (r < R) {
          const float4 qq = *reinterpret_cast<const float4*>(&qs[r * D + d4]);
          const float4 q2 = *reinterpret_cast<const float4*>(&qs[r * D + d4 + 4]);
          acc[i] = fmaf(qq.x, kk.x, fmaf(qq.y, kk.y, fmaf(qq.z, kk.z, fmaf(qq.w, kk.w, acc[i]))));
          acc2[i] = fmaf(q2.x, k2.x, fmaf(q2.y, k2.y, fmaf(q2.z, k2.z, fmaf(q2.w, k2.w, acc2[i]))));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MAXR / 2; ++i) acc[i] += acc2[i];
#pragma unroll
    for (int i = 0; i < MAXR / 2; ++i) {
      const int r = rh + 2 * i;
      if (r < R) {
        const int qpos = p0 + r / G;  // causal: this row sees keys <= its position
        sc[r * KC + j] = (j < nk && jabs <= qpos) ? acc[i] : -INFINITY;
      }
    }
  }
  __syncthreads();
  // per-row max / sum over the split; probabilities back into sc
  for (int r = wid; r < R; r += 4) {
    const float s0 = sc[r * KC + lane], s1 = sc[r * KC + lane + 64];
    const float m = nos::wave_max(fmaxf(s0, s1));
    const float e0 = m == -INFINITY ? 0.f : __expf(s0 - m), e1 = m == -INFINITY ? 0.f : __expf(s1 - m);
    sc[r * KC + lane] = e0;
    sc[r * KC + lane + 64] = e1;
    const float l = nos::wave_sum(e0 + e1);
    if (lane == 0) {
      mrow[r] = m;
      lrow[r] = l;
    }
  }
  __syncthreads();  // every wave is done with the keys
  stage(vr);
  overlay(false);
  __syncthreads();
  // P V: thread -> column d, rows of one residue
  {
    constexpr int RS = 256 / D;  // rows in parallel
    const int d = tid % D, r0 = tid / D;
    for (int r = r0; r < R; r += RS) {
      // four partial sums: a chain of nk dependent FMAs (each behind two LDS reads) was
      // latency-bound; keys past nk hold P = 0 and zero V rows, so the unrolled tail adds 0
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      for (int j = 0; j < nk; j += 4) {
        a0 = fmaf(sc[r * KC + j], kv[j * DP + d], a0);
        a1 = fmaf(sc[r * KC + j + 1], kv[(j + 1) * DP + d], a1);
        a2 = fmaf(sc[r * KC + j + 2], kv[(j + 2) * DP + d], a2);
        a3 = fmaf(sc[r * KC + j + 3], kv[(j + 3) * DP + d], a3);
      }
      out[r * (D + 2) + d] = (a0 + a1) + (a2 + a3);
    }
    for (int r = tid; r < R; r += 256) {
      out[r * (D + 2) + D] = mrow[r];
      out[r * (D + 2) + D + 1] = lrow[r];
    }
  }
  decode_combine_last<D>(ws, sync, o, obf, bk, NS, G, R, H, Hkv, Sq_total, q0, tid);
}

// out[b, q0 + qi, h, :] = sum_s e^(m_s - M) acc_s / sum_s e^(m_s - M) l_s over the splits
template <int D>
__global__ __launch_bounds__(D) void attn_decode_combine_kernel(const float* __restrict__ ws, void* __restrict__ o,
                                                                int obf, int B, int H, int Hkv, int Sq, int q0,
                                                                int Sq_total, int NS) {
  const int G = H / Hkv, R = G * Sq;
  const int row = blockIdx.x;  // (b, kvh, r)
  decode_combine_row<D>(ws, o, obf, row / R, row % R, threadIdx.x, NS, G, R, H, Hkv, Sq_total, q0);
}

// ------------------------------------------------------------------ positions, argmax
__global__ void pos_update_kernel(int* __restrict__ pos, int B, int add, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) pos[i] = add ? pos[i] + n : n;
}

// first index of the row maximum (torch.argmax's tie rule); NaN rows give the NaN's index
// (value, index) b better than a: NaN beats numbers (torch.argmax), then the
// larger value, then the smaller index -- the first maximum
__device__ __forceinline__ bool am_better(float bv, int bi, float av, int ai) {
  const bool bn = bv != bv, an = av != av;
  if (bn != an) return bn;
  if (bn) return bi < ai;
  return bv > av || (bv == av && bi < ai);
}

// one workgroup of NT threads per row: 4 independent loads in flight per thread
// per step (a wave per row left a 32000-wide vocabulary row latency-bound at
// ~180 us), wave shuffles, then the waves' winners through LDS
template <int NT>
__global__ __launch_bounds__(NT) void argmax_kernel(const void* __restrict__ x, int bf, int rows, int L, int ldx,
                                                    int* __restrict__ out, int* __restrict__ pos, int pos_n) {
  __shared__ float sv[NT / 64];
  __shared__ int si[NT / 64];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const long long base = (long long)row * ldx;
  float best = -INFINITY;
  int bi = INT_MAX;
  for (int j0 = tid; j0 < L; j0 += 4 * NT) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * NT;
      v[u] = j < L ? ldf(x, base + j, bf) : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * NT;
      if (j < L && am_better(v[u], j, best, bi)) {
        best = v[u];
        bi = j;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (am_better(ob, oi, best, bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) {
    sv[wid] = best;
    si[wid] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < NT / 64; ++w)
      if (am_better(sv[w], si[w], best, bi)) {
        best = sv[w];
        bi = si[w];
      }
    out[row] = bi >= L ? 0 : bi;  // an all -inf row: index 0
    if (pos != nullptr) pos[row] += pos_n;  // the step's position advance folded in (row = sequence)
  }
}

// ------------------------------------------------------------------ GEMV (M <= 8)
// x given as the decode attention's split partials (ws != null): x row m = sequence m's
// single query token, x[m][h * D + d] combined from the NS splits of (m, h / G) exactly as
// attn_decode_combine_kernel does -- the combine launch folded into the O-projection
struct Parts {
  const float* ws = nullptr;
  int NS = 0, R = 0, G = 0, Hkv = 0, D = 0;
};

__device__ __forceinline__ float4 parts_x4(const Parts& pt, int m, int k) {
  const int h = k / pt.D, d = k % pt.D, kvh = h / pt.G, r = h % pt.G;  // r = g (one query token)
  const int bk = m * pt.Hkv + kvh;
  const long long row = (long long)(pt.D + 2);
  float M = -INFINITY;
  for (int s = 0; s < pt.NS; ++s) {
    const float* p = pt.ws + ((long long)(bk * pt.NS + s) * pt.R + r) * row;
    if (p[pt.D + 1] > 0.f) M = fmaxf(M, p[pt.D]);
  }
  float n0 = 0.f, n1 = 0.f, n2 = 0.f, n3 = 0.f, den = 0.f;
  for (int s = 0; s < pt.NS; ++s) {
    const float* p = pt.ws + ((long long)(bk * pt.NS + s) * pt.R + r) * row;
    if (p[pt.D + 1] > 0.f) {
      const float w = __expf(p[pt.D] - M);
      n0 = fmaf(w, p[d], n0);
      n1 = fmaf(w, p[d + 1], n1);
      n2 = fmaf(w, p[d + 2], n2);
      n3 = fmaf(w, p[d + 3], n3);
      den = fmaf(w, p[pt.D + 1], den);
    }
  }
  return den > 0.f ? float4{n0 / den, n1 / den, n2 / den, n3 / den} : float4{0.f, 0.f, 0.f, 0.f};
}

template <int M, int WBF, int KU>
__global__ __launch_bounds__(256) void gemv_kernel(const void* __restrict__ x, int xbf, int ldx,
                                                   const void* __restrict__ w, int /*wbf = WBF*/, int ldw,
                                                   const void* __restrict__ bias, const void* __restrict__ res,
                                                   int ldr, void* __restrict__ y, int ldy, int N, int K, int epi,
                                                   float rms_eps, Parts pt) {
  constexpr int wbf = WBF;  // the weight dtype fixed at compile time: no per-load dtype branch
  extern __shared__ __attribute__((aligned(16))) float xs[];  // [M][K] fp32
  __shared__ float rsc[M];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool glu = (epi & EPI_GLU) != 0;
  const int Nh = N / 2;                                          // GLU: output columns
  const int ngrp = glu ? (Nh + 3) / 4 : (N + 7) / 8;             // 8 columns per pass: 4 waves x 2
  // the weight rows (two per wave) of column group grp: GLU pairs gate n0 with up n0 + Nh
  auto rows_of = [&](int grp, int& n0, long long& w0, long long& w1) {
    n0 = glu ? grp * 4 + wid : grp * 8 + wid * 2;
    const int nc0 = glu ? min(n0, Nh - 1) : min(n0, N - 1);
    const int nc1 = glu ? min(n0, Nh - 1) + Nh : min(n0 + 1, N - 1);
    w0 = (long long)nc0 * ldw;
    w1 = (long long)nc1 * ldw;
  };
  auto load_chunk = [&](long long w0, long long w1, int k0, uint4 (&a)[KU], uint4 (&c4)[KU]) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = k0 + 256 * u;
      a[u] = k < K ? ld4raw(w, w0 + k, wbf) : uint4{0u, 0u, 0u, 0u};
      c4[u] = k < K ? ld4raw(w, w1 + k, wbf) : uint4{0u, 0u, 0u, 0u};
    }
  };
  // the first group's first K chunk of weights in flight while x is staged and normalised:
  // the weights do not depend on x, and the two memory latencies were back to back
  uint4 pa[KU], pc[KU];
  if ((int)blockIdx.x < ngrp) {
    int n0;
    long long w0, w1;
    rows_of(blockIdx.x, n0, w0, w1);
    load_chunk(w0, w1, lane * 4, pa, pc);
  }
  for (int e = tid * 4; e < M * K; e += 1024) {
    const int m = e / K, k = e % K;
    *reinterpret_cast<float4*>(&xs[e]) = pt.ws ? parts_x4(pt, m, k) : ld4(x, (long long)m * ldx + k, xbf);
  }
  __syncthreads();
  if (rms_eps > 0.f) {  // RMSNorm of each row, gamma folded into W
    for (int m = wid; m < M; m += 4) {
      float q = 0.f;
      for (int k = lane; k < K; k += 64) q = fmaf(xs[m * K + k], xs[m * K + k], q);
      q = nos::wave_sum(q);
      if (lane == 0) rsc[m] = rsqrtf(q / (float)K + rms_eps);
    }
  } else if (tid < M) {
    rsc[tid] = 1.f;
  }
  __syncthreads();
  for (int grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {
    int n0;
    long long w0, w1;
    rows_of(grp, n0, w0, w1);
    float acc[2][M];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[c][m] = 0.f;
    // KU K steps' weight loads issued together (2 KU float4 in flight per lane): the
    // one-step loop waited a full memory latency per 256 columns of K; KU = 12 takes
    // K <= 3072 (a down projection) in one batch (the same summation order as KU = 4)
    for (int k0 = lane * 4; k0 < K; k0 += 256 * KU) {
      uint4 ra[KU], rc[KU];
      if (grp == (int)blockIdx.x && k0 == lane * 4) {
#pragma unroll
        for (int u = 0; u < KU; ++u) {
          ra[u] = pa[u];
          rc[u] = pc[u];
        }
      } else {
        load_chunk(w0, w1, k0, ra, rc);
      }
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int k = k0 + 256 * u;
        if (k < K) {
          const float4 a = cvt4(ra[u], wbf), c4 = cvt4(rc[u], wbf);
#pragma unroll
          for (int m = 0; m < M; ++m) {
            const float4 xv = *reinterpret_cast<const float4*>(&xs[m * K + k]);
            acc[0][m] = fmaf(a.x, xv.x, fmaf(a.y, xv.y, fmaf(a.z, xv.z, fmaf(a.w, xv.w, acc[0][m]))));
            acc[1][m] = fmaf(c4.x, xv.x, fmaf(c4.y, xv.y, fmaf(c4.z, xv.z, fmaf(c4.w, xv.w, acc[1][m]))));
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[c][m] = nos::wave_sum(acc[c][m]);
    if (glu) {  // lane m finishes output (m, n0): silu(gate) * up
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (lane == m && n0 < Nh) {
          float g = acc[0][m] * rsc[m], u = acc[1][m] * rsc[m];
          if (epi & EPI_BIAS) {
            g += ldf(bias, n0, wbf);
            u += ldf(bias, n0 + Nh, wbf);
          }
          stf(y, (long long)m * ldy + n0, g / (1.f + __expf(-g)) * u, xbf);
        }
      continue;
    }
    // lane (c * M + m) finishes output (m, n0 + c)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int n = n0 + c;
        if (lane == c * M + m && n < N) {
          float v = acc[c][m] * rsc[m];
          if (epi & EPI_BIAS) v += ldf(bias, n, wbf);
          if (epi & EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
          if (epi & EPI_RELU) v = fmaxf(v, 0.f);
          if (epi & EPI_SILU) v = v / (1.f + __expf(-v));
          if (epi & EPI_RESID) v += ldf(res, (long long)m * ldr + n, xbf);
          stf(y, (long long)m * ldy + n, v, xbf);
        }
      }
  }
}

}  // namespace

// x2 / cache2 (optional, same shapes and dtypes): a second write in the same
// launch without rotation -- a layer's V beside its rotated K
NOS_API int nos_kv_write(const void* x, int xbf, int ldx, long long bsx, void* cache, int cbf, const int* pos,
                         const float* cos_t, const float* sin_t, int R, int B, int S, int H, int D, int L,
                         const void* x2, int ldx2, long long bsx2, void* cache2, hipStream_t stream) {
  if (B <= 0 || S <= 0 || H <= 0 || D <= 0 || (D % 2) || L <= 0 || S > L || ldx < H * D || !x || !cache || !pos ||
      (B > 1 && bsx < (long long)(S - 1) * ldx + H * D) || (xbf != 0 && xbf != 1) || (cbf != 0 && cbf != 1) ||
      ((cos_t == nullptr) != (sin_t == nullptr)) || (cos_t && R <= 0) || ((x2 == nullptr) != (cache2 == nullptr)) ||
      (x2 && (ldx2 < H * D || (B > 1 && bsx2 < (long long)(S - 1) * ldx2 + H * D))))
    return (int)hipErrorInvalidValue;
  const long long n = (long long)B * S * H * (D / 2);
  hipLaunchKernelGGL(kv_write_kernel, dim3((unsigned)((n + 255) / 256), x2 ? 2u : 1u), dim3(256), 0, stream, x, xbf,
                     ldx, bsx, cache, cbf, pos, cos_t, sin_t, R, B, S, H, D, L, KvPair{x2, ldx2, bsx2, cache2});
  return (int)hipGetLastError();
}

NOS_API int nos_rotary_pos(const void* x, int ldx, long long bsx, void* y, const int* pos, const float* cos_t,
                           const float* sin_t, int R, int B, int S, int H, int D, int bf16, hipStream_t stream) {
  if (B <= 0 || S <= 0 || H <= 0 || D <= 0 || (D % 2) || R <= 0 || ldx < H * D || !cos_t || !sin_t || !pos ||
      (B > 1 && bsx < (long long)(S - 1) * ldx + H * D) || (bf16 != 0 && bf16 != 1))
    return (int)hipErrorInvalidValue;
  const long long n = (long long)B * S * H * (D / 2);
  hipLaunchKernelGGL(rotary_pos_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, ldx, bsx, y, pos,
                     cos_t, sin_t, R, B, S, H, D, bf16);
  return (int)hipGetLastError();
}

// bytes of nos_attn_decode's workspace
NOS_API long long nos_attn_decode_workspace(int B, int H, int Hkv, int Sq, int L, int D) {
  if (B <= 0 || H <= 0 || Hkv <= 0 || Sq <= 0 || L <= 0 || H % Hkv) return -1;
  const int G = H / Hkv, rows = G * (Sq < MAXR / G ? Sq : (MAXR / G > 0 ? MAXR / G : 1));
  const long long NS = (L + KC - 1) / KC;
  return (long long)B * Hkv * NS * rows * (D + 2) * 4;
}

// q [B, Sq, H, D] (heads contiguous per token; token stride ldq, batch stride
// bsq; fp32 / bf16), caches [B, L, Hkv, D] contiguous (fp32 / bf16), pos [B]
// i32: query i at position pos[b] + i sees keys 0 .. min(pos[b] + i, L - 1).
// cos / sin [R, D] fp32 (or null): q rotated at its positions.  out [B, Sq, H,
// D] contiguous (obf: bf16).  Query tokens are processed in launches of at
// most 32 / G (the rows a workgroup holds), each a decode pass + combine.
// kn / vn (nfresh > 0): the step's own K / V rows [B, nfresh, Hkv, D] (token stride
// ldk / ldv, batch stride bsk / bsv; nbf: bf16) -- written into the caches at
// pos[b] + t (K rotated with cos / sin) by the attention itself, which reads them
// from there: the kv_write launch of the step folded in (nfresh == Sq).  sync
// (sync_n >= B x Hkv i32, zero before the first call, left zero by each): the
// combine folded into the decode launch (its last workgroup per (b, kv head)).
NOS_API int nos_attn_decode(const void* q, int qbf, int ldq, long long bsq, const void* kc, const void* vc, int cbf,
                            const int* pos, const float* cos_t, const float* sin_t, int R, void* out, int obf, int B,
                            int H, int Hkv, int Sq, int L, int D, float scale, void* ws, long long ws_bytes,
                            const void* kn, const void* vn, int nbf, int ldk, long long bsk, int ldv, long long bsv,
                            int nfresh, int* sync, long long sync_n, int partials_only, hipStream_t stream) {
  if (B <= 0 || H <= 0 || Hkv <= 0 || H % Hkv || H / Hkv > MAXR || Sq <= 0 || L <= 0 || (D != 64 && D != 128) ||
      ldq < H * D || (B > 1 && bsq < (long long)(Sq - 1) * ldq + H * D) || !q || !kc || !vc || !pos || !out ||
      !ws || ((cos_t == nullptr) != (sin_t == nullptr)) || (cos_t && R <= 0) || (qbf != 0 && qbf != 1) ||
      (cbf != 0 && cbf != 1) || (obf != 0 && obf != 1) || !(scale > 0.f))
    return (int)hipErrorInvalidValue;
  if (ws_bytes < nos_attn_decode_workspace(B, H, Hkv, Sq, L, D)) return (int)hipErrorInvalidValue;
  if (sync != nullptr && sync_n < (long long)B * Hkv) return (int)hipErrorInvalidValue;
  // partials_only: the splits' partials stay in ws for nos_gemv_partials (one query token)
  if (partials_only && (sync != nullptr || Sq != 1)) return (int)hipErrorInvalidValue;
  Fresh fr;
  if (nfresh != 0) {
    if (nfresh != Sq || !kn || !vn || (nbf != 0 && nbf != 1) || ldk < Hkv * D || ldv < Hkv * D ||
        (B > 1 && (bsk < (long long)(Sq - 1) * ldk + Hkv * D || bsv < (long long)(Sq - 1) * ldv + Hkv * D)))
      return (int)hipErrorInvalidValue;
    fr.k = kn;
    fr.v = vn;
    fr.kc = const_cast<void*>(kc);
    fr.vc = const_cast<void*>(vc);
    fr.bsk = bsk;
    fr.bsv = bsv;
    fr.ldk = ldk;
    fr.ldv = ldv;
    fr.bf = nbf;
    fr.n = nfresh;
  }
  const int G = H / Hkv, chunk = MAXR / G;
  const int NS = (L + KC - 1) / KC;
  for (int q0 = 0; q0 < Sq; q0 += chunk) {
    const int sq = Sq - q0 < chunk ? Sq - q0 : chunk;
    const unsigned grid = (unsigned)(B * Hkv * NS);
    const unsigned rows = (unsigned)(B * Hkv * G * sq);
#define NOS_ATTN_DECODE(d, c)                                                                                   \
  hipLaunchKernelGGL((attn_decode_kernel<d, c>), dim3(grid), dim3(256), 0, stream, q, qbf, ldq, bsq, kc, vc, cbf, pos, \
                     cos_t, sin_t, R, static_cast<float*>(ws), B, H, Hkv, sq, q0, L, NS, scale, fr, sync, out, obf, Sq)
    if (D == 64) {
      if (cbf)
        NOS_ATTN_DECODE(64, 1);
      else
        NOS_ATTN_DECODE(64, 0);
      if (!sync && !partials_only)
        hipLaunchKernelGGL(attn_decode_combine_kernel<64>, dim3(rows), dim3(64), 0, stream,
                           static_cast<const float*>(ws), out, obf, B, H, Hkv, sq, q0, Sq, NS);
    } else {
      if (cbf)
        NOS_ATTN_DECODE(128, 1);
      else
        NOS_ATTN_DECODE(128, 0);
      if (!sync && !partials_only)
        hipLaunchKernelGGL(attn_decode_combine_kernel<128>, dim3(rows), dim3(128), 0, stream,
                           static_cast<const float*>(ws), out, obf, B, H, Hkv, sq, q0, Sq, NS);
    }
  }
  #undef NOS_ATTN_DECODE
  return (int)hipGetLastError();
}

NOS_API int nos_pos_update(int* pos, int B, int add, int n, hipStream_t stream) {
  if (!pos || B <= 0 || n < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(pos_update_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, stream, pos, B, add, n);
  return (int)hipGetLastError();
}

// pos (or null): pos[row] += pos_n after row's maximum (a decode step's
// position advance in the same launch; rows = the sequences)
NOS_API int nos_argmax(const void* x, int bf16, int rows, int L, int ldx, int* out, int* pos, int pos_n,
                       hipStream_t stream) {
  if (!x || !out || rows <= 0 || L <= 0 || ldx < L || (bf16 != 0 && bf16 != 1) || pos_n < 0)
    return (int)hipErrorInvalidValue;
  if (L >= 4096)
    hipLaunchKernelGGL(argmax_kernel<1024>, dim3((unsigned)rows), dim3(1024), 0, stream, x, bf16, rows, L, ldx, out,
                       pos, pos_n);
  else
    hipLaunchKernelGGL(argmax_kernel<256>, dim3((unsigned)rows), dim3(256), 0, stream, x, bf16, rows, L, ldx, out,
                       pos, pos_n);
  return (int)hipGetLastError();
}

// y [M, N] = act(rms(x) x [M, K] . W [N, K]^T + bias) + res, M <= 8; x, y, res
// share x's dtype (xbf), W and bias W's (wbf); K % 4 == 0, rows 16-byte
// (fp32) / 8-byte (bf16) aligned, M x K x 4 <= 64 KiB (the x rows in LDS).
// rms_eps > 0: each x row RMS-normalised first.  grid: up to 16 workgroups per CU
// walk the N / 8 column groups.
static int gemv_launch(const void* x, int xbf, int ldx, const void* w, int wbf, int ldw, const void* bias,
                       const void* res, int ldr, void* y, int ldy, int M, int N, int K, int epi, float rms_eps,
                       Parts pt, hipStream_t stream);

NOS_API int nos_gemv(const void* x, int xbf, int ldx, const void* w, int wbf, int ldw, const void* bias,
                     const void* res, int ldr, void* y, int ldy, int M, int N, int K, int epi, float rms_eps,
                     hipStream_t stream) {
  if (!x || !w || !y || M <= 0 || M > 8 || N <= 0 || K <= 0 || (K % 4) || ldx < K || ldw < K || ldy < ((epi & EPI_GLU) ? N / 2 : N) ||
      (long long)M * K * 4 > 65536 || (xbf != 0 && xbf != 1) || (wbf != 0 && wbf != 1) ||
      ((epi & EPI_BIAS) && !bias) || ((epi & EPI_RESID) && (!res || ldr < N)) || (ldx % 4) || (ldw % 4) ||
      ((uintptr_t)x & (xbf ? 7 : 15)) || ((uintptr_t)w & (wbf ? 7 : 15)))
    return (int)hipErrorInvalidValue;
  if ((epi & EPI_GLU) && ((N % 2) || (epi & (EPI_RESID | EPI_GELU | EPI_RELU | EPI_SILU)) || ldy < N / 2))
    return (int)hipErrorInvalidValue;
  return gemv_launch(x, xbf, ldx, w, wbf, ldw, bias, res, ldr, y, ldy, M, N, K, epi, rms_eps, Parts{}, stream);
}

// y [M, N] = act(x W^T + b) + R with x = the decode attention's split partials
// (nos_attn_decode with partials_only: ws [M x Hkv, NS, R = G, D + 2] fp32, one
// query token per sequence), combined in the GEMV's x staging: the combine launch
// folded into the O-projection.  ybf: y / R dtype; K = Hkv x G x D.
NOS_API int nos_gemv_partials(const float* ws, long long ws_n, int NS, int R, int G, int Hkv, int D, int ybf,
                              const void* w, int wbf, int ldw, const void* bias, const void* res, int ldr, void* y,
                              int ldy, int M, int N, int K, int epi, hipStream_t stream) {
  if (!ws || NS <= 0 || G <= 0 || Hkv <= 0 || (D != 64 && D != 128) || R != G || K != Hkv * G * D || !w || !y ||
      M <= 0 || M > 8 || N <= 0 || ws_n < (long long)M * Hkv * NS * R * (D + 2) || (long long)M * K * 4 > 65536 ||
      (ybf != 0 && ybf != 1) || (wbf != 0 && wbf != 1) || ((epi & EPI_BIAS) && !bias) ||
      ((epi & EPI_RESID) && (!res || ldr < N)) || ldy < N || (epi & EPI_GLU) || (ldw % 4) || ldw < K ||
      ((uintptr_t)w & (wbf ? 7 : 15)))
    return (int)hipErrorInvalidValue;
  Parts pt;
  pt.ws = ws;
  pt.NS = NS;
  pt.R = R;
  pt.G = G;
  pt.Hkv = Hkv;
  pt.D = D;
  return gemv_launch(nullptr, ybf, K, w, wbf, ldw, bias, res, ldr, y, ldy, M, N, K, epi, 0.f, pt, stream);
}

static int gemv_launch(const void* x, int xbf, int ldx, const void* w, int wbf, int ldw, const void* bias,
                       const void* res, int ldr, void* y, int ldy, int M, int N, int K, int epi, float rms_eps,
                       Parts pt, hipStream_t stream) {
  const int ngrp = (epi & EPI_GLU) ? (N / 2 + 3) / 4 : (N + 7) / 8;
  // every column group its own workgroup up to 16 per CU: a vocabulary head (4000 groups) no
  // longer walks 4 groups per workgroup one memory round trip after another
  const int cap = 16 * nos_effective_cus();
  const unsigned grid = (unsigned)(ngrp < cap ? ngrp : cap);
  const size_t lds = (size_t)M * K * 4;
#define NOS_GEMV_KU(m, b, ku)                                                                                         \
  hipLaunchKernelGGL((gemv_kernel<m, b, ku>), dim3(grid), dim3(256), lds, stream, x, xbf, ldx, w, wbf, ldw, bias, res, \
                     ldr, y, ldy, N, K, epi, rms_eps, pt)
#define NOS_GEMV(m)                                                                                                   \
  if (K > 1024) {                                                                                                     \
    if (wbf)                                                                                                          \
      NOS_GEMV_KU(m, 1, 12);                                                                                          \
    else                                                                                                              \
      NOS_GEMV_KU(m, 0, 12);                                                                                          \
  } else if (wbf) {                                                                                                   \
    NOS_GEMV_KU(m, 1, 4);                                                                                             \
  } else {                                                                                                            \
    NOS_GEMV_KU(m, 0, 4);                                                                                             \
  }
  switch (M) {
    case 1: NOS_GEMV(1); break;
    case 2: NOS_GEMV(2); break;
    case 3: NOS_GEMV(3); break;
    case 4: NOS_GEMV(4); break;
    case 5: NOS_GEMV(5); break;
    case 6: NOS_GEMV(6); break;
    case 7: NOS_GEMV(7); break;
    default: NOS_GEMV(8); break;
  }
#undef NOS_GEMV
#undef NOS_GEMV_KU
  return (int)hipGetLastError();
}
