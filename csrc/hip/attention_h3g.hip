// General fp32 attention on the fp16x3 ("h3") matrix pipes: the attention of
// tenant programs that are not ViT encoders -- decoder LLMs (causal, head_dim
// 128, grouped-query K/V heads, rotary position embeddings), and any
// head_dim-64 attention whose K / V are not the output of a fused LN-QKV GEMM.
//
//   O = softmax(scale Q K^T [+ causal mask]) V,   q / k / v fp32 [B, S, H(kv), D]
//
// Same numerics as the YOLOS h3 kernel (attention_f32x.hip; split_f16.h):
// every operand is two fp16 pieces on a power-of-two scale and every product
// the three piece products ah.bh + ah.bl + al.bh on v_mfma_f32_32x32x16_f16
// (22 of an fp32's 24 bits, fp32 accumulation), within the exact-f32
// kernel's error against fp64 (tests/test_tenant_ops_gpu.py).  What differs
// is where the K / V scales come from: here K / V are arbitrary activations,
// so a pre-pass measures them --
//
//  1. kv_absmax: max |k| and |v| per (batch, kv head) over row chunks;
//  2. kv_scale: the power of two that puts each head's max just under 2^14
//     (for rotated keys: the host's bound max|cos| + max|sin| on top);
//  3. split_kv: K (rotated on the fly) and V as four fp16 planes per token,
//     [b][kv head][token][K hi, K lo, V hi, V lo][D], 16-byte stores;
//  4. the attention: one workgroup = 8 waves x 32 query rows of one (batch,
//     head); 32-key tiles of the four planes arrive by LDS-DMA
//     (global_load_lds_dwordx4) into a 2-deep ring, each 64-dim half of a
//     plane as its own XOR-swizzled 4 KiB image (head_dim 128 = two halves
//     of the head_dim-64 layout); swapped S^T = K Q^T with Q's pieces (its
//     per-row scale and the softmax scale folded in, rotated on load) in
//     registers; P = exp2(S - m) split in registers and fed straight to
//     O^T = V^T P^T through ds_read_b64_tr_b16; deferred rescale (P <= 2^8);
//     causal tiles past a workgroup's last query are never loaded, the
//     diagonal tiles masked per lane, heavy (late) query blocks first;
//     grouped-query heads read their K / V head's planes (h * Hkv / H);
//     key splits (merged by merge_kernel) when the grid leaves CU slots idle;
//     slice-sized persistent grids under a CU budget (nos::xcd_chunk).
#include <float.h>
#include <limits.h>
#include <math.h>

#include "common.h"
#include "split_f16.h"

namespace {

constexpr int KVB = 32;                 // keys per tile
constexpr int IMG = KVB * 64 * 2;       // one 64-dim fp16 piece image: 32 rows x 128 B = 4 KiB
constexpr float RESCALE_THR = 8.f;      // log2 units
constexpr int MAX_SPLIT = 4;
constexpr int HW = 8;                   // waves per workgroup
constexpr int QB = 32 * HW;             // query rows per workgroup
constexpr int ABS_ROWS = 256;           // rows per absmax chunk

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

// LDS-DMA of 16 bytes per lane as inline asm (see attention_f32x.hip: the
// builtin makes hipcc drain in-flight tiles before every LDS read)
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds) : "memory");
}

// LDS-DMA from a wave-uniform tile base (SGPR pair) plus a per-lane 32-bit byte
// offset: the steady-state tiles need no 64-bit VALU address arithmetic
__device__ __forceinline__ void glds16_s(const void* sbase, unsigned voff, unsigned char* lds_wave_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(lds) : "memory");
}

__device__ __forceinline__ void dma_wait_publish() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// ---------------------------------------------------------------- 1. absmax
// part[(bh * nchunk + chunk) * 2 + (0: K, 1: V)] = max |x| over the chunk's rows
__global__ __launch_bounds__(256) void kv_absmax_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                        float* __restrict__ part, int S, int Hkv, int D, int ldk,
                                                        long long bsk, int ldv, long long bsv, int nchunk) {
  __shared__ float red[2][4];
  const int bh = blockIdx.y, chunk = blockIdx.x;
  const int b = bh / Hkv, h = bh - b * Hkv;
  const int r0 = chunk * ABS_ROWS, r1 = min(S, r0 + ABS_ROWS);
  const int d4 = D / 4;
  const int n = (r1 - r0) * d4;
  float mk = 0.f, mv = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int r = r0 + i / d4, c = (i % d4) * 4;
    const float4 a = *reinterpret_cast<const float4*>(k + b * bsk + (long long)r * ldk + h * D + c);
    const float4 e = *reinterpret_cast<const float4*>(v + b * bsv + (long long)r * ldv + h * D + c);
    mk = fmaxf(mk, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
    mv = fmaxf(mv, fmaxf(fmaxf(fabsf(e.x), fabsf(e.y)), fmaxf(fabsf(e.z), fabsf(e.w))));
  }
  mk = nos::wave_max(mk);
  mv = nos::wave_max(mv);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mk;
    red[1][threadIdx.x >> 6] = mv;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const float* r = red[threadIdx.x];
    part[((long long)bh * nchunk + chunk) * 2 + threadIdx.x] = fmaxf(fmaxf(r[0], r[1]), fmaxf(r[2], r[3]));
  }
}

// ---------------------------------------------------------------- 2. scales
// kvsc[bh * 2 + t] = 2^e with (max_t * bound_t) 2^e < 2^14 (bound: K's rotary growth)
__global__ __launch_bounds__(256) void kv_scale_kernel(const float* __restrict__ part, float* __restrict__ kvsc,
                                                       int n, int nchunk, float kbound) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int bh = i >> 1, t = i & 1;
  float m = 0.f;
  for (int c = 0; c < nchunk; ++c) m = fmaxf(m, part[((long long)bh * nchunk + c) * 2 + t]);
  kvsc[i] = nos::pow2i(nos::h3_scale_exp(t == 0 ? m * kbound : m));
}

// ---------------------------------------------------------------- 3. split
// one thread: 8 dims of one (b, kv head, token, K|V): planes
// kvs[(bh * skvp + s) * 4 + 2t + piece][D]; K rotated first when cos != null
// (rows of the [Skv][D] tables = key positions)
__global__ __launch_bounds__(256) void split_kv_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                       const float* __restrict__ kvsc, _Float16* __restrict__ kvs,
                                                       int S, int skvp, int Hkv, int D, int ldk, long long bsk,
                                                       int ldv, long long bsv, const float* __restrict__ rc,
                                                       const float* __restrict__ rs, long long n8) {
  typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const int c8 = D / 8;
  const int ch = (int)(i % c8);
  long long rest = i / c8;
  const int t = (int)(rest & 1);
  rest >>= 1;
  const int s = (int)(rest % S);
  const int bh = (int)(rest / S);
  const int b = bh / Hkv, h = bh - b * Hkv;
  const float* src = t == 0 ? k + b * bsk + (long long)s * ldk + h * D : v + b * bsv + (long long)s * ldv + h * D;
  float x[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(src + ch * 8);
    const float4 e = *reinterpret_cast<const float4*>(src + ch * 8 + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = e.x; x[5] = e.y; x[6] = e.z; x[7] = e.w;
  }
  if (t == 0 && rc != nullptr) {  // rotate_half: partner chunk D/16 away
    const int half = c8 / 2;
    const bool lo = ch < half;
    const int pc = lo ? ch + half : ch - half;
    const float4 a = *reinterpret_cast<const float4*>(src + pc * 8);
    const float4 e = *reinterpret_cast<const float4*>(src + pc * 8 + 4);
    const float p[8] = {a.x, a.y, a.z, a.w, e.x, e.y, e.z, e.w};
    const float* cr = rc + (long long)s * D + ch * 8;
    const float* sr = rs + (long long)s * D + ch * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = lo ? fmaf(x[j], cr[j], -p[j] * sr[j]) : fmaf(x[j], cr[j], p[j] * sr[j]);
  }
  const float sc = kvsc[bh * 2 + t];
  f16x8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    f16x2_t h2, l2;
    nos::split2h(f32x2_t{x[j] * sc, x[j + 1] * sc}, h2, l2);
    hi[j] = h2.x; hi[j + 1] = h2.y;
    lo[j] = l2.x; lo[j + 1] = l2.y;
  }
  _Float16* dst = kvs + (((long long)bh * skvp + s) * 4 + 2 * t) * D + ch * 8;
  *reinterpret_cast<f16x8*>(dst) = hi;
  *reinterpret_cast<f16x8*>(dst + D) = lo;
}

// ---------------------------------------------------------------- 4. attention
template <int D, bool CAUSAL, bool ROPE, bool PERSIST>
__global__ __launch_bounds__(64 * HW, D == 64 ? 2 : 1) void attn_h3g_kernel(
    const float* __restrict__ q, int ldq, long long bsq, const _Float16* __restrict__ kvs,
    const float* __restrict__ kvsc, float* __restrict__ o, int ldo, long long bso, int B, int H, int Hkv, int Sq,
    int Skv, float c, int nqb, int nsplit, float* __restrict__ part, const float* __restrict__ rc,
    const float* __restrict__ rs) {
  constexpr int NH = D / 64;                 // 64-dim halves
  constexpr int NKS = D / 16;                // 16-deep MFMA steps over D
  constexpr int STAGE = 4 * NH * IMG;
  constexpr int PPW = 16 * NH / HW;          // 1 KiB DMA pieces per wave per tile
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
  const int off = Skv - Sq;  // query i sees keys <= i + off (causal; 0 for self-attention)
  int soff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = wid * PPW + i;
    const int img = p >> 2, plane = img / NH, half = img % NH;
    const int row = (p & 3) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (plane < 2 ? kswz(row) : vswz(row));
    soff[i] = (row * 4 + plane) * D + half * 64 + lc * 8;
  }

  for (int w = chunk.first; w < chunk.end; w += chunk.step) {
    if (PERSIST && w != chunk.first) __syncthreads();
    const int sp = w % nsplit;
    const int wq = w / nsplit;
    const int b = wq / (H * nqb);
    const int rem = wq - b * (H * nqb);
    const int h = rem / nqb;
    const int qb = CAUSAL ? nqb - 1 - (rem - h * nqb) : rem - h * nqb;  // causal: the longest rows first
    const int hk = h / (H / Hkv);
    const int q0 = qb * QB;
    const int nt_item = CAUSAL ? min(ntiles, (min(q0 + QB, Sq) - 1 + off) / KVB + 1) : ntiles;
    const int tps = (nt_item + nsplit - 1) / nsplit;
    const int t0 = sp * tps, t1 = min(nt_item, t0 + tps);
    const float ksc = kvsc[(b * Hkv + hk) * 2], vinv = 1.f / kvsc[(b * Hkv + hk) * 2 + 1];

    // ---- Q pieces: lane holds Q[row][16 ks + 8 hh .. +7] * c * 2^e (rotated first)
    const int qrow = q0 + wid * 32 + r;
    const int qr = min(qrow, Sq - 1);
    f16x8_t qf[NKS][2];
    float fs;
    {
      const float* qp = q + b * bsq + (long long)qr * ldq + h * D + 8 * hh;
      float x[NKS][8];
      float mx = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const float4 x0 = *reinterpret_cast<const float4*>(qp + 16 * ks);
        const float4 x1 = *reinterpret_cast<const float4*>(qp + 16 * ks + 4);
        x[ks][0] = x0.x; x[ks][1] = x0.y; x[ks][2] = x0.z; x[ks][3] = x0.w;
        x[ks][4] = x1.x; x[ks][5] = x1.y; x[ks][6] = x1.z; x[ks][7] = x1.w;
      }
      if constexpr (ROPE) {  // partner dims d +- D/2 are ks +- NKS/2 of this same lane
        const float* cr = rc + (long long)(qr + off) * D + 8 * hh;
        const float* sr = rs + (long long)(qr + off) * D + 8 * hh;
        float y[NKS][8];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float cv = cr[16 * ks + j], sv = sr[16 * ks + j];
            y[ks][j] = ks < NKS / 2 ? fmaf(x[ks][j], cv, -x[ks + NKS / 2][j] * sv)
                                    : fmaf(x[ks][j], cv, x[ks - NKS / 2][j] * sv);
          }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) x[ks][j] = y[ks][j];
      }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(x[ks][j]));
      const int e = nos::h3_scale_exp(xor32_max(mx) * c);
      const float qm = c * nos::pow2i(e);
      fs = nos::pow2i(-e) / ksc;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          f16x2_t hi, lo;
          nos::split2h(f32x2_t{x[ks][j] * qm, x[ks][j + 1] * qm}, hi, lo);
          qf[ks][0][j] = hi.x; qf[ks][0][j + 1] = hi.y;
          qf[ks][1][j] = lo.x; qf[ks][1][j + 1] = lo.y;
        }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int p = 0; p < 2; ++p) asm volatile("" : "+v"(qf[ks][p]));
    }

    const _Float16* pb = kvs + (long long)(b * Hkv + hk) * skvp * 4 * D;
    auto stage_piece = [&](int t, int buf, int i) {
      const int p = wid * PPW + i;
      long long o2 = (long long)t * (KVB * 4) * D + soff[i];
      if ((t + 1) * KVB > Skv) {  // tail tile: rows past Skv re-read the last key (masked)
        const int over = t * KVB + (p & 3) * 8 + (lane >> 3) - (Skv - 1);
        if (over > 0) o2 -= (long long)over * 4 * D;
      }
      glds16(pb + o2, smem + buf * STAGE + (p >> 2) * IMG + (p & 3) * 8 * 128);
    };
    auto stage_full = [&](int t, int buf, int i) {  // full tiles: uniform base + per-lane byte offset
      const int p = wid * PPW + i;
      glds16_s(pb + (long long)t * (KVB * 4) * D, (unsigned)soff[i] * 2u,
               smem + buf * STAGE + (p >> 2) * IMG + (p & 3) * 8 * 128);
    };

    f32x16_t oacc[2 * NH];
#pragma unroll
    for (int db = 0; db < 2 * NH; ++db)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[db][i] = 0.f;
    float m = 0.f, l = 0.f;

    if (t0 < t1) {
#pragma unroll
      for (int i = 0; i < PPW; ++i) stage_piece(t0, 0, i);
      dma_wait_publish();
    }
    const int qw0 = q0 + wid * 32;  // this wave's first query row (wave-uniform mask test)
    for (int t = t0; t < t1; ++t) {
      const int buf = (t - t0) & 1;
      if (t + 1 < t1) {
        if ((t + 2) * KVB <= Skv) {
#pragma unroll
          for (int i = 0; i < PPW; ++i) stage_full(t + 1, buf ^ 1, i);
        } else {
#pragma unroll
          for (int i = 0; i < PPW; ++i) stage_piece(t + 1, buf ^ 1, i);
        }
      }
      const unsigned char* st = smem + buf * STAGE;

      f32x16_t s;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = 0.f;
#pragma unroll
      for (int hf = 0; hf < NH; ++hf)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          f16x8_t a[2];
#pragma unroll
          for (int pc = 0; pc < 2; ++pc)
            a[pc] = *reinterpret_cast<const f16x8_t*>(st + (pc * NH + hf) * IMG + koff[ks]);
          s = nos::mma3h(a, qf[hf * 4 + ks], s);
        }
      if ((t + 1) * KVB > Skv) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (t * KVB + (i & 3) + 8 * (i >> 2) + 4 * hh >= Skv) s[i] = -INFINITY;
      }
      if (CAUSAL && t * KVB + KVB - 1 > qw0 + off) {  // a diagonal tile of this wave
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (t * KVB + (i & 3) + 8 * (i >> 2) + 4 * hh > qrow + off) s[i] = -INFINITY;
      }
      float mt = s[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mt = fmaxf(mt, s[i]);
      // a fully masked row (causal; a split of early keys) keeps a finite
      // reference -1e30; the new reference is set directly (m + delta would
      // lose a real maximum against 1e30 and break P <= 2^8)
      const float mnew = fmaxf(xor32_max(mt) * fs, -1e30f);
      if (t == t0) {
        m = mnew;
      } else if (!__all(mnew - m <= RESCALE_THR)) {
        const float mref = fmaxf(mnew, m);
        const float alpha = __builtin_amdgcn_exp2f(m - mref);
        m = mref;
        l *= alpha;
#pragma unroll
        for (int db = 0; db < 2 * NH; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) oacc[db][i] *= alpha;
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
      for (int db = 0; db < 2 * NH; ++db)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          f16x8_t a[2];
#pragma unroll
          for (int pc = 0; pc < 2; ++pc) {
            const unsigned char* base = st + ((2 + pc) * NH + (db >> 1)) * IMG + voff[db & 1] + s2 * 16 * 128;
            const s16x4_t lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base));
            const s16x4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + 8 * 128));
            const s16x8_t a16 = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            a[pc] = __builtin_bit_cast(f16x8_t, a16);
          }
          oacc[db] = nos::mma3h(a, pf[s2], oacc[db]);
        }
      dma_wait_publish();
    }

    const float lt = xor32_sum(l);
    const int ldh = H * D;
    if (nsplit > 1) {  // unnormalised partial (O on the unit scale, m, l) of this key range
      if (qrow < Sq) {
        const long long row = ((long long)sp * B + b) * Sq + qrow;
        float* op = part + row * ldh + h * D;
#pragma unroll
        for (int db = 0; db < 2 * NH; ++db)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(op + 32 * db + 8 * g + 4 * hh) =
                float4{oacc[db][4 * g + 0] * vinv, oacc[db][4 * g + 1] * vinv, oacc[db][4 * g + 2] * vinv,
                       oacc[db][4 * g + 3] * vinv};
        if (hh == 0) {
          float* ml = part + (long long)nsplit * B * Sq * ldh + (row * H + h) * 2;
          ml[0] = t0 < t1 ? m : -1e30f;
          ml[1] = lt;
        }
      }
      continue;
    }
    const float inv = vinv / lt;
    if (qrow < Sq) {
      float* op = o + b * bso + (long long)qrow * ldo + h * D;
#pragma unroll
      for (int db = 0; db < 2 * NH; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(op + 32 * db + 8 * g + 4 * hh) =
              float4{oacc[db][4 * g + 0] * inv, oacc[db][4 * g + 1] * inv, oacc[db][4 * g + 2] * inv,
                     oacc[db][4 * g + 3] * inv};
    }
  }  // items
}

// key-split merge: O = sum_i O_i 2^(m_i - M) / sum_i l_i 2^(m_i - M)
__global__ __launch_bounds__(256) void merge_kernel(const float* __restrict__ part, float* __restrict__ o, int B,
                                                    int H, int D, int Sq, int nsplit, int ldo, long long bso,
                                                    long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int ldh = H * D;
  const long long row = i / (ldh / 4);
  const int col = (int)(i - row * (ldh / 4)) * 4;
  const int h = col / D;
  const long long per_split = (long long)B * Sq;
  const float* ml = part + (long long)nsplit * per_split * ldh;
  float mx = -INFINITY;
  for (int sp = 0; sp < nsplit; ++sp) mx = fmaxf(mx, ml[((sp * per_split + row) * H + h) * 2]);
  float L = 0.f;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < nsplit; ++sp) {
    const long long r = sp * per_split + row;
    const float a = __builtin_amdgcn_exp2f(ml[(r * H + h) * 2] - mx);
    L = fmaf(ml[(r * H + h) * 2 + 1], a, L);
    const float4 v = *reinterpret_cast<const float4*>(part + r * ldh + col);
    acc.x = fmaf(v.x, a, acc.x);
    acc.y = fmaf(v.y, a, acc.y);
    acc.z = fmaf(v.z, a, acc.z);
    acc.w = fmaf(v.w, a, acc.w);
  }
  const float inv = 1.f / L;
  const long long b = row / Sq, s = row - b * Sq;
  *reinterpret_cast<float4*>(o + b * bso + s * ldo + col) = float4{acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
}

struct Layout {
  long long planes, absmax, scales, part, total;
  int nchunk, skvp;
};

Layout layout(int B, int H, int Hkv, int Sq, int Skv, int D) {
  Layout L;
  L.skvp = (Skv + KVB - 1) / KVB * KVB;
  L.nchunk = (Skv + ABS_ROWS - 1) / ABS_ROWS;
  auto al = [](long long x) { return (x + 255) / 256 * 256; };
  L.planes = 0;
  L.absmax = al((long long)B * Hkv * L.skvp * 4 * D * 2);
  L.scales = L.absmax + al((long long)B * Hkv * L.nchunk * 2 * 4);
  L.part = L.scales + al((long long)B * Hkv * 2 * 4);
  L.total = L.part + (long long)MAX_SPLIT * B * Sq * H * (D + 2) * 4;
  return L;
}

int g_kvsplit = 0;  // 0: auto

int pick_split(long long nwg1, int ntiles, int wg_per_cu) {
  int n = g_kvsplit;
  if (n == 0) {
    const long long slots = (long long)wg_per_cu * nos_effective_cus();
    n = nwg1 >= slots ? 1 : (int)(slots / nwg1);
  }
  n = n < 1 ? 1 : (n > MAX_SPLIT ? MAX_SPLIT : n);
  while (n > 1 && (long long)(n - 1) * ((ntiles + n - 1) / n) >= ntiles) --n;
  return n;
}

template <int D, bool CAUSAL, bool ROPE>
int launch(const float* q, int ldq, long long bsq, const _Float16* kvs, const float* kvsc, float* o, int ldo,
           long long bso, int B, int H, int Hkv, int Sq, int Skv, float c, int nqb, int nsplit, float* part,
           const float* rc, const float* rs, hipStream_t stream) {
  constexpr int lds = 2 * 4 * (D / 64) * IMG;
  const long long nwg = (long long)B * H * nqb * nsplit;
  const int grid = nos_grid_for((const void*)attn_h3g_kernel<D, CAUSAL, ROPE, true>, 64 * HW, lds, nwg);
  if (grid < nwg)
    hipLaunchKernelGGL((attn_h3g_kernel<D, CAUSAL, ROPE, true>), dim3((unsigned)grid), dim3(64 * HW), lds, stream, q,
                       ldq, bsq, kvs, kvsc, o, ldo, bso, B, H, Hkv, Sq, Skv, c, nqb, nsplit, part, rc, rs);
  else
    hipLaunchKernelGGL((attn_h3g_kernel<D, CAUSAL, ROPE, false>), dim3((unsigned)nwg), dim3(64 * HW), lds, stream,
                       q, ldq, bsq, kvs, kvsc, o, ldo, bso, B, H, Hkv, Sq, Skv, c, nqb, nsplit, part, rc, rs);
  return (int)hipGetLastError();
}

}  // namespace

// Workspace bytes of nos_attn_h3g (K / V planes, scales, key-split partials).
NOS_API long long nos_attn_h3g_workspace(int B, int H, int Hkv, int Sq, int Skv, int D) {
  if (B <= 0 || H <= 0 || Hkv <= 0 || Sq <= 0 || Skv <= 0 || (D != 64 && D != 128)) return -1;
  return layout(B, H, Hkv, Sq, Skv, D).total;
}

NOS_API int nos_attn_h3g_set_kvsplit(int n) {
  if (n < 0 || n > MAX_SPLIT) return (int)hipErrorInvalidValue;
  g_kvsplit = n;
  return 0;
}

// O = softmax(scale Q K^T [causal]) V for fp32 q [B, Sq, H, D], k / v
// [B, Skv, Hkv, D] (token row strides ld*, batch strides bs*, each head's D
// dims contiguous; H % Hkv == 0: grouped-query heads) into o [B, Sq, H, D]
// (ldo, bso).  D = 64 or 128.  causal: query i attends keys <= i + Skv - Sq.
// rope_cos / rope_sin (fp32 [Skv][D], or null): rotate Q (rows i + Skv - Sq)
// and K (rows = key positions) by rotate_half first; rope_bound >=
// max |cos| + max |sin| of the tables (bounds the rotated keys).  ws: at
// least nos_attn_h3g_workspace() bytes, 256-byte aligned.
NOS_API int nos_attn_h3g(const float* q, int ldq, long long bsq, const float* k, int ldk, long long bsk,
                         const float* v, int ldv, long long bsv, float* o, int ldo, long long bso, int B, int H, int Hkv,
                         int Sq, int Skv, int D, int causal, float scale, const float* rope_cos, const float* rope_sin,
                         float rope_bound, void* ws, long long ws_bytes, hipStream_t stream) {
  if (B <= 0 || H <= 0 || Hkv <= 0 || H % Hkv || Sq <= 0 || Skv <= 0 || (D != 64 && D != 128) || !(scale > 0.f))
    return (int)hipErrorInvalidValue;
  if (causal && Sq > Skv) return (int)hipErrorInvalidValue;
  if (ldq < H * D || ldo < H * D || ldk < Hkv * D || ldv < Hkv * D) return (int)hipErrorInvalidValue;
  if ((ldq | ldk | ldv | ldo) & 3 || (bsq | bsk | bsv | bso) & 3) return (int)hipErrorInvalidValue;
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15 || ((uintptr_t)ws) & 255)
    return (int)hipErrorInvalidValue;
  if ((rope_cos == nullptr) != (rope_sin == nullptr) || (rope_cos && !(rope_bound > 0.f)))
    return (int)hipErrorInvalidValue;
  const Layout L = layout(B, H, Hkv, Sq, Skv, D);
  if (ws == nullptr || ws_bytes < L.total) return (int)hipErrorInvalidValue;
  if ((long long)B * H * ((Sq + QB - 1) / QB) * MAX_SPLIT > (1LL << 30) || (long long)B * Hkv * L.skvp * 4 * D > INT_MAX * 8LL)
    return (int)hipErrorInvalidValue;
  auto* base = static_cast<unsigned char*>(ws);
  auto* kvs = reinterpret_cast<_Float16*>(base + L.planes);
  auto* absmax = reinterpret_cast<float*>(base + L.absmax);
  auto* kvsc = reinterpret_cast<float*>(base + L.scales);
  auto* part = reinterpret_cast<float*>(base + L.part);
  const int nbh = B * Hkv;
  hipLaunchKernelGGL(kv_absmax_kernel, dim3((unsigned)L.nchunk, (unsigned)nbh), dim3(256), 0, stream, k, v, absmax,
                     Skv, Hkv, D, ldk, bsk, ldv, bsv, L.nchunk);
  hipLaunchKernelGGL(kv_scale_kernel, dim3((unsigned)((2 * nbh + 255) / 256)), dim3(256), 0, stream, absmax, kvsc,
                     2 * nbh, L.nchunk, rope_cos ? rope_bound : 1.f);
  const long long n8 = (long long)nbh * Skv * 2 * (D / 8);
  hipLaunchKernelGGL(split_kv_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, stream, k, v, kvsc, kvs, Skv,
                     L.skvp, Hkv, D, ldk, bsk, ldv, bsv, rope_cos, rope_sin, n8);
  if (int rc = (int)hipGetLastError()) return rc;
  const float c = scale * 1.4426950408889634f;
  const int nqb = (Sq + QB - 1) / QB;
  const long long nwg1 = (long long)B * H * nqb;
  const int nsplit = pick_split(nwg1, L.skvp / KVB, D == 64 ? 2 : 1);
  int rc;
  const bool rope = rope_cos != nullptr;
#define NOS_H3G(d, cz, rp)                                                                                          \
  rc = launch<d, cz, rp>(q, ldq, bsq, kvs, kvsc, o, ldo, bso, B, H, Hkv, Sq, Skv, c, nqb, nsplit, part, rope_cos, \
                         rope_sin, stream)
  if (D == 64) {
    if (causal) {
      if (rope) NOS_H3G(64, true, true); else NOS_H3G(64, true, false);
    } else {
      if (rope) NOS_H3G(64, false, true); else NOS_H3G(64, false, false);
    }
  } else {
    if (causal) {
      if (rope) NOS_H3G(128, true, true); else NOS_H3G(128, true, false);
    } else {
      if (rope) NOS_H3G(128, false, true); else NOS_H3G(128, false, false);
    }
  }
#undef NOS_H3G
  if (rc != 0 || nsplit == 1) return rc;
  const long long n4 = (long long)B * Sq * H * (D / 4);
  hipLaunchKernelGGL(merge_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, stream, part, o, B, H, D, Sq,
                     nsplit, ldo, bso, n4);
  return (int)hipGetLastError();
}
