// Fused multi-head self-attention forward (flash-style, non-causal) for the
// YOLOS-family tenant model, bf16 in / bf16 out, fp32 softmax, head_dim 64.
//
// CDNA4 design (not a port of any CUDA kernel):
//  * one workgroup = 8 waves = 128 query rows of one (batch, head), split in
//    two wave groups that walk interleaved 64-key tiles of the same K/V
//    stream (group 0: even tiles, group 1: odd tiles); the groups' partial
//    (m, l, O) are merged through LDS at the end.  One workgroup per CU, two
//    waves per SIMD, up to 256 registers per wave;
//  * software pipeline inside each wave: while the VALU computes the softmax
//    of tile j, the matrix pipe runs O += P(j-1) V(j-1) and S(j+1) = K(j+1) Q^T
//    -- the three steps are independent, so MFMA and VALU work of the SAME
//    wave overlap (for head_dim 64 the exp/max/sum work per score is about
//    as long as the MFMA work per score, so serialising them halves speed);
//  * "swapped" QK^T: S^T = K . Q^T, so every lane holds 16 of the 32 key
//    scores of ONE query row (column = lane & 31): row max / sum are
//    lane-local plus one v_permlane32_swap;
//  * V^T fragments come from a row-major, XOR-swizzled V tile through the
//    gfx950 transposing LDS read ds_read_b64_tr_b16; K is read with
//    ds_read_b128 from an XOR-swizzled image (both conflict-free).  Both are
//    issued as inline asm with explicit lgkmcnt waits: the compiler's own
//    waits serialised the K reads with the MFMAs and waited for in-flight
//    LDS-DMA before every V read;
//  * K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4) into 3-deep rings
//    (K and V separately, 96 KiB), issued two iterations ahead; a counted
//    s_waitcnt vmcnt + raw s_barrier closes each iteration;
//  * deferred rescale (T13): O and l are only rescaled when some row's max
//    grows by more than 8 (log2 units).  The rare rescale path first folds
//    the pending P(j-1) V(j-1) into O (and zeroes P(j-1)) so the main block
//    stays branch-free;
//  * XCD-aware workgroup -> (batch, head, q-block) map: q-blocks of one
//    head share an XCD's L2.
#include "common.h"

namespace {

constexpr int D = 64;
constexpr int QBLK = 128;           // query rows per workgroup (4 waves x 32)
constexpr int KVBLK = 64;           // keys per tile
constexpr int NT = 512;             // 8 waves
constexpr int TILE_BYTES = KVBLK * D * 2;   // 8 KiB
constexpr int PAIR_BYTES = 2 * TILE_BYTES;  // tiles 2p (group 0) and 2p+1 (group 1)
constexpr int NSLOT = 3;                    // ring depth
constexpr int V_OFF = NSLOT * PAIR_BYTES;   // V ring after the K ring
constexpr int LDS_BYTES = 2 * NSLOT * PAIR_BYTES;  // 96 KiB
constexpr float RESCALE_THR = 8.f;          // log2 units

typedef __attribute__((ext_vector_type(4))) int i32x4_t;

__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int vswz(int row) { return ((row >> 1) & 1) << 2; }

__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
template <int OFF>
__device__ __forceinline__ i32x4_t ds_b128(unsigned a) {
  i32x4_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ s16x4_t ds_tr16(unsigned a) {
  s16x4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0)

struct KFrag { i32x4_t k[2][4]; };        // [kb][ks]
struct VFrag { s16x4_t lo[2][2][2], hi[2][2][2]; };  // [db][kb][s2]

__device__ __forceinline__ void read_k(KFrag& f, unsigned kbase, const int (&koff)[4]) {
  const unsigned a0 = kbase + koff[0], a1 = kbase + koff[1], a2 = kbase + koff[2], a3 = kbase + koff[3];
  f.k[0][0] = ds_b128<0>(a0); f.k[0][1] = ds_b128<0>(a1); f.k[0][2] = ds_b128<0>(a2); f.k[0][3] = ds_b128<0>(a3);
  f.k[1][0] = ds_b128<4096>(a0); f.k[1][1] = ds_b128<4096>(a1);
  f.k[1][2] = ds_b128<4096>(a2); f.k[1][3] = ds_b128<4096>(a3);
}

__device__ __forceinline__ void read_v(VFrag& f, unsigned vbase, const int (&voff)[2]) {
#define TRP(DB, KB, S2, A)                                                \
  f.lo[DB][KB][S2] = ds_tr16<(KB * 32 + S2 * 16) * 128>(A);               \
  f.hi[DB][KB][S2] = ds_tr16<(KB * 32 + S2 * 16 + 8) * 128>(A);
  const unsigned a0 = vbase + voff[0], a1 = vbase + voff[1];
  TRP(0, 0, 0, a0) TRP(0, 0, 1, a0) TRP(0, 1, 0, a0) TRP(0, 1, 1, a0)
  TRP(1, 0, 0, a1) TRP(1, 0, 1, a1) TRP(1, 1, 0, a1) TRP(1, 1, 1, a1)
#undef TRP
}

// wait until at most N LDS reads are outstanding; ties the fragment registers
// so no consumer is scheduled above the wait
template <int N>
__device__ __forceinline__ void wait_k(KFrag& f) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f.k[0][0]), "+v"(f.k[0][1]), "+v"(f.k[0][2]), "+v"(f.k[0][3]), "+v"(f.k[1][0]),
                 "+v"(f.k[1][1]), "+v"(f.k[1][2]), "+v"(f.k[1][3])
               : "i"(N));
}
template <int N>
__device__ __forceinline__ void wait_v(VFrag& f) {
  asm volatile("s_waitcnt lgkmcnt(%16)"
               : "+v"(f.lo[0][0][0]), "+v"(f.lo[0][0][1]), "+v"(f.lo[0][1][0]), "+v"(f.lo[0][1][1]),
                 "+v"(f.lo[1][0][0]), "+v"(f.lo[1][0][1]), "+v"(f.lo[1][1][0]), "+v"(f.lo[1][1][1]),
                 "+v"(f.hi[0][0][0]), "+v"(f.hi[0][0][1]), "+v"(f.hi[0][1][0]), "+v"(f.hi[0][1][1]),
                 "+v"(f.hi[1][0][0]), "+v"(f.hi[1][0][1]), "+v"(f.hi[1][1][0]), "+v"(f.hi[1][1][1])
               : "i"(N));
}

__device__ __forceinline__ bf16x8_t vcat(s16x4_t lo, s16x4_t hi) {
  const s16x8_t a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, a);
}

__device__ __forceinline__ void qk(f32x16_t (&s)[2], const KFrag& f, const bf16x8_t (&qf)[4]) {
  const f32x16_t zero = {};
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    s[kb] = MFMA(__builtin_bit_cast(bf16x8_t, f.k[kb][0]), qf[0], zero);
#pragma unroll
    for (int ks = 1; ks < 4; ++ks) s[kb] = MFMA(__builtin_bit_cast(bf16x8_t, f.k[kb][ks]), qf[ks], s[kb]);
  }
}

__device__ __forceinline__ void pv(f32x16_t (&o)[2], const VFrag& f, const bf16x8_t (&pf)[2][2]) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < 2; ++db) o[db] = MFMA(vcat(f.lo[db][kb][s2], f.hi[db][kb][s2]), pf[kb][s2], o[db]);
}

__global__ __launch_bounds__(NT, 1) void attn_fwd_d64_kernel(
    const unsigned short* __restrict__ q, const unsigned short* __restrict__ k,
    const unsigned short* __restrict__ v, unsigned short* __restrict__ o, int B, int H, int Sq, int Skv,
    int ld_in, long long bs_in, int ld_out, long long bs_out, float c /* scale * log2(e) */, int nqb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = B * H * nqb;
  const int w = nos::xcd_remap(blockIdx.x, nwg);
  const int b = w / (H * nqb);
  const int rem = w - b * (H * nqb);
  const int h = rem / nqb;
  const int qb = rem - h * nqb;

  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR branches
  const int grp = wid >> 2;     // wave group: 0 even tiles, 1 odd tiles
  const int wq = wid & 3;       // query slice of the wave
  const int lane = tid & 63;
  const int r = lane & 31;
  const int hh = lane >> 5;

  const unsigned short* qb_ptr = q + b * bs_in + h * D;
  const unsigned short* kb_ptr = k + b * bs_in + h * D;
  const unsigned short* vb_ptr = v + b * bs_in + h * D;

  // ---- Q fragments (B operand): lane holds Q[row r][d = 16ks + 8hh .. +7]
  const int qrow = qb * QBLK + wq * 32 + r;
  const int qrow_c = qrow < Sq ? qrow : Sq - 1;
  bf16x8_t qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8_t*>(qb_ptr + (long long)qrow_c * ld_in + ks * 16 + hh * 8);

  // ---- LDS-DMA staging of one pair (tiles 2p, 2p+1) of K or V: 16 x 1 KiB
  // pieces, 2 per wave.  Lane L writes row R + L/8, physical chunk L%8 =
  // logical chunk ^ swizzle (swizzle applied to the source address).
  const unsigned char* src_base[2] = {(const unsigned char*)kb_ptr, (const unsigned char*)vb_ptr};
  auto stage = [&](int is_v, int p) {
    const int slot = p % NSLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = wid * 2 + i;     // 0..15
      const int g = piece >> 3;          // tile of the pair
      const int R = (piece & 7) * 8;     // row block in the tile
      const int row = R + (lane >> 3);
      const int pc = lane & 7;
      const int lc = pc ^ (is_v ? vswz(row) : kswz(row));
      int kv = (2 * p + g) * KVBLK + row;
      kv = kv < Skv ? kv : Skv - 1;
      const unsigned char* src = src_base[is_v] + ((long long)kv * ld_in + lc * 8) * 2;
      unsigned char* dst = smem + is_v * V_OFF + slot * PAIR_BYTES + g * TILE_BYTES + R * 128;
      glds16(src, dst);
    }
  };

  const int ntiles = (Skv + KVBLK - 1) / KVBLK;
  const int niters = (ntiles + 1) / 2;   // pairs

  // prologue: K pairs 0..2, V pair 0
  stage(0, 0);
  stage(0, 1);
  stage(0, 2);
  stage(1, 0);

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

  const unsigned lds0 = lds_u32(smem);
  const unsigned kgrp = lds0 + grp * TILE_BYTES;
  const unsigned vgrp = lds0 + V_OFF + grp * TILE_BYTES;

  f32x16_t oacc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; }
  bf16x8_t pprev[2][2];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) pprev[kb][s2][j] = (__bf16)0.f;
  float m = 0.f, l = 0.f;

  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  // prologue QK of this group's first tile (pair 0)
  f32x16_t sacc[2];
  {
    KFrag kf;
    read_k(kf, kgrp, koff);
    wait_k<0>(kf);
    qk(sacc, kf, qf);
  }
  // every wave is done reading pair 0 before iteration 0 restages its slot
  asm volatile("s_barrier" ::: "memory");

  for (int it = 0; it < niters; ++it) {
    // prefetch two iterations ahead (slots freed by the barrier that ended it-1)
    stage(0, it + 3);
    stage(1, it + 1);

    const int t = 2 * it + grp;               // tile whose softmax runs now
    const bool valid = t < ntiles;
    // fragments: K of this group's next tile (pair it+1), V of its previous tile (pair it-1)
    KFrag kf;
    VFrag vf;
    read_k(kf, kgrp + ((it + 1) % NSLOT) * PAIR_BYTES, koff);
    read_v(vf, vgrp + ((it + NSLOT - 1) % NSLOT) * PAIR_BYTES * (it > 0), voff);

    if (!valid || (t + 1) * KVBLK > Skv) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kv = t * KVBLK + kb * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
          if (kv >= Skv) sacc[kb][i] = -INFINITY;
        }
    }
    float mt = sacc[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mt = fmaxf(mt, sacc[0][i]);
#pragma unroll
    for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sacc[1][i]);
    const float mrel = fmaf(xor32_max(mt), c, -m);  // tile max - m (log2 units)
    const bool first = it == 0 && valid;
    if (first || !__all(mrel <= RESCALE_THR)) {
      // rare: fold the pending P(j-1) V(j-1) into O at the old scale, then rescale
      wait_v<0>(vf);
      pv(oacc, vf, pprev);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 8; ++j) pprev[kb][s2][j] = (__bf16)0.f;
      const float delta = first ? mrel : fmaxf(mrel, 0.f);
      const float alpha = __builtin_amdgcn_exp2f(-delta);
      m += delta;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        oacc[0][i] *= alpha;
        oacc[1][i] *= alpha;
      }
    }

    // main block: softmax(t) on the VALU || PV(t-2) and QK(t+2) on the matrix pipe
    wait_k<15>(kf);  // lgkmcnt is 4 bits: <= 15 outstanding covers the 8 K reads (issued before 16 V reads)
    f32x16_t snext[2];
    qk(snext, kf, qf);
    float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[0][i], c, -m));
      const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[1][i], c, -m));
      sacc[0][i] = p0;
      sacc[1][i] = p1;
      ps0 += p0;
      ps1 += p1;
    }
    l += ps0 + ps1;
    wait_v<0>(vf);
    pv(oacc, vf, pprev);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) pprev[kb][s2][j] = (__bf16)sacc[kb][8 * s2 + j];
    sacc[0] = snext[0];
    sacc[1] = snext[1];

    // pairs issued this iteration may stay in flight; older ones have landed
    asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  }

  // epilogue: PV of the group's last tile (pair niters-1)
  {
    VFrag vf;
    read_v(vf, vgrp + ((niters - 1) % NSLOT) * PAIR_BYTES, voff);
    wait_v<0>(vf);
    pv(oacc, vf, pprev);
  }

  // ---- merge the two groups' partial softmax states through LDS
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  float* xch = reinterpret_cast<float*>(smem) + wq * (34 * 64);
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
  if (grp == 0) {
    const float m1 = xch[32 * 64 + lane];
    const float l1 = xch[33 * 64 + lane];
    // group 1 saw no tile when the sequence has a single tile: it must not set
    // the reference max (a per-lane l1 == 0 test would be wrong: each lane
    // holds a partial sum over half of the keys)
    const bool g1 = ntiles > 1;
    const float mf = g1 ? fmaxf(m, m1) : m;
    const float a0 = __builtin_amdgcn_exp2f(m - mf);
    const float a1 = g1 ? __builtin_amdgcn_exp2f(m1 - mf) : 0.f;
    float lt = l * a0 + l1 * a1;
    lt += __shfl_xor(lt, 32, 64);
    const float inv = 1.f / lt;
    if (qrow < Sq) {
      unsigned short* op = o + b * bs_out + (long long)qrow * ld_out + h * D;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 32 * db + 8 * g + 4 * hh;
          bf16x4_t ov;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ri = 4 * g + e;
            const float o1 = xch[(16 * db + ri) * 64 + lane];
            ov[e] = (__bf16)((oacc[db][ri] * a0 + o1 * a1) * inv);
          }
          *reinterpret_cast<bf16x4_t*>(op + d) = ov;
        }
    }
  }
}

}  // namespace

// q/k/v: bf16 [B, S, *] rows with row stride ld_in (elements) and batch stride
// bs_in; head h occupies columns [h*64, h*64+64) relative to each pointer.
// o: bf16 [B, Sq, H*64 (+pad)] with row stride ld_out and batch stride bs_out.
NOS_API int nos_attn_fwd_d64(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq,
                             int Skv, int ld_in, long long bs_in, int ld_out, long long bs_out, float scale,
                             hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Skv <= 0) return (int)hipErrorInvalidValue;
  if ((ld_in % 8) != 0 || (ld_out % 4) != 0) return (int)hipErrorInvalidValue;
  const int nqb = (Sq + QBLK - 1) / QBLK;
  const int nwg = B * H * nqb;
  const float c = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(attn_fwd_d64_kernel, dim3(nwg), dim3(NT), LDS_BYTES, stream, (const unsigned short*)q,
                     (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o, B, H, Sq, Skv, ld_in,
                     bs_in, ld_out, bs_out, c, nqb);
  return (int)hipGetLastError();
}
