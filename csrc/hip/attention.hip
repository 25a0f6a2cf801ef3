// Fused multi-head self-attention forward (flash-style, non-causal) for the
// YOLOS-family tenant model, bf16 in / bf16 out, fp32 softmax, head_dim 64.
//
// CDNA4 design (not a port of any CUDA kernel):
//  * one workgroup = 8 waves = 128 query rows of one (batch, head), split in
//    two wave groups that walk interleaved 64-key tiles of the same K/V
//    stream (group 0: even tiles, group 1: odd tiles) -- two waves per SIMD
//    from one workgroup, so one wave's MFMAs overlap the other's softmax,
//    without shrinking the grid (one inference has only ~160 128-row blocks);
//    the groups' partial (m, l, O) are merged through LDS at the end;
//  * each wave owns 32 query rows, held for the whole kernel as the B
//    operand of v_mfma_f32_32x32x16_bf16;
//  * "swapped" QK^T: S^T = K . Q^T, so every lane holds 16 of the 32 key
//    scores of ONE query row (column = lane & 31): row max / sum are
//    lane-local plus one v_permlane32_swap;
//  * the S^T accumulator is re-used in registers as the B operand of
//    O^T = V^T . P^T (no LDS round trip for P);
//  * V^T fragments come from a row-major, XOR-swizzled V tile through the
//    gfx950 transposing LDS read ds_read_b64_tr_b16; K is read with
//    ds_read_b128 from an XOR-swizzled image (both conflict-free);
//  * K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//    instruction) into a 2-deep ring: no staging registers, no ds_write;
//    the swizzle is applied to the per-lane SOURCE address (linear LDS
//    destination, cdna_hip_programming.md rule 21);
//  * every LDS address is a per-lane base register + an immediate: the
//    swizzle terms that vary per lane are hoisted out of the key loop;
//  * deferred rescale (T13): O and l are only rescaled when some row's max
//    grows by more than 8 (log2 units; P <= 2^8); the reference max starts
//    at the group's first tile max, so no -inf sentinels are needed;
//  * XCD-aware workgroup -> (batch, head, q-block) map: q-blocks of one
//    head share an XCD's L2 (K/V of one head = 870 KB at S = 3401).
#include "common.h"

namespace {

constexpr int D = 64;
constexpr int QBLK = 128;          // query rows per workgroup (4 waves x 32)
constexpr int KVBLK = 64;          // keys per tile (per wave group)
constexpr int NT = 512;            // 8 waves
constexpr int TILE_BYTES = KVBLK * D * 2;   // 8 KiB
constexpr int PAIR_BYTES = 4 * TILE_BYTES;  // K0 V0 K1 V1 (one tile per group)
constexpr int LDS_BYTES = 2 * PAIR_BYTES;   // 2-deep ring: 64 KiB
constexpr float RESCALE_THR = 8.f;          // log2 units

__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int vswz(int row) { return ((row >> 1) & 1) << 2; }

__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__global__ __launch_bounds__(NT, 4) void attn_fwd_d64_kernel(
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

  // ---- LDS-DMA staging: per iteration 2 tiles x (K + V) = 32 x 1 KiB pieces,
  // 4 per wave.  Piece p (0..31): tensor p>>4 (K/V), tile-row block (p&15)*8.
  // Lane L writes row R + L/8, physical chunk L%8 = logical chunk ^ swizzle.
  auto stage = [&](int it, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = wid * 4 + i;
      const int is_v = p >> 4;
      const int R = (p & 15) * 8;          // 0..120 across the two tiles
      const int row = R + (lane >> 3);     // 0..127
      const int g = row >> 6, lr = row & 63;
      const int pc = lane & 7;
      const int lc = pc ^ (is_v ? vswz(lr) : kswz(lr));
      int kv = it * 2 * KVBLK + row;
      kv = kv < Skv ? kv : Skv - 1;
      const unsigned short* src = (is_v ? vb_ptr : kb_ptr) + (long long)kv * ld_in + lc * 8;
      unsigned char* dst = smem + buf * PAIR_BYTES + g * 2 * TILE_BYTES + is_v * TILE_BYTES + (R & 63) * 128;
      glds16(src, dst);
    }
  };

  const int ntiles = (Skv + KVBLK - 1) / KVBLK;
  const int niters = (ntiles + 1) / 2;
  stage(0, 0);

  // hoisted per-lane LDS offsets (relative to the group's K / V tile)
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = r * 128 + (((2 * ks + hh) ^ kswz(r)) << 4);
  const int g16 = (lane >> 4) & 1;
  const int tq = (lane & 15) >> 2;
  const int tp = lane & 3;
  const int vlb = (tq >> 1) & 1;  // (row >> 1) & 1 of every row this lane's tr-reads touch
  int voff[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
    voff[db] = (4 * hh + tq) * 128 + (((4 * (db ^ vlb)) + 2 * g16 + (tp >> 1)) << 4) + 8 * (tp & 1);

  f32x16_t oacc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; }
  // m: the row's reference max in log2 units (scores x c); p = exp2(s*c - m)
  // is one FMA + one v_exp per score.  m only moves on the group's first tile
  // and when a row's max exceeds it by more than RESCALE_THR (then
  // p <= 2^RESCALE_THR in between).  (Pre-scaling Q by c instead would add a
  // bf16 rounding of Q*c: ~0.1 abs error on peaky rows.)
  float m = 0.f, l = 0.f;

  __syncthreads();  // drains stage 0 (vmcnt(0)) and publishes it

  for (int it = 0; it < niters; ++it) {
    const int buf = it & 1;
    if (it + 1 < niters) stage(it + 1, buf ^ 1);  // buffer freed by the barrier that ended it-1

    const int t = 2 * it + grp;  // this group's tile
    if (t < ntiles) {
      const unsigned char* kl = smem + buf * PAIR_BYTES + grp * 2 * TILE_BYTES;
      const unsigned char* vl = kl + TILE_BYTES;

      f32x16_t sacc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kb][i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(kl + koff[ks] + kb * 32 * 128);
          sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], sacc[kb], 0, 0, 0);
        }
      }
      if ((t + 1) * KVBLK > Skv) {
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
      if (it == 0 || !__all(mrel <= RESCALE_THR)) {
        // first tile: m := tile max; later: raise m where the max grew
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
      // p = exp2(s*c - m): scalar FMA / add beside the MFMAs (a v_pk_*_f32
      // costs more issue cycles than the two scalar ops it replaces,
      // MI355X_MICROARCH 'price of one filler'), two row-sum accumulators
      // (even / odd scores: the packed form's order), packed bf16 conversion
      float ps0 = 0.f, ps1 = 0.f;
      const float nm = -m;
      bf16x8_t pf[2][2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j2 = 0; j2 < 8; ++j2) {
          f32x2_t x;
          x.x = __builtin_amdgcn_exp2f(fmaf(sacc[kb][2 * j2], c, nm));
          x.y = __builtin_amdgcn_exp2f(fmaf(sacc[kb][2 * j2 + 1], c, nm));
          ps0 += x.x;
          ps1 += x.y;
          const bf16x2_t pb = __builtin_convertvector(x, bf16x2_t);
          pf[kb][j2 >> 2][2 * (j2 & 3)] = pb.x;
          pf[kb][j2 >> 2][2 * (j2 & 3) + 1] = pb.y;
        }
      l += ps0 + ps1;

#pragma unroll
      for (int db = 0; db < 2; ++db) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const unsigned char* base = vl + voff[db] + (kb * 32 + s2 * 16) * 128;
            const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base));
            const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4_t, base + 8 * 128));
            const s16x8_t a16 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a16), pf[kb][s2],
                                                               oacc[db], 0, 0, 0);
          }
      }
    }
    __syncthreads();  // next stage landed (vmcnt(0)); everyone done with `buf`
  }

  // ---- merge the two groups' partial softmax states through LDS
  // layout per group-1 wave: [32 O floats][m][l] per lane, 34 x 64 floats
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
