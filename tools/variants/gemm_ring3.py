import sys; p=sys.argv[1]+'/gemm.hip'
s=open(p).read()
rep=[
('''//  * two LDS buffers: tile k+1 is in flight while tile k is consumed;''',
'''//  * three-stage LDS ring: tiles k+1 and k+2 are in flight while tile k is
//    consumed; counted `s_waitcnt vmcnt(8)` + raw s_barrier keep the next
//    tile's DMA alive across the barrier (a __syncthreads would drain it);
//    96 KiB, so one GEMM workgroup and one attention workgroup (64 KiB) of
//    another tenant still fit one CU's 160 KiB LDS;'''),
('''constexpr int CT_LD = BN + 4;                        // fp32 C tile row stride (floats)
constexpr int CT_BYTES = BM * CT_LD * 4;             // 67,584 B
constexpr int MAIN_BYTES = (2 * STAGE_BYTES > CT_BYTES) ? 2 * STAGE_BYTES : CT_BYTES;
constexpr int STATS_OFF = MAIN_BYTES;                // mu[128], rstd[128], p1[128], p2[128]
constexpr int LDS_BYTES = MAIN_BYTES + 4 * BM * 4;''',
'''constexpr int NSTAGE = 3;
constexpr int GLDS_PER_STAGE = 8;                    // per wave: 4 for A + 4 for W
constexpr int CT_LD = BN + 4;                        // fp32 C tile row stride (floats)
constexpr int CT_BYTES = BM * CT_LD * 4;             // 67,584 B
constexpr int RING_BYTES = NSTAGE * STAGE_BYTES;     // 96 KiB
constexpr int STATS_OFF = CT_BYTES;                  // mu[128], rstd[128], p1[128], p2[128] (epilogue only)
constexpr int LDS_BYTES = RING_BYTES;
static_assert(STATS_OFF + 4 * BM * 4 <= RING_BYTES, "epilogue scratch must fit in the ring");

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}'''),
('''    stage_tile(A, lda, m0, M, 0, smem, wid, lane);
    stage_tile(W, ldw, n0, N, 0, smem + TILE_A_BYTES, wid, lane);
    __syncthreads();  // drains the DMA (vmcnt(0)) and publishes the tile

    for (int kt = 0; kt < nk; ++kt) {
      unsigned char* cur = smem + (kt & 1) * STAGE_BYTES;
      if (kt + 1 < nk) {
        unsigned char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
        stage_tile(A, lda, m0, M, (kt + 1) * BK, nxt, wid, lane);
        stage_tile(W, ldw, n0, N, (kt + 1) * BK, nxt + TILE_A_BYTES, wid, lane);
      }
      const unsigned char* ta = cur;''',
'''#pragma unroll
    for (int s = 0; s < NSTAGE - 1; ++s)
      if (s < nk) {
        stage_tile(A, lda, m0, M, s * BK, smem + s * STAGE_BYTES, wid, lane);
        stage_tile(W, ldw, n0, N, s * BK, smem + s * STAGE_BYTES + TILE_A_BYTES, wid, lane);
      }

    int slot = 0;  // ring slot of tile kt
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt landed (this wave's DMA: only tile kt+1's 8 loads may remain),
      // then the barrier publishes every wave's share and retires the reads of
      // tile kt-1, whose slot is restaged next
      if (kt + 1 < nk)
        wait_vmcnt<GLDS_PER_STAGE>();
      else
        wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + NSTAGE - 1 < nk) {
        const int ns = slot == 0 ? NSTAGE - 1 : slot - 1;
        unsigned char* nxt = smem + ns * STAGE_BYTES;
        stage_tile(A, lda, m0, M, (kt + NSTAGE - 1) * BK, nxt, wid, lane);
        stage_tile(W, ldw, n0, N, (kt + NSTAGE - 1) * BK, nxt + TILE_A_BYTES, wid, lane);
      }
      unsigned char* cur = smem + slot * STAGE_BYTES;
      slot = slot + 1 == NSTAGE ? 0 : slot + 1;
      const unsigned char* ta = cur;'''),
('''            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
      }
      __syncthreads();  // next tile landed; everyone done with `cur`
    }
''','''            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave done with the ring (all DMA retired above): reuse it
'''),
]
for a,b in rep:
    assert a in s, a[:80]
    s=s.replace(a,b)
open(p,'w').write(s)
