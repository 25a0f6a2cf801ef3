// Host-side tile choice of the bf16 GEMM (gemm.hip), kept free of HIP so the
// CPU test suite can compile and check it (tests/test_gemm_tile_choice.py).
#pragma once

namespace nos_gemm {

enum TileKind : int { T_BASE, T_NARROW, T_WIDE, T_BIG };

// Tile choice by a cost model: (tiles or rounds of tiles) x tile area /
// relative efficiency.  The efficiencies are measured per output element on
// the batch-8 YOLOS shapes and 4096^3 (profiles/r02_gemm_bf16_tiles.json):
// the 8-wave 256-row tiles read half the L2 bytes per FLOP and 0.75-0.83 LDS
// fragments per MFMA; 128x64 reads 1.5.
//  * latency policy: ceil(tiles / CUs) x area -- the rounds a single tenant waits;
//  * throughput policy: tiles x area -- the work co-running pods share (and
//    no 128x64, which costs them ~4 %);
// the 512-thread tiles only when they occupy at least half the CUs (a few big
// tiles would serialise one tenant on a handful of CUs).
inline int pick_tile(int M, int N, int policy, int cus) {
  if (policy == 2) return T_NARROW;
  if (policy == 3) return T_BIG;
  if (policy == 4) return T_WIDE;
  struct Cand {
    int kind, bm, bn;
    double eff;
  };
  static constexpr Cand cands[] = {{T_BASE, 128, 128, 1.0}, {T_NARROW, 128, 64, 0.8}, {T_WIDE, 256, 192, 1.2},
                                   {T_BIG, 256, 256, 1.25}};
  int pick = T_BASE;
  double best = 1e300;
  for (const Cand& c : cands) {
    if (policy == 0 && c.kind == T_NARROW) continue;
    const long long tiles = (long long)((M + c.bm - 1) / c.bm) * ((N + c.bn - 1) / c.bn);
    if (c.bm == 256 && 2 * tiles < cus) continue;
    const double per = (double)c.bm * c.bn / c.eff;
    const double cost = policy == 1 ? (double)((tiles + cus - 1) / cus) * per : (double)tiles * per;
    if (cost < best * 0.99) {  // ties keep the earlier (smaller) tile
      best = cost;
      pick = c.kind;
    }
  }
  return pick;
}

}  // namespace nos_gemm
