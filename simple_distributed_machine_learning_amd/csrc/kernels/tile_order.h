// Tile order of the output-tiled GEMMs (gemm_bf16.hip, gemm_f16x2.hip): logical tile id -> (tm, tn).
// The launch remaps blockIdx XCD-aware first, so consecutive logical ids share an XCD and its L2; one XCD runs ~32
// tiles at once. group_m = 0: M fastest, those 32 tiles are 32 m-panels of ONE n-panel (only B is re-read from L2).
// group_m = g > 0: tiles walk groups of g m-tiles x every n-tile, m fastest inside a group, so the 32 tiles cover
// g m-panels x 32 / g n-panels and both operands are re-read from the XCD's L2 (the grouped order of tiled GEMM
// schedulers). Measured at the GPT-2 shapes: profiles/r6_gemm_group_ab.jsonl.
#pragma once

namespace sdml {

__device__ __forceinline__ void tile_of(int wg, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 0) {
    tm = wg % tiles_m;
    tn = wg / tiles_m;
    return;
  }
  const int per = gm * tiles_n;
  const int grp = wg / per, first = grp * gm;
  const int rows = tiles_m - first < gm ? tiles_m - first : gm;
  const int loc = wg - grp * per;
  tm = first + loc % rows;
  tn = loc / rows;
}

}  // namespace sdml
