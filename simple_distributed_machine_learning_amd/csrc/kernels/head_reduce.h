// The fused head's per-block slab reduction as a block-level device function, shared by
// head_xent.hip's head_reduce_kernel and mlp_u8.hip's combined weight-gradient + head reduction
// (one launch for both deterministic reductions of the MLP step: HeadReduceArgs in kernels.h).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdml {

// out[o] += sum_b part[b][o] in a fixed order (deterministic) for the 64 outputs of block `bx`.
// 1024 threads = 64 outputs x 16 waves; wave w sums slabs b = w, w+16, ... with 16 loads in flight,
// then the 16 wave partials are added in LDS (acc, 16 x 64 floats) in wave order.
// flags: bit 0 = training (accumulate gW/gb), bit 1 = overwrite stats instead of adding.
__device__ __forceinline__ void head_reduce_block(const HeadReduceArgs& a, int bx, float (*acc)[64]) {
  const int train = a.flags & 1;
  const int width = a.CK + a.C + 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = bx * 64 + lane;
  float s = 0.f;
  if (o < width) {  // 16 loads in flight per lane (512 slabs: two round trips per wave)
    float v[16];
    int b = w;
    for (; b + 16 * 15 < a.nblocks; b += 16 * 16) {
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = a.part[(size_t)(b + 16 * u) * width + o];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; b < a.nblocks; b += 16) s += a.part[(size_t)b * width + o];
  }
  acc[w][lane] = s;
  __syncthreads();
  if (w == 0 && o < width) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += acc[i][lane];
    if (o < a.CK) {
      if (train) a.gW[o] += t;
    } else if (o < a.CK + a.C) {
      if (train) a.gb[o - a.CK] += t;
    } else if (a.flags & 2) {
      a.stats[o - a.CK - a.C] = t;
    } else {
      a.stats[o - a.CK - a.C] += t;
    }
  }
}

inline int head_reduce_blocks(const HeadReduceArgs& a) { return (a.CK + a.C + 2 + 63) / 64; }

}  // namespace sdml
