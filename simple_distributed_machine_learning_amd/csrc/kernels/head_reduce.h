// The fused head's per-block slab reduction as a block-level device function, shared by
// head_xent.hip's head_reduce_kernel and mlp_u8.hip's combined weight-gradient + head reduction
// (one launch for both deterministic reductions of the MLP step: HeadReduceArgs in kernels.h).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "sgd_rule.h"

namespace sdml {

// out[o] += sum_b part[b][o] in a fixed order (deterministic) for the 64 outputs of block `bx`.
// 1024 threads = 64 outputs x 16 waves; wave w sums slabs b = w, w+16, ... with 16 loads in flight,
// then the 16 wave partials are added in LDS (acc, 16 x 64 floats) in wave order.
// flags: bit 0 = training (accumulate gW/gb), bit 1 = overwrite stats instead of adding.
// sg (optional, sg->hp set): apply the optimizer step to gW / gb's parameters right here (the
// step's last gradient contribution), with the same rule as the SGD kernel.
__device__ __forceinline__ void head_reduce_block(const HeadReduceArgs& a, int bx, float (*acc)[64],
                                                  const SgdFuse* sg = nullptr) {
  const int train = a.flags & 1;
  const int width = a.CK + a.C + 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = bx * 64 + lane;
  // the fused step's epilogue operands (gW / gb, the head parameters and momentum), loaded with the slabs
  const int o4p = bx * 64 + 4 * lane;
  const bool pre = sg && sg->hp && (a.flags & 1) && w == 0 && lane < 16 && o4p + 4 <= a.CK + a.C;
  sgd_f32x4 g0 = {0.f, 0.f, 0.f, 0.f}, p0 = {0.f, 0.f, 0.f, 0.f}, b0 = {0.f, 0.f, 0.f, 0.f};
  if (pre) {
    g0 = *reinterpret_cast<const sgd_f32x4*>(a.gW + o4p);
    p0 = *reinterpret_cast<const sgd_f32x4*>(sg->hp + o4p);
    if (sg->mom != 0.f && !sg->first) b0 = *reinterpret_cast<const sgd_f32x4*>(sg->hbuf + o4p);
  }
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
  if (sg && sg->hp && (a.flags & 1)) {  // fused step: 4 consecutive outputs per lane (gb follows gW)
    __syncthreads();
    if (w == 0 && o < width) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) t += acc[i][lane];
      acc[0][lane] = t;  // (row 0 was wave 0's own partial: read above)
    }
    __syncthreads();
    const int o4 = bx * 64 + 4 * lane;
    if (w == 0 && lane < 16 && o4 < a.CK + a.C) {
      const int n4 = min(4, a.CK + a.C - o4);  // the last group may hold the 2 stats or padding
      float* gp = a.gW + o4;
      sgd_f32x4 d;
      if (n4 == 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = g0[j] + acc[0][4 * lane + j];
        sgd_update4_pre(sg->hp + o4, sg->hbuf + o4, d, SgdRule{sg->lr, sg->mom, sg->damp, sg->wd, sg->nesterov, sg->first},
                        p0, b0);
        *reinterpret_cast<sgd_f32x4*>(gp) = sg->zero_grad ? sgd_f32x4{0.f, 0.f, 0.f, 0.f} : d;
      } else {  // ragged tail (CK + C not a multiple of 4): the padding after gb is zero in every buffer
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = j < n4 ? gp[j] + acc[0][4 * lane + j] : 0.f;
        sgd_f32x4 pt, bt;  // 16-B aligned locals (hbuf is null without momentum: the rule then never reads it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pt[j] = j < n4 ? sg->hp[o4 + j] : 0.f;
          bt[j] = (j < n4 && sg->hbuf) ? sg->hbuf[o4 + j] : 0.f;
        }
        sgd_update4(reinterpret_cast<float*>(&pt), reinterpret_cast<float*>(&bt), d,
                    SgdRule{sg->lr, sg->mom, sg->damp, sg->wd, sg->nesterov, sg->first});
        for (int j = 0; j < n4; ++j) {
          sg->hp[o4 + j] = pt[j];
          if (sg->hbuf) sg->hbuf[o4 + j] = bt[j];
          gp[j] = sg->zero_grad ? 0.f : d[j];
        }
      }
    }
    if (w == 1 && lane < 2 && bx * 64 <= a.CK + a.C + lane && a.CK + a.C + lane < bx * 64 + 64) {  // stats
      const int so = a.CK + a.C + lane;
      float t = acc[0][so - bx * 64];
      if (a.flags & 2) a.stats[lane] = t;
      else a.stats[lane] += t;
    }
    return;
  }
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
