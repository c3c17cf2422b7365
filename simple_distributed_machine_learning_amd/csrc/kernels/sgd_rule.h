// torch.optim.SGD's update for 4 consecutive parameters, shared by the fused SGD kernel
// (elementwise.hip) and the reduction that applies the step itself on the one-rank MLP step
// (mlp_u8.hip's slab_head_reduce_kernel): d = g + wd p; buf = first ? d : mom buf + (1 - damp) d;
// d = nesterov ? d + mom buf : buf; p -= lr d. (/root/reference/simple_distributed.py:100-104)
#pragma once

#include <hip/hip_runtime.h>

#include "u8_planes.h"

namespace sdml {

typedef float sgd_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short sgd_u16x4 __attribute__((ext_vector_type(4)));

struct SgdRule {
  float lr, mom, damp, wd;
  int nesterov, first;
};

// p4 / buf4: the 4 parameters and their momentum (16-B aligned); returns the updated parameters.
// Every multiply-add is an explicit fma and contraction is off, so each kernel that inlines this rule
// (the SGD kernel, the reductions that apply the step themselves) produces the same bits: left to the
// compiler, "mom * b + (1 - damp) * d" may be fused around either product depending on the context.
// pv / bv0: the parameter and momentum values, loaded by the caller (ahead of its other loads: one memory round trip
// instead of a dependent one after the gradient sum); bv0 is read only with momentum and !first
__device__ __forceinline__ sgd_f32x4 sgd_update4_pre(float* p4, float* buf4, sgd_f32x4 d, const SgdRule& r,
                                                    const sgd_f32x4 pv, const sgd_f32x4 bv0) {
#pragma clang fp contract(off)
  if (r.wd != 0.f) {
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = __builtin_fmaf(r.wd, pv[j], d[j]);
  }
  if (r.mom != 0.f) {
    sgd_f32x4 b;
    if (r.first) {
      b = d;
    } else {
      b = bv0;
      const float keep = 1.f - r.damp;
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = __builtin_fmaf(r.mom, b[j], keep * d[j]);
    }
    *reinterpret_cast<sgd_f32x4*>(buf4) = b;
    if (r.nesterov) {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = __builtin_fmaf(r.mom, b[j], d[j]);
    } else {
      d = b;
    }
  }
  sgd_f32x4 nv;
#pragma unroll
  for (int j = 0; j < 4; ++j) nv[j] = __builtin_fmaf(-r.lr, d[j], pv[j]);
  *reinterpret_cast<sgd_f32x4*>(p4) = nv;
  return nv;
}

// the uint8 forward's fp16 weight planes of 4 updated weights at plane element q (u8_planes.h)
__device__ __forceinline__ sgd_f32x4 sgd_update4(float* p4, float* buf4, sgd_f32x4 d, const SgdRule& r) {
  const sgd_f32x4 pv = *reinterpret_cast<const sgd_f32x4*>(p4);
  const sgd_f32x4 bv = (r.mom != 0.f && !r.first) ? *reinterpret_cast<const sgd_f32x4*>(buf4) : sgd_f32x4{0.f, 0.f, 0.f, 0.f};
  return sgd_update4_pre(p4, buf4, d, r, pv, bv);
}

__device__ __forceinline__ void sgd_write_planes4(unsigned short* q, int64_t plane_stride, sgd_f32x4 nv) {
  sgd_u16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned short hj, lj;
    u8_fwd_planes_of(nv[j], hj, lj);
    h[j] = hj;
    l[j] = lj;
  }
  *reinterpret_cast<sgd_u16x4*>(q) = h;
  *reinterpret_cast<sgd_u16x4*>(q + plane_stride) = l;
}

}  // namespace sdml
