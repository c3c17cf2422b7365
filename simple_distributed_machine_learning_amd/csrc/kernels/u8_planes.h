// Weight planes of the uint8-fed first layer (mlp_u8.hip's forward), written by split_planes_pad
// and by the fused SGD step (elementwise.hip) with this one function, so both writers agree bit
// for bit.
//
// W (fp32) is stored as two fp16 planes of W' = W * 2^8: hi = fp16(W') (round to nearest even) and
// lo = fp16(W' - hi). W' - hi is exact in fp32 (hi is W' rounded to 11 significant bits), and lo
// keeps 11 more bits of it, so |hi + lo - W'| <= 2^-23 |W'|: the pair is W to within one fp32
// ulp. A pixel byte is exact in fp16, so x * W costs 2 fp16 MFMA products (bf16 needs 3
// planes for the same 24 bits). The 2^8 keeps that bound for |W| >= 2^-9 (lo's absolute precision is
// 2^-25 or better in units of W * 2^8); smaller weights keep an absolute error below 2^-33. |W| >= 255.9
// overflows hi to inf, so a diverged weight shows up as a non-finite output instead of a silent
// error. The forward folds the 2^-8 into its epilogue scale.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"  // kU8FwdPlanes

namespace sdml {

constexpr float kU8FwdWScale = 256.f;

__device__ __forceinline__ void u8_fwd_planes_of(float w, unsigned short& hi, unsigned short& lo) {
  const float s = w * kU8FwdWScale;
  const _Float16 h = static_cast<_Float16>(s);
  const _Float16 l = static_cast<_Float16>(s - static_cast<float>(h));
  hi = __builtin_bit_cast(unsigned short, h);
  lo = __builtin_bit_cast(unsigned short, l);
}

}  // namespace sdml
