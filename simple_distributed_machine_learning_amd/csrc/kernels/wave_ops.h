// Cross-lane reductions on gfx950 that stay on the VALU: DPP (quad_perm, row_half_mirror, row_mirror) inside a row
// of 16 lanes, v_permlane16_swap / v_permlane32_swap across rows. __shfl_xor lowers to ds_bpermute_b32, an LDS
// crossbar round trip per step; a reduction chain of those is latency-bound (the head epilogue had ~50 of them).
//
// Every combine here is symmetric in its two operands (a + b, fmaxf, the argmax rule), and a permlane swap of a
// register with itself leaves lane l holding {x[l], x[l ^ 16]} (resp. ^ 32) as its two results, so every lane of a
// group ends with the same bits - whichever half of the swap pair is "own".
#pragma once

#include <hip/hip_runtime.h>

namespace sdml {
namespace wv {

constexpr int XOR1 = 0xB1;         // quad_perm [1, 0, 3, 2]
constexpr int XOR2 = 0x4E;         // quad_perm [2, 3, 0, 1]
constexpr int HALF_MIRROR = 0x141;  // lane i <-> 7 - i within each 8
constexpr int MIRROR = 0x140;       // lane i <-> 15 - i within each 16

template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

// {x[l], x[l ^ 16]} / {x[l], x[l ^ 32]} in an unspecified order
__device__ __forceinline__ void pair16(float x, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair32(float x, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair16(int x, int& a, int& b) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
  a = (int)r[0];
  b = (int)r[1];
}
__device__ __forceinline__ void pair32(int x, int& a, int& b) {
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
  a = (int)r[0];
  b = (int)r[1];
}

// sum / max over the 16 lanes of a row (every lane of the row gets the result)
__device__ __forceinline__ float sum16(float x) {
  x += dpp<XOR1>(x);
  x += dpp<XOR2>(x);
  x += dpp<HALF_MIRROR>(x);
  return x + dpp<MIRROR>(x);
}
__device__ __forceinline__ float max16(float x) {
  x = fmaxf(x, dpp<XOR1>(x));
  x = fmaxf(x, dpp<XOR2>(x));
  x = fmaxf(x, dpp<HALF_MIRROR>(x));
  return fmaxf(x, dpp<MIRROR>(x));
}
// x[l] + x[l ^ 16] + x[l ^ 32] + x[l ^ 48] (the 4 row groups of a 16x16 MFMA accumulator)
__device__ __forceinline__ float sum_rows(float x) {
  float a, b;
  pair16(x, a, b);
  x = a + b;
  pair32(x, a, b);
  return a + b;
}
__device__ __forceinline__ float max_rows(float x) {
  float a, b;
  pair16(x, a, b);
  x = fmaxf(a, b);
  pair32(x, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float sum64(float x) { return sum_rows(sum16(x)); }
__device__ __forceinline__ float max64(float x) { return max_rows(max16(x)); }

// (max, first index) over the 4 row groups: the larger value wins, ties go to the smaller index
__device__ __forceinline__ void argmax_rows(float& mx, int& am) {
  float m0, m1;
  int a0, a1;
  pair16(mx, m0, m1);
  pair16(am, a0, a1);
  bool take = (m1 > m0) | ((m1 == m0) & (a1 < a0));  // (bitwise: no short-circuit branches)
  mx = take ? m1 : m0;
  am = take ? a1 : a0;
  pair32(mx, m0, m1);
  pair32(am, a0, a1);
  take = (m1 > m0) | ((m1 == m0) & (a1 < a0));
  mx = take ? m1 : m0;
  am = take ? a1 : a0;
}

}  // namespace wv
}  // namespace sdml
