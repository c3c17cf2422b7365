// One 16-row tile of the MFMA classifier head (K = 128 hidden, C <= 16 classes), shared by
// head_xent.hip's head_mfma_kernel (h read from HBM) and mlp_u8.hip's fused uint8 forward + head
// (h never leaves the workgroup: it is staged in LDS straight from the forward's accumulators).
// Both call the same two device functions, so their logits, dlogits and dW^T products are the same
// operations in the same order (the fused kernel's dl is bit-identical to the standalone head's).
//
// Lane l = (r = l % 16, g = l / 16), fp32 MFMAs (v_mfma_f32_16x16x4_f32):
//   logits^T = W x^T : A = W (lane: class r), B = x^T (lane: row r), k = 16u + 4g + e over 32 MFMAs;
//     lane (r, g) ends with row r's logits of classes 4g .. 4g+3 (bias as the initial value), so
//     softmax / NLL / argmax reduce 4 values in-lane plus two symmetric permlane swaps (wave_ops.h)
//   dW^T += x^T dz : x read back transposed from the tile's LDS image (xt_at layout) and dz through a
//     wave-private 16 x 16 transpose; dW^T stays in registers across the wave's tiles.
// Reference op: /root/reference/simple_distributed.py:77-79 (fc2, log_softmax), :111 (nll_loss).
#pragma once

#include <hip/hip_runtime.h>

#include "wave_ops.h"

namespace sdml {
namespace headtile {

typedef float f32x4m __attribute__((ext_vector_type(4)));
constexpr int HKT = 128;  // hidden width
constexpr int DTP = 16;   // dz transpose pitch

// x tile image [16 rows][128] with the 16-B chunk c of row rho's 16-float group at c ^ swz(rho) and
// group q at q ^ (rho & 3): the column reads (rows 4kk + g, columns 16t + r) cover 64 distinct banks, and
// the row reads xt_at(r, u, 4g) (ds_read_b128, lane (r, g)) are conflict-free: in each 16-lane group of a
// b128 read the four (g, r >> 2) classes present get the 4 distinct chunk slots g ^ h(r >> 2), h = {0, 2,
// 3, 1} (with h(r >> 2) = r >> 2 two classes shared a slot: 2-way conflicts on every x-tile read of the
// fused uint8 forward's head epilogue; checked by enumeration, r4).
__device__ __forceinline__ int swz(int rho) { return 4 * ((0x78 >> (2 * ((rho >> 2) & 3))) & 3); }
__device__ __forceinline__ int xt_at(int rho, int q, int j) {
  return rho * HKT + 16 * (q ^ (rho & 3)) + (j ^ swz(rho));
}

__device__ __forceinline__ f32x4m mfma4(float a, float b, f32x4m c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct TileAcc {
  f32x4m gw[8];  // dW^T: gw[t][v] = dW[class r][hidden 16 t + 4 g + v]
  float gbp, loss, corr, amx;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < 8; ++t) gw[t] = f32x4m{0.f, 0.f, 0.f, 0.f};
    gbp = loss = corr = amx = 0.f;
  }
};

// softmax_dz: log_softmax, NLL (loss accumulated for valid rows), argmax (correct), and when `train`
// dz = scale (softmax - onehot) for the lane's 4 classes (0 for invalid rows / classes >= C); amx tracks
// max_row sum_c |dz_c| (the |dl @ W| bound). Given lane (r, g)'s logits z of classes 4g .. 4g+3 of row r (the layout of a
// 16x16 MFMA accumulator: head_block.h's fp16-plane head produces it too)
template <int C>
__device__ __forceinline__ void softmax_dz(const f32x4m& z, int tg_raw, bool valid, bool train, float scale, int g,
                                           TileAcc& a, float (&dz)[4], bool track_amax) {
  constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  float zc[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) zc[v] = (4 * g + v) < C ? z[v] : -INFINITY;
  // row max and first argmax over the 4 lane groups (symmetric, branch-free combines)
  float mx = zc[0];
  int am = 4 * g;
#pragma unroll
  for (int v = 1; v < 4; ++v) {
    const bool t = zc[v] > mx;
    mx = t ? zc[v] : mx;
    am = t ? 4 * g + v : am;
  }
  wv::argmax_rows(mx, am);
  // p = exp(z - max) once (one fma + v_exp each); the softmax is p / sum p, the log-sum-exp max + log(sum p)
  const float mxl = mx * LOG2E;
  float p[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) p[v] = __builtin_amdgcn_exp2f(fmaf(zc[v], LOG2E, -mxl));
  const float se = wv::sum_rows((p[0] + p[1]) + (p[2] + p[3]));
  const float lse = fmaf(__builtin_amdgcn_logf(se), LN2, mx);
  const int tg = valid ? tg_raw : -1;
  float zt = zc[0];
#pragma unroll
  for (int v = 1; v < 4; ++v) zt = (tg & 3) == v ? zc[v] : zt;
  a.loss += (valid && (tg >> 2) == g) ? lse - zt : 0.f;
  a.corr += (valid && g == 0 && am == tg) ? 1.f : 0.f;
  if (!train) return;
  const float rs = scale * __builtin_amdgcn_rcpf(se);
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int c = 4 * g + v;
    dz[v] = (valid && c < C) ? fmaf(p[v], rs, c == tg ? -scale : 0.f) : 0.f;
  }
  if (track_amax) {  // (invalid rows and classes >= C hold dz == 0)
    const float sa = (fabsf(dz[0]) + fabsf(dz[1])) + (fabsf(dz[2]) + fabsf(dz[3]));
    a.amx = fmaxf(a.amx, wv::sum_rows(sa));
  }
}

// dW^T += x^T dz, db += dz: xw = this tile's x image (xt_at layout, complete and visible to the wave),
// dw = the wave's 16 x DTP dz transpose scratch
__device__ __forceinline__ void dw_accum(const float* xw, float* dw, const float (&dz)[4], int r, int g, TileAcc& a) {
  *reinterpret_cast<f32x4m*>(dw + r * DTP + ((4 * g) ^ swz(r))) = f32x4m{dz[0], dz[1], dz[2], dz[3]};
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float db[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    db[kk] = dw[(4 * kk + g) * DTP + (r ^ swz(4 * kk + g))];
    a.gbp += db[kk];
  }
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) a.gw[t] = mfma4(xw[xt_at(4 * kk + g, t, r)], db[kk], a.gw[t]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
  __builtin_amdgcn_wave_barrier();
}

}  // namespace headtile
}  // namespace sdml
