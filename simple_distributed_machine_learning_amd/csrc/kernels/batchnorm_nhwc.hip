// Training-mode BatchNorm (+ residual add) (+ ReLU) on channels-last bf16 activations, for the
// ResNet-18-style stages (models/resnet.py). x is viewed as [M = N*H*W][C] (channels contiguous).
//
// forward : stats   per-channel sum / sum of squares -> per-block fp32 partials
//           finalize fixed-order fp64 reduction of the partials -> mean, rstd, the folded
//                    scale = gamma * rstd and shift = beta - mean * scale, running-stat update
//           apply    y = relu?(x * scale + shift (+ residual))        (one read, one write)
// backward: partial  per-channel sums of g and g * xhat, g = dy * (y > 0 if relu)
//           finalize dgamma / dbeta added into the bf16 parameter gradients, the two means
//           apply    dx = gamma * rstd * (g - mean(g) - xhat * mean(g * xhat)); dres = g
//                    (folded per channel into dx = a * (g - mean(g)) + b * (x - mean))
// Every pass streams 16 B per thread (8 channels); reductions are deterministic (per-block
// partials summed in block order). PyTorch's channels-last BatchNorm kernels ran 100-800 us per
// call on these shapes (0.1-0.5 TB/s, profiles/r1_resnet_bf16_kernel_stats.txt).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, static_cast<__bf16>(f)); }

constexpr int BT = 256;

// rows of this block: [blockIdx.x * rpb, +rpb); thread = (row lane, 8-channel group)
// relu (backward): 0 none, 1 mask from the saved output y > 0, 2 mask recomputed from the input
// (x * gamma * rstd + beta - mean * gamma * rstd > 0: BatchNorm + ReLU without a residual, so the
// output need not be kept or re-read)
template <bool BWD>
__global__ void __launch_bounds__(BT) bn_partial_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                        const u16* __restrict__ y, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, const u16* __restrict__ gamma,
                                                        const u16* __restrict__ beta, int M, int C, int rpb,
                                                        int relu, float* __restrict__ part) {
  __shared__ float red[BT * 16];
  const int G = C / 8;  // channel groups
  const int lanes = BT / G;
  const int cg = threadIdx.x % G, rl = threadIdx.x / G;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  float mu[8], rs[8], sc[8], sh[8];
  if (BWD) {  // (16-B loads, all issued before the first use)
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const f32x4 m0 = reinterpret_cast<const f32x4*>(mean + 8 * cg)[0], m1 = reinterpret_cast<const f32x4*>(mean + 8 * cg)[1];
    const f32x4 q0 = reinterpret_cast<const f32x4*>(rstd + 8 * cg)[0], q1 = reinterpret_cast<const f32x4*>(rstd + 8 * cg)[1];
    u16x8 gm = {0, 0, 0, 0, 0, 0, 0, 0}, bt = {0, 0, 0, 0, 0, 0, 0, 0};
    if (relu == 2) {  // (uniform)
      gm = *reinterpret_cast<const u16x8*>(gamma + 8 * cg);
      bt = *reinterpret_cast<const u16x8*>(beta + 8 * cg);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = e < 4 ? m0[e & 3] : m1[e & 3];
      rs[e] = e < 4 ? q0[e & 3] : q1[e & 3];
      sc[e] = bf2f(gm[e]) * rs[e];
      sh[e] = bf2f(bt[e]) - mu[e] * sc[e];
    }
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  if (rl < lanes) {
    // RU rows per round, all their loads issued before the first use (clamped row, the extra rows dropped by a
    // select): a round is one memory latency, not RU. Rows are still added in order. (One row per round waited out
    // ~25 dependent round trips per thread at C = 64, M = 401K: ~19 us per call.)
    constexpr int RU = 4;
    for (int rb = r0 + rl; rb < r1; rb += RU * lanes) {
      u16x8 xv[RU], gv[RU], yv[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const size_t o = (size_t)min(rb + u * lanes, r1 - 1) * C + 8 * cg;
        xv[u] = *reinterpret_cast<const u16x8*>(x + o);
        if (BWD) {
          gv[u] = *reinterpret_cast<const u16x8*>(dy + o);
          yv[u] = relu == 1 ? *reinterpret_cast<const u16x8*>(y + o) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const bool in = rb + u * lanes < r1;
        if (!BWD) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = bf2f(xv[u][e]);
            s1[e] = in ? s1[e] + v : s1[e];
            s2[e] = in ? s2[e] + v * v : s2[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float g = bf2f(gv[u][e]);
            if (relu == 1 && !(bf2f(yv[u][e]) > 0.f)) g = 0.f;
            if (relu == 2 && !(fmaf(bf2f(xv[u][e]), sc[e], sh[e]) > 0.f)) g = 0.f;
            s1[e] = in ? s1[e] + g : s1[e];
            s2[e] = in ? s2[e] + g * (bf2f(xv[u][e]) - mu[e]) * rs[e] : s2[e];
          }
        }
      }
    }
  }
  // block reduction over the row lanes (fixed order)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(rl * G + cg) * 16 + e] = s1[e];
    red[(rl * G + cg) * 16 + 8 + e] = s2[e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * 16; i += BT) {
    const int g = i / 16, e = i % 16;
    float a = 0.f;
    for (int l = 0; l < lanes; ++l) a += red[(l * G + g) * 16 + e];
    const int c = 8 * g + (e & 7);
    part[(size_t)blockIdx.x * 2 * C + (e < 8 ? c : C + c)] = a;
  }
}

// one wave per channel: lane l sums partials l, l+64, ... in order (fp64), then a fixed shuffle tree
__device__ __forceinline__ void wave_sum2(const float* __restrict__ part, int nblk, int C, int c, double& s1,
                                          double& s2) {
  const int lane = threadIdx.x & 63;
  s1 = 0.0;
  s2 = 0.0;
  // 4 partials per lane per round, loads unconditional (clamped) and added in block order: one memory latency per
  // round (the one-at-a-time loop waited ~25 round trips at 1568 conv tiles)
  for (int b0 = lane; b0 < nblk; b0 += 4 * 64) {
    float v1[4], v2[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = min(b0 + 64 * u, nblk - 1);
      v1[u] = part[(size_t)b * 2 * C + c];
      v2[u] = part[(size_t)b * 2 * C + C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool in = b0 + 64 * u < nblk;
      s1 = in ? s1 + v1[u] : s1;
      s2 = in ? s2 + v2[u] : s2;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
}

// the 4 waves of a block split channel c's partials into 4 contiguous quarters (each summed as wave_sum2 does), the
// quarters added in order: a quarter of the dependent load rounds per wave (the conv epilogue writes ~1.5K partial
// rows, 6 rounds for one wave). sum4 = ((q0 + q1) + q2) + q3 in fp64.
__device__ __forceinline__ void block_sum2(const float* __restrict__ part, int nblk, int C, int c, double& s1,
                                           double& s2, double (*red)[2]) {
  const int w = threadIdx.x >> 6;
  const int q = (nblk + 3) / 4, b0 = min(nblk, w * q), b1 = min(nblk, b0 + q);
  double a1, a2;
  wave_sum2(part + (size_t)b0 * 2 * C, b1 - b0, C, c, a1, a2);
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = a1;
    red[w][1] = a2;
  }
  __syncthreads();
  s1 = ((red[0][0] + red[1][0]) + red[2][0]) + red[3][0];
  s2 = ((red[0][1] + red[1][1]) + red[2][1]) + red[3][1];
}

__global__ void __launch_bounds__(BT) bn_fwd_finalize_kernel(const float* __restrict__ part, int nblk, int C, int M,
                                                             float eps, float momentum, const u16* __restrict__ gamma,
                                                             const u16* __restrict__ beta, u16* __restrict__ rmean,
                                                             u16* __restrict__ rvar, float* __restrict__ mean,
                                                             float* __restrict__ rstd, float* __restrict__ scale,
                                                             float* __restrict__ shift, int64_t* __restrict__ nbt) {
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) ++*nbt;  // BatchNorm2d.num_batches_tracked (one launch less)
  __shared__ double red[BT / 64][2];
  const int c = blockIdx.x;  // one channel per block, its partials over the block's 4 waves
  double s1, s2;
  block_sum2(part, nblk, C, c, s1, s2, red);
  if (threadIdx.x != 0) return;
  const double mu = s1 / M;
  double var = s2 / M - mu * mu;
  if (var < 0.0) var = 0.0;
  const float r = (float)(1.0 / sqrt(var + (double)eps));
  const float g = bf2f(gamma[c]), bta = bf2f(beta[c]);
  mean[c] = (float)mu;
  rstd[c] = r;
  scale[c] = g * r;
  shift[c] = bta - (float)mu * (g * r);  // bit-identical to the backward's recomputed ReLU mask
  if (rmean) {
    const double unb = M > 1 ? var * M / (M - 1) : var;
    rmean[c] = f2bf((1.f - momentum) * bf2f(rmean[c]) + momentum * (float)mu);
    rvar[c] = f2bf((1.f - momentum) * bf2f(rvar[c]) + momentum * (float)unb);
  }
}

// y = relu?(x * scale + shift (+ res)), 8 channels per thread, grid-stride. The block size (and so
// the grid stride) is a multiple of C / 8 (apply_threads), so a thread's channel group never changes: the folded
// coefficients live in registers and the loop is a pure 16 B-per-tensor stream (the first version
// re-loaded them per element and ran at ~1.6 TB/s).
template <bool RES, bool RELU>
__global__ void __launch_bounds__(BT) bn_apply_kernel(const u16* __restrict__ x, const u16* __restrict__ res,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      int64_t n8, int C, u16* __restrict__ y) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = 8 * (threadIdx.x % (C / 8));
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c0 + e];
    sh[e] = shift[c0 + e];
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = i0; i < n8; i += stride) {
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[i];
    u16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (RES) rv = reinterpret_cast<const u16x8*>(res)[i];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = fmaf(bf2f(xv[e]), sc[e], sh[e]);
      if (RES) v += bf2f(rv[e]);
      if (RELU) v = fmaxf(v, 0.f);
      o[e] = f2bf(v);
    }
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

// per channel: dbeta = sum g, dgamma = sum g*xhat (added into the bf16 grads), and the folded
// input-gradient coefficients dx = a * (g - mg) + b * (x - mean) with a = gamma * rstd,
// b = -a * rstd * mean(g * xhat)
__global__ void __launch_bounds__(BT) bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C, int M,
                                                             const float* __restrict__ rstd,
                                                             const u16* __restrict__ gamma, u16* __restrict__ ggamma,
                                                             u16* __restrict__ gbeta, float* __restrict__ coef) {
  __shared__ double red[BT / 64][2];
  const int c = blockIdx.x;  // one channel per block (block_sum2)
  double s1, s2;
  block_sum2(part, nblk, C, c, s1, s2, red);
  if (threadIdx.x != 0) return;
  const float a = bf2f(gamma[c]) * rstd[c];
  coef[c] = a;
  coef[C + c] = (float)(s1 / M);
  coef[2 * C + c] = -a * rstd[c] * (float)(s2 / M);
  if (gbeta) gbeta[c] = f2bf(bf2f(gbeta[c]) + (float)s1);
  if (ggamma) ggamma[c] = f2bf(bf2f(ggamma[c]) + (float)s2);
}

// dx = a * (g - mg) + b * (x - mean); dres = g (optional). Coefficients in registers (see apply);
// RELU as in bn_partial_kernel (2: the mask from x, with the forward's folded scale/shift)
template <int RELU, bool DRES>
__global__ void __launch_bounds__(BT) bn_bwd_apply_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                          const u16* __restrict__ y, const float* __restrict__ mean,
                                                          const float* __restrict__ coef, const u16* __restrict__ gamma,
                                                          const u16* __restrict__ beta, int64_t n8, int C,
                                                          u16* __restrict__ dx, u16* __restrict__ dres) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = 8 * (threadIdx.x % (C / 8));
  float ca[8], cm[8], cb[8], mu[8], fs[8], fh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ca[e] = coef[c0 + e];
    cm[e] = coef[C + c0 + e];
    cb[e] = coef[2 * C + c0 + e];
    mu[e] = mean[c0 + e];
    if (RELU == 2) {  // a = gamma * rstd is the forward scale
      fs[e] = ca[e];
      fh[e] = bf2f(beta[c0 + e]) - mu[e] * ca[e];
    }
  }
  (void)gamma;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = i0; i < n8; i += stride) {
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[i];
    const u16x8 gv = reinterpret_cast<const u16x8*>(dy)[i];
    u16x8 yv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (RELU == 1) yv = reinterpret_cast<const u16x8*>(y)[i];
    u16x8 o, og;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float g = bf2f(gv[e]);
      if (RELU == 1 && !(bf2f(yv[e]) > 0.f)) g = 0.f;
      if (RELU == 2 && !(fmaf(bf2f(xv[e]), fs[e], fh[e]) > 0.f)) g = 0.f;
      o[e] = f2bf(fmaf(ca[e], g - cm[e], cb[e] * (bf2f(xv[e]) - mu[e])));
      og[e] = f2bf(g);
    }
    reinterpret_cast<u16x8*>(dx)[i] = o;
    if (DRES) reinterpret_cast<u16x8*>(dres)[i] = og;
  }
}

int bn_blocks(int M, int C, int* rpb) {
  // one partial row per block, at most 512 of them (>= 2 blocks per CU for the streaming pass)
  int blocks = std::min(512, std::max(1, M / 64));
  *rpb = (M + blocks - 1) / blocks;
  blocks = (M + *rpb - 1) / *rpb;
  return blocks;
}

// largest multiple of the channel-group count C / 8 that fits a BT-thread block
int apply_threads(int C) { return (BT / (C / 8)) * (C / 8); }
int elem_blocks(int64_t n8, int nt) { return (int)std::min<int64_t>((n8 + nt - 1) / nt, 8192); }

void launch_apply(const void* x, const void* res, const float* scale, const float* shift, int64_t n8, int C, bool relu,
                  void* y, hipStream_t stream) {
  const dim3 g(elem_blocks(n8, apply_threads(C))), b(apply_threads(C));
  const u16 *xp = static_cast<const u16*>(x), *rp = static_cast<const u16*>(res);
  u16* yp = static_cast<u16*>(y);
  if (res && relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), g, b, 0, stream, xp, rp, scale, shift, n8, C, yp);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<true, false>), g, b, 0, stream, xp, rp, scale, shift, n8, C, yp);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), g, b, 0, stream, xp, rp, scale, shift, n8, C, yp);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, false>), g, b, 0, stream, xp, rp, scale, shift, n8, C, yp);
}

}  // namespace

bool bn_nhwc_supported(int C) { return C % 8 == 0 && C >= 8 && C <= 2048; }

size_t bn_nhwc_workspace_floats(int M, int C) {
  int rpb;
  return (size_t)bn_blocks(M, C, &rpb) * 2 * C + 8 * (size_t)C;
}

void bn_nhwc_fwd_bf16(const void* x, const void* res, const void* gamma, const void* beta, void* rmean, void* rvar,
                      int M, int C, float eps, float momentum, bool relu, void* y, float* mean, float* rstd,
                      float* workspace, hipStream_t stream, int64_t* num_batches_tracked, const float* part_in,
                      int part_rows) {
  int rpb;
  int nblk = bn_blocks(M, C, &rpb);
  const float* part = workspace;
  float* scale = workspace + (size_t)nblk * 2 * C;
  float* shift = scale + C;
  if (part_in) {  // the producing convolution's epilogue already summed y per tile (conv_bf16.hip)
    part = part_in;
    nblk = part_rows;
  } else {
    hipLaunchKernelGGL(bn_partial_kernel<false>, dim3(nblk), dim3(BT), 0, stream, static_cast<const u16*>(x), nullptr,
                       nullptr, nullptr, nullptr, nullptr, nullptr, M, C, rpb, 0, workspace);
  }
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(C), dim3(BT), 0, stream, part, nblk, C, M, eps,
                     momentum, static_cast<const u16*>(gamma), static_cast<const u16*>(beta), static_cast<u16*>(rmean),
                     static_cast<u16*>(rvar), mean, rstd, scale, shift, num_batches_tracked);
  const int64_t n8 = (int64_t)M * C / 8;
  launch_apply(x, res, scale, shift, n8, C, relu, y, stream);
}

void bn_nhwc_bwd_bf16(const void* x, const void* dy, const void* y, const float* mean, const float* rstd,
                      const void* gamma, int M, int C, bool relu, void* dx, void* dres, void* ggamma, void* gbeta,
                      float* workspace, hipStream_t stream, const void* beta, const float* part_in, int part_rows) {
  int rpb;
  int nblk = bn_blocks(M, C, &rpb);
  const float* part = workspace;
  float* coef = workspace + (size_t)nblk * 2 * C;  // [3][C]
  // ReLU mask: from y when given, else recomputed from x (needs beta; BatchNorm + ReLU, no residual)
  const int rmode = !relu ? 0 : (y ? 1 : 2);
  const u16 *gp = static_cast<const u16*>(gamma), *bp = static_cast<const u16*>(beta);
  if (part_in) {  // the convolution that produced dy summed g and g * xhat per tile (conv_bf16.hip BnBack)
    part = part_in;
    nblk = part_rows;
  } else {
    hipLaunchKernelGGL(bn_partial_kernel<true>, dim3(nblk), dim3(BT), 0, stream, static_cast<const u16*>(x),
                       static_cast<const u16*>(dy), static_cast<const u16*>(y), mean, rstd, gp, bp, M, C, rpb, rmode,
                       workspace);
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(BT), 0, stream, part, nblk, C, M,
                     rstd, gp, static_cast<u16*>(ggamma), static_cast<u16*>(gbeta), coef);
  const int64_t n8 = (int64_t)M * C / 8;
  const dim3 g(elem_blocks(n8, apply_threads(C))), b(apply_threads(C));
  const u16 *xp = static_cast<const u16*>(x), *dyp = static_cast<const u16*>(dy), *yp = static_cast<const u16*>(y);
  u16 *dxp = static_cast<u16*>(dx), *drp = static_cast<u16*>(dres);
#define BNB(R, D) \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<R, D>), g, b, 0, stream, xp, dyp, yp, mean, coef, gp, bp, n8, C, dxp, drp)
  if (rmode == 1 && dres) BNB(1, true);
  else if (rmode == 1) BNB(1, false);
  else if (rmode == 2 && dres) BNB(2, true);
  else if (rmode == 2) BNB(2, false);
  else if (dres) BNB(0, true);
  else BNB(0, false);
#undef BNB
}

// eval mode: y = relu?(x * scale + shift (+ res)) from the running statistics
void bn_nhwc_eval_bf16(const void* x, const void* res, const float* scale, const float* shift, int M, int C, bool relu,
                       void* y, hipStream_t stream) {
  const int64_t n8 = (int64_t)M * C / 8;
  launch_apply(x, res, scale, shift, n8, C, relu, y, stream);
}

}  // namespace sdml
