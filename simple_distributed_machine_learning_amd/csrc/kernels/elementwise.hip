// Bandwidth-bound kernels: fused SGD-momentum over the flat parameter buffer, and the
// on-device synthetic MNIST-shape data generator.
#include <hip/hip_runtime.h>

#include <hip/hip_bf16.h>

#include "kernels.h"
#include "synth_hash.h"
#include "sgd_rule.h"
#include "u8_planes.h"

namespace sdml {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// torch.optim.SGD semantics (reference DistributedOptimizer(optim.SGD, lr, momentum),
// /root/reference/simple_distributed.py:100-104): d = g + wd*p; buf = first ? d :
// momentum*buf + (1-dampening)*d; d = nesterov ? d + momentum*buf : buf; p -= lr*d.
// One launch for all parameters of all stages a rank owns; 16 B per lane per stream.
typedef unsigned short u16x4s __attribute__((ext_vector_type(4)));

// pl: optional weight-plane cache written from the UPDATED weights (the uint8 first layer's
// forward reads W as zero-padded fp16 planes [2][rows][Kp], u8_planes.h - the same function as
// mlp_u8.hip's split kernel, so both writers agree bit for bit; writing them here saves a separate
// split launch per step). pl.n4 float4 of the flat buffer starting at float4 pl.off4 form a
// [rows][K] matrix, K % 4 == 0.
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, float* __restrict__ g,
                                                  float* __restrict__ buf, int64_t n4, float lr, float mom,
                                                  float damp, float wd, int nesterov, int first, int zero_grad,
                                                  SgdPlanes pl) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const SgdRule rule{lr, mom, damp, wd, nesterov, first};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 d = reinterpret_cast<const f32x4*>(g)[i];
    if (zero_grad) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 nv = sgd_update4(p + 4 * i, buf + 4 * i, d, rule);
    if (pl.planes && i >= pl.off4 && i < pl.off4 + pl.n4) {
      const int64_t e = 4 * (i - pl.off4);
      const int64_t r = e / pl.K, k = e % pl.K;
      sgd_write_planes4(pl.planes + r * pl.Kp + k, pl.plane_stride, nv);
    }
  }
}

// Mixed precision: fp32 master weights + momentum, bf16 gradients in, bf16 model weights out
// (round-to-nearest-even via the hardware cvt). One pass: 2 B (g) + 8 B (master) + 8 B (buf)
// read/written + 2 B (p) written per element; 8 elements per lane so every stream moves 16 B per
// access (the 4-element form wrote the bf16 weights 2 B at a time: 3.3 TB/s on GPT-2's 124 M).
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ float bf16_to_f32(unsigned short v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f));
}

// one 8-element chunk i: loads (issued by the caller before any use), then the update and its stores
struct MixedIn {
  f32x4 mv[2], bo[2];
  u16x8 gr;
};

// (plain loads: nontemporal loads measured 2x slower on this stream, round 3 tools/probes/sgd_nt_ab.py)
__device__ __forceinline__ MixedIn mixed_load(const float* master, const unsigned short* g, const float* buf, int64_t i,
                                              bool use_buf) {
  MixedIn in;
  const f32x4* m4 = reinterpret_cast<const f32x4*>(master) + 2 * i;
  const f32x4* b4 = reinterpret_cast<const f32x4*>(buf) + 2 * i;
  in.mv[0] = m4[0];
  in.mv[1] = m4[1];
  in.gr = *(reinterpret_cast<const u16x8*>(g) + i);
  if (use_buf) {
    in.bo[0] = b4[0];
    in.bo[1] = b4[1];
  }
  return in;
}

template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, const T& v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT>
__device__ __forceinline__ void mixed_update(MixedIn in, float* master, unsigned short* p, unsigned short* g,
                                             float* buf, int64_t i, float lr, float mom, float damp, float wd,
                                             int nesterov, int first, int zero_grad) {
  if (zero_grad) st<NT>(reinterpret_cast<u16x8*>(g) + i, u16x8{0, 0, 0, 0, 0, 0, 0, 0});
  u16x8 po;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 d = {bf16_to_f32(in.gr[4 * h]), bf16_to_f32(in.gr[4 * h + 1]), bf16_to_f32(in.gr[4 * h + 2]),
               bf16_to_f32(in.gr[4 * h + 3])};
    if (wd != 0.f) d += wd * in.mv[h];
    if (mom != 0.f) {
      const f32x4 b = first ? d : mom * in.bo[h] + (1.f - damp) * d;
      st<NT>(reinterpret_cast<f32x4*>(buf) + 2 * i + h, b);
      d = nesterov ? d + mom * b : b;
    }
    in.mv[h] = in.mv[h] - lr * d;
    st<NT>(reinterpret_cast<f32x4*>(master) + 2 * i + h, in.mv[h]);
#pragma unroll
    for (int e = 0; e < 4; ++e) po[4 * h + e] = f32_to_bf16(in.mv[h][e]);
  }
  st<NT>(reinterpret_cast<u16x8*>(p) + i, po);
}

// V = 0: one chunk per loop trip; V = 1: two chunks (i, i + stride) per trip, both chunks' loads issued before either
// update; V = 2: one chunk, nontemporal stores. Same arithmetic, bit-identical results.
template <int V>
__global__ void __launch_bounds__(256) sgd_mixed_kernel(float* __restrict__ master, unsigned short* __restrict__ p,
                                                        unsigned short* __restrict__ g, float* __restrict__ buf,
                                                        int64_t n8, float lr, float mom, float damp, float wd,
                                                        int nesterov, int first, int zero_grad) {
  constexpr bool NT = V == 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool use_buf = mom != 0.f && !first;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (V == 1) {
    for (; i + stride < n8; i += 2 * stride) {
      const MixedIn a = mixed_load(master, g, buf, i, use_buf);
      const MixedIn b = mixed_load(master, g, buf, i + stride, use_buf);
      mixed_update<NT>(a, master, p, g, buf, i, lr, mom, damp, wd, nesterov, first, zero_grad);
      mixed_update<NT>(b, master, p, g, buf, i + stride, lr, mom, damp, wd, nesterov, first, zero_grad);
    }
  }
  for (; i < n8; i += stride)
    mixed_update<NT>(mixed_load(master, g, buf, i, use_buf), master, p, g, buf, i, lr, mom, damp, wd, nesterov,
                     first, zero_grad);
}

__global__ void __launch_bounds__(256) synth_kernel(uint64_t seed, int64_t start, int64_t n, int H, int W, int mode,
                                                    float* __restrict__ x, int64_t* __restrict__ y) {
  const int D = H * W;
  const int64_t total = n * D;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t s = i / D;
    int pix = (int)(i - s * D);
    uint64_t smp = (uint64_t)(start + s);
    x[i] = synth_pixel(seed, smp, pix, H, W, mode);
    if (pix == 0 && y) y[s] = synth_label(seed, smp);
  }
}

}  // namespace

void sgd_momentum(float* p, float* g, float* buf, int64_t n, float lr, float momentum, float dampening,
                  float wd, bool nesterov, bool first, bool zero_grad, hipStream_t stream, SgdPlanes planes) {
  // flat buffers are padded to 64 elements, so n is a multiple of 4
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p, g, buf, n4, lr, momentum, dampening,
                     wd, nesterov ? 1 : 0, first ? 1 : 0, zero_grad ? 1 : 0, planes);
}

void sgd_momentum_mixed(float* master, void* p_bf16, void* g_bf16, float* buf, int64_t n, float lr, float momentum,
                        float dampening, float wd, bool nesterov, bool first, bool zero_grad, hipStream_t stream) {
  // flat buffers are padded to 64 elements, so n is a multiple of 8
  const int64_t n8 = n / 8;
  int64_t blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const int v = knob(KNOB_SGD_MIXED_V);
  auto* k = v == 1 ? sgd_mixed_kernel<1> : v == 2 ? sgd_mixed_kernel<2> : sgd_mixed_kernel<0>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), 0, stream, master, static_cast<unsigned short*>(p_bf16),
                     static_cast<unsigned short*>(g_bf16), buf, n8, lr, momentum, dampening, wd, nesterov ? 1 : 0,
                     first ? 1 : 0, zero_grad ? 1 : 0);
}

void synth_mnist(uint64_t seed, int64_t start, int64_t n, int H, int W, int mode, float* x, int64_t* y,
                 hipStream_t stream) {
  if (n <= 0) return;
  int64_t total = n * H * W;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, seed, start, n, H, W, mode, x, y);
}

}  // namespace sdml
