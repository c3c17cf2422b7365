// The whole training step of the 784-128-10 MLP at the reference's batch sizes (B <= 128; the
// reference trains at B = 60: /root/reference/simple_distributed.py:18) as TWO launches: stage 0
// forward, stage 1 forward + log_softmax + NLL + backward, stage 0 backward and the SGD update of all
// four parameter tensors (:63-64, :75-79, :111-113). At this size every kernel is a few microseconds
// of work and the multi-kernel step (6 launches + the host work between them) is launch-bound:
//
//   kernel A (block g owns hidden units 2g, 2g+1; 64 blocks): h[:, own] = relu(x W1[own]^T + b1[own])
//   kernel B (every block, redundantly): logits of all rows from the full h (one thread per (row, class)
//            dot product), log_softmax, NLL,
//            dl = scale (softmax - onehot) (identical bits in every block: same operations, same order)
//            own part: dz = (dl W2[:, own]) * (h > 0); gW1[own] = dz^T x; gb1[own]; gW2[:, own]; block 0:
//            gb2, loss, correct; then torch.optim.SGD's update of exactly the parameters the block owns
//            (sgd_rule.h's fma sequence per element). W2 / b2 are read into LDS before a __syncthreads
//            that precedes every update, and no block reads another block's updated parameters.
// (A first version ran both phases in one cooperative launch with a grid barrier: 29.6 us of kernel
// time, but the cooperative launch API alone held the step at ~50 us of host time.)
// fp32 throughout (VALU fmas, fixed summation orders: deterministic). The flat gradient buffer is not
// touched: the gradients are consumed where they are produced (it stays zero, as after a fused
// zero_grad step).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

namespace sdml {
namespace {

constexpr int SK = 784, SH = 128, SC = 10;
constexpr int ST = 1024;           // threads per block (16 waves: rows spread over more waves)
constexpr int SG = SH / 2;         // blocks: 2 hidden units each
constexpr int SMAXB = 128;         // rows

struct SmallArgs {
  const void* x;  // [B][784] fp32 pixels, or uint8 (x8 = 1; scaled by 1/255)
  int x8;
  const int64_t* target;
  int B;
  float scale;
  float* w1;  // [128][784]
  float* b1;
  float* w2;  // [10][128]
  float* b2;
  float* m1;  // momentum buffers aligned with the parameters (null without momentum)
  float* mb1;
  float* m2;
  float* mb2;
  float lr, mom, damp, wd;
  int nesterov, first;
  float* h;      // scratch [B][128]
  float* snap;   // scratch [10 * 128 + 10]: W2 and b2 as kernel B must read them (before any update)
  float* stats;  // [2] loss sum, correct (overwritten)
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// X8 is a template parameter: a runtime "uint8 or float" select inside the unrolled load batches makes
// hipcc branch around every load and wait for each one (no loads in flight)
template <bool X8>
__device__ __forceinline__ float xval(const SmallArgs& a, int b, int k) {
  if constexpr (X8) return static_cast<float>(static_cast<const unsigned char*>(a.x)[(size_t)b * SK + k]) * (1.f / 255.f);
  else return static_cast<const float*>(a.x)[(size_t)b * SK + k];
}

// torch.optim.SGD on one parameter, with sgd_rule.h's operation sequence (explicit fmas)
__device__ __forceinline__ void sgd1(float* p, float* buf, float d, const SmallArgs& a) {
#pragma clang fp contract(off)
  const float pv = *p;
  if (a.wd != 0.f) d = __builtin_fmaf(a.wd, pv, d);
  if (a.mom != 0.f) {
    const float b = a.first ? d : __builtin_fmaf(a.mom, *buf, (1.f - a.damp) * d);
    *buf = b;
    d = a.nesterov ? __builtin_fmaf(a.mom, b, d) : b;
  }
  *p = __builtin_fmaf(-a.lr, d, pv);
}

template <bool X8>
__global__ void __launch_bounds__(ST) mlp_small_fwd_kernel(SmallArgs a) {
  __shared__ float w1s[2][SK];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int j0 = 2 * blockIdx.x;
  const int B = a.B;
  {  // (both loads per thread issued before the stores)
    float wv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = min(t + ST * u, 2 * SK - 1);
      wv[u] = a.w1[(size_t)(j0 + i / SK) * SK + i % SK];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (t + ST * u < 2 * SK) w1s[(t + ST * u) / SK][(t + ST * u) % SK] = wv[u];
  }
  const float bj0 = a.b1[j0], bj1 = a.b1[j0 + 1];
  // snapshot of W2 / b2 for kernel B: its blocks update W2's columns (and block 0 b2) while other blocks
  // may still be starting, so they read the values of this step from here (stream order: A before B)
  if (t < 2 * SC) a.snap[(t >> 1) * SH + j0 + (t & 1)] = a.w2[(t >> 1) * SH + j0 + (t & 1)];
  if (blockIdx.x == 0 && t >= 64 && t < 64 + SC) a.snap[SC * SH + t - 64] = a.b2[t - 64];
  __syncthreads();
  for (int b = wave; b < B; b += ST / 64) {
    // the row's 13 loads are issued together (fully unrolled, the partial 13th masked)
    float xv[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) xv[i] = (lane + 64 * i < SK) ? xval<X8>(a, b, lane + 64 * i) : 0.f;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const int k = min(lane + 64 * i, SK - 1);
      s0 = __builtin_fmaf(xv[i], w1s[0][k], s0);
      s1 = __builtin_fmaf(xv[i], w1s[1][k], s1);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
      a.h[(size_t)b * SH + j0] = fmaxf(s0 + bj0, 0.f);
      a.h[(size_t)b * SH + j0 + 1] = fmaxf(s1 + bj1, 0.f);
    }
  }
}

template <bool X8>
__global__ void __launch_bounds__(ST) mlp_small_bwd_kernel(SmallArgs a) {
  __shared__ float w2s[SC][SH + 1];  // padded: the (row, class) threads of a wave read 10 rows of it at once
  __shared__ float b2s[SC];
  __shared__ float hs[SMAXB][SH + 1];
  __shared__ float dls[SMAXB][SC];
  __shared__ float dzs[SMAXB][2];
  __shared__ float zs[SMAXB][SC];
  __shared__ float rowl[SMAXB][2];
  const int t = threadIdx.x;
  const int j0 = 2 * blockIdx.x;
  const int B = a.B;
  // staging: 8 loads per thread in flight per round (clamped index, stored only when in range); a plain
  // strided copy loop waited out each load before the next (8 serial round trips for h at B = 60)
  {
    float wv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) wv[u] = a.snap[min(t + ST * u, SC * SH - 1)];
    const float bv = t < SC ? a.snap[SC * SH + t] : 0.f;
    const int n = B * SH;
    for (int i0 = t; i0 < n; i0 += 8 * ST) {
      float hv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) hv[u] = a.h[min(i0 + ST * u, n - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + ST * u < n) hs[(i0 + ST * u) / SH][(i0 + ST * u) % SH] = hv[u];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (t + ST * u < SC * SH) w2s[(t + ST * u) / SH][(t + ST * u) % SH] = wv[u];
    if (t < SC) b2s[t] = bv;
  }
  __syncthreads();
  // logits: one (row, class) dot product of length 128 per thread (no cross-lane reductions on the
  // critical path), then one thread per row: log_softmax, NLL, argmax, dl
  for (int i = t; i < B * SC; i += ST) {
    const int b = i / SC, c = i % SC;
    float p = b2s[c];
#pragma unroll 16
    for (int k = 0; k < SH; ++k) p = __builtin_fmaf(hs[b][k], w2s[c][k], p);
    zs[b][c] = p;
  }
  __syncthreads();
  if (t < B) {
    const int b = t;
    float z[SC];
#pragma unroll
    for (int c = 0; c < SC; ++c) z[c] = zs[b][c];
    float mx = z[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < SC; ++c)
      if (z[c] > mx) {
        mx = z[c];
        am = c;
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < SC; ++c) se += __expf(z[c] - mx);
    const float lse = mx + __logf(se);
    const int tg = (int)a.target[b];
    float zt = 0.f;
#pragma unroll
    for (int c = 0; c < SC; ++c) zt = c == tg ? z[c] : zt;
    rowl[b][0] = lse - zt;
    rowl[b][1] = am == tg ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < SC; ++c) dls[b][c] = a.scale * (__expf(z[c] - lse) - (c == tg ? 1.f : 0.f));
  }
  __syncthreads();
  if (blockIdx.x == 0 && t == 0) {  // loss sum and correct count, in row order
    float l = 0.f, c = 0.f;
    for (int b = 0; b < B; ++b) {
      l += rowl[b][0];
      c += rowl[b][1];
    }
    a.stats[0] = l;
    a.stats[1] = c;
  }
  // dz of the own hidden units (the ReLU backward from h > 0)
  for (int i = t; i < 2 * B; i += ST) {
    const int b = i >> 1, jj = i & 1;
    float d = 0.f;
#pragma unroll
    for (int c = 0; c < SC; ++c) d = __builtin_fmaf(dls[b][c], w2s[c][j0 + jj], d);
    dzs[b][jj] = hs[b][j0 + jj] > 0.f ? d : 0.f;
  }
  __syncthreads();
  // gW1[own rows] = dz^T x, then the update of those rows (each element by the thread that reduced it)
  for (int k = t; k < SK; k += ST) {
    float g0 = 0.f, g1 = 0.f;
    for (int b = 0; b < B; b += 32) {
      // 32 unconditional loads in flight (ragged-tail rows clamped to row B - 1, their terms skipped),
      // then the fmas in row order
      float xv[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) xv[u] = xval<X8>(a, min(b + u, B - 1), k);
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        if (b + u < B) {
          g0 = __builtin_fmaf(dzs[b + u][0], xv[u], g0);
          g1 = __builtin_fmaf(dzs[b + u][1], xv[u], g1);
        }
      }
    }
    const size_t o0 = (size_t)j0 * SK + k, o1 = o0 + SK;
    sgd1(a.w1 + o0, a.m1 ? a.m1 + o0 : nullptr, g0, a);
    sgd1(a.w1 + o1, a.m1 ? a.m1 + o1 : nullptr, g1, a);
  }
  if (t < 2) {  // gb1[own]
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += dzs[b][t];
    sgd1(a.b1 + j0 + t, a.mb1 ? a.mb1 + j0 + t : nullptr, g, a);
  } else if (t >= 64 && t < 64 + 2 * SC) {  // gW2[:, own]
    const int c = (t - 64) >> 1, jj = (t - 64) & 1;
    float g = 0.f;
    for (int b = 0; b < B; ++b) g = __builtin_fmaf(dls[b][c], hs[b][j0 + jj], g);
    const size_t o = (size_t)c * SH + j0 + jj;
    sgd1(a.w2 + o, a.m2 ? a.m2 + o : nullptr, g, a);
  } else if (blockIdx.x == 0 && t >= 128 && t < 128 + SC) {  // gb2
    const int c = t - 128;
    float g = 0.f;
    for (int b = 0; b < B; ++b) g += dls[b][c];
    sgd1(a.b2 + c, a.mb2 ? a.mb2 + c : nullptr, g, a);
  }
}

}  // namespace

int mlp_small_step_max_batch() { return SMAXB; }

bool mlp_small_step(const void* x, bool x_u8, const int64_t* target, int B, float scale, float* w1, float* b1,
                    float* w2, float* b2, float* m1, float* mb1, float* m2, float* mb2, float lr, float mom,
                    float damp, float wd, bool nesterov, bool first, float* h_scratch, float* snap_scratch,
                    float* stats, hipStream_t stream) {
  if (B < 1 || B > SMAXB) return false;
  SmallArgs a;
  a.x = x;
  a.x8 = x_u8 ? 1 : 0;
  a.target = target;
  a.B = B;
  a.scale = scale;
  a.w1 = w1;
  a.b1 = b1;
  a.w2 = w2;
  a.b2 = b2;
  a.m1 = m1;
  a.mb1 = mb1;
  a.m2 = m2;
  a.mb2 = mb2;
  a.lr = lr;
  a.mom = mom;
  a.damp = damp;
  a.wd = wd;
  a.nesterov = nesterov ? 1 : 0;
  a.first = first ? 1 : 0;
  a.h = h_scratch;
  a.snap = snap_scratch;
  a.stats = stats;
  if (x_u8) {
    hipLaunchKernelGGL(mlp_small_fwd_kernel<true>, dim3(SG), dim3(ST), 0, stream, a);
    hipLaunchKernelGGL(mlp_small_bwd_kernel<true>, dim3(SG), dim3(ST), 0, stream, a);
  } else {
    hipLaunchKernelGGL(mlp_small_fwd_kernel<false>, dim3(SG), dim3(ST), 0, stream, a);
    hipLaunchKernelGGL(mlp_small_bwd_kernel<false>, dim3(SG), dim3(ST), 0, stream, a);
  }
  return true;
}

}  // namespace sdml
