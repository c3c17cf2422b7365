// The reference CNN's two pipeline stages as fused gfx950 kernels
// (/root/reference/simple_distributed.py:26-80).
//
// Stage 0 (Network1): conv1(1->10,k5) -> maxpool2 -> relu -> conv2(10->20,k5) -> Dropout2d(p)
//                     -> maxpool2 -> relu -> flatten(320)
//   * cnn_s0_fwd: ONE launch, one workgroup per sample; the image, both filter banks and the
//     12x12 intermediate live in LDS; pooling, ReLU and the per-(sample, channel) dropout mask
//     are fused into the convolution loops (the pool is evaluated on the fly: each pooled output
//     computes its 2x2 conv window and keeps the max).
//   * cnn_s0_bwd: ONE launch; recomputes the (cheap) forward in LDS, routes the incoming
//     gradient through ReLU / max-pool argmax / dropout, and accumulates dW2, db2, dW1, db1
//     (no dX: the first stage's input is data). Per-block partials go out as one fp32 atomic per
//     weight per block (60 blocks at the reference batch).
// Stage 1 (Network2): fc1(320->50) -> relu -> dropout(p) -> fc2(50->10) -> log_softmax -> NLL
//   * cnn_s1: ONE launch for forward, loss/accuracy and the whole backward (dX, dW1, db1, dW2,
//     db2); each workgroup handles up to 64 samples, keeps their inputs and dh in LDS and
//     reduces dW1 = dh^T x over them before a single atomic per weight.
// Dropout masks come from a counter hash of (seed, sample, unit): the backward regenerates the
// forward's mask exactly, nothing is stored. At batch 60 these layers are launch-bound, so the
// design goal is the minimum number of launches per step (3 + the optimizer), not MFMA use.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdml {
namespace {

constexpr int IMG = 28, KS = 5, C1 = 10, O1 = 24, P1 = 12, C2 = 20, O2 = 8, P2 = 4;
constexpr int FLAT = C2 * P2 * P2;  // 320
constexpr int HID = 50, NCLS = 10;
constexpr int T = 256;

__device__ __forceinline__ unsigned drop_hash(unsigned long long seed, unsigned a, unsigned b) {
  unsigned long long x = seed ^ (0x9E3779B97F4A7C15ull * (a + 1)) ^ (0xC2B2AE3D27D4EB4Full * (b + 7));
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return (unsigned)x;
}
__device__ __forceinline__ float keep_scale(unsigned long long seed, unsigned a, unsigned b, float p) {
  if (p <= 0.f) return 1.f;
  float u = (float)(drop_hash(seed, a, b) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

struct S0Smem {
  float x[IMG * IMG];
  float w1[C1 * KS * KS];
  float b1[C1];
  float w2[C2 * C1 * KS * KS];
  float b2[C2];
  float z1[C1 * P1 * P1];      // relu(maxpool(conv1))
  float dsc[C2];               // dropout2d scale per channel
  unsigned char a1[C1 * P1 * P1];
  unsigned char a2[FLAT];
  float m2[FLAT];              // pre-relu pooled conv2 value (after dropout)
};

__device__ void s0_load(S0Smem& s, const float* x, const float* w1, const float* b1, const float* w2,
                        const float* b2) {
  for (int i = threadIdx.x; i < IMG * IMG; i += T) s.x[i] = x[i];
  for (int i = threadIdx.x; i < C1 * KS * KS; i += T) s.w1[i] = w1[i];
  for (int i = threadIdx.x; i < C2 * C1 * KS * KS; i += T) s.w2[i] = w2[i];
  if (threadIdx.x < C1) s.b1[threadIdx.x] = b1[threadIdx.x];
  if (threadIdx.x < C2) s.b2[threadIdx.x] = b2[threadIdx.x];
}

// forward into LDS (z1, a1, a2, m2); returns nothing, out written by caller from m2
__device__ void s0_forward(S0Smem& s, unsigned long long seed, unsigned sample, float p, bool drop) {
  if (threadIdx.x < C2) s.dsc[threadIdx.x] = drop ? keep_scale(seed, sample, threadIdx.x, p) : 1.f;
  for (int o = threadIdx.x; o < C1 * P1 * P1; o += T) {
    const int c = o / (P1 * P1), py = (o / P1) % P1, px = o % P1;
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y0 = 2 * py + (d >> 1), x0 = 2 * px + (d & 1);
      float acc = s.b1[c];
#pragma unroll
      for (int ky = 0; ky < KS; ++ky)
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) acc += s.w1[(c * KS + ky) * KS + kx] * s.x[(y0 + ky) * IMG + x0 + kx];
      if (acc > best) {
        best = acc;
        arg = d;
      }
    }
    s.z1[o] = fmaxf(best, 0.f);
    s.a1[o] = (unsigned char)arg;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < FLAT; o += T) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    const float sc = s.dsc[c];
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int y0 = 2 * py + (d >> 1), x0 = 2 * px + (d & 1);
      float acc = s.b2[c];
      for (int ci = 0; ci < C1; ++ci)
#pragma unroll
        for (int ky = 0; ky < KS; ++ky)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx)
            acc += s.w2[((c * C1 + ci) * KS + ky) * KS + kx] * s.z1[(ci * P1 + y0 + ky) * P1 + x0 + kx];
      const float v = acc * sc;  // Dropout2d before the pool (reference order, :45)
      if (v > best) {
        best = v;
        arg = d;
      }
    }
    s.m2[o] = best;
    s.a2[o] = (unsigned char)arg;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(T) cnn_s0_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, float* __restrict__ out,
                                                       unsigned long long seed, unsigned sample0, float p, int drop) {
  __shared__ S0Smem s;
  const int n = blockIdx.x;
  s0_load(s, x + (size_t)n * IMG * IMG, w1, b1, w2, b2);
  __syncthreads();
  s0_forward(s, seed, sample0 + n, p, drop != 0);
  for (int o = threadIdx.x; o < FLAT; o += T) out[(size_t)n * FLAT + o] = fmaxf(s.m2[o], 0.f);
}

__global__ void __launch_bounds__(T) cnn_s0_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, const float* __restrict__ gout,
                                                       unsigned long long seed, unsigned sample0, float p, int drop,
                                                       float* __restrict__ gw1, float* __restrict__ gb1,
                                                       float* __restrict__ gw2, float* __restrict__ gb2) {
  __shared__ S0Smem s;
  __shared__ float G2[C2 * O2 * O2];
  __shared__ float G1[C1 * O1 * O1];
  const int n = blockIdx.x;
  s0_load(s, x + (size_t)n * IMG * IMG, w1, b1, w2, b2);
  for (int i = threadIdx.x; i < C2 * O2 * O2; i += T) G2[i] = 0.f;
  for (int i = threadIdx.x; i < C1 * O1 * O1; i += T) G1[i] = 0.f;
  __syncthreads();
  s0_forward(s, seed, sample0 + n, p, drop != 0);
  // relu -> maxpool2 (argmax) -> dropout2d scale: gradient of the conv2 output
  for (int o = threadIdx.x; o < FLAT; o += T) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    const float g = s.m2[o] > 0.f ? gout[(size_t)n * FLAT + o] * s.dsc[c] : 0.f;
    const int d = s.a2[o];
    G2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)] = g;
  }
  __syncthreads();
  // dW2, db2
  for (int o = threadIdx.x; o < C2 * C1 * KS * KS; o += T) {
    const int c = o / (C1 * KS * KS), ci = (o / (KS * KS)) % C1, ky = (o / KS) % KS, kx = o % KS;
    float acc = 0.f;
    for (int y = 0; y < O2; ++y)
#pragma unroll
      for (int xx = 0; xx < O2; ++xx) acc += G2[(c * O2 + y) * O2 + xx] * s.z1[(ci * P1 + y + ky) * P1 + xx + kx];
    atomicAdd(gw2 + o, acc);
  }
  if (threadIdx.x < C2) {
    float acc = 0.f;
    for (int i = 0; i < O2 * O2; ++i) acc += G2[threadIdx.x * O2 * O2 + i];
    atomicAdd(gb2 + threadIdx.x, acc);
  }
  // dz1 -> relu mask -> maxpool1 argmax -> gradient of the conv1 output
  for (int o = threadIdx.x; o < C1 * P1 * P1; o += T) {
    if (s.z1[o] <= 0.f) continue;
    const int ci = o / (P1 * P1), yy = (o / P1) % P1, xx = o % P1;
    float acc = 0.f;
    for (int c = 0; c < C2; ++c)
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const int y = yy - ky;
        if (y < 0 || y >= O2) continue;
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const int xo = xx - kx;
          if (xo < 0 || xo >= O2) continue;
          acc += G2[(c * O2 + y) * O2 + xo] * s.w2[((c * C1 + ci) * KS + ky) * KS + kx];
        }
      }
    const int d = s.a1[o];
    G1[(ci * O1 + 2 * yy + (d >> 1)) * O1 + 2 * xx + (d & 1)] = acc;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < C1 * KS * KS; o += T) {
    const int c = o / (KS * KS), ky = (o / KS) % KS, kx = o % KS;
    float acc = 0.f;
    for (int y = 0; y < O1; ++y)
      for (int xx = 0; xx < O1; ++xx) acc += G1[(c * O1 + y) * O1 + xx] * s.x[(y + ky) * IMG + xx + kx];
    atomicAdd(gw1 + o, acc);
  }
  if (threadIdx.x < C1) {
    float acc = 0.f;
    for (int i = 0; i < O1 * O1; ++i) acc += G1[threadIdx.x * O1 * O1 + i];
    atomicAdd(gb1 + threadIdx.x, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// stage 1
constexpr int S1_ROWS = 64;
constexpr int XP1 = FLAT + 1;  // LDS pitch (odd: conflict-free column walks)

__global__ void __launch_bounds__(T) cnn_s1_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                   const float* __restrict__ b1, const float* __restrict__ w2,
                                                   const float* __restrict__ b2, const int64_t* __restrict__ tgt,
                                                   int B, unsigned long long seed, unsigned sample0, float p,
                                                   int drop, float scale, float* __restrict__ stats,
                                                   float* __restrict__ dx, float* __restrict__ gw1,
                                                   float* __restrict__ gb1, float* __restrict__ gw2,
                                                   float* __restrict__ gb2) {
  __shared__ float xs[S1_ROWS * XP1];
  __shared__ float dhs[S1_ROWS * HID];
  __shared__ float w2s[NCLS * HID];
  __shared__ float dsh[4][HID];
  __shared__ float lsh[4][NCLS];
  __shared__ float red[4][NCLS * HID + NCLS + 2];
  const int r0 = blockIdx.x * S1_ROWS;
  const int nr = min(S1_ROWS, B - r0);
  const bool train = dx != nullptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < nr * FLAT; i += T) xs[(i / FLAT) * XP1 + i % FLAT] = x[(size_t)r0 * FLAT + i];
  for (int i = threadIdx.x; i < NCLS * HID; i += T) w2s[i] = w2[i];
  __syncthreads();
  float gw2acc[NCLS];  // lane j < 50: dW2[c][j]
#pragma unroll
  for (int c = 0; c < NCLS; ++c) gw2acc[c] = 0.f;
  float gb2acc = 0.f, loss_acc = 0.f, ok_acc = 0.f;
  for (int rr = w; rr < nr; rr += 4) {
    const int n = r0 + rr;
    // fc1 + relu + dropout: lane j < 50
    float h = 0.f, ms = 0.f;
    if (lane < HID) {
      float acc = b1[lane];
      const float* wr = w1 + (size_t)lane * FLAT;
      for (int k = 0; k < FLAT; ++k) acc += wr[k] * xs[rr * XP1 + k];
      h = fmaxf(acc, 0.f);
      ms = drop ? keep_scale(seed, sample0 + n, lane, p) : 1.f;
      dsh[w][lane] = h * ms;
    }
    __builtin_amdgcn_wave_barrier();
    // fc2 + log_softmax: lane c < 10
    float z = -INFINITY;
    if (lane < NCLS) {
      float acc = b2[lane];
#pragma unroll 10
      for (int j = 0; j < HID; ++j) acc += w2s[lane * HID + j] * dsh[w][j];
      z = acc;
    }
    float mx = z;
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float e = lane < NCLS ? __expf(z - mx) : 0.f;
    float se = e;
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = mx + __logf(se);
    const int y = (int)tgt[n];
    // argmax (first max) among lanes 0..9
    unsigned long long bal = __ballot(lane < NCLS && z == mx);
    const int am = __ffsll((long long)bal) - 1;
    const float zy = __shfl(z, y);
    if (lane == 0) {
      loss_acc += lse - zy;
      ok_acc += (am == y) ? 1.f : 0.f;
    }
    if (!train) continue;
    const float dl = lane < NCLS ? scale * (__expf(z - lse) - (lane == y ? 1.f : 0.f)) : 0.f;
    if (lane < NCLS) lsh[w][lane] = dl;
    __builtin_amdgcn_wave_barrier();
    gb2acc += dl;
    float dh = 0.f;
    if (lane < HID) {
      float dd = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) {
        const float lc = lsh[w][c];
        dd += w2s[c * HID + lane] * lc;
        gw2acc[c] += lc * dsh[w][lane];
      }
      dh = (h > 0.f) ? dd * ms : 0.f;
      dhs[rr * HID + lane] = dh;
    }
    __builtin_amdgcn_wave_barrier();
    // dx[n][k] = sum_j W1[j][k] dh_j  (lanes over k: coalesced W1 reads)
    for (int k = lane; k < FLAT; k += 64) {
      float acc = 0.f;
      for (int j = 0; j < HID; ++j) acc += w1[(size_t)j * FLAT + k] * dhs[rr * HID + j];
      dx[(size_t)n * FLAT + k] = acc;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // per-wave partials -> LDS -> one atomic per output per block
  if (train && lane < HID) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) red[w][c * HID + lane] = gw2acc[c];
  }
  if (lane < NCLS) red[w][NCLS * HID + lane] = train ? gb2acc : 0.f;
  if (lane == 0) {
    red[w][NCLS * HID + NCLS] = loss_acc;
    red[w][NCLS * HID + NCLS + 1] = ok_acc;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < NCLS * HID + NCLS + 2; o += T) {
    const float v = red[0][o] + red[1][o] + red[2][o] + red[3][o];
    if (o < NCLS * HID) {
      if (train) atomicAdd(gw2 + o, v);
    } else if (o < NCLS * HID + NCLS) {
      if (train) atomicAdd(gb2 + o - NCLS * HID, v);
    } else {
      atomicAdd(stats + o - NCLS * HID - NCLS, v);
    }
  }
  if (!train) return;
  // dW1[j][k] = sum_rows dh[r][j] x[r][k]; db1[j] = sum_rows dh[r][j]
  for (int o = threadIdx.x; o < HID * FLAT; o += T) {
    const int j = o / FLAT, k = o % FLAT;
    float acc = 0.f;
    for (int r = 0; r < nr; ++r) acc += dhs[r * HID + j] * xs[r * XP1 + k];
    atomicAdd(gw1 + o, acc);
  }
  if (threadIdx.x < HID) {
    float acc = 0.f;
    for (int r = 0; r < nr; ++r) acc += dhs[r * HID + threadIdx.x];
    atomicAdd(gb1 + threadIdx.x, acc);
  }
}

}  // namespace

void ref_cnn_stage0_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                        int B, unsigned long long seed, unsigned sample0, float p, bool drop, hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cnn_s0_fwd_kernel, dim3(B), dim3(T), 0, stream, x, w1, b1, w2, b2, out, seed, sample0, p,
                     drop ? 1 : 0);
}

void ref_cnn_stage0_bwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                        const float* gout, int B, unsigned long long seed, unsigned sample0, float p, bool drop,
                        float* gw1, float* gb1, float* gw2, float* gb2, hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cnn_s0_bwd_kernel, dim3(B), dim3(T), 0, stream, x, w1, b1, w2, b2, gout, seed, sample0, p,
                     drop ? 1 : 0, gw1, gb1, gw2, gb2);
}

void ref_cnn_stage1(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                    const int64_t* target, int B, unsigned long long seed, unsigned sample0, float p, bool drop,
                    float scale, float* stats, float* dx, float* gw1, float* gb1, float* gw2, float* gb2,
                    hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cnn_s1_kernel, dim3((B + S1_ROWS - 1) / S1_ROWS), dim3(T), 0, stream, x, w1, b1, w2, b2, target,
                     B, seed, sample0, p, drop ? 1 : 0, scale, stats, dx, gw1, gb1, gw2, gb2);
}

}  // namespace sdml
