// The reference CNN's two pipeline stages as fused gfx950 kernels
// (/root/reference/simple_distributed.py:26-80).
//
// Stage 0 (Network1): conv1(1->10,k5) -> maxpool2 -> relu -> conv2(10->20,k5) -> Dropout2d(p)
//                     -> maxpool2 -> relu -> flatten(320)
//   * cnn_s0_fwd: one workgroup (512 threads) per sample. The image, both filter banks and
//     every intermediate live in LDS. Conv1 is evaluated per pooled output: each one computes
//     its 2x2 conv window and keeps the max and its argmax. Conv2 is register-blocked: one
//     thread computes a full 8-wide output row, sliding a 12-value input window over 5 taps.
//     ReLU and the per-(sample, channel) Dropout2d scale are fused in. For training, the
//     pooled conv1 activations and both pool argmaxes (1.4K floats + 1.7K bytes per sample)
//     are saved so that the backward does not recompute.
//   * cnn_s0_bwd: one workgroup (1024 threads) per sample, in three phases:
//       1. route the incoming gradient through ReLU, pool argmax and dropout into a dense
//          conv2-output gradient held in LDS;
//       2. dW2 over 1000 (c, ci, ky) rows, register-blocked over kx with a sliding input
//          window; dZ1 as 4-wide strips x 2 channel halves (combined by LDS float atomics),
//          fused with the ReLU mask;
//       3. dW1 over the 144 argmax positions per channel (pooling makes conv1's output
//          gradient 3/4 zeros, so those are never touched), reduced across 4-lane groups.
//     Per-block partial weight grads go out as one fp32 atomic per weight.
// Stage 1 (Network2): fc1(320->50) -> relu -> dropout(p) -> fc2(50->10) -> log_softmax -> NLL
//   * cnn_s1: ONE launch for forward, loss/accuracy and the whole backward (dX, dW1, db1, dW2,
//     db2). A workgroup handles ROWS samples (8 at small batch, so the batch spreads over many
//     CUs) and first stages all of W1 (64 KB) in LDS. Each wave runs one sample at a time: fc1
//     by lane-per-row dot products, softmax by wave shuffles, dX by lane-per-column walks. dW1 = dh^T x is then reduced over the
//     block's rows before a single atomic per weight.
// Dropout masks come from a counter hash of (seed, sample, unit). The backward regenerates the
// forward's mask exactly, so no mask is stored.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdml {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int IMG = 28, KS = 5, C1 = 10, O1 = 24, P1 = 12, C2 = 20, O2 = 8, P2 = 4;
constexpr int FLAT = C2 * P2 * P2;  // 320
constexpr int HID = 50, NCLS = 10;
constexpr int NZ1 = C1 * P1 * P1;   // 1440 pooled conv1 activations per sample
constexpr int NIDX = NZ1 + FLAT;    // saved argmax bytes per sample (conv1 pool, conv2 pool)

__device__ __forceinline__ unsigned drop_hash(unsigned long long seed, unsigned a, unsigned b) {
  unsigned long long x = seed ^ (0x9E3779B97F4A7C15ull * (a + 1)) ^ (0xC2B2AE3D27D4EB4Full * (b + 7));
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return (unsigned)x;
}
// per-pass seed + a device step counter (advanced inside captured hipGraphs, so replays
// draw fresh masks): seed_eff = seed + golden * ctr  (mod 2^64)
__device__ __forceinline__ unsigned long long eff_seed(unsigned long long seed, const long long* ctr) {
  return ctr ? seed + 0x9E3779B97F4A7C15ull * (unsigned long long)(*ctr) : seed;
}
__device__ __forceinline__ float keep_scale(unsigned long long seed, unsigned a, unsigned b, float p) {
  if (p <= 0.f) return 1.f;
  float u = (float)(drop_hash(seed, a, b) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

// ---------------------------------------------------------------------------------------------
// stage 0 forward
constexpr int TF = 512;

__global__ void __launch_bounds__(TF) cnn_s0_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ out,
                                                        float* __restrict__ z1_save, unsigned char* __restrict__ idx_save,
                                                        unsigned long long seed0, const long long* ctr,
                                                        unsigned sample0, float p, int drop) {
  __shared__ float xs[IMG * IMG];
  __shared__ float w1s[C1 * KS * KS];
  __shared__ float w2s[C2 * C1 * KS * KS];
  __shared__ float z1[NZ1];
  __shared__ float c2[C2 * O2 * O2];
  __shared__ float dsc[C2];
  const int n = blockIdx.x, t = threadIdx.x;
  const float* xn = x + (size_t)n * IMG * IMG;
  for (int i = t; i < IMG * IMG; i += TF) xs[i] = xn[i];
  for (int i = t; i < C1 * KS * KS; i += TF) w1s[i] = w1[i];
  for (int i = t; i < C2 * C1 * KS * KS; i += TF) w2s[i] = w2[i];
  if (t < C2) dsc[t] = drop ? keep_scale(eff_seed(seed0, ctr), sample0 + n, t, p) : 1.f;
  __syncthreads();
  // conv1 -> maxpool2 (argmax) -> relu, one pooled output per item
  for (int o = t; o < NZ1; o += TF) {
    const int c = o / (P1 * P1), py = (o / P1) % P1, px = o % P1;
    float win[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int q = 0; q < 6; ++q) win[r][q] = xs[(2 * py + r) * IMG + 2 * px + q];
    float acc[4];
    const float bias = b1[c];
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] = bias;
#pragma unroll
    for (int ky = 0; ky < KS; ++ky)
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float w = w1s[(c * KS + ky) * KS + kx];
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[d] += w * win[(d >> 1) + ky][(d & 1) + kx];
      }
    float best = acc[0];
    int arg = 0;
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (acc[d] > best) {
        best = acc[d];
        arg = d;
      }
    const float v = fmaxf(best, 0.f);
    z1[o] = v;
    if (z1_save) {
      z1_save[(size_t)n * NZ1 + o] = v;
      idx_save[(size_t)n * NIDX + o] = (unsigned char)arg;
    }
  }
  __syncthreads();
  // conv2 (+ dropout2d scale): one output row (c, y) of 8 per item, sliding window over kx
  for (int it = t; it < C2 * O2; it += TF) {
    const int c = it / O2, y = it % O2;
    float acc[O2];
#pragma unroll
    for (int xo = 0; xo < O2; ++xo) acc[xo] = 0.f;
    for (int ci = 0; ci < C1; ++ci)
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const float* zr = z1 + (ci * P1 + y + ky) * P1;
        const float* wr = w2s + ((c * C1 + ci) * KS + ky) * KS;
        float zv[P1], wv[KS];
#pragma unroll
        for (int q = 0; q < P1; ++q) zv[q] = zr[q];
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) wv[kx] = wr[kx];
#pragma unroll
        for (int xo = 0; xo < O2; ++xo)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) acc[xo] += wv[kx] * zv[xo + kx];
      }
    const float bias = b2[c], sc = dsc[c];
#pragma unroll
    for (int xo = 0; xo < O2; ++xo) c2[(c * O2 + y) * O2 + xo] = (acc[xo] + bias) * sc;  // Dropout2d before pool (:45)
  }
  __syncthreads();
  // maxpool2 (argmax) -> relu -> flatten
  for (int o = t; o < FLAT; o += TF) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float v = c2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)];
      if (v > best) {
        best = v;
        arg = d;
      }
    }
    out[(size_t)n * FLAT + o] = fmaxf(best, 0.f);
    if (idx_save) idx_save[(size_t)n * NIDX + NZ1 + o] = (unsigned char)arg;
  }
}

// ---------------------------------------------------------------------------------------------
// stage 0 backward (uses the forward's saved z1 / argmaxes and its output for the ReLU mask)
constexpr int TB = 1024;

__global__ void __launch_bounds__(TB) cnn_s0_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w2,
                                                        const float* __restrict__ out, const float* __restrict__ gout,
                                                        const float* __restrict__ z1_save,
                                                        const unsigned char* __restrict__ idx_save,
                                                        unsigned long long seed0, const long long* ctr,
                                                        unsigned sample0, float p, int drop, float* __restrict__ gw1,
                                                        float* __restrict__ gb1, float* __restrict__ gw2,
                                                        float* __restrict__ gb2) {
  __shared__ float xs[IMG * IMG];
  __shared__ float w2s[C2 * C1 * KS * KS];
  __shared__ float z1[NZ1];
  __shared__ float G2[C2 * O2 * O2];
  __shared__ float g1[NZ1];  // d loss / d (pooled conv1 output), ReLU-masked
  __shared__ unsigned char a1[NZ1];
  __shared__ float dsc[C2];
  const int n = blockIdx.x, t = threadIdx.x;
  const float* xn = x + (size_t)n * IMG * IMG;
  for (int i = t; i < IMG * IMG; i += TB) xs[i] = xn[i];
  for (int i = t; i < C2 * C1 * KS * KS; i += TB) w2s[i] = w2[i];
  for (int i = t; i < NZ1; i += TB) {
    z1[i] = z1_save[(size_t)n * NZ1 + i];
    a1[i] = idx_save[(size_t)n * NIDX + i];
  }
  for (int i = t; i < C2 * O2 * O2; i += TB) G2[i] = 0.f;
  for (int i = t; i < NZ1; i += TB) g1[i] = 0.f;
  if (t < C2) dsc[t] = drop ? keep_scale(eff_seed(seed0, ctr), sample0 + n, t, p) : 1.f;
  __syncthreads();
  // 1. relu (out > 0 <=> pooled pre-relu > 0) -> pool argmax -> dropout scale
  for (int o = t; o < FLAT; o += TB) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    const float g = out[(size_t)n * FLAT + o] > 0.f ? gout[(size_t)n * FLAT + o] * dsc[c] : 0.f;
    const int d = idx_save[(size_t)n * NIDX + NZ1 + o];
    G2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)] = g;
  }
  __syncthreads();
  // 2a. dW2[c][ci][ky][:] for 1000 (c, ci, ky) rows; db2 on the spare threads
  if (t < C2 * C1 * KS) {
    const int c = t / (C1 * KS), ci = (t / KS) % C1, ky = t % KS;
    float acc[KS] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int y = 0; y < O2; ++y) {
      const float* zr = z1 + (ci * P1 + y + ky) * P1;
      const float* gr = G2 + (c * O2 + y) * O2;
      float zv[P1], gv[O2];
#pragma unroll
      for (int q = 0; q < P1; ++q) zv[q] = zr[q];
#pragma unroll
      for (int q = 0; q < O2; ++q) gv[q] = gr[q];
#pragma unroll
      for (int xo = 0; xo < O2; ++xo)
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) acc[kx] += gv[xo] * zv[xo + kx];
    }
    float* dst = gw2 + ((c * C1 + ci) * KS + ky) * KS;
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) atomicAdd(dst + kx, acc[kx]);
  } else if (t < C2 * C1 * KS + C2) {
    const int c = t - C2 * C1 * KS;
    float acc = 0.f;
    for (int i = 0; i < O2 * O2; ++i) acc += G2[c * O2 * O2 + i];
    atomicAdd(gb2 + c, acc);
  }
  // 2b. dZ1 = full correlation of G2 with W2, 4-wide strips (ci, Y, X0..X0+3) x 2 halves of
  //     the conv2 channels (720 items: the block's critical path), halves combined by LDS atomics
  for (int it = t; it < 2 * C1 * P1 * (P1 / 4); it += TB) {
    const int half = it / (C1 * P1 * 3), r = it % (C1 * P1 * 3);
    const int ci = r / (P1 * 3), Y = (r / 3) % P1, X0 = (r % 3) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = half * (C2 / 2); c < (half + 1) * (C2 / 2); ++c)
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const int y = Y - ky;
        if (y < 0 || y >= O2) continue;
        const float* gr = G2 + (c * O2 + y) * O2;
        const float* wr = w2s + ((c * C1 + ci) * KS + ky) * KS;
        float gv[8], wv[KS];
#pragma unroll
        for (int q = 0; q < 8; ++q) {  // G2 row at x = X0 - 4 + q (zero outside 0..7)
          const int xx = X0 - 4 + q;
          gv[q] = (xx >= 0 && xx < O2) ? gr[xx] : 0.f;
        }
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) wv[kx] = wr[kx];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) acc[j] += wv[kx] * gv[j - kx + 4];
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = (ci * P1 + Y) * P1 + X0 + j;
      if (z1[o] > 0.f) atomicAdd(&g1[o], acc[j]);  // ReLU mask; g1 pre-zeroed
    }
  }
  __syncthreads();
  // 3. dW1[c][ky][kx] = sum over pooled positions of g1 * x at the argmax tap; 4 lanes per weight
  if (t < C1 * KS * KS * 4) {
    const int wi = t >> 2, part = t & 3;
    const int c = wi / (KS * KS), ky = (wi / KS) % KS, kx = wi % KS;
    float acc = 0.f;
    for (int q = part; q < P1 * P1; q += 4) {
      const int o = c * P1 * P1 + q;
      const int py = q / P1, px = q % P1, d = a1[o];
      acc += g1[o] * xs[(2 * py + (d >> 1) + ky) * IMG + 2 * px + (d & 1) + kx];
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part == 0) atomicAdd(gw1 + wi, acc);
  } else if (t < C1 * KS * KS * 4 + C1) {
    const int c = t - C1 * KS * KS * 4;
    float acc = 0.f;
    for (int q = 0; q < P1 * P1; ++q) acc += g1[c * P1 * P1 + q];
    atomicAdd(gb1 + c, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// stage 1
constexpr int T1 = 256;
constexpr int XP1 = FLAT + 4;  // LDS row pitch of the inputs (16-B aligned rows)
constexpr int WP1 = FLAT + 1;  // LDS row pitch of W1 (odd: lane-per-row walks are conflict-free)

template <int ROWS>
__global__ void __launch_bounds__(T1) cnn_s1_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                    const float* __restrict__ b1, const float* __restrict__ w2,
                                                    const float* __restrict__ b2, const int64_t* __restrict__ tgt,
                                                    int B, unsigned long long seed0, const long long* ctr,
                                                    unsigned sample0, float p, int drop, float scale,
                                                    float* __restrict__ stats, float* __restrict__ dx,
                                                    float* __restrict__ gw1, float* __restrict__ gb1,
                                                    float* __restrict__ gw2, float* __restrict__ gb2) {
  __shared__ __attribute__((aligned(16))) float xs[ROWS * XP1];
  __shared__ float w1s[HID * WP1];  // 64 KB: fc1 and dX read W1 from LDS, not L2
  __shared__ float dhs[ROWS * HID];
  __shared__ float w2s[NCLS * HID];
  __shared__ float dsh[4][HID];
  __shared__ float lsh[4][NCLS];
  __shared__ float red[4][NCLS * HID + NCLS + 2];
  const unsigned long long seed = eff_seed(seed0, ctr);
  const int r0 = blockIdx.x * ROWS;
  const int nr = min(ROWS, B - r0);
  const bool train = dx != nullptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < nr * (FLAT / 4); i += T1) {
    const int r = i / (FLAT / 4), k4 = i % (FLAT / 4);
    *reinterpret_cast<float4*>(xs + r * XP1 + 4 * k4) =
        *reinterpret_cast<const float4*>(x + (size_t)(r0 + r) * FLAT + 4 * k4);
  }
  for (int i = threadIdx.x; i < HID * (FLAT / 4); i += T1) {
    const int j = i / (FLAT / 4), k4 = i % (FLAT / 4);
    const float4 v = *reinterpret_cast<const float4*>(w1 + (size_t)j * FLAT + 4 * k4);
    float* d = w1s + j * WP1 + 4 * k4;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  for (int i = threadIdx.x; i < NCLS * HID; i += T1) w2s[i] = w2[i];
  __syncthreads();
  float gw2acc[NCLS];  // lane j < 50: dW2[c][j]
#pragma unroll
  for (int c = 0; c < NCLS; ++c) gw2acc[c] = 0.f;
  float gb2acc = 0.f, loss_acc = 0.f, ok_acc = 0.f;
  for (int rr = w; rr < nr; rr += 4) {
    const int n = r0 + rr;
    // fc1 + relu + dropout: lane j < 50 (W1 row j from LDS, x broadcast as float4)
    float h = 0.f, ms = 0.f;
    if (lane < HID) {
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
      const float* wr = w1s + lane * WP1;
      const float4* xr = reinterpret_cast<const float4*>(xs + rr * XP1);
#pragma unroll 8
      for (int k4 = 0; k4 < FLAT / 4; ++k4) {
        const float4 xv = xr[k4];
        a4[0] += wr[4 * k4] * xv.x;
        a4[1] += wr[4 * k4 + 1] * xv.y;
        a4[2] += wr[4 * k4 + 2] * xv.z;
        a4[3] += wr[4 * k4 + 3] * xv.w;
      }
      h = fmaxf(b1[lane] + ((a4[0] + a4[1]) + (a4[2] + a4[3])), 0.f);
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
    float se = lane < NCLS ? __expf(z - mx) : 0.f;
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = mx + __logf(se);
    const int y = (int)tgt[n];
    const unsigned long long bal = __ballot(lane < NCLS && z == mx);  // first max = torch argmax
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
    if (lane < HID) {
      float dd = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) {
        const float lc = lsh[w][c];
        dd += w2s[c * HID + lane] * lc;
        gw2acc[c] += lc * dsh[w][lane];
      }
      dhs[rr * HID + lane] = (h > 0.f) ? dd * ms : 0.f;
    }
    __builtin_amdgcn_wave_barrier();
    // dx[n][k] = sum_j W1[j][k] dh_j  (lanes over k)
    for (int k = lane; k < FLAT; k += 64) {
      float acc = 0.f;
#pragma unroll 10
      for (int j = 0; j < HID; ++j) acc += w1s[j * WP1 + k] * dhs[rr * HID + j];
      dx[(size_t)n * FLAT + k] = acc;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // per-wave partials -> LDS -> one atomic per output per block
  if (lane < HID) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) red[w][c * HID + lane] = gw2acc[c];
  }
  if (lane < NCLS) red[w][NCLS * HID + lane] = gb2acc;
  if (lane == 0) {
    red[w][NCLS * HID + NCLS] = loss_acc;
    red[w][NCLS * HID + NCLS + 1] = ok_acc;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < NCLS * HID + NCLS + 2; o += T1) {
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
  for (int o = threadIdx.x; o < HID * FLAT; o += T1) {
    const int j = o / FLAT, k = o % FLAT;
    float acc = 0.f;
#pragma unroll 4
    for (int r = 0; r < nr; ++r) acc += dhs[r * HID + j] * xs[r * XP1 + k];
    atomicAdd(gw1 + o, acc);
  }
  if (threadIdx.x < HID) {
    float acc = 0.f;
    for (int r = 0; r < nr; ++r) acc += dhs[r * HID + threadIdx.x];
    atomicAdd(gb1 + threadIdx.x, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// The whole training step of the 2-stage CNN (both stages on one rank, the reference's B = 60) in two
// launches: cnn_step_sample runs, per sample, stage 0's forward, stage 1's forward + NLL + backward and
// stage 0's backward in ONE workgroup (the sample's activations never leave LDS), and writes the sample's
// weight-gradient contributions as one record (no float atomics: the per-block atomics of the three-kernel
// form queued 60 deep on every conv weight); cnn_step_update sums the records in sample order
// (deterministic), applies torch.optim.SGD's update to all 8 parameter tensors, writes (loss sum, correct)
// and advances the device dropout counter. The fc layers' gradients are rank 1 per sample (dh z3^T,
// dl hd^T), so a record holds the factors (380 + 60 floats), not the 16,500-float products.
constexpr int TS = 1024;
// diagnostic phase stamps (stamps != nullptr, tools/probes): s_memtime after each barrier, per block
#define STAMP(k)                                                                  \
  do {                                                                            \
    if (stamps && t == 0) stamps[(size_t)blockIdx.x * 16 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
constexpr int R_W2C = 0, R_B2C = R_W2C + C2 * C1 * KS * KS, R_W1C = R_B2C + C2, R_B1C = R_W1C + C1 * KS * KS,
              R_DH = R_B1C + C1, R_Z3 = R_DH + HID, R_DL = R_Z3 + FLAT, R_HD = R_DL + NCLS, R_LOSS = R_HD + HID,
              REC = R_LOSS + 2;
static_assert(REC == 5712, "record layout");
// split-backward workspace per sample: G2 [20][8][8], z1 [10][12][12], the conv1 pool argmaxes (bytes)
constexpr int BWS = C2 * O2 * O2 + NZ1 + NZ1 / 4;

__global__ void __launch_bounds__(TS) cnn_step_sample_kernel(const float* __restrict__ x, const int64_t* __restrict__ tgt,
                                                             const float* __restrict__ cw1, const float* __restrict__ cb1,
                                                             const float* __restrict__ cw2, const float* __restrict__ cb2,
                                                             const float* __restrict__ fw1, const float* __restrict__ fb1,
                                                             const float* __restrict__ fw2, const float* __restrict__ fb2,
                                                             unsigned long long seed0, unsigned long long seed1,
                                                             const long long* ctr, float p0, int drop0, float p1,
                                                             int drop1, float scale, float* __restrict__ rec,
                                                             long long* __restrict__ stamps, float* __restrict__ bws) {
  __shared__ float xs[IMG * IMG];
  __shared__ float w1s[C1 * KS * KS];
  __shared__ float w2s[C2 * C1 * KS * KS];
  __shared__ float z1[NZ1];
  __shared__ unsigned char a1[NZ1];
  __shared__ float c2[C2 * O2 * O2];  // conv2 output, then its gradient G2
  __shared__ float c2p[5][C2 * O2 * O2];  // conv2 partials per group of 2 input channels
  __shared__ float z3[FLAT];
  __shared__ unsigned char a2[FLAT];
  __shared__ float g1[NZ1];
  __shared__ float dsc[C2];
  __shared__ float hraw[HID], hd[HID], msk[HID], dh[HID], dl[NCLS];
  __shared__ float fw2s[NCLS * HID], fb1s[HID], fb2s[NCLS];
  __shared__ float dzp[TS / 64][FLAT];  // per-wave partials of W1^T dh (the wave's 4 fc1 rows)
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float* R = rec + (size_t)n * REC;
  STAMP(0);
  // fc1 rows of this wave (hidden units wv, wv + 16, wv + 32, wv + 48 < 50), 5 per lane: loaded here so their
  // HBM latency (the weights were just rewritten by the previous step's update) hides under the conv phases
  float w1r[4][5];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = wv + 16 * u;
#pragma unroll
    for (int i = 0; i < 5; ++i) w1r[u][i] = j < HID ? fw1[(size_t)j * FLAT + lane + 64 * i] : 0.f;
  }
  const float* xn = x + (size_t)n * IMG * IMG;
  {  // every global load issued before the first LDS store: one latency instead of one per loop round
    constexpr int NW2 = (C2 * C1 * KS * KS + TS - 1) / TS;  // 5
    float w2v[NW2];
#pragma unroll
    for (int u = 0; u < NW2; ++u) w2v[u] = t + TS * u < C2 * C1 * KS * KS ? cw2[t + TS * u] : 0.f;
    const float xv = t < IMG * IMG ? xn[t] : 0.f;
    const float w1v = t < C1 * KS * KS ? cw1[t] : 0.f;
    // stage 1's small operands too (fc2 weights, both biases): their phases then read LDS, not HBM
    const float f2v = t < NCLS * HID ? fw2[t] : 0.f;
    const float fbv = t < HID ? fb1[t] : (t >= 64 && t < 64 + NCLS ? fb2[t - 64] : 0.f);
#pragma unroll
    for (int u = 0; u < NW2; ++u)
      if (t + TS * u < C2 * C1 * KS * KS) w2s[t + TS * u] = w2v[u];
    if (t < IMG * IMG) xs[t] = xv;
    if (t < C1 * KS * KS) w1s[t] = w1v;
    if (t < NCLS * HID) fw2s[t] = f2v;
    if (t < HID) fb1s[t] = fbv;
    else if (t >= 64 && t < 64 + NCLS) fb2s[t - 64] = fbv;
  }
  for (int i = t; i < NZ1; i += TS) g1[i] = 0.f;
  if (t < C2) dsc[t] = drop0 ? keep_scale(eff_seed(seed0, ctr), n, t, p0) : 1.f;
  __syncthreads();
  STAMP(1);
  // ---- stage 0 forward (cnn_s0_fwd_kernel's arithmetic) ----
  for (int o = t; o < NZ1; o += TS) {
    const int c = o / (P1 * P1), py = (o / P1) % P1, px = o % P1;
    float win[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int q = 0; q < 6; ++q) win[r][q] = xs[(2 * py + r) * IMG + 2 * px + q];
    float acc[4];
    const float bias = cb1[c];
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] = bias;
#pragma unroll
    for (int ky = 0; ky < KS; ++ky)
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float w = w1s[(c * KS + ky) * KS + kx];
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[d] += w * win[(d >> 1) + ky][(d & 1) + kx];
      }
    float best = acc[0];
    int arg = 0;
#pragma unroll
    for (int d = 1; d < 4; ++d)
      if (acc[d] > best) {
        best = acc[d];
        arg = d;
      }
    z1[o] = fmaxf(best, 0.f);
    a1[o] = (unsigned char)arg;
  }
  __syncthreads();
  STAMP(2);
  // conv2 as 800 items (output row (c, y) x 5 groups of 2 input channels; the 160-row form left 864 of the
  // 1024 threads idle on a 2000-FMA chain), group partials summed in a fixed order below
  for (int it = t; it < C2 * O2 * 5; it += TS) {
    const int cg = it / (C2 * O2), c = (it / O2) % C2, y = it % O2;
    float acc[O2];
#pragma unroll
    for (int xo = 0; xo < O2; ++xo) acc[xo] = 0.f;
#pragma unroll
    for (int ci = 2 * cg; ci < 2 * cg + 2; ++ci)
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const float* zr = z1 + (ci * P1 + y + ky) * P1;
        const float* wr = w2s + ((c * C1 + ci) * KS + ky) * KS;
        float zv[P1], wv5[KS];
#pragma unroll
        for (int q = 0; q < P1; ++q) zv[q] = zr[q];
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) wv5[kx] = wr[kx];
#pragma unroll
        for (int xo = 0; xo < O2; ++xo)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) acc[xo] += wv5[kx] * zv[xo + kx];
      }
#pragma unroll
    for (int xo = 0; xo < O2; ++xo) c2p[cg][(c * O2 + y) * O2 + xo] = acc[xo];
  }
  __syncthreads();
  STAMP(3);
  for (int o = t; o < C2 * O2 * O2; o += TS) {
    const int c = o / (O2 * O2);
    const float v = (((c2p[0][o] + c2p[1][o]) + (c2p[2][o] + c2p[3][o])) + c2p[4][o]) + cb2[c];
    c2[o] = v * dsc[c];
  }
  __syncthreads();
  STAMP(4);
  for (int o = t; o < FLAT; o += TS) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float v = c2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)];
      if (v > best) {
        best = v;
        arg = d;
      }
    }
    const float v = fmaxf(best, 0.f);
    z3[o] = v;
    a2[o] = (unsigned char)arg;
    R[R_Z3 + o] = v;
  }
  __syncthreads();
  STAMP(5);
  for (int i = t; i < C2 * O2 * O2; i += TS) c2[i] = 0.f;  // becomes G2
  // ---- stage 1: fc1 + relu + dropout (wave w: hidden units w, w + 16, w + 32, w + 48) ----
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = wv + 16 * u;
    if (j >= HID) break;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 5; ++i) a += w1r[u][i] * z3[lane + 64 * i];
    for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
    if (lane == 0) {
      const float h = fmaxf(fb1s[j] + a, 0.f);
      const float ms = drop1 ? keep_scale(eff_seed(seed1, ctr), n, j, p1) : 1.f;
      hraw[j] = h;
      msk[j] = ms;
      hd[j] = h * ms;
      R[R_HD + j] = h * ms;
    }
  }
  __syncthreads();
  STAMP(6);
  // fc2 + log_softmax + NLL + dlogits, then dh = (W2^T dl) * relu' * dropout (wave 0)
  if (wv == 0) {
    float z = -INFINITY;
    if (lane < NCLS) {
      float acc = fb2s[lane];
      for (int j = 0; j < HID; ++j) acc += fw2s[lane * HID + j] * hd[j];
      z = acc;
    }
    float mx = z;
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float se = lane < NCLS ? __expf(z - mx) : 0.f;
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const float lse = mx + __logf(se);
    const int y = (int)tgt[n];
    const unsigned long long bal = __ballot(lane < NCLS && z == mx);  // first max = torch argmax
    const int am = __ffsll((long long)bal) - 1;
    const float zy = __shfl(z, y);
    const float d = lane < NCLS ? scale * (__expf(z - lse) - (lane == y ? 1.f : 0.f)) : 0.f;
    if (lane < NCLS) {
      dl[lane] = d;
      R[R_DL + lane] = d;
    }
    if (lane == 0) {
      R[R_LOSS] = lse - zy;
      R[R_LOSS + 1] = (am == y) ? 1.f : 0.f;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < HID) {
      float dd = 0.f;
#pragma unroll
      for (int c = 0; c < NCLS; ++c) dd += fw2s[c * HID + lane] * dl[c];
      const float v = hraw[lane] > 0.f ? dd * msk[lane] : 0.f;
      dh[lane] = v;
      R[R_DH + lane] = v;
    }
  }
  __syncthreads();
  STAMP(7);
  // dz3 = W1^T dh, routed through relu (z3 > 0), pool argmax and the Dropout2d scale into G2. Wave w holds fc1
  // rows w + 16 u in registers (w1r, loaded for the forward): it writes its 4-row partial of every column, and
  // column t sums the 16 wave partials in wave order (re-reading W1 column-wise from memory cost 50 loads per
  // thread, 5 dependent L2 round trips)
  {
    float pz[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = wv + 16 * u;
      const float dj = j < HID ? dh[j] : 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) pz[i] = __builtin_fmaf(w1r[u][i], dj, pz[i]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) dzp[wv][lane + 64 * i] = pz[i];
  }
  __syncthreads();
  if (t < FLAT) {
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < TS / 64; ++w) acc += dzp[w][t];
    const int c = t / (P2 * P2), py = (t / P2) % P2, px = t % P2, d = a2[t];
    c2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)] = z3[t] > 0.f ? acc * dsc[c] : 0.f;
  }
  __syncthreads();
  STAMP(8);
  if (bws) {  // split backward: hand G2, z1 and the conv1 pool argmaxes to cnn_step_bwd_kernel (10 workgroups per sample)
    float* wsn = bws + (size_t)n * BWS;
    for (int i = t; i < C2 * O2 * O2; i += TS) wsn[i] = c2[i];
    for (int i = t; i < NZ1; i += TS) wsn[C2 * O2 * O2 + i] = z1[i];
    unsigned char* ab = reinterpret_cast<unsigned char*>(wsn + C2 * O2 * O2 + NZ1);
    for (int i = t; i < NZ1; i += TS) ab[i] = a1[i];
    return;
  }
  const float* G2 = c2;
  // ---- stage 0 backward (cnn_s0_bwd_kernel's phases), contributions into the record ----
  if (t < C2 * C1 * KS) {
    // dW2 from the 16 nonzeros of each channel's G2 (one per pooled cell, at its argmax; the other 48 of
    // the 64 positions are zero): 16 instead of 64 terms per weight
    const int c = t / (C1 * KS), ci = (t / KS) % C1, ky = t % KS;
    float acc[KS] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int q = 0; q < P2 * P2; ++q) {
      const int py = q / P2, px = q % P2, d = a2[c * P2 * P2 + q];
      const int y = 2 * py + (d >> 1), x = 2 * px + (d & 1);
      const float g = G2[(c * O2 + y) * O2 + x];
      const float* zr = z1 + (ci * P1 + y + ky) * P1 + x;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) acc[kx] += g * zr[kx];
    }
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) R[R_W2C + ((c * C1 + ci) * KS + ky) * KS + kx] = acc[kx];
  } else if (t < C2 * C1 * KS + C2) {
    const int c = t - C2 * C1 * KS;
    float acc = 0.f;
    for (int i = 0; i < O2 * O2; ++i) acc += G2[c * O2 * O2 + i];
    R[R_B2C + c] = acc;
  }
  if (stamps) {
    __syncthreads();
    STAMP(10);
  }
  // dZ1 as 3-wide strips: 2 halves x 10 ci x 12 rows x 4 strips = 960 items (720 4-wide strips left 304
  // threads idle on the phase's critical path)
  for (int it = t; it < 2 * C1 * P1 * (P1 / 3); it += TS) {
    const int half = it / (C1 * P1 * 4), r = it % (C1 * P1 * 4);
    const int ci = r / (P1 * 4), Y = (r / 4) % P1, X0 = (r % 4) * 3;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int c = half * (C2 / 2); c < (half + 1) * (C2 / 2); ++c)
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) {
        const int y = Y - ky;
        if (y < 0 || y >= O2) continue;
        const float* gr = G2 + (c * O2 + y) * O2;
        const float* wr = w2s + ((c * C1 + ci) * KS + ky) * KS;
        float gv[7], wv5[KS];
#pragma unroll
        for (int q = 0; q < 7; ++q) {  // G2 row at x = X0 - 4 + q (zero outside 0..7)
          const int xx = X0 - 4 + q;
          gv[q] = (xx >= 0 && xx < O2) ? gr[xx] : 0.f;
        }
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) wv5[kx] = wr[kx];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) acc[j] += wv5[kx] * gv[j - kx + 4];
      }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int o = (ci * P1 + Y) * P1 + X0 + j;
      if (z1[o] > 0.f) atomicAdd(&g1[o], acc[j]);  // ReLU mask; LDS, two halves (a + b == b + a: deterministic)
    }
  }
  __syncthreads();
  STAMP(9);
  if (t < C1 * KS * KS * 4) {
    const int wi = t >> 2, prt = t & 3;
    const int c = wi / (KS * KS), ky = (wi / KS) % KS, kx = wi % KS;
    float acc = 0.f;
    for (int q = prt; q < P1 * P1; q += 4) {
      const int o = c * P1 * P1 + q;
      const int py = q / P1, px = q % P1, d = a1[o];
      acc += g1[o] * xs[(2 * py + (d >> 1) + ky) * IMG + 2 * px + (d & 1) + kx];
    }
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (prt == 0) R[R_W1C + wi] = acc;
  } else if (t < C1 * KS * KS * 4 + C1) {
    const int c = t - C1 * KS * KS * 4;
    float acc = 0.f;
    for (int q = 0; q < P1 * P1; ++q) acc += g1[c * P1 * P1 + q];
    R[R_B1C + c] = acc;
  }
  __syncthreads();
  STAMP(15);
}

// Stage 0's backward of one sample, split over its 10 conv1 channels (one workgroup per (sample, ci), 576
// threads): the batch of 60 then spreads over 600 workgroups instead of 60, which cuts the sample kernel's
// critical path roughly in half (its backward phases ran on one CU per sample). Partitioning by the conv1
// channel ci keeps every output private to one workgroup: dW2[:, ci], dZ1[ci] (all 20 conv2 channels
// contribute, summed as 4 fixed quarters), the ReLU mask, dW1[ci], db1[ci]; db2 by the ci = 0 workgroup.
// Fixed summation orders: deterministic. Inputs: x, W2, the forward's G2 / z1 / argmaxes (workspace bws).
constexpr int TBW = 576;
// the last phase: dW1 on threads 0..399, db1 on 400..415, dW2 on 416..515, db2 (ci == 0) on 520..559
constexpr int DW2_T0 = 416, DB2_T0 = 520;
__global__ void __launch_bounds__(TBW, 7) cnn_step_bwd_kernel(const float* __restrict__ x, const float* __restrict__ cw2,
                                                           const float* __restrict__ bws, float* __restrict__ rec,
                                                           long long* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) float G2[C2 * O2 * O2];
  __shared__ float z1c[P1 * P1];
  __shared__ unsigned char a1c[P1 * P1];
  __shared__ unsigned char a2s[FLAT];
  __shared__ float cellg[FLAT];        // G2 at each pooled cell's argmax (its one nonzero)
  __shared__ __attribute__((aligned(16))) float xs[IMG * IMG];
  __shared__ float w2c[C2 * KS * KS];  // W2[c][ci][ky][kx] of this ci
  __shared__ float gq[4][P1 * P1];     // dZ1 quarter sums (conv2 channels 5 q .. 5 q + 4)
  __shared__ float g1[P1 * P1];
  const int n = blockIdx.x / C1, ci = blockIdx.x % C1, t = threadIdx.x;
  STAMP(0);
  if (stamps && t == 0) stamps[(size_t)blockIdx.x * 16 + 14] = (long long)__builtin_amdgcn_s_memrealtime();
  const float* wsn = bws + (size_t)n * BWS;
  float* R = rec + (size_t)n * REC;
  // every global load of the workgroup is issued before the first LDS store (one latency, not one per loop
  // round: these bytes were just written by the sample kernel on other XCDs); 16-B loads where aligned
  // (BWS and 784 floats are multiples of 4)
  f32x4 g2v = {}, xv = {};
  float w2v = 0.f, z1v = 0.f;
  unsigned char a1v = 0;
  if (t < C2 * O2 * O2 / 4) g2v = reinterpret_cast<const f32x4*>(wsn)[t];
  if (t < IMG * IMG / 4) xv = reinterpret_cast<const f32x4*>(x + (size_t)n * IMG * IMG)[t];
  if (t < C2 * KS * KS) w2v = cw2[((t / (KS * KS)) * C1 + ci) * KS * KS + t % (KS * KS)];
  if (t < P1 * P1) {
    z1v = wsn[C2 * O2 * O2 + ci * P1 * P1 + t];
    a1v = reinterpret_cast<const unsigned char*>(wsn + C2 * O2 * O2 + NZ1)[ci * P1 * P1 + t];
  }
  if (t < C2 * O2 * O2 / 4) reinterpret_cast<f32x4*>(G2)[t] = g2v;
  if (t < IMG * IMG / 4) reinterpret_cast<f32x4*>(xs)[t] = xv;
  if (t < C2 * KS * KS) w2c[t] = w2v;
  if (t < P1 * P1) {
    z1c[t] = z1v;
    a1c[t] = a1v;
  }
  __syncthreads();
  STAMP(1);
  // the conv2 pool argmax of every pooled cell: the one nonzero of G2 in it (G2 is zero elsewhere)
  for (int o = t; o < FLAT; o += TBW) {
    const int c = o / (P2 * P2), py = (o / P2) % P2, px = o % P2;
    int arg = 0;
    float gv = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const float v = G2[(c * O2 + 2 * py + (d >> 1)) * O2 + 2 * px + (d & 1)];
      if (v != 0.f) {
        arg = d;
        gv = v;
      }
    }
    a2s[o] = (unsigned char)arg;
    cellg[o] = gv;
  }
  __syncthreads();
  STAMP(2);
  // dZ1[ci][Y][X] = sum_c sum_{ky,kx} G2[c][Y - ky][X - kx] W2[c][ci][ky][kx]: 4 channel quarters x 144 positions.
  // G2 has one nonzero per pooled cell (at its argmax), so the 5 x 5 window of (Y, X) meets at most 3 x 3
  // cells per channel: 45 candidate terms per thread instead of the dense 125 (fixed trip counts, predicated)
  {
    const int q = t / (P1 * P1), pos = t % (P1 * P1);  // t < 576 = 4 x 144
    const int Y = pos / P1, X = pos % P1;
    const int py0 = max(Y - (KS - 1), 0) >> 1, px0 = max(X - (KS - 1), 0) >> 1;
    float acc = 0.f;
    // candidate cell k = (py, px) of the 3 x 3 around (Y, X): the cell's nonzero sits at (2 py + (d >> 1),
    // 2 px + (d & 1)), d its argmax; tap (ky, kx) = (by - (d >> 1), bx - (d & 1)) with (by, bx) = (Y - 2 py,
    // X - 2 px). Which d land inside the 5 x 5 window is fixed per candidate (a 4-bit mask), so per channel
    // a candidate costs 3 LDS reads (argmax byte, the cell's G2 value, the W2 tap) and a select. The index
    // math of the per-channel form was VALU-bound across the 27 waves a CU holds (13.8K of the block's 20K
    // cycles); invalid candidates add an exact 0.
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int py = py0 + k / 3, px = px0 + k % 3;
      const int by = Y - 2 * py, bx = X - 2 * px;
      unsigned vm = 0u;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int ky = by - (d >> 1), kx = bx - (d & 1);
        vm |= (py < P2 && px < P2 && ky >= 0 && ky < KS && kx >= 0 && kx < KS) ? (1u << d) : 0u;
      }
      const int cell = min(py, P2 - 1) * P2 + min(px, P2 - 1);
      const int wb = by * KS + bx;  // tap index of d = 0 (out of range for invalid candidates: clamped below)
#pragma unroll
      for (int c = 5 * q; c < 5 * q + 5; ++c) {
        const int d = a2s[c * P2 * P2 + cell];
        const float g = cellg[c * P2 * P2 + cell];
        const float w = w2c[c * KS * KS + min(max(wb - (d >> 1) * KS - (d & 1), 0), KS * KS - 1)];
        acc += ((vm >> d) & 1u) ? g * w : 0.f;
      }
    }
    gq[q][pos] = acc;
  }
  __syncthreads();
  STAMP(3);
  if (t < P1 * P1) g1[t] = z1c[t] > 0.f ? (gq[0][t] + gq[1][t]) + (gq[2][t] + gq[3][t]) : 0.f;  // ReLU mask
  __syncthreads();
  STAMP(4);
  // dW1[ci][ky][kx] = sum over the 144 pooled positions of g1 * x at the argmax tap: 16 lanes per weight
  // (positions p, p + 16, ...), then a fixed xor tree over the 16; db1 by the threads after them
  if (t < KS * KS * 16) {
    const int wi = t >> 4, prt = t & 15;
    const int ky = wi / KS, kx = wi % KS;
    float acc = 0.f;
    float gv[9], xv9[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {  // (reads first, then the 9 FMAs in position order)
      const int q = prt + 16 * k;
      const int py = q / P1, px = q % P1, d = a1c[q];
      gv[k] = g1[q];
      xv9[k] = xs[(2 * py + (d >> 1) + ky) * IMG + 2 * px + (d & 1) + kx];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) acc += gv[k] * xv9[k];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    acc += __shfl_xor(acc, 8);
    if (prt == 0) R[R_W1C + ci * KS * KS + wi] = acc;
  } else if (t < KS * KS * 16 + 16) {  // db1: 16 lanes (9 positions each) and the same xor tree
    const int prt = t & 15;
    float acc = 0.f;
#pragma unroll
    for (int q = prt; q < P1 * P1; q += 16) acc += g1[q];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    acc += __shfl_xor(acc, 8);
    if (prt == 0) R[R_B1C + ci] = acc;
  } else if (t >= DW2_T0 && t < DW2_T0 + C2 * KS) {  // dW2 (moved here: beside dW1, not before dZ1)
    // dW2[c][ci][ky][:] from the 16 cells of channel c (their argmax entries; G2 is 0 at the other 48)
    const int c = (t - DW2_T0) / KS, ky = (t - DW2_T0) % KS;
    float acc[KS] = {0.f, 0.f, 0.f, 0.f, 0.f};
    // all 16 argmax reads first, then every G2 / z1 read, then the FMAs in cell order (one LDS latency per
    // step instead of one per cell)
    int dq[P2 * P2];
#pragma unroll
    for (int q = 0; q < P2 * P2; ++q) dq[q] = a2s[c * P2 * P2 + q];
#pragma unroll
    for (int q = 0; q < P2 * P2; ++q) {
      const int py = q / P2, px = q % P2, d = dq[q];
      const int y = 2 * py + (d >> 1), xx = 2 * px + (d & 1);
      const float g = G2[(c * O2 + y) * O2 + xx];
      const float* zr = z1c + (y + ky) * P1 + xx;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) acc[kx] += g * zr[kx];
    }
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) R[R_W2C + ((c * C1 + ci) * KS + ky) * KS + kx] = acc[kx];
  } else if (ci == 0 && t >= DB2_T0 && t < DB2_T0 + 2 * C2) {  // db2: 2 lanes per channel (32 cells each)
    const int c = (t - DB2_T0) >> 1, k = t & 1;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < O2 * O2 / 2; ++i) acc += G2[c * O2 * O2 + k + 2 * i];
    acc += __shfl_xor(acc, 1);
    if (k == 0) R[R_B2C + c] = acc;
  }
  if (stamps) {
    __syncthreads();
    STAMP(5);
    if (t == 0) stamps[(size_t)blockIdx.x * 16 + 15] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

struct CnnParams {
  float* p[8];    // conv1.w, conv1.b, conv2.w, conv2.b, fc1.w, fc1.b, fc2.w, fc2.b
  float* buf[8];  // momentum buffers (nullptr without momentum)
  float lr, mom, damp, wd;
  int nesterov, first;
};

// torch.optim.SGD on one parameter (sgd_rule.h's operations, explicit fmas); pv / bv: the parameter and its
// momentum buffer, loaded by the caller ahead of the gradient sums (their latency overlaps the record loads)
__device__ __forceinline__ void sgd_update1(float* pp, float* bp, float d, const CnnParams& a, float pv, float bv) {
#pragma clang fp contract(off)
  if (a.wd != 0.f) d = __builtin_fmaf(a.wd, pv, d);
  if (a.mom != 0.f) {
    float b = d;
    if (!a.first) b = __builtin_fmaf(a.mom, bv, (1.f - a.damp) * d);
    *bp = b;
    d = a.nesterov ? __builtin_fmaf(a.mom, b, d) : b;
  }
  *pp = __builtin_fmaf(-a.lr, d, pv);
}

// The update: a block = 32 parameters x 8 sample groups (group g sums samples g, g + 8, g + 16, ... with up to
// 8 loads in flight), the 8 group partials meet in LDS and are added in a fixed order (deterministic). A
// thread per parameter summing all B records in sequence was bound by B dependent round trips to records
// that other XCDs had just written (37 us at B = 60; 8-way unrolled, 14 us).
constexpr int UP = 32, UG = 8;  // parameters and sample groups per block (256 threads)

// (the loads are unconditional - past-the-end samples re-read sample B - 1 and are dropped by a select - so all
// 8 (16) of them are in flight at once: with `if (s < B) acc += r[o]` hipcc put each load in its own branch with
// a vmcnt(0) behind it, 8 serial round trips, 10.8 us at B = 60)
template <bool PROD>
__device__ __forceinline__ float group_sum(const float* __restrict__ rec, int B, int g, int o, int o2) {
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s0 = g; s0 < B; s0 += UG * 8) {
    float xa[8], xb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float* r = rec + (size_t)min(s0 + UG * u, B - 1) * REC;
      xa[u] = r[o];
      xb[u] = PROD ? r[o2] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float v = PROD ? __builtin_fmaf(xa[u], xb[u], acc[u]) : acc[u] + xa[u];
      acc[u] = s0 + UG * u < B ? v : acc[u];
    }
  }
  return ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

// parameter tensor q's pointer without indexing the kernel-argument array by a per-thread value (that put the
// array in scratch memory; a plain select chain became a vector load from the argument segment, one more
// dependent round trip): the 8 pointers are pinned in SGPRs first, then selected per lane
__device__ __forceinline__ float* pick8(float* const (&v)[8], int q) {
  float* w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[k] = v[k];
    asm volatile("" : "+s"(w[k]));
  }
  float* r = w[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) r = q == k ? w[k] : r;
  return r;
}

__global__ void __launch_bounds__(256) cnn_step_update_kernel(const float* __restrict__ rec, int B, CnnParams a,
                                                              float* __restrict__ stats, long long* ctr) {
  constexpr int n0 = C1 * KS * KS, n1 = C1, n2 = C2 * C1 * KS * KS, n3 = C2, n4 = HID * FLAT, n5 = HID,
                n6 = NCLS * HID, n7 = NCLS;
  constexpr int total = n0 + n1 + n2 + n3 + n4 + n5 + n6 + n7;
  __shared__ float part[UG][UP];
  const int j = threadIdx.x % UP, g = threadIdx.x / UP;
  const int i = blockIdx.x * UP + j;
  // the parameter this column updates (tensor ti, element): its value and momentum are loaded now, under the
  // record loads below
  float pv = 0.f, bv = 0.f;
  if (g == 0 && i < total) {
    int tt = 0, ee = i;
    const int sizes[8] = {n0, n1, n2, n3, n4, n5, n6, n7};
#pragma unroll
    for (int q = 0; q < 7; ++q)
      if (tt == q && ee >= sizes[q]) {
        ee -= sizes[q];
        tt = q + 1;
      }
    pv = pick8(a.p, tt)[ee];
    float* bq = pick8(a.buf, tt);
    if (bq && !a.first) bv = bq[ee];
  }
  int ti = -1, e = i;
  float v = 0.f;
  if (i < total) {
    if (e < n0) {
      ti = 0;
      v = group_sum<false>(rec, B, g, R_W1C + e, 0);
    } else if ((e -= n0) < n1) {
      ti = 1;
      v = group_sum<false>(rec, B, g, R_B1C + e, 0);
    } else if ((e -= n1) < n2) {
      ti = 2;
      v = group_sum<false>(rec, B, g, R_W2C + e, 0);
    } else if ((e -= n2) < n3) {
      ti = 3;
      v = group_sum<false>(rec, B, g, R_B2C + e, 0);
    } else if ((e -= n3) < n4) {
      ti = 4;
      v = group_sum<true>(rec, B, g, R_DH + e / FLAT, R_Z3 + e % FLAT);
    } else if ((e -= n4) < n5) {
      ti = 5;
      v = group_sum<false>(rec, B, g, R_DH + e, 0);
    } else if ((e -= n5) < n6) {
      ti = 6;
      v = group_sum<true>(rec, B, g, R_DL + e / HID, R_HD + e % HID);
    } else {
      e -= n6;
      ti = 7;
      v = group_sum<false>(rec, B, g, R_DL + e, 0);
    }
  }
  part[g][j] = v;
  __syncthreads();
  if (g == 0 && ti >= 0) {
    const float gr = ((part[0][j] + part[1][j]) + (part[2][j] + part[3][j])) +
                     ((part[4][j] + part[5][j]) + (part[6][j] + part[7][j]));
    float* bq = pick8(a.buf, ti);
    sgd_update1(pick8(a.p, ti) + e, bq ? bq + e : nullptr, gr, a, pv, bv);
  }
  if (blockIdx.x == 0) {  // (loss sum, correct): 256 strided partials, then a fixed-order tree (deterministic).
    // (A serial loop over the B records on two threads was B dependent round trips to records other XCDs had
    // just written: it set this kernel's length, ~14 us at B = 60.)
    __shared__ float st[2][256];
    float l = 0.f, c = 0.f;
    for (int s = threadIdx.x; s < B; s += 256) {
      l += rec[(size_t)s * REC + R_LOSS];
      c += rec[(size_t)s * REC + R_LOSS + 1];
    }
    st[0][threadIdx.x] = l;
    st[1][threadIdx.x] = c;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) {
        st[0][threadIdx.x] += st[0][threadIdx.x + w];
        st[1][threadIdx.x] += st[1][threadIdx.x + w];
      }
      __syncthreads();
    }
    if (threadIdx.x < 2) stats[threadIdx.x] = st[threadIdx.x][0];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0 && ctr) *ctr += 1;  // this step's masks are drawn
}

}  // namespace


int ref_cnn_idx_bytes() { return NIDX; }
int ref_cnn_z1_floats() { return NZ1; }

void ref_cnn_stage0_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                        float* z1_save, unsigned char* idx_save, int B, unsigned long long seed, const long long* ctr,
                        unsigned sample0, float p, bool drop, hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cnn_s0_fwd_kernel, dim3(B), dim3(TF), 0, stream, x, w1, b1, w2, b2, out, z1_save, idx_save,
                     seed, ctr, sample0, p, drop ? 1 : 0);
}

void ref_cnn_stage0_bwd(const float* x, const float* w2, const float* out, const float* gout, const float* z1_save,
                        const unsigned char* idx_save, int B, unsigned long long seed, const long long* ctr,
                        unsigned sample0, float p, bool drop, float* gw1, float* gb1, float* gw2, float* gb2,
                        hipStream_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(cnn_s0_bwd_kernel, dim3(B), dim3(TB), 0, stream, x, w2, out, gout, z1_save, idx_save, seed, ctr,
                     sample0, p, drop ? 1 : 0, gw1, gb1, gw2, gb2);
}

void ref_cnn_stage1(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                    const int64_t* target, int B, unsigned long long seed, const long long* ctr, unsigned sample0,
                    float p, bool drop, float scale, float* stats, float* dx, float* gw1, float* gb1, float* gw2,
                    float* gb2, hipStream_t stream) {
  if (B <= 0) return;
  // small batches: 8 rows per block (spread over CUs); large: 32 (fewer dW1 atomics per sample)
  if (B <= 4096) {
    hipLaunchKernelGGL(cnn_s1_kernel<8>, dim3((B + 7) / 8), dim3(T1), 0, stream, x, w1, b1, w2, b2, target, B, seed,
                       ctr, sample0, p, drop ? 1 : 0, scale, stats, dx, gw1, gb1, gw2, gb2);
  } else {
    hipLaunchKernelGGL(cnn_s1_kernel<32>, dim3((B + 31) / 32), dim3(T1), 0, stream, x, w1, b1, w2, b2, target, B,
                       seed, ctr, sample0, p, drop ? 1 : 0, scale, stats, dx, gw1, gb1, gw2, gb2);
  }
}

int ref_cnn_step_record_floats() { return REC; }
int ref_cnn_step_workspace_floats(int B) { return B * REC + (B <= 128 ? B * BWS : 0); }

void ref_cnn_step(const float* x, const int64_t* target, int B, float* const* params, float* const* bufs,
                  unsigned long long seed0, unsigned long long seed1, long long* ctr, float p0, bool drop0, float p1,
                  bool drop1, float scale, float lr, float mom, float damp, float wd, bool nesterov, bool first,
                  float* rec, float* stats, hipStream_t stream, long long* stamps) {
  if (B <= 0) return;
  // B <= 128 (the reference's 60): stage 0's backward as its own launch over 10 workgroups per sample
  // stamps (diagnostics, tools/probes): the sample kernel's phases on the unsplit path, or with knob CNN_SPLIT_BWD = 2
  // the split backward kernel's ([B * 10][16] slots)
  const int split = knob(KNOB_CNN_SPLIT_BWD);
  float* bws = (B <= 128 && split && (!stamps || split == 2)) ? rec + (size_t)B * REC : nullptr;
  hipLaunchKernelGGL(cnn_step_sample_kernel, dim3(B), dim3(TS), 0, stream, x, target, params[0], params[1], params[2],
                     params[3], params[4], params[5], params[6], params[7], seed0, seed1, ctr, p0, drop0 ? 1 : 0, p1,
                     drop1 ? 1 : 0, scale, rec, bws ? nullptr : stamps, bws);
  if (bws)
    hipLaunchKernelGGL(cnn_step_bwd_kernel, dim3(B * C1), dim3(TBW), 0, stream, x, params[2], bws, rec,
                       split == 2 ? stamps : nullptr);
  CnnParams a;
  for (int i = 0; i < 8; ++i) {
    a.p[i] = params[i];
    a.buf[i] = bufs[i];
  }
  a.lr = lr;
  a.mom = mom;
  a.damp = damp;
  a.wd = wd;
  a.nesterov = nesterov ? 1 : 0;
  a.first = first ? 1 : 0;
  constexpr int total = C1 * KS * KS + C1 + C2 * C1 * KS * KS + C2 + HID * FLAT + HID + NCLS * HID + NCLS;
  hipLaunchKernelGGL(cnn_step_update_kernel, dim3((total + UP - 1) / UP), dim3(256), 0, stream, rec, B, a, stats, ctr);
}

}  // namespace sdml
