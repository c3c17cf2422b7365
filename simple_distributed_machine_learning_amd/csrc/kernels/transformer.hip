// Transformer-stage kernels for the GPT-2 pipeline config (BASELINE config 5, bf16):
//
// * vocab cross-entropy: bf16 logits [rows, V] -> per-row loss, argmax-correct and (training)
//   dlogits = scale * (softmax - onehot) in bf16. One read pass for max/sum (online softmax),
//   one read+write pass for the gradient: no fp32 copy of the [rows, 50257] logits.
// * LayerNorm forward/backward: bf16 I/O, fp32 statistics (mean, rstd saved for backward),
//   weight/bias grads reduced per block into an fp32 slab and summed by a second pass.
//
// One workgroup (256 threads) per row for the vocab kernels (a 50257-wide row is 98 KiB of
// bf16), grid-stride over rows for LayerNorm (768-wide rows, one wave per row, 16-B loads).
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // RNE, NaN-preserving (hardware cvt)
  return *reinterpret_cast<u16*>(&h);
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// ---------------------------------------------------------------------------------------------
// vocab cross-entropy
constexpr int CE_T = 256;

__global__ void __launch_bounds__(CE_T) ce_fwd_bwd_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                          int rows, int V, int ld, float scale, int ignore_index,
                                                          float* __restrict__ row_loss, float* __restrict__ row_ok,
                                                          u16* __restrict__ dlogits) {
  __shared__ float sm[CE_T / 64], ss[CE_T / 64];
  __shared__ int si[CE_T / 64];
  const int row = blockIdx.x;
  if (row >= rows) return;
  const u16* z = logits + (size_t)row * ld;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // pass 1: online max / sum-exp + argmax (vectorised 8 x bf16 when aligned)
  float m = -INFINITY, s = 0.f;
  int am = 0;
  const bool vec = (V % 8 == 0) && (ld % 8 == 0) && ((reinterpret_cast<uintptr_t>(z) & 15) == 0);
  auto consume = [&](float v, int idx) {
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
      am = idx;
    } else {
      s += __expf(v - m);
    }
  };
  if (vec) {
    for (int i = t * 8; i < V; i += CE_T * 8) {
      u16x8 v = *reinterpret_cast<const u16x8*>(z + i);
#pragma unroll
      for (int e = 0; e < 8; ++e) consume(bf2f(v[e]), i + e);
    }
  } else {
    for (int i = t; i < V; i += CE_T) consume(bf2f(z[i]), i);
  }
  // combine (m, s, argmax) across the wave, then across waves
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
    int a2 = __shfl_xor(am, o);
    float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    if (m2 > m || (m2 == m && a2 < am)) am = a2;
    m = mn;
  }
  if (lane == 0) {
    sm[w] = m;
    ss[w] = s;
    si[w] = am;
  }
  __syncthreads();
  float M = sm[0], S = 0.f;
  int AM = si[0];
  for (int i = 1; i < CE_T / 64; ++i)
    if (sm[i] > M || (sm[i] == M && si[i] < AM)) {
      M = sm[i];
      AM = si[i];
    }
  for (int i = 0; i < CE_T / 64; ++i) S += ss[i] * __expf(sm[i] - M);
  const float lse = M + __logf(S);
  const int y = (int)tgt[row];
  const bool valid = y != ignore_index && y >= 0 && y < V;
  if (t == 0) {
    row_loss[row] = valid ? lse - bf2f(z[y]) : 0.f;
    row_ok[row] = (valid && AM == y) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  u16* g = dlogits + (size_t)row * ld;
  const float sc = valid ? scale : 0.f;
  if (vec) {
    for (int i = t * 8; i < V; i += CE_T * 8) {
      u16x8 v = *reinterpret_cast<const u16x8*>(z + i);
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float p = __expf(bf2f(v[e]) - lse);
        o[e] = f2bf(sc * (p - (i + e == y ? 1.f : 0.f)));
      }
      *reinterpret_cast<u16x8*>(g + i) = o;
    }
  } else {
    for (int i = t; i < V; i += CE_T) {
      float p = __expf(bf2f(z[i]) - lse);
      g[i] = f2bf(sc * (p - (i == y ? 1.f : 0.f)));
    }
  }
  for (int i = V + t; i < ld; i += CE_T) g[i] = 0;  // padded rows (ld > V): zero gradient columns
}

// Register-resident variant (V <= 512 threads * 8 * CE_NVMAX): the row is read from HBM ONCE
// into registers (16-B loads over the row's 16-B aligned body; the unaligned head/tail elements of
// an odd vocabulary like GPT-2's 50257 go one per thread), then max/argmax, sum-exp and dlogits
// are all computed from registers: one read and one write of the logits per row (the online
// kernel above reads them twice and, for odd V, element by element).
constexpr int CER_T = 512;  // 2 waves/SIMD per workgroup: up to 256 VGPRs for the resident row
constexpr int CE_NVMAX = 16;
constexpr u16 BF16_NEG_INF = 0xFF80;

// MINW: waves per SIMD the register budget is held to. GPT-2's rows (13 vectors per thread) at MINW = 4 (<= 128 VGPRs,
// 10 spilled) run two 8-wave rows per CU instead of one: 792 -> 697 us per call (one rocprofv3 pair, round 6)
template <int NV, int MINW = 1>
__global__ void __launch_bounds__(CER_T, MINW) ce_reg_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       int rows, int V, int ld, float scale, int ignore_index,
                                                       float* __restrict__ row_loss, float* __restrict__ row_ok,
                                                       u16* __restrict__ dlogits) {
  __shared__ float red_m[CER_T / 64], red_s[CER_T / 64];
  __shared__ int red_i[CER_T / 64];
  const int row = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const u16* z = logits + (size_t)row * ld;
  int head = (int)(((16 - (reinterpret_cast<uintptr_t>(z) & 15)) & 15) >> 1);
  if (head > V) head = V;
  const int nvec = (V - head) >> 3;
  const int tail0 = head + 8 * nvec, ntail = V - tail0;
  u16x8 v[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int vi = t + u * CER_T;
    if (vi < nvec) {
      v[u] = *reinterpret_cast<const u16x8*>(z + head + 8 * vi);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[u][e] = BF16_NEG_INF;
    }
  }
  // unaligned head (t < head) and tail (t < ntail) elements, one each per thread
  const float xh = t < head ? bf2f(z[t]) : -INFINITY;
  const float xt = t < ntail ? bf2f(z[tail0 + t]) : -INFINITY;
  // block max (values stay packed bf16 in registers; unpacking is one shift)
  float mx = fmaxf(xh, xt);
#pragma unroll
  for (int u = 0; u < NV; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) mx = fmaxf(mx, bf2f(v[u][e]));
  mx = wave_max(mx);
  if (lane == 0) red_m[w] = mx;
  __syncthreads();
  float M = red_m[0];
#pragma unroll
  for (int i = 1; i < CER_T / 64; ++i) M = fmaxf(M, red_m[i]);
  // first index holding the max (torch.argmax semantics)
  int am = 0x7fffffff;
  if (xh == M) am = t;
#pragma unroll
  for (int u = 0; u < NV; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (bf2f(v[u][e]) == M) am = min(am, head + 8 * (t + u * CER_T) + e);
  if (xt == M) am = min(am, tail0 + t);
  for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o));
  if (lane == 0) red_i[w] = am;
  __syncthreads();
  int AM = red_i[0];
#pragma unroll
  for (int i = 1; i < CER_T / 64; ++i) AM = min(AM, red_i[i]);
  // sum of exp from registers
  float se = 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) se += __expf(bf2f(v[u][e]) - M);
  se += __expf(xh - M) + __expf(xt - M);
  se = wave_sum(se);
  if (lane == 0) red_s[w] = se;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int i = 0; i < CER_T / 64; ++i) S += red_s[i];
  const float lse = M + __logf(S);
  const int y = (int)tgt[row];
  const bool valid = y != ignore_index && y >= 0 && y < V;
  if (t == 0) {
    row_loss[row] = valid ? lse - bf2f(z[y]) : 0.f;
    row_ok[row] = (valid && AM == y) ? 1.f : 0.f;
  }
  if (!dlogits) return;
  u16* g = dlogits + (size_t)row * ld;  // same alignment as the logits row (same ld)
  const float sc = valid ? scale : 0.f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int vi = t + u * CER_T;
    if (vi < nvec) {
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int idx = head + 8 * vi + e;
        o[e] = f2bf(sc * (__expf(bf2f(v[u][e]) - lse) - (idx == y ? 1.f : 0.f)));
      }
      *reinterpret_cast<u16x8*>(g + head + 8 * vi) = o;
    }
  }
  if (t < head) g[t] = f2bf(sc * (__expf(xh - lse) - (t == y ? 1.f : 0.f)));
  if (t < ntail) g[tail0 + t] = f2bf(sc * (__expf(xt - lse) - (tail0 + t == y ? 1.f : 0.f)));
  // padded rows (ld > V, the lm_head's vocabulary padded to a multiple of 64 in ops/linear.py lm_head): the pad
  // columns' gradient is zero, so the GEMMs that read the padded dlogits (input and weight gradient) see exact zeros
  for (int i = V + t; i < ld; i += CER_T) g[i] = 0;
}

// ---------------------------------------------------------------------------------------------
// LayerNorm (row width D <= 4096, D % 8 == 0): one wave per row, fp32 statistics.
constexpr int LN_T = 256;
// LN_MAXV = 16-B chunks per lane (template): D <= 64 lanes * 8 elems * LN_MAXV

// res != nullptr: the row is first the residual sum xs = bf16(x + res) (stored to xs, exactly the
// unfused bf16 add), and the statistics are those of xs — one pass instead of add + LayerNorm
template <int LN_MAXV>
__global__ void __launch_bounds__(LN_T) ln_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ res,
                                                      const u16* __restrict__ w, const u16* __restrict__ b,
                                                      u16* __restrict__ xs, u16* __restrict__ y,
                                                      float* __restrict__ mean, float* __restrict__ rstd, int rows,
                                                      int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int nch = D / 8;
  // this lane's gamma / beta chunks, once (they were re-read for every row)
  u16x8 wv[LN_MAXV], bv[LN_MAXV];
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    const int ch = min(lane + 64 * c, nch - 1);
    wv[c] = *reinterpret_cast<const u16x8*>(w + 8 * ch);
    bv[c] = *reinterpret_cast<const u16x8*>(b + 8 * ch);
  }
  for (int row = blockIdx.x * (LN_T / 64) + (threadIdx.x >> 6); row < rows; row += gridDim.x * (LN_T / 64)) {
    const u16* xr = x + (size_t)row * D;
    u16x8 v[LN_MAXV];
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch) {
        v[c] = *reinterpret_cast<const u16x8*>(xr + 8 * ch);
        if (res) {
          const u16x8 rv = *reinterpret_cast<const u16x8*>(res + (size_t)row * D + 8 * ch);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[c][e] = f2bf(bf2f(v[c][e]) + bf2f(rv[e]));
          *reinterpret_cast<u16x8*>(xs + (size_t)row * D + 8 * ch) = v[c];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) sum += bf2f(v[c][e]);
      }
    }
    const float mu = wave_sum(sum) / D;
    float var = 0.f;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float d = bf2f(v[c][e]) - mu;
          var += d * d;
        }
    }
    const float rs = rsqrtf(wave_sum(var) / D + eps);
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
    u16* yr = y + (size_t)row * D;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch) {
        u16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf((bf2f(v[c][e]) - mu) * rs * bf2f(wv[c][e]) + bf2f(bv[c][e]));
        *reinterpret_cast<u16x8*>(yr + 8 * ch) = o;
      }
    }
  }
}

// dx = rstd * (g*w - mean(g*w) - xhat * mean(g*w*xhat)) (+ gadd: the residual-path gradient of
// a fused add + LayerNorm, summed in fp32 and rounded once); dw += g*xhat; db += g (per-block slabs)
template <int LN_MAXV>
__global__ void __launch_bounds__(LN_T) ln_bwd_kernel(const u16* __restrict__ x, const u16* __restrict__ w,
                                                      const u16* __restrict__ gy, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, const u16* __restrict__ gadd,
                                                      u16* __restrict__ dx, float* __restrict__ part, int rows, int D) {
  const int lane = threadIdx.x & 63, wv_id = threadIdx.x >> 6;
  const int nch = D / 8;
  // per-thread partial dW/dB for the chunks this lane owns (reduced over the block's rows)
  float pw[LN_MAXV][8], pb[LN_MAXV][8];
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) pw[c][e] = pb[c][e] = 0.f;
  // this lane's gamma chunks, once (they were re-read twice per row)
  u16x8 wc[LN_MAXV];
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) wc[c] = *reinterpret_cast<const u16x8*>(w + 8 * min(lane + 64 * c, nch - 1));
  for (int row = blockIdx.x * (LN_T / 64) + wv_id; row < rows; row += gridDim.x * (LN_T / 64)) {
    const u16* xr = x + (size_t)row * D;
    const u16* gr = gy + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    u16x8 xv[LN_MAXV], gv[LN_MAXV], av[LN_MAXV];
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch) {
        xv[c] = *reinterpret_cast<const u16x8*>(xr + 8 * ch);
        gv[c] = *reinterpret_cast<const u16x8*>(gr + 8 * ch);
        // the residual-path gradient with the row's other loads (it was a second round trip after the reductions)
        av[c] = gadd ? *reinterpret_cast<const u16x8*>(gadd + (size_t)row * D + 8 * ch) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        const u16x8 wv = wc[c];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float xh = (bf2f(xv[c][e]) - mu) * rs;
          float g = bf2f(gv[c][e]);
          float gw = g * bf2f(wv[e]);
          s1 += gw;
          s2 += gw * xh;
          pw[c][e] += g * xh;
          pb[c][e] += g;
        }
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
    u16* dr = dx + (size_t)row * D;
#pragma unroll
    for (int c = 0; c < LN_MAXV; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch) {
        const u16x8 wv = wc[c];
        u16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float xh = (bf2f(xv[c][e]) - mu) * rs;
          o[e] = f2bf(rs * (bf2f(gv[c][e]) * bf2f(wv[e]) - s1 - xh * s2) + bf2f(av[c][e]));
        }
        *reinterpret_cast<u16x8*>(dr + 8 * ch) = o;
      }
    }
  }
  // block reduction of the 4 waves' partials through LDS, then one slab row per block
  __shared__ float red[LN_T / 64][2 * 64 * 8];
  float* slab = part + (size_t)blockIdx.x * 2 * D;
#pragma unroll
  for (int c = 0; c < LN_MAXV; ++c) {
    int ch = lane + 64 * c;
    if (64 * c >= nch) break;  // uniform
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wv_id][lane * 8 + e] = pw[c][e];
      red[wv_id][512 + lane * 8 + e] = pb[c][e];
    }
    __syncthreads();
    if (wv_id == 0 && ch < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float a = 0.f, bsum = 0.f;
        for (int q = 0; q < LN_T / 64; ++q) {
          a += red[q][lane * 8 + e];
          bsum += red[q][512 + lane * 8 + e];
        }
        slab[8 * ch + e] = a;
        slab[D + 8 * ch + e] = bsum;
      }
    }
    __syncthreads();
  }
}

// out[o] += sum_b part[b][o] (deterministic order). 64 outputs x 16 waves per block; wave w
// sums slabs w, w+16, ... with 8 loads in flight, partials added in LDS in wave order.
__global__ void __launch_bounds__(1024) slab_sum_kernel(const float* __restrict__ part, int nblocks, int width,
                                                        float* __restrict__ out) {
  __shared__ float acc[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (o < width) {
    int b = w;
    for (; b + 16 * 7 < nblocks; b += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(b + 16 * u) * width + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nblocks; b += 16) s += part[(size_t)b * width + o];
  }
  acc[w][lane] = s;
  __syncthreads();
  if (w == 0 && o < width) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += acc[i][lane];
    out[o] += t;
  }
}

// same reduction, accumulated straight into bf16 parameter gradients: outputs [0, split) go to
// lo[o], [split, width) to hi[o - split] (hi may be null when split == width)
__global__ void __launch_bounds__(1024) slab_sum_bf16_kernel(const float* __restrict__ part, int nblocks, int width,
                                                             int split, u16* __restrict__ lo, u16* __restrict__ hi) {
  __shared__ float acc[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (o < width) {
    int b = w;
    for (; b + 16 * 7 < nblocks; b += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(b + 16 * u) * width + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nblocks; b += 16) s += part[(size_t)b * width + o];
  }
  acc[w][lane] = s;
  __syncthreads();
  if (w == 0 && o < width) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += acc[i][lane];
    u16* dst = o < split ? lo + o : hi + (o - split);
    *dst = f2bf(bf2f(*dst) + t);
  }
}

// bias gradient partials: part[blockIdx.y][n] = sum over this block's rows of gy[m][n] (fp32).
// Block = 64 columns x 4 row lanes; rows of the block's range are strided by 4.
constexpr int CS_T = 256;
__global__ void __launch_bounds__(CS_T) colsum_partial_kernel(const u16* __restrict__ gy, int M, int N, int ld,
                                                              int rows_per_block, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s = 0.f;
  if (n < N) {
    int r = r0 + rl;
    for (; r + 12 < r1; r += 16) {
      const float a = bf2f(gy[(size_t)r * ld + n]), b = bf2f(gy[(size_t)(r + 4) * ld + n]);
      const float c = bf2f(gy[(size_t)(r + 8) * ld + n]), d = bf2f(gy[(size_t)(r + 12) * ld + n]);
      s += (a + b) + (c + d);
    }
    for (; r < r1; r += 4) s += bf2f(gy[(size_t)r * ld + n]);
  }
  red[rl][lane] = s;
  __syncthreads();
  if (rl == 0 && n < N) part[(size_t)blockIdx.y * N + n] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

}  // namespace

int bias_grad_blocks(int M) {
  int r = (M + 63) / 64;
  return r > 64 ? 64 : (r < 1 ? 1 : r);
}

void bias_grad_bf16(const void* gy, int M, int N, int ld, void* gb, float* workspace, hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  const int R = bias_grad_blocks(M);
  const int rpb = (M + R - 1) / R;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 63) / 64, R), dim3(CS_T), 0, stream,
                     reinterpret_cast<const u16*>(gy), M, N, ld, rpb, workspace);
  hipLaunchKernelGGL(slab_sum_bf16_kernel, dim3((N + 63) / 64), dim3(1024), 0, stream, workspace, R, N, N,
                     reinterpret_cast<u16*>(gb), nullptr);
}

void cross_entropy_bf16(const void* logits, const int64_t* target, int rows, int V, int ld, float scale,
                        int ignore_index, float* row_loss, float* row_ok, void* dlogits, hipStream_t stream) {
  if (rows <= 0) return;
  // register-resident kernel when the row fits (and dlogits shares the logits' alignment)
  const int nvec = (V + 7) / 8;
  const int nv = (nvec + CER_T - 1) / CER_T;
  const bool same_align = !dlogits || ((reinterpret_cast<uintptr_t>(logits) ^ reinterpret_cast<uintptr_t>(dlogits)) & 15) == 0;
  if (nv <= CE_NVMAX && same_align) {
    const u16* L = reinterpret_cast<const u16*>(logits);
    u16* G = reinterpret_cast<u16*>(dlogits);
#define CER(NVV, MW)                                                                                               \
  hipLaunchKernelGGL((ce_reg_kernel<NVV, MW>), dim3(rows), dim3(CER_T), 0, stream, L, target, rows, V, ld, scale, \
                     ignore_index, row_loss, row_ok, G)
    if (nv <= 4) CER(4, 1);
    else if (nv <= 8) CER(8, 1);
    else if (nv <= 13) CER(13, 4);  // GPT-2: V = 50257 -> 13 vectors of 8 per thread, two rows per CU
    else CER(16, 1);
#undef CER
    return;
  }
  hipLaunchKernelGGL(ce_fwd_bwd_kernel, dim3(rows), dim3(CE_T), 0, stream, reinterpret_cast<const u16*>(logits),
                     target, rows, V, ld, scale, ignore_index, row_loss, row_ok, reinterpret_cast<u16*>(dlogits));
}

int layernorm_bwd_blocks(int rows) {
  // one wave per row in flight: 1024 blocks x 4 waves = 16 waves per CU keep enough loads in
  // flight (256 blocks left 4 waves per CU latency-bound: 43 us -> see profiles/); the dW/dB
  // slabs this adds (blocks x 2D fp32) are summed by one extra 6 MB pass
  int b = (rows + 3) / 4;
  return b > 1024 ? 1024 : (b < 1 ? 1 : b);
}

void layernorm_fwd_bf16(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int rows,
                        int D, float eps, hipStream_t stream, const void* res, void* xs) {
  if (rows <= 0) return;
  int blocks = (rows + 3) / 4;
  if (blocks > 4096) blocks = 4096;
#define LNF(V)                                                                                                 \
  hipLaunchKernelGGL((ln_fwd_kernel<V>), dim3(blocks), dim3(LN_T), 0, stream, reinterpret_cast<const u16*>(x), \
                     reinterpret_cast<const u16*>(res), reinterpret_cast<const u16*>(w),                         \
                     reinterpret_cast<const u16*>(b), reinterpret_cast<u16*>(xs), reinterpret_cast<u16*>(y),     \
                     mean, rstd, rows, D, eps)
  if (D <= 512) LNF(1);
  else if (D <= 1024) LNF(2);
  else if (D <= 2048) LNF(4);
  else LNF(8);
#undef LNF
}

void layernorm_bwd_bf16(const void* x, const void* w, const void* gy, const float* mean, const float* rstd, void* dx,
                        float* workspace, float* dw_acc, float* db_acc, int rows, int D, hipStream_t stream) {
  if (rows <= 0) return;
  const int blocks = layernorm_bwd_blocks(rows);
#define LNB(V)                                                                                                 \
  hipLaunchKernelGGL((ln_bwd_kernel<V>), dim3(blocks), dim3(LN_T), 0, stream, reinterpret_cast<const u16*>(x), \
                     reinterpret_cast<const u16*>(w), reinterpret_cast<const u16*>(gy), mean, rstd, nullptr,    \
                     reinterpret_cast<u16*>(dx), workspace, rows, D)
  if (D <= 512) LNB(1);
  else if (D <= 1024) LNB(2);
  else if (D <= 2048) LNB(4);
  else LNB(8);
#undef LNB
  // workspace rows are [dw (D) | db (D)]; sum them separately into the two accumulators
  hipLaunchKernelGGL(slab_sum_kernel, dim3((2 * D + 63) / 64), dim3(1024), 0, stream, workspace, blocks, 2 * D,
                     dw_acc);
  (void)db_acc;  // dw_acc is [2*D]: dw followed by db (caller splits)
}

void layernorm_bwd_bf16_accum(const void* x, const void* w, const void* gy, const float* mean, const float* rstd,
                              void* dx, float* workspace, void* gw, void* gb, int rows, int D, hipStream_t stream,
                              const void* gadd) {
  if (rows <= 0) return;
  const int blocks = layernorm_bwd_blocks(rows);
#define LNB(V)                                                                                                 \
  hipLaunchKernelGGL((ln_bwd_kernel<V>), dim3(blocks), dim3(LN_T), 0, stream, reinterpret_cast<const u16*>(x), \
                     reinterpret_cast<const u16*>(w), reinterpret_cast<const u16*>(gy), mean, rstd,             \
                     reinterpret_cast<const u16*>(gadd), reinterpret_cast<u16*>(dx), workspace, rows, D)
  if (D <= 512) LNB(1);
  else if (D <= 1024) LNB(2);
  else if (D <= 2048) LNB(4);
  else LNB(8);
#undef LNB
  hipLaunchKernelGGL(slab_sum_bf16_kernel, dim3((2 * D + 63) / 64), dim3(1024), 0, stream, workspace, blocks, 2 * D, D,
                     reinterpret_cast<u16*>(gw), reinterpret_cast<u16*>(gb));
}

}  // namespace sdml
