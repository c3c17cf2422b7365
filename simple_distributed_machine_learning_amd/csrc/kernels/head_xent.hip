// Fused classifier head: fc (K -> C) + log_softmax + NLL + the full backward, in ONE launch.
//
// For the 784-128-10 MLP this kernel IS the whole last pipeline stage (reference stage 1
// does fc2 -> log_softmax on worker1 and nll_loss + backward on the master over RPC:
// /root/reference/simple_distributed.py:77-79, :111-112). Per 64-row chunk:
//   1. x chunk [64][128] -> LDS (float4, coalesced); W [C][128], b -> LDS once per block
//   2. 4 threads per row: partial logits over 32 k each, 2-step xor-shuffle reduction
//      -> log-sum-exp, NLL, argmax (correct), dz = scale * (softmax - onehot)
//   3. dx[row][k] = sum_c dz_c W[c][k] written straight from registers (float4)
//   4. dW partial (C x 128 outputs, 5 per thread for C=10) accumulated in registers across
//      all chunks of the block; each block writes one partial slab (dW, db, loss, correct)
//      and a second tiny pass sums the slabs in block order (deterministic, no contention).
// Memory-bound by design (0.5 KiB read + 0.5 KiB written per sample); all MACs on VALU.
// Small batches (<= 2048 rows) use 16-row chunks with 16 threads per row instead.
// Measured and rejected (round 2): 32 lanes per row with W and the dW partial in registers and no
// LDS in the row loop - 75 us vs 49 us at 131072 rows: every lane of a row then redoes the
// row's reduction and softmax, ~2.8x the VALU work per row of this 4-lanes-per-row layout.
//
// head_generic: any K (multiple of 4) / C <= 32: computes loss/dz/dx per row (one wave per
// row); dW/db are then done by the MFMA GEMM (gemm_f32 with fused row-sum).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "head_reduce.h"
#include "head_block.h"
#include "head_tile.h"
#include "kernels.h"

namespace sdml {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HK = 128;     // fused kernel: hidden width
constexpr int CMAX = 16;    // fused kernel: max classes
constexpr int HTHR = 256;
constexpr int XP = HK + 4;  // LDS row pitch of the x chunk

// TPR threads per row: 4 (64-row chunks) for large batches, 16 (16-row chunks) for small ones,
// so a batch of 60 spreads over 4 workgroups instead of serialising through one.
template <int C, int TPR>
__global__ void __launch_bounds__(HTHR) head_fused_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                          const float* __restrict__ bias,
                                                          const int64_t* __restrict__ target, int M, float scale,
                                                          float* __restrict__ part, float* __restrict__ dx,
                                                          int chunks_per_block, int mask_dx, float* __restrict__ dl) {
  constexpr int RWS = HTHR / TPR;  // rows per chunk
  // x chunk; reused at the end for the dW partial reduction ([4 waves][C * HK])
  constexpr int XS = RWS * XP > (HTHR / 64) * C * HK ? RWS * XP : (HTHR / 64) * C * HK;
  __shared__ __attribute__((aligned(16))) float xs[XS];
  __shared__ __attribute__((aligned(16))) float ws[C * HK];
  __shared__ float bs[CMAX];
  constexpr int DZP = (C + 3) / 4 * 4;  // dz row pitch (16-B aligned rows for b128 broadcasts)
  __shared__ __attribute__((aligned(16))) float dzs[RWS * DZP];
  __shared__ float red[2 * HTHR / 64];
  const int t = threadIdx.x;
  // dl: the row's scaled dlogits dz [M][C] instead of (or besides) dx = dz @ W, the factor form of
  // the boundary gradient (head_dx_from_dl rebuilds dx from it bit for bit)
  const bool train = dx != nullptr || dl != nullptr;
  for (int i = t; i < C * HK / 4; i += HTHR)
    reinterpret_cast<f32x4*>(ws)[i] = reinterpret_cast<const f32x4*>(W)[i];
  if (t < C) bs[t] = bias[t];

  constexpr int NOUT = (C * HK + HTHR - 1) / HTHR;  // dW outputs per thread (slab write)
  // dW partial: thread owns k = 4*kq .. 4*kq+3 for every class c, over rows rq, rq+RG, ...
  // of each chunk (one float4 of x and one broadcast dz row per row: 40 FMAs per 4 LDS reads)
  constexpr int RG = HTHR / (HK / 4);  // row groups (8)
  const int kq = t % (HK / 4), rq = t / (HK / 4);
  f32x4 gacc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) gacc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gbacc = 0.f;
  float loss_acc = 0.f, corr_acc = 0.f;

  const int row_in = t / TPR, q = t % TPR;  // TPR threads per row, HK / TPR k each
  // x chunks are prefetched one ahead into registers: chunk ch+1's loads are in flight while
  // chunk ch is computed (the loop is otherwise load -> barrier -> compute, memory idle meanwhile)
  constexpr int NPRE = RWS * HK / 4 / HTHR;
  f32x4 pre[NPRE];
  auto gload = [&](int r0) {
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
      const int idx = t + HTHR * i;
      const int r = idx >> 5, k4 = idx & 31;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (r0 + r < M) v = *reinterpret_cast<const f32x4*>(x + (size_t)(r0 + r) * HK + 4 * k4);
      pre[i] = v;
    }
  };
  gload(blockIdx.x * chunks_per_block * RWS);
  for (int ch = 0; ch < chunks_per_block; ++ch) {
    const int r0 = (blockIdx.x * chunks_per_block + ch) * RWS;
    if (r0 >= M) break;
    __syncthreads();  // previous chunk fully consumed (and ws/bs visible on first pass)
    // stage x chunk
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
      const int idx = t + HTHR * i;
      const int r = idx >> 5, k4 = idx & 31;
      *reinterpret_cast<f32x4*>(xs + r * XP + 4 * k4) = pre[i];
    }
    if (ch + 1 < chunks_per_block) gload(r0 + RWS);
    __syncthreads();
    const int grow = r0 + row_in;
    const bool valid = grow < M;
    float z[C];
#pragma unroll
    for (int c = 0; c < C; ++c) z[c] = 0.f;
    // thread q covers k = 4*(q + TPR*j) .. +3 (interleaved -> conflict-light LDS reads)
#pragma unroll
    for (int j = 0; j < HK / (4 * TPR); ++j) {
      const int k = 4 * (q + TPR * j);
      f32x4 xv = *reinterpret_cast<const f32x4*>(xs + row_in * XP + k);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        f32x4 wv = *reinterpret_cast<const f32x4*>(ws + c * HK + k);
        z[c] += xv[0] * wv[0] + xv[1] * wv[1] + xv[2] * wv[2] + xv[3] * wv[3];
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int off = 1; off < TPR; off <<= 1) z[c] += __shfl_xor(z[c], off);
      z[c] += bs[c];
    }
    float mx = z[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < C; ++c)
      if (z[c] > mx) {
        mx = z[c];
        am = c;
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) se += __expf(z[c] - mx);
    const float lse = mx + __logf(se);
    const int tg = valid ? (int)target[grow] : 0;
    if (valid && q == 0) {
      float zt = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) zt = (c == tg) ? z[c] : zt;
      loss_acc += lse - zt;
      corr_acc += (am == tg) ? 1.f : 0.f;
    }
    if (train) {
      float dz[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float pr = __expf(z[c] - lse);
        dz[c] = valid ? scale * (pr - (c == tg ? 1.f : 0.f)) : 0.f;
      }
      if (q == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) dzs[row_in * DZP + c] = dz[c];
        if (dl && valid) {
#pragma unroll
          for (int c = 0; c < C; ++c) dl[(size_t)grow * C + c] = dz[c];
        }
      }
      if (valid && dx) {
#pragma unroll
        for (int j = 0; j < HK / (4 * TPR); ++j) {
          const int k = 4 * (q + TPR * j);
          f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < C; ++c) {
            f32x4 wv = *reinterpret_cast<const f32x4*>(ws + c * HK + k);
            o += dz[c] * wv;
          }
          if (mask_dx) {  // ReLU backward of the producing stage, fused: x = relu(z) > 0 <=> z > 0
            f32x4 xv = *reinterpret_cast<const f32x4*>(xs + row_in * XP + k);
            o[0] = xv[0] > 0.f ? o[0] : 0.f;
            o[1] = xv[1] > 0.f ? o[1] : 0.f;
            o[2] = xv[2] > 0.f ? o[2] : 0.f;
            o[3] = xv[3] > 0.f ? o[3] : 0.f;
          }
          *reinterpret_cast<f32x4*>(dx + (size_t)grow * HK + k) = o;
        }
      }
      __syncthreads();  // dzs complete
#pragma unroll 2
      for (int r = rq; r < RWS; r += RG) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(xs + r * XP + 4 * kq);
        float d[DZP];
#pragma unroll
        for (int c4 = 0; c4 < DZP / 4; ++c4) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(dzs + r * DZP + 4 * c4);
          d[4 * c4] = v[0];
          d[4 * c4 + 1] = v[1];
          d[4 * c4 + 2] = v[2];
          d[4 * c4 + 3] = v[3];
        }
#pragma unroll
        for (int c = 0; c < C; ++c) gacc[c] += d[c] * xv;
      }
      if (t < C) {
        float s = 0.f;
        for (int r = 0; r < RWS; ++r) s += dzs[r * DZP + t];
        gbacc += s;
      }
    }
  }
  // ---- block partials -> slab (no cross-block atomics: 512 blocks adding into the same
  // 1.3K addresses serialises at the memory side; a slab + one reduce pass does not) ----
  float* slab = part + (size_t)blockIdx.x * (C * HK + C + 2);
  if (train) {
    // row groups rq and rq^1 are lanes l and l^32 of one wave; the 4 waves meet in LDS (the x
    // chunk buffer is free now) in wave order
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) gacc[c][e] += __shfl_xor(gacc[c][e], 32);
    static_assert(RG == 8 && HTHR == 256, "dW partial reduction assumes 8 row groups in 4 waves");
    __syncthreads();  // everyone done reading xs
    float* red4 = xs;  // [4 waves][C * HK]
    if ((t & 63) < 32) {
#pragma unroll
      for (int c = 0; c < C; ++c)
        *reinterpret_cast<f32x4*>(red4 + (t >> 6) * C * HK + c * HK + 4 * kq) = gacc[c];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NOUT; ++u) {
      const int o = t + HTHR * u;
      if (o < C * HK) slab[o] = (red4[o] + red4[C * HK + o]) + (red4[2 * C * HK + o] + red4[3 * C * HK + o]);
    }
    if (t < C) slab[C * HK + t] = gbacc;
  }
  for (int off = 32; off > 0; off >>= 1) {
    loss_acc += __shfl_xor(loss_acc, off);
    corr_acc += __shfl_xor(corr_acc, off);
  }
  if ((t & 63) == 0) {
    red[2 * (t >> 6)] = loss_acc;
    red[2 * (t >> 6) + 1] = corr_acc;
  }
  __syncthreads();
  if (t == 0) {
    float l = 0.f, c = 0.f;
    for (int w = 0; w < HTHR / 64; ++w) {
      l += red[2 * w];
      c += red[2 * w + 1];
    }
    slab[C * HK + C] = l;
    slab[C * HK + C + 1] = c;
  }
}

// sum the per-block slabs: out[o] += sum_b part[b][o] (fixed order -> deterministic), head_reduce.h
__global__ void __launch_bounds__(1024) head_reduce_kernel(HeadReduceArgs a) {
  __shared__ float acc[16][64];
  head_reduce_block(a, blockIdx.x, acc);
}

// grid-stride, one wave per row at a time, any K / C <= 32: loss/correct, dz (to dz_out) and
// dx. Loss/correct stay in registers per wave and leave as one atomic pair per block.
__global__ void __launch_bounds__(256) head_generic_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const int64_t* __restrict__ target, int M, int K, int C,
                                                           float scale, float* __restrict__ stats,
                                                           float* __restrict__ dx, float* __restrict__ dz_out,
                                                           int mask_dx) {
  __shared__ float red[8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float loss_acc = 0.f, corr_acc = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < M; row += gridDim.x * 4) {
    const float* xr = x + (size_t)row * K;
    float z[32];
    for (int c = 0; c < 32; ++c) z[c] = 0.f;
    for (int k = lane; k < K; k += 64) {
      float xv = xr[k];
      for (int c = 0; c < C; ++c) z[c] += xv * W[(size_t)c * K + k];
    }
    for (int c = 0; c < C; ++c) {
      float v = z[c];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      z[c] = v + bias[c];
    }
    float mx = z[0];
    int am = 0;
    for (int c = 1; c < C; ++c)
      if (z[c] > mx) {
        mx = z[c];
        am = c;
      }
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(z[c] - mx);
    const float lse = mx + __logf(se);
    const int tg = (int)target[row];
    float zt = 0.f;
    for (int c = 0; c < C; ++c) zt = (c == tg) ? z[c] : zt;
    loss_acc += lse - zt;
    corr_acc += am == tg ? 1.f : 0.f;
    if (dx || dz_out) {
      float dz[32];
      for (int c = 0; c < C; ++c) dz[c] = scale * (__expf(z[c] - lse) - (c == tg ? 1.f : 0.f));
      if (dz_out && lane < C) {
        float v = 0.f;
        for (int c = 0; c < C; ++c) v = (c == lane) ? dz[c] : v;
        dz_out[(size_t)row * C + lane] = v;
      }
      if (dx)
        for (int k = lane; k < K; k += 64) {
          float o = 0.f;
          for (int c = 0; c < C; ++c) o += dz[c] * W[(size_t)c * K + k];
          dx[(size_t)row * K + k] = (mask_dx && xr[k] <= 0.f) ? 0.f : o;
        }
    }
  }
  if (lane == 0) {
    red[2 * wave] = loss_acc;
    red[2 * wave + 1] = corr_acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = red[0] + red[2] + red[4] + red[6];
    float c = red[1] + red[3] + red[5] + red[7];
    atomicAdd(stats, l);
    atomicAdd(stats + 1, c);
  }
}

// wide-K heads (the 4x1024 MLP: K = 1024, C = 10, 65536 rows): W [C][K] staged in LDS once per
// block and every W chunk read serves two rows; x and dx move as float4. The per-row generic
// kernel above re-read W through the cache for every row (twice): 1.25 ms at 65536 x 1024.
constexpr int HL_MAXJ = 4;  // float4 chunks per lane: K <= 64 * 4 * HL_MAXJ = 1024

// DW: the weight/bias gradients are accumulated per lane (dW[c][its 16 k] += dz[c] x[k]) over the
// block's rows, reduced over the 4 waves through LDS in wave order and written, with the loss and
// correct count, as one slab row [dW | db | loss, correct] per block for head_reduce_kernel (no
// separate dz^T x GEMM re-reading x: 250 us at 65536 x 1024)
template <int C, bool DW>
__global__ void __launch_bounds__(256) head_lds_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                       const float* __restrict__ bias,
                                                       const int64_t* __restrict__ target, int M, int K, float scale,
                                                       float* __restrict__ stats, float* __restrict__ dx,
                                                       float* __restrict__ dz_out, int mask_dx,
                                                       float* __restrict__ part, float* __restrict__ dx_amax) {
  extern __shared__ float4 Ws4[];  // [C][K / 4]
  __shared__ float red[8];
  __shared__ float amx[4];
  float vmax = 0.f;  // max |dx| this wave wrote (dx_amax: per-block bounds for the next split)
  const int nch = K / 4;
  for (int i = threadIdx.x; i < C * nch; i += 256) Ws4[i] = reinterpret_cast<const float4*>(W)[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float bv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) bv[c] = bias[c];
  constexpr int R = 2;  // rows per W read (1 row with DW measured no better: hipcc keeps ~300 registers either way)
  float loss_acc = 0.f, corr_acc = 0.f;
  float4 gacc[DW ? C : 1][HL_MAXJ];
  float gbacc[DW ? C : 1];
  if constexpr (DW) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      gbacc[c] = 0.f;
#pragma unroll
      for (int j = 0; j < HL_MAXJ; ++j) gacc[c][j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  for (int row0 = (blockIdx.x * 4 + wave) * R; row0 < M; row0 += gridDim.x * 4 * R) {
    float4 xv[R][HL_MAXJ];
    float z[R][C];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
#pragma unroll
      for (int c = 0; c < C; ++c) z[rr][c] = 0.f;
#pragma unroll
      for (int j = 0; j < HL_MAXJ; ++j) {
        const int ch = lane + 64 * j;
        xv[rr][j] = (row0 + rr < M && ch < nch) ? reinterpret_cast<const float4*>(x + (size_t)(row0 + rr) * K)[ch]
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < HL_MAXJ; ++j) {
      const int ch = lane + 64 * j;
      if (ch < nch)
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const float4 w = Ws4[c * nch + ch];
#pragma unroll
          for (int rr = 0; rr < R; ++rr)
            z[rr][c] += xv[rr][j].x * w.x + xv[rr][j].y * w.y + xv[rr][j].z * w.z + xv[rr][j].w * w.w;
        }
    }
    float dz[R][C];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float v = z[rr][c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        z[rr][c] = v + bv[c];
      }
      const int row = row0 + rr;
      if (row >= M) {
#pragma unroll
        for (int c = 0; c < C; ++c) dz[rr][c] = 0.f;
        continue;
      }
      float mx = z[rr][0];
      int am = 0;
#pragma unroll
      for (int c = 1; c < C; ++c)
        if (z[rr][c] > mx) {
          mx = z[rr][c];
          am = c;
        }
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) se += __expf(z[rr][c] - mx);
      const float lse = mx + __logf(se);
      const int tg = (int)target[row];
      float zt = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) zt = (c == tg) ? z[rr][c] : zt;
      loss_acc += lse - zt;
      corr_acc += am == tg ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) dz[rr][c] = scale * (__expf(z[rr][c] - lse) - (c == tg ? 1.f : 0.f));
      if (dz_out && lane < C) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) v = (c == lane) ? dz[rr][c] : v;
        dz_out[(size_t)row * C + lane] = v;
      }
    }
    if constexpr (DW) {  // rows past M have dz = 0 and zero x: they add nothing
#pragma unroll
      for (int c = 0; c < C; ++c) {
        #pragma unroll
        for (int rr = 0; rr < R; ++rr) gbacc[c] += dz[rr][c];
#pragma unroll
        for (int j = 0; j < HL_MAXJ; ++j)
#pragma unroll
          for (int rr = 0; rr < R; ++rr) {
            gacc[c][j].x += dz[rr][c] * xv[rr][j].x;
            gacc[c][j].y += dz[rr][c] * xv[rr][j].y;
            gacc[c][j].z += dz[rr][c] * xv[rr][j].z;
            gacc[c][j].w += dz[rr][c] * xv[rr][j].w;
          }
      }
    }
    if (dx)
#pragma unroll
      for (int j = 0; j < HL_MAXJ; ++j) {
        const int ch = lane + 64 * j;
        if (ch >= nch) continue;
        float4 o[R];
#pragma unroll
        for (int rr = 0; rr < R; ++rr) o[rr] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const float4 w = Ws4[c * nch + ch];
#pragma unroll
          for (int rr = 0; rr < R; ++rr) {
            o[rr].x += dz[rr][c] * w.x;
            o[rr].y += dz[rr][c] * w.y;
            o[rr].z += dz[rr][c] * w.z;
            o[rr].w += dz[rr][c] * w.w;
          }
        }
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          if (row0 + rr >= M) continue;
          if (mask_dx) {
            o[rr].x = xv[rr][j].x <= 0.f ? 0.f : o[rr].x;
            o[rr].y = xv[rr][j].y <= 0.f ? 0.f : o[rr].y;
            o[rr].z = xv[rr][j].z <= 0.f ? 0.f : o[rr].z;
            o[rr].w = xv[rr][j].w <= 0.f ? 0.f : o[rr].w;
          }
          reinterpret_cast<float4*>(dx + (size_t)(row0 + rr) * K)[ch] = o[rr];
          vmax = fmaxf(fmaxf(vmax, fmaxf(fabsf(o[rr].x), fabsf(o[rr].y))), fmaxf(fabsf(o[rr].z), fabsf(o[rr].w)));
        }
      }
  }
  if (lane == 0) {
    red[2 * wave] = loss_acc;
    red[2 * wave + 1] = corr_acc;
  }
  if (dx_amax) {
    for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off));
    if (lane == 0) amx[wave] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) dx_amax[blockIdx.x] = fmaxf(fmaxf(amx[0], amx[1]), fmaxf(amx[2], amx[3]));
  }
  if constexpr (DW) {
    __shared__ float gbs[4][C];
    if (lane == 0)
#pragma unroll
      for (int c = 0; c < C; ++c) gbs[wave][c] = gbacc[c];
    // the W image is dead: reuse it for the dW partial, the waves adding in order 0, 1, 2, 3
    for (int wv = 0; wv < 4; ++wv) {
      __syncthreads();
      if (wave == wv)
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int j = 0; j < HL_MAXJ; ++j) {
            const int ch = lane + 64 * j;
            if (ch >= nch) continue;
            float4 v = gacc[c][j];
            if (wv > 0) {
              const float4 q = Ws4[c * nch + ch];
              v.x += q.x;
              v.y += q.y;
              v.z += q.z;
              v.w += q.w;
            }
            Ws4[c * nch + ch] = v;
          }
    }
    __syncthreads();
    const int width = C * K + C + 2;
    float* slab = part + (size_t)blockIdx.x * width;
    for (int i = threadIdx.x; i < C * nch; i += 256) reinterpret_cast<float4*>(slab)[i] = Ws4[i];
    if (threadIdx.x < C) slab[C * K + threadIdx.x] = gbs[0][threadIdx.x] + gbs[1][threadIdx.x] +
                                                     gbs[2][threadIdx.x] + gbs[3][threadIdx.x];
    if (threadIdx.x == 0) {
      slab[C * K + C] = red[0] + red[2] + red[4] + red[6];
      slab[C * K + C + 1] = red[1] + red[3] + red[5] + red[7];
    }
    return;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(stats, red[0] + red[2] + red[4] + red[6]);
    atomicAdd(stats + 1, red[1] + red[3] + red[5] + red[7]);
  }
}


// ==== MFMA head (K = 128, C <= 16) =============================================================
// The whole head as fp32 MFMAs (v_mfma_f32_16x16x4_f32: fp32 operands and accumulation, the
// same product precision as the VALU path), one wave per 16-row tile, no block-level barriers in
// the row loop. Lane l = (r = l % 16, g = l / 16):
//   logits^T = W x^T : A = W (lane: class r), B = x^T (lane: row r), k = 16u + 4g + e over 32 MFMAs;
//     D leaves lane (r, g) with row r's logits of classes 4g .. 4g+3 (bias as the initial value),
//     so softmax/NLL/argmax reduce 4 values in-lane plus two xor-shuffles (symmetric: every lane
//     of a row ends with bitwise the same max / sum)
//   dx^T = W^T dz^T : MFMA kk feeds each lane's own dz[row r][4g + kk] (the k index is the class,
//     permuted so no shuffle is needed); D = dx[row r][16 t + 4g .. +3], exactly the x elements
//     lane (r, g) loaded -> fused ReLU mask
//   dW^T += x^T dz : needs row-indexed K and hidden-/class-indexed lanes, so the tile and its dz
//     go through a wave-private LDS transpose (8 + 1 ds_write_b128, 36 ds_read_b32, swizzled so
//     both sides are bank-conflict-free); the dW^T accumulators stay in registers across the
//     wave's tiles.
// Both W fragment sets live in registers for the whole kernel (2 waves per SIMD); the next tile's
// x and targets are loaded while the current one is computed (ping-pong registers, no copies).
// Loads are unpredicated (rows clamped); a full tile stores without per-lane predicates, so its
// loop body is one basic block. Measured and rejected: 16-wave blocks at <= 128 VGPRs (W re-read
// from LDS per tile, 4 waves per SIMD) - spills, and its scratch reloads wait on every outstanding
// store (40.9 vs 38.2 us); 3 waves per SIMD (W re-read from LDS per tile, no register prefetch,
// 158 VGPRs, 512-1024 blocks) - 38.6 vs 36.5 us. Per block (4 waves) the dW, db, loss and correct partials meet in LDS
// in wave order and leave as one slab row (head_reduce_kernel sums the slabs in block order).
using headtile::f32x4m;
using headtile::mfma4;
using headtile::swz;
using headtile::xt_at;
constexpr int MW = 4;          // waves per block
constexpr int WSP = HK + 4;    // W pitch in LDS: the per-wave fragment reads hit distinct banks
constexpr int DTP = headtile::DTP;  // dz tile pitch

__device__ __forceinline__ void stage_w16(const float* __restrict__ W, int C, float* ws, int tid, int nthr) {
  for (int i = tid; i < 16 * HK / 4; i += nthr) {
    const int c = i / (HK / 4), k4 = i % (HK / 4);
    *reinterpret_cast<f32x4m*>(ws + c * WSP + 4 * k4) =
        c < C ? reinterpret_cast<const f32x4m*>(W)[i] : f32x4m{0.f, 0.f, 0.f, 0.f};
  }
}

// wd[t][kk] = W[class 4 g + kk][hidden 16 t + r] (zero for classes >= C)
__device__ __forceinline__ void load_wd(const float* ws, int r, int g, float (&wd)[8][4]) {
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) wd[t][kk] = ws[(4 * g + kk) * WSP + 16 * t + r];
}

// row clamped into [0, M): past-the-end rows of a partial tile read (and compute on) real data,
// their results are never stored or counted
__device__ __forceinline__ void load_x_tile(const float* __restrict__ x, int row, int g, f32x4m (&xv)[8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) xv[u] = *reinterpret_cast<const f32x4m*>(x + (size_t)row * HK + 16 * u + 4 * g);
}

// dx columns 16 t + 4 g .. +3 of row r: dx = sum_c dz[r][c] W[c][.], then the ReLU mask. The head
// and head_mfma_dx_from_dl_kernel both go through here, so their dx agree bit for bit.
__device__ __forceinline__ f32x4m dx_t(const float (&w4)[4], const float (&dz)[4], const f32x4m& xv, int mask) {
  f32x4m o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) o = mfma4(w4[kk], dz[kk], o);
  if (mask) {  // ReLU backward of the producing stage: x = relu(z) > 0 <=> z > 0
#pragma unroll
    for (int v = 0; v < 4; ++v) o[v] = xv[v] > 0.f ? o[v] : 0.f;
  }
  return o;
}

// dx from the factor dl with the MFMA head's exact operations (bit-identical to its dx)
template <int C>
__global__ void __launch_bounds__(256) head_mfma_dx_from_dl_kernel(const float* __restrict__ dl, const float* __restrict__ W,
                                                                   const float* __restrict__ x, float* __restrict__ dx,
                                                                   int M, int mask) {
  __shared__ __attribute__((aligned(16))) float ws[16 * WSP];
  stage_w16(W, C, ws, threadIdx.x, 256);
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  float wd[8][4];
  load_wd(ws, r, g, wd);
  const int tiles = (M + 15) / 16;
  for (int tile = blockIdx.x * 4 + (threadIdx.x >> 6); tile < tiles; tile += gridDim.x * 4) {
    const int row = tile * 16 + r;
    const bool valid = row < M;
    const int crow = min(row, M - 1);
    f32x4m xv[8];
    if (mask) load_x_tile(x, crow, g, xv);
    float dz[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) dz[v] = (valid && 4 * g + v < C) ? dl[(size_t)crow * C + 4 * g + v] : 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const f32x4m o = dx_t(wd[t], dz, xv[t], mask);
      if (valid) *reinterpret_cast<f32x4m*>(dx + (size_t)row * HK + 16 * t + 4 * g) = o;
    }
  }
}

// The standalone head for K = 128, C <= 16: head_block.h on 256-row blocks of x read from HBM, in the C layout the
// fused uint8 forward holds its accumulators in, so this kernel and the fused one run identical operations on the
// same rows (bit-identical logits, dl, loss). dx (DXP) from dl with dx_t, as head_mfma_dx_from_dl_kernel.
template <int C, bool DXP>
__global__ void __launch_bounds__(hblk::NT) head_block_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                               const float* __restrict__ bias,
                                                               const int64_t* __restrict__ target, int M, float scale,
                                                               float* __restrict__ part, float* __restrict__ dx,
                                                               int mask_dx, float* __restrict__ dl,
                                                               float* __restrict__ dxmax) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[hblk::LDS_BYTES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 3, wn = wave >> 2, h2 = lane >> 5, r32 = lane & 31;
  const int r = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * hblk::ROWS;
  auto prep = [&](hblk::hb_f32x16 (&y)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = m0 + 64 * wm + 32 * i + 8 * (q >> 2) + 4 * h2 + (q & 3);
          const float v = x[(size_t)min(row, M - 1) * HK + 64 * wn + 32 * j + r32];
          y[i][j][q] = row < M ? v : 0.f;
        }
  };
  float wd[8][4];  // wd[t][kk] = W[class 4 g + kk][hidden 16 t + r] (zero for classes >= C)
  if constexpr (DXP) {
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) wd[t][kk] = 4 * g + kk < C ? W[(size_t)(4 * g + kk) * HK + 16 * t + r] : 0.f;
  }
  hblk::Args a;
  a.w2 = W;
  a.b2 = bias;
  a.target = target;
  a.loss_scale = scale;
  a.train = dx != nullptr || dl != nullptr;
  a.dl = dl;
  a.part = part + (size_t)blockIdx.x * (C * HK + C + 2);
  a.bound = dxmax ? dxmax + blockIdx.x : nullptr;
  hblk::Operands ops;
  hblk::load_operands<C>(a, m0, M, wave, lane, ops);
  hblk::block_head<C>(
      prep, smem, a, ops, m0, M, wave, lane,
      [&](int, int row, bool valid, const float (&dz)[4]) {
        if constexpr (DXP) {
          if (dx) {
            f32x4m xv[8];
            load_x_tile(x, min(row, M - 1), g, xv);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const f32x4m o = dx_t(wd[t], dz, xv[t], mask_dx);
              if (valid) *reinterpret_cast<f32x4m*>(dx + (size_t)row * HK + 16 * t + 4 * g) = o;
            }
          }
        }
      },
      nullptr);
}

}  // namespace

bool head_fused_supported(int K, int C) { return K == HK && (C == 10 || C == 2 || C == 16); }

// the LDS-staged wide-K head (C = 10, K % 4 == 0, K <= 1024, large batches)
bool head_lds_supported(int M, int K, int C) { return C == 10 && K % 4 == 0 && K <= 64 * 4 * HL_MAXJ && M >= 4096; }
int head_lds_blocks(int M) { return (int)std::min<int64_t>(((int64_t)M + 7) / 8, 1024); }

// grid of the fused kernel: enough blocks to fill the chip, each keeping its dW partial in
// registers over several 64-row chunks (fewer slabs to reduce)
constexpr int SMALL_BATCH = 2048;  // <= this many rows: 16-row chunks (TPR = 16)
int head_rows_per_chunk(int M) { return M <= SMALL_BATCH ? HTHR / 16 : HTHR / 4; }

// the MFMA head (default) or the 4-lanes-per-row VALU head (SDML_HEAD=v1, A/B only)
static bool head_use_mfma() {
  return knob(KNOB_HEAD_VALU) == 0;
}

// MFMA head grid: 16-row tiles, ~2 waves per SIMD, each wave several tiles (its dW partial stays
// in registers across them)
static int head_mfma_blocks(int M, int* tiles_per_wave) {
  *tiles_per_wave = hblk::ROWS / 16;  // (head_block_kernel: one 256-row block per workgroup)
  return (M + hblk::ROWS - 1) / hblk::ROWS;
}

int head_fused_blocks(int M, int* chunks_per_block) {
  if (head_use_mfma()) return head_mfma_blocks(M, chunks_per_block);
  const int rows = head_rows_per_chunk(M);
  const int chunks = (M + rows - 1) / rows;
  const int max_blocks = std::max(1, knob(KNOB_HEAD_MAX_BLOCKS));  // A/B knob
  int blocks = chunks < max_blocks ? chunks : max_blocks;
  int cpb = (chunks + blocks - 1) / blocks;
  blocks = (chunks + cpb - 1) / cpb;
  *chunks_per_block = cpb;
  return blocks;
}

size_t head_workspace_floats(int M, int K, int C) {
  if (head_lds_supported(M, K, C)) return (size_t)head_lds_blocks(M) * (C * K + C + 2);
  if (!head_fused_supported(K, C)) return 0;
  int cpb;
  return (size_t)head_fused_blocks(M, &cpb) * (C * K + C + 2);
}

// dx[m][k] = (sum_c dl[m][c] W[c][k]) * (mask ? x[m][k] > 0 : 1): the fused head's dx, rebuilt from its
// factor with the SAME operations in the same order (f32x4 accumulation over c from zero), so the
// result is bit-identical to the dx the head would have written. K == HK (128).
template <int C>
__global__ void __launch_bounds__(256) head_dx_from_dl_kernel(const float* __restrict__ dl, const float* __restrict__ W,
                                                              const float* __restrict__ x, float* __restrict__ dx,
                                                              int M, int mask) {
  __shared__ __attribute__((aligned(16))) float ws[C * HK];
  for (int i = threadIdx.x; i < C * HK / 4; i += 256)
    reinterpret_cast<f32x4*>(ws)[i] = reinterpret_cast<const f32x4*>(W)[i];
  __syncthreads();
  const int q = threadIdx.x & 31;  // float4 column of the row
  for (int row = blockIdx.x * 8 + (threadIdx.x >> 5); row < M; row += gridDim.x * 8) {
    float dz[C];
#pragma unroll
    for (int c = 0; c < C; ++c) dz[c] = dl[(size_t)row * C + c];
    const int k = 4 * q;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < C; ++c) {
      f32x4 wv = *reinterpret_cast<const f32x4*>(ws + c * HK + k);
      o += dz[c] * wv;
    }
    if (mask) {
      f32x4 xv = *reinterpret_cast<const f32x4*>(x + (size_t)row * HK + k);
      o[0] = xv[0] > 0.f ? o[0] : 0.f;
      o[1] = xv[1] > 0.f ? o[1] : 0.f;
      o[2] = xv[2] > 0.f ? o[2] : 0.f;
      o[3] = xv[3] > 0.f ? o[3] : 0.f;
    }
    *reinterpret_cast<f32x4*>(dx + (size_t)row * HK + k) = o;
  }
}

void head_dx_from_dl(const float* dl, const float* W, const float* x, float* dx, int M, int K, int C, bool mask,
                     hipStream_t stream) {
  if (M <= 0) return;
  if (K != HK) abort();  // host contract (checked by the binding)
  if (head_use_mfma()) {
    const int blocks = std::min(2048, (M + 63) / 64);
#define DX_MFMA(CC) \
  hipLaunchKernelGGL((head_mfma_dx_from_dl_kernel<CC>), dim3(blocks), dim3(256), 0, stream, dl, W, x, dx, M, mask ? 1 : 0)
    switch (C) {
      case 10: DX_MFMA(10); break;
      case 2: DX_MFMA(2); break;
      case 16: DX_MFMA(16); break;
      default: abort();  // host contract: C in {2, 10, 16} (head_fused_supported)
    }
#undef DX_MFMA
    return;
  }
  int blocks = (M + 7) / 8;
  if (blocks > 2048) blocks = 2048;
  switch (C) {
    case 10: hipLaunchKernelGGL(head_dx_from_dl_kernel<10>, dim3(blocks), dim3(256), 0, stream, dl, W, x, dx, M, mask ? 1 : 0); break;
    case 2: hipLaunchKernelGGL(head_dx_from_dl_kernel<2>, dim3(blocks), dim3(256), 0, stream, dl, W, x, dx, M, mask ? 1 : 0); break;
    case 16: hipLaunchKernelGGL(head_dx_from_dl_kernel<16>, dim3(blocks), dim3(256), 0, stream, dl, W, x, dx, M, mask ? 1 : 0); break;
    default: abort();  // host contract: C in {2, 10, 16} (head_fused_supported)
  }
}

void head_reduce_run(const HeadReduceArgs& a, hipStream_t stream) {
  if (!a.part) return;
  hipLaunchKernelGGL(head_reduce_kernel, dim3(head_reduce_blocks(a)), dim3(1024), 0, stream, a);
}

void head_logsoftmax_nll(const float* x, const float* W, const float* b, const int64_t* target, int M, int K, int C,
                         float scale, float* stats, float* dx, float* gW, float* gb, float* dz_out,
                         float* workspace, bool mask_dx, hipStream_t stream, float* dl, bool stats_overwrite,
                         float* dx_amax, int* n_amax, HeadReduceArgs* defer) {
  if (n_amax) *n_amax = 0;
  if (defer) *defer = HeadReduceArgs();
  if (M <= 0) {
    if (stats_overwrite) (void)hipMemsetAsync(stats, 0, 2 * sizeof(float), stream);
    return;
  }
  const int rflags = ((dx != nullptr || dl != nullptr) ? 1 : 0) | (stats_overwrite ? 2 : 0);
  if (head_fused_supported(K, C) && dz_out == nullptr && workspace != nullptr && head_use_mfma()) {
    int tpw = 0;
    const int blocks = head_mfma_blocks(M, &tpw);
    float* amx = ((dx || dl) && dx_amax && n_amax && blocks <= kHeadAmaxMax) ? dx_amax : nullptr;
    if (amx) *n_amax = blocks;
#define HEAD_MFMA(CC)                                                                                          \
  do {                                                                                                     \
    if (dx)                                                                                                \
      hipLaunchKernelGGL((head_block_kernel<CC, true>), dim3(blocks), dim3(hblk::NT), 0, stream, x, W, b, target, M, \
                         scale, workspace, dx, mask_dx ? 1 : 0, dl, amx);                                   \
    else                                                                                                   \
      hipLaunchKernelGGL((head_block_kernel<CC, false>), dim3(blocks), dim3(hblk::NT), 0, stream, x, W, b, target, \
                         M, scale, workspace, dx, mask_dx ? 1 : 0, dl, amx);                                \
  } while (0)
    switch (C) {
      case 10: HEAD_MFMA(10); break;
      case 2: HEAD_MFMA(2); break;
      default: HEAD_MFMA(16); break;
    }
#undef HEAD_MFMA
    HeadReduceArgs ra;
    ra.part = workspace;
    ra.nblocks = blocks;
    ra.CK = C * K;
    ra.C = C;
    ra.gW = gW;
    ra.gb = gb;
    ra.stats = stats;
    ra.flags = rflags;
    if (defer) *defer = ra;  // the caller runs it (u8_wgrad_dl's reduction, or head_reduce_run)
    else head_reduce_run(ra, stream);
    return;
  }
  if (head_fused_supported(K, C) && dz_out == nullptr && workspace != nullptr) {
    int cpb = 0, blocks = head_fused_blocks(M, &cpb);
#define HEAD_LAUNCH(CC, TT)                                                                             \
  hipLaunchKernelGGL((head_fused_kernel<CC, TT>), dim3(blocks), dim3(HTHR), 0, stream, x, W, b, target, M, scale, \
                     workspace, dx, cpb, mask_dx ? 1 : 0, dl)
    const bool small = M <= SMALL_BATCH;
    switch (C) {
      case 10:
        if (small) HEAD_LAUNCH(10, 16); else HEAD_LAUNCH(10, 4);
        break;
      case 2:
        if (small) HEAD_LAUNCH(2, 16); else HEAD_LAUNCH(2, 4);
        break;
      default:
        if (small) HEAD_LAUNCH(16, 16); else HEAD_LAUNCH(16, 4);
        break;
    }
#undef HEAD_LAUNCH
    HeadReduceArgs ra;
    ra.part = workspace;
    ra.nblocks = blocks;
    ra.CK = C * K;
    ra.C = C;
    ra.gW = gW;
    ra.gb = gb;
    ra.stats = stats;
    ra.flags = rflags;
    head_reduce_run(ra, stream);
    return;
  }
  if (dl) abort();  // host contract: the dlogits output exists on the fused path only (head_fused_supported)
  if (head_lds_supported(M, K, C)) {
    const int lblocks = head_lds_blocks(M);
    const size_t lds = (size_t)C * K * sizeof(float);
    if (gW && gb && workspace && dz_out == nullptr) {
      float* am = (dx && dx_amax && n_amax && lblocks <= kHeadAmaxMax) ? dx_amax : nullptr;
      hipLaunchKernelGGL((head_lds_kernel<10, true>), dim3(lblocks), dim3(256), lds, stream, x, W, b, target, M, K,
                         scale, stats, dx, nullptr, mask_dx ? 1 : 0, workspace, am);
      if (am) *n_amax = lblocks;  // exact per-block max |dx|
      HeadReduceArgs ra;
      ra.part = workspace;
      ra.nblocks = lblocks;
      ra.CK = C * K;
      ra.C = C;
      ra.gW = gW;
      ra.gb = gb;
      ra.stats = stats;
      ra.flags = 1 | (stats_overwrite ? 2 : 0);
      head_reduce_run(ra, stream);
    } else {
      if (stats_overwrite) (void)hipMemsetAsync(stats, 0, 2 * sizeof(float), stream);  // this variant adds
      hipLaunchKernelGGL((head_lds_kernel<10, false>), dim3(lblocks), dim3(256), lds, stream, x, W, b, target, M, K,
                         scale, stats, dx, dz_out, mask_dx ? 1 : 0, nullptr, nullptr);
    }
    return;
  }
  if (stats_overwrite) (void)hipMemsetAsync(stats, 0, 2 * sizeof(float), stream);  // the generic kernel adds
  int gblocks = (M + 3) / 4;
  if (gblocks > 1024) gblocks = 1024;
  hipLaunchKernelGGL(head_generic_kernel, dim3(gblocks), dim3(256), 0, stream, x, W, b, target, M, K, C, scale, stats,
                     dx, dz_out, mask_dx ? 1 : 0);
}

}  // namespace sdml
