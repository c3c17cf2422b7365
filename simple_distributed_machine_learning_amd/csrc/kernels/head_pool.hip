// Pooled classifier head for the ResNet-18 stages' last layer (BASELINE config 4): global average pool ->
// Linear(K -> C) -> log_softmax -> NLL (sum) and the whole backward, in one launch plus one fixed-order
// reduction launch. Replaces adaptive_avg_pool2d + a hipBLASLt GEMM + ATen log_softmax / nll_loss forward
// and backward + the dW / db GEMMs (the reference's loss, /root/reference/simple_distributed.py:111, on the
// ResNet's logits).
//
// x [M][P][K] channels-last (P = H * W positions, K channels), bf16 or fp32; W [C][K], b [C] of the same
// type (the stage's parameters). Per row m (one wave): feats = mean_p x (fp32), z = feats W^T + b (fp32),
// loss = logsumexp(z) - z[y], correct = (first argmax == y), dl = scale (softmax(z) - onehot(y)),
// dfeat = dl W, dx[m][p][k] = dfeat[k] / P (the pool's backward; written in x's type). A workgroup holds
// RB = 4 rows (4 waves) and writes its dW / db / (loss, correct) partial sums over its rows, in row order,
// to a workspace slab; head_pool_reduce adds the slabs in block order into gW / gb (accumulated, in the
// parameters' type) and stats (added, or overwritten) - deterministic. Rows with a label outside [0, C)
// get no loss term and no gradient (as head_xent.hip's heads).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace sdml {
namespace {

constexpr int HP_RB = 4;       // rows (waves) per workgroup
constexpr int HP_MAXKL = 16;   // K / 64 per lane (K <= 1024)
constexpr int HP_MAXC = 16;

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const __bf16* p) { return static_cast<float>(*p); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void stf(__bf16* p, float v) { *p = static_cast<__bf16>(v); }

template <typename T>
__global__ void __launch_bounds__(256) head_pool_kernel(const T* __restrict__ x, const T* __restrict__ W,
                                                        const T* __restrict__ b, const int64_t* __restrict__ tgt,
                                                        int M, int P, int K, int C, float scale, T* __restrict__ dx,
                                                        float* __restrict__ part) {
  extern __shared__ float sm[];
  float* Ws = sm;                         // [C][K]
  float* fS = Ws + C * K;                 // [RB][K] pooled features
  float* dS = fS + HP_RB * K;             // [RB][C] dl (0 for rows past M / bad labels)
  float* lS = dS + HP_RB * HP_MAXC;       // [RB][2] loss, correct
  const int t = threadIdx.x, lane = t & 63, r = t >> 6;
  for (int i = t; i < C * K; i += 256) Ws[i] = ldf(W + i);
  __syncthreads();
  const int m = blockIdx.x * HP_RB + r;
  const int KL = K / 64;
  float dl[HP_MAXC];
#pragma unroll
  for (int c = 0; c < HP_MAXC; ++c) dl[c] = 0.f;
  float loss = 0.f, corr = 0.f;
  if (m < M) {
    const float inv = 1.f / (float)P;
    float f[HP_MAXKL];
#pragma unroll
    for (int j = 0; j < HP_MAXKL; ++j) {
      f[j] = 0.f;
      if (j < KL) {
        const T* xp = x + (size_t)m * P * K + lane + 64 * j;
        float s = 0.f;
        for (int p = 0; p < P; ++p) s += ldf(xp + (size_t)p * K);
        f[j] = s * inv;
        fS[r * K + lane + 64 * j] = f[j];
      }
    }
    float z[HP_MAXC];
#pragma unroll
    for (int c = 0; c < HP_MAXC; ++c) {
      float a = 0.f;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < HP_MAXKL; ++j)
          if (j < KL) a += f[j] * Ws[c * K + lane + 64 * j];
        for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
        a += ldf(b + c);
      }
      z[c] = a;
    }
    const int y = (int)tgt[m];
    float mx = -INFINITY;
    int am = 0;
#pragma unroll
    for (int c = 0; c < HP_MAXC; ++c)
      if (c < C && z[c] > mx) {
        mx = z[c];
        am = c;
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < HP_MAXC; ++c)
      if (c < C) se += __expf(z[c] - mx);
    const float lse = mx + __logf(se);
    if (y >= 0 && y < C) {
      float zy = 0.f;
#pragma unroll
      for (int c = 0; c < HP_MAXC; ++c)
        if (c == y) zy = z[c];
      loss = lse - zy;
      corr = am == y ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < HP_MAXC; ++c)
        if (c < C) dl[c] = scale * (__expf(z[c] - lse) - (c == y ? 1.f : 0.f));
    }
    // dfeat = dl W -> dx (the pool's backward spreads it evenly over the P positions)
#pragma unroll
    for (int j = 0; j < HP_MAXKL; ++j) {
      if (j < KL) {
        const int k = lane + 64 * j;
        float g = 0.f;
#pragma unroll
        for (int c = 0; c < HP_MAXC; ++c)
          if (c < C) g += dl[c] * Ws[c * K + k];
        g *= inv;
        T* dp = dx + (size_t)m * P * K + k;
        for (int p = 0; p < P; ++p) stf(dp + (size_t)p * K, g);
      }
    }
  } else {
    for (int k = lane; k < K; k += 64) fS[r * K + k] = 0.f;
  }
  if (lane < HP_MAXC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < HP_MAXC; ++c)
      if (c == lane) v = dl[c];
    dS[r * HP_MAXC + lane] = v;
  }
  if (lane == 0) {
    lS[2 * r] = loss;
    lS[2 * r + 1] = corr;
  }
  __syncthreads();
  // block partials over its rows, rows in order: dW [C][K], db [C], loss, correct
  const int CK = C * K;
  float* out = part + (size_t)blockIdx.x * (CK + C + 2);
  for (int i = t; i < CK + C + 2; i += 256) {
    float s = 0.f;
    if (i < CK) {
      const int c = i / K, k = i % K;
#pragma unroll
      for (int q = 0; q < HP_RB; ++q) s += dS[q * HP_MAXC + c] * fS[q * K + k];
    } else if (i < CK + C) {
#pragma unroll
      for (int q = 0; q < HP_RB; ++q) s += dS[q * HP_MAXC + (i - CK)];
    } else {
#pragma unroll
      for (int q = 0; q < HP_RB; ++q) s += lS[2 * q + (i - CK - C)];
    }
    out[i] = s;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) head_pool_reduce_kernel(const float* __restrict__ part, int nblocks, int CK, int C,
                                                               T* __restrict__ gW, T* __restrict__ gb,
                                                               float* __restrict__ stats, int overwrite) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = CK + C + 2;
  if (i >= n) return;
  float s = 0.f;
  for (int q = 0; q < nblocks; ++q) s += part[(size_t)q * n + i];
  if (i < CK) {
    stf(gW + i, ldf(gW + i) + s);
  } else if (i < CK + C) {
    stf(gb + (i - CK), ldf(gb + (i - CK)) + s);
  } else if (stats) {
    const int k = i - CK - C;
    stats[k] = overwrite ? s : stats[k] + s;
  }
}

template <typename T>
void launch(const T* x, const T* W, const T* b, const int64_t* tgt, int M, int P, int K, int C, float scale, T* dx,
            T* gW, T* gb, float* stats, bool overwrite, float* ws, hipStream_t stream) {
  const int nb = (M + HP_RB - 1) / HP_RB;
  const size_t lds = (size_t)(C * K + HP_RB * K + HP_RB * HP_MAXC + 2 * HP_RB) * sizeof(float);
  hipLaunchKernelGGL((head_pool_kernel<T>), dim3(nb), dim3(256), lds, stream, x, W, b, tgt, M, P, K, C, scale, dx, ws);
  const int n = C * K + C + 2;
  hipLaunchKernelGGL((head_pool_reduce_kernel<T>), dim3((n + 255) / 256), dim3(256), 0, stream, ws, nb, C * K, C, gW, gb,
                     stats, overwrite ? 1 : 0);
}

}  // namespace

bool head_pool_supported(int M, int P, int K, int C) {
  // LDS: W + RB feature rows (<= 160 KiB); K a multiple of 64 up to 1024 (16 per lane)
  return M >= 1 && P >= 1 && C >= 1 && C <= HP_MAXC && K % 64 == 0 && K <= 64 * HP_MAXKL &&
         (size_t)(C * K + HP_RB * K + HP_RB * HP_MAXC + 2 * HP_RB) * 4 <= 160 * 1024;
}

int64_t head_pool_workspace_floats(int M, int K, int C) {
  return (int64_t)((M + HP_RB - 1) / HP_RB) * (C * K + C + 2);
}

void head_pool_xent(const void* x, const void* W, const void* b, const int64_t* tgt, int M, int P, int K, int C,
                    float scale, void* dx, void* gW, void* gb, float* stats, bool stats_overwrite, float* ws, bool bf16,
                    hipStream_t stream) {
  if (M <= 0) return;
  if (bf16)
    launch<__bf16>(static_cast<const __bf16*>(x), static_cast<const __bf16*>(W), static_cast<const __bf16*>(b), tgt, M,
                   P, K, C, scale, static_cast<__bf16*>(dx), static_cast<__bf16*>(gW), static_cast<__bf16*>(gb), stats,
                   stats_overwrite, ws, stream);
  else
    launch<float>(static_cast<const float*>(x), static_cast<const float*>(W), static_cast<const float*>(b), tgt, M, P,
                  K, C, scale, static_cast<float*>(dx), static_cast<float*>(gW), static_cast<float*>(gb), stats,
                  stats_overwrite, ws, stream);
}

}  // namespace sdml
