// Pooled classifier head for the ResNet-18 stages' last layer (BASELINE config 4): global average pool ->
// Linear(K -> C) -> log_softmax -> NLL (sum) and the whole backward, in one launch plus one fixed-order
// reduction launch. Replaces adaptive_avg_pool2d + a hipBLASLt GEMM + ATen log_softmax / nll_loss forward
// and backward + the dW / db GEMMs (the reference's loss, /root/reference/simple_distributed.py:111, on the
// ResNet's logits).
//
// x [M][P][K] channels-last (P = H * W positions, K channels), bf16 or fp32; W [C][K], b [C] of the same
// type (the stage's parameters). Per row m (one wave; lane l owns channels 8 l .. 8 l + 7 (+ 512 ...), so
// every load and store moves 16 B (bf16) per lane): feats = mean_p x (fp32), z = feats W^T + b (fp32),
// loss = logsumexp(z) - z[y], correct = (first argmax == y), dl = scale (softmax(z) - onehot(y)),
// dfeat = dl W, dx[m][p][k] = dfeat[k] / P (the pool's backward; written in x's type). A workgroup (4 waves)
// runs HP_ROWS = 4 rows, 1 per wave, and writes its dW / db / (loss, correct) sums over those rows, in row
// order, to a workspace slab; head_pool_reduce adds the slabs (4 strided groups per entry, combined in a fixed
// order) into gW / gb (accumulated, in the parameters' type) and stats (added, or overwritten) -
// deterministic. Rows with a label outside [0, C) get no loss term and no gradient (as head_xent.hip's heads).
//
// Round 4 first version: one row per wave with scalar loads and a serial slab reduction ran 56 + 32 us at
// ResNet's 512 x 16 x 512 (profiles/r4_resnet18_bf16_kernel_stats.txt), slower than the ATen head. The second
// (16 rows per workgroup, 4 per wave, one position load in flight per lane) still took 58 us: 32 workgroups, each
// wave waiting out 64 dependent HBM round trips. Now: one row per wave (128 workgroups at M = 512) and the
// positions' loads issued HP_PU at a time.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace sdml {
namespace {

constexpr int HP_WAVES = 4;
constexpr int HP_RPW = 1;                     // rows per wave
constexpr int HP_PU = 8;                      // positions loaded per batch (independent loads in flight)
constexpr int HP_ROWS = HP_WAVES * HP_RPW;    // rows per workgroup
constexpr int HP_MAXCH = 2;                   // 8-channel chunks per lane: K <= 1024
constexpr int HP_MAXC = 16;
constexpr int HP_RG = 4;                      // reduction: partial groups per entry

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, static_cast<__bf16>(f)); }

// 8 consecutive elements <-> floats
__device__ __forceinline__ void ld8(const __bf16* p, float (&v)[8]) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
}
__device__ __forceinline__ void st8(__bf16* p, const float (&v)[8]) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  *reinterpret_cast<u16x8*>(p) = u;
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  reinterpret_cast<f32x4*>(p)[0] = f32x4{v[0], v[1], v[2], v[3]};
  reinterpret_cast<f32x4*>(p)[1] = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const __bf16* p) { return static_cast<float>(*p); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void stf(__bf16* p, float v) { *p = static_cast<__bf16>(v); }

template <typename T>
__global__ void __launch_bounds__(64 * HP_WAVES) head_pool_kernel(const T* __restrict__ x, const T* __restrict__ W,
                                                                 const T* __restrict__ b,
                                                                 const int64_t* __restrict__ tgt, int M, int P, int K,
                                                                 int C, float scale, T* __restrict__ dx,
                                                                 float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ws = sm;                         // [C][K]
  float* fS = Ws + C * K;                 // [HP_ROWS][K] pooled features
  float* dS = fS + HP_ROWS * K;           // [HP_ROWS][HP_MAXC] dl (0 for rows past M / bad labels)
  float* lS = dS + HP_ROWS * HP_MAXC;     // [HP_ROWS][2] loss, correct
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int i = 8 * t; i < C * K; i += 8 * 64 * HP_WAVES) {
    float v[8];
    ld8(W + i, v);
    st8(Ws + i, v);
  }
  __syncthreads();
  const int nch = K / 512 + (K % 512 ? 1 : 0);  // this lane's chunks: 8 lane + 512 q, q < nch (when < K)
  const float inv = 1.f / (float)P;
  for (int rr = 0; rr < HP_RPW; ++rr) {
    const int r = w * HP_RPW + rr, m = blockIdx.x * HP_ROWS + r;
    float dl[HP_MAXC];
#pragma unroll
    for (int c = 0; c < HP_MAXC; ++c) dl[c] = 0.f;
    float loss = 0.f, corr = 0.f;
    if (m < M) {  // (wave-uniform)
      float f[HP_MAXCH][8];
#pragma unroll
      for (int q = 0; q < HP_MAXCH; ++q) {
        const int k0 = 8 * lane + 512 * q;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[q][e] = 0.f;
        if (q < nch && k0 < K) {
          const T* xp = x + (size_t)m * P * K + k0;
          int p = 0;
          for (; p + HP_PU <= P; p += HP_PU) {  // HP_PU loads in flight, added in position order
            float v[HP_PU][8];
#pragma unroll
            for (int u = 0; u < HP_PU; ++u) ld8(xp + (size_t)(p + u) * K, v[u]);
#pragma unroll
            for (int u = 0; u < HP_PU; ++u)
#pragma unroll
              for (int e = 0; e < 8; ++e) f[q][e] += v[u][e];
          }
          for (; p < P; ++p) {
            float v[8];
            ld8(xp + (size_t)p * K, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[q][e] += v[e];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) f[q][e] *= inv;
          st8(fS + r * K + k0, f[q]);
        }
      }
      float z[HP_MAXC];
#pragma unroll
      for (int c = 0; c < HP_MAXC; ++c) {
        float a = 0.f;
        if (c < C) {
#pragma unroll
          for (int q = 0; q < HP_MAXCH; ++q) {
            const int k0 = 8 * lane + 512 * q;
            if (q < nch && k0 < K) {
              float wv[8];
              ld8(Ws + c * K + k0, wv);
#pragma unroll
              for (int e = 0; e < 8; ++e) a += f[q][e] * wv[e];
            }
          }
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
      for (int q = 0; q < HP_MAXCH; ++q) {
        const int k0 = 8 * lane + 512 * q;
        if (q < nch && k0 < K) {
          float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < HP_MAXC; ++c)
            if (c < C) {
              float wv[8];
              ld8(Ws + c * K + k0, wv);
#pragma unroll
              for (int e = 0; e < 8; ++e) g[e] += dl[c] * wv[e];
            }
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] *= inv;
          T* dp = dx + (size_t)m * P * K + k0;
          for (int p = 0; p < P; ++p) st8(dp + (size_t)p * K, g);
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
  }
  __syncthreads();
  // block partials over its rows, rows in order: dW [C][K], db [C], loss, correct
  const int CK = C * K;
  float* out = part + (size_t)blockIdx.x * (CK + C + 2);
  for (int i = t; i < CK + C + 2; i += 64 * HP_WAVES) {
    float s = 0.f;
    if (i < CK) {
      const int c = i / K, k = i % K;
#pragma unroll
      for (int q = 0; q < HP_ROWS; ++q) s += dS[q * HP_MAXC + c] * fS[q * K + k];
    } else if (i < CK + C) {
#pragma unroll
      for (int q = 0; q < HP_ROWS; ++q) s += dS[q * HP_MAXC + (i - CK)];
    } else {
#pragma unroll
      for (int q = 0; q < HP_ROWS; ++q) s += lS[2 * q + (i - CK - C)];
    }
    out[i] = s;
  }
}

// entry i of the slab: HP_RG strided groups of the nblocks partials (loads independent, 8 in flight), then the
// groups added in order
template <typename T>
__global__ void __launch_bounds__(64 * HP_RG) head_pool_reduce_kernel(const float* __restrict__ part, int nblocks,
                                                                     int CK, int C, T* __restrict__ gW,
                                                                     T* __restrict__ gb, float* __restrict__ stats,
                                                                     int overwrite) {
  __shared__ float red[HP_RG][64];
  const int l = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + l;
  const int n = CK + C + 2;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < n) {
    // loads unconditional (clamped block index, the extra terms dropped by a select): with `if (q < nblocks)`
    // around each load hipcc waited out every load on its own (11 serial round trips, 11.8 us)
    for (int q0 = grp; q0 < nblocks; q0 += 8 * HP_RG) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)min(q0 + HP_RG * u, nblocks - 1) * n + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = q0 + HP_RG * u < nblocks ? acc[u] + v[u] : acc[u];
    }
  }
  red[grp][l] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (grp != 0 || i >= n) return;
  float s = red[0][l];
#pragma unroll
  for (int g = 1; g < HP_RG; ++g) s += red[g][l];
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
  const int nb = (M + HP_ROWS - 1) / HP_ROWS;
  const size_t lds = (size_t)(C * K + HP_ROWS * K + HP_ROWS * HP_MAXC + 2 * HP_ROWS) * sizeof(float);
  hipLaunchKernelGGL((head_pool_kernel<T>), dim3(nb), dim3(64 * HP_WAVES), lds, stream, x, W, b, tgt, M, P, K, C, scale,
                     dx, ws);
  const int n = C * K + C + 2;
  hipLaunchKernelGGL((head_pool_reduce_kernel<T>), dim3((n + 63) / 64), dim3(64 * HP_RG), 0, stream, ws, nb, C * K, C,
                     gW, gb, stats, overwrite ? 1 : 0);
}

}  // namespace

bool head_pool_supported(int M, int P, int K, int C) {
  // K a multiple of 8 up to 1024 (two 8-channel chunks per lane); W + HP_ROWS feature rows in LDS
  return M >= 1 && P >= 1 && C >= 1 && C <= HP_MAXC && K % 8 == 0 && K <= 512 * HP_MAXCH &&
         (size_t)(C * K + HP_ROWS * K + HP_ROWS * HP_MAXC + 2 * HP_ROWS) * 4 <= 64 * 1024;
}

int64_t head_pool_workspace_floats(int M, int K, int C) {
  return (int64_t)((M + HP_ROWS - 1) / HP_ROWS) * (C * K + C + 2);
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
