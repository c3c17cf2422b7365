// GPT-2 stage kernels outside the GEMMs/attention/LayerNorm (BASELINE config 5, bf16):
//
// * tanh-GELU forward and backward (the MLP activation, models/gpt2.py MLP; gelu.h): fp32 math on bf16 I/O,
//   PyTorch's approximate="tanh" functions in sigmoid form (one __expf), 8 elements (16 B) per lane.
// * token + position embedding: out[b][s] = wte[tok[b][s]] + wpe[s], one wave per token row.
// * embedding backward, deterministic: wpe.grad[s] += sum_b g[b][s] in batch order; wte.grad[v] +=
//   sum of g over the positions holding token v, in position order - the tokens arrive stably sorted
//   (key = token, value = position) and one wave per sorted segment sums its rows; no float atomics,
//   so repeated runs produce the same bits. Gradients are added in fp32 and rounded into the bf16
//   parameter gradients in place (the flat gradient buffer, utils/flat.py).
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include "gelu.h"
#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // RNE, NaN-preserving
  return *reinterpret_cast<u16*>(&h);
}

__global__ void __launch_bounds__(256) gelu_fwd_kernel(const u16x8* __restrict__ x, u16x8* __restrict__ y,
                                                       int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const u16x8 v = x[i];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(gelu_f(bf2f(v[e])));
    y[i] = o;
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const u16x8* __restrict__ gy, const u16x8* __restrict__ x,
                                                       u16x8* __restrict__ gx, int64_t n8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const u16x8 g = gy[i], v = x[i];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(gelu_grad_f(bf2f(g[e]), bf2f(v[e])));
    gx[i] = o;
  }
}

// one wave per token row: 4 bf16 (8 B) per lane per step
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ tok, const u16* __restrict__ wte,
                                                        const u16* __restrict__ wpe, u16* __restrict__ out, int rows,
                                                        int S, int C, int V) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  int64_t t = tok[row];
  t = t < 0 ? 0 : (t >= V ? V - 1 : t);  // (host validates the range in debug mode)
  const u16x4* a = reinterpret_cast<const u16x4*>(wte + t * C);
  const u16x4* p = reinterpret_cast<const u16x4*>(wpe + (int64_t)(row % S) * C);
  u16x4* o = reinterpret_cast<u16x4*>(out + (int64_t)row * C);
  for (int c = lane; c < C / 4; c += 64) {
    const u16x4 va = a[c], vp = p[c];
    u16x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = f2bf(bf2f(va[e]) + bf2f(vp[e]));
    o[c] = r;
  }
}

// wpe.grad[s] += sum_b g[b][s] (batch order); one wave per position
__global__ void __launch_bounds__(256) wpe_bwd_kernel(const u16* __restrict__ g, u16* __restrict__ gw, int B, int S,
                                                      int C) {
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (s >= S) return;
  for (int c = lane; c < C / 4; c += 64) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
      const u16x4 v = reinterpret_cast<const u16x4*>(g + ((int64_t)b * S + s) * C)[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += bf2f(v[e]);
    }
    u16x4* dst = reinterpret_cast<u16x4*>(gw + (int64_t)s * C) + c;
    const u16x4 old = *dst;
    u16x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = f2bf(bf2f(old[e]) + acc[e]);
    *dst = r;
  }
}

// wte.grad[key] += sum of g[perm[j]] over the sorted segment of `key`, in position order; one wave per
// sorted index, the waves that do not start a segment exit at once
__global__ void __launch_bounds__(256) wte_bwd_kernel(const u16* __restrict__ g, const int64_t* __restrict__ keys,
                                                      const int64_t* __restrict__ perm, u16* __restrict__ gw, int n,
                                                      int C, int V) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t key = keys[i];
  if ((i > 0 && keys[i - 1] == key) || key < 0 || key >= V) return;
  int end = i + 1;
  while (end < n && keys[end] == key) ++end;
  for (int c = lane; c < C / 4; c += 64) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = i; j < end; ++j) {
      const u16x4 v = reinterpret_cast<const u16x4*>(g + perm[j] * C)[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += bf2f(v[e]);
    }
    u16x4* dst = reinterpret_cast<u16x4*>(gw + key * C) + c;
    const u16x4 old = *dst;
    u16x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = f2bf(bf2f(old[e]) + acc[e]);
    *dst = r;
  }
}

int grid_for(int64_t n8) {
  const int64_t b = (n8 + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

// ---- batched 2-D transpose (the hand NT GEMM's W^T operands, once per optimizer step) ----------------------
// dst[c][r] = src[r][c] for up to kTransposeBatchMax bf16 matrices in ONE launch: a ResNet-like per-weight loop of 48
// small copies per GPT-2 step was 48 launches of ~5 us. 64 x 64 tiles through LDS (pitch 66 u16: the column reads
// of the write phase spread over the banks), 16-B loads and stores (R, C multiples of 8).
struct TrBatch {
  const u16* src[kTransposeBatchMax];
  u16* dst[kTransposeBatchMax];
  int R[kTransposeBatchMax], C[kTransposeBatchMax], block0[kTransposeBatchMax + 1];
  int n;
};

__global__ void __launch_bounds__(256) transpose_batched_kernel(TrBatch b) {
  __shared__ u16 tile[64][66];
  const int blk = blockIdx.x;
  int e = 0;
  while (e + 1 < b.n && b.block0[e + 1] <= blk) ++e;
  const int R = b.R[e], C = b.C[e];
  const int tcn = (C + 63) / 64;
  const int t = blk - b.block0[e], r0 = (t / tcn) * 64, c0 = (t % tcn) * 64;
  const u16* src = b.src[e];
  u16* dst = b.dst[e];
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // 64 rows x 8 chunks of 8
    const int idx = threadIdx.x + 256 * u, rr = idx >> 3, ch = idx & 7;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + rr < R && c0 + 8 * ch < C) v = *reinterpret_cast<const u16x8*>(src + (size_t)(r0 + rr) * C + c0 + 8 * ch);
#pragma unroll
    for (int k = 0; k < 8; ++k) tile[rr][8 * ch + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // dst rows c0 + cc, 8 chunks of 8 source rows each
    const int idx = threadIdx.x + 256 * u, cc = idx >> 3, ch = idx & 7;
    if (c0 + cc >= C || r0 + 8 * ch >= R) continue;
    u16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tile[8 * ch + k][cc];
    *reinterpret_cast<u16x8*>(dst + (size_t)(c0 + cc) * R + r0 + 8 * ch) = v;
  }
}

}  // namespace

void gelu_fwd_bf16(const void* x, void* y, int64_t n, hipStream_t stream) {
  if (n % 8) abort();  // host contract
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream,
                     reinterpret_cast<const u16x8*>(x), reinterpret_cast<u16x8*>(y), n / 8);
}

void gelu_bwd_bf16(const void* gy, const void* x, void* gx, int64_t n, hipStream_t stream) {
  if (n % 8) abort();  // host contract
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(grid_for(n / 8)), dim3(256), 0, stream,
                     reinterpret_cast<const u16x8*>(gy), reinterpret_cast<const u16x8*>(x),
                     reinterpret_cast<u16x8*>(gx), n / 8);
}

void embedding_fwd_bf16(const int64_t* tok, const void* wte, const void* wpe, void* out, int rows, int S, int C, int V,
                        hipStream_t stream) {
  if (C % 4 || rows <= 0) return;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, tok,
                     reinterpret_cast<const u16*>(wte), reinterpret_cast<const u16*>(wpe), reinterpret_cast<u16*>(out),
                     rows, S, C, V);
}

void embedding_bwd_bf16(const void* g, const int64_t* sorted_tok, const int64_t* perm, void* gwte, void* gwpe, int B,
                        int S, int C, int V, hipStream_t stream) {
  const int n = B * S;
  if (C % 4 || n <= 0) return;
  if (gwpe)
    hipLaunchKernelGGL(wpe_bwd_kernel, dim3((S + 3) / 4), dim3(256), 0, stream, reinterpret_cast<const u16*>(g),
                       reinterpret_cast<u16*>(gwpe), B, S, C);
  if (gwte)
    hipLaunchKernelGGL(wte_bwd_kernel, dim3((n + 3) / 4), dim3(256), 0, stream, reinterpret_cast<const u16*>(g),
                       sorted_tok, perm, reinterpret_cast<u16*>(gwte), n, C, V);
}

void transpose_batched_bf16(const void* const* src, void* const* dst, const int* R, const int* C, int n,
                            hipStream_t stream) {
  if (n <= 0) return;
  TrBatch b{};
  int blocks = 0;
  for (int k = 0; k < n; ++k) {
    b.src[k] = static_cast<const u16*>(src[k]);
    b.dst[k] = static_cast<u16*>(dst[k]);
    b.R[k] = R[k];
    b.C[k] = C[k];
    b.block0[k] = blocks;
    blocks += ((R[k] + 63) / 64) * ((C[k] + 63) / 64);
  }
  b.block0[n] = blocks;
  b.n = n;
  hipLaunchKernelGGL(transpose_batched_kernel, dim3(blocks), dim3(256), 0, stream, b);
}

}  // namespace sdml
