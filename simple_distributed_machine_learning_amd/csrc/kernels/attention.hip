// Causal flash attention (forward + backward) for the GPT-2 stages, bf16 in/out, fp32 math,
// head_dim 64, on v_mfma_f32_32x32x16_bf16. Replaces torch SDPA (which dispatches to
// AOTriton-generated kernels on ROCm): everything here is plain HIP for gfx950.
//
// Layout conventions (gfx950 MFMA 32x32x16 bf16, wave64):
//   A operand: lane (r = l&31, h = l>>5) holds A[row r][k = 8h + j], j = 0..7
//   B operand: lane (r, h) holds B[k = 8h + j][col r]
//   C/D      : lane holds column (l&31); register i holds row (i&3) + 8(i>>2) + 4h
//   An accumulator X (rows in registers, column on the lane) is reused as the B operand of the
//   next product by packing registers 8s..8s+7 to bf16: element j of lane half h then stands
//   for X row 16s + 8(j>>2) + 4h + (j&3) (cdna_hip_programming.md §3), so the A operand must
//   be read in that same k order.
//
// Forward (one workgroup = 4 waves = 128 queries of one (batch, head); wave = 32 queries):
//   S^T = K Q^T  (A = K rows from LDS, B = this wave's Q rows, kept in registers)
//     -> each lane owns ONE query column: the online-softmax max/sum are in-lane + one
//        xor-32 shuffle; no cross-lane reductions over the key axis.
//   O^T += V^T P^T (A = V^T from a transposed V image in LDS, B = P straight from registers)
//     -> O^T has the query on the lane too, so the rescale by exp(m_old - m_new) is a per-lane
//        scalar multiply. LSE (log2 domain) is saved for the backward pass.
// Backward: dK/dV kernel (workgroup = 128 keys; loops over query blocks) and dQ kernel
// (workgroup = 128 queries; loops over key blocks) — no atomics, P recomputed from LSE.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA operand (8 x bf16)
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));

constexpr int HD = 64;             // head dim
constexpr int QW = 32;             // queries per wave
constexpr int NW = 4;              // waves per workgroup
constexpr int QB = QW * NW;        // queries per workgroup
constexpr int KB = 64;             // keys per iteration
constexpr int KP = HD + 8;         // LDS pitch (bf16) of row-major [key][d] tiles: 144 B rows
constexpr int TP = KB + 8;         // LDS pitch (bf16) of transposed [d][key] tiles
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<u16*>(&h);
}
__device__ __forceinline__ short f2bfs(float f) { return (short)f2bf(f); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// pack accumulator registers 8s..8s+7 to a bf16 B/A fragment
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bfs(x[8 * s + j]);
  return r;
}

// fragment in the accumulator k-order from a transposed image T[row][key]:
// element j = T[row][k0 + 8(j>>2) + 4h + (j&3)]  (two 8-byte reads)
__device__ __forceinline__ bf16x8 tr_frag(const u16* T, int pitch, int row, int k0, int h) {
  const u16* p = T + row * pitch + k0 + 4 * h;
  bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
  bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 8);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// natural-order fragment of row `row` of a row-major [row][d] image: element j = X[row][k0 + 8h + j]
__device__ __forceinline__ bf16x8 row_frag(const u16* X, int pitch, int row, int k0, int h) {
  return *reinterpret_cast<const bf16x8*>(X + row * pitch + k0 + 8 * h);
}

struct AttnArgs {
  const u16 *q, *k, *v, *o, *dout;
  u16 *out, *dq, *dk, *dv;
  float *lse, *delta;
  int B, H, S;
  long sqb, sqh, sqs;  // strides (elements) of q/k/v and of dq/dk/dv: batch, head, seq
  long sob, soh, sos;  // strides of o / dout
  float scale;         // softmax scale (1/sqrt(d))
  int causal;
};

// cooperative copy of `rows` rows x 64 d (bf16) starting at global row r0 into a row-major
// LDS image [row][KP]; rows beyond S are zero-filled. 256 threads, 16 B each.
__device__ __forceinline__ void stage_rows(u16* L, const u16* G, long srow, int r0, int rows, int S) {
  for (int c = threadIdx.x; c < rows * 8; c += 256) {
    int r = c >> 3, ch = c & 7;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < S) v = *reinterpret_cast<const u16x8*>(G + (long)(r0 + r) * srow + 8 * ch);
    *reinterpret_cast<u16x8*>(L + r * KP + 8 * ch) = v;
  }
}

// same rows stored transposed: T[d][row] with pitch TP
__device__ __forceinline__ void stage_rows_tr(u16* T, const u16* G, long srow, int r0, int rows, int S) {
  for (int c = threadIdx.x; c < rows * 8; c += 256) {
    int r = c >> 3, ch = c & 7;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < S) v = *reinterpret_cast<const u16x8*>(G + (long)(r0 + r) * srow + 8 * ch);
#pragma unroll
    for (int e = 0; e < 8; ++e) T[(8 * ch + e) * TP + r] = v[e];
  }
}

// ============================================================================================
// forward
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) u16 Ks[KB * KP];
  __shared__ __attribute__((aligned(16))) u16 Vt[HD * TP];
  const int nqb = (a.S + QB - 1) / QB;
  const int bh = blockIdx.x / nqb;
  const int qb = nqb - 1 - (blockIdx.x % nqb);  // heaviest (causal) blocks first
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long qoff = (long)b * a.sqb + (long)hh * a.sqh;
  const u16* Q = a.q + qoff;
  const u16* K = a.k + qoff;
  const u16* V = a.v + qoff;
  const int q0w = qb * QB + w * QW;  // this wave's first query
  const int qi = q0w + r;            // this lane's query
  // Q fragments (B operand of S^T = K Q^T): element j = Q[qi][16t + 8h + j]
  bf16x8 qf[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (qi < a.S) qf[t] = *reinterpret_cast<const bf16x8*>(Q + (long)qi * a.sqs + 16 * t + 8 * h);
    else qf[t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const float sl2 = a.scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x16 o[2] = {zero16(), zero16()};  // O^T[d][q]: d tile 0..1
  const int kend = a.causal ? min(a.S, qb * QB + QB) : a.S;
  for (int k0 = 0; k0 < kend; k0 += KB) {
    __syncthreads();
    stage_rows(Ks, K, a.sqs, k0, KB, a.S);
    stage_rows_tr(Vt, V, a.sqs, k0, KB, a.S);
    __syncthreads();
    if (a.causal && k0 > q0w + QW - 1) continue;  // this wave's queries are all before k0
    // S^T for two 32-key sub-blocks
    f32x16 s[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      s[c] = zero16();
#pragma unroll
      for (int t = 0; t < 4; ++t) s[c] = mfma(row_frag(Ks, KP, 32 * c + r, 16 * t, h), qf[t], s[c]);
    }
    // scale, mask, running max
    float mx = m;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kj = k0 + 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
        float v = s[c][i] * sl2;
        if (kj >= a.S || (a.causal && kj > qi)) v = -INFINITY;
        s[c][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mx);
    float rs = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = (mx == -INFINITY) ? 0.f : exp2f(s[c][i] - mx);
        s[c][i] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 32);
    l = l * alpha + rs;
    m = mx;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
    // O^T[d][q] += sum_k V^T[d][k] P^T[k][q]
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pb = pack8(s[c], st);
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mfma(tr_frag(Vt, TP, 32 * d + r, 32 * c + 16 * st, h), pb, o[d]);
      }
  }
  if (qi >= a.S) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  u16* O = a.out + (long)b * a.sob + (long)hh * a.soh + (long)qi * a.sos;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = f2bf(o[d][4 * g + e] * inv);
      *reinterpret_cast<u16x4*>(O + 32 * d + 8 * g + 4 * h) = v;
    }
  if (h == 0) a.lse[(long)bh * a.S + qi] = m + log2f(l);
}

// ============================================================================================
// backward, part 0: delta[q] = sum_d dO[q][d] * O[q][d]   (one wave per 64 queries... per row)
__global__ void __launch_bounds__(256) attn_delta_kernel(AttnArgs a) {
  const long rows = (long)a.B * a.H * a.S;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < rows; i += (long)gridDim.x * 256) {
    const int qi = (int)(i % a.S);
    const long bh = i / a.S;
    const int b = (int)(bh / a.H), hh = (int)(bh % a.H);
    const long off = (long)b * a.sob + (long)hh * a.soh + (long)qi * a.sos;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      u16x8 x = *reinterpret_cast<const u16x8*>(a.o + off + 8 * c);
      u16x8 y = *reinterpret_cast<const u16x8*>(a.dout + off + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += bf2f(x[e]) * bf2f(y[e]);
    }
    a.delta[i] = s;
  }
}

// backward, part 1: dK, dV. Workgroup = 128 keys (wave = 32 keys); loop over query blocks of 64.
//   S  = Q K^T      (A = Q rows from LDS, B = K rows of this wave -> registers); C: key on lane
//   P  = exp2(S*c - lse[q])                       (lse per register row, from LDS)
//   dV^T[d][k] += dO^T[d][q] P[q][k]              (A = dO^T transposed image, B = P registers)
//   dP = dO V^T     (A = dO rows from LDS, B = V rows of this wave -> registers)
//   dS = P (dP - delta[q])
//   dK^T[d][k] += Q^T[d][q] dS[q][k]              (A = Q^T transposed image, B = dS registers)
constexpr int BQ = 64;  // queries per iteration (backward)

__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) u16 Qs[BQ * KP];
  __shared__ __attribute__((aligned(16))) u16 Qt[HD * TP];
  __shared__ __attribute__((aligned(16))) u16 Ds[BQ * KP];
  __shared__ __attribute__((aligned(16))) u16 Dt[HD * TP];
  __shared__ float Ls[BQ], Dl[BQ];
  const int nkb = (a.S + QB - 1) / QB;
  const int bh = blockIdx.x / nkb;
  const int kb = blockIdx.x % nkb;  // light blocks (early keys see many queries) first... any order
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long off = (long)b * a.sqb + (long)hh * a.sqh;
  const long ooff = (long)b * a.sob + (long)hh * a.soh;
  const int k0w = kb * QB + w * QW;
  const int kj = k0w + r;  // this lane's key (column of S, dP, dV^T, dK^T)
  bf16x8 kf[4], vf[4];     // B operands: K[kj][16t + 8h + j], V[kj][...]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (kj < a.S) {
      kf[t] = *reinterpret_cast<const bf16x8*>(a.k + off + (long)kj * a.sqs + 16 * t + 8 * h);
      vf[t] = *reinterpret_cast<const bf16x8*>(a.v + off + (long)kj * a.sqs + 16 * t + 8 * h);
    } else {
      kf[t] = vf[t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const float sl2 = a.scale * LOG2E;
  f32x16 dv[2] = {zero16(), zero16()}, dk[2] = {zero16(), zero16()};
  const int qstart = a.causal ? (kb * QB) / BQ * BQ : 0;
  for (int q0 = qstart; q0 < a.S; q0 += BQ) {
    __syncthreads();
    stage_rows(Qs, a.q + off, a.sqs, q0, BQ, a.S);
    stage_rows_tr(Qt, a.q + off, a.sqs, q0, BQ, a.S);
    stage_rows(Ds, a.dout + ooff, a.sos, q0, BQ, a.S);
    stage_rows_tr(Dt, a.dout + ooff, a.sos, q0, BQ, a.S);
    if (threadIdx.x < BQ) {
      const int qi = q0 + threadIdx.x;
      Ls[threadIdx.x] = qi < a.S ? a.lse[(long)bh * a.S + qi] : 0.f;
      Dl[threadIdx.x] = qi < a.S ? a.delta[(long)bh * a.S + qi] : 0.f;
    }
    __syncthreads();
    if (a.causal && q0 + BQ - 1 < k0w) continue;  // all these queries precede this wave's keys
#pragma unroll
    for (int c = 0; c < 2; ++c) {  // 32-query sub-blocks
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s = mfma(row_frag(Qs, KP, 32 * c + r, 16 * t, h), kf[t], s);
        dp = mfma(row_frag(Ds, KP, 32 * c + r, 16 * t, h), vf[t], dp);
      }
      // rows of s/dp are queries: q = q0 + 32c + (i&3) + 8(i>>2) + 4h
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
        const int qi = q0 + ql;
        float p = exp2f(s[i] * sl2 - Ls[ql]);
        if (qi >= a.S || kj >= a.S || (a.causal && kj > qi)) p = 0.f;
        s[i] = p;
        dp[i] = p * (dp[i] - Dl[ql]);  // dS (scale applied to dK at the end)
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pb = pack8(s, st), db = pack8(dp, st);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = mfma(tr_frag(Dt, TP, 32 * d + r, 32 * c + 16 * st, h), pb, dv[d]);
          dk[d] = mfma(tr_frag(Qt, TP, 32 * d + r, 32 * c + 16 * st, h), db, dk[d]);
        }
      }
    }
  }
  if (kj >= a.S) return;
  // dV^T / dK^T: lane = key, register rows = d
  u16* DV = a.dv + off + (long)kj * a.sqs;  // grads use the q/k/v layout
  u16* DK = a.dk + off + (long)kj * a.sqs;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u16x4 x, y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[e] = f2bf(dv[d][4 * g + e]);
        y[e] = f2bf(dk[d][4 * g + e] * a.scale);
      }
      *reinterpret_cast<u16x4*>(DV + 32 * d + 8 * g + 4 * h) = x;
      *reinterpret_cast<u16x4*>(DK + 32 * d + 8 * g + 4 * h) = y;
    }
}

// backward, part 2: dQ. Workgroup = 128 queries (wave = 32); loop over key blocks of 64.
//   S^T  = K Q^T     (A = K rows from LDS, B = Q rows of this wave -> registers); lane = query
//   P^T  = exp2(S^T c - lse[q])      (lse per lane)
//   dP^T = V dO^T    (A = V rows from LDS, B = dO rows of this wave -> registers)
//   dS^T = P^T (dP^T - delta[q])
//   dQ^T[d][q] += K^T[d][k] dS^T[k][q]   (A = K^T transposed image, B = dS^T registers)
__global__ void __launch_bounds__(256, 2) attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) u16 Ks[KB * KP];
  __shared__ __attribute__((aligned(16))) u16 Kt[HD * TP];
  __shared__ __attribute__((aligned(16))) u16 Vs[KB * KP];
  const int nqb = (a.S + QB - 1) / QB;
  const int bh = blockIdx.x / nqb;
  const int qb = nqb - 1 - (blockIdx.x % nqb);
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long off = (long)b * a.sqb + (long)hh * a.sqh;
  const long ooff = (long)b * a.sob + (long)hh * a.soh;
  const int q0w = qb * QB + w * QW;
  const int qi = q0w + r;
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (qi < a.S) {
      qf[t] = *reinterpret_cast<const bf16x8*>(a.q + off + (long)qi * a.sqs + 16 * t + 8 * h);
      df[t] = *reinterpret_cast<const bf16x8*>(a.dout + ooff + (long)qi * a.sos + 16 * t + 8 * h);
    } else {
      qf[t] = df[t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const float lse = qi < a.S ? a.lse[(long)bh * a.S + qi] : 0.f;
  const float dl = qi < a.S ? a.delta[(long)bh * a.S + qi] : 0.f;
  const float sl2 = a.scale * LOG2E;
  f32x16 dq[2] = {zero16(), zero16()};
  const int kend = a.causal ? min(a.S, qb * QB + QB) : a.S;
  for (int k0 = 0; k0 < kend; k0 += KB) {
    __syncthreads();
    stage_rows(Ks, a.k + off, a.sqs, k0, KB, a.S);
    stage_rows_tr(Kt, a.k + off, a.sqs, k0, KB, a.S);
    stage_rows(Vs, a.v + off, a.sqs, k0, KB, a.S);
    __syncthreads();
    if (a.causal && k0 > q0w + QW - 1) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s = mfma(row_frag(Ks, KP, 32 * c + r, 16 * t, h), qf[t], s);
        dp = mfma(row_frag(Vs, KP, 32 * c + r, 16 * t, h), df[t], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kj = k0 + 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
        float p = exp2f(s[i] * sl2 - lse);
        if (qi >= a.S || kj >= a.S || (a.causal && kj > qi)) p = 0.f;
        dp[i] = p * (dp[i] - dl);
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 db = pack8(dp, st);
#pragma unroll
        for (int d = 0; d < 2; ++d) dq[d] = mfma(tr_frag(Kt, TP, 32 * d + r, 32 * c + 16 * st, h), db, dq[d]);
      }
    }
  }
  if (qi >= a.S) return;
  u16* DQ = a.dq + off + (long)qi * a.sqs;
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u16x4 x;
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = f2bf(dq[d][4 * g + e] * a.scale);
      *reinterpret_cast<u16x4*>(DQ + 32 * d + 8 * g + 4 * h) = x;
    }
}

AttnArgs make_args(const AttnShape& s) {
  AttnArgs a;
  a.q = reinterpret_cast<const u16*>(s.q);
  a.k = reinterpret_cast<const u16*>(s.k);
  a.v = reinterpret_cast<const u16*>(s.v);
  a.o = reinterpret_cast<const u16*>(s.o);
  a.dout = reinterpret_cast<const u16*>(s.dout);
  a.out = reinterpret_cast<u16*>(s.out);
  a.dq = reinterpret_cast<u16*>(s.dq);
  a.dk = reinterpret_cast<u16*>(s.dk);
  a.dv = reinterpret_cast<u16*>(s.dv);
  a.lse = s.lse;
  a.delta = s.delta;
  a.B = s.B;
  a.H = s.H;
  a.S = s.S;
  a.sqb = s.sqb;
  a.sqh = s.sqh;
  a.sqs = s.sqs;
  a.sob = s.sob;
  a.soh = s.soh;
  a.sos = s.sos;
  a.scale = s.scale;
  a.causal = s.causal;
  return a;
}

}  // namespace

void attention_fwd_bf16(const AttnShape& s, hipStream_t stream) {
  AttnArgs a = make_args(s);
  const int nqb = (s.S + QB - 1) / QB;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
}

void attention_bwd_bf16(const AttnShape& s, hipStream_t stream) {
  AttnArgs a = make_args(s);
  const long rows = (long)s.B * s.H * s.S;
  long db = (rows + 255) / 256;
  if (db > 4096) db = 4096;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)db), dim3(256), 0, stream, a);
  const int nb = (s.S + QB - 1) / QB;
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3(nb * s.B * s.H), dim3(256), 0, stream, a);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(nb * s.B * s.H), dim3(256), 0, stream, a);
}

}  // namespace sdml
