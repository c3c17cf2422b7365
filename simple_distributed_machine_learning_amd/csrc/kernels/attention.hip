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
// Backward: dQ kernel (workgroup = 128 queries; loops over key blocks; also writes delta = rowsum(dO * O)), then
// dK/dV kernel (workgroup = 128 keys; loops over query blocks) — no atomics, P recomputed from LSE.
//
// Tiles (64 rows x 64 d, bf16) live in LDS as ONE swizzled row-major image each, read two ways:
//   * by rows with ds_read_b128 (operands whose MFMA k is d: S = K Q^T, dP = dO V^T, ...)
//   * by columns with ds_read_b64_tr_b16 (operands whose MFMA k is the key/query axis:
//     V^T P^T, dO^T P, Q^T dS, K^T dS^T) — the hardware transpose read replaces a transposed
//     second copy written element by element.
//   Chunk c (16 B) of row r is stored at chunk c ^ f(r), f(r) = ((r>>1)&1)<<2 | ((r>>2)&3):
//   both read kinds are bank-conflict-free on 128-B rows (the row reads' 16-lane groups hit
//   16 distinct 16-B slots; each 32-lane half of a transposed read covers 4 rows x 4 chunks in
//   16 distinct slots).
// Every loop double-buffers its tiles: the next tile's global loads are issued into registers
// before the current tile's MFMAs and written to the other LDS buffer after them, so the HBM/L2
// latency hides behind compute and each iteration has one barrier.
// Measured and rejected (forward, GPT-2 shape, tools/attn_prof.py): the softmax denominator on the
// matrix core (an all-ones d tile) plus FA4-style lazy rescaling removed 34 VALU adds and 16
// packed multiplies per tile but ran 93 vs 87 us: the loop is not VALU-issue bound; at ~12 % MFMA
// busy (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES). A two-tile-deep prefetch (K/V by global_load_lds into
// a 3-buffer ring, counted vmcnt + raw barriers, the V^T reads as inline-asm ds_read_b64_tr_b16 so
// hipcc stops draining the DMA before them) ran 90-91 vs 88 us as well: neither VALU issue nor the
// tile prefetch depth is what bounds this loop.
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

// v_exp_f32 directly (exp2f adds denormal range fix-ups we do not need: arguments are <= 0 or
// -inf, and flushing tiny probabilities to 0 is harmless)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

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

// ---- swizzled tile image ----------------------------------------------------------------------
constexpr int TR = 64;  // rows per staged tile (KB keys or BQ queries)
__device__ __forceinline__ int swz(int r, int ch) {
  return r * HD + 8 * (ch ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3)));
}
// row fragment (A/B operand with k = d): element j = X[row][16t + 8h + j]
__device__ __forceinline__ bf16x8 rowf(const u16* X, int row, int t, int h) {
  return *reinterpret_cast<const bf16x8*>(X + swz(row, 2 * t + h));
}
typedef __attribute__((ext_vector_type(4))) short s16x4;
__device__ __forceinline__ s16x4 ds_tr16(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
// transposed fragment in the accumulator k-order: element j = X[k0 + 8(j>>2) + 4h + (j&3)][c0 + (lane&31)]
// (k0 % 8 == 0, c0 % 32 == 0). Two ds_read_b64_tr_b16: each 16-lane group g reads rows
// k0 + 4(g>>1) + q (q = 0..3) at columns c0 + 16(g&1) + 0..15; lane 4q+p supplies row q, cols 4p..4p+3.
// Must run with all 64 lanes active.
__device__ __forceinline__ bf16x8 trf(const u16* X, int k0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int R = k0 + 4 * (g >> 1) + q;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const s16x4 lo = ds_tr16(X + swz(R, col >> 3) + (col & 7));
  const s16x4 hi = ds_tr16(X + swz(R + 8, col >> 3) + (col & 7));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// a tile of ROWS rows in registers (ROWS * 8 / NTH x 16 B per thread of an NTH-thread block) on its way from global
// memory to LDS
template <int ROWS, int NTH = 256>
struct TileRegs {
  u16x8 v[ROWS * 8 / NTH];
};
template <int ROWS, int NTH>
__device__ __forceinline__ void tile_load(TileRegs<ROWS, NTH>& t, const u16* G, long srow, int r0, int S) {
#pragma unroll
  for (int u = 0; u < ROWS * 8 / NTH; ++u) {
    const int idx = threadIdx.x + NTH * u, r = idx >> 3, ch = idx & 7;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < S) v = *reinterpret_cast<const u16x8*>(G + (long)(r0 + r) * srow + 8 * ch);
    t.v[u] = v;
  }
}
// rows past S re-read row S - 1 (unconditional loads, no exec-masked branches): only for consumers that mask those
// keys themselves (the forward's edge tiles set their scores to -inf, so their V rows meet P = 0)
template <int ROWS, int NTH>
__device__ __forceinline__ void tile_load_clamped(TileRegs<ROWS, NTH>& t, const u16* G, long srow, int r0, int S) {
#pragma unroll
  for (int u = 0; u < ROWS * 8 / NTH; ++u) {
    const int idx = threadIdx.x + NTH * u, r = idx >> 3, ch = idx & 7;
    t.v[u] = *reinterpret_cast<const u16x8*>(G + (long)min(r0 + r, S - 1) * srow + 8 * ch);
  }
}
template <int ROWS, int NTH>
__device__ __forceinline__ void tile_store(u16* L, const TileRegs<ROWS, NTH>& t) {
#pragma unroll
  for (int u = 0; u < ROWS * 8 / NTH; ++u) {
    const int idx = threadIdx.x + NTH * u, r = idx >> 3, ch = idx & 7;
    *reinterpret_cast<u16x8*>(L + swz(r, ch)) = t.v[u];
  }
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

// XCD-aware block order: the dispatcher deals consecutive workgroup ids round-robin to the 8 XCDs, so
// the blocks of one (batch, head) - which all read the same K/V (or Q/dO) tiles - would land on 8
// different L2s. Logical block L = (id % 8) * (n / 8) + id / 8 keeps consecutive L (same (b, h)) on one
// XCD (bijective when n % 8 == 0; otherwise the plain order).
__device__ __forceinline__ int xcd_block(int id, int n) { return (n % 8 == 0) ? (id % 8) * (n / 8) + id / 8 : id; }

// ============================================================================================
// forward
// QS: 32-query sub-blocks per wave (1: 32 queries per wave; 2: 64). With QS = 2 each K / V fragment read from LDS
// feeds both sub-blocks' MFMAs and the wave carries two independent score -> softmax -> PV chains, so one sub-block's
// exp / max / sum VALU work can issue beside the other's MFMAs. NWV waves per workgroup (4, or 2 with QS = 2: the
// same 128 queries per workgroup, four workgroups per CU).
template <int KBT, int QS, int NWV = NW, int MINW = 8 / NWV>  // keys per tile (64 or 128); MINW: waves per SIMD bound
__global__ void __launch_bounds__(64 * NWV, MINW) attn_fwd_kernel(AttnArgs a) {
  constexpr int NC = KBT / 32;  // 32-key sub-blocks per tile
  constexpr int QWV = QW * QS;  // queries per wave
  constexpr int QBW = QWV * NWV;  // queries per workgroup
  constexpr int NTH = 64 * NWV;
  __shared__ __attribute__((aligned(16))) u16 Ks[2][KBT * HD];
  __shared__ __attribute__((aligned(16))) u16 Vs[2][KBT * HD];
  const int nqb = (a.S + QBW - 1) / QBW;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int bh = blk / nqb;
  const int qb = nqb - 1 - (blk % nqb);  // heaviest (causal) blocks first
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 31,
            h = lane >> 5;
  const long qoff = (long)b * a.sqb + (long)hh * a.sqh;
  const u16* Q = a.q + qoff;
  const u16* K = a.k + qoff;
  const u16* V = a.v + qoff;
  const int q0w = qb * QBW + w * QWV;  // this wave's first query
  int qi[QS];                          // this lane's query in each sub-block
  // Q fragments (B operand of S^T = K Q^T): element j = Q[qi][16t + 8h + j]
  bf16x8 qf[QS][4];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    qi[u] = q0w + QW * u + r;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (qi[u] < a.S) qf[u][t] = *reinterpret_cast<const bf16x8*>(Q + (long)qi[u] * a.sqs + 16 * t + 8 * h);
      else qf[u][t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const float sl2 = a.scale * LOG2E;
  float m[QS], l[QS];
  f32x16 o[QS][2];  // O^T[d][q]: d tile 0..1
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    m[u] = -INFINITY;
    l[u] = 0.f;
    o[u][0] = o[u][1] = zero16();
  }
  const int kend = a.causal ? min(a.S, qb * QBW + QBW) : a.S;
  TileRegs<KBT, NTH> kr, vr;
  tile_load_clamped(kr, K, a.sqs, 0, a.S);
  tile_load_clamped(vr, V, a.sqs, 0, a.S);
  tile_store(Ks[0], kr);
  tile_store(Vs[0], vr);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < kend; k0 += KBT, buf ^= 1) {
    const bool more = k0 + KBT < kend;
    if (more) {  // next tile's loads fly during this tile's MFMAs
      tile_load_clamped(kr, K, a.sqs, k0 + KBT, a.S);
      tile_load_clamped(vr, V, a.sqs, k0 + KBT, a.S);
    }
    if (!(a.causal && k0 > q0w + QWV - 1)) {  // else: all this wave's queries precede k0
      const u16* Kt = Ks[buf];
      const u16* Vt = Vs[buf];
      // S^T for the 32-key sub-blocks of every query sub-block (one K fragment read feeds all QS of them). A query
      // sub-block that lies wholly before k0 (QS = 2, diagonal tiles) computes scores that the mask turns to -inf:
      // its p are 0 and its m, l, o stay unchanged (alpha = 1)
      f32x16 s[QS][NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int u = 0; u < QS; ++u) s[u][c] = zero16();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 kfr = rowf(Kt, 32 * c + r, t, h);
#pragma unroll
          for (int u = 0; u < QS; ++u) s[u][c] = mfma(kfr, qf[u][t], s[u][c]);
        }
      }
      // mask (diagonal / ragged tiles only) and running max on the RAW scores; the softmax scale
      // is folded into one FMA per score: p = exp2(s * c - max * c), c = scale * log2(e) > 0
      const bool edge = (a.causal && k0 + KBT - 1 > q0w) || k0 + KBT > a.S;
      float alpha[QS];
#pragma unroll
      for (int u = 0; u < QS; ++u) {
        if (edge) {  // (one uniform branch; per element a compare + select: hipcc turned the per-element `if` into 2
                     // scalar branches per score, on the unmasked tiles too)
          const int lim = (a.causal ? min(qi[u], a.S - 1) : a.S - 1) - (k0 + 4 * h);  // last key this lane may see
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              s[u][c][i] = (32 * c + (i & 3) + 8 * (i >> 2) > lim) ? -INFINITY : s[u][c][i];
        }
        float mr = -INFINITY;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int i = 0; i < 16; ++i) mr = fmaxf(mr, s[u][c][i]);
        mr = fmaxf(mr, __shfl_xor(mr, 32));
        const float mx = fmaxf(m[u], mr * sl2);  // running max, log2 domain
        alpha[u] = (m[u] == -INFINITY) ? 0.f : ex2(m[u] - mx);
        const float msub = (mx == -INFINITY) ? 0.f : mx;  // all-masked so far: exp2(-inf) = 0
        float rs = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = ex2(__builtin_fmaf(s[u][c][i], sl2, -msub));
            s[u][c][i] = p;
            rs += p;
          }
        rs += __shfl_xor(rs, 32);
        l[u] = l[u] * alpha[u] + rs;
        m[u] = mx;
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[u][d][i] *= alpha[u];
      }
      // O^T[d][q] += sum_k V^T[d][k] P^T[k][q]   (V^T by transposed reads of the V image, shared by the sub-blocks)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 pb[QS];
#pragma unroll
          for (int u = 0; u < QS; ++u) pb[u] = pack8(s[u][c], st);
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const bf16x8 vt = trf(Vt, 32 * c + 16 * st, 32 * d, lane);
#pragma unroll
            for (int u = 0; u < QS; ++u) o[u][d] = mfma(vt, pb[u], o[u][d]);
          }
        }
    }
    if (more) {
      tile_store(Ks[buf ^ 1], kr);
      tile_store(Vs[buf ^ 1], vr);
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    if (qi[u] >= a.S) continue;
    const float inv = l[u] > 0.f ? 1.f / l[u] : 0.f;
    u16* O = a.out + (long)b * a.sob + (long)hh * a.soh + (long)qi[u] * a.sos;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[u][d][4 * g + e] * inv);
        *reinterpret_cast<u16x4*>(O + 32 * d + 8 * g + 4 * h) = v;
      }
    if (h == 0) a.lse[(long)bh * a.S + qi[u]] = m[u] + log2f(l[u]);
  }
}

// ============================================================================================
// backward, part 1: dK, dV. Workgroup = 128 keys (wave = 32 keys); loop over query blocks of 64.
//   S  = Q K^T      (A = Q rows, B = K rows of this wave -> registers); C: key on lane
//   P  = exp2(S*c - lse[q])                       (lse per register row, from LDS)
//   dV^T[d][k] += dO^T[d][q] P[q][k]              (A = dO^T by transposed reads, B = P registers)
//   dP = dO V^T     (A = dO rows, B = V rows of this wave -> registers)
//   dS = P (dP - delta[q])
//   dK^T[d][k] += Q^T[d][q] dS[q][k]              (A = Q^T by transposed reads, B = dS registers)
constexpr int BQ = 64;  // queries per iteration (backward)

// NKT: 32-key tiles per wave (1: 128 keys per workgroup, 2 waves per SIMD; 2: 256 keys per workgroup, one wave per
// SIMD with up to 512 registers: every Q / dO fragment read from LDS (rows and transposed) feeds both key tiles'
// MFMAs, so the LDS reads per MFMA halve and each wave carries two independent accumulation chains)
template <int NKT>
__global__ void __launch_bounds__(256, NKT == 1 ? 2 : 1) attn_bwd_dkdv_kernel(AttnArgs a) {
  constexpr int KW = QW * NKT;  // keys per wave
  constexpr int KBW = KW * NW;  // keys per workgroup
  __shared__ __attribute__((aligned(16))) u16 Qs[2][TR * HD];
  __shared__ __attribute__((aligned(16))) u16 Ds[2][TR * HD];
  __shared__ float Ls[2][BQ], Dl[2][BQ];
  const int nkb = (a.S + KBW - 1) / KBW;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int bh = blk / nkb;
  const int kb = blk % nkb;
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 31,
            h = lane >> 5;
  const long off = (long)b * a.sqb + (long)hh * a.sqh;
  const long ooff = (long)b * a.sob + (long)hh * a.soh;
  const int k0w = kb * KBW + w * KW;
  int kj[NKT];  // this lane's keys (column of S, dP, dV^T, dK^T), one per key tile
  bf16x8 kf[NKT][4], vf[NKT][4];  // B operands: K[kj][16t + 8h + j], V[kj][...]
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    kj[kt] = k0w + QW * kt + r;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (kj[kt] < a.S) {
        kf[kt][t] = *reinterpret_cast<const bf16x8*>(a.k + off + (long)kj[kt] * a.sqs + 16 * t + 8 * h);
        vf[kt][t] = *reinterpret_cast<const bf16x8*>(a.v + off + (long)kj[kt] * a.sqs + 16 * t + 8 * h);
      } else {
        kf[kt][t] = vf[kt][t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }
  const float sl2 = a.scale * LOG2E;
  f32x16 dv[NKT][2], dk[NKT][2];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
    for (int d = 0; d < 2; ++d) dv[kt][d] = dk[kt][d] = zero16();
  const int qstart = a.causal ? (kb * KBW) / BQ * BQ : 0;
  const float* LSE = a.lse + (long)bh * a.S;
  const float* DEL = a.delta + (long)bh * a.S;
  TileRegs<TR> qr, dr;
  float lr = 0.f, dlr = 0.f;
  auto load = [&](int q0) {
    tile_load(qr, a.q + off, a.sqs, q0, a.S);
    tile_load(dr, a.dout + ooff, a.sos, q0, a.S);
    if (threadIdx.x < BQ) {
      const int qi = q0 + threadIdx.x;
      lr = qi < a.S ? LSE[qi] : 0.f;
      dlr = qi < a.S ? DEL[qi] : 0.f;
    }
  };
  auto store = [&](int bi) {
    tile_store(Qs[bi], qr);
    tile_store(Ds[bi], dr);
    if (threadIdx.x < BQ) {
      Ls[bi][threadIdx.x] = lr;
      Dl[bi][threadIdx.x] = dlr;
    }
  };
  if (qstart < a.S) {
    load(qstart);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int q0 = qstart; q0 < a.S; q0 += BQ, buf ^= 1) {
    const bool more = q0 + BQ < a.S;
    if (more) load(q0 + BQ);
    if (!(a.causal && q0 + BQ - 1 < k0w)) {  // else: all these queries precede this wave's keys
      const u16* Qt = Qs[buf];
      const u16* Dt = Ds[buf];
      // only the causal diagonal needs a mask: rows past S are zero-filled Q/dO (their P and dS
      // terms multiply zero rows), and lanes with kj >= S are never stored
      const bool edge = a.causal && q0 < k0w + KW - 1;
      // (NKT == 2: the two 32-query sub-blocks one after the other; unrolled, hipcc overlapped their score
      // registers and spilled)
#pragma unroll (NKT == 1 ? 2 : 1)
      for (int c = 0; c < 2; ++c) {  // 32-query sub-blocks
        f32x16 s[NKT], dp[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) s[kt] = dp[kt] = zero16();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16x8 qa = rowf(Qt, 32 * c + r, t, h), da = rowf(Dt, 32 * c + r, t, h);
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt) {
            s[kt] = mfma(qa, kf[kt][t], s[kt]);
            dp[kt] = mfma(da, vf[kt][t], dp[kt]);
          }
        }
        // rows of s/dp are queries: q = q0 + 32c + (i&3) + 8(i>>2) + 4h
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int ql = 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
          const float lq = Ls[buf][ql], dq = Dl[buf][ql];
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt) {
            float p = ex2(s[kt][i] * sl2 - lq);
            if (edge && kj[kt] > q0 + ql) p = 0.f;
            s[kt][i] = p;
            dp[kt][i] = p * (dp[kt][i] - dq);  // dS (scale applied to dK at the end)
          }
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const bf16x8 dta = trf(Dt, 32 * c + 16 * st, 32 * d, lane), qta = trf(Qt, 32 * c + 16 * st, 32 * d, lane);
#pragma unroll
            for (int kt = 0; kt < NKT; ++kt) {
              dv[kt][d] = mfma(dta, pack8(s[kt], st), dv[kt][d]);
              dk[kt][d] = mfma(qta, pack8(dp[kt], st), dk[kt][d]);
            }
          }
        }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
  // dV^T / dK^T: lane = key, register rows = d
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kj[kt] >= a.S) continue;
    u16* DV = a.dv + off + (long)kj[kt] * a.sqs;  // grads use the q/k/v layout
    u16* DK = a.dk + off + (long)kj[kt] * a.sqs;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 x, y;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = f2bf(dv[kt][d][4 * g + e]);
          y[e] = f2bf(dk[kt][d][4 * g + e] * a.scale);
        }
        *reinterpret_cast<u16x4*>(DV + 32 * d + 8 * g + 4 * h) = x;
        *reinterpret_cast<u16x4*>(DK + 32 * d + 8 * g + 4 * h) = y;
      }
  }
}

// backward, part 2: dQ. Workgroup = 128 queries (wave = 32); loop over key blocks of 64.
//   S^T  = K Q^T     (A = K rows, B = Q rows of this wave -> registers); lane = query
//   P^T  = exp2(S^T c - lse[q])      (lse per lane)
//   dP^T = V dO^T    (A = V rows, B = dO rows of this wave -> registers)
//   dS^T = P^T (dP^T - delta[q])
//   dQ^T[d][q] += K^T[d][k] dS^T[k][q]   (A = K^T by transposed reads, B = dS^T registers)
__global__ void __launch_bounds__(256, 2) attn_bwd_dq_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) u16 Ks[2][TR * HD];
  __shared__ __attribute__((aligned(16))) u16 Vs[2][TR * HD];
  const int nqb = (a.S + QB - 1) / QB;
  const int blk = xcd_block(blockIdx.x, gridDim.x);
  const int bh = blk / nqb;
  const int qb = nqb - 1 - (blk % nqb);
  const int b = bh / a.H, hh = bh % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 31,
            h = lane >> 5;
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
  // delta[q] = sum_d dO[q][d] O[q][d] from the dO fragments already in registers (this lane: d = 16t + 8h + j) and
  // the same elements of O, the two lane halves combined by one xor-32 exchange; written for the dK/dV kernel, which
  // runs after this one (no separate delta pass over O and dO)
  float dl = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    bf16x8 of = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (qi < a.S) of = *reinterpret_cast<const bf16x8*>(a.o + ooff + (long)qi * a.sos + 16 * t + 8 * h);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf(bf2f((u16)df[t][j]), bf2f((u16)of[j]), dl);
  }
  dl += __shfl_xor(dl, 32);
  if (h == 0 && qi < a.S) a.delta[(long)bh * a.S + qi] = dl;
  const float sl2 = a.scale * LOG2E;
  f32x16 dq[2] = {zero16(), zero16()};
  const int kend = a.causal ? min(a.S, qb * QB + QB) : a.S;
  TileRegs<TR> kr, vr;
  tile_load(kr, a.k + off, a.sqs, 0, a.S);
  tile_load(vr, a.v + off, a.sqs, 0, a.S);
  tile_store(Ks[0], kr);
  tile_store(Vs[0], vr);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < kend; k0 += KB, buf ^= 1) {
    const bool more = k0 + KB < kend;
    if (more) {
      tile_load(kr, a.k + off, a.sqs, k0 + KB, a.S);
      tile_load(vr, a.v + off, a.sqs, k0 + KB, a.S);
    }
    if (!(a.causal && k0 > q0w + QW - 1)) {
      const u16* Kt = Ks[buf];
      const u16* Vt = Vs[buf];
      // causal diagonal only: keys past S have zero K/V rows (their dS^T terms multiply zero
      // K^T columns) and lanes with qi >= S are never stored
      const bool edge = a.causal && k0 + KB - 1 > q0w;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f32x16 s = zero16(), dp = zero16();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s = mfma(rowf(Kt, 32 * c + r, t, h), qf[t], s);
          dp = mfma(rowf(Vt, 32 * c + r, t, h), df[t], dp);
        }
        const int lim = edge ? qi - (k0 + 32 * c + 4 * h) : 1000000;  // (branch-free causal mask, as in the forward)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float p = ex2(s[i] * sl2 - lse);
          p = ((i & 3) + 8 * (i >> 2) > lim) ? 0.f : p;
          dp[i] = p * (dp[i] - dl);
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 db = pack8(dp, st);
#pragma unroll
          for (int d = 0; d < 2; ++d) dq[d] = mfma(trf(Kt, 32 * c + 16 * st, 32 * d, lane), db, dq[d]);
        }
      }
    }
    if (more) {
      tile_store(Ks[buf ^ 1], kr);
      tile_store(Vs[buf ^ 1], vr);
    }
    __syncthreads();
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

static int g_fwd_kb = 0;  // 0: default; 64 / 128 (A/B experiments)
void attention_set_fwd_kb(int kb) { g_fwd_kb = kb; }

void attention_fwd_bf16(const AttnShape& s, hipStream_t stream) {
  AttnArgs a = make_args(s);
  const int qs = knob(KNOB_ATTN_FWD_QS);
  if (qs == 2) {  // 64 queries per wave (two sub-blocks), 4 waves: 256 per workgroup
    const int nqb = (s.S + 2 * QB - 1) / (2 * QB);
    hipLaunchKernelGGL((attn_fwd_kernel<64, 2>), dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
    return;
  }
  if (qs == 3) {  // 64 queries per wave, 2 waves: 128 per workgroup (the QS = 1 grid)
    const int nqb = (s.S + QB - 1) / QB;
    hipLaunchKernelGGL((attn_fwd_kernel<64, 2, 2>), dim3(nqb * s.B * s.H), dim3(128), 0, stream, a);
    return;
  }
  const int nqb = (s.S + QB - 1) / QB;
  const int occ = knob(KNOB_ATTN_OCC);  // (A/B) register bound for 3 or 4 waves per SIMD instead of 2
  if (g_fwd_kb == 128)
    hipLaunchKernelGGL((attn_fwd_kernel<128, 1>), dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
  else if (occ == 3)
    hipLaunchKernelGGL((attn_fwd_kernel<64, 1, NW, 3>), dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
  else if (occ == 4)
    hipLaunchKernelGGL((attn_fwd_kernel<64, 1, NW, 4>), dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<64, 1>), dim3(nqb * s.B * s.H), dim3(256), 0, stream, a);
}

void attention_bwd_bf16(const AttnShape& s, hipStream_t stream) {
  AttnArgs a = make_args(s);
  const int nb = (s.S + QB - 1) / QB;
  // dQ first: it computes delta = rowsum(dO * O) for its own queries and writes it for dK/dV
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3(nb * s.B * s.H), dim3(256), 0, stream, a);
  // dK/dV: 128 keys per workgroup (one 32-key tile per wave); knob ATTN_DKDV_KT = 2: 256 (measured slower)
  if (knob(KNOB_ATTN_DKDV_KT) == 2) {
    const int nk2 = (s.S + 2 * QB - 1) / (2 * QB);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<2>, dim3(nk2 * s.B * s.H), dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<1>, dim3(nb * s.B * s.H), dim3(256), 0, stream, a);
  }
}

}  // namespace sdml
