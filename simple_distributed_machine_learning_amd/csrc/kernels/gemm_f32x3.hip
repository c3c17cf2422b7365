// fp32 GEMM on the bf16 matrix cores: every fp32 operand is split into three bf16 terms
// x = hi + mid + lo (round-to-nearest at each step; the split is EXACT: 8 + 8 + 8 significant
// bits = the fp32 mantissa) and the product is formed from the six terms that matter,
//   a*b ~= hi*hi + (hi*mid + mid*hi) + (hi*lo + lo*hi + mid*mid),
// each term an exact bf16 x bf16 product accumulated in fp32 by v_mfma_f32_32x32x16_bf16.
// The dropped terms (mid*lo, lo*mid, lo*lo) are below 2^-24 |a*b|: the result has fp32
// accuracy (compared against an fp64 reference together with the
// error of the exact-fp32 v_mfma_f32_32x32x2_f32 path; tests/test_gemm_x3_gpu.py), at 6 bf16 MFMAs per fp32 product:
// bf16 MFMA runs 16x the fp32-input MFMA rate on gfx950, so this is 2.67x the fp32 matrix
// peak and turns the MLP GEMMs (K = 784, 128-wide) from MFMA-bound into HBM-bound.
//
// Same contract as gemm_f32.hip (C[M,N] op= sum_k A(m,k) B(n,k), any of the four operand
// layouts, the same epilogues, ReLU masks and fused bias-gradient row sums); it replaces the
// ATen fc-layer GEMMs of the reference (/root/reference/simple_distributed.py:63-64, :75-77).
//
// Geometry (gfx950, wave64): 512 threads = 8 waves, K-step 32, one workgroup per CU.
// (Measured alternative: 256-thread 128 x 128 workgroups with one LDS buffer, two per CU so one's
//  barrier/split phases run under the other's MFMAs: 205 vs 182 us for the headline forward.)
//   A k-contiguous: block tile 256 x 128, waves 4 x 2, 64 x 64 per wave (2 x 2 MFMA tiles)
//   A k-major     : block tile 128 x 128, waves 2 x 4, 64 x 32 per wave (2 x 1 MFMA tiles)
//   (a 128 x 256 tile for the weight gradient, B = X widened to 256 columns, measured slower:
//    784 columns -> 4 tiles with 31 % padding; 250 vs 217 us at the headline shape)
// LDS holds each operand as three bf16 planes (hi/mid/lo), double-buffered: 144 KiB / 96 KiB.
//   * k-contiguous operand: image [rows][32 k], 64-B rows, 16-B chunk c of row r stored at
//     chunk c ^ ((r >> 2) & 3): the ds_read_b128 fragment reads (8 consecutive k of one row per
//     lane) hit 16 distinct 16-B slots per lane group -> conflict-free.
//   * k-major operand (rows contiguous in memory, e.g. dZ^T or X in the weight gradient):
//     image [32 k][128 rows], 256-B rows, chunk c of row k at c ^ (((k&3)<<2) | ((k>>2)&3));
//     written straight from float4 loads (no transpose in registers) and read by two
//     ds_read_b64_tr_b16 per fragment (hardware transpose), conflict-free on both sides.
// Global -> registers -> (split) -> LDS staging is prefetched one K-step ahead; one barrier
// per K-step (the split of tile t+1 is written to the other buffer after tile t's MFMAs).
// MFMA maps (gfx950): A lane (r = l&31, h = l>>5) holds A[r][k = 8h + j]; B lane holds
// B[k = 8h + j][col r]; C/D: col = l&31, row = (i&3) + 8(i>>2) + 4h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int NT = 512;  // threads per workgroup (main kernel)
constexpr int BK = 32;   // k per K-step
constexpr int BN = 128;  // block tile columns (B operand rows)

struct X3Params {
  const float* A;
  const float* amask;
  const float* B;
  const u16* Bp;  // B pre-split into bf16 planes [3][N][ldb] (k-contiguous B only) or nullptr
  float* C;
  const float* bias;
  float* rowsum;
  const float* cmask;
  int M, N, K, lda, ldb, ldc;
  int epi;
  int kps;  // K per split (multiple of BK)
  int tiles_m, tiles_n;
  const unsigned char* X8;  // U8 kernels: the uint8 pixel operand (A for U8_A, B for U8_B)
  float scale;              // U8 kernels: C = scale * acc (+ bias); 1/255 = ToTensor's scaling
  float* slab;              // split-K partials: split s writes slab + s * slab_stride ([M][ldc]) with
  int64_t slab_stride;      // plain stores instead of atomics (reduced in fixed order afterwards)
};

// which operand (if any) is a uint8 pixel matrix: integers 0..255 have at most 8 significant
// bits, so the operand is EXACT in one bf16 plane and each product needs 3 MFMAs, not 6
enum { U8_NONE = 0, U8_A = 1, U8_B = 2 };

// ---- the split ---------------------------------------------------------------------------------
__device__ __forceinline__ u16 bf16_bits(float f) {
  __bf16 h = static_cast<__bf16>(f);  // round-to-nearest-even (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(u16, h);
}
__device__ __forceinline__ float bf16_val(u16 b) { return __uint_as_float(((unsigned)b) << 16); }

// x -> (hi, mid, lo), x == hi + mid + lo exactly for normal-range x
template <int N>
__device__ __forceinline__ void split3(const float (&x)[N], u16 (&h)[N], u16 (&m)[N], u16 (&l)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    h[j] = bf16_bits(x[j]);
    const float r1 = x[j] - bf16_val(h[j]);
    m[j] = bf16_bits(r1);
    const float r2 = r1 - bf16_val(m[j]);
    l[j] = bf16_bits(r2);
  }
}

// ---- LDS images (offsets in u16 elements) ------------------------------------------------------
// k-contiguous image [rows][32]: chunk ch (8 k) of row r
__device__ __forceinline__ int kc_off(int r, int ch) { return r * BK + 8 * (ch ^ ((r >> 2) & 3)); }
// k-major image [32][128]: 16-B chunk ch (8 rows) of k-row k
__device__ __forceinline__ int km_off(int k, int ch) {
  return k * 128 + 8 * (ch ^ (((k & 3) << 2) | ((k >> 2) & 3)));
}

__device__ __forceinline__ s16x4 ds_tr16(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// A/B fragment of the 32-row sub-tile at r0, k-substep s (k = 16s + 8h + j), natural k order
template <bool KM>
__device__ __forceinline__ bf16x8 frag(const u16* P, int r0, int s, int lane) {
  if constexpr (!KM) {
    const int r = r0 + (lane & 31), h = lane >> 5;
    return *reinterpret_cast<const bf16x8*>(P + kc_off(r, 2 * s + h));
  } else {
    // two ds_read_b64_tr_b16: 16-lane group g reads k-rows 16s + 8(g>>1) + q (+4), q = 0..3, at
    // rows r0 + 16(g&1) + 4p .. +3; lane i of the group receives row r0 + 16(g&1) + i.
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = 16 * s + 8 * (g >> 1) + q;
    const int col = r0 + 16 * (g & 1) + 4 * p;
    const s16x4 lo = ds_tr16(P + km_off(k, col >> 3) + (col & 7));
    const s16x4 hi = ds_tr16(P + km_off(k + 4, col >> 3) + (col & 7));
    bf16x8 f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
}

__device__ __forceinline__ f32x4 mask4(f32x4 x, f32x4 mk) {
  x[0] = mk[0] > 0.f ? x[0] : 0.f;
  x[1] = mk[1] > 0.f ? x[1] : 0.f;
  x[2] = mk[2] > 0.f ? x[2] : 0.f;
  x[3] = mk[3] > 0.f ? x[3] : 0.f;
  return x;
}

// ---- staging of one operand tile (ROWS x BK) ---------------------------------------------------
// k-contiguous: ROWS*4 chunks of 8 k; a thread owns NC = ROWS*4/NT chunks (2 float4 each).
// k-major (ROWS == 128): 32 k-rows x 32 float4; a thread owns 2 float4 (4 rows at one k each).
template <bool KM, int ROWS, int NT = ::sdml::NT>
struct Stage {
  static constexpr int NV = ROWS * BK / 4 / NT;  // float4 per thread
  f32x4 v[NV];

  // Branch-free and select-free: indices are clamped into the operand (rows past the end re-read
  // the last row / float4 and only feed outputs that are never stored; k past kend is zeroed at
  // split time by store()), so the loads' results are not needed until the split and the whole
  // K-step stays one basic block the scheduler can interleave.
  template <bool MASK>
  __device__ __forceinline__ void load(const float* __restrict__ P, const float* __restrict__ mask, int ld,
                                       int rows, int r0, int k0, int K) {
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      size_t o;
      if constexpr (!KM) {
        const int id = t + NT * (u >> 1);  // chunk
        const int gr = min(r0 + (id >> 2), rows - 1);
        const int gk = min(k0 + 8 * (id & 3) + 4 * (u & 1), K - 4);
        o = (size_t)gr * ld + gk;
      } else {
        const int id = t + NT * u;
        const int gk = min(k0 + (id >> 5), K - 1);
        const int gr = min(r0 + 4 * (id & 31), rows - 4);  // rows % 4 == 0 (host check)
        o = (size_t)gk * ld + gr;
      }
      f32x4 x = *reinterpret_cast<const f32x4*>(P + o);
      if constexpr (MASK) x = mask4(x, *reinterpret_cast<const f32x4*>(mask + o));
      v[u] = x;
    }
  }

  // zero the k >= kend part of the tile staged for k0 (the K tail / past the end of a split)
  __device__ __forceinline__ void zero_tail(int k0, int kend) {
    const int t = threadIdx.x;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      int gk;
      if constexpr (!KM) gk = k0 + 8 * ((t + NT * (u >> 1)) & 3) + 4 * (u & 1);
      else gk = k0 + ((t + NT * u) >> 5);
      v[u] = gk < kend ? v[u] : z;
    }
  }

  // fp32 row sums of the staged values (bias gradient): k-contiguous -> one row per chunk,
  // k-major -> 4 rows per float4
  __device__ __forceinline__ void accum_rowsum(float (&rs)[4]) const {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      if constexpr (!KM) {
        rs[u >> 1] += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rs[e] += v[u][e];
      }
    }
  }

  // split into hi/mid/lo and write the three planes (plane stride PL u16)
  template <int PL>
  __device__ __forceinline__ void store(u16* L) const {
    const int t = threadIdx.x;
    if constexpr (!KM) {
#pragma unroll
      for (int c = 0; c < NV / 2; ++c) {
        const int id = t + NT * c;
        float x[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] = v[2 * c][e];
          x[4 + e] = v[2 * c + 1][e];
        }
        u16 h[8], m[8], l[8];
        split3<8>(x, h, m, l);
        const int o = kc_off(id >> 2, id & 3);
        u16x8 H, Mi, Lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          H[e] = h[e];
          Mi[e] = m[e];
          Lo[e] = l[e];
        }
        *reinterpret_cast<u16x8*>(L + o) = H;
        *reinterpret_cast<u16x8*>(L + PL + o) = Mi;
        *reinterpret_cast<u16x8*>(L + 2 * PL + o) = Lo;
      }
    } else {
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int id = t + NT * u;
        const int k = id >> 5, row = 4 * (id & 31);
        float x[4] = {v[u][0], v[u][1], v[u][2], v[u][3]};
        u16 h[4], m[4], l[4];
        split3<4>(x, h, m, l);
        const int o = km_off(k, row >> 3) + (row & 7);
        u16x4 H = {h[0], h[1], h[2], h[3]}, Mi = {m[0], m[1], m[2], m[3]}, Lo = {l[0], l[1], l[2], l[3]};
        *reinterpret_cast<u16x4*>(L + o) = H;
        *reinterpret_cast<u16x4*>(L + PL + o) = Mi;
        *reinterpret_cast<u16x4*>(L + 2 * PL + o) = Lo;
      }
    }
  }
};

// k-contiguous operand already split into bf16 planes in global memory ([3][rows][ld] u16, ld %
// 8 == 0): a plain copy into the LDS image, no VALU split. A thread owns one 8-k chunk per plane.
template <int ROWS, int NT = ::sdml::NT>
struct StagePre {
  static constexpr int NC = ROWS * 4 / NT;  // chunks per thread per plane
  u16x8 v[3][NC];

  __device__ __forceinline__ void load(const u16* __restrict__ P, int ld, int rows, int r0, int k0, int K) {
    const size_t plane = (size_t)rows * ld;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int id = threadIdx.x + NT * c;
      const int gr = min(r0 + (id >> 2), rows - 1);
      const int gk = min(k0 + 8 * (id & 3), K - 8);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) v[pl][c] = *reinterpret_cast<const u16x8*>(P + pl * plane + (size_t)gr * ld + gk);
    }
  }
  __device__ __forceinline__ void zero_tail(int k0, int kend) {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const bool ok = k0 + 8 * ((threadIdx.x + NT * c) & 3) < kend;  // K % 8 == 0: chunk all in or out
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) v[pl][c] = ok ? v[pl][c] : z;
    }
  }
  template <int PL>
  __device__ __forceinline__ void store(u16* L) const {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int id = threadIdx.x + NT * c;
      const int o = kc_off(id >> 2, id & 3);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u16x8*>(L + pl * PL + o) = v[pl][c];
    }
  }
};

// uint8 pixel operand -> one exact bf16 plane.
//   k-contiguous (ROWS x 32 bytes per K-step): a thread owns one 16-B chunk = 16 k of one row
//   (rows r0 + id/2, k0 + 16*(id&1)); host contract K % 16 == 0, ld % 16 == 0, 16-B aligned base.
//   k-major (32 k-rows x ROWS bytes): a thread owns 8 bytes = 8 rows at one k (k0 + id/16, rows
//   r0 + 8*(id&15)); host contract rows % 8 == 0, ld % 8 == 0, 8-B aligned base.
// Same clamped, branch-free loads as Stage; past-the-end k is zeroed by zero_tail.
template <bool KM, int ROWS, int NT = ::sdml::NT>
struct StageU8 {
  static constexpr int NC = KM ? (BK * ROWS / 8) / NT : (ROWS * 2) / NT;
  static_assert(NC >= 1, "tile too small for the thread count");

  // k-contiguous: row of the 16-k chunk pair owned by thread id (h = id & 1 picks the half).
  // ds_write_b128 banks 8 contiguous lanes over 32 banks (128 B): lanes 2j, 2j+1 of an 8-lane
  // group take rows base + {0, 1, 4, 5} (base = 8*(id>>4) + 2*((id>>3)&1)), so the two rows of
  // each parity have swizzles differing in bit 0 and the group's 8 chunks land in 8 distinct
  // 16-B bank slots (rows id>>1 put 2 rows of one parity on the same slots: 2-way conflicts,
  // 1.7M SQ_LDS_BANK_CONFLICT cycles per forward at the headline shape).
  __device__ __forceinline__ static int kc_row(int id) {
    const int rr = (id >> 1) & 3;
    return 8 * (id >> 4) + 2 * ((id >> 3) & 1) + (rr & 1) + 4 * (rr >> 1);
  }
  // native vectors: a ?: select on HIP's uint4/uint2 structs is lowered through scratch memory
  // (a scratch store + load and an s_waitcnt vmcnt(0) per K-step)
  typedef typename std::conditional<KM, u32x2, u32x4>::type V;
  V v[NC];

  __device__ __forceinline__ void load(const unsigned char* __restrict__ P, int ld, int rows, int r0, int k0, int K) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int id = threadIdx.x + NT * c;
      size_t o;
      if constexpr (!KM) {
        const int gr = min(r0 + kc_row(id), rows - 1);
        const int gk = min(k0 + 16 * (id & 1), K - 16);
        o = (size_t)gr * ld + gk;
      } else {
        const int gk = min(k0 + (id >> 4), K - 1);
        const int gr = min(r0 + 8 * (id & 15), rows - 8);
        o = (size_t)gk * ld + gr;
      }
      v[c] = *reinterpret_cast<const V*>(P + o);
    }
  }
  __device__ __forceinline__ void zero_tail(int k0, int kend) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int id = threadIdx.x + NT * c;
      const int gk = KM ? k0 + (id >> 4) : k0 + 16 * (id & 1);
      const V z = {};
      v[c] = gk < kend ? v[c] : z;
    }
  }
  __device__ __forceinline__ void accum_rowsum(float (&)[4]) const {}

  // bytes -> bf16 bit patterns: (float)b has its significant bits in the upper half
  __device__ __forceinline__ static u16x8 widen8(unsigned lo, unsigned hi) {
    u16x8 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[e] = (u16)(__float_as_uint((float)((lo >> (8 * e)) & 0xffu)) >> 16);
      r[4 + e] = (u16)(__float_as_uint((float)((hi >> (8 * e)) & 0xffu)) >> 16);
    }
    return r;
  }
  template <int PL>
  __device__ __forceinline__ void store(u16* L) const {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int id = threadIdx.x + NT * c;
      if constexpr (!KM) {
        const int r = kc_row(id), h = id & 1;
        *reinterpret_cast<u16x8*>(L + kc_off(r, 2 * h)) = widen8(v[c][0], v[c][1]);
        *reinterpret_cast<u16x8*>(L + kc_off(r, 2 * h + 1)) = widen8(v[c][2], v[c][3]);
      } else {
        const int k = id >> 4, row = 8 * (id & 15);
        *reinterpret_cast<u16x8*>(L + km_off(k, row >> 3)) = widen8(v[c][0], v[c][1]);
      }
    }
  }
};

// fp32 -> three bf16 planes (hi, mid, lo), 4 elements per thread (n % 4 == 0)
__global__ void __launch_bounds__(256) split3_planes_kernel(const float* __restrict__ x, u16* __restrict__ out,
                                                            int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
  float a[4] = {v[0], v[1], v[2], v[3]};
  u16 h[4], m[4], l[4];
  split3<4>(a, h, m, l);
  *reinterpret_cast<u16x4*>(out + i) = u16x4{h[0], h[1], h[2], h[3]};
  *reinterpret_cast<u16x4*>(out + n + i) = u16x4{m[0], m[1], m[2], m[3]};
  *reinterpret_cast<u16x4*>(out + 2 * n + i) = u16x4{l[0], l[1], l[2], l[3]};
}

// transposed split: w [R][Cc] fp32 -> planes [3][Cc][R] (the dX GEMM's B = W^T, k-contiguous, so
// the input gradient takes the same pre-split path as the forward). 64 x 64 tiles through LDS:
// coalesced float4 reads of w rows, coalesced u16 writes of the transposed plane rows.
__global__ void __launch_bounds__(256) split3_planes_t_kernel(const float* __restrict__ w, u16* __restrict__ out,
                                                              int R, int Cc) {
  __shared__ u16 t[3][64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 16; i += 256) {  // 64 rows x 16 float4
    const int rr = i / 16, c4 = (i % 16) * 4;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (r0 + rr < R && c0 + c4 + 3 < Cc) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(w + (size_t)(r0 + rr) * Cc + c0 + c4);
      a[0] = v[0];
      a[1] = v[1];
      a[2] = v[2];
      a[3] = v[3];
    } else {
      for (int e = 0; e < 4; ++e)
        if (r0 + rr < R && c0 + c4 + e < Cc) a[e] = w[(size_t)(r0 + rr) * Cc + c0 + c4 + e];
    }
    u16 h[4], m[4], l[4];
    split3<4>(a, h, m, l);
    for (int e = 0; e < 4; ++e) {
      t[0][c4 + e][rr] = h[e];
      t[1][c4 + e][rr] = m[e];
      t[2][c4 + e][rr] = l[e];
    }
  }
  __syncthreads();
  const size_t plane = (size_t)R * Cc;
  for (int i = threadIdx.x; i < 3 * 64 * 64; i += 256) {
    const int pl = i / 4096, cc = (i / 64) % 64, rr = i % 64;
    if (c0 + cc < Cc && r0 + rr < R) out[pl * plane + (size_t)(c0 + cc) * R + r0 + rr] = t[pl][cc][rr];
  }
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// FRESH: each K-step's 12 MFMAs accumulate into a zeroed partial tile that is then added to the
// fp32 accumulator with one round-to-nearest VALU add: the matrix core's internal accumulation
// then only ever sees a 32-deep partial sum (its rounding error scales with that magnitude, not
// with the running total's).
// EARLY: the split + LDS write of tile t+1 and the global loads of tile t+2 are issued in the
// same basic block as tile t's MFMAs (the scheduler interleaves the VALU/LDS work into the
// matrix-core shadow); otherwise they follow the MFMAs (tile t+1 loaded during tile t).
// BPRE: B arrives pre-split (p.Bp; k-contiguous B only)
// U8: U8_A = A is a k-contiguous uint8 matrix (p.X8), U8_B = B is a k-major uint8 matrix; that
// operand takes one LDS plane and each product 3 MFMAs; the epilogue scales by p.scale.
// DEEP (EARLY only): two tiles in flight in registers instead of one (LEAD = 2 K-steps of load
// latency cover instead of 1)
template <bool A_KM, bool B_KM, bool AMASK, bool EARLY, bool BPRE = false, int U8 = U8_NONE, bool DEEP = false,
          bool FRESH = true, bool NOEPI = false>
__global__ void __launch_bounds__(NT) gemm_x3_kernel(X3Params p) {
  constexpr int BM = A_KM ? 128 : 256;
  constexpr int WGM = BM / 64, WGN = 8 / WGM;  // wave grid
  constexpr int TN = BN / WGN / 32;             // 32-col MFMA tiles per wave (TM = 2)
  constexpr int AP = BM * BK, BP = BN * BK;     // u16 per plane
  constexpr int NPA = U8 == U8_A ? 1 : 3, NPB = U8 == U8_B ? 1 : 3;  // bf16 planes per operand
  static_assert(U8 != U8_A || (!A_KM && !AMASK), "uint8 A: k-contiguous, unmasked");
  static_assert(U8 != U8_B || (B_KM && !BPRE), "uint8 B: k-major");
  constexpr int BUF = NPA * AP + NPB * BP;
  __shared__ __attribute__((aligned(16))) u16 smem[2 * BUF];

  // XCD-aware bijective remap over tiles x splits (blocks b, b+8 share an XCD): each XCD gets a
  // contiguous run of logical ids; logical id = split * ntiles + tile, so the tiles that stream
  // the same K-slice of the shared operand read it through one L2.
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nwg = ntiles * gridDim.y;
  const int orig = blockIdx.y * gridDim.x + blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WGM, wn = wave / WGM;
  const int h = lane >> 5;

  f32x16 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x16 part[2][TN];  // FRESH: the K-step's partial tile
  const bool do_rowsum = p.rowsum != nullptr && tn == 0;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};

  typedef typename std::conditional<U8 == U8_A, StageU8<false, BM>, Stage<A_KM, BM>>::type SA;
  typedef typename std::conditional<BPRE, StagePre<BN>,
                                    typename std::conditional<U8 == U8_B, StageU8<true, BN>, Stage<B_KM, BN>>::type>::type SB;
  SA sa, sa2;  // register stages (sa2: second in-flight tile of the DEEP pipeline)
  SB sb, sb2;
  auto load = [&](SA& ra, SB& rb, int k0) {
    if constexpr (U8 == U8_A) ra.load(p.X8, p.lda, p.M, m0, k0, p.K);
    else ra.template load<AMASK>(p.A, p.amask, p.lda, p.M, m0, k0, p.K);
    if constexpr (BPRE) rb.load(p.Bp, p.ldb, p.N, n0, k0, p.K);
    else if constexpr (U8 == U8_B) rb.load(p.X8, p.ldb, p.N, n0, k0, p.K);
    else rb.template load<false>(p.B, nullptr, p.ldb, p.N, n0, k0, p.K);
  };
  // tile staged for k0 -> K-tail zeroing -> bias-grad row sums -> split -> LDS buffer `buf`
  auto store = [&](SA& ra, SB& rb, int buf, int k0) {
    ra.zero_tail(k0, kend);
    rb.zero_tail(k0, kend);
    ra.accum_rowsum(rs);
    u16* L = smem + buf * BUF;
    ra.template store<AP>(L);
    rb.template store<BP>(L + NPA * AP);
  };

  // one K-step on LDS buffer t & 1. EARLY: (ra, rb) hold tile t+1 (loaded LEAD K-steps ago); it is
  // split into the other buffer, whose last readers passed the previous barrier, and tile
  // t+1+LEAD is loaded in its place. Past the end both are harmless: zero tiles written to a
  // buffer nobody reads again.
  constexpr int LEAD = DEEP ? 2 : 1;
  const int nk = (kend - kbeg + BK - 1) / BK;
  auto kstep = [&](int t, SA& ra, SB& rb) {
    const int cur = t & 1;
    const u16* As = smem + cur * BUF;
    const u16* Bs = As + NPA * AP;
    if constexpr (!EARLY) {
      if (t + 1 < nk) load(ra, rb, kbeg + (t + 1) * BK);  // next tile -> registers (latency under the MFMAs)
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 a[2][NPA], b[TN][NPB];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) a[i][pl] = frag<A_KM>(As + pl * AP, wm * 64 + i * 32, s, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int pl = 0; pl < NPB; ++pl) b[j][pl] = frag<B_KM>(Bs + pl * BP, wn * (32 * TN) + j * 32, s, lane);
      if constexpr (EARLY) {
        if (s == 0) {
          store(ra, rb, cur ^ 1, kbeg + (t + 1) * BK);
          load(ra, rb, kbeg + (t + 1 + LEAD) * BK);
        }
      }
      // small terms first, the leading hi*hi term last
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x16 c = (FRESH && s == 0) ? f32x16{} : (FRESH ? part[i][j] : acc[i][j]);
          if constexpr (U8 == U8_A) {  // exact A: a*b = a*(hi + mid + lo)
            c = mfma(a[i][0], b[j][NPB - 1], c);
            c = mfma(a[i][0], b[j][NPB > 1 ? 1 : 0], c);
            c = mfma(a[i][0], b[j][0], c);
          } else if constexpr (U8 == U8_B) {
            c = mfma(a[i][NPA - 1], b[j][0], c);
            c = mfma(a[i][NPA > 1 ? 1 : 0], b[j][0], c);
            c = mfma(a[i][0], b[j][0], c);
          } else {
            c = mfma(a[i][1], b[j][1], c);  // mid*mid
            c = mfma(a[i][2], b[j][0], c);  // lo*hi
            c = mfma(a[i][0], b[j][2], c);  // hi*lo
            c = mfma(a[i][1], b[j][0], c);  // mid*hi
            c = mfma(a[i][0], b[j][1], c);  // hi*mid
            c = mfma(a[i][0], b[j][0], c);  // hi*hi
          }
          if constexpr (FRESH) {
            if (s == BK / 16 - 1) acc[i][j] += c;
            else part[i][j] = c;
          } else {
            acc[i][j] = c;
          }
        }
    }
    if constexpr (!EARLY) {
      if (t + 1 < nk) store(ra, rb, cur ^ 1, kbeg + (t + 1) * BK);
    }
    __syncthreads();
  };

  if (nk > 0) {
    load(sa, sb, kbeg);
    store(sa, sb, 0, kbeg);
    if constexpr (DEEP) {
      load(sa2, sb2, kbeg + BK);  // tiles 1 and 2 in flight (zeroed at split time past kend)
      load(sa, sb, kbeg + 2 * BK);
    } else if constexpr (EARLY) {
      load(sa, sb, kbeg + BK);
    }
  }
  __syncthreads();
  if constexpr (DEEP) {
    // two register stages alternate: K-step t splits the stage holding tile t+1
    for (int t = 0; t < nk; t += 2) {
      kstep(t, sa2, sb2);
      if (t + 1 < nk) kstep(t + 1, sa, sb);
    }
  } else {
    for (int t = 0; t < nk; ++t) kstep(t, sa, sb);
  }
  // EARLY staged LEAD tiles past the end: zeroed, row sums unaffected

  if (do_rowsum) {
    if constexpr (!A_KM) {
      // thread's chunks: rows (t + NT*c) >> 2; the 4 threads of a row are adjacent lanes
#pragma unroll
      for (int c = 0; c < Stage<A_KM, BM>::NV / 2; ++c) {
        float v = rs[c];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        const int row = m0 + ((threadIdx.x + NT * c) >> 2);
        if ((lane & 3) == 0 && row < p.M) atomicAdd(p.rowsum + row, v);
      }
    } else {
      // rows m0 + 4*(t & 31) + e: lanes l and l^32 share them
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = rs[e] + __shfl_xor(rs[e], 32);
        const int row = m0 + 4 * (threadIdx.x & 31) + e;
        if (lane < 32 && row < p.M) atomicAdd(p.rowsum + row, v);
      }
    }
  }

  // ---- epilogue ----
  if constexpr (NOEPI) {  // timing experiments only: keep the accumulators live, store nothing
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) z += acc[i][j][0] + acc[i][j][15];
    if (z == 1234.5f) p.C[0] = z;
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
      if (col >= p.N) continue;
      const float bv = (p.epi == EPI_BIAS || p.epi == EPI_BIAS_RELU) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        const float v = U8 != U8_NONE ? acc[i][j][r] * p.scale : acc[i][j][r];
        if (p.slab) {
          p.slab[split * p.slab_stride + (size_t)row * p.ldc + col] = v;
          continue;
        }
        float* dst = p.C + (size_t)row * p.ldc + col;
        switch (p.epi) {
          case EPI_STORE:
            *dst = (p.cmask && p.cmask[(size_t)row * p.ldc + col] <= 0.f) ? 0.f : v;
            break;
          case EPI_BIAS: *dst = v + bv; break;
          case EPI_BIAS_RELU: *dst = fmaxf(v + bv, 0.f); break;
          case EPI_ACCUM: *dst += v; break;
          default: atomicAdd(dst, v); break;
        }
      }
    }
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

// operand staging needs whole, aligned float4s: a k-contiguous operand K % 4 == 0, a k-major
// one rows % 4 == 0, and ld % 4 == 0 with 16-B aligned bases (masks laid out like the operand)
bool operand_ok(const float* P, const float* mask, int ld, bool kmajor, int rows, int K) {
  if (!P || !al16(P) || (mask && !al16(mask)) || ld % 4) return false;
  return kmajor ? rows % 4 == 0 : K % 4 == 0;
}

}  // namespace

static int g_x3_variant = 0;  // pipeline A/B: 0 = EARLY split (default), 1 = split after the MFMAs

// DEEP register pipeline (two tiles in flight) for the uint8 kernels. Measured at 131072 x 784 -> 128
// (tools/bench_u8.py, profiles/r1_u8_gemm_ab.txt): forward 114 us 1-deep vs 111 us DEEP; weight
// gradient 161 us 1-deep (167 us with 2 workgroups/CU) vs 154 us DEEP. SDML_X3_DEEP=0/1 forces one
// for both (A/B).
static bool x3_deep(bool dflt) {
  const int force = knob(KNOB_X3_DEEP);
  return force < 0 ? dflt : force == 1;
}

// experiment selector for the uint8 kernels (SDML_U8_VARIANT). Forward (engine path, SDML_U8_FWD=x3):
// 1 = no FRESH partials, 2 = no epilogue (timing only), 3 = both. Weight gradient: 1 = FRESH partials.
static int u8_variant() {
  return knob(KNOB_U8_VARIANT);  // timing variants: pinned to 0 in production builds
}

bool gemm_f32x3_eligible(const GemmArgs& g) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return false;
  if (g.epi == EPI_ATOMIC ? false : g.splits > 1) return false;
  return operand_ok(g.A, g.amask, g.lda, g.a_kmajor, g.M, g.K) && operand_ok(g.B, nullptr, g.ldb, g.b_kmajor, g.N, g.K);
}

int gemm_f32x3_pick_splits(int M, int N, int K, bool a_kmajor) {
  const int bm = a_kmajor ? 128 : 256;
  const int tiles = ((M + bm - 1) / bm) * ((N + BN - 1) / BN);
  // one 512-thread workgroup per CU (LDS): aim at one full wave of 256 workgroups, with at
  // least 16 K-steps per split (each split adds a whole C tile with fp32 atomics)
  int splits = 256 / tiles;
  const int max_by_k = K / (16 * BK);
  if (splits > max_by_k) splits = max_by_k;
  return splits < 1 ? 1 : splits;
}

void gemm_f32x3(const GemmArgs& g, hipStream_t stream) {
  X3Params p{};
  p.A = g.A;
  p.amask = g.amask;
  p.B = g.B;
  p.C = g.C;
  p.bias = g.bias;
  p.rowsum = g.rowsum;
  p.cmask = g.cmask;
  p.M = g.M;
  p.N = g.N;
  p.K = g.K;
  p.lda = g.lda;
  p.ldb = g.ldb;
  p.ldc = g.ldc;
  p.epi = g.epi;
  p.X8 = nullptr;
  p.scale = 1.f;
  const int bm = g.a_kmajor ? 128 : 256;
  // atomic epilogues are split-invariant: pick the split count for THIS kernel's geometry
  int splits = g.epi == EPI_ATOMIC ? gemm_f32x3_pick_splits(g.M, g.N, g.K, g.a_kmajor) : 1;
  int kps = (g.K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (g.K + kps - 1) / kps;
  p.kps = kps;
  p.tiles_m = (g.M + bm - 1) / bm;
  p.tiles_n = (g.N + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n, splits, 1);
  dim3 block(NT);
#define X3_LAUNCH(AM, E)                                                                      \
  if (!g.a_kmajor && !g.b_kmajor)                                                             \
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, AM, E>), grid, block, 0, stream, p);     \
  else if (!g.a_kmajor && g.b_kmajor)                                                         \
    hipLaunchKernelGGL((gemm_x3_kernel<false, true, AM, E>), grid, block, 0, stream, p);      \
  else if (g.a_kmajor && !g.b_kmajor)                                                         \
    hipLaunchKernelGGL((gemm_x3_kernel<true, false, AM, E>), grid, block, 0, stream, p);      \
  else                                                                                        \
    hipLaunchKernelGGL((gemm_x3_kernel<true, true, AM, E>), grid, block, 0, stream, p);
  p.Bp = reinterpret_cast<const u16*>(g.b_split);
  const bool early = g_x3_variant != 1;
  if (p.Bp) {  // the forward of a Linear layer: W pre-split once per call (split3_planes)
    if (g.a_kmajor || g.b_kmajor || g.ldb % 8 || g.K % 8) abort();  // host contract, checked by callers
    if (g.amask) hipLaunchKernelGGL((gemm_x3_kernel<false, false, true, true, true>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true>), grid, block, 0, stream, p);
    return;
  }
  if (g.amask) {
    if (early) {
      X3_LAUNCH(true, true)
    } else {
      X3_LAUNCH(true, false)
    }
  } else {
    if (early) {
      X3_LAUNCH(false, true)
    } else {
      X3_LAUNCH(false, false)
    }
  }
#undef X3_LAUNCH
}

void gemm_f32x3_set_variant(int v) { g_x3_variant = v; }

void split3_planes(const float* x, unsigned short* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t blocks = (n / 4 + 255) / 256;
  hipLaunchKernelGGL(split3_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, out, n);
}

void split3_planes_t(const float* w, unsigned short* out, int R, int C, hipStream_t stream) {
  if (R <= 0 || C <= 0) return;
  hipLaunchKernelGGL(split3_planes_t_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, stream, w, out, R, C);
}

bool gemm_f32x3_can_presplit_b(const GemmArgs& g) {
  return !g.a_kmajor && !g.b_kmajor && g.ldb % 8 == 0 && g.K % 8 == 0 && (size_t)g.N * g.ldb % 4 == 0;
}

// ---- uint8 pixel GEMMs (first layer fed straight from MNIST bytes) ----------------------------
void gemm_u8x3_fwd(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_split, int N,
                   const float* bias, float* C, int ldc, bool relu, float scale, hipStream_t stream) {
  X3Params p{};
  p.X8 = X;
  p.Bp = w_split;
  p.C = C;
  p.bias = bias;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = ldx;
  p.ldb = K;
  p.ldc = ldc;
  p.epi = bias ? (relu ? EPI_BIAS_RELU : EPI_BIAS) : EPI_STORE;
  p.scale = scale;
  p.kps = (K + BK - 1) / BK * BK;
  p.tiles_m = (M + 255) / 256;
  p.tiles_n = (N + BN - 1) / BN;
  const dim3 grid(p.tiles_m * p.tiles_n, 1, 1);
  const int v = u8_variant();
  if (v == 1)
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true, U8_A, true, false>), grid, dim3(NT), 0, stream, p);
  else if (v == 2)
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true, U8_A, true, true, true>), grid, dim3(NT), 0, stream, p);
  else if (v == 3)
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true, U8_A, true, false, true>), grid, dim3(NT), 0, stream, p);
  else if (x3_deep(true))
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true, U8_A, true>), grid, dim3(NT), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_x3_kernel<false, false, false, true, true, U8_A>), grid, dim3(NT), 0, stream, p);
}

// deterministic split-K reduction: out[i] += sum_s slab[s][i] in a fixed order (n % 4 == 0). A block
// owns 256 outputs (64 float4 lanes) and its 4 waves take every 4th split (n = 100K floats is only
// ~390 float4 lane groups: one wave each left the memory system underfed, 13.6 us for 51 MB at the
// headline shape), each lane with 4 independent partial sums and 8 loads in flight; the wave
// partials meet in LDS in wave order.
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, int64_t stride, int splits,
                                                          float* __restrict__ out, int64_t n) {
  __shared__ f32x4 part[4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t i = ((int64_t)blockIdx.x * 64 + l) * 4;
  f32x4 a[4] = {};
  if (i < n) {
    int s = w;  // wave w: splits w, w + 4, ...
    for (; s + 4 * 7 < splits; s += 4 * 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u & 3] += *reinterpret_cast<const f32x4*>(slab + (int64_t)(s + 4 * u) * stride + i);
    }
    for (; s < splits; s += 4) a[0] += *reinterpret_cast<const f32x4*>(slab + (int64_t)s * stride + i);
  }
  part[w][l] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w == 0 && i < n) {
    f32x4 acc = *reinterpret_cast<const f32x4*>(out + i);
    acc += (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
    *reinterpret_cast<f32x4*>(out + i) = acc;
  }
}

void slab_reduce(const float* slab, int64_t stride, int splits, float* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((n / 4 + 63) / 64)), dim3(256), 0, stream, slab, stride, splits,
                     out, n);
}

int u8x3_wgrad_splits(int M, int N, int K) {
  int splits = gemm_f32x3_pick_splits(N, K, M, true);
  int kps = (M + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  return (M + kps - 1) / kps;
}

// gw[N,K] += scale * sum_m gz[m,n] X[m,k]; gb[n] += sum_m gz[m,n] (gb optional).
// Split-K partial tiles go to `slab` ([splits][N][K] fp32, u8x3_wgrad_splits(M, N, K) splits) with
// plain stores and are summed in split order by slab_reduce_kernel: deterministic, and cheaper than
// fp32 atomics (measured: the atomic epilogue cost ~14 us of 153 at the headline shape). With
// slab == nullptr the partials are added atomically. Straight MFMA accumulation (no per-K-step
// fp32 partials: tools/probes/mfma_acc_probe.hip) - measured 153 -> 142 us.
void gemm_u8x3_wgrad(const float* gz, const unsigned char* X, int M, int N, int K, int ldx, float* gw, float* gb,
                     float scale, float* slab, hipStream_t stream) {
  X3Params p{};
  p.A = gz;
  p.X8 = X;
  p.C = gw;
  p.rowsum = gb;
  p.M = N;
  p.N = K;
  p.K = M;
  p.lda = N;
  p.ldb = ldx;
  p.ldc = K;
  p.epi = EPI_ATOMIC;
  p.scale = scale;
  p.slab = slab;
  p.slab_stride = (int64_t)N * K;
  const int splits = u8x3_wgrad_splits(M, N, K);
  int kps = (M + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  p.kps = kps;
  p.tiles_m = (N + 127) / 128;
  p.tiles_n = (K + BN - 1) / BN;
  const dim3 grid(p.tiles_m * p.tiles_n, (M + kps - 1) / kps, 1);
  const int v = u8_variant();
  if (v == 1)  // A/B: per-K-step fp32 partials (FRESH), as in round 1
    hipLaunchKernelGGL((gemm_x3_kernel<true, true, false, true, false, U8_B, true, true>), grid, dim3(NT), 0, stream, p);
  else
    hipLaunchKernelGGL((gemm_x3_kernel<true, true, false, true, false, U8_B, true, false>), grid, dim3(NT), 0, stream, p);
  if (slab) {
    slab_reduce(slab, p.slab_stride, (int)grid.y, gw, (int64_t)N * K, stream);
  }
}

}  // namespace sdml
