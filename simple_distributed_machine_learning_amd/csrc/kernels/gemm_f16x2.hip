// fp32-accurate GEMMs of the 4x1024 MLP's hidden layers (BASELINE config 3) on the fp16 matrix cores,
// from operands PRE-SPLIT into two fp16 planes (round 3; the bf16x3 engine in gemm_f32x3.hip splits both
// operands into three bf16 planes inside its K loop and pays 6 MFMAs per product).
//
// Numerics. An fp32 tensor X is stored as two fp16 planes of X * 2^s: hi = fp16(X 2^s), lo = fp16(X 2^s -
// hi) (the difference is exact in fp32), with 2^s chosen from a bound |X| < 2^E as 2^(14 - E): every
// element fits fp16's range, and hi + lo carries 22 significant bits (|hi + lo - X 2^s| <= 2^-23 |X 2^s|)
// for |X| >= 2^(E - 17); smaller elements keep an absolute error below 2^(E - 39). A product is then
//   a b ~= (ah + al)(bh + bl) ~= ah bh + ah bl + al bh      (al bl <= 2^-22 |a b| is dropped),
// three exact fp16 x fp16 MFMA products accumulated in fp32: half the MFMAs of the bf16x3 split, and no
// split work in the GEMM at all. The three products are ONE fp16 GEMM over a K axis three times as long,
//   A' = [Ah | Ah | Al],  B' = [Bh ; Bl ; Bh],
// so the kernels below are plain LDS-DMA fp16 GEMMs whose K-step t reads plane pair (t / nk) of
// {(h, h), (h, l), (l, h)}; the epilogue multiplies by 2^-(sA + sB).
// Reference numerics: the reference's fp32 nn.Linear on the CPU (/root/reference/simple_distributed.py:63-64,
// :75-77); tests/test_gemm_x2_gpu.py compares against fp64 within the fp32 GEMM error bound.
//
// Kernels:
//   x2_split_kernel   fp32 [M][K] -> planes [2][M][K] (K % 8 == 0), scale from a bound (a max over `namax` floats:
//                     a torch inf-norm, the producing GEMM's per-wave maxima or the head's per-block bounds)
//   x2_gemm_kernel    C[M][N] = A'[M][K'] . op(B') : BL = 0 "NT" (B [N][K], forward), BL = 1 "NN" (B [K][N],
//                     input gradient); 256 x 256 tile, 8 waves of 128 x 64 (v_mfma_f32_16x16x32_f16),
//                     K-step 64 by LDS-DMA into 2 x 64 KiB stages (gemm_bf16.hip's 2-phase loop and swizzles);
//                     fp32 epilogue through LDS (16-B row stores): bias, ReLU, ReLU mask of the layer input,
//                     per-wave max |C| for the consumer's split
//   x2_wgrad_kernel   gW[N][K] += sum_m dz[m][n] x[m][k] (both operands k-major, hardware transpose reads),
//                     the 3 plane pairs as 3 token segments of one extended K axis, cut into equal splits over
//                     workgroups (one grid wave), fp32 slabs reduced in a fixed order (deterministic) with the
//                     bias gradient (column sums of dz: hi in segment 0, lo in segment 2). Two main loops:
//                     x2_wgrad_dma_kernel (T % 64 == 0, default) fills a 3-stage LDS ring by LDS-DMA with two
//                     K-steps in flight (gemm_bf16_wgrad.hip's wgrad_dma_kernel); x2_wgrad_kernel stages
//                     through VGPRs (any T; SDML_WGRAD_DMA=0). 588 -> 502 us at 65536 x 1024 x 1024
//                     (profiles/r3_wgrad_dma_vs_staged.json)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "kernels.h"
#include "tile_order.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

// exponent E with |v| < 2^E for finite v >= 0, clamped so 2^(14 - E) and 2^(E - 14) stay normal floats
__device__ __forceinline__ int bound_exp(float v) {
  const unsigned b = __float_as_uint(v);
  const int e = (int)((b >> 23) & 0xffu) - 126;
  return (b & 0x7fffffffu) == 0u ? -100 : min(max(e, -100), 120);
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }

// ================================================================================================
// split: planes [2][rows][ld] of X * 2^(14 - E); scale_out = 2^(E - 14) (the dequantisation factor)
__global__ void __launch_bounds__(256) x2_split_kernel(const float* __restrict__ X, int rows, int cols, int ldx,
                                                       const float* __restrict__ amax, int namax, u16* __restrict__ P,
                                                       int64_t ps, int ldp, float* __restrict__ scale_out) {
  __shared__ float red[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < namax; i += 256) m = fmaxf(m, fabsf(amax[i]));
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int E = bound_exp(m);
  const float up = pow2f(14 - E);
  if (blockIdx.x == 0 && threadIdx.x == 0) *scale_out = pow2f(E - 14);
  // 8 consecutive columns per thread (cols % 8 == 0): two 16-B loads, one 16-B store per plane
  const unsigned c8 = (unsigned)cols / 8u;
  const unsigned n8 = (unsigned)rows * c8;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n8; i += gridDim.x * 256u) {
    const unsigned r = i / c8, c = 8u * (i - r * c8);
    const float* src = X + (int64_t)r * ldx + c;
    const f32x4 v0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src));
    const f32x4 v1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(src) + 1);
    u16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = (e < 4 ? v0[e] : v1[e - 4]) * up;  // exact (power of two)
      const _Float16 h = static_cast<_Float16>(x);
      hi[e] = __builtin_bit_cast(u16, h);
      lo[e] = __builtin_bit_cast(u16, static_cast<_Float16>(x - static_cast<float>(h)));
    }
    *reinterpret_cast<u16x8*>(P + (int64_t)r * ldp + c) = hi;
    *reinterpret_cast<u16x8*>(P + ps + (int64_t)r * ldp + c) = lo;
  }
}

// ================================================================================================
// GEMM
constexpr int GT = 512, TM = 256, TN = 256, TK = 64;
constexpr int A_BYTES = TM * TK * 2;     // 32 KiB
constexpr int STAGE = 2 * A_BYTES;       // A + B
constexpr int SMEM = 2 * STAGE;          // 128 KiB
constexpr int GLDS = STAGE / 1024 / 8;   // DMA instructions per wave per stage (8)

enum : int { X2_RELU = 1, X2_MASK = 2 };

struct X2Gemm {
  const u16* A;  // plane 0 (hi) [M][lda]; plane 1 (lo) at A + a_ps
  const u16* B;  // NT: [N][ldb]; NN: [K][ldb]; plane 1 at B + b_ps
  int64_t a_ps, b_ps;
  float* C;
  const float* bias;  // [N] or nullptr
  const float* mask;  // X2_MASK: [M][ldm], C element kept where mask > 0
  const float* sa;    // dequantisation factors 2^(E - 14) of A and B (device scalars, x2_split)
  const float* sb;
  float* wmax;        // optional [grid][8]: per-wave max |C| (after the epilogue ops)
  int M, N, K, lda, ldb, ldc, ldm;
  int tiles_m, tiles_n;
  int ntstore;  // SDML_GEMM_NT_STORE=1: nontemporal epilogue stores (A/B)
  int group_m;  // tile order (tile_order.h): 0 = M fastest; g > 0 = groups of g m-tiles x every n-tile
};

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

__device__ __forceinline__ int rk_swz(int r) { return (r >> 1) & 7; }                          // [rows][64]
__device__ __forceinline__ int kn_swz(int r) { return ((r & 3) | ((r >> 1) & 4)) << 1; }       // [64][256]

// K-step t of the extended K axis: plane pair (t / nk) of {(hi, hi), (hi, lo), (lo, hi)}, k0 in the segment
template <int BL>
__device__ __forceinline__ void issue_stage(const X2Gemm& p, unsigned char* st, int m0, int n0, int t, int nk,
                                            int wave, int lane) {
  const int seg = t / nk, k0 = (t - seg * nk) * TK;
  const u16* A = p.A + (seg == 2 ? p.a_ps : 0);
  const u16* B = p.B + (seg == 1 ? p.b_ps : 0);
#pragma unroll
  for (int u = 0; u < GLDS / 2; ++u) {  // A: 32 instructions of 8 rows x 128 B
    const int q = wave + 8 * u;
    const int r = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ rk_swz(r);
    const int gr = min(m0 + r, p.M - 1);
    glds16(A + (size_t)gr * p.lda + k0 + 8 * c, st + 1024 * q);
  }
#pragma unroll
  for (int u = 0; u < GLDS / 2; ++u) {
    const int q = wave + 8 * u;
    if constexpr (BL == 0) {  // B [N][K]: like A
      const int r = 8 * q + (lane >> 3);
      const int c = (lane & 7) ^ rk_swz(r);
      const int gr = min(n0 + r, p.N - 1);
      glds16(B + (size_t)gr * p.ldb + k0 + 8 * c, st + A_BYTES + 1024 * q);
    } else {  // B [K][N]: 2 k-rows x 512 B
      const int r = 2 * q + (lane >> 5);
      const int c = (lane & 31) ^ kn_swz(r);
      const int gc = min(n0 + 8 * c, p.N - 8);
      glds16(B + (size_t)(k0 + r) * p.ldb + gc, st + A_BYTES + 1024 * q);
    }
  }
}

__device__ __forceinline__ f16x8 ld_b128(const unsigned char* p) { return *reinterpret_cast<const f16x8*>(p); }
__device__ __forceinline__ s16x4 ds_tr16(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// fp32 epilogue: each wave's 128 x 64 tile in two 64-row halves through a wave-private [64][64] fp32 LDS
// image (16-B chunk c of row r at c ^ (((r >> 2) & 3) << 2): conflict-free writes from the MFMA layout
// and conflict-free 16-B row reads), then every lane moves whole 16-B row pieces
template <int EPI>
__device__ __forceinline__ void x2_epilogue(const X2Gemm& p, const f32x4 (&acc)[8][4], unsigned char* smem, int m0,
                                            int n0, int wave, int lane) {
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l16 = lane & 15;
  float* W = reinterpret_cast<float*>(smem) + wave * (64 * 64);
  const float sc = *p.sa * *p.sb;
  const int ch = lane & 15;
  const int gcol = n0 + wn * 64 + 4 * ch;
  f32x4 bv = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && gcol < p.N) bv = *reinterpret_cast<const f32x4*>(p.bias + gcol);
  float vmax = 0.f;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (hh) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // half 0's reads done before the overwrite
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * g + r, col = 16 * j + l16;
          W[row * 64 + 4 * ((col >> 2) ^ (((row >> 2) & 3) << 2)) + (col & 3)] = acc[4 * hh + i][j][r];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int rr = 4 * it + (lane >> 4);
      f32x4 v = *reinterpret_cast<const f32x4*>(W + rr * 64 + 4 * (ch ^ (((rr >> 2) & 3) << 2)));
      const int grow = m0 + wm * 128 + 64 * hh + rr;
      if (grow >= p.M || gcol >= p.N) continue;  // (N % 4 == 0: a chunk is all in or all out)
      v = v * sc + bv;
      if constexpr (EPI & X2_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (EPI & X2_MASK) {
        const f32x4 mk = *reinterpret_cast<const f32x4*>(p.mask + (size_t)grow * p.ldm + gcol);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) vmax = fmaxf(vmax, fabsf(v[e]));
      f32x4* cp = reinterpret_cast<f32x4*>(p.C + (size_t)grow * p.ldc + gcol);
      if (p.ntstore) __builtin_nontemporal_store(v, cp);
      else *cp = v;
    }
  }
  if (p.wmax) {
    for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off));
    if (lane == 0) p.wmax[(size_t)blockIdx.x * 8 + wave] = vmax;
  }
}

template <int BL, int EPI>
__global__ void __launch_bounds__(GT) x2_gemm_kernel(X2Gemm p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  const int nwg = p.tiles_m * p.tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 16) {  // XCD-aware bijective remap: blocks sharing an XCD get consecutive tile ids
    const int q = nwg / 8, r = nwg % 8, xcd = wg % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wg / 8;
  }
  int tm, tn;
  tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, l16 = lane & 15;
  int aoff[2][8];  // [substep][m-tile]: A row wm*128 + 16 i + l16, chunk 4 s + g
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wm * 128 + 16 * i + l16;
      aoff[s][i] = r * 128 + 16 * ((4 * s + g) ^ rk_swz(r));
    }
  int boff[2][4][2];  // NT: [s][j][0]; NN: the two transposed reads
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (BL == 0) {
        const int r = wn * 64 + 16 * j + l16;
        boff[s][j][0] = A_BYTES + r * 128 + 16 * ((4 * s + g) ^ rk_swz(r));
        boff[s][j][1] = 0;
      } else {
        const int q = l16 >> 2, pp = l16 & 3;
        const int n = wn * 64 + 16 * j + 4 * pp;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int r = 32 * s + 8 * g + 4 * h + q;
          boff[s][j][h] = A_BYTES + r * 512 + 16 * ((n >> 3) ^ kn_swz(r)) + 2 * (n & 7);
        }
      }
    }

  const int nkseg = p.K / TK, nk = 3 * nkseg;
  issue_stage<BL>(p, smem, m0, n0, 0, nkseg, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const unsigned char* st = smem + (t & 1) * STAGE;
    if (t + 1 < nk) issue_stage<BL>(p, smem + ((t + 1) & 1) * STAGE, m0, n0, t + 1, nkseg, wave, lane);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f16x8 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (BL == 0) {
          b[j] = ld_b128(st + boff[s][j][0]);
        } else {
          const s16x4 lo = ds_tr16(st + boff[s][j][0]), hi = ds_tr16(st + boff[s][j][1]);
          b[j] = __builtin_bit_cast(f16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const f16x8 a = ld_b128(st + aoff[s][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[j], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  x2_epilogue<EPI>(p, acc, smem, m0, n0, wave, lane);
}

// ---- NT form, 4-phase K-step schedule (gemm_bf16.hip's gemm_bf16_nt4_kernel with plane pairs) -----------
// Each 64-deep K-step runs as 4 phases, one per 64 x 32 quadrant of every wave's 128 x 64 output (16 MFMAs
// at raised priority); the LDS-DMA prefetch is cut into half-tiles of 128 rows x 64 k (16 KiB) streamed one
// per phase, 3 in flight behind a counted vmcnt(6); the two wave rows run one barrier apart. Half-tile q of
// K-step u (h = 4u + q) lives in slot h % 10 (10 x 16 KiB = all 160 KiB): q 0 / 3 = A rows of quadrant-row
// 0 / 1, q 1 / 2 = B rows of quadrant-col 0 / 1. RAW/WAR reasoning: gemm_bf16.hip.
constexpr int HT = 16384, NSLOT = 10;

template <int Q>
__device__ __forceinline__ void issue_half(const X2Gemm& p, unsigned char* smem, int h, int nk, int nkseg, int m0,
                                           int n0, int wave, int lane) {
  const int t = min(h >> 2, nk - 1);
  const int seg = t / nkseg, k0 = (t - seg * nkseg) * TK;
  unsigned char* slot = smem + (h % NSLOT) * HT;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int qq = wave + 8 * v;          // 1-KiB DMA block of the slot
    const int lr = 8 * qq + (lane >> 3);  // slot row 0..127
    const int c = (lane & 7) ^ rk_swz(lr);
    if constexpr (Q == 0 || Q == 3) {
      const int tr = (lr >> 6) * 128 + (Q == 3 ? 64 : 0) + (lr & 63);
      const u16* A = p.A + (seg == 2 ? p.a_ps : 0);
      glds16(A + (size_t)min(m0 + tr, p.M - 1) * p.lda + k0 + 8 * c, slot + 1024 * qq);
    } else {
      const int tr = (lr >> 5) * 64 + (Q == 2 ? 32 : 0) + (lr & 31);
      const u16* B = p.B + (seg == 1 ? p.b_ps : 0);
      glds16(B + (size_t)min(n0 + tr, p.N - 1) * p.ldb + k0 + 8 * c, slot + 1024 * qq);
    }
  }
}

template <int EPI>
__global__ void __launch_bounds__(GT) x2_gemm_nt4_kernel(X2Gemm p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[NSLOT * HT];  // the epilogue reuses it
  const int nwg = p.tiles_m * p.tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = wg % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wg / 8;
  }
  int tm, tn;
  tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l16 = lane & 15;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r = wm * 64 + 16 * i + l16;
      aoff[i][s2] = r * 128 + 16 * ((4 * s2 + g) ^ rk_swz(r));
    }
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r = wn * 32 + 16 * jj + l16;
      boff[jj][s2] = r * 128 + 16 * ((4 * s2 + g) ^ rk_swz(r));
    }

  const int nkseg = p.K / TK, nk = 3 * nkseg;
  issue_half<0>(p, smem, 0, nk, nkseg, m0, n0, wave, lane);
  issue_half<1>(p, smem, 1, nk, nkseg, m0, n0, wave, lane);
  issue_half<2>(p, smem, 2, nk, nkseg, m0, n0, wave, lane);
  issue_half<3>(p, smem, 3, nk, nkseg, m0, n0, wave, lane);
  issue_half<0>(p, smem, 4, nk, nkseg, m0, n0, wave, lane);
  issue_half<1>(p, smem, 5, nk, nkseg, m0, n0, wave, lane);
  issue_half<2>(p, smem, 6, nk, nkseg, m0, n0, wave, lane);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K-step 0's 4 half-tiles
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // wave row 1 runs one barrier behind row 0

  f16x8 a[4][2], b0[2][2], b1[2][2];
  auto mfma_quadrant = [&](int qm, const f16x8 (&bb)[2][2], int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[4 * qm + i][2 * qn + jj] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][s2], bb[jj][s2], acc[4 * qm + i][2 * qn + jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_mid = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto sync_end = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  for (int t = 0; t < nk; ++t) {
    const int h = 4 * t + 7;
    const unsigned char* s0 = smem + ((4 * t) % NSLOT) * HT;
    const unsigned char* s1 = smem + ((4 * t + 1) % NSLOT) * HT;
    const unsigned char* s2p = smem + ((4 * t + 2) % NSLOT) * HT;
    const unsigned char* s3 = smem + ((4 * t + 3) % NSLOT) * HT;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) b0[jj][s2] = ld_b128(s1 + boff[jj][s2]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s0 + aoff[i][s2]);
    issue_half<3>(p, smem, h, nk, nkseg, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(0, b0, 0);
    sync_end();
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) b1[jj][s2] = ld_b128(s2p + boff[jj][s2]);
    issue_half<0>(p, smem, h + 1, nk, nkseg, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(0, b1, 1);
    sync_end();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s3 + aoff[i][s2]);
    issue_half<1>(p, smem, h + 2, nk, nkseg, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(1, b1, 1);
    sync_end();
    issue_half<2>(p, smem, h + 3, nk, nkseg, m0, n0, wave, lane);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    sync_mid();
    mfma_quadrant(1, b0, 0);
    sync_end();
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // rejoin wave row 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-the-end half-tiles, before the epilogue reuses LDS
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  x2_epilogue<EPI>(p, acc, smem, m0, n0, wave, lane);
}

// W [rows][cols] fp32 -> planes of W^T [cols][rows] (the input gradient's NT operand): 64 x 64 tiles through LDS
__global__ void __launch_bounds__(256) x2_split_t_kernel(const float* __restrict__ X, int rows, int cols, int ldx,
                                                         const float* __restrict__ amax, int namax,
                                                         u16* __restrict__ P, int64_t ps, int ldp,
                                                         float* __restrict__ scale_out) {
  __shared__ float tile[64][65];
  __shared__ float red[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < namax; i += 256) m = fmaxf(m, fabsf(amax[i]));
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int E = bound_exp(m);
  const float up = pow2f(14 - E);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *scale_out = pow2f(E - 14);
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    tile[r][c] = (r0 + r < rows && c0 + c < cols) ? X[(int64_t)(r0 + r) * ldx + c0 + c] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i >> 6, r = i & 63;  // output row c0 + c, column r0 + r
    if (c0 + c >= cols || r0 + r >= rows) continue;
    const float x = tile[r][c] * up;
    const _Float16 h = static_cast<_Float16>(x);
    const int64_t o = (int64_t)(c0 + c) * ldp + r0 + r;
    P[o] = __builtin_bit_cast(u16, h);
    P[ps + o] = __builtin_bit_cast(u16, static_cast<_Float16>(x - static_cast<float>(h)));
  }
}

// ================================================================================================
// weight gradient: gW[M][N] += sum_t A[t][m] B[t][n] with A = dz planes [T][lda], B = x planes [T][ldb]
// (gemm_bf16_wgrad.hip's geometry: 256 x 128 tile, 8 waves of 64 x 64, 32x32x16 MFMAs, register-staged
// k-major images read by ds_read_b64_tr_b16). The 3 plane pairs form one extended K axis of 3 ceil(T / 64)
// K-steps; split s covers K-steps [s kps, (s + 1) kps), and every tile of one split runs on one XCD.
constexpr int WNT = 512, WBM = 256, WBN = 128, WBK = 64;
constexpr int IMG = WBK * 128;  // u16 per 128-column image

struct X2Wg {
  const u16* A;  // dz planes
  const u16* B;  // x planes
  int64_t a_ps, b_ps;
  float* slab;  // [splits][M][N] fp32, then [splits][M] bias partials
  int M, N, T, lda, ldb;
  int nks;     // K-steps per plane pair (ceil(T / WBK)); the extended axis has 3 nks K-steps
  int kps;     // K-steps per split
  int splits;
  int tiles_m, tiles_n;
  int bparts;  // bias partials per split (x2_wgrad_dma_kernel: tiles_n, block tn sums K-steps e % tiles_n == tn)
};

__device__ __forceinline__ int km_off(int k, int ch) { return k * 128 + 8 * (ch ^ (((k & 3) << 2) | ((k >> 2) & 3))); }

__device__ __forceinline__ f16x8 trfrag(const u16* P, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k = 16 * s + 8 * (g >> 1) + q;
  const int col = c0 + 16 * (g & 1) + 4 * pp;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(P + km_off(k, col >> 3) + (col & 7)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(P + km_off(k + 4, col >> 3) + (col & 7)));
  return __builtin_bit_cast(f16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

__device__ __forceinline__ float h2f(u16 v) { return static_cast<float>(__builtin_bit_cast(_Float16, v)); }

template <int COLS>
struct KmTile {
  static constexpr int CPR = COLS / 8;      // chunks per k-row
  static constexpr int NV = WBK * CPR / WNT;  // chunks per thread
  u16x8 v[NV];
  // the K-step's rows k0 .. k0 + 63 of plane P (rows past T re-read row T - 1; zeroed in store)
  __device__ __forceinline__ void load(const u16* __restrict__ P, int ld, int cols, int c0, int k0, int T) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int id = threadIdx.x + WNT * u;
      const int k = min(k0 + id / CPR, T - 1);
      const int c = min(c0 + 8 * (id % CPR), cols - 8);
      v[u] = *reinterpret_cast<const u16x8*>(P + (size_t)k * ld + c);
    }
  }
  // rows k0 + k >= T are stored as zeros; colsum[e] += the staged values when `sum`
  template <bool ROWSUM>
  __device__ __forceinline__ void store(u16* L, int k0, int T, bool sum, float (&colsum)[8]) const {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int id = threadIdx.x + WNT * u;
      const int k = id / CPR, ch = id % CPR;
      const u16x8 val = (k0 + k < T) ? v[u] : z;
      *reinterpret_cast<u16x8*>(L + (ch >> 4) * IMG + km_off(k, ch & 15)) = val;
      if constexpr (ROWSUM) {
        if (sum) {
#pragma unroll
          for (int e = 0; e < 8; ++e) colsum[e] += h2f(val[e]);
        }
      }
    }
  }
};

// bias partials (16 row groups -> LDS -> 256 column sums) and the partial tile -> slab; smem must be free
__device__ __forceinline__ void x2w_finish(const X2Wg& p, const f32x16 (&acc)[2][2], const float (&cs)[8], u16* smem,
                                           bool do_bias, int split, int bslot, int m0, int n0, int wm, int wn,
                                           int lane) {
  if (do_bias) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [16][256]
    const int chn = threadIdx.x & 31, part = threadIdx.x >> 5;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[part * 256 + 8 * chn + e] = cs[e];
    __syncthreads();
    if (threadIdx.x < WBM) {
      float sum = 0.f;
      for (int q = 0; q < 16; ++q) sum += red[q * 256 + threadIdx.x];
      const int m = m0 + threadIdx.x;
      if (m < p.M) p.slab[(size_t)p.splits * p.M * p.N + ((size_t)split * p.bparts + bslot) * p.M + m] = sum;
    }
  }

  // partial tile -> slab; C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        p.slab[((size_t)split * p.M + row) * p.N + col] = acc[i][j][r];
      }
    }
}

// K-step e of the extended axis: plane pair seg = e / nks ({(dz hi, x hi), (dz hi, x lo), (dz lo, x hi)}),
// tokens (e - seg nks) * 64 ..; a split covers K-steps [split * kps, ...) and may cross a pair boundary
template <bool BIAS>
__global__ void __launch_bounds__(WNT) x2_wgrad_kernel(X2Wg p) {
  constexpr int BUF = 3 * IMG;  // A: two 128-col images, B: one
  __shared__ __attribute__((aligned(16))) u16 smem[2 * BUF];
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nwg = ntiles * p.splits;
  const int orig = blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {  // XCD-aware: the tiles of one split (same token range) share an XCD's L2
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int m0 = tm * WBM, n0 = tn * WBN;
  const int ebeg = split * p.kps, eend = min(3 * p.nks, ebeg + p.kps);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 3, wn = wave >> 2;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  KmTile<WBM> ta;
  KmTile<WBN> tb;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool do_bias = BIAS && tn == 0;
  auto seg_of = [&](int e) { return e / p.nks; };
  auto load = [&](int e) {
    const int seg = seg_of(e), k0 = (e - seg * p.nks) * WBK;
    ta.load(p.A + (seg == 2 ? p.a_ps : 0), p.lda, p.M, m0, k0, p.T);
    tb.load(p.B + (seg == 1 ? p.b_ps : 0), p.ldb, p.N, n0, k0, p.T);
  };
  auto store = [&](u16* L, int e) {  // bias: dz hi (pair 0) + dz lo (pair 2)
    const int seg = seg_of(e), k0 = (e - seg * p.nks) * WBK;
    if (do_bias) ta.template store<true>(L, k0, p.T, seg != 1, cs);
    else ta.template store<false>(L, k0, p.T, false, cs);
    tb.template store<false>(L + 2 * IMG, k0, p.T, false, cs);
  };
  const int nk = max(0, eend - ebeg);
  if (nk > 0) {
    load(ebeg);
    store(smem, ebeg);
    if (nk > 1) load(ebeg + 1);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const u16* L = smem + (t & 1) * BUF;
    u16* Ln = smem + ((t + 1) & 1) * BUF;
#pragma unroll
    for (int s = 0; s < WBK / 16; ++s) {
      f16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = trfrag(L + (wm >> 1) * IMG, (wm & 1) * 64 + 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = trfrag(L + 2 * IMG, wn * 64 + 32 * j, s, lane);
      if (s == 0 && t + 1 < nk) {  // K-step t+1 (registers) -> the other buffer; K-step t+2 -> registers
        store(Ln, ebeg + t + 1);
        if (t + 2 < nk) load(ebeg + t + 2);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  x2w_finish(p, acc, cs, smem, do_bias, split, 0, m0, n0, wm, wn, lane);
}

// ---- LDS-DMA form of the weight gradient (T % 64 == 0; gemm_bf16_wgrad.hip's wgrad_dma_kernel with the
// plane pair chosen per K-step): 3-stage ring of [A 2 x 128 cols | B 128 cols] images filled by
// global_load_lds (the km_off swizzle on the per-lane source address), two K-steps in flight, one
// counted vmcnt(6) + barrier per K-step, fragments by inline-asm transposed reads (see x2w_tr16).
__device__ __forceinline__ void x2w_issue(const X2Wg& p, u16* st, int m0, int n0, int e, int wave, int lane) {
  const int seg = e / p.nks, k0 = (e - seg * p.nks) * WBK;
  const u16* A = p.A + (seg == 2 ? p.a_ps : 0);
  const u16* B = p.B + (seg == 1 ? p.b_ps : 0);
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int q = wave + 8 * u;
    const int img = u >> 1, r = 4 * (wave + 8 * (u & 1)) + (lane >> 4);
    const int c = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    const u16* src = img < 2 ? A + (size_t)(k0 + r) * p.lda + min(m0 + 128 * img + 8 * c, p.M - 8)
                             : B + (size_t)(k0 + r) * p.ldb + min(n0 + 8 * c, p.N - 8);
    glds16(src, reinterpret_cast<unsigned char*>(st + q * 512));
  }
}

// inline-asm ds_read_b64_tr_b16: the builtin makes the compiler wait for every LDS-DMA in flight
// (vmcnt(0)) before each read; these are invisible to its wait pass, so lgkmcnt is waited explicitly
// with the fragments as "+v" operands (no MFMA can move above the wait)
__device__ __forceinline__ s16x4 x2w_tr16(const u16* p) {
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) u16*)p;
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

__device__ __forceinline__ void x2w_read(const u16* L, int wm, int wn, int s, int lane, s16x4 (&f)[8]) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k = 16 * s + 8 * (g >> 1) + q;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const u16* P = x < 2 ? L + (wm >> 1) * IMG : L + 2 * IMG;
    const int c0 = x < 2 ? (wm & 1) * 64 + 32 * x : wn * 64 + 32 * (x - 2);
    const int col = c0 + 16 * (g & 1) + 4 * pp;
    f[2 * x] = x2w_tr16(P + km_off(k, col >> 3) + (col & 7));
    f[2 * x + 1] = x2w_tr16(P + km_off(k + 4, col >> 3) + (col & 7));
  }
}

template <int N>
__device__ __forceinline__ void x2w_wait(s16x4 (&f)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
               : "n"(N));
}

__device__ __forceinline__ f16x8 x2w_cat(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(f16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

template <bool BIAS>
__global__ void __launch_bounds__(WNT) x2_wgrad_dma_kernel(X2Wg p) {
  constexpr int BUF = 3 * IMG;
  __shared__ __attribute__((aligned(16))) u16 smem[3 * BUF];
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nwg = ntiles * p.splits;
  const int orig = blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int m0 = tm * WBM, n0 = tn * WBN;
  const int ebeg = split * p.kps, eend = min(3 * p.nks, ebeg + p.kps);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 3, wn = wave >> 2;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int nk = max(0, eend - ebeg);
  auto estep = [&](int t) { return ebeg + min(t, nk - 1); };  // past the end: re-read the last K-step
  if (nk > 0) {
    x2w_issue(p, smem, m0, n0, estep(0), wave, lane);
    x2w_issue(p, smem + BUF, m0, n0, estep(1), wave, lane);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const int bch = threadIdx.x & 31, brg = threadIdx.x >> 5;
  for (int t = 0; t < nk; ++t) {
    const u16* L = smem + (t % 3) * BUF;
    x2w_issue(p, smem + ((t + 2) % 3) * BUF, m0, n0, estep(t + 2), wave, lane);
    s16x4 fr[2][8];
    x2w_read(L, wm, wn, 0, lane, fr[0]);
#pragma unroll
    for (int s = 0; s < WBK / 16; ++s) {
      if (s + 1 < WBK / 16) {
        x2w_read(L, wm, wn, s + 1, lane, fr[(s + 1) & 1]);
        x2w_wait<8>(fr[s & 1]);
      } else {
        x2w_wait<0>(fr[s & 1]);
      }
      const f16x8 a[2] = {x2w_cat(fr[s & 1][0], fr[s & 1][1]), x2w_cat(fr[s & 1][2], fr[s & 1][3])};
      const f16x8 b[2] = {x2w_cat(fr[s & 1][4], fr[s & 1][5]), x2w_cat(fr[s & 1][6], fr[s & 1][7])};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    // bias (dz hi in pair 0 + dz lo in pair 2), after the K-step's MFMAs are issued, before the barrier
    const int e = ebeg + t;
    if (BIAS && e / p.nks != 1 && e % p.bparts == tn) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const u16x8 v = *reinterpret_cast<const u16x8*>(L + (bch >> 4) * IMG + km_off(brg + 16 * u, bch & 15));
#pragma unroll
        for (int x = 0; x < 8; ++x) cs[x] += h2f(v[x]);
      }
    }
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  x2w_finish(p, acc, cs, smem, BIAS, split, tn, m0, n0, wm, wn, lane);
}

// gW[m][n] (fp32) += sa sb sum_s slab[s][m][n] (fixed order); gb[m] += sa sum_j bias_slab[j][m]
// (j < splits * bparts) in the blocks past `main_blocks`: 16 columns x 16 row groups, combined in a fixed order
__global__ void __launch_bounds__(256) x2_wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int bparts,
                                                              int M, int N, float* __restrict__ C, int ldc,
                                                              float* __restrict__ gb, const float* __restrict__ sa,
                                                              const float* __restrict__ sb, int main_blocks) {
  const float da = *sa, dq = da * *sb;
  const int64_t MN = (int64_t)M * N;
  if ((int)blockIdx.x >= main_blocks) {
    __shared__ float red[16][16];
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int m = ((int)blockIdx.x - main_blocks) * 16 + c;
    const float* bs = slab + (size_t)splits * MN;
    float s = 0.f;
    if (m < M)
      for (int k = g; k < splits * bparts; k += 16) s += bs[(size_t)k * M + m];
    red[g][c] = s;
    __syncthreads();
    if (g == 0 && m < M) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += red[q][c];
      gb[m] += da * t;
    }
    return;
  }
  const int64_t n4 = MN / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)main_blocks * 256) {
    f32x4 s = *reinterpret_cast<const f32x4*>(slab + 4 * i);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(slab + k * MN + 4 * i);
    const int64_t e = 4 * i;
    const int m = (int)(e / N), n = (int)(e % N);
    f32x4* dst = reinterpret_cast<f32x4*>(C + (size_t)m * ldc + n);
    *dst += s * dq;
  }
}

// splits of the extended K axis (3 ceil(T / 64) K-steps): enough to cover the 256 CUs once, >= 8 K-steps each
int x2_wgrad_splits(int M, int N, int T) {
  const int tiles = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
  const int steps = 3 * ((T + WBK - 1) / WBK);
  int s = std::max(1, 256 / tiles);
  return std::max(1, std::min(s, steps / 8));
}

}  // namespace

bool x2_gemm_supported(int M, int N, int K, int lda, int ldb, int ldc, bool b_kn) {
  return M >= 1 && N >= 8 && K >= TK && K % TK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 &&
         (b_kn ? ldb >= N : ldb >= K) && lda >= K && ldc >= N;
}

int x2_gemm_wmax_slots(int M, int N) { return ((M + TM - 1) / TM) * ((N + TN - 1) / TN) * 8; }

void x2_split(const float* X, int rows, int cols, int ldx, const float* amax, int namax, void* planes, int64_t ps,
              int ldp, float* scale_out, hipStream_t stream) {
  const int64_t n8 = (int64_t)rows * (cols / 8);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n8 + 255) / 256, 4096));
  hipLaunchKernelGGL(x2_split_kernel, dim3(blocks), dim3(256), 0, stream, X, rows, cols, ldx, amax, namax,
                     static_cast<u16*>(planes), ps, ldp, scale_out);
}

void x2_split_t(const float* X, int rows, int cols, int ldx, const float* amax, int namax, void* planes, int64_t ps,
                int ldp, float* scale_out, hipStream_t stream) {
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  hipLaunchKernelGGL(x2_split_t_kernel, grid, dim3(256), 0, stream, X, rows, cols, ldx, amax, namax,
                     static_cast<u16*>(planes), ps, ldp, scale_out);
}

void x2_gemm(const void* A, int64_t a_ps, const void* B, int64_t b_ps, float* C, int M, int N, int K, int lda, int ldb,
             int ldc, bool b_kn, const float* sa, const float* sb, const float* bias, bool relu, const float* mask,
             int ldm, float* wmax, hipStream_t stream) {
  X2Gemm p;
  p.A = static_cast<const u16*>(A);
  p.B = static_cast<const u16*>(B);
  p.a_ps = a_ps;
  p.b_ps = b_ps;
  p.C = C;
  p.bias = bias;
  p.mask = mask;
  p.sa = sa;
  p.sb = sb;
  p.wmax = wmax;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.ldm = ldm;
  p.tiles_m = (M + TM - 1) / TM;
  p.tiles_n = (N + TN - 1) / TN;
  p.ntstore = knob(KNOB_GEMM_NT_STORE) == 1;
  p.group_m = std::max(0, knob(KNOB_GEMM_GROUP_M));
  const dim3 grid(p.tiles_m * p.tiles_n);
  const int epi = (relu ? X2_RELU : 0) | (mask ? X2_MASK : 0);
#define X2_LAUNCH(BLV, E) hipLaunchKernelGGL((x2_gemm_kernel<BLV, E>), grid, dim3(GT), 0, stream, p)
#define X2_EPI(BLV)                                            \
  do {                                                         \
    switch (epi) {                                             \
      case X2_RELU: X2_LAUNCH(BLV, X2_RELU); break;            \
      case X2_MASK: X2_LAUNCH(BLV, X2_MASK); break;            \
      case X2_RELU | X2_MASK: X2_LAUNCH(BLV, X2_RELU | X2_MASK); break; \
      default: X2_LAUNCH(BLV, 0); break;                       \
    }                                                          \
  } while (0)
#define X2_NT4(E) hipLaunchKernelGGL((x2_gemm_nt4_kernel<E>), grid, dim3(GT), 0, stream, p)
  const bool nt4 = knob(KNOB_X2_2PHASE) == 0;  // 1: the one-barrier-per-K-step loop (A/B)
  if (b_kn) {
    X2_EPI(1);
  } else if (nt4) {
    switch (epi) {
      case X2_RELU: X2_NT4(X2_RELU); break;
      case X2_MASK: X2_NT4(X2_MASK); break;
      case X2_RELU | X2_MASK: X2_NT4(X2_RELU | X2_MASK); break;
      default: X2_NT4(0); break;
    }
  } else {
    X2_EPI(0);
  }
#undef X2_NT4
#undef X2_EPI
#undef X2_LAUNCH
}

bool x2_wgrad_supported(int M, int N, int T, int lda, int ldb) {
  return M >= 8 && N >= 8 && T >= 1 && M % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0;
}

size_t x2_wgrad_workspace_floats(int M, int N, int T) {
  const int splits = x2_wgrad_splits(M, N, T);
  const int tiles_n = (N + WBN - 1) / WBN;  // bias partials: splits x tiles_n rows of M (the DMA loop)
  return (size_t)splits * M * N + (size_t)splits * tiles_n * M;
}

void x2_wgrad(const void* dz, int64_t dz_ps, const void* x, int64_t x_ps, const float* sdz, const float* sx, float* gw,
              int ldc, float* gb, float* workspace, int M, int N, int T, int lda, int ldb, hipStream_t stream) {
  X2Wg p;
  p.A = static_cast<const u16*>(dz);
  p.B = static_cast<const u16*>(x);
  p.a_ps = dz_ps;
  p.b_ps = x_ps;
  p.slab = workspace;
  p.M = M;
  p.N = N;
  p.T = T;
  p.lda = lda;
  p.ldb = ldb;
  p.nks = (T + WBK - 1) / WBK;
  int splits = x2_wgrad_splits(M, N, T);
  p.kps = (3 * p.nks + splits - 1) / splits;
  splits = (3 * p.nks + p.kps - 1) / p.kps;  // (never more than the workspace was sized for)
  p.splits = splits;
  p.tiles_m = (M + WBM - 1) / WBM;
  p.tiles_n = (N + WBN - 1) / WBN;
  const dim3 grid(p.tiles_m * p.tiles_n * p.splits);
  const bool dma = knob(KNOB_WGRAD_DMA) != 0 && T % WBK == 0 &&  // (tests A/B the two loops)
                   (reinterpret_cast<uintptr_t>(dz) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (dz_ps % 8) == 0 && (x_ps % 8) == 0;
  p.bparts = dma ? p.tiles_n : 1;
  if (dma) {
    if (gb) hipLaunchKernelGGL(x2_wgrad_dma_kernel<true>, grid, dim3(WNT), 0, stream, p);
    else hipLaunchKernelGGL(x2_wgrad_dma_kernel<false>, grid, dim3(WNT), 0, stream, p);
  } else if (gb) {
    hipLaunchKernelGGL(x2_wgrad_kernel<true>, grid, dim3(WNT), 0, stream, p);
  } else {
    hipLaunchKernelGGL(x2_wgrad_kernel<false>, grid, dim3(WNT), 0, stream, p);
  }
  const int64_t n4 = (int64_t)M * N / 4;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
  const int bblocks = gb ? (M + 15) / 16 : 0;
  hipLaunchKernelGGL(x2_wgrad_reduce_kernel, dim3(blocks + bblocks), dim3(256), 0, stream, workspace, p.splits,
                     p.bparts, M, N, gw, ldc, gb, sdz, sx, blocks);
}

}  // namespace sdml
