// Weight-gradient GEMM of a bf16 Linear layer: gW[M,N] (bf16, in place) += sum_t gy[t][m] x[t][n]
// over the T tokens of a (micro-)batch — the "small output, huge reduction" GEMM (GPT-2:
// 768..3072 x 768..3072 outputs, T = 16384) that hipBLASLt runs at 180-470 TF/s on gfx950
// because 36-144 output tiles cannot fill 256 CUs (tools/bench_gpt2_gemms.py).
//
// Both operands are k-major (the token index t is the row of gy and x), so their tiles are copied
// into LDS exactly as they sit in memory and the MFMA fragments come out of the hardware
// transpose read (ds_read_b64_tr_b16) — no transpose pass, no extra copy of gy or x.
//   block 512 threads = 8 waves (4 x 2), tile 256 (m) x 128 (n), K-step 64, wave tile 64 x 64
//   (2 x 2 v_mfma_f32_32x32x16_bf16, 16 MFMAs per wave per K-step); LDS double-buffered
//   48 KiB per stage; images [64 k][128 cols] with 16-B chunk c of row k at
//   c ^ (((k&3)<<2) | ((k>>2)&3)) (conflict-free tr reads and 16-B writes).
// The token range is split over workgroups until the grid covers the chip; each split writes
// an fp32 slab and a second pass adds the slabs, in a fixed order, to the bf16 gradient
// (deterministic: no float atomics). With one split the block adds its tile directly.
// The bias gradient (column sums of gy) is fused: the first column tile's blocks sum the gy tile
// they stage anyway, so the separate bias reduction pass over gy disappears.
// Replaces the autograd weight gradient of the GPT-2 stages' projections (ops/linear.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512, BM = 256, BN = 128, BK = 64;
constexpr int IMG = BK * 128;  // u16 per 128-column image

struct WgParams {
  const u16* A;  // gy [T][lda]
  const u16* B;  // x  [T][ldb]
  u16* C;        // gW [M][ldc] (bf16, accumulated)
  u16* gb;       // bias gradient [M] (bf16, accumulated) or nullptr: column sums of gy
  float* slab;   // [splits][M][N] fp32, then [splits][M] bias partials (splits > 1)
  int M, N, T, lda, ldb, ldc;
  int tps;  // tokens per split (multiple of BK)
  int tiles_m, tiles_n, splits;
};

__device__ __forceinline__ int km_off(int k, int ch) { return k * 128 + 8 * (ch ^ (((k & 3) << 2) | ((k >> 2) & 3))); }

__device__ __forceinline__ s16x4 ds_tr16(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// fragment of the 32-column block at c0 of a [64][128] image, k-substep s: element j = X[16s + 8h + j][c0 + lane&31]
__device__ __forceinline__ bf16x8 trfrag(const u16* P, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k = 16 * s + 8 * (g >> 1) + q;
  const int col = c0 + 16 * (g & 1) + 4 * p;
  const s16x4 lo = ds_tr16(P + km_off(k, col >> 3) + (col & 7));
  const s16x4 hi = ds_tr16(P + km_off(k + 4, col >> 3) + (col & 7));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, static_cast<__bf16>(f)); }

// a COLS-wide k-major tile (64 k x COLS) in registers: COLS/8 chunks of 16 B per k-row
template <int COLS>
struct KmTile {
  static constexpr int CPR = COLS / 8;            // chunks per k-row
  static constexpr int NV = BK * CPR / NT;        // chunks per thread
  u16x8 v[NV];
  // clamped loads (rows past T / cols past the end re-read valid memory; zeroed in store)
  __device__ __forceinline__ void load(const u16* __restrict__ P, int ld, int cols, int c0, int k0, int T) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int id = threadIdx.x + NT * u;
      const int k = min(k0 + id / CPR, T - 1);
      const int c = min(c0 + 8 * (id % CPR), cols - 8);
      v[u] = *reinterpret_cast<const u16x8*>(P + (size_t)k * ld + c);
    }
  }
  // ROWSUM: colsum[e] += the 8 staged values of this thread's column chunk (every u of a
  // thread has the same chunk index: NT is a multiple of CPR), k >= kend excluded
  template <bool ROWSUM>
  __device__ __forceinline__ void store(u16* L, int k0, int kend, float (&colsum)[8]) const {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int id = threadIdx.x + NT * u;
      const int k = id / CPR, ch = id % CPR;
      const u16x8 val = (k0 + k < kend) ? v[u] : z;
      *reinterpret_cast<u16x8*>(L + (ch >> 4) * IMG + km_off(k, ch & 15)) = val;
      if constexpr (ROWSUM) {
#pragma unroll
        for (int e = 0; e < 8; ++e) colsum[e] += bf2f(val[e]);
      }
    }
  }
};

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// BIAS: the tn == 0 blocks also reduce the staged gy tile over tokens (the bias gradient)
template <bool BIAS>
__global__ void __launch_bounds__(NT) wgrad_kernel(WgParams p) {
  constexpr int BUF = 3 * IMG;  // A: two 128-col images, B: one
  __shared__ __attribute__((aligned(16))) u16 smem[2 * BUF];
  // XCD-aware bijective remap: the splits of one tile (which read disjoint token ranges) and the
  // tiles that share an A/B column panel land on one XCD's L2
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
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.tps, kend = min(p.T, kbeg + p.tps);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 3, wn = wave >> 2;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  KmTile<BM> ta;
  KmTile<BN> tb;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // bias partials (BIAS, tn == 0)
  float dummy[8];
  const bool do_bias = BIAS && tn == 0;
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    ta.load(p.A, p.lda, p.M, m0, kbeg, p.T);
    tb.load(p.B, p.ldb, p.N, n0, kbeg, p.T);
    if (do_bias) ta.template store<true>(smem, kbeg, kend, cs);
    else ta.template store<false>(smem, kbeg, kend, dummy);
    tb.template store<false>(smem + 2 * IMG, kbeg, kend, dummy);
    ta.load(p.A, p.lda, p.M, m0, kbeg + BK, p.T);
    tb.load(p.B, p.ldb, p.N, n0, kbeg + BK, p.T);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const u16* L = smem + (t & 1) * BUF;
    u16* Ln = smem + ((t + 1) & 1) * BUF;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 a[2], b[2];
      // wave rows wm*64 .. +63 lie in image (wm >> 1), columns (wm & 1) * 64
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = trfrag(L + (wm >> 1) * IMG, (wm & 1) * 64 + 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = trfrag(L + 2 * IMG, wn * 64 + 32 * j, s, lane);
      if (s == 0) {  // tile t+1 (registers) -> the other buffer; tile t+2 -> registers
        if (do_bias) ta.template store<true>(Ln, kbeg + (t + 1) * BK, kend, cs);
        else ta.template store<false>(Ln, kbeg + (t + 1) * BK, kend, dummy);
        tb.template store<false>(Ln + 2 * IMG, kbeg + (t + 1) * BK, kend, dummy);
        ta.load(p.A, p.lda, p.M, m0, kbeg + (t + 2) * BK, p.T);
        tb.load(p.B, p.ldb, p.N, n0, kbeg + (t + 2) * BK, p.T);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }

  if (do_bias) {
    // the 16 threads t, t+32, ..., t+480 own the same 8 columns m0 + 8*(t&31) + e: meet in LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [16][256]
    const int ch = threadIdx.x & 31, part = threadIdx.x >> 5;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[part * 256 + 8 * ch + e] = cs[e];
    __syncthreads();
    if (threadIdx.x < BM) {
      float sum = 0.f;
      for (int q = 0; q < 16; ++q) sum += red[q * 256 + threadIdx.x];
      const int m = m0 + threadIdx.x;
      if (m < p.M) {
        if (p.splits == 1) p.gb[m] = f2bf(bf2f(p.gb[m]) + sum);
        else p.slab[(size_t)p.splits * p.M * p.N + (size_t)split * p.M + m] = sum;
      }
    }
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
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
        if (p.splits == 1) {
          u16* dst = p.C + (size_t)row * p.ldc + col;
          *dst = f2bf(bf2f(*dst) + acc[i][j][r]);
        } else {
          p.slab[((size_t)split * p.M + row) * p.N + col] = acc[i][j][r];
        }
      }
    }
}

// C[m][n] (bf16) += sum_s slab[s][m][n], fixed order; 4 elements per thread (N % 4 == 0);
// gb[m] += sum_s bias_slab[s][m] when gb is given
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                           u16* __restrict__ C, int ldc, u16* __restrict__ gb) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t MN = (int64_t)M * N;
  if (gb) {
    const float* bs = slab + (size_t)splits * MN;
    for (int64_t m = blockIdx.x * 256 + threadIdx.x; m < M; m += (int64_t)gridDim.x * 256) {
      float s = 0.f;
      for (int k = 0; k < splits; ++k) s += bs[(size_t)k * M + m];
      gb[m] = f2bf(bf2f(gb[m]) + s);
    }
  }
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 s = *reinterpret_cast<const f32x4*>(slab + 4 * i);
    for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const f32x4*>(slab + k * MN + 4 * i);
    const int64_t e = 4 * i;
    const int m = (int)(e / N), n = (int)(e % N);
    u16* dst = C + (size_t)m * ldc + n;
#pragma unroll
    for (int c = 0; c < 4; ++c) dst[c] = f2bf(bf2f(dst[c]) + s[c]);
  }
}

}  // namespace

bool wgrad_bf16_supported(int M, int N, int T, int lda, int ldb, int ldc) {
  return M >= 8 && N >= 8 && T >= 1 && M % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc >= N;
}

int wgrad_bf16_splits(int M, int N, int T) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // one 512-thread workgroup per CU (96 KB LDS): SDML_WGRAD_WAVES = how many times the grid may
  // cover the 256 CUs (default 1: floor(256 / tiles) splits); >= 8 K-steps per split. Measured on
  // the GPT-2 shapes (tools/bench_gpt2_gemms.py): 2 or 3 grid waves are 5-25 % slower — the larger
  // fp32 slab reduction costs more than the idle CUs of one partial wave.
  static const int waves = [] {
    const char* e = std::getenv("SDML_WGRAD_WAVES");
    return e ? std::max(1, std::atoi(e)) : 1;
  }();
  int s = 256 * waves / tiles;
  const int max_by_t = T / (8 * BK);
  if (s > max_by_t) s = max_by_t;
  return s < 1 ? 1 : s;
}

size_t wgrad_bf16_workspace_floats(int M, int N, int T) {
  const int s = wgrad_bf16_splits(M, N, T);
  return s > 1 ? (size_t)s * M * N + (size_t)s * M : 0;
}

void wgrad_bf16(const void* gy, const void* x, void* gw, void* gb, float* workspace, int M, int N, int T, int lda,
                int ldb, int ldc, hipStream_t stream) {
  WgParams p;
  p.A = static_cast<const u16*>(gy);
  p.B = static_cast<const u16*>(x);
  p.C = static_cast<u16*>(gw);
  p.gb = static_cast<u16*>(gb);
  p.slab = workspace;
  p.M = M;
  p.N = N;
  p.T = T;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  int s = wgrad_bf16_splits(M, N, T);
  int tps = (T + s - 1) / s;
  tps = (tps + BK - 1) / BK * BK;
  s = (T + tps - 1) / tps;
  p.tps = tps;
  p.splits = s;
  p.tiles_m = (M + BM - 1) / BM;
  p.tiles_n = (N + BN - 1) / BN;
  if (gb) hipLaunchKernelGGL(wgrad_kernel<true>, dim3(p.tiles_m * p.tiles_n * s), dim3(NT), 0, stream, p);
  else hipLaunchKernelGGL(wgrad_kernel<false>, dim3(p.tiles_m * p.tiles_n * s), dim3(NT), 0, stream, p);
  if (s > 1) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, workspace, s, M, N,
                       static_cast<u16*>(gw), ldc, static_cast<u16*>(gb));
  }
}

}  // namespace sdml
