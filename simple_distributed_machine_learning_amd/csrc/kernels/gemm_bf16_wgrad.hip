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
//
// Two main loops over the same tile, fragments and epilogue:
//   wgrad_dma_kernel (T % 64 == 0, 16-B aligned operands; the default): the tiles go HBM -> LDS by
//     LDS-DMA (global_load_lds_dwordx4) into a ring of 3 stages (144 KiB), two K-steps in flight and
//     one counted `s_waitcnt vmcnt(6)` + barrier per K-step. The XOR swizzle moves to the per-lane
//     source address (a DMA instruction writes 4 image rows lane-linearly), so the images are the
//     same as below. No VGPR staging: the 48 KiB per K-step of ds_write_b128 (~13 LDS cycles per
//     wave-instruction, MI355X_MICROARCH.md LDS table) that made the staged loop LDS-bound are gone.
//     The bias gradient's column sums are read back from the A images (4 ds_read_b128 per thread
//     per K-step, in the tn == 0 blocks only).
//   wgrad_kernel (any T; SDML_WGRAD_DMA=0): register-staged double buffer (the loads of K-step t+2
//     are in flight while K-step t+1 is written to LDS), rows past T zeroed on the store.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

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
  int bparts;  // bias partial sums per split (the DMA loop: tiles_n, each tn block sums K-steps t % tiles_n == tn)
  int nfast;   // tile order: 0 = M fastest (neighbouring blocks share the x panel), 1 = N fastest (they share the gy
               // panel: the lm_head's 1.6 GB dlogits, read once from HBM instead of once per column tile)
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

// bias partials (16 row groups of 8 columns per thread -> LDS -> 256 column sums) and the
// accumulator tile (bf16 in place with one split, an fp32 slab otherwise); smem must be free
__device__ __forceinline__ void wgrad_finish(const WgParams& p, const f32x16 (&acc)[2][2], const float (&cs)[8],
                                             u16* smem, bool do_bias, int split, int bslot, int m0, int n0, int wm,
                                             int wn, int lane) {
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
        else p.slab[(size_t)p.splits * p.M * p.N + ((size_t)split * p.bparts + bslot) * p.M + m] = sum;
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
  const int tm = p.nfast ? tile / p.tiles_n : tile % p.tiles_m, tn = p.nfast ? tile % p.tiles_n : tile / p.tiles_m;
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

  wgrad_finish(p, acc, cs, smem, do_bias, split, p.bparts > 1 ? tn : 0, m0, n0, wm, wn, lane);
}

__device__ __forceinline__ void glds16(const void* src, u16* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

// one K-step (64 tokens at k0) -> stage st = [A cols m0..+127 | A cols m0+128..+255 | B cols n0..+127],
// each a [64 k][128] image: 16 DMA instructions of 4 rows x 256 B per image, 6 per wave. Lane l of an
// instruction writes image position (row 4q + l/16, chunk l%16), i.e. it loads logical chunk
// (l%16) ^ swz(row) (the km_off swizzle is an involution). Columns past M / N re-read valid memory
// (chunks are whole: M, N % 8 == 0); they only feed output rows / columns that are never written.
__device__ __forceinline__ void wgrad_issue(const WgParams& p, u16* st, int m0, int n0, int k0, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int q = wave + 8 * u;  // 0..47: image u / 2 (compile-time), rows 4 (q & 15) ..
    const int img = u >> 1, r = 4 * (wave + 8 * (u & 1)) + (lane >> 4);
    const int c = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    const u16* src = img < 2 ? p.A + (size_t)(k0 + r) * p.lda + min(m0 + 128 * img + 8 * c, p.M - 8)
                             : p.B + (size_t)(k0 + r) * p.ldb + min(n0 + 8 * c, p.N - 8);
    glds16(src, st + q * 512);
  }
}

// The DMA loop reads its fragments with inline-asm ds_read_b64_tr_b16: the compiler's wait pass
// puts an `s_waitcnt vmcnt(0)` (every LDS-DMA in flight, K-step t+2 included) in front of each
// __builtin_amdgcn_ds_read_tr16_b64 it cannot tell apart from the DMA stores, which serialises the
// ring. The asm reads are invisible to that pass, so their lgkmcnt waits are explicit (lgkm_wait):
// LDS returns in order, and the fragments are "+v" operands of the wait, so no MFMA moves above it.
__device__ __forceinline__ s16x4 ds_tr16_asm(const u16* p) {
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) u16*)p;
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

// the 8 half-fragments of one 16-deep substep: A (2 x lo/hi) then B (2 x lo/hi), as trfrag reads them
__device__ __forceinline__ void read_substep(const u16* L, int wm, int wn, int s, int lane, s16x4 (&f)[8]) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int k = 16 * s + 8 * (g >> 1) + q;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const u16* P = x < 2 ? L + (wm >> 1) * IMG : L + 2 * IMG;
    const int c0 = x < 2 ? (wm & 1) * 64 + 32 * x : wn * 64 + 32 * (x - 2);
    const int col = c0 + 16 * (g & 1) + 4 * pp;
    f[2 * x] = ds_tr16_asm(P + km_off(k, col >> 3) + (col & 7));
    f[2 * x + 1] = ds_tr16_asm(P + km_off(k + 4, col >> 3) + (col & 7));
  }
}

template <int N>
__device__ __forceinline__ void lgkm_wait(s16x4 (&f)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
               : "n"(N));
}

__device__ __forceinline__ bf16x8 cat(s16x4 lo, s16x4 hi) {
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <bool BIAS>
__global__ void __launch_bounds__(NT) wgrad_dma_kernel(WgParams p) {
  constexpr int BUF = 3 * IMG;  // u16 per stage: A two 128-col images, B one
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
  const int tm = p.nfast ? tile / p.tiles_n : tile % p.tiles_m, tn = p.nfast ? tile % p.tiles_n : tile / p.tiles_m;
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
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // bias: with bparts > 1 every tn block sums the K-steps t % bparts == tn (no straggler column of blocks)
  const bool do_bias = BIAS && (p.bparts > 1 || tn == 0);
  const int nk = (kend - kbeg) / BK;  // whole K-steps (T % BK == 0, tps % BK == 0)
  // K-steps past the end re-read the last one into a stage that is never read again (uniform counting)
  auto kstep = [&](int t) { return kbeg + min(t, nk - 1) * BK; };
  if (nk > 0) {
    wgrad_issue(p, smem, m0, n0, kstep(0), wave, lane);
    wgrad_issue(p, smem + BUF, m0, n0, kstep(1), wave, lane);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K-step 0 landed (this wave's part)
  }
  __builtin_amdgcn_s_barrier();  // (not __syncthreads: its fence would wait for K-step 1 too)
  asm volatile("" ::: "memory");
  // bias: thread = (logical chunk id & 31 of the 256 A columns, row group id >> 5); rows rg + 16 u
  const int bch = threadIdx.x & 31, brg = threadIdx.x >> 5;
  for (int t = 0; t < nk; ++t) {
    const u16* L = smem + (t % 3) * BUF;
    wgrad_issue(p, smem + ((t + 2) % 3) * BUF, m0, n0, kstep(t + 2), wave, lane);
    s16x4 fr[2][8];  // substep s's fragments in fr[s & 1]; s + 1's reads are issued before s's MFMAs
    read_substep(L, wm, wn, 0, lane, fr[0]);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      if (s + 1 < BK / 16) {
        read_substep(L, wm, wn, s + 1, lane, fr[(s + 1) & 1]);
        lgkm_wait<8>(fr[s & 1]);
      } else {
        lgkm_wait<0>(fr[s & 1]);
      }
      const bf16x8 a[2] = {cat(fr[s & 1][0], fr[s & 1][1]), cat(fr[s & 1][2], fr[s & 1][3])};
      const bf16x8 b[2] = {cat(fr[s & 1][4], fr[s & 1][5]), cat(fr[s & 1][6], fr[s & 1][7])};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
    // bias: after the K-step's MFMAs are issued (its VALU work overlaps their tail), before the barrier
    if (do_bias && (p.bparts == 1 || t % p.bparts == tn)) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = brg + 16 * u;
        const u16x8 v = *reinterpret_cast<const u16x8*>(L + (bch >> 4) * IMG + km_off(r, bch & 15));
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += bf2f(v[e]);
      }
    }
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");  // K-step t+1 landed; this wave's reads done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-read stages, before smem is reused
  __syncthreads();
  wgrad_finish(p, acc, cs, smem, do_bias, split, p.bparts > 1 ? tn : 0, m0, n0, wm, wn, lane);
}

// C[m][n] (bf16) += sum_s slab[s][m][n], fixed order; 4 elements per thread (N % 4 == 0);
// gb[m] += sum_j bias_slab[j][m] (j < splits * bparts) when gb is given: blocks past `main_blocks`, 16
// columns x 16 row groups each (a short dependent chain per thread), the groups combined in a fixed order
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int bparts,
                                                           int M, int N, u16* __restrict__ C, int ldc,
                                                           u16* __restrict__ gb, int main_blocks) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t MN = (int64_t)M * N;
  if ((int)blockIdx.x >= main_blocks) {
    __shared__ float red[16][16];
    const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int m = ((int)blockIdx.x - main_blocks) * 16 + c;
    const float* bs = slab + (size_t)splits * MN;
    float s = 0.f;
    const int nb = splits * bparts;
    if (m < M)
      for (int k0 = g; k0 < nb; k0 += 64) {  // 4 per batch (clamped loads, in order)
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = bs[(size_t)min(k0 + 16 * u, nb - 1) * M + m];
#pragma unroll
        for (int u = 0; u < 4; ++u) s = k0 + 16 * u < nb ? s + v[u] : s;
      }
    red[g][c] = s;
    __syncthreads();
    if (g == 0 && m < M) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += red[q][c];
      gb[m] = f2bf(bf2f(gb[m]) + t);
    }
    return;
  }
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)main_blocks * 256) {
    f32x4 s = *reinterpret_cast<const f32x4*>(slab + 4 * i);
    // 4 splits per batch with unconditional (clamped) loads, added in split order: one round trip per batch
    for (int k0 = 1; k0 < splits; k0 += 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4*>(slab + (int64_t)min(k0 + u, splits - 1) * MN + 4 * i);
#pragma unroll
      for (int u = 0; u < 4; ++u) s = k0 + u < splits ? s + v[u] : s;  // (select: keeps the loads hoisted)
    }
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
  const int waves = std::max(1, knob(KNOB_WGRAD_WAVES));
  int s = 256 * waves / tiles;
  const int max_by_t = T / (8 * BK);
  if (s > max_by_t) s = max_by_t;
  return s < 1 ? 1 : s;
}

size_t wgrad_bf16_workspace_floats(int M, int N, int T) {
  const int s = wgrad_bf16_splits(M, N, T);
  const int tiles_n = (N + BN - 1) / BN;  // bias partials: splits x tiles_n rows of M (the DMA loop's layout)
  return s > 1 ? (size_t)s * M * N + (size_t)s * tiles_n * M : 0;
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
  // N fastest when gy (the M-side operand, read once per column tile in M-fastest order) cannot stay in the 256 MiB
  // Infinity Cache between its column tiles: GPT-2's lm_head, M = 50304 vocabulary rows x 16384 tokens (1.6 GB).
  // Round 6, one MI355X: 1.60 ms per lm_head weight gradient in M-fastest order (~6 TB/s: gy streamed from HBM six
  // times, gpurun_out/gpt2_r6 kernel trace); the order is knob WGRAD_NFAST (-1 auto, 0, 1)
  const int nf = knob(KNOB_WGRAD_NFAST);
  p.nfast = nf >= 0 ? nf : ((int64_t)M * T * 2 > ((int64_t)128 << 20) && p.tiles_n <= 8 ? 1 : 0);
  const dim3 grid(p.tiles_m * p.tiles_n * s);
  const bool dma = knob(KNOB_WGRAD_DMA) != 0 && T % BK == 0 &&  // (tests A/B the two loops)
                   (reinterpret_cast<uintptr_t>(gy) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  p.bparts = dma && s > 1 ? p.tiles_n : 1;
  if (dma) {
    if (gb) hipLaunchKernelGGL(wgrad_dma_kernel<true>, grid, dim3(NT), 0, stream, p);
    else hipLaunchKernelGGL(wgrad_dma_kernel<false>, grid, dim3(NT), 0, stream, p);
  } else if (gb) {
    hipLaunchKernelGGL(wgrad_kernel<true>, grid, dim3(NT), 0, stream, p);
  } else {
    hipLaunchKernelGGL(wgrad_kernel<false>, grid, dim3(NT), 0, stream, p);
  }
  if (s > 1) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    const int bblocks = gb ? (M + 15) / 16 : 0;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks + bblocks), dim3(256), 0, stream, workspace, s, p.bparts, M,
                       N, static_cast<u16*>(gw), ldc, static_cast<u16*>(gb), blocks);
  }
}

}  // namespace sdml
