// 3x3 / stride 1 / pad 1 convolution, bf16 NHWC, as implicit GEMMs on v_mfma_f32_32x32x16_bf16.
// These carry the twelve stride-1 3x3 convolutions of the ResNet-18-style stages (88 % of the
// model's MACs; models/resnet.py), replacing MIOpen for them:
//
//   forward  y[p][co]        = sum_{tap, ci} x[p + off(tap)][ci] * w[co][tap][ci]
//            GEMM M = pixels (N*H*W), N = Cout, K = 9*Cin; A = im2col(x) gathered on the fly
//            (a K-step of 64 lies inside one tap because Cin % 64 == 0: 128 contiguous bytes of
//            one shifted pixel per row, zero outside the image), B = weights [Cout][9*Cin].
//   dgrad    dx = the same kernel on dy with the flipped, transposed weights w'[ci][8-tap][co].
//   wgrad    dw[co][tap][ci] = sum_p dy[p][co] * x[p + off(tap)][ci]: M = Cout, N = 9*Cin,
//            K = pixels, both operands k-major (pixel rows), fragments through the hardware
//            transpose read; the pixel range is split over workgroups and reduced in fixed order.
//
// Forward/dgrad tiles: 512 threads, 256 pixels x BN (128, or 64 for 64-channel layers), K-step 64,
// double-buffered LDS images [rows][64] bf16 with the 16-B chunk swizzle of attention.hip
// (conflict-free row reads); the next tile's global loads are issued before the current tile's
// MFMAs and written (with the padding zeros) after them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 512, BM = 256, BK = 64;

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, static_cast<__bf16>(f)); }

// [rows][64] bf16 image, 16-B chunk ch of row r at ch ^ f(r)
__device__ __forceinline__ int swz(int r, int ch) { return r * 64 + 8 * (ch ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))); }
// A/B operand fragment, k-substep s: element j = X[row][16s + 8h + j]
__device__ __forceinline__ bf16x8 rowf(const u16* X, int row, int s, int h) {
  return *reinterpret_cast<const bf16x8*>(X + swz(row, 2 * s + h));
}

// BatchNorm backward statistics of a stored output tile: when the output is the input gradient dy of a
// training BatchNorm (x its forward input, same layout), the epilogue sums g = dy * mask and g * xhat per
// channel (xhat = (x - mean) * rstd; mask 1, y > 0 from its saved output, or x * gamma rstd + beta - mean
// gamma rstd > 0 recomputed from x, exactly as batchnorm_nhwc.hip's bn_partial_kernel), so the backward
// skips its statistics pass over dy and x.
struct BnBack {
  const u16* x = nullptr;  // null: off
  const u16* y = nullptr;  // relu 1: the saved output
  const float* mean = nullptr;
  const float* rstd = nullptr;
  const u16* gamma = nullptr;
  const u16* beta = nullptr;
  int relu = 0;  // 0 none, 1 mask from y, 2 mask recomputed from x
};

struct ConvArgs {
  const u16* x;  // NHWC input [Nb][H][W][C]
  const u16* w;  // [Co][KS*KS][C]
  u16* y;        // NHWC output [Nb][OH][OW][Co]
  int Nb, H, W, C, Co;
  int M;         // Nb*OH*OW
  int tiles_m, tiles_n;
  int OH, OW, S, KS, P;  // output size, stride, kernel size (3 or 1), padding (the halo kernel: 1 / 3 / 1)
  const u16* add;  // optional addend in y's layout: y = bf16(acc + add) (the residual branch's input gradient)
  float* part;     // optional BatchNorm partials [tiles_m][2][Co]: per-tile sums of y and y^2 (bf16-rounded y)
  BnBack bb;       // bb.x set: part holds the backward sums of g and g * xhat instead (BnBack)
};

// Output tile store shared by the im2col, halo and strided-dgrad kernels. The MFMA accumulators
// (C/D map: col = lane&31, row = (r&3) + 8(r>>2) + 4h) are rounded to bf16 into an LDS image
// [BM][BN + 8] (padded rows), then written out as 16-B row chunks: a thread owns one 8-channel chunk of
// BM / (NT / (BN / 8)) rows, so every global access is a full 16-B vector and the output row's address
// (rowoff: element offset of channel n0 of tile row r in y, < 0 = no such row) is decoded once per row,
// not once per element. EPI = 1 adds the optional addend (same layout as y; y = bf16(bf16(acc) + add),
// the rounding of the separate add it replaces) and the optional BatchNorm partials of the stored y:
// per channel, sums of y and y^2 over the tile's rows in a fixed order (the thread's rows, then the
// row groups through LDS), written to part_row[0][0..BN) and part_row[0][Co..Co+BN) - the forward
// BatchNorm (batchnorm_nhwc.hip) then finalizes these rows instead of re-reading y. With bb.x set the two sums
// are the BatchNorm backward's instead (BnBack: sums of g and g * xhat of the stored y as that BatchNorm's dy).
// LDS: max(BM * (BN + 8) * 2, 32 KB) bytes; the caller's main loop has finished with its images.
constexpr int store_tile_lds(int BN) { return BM * (BN + 8) * 2 > 32768 ? BM * (BN + 8) * 2 : 32768; }

template <int TM, int WTM, int WGM, int BN, int EPI, class RowOff>
__device__ __forceinline__ void store_tile(const f32x16 (&acc)[TM][2], int wm, int wn, int lane, u16* lds,
                                           RowOff rowoff, u16* __restrict__ y, const u16* __restrict__ add,
                                           float* __restrict__ part_row, int Co, const BnBack& bb = BnBack(),
                                           int n0 = 0) {
  constexpr int LP = BN + 8;
  constexpr int CPR = BN / 8;    // 16-B chunks per row
  constexpr int RPP = NT / CPR;  // rows per pass
  constexpr int NR = BM / RPP;   // rows per thread
  const int h = lane >> 5;
  const int t = threadIdx.x, c = t % CPR, r0 = t / CPR;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * WTM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        lds[row * LP + col] = f2bf(acc[i][j][r]);
      }
    }
  // every global operand of the thread's rows is loaded before the barrier (one memory latency for the whole
  // epilogue instead of one per row: the stores to y would otherwise order each row's loads after the last row's)
  long long offs[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) offs[k] = rowoff(r0 + k * RPP);
  const bool bwd = EPI == 1 && part_row && bb.x;
  u16x8 av[NR], xv[NR], yv[NR];
  float mu[8], rs[8], sc[8], sh[8];  // backward statistics (bb.x): this thread's 8 channels' coefficients
  if constexpr (EPI == 1) {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const long long o = (offs[k] < 0 ? 0 : offs[k]) + 8 * c;
      av[k] = add ? *reinterpret_cast<const u16x8*>(add + o) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      xv[k] = bwd ? *reinterpret_cast<const u16x8*>(bb.x + o) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      yv[k] = bwd && bb.relu == 1 ? *reinterpret_cast<const u16x8*>(bb.y + o) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    if (bwd) {
      const u16x8 gm = *reinterpret_cast<const u16x8*>(bb.gamma + n0 + 8 * c);
      const u16x8 bt = *reinterpret_cast<const u16x8*>(bb.beta + n0 + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mu[e] = bb.mean[n0 + 8 * c + e];
        rs[e] = bb.rstd[n0 + 8 * c + e];
        sc[e] = bf2f(gm[e]) * rs[e];
        sh[e] = bf2f(bt[e]) - mu[e] * sc[e];
      }
    }
  }
  __syncthreads();
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const int rr = r0 + k * RPP;
    const long long off = offs[k];
    if (off < 0) continue;
    u16x8 v = *reinterpret_cast<const u16x8*>(lds + rr * LP + 8 * c);
    if constexpr (EPI == 1) {
      if (add) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(av[k][e]));
      }
      if (bwd) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float g = bf2f(v[e]);
          const float xf = bf2f(xv[k][e]);
          if (bb.relu == 1 && !(bf2f(yv[k][e]) > 0.f)) g = 0.f;
          if (bb.relu == 2 && !(__builtin_fmaf(xf, sc[e], sh[e]) > 0.f)) g = 0.f;
          s1[e] += g;
          s2[e] += g * (xf - mu[e]) * rs[e];
        }
      } else if (part_row) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf2f(v[e]);
          s1[e] += f;
          s2[e] = __builtin_fmaf(f, f, s2[e]);
        }
      }
    }
    *reinterpret_cast<u16x8*>(y + off + 8 * c) = v;
  }
  if constexpr (EPI == 1) {
    if (!part_row) return;
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [RPP][2][BN]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(r0 * 2 + 0) * BN + 8 * c + e] = s1[e];
      red[(r0 * 2 + 1) * BN + 8 * c + e] = s2[e];
    }
    __syncthreads();
    // QN adjacent lanes per output, each summing RPP / QN row groups in order, then a fixed xor tree
    constexpr int QN = NT / (2 * BN), PER = RPP / QN;
    const int o = t / QN, q = t % QN, k = o / BN, cc = o % BN;
    float v = 0.f;
#pragma unroll
    for (int g = q * PER; g < (q + 1) * PER; ++g) v += red[(g * 2 + k) * BN + cc];
#pragma unroll
    for (int m = 1; m < QN; m <<= 1) v += __shfl_xor(v, m);
    if (q == 0) part_row[(size_t)k * Co + cc] = v;
  }
}

// the im2col / halo kernels' output: tile row r = pixel m0 + r of y [M][Co]
template <int TM, int WTM, int WGM, int BN, int EPI>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x16 (&acc)[TM][2], int tm, int m0, int n0,
                                              int wm, int wn, int lane, u16* lds) {
  const int M = a.M, Co = a.Co;
  auto rowoff = [=](int r) -> long long { return m0 + r < M ? (long long)(m0 + r) * Co + n0 : -1; };
  store_tile<TM, WTM, WGM, BN, EPI>(acc, wm, wn, lane, lds, rowoff, a.y, a.add,
                                    a.part ? a.part + (size_t)tm * 2 * Co + n0 : nullptr, Co, a.bb, n0);
}

template <int BN, int EPI>  // EPI: 0 plain store, 1 addend and/or BatchNorm partials (conv_epilogue)
__global__ void __launch_bounds__(NT) conv3x3_fwd_kernel(ConvArgs a) {
  constexpr int WGN = BN / 64;           // 2 (BN 128) or 1 (BN 64)
  constexpr int WGM = 8 / WGN;           // 4 or 8
  constexpr int WTM = BM / WGM;          // wave rows: 64 or 32
  constexpr int TM = WTM / 32;           // 2 or 1
  constexpr int AI = BM * BK, BI = BN * BK;
  constexpr int NB = BN * 8 / NT;        // B chunks per thread: 2 or 1
  __shared__ __attribute__((aligned(16))) u16 smem[2 * (AI + BI)];
  const int ntiles = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x;
  int wg = orig;
  if (ntiles >= 16) {  // XCD-aware bijective remap: neighbouring pixel tiles share an L2
    const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int tn = wg % a.tiles_n, tm = wg / a.tiles_n;  // the Cout tiles of a pixel tile are adjacent
  const int m0 = tm * BM, n0 = tn * BN;
  const int K = a.KS * a.KS * a.C;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WGM, wn = wave / WGM;
  const int t = threadIdx.x, ch = t & 7;

  // this thread's 4 A rows (pixels m0 + (t >> 3) + 64u), decoded once
  int pn[4], ph[4], pw[4];
  bool pv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = m0 + (t >> 3) + 64 * u;
    pv[u] = p < a.M;
    const int pp = pv[u] ? p : 0;
    pw[u] = pp % a.OW;
    const int q = pp / a.OW;
    ph[u] = q % a.OH;
    pn[u] = q / a.OH;
  }
  u16x8 va[4], vb[NB];
  auto inb = [&](int u, int k0) {  // is row u's shifted pixel inside the image for tap(k0)?
    const int tap = k0 / a.C;
    const int ih = ph[u] * a.S + tap / a.KS - a.P, iw = pw[u] * a.S + tap % a.KS - a.P;
    return pv[u] && k0 < K && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
  };
  auto load = [&](int k0) {
    const int tap = min(k0, K - BK) / a.C, ci0 = min(k0, K - BK) % a.C;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ih = ph[u] * a.S + tap / a.KS - a.P, iw = pw[u] * a.S + tap % a.KS - a.P;
      const bool ok = pv[u] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      const size_t off = ok ? (((size_t)pn[u] * a.H + ih) * a.W + iw) * a.C + ci0 + 8 * ch : 0;
      va[u] = *reinterpret_cast<const u16x8*>(a.x + off);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int n = n0 + (t >> 3) + 64 * u;
      vb[u] = *reinterpret_cast<const u16x8*>(a.w + (size_t)n * K + min(k0, K - BK) + 8 * ch);
    }
  };
  auto store = [&](u16* L, int k0) {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<u16x8*>(L + swz((t >> 3) + 64 * u, ch)) = inb(u, k0) ? va[u] : z;
#pragma unroll
    for (int u = 0; u < NB; ++u) *reinterpret_cast<u16x8*>(L + AI + swz((t >> 3) + 64 * u, ch)) = vb[u];
  };

  f32x16 acc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = K / BK;
  load(0);
  store(smem, 0);
  load(BK);
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const u16* L = smem + (it & 1) * (AI + BI);
    u16* Ln = smem + ((it + 1) & 1) * (AI + BI);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[TM], bf[2];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = rowf(L, wm * WTM + 32 * i + (lane & 31), s, h);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = rowf(L + AI, wn * 64 + 32 * j + (lane & 31), s, h);
      if (s == 0) {  // tile it+1 -> other buffer (its readers passed the last barrier); it+2 -> regs
        store(Ln, (it + 1) * BK);
        load((it + 2) * BK);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(af[i], bf[j], acc[i][j]);
    }
    __syncthreads();
  }
  conv_epilogue<TM, WTM, WGM, BN, EPI>(a, acc, tm, m0, n0, wm, wn, lane, smem);
}

// ---- input gradient of a stride-2 convolution (3x3 pad 1 / 1x1 pad 0): parity-class GEMMs ------
// dx[n][iy][ix][ci] = sum over (ky, kx, co) with iy + P - ky = 2 oy, ix + P - kx = 2 ox of
// dy[n][oy][ox][co] * w[co][ci][ky][kx]. Which taps reach an input pixel depends only on the parity
// (py, px) of (iy, ix): ky = ky0 + 2j with ky0 = (py + P) & 1 (3x3 pad 1: one tap for even rows, two
// for odd ones; 1x1 pad 0: one for even rows, none for odd ones). Each of the four parity classes is
// a dense implicit GEMM - M = its pixels, N = Cin, K = its taps x Cout, A gathered from dy (a K-step
// of 64 lies inside one tap), B = the class's weights packed [Cin][taps][Cout] - so no MAC is spent
// on the zeros of the transposed convolution, and one launch covers all four classes (class-major
// tile order, most taps first; a class without taps writes its zeros through the same epilogue).
struct DgArgs {
  const u16* dy;  // [Nb][OH][OW][Cg] (the convolution's output gradient, NHWC)
  const u16* w;   // the classes' packed weights, class-major in dg_order, each [Cn][taps][Cg]
  u16* dx;        // [Nb][H][W][Cn]
  const u16* add;  // optional addend in dx's layout (dx = bf16(acc + add))
  int Nb, H, W, OH, OW, Cg, Cn, KS, P, tiles_n, tiles;
  float* part;     // optional BatchNorm backward partials of dx (BnBack), one row per class pixel tile:
  BnBack bb;       // [sum over classes of tiles_m][2][Cn], the classes in dg_order
};

struct DgClass {
  int py, px, ky0, kx0, nkx, taps, Ha, Wb, M, tiles_m, woff, tile0;
};

// class processed j-th: most taps first (3x3: (1,1) 4, (0,1) 2, (1,0) 2, (0,0) 1; 1x1: (0,0) only)
__host__ __device__ inline int dg_order(int j, int KS) { return KS == 3 ? (j == 0 ? 3 : j == 3 ? 0 : j) : j; }

__host__ __device__ inline DgClass dg_class(int j, int Nb, int H, int W, int KS, int P, int Cg, int Cn, int tiles_n) {
  DgClass c{};
  int woff = 0, tile0 = 0;
  for (int i = 0; i <= j; ++i) {
    const int cls = dg_order(i, KS);
    c.py = cls >> 1;
    c.px = cls & 1;
    c.ky0 = (c.py + P) & 1;
    c.kx0 = (c.px + P) & 1;
    const int nky = (KS - c.ky0 + 1) / 2;
    c.nkx = (KS - c.kx0 + 1) / 2;
    c.taps = nky * c.nkx;
    c.Ha = (H - c.py + 1) / 2;
    c.Wb = (W - c.px + 1) / 2;
    c.M = Nb * c.Ha * c.Wb;
    c.tiles_m = (c.M + BM - 1) / BM;
    c.woff = woff;
    c.tile0 = tile0;
    woff += c.taps * Cn * Cg;
    tile0 += c.tiles_m * tiles_n;
  }
  return c;
}

template <int BN>
__global__ void __launch_bounds__(NT) conv_dgrad_s2_kernel(DgArgs a) {
  constexpr int WGN = BN / 64;
  constexpr int WGM = 8 / WGN;
  constexpr int WTM = BM / WGM;
  constexpr int TM = WTM / 32;
  constexpr int AI = BM * BK, BI = BN * BK;
  constexpr int NB = BN * 8 / NT;
  __shared__ __attribute__((aligned(16))) u16 smem[2 * (AI + BI)];
  const int orig = blockIdx.x;
  int wg = orig;
  if (a.tiles >= 16) {  // XCD-aware bijective remap
    const int q = a.tiles / 8, r = a.tiles % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  int j = 0;
  DgClass c = dg_class(0, a.Nb, a.H, a.W, a.KS, a.P, a.Cg, a.Cn, a.tiles_n);
  for (int jj = 1; jj < 4; ++jj) {
    const DgClass d = dg_class(jj, a.Nb, a.H, a.W, a.KS, a.P, a.Cg, a.Cn, a.tiles_n);
    if (wg >= d.tile0 && d.tiles_m > 0) {
      c = d;
      j = jj;
    }
  }
  (void)j;
  const int local = wg - c.tile0;
  const int tn = local % a.tiles_n, tm = local / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int K = c.taps * a.Cg;
  const u16* __restrict__ wc = a.w + c.woff;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WGM, wn = wave / WGM;
  const int t = threadIdx.x, ch = t & 7;

  int pn[4], py[4], px[4];  // this thread's 4 A rows: image, input row / column of the class pixel
  bool pv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int p = m0 + (t >> 3) + 64 * u;
    pv[u] = p < c.M;
    const int pp = pv[u] ? p : 0;
    px[u] = 2 * (pp % c.Wb) + c.px;
    const int q = pp / c.Wb;
    py[u] = 2 * (q % c.Ha) + c.py;
    pn[u] = q / c.Ha;
  }
  u16x8 va[4], vb[NB];
  bool ok[4];
  auto load = [&](int k0) {
    const int kk = min(k0, K - BK);
    const int tt = kk / a.Cg, co0 = kk % a.Cg;
    const int ky = c.ky0 + 2 * (tt / c.nkx), kx = c.kx0 + 2 * (tt % c.nkx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int dh = py[u] + a.P - ky, dw = px[u] + a.P - kx;  // even by the class
      const int oy = dh >> 1, ox = dw >> 1;
      ok[u] = pv[u] && k0 < K && dh >= 0 && oy < a.OH && dw >= 0 && ox < a.OW;
      const size_t off = ok[u] ? (((size_t)pn[u] * a.OH + oy) * a.OW + ox) * a.Cg + co0 + 8 * ch : 0;
      va[u] = *reinterpret_cast<const u16x8*>(a.dy + off);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int n = n0 + (t >> 3) + 64 * u;
      vb[u] = *reinterpret_cast<const u16x8*>(wc + (size_t)n * K + kk + 8 * ch);
    }
  };
  auto store = [&](u16* L) {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<u16x8*>(L + swz((t >> 3) + 64 * u, ch)) = ok[u] ? va[u] : z;
#pragma unroll
    for (int u = 0; u < NB; ++u) *reinterpret_cast<u16x8*>(L + AI + swz((t >> 3) + 64 * u, ch)) = vb[u];
  };

  f32x16 acc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][jn][r] = 0.f;

  const int nk = K / BK;
  if (nk > 0) {
    load(0);
    store(smem);
    load(BK);
    __syncthreads();
    for (int it = 0; it < nk; ++it) {
      const u16* L = smem + (it & 1) * (AI + BI);
      u16* Ln = smem + ((it + 1) & 1) * (AI + BI);
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 af[TM], bf[2];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = rowf(L, wm * WTM + 32 * i + (lane & 31), s, h);
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) bf[jn] = rowf(L + AI, wn * 64 + 32 * jn + (lane & 31), s, h);
        if (s == 0) {
          store(Ln);
          load((it + 2) * BK);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int jn = 0; jn < 2; ++jn) acc[i][jn] = mfma(af[i], bf[jn], acc[i][jn]);
      }
      __syncthreads();
    }
  }
  const int H = a.H, W = a.W, Cn = a.Cn, Ha = c.Ha, Wb = c.Wb, cpy = c.py, cpx = c.px, Mc = c.M;
  auto rowoff = [=](int r) -> long long {  // class pixel m0 + r -> dx element offset of channel n0
    const int p = m0 + r;
    if (p >= Mc) return -1;
    const int ix = 2 * (p % Wb) + cpx, q = p / Wb;
    const int iy = 2 * (q % Ha) + cpy, n = q / Ha;
    return (((long long)n * H + iy) * W + ix) * Cn + n0;
  };
  float* prow = a.part ? a.part + ((size_t)(c.tile0 / a.tiles_n + tm) * 2 * Cn + n0) : nullptr;
  store_tile<TM, WTM, WGM, BN, 1>(acc, wm, wn, lane, smem, rowoff, a.dx, a.add, prow, Cn, a.bb, n0);
}

// torch weight [Cg][Cn][KS][KS] -> the parity classes' packed [Cn][taps][Cg] images (dg_class)
__global__ void __launch_bounds__(256) conv_dgrad_s2_weight_kernel(const u16* __restrict__ w, u16* __restrict__ out,
                                                                   int Cg, int Cn, int KS, int P) {
  const int64_t n = (int64_t)Cg * Cn * KS * KS;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    DgClass c = dg_class(0, 1, 2, 2, KS, P, Cg, Cn, 1);
    for (int j = 1; j < 4; ++j) {
      const DgClass d = dg_class(j, 1, 2, 2, KS, P, Cg, Cn, 1);
      if (e >= d.woff && d.taps > 0) c = d;
    }
    const int64_t r = e - c.woff;  // [ci][t][co]
    const int co = (int)(r % Cg);
    const int64_t q = r / Cg;
    const int tt = (int)(q % c.taps), ci = (int)(q / c.taps);
    const int ky = c.ky0 + 2 * (tt / c.nkx), kx = c.kx0 + 2 * (tt % c.nkx);
    out[e] = w[(((int64_t)co * Cn + ci) * KS + ky) * KS + kx];
  }
}

// ---- forward / dgrad, halo-staged ("direct") variant ------------------------------------------
// The im2col kernel above re-reads every input pixel once per tap (9x the input bytes through L2
// per output tile). This one stages, per 64-channel chunk, the block's BM output pixels plus a
// halo of W + 1 flattened pixels on either side ([m0 - W - 1, m0 + BM + W + 1), the only input
// rows any tap of the tile touches) in LDS once; the nine taps are then row-shifted reads of that
// image (row = pixel + dh * W + dw), zeroed per lane where the shifted pixel leaves the image.
// Steps run chunk-major, tap-minor; the weight tile of step st + 1 is stored (and st + 2 loaded)
// during step st, the halo of chunk cc + 1 is stored at tap 4 of chunk cc (its buffer's readers
// finished with chunk cc - 1) and chunk cc + 2's halo loaded into registers then.
// HL = 16-B halo chunks per thread: 5 covers W <= 31 (halo rows <= 320), 7 covers W <= 95 (448).
// The 64-channel-tile, HL = 5 form fits 128 VGPRs: two workgroups (4 waves per SIMD) per CU.
constexpr int HALO_MAX_W = 95;
constexpr int halo_hl(int W) { return (BM + 2 * W + 2) * 8 <= 5 * NT ? 5 : 7; }
constexpr int halo_occ(int BN, int HL) { return BN == 64 && HL == 5 ? 4 : 2; }

template <int BN, int HL, int EPI>
__global__ void __launch_bounds__(NT, halo_occ(BN, HL)) conv3x3_halo_kernel(ConvArgs a) {
  constexpr int WGN = BN / 64;
  constexpr int WGM = 8 / WGN;
  constexpr int WTM = BM / WGM;
  constexpr int TM = WTM / 32;
  constexpr int BI = BN * BK;
  constexpr int NB = BN * 8 / NT;
  extern __shared__ __attribute__((aligned(16))) u16 dsm[];
  const int HR = BM + 2 * a.W + 2;  // halo rows
  // one halo buffer when C == 64 (a single chunk): 56 KB at W = 28, two workgroups per CU
  const int nhb = a.C > 64 ? 2 : 1;
  u16* const HB[2] = {dsm, dsm + (nhb - 1) * HR * 64};
  u16* const BB[2] = {dsm + nhb * HR * 64, dsm + nhb * HR * 64 + BI};
  const int ntiles = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x;
  int wg = orig;
  if (ntiles >= 16) {
    const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int tn = wg % a.tiles_n, tm = wg / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int K = 9 * a.C;
  const int nch = a.C / 64, NS = 9 * nch;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WGM, wn = wave / WGM;
  const int t = threadIdx.x, ch = t & 7;

  // this lane's A rows: local row lr[i]; vm[i] bit tap = shifted pixel inside the image
  int lr[TM];
  unsigned vm[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    lr[i] = wm * WTM + 32 * i + (lane & 31);
    const int p = min(m0 + lr[i], a.M - 1);
    const int pw = p % a.W, q = p / a.W, ph = q % a.H;
    unsigned m = 0;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int ih = ph + tp / 3 - 1, iw = pw + tp % 3 - 1;
      m |= (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) ? (1u << tp) : 0u;
    }
    vm[i] = m;
  }

  u16x8 vh[HL], vb[2][NB];  // weight tiles: two register sets, loaded 2 steps before their store
  const int hbase = m0 - a.W - 1;
  auto load_halo = [&](int cc) {
#pragma unroll
    for (int u = 0; u < HL; ++u) {
      const int id = t + NT * u;
      // clamped rows (outside [0, M) or past the halo) load valid memory that no unmasked tap reads;
      // unconditional, so the compiler does not wait on each load separately
      const int q = min(max(hbase + (id >> 3), 0), a.M - 1);
      vh[u] = *reinterpret_cast<const u16x8*>(a.x + (size_t)q * a.C + cc * 64 + 8 * (id & 7));
    }
  };
  auto store_halo = [&](u16* L) {
#pragma unroll
    for (int u = 0; u < HL; ++u) {
      const int id = t + NT * u;
      if (id < HR * 8) *reinterpret_cast<u16x8*>(L + swz(id >> 3, id & 7)) = vh[u];
    }
  };
  auto load_b = [&](u16x8* v, int st) {
    st = min(st, NS - 1);
    const int cc = st / 9, tap = st % 9;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int n = n0 + (t >> 3) + 64 * u;
      v[u] = *reinterpret_cast<const u16x8*>(a.w + (size_t)n * K + tap * a.C + cc * 64 + 8 * ch);
    }
  };
  auto store_b = [&](u16* L, const u16x8* v) {
#pragma unroll
    for (int u = 0; u < NB; ++u) *reinterpret_cast<u16x8*>(L + swz((t >> 3) + 64 * u, ch)) = v[u];
  };

  f32x16 acc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_halo(0);
  load_b(vb[0], 0);
  store_halo(HB[0]);
  store_b(BB[0], vb[0]);
  load_b(vb[1], 1);
  load_b(vb[0], 2);
  if (nch > 1) load_halo(1);
  __syncthreads();
  const bf16x8 zf = {0, 0, 0, 0, 0, 0, 0, 0};
  // step st stores weight tile st + 1 (register set (st + 1) & 1) and refills that set with
  // tile st + 3; the parity is a template constant so the register sets stay in registers
  auto step = [&](auto parity, int st) {
    constexpr int P = decltype(parity)::value;
    const int cc = st / 9, tap = st % 9;
    const u16* HA = HB[cc & 1];
    const u16* L = BB[P];
    const int shift = (tap / 3) * a.W + tap % 3;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[TM], bf[2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 v = rowf(HA, lr[i] + shift, s, h);
        af[i] = ((vm[i] >> tap) & 1) ? v : zf;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = rowf(L, wn * 64 + 32 * j + (lane & 31), s, h);
      if (s == 0) {
        store_b(BB[P ^ 1], vb[P ^ 1]);
        load_b(vb[P ^ 1], st + 3);
        if (tap == 4 && cc + 1 < nch) {
          store_halo(HB[(cc + 1) & 1]);
          if (cc + 2 < nch) load_halo(cc + 2);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(af[i], bf[j], acc[i][j]);
    }
    __syncthreads();
  };
  int st = 0;
  for (; st + 1 < NS; st += 2) {  // NS = 9 * nch is odd for odd nch: one tail step
    step(std::integral_constant<int, 0>(), st);
    step(std::integral_constant<int, 1>(), st + 1);
  }
  if (st < NS) step(std::integral_constant<int, 0>(), st);
  conv_epilogue<TM, WTM, WGM, BN, EPI>(a, acc, tm, m0, n0, wm, wn, lane, dsm);
}

// ---- weight gradient: dw[co][tap][ci] (fp32 slabs) = sum_p dy[p][co] x[p + off(tap)][ci] ---------
// tile 128 (co) x 128 (tap, ci), K-step 64 pixels; both operands k-major images [64][128] read by
// ds_read_b64_tr_b16 (same image/swizzle as gemm_bf16_wgrad.hip)
__device__ __forceinline__ int km_off(int k, int c) { return k * 128 + 8 * (c ^ (((k & 3) << 2) | ((k >> 2) & 3))); }
__device__ __forceinline__ s16x4 ds_tr16(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}
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

struct WgArgs {
  const u16* dy;  // [M][Co] (NHWC output gradient, M = Nb*OH*OW)
  const u16* x;   // [Nb][H][W][C] (NHWC)
  float* slab;    // [splits][Co][KS*KS*C]
  int Nb, H, W, C, Co, M;
  int OH, OW, S, KS, P;
  int pps;        // pixels per split (multiple of 64)
  int tiles_m, tiles_n, splits;
};

template <int TMR>  // output-channel rows per tile: 128 (waves 64 x 32) or 64 (waves 32 x 32; Cout = 64)
__global__ void __launch_bounds__(NT) conv3x3_wgrad_kernel(WgArgs a) {
  constexpr int IMG = 64 * 128;
  constexpr int TI = TMR / 64;       // 32-row blocks per wave
  constexpr int ACPR = TMR / 8;      // dy chunks per pixel row of the tile
  constexpr int NA = 64 * ACPR / NT;  // dy chunks per thread per K-step
  __shared__ __attribute__((aligned(16))) u16 smem[2 * 2 * IMG];
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nwg = ntiles * a.splits;
  const int orig = blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % a.tiles_m, tn = tile / a.tiles_m;
  const int m0 = tm * TMR, n0 = tn * 128;  // m: co, n: tap*C + ci
  const int K9 = a.KS * a.KS * a.C;  // GEMM N: (tap, ci)
  const int pbeg = split * a.pps, pend = min(a.M, pbeg + a.pps);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;  // 2 x 4 waves: TMR / 2 (co) x 32 (n) each
  const int t = threadIdx.x;
  // per K-step: the dy tile is 64 pixels x TMR channels, the x tile 64 pixels x 128 columns (2 16-B
  // chunks per thread: pixel row kk = id >> 4, 8-column chunk c = id & 15)
  u16x8 va[NA], vb[2];
  unsigned okb = 0;  // bit u: chunk u of vb is inside the image (zeroed at store time otherwise)
  // this thread's x chunks: one column chunk (tap, ci fixed) on pixel rows kk0 and kk0 + 32; the
  // pixel coordinates advance by 64 pixels per K-step incrementally (no integer division in the loop)
  const int kk0 = t >> 4, cb = t & 15;
  const int nb_col = min(n0 + 8 * cb, K9 - 8);
  const int tap = nb_col / a.C, ci = nb_col % a.C, dh = tap / a.KS - a.P, dw = tap % a.KS - a.P;
  const int HW = a.OH * a.OW;  // output-pixel coordinates (the GEMM's K axis)
  const int st_n = 64 / HW, st_h = (64 % HW) / a.OW, st_w = 64 % a.OW;
  int pn[2], ph[2], pw[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = pbeg + kk0 + 32 * u;
    pw[u] = p % a.OW;
    ph[u] = (p / a.OW) % a.OH;
    pn[u] = p / HW;
  }
  auto load = [&](int p0) {
    okb = 0;
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int id = t + NT * u, kk = id / ACPR, c = id % ACPR;
      const int p = min(p0 + kk, a.M - 1);
      va[u] = *reinterpret_cast<const u16x8*>(a.dy + (size_t)p * a.Co + min(m0 + 8 * c, a.Co - 8));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int ih = ph[u] * a.S + dh, iw = pw[u] * a.S + dw;
      const bool ok = pn[u] < a.Nb && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      vb[u] = *reinterpret_cast<const u16x8*>(a.x + (ok ? (((size_t)pn[u] * a.H + ih) * a.W + iw) * a.C + ci : 0));
      okb |= ok ? (1u << u) : 0u;
      pw[u] += st_w;  // next call loads the rows 64 pixels further
      if (pw[u] >= a.OW) {
        pw[u] -= a.OW;
        ++ph[u];
      }
      ph[u] += st_h;
      if (ph[u] >= a.OH) {
        ph[u] -= a.OH;
        ++pn[u];
      }
      pn[u] += st_n;
    }
  };
  auto store = [&](u16* L, int p0) {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int id = t + NT * u, kk = id / ACPR, c = id % ACPR;
      *reinterpret_cast<u16x8*>(L + km_off(kk, c)) = p0 + kk < pend ? va[u] : z;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = t + NT * u, kk = id >> 4, c = id & 15;
      const bool in = p0 + kk < pend;
      *reinterpret_cast<u16x8*>(L + IMG + km_off(kk, c)) = (in && ((okb >> u) & 1)) ? vb[u] : z;
    }
  };
  f32x16 acc[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int nk = (pend - pbeg + 63) / 64;
  if (nk > 0) {
    load(pbeg);
    store(smem, pbeg);
    load(pbeg + 64);
  }
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const u16* L = smem + (it & 1) * 2 * IMG;
    u16* Ln = smem + ((it + 1) & 1) * 2 * IMG;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 af[TI], bfr;
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = trfrag(L, wm * (TMR / 2) + 32 * i, s, lane);
      bfr = trfrag(L + IMG, wn * 32, s, lane);
      if (s == 0) {
        store(Ln, pbeg + (it + 1) * 64);
        load(pbeg + (it + 2) * 64);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) acc[i] = mfma(af[i], bfr, acc[i]);
    }
    __syncthreads();
  }
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= K9) return;
  float* S = a.slab + (size_t)split * a.Co * K9;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * (TMR / 2) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < a.Co) S[(size_t)co * K9 + col] = acc[i][r];
    }
}

// ---- LDS-DMA form of the weight gradient (opt-in: SDML_CONV_WGRAD_DMA=1) ---------------------------
// Measured on ResNet-18 bf16 (batch 512, one MI355X): 40.6 us vs the staged loop's 40.9 for the 128-row
// tile, 78.9 vs 72.4 for the 64-row one, the 3-stage ring slower still (4.89 vs 4.57 ms per step) — unlike
// the dense weight gradients (gemm_bf16_wgrad.hip), this loop is not bound by the LDS staging writes, so
// the staged loop stays the default.
// Same tile, waves, images and slab as conv3x3_wgrad_kernel, but both images are filled by
// global_load_lds (16 B per lane, 2 + 2 instructions per wave per K-step) into a 3-stage ring with two
// K-steps in flight and one counted vmcnt(4) + barrier per K-step: no VGPR staging and no ds_write of
// the 32 KiB per K-step. A DMA instruction writes 4 image rows lane-linearly, so lane l owns rows
// 4 wave + l/16 (+ 32) and the logical chunk (l % 16) ^ swz(row) of both images (swz(r) = swz(r + 32)).
// Taps outside the image, pixels past the split and dy rows past it read a zero page in global memory
// (a DMA cannot zero-fill). Fragments by inline-asm transposed reads (the builtin made the compiler wait
// for every DMA in flight before each read), lgkmcnt waited explicitly.
__device__ __attribute__((aligned(16))) u16 g_zero16[8] = {0, 0, 0, 0, 0, 0, 0, 0};

__device__ __forceinline__ void glds16(const void* src, u16* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

__device__ __forceinline__ s16x4 ds_tr16_asm(const u16* p) {
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) u16*)p;
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

template <int NR>
__device__ __forceinline__ void lgkm_wait6(s16x4 (&f)[6]) {
  asm volatile("s_waitcnt lgkmcnt(%6)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5])
               : "n"(NR));
}

// NSTG = 2: 64 KiB of LDS, two workgroups per CU, one K-step in flight; 3: 96 KiB, one workgroup, two
template <int TMR, int NSTG>
__global__ void __launch_bounds__(NT) conv3x3_wgrad_dma_kernel(WgArgs a) {
  constexpr int IMG = 64 * 128;
  constexpr int TI = TMR / 64;
  constexpr int NR = 2 * (TI + 1);  // transposed reads per substep
  constexpr int BUF = 2 * IMG;      // A (dy) image, B (x) image
  __shared__ __attribute__((aligned(16))) u16 smem[NSTG * BUF];
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nwg = ntiles * a.splits;
  const int orig = blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % a.tiles_m, tn = tile / a.tiles_m;
  const int m0 = tm * TMR, n0 = tn * 128;
  const int K9 = a.KS * a.KS * a.C;
  const int pbeg = split * a.pps, pend = min(a.M, pbeg + a.pps);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  // this lane's DMA rows r0 = 4 wave + lane / 16 and r0 + 32, logical chunk c of both images
  const int r0 = 4 * wave + (lane >> 4);
  const int c = (lane & 15) ^ (((r0 & 3) << 2) | ((r0 >> 2) & 3));
  const int acol = min(m0 + 8 * c, a.Co - 8);
  const int nb_col = min(n0 + 8 * c, K9 - 8);
  const int tap = nb_col / a.C, ci = nb_col % a.C, dh = tap / a.KS - a.P, dw = tap % a.KS - a.P;
  const int HW = a.OH * a.OW;
  const int st_n = 64 / HW, st_h = (64 % HW) / a.OW, st_w = 64 % a.OW;
  int pn[2], ph[2], pw[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = pbeg + r0 + 32 * u;
    pw[u] = p % a.OW;
    ph[u] = (p / a.OW) % a.OH;
    pn[u] = p / HW;
  }
  int pnext = pbeg;  // first pixel of the next K-step to issue
  auto issue = [&](u16* st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = pnext + r0 + 32 * u;
      const bool in = p < pend;
      glds16(in ? a.dy + (size_t)p * a.Co + acol : g_zero16, st + (wave + 8 * u) * 512);
      const int ih = ph[u] * a.S + dh, iw = pw[u] * a.S + dw;
      const bool ok = in && pn[u] < a.Nb && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      glds16(ok ? a.x + (((size_t)pn[u] * a.H + ih) * a.W + iw) * a.C + ci : g_zero16,
             st + IMG + (wave + 8 * u) * 512);
      pw[u] += st_w;
      if (pw[u] >= a.OW) {
        pw[u] -= a.OW;
        ++ph[u];
      }
      ph[u] += st_h;
      if (ph[u] >= a.OH) {
        ph[u] -= a.OH;
        ++pn[u];
      }
      pn[u] += st_n;
    }
    pnext += 64;
  };
  f32x16 acc[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const int nk = (pend - pbeg + 63) / 64;
  if (nk > 0) {
    issue(smem);
    if constexpr (NSTG == 3) {
      issue(smem + BUF);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // fragment read addresses: trfrag's (k, col) for the A blocks (wm * TMR/2 + 32 i) and the B block (wn * 32)
  const int g = lane >> 4, il = lane & 15, qq = il >> 2, pp = il & 3;
  auto rd = [&](const u16* L, int s, s16x4 (&f)[6]) {
    const int k = 16 * s + 8 * (g >> 1) + qq;
#pragma unroll
    for (int x = 0; x <= TI; ++x) {
      const u16* P = x < TI ? L : L + IMG;
      const int col = (x < TI ? wm * (TMR / 2) + 32 * x : wn * 32) + 16 * (g & 1) + 4 * pp;
      f[2 * x] = ds_tr16_asm(P + km_off(k, col >> 3) + (col & 7));
      f[2 * x + 1] = ds_tr16_asm(P + km_off(k + 4, col >> 3) + (col & 7));
    }
  };
  for (int it = 0; it < nk; ++it) {
    const u16* L = smem + (it % NSTG) * BUF;
    issue(smem + ((it + NSTG - 1) % NSTG) * BUF);
    s16x4 fr[2][6];
    rd(L, 0, fr[0]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s < 3) {
        rd(L, s + 1, fr[(s + 1) & 1]);
        lgkm_wait6<NR>(fr[s & 1]);
      } else {
        lgkm_wait6<0>(fr[s & 1]);
      }
      const s16x4* f = fr[s & 1];
      const bf16x8 bfr = {f[2 * TI][0], f[2 * TI][1], f[2 * TI][2], f[2 * TI][3],
                          f[2 * TI + 1][0], f[2 * TI + 1][1], f[2 * TI + 1][2], f[2 * TI + 1][3]};
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const bf16x8 af = {f[2 * i][0], f[2 * i][1], f[2 * i][2], f[2 * i][3],
                           f[2 * i + 1][0], f[2 * i + 1][1], f[2 * i + 1][2], f[2 * i + 1][3]};
        acc[i] = mfma(af, bfr, acc[i]);
      }
    }
    if constexpr (NSTG == 3) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-the-end stages (zero-page reads)
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= K9) return;
  float* S = a.slab + (size_t)split * a.Co * K9;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * (TMR / 2) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < a.Co) S[(size_t)co * K9 + col] = acc[i][r];
    }
}

// gw[co][ci][kh][kw] (bf16, torch layout, accumulated) += sum_s slab[s][co][tap][ci]. A block is 32
// float4 outputs (slab order, coalesced) x 8 split groups: group g sums splits g, g + 8, ... in
// order, then the 8 partials are added in fixed order through LDS (deterministic); the 4 results
// of a thread are scattered to the torch layout.
constexpr int RD_OUT = 32, RD_GRP = 8;

__global__ void __launch_bounds__(RD_OUT * RD_GRP) conv_wgrad_reduce_kernel(const float* __restrict__ slab, int splits,
                                                                           int Co, int C, int T, u16* __restrict__ gw) {
  __shared__ float4 red[RD_GRP][RD_OUT];
  const int64_t n = (int64_t)Co * T * C, n4 = n / 4;
  const int o = threadIdx.x % RD_OUT, g = threadIdx.x / RD_OUT;
  for (int64_t base = (int64_t)blockIdx.x * RD_OUT; base < n4; base += (int64_t)gridDim.x * RD_OUT) {
    const int64_t i = base + o;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n4)
      // 4 splits per batch, loads unconditional (clamped split, the extra terms dropped by a select) so they
      // are in flight together; the sum order is unchanged (k = g, g + RD_GRP, ... in sequence)
      for (int k0 = g; k0 < splits; k0 += 4 * RD_GRP) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = reinterpret_cast<const float4*>(slab + (size_t)min(k0 + RD_GRP * u, splits - 1) * n)[i];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool in = k0 + RD_GRP * u < splits;  // (a select, not a branch: keeps the loads hoisted)
          acc.x = in ? acc.x + v[u].x : acc.x;
          acc.y = in ? acc.y + v[u].y : acc.y;
          acc.z = in ? acc.z + v[u].z : acc.z;
          acc.w = in ? acc.w + v[u].w : acc.w;
        }
      }
    red[g][o] = acc;
    __syncthreads();
    if (g == 0 && i < n4) {
      float4 t = red[0][o];
#pragma unroll
      for (int gg = 1; gg < RD_GRP; ++gg) {
        t.x += red[gg][o].x;
        t.y += red[gg][o].y;
        t.z += red[gg][o].z;
        t.w += red[gg][o].w;
      }
      const int64_t e = 4 * i;  // slab layout [co][tap][ci]
      const int ci = (int)(e % C);
      const int64_t r = e / C;
      const int tap = (int)(r % T), co = (int)(r / T);
      const float sv[4] = {t.x, t.y, t.z, t.w};
      u16 old[4];  // the 4 reads first (before any store: the compiler cannot tell the addresses apart)
#pragma unroll
      for (int j = 0; j < 4; ++j) old[j] = gw[((int64_t)co * C + ci + j) * T + tap];
#pragma unroll
      for (int j = 0; j < 4; ++j) gw[((int64_t)co * C + ci + j) * T + tap] = f2bf(bf2f(old[j]) + sv[j]);
    }
    __syncthreads();
  }
}

// torch weight [co][ci][3][3] -> the forward layout [co][tap][ci] and/or the dgrad layout
// [ci][8 - tap][co] (either output may be null)
// element-wise: one load, two stores per weight element (8.8 us per call at ResNet's shapes). A 64 x 64 x 9 LDS-tile
// form (128-byte rows on both outputs) measured slower in round 4 (ResNet step 4.49 -> 4.87 ms): 64 workgroups at
// 512 channels, each thread's 144 tile loads waited out one by one
__global__ void __launch_bounds__(256) conv_weight_transform_kernel(const u16* __restrict__ w, u16* __restrict__ fwd,
                                                                    u16* __restrict__ dgrad, int Co, int C) {
  const int64_t n = (int64_t)Co * C * 9;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int tap = (int)(i % 9);
    const int64_t r = i / 9;
    const int ci = (int)(r % C), co = (int)(r / C);
    const u16 v = w[i];
    if (fwd) fwd[((int64_t)co * 9 + tap) * C + ci] = v;
    if (dgrad) dgrad[((int64_t)ci * 9 + (8 - tap)) * Co + co] = v;
  }
}

// every 3x3 weight of a step in one launch (ResNet-18: 16 weights, 16 launches of ~9 us, mostly launch latency):
// block b works on the weight whose block range holds it (a uniform scan of the kernel-argument table)
struct WtBatch {
  const u16* w[kWtBatchMax];
  u16* fwd[kWtBatchMax];
  u16* dgrad[kWtBatchMax];
  int Co[kWtBatchMax], C[kWtBatchMax], block0[kWtBatchMax + 1];
  int n;
};

// A block transposes a tile of 32 output x 32 input channels through LDS: it reads the 32 rows of 32 x 9
// contiguous weights (576 B each) and writes 64-B runs of both layouts (fwd [co][tap][ci0..+31], dgrad
// [ci][8 - tap][co0..+31]); an element-wise loop wrote each layout with 2-byte stores strided by C or 9 Co (36 us
// for ResNet-18's 11M weights, most of it write amplification).
constexpr int WT_T = 32;

__global__ void __launch_bounds__(256) conv_weight_transform_batched_kernel(WtBatch b) {
  __shared__ u16 tile[WT_T][WT_T * 9 + 2];  // [co][ci * 9 + tap] (+2: row starts on distinct banks)
  int k = 0;
  for (int j = 1; j < b.n; ++j) k = (int)blockIdx.x >= b.block0[j] ? j : k;
  const int Co = b.Co[k], C = b.C[k];
  const int tiles_c = (C + WT_T - 1) / WT_T;
  const int t = blockIdx.x - b.block0[k];
  const int co0 = (t / tiles_c) * WT_T, ci0 = (t % tiles_c) * WT_T;
  const int nco = min(WT_T, Co - co0), nci = min(WT_T, C - ci0);
  const u16* w = b.w[k];
  for (int i = threadIdx.x; i < WT_T * WT_T * 9; i += 256) {
    const int r = i / (WT_T * 9), c = i % (WT_T * 9);
    if (r < nco && c < nci * 9) tile[r][c] = w[((int64_t)(co0 + r) * C + ci0) * 9 + c];
  }
  __syncthreads();
  u16* fwd = b.fwd[k];
  for (int i = threadIdx.x; i < WT_T * 9 * WT_T; i += 256) {  // fwd: (co, tap) rows of ci0..
    const int ci = i % WT_T, rt = i / WT_T, tap = rt % 9, co = rt / 9;
    if (co < nco && ci < nci) fwd[((int64_t)(co0 + co) * 9 + tap) * C + ci0 + ci] = tile[co][ci * 9 + tap];
  }
  u16* dgrad = b.dgrad[k];
  if (dgrad) {
    for (int i = threadIdx.x; i < WT_T * 9 * WT_T; i += 256) {  // dgrad: (ci, tap) rows of co0..
      const int co = i % WT_T, rt = i / WT_T, tap = rt % 9, ci = rt / 9;
      if (co < nco && ci < nci) dgrad[((int64_t)(ci0 + ci) * 9 + (8 - tap)) * Co + co0 + co] = tile[co][ci * 9 + tap];
    }
  }
}

// ---- stem: one input channel (MNIST), 3x3 / stride 1 / pad 1 -----------------------------------
// K = 9 is far too short for the matrix cores: both passes are plain streaming kernels at the
// output/gradient bandwidth. Forward: a thread owns 16 output channels of one pixel (weights in
// LDS as fp32 [tap][co]); it writes NHWC directly, so no layout copy follows (MIOpen produced NCHW
// here, 68 us + a 24 us channels-last copy at batch 512).
constexpr int STEM_T = 256;

__global__ void __launch_bounds__(STEM_T) conv_c1_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ w,
                                                             u16* __restrict__ y, int Nb, int H, int W, int Co) {
  __shared__ float ws[9 * 512];
  for (int i = threadIdx.x; i < 9 * Co; i += STEM_T) {  // w [co][tap] -> ws [tap][co]
    const int co = i / 9, tap = i % 9;
    ws[tap * Co + co] = bf2f(w[i]);
  }
  __syncthreads();
  const int G = Co / 16;
  const int64_t M = (int64_t)Nb * H * W, total = M * G;
  for (int64_t idx = (int64_t)blockIdx.x * STEM_T + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * STEM_T) {
    const int64_t p = idx / G;
    const int c0 = 16 * (int)(idx % G);
    const int pw = (int)(p % W);
    const int64_t q = p / W;
    const int ph = (int)(q % H);
    float acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ih = ph + tap / 3 - 1, iw = pw + tap % 3 - 1;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
      const float xv = bf2f(x[p + (int64_t)(tap / 3 - 1) * W + (tap % 3 - 1)]);
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = fmaf(xv, ws[tap * Co + c0 + e], acc[e]);
    }
    u16x8 o0, o1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o0[e] = f2bf(acc[e]);
      o1[e] = f2bf(acc[8 + e]);
    }
    u16x8* dst = reinterpret_cast<u16x8*>(y + p * Co + c0);
    dst[0] = o0;
    dst[1] = o1;
  }
}

// weight gradient: per-block partial [9][Co] over a pixel range; thread = (pixel lane, 8 channels),
// 72 fp32 accumulators; block reduction over the pixel lanes in fixed order
__global__ void __launch_bounds__(STEM_T) conv_c1_wgrad_kernel(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                               int Nb, int H, int W, int Co, int ppb,
                                                               float* __restrict__ part) {
  __shared__ float red[STEM_T * 8];
  const int G = Co / 8, lanes = STEM_T / G;
  const int g = threadIdx.x % G, rl = threadIdx.x / G;
  const int64_t M = (int64_t)Nb * H * W;
  const int64_t p0 = (int64_t)blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  if (rl < lanes) {
    for (int64_t p = p0 + rl; p < p1; p += lanes) {
      const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + p * Co + 8 * g);
      const int pw = (int)(p % W), ph = (int)((p / W) % H);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ih = ph + tap / 3 - 1, iw = pw + tap % 3 - 1;
        const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float xv = ok ? bf2f(x[p + (int64_t)(tap / 3 - 1) * W + (tap % 3 - 1)]) : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[tap][e] = fmaf(bf2f(gv[e]), xv, acc[tap][e]);
      }
    }
  }
  // reduce over the row lanes, one tap at a time through LDS (fixed order)
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = acc[tap][e];
    __syncthreads();
    for (int i = threadIdx.x; i < Co; i += STEM_T) {
      const int gg = i / 8, e = i % 8;
      float s2 = 0.f;
      for (int l = 0; l < lanes; ++l) s2 += red[(l * G + gg) * 8 + e];
      part[((size_t)blockIdx.x * 9 + tap) * Co + i] = s2;
    }
    __syncthreads();
  }
}

// gw[co][0][tap] (bf16, accumulated) += sum over blocks of part[b][tap][co]: one wave per output,
// lane l sums blocks l, l + 64, ... in order, then a fixed shuffle tree (deterministic)
__global__ void __launch_bounds__(STEM_T) conv_c1_wgrad_reduce_kernel(const float* __restrict__ part, int nblk, int Co,
                                                                      u16* __restrict__ gw) {
  const int i = blockIdx.x * (STEM_T / 64) + (threadIdx.x >> 6);  // over [tap][co]
  if (i >= 9 * Co) return;
  const int lane = threadIdx.x & 63;
  float s2 = 0.f;
  for (int b = lane; b < nblk; b += 64) s2 += part[(size_t)b * 9 * Co + i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s2 += __shfl_xor(s2, off);
  if (lane != 0) return;
  const int tap = i / Co, co = i % Co;
  gw[co * 9 + tap] = f2bf(bf2f(gw[co * 9 + tap]) + s2);
}

}  // namespace

bool conv3x3_bf16_supported(int C, int Co) { return C >= 64 && Co >= 64 && C % 64 == 0 && Co % 64 == 0; }

void conv3x3_weight_transform_bf16(const void* w_torch, void* fwd, void* dgrad, int Co, int C, hipStream_t stream) {
  const int64_t n = (int64_t)Co * C * 9;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(conv_weight_transform_kernel, dim3(blocks), dim3(256), 0, stream,
                     static_cast<const u16*>(w_torch), static_cast<u16*>(fwd), static_cast<u16*>(dgrad), Co, C);
}

void conv3x3_weight_transform_batched_bf16(const void* const* w, void* const* fwd, void* const* dgrad, const int* Co,
                                           const int* C, int n, hipStream_t stream) {
  WtBatch b{};
  b.n = n;
  int blocks = 0;
  for (int k = 0; k < n; ++k) {
    b.w[k] = static_cast<const u16*>(w[k]);
    b.fwd[k] = static_cast<u16*>(fwd[k]);
    b.dgrad[k] = static_cast<u16*>(dgrad[k]);
    b.Co[k] = Co[k];
    b.C[k] = C[k];
    b.block0[k] = blocks;
    blocks += ((Co[k] + WT_T - 1) / WT_T) * ((C[k] + WT_T - 1) / WT_T);  // one 32 x 32-channel tile per block
  }
  b.block0[n] = blocks;
  if (blocks > 0) hipLaunchKernelGGL(conv_weight_transform_batched_kernel, dim3(blocks), dim3(256), 0, stream, b);
}

int conv_part_rows(int Nb, int OH, int OW) { return (Nb * OH * OW + BM - 1) / BM; }

static void launch_im2col(ConvArgs& a, bool bn128, hipStream_t stream) {
  a.tiles_n = a.Co / (bn128 ? 128 : 64);
  const dim3 grid(a.tiles_m * a.tiles_n), block(NT);
  const bool epi = a.add || a.part;
  if (bn128 && epi) hipLaunchKernelGGL((conv3x3_fwd_kernel<128, 1>), grid, block, 0, stream, a);
  else if (bn128) hipLaunchKernelGGL((conv3x3_fwd_kernel<128, 0>), grid, block, 0, stream, a);
  else if (epi) hipLaunchKernelGGL((conv3x3_fwd_kernel<64, 1>), grid, block, 0, stream, a);
  else hipLaunchKernelGGL((conv3x3_fwd_kernel<64, 0>), grid, block, 0, stream, a);
}

static BnBack bn_back(const ConvBnBack* b) {
  BnBack r;
  if (b && b->x) {
    r.x = static_cast<const u16*>(b->x);
    r.y = static_cast<const u16*>(b->y);
    r.mean = b->mean;
    r.rstd = b->rstd;
    r.gamma = static_cast<const u16*>(b->gamma);
    r.beta = static_cast<const u16*>(b->beta);
    r.relu = b->relu;
    if (r.relu == 1 && !r.y) abort();  // host contract: the mask source is given
    if (!r.mean || !r.rstd || !r.gamma || !r.beta) abort();
  }
  return r;
}

void conv3x3_fwd_bf16(const void* x, const void* wt, void* y, int Nb, int H, int W, int C, int Co,
                      hipStream_t stream, const void* add, float* part, const ConvBnBack* bnb) {
  ConvArgs a;
  a.add = static_cast<const u16*>(add);
  a.part = part;
  a.bb = bn_back(bnb);
  if (a.bb.x && !part) abort();  // host contract: the backward statistics need their partial rows
  a.x = static_cast<const u16*>(x);
  a.w = static_cast<const u16*>(wt);
  a.y = static_cast<u16*>(y);
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.M = Nb * H * W;
  a.OH = H;
  a.OW = W;
  a.S = 1;
  a.KS = 3;
  a.P = 1;
  a.tiles_m = (a.M + BM - 1) / BM;
  const int engine = knob(KNOB_CONV_FWD_IM2COL) ? 0 : 1;  // im2col kernel on request (A/B tuning)
  const int bn128_min = knob(KNOB_CONV_BN128_MIN);  // BN 128 needs this many tiles, else BN 64 (more workgroups)
  if (engine == 1 && W <= HALO_MAX_W) {
    const bool big = Co % 128 == 0 && a.tiles_m * (Co / 128) >= bn128_min;
    const int bn = big ? 128 : 64;
    a.tiles_n = Co / bn;
    size_t lds = std::max<size_t>((size_t)((C > 64 ? 2 : 1) * (BM + 2 * W + 2) * 64 + 2 * bn * BK) * sizeof(u16),
                                  (size_t)store_tile_lds(bn));
    if (knob(KNOB_CONV_HALO_1WG) == 1) lds = std::max<size_t>(lds, 81 * 1024);  // (A/B) one workgroup per CU
    static bool attr = [] {
      for (const void* f : {reinterpret_cast<const void*>(conv3x3_halo_kernel<128, 5, 0>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<128, 7, 0>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<64, 5, 0>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<64, 7, 0>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<128, 5, 1>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<128, 7, 1>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<64, 5, 1>),
                             reinterpret_cast<const void*>(conv3x3_halo_kernel<64, 7, 1>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      return true;
    }();
    (void)attr;
    const dim3 grid(a.tiles_m * a.tiles_n), block(NT);
    const bool h5 = halo_hl(W) == 5;
    auto go = [&](auto epi) {
      constexpr int E = decltype(epi)::value;
      if (big && h5) hipLaunchKernelGGL((conv3x3_halo_kernel<128, 5, E>), grid, block, lds, stream, a);
      else if (big) hipLaunchKernelGGL((conv3x3_halo_kernel<128, 7, E>), grid, block, lds, stream, a);
      else if (h5) hipLaunchKernelGGL((conv3x3_halo_kernel<64, 5, E>), grid, block, lds, stream, a);
      else hipLaunchKernelGGL((conv3x3_halo_kernel<64, 7, E>), grid, block, lds, stream, a);
    };
    if (a.add || a.part) go(std::integral_constant<int, 1>());
    else go(std::integral_constant<int, 0>());
    return;
  }
  launch_im2col(a, Co % 128 == 0, stream);
}

int conv_out_size(int in, int ks, int stride, int pad) { return (in + 2 * pad - ks) / stride + 1; }

bool conv_general_supported(int C, int Co, int ks, int stride, int pad) {
  return C >= 64 && Co >= 64 && C % 64 == 0 && Co % 64 == 0 && ((ks == 3 && pad == 1) || (ks == 1 && pad == 0)) &&
         (stride == 1 || stride == 2);
}

void conv_fwd_bf16(const void* x, const void* wt, void* y, int Nb, int H, int W, int C, int Co, int ks, int stride,
                   int pad, hipStream_t stream, const void* add, float* part) {
  ConvArgs a;
  a.add = static_cast<const u16*>(add);
  a.part = part;
  a.bb = BnBack();
  a.x = static_cast<const u16*>(x);
  a.w = static_cast<const u16*>(wt);
  a.y = static_cast<u16*>(y);
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.OH = conv_out_size(H, ks, stride, pad);
  a.OW = conv_out_size(W, ks, stride, pad);
  a.S = stride;
  a.KS = ks;
  a.P = pad;
  a.M = Nb * a.OH * a.OW;
  a.tiles_m = (a.M + BM - 1) / BM;
  launch_im2col(a, Co % 128 == 0 && a.tiles_m * (Co / 128) >= 160, stream);
}

int conv_dgrad_s2_part_rows(int Nb, int H, int W, int ks, int pad) {
  const DgClass last = dg_class(3, Nb, H, W, ks, pad, 64, 64, 1);
  return last.tile0 + last.tiles_m;  // tiles_n = 1: tile0 counts the earlier classes' pixel tiles
}

size_t conv_dgrad_s2_weight_elems(int Co, int C, int ks) { return (size_t)Co * C * ks * ks; }

void conv_dgrad_s2_weight_bf16(const void* w_torch, void* packed, int Co, int C, int ks, int pad, hipStream_t stream) {
  const int64_t n = (int64_t)Co * C * ks * ks;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(conv_dgrad_s2_weight_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<const u16*>(w_torch),
                     static_cast<u16*>(packed), Co, C, ks, pad);
}

void conv_dgrad_s2_bf16(const void* dy, const void* packed, void* dx, int Nb, int H, int W, int C, int Co, int ks,
                        int pad, hipStream_t stream, const void* add, float* part, const ConvBnBack* bnb) {
  DgArgs a;
  a.add = static_cast<const u16*>(add);
  a.part = part;
  a.bb = bn_back(bnb);
  if (a.bb.x && !part) abort();  // host contract: the backward statistics need their partial rows
  a.dy = static_cast<const u16*>(dy);
  a.w = static_cast<const u16*>(packed);
  a.dx = static_cast<u16*>(dx);
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.OH = conv_out_size(H, ks, 2, pad);
  a.OW = conv_out_size(W, ks, 2, pad);
  a.Cg = Co;
  a.Cn = C;
  a.KS = ks;
  a.P = pad;
  // BN 128 when that still gives >= 160 workgroups, else BN 64 (more workgroups)
  int bn = 64;
  if (C % 128 == 0) {
    const DgClass last = dg_class(3, Nb, H, W, ks, pad, Co, C, C / 128);
    if (last.tile0 + last.tiles_m * (C / 128) >= 160) bn = 128;
  }
  a.tiles_n = C / bn;
  const DgClass last = dg_class(3, Nb, H, W, ks, pad, Co, C, a.tiles_n);
  a.tiles = last.tile0 + last.tiles_m * a.tiles_n;
  if (a.tiles <= 0) return;
  if (bn == 128) hipLaunchKernelGGL(conv_dgrad_s2_kernel<128>, dim3(a.tiles), dim3(NT), 0, stream, a);
  else hipLaunchKernelGGL(conv_dgrad_s2_kernel<64>, dim3(a.tiles), dim3(NT), 0, stream, a);
}

static int wgrad_rows(int Co) {
  const bool rows64 = knob(KNOB_CONV_WG_ROWS64) != 0;  // 0: 128-row tiles (half idle) for Cout = 64 too
  return Co % 128 == 0 || !rows64 ? 128 : 64;
}

static int wgrad_splits(int M, int KT, int Co) {
  // the pixel range is split until the grid reaches ~two workgroups per CU (64 KB LDS, <= 128 VGPRs)
  const int target = std::max(1, knob(KNOB_CONV_WG_BLOCKS));
  const int tr = wgrad_rows(Co);
  const int tiles = ((Co + tr - 1) / tr) * ((KT + 127) / 128);
  int s = target / tiles;
  const int max_by_m = M / (8 * 64);  // >= 8 K-steps per workgroup
  if (s > max_by_m) s = max_by_m;
  return s < 1 ? 1 : s;
}

int conv3x3_wgrad_splits(int Nb, int H, int W, int C, int Co) { return wgrad_splits(Nb * H * W, 9 * C, Co); }

size_t conv_wgrad_workspace_floats(int Nb, int H, int W, int C, int Co, int ks, int stride, int pad) {
  const int M = Nb * conv_out_size(H, ks, stride, pad) * conv_out_size(W, ks, stride, pad);
  return (size_t)wgrad_splits(M, ks * ks * C, Co) * Co * ks * ks * C;
}

size_t conv3x3_wgrad_workspace_floats(int Nb, int H, int W, int C, int Co) {
  return conv_wgrad_workspace_floats(Nb, H, W, C, Co, 3, 1, 1);
}

void conv_wgrad_bf16(const void* dy, const void* x, void* gw_torch, float* workspace, int Nb, int H, int W, int C,
                     int Co, int ks, int stride, int pad, hipStream_t stream) {
  WgArgs a;
  a.dy = static_cast<const u16*>(dy);
  a.x = static_cast<const u16*>(x);
  a.slab = workspace;
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.OH = conv_out_size(H, ks, stride, pad);
  a.OW = conv_out_size(W, ks, stride, pad);
  a.S = stride;
  a.KS = ks;
  a.P = pad;
  a.M = Nb * a.OH * a.OW;
  const int T = ks * ks;
  int s = wgrad_splits(a.M, T * C, Co);
  int pps = (a.M + s - 1) / s;
  pps = (pps + 63) / 64 * 64;
  s = (a.M + pps - 1) / pps;
  a.pps = pps;
  a.splits = s;
  const int tr = wgrad_rows(Co);
  a.tiles_m = (Co + tr - 1) / tr;
  a.tiles_n = (T * C + 127) / 128;
  const dim3 grid(a.tiles_m * a.tiles_n * s);
  const bool dma = knob(KNOB_CONV_WGRAD_DMA) == 1 && C % 8 == 0 && Co % 8 == 0 &&  // (tests A/B the loops)
                   (reinterpret_cast<uintptr_t>(dy) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const bool st3 = knob(KNOB_CONV_WGRAD_STAGES) == 3;
  if (dma && tr == 128 && st3)
    hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<128, 3>), grid, dim3(NT), 0, stream, a);
  else if (dma && tr == 128)
    hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<128, 2>), grid, dim3(NT), 0, stream, a);
  else if (dma && st3)
    hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<64, 3>), grid, dim3(NT), 0, stream, a);
  else if (dma)
    hipLaunchKernelGGL((conv3x3_wgrad_dma_kernel<64, 2>), grid, dim3(NT), 0, stream, a);
  else if (tr == 128)
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<128>, grid, dim3(NT), 0, stream, a);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<64>, grid, dim3(NT), 0, stream, a);
  const int64_t n4 = (int64_t)Co * T * C / 4;
  const int blocks = (int)std::min<int64_t>((n4 + RD_OUT - 1) / RD_OUT, 8192);
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(blocks), dim3(RD_OUT * RD_GRP), 0, stream, workspace, s, Co, C, T,
                     static_cast<u16*>(gw_torch));
}

void conv3x3_wgrad_bf16(const void* dy, const void* x, void* gw_torch, float* workspace, int Nb, int H, int W, int C,
                        int Co, hipStream_t stream) {
  conv_wgrad_bf16(dy, x, gw_torch, workspace, Nb, H, W, C, Co, 3, 1, 1, stream);
}

// ---- stem (one input channel) ----------------------------------------------------------------
bool conv_c1_supported(int Co) { return Co % 16 == 0 && Co <= 512; }

void conv_c1_fwd_bf16(const void* x, const void* w, void* y, int Nb, int H, int W, int Co, hipStream_t stream) {
  const int64_t total = (int64_t)Nb * H * W * (Co / 16);
  const int blocks = (int)std::min<int64_t>((total + STEM_T - 1) / STEM_T, 8192);
  hipLaunchKernelGGL(conv_c1_fwd_kernel, dim3(blocks), dim3(STEM_T), 0, stream, static_cast<const u16*>(x),
                     static_cast<const u16*>(w), static_cast<u16*>(y), Nb, H, W, Co);
}

static int c1_wgrad_blocks(int64_t M, int* ppb) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(1024, M / 64));
  *ppb = (int)((M + blocks - 1) / blocks);
  return (int)((M + *ppb - 1) / *ppb);
}

size_t conv_c1_wgrad_workspace_floats(int Nb, int H, int W, int Co) {
  int ppb;
  return (size_t)c1_wgrad_blocks((int64_t)Nb * H * W, &ppb) * 9 * Co;
}

void conv_c1_wgrad_bf16(const void* dy, const void* x, void* gw, float* workspace, int Nb, int H, int W, int Co,
                        hipStream_t stream) {
  int ppb;
  const int nblk = c1_wgrad_blocks((int64_t)Nb * H * W, &ppb);
  hipLaunchKernelGGL(conv_c1_wgrad_kernel, dim3(nblk), dim3(STEM_T), 0, stream, static_cast<const u16*>(dy),
                     static_cast<const u16*>(x), Nb, H, W, Co, ppb, workspace);
  hipLaunchKernelGGL(conv_c1_wgrad_reduce_kernel, dim3((9 * Co + STEM_T / 64 - 1) / (STEM_T / 64)), dim3(STEM_T), 0, stream,
                     workspace, nblk, Co, static_cast<u16*>(gw));
}

}  // namespace sdml
