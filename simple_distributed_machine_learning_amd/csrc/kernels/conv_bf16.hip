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

struct ConvArgs {
  const u16* x;  // NHWC input [Nb][H][W][C]
  const u16* w;  // [Co][9][C]
  u16* y;        // NHWC output [Nb][H][W][Co]
  int Nb, H, W, C, Co;
  int M;         // Nb*H*W
  int tiles_m, tiles_n;
};

template <int BN>
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
  const int K = 9 * a.C;
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
    pw[u] = pp % a.W;
    const int q = pp / a.W;
    ph[u] = q % a.H;
    pn[u] = q / a.H;
  }
  u16x8 va[4], vb[NB];
  auto inb = [&](int u, int k0) {  // is row u's shifted pixel inside the image for tap(k0)?
    const int tap = k0 / a.C;
    const int ih = ph[u] + tap / 3 - 1, iw = pw[u] + tap % 3 - 1;
    return pv[u] && k0 < K && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
  };
  auto load = [&](int k0) {
    const int tap = min(k0, K - BK) / a.C, ci0 = min(k0, K - BK) % a.C;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ih = ph[u] + tap / 3 - 1, iw = pw[u] + tap % 3 - 1;
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
  // epilogue: C/D map col = lane&31 (cout), row = (r&3) + 8(r>>2) + 4h (pixel)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = n0 + wn * 64 + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = m0 + wm * WTM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (p < a.M) a.y[(size_t)p * a.Co + co] = f2bf(acc[i][j][r]);
      }
    }
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
  const u16* dy;  // [M][Co]
  const u16* x;   // [M][C] (NHWC)
  float* slab;    // [splits][Co][9C]
  int Nb, H, W, C, Co, M;
  int pps;        // pixels per split (multiple of 64)
  int tiles_m, tiles_n, splits;
};

__global__ void __launch_bounds__(NT) conv3x3_wgrad_kernel(WgArgs a) {
  constexpr int IMG = 64 * 128;
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
  const int m0 = tm * 128, n0 = tn * 128;  // m: co, n: tap*C + ci
  const int K9 = 9 * a.C;
  const int pbeg = split * a.pps, pend = min(a.M, pbeg + a.pps);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;  // 2 x 4 waves: 64 (co) x 32 (n) each
  const int t = threadIdx.x;
  // per K-step each operand tile is 64 pixels x 128 columns = 1024 16-B chunks: 2 per thread
  // (pixel row kk = id >> 4, 8-column chunk c = id & 15)
  u16x8 va[2], vb[2];
  unsigned okb = 0;  // bit u: chunk u of vb is inside the image (zeroed at store time otherwise)
  auto load = [&](int p0) {
    okb = 0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = t + NT * u, kk = id >> 4, c = id & 15;
      const int p = min(p0 + kk, a.M - 1);
      va[u] = *reinterpret_cast<const u16x8*>(a.dy + (size_t)p * a.Co + min(m0 + 8 * c, a.Co - 8));
      const int n = n0 + 8 * c;
      const int tap = min(n, K9 - 8) / a.C, ci = min(n, K9 - 8) % a.C;
      const int ow = p % a.W, q = p / a.W, oh = q % a.H, nb = q / a.H;
      const int ih = oh + tap / 3 - 1, iw = ow + tap % 3 - 1;
      const bool ok = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      vb[u] = *reinterpret_cast<const u16x8*>(a.x + (ok ? (((size_t)nb * a.H + ih) * a.W + iw) * a.C + ci : 0));
      okb |= ok ? (1u << u) : 0u;
    }
  };
  auto store = [&](u16* L, int p0) {
    const u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int id = t + NT * u, kk = id >> 4, c = id & 15;
      const bool in = p0 + kk < pend;
      *reinterpret_cast<u16x8*>(L + km_off(kk, c)) = in ? va[u] : z;
      *reinterpret_cast<u16x8*>(L + IMG + km_off(kk, c)) = (in && ((okb >> u) & 1)) ? vb[u] : z;
    }
  };
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
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
      bf16x8 af[2], bfr;
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = trfrag(L, wm * 64 + 32 * i, s, lane);
      bfr = trfrag(L + IMG, wn * 32, s, lane);
      if (s == 0) {
        store(Ln, pbeg + (it + 1) * 64);
        load(pbeg + (it + 2) * 64);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i] = mfma(af[i], bfr, acc[i]);
    }
    __syncthreads();
  }
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= K9) return;
  float* S = a.slab + (size_t)split * a.Co * K9;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < a.Co) S[(size_t)co * K9 + col] = acc[i][r];
    }
}

// gw[co][ci][kh][kw] (bf16, torch layout, accumulated) += sum_s slab[s][co][tap][ci]
__global__ void __launch_bounds__(256) conv_wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int Co,
                                                                int C, u16* __restrict__ gw) {
  const int64_t n = (int64_t)Co * 9 * C;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    // i indexes the torch layout [co][ci][tap]
    const int tap = (int)(i % 9);
    const int64_t r = i / 9;
    const int ci = (int)(r % C), co = (int)(r / C);
    const int64_t src = ((int64_t)co * 9 + tap) * C + ci;
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += slab[(size_t)k * n + src];
    gw[i] = f2bf(bf2f(gw[i]) + s);
  }
}

// torch weight [co][ci][3][3] -> [co][tap][ci] (forward) or the dgrad weight [ci][8 - tap][co]
__global__ void __launch_bounds__(256) conv_weight_transform_kernel(const u16* __restrict__ w, u16* __restrict__ out,
                                                                    int Co, int C, int dgrad) {
  const int64_t n = (int64_t)Co * C * 9;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int tap = (int)(i % 9);
    const int64_t r = i / 9;
    const int ci = (int)(r % C), co = (int)(r / C);
    const int64_t dst = dgrad ? ((int64_t)ci * 9 + (8 - tap)) * Co + co : ((int64_t)co * 9 + tap) * C + ci;
    out[dst] = w[i];
  }
}

}  // namespace

bool conv3x3_bf16_supported(int C, int Co) { return C >= 64 && Co >= 64 && C % 64 == 0 && Co % 64 == 0; }

void conv3x3_weight_transform_bf16(const void* w_torch, void* out, int Co, int C, bool dgrad, hipStream_t stream) {
  const int64_t n = (int64_t)Co * C * 9;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(conv_weight_transform_kernel, dim3(blocks), dim3(256), 0, stream,
                     static_cast<const u16*>(w_torch), static_cast<u16*>(out), Co, C, dgrad ? 1 : 0);
}

void conv3x3_fwd_bf16(const void* x, const void* wt, void* y, int Nb, int H, int W, int C, int Co,
                      hipStream_t stream) {
  ConvArgs a;
  a.x = static_cast<const u16*>(x);
  a.w = static_cast<const u16*>(wt);
  a.y = static_cast<u16*>(y);
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.M = Nb * H * W;
  a.tiles_m = (a.M + BM - 1) / BM;
  if (Co % 128 == 0) {
    a.tiles_n = Co / 128;
    hipLaunchKernelGGL(conv3x3_fwd_kernel<128>, dim3(a.tiles_m * a.tiles_n), dim3(NT), 0, stream, a);
  } else {
    a.tiles_n = Co / 64;
    hipLaunchKernelGGL(conv3x3_fwd_kernel<64>, dim3(a.tiles_m * a.tiles_n), dim3(NT), 0, stream, a);
  }
}

int conv3x3_wgrad_splits(int Nb, int H, int W, int C, int Co) {
  const int tiles = ((Co + 127) / 128) * ((9 * C + 127) / 128);
  const int M = Nb * H * W;
  int s = 256 / tiles;
  const int max_by_m = M / (8 * 64);
  if (s > max_by_m) s = max_by_m;
  return s < 1 ? 1 : s;
}

size_t conv3x3_wgrad_workspace_floats(int Nb, int H, int W, int C, int Co) {
  return (size_t)conv3x3_wgrad_splits(Nb, H, W, C, Co) * Co * 9 * C;
}

void conv3x3_wgrad_bf16(const void* dy, const void* x, void* gw_torch, float* workspace, int Nb, int H, int W, int C,
                        int Co, hipStream_t stream) {
  WgArgs a;
  a.dy = static_cast<const u16*>(dy);
  a.x = static_cast<const u16*>(x);
  a.slab = workspace;
  a.Nb = Nb;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Co = Co;
  a.M = Nb * H * W;
  int s = conv3x3_wgrad_splits(Nb, H, W, C, Co);
  int pps = (a.M + s - 1) / s;
  pps = (pps + 63) / 64 * 64;
  s = (a.M + pps - 1) / pps;
  a.pps = pps;
  a.splits = s;
  a.tiles_m = (Co + 127) / 128;
  a.tiles_n = (9 * C + 127) / 128;
  hipLaunchKernelGGL(conv3x3_wgrad_kernel, dim3(a.tiles_m * a.tiles_n * s), dim3(NT), 0, stream, a);
  const int64_t n = (int64_t)Co * 9 * C;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, workspace, s, Co, C,
                     static_cast<u16*>(gw_torch));
}

}  // namespace sdml
