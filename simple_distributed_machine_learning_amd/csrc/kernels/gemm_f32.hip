// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32: bitwise an fmaf chain).
//
// Used for every Linear of the MNIST MLPs (forward with fused bias+ReLU, dX with the ReLU
// mask fused into the A-operand staging, dW split-K with atomic accumulation straight into
// the flat gradient buffer and the bias gradient fused as a row-sum of the staged A tile).
// These replace the ATen CPU GEMMs of the reference's fc layers
// (/root/reference/simple_distributed.py:63-64, :75-77).
//
// Tiling (gfx950, wave64):
//   block 256 threads = 4 waves in a 2x2 grid, block tile 128x128, K-step 32 floats;
//   each wave owns a 64x64 output = 2x2 MFMA 32x32 accumulators (64 AGPR/VGPR floats).
//   LDS: double-buffered A and B tiles (2 x 2 x 18 KiB = 72 KiB -> 2 blocks/CU).
//   * K-contiguous operand tile is stored [row][32 + 4 pad] floats: one ds_read_b128 gives a
//     lane 4 consecutive k of its row -> 4 MFMAs per read. The 144-B row pitch makes the
//     16-lane groups of ds_read_b128 conflict-free (lanes l and l+16 never share a group).
//   * K-major operand tile is stored [k][128] (straight copy of the global layout, no
//     transpose in staging): fragments are ds_read_b32 of 32 consecutive floats (conflict-free).
//   Both layouts use the same k permutation inside a k-group of 8: MFMA j of group s sums
//   k = 8s+j (lanes 0-31) and 8s+4+j (lanes 32-63). Any permutation of the reduction is valid
//   as long as A and B agree; the result is the same set of fmaf terms in a different order.
//   Global->LDS staging is register-prefetched one K-step ahead (issue before the MFMAs,
//   write after), so HBM latency hides under the matrix work.
// MFMA C/D map (gfx950, dtype-independent): col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "kernels.h"

namespace sdml {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, NTHR = 256;
constexpr int BK_MAX = 32;
template <int BK>
struct TileCfg {
  static constexpr int KC_PITCH = BK + 4;            // K-contiguous tile row pitch (floats)
  static constexpr int TILE_FLOATS = BM * KC_PITCH;  // >= BK*BM (K-major tile)
  static constexpr int NV = BM * BK / 4 / NTHR;      // float4 per thread per operand tile
  static_assert(BK * BM <= TILE_FLOATS, "tile size");
};

struct KParams {
  const float* A;
  const float* amask;
  const float* B;
  float* C;
  const float* bias;
  float* rowsum;
  const float* cmask;
  int M, N, K, lda, ldb, ldc;
  int epi;
  int a_vec, b_vec;  // 16-B vector loads legal for the operand
  int kps;  // K elements per split (multiple of BK)
  int tiles_m, tiles_n;
};

// ---- staging ---------------------------------------------------------------------------------
// K-contiguous operand: tile rows [r0, r0+128), k [k0, k0+BK): NV float4 per thread.
template <int BK>
__device__ __forceinline__ void load_kc(const float* __restrict__ P, const float* __restrict__ mask, int ld,
                                        int rows, int r0, int k0, int kend, bool vec, f32x4 (&v)[TileCfg<BK>::NV]) {
#pragma unroll
  for (int i = 0; i < TileCfg<BK>::NV; ++i) {
    int idx = threadIdx.x + NTHR * i;
    int r = idx / (BK / 4), k4 = idx % (BK / 4);
    int gr = r0 + r, gk = k0 + 4 * k4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (!vec) {  // unaligned / K % 4 != 0: element loads (slow path, odd shapes only)
      if (gr < rows) {
        const float* src = P + (size_t)gr * ld;
        const float* msk = mask ? mask + (size_t)gr * ld : nullptr;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (gk + e < kend) x[e] = (!msk || msk[gk + e] > 0.f) ? src[gk + e] : 0.f;
      }
    } else if (gr < rows && gk < kend) {
      x = *reinterpret_cast<const f32x4*>(P + (size_t)gr * ld + gk);
      if (mask) {
        f32x4 mk = *reinterpret_cast<const f32x4*>(mask + (size_t)gr * ld + gk);
        x[0] = mk[0] > 0.f ? x[0] : 0.f;
        x[1] = mk[1] > 0.f ? x[1] : 0.f;
        x[2] = mk[2] > 0.f ? x[2] : 0.f;
        x[3] = mk[3] > 0.f ? x[3] : 0.f;
      }
    }
    v[i] = x;
  }
}

template <int BK>
__device__ __forceinline__ void store_kc(float* __restrict__ T, const f32x4 (&v)[TileCfg<BK>::NV]) {
#pragma unroll
  for (int i = 0; i < TileCfg<BK>::NV; ++i) {
    int idx = threadIdx.x + NTHR * i;
    int r = idx / (BK / 4), k4 = idx % (BK / 4);
    *reinterpret_cast<f32x4*>(T + r * TileCfg<BK>::KC_PITCH + 4 * k4) = v[i];
  }
}

// K-major operand: tile k [k0, k0+BK), rows [r0, r0+128): float4 along rows.
template <int BK>
__device__ __forceinline__ void load_km(const float* __restrict__ P, const float* __restrict__ mask, int ld,
                                        int rows, int r0, int k0, int kend, bool vec, f32x4 (&v)[TileCfg<BK>::NV]) {
#pragma unroll
  for (int i = 0; i < TileCfg<BK>::NV; ++i) {
    int idx = threadIdx.x + NTHR * i;
    int kk = idx >> 5, r4 = idx & 31;
    int gk = k0 + kk, gr = r0 + 4 * r4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (gk < kend) {
      const float* src = P + (size_t)gk * ld + gr;
      const float* msk = mask ? mask + (size_t)gk * ld + gr : nullptr;
      if (vec && gr + 3 < rows) {
        x = *reinterpret_cast<const f32x4*>(src);
        if (msk) {
          f32x4 mk = *reinterpret_cast<const f32x4*>(msk);
          x[0] = mk[0] > 0.f ? x[0] : 0.f;
          x[1] = mk[1] > 0.f ? x[1] : 0.f;
          x[2] = mk[2] > 0.f ? x[2] : 0.f;
          x[3] = mk[3] > 0.f ? x[3] : 0.f;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (gr + e < rows) {
            float a = src[e];
            x[e] = (!msk || msk[e] > 0.f) ? a : 0.f;
          }
      }
    }
    v[i] = x;
  }
}

template <int BK>
__device__ __forceinline__ void store_km(float* __restrict__ T, const f32x4 (&v)[TileCfg<BK>::NV]) {
#pragma unroll
  for (int i = 0; i < TileCfg<BK>::NV; ++i) {
    int idx = threadIdx.x + NTHR * i;
    int kk = idx >> 5, r4 = idx & 31;
    *reinterpret_cast<f32x4*>(T + kk * BM + 4 * r4) = v[i];
  }
}

// fragment of a 32-row sub-tile for k-group s: f[j] = X(row, k = 8s + 4h + j)
template <bool KM, int BK>
__device__ __forceinline__ f32x4 frag(const float* __restrict__ T, int row, int s, int h) {
  if constexpr (!KM) {
    return *reinterpret_cast<const f32x4*>(T + row * TileCfg<BK>::KC_PITCH + 8 * s + 4 * h);
  } else {
    const float* p = T + (8 * s + 4 * h) * BM + row;
    f32x4 f;
    f[0] = p[0];
    f[1] = p[BM];
    f[2] = p[2 * BM];
    f[3] = p[3 * BM];
    return f;
  }
}

template <bool A_KM, bool B_KM, int BK>
__global__ void __launch_bounds__(NTHR, 2) gemm_f32_kernel(KParams p) {
  constexpr int TILE_FLOATS = TileCfg<BK>::TILE_FLOATS;
  constexpr int KC_PITCH = TileCfg<BK>::KC_PITCH;
  constexpr int NV = TileCfg<BK>::NV;
  __shared__ __attribute__((aligned(16))) float smem[4 * TILE_FLOATS];  // [buf][A|B]
  // XCD-aware, bijective remap over ALL blocks (tiles x splits): blocks b and b+8 share an
  // XCD, so hand each XCD a contiguous run of logical ids. Logical id = split * ntiles + tile:
  // the tiles of one K-split (which stream the SAME A/B K-slices) then sit on one XCD and
  // read those slices through its L2 instead of once per tile from HBM.
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nwg = ntiles * gridDim.y;
  int orig = blockIdx.y * gridDim.x + blockIdx.x;
  int wg = orig;
  if (nwg >= 16) {
    int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int l32 = lane & 31, h = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const bool do_rowsum = p.rowsum != nullptr && tn == 0;
  float rs = 0.f;  // thread's partial row-sum of A (bias gradient)

  f32x4 va[NV], vb[NV];
  auto load = [&](int k0) {
    if constexpr (A_KM) load_km<BK>(p.A, p.amask, p.lda, p.M, m0, k0, kend, p.a_vec, va);
    else load_kc<BK>(p.A, p.amask, p.lda, p.M, m0, k0, kend, p.a_vec, va);
    if constexpr (B_KM) load_km<BK>(p.B, nullptr, p.ldb, p.N, n0, k0, kend, p.b_vec, vb);
    else load_kc<BK>(p.B, nullptr, p.ldb, p.N, n0, k0, kend, p.b_vec, vb);
  };
  auto store = [&](int buf) {
    float* As = smem + (2 * buf) * TILE_FLOATS;
    float* Bs = As + TILE_FLOATS;
    if constexpr (A_KM) store_km<BK>(As, va);
    else store_kc<BK>(As, va);
    if constexpr (B_KM) store_km<BK>(Bs, vb);
    else store_kc<BK>(Bs, vb);
  };

  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) load(kbeg + (t + 1) * BK);  // prefetch next tile into registers
    const float* As = smem + (2 * cur) * TILE_FLOATS;
    const float* Bs = As + TILE_FLOATS;
    if (do_rowsum) {  // rows of the A tile (bias grad): thread -> row t%128, half of the k range
      const int row = threadIdx.x & (BM - 1), half = threadIdx.x >> 7;
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        int k = half * (BK / 2) + kk;
        rs += A_KM ? As[k * BM + row] : As[row * KC_PITCH + k];
      }
    }
#pragma unroll
    for (int s = 0; s < BK / 8; ++s) {
      f32x4 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = frag<A_KM, BK>(As, wm * 64 + i * 32 + l32, s, h);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = frag<B_KM, BK>(Bs, wn * 64 + j * 32 + l32, s, h);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  if (do_rowsum) {
    const int row = threadIdx.x & (BM - 1);
    if (m0 + row < p.M) atomicAdd(p.rowsum + m0 + row, rs);
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + l32;
      if (col >= p.N) continue;
      const float bv = (p.epi == EPI_BIAS || p.epi == EPI_BIAS_RELU) ? p.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        float v = acc[i][j][r];
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

}  // namespace

static bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

// 16-B loads are legal when the base is aligned, the leading dimension keeps every row
// aligned, and (for a k-contiguous operand) K is whole float4s
static bool vec_ok(const float* P, const float* mask, int ld, bool kmajor, int K) {
  if (!al16(P) || (mask && !al16(mask)) || ld % 4) return false;
  return kmajor || K % 4 == 0;
}

bool gemm_f32_supported(const GemmArgs& g) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return false;
  if (g.splits > 1 && g.epi != EPI_ATOMIC) return false;
  return true;
}

static int g_variant = 0;  // 0: auto, 32: BK=32, 16: BK=16 (A/B experiments)
void gemm_f32_set_variant(int v) { g_variant = v; }

static int g_mode = -1;  // -1: not yet read from the environment
void gemm_f32_set_mode(int mode) { g_mode = mode; }
int gemm_f32_mode() {
  if (g_mode < 0) {
    const char* e = getenv("SDML_F32_GEMM");
    g_mode = (e && std::string(e) == "mfma") ? 0 : 1;
  }
  return g_mode;
}

int gemm_f32_pick_splits(int M, int N, int K) {
  constexpr int BK = BK_MAX;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  // fill the chip with one wave of blocks (2 resident per CU = 512 slots) while keeping
  // >= 32 K-steps per split: every split adds its whole C tile with fp32 atomics
  // (~1.3 TB/s chip-wide), so splits cost output bandwidth
  int splits = 512 / tiles;
  const int max_by_k = K / (32 * BK);
  if (splits > max_by_k) splits = max_by_k;
  return splits < 1 ? 1 : splits;
}

namespace {
// skinny-GEMM helpers: C rows <- bias (or 0) before a split-K atomic GEMM; relu / x>0 mask after
__global__ void __launch_bounds__(256) rows_init_kernel(float* __restrict__ C, const float* __restrict__ bias, int M,
                                                        int N, int ldc) {
  const int64_t n = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / N), c = (int)(i % N);
    C[(int64_t)m * ldc + c] = bias ? bias[c] : 0.f;
  }
}
__global__ void __launch_bounds__(256) post_epi_kernel(float* __restrict__ C, const float* __restrict__ cmask, int M,
                                                       int N, int ldc, int relu) {
  const int64_t n = (int64_t)M * N;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / N), c = (int)(i % N);
    float v = C[(int64_t)m * ldc + c];
    if (relu) v = fmaxf(v, 0.f);
    if (cmask && !(cmask[(int64_t)m * ldc + c] > 0.f)) v = 0.f;
    C[(int64_t)m * ldc + c] = v;
  }
}
// dW for a SMALL batch (the GEMM's K): gw[n][k] += sum_m gz(m,n) x[m][k], gb[n] += sum_m gz(m,n),
// gz(m,n) = gy[m][n] * (mask[m][n] > 0). One thread owns DW_NG n x 4 k outputs (plain
// read-modify-write: deterministic, no atomics, no 128x128 tile epilogue funnelled through a
// few CUs); gy values are wave-broadcast. DW_NG = 1 maximises the wave count: with ~100
// waves (DW_NG = 4) the kernel was VALU-issue bound on a quarter of the CUs.
constexpr int DW_NG = 1;
__global__ void __launch_bounds__(256) dw_smallk_kernel(const float* __restrict__ gy, const float* __restrict__ mask,
                                                        const float* __restrict__ x, float* __restrict__ gw,
                                                        float* __restrict__ gb, int M, int N, int K, int vec) {
  const int K4 = (K + 3) / 4;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int ng = idx / K4, k4 = idx % K4;
  const int n0 = ng * DW_NG;
  if (n0 >= N) return;
  float acc[DW_NG][4] = {};
  float gs[DW_NG] = {};
  const int k0 = 4 * k4;
  // batches of DW_MB rows: all their loads are issued before the FMAs (latency, not
  // bandwidth, bounds this kernel: a few hundred waves, L2-resident operands)
  constexpr int DW_MB = 8;
  for (int mb = 0; mb < M; mb += DW_MB) {
    float xv[DW_MB][4], gv[DW_MB][DW_NG];
#pragma unroll
    for (int u = 0; u < DW_MB; ++u) {
      const int m = mb + u;
      const bool ok = m < M;
      const float* xr = x + (size_t)m * K + k0;
      if (vec && ok) {
        const float4 v = *reinterpret_cast<const float4*>(xr);
        xv[u][0] = v.x;
        xv[u][1] = v.y;
        xv[u][2] = v.z;
        xv[u][3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[u][j] = (ok && k0 + j < K) ? xr[j] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < DW_NG; ++i) {
        const int n = n0 + i;
        float g = 0.f;
        if (ok && n < N) {
          g = gy[(size_t)m * N + n];
          if (mask && !(mask[(size_t)m * N + n] > 0.f)) g = 0.f;
        }
        gv[u][i] = g;
      }
    }
#pragma unroll
    for (int u = 0; u < DW_MB; ++u)
#pragma unroll
      for (int i = 0; i < DW_NG; ++i) {
        gs[i] += gv[u][i];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += gv[u][i] * xv[u][j];
      }
  }
#pragma unroll
  for (int i = 0; i < DW_NG; ++i) {
    const int n = n0 + i;
    if (n >= N) break;
    float* dst = gw + (size_t)n * K + k0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (k0 + j < K) dst[j] += acc[i][j];
    if (gb && k4 == 0) gb[n] += gs[i];
  }
}
// Forward GEMM for a SMALL batch: C[m][n] = epi(sum_k A[m][k] B[n][k] + bias[n]), both operands
// k-contiguous (x @ W^T). A workgroup owns one row m and 64 outputs n (one per lane); its 4 waves
// split K into quarters (float4 steps: the x row is wave-broadcast, every lane streams its own
// W row from L2) and meet in LDS for the bias/ReLU epilogue. Grid M x N/64 (120 WGs at the
// reference's 60 x 784 -> 128), versus a single 128x128 MFMA tile walking all of K.
__global__ void __launch_bounds__(256) fwd_smallm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                         const float* __restrict__ bias, float* __restrict__ C, int N,
                                                         int K, int lda, int ldb, int ldc, int relu) {
  __shared__ float red[4][64];
  const int m = blockIdx.x, n0 = blockIdx.y * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = n0 + lane;
  const int K4 = K / 4, q = (K4 + 3) / 4;
  const int kb = w * q, ke = min(K4, kb + q);
  const float4* a = reinterpret_cast<const float4*>(A + (size_t)m * lda);
  const float4* b = reinterpret_cast<const float4*>(B + (size_t)(n < N ? n : 0) * ldb);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k4 = kb; k4 < ke; ++k4) {
    const float4 av = a[k4], bv = b[k4];
    acc[0] += av.x * bv.x;
    acc[1] += av.y * bv.y;
    acc[2] += av.z * bv.z;
    acc[3] += av.w * bv.w;
  }
  red[w][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (w == 0 && n < N) {
    float v = ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) + (bias ? bias[n] : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    C[(size_t)m * ldc + n] = v;
  }
}

}  // namespace

void dw_smallk(const float* gy, const float* mask, const float* x, float* gw, float* gb, int M, int N, int K,
               hipStream_t stream) {
  const bool vec = (K % 4 == 0) && al16(x);
  const int64_t threads = (int64_t)((N + DW_NG - 1) / DW_NG) * ((K + 3) / 4);
  hipLaunchKernelGGL(dw_smallk_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, gy, mask, x, gw,
                     gb, M, N, K, vec ? 1 : 0);
}

// Few output tiles and a long K (e.g. a batch-60 forward: ONE 128x128 tile, K = 784) leave
// the chip idle and run one block through the whole K. Split K instead and accumulate with
// fp32 atomics into C pre-set to the bias, then apply ReLU / the x>0 mask in a light pass:
// three short launches instead of one long serial one. 0 = not worth it.
int gemm_f32_skinny_splits(int M, int N, int K, int epi) {
  if (epi == EPI_ATOMIC) return 0;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles > 32 || K < 256) return 0;
  int splits = 256 / tiles;
  const int max_by_k = K / (2 * BK_MAX);  // >= 2 K-steps per split
  if (splits > max_by_k) splits = max_by_k;
  return splits >= 4 ? splits : 0;
}

bool gemm_f32_uses_x3(const GemmArgs& g) {
  return gemm_f32_mode() == 1 && (int64_t)g.M * g.N * g.K >= (int64_t(1) << 26) && gemm_f32x3_eligible(g);
}

void gemm_f32(const GemmArgs& g, hipStream_t stream) {
  if (g.M <= FWD_SMALLM_MAX_M && !g.a_kmajor && !g.b_kmajor && g.splits <= 1 && !g.amask && !g.rowsum &&
      (g.epi == EPI_BIAS || g.epi == EPI_BIAS_RELU || (g.epi == EPI_STORE && !g.cmask)) && g.K % 4 == 0 &&
      al16(g.A) && al16(g.B) && g.lda % 4 == 0 && g.ldb % 4 == 0) {
    hipLaunchKernelGGL(fwd_smallm_kernel, dim3(g.M, (g.N + 63) / 64), dim3(256), 0, stream, g.A, g.B,
                       g.epi == EPI_STORE ? nullptr : g.bias, g.C, g.N, g.K, g.lda, g.ldb, g.ldc,
                       g.epi == EPI_BIAS_RELU ? 1 : 0);
    return;
  }
  // large shapes: fp32 via the bf16x3 split on the bf16 matrix cores (2.67x the fp32 MFMA rate)
  if (gemm_f32_uses_x3(g)) {
    gemm_f32x3(g, stream);
    return;
  }
  if (g.splits <= 1 && g.epi != EPI_ATOMIC) {
    const int sk = gemm_f32_skinny_splits(g.M, g.N, g.K, g.epi);
    if (sk > 0) {
      const int64_t n = (int64_t)g.M * g.N;
      const int eb = (int)std::min<int64_t>((n + 255) / 256, 1024);
      if (g.epi != EPI_ACCUM)
        hipLaunchKernelGGL(rows_init_kernel, dim3(eb), dim3(256), 0, stream, g.C,
                           (g.epi == EPI_BIAS || g.epi == EPI_BIAS_RELU) ? g.bias : nullptr, g.M, g.N, g.ldc);
      GemmArgs a = g;
      a.epi = EPI_ATOMIC;
      a.splits = sk;
      a.bias = nullptr;
      a.cmask = nullptr;  // rowsum (bias grad) is split-K safe: it stays
      gemm_f32(a, stream);
      const bool relu = g.epi == EPI_BIAS_RELU;
      if (relu || (g.cmask && g.epi == EPI_STORE))
        hipLaunchKernelGGL(post_epi_kernel, dim3(eb), dim3(256), 0, stream, g.C,
                           g.epi == EPI_STORE ? g.cmask : nullptr, g.M, g.N, g.ldc, relu ? 1 : 0);
      return;
    }
  }
  KParams p;
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
  p.a_vec = vec_ok(g.A, g.amask, g.lda, g.a_kmajor, g.K);
  p.b_vec = vec_ok(g.B, nullptr, g.ldb, g.b_kmajor, g.K);
  const int BK = (g_variant == 16) ? 16 : 32;
  int splits = g.splits < 1 ? 1 : g.splits;
  int kps = (g.K + splits - 1) / splits;
  kps = (kps + BK_MAX - 1) / BK_MAX * BK_MAX;
  splits = (g.K + kps - 1) / kps;
  p.kps = kps;
  p.tiles_m = (g.M + BM - 1) / BM;
  p.tiles_n = (g.N + BN - 1) / BN;
  dim3 grid(p.tiles_m * p.tiles_n, splits, 1);
  dim3 block(NTHR);
#define GEMM_LAUNCH(BKV)                                                                         \
  if (!g.a_kmajor && !g.b_kmajor)                                                                \
    hipLaunchKernelGGL((gemm_f32_kernel<false, false, BKV>), grid, block, 0, stream, p);        \
  else if (!g.a_kmajor && g.b_kmajor)                                                            \
    hipLaunchKernelGGL((gemm_f32_kernel<false, true, BKV>), grid, block, 0, stream, p);         \
  else if (g.a_kmajor && !g.b_kmajor)                                                            \
    hipLaunchKernelGGL((gemm_f32_kernel<true, false, BKV>), grid, block, 0, stream, p);         \
  else                                                                                           \
    hipLaunchKernelGGL((gemm_f32_kernel<true, true, BKV>), grid, block, 0, stream, p);
  if (BK == 16) {
    GEMM_LAUNCH(16)
  } else {
    GEMM_LAUNCH(32)
  }
#undef GEMM_LAUNCH
}

}  // namespace sdml
