// First layer of the MNIST MLPs fed straight from uint8 pixels (BASELINE configs 1-3): the
// forward GEMM y = relu(scale * X W^T + b) with X [M][K] uint8 and W [N][K] fp32.
//
// Numerics (same contract as gemm_f32x3.hip's uint8 path): a pixel byte is exact in one bf16, W is
// split exactly into three bf16 planes (hi + mid + lo = W), so every product is 3 exact bf16 MFMA
// products accumulated in fp32; ToTensor's 1/255 is applied in the epilogue. The reference does the
// same layer in fp32 on the CPU (/root/reference/simple_distributed.py:63, :75 for its fc layers,
// :87-88 for ToTensor).
//
// Accumulation: straight MFMA chains (no per-K-step fp32 partials). tools/probes/mfma_acc_probe.hip
// measured v_mfma_f32_32x32x16_bf16's accumulation on gfx950 as unbiased and more accurate than a
// k-ordered fp32 fmaf chain (K = 4096: 2.7e-7 vs 7.6e-7 mean relative error, bias 4e-9).
//
// Structure (gfx950, wave64): 512 threads = 8 waves as 4 (rows) x 2 (cols), block tile 256 x 128,
// wave tile 64 x 64 = 2 x 2 tiles of v_mfma_f32_32x32x16_bf16, K-step 64 (4 MFMA k-substeps).
// Both operands reach LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane, no VGPR staging)
// into a ring of NS stages (2 x 64 KiB; the DMA of K-step t+1 flies under K-step t's 48 MFMAs per
// wave). Measured alternative: 32-deep K-steps in a 4-stage ring (3 K-steps in flight), slower
// (102.6 vs 93.8 us at the headline shape: half the MFMAs per barrier).
// The LDS images are swizzled on the DMA's per-lane source address (the DMA writes 1 KiB
// lane-linearly) so the fragment ds_read_b128s are conflict-free; k order inside a K-step is
// permuted identically for both operands (lane half h, substep s, element j <-> k = 32h + 8s + j),
// so one 32-byte read per row tile feeds all four substeps of the pixel operand. Bytes are widened to
// bf16 in registers. The epilogue goes through LDS so every lane stores whole 16-byte row pieces.
// W is pre-split into zero-padded planes [3][N][Kp] (Kp = K rounded up to FBK), so the K tail needs
// no masking: past-the-end pixel bytes (clamped, finite) meet zero weights.
// Measured at 131072 x 784 -> 128 (tools/bench_u8.py): see README "uint8 pixels".
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "kernels.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int FT = 512;                       // threads
constexpr int FBM = 256;                      // rows per block
constexpr int FBN = 128;                      // columns per block
constexpr int FBK = 64;                       // k per K-step (FBK / 16 MFMA k-substeps)
constexpr int NS = 2;                         // LDS stages
constexpr int NSUB = FBK / 16;
constexpr int A_BYTES = FBM * FBK;            // raw pixel bytes per stage
constexpr int B_PLANE = FBN * FBK * 2;        // bytes per bf16 plane per stage
constexpr int STAGE = A_BYTES + 3 * B_PLANE;
constexpr int XCH = FBK / 16;                 // 16-B chunks per pixel row (2 or 4)
constexpr int WCH = FBK / 8;                  // 16-B chunks per weight row (4 or 8)
constexpr int GLDS_X = A_BYTES / 1024 / (FT / 64), GLDS_W = 3 * B_PLANE / 1024 / (FT / 64);
constexpr int GLDS_PER_STAGE = GLDS_X + GLDS_W;  // DMA instructions per wave per stage
static_assert(FBK == 32 || FBK == 64, "swizzles below are written for 32- and 64-deep K-steps");
static_assert(NS * STAGE <= 160 * 1024, "LDS");
static_assert(NS * STAGE >= (FT / 64) * 64 * 64 * 4, "the epilogue transposes each wave's 64 x 64 fp32 tile in the stage buffers");

// swizzled 16-B chunk positions: every 16-lane group of a fragment ds_read_b128 (16 rows, one
// logical chunk) hits 16 distinct bank groups
__device__ __forceinline__ int xpos(int r, int c) { return c ^ (XCH == 2 ? (r >> 3) & 1 : (r >> 2) & 3); }
__device__ __forceinline__ int wpos(int r, int c) { return c ^ (WCH == 4 ? (r >> 2) & 3 : (r >> 1) & 7); }

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ u16 bf16_bits(float f) { return __builtin_bit_cast(u16, static_cast<__bf16>(f)); }
__device__ __forceinline__ float bf16_val(u16 b) { return __uint_as_float(((unsigned)b) << 16); }

// 8 bytes -> 8 bf16 (exact: (float)b has its significant bits in the upper half)
__device__ __forceinline__ bf16x8 widen8(unsigned lo, unsigned hi) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = (short)(__float_as_uint((float)((lo >> (8 * e)) & 0xffu)) >> 16);
    r[4 + e] = (short)(__float_as_uint((float)((hi >> (8 * e)) & 0xffu)) >> 16);
  }
  return r;
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct FwdParams {
  const unsigned char* X;
  const u16* Wp;  // [3][N][Kp]
  const float* bias;
  float* C;
  int M, N, K, Kp, ldx, ldc;
  float scale;
  int relu;
};

// LDS images of one stage: X [256 rows][FBK bytes], W [3 planes][128 rows][FBK bf16], chunks at
// xpos / wpos. The DMA writes 1 KiB per wave-instruction lane-linearly (lane i -> bytes 16i..), so
// the swizzle goes on the per-lane SOURCE address.
__device__ __forceinline__ void issue_stage(const FwdParams& p, unsigned char* st, int m0, int n0, int k0, int wave,
                                           int lane) {
  constexpr int XROWS = 1024 / FBK;  // pixel rows per DMA instruction
#pragma unroll
  for (int u = 0; u < GLDS_X; ++u) {
    const int q = wave + (FT / 64) * u;
    const int row = XROWS * q + lane / XCH;
    const int pos = lane % XCH;
    const int ch = xpos(row, pos);  // xpos is an involution: the chunk stored at `pos`
    const int gr = min(m0 + row, p.M - 1);
    const int gk = min(k0 + 16 * ch, p.K - 16);  // past the end: finite bytes meeting zero weights
    glds16(p.X + (size_t)gr * p.ldx + gk, st + 1024 * q);
  }
  constexpr int WROWS = 1024 / (2 * FBK);  // weight rows per DMA instruction
  constexpr int WINST = FBN / WROWS;       // instructions per plane
  const size_t plane = (size_t)p.N * p.Kp;
#pragma unroll
  for (int u = 0; u < GLDS_W; ++u) {
    const int q = wave + (FT / 64) * u;
    const int pl = q / WINST;
    const int row = WROWS * (q % WINST) + lane / WCH;
    const int ch = wpos(row, lane % WCH);
    glds16(p.Wp + pl * plane + (size_t)(n0 + row) * p.Kp + k0 + 8 * ch, st + A_BYTES + 1024 * q);
  }
}

// MODE (timing experiments only): 0 = normal, 1 = no MFMA/LDS reads (DMA pipeline alone),
// 2 = no DMA in the K loop (compute on stale LDS), 3 = no LDS reads (MFMA on register data)
template <int MODE = 0>
__global__ void __launch_bounds__(FT) u8_fwd_kernel(FwdParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE];
  const int m0 = blockIdx.x * FBM, n0 = blockIdx.y * FBN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  const int h = lane >> 5, r32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // per-lane LDS read offsets (bytes, within a stage). k order inside a K-step, identical for both
  // operands: lane half h, substep s, element j <-> k = (FBK / 2) h + 8 s + j, so the lane's
  // FBK / 2 contiguous pixel bytes of a row feed all substeps of the X operand.
  int aoff[2][XCH / 2], boff[2][NSUB];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wm * 64 + 32 * i + r32;
#pragma unroll
    for (int c = 0; c < XCH / 2; ++c) aoff[i][c] = row * FBK + 16 * xpos(row, (XCH / 2) * h + c);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wn * 64 + 32 * j + r32;
#pragma unroll
    for (int s = 0; s < NSUB; ++s) boff[j][s] = A_BYTES + row * (2 * FBK) + 16 * wpos(row, NSUB * h + s);
  }

  // NS_ = substeps to run: NSUB, or fewer in the last K-step when only lane half 0's first
  // substeps hold k < K (the rest multiply zero-padded weights)
  auto kstep = [&](const unsigned char* st, auto ns_c) {
    constexpr int NS_ = decltype(ns_c)::value;
    if constexpr (MODE == 1) return;
    u32x4 araw[2][XCH / 2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < XCH / 2; ++c) {
        if constexpr (MODE == 3) araw[i][c] = u32x4{(unsigned)aoff[i][c], 1u, 2u, 3u};
        else araw[i][c] = *reinterpret_cast<const u32x4*>(st + aoff[i][c]);
      }
#pragma unroll
    for (int s = 0; s < NS_; ++s) {
      bf16x8 b[2][3];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          if constexpr (MODE == 3) b[j][pl] = bf16x8{(short)boff[j][s], (short)pl, 1, 2, 3, 4, 5, 6};
          else b[j][pl] = *reinterpret_cast<const bf16x8*>(st + boff[j][s] + pl * B_PLANE);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const u32x4 v = araw[i][s >> 1];
        const bf16x8 a = (s & 1) ? widen8(v[2], v[3]) : widen8(v[0], v[1]);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma(a, b[j][2], acc[i][j]);  // lo
          acc[i][j] = mfma(a, b[j][1], acc[i][j]);  // mid
          acc[i][j] = mfma(a, b[j][0], acc[i][j]);  // hi
        }
      }
    }
  };

  // NS-stage ring: K-step t computes stage t % NS while the DMA of K-steps t+1 .. t+NS-1 is in
  // flight. A stage is refilled only after the barrier that follows its last reads, and read only
  // after every wave's counted vmcnt for it plus the following barrier (a raw s_barrier keeps the
  // younger DMAs in flight: __syncthreads() would drain them). Full K-steps only: the W planes are
  // zero-padded to Kp.
  const int nk = p.Kp / FBK;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue_stage(p, smem + t * STAGE, m0, n0, t * FBK, wave, lane);
  auto sync_step = [&](int t) {  // stage t % NS landed and visible; stage (t - 1) % NS free
    const int ahead = min(NS - 2, nk - 1 - t);  // K-steps issued after t that may stay in flight
    if constexpr (NS >= 4) {
      if (ahead >= 2) wait_vmcnt<2 * GLDS_PER_STAGE>();
      else if (ahead == 1) wait_vmcnt<GLDS_PER_STAGE>();
      else wait_vmcnt<0>();
    } else if constexpr (NS == 3) {
      if (ahead >= 1) wait_vmcnt<GLDS_PER_STAGE>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS access moves across the barrier
    if constexpr (MODE != 2) {
      if (t + NS - 1 < nk) issue_stage(p, smem + ((t + NS - 1) % NS) * STAGE, m0, n0, (t + NS - 1) * FBK, wave, lane);
    }
  };
  for (int t = 0; t + 1 < nk; ++t) {
    sync_step(t);
    kstep(smem + (t % NS) * STAGE, std::integral_constant<int, NSUB>{});
  }
  {  // last K-step: only the substeps holding k < K (lane half 0 covers the first FBK / 2 k)
    sync_step(nk - 1);
    const unsigned char* st = smem + ((nk - 1) % NS) * STAGE;
    const int v = p.K - (nk - 1) * FBK;
    if (v > FBK / 2 - 8) kstep(st, std::integral_constant<int, NSUB>{});
    else if (NSUB == 4 && v > 16) kstep(st, std::integral_constant<int, 3>{});
    else if (NSUB == 4 && v > 8) kstep(st, std::integral_constant<int, 2>{});
    else kstep(st, std::integral_constant<int, 1>{});
  }

  // epilogue: relu(scale * acc + bias), transposed through LDS so that every lane stores whole
  // 16-byte row pieces (a wave's 64 x 64 fp32 tile = 16 KiB; the 8 tiles reuse the 128 KiB of
  // stage buffers, free after the barrier that ended the last K-step)
  __syncthreads();
  float* T = reinterpret_cast<float*>(smem) + wave * 64 * 64;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + 32 * j + r32;
    const float bv = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float y = acc[i][j][r] * p.scale + bv;
        if (p.relu) y = fmaxf(y, 0.f);
        T[(32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * 64 + 32 * j + r32] = y;
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile is in LDS (wave-private region)
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int rr = 4 * q + (lane >> 4);
    const int row = m0 + wm * 64 + rr;
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + rr * 64 + 4 * (lane & 15));
    if (row < p.M) *reinterpret_cast<f32x4*>(p.C + (size_t)row * p.ldc + n0 + wn * 64 + 4 * (lane & 15)) = v;
  }
}

// fp32 [N][K] -> three zero-padded bf16 planes [3][N][Kp] (hi + mid + lo == w exactly)
__global__ void __launch_bounds__(256) split3_pad_kernel(const float* __restrict__ w, u16* __restrict__ out, int N,
                                                         int K, int Kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element of the padded [N][Kp]
  const int64_t n = (int64_t)N * Kp;
  if (i >= n) return;
  const int r = (int)(i / Kp), k = (int)(i % Kp);
  const float x = k < K ? w[(size_t)r * K + k] : 0.f;
  const u16 hi = bf16_bits(x);
  const float r1 = x - bf16_val(hi);
  const u16 mi = bf16_bits(r1);
  const u16 lo = bf16_bits(r1 - bf16_val(mi));
  out[i] = hi;
  out[n + i] = mi;
  out[2 * n + i] = lo;
}

}  // namespace

int u8_fwd_kpad(int K) { return (K + FBK - 1) / FBK * FBK; }  // zero-padded W planes

bool u8_fwd_supported(int M, int N, int K, int ldx, const void* X) {
  // (the epilogue stores 16-B row pieces: C 16-B aligned with ldc % 4 == 0, checked by the caller)
  return M >= FBM && N % FBN == 0 && K >= 16 && K % 16 == 0 && ldx % 16 == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (int64_t)M * ldx < (int64_t(1) << 31);
}

void split3_pad(const float* w, unsigned short* out, int N, int K, int Kp, hipStream_t stream) {
  const int64_t n = (int64_t)N * Kp;
  hipLaunchKernelGGL(split3_pad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, w, out, N, K, Kp);
}

void u8_fwd(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_planes, int N, int Kp,
            const float* bias, float* C, int ldc, bool relu, float scale, hipStream_t stream) {
  FwdParams p;
  p.X = X;
  p.Wp = w_planes;
  p.bias = bias;
  p.C = C;
  p.M = M;
  p.N = N;
  p.K = K;
  p.Kp = Kp;
  p.ldx = ldx;
  p.ldc = ldc;
  p.scale = scale;
  p.relu = relu ? 1 : 0;
  static const int mode = [] {
    const char* e = getenv("SDML_U8_FWD_MODE");
    return e ? atoi(e) : 0;
  }();
  const dim3 grid((M + FBM - 1) / FBM, N / FBN);
  if (mode == 1) hipLaunchKernelGGL(u8_fwd_kernel<1>, grid, dim3(FT), 0, stream, p);
  else if (mode == 2) hipLaunchKernelGGL(u8_fwd_kernel<2>, grid, dim3(FT), 0, stream, p);
  else if (mode == 3) hipLaunchKernelGGL(u8_fwd_kernel<3>, grid, dim3(FT), 0, stream, p);
  else hipLaunchKernelGGL(u8_fwd_kernel<0>, grid, dim3(FT), 0, stream, p);
}

}  // namespace sdml
