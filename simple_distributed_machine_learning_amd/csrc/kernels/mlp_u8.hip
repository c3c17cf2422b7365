// First layer of the MNIST MLPs fed straight from uint8 pixels (BASELINE configs 1-3): the
// forward GEMM y = relu(scale * X W^T + b) with X [M][K] uint8 and W [N][K] fp32.
//
// Numerics: a pixel byte is exact in one fp16, and W is held as two fp16 planes of W * 2^8
// (u8_planes.h: hi + lo is W to within one fp32 ulp), so every product is 2 exact
// fp16 MFMA products accumulated in fp32; ToTensor's 1/255 and the 2^-8 are applied in the
// epilogue. (Round 1 and the first half of round 2 used 3 exact bf16 planes, 3 MFMAs per product;
// the pair of fp16 planes carries the same 24 bits in 2.) The reference does the same layer in fp32
// on the CPU (/root/reference/simple_distributed.py:63, :75 for its fc layers, :87-88 for ToTensor).
//
// Accumulation: straight MFMA chains (no per-K-step fp32 partials). tools/probes/mfma_acc_probe.hip
// measured v_mfma_f32_32x32x16_bf16's accumulation on gfx950 as unbiased and more accurate than a
// k-ordered fp32 fmaf chain (K = 4096: 2.7e-7 vs 7.6e-7 mean relative error, bias 4e-9).
//
// Structure (gfx950, wave64): NWR x 2 waves (4 x 2 = 512 threads, or 8 x 2 = 1024 threads for the
// 512-row blocks of large batches, 4 waves per SIMD), wave tile 32 WMT x 64 = WMT x 2 tiles of
// v_mfma_f32_32x32x16_f16, block tile 32 WMT NWR x 128, K-step 64 (4 MFMA k-substeps).
// Both operands reach LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane, no VGPR staging)
// into a ring of NS stages (the DMA of K-step t+1 flies under K-step t's MFMAs). Measured
// alternatives (on the 3-plane bf16 form): 32-deep K-steps in a 4-stage ring (3 K-steps in flight),
// slower (102.6 vs 93.8 us at the headline shape: half the MFMAs per barrier); weight fragments of
// substep s+1 pinned ahead of substep s's MFMAs with sched_barrier (register double buffer),
// 2-3 % slower than the compiler's own placement; 1024-thread blocks of 512 rows did not fit 4 waves
// per SIMD with 3 planes (~400 VGPRs spilled at 128) - with 2 planes they need 115 and are the
// default for large batches (62-65 vs 66.5-67.3 us for 8 waves of 128 x 64).
// The LDS images are swizzled on the DMA's per-lane source address (the DMA writes 1 KiB
// lane-linearly) so the fragment ds_read_b128s are conflict-free; k order inside a K-step is
// permuted identically for both operands (lane half h, substep s, element j <-> k = 32h + 8s + j),
// so one 32-byte read per row tile feeds all four substeps of the pixel operand. Bytes are widened to
// fp16 in registers (a byte permute builds 1024 + b, one packed subtract removes the 1024). The
// epilogue goes through LDS so every lane stores whole 16-byte row pieces.
// W is pre-split into zero-padded planes [2][N][Kp] (Kp = K rounded up to FBK), so the K tail needs
// no masking: past-the-end pixel bytes (clamped, finite) meet zero weights.
// Measured at 131072 x 784 -> 128 (tools/bench_u8.py): see README "uint8 pixels".
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "head_block.h"
#include "head_reduce.h"
#include "head_tile.h"
#include "lds_dma.h"
#include "kernels.h"
#include "sgd_rule.h"
#include "wave_ops.h"
#include "u8_planes.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr int FBN = 128;                      // columns per block
constexpr int FBK = 64;                       // k per K-step (FBK / 16 MFMA k-substeps)
constexpr int NS = 2;                         // LDS stages
constexpr int NSUB = FBK / 16;
constexpr int NPL = kU8FwdPlanes;            // fp16 weight planes
constexpr int B_PLANE = FBN * FBK * 2;        // bytes per fp16 plane per stage
constexpr int XCH = FBK / 16;                 // 16-B chunks per pixel row (2 or 4)
constexpr int WCH = FBK / 8;                  // 16-B chunks per weight row (4 or 8)
static_assert(FBK == 32 || FBK == 64, "swizzles below are written for 32- and 64-deep K-steps");

// block geometry per WMT = 32-row MFMA tiles per wave and NWR = row waves (the block is NWR x 2
// waves; wave tile 32 WMT x 64, block 32 WMT NWR x 128). NWR = 4: 512 threads (2 waves per SIMD);
// NWR = 8: 1024 threads (4 waves per SIMD, <= 128 VGPRs)
template <int WMT, int NWR = 4, int NSG = NS>
struct Geo {
  static constexpr int THREADS = 128 * NWR;
  static constexpr int WAVES = THREADS / 64;
  static constexpr int BM = NWR * 32 * WMT;         // rows per block
  static constexpr int A_BYTES = BM * FBK;          // raw pixel bytes per stage
  static constexpr int STAGE = A_BYTES + NPL * B_PLANE;
  static constexpr int GLDS_X = A_BYTES / 1024 / WAVES;
  static constexpr int GLDS_W = NPL * B_PLANE / 1024 / WAVES;
  static constexpr int GLDS_PER_STAGE = GLDS_X + GLDS_W;  // DMA instructions per wave per stage
  static_assert(GLDS_X * 1024 * WAVES == A_BYTES && GLDS_W * 1024 * WAVES == NPL * B_PLANE, "DMA split");
  // the epilogue transposes EPR x 64 fp32 per wave through the (then free) stage buffers
  static constexpr int EPR = WAVES * 64 * 64 * 4 <= 128 * 1024 ? 64 : 32;
  static constexpr int SMEM = std::max(NSG * STAGE, WAVES * EPR * 64 * 4);
  static_assert(SMEM <= 160 * 1024, "LDS");
};

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

// 8 bytes -> 8 fp16 (exact): a byte permute puts b under the exponent of 1024 (fp16 0x6400 | b ==
// 1024 + b), one packed subtract per pair removes the 1024
__device__ __forceinline__ f16x2 h2_of(unsigned v, unsigned sel) {
  const unsigned t = __builtin_amdgcn_perm(0x64646464u, v, sel);
  return __builtin_bit_cast(f16x2, t) - f16x2{(_Float16)1024.f, (_Float16)1024.f};
}
__device__ __forceinline__ f16x8 widen8h(unsigned lo, unsigned hi) {
  const f16x2 a = h2_of(lo, 0x04010400u), b = h2_of(lo, 0x04030402u);
  const f16x2 c = h2_of(hi, 0x04010400u), d = h2_of(hi, 0x04030402u);
  return f16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

struct FwdParams {
  const unsigned char* X;
  const u16* Wp;  // [NPL][N][Kp] fp16 bits
  const float* bias;
  float* C;
  int M, N, K, Kp, ldx, ldc;
  float scale;
  int relu;
  int prio;        // 1: s_setprio 1 on the second half of the waves (each SIMD's younger wave; A/B knob U8_FWD_PRIO)
  unsigned* mask;  // optional [M][N / 32] ReLU bits (plain epilogue)
  float* wmax;     // optional [blocks][WAVES] per-wave max of the stored outputs (plain epilogue): a bound the
                   // next layer's two-plane split (gemm_f16x2.hip) reads instead of an inf-norm pass
  U8HeadArgs head;  // fused head epilogue (HEADC > 0)
  int pf_stride;   // fused head: > 0 = during the epilogue, LDS-DMA block blockIdx + pf_stride's first two K-steps of
                   // pixels into a scratch KiB, so they sit in this XCD's L2 when that block starts (knob U8_FWD_PREFETCH)
  long long* stamps;  // MODE 7 (experiments builds only): per-wave phase stamps, U8_NSTAMP per (block, wave)
};

// MODE 7 diagnostic stamps (tools/probes/u8_fwd_stamps.py): lane 0 of every wave writes s_memtime after each
// phase (vector stores into a buffer nothing else reads); slots 0 / U8_NSTAMP - 1 hold s_memrealtime
constexpr int U8_NSTAMP = 24;
#ifdef SDML_KERNEL_EXPERIMENTS
long long* g_u8_stamps = nullptr;   // u8_set_stamps: the fused forward's MODE 7 buffer
long long* g_u8w_stamps = nullptr;  // u8_set_wgrad_stamps: the weight gradient's phase stamps
#endif
#define U8_STAMP(k, fn)                                                                                  \
  do {                                                                                                   \
    if constexpr (MODE == 7) {                                                                           \
      if (lane == 0) p.stamps[((size_t)blockIdx.x * G::WAVES + wave) * U8_NSTAMP + (k)] = (long long)fn(); \
    }                                                                                                    \
  } while (0)

// ---- fused classifier-head epilogue (HEADC > 0; WMT = 2, NWR = 4: 8 waves, 256 rows x 128 hidden per block):
// head_block.h (fp16-plane MFMA head, its LDS image in the then free stage buffers). Round 4's 4-wave 128-row
// variant (knob U8_FH_WAVES = 4, two blocks per CU) measured slower and is gone with the fp32-MFMA epilogue.

// LDS images of one stage: X [BM rows][FBK bytes], W [NPL planes][128 rows][FBK fp16], chunks at
// xpos / wpos. The DMA writes 1 KiB per wave-instruction lane-linearly (lane i -> bytes 16i..), so
// the swizzle goes on the per-lane SOURCE address.
// pieces [U0, U1) of the wave's GLDS_X + GLDS_W DMA pieces of the stage (the spread K-step issues them in parts)
template <int WMT, int NWR, int U0 = 0, int U1 = 1 << 20>
__device__ __forceinline__ void issue_stage(const FwdParams& p, unsigned char* st, int m0, int n0, int k0, int wave,
                                           int lane) {
  using G = Geo<WMT, NWR>;
  // buffer-form DMA (lds_dma.h: keeps the fragment reads' lgkmcnt waits counted); u8_fwd_supported keeps
  // M * ldx < 2^31, the planes are small
  const __amdgpu_buffer_rsrc_t rx = dma_rsrc(p.X, (unsigned)((size_t)p.M * p.ldx));
  const __amdgpu_buffer_rsrc_t rw = dma_rsrc(p.Wp, (unsigned)((size_t)NPL * p.N * p.Kp * 2));
  constexpr int XROWS = 1024 / FBK;  // pixel rows per DMA instruction
#pragma unroll
  for (int u = 0; u < G::GLDS_X; ++u) {
    if (u < U0 || u >= U1) continue;
    const int q = wave + G::WAVES * u;
    const int row = XROWS * q + lane / XCH;
    const int pos = lane % XCH;
    const int ch = xpos(row, pos);  // xpos is an involution: the chunk stored at `pos`
    const int gr = min(m0 + row, p.M - 1);
    const int gk = min(k0 + 16 * ch, p.K - 16);  // past the end: finite bytes meeting zero weights
    bdma16(rx, (unsigned)((size_t)gr * p.ldx + gk), st + 1024 * q);
  }
  constexpr int WROWS = 1024 / (2 * FBK);  // weight rows per DMA instruction
  constexpr int WINST = FBN / WROWS;       // instructions per plane
  const size_t plane = (size_t)p.N * p.Kp;
#pragma unroll
  for (int u = 0; u < G::GLDS_W; ++u) {
    if (G::GLDS_X + u < U0 || G::GLDS_X + u >= U1) continue;
    const int q = wave + G::WAVES * u;
    const int pl = q / WINST;
    const int row = WROWS * (q % WINST) + lane / WCH;
    const int ch = wpos(row, lane % WCH);
    bdma16(rw, (unsigned)(2 * (pl * plane + (size_t)(n0 + row) * p.Kp + k0 + 8 * ch)), st + G::A_BYTES + 1024 * q);
  }
}

// MODE (timing experiments only): 0 = normal, 1 = no MFMA/LDS reads (DMA pipeline alone),
// 4 = no DMA and no barrier in the K loop, 5 = no byte widening (MFMA on raw bytes), 6 = no output stores,
// 2 = no DMA in the K loop (compute on stale LDS), 3 = no LDS reads (MFMA on register data)
// TAIL = MFMA substeps of the last K-step (tail_substeps: only those holding k < K; chosen on the
// host so the kernel carries one straight-line tail)
template <int C, int NWR>
__device__ __forceinline__ void fused_head_epilogue(const FwdParams& p, const f32x16 (&acc)[2][2], unsigned char* smem,
                                                    int m0, int wave, int lane, int wm, int wn,
                                                    const hblk::Operands& ops, const float (&bv1)[2], long long* stamp,
                                                    int hb);
template <int C>
__device__ __forceinline__ void fused_head_prefetch(const FwdParams& p, int m0, int wave, int lane, int wn,
                                                    hblk::Operands& ops, float (&bv1)[2]);

// HEADC = 0: store h = act(scale acc + b) (+ its ReLU bits when p.mask); HEADC = C > 0: the fused
// classifier head on h (fused_head_epilogue), h is never stored
// NSK: LDS ring stages. The fused-head variant may take 3 (the head epilogue needs 148 KiB anyway, so a third
// 48 KiB stage costs no occupancy: two K-steps of pixel DMA in flight instead of one).
// DMAS: 0 = the next stage's DMA issued right after the K-step's barrier (all pieces before the first MFMA), 1 = spread
// over the first substeps (two pieces after each substep's MFMAs: the issue cost of a piece hides under MFMAs instead
// of delaying the first ones; knob U8_FWD_DMA_SPREAD, NS == 2 only), 2 = 1 + each substep's fragments read one substep
// ahead
template <int MODE, int WMT, int TAIL, int NWR, int HEADC = 0, int NSK = NS, int DMAS = 0>
__global__ void __launch_bounds__(128 * NWR, NWR == 2 ? 2 : 1) u8_fwd_kernel(FwdParams p) {  // (4-wave blocks: 2 waves per SIMD, <= 256 VGPRs, two blocks per CU)
  constexpr int NS = NSK;  // (shadows the file-wide default inside this kernel)
  using G = Geo<WMT, NWR, NSK>;
  static_assert(HEADC == 0 || ((WMT == 2 || WMT == 4) && NWR == 4), "the fused head epilogue: 8 waves of 64 x 64");
  // HALVES (fused head, WMT = 4: 512-row blocks): a wave's four 32-row tiles are rows 64 wm + {0, 32} of each 256-row
  // half of the block (not 128 consecutive rows), so tiles 0, 1 of every wave are the first half's h in exactly the
  // layout head_block.h takes for a 256-row block, and tiles 2, 3 the second's: the head runs twice on unchanged code.
  // Why 512 rows: every block streams all of W's planes through LDS per K-step (32 KiB), once per 256 rows before;
  // now once per 512 (a third less LDS-DMA per row), one block per CU in one round instead of two.
  constexpr bool HALVES = HEADC > 0 && WMT == 4;
  auto tile_row = [](int i) { return HALVES ? 32 * (i & 1) + 256 * (i >> 1) : 32 * i; };
  static_assert(HEADC == 0 || G::SMEM <= hblk::LDS_BYTES, "the prefetch scratch KiB sits past the ring and the head");
  constexpr int STAGE = G::STAGE, GLDS_PER_STAGE = G::GLDS_PER_STAGE;
  constexpr int SMEM_BYTES = HEADC ? std::max(G::SMEM, hblk::LDS_BYTES) + 1024 : G::SMEM;  // (+ the prefetch scratch)
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
  const int m0 = blockIdx.x * G::BM, n0 = blockIdx.y * FBN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % NWR, wn = wave / NWR;
  // static priority for the second-dispatched half (waves w and w + WAVES / 2 share a SIMD): the guide's
  // MI355X_MICROARCH "Two waves per SIMD" item 4 (knob, off by default until measured here)
  if (p.prio && wave >= G::WAVES / 2) __builtin_amdgcn_s_setprio(1);
  const int h = lane >> 5, r32 = lane & 31;
  U8_STAMP(0, __builtin_amdgcn_s_memrealtime);
  U8_STAMP(1, __builtin_amdgcn_s_memtime);
  // the head's W2, biases and targets (and fc1's bias): requested inside the K loop (K-step nk - 4), used after it.
  // (Requested here, at the start, they cost as much in the prologue as they saved in the epilogue: 256 blocks x 8
  // waves x 8 KB of W2 reads in one burst with the first DMA stages, stamps r5)
  hblk::Operands hops;
  float hb1[2];

  f32x16 acc[WMT][2];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // per-lane LDS read offsets (bytes, within a stage). k order inside a K-step, identical for both
  // operands: lane half h, substep s, element j <-> k = (FBK / 2) h + 8 s + j, so the lane's
  // FBK / 2 contiguous pixel bytes of a row feed all substeps of the X operand.
  // (the swizzles use row bits below 5 only, so tiles 32 rows apart differ by a constant offset)
  int aoff[XCH / 2], boff[NSUB];
  {
    const int row = (HALVES ? wm * 64 : wm * 32 * WMT) + r32;
#pragma unroll
    for (int c = 0; c < XCH / 2; ++c) aoff[c] = row * FBK + 16 * xpos(row, (XCH / 2) * h + c);
  }
  {
    const int row = wn * 64 + r32;
#pragma unroll
    for (int s = 0; s < NSUB; ++s) boff[s] = G::A_BYTES + row * (2 * FBK) + 16 * wpos(row, NSUB * h + s);
  }

  // NS_ = substeps to run: NSUB, or fewer in the last K-step when only lane half 0's first
  // substeps hold k < K (the rest multiply zero-padded weights)
  auto load_a = [&](const unsigned char* st, int s2, u32x4 (&ar)[WMT]) {  // 16 B = substeps 2 s2, 2 s2 + 1
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      if constexpr (MODE == 3) ar[i] = u32x4{(unsigned)aoff[s2], 1u, 2u, 3u};
      else ar[i] = *reinterpret_cast<const u32x4*>(st + aoff[s2] + FBK * tile_row(i));
    }
  };
  auto load_b = [&](const unsigned char* st, int s, f16x8 (&b)[2][NPL]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        if constexpr (MODE == 3) b[j][pl] = __builtin_bit_cast(f16x8, bf16x8{(short)boff[s], (short)pl, (short)j, 2, 3, 4, 5, 6});
        else b[j][pl] = *reinterpret_cast<const f16x8*>(st + boff[s] + 64 * FBK * j + pl * B_PLANE);
      }
  };
  auto compute = [&](int s, const u32x4 (&ar)[WMT], const f16x8 (&b)[2][NPL]) {
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      const u32x4 v = ar[i];
      f16x8 a;
      if constexpr (MODE == 5) a = __builtin_bit_cast(f16x8, v);  // timing only: no widening
      else a = (s & 1) ? widen8h(v[2], v[3]) : widen8h(v[0], v[1]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pl = NPL - 1; pl >= 0; --pl) acc[i][j] = mfma(a, b[j][pl], acc[i][j]);  // lo first
    }
  };
  // DMA_AT: substep after whose MFMAs a K-step issues the next stage's DMA (-1: right after the barrier, the
  // production schedule; MODE 8 / 9, experiments: after substep 0 / 1)
  constexpr int DMA_AT = MODE == 8 ? 0 : (MODE == 9 ? 1 : -1);
  static_assert(DMAS == 0 || (NSK == 2 && DMA_AT < 0 && MODE != 11 && GLDS_PER_STAGE == 6),
                "spread DMA: the 2-stage production loop, 6 pieces per wave");
  // PIPE: the pipelined K-step (MODE 11, experiments)
  constexpr bool PIPE = MODE == 11;
  auto kstep = [&](const unsigned char* st, auto ns_c, auto&& dma, auto&& dma_part) {
    constexpr int NS_ = decltype(ns_c)::value;
    if constexpr (MODE == 1) return;
    // (reading substep s+1's fragments ahead of substep s's MFMAs, pinned with sched_barrier,
    // measured no faster at either geometry: 87.2 vs 87.5 us; neither did s_setprio 1 around
    // each substep's MFMAs: 92.3-92.9 vs 91.5-93.4 us)
    if constexpr (PIPE) {
      // register double buffer: substep s + 1's fragment reads are issued before substep s's MFMAs (pinned
      // with sched_barrier), so each counted lgkmcnt wait covers reads that had a whole substep of MFMAs
      // to land; the next stage's DMA goes out while substep 0's reads are in flight
      u32x4 ar[2][WMT];
      f16x8 b[2][2][NPL];
      load_a(st, 0, ar[0]);
      load_b(st, 0, b[0]);
      dma();
#pragma unroll
      for (int s = 0; s < NS_; ++s) {
        if (s + 1 < NS_) {
          if ((s + 1) % 2 == 0) load_a(st, (s + 1) >> 1, ar[((s + 1) >> 1) & 1]);
          load_b(st, s + 1, b[(s + 1) & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        compute(s, ar[(s >> 1) & 1], b[s & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (DMAS == 2) {
      // spread DMA + substep s + 1's fragment reads issued ahead of substep s's MFMAs (register double buffer, the
      // compiler's own placement: no sched_barrier)
      u32x4 ar[2][WMT];
      f16x8 b[2][2][NPL];
      load_a(st, 0, ar[0]);
      load_b(st, 0, b[0]);
#pragma unroll
      for (int s = 0; s < NS_; ++s) {
        if (s + 1 < NS_) {
          if ((s + 1) % 2 == 0) load_a(st, (s + 1) >> 1, ar[((s + 1) >> 1) & 1]);
          load_b(st, s + 1, b[(s + 1) & 1]);
        }
        compute(s, ar[(s >> 1) & 1], b[s & 1]);
        dma_part(s);
      }
    } else {
      u32x4 ar[WMT];
      f16x8 b[2][NPL];
#pragma unroll
      for (int s = 0; s < NS_; ++s) {
        if (s % 2 == 0) load_a(st, s >> 1, ar);
        load_b(st, s, b);
        compute(s, ar, b);
        if (s == DMA_AT) dma();
        if constexpr (DMAS == 1) dma_part(s);
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
    if (t < nk) issue_stage<WMT, NWR>(p, smem + t * STAGE, m0, n0, t * FBK, wave, lane);
  // stage t % NS landed and visible; stage (t - 1) % NS free; ISSUE: refill it with K-step t+NS-1
  // (the main loop passes a compile-time true so its body stays one basic block)
  auto sync_step = [&](int t, auto issue_c) {
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
    if constexpr (MODE != 4) {  // (MODE 4, timing only: no DMA and no barrier)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("" ::: "memory");  // no LDS access moves across the barrier
    if constexpr (MODE != 2 && MODE != 4 && decltype(issue_c)::value) {
      if (NS == 2 || t + NS - 1 < nk)
        issue_stage<WMT, NWR>(p, smem + ((t + NS - 1) % NS) * STAGE, m0, n0, (t + NS - 1) * FBK, wave, lane);
    }
  };
  auto no_dma = [] {};
  auto no_dma_part = [](int) {};
  for (int t = 0; t + 1 < nk; ++t) {  // NS == 2: K-step t + 1 always exists here
    sync_step(t, std::integral_constant<bool, (DMA_AT < 0 && !PIPE && DMAS == 0)>{});
    if (t < 13) U8_STAMP(2 + t, __builtin_amdgcn_s_memtime);
    if constexpr (HEADC > 0) {
      if (t == nk - 4) fused_head_prefetch<HEADC>(p, m0, wave, lane, wn, hops, hb1);
    }
    unsigned char* nxt = smem + ((t + NS - 1) % NS) * STAGE;
    const int k1 = (t + NS - 1) * FBK;
    kstep(
        smem + (t % NS) * STAGE, std::integral_constant<int, NSUB>{},
        [&] {
          if (NS == 2 || t + NS - 1 < nk) issue_stage<WMT, NWR>(p, nxt, m0, n0, k1, wave, lane);
        },
        [&](int sub) {  // DMAS == 1 (NS == 2): two of the 6 pieces after each of the first three substeps
          if (sub == 0) issue_stage<WMT, NWR, 0, 2>(p, nxt, m0, n0, k1, wave, lane);
          else if (sub == 1) issue_stage<WMT, NWR, 2, 4>(p, nxt, m0, n0, k1, wave, lane);
          else if (sub == 2) issue_stage<WMT, NWR, 4, 1 << 20>(p, nxt, m0, n0, k1, wave, lane);
        });
  }
  {  // last K-step: only the substeps holding k < K (lane half 0 covers the first FBK / 2 k)
    sync_step(nk - 1, std::integral_constant<bool, (NS > 2)>{});
    kstep(smem + ((nk - 1) % NS) * STAGE, std::integral_constant<int, TAIL>{}, no_dma, no_dma_part);
  }
  U8_STAMP(15, __builtin_amdgcn_s_memtime);
  if constexpr (MODE == 10) {  // timing only: the K loop alone (keep the accumulators alive)
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < WMT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) keep += acc[i][j][r];
    if (keep == 12345.f && lane == 99) p.stamps[0] = 1;
    return;
  }

  if constexpr (HEADC > 0) {
    long long* stp = MODE == 7 ? p.stamps + ((size_t)blockIdx.x * G::WAVES + wave) * U8_NSTAMP : nullptr;
    if constexpr (!HALVES) {
      fused_head_epilogue<HEADC, NWR>(p, acc, smem, m0, wave, lane, wm, wn, hops, hb1, stp, (int)blockIdx.x);
    } else {  // two 256-row head blocks: tiles 0, 1 then 2, 3 of every wave (see HALVES)
      typedef const f32x16 Half[2][2];
      fused_head_epilogue<HEADC, NWR>(p, *reinterpret_cast<Half*>(&acc[0][0]), smem, m0, wave, lane, wm, wn, hops, hb1,
                                      stp, 2 * (int)blockIdx.x);
      if (m0 + hblk::ROWS < p.M) {  // (block-uniform) the second half holds rows
        __syncthreads();  // every wave is done with the first head's LDS
        fused_head_prefetch<HEADC>(p, m0 + hblk::ROWS, wave, lane, wn, hops, hb1);
        fused_head_epilogue<HEADC, NWR>(p, *reinterpret_cast<Half*>(&acc[2][0]), smem, m0 + hblk::ROWS, wave, lane, wm,
                                        wn, hops, hb1, nullptr, 2 * (int)blockIdx.x + 1);
      }
    }
    U8_STAMP(22, __builtin_amdgcn_s_memtime);
    U8_STAMP(U8_NSTAMP - 1, __builtin_amdgcn_s_memrealtime);
    return;
  }
  // epilogue: relu(scale * acc + bias), transposed through LDS so that every lane stores whole
  // 16-byte row pieces, EPR rows of the wave tile at a time (EPR x 64 fp32 per wave; the waves'
  // pieces reuse the stage buffers, free after the barrier that ended the last K-step)
  __syncthreads();
  constexpr int EPR = G::EPR, NI2 = EPR / 32;
  float* T = reinterpret_cast<float*>(smem) + wave * EPR * 64;
  float bv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bv[j] = p.bias ? p.bias[n0 + wn * 64 + 32 * j + r32] : 0.f;
  float vmax = 0.f;
#pragma unroll
  for (int ip = 0; ip < WMT / NI2; ++ip) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous piece's reads are done
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i2 = 0; i2 < NI2; ++i2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float y = acc[NI2 * ip + i2][j][r] * p.scale + bv[j];
          if (p.relu) y = fmaxf(y, 0.f);
          T[(32 * i2 + (r & 3) + 8 * (r >> 2) + 4 * h) * 64 + 32 * j + r32] = y;
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's piece is in LDS (wave-private region)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < EPR / 4; ++q) {
      const int rr = 4 * q + (lane >> 4);
      const int row = m0 + wm * 32 * WMT + EPR * ip + rr;
      const f32x4 v = *reinterpret_cast<const f32x4*>(T + rr * 64 + 4 * (lane & 15));
      if constexpr (MODE == 6) {  // timing only: no global stores (keep the values alive)
        if (v[0] == 12345.f && row < 0) *reinterpret_cast<f32x4*>(p.C) = v;
      } else if (row < p.M) {
        *reinterpret_cast<f32x4*>(p.C + (size_t)row * p.ldc + n0 + wn * 64 + 4 * (lane & 15)) = v;
        vmax = fmaxf(fmaxf(vmax, fmaxf(fabsf(v[0]), fabsf(v[1]))), fmaxf(fabsf(v[2]), fabsf(v[3])));
      }
      if (p.mask) {  // ReLU bits: the 8 lanes holding 32 columns of the row OR their nibbles into one word
        unsigned w = ((v[0] > 0.f ? 1u : 0u) | (v[1] > 0.f ? 2u : 0u) | (v[2] > 0.f ? 4u : 0u) |
                      (v[3] > 0.f ? 8u : 0u)) << (4 * (lane & 7));
        w |= __shfl_xor(w, 1);
        w |= __shfl_xor(w, 2);
        w |= __shfl_xor(w, 4);
        if ((lane & 7) == 0 && row < p.M)
          p.mask[(size_t)row * (p.N / 32) + (n0 + wn * 64) / 32 + ((lane & 15) >> 3)] = w;
      }
    }
  }
  if (p.wmax) {
    for (int off = 32; off > 0; off >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, off));
    if (lane == 0) p.wmax[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * G::WAVES + wave] = vmax;
  }
}

// ReLU-bit words of tile (i, j) = (Q >> 5, (Q >> 4) & 1), registers r = Q & 15 .. +3 (rows rw = 32 i + 8 (r >> 2) + e
// and rw + 4 of the wave, e = 0..3): each ballot's halves go to lanes rw and rw + 4 of mw[j] (lane selects inline
// constants). The ballots are VALU writes of SGPRs that v_writelane reads as data: the hazard recognizer does not look
// into the asm string, so it opens with the wait states itself (without them a writelane read the previous ballot).
template <int Q>
__device__ __forceinline__ void mask_words(const f32x16 (&y)[2][2], int (&mw)[2]) {
  if constexpr (Q < 64) {
    constexpr int i = Q >> 5, j = (Q >> 4) & 1, r = Q & 15, rw = 32 * i + 8 * (r >> 2);
    const unsigned long long b0 = __ballot(y[i][j][r] > 0.f), b1 = __ballot(y[i][j][r + 1] > 0.f);
    const unsigned long long b2 = __ballot(y[i][j][r + 2] > 0.f), b3 = __ballot(y[i][j][r + 3] > 0.f);
    asm("s_nop 4\n\t"
        "v_writelane_b32 %0, %1, %9\n\tv_writelane_b32 %0, %2, %10\n\t"
        "v_writelane_b32 %0, %3, %11\n\tv_writelane_b32 %0, %4, %12\n\t"
        "v_writelane_b32 %0, %5, %13\n\tv_writelane_b32 %0, %6, %14\n\t"
        "v_writelane_b32 %0, %7, %15\n\tv_writelane_b32 %0, %8, %16"
        : "+v"(mw[j])
        : "s"((unsigned)b0), "s"((unsigned)(b0 >> 32)), "s"((unsigned)b1), "s"((unsigned)(b1 >> 32)),
          "s"((unsigned)b2), "s"((unsigned)(b2 >> 32)), "s"((unsigned)b3), "s"((unsigned)(b3 >> 32)),
          "i"(rw), "i"(rw + 4), "i"(rw + 1), "i"(rw + 5), "i"(rw + 2), "i"(rw + 6), "i"(rw + 3), "i"(rw + 7));
    mask_words<Q + 4>(y, mw);
  }
}

// The classifier head on the block's h, straight from the forward's accumulators (no HBM round trip): h = relu(scale
// acc + b1) (rows past M zero) handed to head_block.h: fp16-plane MFMA logits, softmax / NLL / dl, dW2 and the block's
// slab row, bit-identical dl to head_xent.hip's standalone block head on the same rows. The ReLU bits leave by one
// 8-byte store per lane: each register's ballot holds one word of two rows of the wave (lanes 0..31: row rw, 32..63:
// row rw + 4), deposited straight into those rows' lanes by v_writelane (round 4 selected them with compares, and the
// 64 ballot SGPR pairs spilled)
template <int C>
__device__ __forceinline__ hblk::Args fused_head_args(const FwdParams& p, int hb) {  // hb: 256-row head block index
  const U8HeadArgs& hd = p.head;
  hblk::Args a;
  a.w2 = hd.w2;
  a.b2 = hd.b2;
  a.target = hd.target;
  a.loss_scale = hd.loss_scale;
  a.train = true;
  a.dl = hd.dl;
  a.part = hd.part + (size_t)hb * (C * 128 + C + 2);
  a.bound = hd.bound + hb;
  return a;
}

template <int C>
__device__ __forceinline__ void fused_head_prefetch(const FwdParams& p, int m0, int wave, int lane, int wn,
                                                    hblk::Operands& ops, float (&bv1)[2]) {
  hblk::load_operands<C>(fused_head_args<C>(p, 0), m0, p.M, wave, lane, ops);
#pragma unroll
  for (int j = 0; j < 2; ++j) bv1[j] = p.bias[wn * 64 + 32 * j + (lane & 31)];
}

template <int C, int NWR>
__device__ __forceinline__ void fused_head_epilogue(const FwdParams& p, const f32x16 (&acc)[2][2], unsigned char* smem,
                                                    int m0, int wave, int lane, int wm, int wn,
                                                    const hblk::Operands& ops, const float (&bv1)[2], long long* stamp,
                                                    int hb) {
  static_assert(NWR == 4, "head_block.h: 8 waves of 64 x 64, 256 rows");
  const U8HeadArgs& hd = p.head;
  const int h2 = lane >> 5;
  if (stamp && lane == 0) stamp[16] = (long long)__builtin_amdgcn_s_memtime();
  const hblk::Args a = fused_head_args<C>(p, hb);
  auto prep = [&](hblk::hb_f32x16 (&y)[2][2]) {
    // the plain epilogue's fmaxf(fma(acc, scale, b), 0), the fmas on pairs (v_pk_fma_f32: the same roundings)
    const hblk::hb_f32x2 sc2 = {p.scale, p.scale};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const hblk::hb_f32x2 b2 = {bv1[j], bv1[j]};
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const hblk::hb_f32x2 v = __builtin_elementwise_fma(hblk::hb_f32x2{acc[i][j][r], acc[i][j][r + 1]}, sc2, b2);
          y[i][j][r] = fmaxf(v[0], 0.f);
          y[i][j][r + 1] = fmaxf(v[1], 0.f);
        }
      }
    if (m0 + hblk::ROWS > p.M) {  // (block-uniform) the last block's rows past M
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h2 >= p.M) y[i][j][r] = 0.f;
    }
    int mw[2] = {0, 0};  // lane L: mask words 2 wn + j of the wave's row L
    mask_words<0>(y, mw);
    const int row = m0 + wm * 64 + lane;
    if (row < p.M) *reinterpret_cast<uint2*>(hd.mask + (size_t)row * 4 + 2 * wn) = uint2{(unsigned)mw[0], (unsigned)mw[1]};
  };
  // after the first barrier (past the epilogue's last compiler-counted load wait, so nothing below waits for these):
  // the pixels of the workgroup that runs next on this XCD - block blockIdx + pf_stride, its first K-step (the one its
  // DMA prologue waits for), 256 rows x 64 B - into this XCD's L2 by LDS-DMA into a scratch KiB. Round-2 workgroups
  // started with ~4.8K cycles of DMA prologue from HBM (stamps: ~2.6-3.2K with the prefetch).
  const bool pf = p.pf_stride > 0 && (int)blockIdx.x + p.pf_stride < (int)gridDim.x;  // (block-uniform)
  auto post_b1 = [&]() {
    if (pf) {
      const int m1 = ((int)blockIdx.x + p.pf_stride) * hblk::ROWS;
      const dma_i32x4 rx = dma_rsrc4(p.X, (unsigned)((size_t)p.M * p.ldx));
#pragma unroll
      for (int u = 0; u < 2; ++u) {  // 16 pieces of 16 rows x 64 B, 2 per wave
        const int row = 16 * (wave + 8 * u) + (lane >> 2);
        const unsigned voff = (unsigned)((size_t)min(m1 + row, p.M - 1) * p.ldx + 16 * (lane & 3));
        bdma16_asm(rx, voff, 0u, smem + hblk::LDS_BYTES);  // (past the ring and the head's LDS)
      }
    }
  };
  hblk::block_head<C>(prep, smem, a, ops, m0, p.M, wave, lane, [](int, int, bool, const float (&)[4]) {}, stamp,
                      post_b1);
  if (pf) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the scratch DMA lands before the LDS is released)
}

// fp32 [N][K] -> zero-padded fp16 planes [NPL][N][Kp] of W * 2^8 (u8_planes.h)
__global__ void __launch_bounds__(256) split_planes_pad_kernel(const float* __restrict__ w, u16* __restrict__ out,
                                                               int N, int K, int Kp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // element of the padded [N][Kp]
  const int64_t n = (int64_t)N * Kp;
  if (i >= n) return;
  const int r = (int)(i / Kp), k = (int)(i % Kp);
  const float x = k < K ? w[(size_t)r * K + k] : 0.f;
  u16 hi, lo;
  u8_fwd_planes_of(x, hi, lo);
  out[i] = hi;
  out[n + i] = lo;
}


// ==== weight gradient of the uint8-fed first layer =============================================
// gW[n][k] += scale * sum_m dz[m][n] X[m][k]   and   gb[n] += sum_m dz[m][n]
// (dz [M][N] fp32 = the boundary gradient, already ReLU-masked; X [M][784] uint8 pixels).
//
// Numerics: a pixel byte is exact in fp16; dz is split into two fp16 planes of dz * 2^s, hi =
// fp16(dz 2^s) and lo = fp16(dz 2^s - hi) (each dz to within one fp32 ulp, as the forward's weight
// planes in u8_planes.h), so every product is 2 fp16 MFMA products accumulated in fp32 and the 2^-s
// is folded into the partial tile's scale. The power of two 2^s = 2^(14 - E) is chosen from a bound
// |dz| < 2^E: the max of the head's per-block bounds when the gradient comes from the fused head
// (head_xent.hip writes them next to dx: 2 max_row sum_c |dl_c| * max |W2|), a torch amax otherwise, and for the factored gradient (FD)
// the workgroup's own bound max_row sum_c |dl| * max |W2| (hidden columns of the workgroup). dz
// elements above 2^(E-15) keep the one-ulp split; smaller ones an absolute error below 2^(E-39).
//
// Why this shape: the reduction runs over the batch (K = 131072 rows), so the work is split over
// row ranges and every workgroup leaves one partial tile. dz must be split into 3 bf16 planes on
// the VALU; in a 128 x 128 output tile (gemm_f32x3's kernel) every dz element is split 7 times
// (once per 128-column tile), which made that kernel VALU-issue-bound (~90 VALU per 12 MFMAs).
// Here a workgroup owns 64 hidden units x ALL 784 columns: each dz element is split exactly once
// and each pixel byte widened twice (once per hidden half), at the price of larger partial tiles
// (written with plain stores, reduced in fixed order by slab_reduce).
//
// Geometry: v_mfma_f32_32x32x16_bf16 (an MFMA holds the SIMD's vector issue 8 of its 32 cycles;
// the 16x16x32 form holds 8 of 16, which left a first version of this kernel issue-bound), the 784
// columns padded to 25 tiles of 32. 8 waves, all computing: wave 0 owns columns 0..127, waves
// 1..7 three 32-column tiles each, every wave all 64 hidden (2 x {4,3} tiles, <= 8 f32x16
// accumulators; measured and rejected: the 25th tile split by hidden half over waves 0 and 1 so no
// SIMD carries more than 13 of the 50 tile pairs, with or without double-buffered staging
// registers - 91-93 vs 85 us, the extra fragment reads and register pressure (spills) outweigh the
// balance). All 8 waves stage the next 32-row K-step (dz float4 -> 3 bf16 planes, 16 pixel
// bytes -> 16 bf16) into the other LDS buffer while the current one is consumed. Both operands
// are k-major in memory (the reduction index is the row), so fragments come from [row][col] LDS
// images through ds_read_b64_tr_b16 (a 16-lane group reads 4 rows x 16 columns, transposed).
constexpr int GT = 512;             // threads
constexpr int GHN = 64;             // hidden units per workgroup
constexpr int GBK = 32;             // rows per K-step (two 32x32x16 MFMA k-substeps)
constexpr int GKC = 784;            // pixel columns (MNIST)
constexpr int GKP = 800;            // padded to 25 column tiles of 32
// LDS row pitches: a transposed read of a 32x32x16 operand has a 32-lane half read 4 consecutive
// rows x 64 B (16 banks each), conflict-free when the row pitch is 16 dwords mod 64 (rows land on
// bank offsets 0, 16, 32, 48 in some order): 1600 B (400 dwords) and 192 B (48 dwords).
// Measured before: pitches 1616 / 144 B -> SQ_LDS_BANK_CONFLICT 47% of LDS-active cycles.
constexpr int GXP = GKP;            // LDS pitch (bf16) of the pixel image rows
constexpr int GDP = GHN + 32;       // LDS pitch (bf16) of the dz plane rows
static_assert((GXP * 2 / 4) % 64 == 16 && (GDP * 2 / 4) % 64 == 48, "conflict-free transposed-read pitches");
constexpr int GX_U16 = GBK * GXP;   // pixel image per buffer (u16)
constexpr int GD_U16 = GBK * GDP;   // one dz plane per buffer (u16)
constexpr int GNPL = 2;              // fp16 planes of dz
constexpr int GBUF_U16 = GX_U16 + GNPL * GD_U16;
constexpr int GXCH = GBK * (GKP / 16);  // 16-byte pixel chunks per K-step incl. the zero pad (1600)
static_assert(2 * GBUF_U16 * 2 <= 160 * 1024, "LDS");

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x4 tr16(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// 32x32x16 operand of the 32 columns c0.. of a [k-row][PITCH] image at k-substep s: lane l
// (r = l & 31, h = l >> 5) gets column c0 + r, k-rows 16 s + 8 h + j (j = 0..7). Two tr16 reads:
// 16-lane group g covers k-rows 16 s + 8 (g >> 1) + q (+4), lane 4q + p addressing columns
// c0 + 16 (g & 1) + 4p .. +3, lane i receiving column c0 + 16 (g & 1) + i.
template <int PITCH>
__device__ __forceinline__ f16x8 frag_tr(const u16* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const u16* p = img + (16 * s + 8 * (g >> 1) + (i >> 2)) * PITCH + c0 + 16 * (g & 1) + 4 * (i & 3);
  const s16x4 lo = tr16(p), hi = tr16(p + 4 * PITCH);
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return __builtin_bit_cast(f16x8, f);
}

// dz plane images: the 8-byte granule g (4 hidden units) of k-row r is stored at g ^ dz_swz(r). The
// factored staging writes one 16-row x 4-column block per 16 lanes (the fd_dz MFMA layout): on the
// 48-dword pitch the even rows of the block share one 16-dword bank half and the odd rows the other, so
// the 8 even (odd) rows need 8 distinct granule slots: (r >> 1) & 7. (Round 3's ((r >> 2) & 3) << 1 gave
// 4, i.e. 2-way write conflicts; no swizzle: 4-way, 7.1e6 conflict cycles.) A transposed read stays
// conflict-free under any XOR below 8: it permutes each row's 8-granule block in place.
__device__ __forceinline__ int dz_swz(int r) { return (r >> 1) & 7; }

// pixel image rows (GXP = 800 fp16): the low 8 fp16 of every 16-column chunk cc at 8 cc, the high 8 at
// 400 + 8 cc. The staging's 16-B stores (lane = chunk, two per chunk) then hit 32 consecutive dwords per
// 8-lane group (the chunk-contiguous row of round 3 put lanes cc and cc + 4 on the same banks: 2-way on
// 400 of 512 store groups); the transposed reads of 4 columns stay inside one half-chunk, conflict-free.
__device__ __forceinline__ int px_col(int col) { return ((col >> 3) & 1) * 400 + (col >> 4) * 8 + (col & 7); }

// frag_tr for the pixel image (px_col layout)
__device__ __forceinline__ f16x8 frag_px(const u16* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const u16* p = img + (16 * s + 8 * (g >> 1) + (i >> 2)) * GXP + px_col(c0 + 16 * (g & 1) + 4 * (i & 3));
  const s16x4 lo = tr16(p), hi = tr16(p + 4 * GXP);
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return __builtin_bit_cast(f16x8, f);
}

template <int PITCH>
__device__ __forceinline__ f16x8 frag_tr_dz(const u16* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int r = 16 * s + 8 * (g >> 1) + (i >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i & 3);
  const s16x4 lo = tr16(img + r * PITCH + (((col >> 2) ^ dz_swz(r)) << 2));
  const s16x4 hi = tr16(img + (r + 4) * PITCH + (((col >> 2) ^ dz_swz(r + 4)) << 2));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return __builtin_bit_cast(f16x8, f);
}

// exponent E with |v| < 2^E for a finite v >= 0 (v = m 2^E, m in [0.5, 1)), clamped so 2^(14 - E)
// and 2^(E - 14) stay normal floats
__device__ __forceinline__ int bound_exp(float v) {
  const unsigned b = __float_as_uint(v);
  const int e = (int)((b >> 23) & 0xffu) - 126;
  return (b & 0x7fffffffu) == 0u ? -100 : min(max(e, -100), 120);
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }

struct WgradParams {
  const float* dz;           // [M][N]
  const unsigned char* X;    // [M][ldx]
  float* slab;               // [splits][N * 784 + N]: gW partial (scaled) then gb partial
  int M, N, ldx;
  int rows_per_split;        // multiple of GBK
  float scale;
  const float* amax;         // optional [namax]: |dz| <= max(amax) (the head's per-block maxima)
  int namax;
  // FD (factored boundary gradient): dz = (dl @ W2) * (h > 0) rebuilt in the staging
  const float* dl;           // [M][C]
  const float* w2;           // [C][N]
  const float* h;            // [M][N] (FD == 1)
  const unsigned* mask;      // [M][N / 32] ReLU bits (FD == 2)
  int C;                     // <= 16
  int groups, splits;        // hidden groups launched x row splits (1-D grid, XCD-aware order)
  int g0;                    // first hidden group launched (hidden units GHN g0 ..)
  int xcd;                   // 0: plain order (split-major), A/B only (SDML_U8_WGRAD_XCD=0)
  int prio;                  // 1: s_setprio 1 on waves 4..7 (knob U8_WGRAD_PRIO)
  long long* stamps;         // experiments builds only: [blocks][8 waves][16] phase stamps (u8_set_wgrad_stamps)
  unsigned* pair;            // ring kernel, pairwise combine (knob U8_WGRAD_PAIR): [groups][splits / 2][2] ticket and
                             // flag words, zero between launches (the second arriver of a pair resets them); null: off
};

// experiments builds: s_memtime stamps of the weight gradient's phases (tools/u8_wgrad_stamps.py); slot 0 / 15 hold
// s_memrealtime at start / end
#ifdef SDML_KERNEL_EXPERIMENTS
#define U8W_STAMP(k, fn)                                                                               \
  do {                                                                                                 \
    if (p.stamps && lane == 0) p.stamps[((size_t)blockIdx.x * 8 + wave) * 16 + (k)] = (long long)fn(); \
  } while (0)
#else
#define U8W_STAMP(k, fn) \
  do {                   \
  } while (0)
#endif

// dx tile of head_xent.hip's MFMA head (dx_t / head_mfma_dx_from_dl_kernel), reproduced operation
// for operation: lane (r, g) of a 16-row tile gets dz[row r][16 t + 4 g + v] =
// sum over the 4 MFMAs kk of W2[4 g + kk][16 t + r] * dl[row r][4 g + kk], then the ReLU mask of h.
__device__ __forceinline__ f32x4 fd_dz(const float (&w4)[4], const float (&d4)[4], const f32x4& hv) {
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) o = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[kk], d4[kk], o, 0, 0, 0);
#pragma unroll
  for (int v = 0; v < 4; ++v) o[v] = hv[v] > 0.f ? o[v] : 0.f;
  return o;
}
// the same with the ReLU mask as 4 bits (bit v <=> h[.][column v] > 0): bit-identical dz
__device__ __forceinline__ f32x4 fd_dz_bits(const float (&w4)[4], const float (&d4)[4], unsigned bits) {
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) o = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[kk], d4[kk], o, 0, 0, 0);
#pragma unroll
  for (int v = 0; v < 4; ++v) o[v] = (bits >> v) & 1u ? o[v] : 0.f;
  return o;
}

// dz bound -> plane scale dz_up = 2^(14 - E) and the partial tile's out_scale = scale 2^(E - 14): block max through
// LDS (red: >= 16 free floats; every thread of the GT-thread block calls this)
template <int FD>
__device__ __forceinline__ void wgrad_scales(const WgradParams& p, int n0, int r0, int t, float* red, float& dz_up,
                                             float& out_scale) {
  const int lane = t & 63, wave = t >> 6;
  float bnd = 0.f;
  if (p.amax) {
    for (int i = t; i < p.namax; i += GT) bnd = fmaxf(bnd, p.amax[i]);
  } else if constexpr (FD != 0) {  // max_row sum_c |dl| over this workgroup's rows, times max |W2| here
    const int nrows = min(p.rows_per_split, p.M - r0);
    for (int i = t; i < nrows; i += GT) {
      const float* d = p.dl + (size_t)(r0 + i) * p.C;
      float sa = 0.f;
      for (int c = 0; c < p.C; ++c) sa += fabsf(d[c]);
      bnd = fmaxf(bnd, sa);
    }
  }
  float wmx = 0.f;
  if constexpr (FD != 0) {
    if (!p.amax)
      for (int i = t; i < p.C * GHN; i += GT) wmx = fmaxf(wmx, fabsf(p.w2[(size_t)(i / GHN) * p.N + n0 + i % GHN]));
  }
  for (int off = 32; off > 0; off >>= 1) {
    bnd = fmaxf(bnd, __shfl_xor(bnd, off));
    wmx = fmaxf(wmx, __shfl_xor(wmx, off));
  }
  if (lane == 0) {
    red[wave] = bnd;
    red[8 + wave] = wmx;
  }
  __syncthreads();
  bnd = red[0];
  wmx = red[8];
#pragma unroll
  for (int w = 1; w < GT / 64; ++w) {
    bnd = fmaxf(bnd, red[w]);
    wmx = fmaxf(wmx, red[8 + w]);
  }
  __syncthreads();
  // FD without amax: |dz_n| <= sum_c |dl_c| |W2_cn|; the product is rounded, so bound it by 2x
  const int E = bound_exp((FD != 0 && !p.amax) ? 2.f * bnd * wmx : bnd);
  dz_up = pow2f(14 - E);
  out_scale = p.scale * pow2f(E - 14);
}

// partial tile -> slab (plain stores); C map: column = lane & 31, row = (r&3) + 8(r>>2) + 4h
// add (pairwise combine, the second arriver): the partner's partial is read from slab row `add_row` and each element
// stored is (own partial) + (partner's) - one fp32 add, commutative, so the pair sum has the same bits whichever of the
// two arrived first
// pairwise-combine memory forms (the write-through hand-off of cdna_hip_programming.md Guideline 16, R1): the first
// arriver stores its partial sc1 (agent-scope relaxed atomic stores), the second loads it sc1 (agent-scope relaxed
// atomic loads, past this CU's L1), so neither needs an L2-wide release / acquire fence
__device__ __forceinline__ void st_sc1(float* a, float v) { __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_sc1(const float* a) {
  return __hip_atomic_load(const_cast<float*>(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// role: -1 no pairing (plain stores), 0 first arriver (sc1 stores, row = own split), 1 second arriver (the partner's
// partial read from add_row, (own + partner) stored plain)
template <int NCT>
__device__ __forceinline__ void wgrad_store_tile(const WgradParams& p, const f32x16 (&acc)[2][NCT], int split, int n0,
                                                 int ct0, int lane, float out_scale, int role = -1, int add_row = 0) {
#pragma clang fp contract(off)  // the pair sum is (rounded product) + partner: never one fma, which would be role-dependent
  float* out = p.slab + (size_t)split * ((size_t)p.N * GKC + p.N);
  const float* pin = p.slab + (size_t)add_row * ((size_t)p.N * GKC + p.N);
#pragma unroll
  for (int j = 0; j < NCT; ++j) {
    const int col = 32 * (ct0 + j) + (lane & 31);
    if (col >= GKC) continue;
    float other[2][16];
    if (role == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          other[i][r] = ld_sc1(pin + (size_t)(n0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * GKC + col);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float v = acc[i][j][r] * out_scale;
        if (role == 0) st_sc1(out + (size_t)n * GKC + col, v);
        else out[(size_t)n * GKC + col] = role == 1 ? v + other[i][r] : v;
      }
  }
}

// Pairwise combine of the ring weight gradient's row splits (knob U8_WGRAD_PAIR): split s < S/2 and split s + S/2 of
// one hidden group (the same XCD under the XCD-aware order) draw a ticket when their K loop ends. The first arriver
// stores its partial into its own slab row and publishes it (every wave's stores drained, barrier, agent-scope release,
// flag); the second waits for the flag (the first is resident and only storing: a bounded wait), acquires, and stores
// (own + partner) into row s, then resets both words for the next launch. The reduction that follows reads S/2 rows
// instead of S. Returns the role: 0 first arriver, 1 second; `red` holds a free LDS int for the broadcast. The
// payload is handed over write-through (st_sc1 / ld_sc1): a release / acquire pair of agent-scope fences instead
// (an L2 write-back on every first arriver) made the kernel ~20 us slower.
__device__ __forceinline__ int wgrad_pair_role(const WgradParams& p, int group, int split, int t, int* red) {
  unsigned* w = p.pair + 2 * ((size_t)group * (p.splits / 2) + (split % (p.splits / 2)));
  __syncthreads();  // every wave's last fragment reads are done before red is written
  if (t == 0) red[0] = (int)__hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int role = red[0];
  __syncthreads();
  if (role == 1) {
    if (t == 0) {
      for (int it = 0; it < (1 << 26) && __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
           ++it)
        __builtin_amdgcn_s_sleep(1);
      __hip_atomic_store(w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(w + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every load of the partner's bytes is sc1 (ld_sc1): no acquire, only keep the compiler from hoisting them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
  }
  return role;
}

// the first arriver's publish, after all of its slab stores
__device__ __forceinline__ void wgrad_pair_publish(const WgradParams& p, int group, int split, int t) {
  unsigned* w = p.pair + 2 * ((size_t)group * (p.splits / 2) + (split % (p.splits / 2)));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (t == 0) __hip_atomic_store(w + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bias-gradient partial: the 32 threads of each hidden float4 meet in LDS (red: 4 GT free floats, after a barrier)
template <int FD>
__device__ __forceinline__ void wgrad_store_bias(const WgradParams& p, const f32x4& bsum, int split, int n0, int t,
                                                 float* red, int role = -1, int add_row = 0) {
  float* out = p.slab + (size_t)split * ((size_t)p.N * GKC + p.N);
  *reinterpret_cast<f32x4*>(red + 4 * t) = bsum;
  __syncthreads();
  if (t < GHN) {  // rows rr = 0 .. 31 in order, whichever thread staged them
    float sacc = 0.f;
    for (int rr = 0; rr < GBK; ++rr) {
      const int owner = FD != 0 ? 64 * ((rr >> 4) * 4 + (t >> 4)) + 16 * ((t >> 2) & 3) + (rr & 15) : rr * 16 + (t >> 2);
      sacc += red[4 * owner + (t & 3)];
    }
    if (role == 1) sacc += ld_sc1(p.slab + (size_t)add_row * ((size_t)p.N * GKC + p.N) + (size_t)p.N * GKC + n0 + t);
    if (role == 0) st_sc1(out + (size_t)p.N * GKC + n0 + t, sacc);
    else out[(size_t)p.N * GKC + n0 + t] = sacc;
  }
}

// FD = 0: dz read as [M][N]. FD > 0: the factored boundary gradient (rotate placement, one-rank step)
// is expanded here instead of by a separate kernel that writes dz to memory and reads it back -
// with head_xent.hip's exact operations, so gW / gb are bit-identical to the unfused pair; the ReLU
// mask comes from h (FD = 1, 16 B per thread and K-step) or from its bits (FD = 2, 4 B).
// ILV: the K-step body carries an explicit instruction interleave (sched_group_barrier): the fragment reads of a
// substep, then its MFMAs each followed by 3 of the staging VALU instructions, so the next K-step's staging runs in
// the MFMA shadows of this one's (without it the compiler emitted compute, then staging, then the barrier: ~3.9K
// cycles per K-step against ~1.8K of MFMA, stamps in profiles/r4_u8_wgrad_stamps.json)
template <int FD, bool ILV = false>
__global__ void __launch_bounds__(GT) u8_wgrad_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) u16 smem[2 * GBUF_U16];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  if (p.prio && wave >= GT / 128) __builtin_amdgcn_s_setprio(1);  // (knob U8_WGRAD_PRIO)
  // XCD-aware order: the hidden groups of one row split read the same pixel rows, so they are given
  // block ids 8 apart (same XCD under the round-robin dispatch, one L2) and run side by side:
  // L = 8 G (s / 8) + 8 g + s % 8. Ids past the last split (splits rounded up to 8) exit here.
  const int L = blockIdx.x, G8 = 8 * p.groups;
  const int split = p.xcd ? (L / G8) * 8 + L % 8 : L / p.groups;
  if (split >= p.splits) return;
  U8W_STAMP(0, __builtin_amdgcn_s_memrealtime);
  U8W_STAMP(1, __builtin_amdgcn_s_memtime);
  const int n0 = (p.g0 + (p.xcd ? (L % G8) / 8 : L % p.groups)) * GHN;
  const int r0 = split * p.rows_per_split;
  const int nk = min(p.rows_per_split, p.M - r0) / GBK;  // host: M % GBK == 0

  // ---- staging: thread t owns dz float4 (row t >> 4, hidden 4 (t & 15)) and pixel chunks
  // t + 512 u (chunk c: row c / 50, columns 16 (c % 50); c % 50 == 49 is the zero pad). The 4th
  // round covers chunks 1536..1599: threads >= 64 repeat chunk 1599 (same bytes to the same
  // place), so staging has no lane-dependent branches ----
  // FD: wave w builds the 16 x 16 dz tile (rows 16 (w >> 2) .., hidden 16 (w & 3) ..) of each
  // K-step with 4 fp32 MFMAs, lane (r, g) holding row r, hidden 4 g .. 4 g + 3 of it
  const int fr = 16 * (wave >> 2) + (lane & 15), fc = 16 * (wave & 3) + 4 * (lane >> 4);
  const int drow = FD ? fr : (t >> 4), dcol = FD ? fc : 4 * (t & 15);  // this thread's dz float4
  const float* dzp = (FD == 1 ? p.h : p.dz) + (size_t)(r0 + drow) * p.N + n0 + dcol;
  const size_t dz_step = (size_t)GBK * p.N;
  const unsigned* mkp = p.mask + (size_t)(r0 + drow) * (p.N / 32) + (n0 + dcol) / 32;  // FD == 2
  const int mshift = (n0 + dcol) & 31;
  unsigned mbits = 0u;
  float dz_up = 1.f, out_scale = p.scale;  // 2^(14 - E) and scale * 2^(E - 14), set below
  float w4[4] = {0.f, 0.f, 0.f, 0.f};  // FD: W2[4 g + kk][n0 + 16 (w & 3) + r]
  const float* dlp = nullptr;
  if constexpr (FD != 0) {
    const int g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      if (4 * g + kk < p.C) w4[kk] = p.w2[(size_t)(4 * g + kk) * p.N + n0 + 16 * (wave & 3) + (lane & 15)];
    dlp = p.dl + (size_t)(r0 + fr) * p.C;
  }
  float d4[4] = {0.f, 0.f, 0.f, 0.f};

  wgrad_scales<FD>(p, n0, r0, t, reinterpret_cast<float*>(smem), dz_up, out_scale);
  U8W_STAMP(2, __builtin_amdgcn_s_memtime);
  constexpr int XU = (GXCH + GT - 1) / GT;  // 4 rounds
  const unsigned char* xp[XU];
  int xoff[XU];
  bool xload[XU];
#pragma unroll
  for (int u = 0; u < XU; ++u) {
    const int c = min(t + GT * u, GXCH - 1);
    const int row = c / 50, cc = c % 50;
    xload[u] = cc < 49;
    xp[u] = p.X + (size_t)(r0 + row) * p.ldx + 16 * min(cc, 48);
    xoff[u] = row * GXP + 8 * cc;  // (px_col: high half at + 400)
  }
  const size_t x_step = (size_t)GBK * p.ldx;
  f32x4 dv;
  u32x4 xv[XU];
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
  auto gload = [&](int kt) {
    if constexpr (FD == 2) mbits = mkp[(size_t)kt * GBK * (p.N / 32)];  // the ReLU bits
    else dv = *reinterpret_cast<const f32x4*>(dzp + kt * dz_step);      // dz, or FD == 1: h (the ReLU mask source)
    if constexpr (FD != 0) {
      const int g = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        d4[kk] = 4 * g + kk < p.C ? dlp[(size_t)kt * GBK * p.C + 4 * g + kk] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) xv[u] = *reinterpret_cast<const u32x4*>(xp[u] + kt * x_step);
  };
  auto stage = [&](int buf) {
    u16* B = smem + buf * GBUF_U16;
    if constexpr (FD == 1) dv = fd_dz(w4, d4, dv);
    if constexpr (FD == 2) dv = fd_dz_bits(w4, d4, (mbits >> mshift) & 15u);
    bsum += dv;
    u16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = dv[e] * dz_up;  // exact (power of two), |x| < 2^14
      const _Float16 h = static_cast<_Float16>(x);
      hi[e] = __builtin_bit_cast(u16, h);
      lo[e] = __builtin_bit_cast(u16, static_cast<_Float16>(x - static_cast<float>(h)));
    }
    const int doff = GX_U16 + drow * GDP + (((dcol >> 2) ^ dz_swz(drow)) << 2);
    *reinterpret_cast<u16x4*>(B + doff) = hi;
    *reinterpret_cast<u16x4*>(B + doff + GD_U16) = lo;
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const u32x4 v = xload[u] ? xv[u] : u32x4{0u, 0u, 0u, 0u};
      *reinterpret_cast<f16x8*>(B + xoff[u]) = widen8h(v[0], v[1]);
      *reinterpret_cast<f16x8*>(B + xoff[u] + 400) = widen8h(v[2], v[3]);
    }
  };

  // ---- compute: wave 0 columns 0..127, wave w >= 1 columns 128 + 96 (w - 1) .. +95; all 64 hidden.
  // The K loop is instantiated per column count, and its body has no branches: the compiler can
  // then interleave the staging VALU work into the MFMA shadows of the same wave.
  auto run = [&](auto nct_c) {
    constexpr int NCT = decltype(nct_c)::value;
    const int ct0 = NCT == 4 ? 0 : 4 + 3 * (wave - 1);  // first 32-column tile
    f32x16 acc[2][NCT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[i][j] = f32x16{};
    auto compute = [&](int buf) {
      const u16* B = smem + buf * GBUF_U16;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 a[2][GNPL];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int pl = 0; pl < GNPL; ++pl) a[i][pl] = frag_tr_dz<GDP>(B + GX_U16 + pl * GD_U16, 32 * i, s, lane);
#pragma unroll
        for (int j = 0; j < NCT; ++j) {
          const f16x8 b = frag_px(B, 32 * (ct0 + j), s, lane);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            acc[i][j] = mfma(a[i][1], b, acc[i][j]);  // lo
            acc[i][j] = mfma(a[i][0], b, acc[i][j]);  // hi
          }
        }
      }
    };
    // buffer kt & 1 is consumed in step kt while step kt+1 is staged into the other one (its last
    // readers passed the previous barrier) and step kt+2's global loads fly
    gload(0);
    stage(0);
    if (nk > 1) gload(1);
    __syncthreads();
    U8W_STAMP(3, __builtin_amdgcn_s_memtime);
    int kt = 0;
    auto interleave = [&]() {
      if constexpr (ILV) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          __builtin_amdgcn_sched_group_barrier(0x100, 8 + 2 * NCT, 0);  // this substep's fragment reads
#pragma unroll
          for (int m = 0; m < 4 * NCT; ++m) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // three staging VALU
          }
        }
      }
    };
    for (; kt + 2 < nk; ++kt) {
      compute(kt & 1);
#ifdef SDML_KERNEL_EXPERIMENTS
      if (kt == 0 || kt == 8 || kt == 16) U8W_STAMP(4 + kt / 8 * 2, __builtin_amdgcn_s_memtime);  // after compute
#endif
      stage((kt + 1) & 1);
      gload(kt + 2);
      interleave();
      __syncthreads();
#ifdef SDML_KERNEL_EXPERIMENTS
      if (kt == 0 || kt == 8 || kt == 16) U8W_STAMP(5 + kt / 8 * 2, __builtin_amdgcn_s_memtime);  // after barrier
#endif
    }
    if (kt + 1 < nk) {
      compute(kt & 1);
      stage((kt + 1) & 1);
      __syncthreads();
      ++kt;
    }
    compute(kt & 1);
    U8W_STAMP(10, __builtin_amdgcn_s_memtime);

    wgrad_store_tile<NCT>(p, acc, split, n0, ct0, lane, out_scale);
    U8W_STAMP(11, __builtin_amdgcn_s_memtime);
  };
  if (nk > 0) {
    if (wave == 0) run(std::integral_constant<int, 4>{});
    else run(std::integral_constant<int, 3>{});
  }
  __syncthreads();
  wgrad_store_bias<FD>(p, bsum, split, n0, t, reinterpret_cast<float*>(smem));
  U8W_STAMP(12, __builtin_amdgcn_s_memtime);
  U8W_STAMP(15, __builtin_amdgcn_s_memrealtime);
}

// ---- the same weight gradient with its operands on LDS-DMA rings (FD = 2: dl + ReLU bits) ----------------------
// Why: u8_wgrad_kernel stages a K-step's pixels through registers (global -> VGPR -> fp16 -> LDS) and reads each
// K-step's fragments only after that K-step's barrier; at ~3.9K cycles per K-step against ~2K of MFMA on its busiest
// SIMD its waves sat in s_waitcnt (SQ_WAIT_INST_ANY 35 % of wave cycles, profiles/r4_pmc_fused_fwd_head_and_wgrad.txt).
// Here:
//  * the raw pixel bytes go to LDS by buffer-DMA into a 4-stage ring, issued three K-steps ahead; the K-step's dl rows
//    and ReLU bits into a 4-stage side ring, four K-steps ahead. The DMA is inline assembly (lds_dma.h bdma16_asm:
//    with the builtin form the compiler drained the ring, s_waitcnt vmcnt(0), before every transposed fragment read);
//  * pixel fragments come straight from the byte image through ds_read_b64_tr_b8 (a 16-lane group reads 8 rows x 16
//    columns: lane = column, byte q = row q) and are widened in registers by the wave that owns the column tile (each
//    pixel once per block, as before); the waves only write the dz planes (8 KB per K-step instead of 59 KB);
//  * software pipeline: the dz planes of K-step kt + 2 are built during kt (three dz buffers), so when the barrier
//    ending kt - 1 has passed, kt + 1's planes and pixels are both published; k-substep 0's fragments of kt + 1 are
//    read into registers during kt's last MFMAs and the MFMAs of kt + 1 start right after its barrier.
// Numerics, tile ownership, k order and the partial-tile / bias outputs are those of u8_wgrad_kernel<2>: the results
// are bit-identical. Measured stamps: tools/u8_wgrad_stamps.py.
constexpr int RX_PITCH = 800;                     // bytes per pixel row in LDS (50 16-B chunks, the last one a pad)
constexpr int RX_PIECES = GBK * RX_PITCH / 1024;  // 25 1-KiB DMA pieces of pixels per K-step
constexpr int RX_STAGE = RX_PIECES * 1024;
constexpr int RNS = 4;                            // stages of both rings
constexpr int RS_STAGE = 3072;                    // side stage: dl rows (2 pieces, 8 C <= 128 chunks), ReLU bits (1)
constexpr int RS_OFF = RNS * RX_STAGE;
constexpr int RDZ_OFF = RS_OFF + RNS * RS_STAGE;  // three dz-plane buffers [GNPL][GBK][GDP] fp16
constexpr int RDZ_BUF = GNPL * GD_U16;            // u16 per dz buffer
constexpr int RSCR_OFF = RDZ_OFF + 3 * RDZ_BUF * 2;  // 1 KiB the null DMA pieces write
constexpr int RSMEM = RSCR_OFF + 1024;
static_assert(GBK * RX_PITCH % 1024 == 0 && RSMEM <= 160 * 1024, "ring LDS");
static_assert((RX_PITCH / 16) % 16 == 2, "tr_b8 reads: rows q = 0..7 of a chunk pair on 16 distinct 16-B bank slots");

typedef int i32x2 __attribute__((ext_vector_type(2)));

// 32x32x16 f16 B operand of the 32 columns c0.. of the byte image at k-substep s, same lane map as frag_px:
// lane l (r = l & 31, h = l >> 5) gets column c0 + r, k-rows 16 s + 8 h + j. Lane 2q + p of 16-lane group g
// addresses row 16 s + 8 (g >> 1) + q, columns c0 + 16 (g & 1) + 8 p .. +7.
template <bool RAW = false>
__device__ __forceinline__ f16x8 frag_x8(const unsigned char* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const unsigned char* a = img + (16 * s + 8 * (g >> 1) + (i >> 1)) * RX_PITCH + c0 + 16 * (g & 1) + 8 * (i & 1);
  const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(a));
  if constexpr (RAW) {  // (timing experiment)
    u32x4 r = {(unsigned)v[0], (unsigned)v[1], (unsigned)v[0], (unsigned)v[1]};
    return __builtin_bit_cast(f16x8, r);
  }
  return widen8h((unsigned)v[0], (unsigned)v[1]);
}

// the same 8 bytes, not widened
__device__ __forceinline__ i32x2 frag_x8_raw(const unsigned char* img, int c0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const unsigned char* a = img + (16 * s + 8 * (g >> 1) + (i >> 1)) * RX_PITCH + c0 + 16 * (g & 1) + 8 * (i & 1);
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(a));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MODE (experiments builds, knob U8_VARIANT; wrong results by design): 1 no dz build in the K loop, 2 no byte
// widening (raw bytes as fp16 bits), 3 no barrier in the K loop, 4 no MFMA, 6 the DMA ring alone (no LDS reads,
// no MFMA, no dz build in the K loop). Measured (tools/u8_wgrad_stamps.py, cycles per K-step, headline shape): normal
// 2.85K, 1: 2.29K, 4: 2.24K, 6: 1.04K; fencing the K-step's phases off from the scheduler (sched_barrier) 3.42K.
// BAL (knob U8_WGRAD_BAL): every wave owns 3 of the 24 full 32-column tiles, and the last 16 columns (768..783) run as
// 16x16x32 MFMAs on waves 4..7 (16 hidden each): every SIMD carries 6 tiles + 1/4 half tile per K-step instead of 7 or
// 6 (wave 0 owned 4 tiles). Those 16 columns then sum in a different MFMA order (fp32-equal, not bit-identical).
template <int MODE = 0, bool BAL = false>
__global__ void __launch_bounds__(GT) u8_wgrad_ring_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char rsm[RSMEM];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int L = blockIdx.x, G8 = 8 * p.groups;
  const int split = p.xcd ? (L / G8) * 8 + L % 8 : L / p.groups;
  if (split >= p.splits) return;
  // waves 4..7 (each SIMD's second wave) at priority 1 (knob U8_WGRAD_PRIO): stamped K-steps 2.98K vs 3.21K cycles on
  // one box, but the un-stamped kernel and the headline step the same (0.1569 / 0.1567 vs 0.1574 / 0.1566 ms): off
  if (p.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  U8W_STAMP(0, __builtin_amdgcn_s_memrealtime);
  U8W_STAMP(1, __builtin_amdgcn_s_memtime);
  const int group = p.xcd ? (L % G8) / 8 : L % p.groups;
  const int n0 = (p.g0 + group) * GHN;
  // pairwise combine of splits s and s + S/2 (wgrad_pair_role); role 0 when off
  const bool pairing = p.pair != nullptr;
  int role = -1;
  const int r0 = split * p.rows_per_split;
  const int nk = min(p.rows_per_split, p.M - r0) / GBK;  // host: M % GBK == 0
  float dz_up = 0.f, out_scale = 0.f;
  // The head's per-block bounds (one per thread): their load goes out with W2's and their block max travels with the
  // prologue's barrier (float slots in dz buffer 2, first written in K-step 0), instead of a phase of its own in front
  // of the DMA (wgrad_scales: a global round trip and two barriers, ~2.5K cycles by the stamps)
  const bool fast_bound = p.amax != nullptr && p.namax <= GT;
  if (!fast_bound) wgrad_scales<2>(p, n0, r0, t, reinterpret_cast<float*>(rsm), dz_up, out_scale);
  if (nk <= 0) return;  // (block-uniform; after wgrad_scales' barriers)
  const float av = fast_bound ? p.amax[min(t, p.namax - 1)] : 0.f;
  float* bred = reinterpret_cast<float*>(rsm + RDZ_OFF + 2 * RDZ_BUF * 2);
  U8W_STAMP(2, __builtin_amdgcn_s_memtime);

  // DMA: one resource per operand from this split's first row (rows past M read as zero), a per-lane offset per piece
  // (chunk 64 j + lane), a scalar advance per K-step. Every wave issues 4 pieces per group, so the loop body has no
  // branches: pixel pieces w, w + 8, w + 16, and a 4th - wave 0 pixel piece 24, waves 1 and 2 the dl pieces, wave 3
  // the ReLU-bit piece, waves 4..7 a null resource (num_records 0: no memory access, zeros into a scratch KiB)
  const int C = p.C, NW = p.N / 32;
  const dma_i32x4 rx = dma_rsrc4(p.X + (size_t)r0 * p.ldx, (unsigned)((p.M - r0) * p.ldx));
  const dma_i32x4 rnull = dma_rsrc4(p.X, 0u);
  dma_i32x4 r3 = rnull;
  const unsigned xstep = GBK * p.ldx;
  unsigned step3 = 0u;
  unsigned voff[4];
#pragma unroll
  for (int u = 0; u < 3; ++u) {  // pixel chunk ci: row ci / 50, 16-B column chunk ci % 50 (49 = pad: repeats 48)
    const int ci = 64 * (wave + 8 * u) + lane, row = ci / (RX_PITCH / 16), cc = ci % (RX_PITCH / 16);
    voff[u] = (unsigned)(row * p.ldx + 16 * min(cc, GKC / 16 - 1));
  }
  voff[3] = 0u;
  if (wave == 0) {
    const int ci = 64 * (RX_PIECES - 1) + lane, row = ci / (RX_PITCH / 16), cc = ci % (RX_PITCH / 16);
    voff[3] = (unsigned)(row * p.ldx + 16 * min(cc, GKC / 16 - 1));
    r3 = rx;
    step3 = xstep;
  } else if (wave < 3) {  // dl chunk (clamped: chunks past 8 C repeat the last one into unused bytes)
    voff[3] = 16u * (unsigned)min(64 * (wave - 1) + lane, 8 * C - 1);
    r3 = dma_rsrc4(p.dl + (size_t)r0 * C, (unsigned)((p.M - r0) * C * 4));
    step3 = GBK * C * 4;
  } else if (wave == 3) {
    voff[3] = 16u * (unsigned)min(lane, 8 * NW - 1);  // ReLU-bit chunk
    r3 = dma_rsrc4(p.mask + (size_t)r0 * NW, (unsigned)((p.M - r0) * NW * 4));
    step3 = GBK * NW * 4;
  }
  // the 4th piece's LDS destination: wave 0 the x stage, waves 1..3 the side stage, waves 4..7 the scratch KiB
  auto dst3 = [&](int kx, int ks) -> unsigned char* {
    if (wave == 0) return rsm + (kx & (RNS - 1)) * RX_STAGE + 1024 * (RX_PIECES - 1);
    if (wave < 4) return rsm + RS_OFF + (ks & (RNS - 1)) * RS_STAGE + 1024 * (wave - 1);
    return rsm + RSCR_OFF;
  };
  auto issue_x3 = [&](int kx) {  // the three pixel pieces of K-step kx
    unsigned char* st = rsm + (kx & (RNS - 1)) * RX_STAGE;
#pragma unroll
    for (int u = 0; u < 3; ++u) bdma16_asm(rx, voff[u], (unsigned)kx * xstep, st + 1024 * (wave + 8 * u));
  };
  // group of K-step kt of the steady loop: pixels of kx = kt + 3 and side data of ks = kt + 4 (null past the end)
  auto issue_group = [&](int kx, int ks, bool side_ok) {
    issue_x3(kx);
    const dma_i32x4 r = (wave == 0 || side_ok) ? r3 : rnull;
    bdma16_asm(r, voff[3], (unsigned)(wave == 0 ? kx : ks) * step3, dst3(kx, ks));
  };

  // dz tile of wave w: rows 16 (w >> 2) + (lane & 15), hidden 16 (w & 3) + 4 (lane >> 4) .. +3 (as u8_wgrad_kernel<2>)
  const int fr = 16 * (wave >> 2) + (lane & 15), fc = 16 * (wave & 3) + 4 * (lane >> 4);
  const int mword = (n0 + fc) / 32, mshift = (n0 + fc) & 31;
  float w4[4];
  {
    const int g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      w4[kk] = 4 * g + kk < C ? p.w2[(size_t)(4 * g + kk) * p.N + n0 + 16 * (wave & 3) + (lane & 15)] : 0.f;
  }
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
  u16* dzb = reinterpret_cast<u16*>(rsm + RDZ_OFF);
  const int doff = fr * GDP + (((fc >> 2) ^ dz_swz(fr)) << 2);
  // dz build of K-step kt in two parts: the side-data reads (issued early in a K-step) and the fp32 MFMAs, split and
  // plane stores (after the first substep's MFMAs)
  struct DzIn {
    float d4[4];
    unsigned bits;
  };
  auto build_dz_load = [&](int kt, DzIn& in) {
    const unsigned char* st = rsm + RS_OFF + (kt & (RNS - 1)) * RS_STAGE;
    const float* sdl = reinterpret_cast<const float*>(st) + fr * C;
    in.bits = reinterpret_cast<const unsigned*>(st + 2048)[fr * NW + mword];
    const int g = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const float v = sdl[min(4 * g + kk, C - 1)];
      in.d4[kk] = 4 * g + kk < C ? v : 0.f;
    }
  };
  auto build_dz_finish = [&](int kt, const DzIn& in) {
    if constexpr (MODE == 1) {
      if (kt > 1) return;
    }
    const f32x4 dv = fd_dz_bits(w4, in.d4, (in.bits >> mshift) & 15u);
    bsum += dv;
    u16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = dv[e] * dz_up;  // exact (power of two), |x| < 2^14
      const _Float16 h = static_cast<_Float16>(x);
      hi[e] = __builtin_bit_cast(u16, h);
      lo[e] = __builtin_bit_cast(u16, static_cast<_Float16>(x - static_cast<float>(h)));
    }
    u16* B = dzb + (kt % 3) * RDZ_BUF;
    *reinterpret_cast<u16x4*>(B + doff) = hi;
    *reinterpret_cast<u16x4*>(B + doff + GD_U16) = lo;
  };
  auto build_dz = [&](int kt) {
    DzIn in;
    build_dz_load(kt, in);
    build_dz_finish(kt, in);
  };

  // EARLY: where the wave builds its dz tile in a K-step - after the first substep's MFMAs (waves 0..3) or after the
  // second (waves 4..7). The two waves of a SIMD (w, w + 4) then never wait on the build's dependent chain (LDS reads,
  // four fp32 MFMAs, the split) at the same time: one issues MFMAs while the other builds.
  auto run = [&](auto nct_c, auto half_c, auto early_c) {
    constexpr int NCT = decltype(nct_c)::value;
    constexpr bool HALF = decltype(half_c)::value;  // BAL: this wave's 16 hidden of columns 768..783
    constexpr bool EARLY = decltype(early_c)::value;
    const int ct0 = BAL ? 3 * wave : NCT == 4 ? 0 : 4 + 3 * (wave - 1);  // first 32-column tile
    f32x16 acc[2][NCT];
    f32x4 hacc = {0.f, 0.f, 0.f, 0.f};
    f16x8 ha[GNPL], hb;
    // 16x16x32 operands of the half tile for the whole K-step (k-rows 8 (lane >> 4) + j): dz rows through two tr16
    // reads (hidden 16 (wave - 4) + (lane & 15)), pixel column 768 + (lane & 15) through one tr8 read
    auto load_half = [&](int kt) {
      if constexpr (HALF) {
        const unsigned char* X8 = rsm + (kt & (RNS - 1)) * RX_STAGE;
        const u16* D = dzb + (kt % 3) * RDZ_BUF;
        const int g = lane >> 4, i = lane & 15;
        const int r = 8 * g + (i >> 2), col = 16 * (wave - 4) + 4 * (i & 3);
#pragma unroll
        for (int pl = 0; pl < GNPL; ++pl) {
          const s16x4 lo = tr16(D + pl * GD_U16 + r * GDP + (((col >> 2) ^ dz_swz(r)) << 2));
          const s16x4 hi = tr16(D + pl * GD_U16 + (r + 4) * GDP + (((col >> 2) ^ dz_swz(r + 4)) << 2));
          bf16x8 f;
          f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
          f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
          ha[pl] = __builtin_bit_cast(f16x8, f);
        }
        const unsigned char* xa = X8 + (8 * g + (i >> 1)) * RX_PITCH + 768 + 8 * (i & 1);
        const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(xa));
        hb = widen8h((unsigned)v[0], (unsigned)v[1]);
      }
    };
    auto mma_half = [&]() {
      if constexpr (HALF) {
        hacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[1], hb, hacc, 0, 0, 0);  // lo
        hacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha[0], hb, hacc, 0, 0, 0);  // hi
      }
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[i][j] = f32x16{};
    // the fragments of one k-substep: dz planes (2 hidden tiles x 2 planes) and the wave's pixel tiles
    struct Frag {
      f16x8 a[2][GNPL];
      i32x2 b[NCT];  // raw pixel bytes (widened next to their MFMAs)
    };
    auto load = [&](int kt, int s, Frag& f) {
      const unsigned char* X8 = rsm + (kt & (RNS - 1)) * RX_STAGE;
      const u16* D = dzb + (kt % 3) * RDZ_BUF;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pl = 0; pl < GNPL; ++pl) f.a[i][pl] = frag_tr_dz<GDP>(D + pl * GD_U16, 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < NCT; ++j) f.b[j] = frag_x8_raw(X8, 32 * (ct0 + j), s, lane);
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
      for (int j = 0; j < NCT; ++j) {
        f16x8 b;
        if constexpr (MODE == 2) {  // (timing: raw bytes as fp16 bits)
          const u32x4 r = {(unsigned)f.b[j][0], (unsigned)f.b[j][1], (unsigned)f.b[j][0], (unsigned)f.b[j][1]};
          b = __builtin_bit_cast(f16x8, r);
        } else {
          b = widen8h((unsigned)f.b[j][0], (unsigned)f.b[j][1]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (MODE == 4) {  // no MFMA: keep the fragments alive with one VALU add each
            acc[i][j][0] += (float)(f.a[i][1][0] + f.a[i][0][1] + b[i]);
          } else {
            acc[i][j] = mfma(f.a[i][1], b, acc[i][j]);  // lo
            acc[i][j] = mfma(f.a[i][0], b, acc[i][j]);  // hi
          }
        }
      }
    };
    // prologue: side data of K-steps 0..3 (one group), pixels of 0, 1, 2 (a group each); wait for all but the last
    // pixel group, build dz 0 and 1, publish them, read k-substep 0 of K-step 0
    // (W2 values in registers first: the compiler's own wait for them would be a vmcnt(0) behind the DMA it cannot see)
    asm volatile("" ::"v"(w4[0]), "v"(w4[1]), "v"(w4[2]), "v"(w4[3]), "v"(av));  // (and the bound: waited here, not behind the DMA)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      bdma16_asm(wave > 0 && wave < 4 && ks < nk ? r3 : rnull, voff[3], (unsigned)ks * step3,
                 wave > 0 && wave < 4 ? dst3(0, ks) : rsm + RSCR_OFF);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      issue_x3(kx < nk ? kx : 0);  // (K-steps past the end re-read step 0 into unused stages)
      bdma16_asm(wave == 0 ? r3 : rnull, voff[3], (unsigned)(kx < nk ? kx : 0) * step3,
                 wave == 0 ? dst3(kx, 0) : rsm + RSCR_OFF);
    }
    if (fast_bound) {
      const float bw = wv::max64(av);
      if (lane == 0) bred[wave] = bw;
    }
    wait_vm<4>();
    __syncthreads();
    if (fast_bound) {  // = wgrad_scales' amax path
      float bnd = bred[0];
#pragma unroll
      for (int w = 1; w < GT / 64; ++w) bnd = fmaxf(bnd, bred[w]);
      const int E = bound_exp(bnd);
      dz_up = pow2f(14 - E);
      out_scale = p.scale * pow2f(E - 14);
    }
    build_dz(0);
    if (nk > 1) build_dz(1);
    __syncthreads();
    Frag f0, f1;
    load(0, 0, f0);
    U8W_STAMP(3, __builtin_amdgcn_s_memtime);
    // K-step kt (one barrier, at its end): pixel group kt + 3 and side group kt + 4 issued; k-substep 1 read and both
    // substeps' MFMAs; dz of kt + 2 built; k-substep 0 of kt + 1 read (published by the barrier that ended kt - 1).
    // The barrier ending kt waits for every DMA group but kt's own: pixels of kt + 2 and side data of kt + 3, which
    // step kt + 1 reads. Stage reuse: pixel stage (kt + 3) % 4 was last read in step kt - 1, side stage (kt + 4) % 4 in
    // step kt - 2, dz buffer (kt + 2) % 3 in step kt - 1.
    int kt = 0;
    for (; kt + 3 < nk; ++kt) {
      issue_group(kt + 3, kt + 4, kt + 4 < nk);
      if constexpr (MODE != 6) {  // (MODE 6, timing: the DMA ring alone)
        load(kt, 1, f1);
        load_half(kt);
        DzIn dzi;
        build_dz_load(kt + 2, dzi);
        mma(f0);
        if constexpr (EARLY) build_dz_finish(kt + 2, dzi);
        mma(f1);
        mma_half();
        if constexpr (!EARLY) build_dz_finish(kt + 2, dzi);
        load(kt + 1, 0, f0);
      }
#ifdef SDML_KERNEL_EXPERIMENTS
      if (kt == 0 || kt == 8 || kt == 16) U8W_STAMP(4 + kt / 8 * 2, __builtin_amdgcn_s_memtime);  // before barrier
#endif
      // The barrier publishes this step's dz-plane stores and the DMA of kt + 2 (wait_vm). Not __syncthreads: its
      // fence would also wait for the substep-0 reads of kt + 1 just issued, which may stay in flight across it (what
      // they read is not rewritten before the barrier ending kt + 1). The plane stores precede those 8 + NCT reads in
      // program order (the compiler cannot separate their addresses) and LDS operations complete in order, so
      // lgkmcnt(8 + NCT) covers the stores.
      wait_vm<4>();
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(8 + NCT) : "memory");
      if constexpr (MODE != 3) __builtin_amdgcn_s_barrier();
#ifdef SDML_KERNEL_EXPERIMENTS
      if (kt == 0 || kt == 8 || kt == 16) U8W_STAMP(5 + kt / 8 * 2, __builtin_amdgcn_s_memtime);  // after barrier
#endif
    }
    for (; kt < nk; ++kt) {  // the last three K-steps: no further DMA
      load(kt, 1, f1);
      load_half(kt);
      mma(f0);
      if (kt + 2 < nk) build_dz(kt + 2);
      mma(f1);
      mma_half();
      if (kt + 1 < nk) {
        load(kt + 1, 0, f0);
        wait_vm<0>();
        __syncthreads();
      }
    }
    U8W_STAMP(10, __builtin_amdgcn_s_memtime);
    if (pairing) role = wgrad_pair_role(p, group, split, t, reinterpret_cast<int*>(rsm));
    const int row = role == 1 ? split % (p.splits / 2) : split;  // the pair sum goes to the lower split's row
    const int add_row = split < p.splits / 2 ? split + p.splits / 2 : split - p.splits / 2;
    wgrad_store_tile<NCT>(p, acc, row, n0, ct0, lane, out_scale, role, add_row);
    if constexpr (HALF) {  // C map of 16x16: column lane & 15, rows 4 (lane >> 4) + v
#pragma clang fp contract(off)
      float* out = p.slab + (size_t)row * ((size_t)p.N * GKC + p.N);
      const float* pin = p.slab + (size_t)add_row * ((size_t)p.N * GKC + p.N);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const size_t e = (size_t)(n0 + 16 * (wave - 4) + 4 * (lane >> 4) + v) * GKC + 768 + (lane & 15);
        const float o = hacc[v] * out_scale;
        if (role == 0) st_sc1(out + e, o);
        else out[e] = role == 1 ? o + ld_sc1(pin + e) : o;
      }
    }
    U8W_STAMP(11, __builtin_amdgcn_s_memtime);
  };
  using I3 = std::integral_constant<int, 3>;
  if constexpr (BAL) {
    if (wave >= 4) run(I3{}, std::true_type{}, std::false_type{});
    else run(I3{}, std::false_type{}, std::true_type{});
  } else {
    if (wave == 0) run(std::integral_constant<int, 4>{}, std::false_type{}, std::true_type{});
    else if (wave < 4) run(I3{}, std::false_type{}, std::true_type{});
    else run(I3{}, std::false_type{}, std::false_type{});
  }
  __syncthreads();
  {
    const int row = role == 1 ? split % (p.splits / 2) : split;
    const int add_row = split < p.splits / 2 ? split + p.splits / 2 : split - p.splits / 2;
    wgrad_store_bias<2>(p, bsum, row, n0, t, reinterpret_cast<float*>(rsm), role, add_row);
  }
  if (pairing && role == 0) wgrad_pair_publish(p, group, split, t);
  U8W_STAMP(12, __builtin_amdgcn_s_memtime);
  U8W_STAMP(15, __builtin_amdgcn_s_memrealtime);
}

// The step's two deterministic reductions in one launch: blocks [0, nhead) run the fused head's reduction
// (head_reduce.h: two dependent round trips of 4-byte loads, so they start first instead of trailing the grid),
// the blocks after them sum the weight gradient's split slabs. Saves the head reduction's own launch (~5 us of
// latency-bound work) on the one-rank MLP step.
// Slab blocks, COLS float4 columns each: wave w's partial of a column is ((a0 + a1) + (a2 + a3)), a[u & 3] summing
// splits w + 16u (u = 0..7, then w + 128, ... into a0), and the 16 wave partials are added in wave order. COLS = 64:
// one lane per column; COLS = 32: lanes 32..63 take a2, a3 of the lane 32 below (twice the blocks, half the loads
// per lane; the same sums in the same order, so the same bits).
// sg.p set: these are the step's last gradients, and the optimizer step is applied here (sgd_rule.h)
// instead of by a separate SGD launch over the flat buffer.
// Segments: slab blocks [0, nA) reduce [a_off, a_end), blocks [nA, nslab) reduce [b_off, b_end) (offsets into the
// [N * 784 + N] gradient, multiples of 4): the whole gradient is one segment; one hidden-group range of a
// split weight gradient is its weight rows plus its bias entries.
struct SlabSegs {
  int64_t a_off, a_end, b_off, b_end;
  int nA;
};

template <int COLS>
__global__ void __launch_bounds__(1024) slab_head_reduce_kernel(const float* __restrict__ slab, int64_t stride,
                                                                int splits, float* __restrict__ out, SlabSegs sgs,
                                                                int nslab, int nhead, HeadReduceArgs head,
                                                                SgdFuse sg) {
  static_assert(COLS == 64 || COLS == 32, "one or two lanes per column");
  __shared__ f32x4 part[16][64];
  if ((int)blockIdx.x < nhead) {
    head_reduce_block(head, blockIdx.x, reinterpret_cast<float(*)[64]>(&part[0][0]), sg.p ? &sg : nullptr);
    return;
  }
  const int bx = (int)blockIdx.x - nhead;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c = l % COLS, half = l / COLS;  // (COLS = 64: half = 0)
  const bool segA = bx < sgs.nA;
  const int64_t i = (segA ? sgs.a_off : sgs.b_off) + ((int64_t)(segA ? bx : bx - sgs.nA) * COLS + c) * 4;
  const int64_t n = segA ? sgs.a_end : sgs.b_end;
  const bool lead = half == 0;
  // wave 0's epilogue operands (the gradient it adds into, the parameter, its momentum) are loaded first, with the
  // partials: one memory round trip for all of them instead of two more after the sum
  f32x4 acc0 = {}, pv0 = {}, bv0 = {};
  if (w == 0 && lead && i < n) {
    acc0 = *reinterpret_cast<const f32x4*>(out + i);
    if (sg.p) {
      pv0 = *reinterpret_cast<const f32x4*>(sg.p + i);
      if (sg.mom != 0.f && !sg.first) bv0 = *reinterpret_cast<const f32x4*>(sg.buf + i);
    }
  }
  f32x4 a[4] = {};
  if (i < n) {
    int s = w;  // wave w: splits w, w + 16, ...
    if constexpr (COLS == 64) {
      for (; s + 16 * 7 < splits; s += 16 * 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u & 3] += *reinterpret_cast<const f32x4*>(slab + (int64_t)(s + 16 * u) * stride + i);
      }
    } else {  // this lane's two of the four: u & 3 in {2 half, 2 half + 1}
      for (; s + 16 * 7 < splits; s += 16 * 8) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int u = (v & 1) + 2 * half + 4 * (v >> 1);
          a[v & 1] += *reinterpret_cast<const f32x4*>(slab + (int64_t)(s + 16 * u) * stride + i);
        }
      }
    }
    if (lead)
      for (; s < splits; s += 16) a[0] += *reinterpret_cast<const f32x4*>(slab + (int64_t)s * stride + i);
  }
  if constexpr (COLS == 64) {
    part[w][l] = (a[0] + a[1]) + (a[2] + a[3]);
  } else {
    part[w][l] = a[0] + a[1];  // lanes c: a0 + a1, lanes 32 + c: a2 + a3
  }
  __syncthreads();
  if (w == 0 && lead && i < n) {
    f32x4 acc = acc0;
    f32x4 t = COLS == 64 ? part[0][l] : part[0][l] + part[0][l + 32];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += COLS == 64 ? part[q][l] : part[q][l] + part[q][l + 32];
    acc += t;
    if (sg.p) {
      const f32x4 nv = sgd_update4_pre(sg.p + i, sg.buf + i, acc, SgdRule{sg.lr, sg.mom, sg.damp, sg.wd, sg.nesterov, sg.first},
                                       pv0, bv0);
      const int64_t i4 = i / 4;
      if (sg.planes && i4 >= sg.pl_off4 && i4 < sg.pl_off4 + sg.pl_n4) {
        const int64_t e = i - 4 * sg.pl_off4;
        sgd_write_planes4(sg.planes + (e / sg.K) * sg.Kp + e % sg.K, sg.plane_stride, nv);
      }
      if (sg.zero_grad) acc = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    *reinterpret_cast<f32x4*>(out + i) = acc;
  }
}

// launch: the segments' slab blocks at COLS columns each, the head's blocks in front
static void launch_slab_head_reduce(const float* slab, int64_t stride, int splits, float* out, int64_t a_off,
                                    int64_t a_end, int64_t b_off, int64_t b_end, const HeadReduceArgs* head,
                                    const SgdFuse* sg, hipStream_t stream) {
  const int cols = knob(KNOB_U8_SLAB_COLS) == 32 ? 32 : 64;
  SlabSegs sgs{a_off, a_end, b_off, b_end, (int)(((a_end - a_off) / 4 + cols - 1) / cols)};
  const int nslab = sgs.nA + (int)(((b_end - b_off) / 4 + cols - 1) / cols);
  const bool hd = head && head->part;
  const int nhead = hd ? head_reduce_blocks(*head) : 0;
  const dim3 grid(nslab + nhead);
  const HeadReduceArgs ha = hd ? *head : HeadReduceArgs();
  const SgdFuse sf = sg ? *sg : SgdFuse();
  if (cols == 32)
    hipLaunchKernelGGL(slab_head_reduce_kernel<32>, grid, dim3(1024), 0, stream, slab, stride, splits, out, sgs, nslab,
                       nhead, ha, sf);
  else
    hipLaunchKernelGGL(slab_head_reduce_kernel<64>, grid, dim3(1024), 0, stream, slab, stride, splits, out, sgs, nslab,
                       nhead, ha, sf);
}

}  // namespace

// substeps of the last K-step that hold k < K (lane half 0 covers its first FBK / 2 k; the rest
// multiply zero-padded weights)
static int wgrad_xcd() {
  return knob(KNOB_U8_WGRAD_XCD);
}

// the pairwise combine's ticket / flag words: one zeroed allocation per device, made on the first eager call (none is
// made while a stream is being captured: the combine is then off for that launch); the kernel leaves them zero
static unsigned* wgrad_pair_words(hipStream_t stream) {
  static unsigned* words[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!words[dev]) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    void* w = nullptr;
    if (hipMalloc(&w, 4096 * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(w, 0, 4096 * sizeof(unsigned)) != hipSuccess) return nullptr;
    words[dev] = static_cast<unsigned*>(w);
  }
  return words[dev];
}

static int tail_substeps(int K) {
  const int v = K - ((K + FBK - 1) / FBK - 1) * FBK;
  if (v > FBK / 2 - 8) return NSUB;
  if (NSUB == 4 && v > 16) return 3;
  if (NSUB == 4 && v > 8) return 2;
  return 1;
}

int u8_fwd_kpad(int K) { return (K + FBK - 1) / FBK * FBK; }  // zero-padded W planes

bool u8_fwd_supported(int M, int N, int K, int ldx, const void* X) {
  // (the epilogue stores 16-B row pieces: C 16-B aligned with ldc % 4 == 0, checked by the caller)
  return M >= 256 && N % FBN == 0 && K >= 16 && K % 16 == 0 && ldx % 16 == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (int64_t)M * ldx < (int64_t(1) << 31);
}

bool u8_wgrad_supported(int M, int N, int K, int ldx, const void* X, const void* dz) {
  return K == GKC && N % GHN == 0 && M % GBK == 0 && M >= GBK && ldx % 16 == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(dz) & 15) == 0 &&
         (int64_t)M * ldx < (int64_t(1) << 31);
}

int u8_wgrad_splits(int M, int N) {
  // one workgroup per CU: (N / 64) hidden groups x splits ~ 256 workgroups, >= 4 K-steps each
  const int groups = N / GHN;
  int splits = std::max(1, 256 / std::max(1, groups));
  splits = std::min(splits, std::max(1, M / (4 * GBK)));
  const int rps = ((M + splits - 1) / splits + GBK - 1) / GBK * GBK;
  return (M + rps - 1) / rps;
}

int u8_wgrad_group_splits(int M, int blocks) {
  const int rps = ((M + std::max(1, blocks) - 1) / std::max(1, blocks) + GBK - 1) / GBK * GBK;
  return (M + rps - 1) / rps;
}

int64_t u8_wgrad_slab_floats(int M, int N, int blocks) {
  const int splits = blocks > 0 ? u8_wgrad_group_splits(M, blocks) : u8_wgrad_splits(M, N);
  return (int64_t)splits * ((int64_t)N * GKC + N);
}

void u8_wgrad(const float* dz, const unsigned char* X, int M, int N, int ldx, float* slab, float* gwb, float scale,
              const float* amax, int namax, hipStream_t stream) {
  if (!amax || namax < 1) abort();  // host contract: the dz bound is given
  WgradParams p{};
  p.dz = dz;
  p.amax = amax;
  p.namax = namax;
  p.X = X;
  p.slab = slab;
  p.M = M;
  p.N = N;
  p.ldx = ldx;
  p.scale = scale;
  const int splits = u8_wgrad_splits(M, N);
  p.rows_per_split = ((M + splits - 1) / splits + GBK - 1) / GBK * GBK;
  p.groups = N / GHN;
  p.splits = splits;
  p.xcd = wgrad_xcd();
  p.prio = knob(KNOB_U8_WGRAD_PRIO);
  hipLaunchKernelGGL(u8_wgrad_kernel<0>, dim3(((splits + 7) / 8) * 8 * p.groups), dim3(GT), 0, stream, p);
  slab_reduce(slab, (int64_t)N * GKC + N, splits, gwb, (int64_t)N * GKC + N, stream);
}

bool u8_wgrad_dl_supported(int M, int N, int K, int ldx, const void* X, const void* h, int C) {
  return u8_wgrad_supported(M, N, K, ldx, X, h) && C >= 1 && C <= 16;
}

void u8_wgrad_dl(const float* dl, const float* w2, const float* h, const unsigned* mask, int C,
                 const unsigned char* X, int M, int N, int ldx, float* slab, float* gwb, float scale,
                 const float* amax, int namax, hipStream_t stream, const HeadReduceArgs* head, const SgdFuse* sgd,
                 const WgradGroups* grp) {
  if ((h == nullptr) == (mask == nullptr)) abort();  // host contract: exactly one ReLU-mask source
  if (grp && (grp->g_count < 1 || grp->g_first < 0 || (grp->g_first + grp->g_count) * GHN > N || grp->blocks < 1))
    abort();  // host contract: a range of whole hidden groups
  WgradParams p{};
  p.amax = namax > 0 ? amax : nullptr;
  p.namax = namax;
  p.X = X;
  p.slab = slab;
  p.M = M;
  p.N = N;
  p.ldx = ldx;
  p.scale = scale;
  p.dl = dl;
  p.w2 = w2;
  p.h = h;
  p.mask = mask;
  p.C = C;
  p.groups = grp ? grp->g_count : N / GHN;
  p.g0 = grp ? grp->g_first : 0;
  const int splits = grp ? u8_wgrad_group_splits(M, grp->blocks) : u8_wgrad_splits(M, N);
  p.rows_per_split = ((M + splits - 1) / splits + GBK - 1) / GBK * GBK;
  p.splits = splits;
  p.xcd = wgrad_xcd();
  p.prio = knob(KNOB_U8_WGRAD_PRIO);
#ifdef SDML_KERNEL_EXPERIMENTS
  p.stamps = g_u8w_stamps;
#endif
  const dim3 wgrid(((splits + 7) / 8) * 8 * p.groups);
  const bool ilv = knob(KNOB_U8_WGRAD_ILV) != 0;
  // pairwise combine (ring kernel, whole weight gradient, XCD-aware order so splits s and s + S/2 share an XCD)
  p.pair = nullptr;
  if (!grp && p.xcd && splits % 16 == 0 && p.groups * splits <= 4096 && knob(KNOB_U8_WGRAD_PAIR) != 0 && mask && !ilv &&
      knob(KNOB_U8_WGRAD_RING) != 0)
    p.pair = wgrad_pair_words(stream);
  // the DMA-ring form: ReLU bits, one DMA piece of them and two of dl rows per K-step, 16-B aligned sources
  const bool ring = mask && !ilv && knob(KNOB_U8_WGRAD_RING) != 0 && N <= 256 && C <= 16 &&
                    (reinterpret_cast<uintptr_t>(dl) & 15) == 0 && (reinterpret_cast<uintptr_t>(mask) & 15) == 0;
  if (ring) {
#ifdef SDML_KERNEL_EXPERIMENTS
    switch (knob(KNOB_U8_VARIANT)) {
      case 1: hipLaunchKernelGGL(u8_wgrad_ring_kernel<1>, wgrid, dim3(GT), 0, stream, p); break;
      case 2: hipLaunchKernelGGL(u8_wgrad_ring_kernel<2>, wgrid, dim3(GT), 0, stream, p); break;
      case 3: hipLaunchKernelGGL(u8_wgrad_ring_kernel<3>, wgrid, dim3(GT), 0, stream, p); break;
      case 4: hipLaunchKernelGGL(u8_wgrad_ring_kernel<4>, wgrid, dim3(GT), 0, stream, p); break;
      case 6: hipLaunchKernelGGL(u8_wgrad_ring_kernel<6>, wgrid, dim3(GT), 0, stream, p); break;
      case 5: hipLaunchKernelGGL((u8_wgrad_ring_kernel<0, true>), wgrid, dim3(GT), 0, stream, p); break;
      default:
        if (knob(KNOB_U8_WGRAD_BAL)) hipLaunchKernelGGL((u8_wgrad_ring_kernel<0, true>), wgrid, dim3(GT), 0, stream, p);
        else hipLaunchKernelGGL((u8_wgrad_ring_kernel<0, false>), wgrid, dim3(GT), 0, stream, p);
    }
#else
    if (knob(KNOB_U8_WGRAD_BAL)) hipLaunchKernelGGL((u8_wgrad_ring_kernel<0, true>), wgrid, dim3(GT), 0, stream, p);
    else hipLaunchKernelGGL((u8_wgrad_ring_kernel<0, false>), wgrid, dim3(GT), 0, stream, p);
#endif
  }
  else if (mask && ilv) hipLaunchKernelGGL((u8_wgrad_kernel<2, true>), wgrid, dim3(GT), 0, stream, p);
  else if (mask) hipLaunchKernelGGL((u8_wgrad_kernel<2, false>), wgrid, dim3(GT), 0, stream, p);
  else if (ilv) hipLaunchKernelGGL((u8_wgrad_kernel<1, true>), wgrid, dim3(GT), 0, stream, p);
  else hipLaunchKernelGGL((u8_wgrad_kernel<1, false>), wgrid, dim3(GT), 0, stream, p);
  const int64_t n = (int64_t)N * GKC + N;
  const int rsplits = (ring && p.pair) ? splits / 2 : splits;  // rows left for the reduction
  if (!ring) p.pair = nullptr;
  if (grp) {  // this hidden-group range only: its weight rows, then its bias entries (+ the head's reduction)
    if (sgd && sgd->p) abort();  // host contract: the split weight gradient is not the fused optimizer step
    const int64_t b_off = (int64_t)N * GKC + grp->g_first * GHN;
    launch_slab_head_reduce(slab, n, splits, gwb, (int64_t)grp->g_first * GHN * GKC,
                            (int64_t)(grp->g_first + grp->g_count) * GHN * GKC, b_off, b_off + grp->g_count * GHN, head,
                            nullptr, stream);
  } else if (head && head->part) {
    launch_slab_head_reduce(slab, n, rsplits, gwb, 0, n, n, n, head, sgd, stream);
  } else {
    if (sgd && sgd->p) abort();  // host contract: the fused step needs the head reduction in the same launch
    slab_reduce(slab, n, rsplits, gwb, n, stream);
  }
}

void split_planes_pad(const float* w, unsigned short* out, int N, int K, int Kp, hipStream_t stream) {
  const int64_t n = (int64_t)N * Kp;
  hipLaunchKernelGGL(split_planes_pad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, w, out, N, K, Kp);
}

// the forward's block geometry for M rows: 16 waves of 512 rows, or 8 waves of 128 WMT rows
static void u8_fwd_geometry(int M, bool& w16, int& wmt, int& bm) {
  const int wmt_env = knob(KNOB_U8_FWD_WMT);
  const int waves_env = knob(KNOB_U8_FWD_WAVES);  // 8 (512 threads) or 16 (1024 threads, 4 waves per SIMD)
  // 512-row blocks (half the LDS weight traffic per MFMA) once they still cover every CU, as 16
  // waves of 64 x 64 (4 waves per SIMD at 115 VGPRs; 8 waves of 128 x 64 need 199: 63.9-65.3 vs
  // 66.5-67.3 us at 131072 rows, tools/gpu_fwd16.sh); smaller batches: 256-row blocks of 8 waves
  const bool big = M >= 256 * Geo<4>::BM;
  w16 = waves_env ? waves_env == 16 : (big && !wmt_env);
  wmt = wmt_env ? wmt_env : (big ? 4 : 2);
  if (w16) wmt = 2;
  bm = w16 ? Geo<2, 8>::BM : (wmt == 4 ? Geo<4>::BM : Geo<2>::BM);
}

int u8_fwd_wmax_slots(int M, int N) {
  bool w16;
  int wmt, bm;
  u8_fwd_geometry(M, w16, wmt, bm);
  return ((M + bm - 1) / bm) * (N / FBN) * (w16 ? 16 : 8);
}

void u8_fwd(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_planes, int N, int Kp,
            const float* bias, float* C, int ldc, bool relu, float scale, hipStream_t stream, unsigned* mask,
            float* wmax) {
  if (mask && !relu) abort();  // host contract: the ReLU bits need the ReLU epilogue
  FwdParams p{};
  p.mask = mask;
  p.wmax = wmax;
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
  p.scale = scale / kU8FwdWScale;  // the planes hold W * 2^8 (exact power of two)
  p.relu = relu ? 1 : 0;
#ifdef SDML_KERNEL_EXPERIMENTS  // timing-experiment variants (tools/bench_u8.py): not in production builds
  static const int mode = [] {
    const char* e = getenv("SDML_U8_FWD_MODE");
    return e ? atoi(e) : 0;
  }();
#else
  constexpr int mode = 0;
#endif
  bool w16;
  int wmt, bm;
  u8_fwd_geometry(M, w16, wmt, bm);
  const dim3 grid((M + bm - 1) / bm, N / FBN);
  const int tail = tail_substeps(K);
#define FWD_LAUNCH(MD, W, T, R) \
  hipLaunchKernelGGL((u8_fwd_kernel<MD, W, T, R>), grid, dim3(Geo<W, R>::THREADS), 0, stream, p)
#define FWD_TAILS(W, R)                          \
  do {                                           \
    switch (tail) {                              \
      case 1: FWD_LAUNCH(0, W, 1, R); break;     \
      case 2: FWD_LAUNCH(0, W, 2, R); break;     \
      case 3: FWD_LAUNCH(0, W, 3, R); break;     \
      default: FWD_LAUNCH(0, W, NSUB, R);        \
    }                                            \
  } while (0)
#define FWD_MODE(MD)                                \
  do {                                              \
    if (w16) FWD_LAUNCH(MD, 2, NSUB, 8);            \
    else if (wmt == 4) FWD_LAUNCH(MD, 4, NSUB, 4);  \
    else FWD_LAUNCH(MD, 2, NSUB, 4);                \
  } while (0)  // timing modes: full last K-step
#ifdef SDML_KERNEL_EXPERIMENTS
  if (mode == 1) FWD_MODE(1);
  else if (mode == 2) FWD_MODE(2);
  else if (mode == 3) FWD_MODE(3);
  else if (mode == 4) FWD_MODE(4);
  else if (mode == 5) FWD_MODE(5);
  else if (mode == 6) FWD_MODE(6);
  else
#endif
  if (w16) FWD_TAILS(2, 8);
  else if (wmt == 4) FWD_TAILS(4, 4);
  else FWD_TAILS(2, 4);
#undef FWD_TAILS
#undef FWD_MODE
#undef FWD_LAUNCH
}

bool u8_fwd_head_supported(int M, int N, int K, int ldx, const void* X, int C) {
  return u8_fwd_supported(M, N, K, ldx, X) && N == FBN && (C == 2 || C == 10 || C == 16);
}

// rows per fused-head block: 256 (8 waves, one block per CU; head_block.h)
static int fh_rows() { return hblk::ROWS; }
int u8_fwd_head_blocks(int M) { return (M + fh_rows() - 1) / fh_rows(); }


bool u8_set_stamps(void* buf) {
#ifdef SDML_KERNEL_EXPERIMENTS
  g_u8_stamps = static_cast<long long*>(buf);
  return true;
#else
  (void)buf;
  return false;  // production builds carry no stamp variant
#endif
}
int u8_stamp_slots() { return U8_NSTAMP; }

namespace {
// one wave: a 1-KiB byte image in LDS, ds_read_b64_tr_b8 at per-lane byte addresses (multiples of 8), the 8 bytes
// each lane gets -> out[lane][2] (tests/test_fused_head_gpu.py pins the lane map frag_x8 assumes)
__global__ void __launch_bounds__(64) tr8_probe_kernel(const unsigned char* img, const int* addr, int* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  const int l = threadIdx.x;
  *reinterpret_cast<u32x4*>(s + 16 * l) = *reinterpret_cast<const u32x4*>(img + 16 * l);
  __syncthreads();
  const int a = addr[l] & 1016;
  const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(s + a));
  out[2 * l] = v[0];
  out[2 * l + 1] = v[1];
}
}  // namespace

void u8_tr8_probe(const unsigned char* img, const int* addr, int* out, hipStream_t stream) {
  hipLaunchKernelGGL(tr8_probe_kernel, dim3(1), dim3(64), 0, stream, img, addr, out);
}
bool u8_set_wgrad_stamps(void* buf) {
#ifdef SDML_KERNEL_EXPERIMENTS
  g_u8w_stamps = static_cast<long long*>(buf);
  return true;
#else
  (void)buf;
  return false;
#endif
}

void u8_fwd_head(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_planes, int N, int Kp,
                 const float* bias, float scale, const U8HeadArgs& head, hipStream_t stream) {
  if (N != FBN || !head.dl || !head.mask || !head.part || !head.bound || !bias) abort();  // host contract
  static_assert(Geo<2, 4>::BM == hblk::ROWS, "one fused-head block = its rows");
  FwdParams p{};
  p.X = X;
  p.Wp = w_planes;
  p.bias = bias;
  p.M = M;
  p.N = N;
  p.K = K;
  p.Kp = Kp;
  p.ldx = ldx;
  p.scale = scale / kU8FwdWScale;
  p.relu = 1;
  p.head = head;
  p.prio = knob(KNOB_U8_FWD_PRIO);
  const dim3 grid(u8_fwd_head_blocks(M), 1);
  {  // the next workgroup on an XCD (blocks are dispatched round-robin over the 8 XCDs) is blockIdx + the CU count
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      hipDeviceProp_t pr;
      cus = hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0 ? pr.multiProcessorCount : 256;
    }
    p.pf_stride = knob(KNOB_U8_FWD_PREFETCH) ? cus : 0;
  }
  const int tail = tail_substeps(K);
  const int spread = knob(KNOB_U8_FWD_DMA_SPREAD);  // 0, 1 (spread DMA), 2 (+ fragment reads one substep ahead)
  // 512-row blocks (u8_fwd_kernel HALVES: two head passes per block) once they still give every CU a block
  const int r512k = knob(KNOB_U8_FH_ROWS512);
  const bool rows512 = (r512k >= 0 ? r512k == 1 : M >= 256 * Geo<4, 4>::BM) && spread == 0 &&
                       knob(KNOB_U8_FH_STAGES) != 3;
#ifdef SDML_KERNEL_EXPERIMENTS  // timing variants (tools/u8_fwd_stamps.py): SDML_U8_FWD_MODE 1-6, 8-10
  static const int fmode = [] {
    const char* e = getenv("SDML_U8_FWD_MODE");
    return e ? atoi(e) : 0;
  }();
  if (head.C == 10 && fmode && fmode != 7 && !g_u8_stamps) {
#define FHM(MD) hipLaunchKernelGGL((u8_fwd_kernel<MD, 2, NSUB, 4, 10>), grid, dim3(512), 0, stream, p)
    switch (fmode) {
      case 1: FHM(1); break;
      case 2: FHM(2); break;
      case 3: FHM(3); break;
      case 4: FHM(4); break;
      case 5: FHM(5); break;
      case 8: FHM(8); break;
      case 9: FHM(9); break;
      case 10: FHM(10); break;
      case 11: FHM(11); break;
      default: abort();
    }
#undef FHM
    return;
  }
  // MODE 7: phase stamps into the buffer set by u8_set_stamps
  if (g_u8_stamps && head.C == 10) {
    p.stamps = g_u8_stamps;
    switch (tail) {
      case 1: hipLaunchKernelGGL((u8_fwd_kernel<7, 2, 1, 4, 10>), grid, dim3(512), 0, stream, p); break;
      case 2: hipLaunchKernelGGL((u8_fwd_kernel<7, 2, 2, 4, 10>), grid, dim3(512), 0, stream, p); break;
      case 3: hipLaunchKernelGGL((u8_fwd_kernel<7, 2, 3, 4, 10>), grid, dim3(512), 0, stream, p); break;
      default: hipLaunchKernelGGL((u8_fwd_kernel<7, 2, NSUB, 4, 10>), grid, dim3(512), 0, stream, p);
    }
    return;
  }
#endif
  const dim3 grid512((M + Geo<4, 4>::BM - 1) / Geo<4, 4>::BM, 1);
  if (rows512) p.pf_stride = 0;  // (one round of blocks: nothing runs next on the CU)
#define FH_LAUNCH(T, CC)                                                                                    \
  do {                                                                                                      \
    if (rows512) hipLaunchKernelGGL((u8_fwd_kernel<0, 4, T, 4, CC>), grid512, dim3(512), 0, stream, p);       \
    else if (spread == 2) hipLaunchKernelGGL((u8_fwd_kernel<0, 2, T, 4, CC, NS, 2>), grid, dim3(512), 0, stream, p); \
    else if (spread) hipLaunchKernelGGL((u8_fwd_kernel<0, 2, T, 4, CC, NS, 1>), grid, dim3(512), 0, stream, p); \
    else hipLaunchKernelGGL((u8_fwd_kernel<0, 2, T, 4, CC>), grid, dim3(512), 0, stream, p);               \
  } while (0)
#define FH_LAUNCH3(T) hipLaunchKernelGGL((u8_fwd_kernel<0, 2, T, 4, 10, 3>), grid, dim3(512), 0, stream, p)
#define FH_TAILS(CC)                      \
  do {                                    \
    switch (tail) {                       \
      case 1: FH_LAUNCH(1, CC); break;    \
      case 2: FH_LAUNCH(2, CC); break;    \
      case 3: FH_LAUNCH(3, CC); break;    \
      default: FH_LAUNCH(NSUB, CC);       \
    }                                     \
  } while (0)
  if (head.C == 10 && knob(KNOB_U8_FH_STAGES) == 3) {  // 3-stage ring (the 784-128-10 MLP)
    switch (tail) {
      case 1: FH_LAUNCH3(1); break;
      case 2: FH_LAUNCH3(2); break;
      case 3: FH_LAUNCH3(3); break;
      default: FH_LAUNCH3(NSUB);
    }
    return;
  }
  switch (head.C) {
    case 10: FH_TAILS(10); break;
    case 2: FH_TAILS(2); break;
    case 16: FH_TAILS(16); break;
    default: abort();  // host contract: u8_fwd_head_supported
  }
#undef FH_TAILS
#undef FH_LAUNCH3
#undef FH_LAUNCH
}

}  // namespace sdml
