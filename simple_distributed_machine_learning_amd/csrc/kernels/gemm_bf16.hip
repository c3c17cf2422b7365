// bf16 GEMMs of the GPT-2 stages (BASELINE config 5) with fused epilogues: the forward of every
// Linear (Y = X W^T + b, optionally Y = gelu(X W^T + b) writing the pre-activation too) and the input
// gradient (dX = dY W, optionally times gelu'(u) of the layer below: the MLP's activation backward).
// They replace the hipBLASLt GEMMs of the forward and input-gradient passes and the two GELU kernels
// (the weight gradient is gemm_bf16_wgrad.hip's).
//
//   C[M][N] = A[M][K] . op(B)   A row-major (the activations / incoming gradient, k contiguous)
//     BL = 0 ("NT"): B stored [N][K] (nn.Linear's weight; forward)       -> C = A B^T
//     BL = 1 ("NN"): B stored [K][N] (the same weight; input gradient)   -> C = A B
//
// Geometry (gfx950): 256 x 256 output tile per 512-thread workgroup, 8 waves as 2 (M) x 4 (N), wave tile
// 128 x 64 = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 VGPRs), K-step 64 (two 32-deep substeps).
// Both operands go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 16 B per lane, no VGPR staging) into
// two 64 KiB stages: K-step t+1's DMA is issued before K-step t's fragment reads + MFMAs, then one
// counted wait + barrier per K-step ("2-phase" form of the guide's T3/T4 schedule).
// LDS images are lane-linear per DMA instruction, so the bank swizzles live on the per-lane SOURCE
// address (an involution applied again on the read):
//   [rows][64 k] images (A, NT B): 16-B chunk c of row r stored at c ^ ((r >> 1) & 7): the 16 rows of a
//     ds_read_b128 lane group land in 16 distinct 16-B bank slots (conflict-free)
//   [64 k][256 n] image (NN B): chunk c of k-row r at c ^ (((r & 3) | ((r >> 1) & 4)) << 1): the 8 rows of
//     a 32-lane half of the ds_read_b64_tr_b16 pair (k-rows q, q + 8 of the block) hit distinct 32-B slots
// The grid is remapped XCD-aware (bijective): consecutive tiles of one M panel run on one XCD's L2.
// Epilogue through LDS (the stage buffers are free then): each wave stores its 128 x 64 tile as bf16 rows,
// then every lane moves whole 16-B row pieces, where the elementwise epilogue runs:
//   EPI_BIAS        C = bf16(acc + b)
//   EPI_BIAS_GELU   U = bf16(acc + b) -> aux, C = bf16(gelu(U))            (exactly the unfused pair)
//   EPI_DGELU       C = bf16(gelu'(U) * bf16(acc)), U read from aux       (exactly the unfused pair)
//   EPI_BIAS_GELU_SAVE_GRAD / EPI_MUL_GRAD: the same pair with bf16(gelu'(U)) in aux instead of U (the forward
//     already holds the sigmoid; the backward epilogue is then one multiply, C = bf16(aux * bf16(acc)))
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "gelu.h"
#include "kernels.h"
#include "lds_dma.h"
#include "tile_order.h"

namespace sdml {
namespace {

typedef unsigned short u16;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef u16 u16x8 __attribute__((ext_vector_type(8)));

constexpr int GT = 512, TM = 256, TN = 256, TK = 64;
constexpr int A_BYTES = TM * TK * 2;     // 32 KiB
constexpr int STAGE = 2 * A_BYTES;       // A + B
constexpr int SMEM = 2 * STAGE;          // 128 KiB
constexpr int GLDS = STAGE / 1024 / 8;   // DMA instructions per wave per stage (8)

struct GP {
  const u16* A;
  const u16* B;
  u16* C;
  const u16* bias;  // [N] bf16 (EPI_BIAS, EPI_BIAS_GELU)
  u16* aux;         // EPI_BIAS_GELU: U out; EPI_DGELU: U in ([M][ldaux])
  int M, N, K, lda, ldb, ldc, ldaux;
  int tiles_m, tiles_n;
  int ntstore;  // SDML_GEMM_NT_STORE=1: nontemporal epilogue stores (A/B)
  int gsave;    // EPI_BIAS_GELU: aux = bf16(gelu'(U)); EPI_DGELU: aux holds it (EPI_*_GRAD host values)
  int nostore;  // timing probe (SDML_GEMM_BF16_NOSTORE=1): the epilogue runs but skips its HBM stores
  int group_m;  // tile order (tile_order.h): 0 = M fastest; g > 0 = groups of g m-tiles x every n-tile
};


__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // RNE, NaN-preserving
  return *reinterpret_cast<u16*>(&h);
}

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

__device__ __forceinline__ int rk_swz(int r) { return (r >> 1) & 7; }                          // [rows][64]
__device__ __forceinline__ int kn_swz(int r) { return ((r & 3) | ((r >> 1) & 4)) << 1; }       // [64][256]

// one stage: A tile rows m0.., k0..k0+63; B tile (NT: rows n0.., NN: k-rows k0.., columns n0..)
template <int BL>
__device__ __forceinline__ void issue_stage(const GP& p, unsigned char* st, int m0, int n0, int k0, int wave,
                                            int lane) {
#pragma unroll
  for (int u = 0; u < GLDS / 2; ++u) {  // A: 32 instructions of 8 rows x 128 B
    const int q = wave + 8 * u;
    const int r = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ rk_swz(r);
    const int gr = min(m0 + r, p.M - 1);
    glds16(p.A + (size_t)gr * p.lda + k0 + 8 * c, st + 1024 * q);
  }
#pragma unroll
  for (int u = 0; u < GLDS / 2; ++u) {
    const int q = wave + 8 * u;
    if constexpr (BL == 0) {  // B [N][K]: like A
      const int r = 8 * q + (lane >> 3);
      const int c = (lane & 7) ^ rk_swz(r);
      const int gr = min(n0 + r, p.N - 1);
      glds16(p.B + (size_t)gr * p.ldb + k0 + 8 * c, st + A_BYTES + 1024 * q);
    } else {  // B [K][N]: 2 k-rows x 512 B
      const int r = 2 * q + (lane >> 5);
      const int c = (lane & 31) ^ kn_swz(r);
      const int gc = min(n0 + 8 * c, p.N - 8);
      glds16(p.B + (size_t)(k0 + r) * p.ldb + gc, st + A_BYTES + 1024 * q);
    }
  }
}

__device__ __forceinline__ bf16x8 ld_b128(const unsigned char* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ s16x4 ds_tr16(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// the elementwise part of the epilogues on one 16-B row piece v (bf16(acc (+ bias)) of 8 columns gcol.. of row grow),
// then its store (shared by the 8-wave and 4-wave kernels)
template <int EPI, typename V = u16x8>
__device__ __forceinline__ void store_piece(const GP& p, const V v, int grow, int gcol, const V* pre = nullptr) {
  constexpr int W = sizeof(V) / sizeof(u16);  // 8 (16-B row pieces) or 4 (the persistent kernel's 8-B pieces)
  V o = v;
  if constexpr (EPI == EPI_BIAS_GELU) {
    V* ap = reinterpret_cast<V*>(p.aux + (size_t)grow * p.ldaux + gcol);
    if (p.gsave) {
      V d;
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const float x = bf2f(v[e]), sg = gelu_sig(x);
        o[e] = f2bf(x * sg);  // gelu_f's bits
        d[e] = f2bf(gelu_grad_f(1.f, x));
      }
      if (p.ntstore) __builtin_nontemporal_store(d, ap);
      else *ap = d;
    } else {
      if (p.ntstore) __builtin_nontemporal_store(v, ap);
      else *ap = v;
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = f2bf(gelu_f(bf2f(v[e])));
    }
  } else if constexpr (EPI == EPI_DGELU) {
    const V u = pre ? *pre : *reinterpret_cast<const V*>(p.aux + (size_t)grow * p.ldaux + gcol);  // (pre: loaded early)
    if (p.gsave) {
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = f2bf(bf2f(u[e]) * bf2f(v[e]));
    } else {
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = f2bf(gelu_grad_f(bf2f(v[e]), bf2f(u[e])));
    }
  }
  V* cp = reinterpret_cast<V*>(p.C + (size_t)grow * p.ldc + gcol);
  if (p.ntstore) __builtin_nontemporal_store(o, cp);
  else *cp = o;
}

// epilogue shared by both main loops: bf16 rows through the (free) stage buffers, 16-B row pieces to HBM
// WNW: waves along N (4: the 256 x 256 tile's 2 x 4 waves; 2: the 256 x 128 tile's 2 x 2)
// NJ: 16-column tiles per wave (4: the wave owns 64 columns; 3: 48, the 256 x 192 tile)
// TR: the accumulators hold the transposed product (the MFMA called with the B fragment as its A operand): lane
// (l16, g) then has row 16 i + l16, columns 16 j + 4 g .. + 3 of tile (i, j) - 4 consecutive bf16, one ds_write_b64
// (32 per lane) instead of 4 ds_write_b16 (128 per lane) of one column's 4 rows
template <int EPI, int WNW = 4, int NJ = 4, bool TR = false>
__device__ __forceinline__ void gemm_bf16_epilogue(const GP& p, const f32x4 (&acc)[8][NJ], unsigned char* smem, int m0,
                                                   int n0, int wave, int lane) {
  const int wm = wave / WNW, wn = wave % WNW;
  const int g = lane >> 4, l16 = lane & 15;
  // EPI_DGELU: every aux piece this lane will need, loaded now (rows / columns clamped into the operand: lanes that store
  // nothing load valid memory and drop it)
  u16x8 auxv[EPI == EPI_DGELU ? 16 : 1];
  if constexpr (EPI == EPI_DGELU) {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int row = 8 * it + (lane >> 3), ch = lane & 7;
      const int grow = min(m0 + wm * 128 + row, p.M - 1), gcol = min(n0 + wn * 16 * NJ + 8 * ch, p.N - 8);
      auxv[it] = *reinterpret_cast<const u16x8*>(p.aux + (size_t)grow * p.ldaux + gcol);
    }
  }
  // wave image [128 rows][64 cols] bf16 (128 B rows, 16-B chunks swizzled like the A image; NJ = 3 uses 48 of them)
  unsigned char* W = smem + wave * (128 * 128);
  if constexpr (TR) {
    float bj[NJ][4] = {};
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) bj[j][r] = bf2f(p.bias[min(n0 + wn * 16 * NJ + 16 * j + 4 * g + r, p.N - 1)]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = 16 * i + l16, col = 16 * j + 4 * g;
        typedef u16 u16x4 __attribute__((ext_vector_type(4)));
        u16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(acc[i][j][r] + bj[j][r]);
        *reinterpret_cast<u16x4*>(W + row * 128 + 16 * ((col >> 3) ^ rk_swz(row)) + 2 * (col & 7)) = v;
      }
  } else {
    float bj[NJ] = {};
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = min(n0 + wn * 16 * NJ + 16 * j + l16, p.N - 1);
        bj[j] = bf2f(p.bias[col]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * g + r, col = 16 * j + l16;
          const float v = acc[i][j][r] + bj[j];
          *reinterpret_cast<u16*>(W + row * 128 + 16 * ((col >> 3) ^ rk_swz(row)) + 2 * (col & 7)) = f2bf(v);
        }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if constexpr (EPI == EPI_DGELU) {
    // the 16 aux pieces were loaded before the image writes (one memory round trip instead of four)
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int row = 8 * it + (lane >> 3), ch = lane & 7;
      const u16x8 v = *reinterpret_cast<const u16x8*>(W + row * 128 + 16 * (ch ^ rk_swz(row)));
      const int grow = m0 + wm * 128 + row, gcol = n0 + wn * 16 * NJ + 8 * ch;
      if (ch >= 2 * NJ || grow >= p.M || gcol >= p.N || p.nostore) continue;
      store_piece<EPI>(p, v, grow, gcol, &auxv[it]);
    }
    return;
  }
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int row = 8 * it + (lane >> 3), ch = lane & 7;
    const u16x8 v = *reinterpret_cast<const u16x8*>(W + row * 128 + 16 * (ch ^ rk_swz(row)));
    const int grow = m0 + wm * 128 + row, gcol = n0 + wn * 16 * NJ + 8 * ch;
    if (ch >= 2 * NJ || grow >= p.M || gcol >= p.N || p.nostore) continue;  // (N % 8 == 0: a chunk is all in or out)
    store_piece<EPI>(p, v, grow, gcol);
  }
}

template <int BL, int EPI>
__global__ void __launch_bounds__(GT) gemm_bf16_kernel(GP p) {
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

  // per-lane LDS byte offsets of the fragments (stage-relative)
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

  const int nk = p.K / TK;
  issue_stage<BL>(p, smem, m0, n0, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const unsigned char* st = smem + (t & 1) * STAGE;
    if (t + 1 < nk) issue_stage<BL>(p, smem + ((t + 1) & 1) * STAGE, m0, n0, (t + 1) * TK, wave, lane);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (BL == 0) {
          b[j] = ld_b128(st + boff[s][j][0]);
        } else {
          const s16x4 lo = ds_tr16(st + boff[s][j][0]), hi = ds_tr16(st + boff[s][j][1]);
          b[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const bf16x8 a = ld_b128(st + aoff[s][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  gemm_bf16_epilogue<EPI>(p, acc, smem, m0, n0, wave, lane);
}

// ---- NT form, 4-phase K-step schedule ("8-phase" per two K-steps; cdna_hip_programming.md §5) --------
// Same tile, waves and fragments as above, but each 64-deep K-step runs as 4 phases, one per 64 x 32
// quadrant of every wave's 128 x 64 output (16 MFMAs each, at raised priority), and the LDS-DMA prefetch
// is cut into half-tiles of 128 rows x 64 k (16 KiB, 2 global_load_lds per thread) streamed one per
// phase, 3 in flight: the counted `s_waitcnt vmcnt(6)` at the last phase of K-step t retires exactly
// K-step t+1, so loads stay in flight across every barrier (never vmcnt(0) in the loop).
// The two wave rows run one barrier apart (ping-pong): while one issues its LDS reads and DMA, the other
// is in its MFMAs. Half-tile q of K-step u (h = 4u + q) lives in LDS slot h % 10 (10 x 16 KiB = all
// 160 KiB):
//   q 0: A rows of quadrant-row 0 (tile rows wm*128 + i, i < 64, for both wm; slot row wm*64 + i)
//   q 1: B rows of quadrant-col 0 (tile rows wn*64 + i, i < 32; slot row wn*32 + i)
//   q 2: B rows of quadrant-col 1 (tile rows wn*64 + 32 + i)
//   q 3: A rows of quadrant-row 1 (tile rows wm*128 + 64 + i)
// Phase p of K-step t reads (p0: q0 -> A regs, q1 -> B0 regs; p1: q2 -> B1 regs; p2: q3 -> A regs;
// p3: nothing), computes quadrant (0,0), (0,1), (1,1), (1,0), and issues half-tile h = 4t + p + 7.
// RAW: a half-tile is retired by every wave's vmcnt(6) before that wave's barrier of phase 4t+3, and
// read only after the next barrier. WAR: with 10 slots a slot is re-filled >= 3 phases after its last
// read, so the lagging wave row's reads (retired by its lgkmcnt(0) after the following barrier) are
// long done. Half-tiles past the last K-step re-read it into consumed slots (uniform vmcnt counting).
constexpr int HT = 16384, NSLOT = 10;

// DMA pieces (1 KiB per wave) of half-tile Q: 2, except the B half-tile of n-tiles 2.. when NJ == 3 (16 rows per wave)
template <int Q, int NJ>
constexpr int half_pieces() {
  return (Q == 2 && NJ == 3) ? 1 : 2;
}

template <int Q, int NJ = 4>
__device__ __forceinline__ void issue_half(const GP& p, unsigned char* smem, int h, int nk, int m0, int n0, int wave,
                                           int lane) {
  const int k0 = min(h >> 2, nk - 1) * TK;
  unsigned char* slot = smem + (h % NSLOT) * HT;
#pragma unroll
  for (int v = 0; v < half_pieces<Q, NJ>(); ++v) {
    const int qq = wave + 8 * v;         // 1-KiB DMA block of the slot
    const int lr = 8 * qq + (lane >> 3);  // slot row 0..127
    const int c = (lane & 7) ^ rk_swz(lr);
    if constexpr (Q == 0 || Q == 3) {
      const int tr = (lr >> 6) * 128 + (Q == 3 ? 64 : 0) + (lr & 63);
      glds16(p.A + (size_t)min(m0 + tr, p.M - 1) * p.lda + k0 + 8 * c, slot + 1024 * qq);
    } else {
      // wave wn's columns wn * 16 NJ ..: n-tiles 0, 1 in half-tile 1 (32 rows each), the rest in half-tile 2
      constexpr int R2 = 16 * (NJ - 2);  // rows per wave in half-tile 2
      const int tr = Q == 1 ? (lr >> 5) * 16 * NJ + (lr & 31) : (lr / R2) * 16 * NJ + 32 + (lr % R2);
      glds16(p.B + (size_t)min(n0 + tr, p.N - 1) * p.ldb + k0 + 8 * c, slot + 1024 * qq);
    }
  }
}

// NJ = 3 (256 x 192 tiles, wave tile 128 x 48): half-tile 2 carries one 16-row n-tile per wave (1 DMA piece instead of
// 2), quadrant-col 1 is that one n-tile, and the counted waits keep exactly the last three half-tiles in flight
// (2 + 2 + 1 pieces). It exists for wave quantization: at N = 768 the 256-wide tiles make 192 tiles of a 16384-row
// GEMM, 3/4 of the 256 CUs; 192-wide ones make 256.
template <int EPI, int NJ = 4, bool TR = false>
__global__ void __launch_bounds__(GT) gemm_bf16_nt4_kernel(GP p) {
  static_assert(NJ == 3 || NJ == 4, "n-tiles per wave");
  constexpr int BN = 64 * NJ, NJ1 = NJ - 2;  // tile width; n-tiles of quadrant-col 1
  constexpr int INFLIGHT = half_pieces<0, NJ>() + half_pieces<1, NJ>() + half_pieces<2, NJ>();
  __shared__ __attribute__((aligned(16))) unsigned char smem[NSLOT * HT];  // the epilogue reuses it
  const int nwg = p.tiles_m * p.tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = wg % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wg / 8;
  }
  int tm, tn;
  tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l16 = lane & 15;

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment byte offsets inside a slot: A (m-tile i of the quadrant, substep s), B (n-tile jj, substep s: boff in
  // half-tile 1, boff1 in half-tile 2)
  int aoff[4][2], boff[2][2], boff1[NJ1][2];
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
#pragma unroll
  for (int jj = 0; jj < NJ1; ++jj)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r = wn * 16 * NJ1 + 16 * jj + l16;
      boff1[jj][s2] = r * 128 + 16 * ((4 * s2 + g) ^ rk_swz(r));
    }

  const int nk = p.K / TK;
  issue_half<0, NJ>(p, smem, 0, nk, m0, n0, wave, lane);
  issue_half<1, NJ>(p, smem, 1, nk, m0, n0, wave, lane);
  issue_half<2, NJ>(p, smem, 2, nk, m0, n0, wave, lane);
  issue_half<3, NJ>(p, smem, 3, nk, m0, n0, wave, lane);
  issue_half<0, NJ>(p, smem, 4, nk, m0, n0, wave, lane);
  issue_half<1, NJ>(p, smem, 5, nk, m0, n0, wave, lane);
  issue_half<2, NJ>(p, smem, 6, nk, m0, n0, wave, lane);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");  // K-step 0's 4 half-tiles
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // wave row 1 runs one barrier behind row 0

  bf16x8 a[4][2], b0[2][2], b1[NJ1][2];
  auto mfma_quadrant = [&](int qm, const auto& bb, auto qn_c) {
    constexpr int QN = decltype(qn_c)::value;
    constexpr int NQ = QN == 0 ? 2 : NJ1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < NQ; ++jj)
          acc[4 * qm + i][2 * QN + jj] =
              TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[jj][s2], a[i][s2], acc[4 * qm + i][2 * QN + jj], 0, 0, 0)
                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], bb[jj][s2], acc[4 * qm + i][2 * QN + jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
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
    // phase 0: A quadrant-row 0 + B quadrant-col 0; quadrant (0, 0)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) b0[jj][s2] = ld_b128(s1 + boff[jj][s2]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s0 + aoff[i][s2]);
    issue_half<3, NJ>(p, smem, h, nk, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(0, b0, Q0{});
    sync_end();
    // phase 1: B quadrant-col 1; quadrant (0, 1)
#pragma unroll
    for (int jj = 0; jj < NJ1; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) b1[jj][s2] = ld_b128(s2p + boff1[jj][s2]);
    issue_half<0, NJ>(p, smem, h + 1, nk, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(0, b1, Q1{});
    sync_end();
    // phase 2: A quadrant-row 1; quadrant (1, 1)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s3 + aoff[i][s2]);
    issue_half<1, NJ>(p, smem, h + 2, nk, m0, n0, wave, lane);
    sync_mid();
    mfma_quadrant(1, b1, Q1{});
    sync_end();
    // phase 3: no reads; quadrant (1, 0); retire K-step t + 1
    issue_half<2, NJ>(p, smem, h + 3, nk, m0, n0, wave, lane);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
    sync_mid();
    mfma_quadrant(1, b0, Q0{});
    sync_end();
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // rejoin wave row 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-the-end half-tiles, before the epilogue reuses LDS
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  gemm_bf16_epilogue<EPI, 4, NJ, TR>(p, acc, smem, m0, n0, wave, lane);
}

// ---- NT form, persistent 4-phase loop (knob GEMM_BF16_PERSIST) ------------------------------------------------
// The nt4 kernel above takes all 160 KiB of LDS, so one workgroup runs per CU and each tile pays a launch, a prologue
// (the first K-step's DMA latency with nothing to compute) and an LDS epilogue behind two barriers. Here one
// workgroup per CU walks the tiles v = blockIdx.x, + G, + 2G, ... (G = min(tiles, CUs); blockIdx % 8 is the XCD, so the
// bijective remap above gives every XCD the same contiguous tile ranges as the one-tile-per-workgroup launch) and
// the half-tile stream runs on across tiles: the global K-step T = nk * k + t (k-th tile of this workgroup) picks
// the slots ((4T + q) % 10) exactly as in nt4, and the loop's past-the-end half-tiles of tile k (K-steps nk, nk + 1)
// are the first K-steps of tile k + 1, so its DMA lands under tile k's last phases. The epilogue cannot take 128 KiB
// of LDS (the ring is busy with tile k + 1): each wave stages its tile 32 rows at a time in a private 4 KiB of the
// two slots that are free at the tile boundary (see the epilogue), then stores 16-B row pieces through store_piece
// (same elementwise math, same bits). Storing the C^T accumulators' 8-B pieces straight from registers measured
// 10-25 % slower per GEMM (four 32-B row fragments per 128-B line). The epilogue has no workgroup barrier: the wave
// rows' one-barrier ping-pong carries on across tiles. The counted vmcnt waits stay
// correct with the epilogue's loads / stores in the count: they are older than the half-tiles a wait leaves in
// flight, so a wait only retires more. nk >= 2 (the next tile's reach is K-steps 0 and 1).
template <int Q, int NJ = 4>
__device__ __forceinline__ void issue_half_at(const GP& p, unsigned char* smem, int h, int ks, int m0, int n0,
                                              int wave, int lane) {
  const int k0 = ks * TK;
  unsigned char* slot = smem + (h % NSLOT) * HT;
#pragma unroll
  for (int v = 0; v < half_pieces<Q, NJ>(); ++v) {
    const int qq = wave + 8 * v;
    const int lr = 8 * qq + (lane >> 3);
    const int c = (lane & 7) ^ rk_swz(lr);
    if constexpr (Q == 0 || Q == 3) {
      const int tr = (lr >> 6) * 128 + (Q == 3 ? 64 : 0) + (lr & 63);
      glds16(p.A + (size_t)min(m0 + tr, p.M - 1) * p.lda + k0 + 8 * c, slot + 1024 * qq);
    } else {
      constexpr int R2 = 16 * (NJ - 2);
      const int tr = Q == 1 ? (lr >> 5) * 16 * NJ + (lr & 31) : (lr / R2) * 16 * NJ + 32 + (lr % R2);
      glds16(p.B + (size_t)min(n0 + tr, p.N - 1) * p.ldb + k0 + 8 * c, slot + 1024 * qq);
    }
  }
}

template <int EPI, int NJ = 4>
__global__ void __launch_bounds__(GT) gemm_bf16_nt4p_kernel(GP p) {
  static_assert(NJ == 3 || NJ == 4, "n-tiles per wave");
  constexpr int BN = 64 * NJ, NJ1 = NJ - 2;
  constexpr int INFLIGHT = half_pieces<0, NJ>() + half_pieces<1, NJ>() + half_pieces<2, NJ>();
  __shared__ __attribute__((aligned(16))) unsigned char smem[NSLOT * HT];
  const int ntiles = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  auto tile_at = [&](int v, int& m0, int& n0) {
    int wg = v;
    if (ntiles >= 16) {
      const int q = ntiles / 8, r = ntiles % 8, xcd = v % 8;
      wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + v / 8;
    }
    int tm, tn;
    tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
    m0 = tm * TM;
    n0 = tn * BN;
  };
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, l16 = lane & 15;

  int aoff[4][2], boff[2][2], boff1[NJ1][2];
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
#pragma unroll
  for (int jj = 0; jj < NJ1; ++jj)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r = wn * 16 * NJ1 + 16 * jj + l16;
      boff1[jj][s2] = r * 128 + 16 * ((4 * s2 + g) ^ rk_swz(r));
    }

  const int nk = p.K / TK;  // >= 2 (host)
  int v = blockIdx.x;
  int m0, n0, nm0, nn0;
  tile_at(v, m0, n0);
  bool has_next = v + G < ntiles;
  if (has_next) tile_at(v + G, nm0, nn0);
  int kbase = 0;  // global K-step of this tile's K-step 0
  // half-tile H (global): this tile's K-step, the next tile's first ones, or (last tile) a re-read of the last K-step
  auto issue = [&](auto qc, int H) {
    constexpr int Q = decltype(qc)::value;
    const int lt = (H >> 2) - kbase;
    if (lt < nk) issue_half_at<Q, NJ>(p, smem, H, lt, m0, n0, wave, lane);
    else if (has_next) issue_half_at<Q, NJ>(p, smem, H, lt - nk, nm0, nn0, wave, lane);
    else issue_half_at<Q, NJ>(p, smem, H, nk - 1, m0, n0, wave, lane);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  issue(I0{}, 0);
  issue(I1{}, 1);
  issue(I2{}, 2);
  issue(I3{}, 3);
  issue(I0{}, 4);
  issue(I1{}, 5);
  issue(I2{}, 6);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) __builtin_amdgcn_s_barrier();  // wave row 1 runs one barrier behind row 0, across all tiles

  f32x4 acc[8][NJ];
  bf16x8 a[4][2], b0[2][2], b1[NJ1][2];
  auto mfma_quadrant = [&](int qm, const auto& bb, auto qn_c) {
    constexpr int QN = decltype(qn_c)::value;
    constexpr int NQ = QN == 0 ? 2 : NJ1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < NQ; ++jj)
          acc[4 * qm + i][2 * QN + jj] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[jj][s2], a[i][s2], acc[4 * qm + i][2 * QN + jj], 0, 0, 0);
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
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K-steps t < nk - 2 fetch within this tile (no tile test per issue); the last two run on into the next tile
    auto kstep = [&](int t, auto tail_c) {
      constexpr bool TAIL = decltype(tail_c)::value;
      const int T = kbase + t;
      const int h = 4 * T + 7;
      auto iss = [&](auto qc, int H) {
        constexpr int Q = decltype(qc)::value;
        if constexpr (TAIL) issue(qc, H);
        else issue_half_at<Q, NJ>(p, smem, H, (H >> 2) - kbase, m0, n0, wave, lane);
      };
      const unsigned char* s0 = smem + ((4 * T) % NSLOT) * HT;
      const unsigned char* s1 = smem + ((4 * T + 1) % NSLOT) * HT;
      const unsigned char* s2p = smem + ((4 * T + 2) % NSLOT) * HT;
      const unsigned char* s3 = smem + ((4 * T + 3) % NSLOT) * HT;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) b0[jj][s2] = ld_b128(s1 + boff[jj][s2]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s0 + aoff[i][s2]);
      iss(I3{}, h);
      sync_mid();
      mfma_quadrant(0, b0, I0{});
      sync_end();
#pragma unroll
      for (int jj = 0; jj < NJ1; ++jj)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) b1[jj][s2] = ld_b128(s2p + boff1[jj][s2]);
      iss(I0{}, h + 1);
      sync_mid();
      mfma_quadrant(0, b1, I1{});
      sync_end();
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = ld_b128(s3 + aoff[i][s2]);
      iss(I1{}, h + 2);
      sync_mid();
      mfma_quadrant(1, b1, I1{});
      sync_end();
      iss(I2{}, h + 3);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
      sync_mid();
      mfma_quadrant(1, b0, I0{});
      sync_end();
    };
    using BF = std::integral_constant<bool, false>;
    using BT = std::integral_constant<bool, true>;
    for (int t = 0; t < nk - 2; ++t) kstep(t, BF{});
    kstep(nk - 2, BT{});
    kstep(nk - 1, BT{});
    // epilogue through a wave-private 4 KiB of the ring, 32 rows per pass (16-B row pieces as in nt4). Free slots: the
    // last K-step's q2 and q3 ((4T + 2) % 10, (4T + 3) % 10, T = kbase + nk - 1): no DMA in flight targets them, every
    // wave's reads of them retired before the barrier that ends row 0's last phase, and the next tile refills them
    // only after barriers that wave row 1 reaches past its own epilogue (row 1 runs one barrier behind row 0)
    {
      const int T = kbase + nk - 1;
      unsigned char* E = smem + ((4 * T + 2 + (wave >> 2)) % NSLOT) * HT + (wave & 3) * 4096;
      float bj[NJ][4] = {};
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) bj[j][r] = bf2f(p.bias[min(n0 + wn * 16 * NJ + 16 * j + 4 * g + r, p.N - 1)]);
      }
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int row = 16 * ii + l16, col = 16 * j + 4 * g;
            typedef u16 u16x4 __attribute__((ext_vector_type(4)));
            u16x4 pv;
#pragma unroll
            for (int r = 0; r < 4; ++r) pv[r] = f2bf(acc[2 * pass + ii][j][r] + bj[j][r]);
            *reinterpret_cast<u16x4*>(E + row * 128 + 16 * ((col >> 3) ^ rk_swz(row)) + 2 * (col & 7)) = pv;
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int row = 8 * it + (lane >> 3), ch = lane & 7;
          const u16x8 pv = *reinterpret_cast<const u16x8*>(E + row * 128 + 16 * (ch ^ rk_swz(row)));
          const int grow = m0 + wm * 128 + 32 * pass + row, gcol = n0 + wn * 16 * NJ + 8 * ch;
          if (ch >= 2 * NJ || grow >= p.M || gcol >= p.N || p.nostore) continue;
          store_piece<EPI>(p, pv, grow, gcol);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this pass's reads done before the next pass rewrites E
        __builtin_amdgcn_wave_barrier();
      }
    }
    v += G;
    if (v >= ntiles) break;
    kbase += nk;
    m0 = nm0;
    n0 = nn0;
    has_next = v + G < ntiles;
    if (has_next) tile_at(v + G, nm0, nn0);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // rejoin wave row 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last tile's past-the-end re-reads land before exit
}

// ---- NT form, 4 waves x 128 x 128 (one wave per SIMD) --------------------------------------------------------
// 256 x 256 tile per 256-thread workgroup, waves 2 (M) x 2 (N), each wave a 128 x 128 output = 4 x 4
// v_mfma_f32_32x32x16_bf16 accumulators (256 registers: one wave per SIMD, up to 512). The 8-wave kernels above
// synchronise every phase (8 barriers per K-step, the two wave rows ping-ponging); here one barrier per 64-deep K-step
// separates 64 MFMAs per wave (2048 cycles). Fragments: A rows and B rows (both k-contiguous) by ds_read_b128 from
// [rows][64 k] images (the rk_swz chunk swizzle), double-buffered in registers one 16-deep substep ahead. Operands
// arrive by LDS-DMA (inline-asm buffer_load ... lds, so the compiler counts only the fragment reads) into two 64 KiB
// stages: K-step t + 1's 16 pieces per wave are issued 8 before each of K-step t's first two substeps' MFMAs and
// retired by one vmcnt(0) before the K-step's barrier. The MFMA takes the B fragment as its first operand, so each lane accumulates
// 4 consecutive output columns of one row (C^T layout): the epilogue writes 8-byte pieces into a [256][264] bf16 image,
// then every thread stores 16-B row pieces through store_piece (all epilogues).
constexpr int W4_GT = 256, W4_STAGE = 2 * A_BYTES, W4_LP = TN + 8;  // 64 KiB per stage; epilogue image pitch (bf16)
constexpr int W4_SMEM = TM * W4_LP * 2 > 2 * W4_STAGE ? TM * W4_LP * 2 : 2 * W4_STAGE;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int EPI>
__global__ void __launch_bounds__(W4_GT, 1) gemm_bf16_w4_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[W4_SMEM];
  const int nwg = p.tiles_m * p.tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = wg % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wg / 8;
  }
  int tm, tn;
  tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int lane = threadIdx.x & 63, r32 = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // DMA pieces of one stage: 64 x 1 KiB, A rows 8q .. 8q + 7 (q < 32) then B rows; wave w issues q = w + 4u
  const dma_i32x4 ra = dma_rsrc4(p.A, (unsigned)((size_t)p.M * p.lda * 2));
  const dma_i32x4 rb = dma_rsrc4(p.B, (unsigned)((size_t)p.N * p.ldb * 2));
  unsigned voff[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int q = wave + 4 * u, lr = 8 * (q & 31) + (lane >> 3);
    const int c = (lane & 7) ^ rk_swz(lr);
    voff[u] = u < 8 ? (unsigned)(((size_t)min(m0 + lr, p.M - 1) * p.lda + 8 * c) * 2)
                    : (unsigned)(((size_t)min(n0 + lr, p.N - 1) * p.ldb + 8 * c) * 2);
  }
  auto issue4 = [&](int kt, unsigned char* stage, int u0) {  // pieces u0 .. u0 + 3 of K-step kt
#pragma unroll
    for (int u = u0; u < u0 + 4; ++u)
      bdma16_asm(u < 8 ? ra : rb, voff[u], (unsigned)kt * TK * 2, stage + 1024 * (wave + 4 * u));
  };
  // fragment byte offsets (stage-relative): row base + the lane's swizzled chunk of substep s; tile i / j at +4096 i
  const int xr = (r32 >> 1) & 7;  // rk_swz of every fragment row (rows 32 i + r32 + multiples of 32)
  const int abase = (wm * 128 + r32) * 128, bbase = A_BYTES + (wn * 128 + r32) * 128;
  int xo[4];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) xo[s2] = 16 * ((2 * s2 + h) ^ xr);

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nk = p.K / TK;
  issue4(0, smem, 0);
  issue4(0, smem, 4);
  issue4(0, smem, 8);
  issue4(0, smem, 12);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 fa[2][4], fb[2][4];
  for (int t = 0; t < nk; ++t) {
    const unsigned char* st = smem + (t & 1) * W4_STAGE;
    unsigned char* nx = smem + ((t + 1) & 1) * W4_STAGE;
    const bool more = t + 1 < nk;
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[0][i] = ld_b128(st + abase + 4096 * i + xo[0]);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[0][j] = ld_b128(st + bbase + 4096 * j + xo[0]);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int cb = s2 & 1;
      if (s2 < 3) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[cb ^ 1][i] = ld_b128(st + abase + 4096 * i + xo[s2 + 1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[cb ^ 1][j] = ld_b128(st + bbase + 4096 * j + xo[s2 + 1]);
      }
      if (more && s2 < 2) {  // the next K-step's DMA early: 8 pieces before substep 0's MFMAs, 8 before substep 1's
        issue4(t + 1, nx, 8 * s2);
        issue4(t + 1, nx, 8 * s2 + 4);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma32(fb[cb][j], fa[cb][i], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // epilogue: acc[i][j] (C^T layout: lane = output row m = wm*128 + 32 i + r32; register e -> column
  // n = wn*128 + 32 j + (e & 3) + 8 (e >> 2) + 4 h) -> bf16(acc (+ bias)) image [256][W4_LP], 8 B per 4 registers
  u16* img = reinterpret_cast<u16*>(smem);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = wn * 128 + 32 * j + 8 * g + 4 * h;
      float bj[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bj[e] = bf2f(p.bias[min(n0 + col + e, p.N - 1)]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        typedef u16 u16x4 __attribute__((ext_vector_type(4)));
        u16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(acc[i][j][4 * g + e] + bj[e]);
        *reinterpret_cast<u16x4*>(img + (wm * 128 + 32 * i + r32) * W4_LP + col) = v;
      }
    }
  __syncthreads();
#pragma unroll 4
  for (int it = 0; it < 32; ++it) {
    const int row = 8 * it + (threadIdx.x >> 5), ch = threadIdx.x & 31;
    const int grow = m0 + row, gcol = n0 + 8 * ch;
    if (grow >= p.M || gcol >= p.N || p.nostore) continue;  // (N % 8 == 0: a piece is all in or out)
    store_piece<EPI>(p, *reinterpret_cast<const u16x8*>(img + row * W4_LP + 8 * ch), grow, gcol);
  }
}

// ---- NT form, 256 x 128 tiles of 4 waves, two workgroups per CU ---------------------------------------
// The 256 x 256 kernels above take all 160 KiB of LDS, so one workgroup runs per CU and every CU reaches its
// epilogue (the bf16 stores of its tile) at the same moment, with no main loop left to hide them under
// (docs/TUNING_NOTES.md: the stores were never overlapped). Here a workgroup is 4 waves (2 x 2, each 128 x 64, the
// same 8 x 4 accumulators) on a 256 x 128 tile, 32-deep K-steps in a 3-stage ring of 24 KiB (72 KiB in all, the
// epilogue's 64 KiB of row images fit in it), and __launch_bounds__(256, 2) keeps it at <= 256 VGPRs: two
// workgroups share each CU, so one's epilogue / prologue runs beside the other's main loop.
// LDS images [rows][32 k] (64-B rows): 16-B chunk c of row r at c ^ ((r >> 2) & 3), so the 16 rows of a
// ds_read_b128 lane group hit 16 distinct 4-bank slots. Operands arrive by buffer-form LDS-DMA (lds_dma.h):
// 6 x 1 KiB per wave per stage, one counted vmcnt(6) + one barrier per K-step, past-the-end K-steps re-read the
// last one into the free stage (uniform counts).
constexpr int T2_TM = 256, T2_TN = 128, T2_TK = 32, T2_GT = 256, T2_NST = 3;
constexpr int T2_A = T2_TM * T2_TK * 2, T2_B = T2_TN * T2_TK * 2, T2_STAGE = T2_A + T2_B;  // 16 + 8 KiB
static_assert(T2_NST * T2_STAGE >= 4 * 128 * 128, "the epilogue's 4 wave images (16 KiB each) fit the ring");

__device__ __forceinline__ int t2_swz(int r) { return (r >> 2) & 3; }

__device__ __forceinline__ void t2_issue(const GP& p, const __amdgpu_buffer_rsrc_t& ra, const __amdgpu_buffer_rsrc_t& rb,
                                         unsigned char* st, int m0, int n0, int k0, int wave, int lane) {
  // A: 16 instructions of 16 rows x 64 B (wave w: w, w + 4, w + 8, w + 12); B: 8 (w, w + 4)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = wave + 4 * u;
    const int r = 16 * q + (lane >> 2);
    const int c = (lane & 3) ^ t2_swz(r);
    const int gr = min(m0 + r, p.M - 1);
    bdma16(ra, (unsigned)(2 * ((size_t)gr * p.lda + k0 + 8 * c)), st + 1024 * q);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = wave + 4 * u;
    const int r = 16 * q + (lane >> 2);
    const int c = (lane & 3) ^ t2_swz(r);
    const int gr = min(n0 + r, p.N - 1);
    bdma16(rb, (unsigned)(2 * ((size_t)gr * p.ldb + k0 + 8 * c)), st + T2_A + 1024 * q);
  }
}

template <int EPI>
__global__ void __launch_bounds__(T2_GT, 2) gemm_bf16_t2_kernel(GP p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[T2_NST * T2_STAGE];
  const int nwg = p.tiles_m * p.tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 16) {  // XCD-aware bijective remap (as the kernels above)
    const int q = nwg / 8, r = nwg % 8, xcd = wg % 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + wg / 8;
  }
  int tm, tn;
  tile_of(wg, p.tiles_m, p.tiles_n, p.group_m, tm, tn);
  const int m0 = tm * T2_TM, n0 = tn * T2_TN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, l16 = lane & 15;
  // gemm_bf16_supported keeps every operand < 2^31 bytes
  const __amdgpu_buffer_rsrc_t ra = dma_rsrc(p.A, (unsigned)((size_t)(p.M - 1) * p.lda * 2 + (size_t)p.K * 2));
  const __amdgpu_buffer_rsrc_t rb = dma_rsrc(p.B, (unsigned)((size_t)(p.N - 1) * p.ldb * 2 + (size_t)p.K * 2));

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int aoff[8], boff[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = wm * 128 + 16 * i + l16;
    aoff[i] = r * 64 + 16 * (g ^ t2_swz(r));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = wn * 64 + 16 * j + l16;
    boff[j] = T2_A + r * 64 + 16 * (g ^ t2_swz(r));
  }

  const int nk = p.K / T2_TK;
  t2_issue(p, ra, rb, smem, m0, n0, 0, wave, lane);
  t2_issue(p, ra, rb, smem + T2_STAGE, m0, n0, min(1, nk - 1) * T2_TK, wave, lane);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // stage t landed (only stage t + 1's 6 DMAs younger)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of stage t - 1 done before its refill
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    t2_issue(p, ra, rb, smem + ((t + 2) % T2_NST) * T2_STAGE, m0, n0, min(t + 2, nk - 1) * T2_TK, wave, lane);
    const unsigned char* st = smem + (t % T2_NST) * T2_STAGE;
    bf16x8 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = ld_b128(st + boff[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bf16x8 a = ld_b128(st + aoff[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-the-end stages, before the epilogue reuses LDS
  __syncthreads();
  gemm_bf16_epilogue<EPI, 2>(p, acc, smem, m0, n0, wave, lane);
}

}  // namespace

// 256 x 192 tiles instead of 256 x 256 when they fill the CUs' rounds better (wave quantization): time ~ rounds x tile
// width, rounds = ceil(tiles / CUs). Knob GEMM_BF16_N192: -1 auto (default), 0 never, 1 always (A/B).
static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t pr;
    cus = hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0 ? pr.multiProcessorCount : 256;
  }
  return cus;
}
static bool nt4_use_192(int tiles_m, int N) {
  const int k = knob(KNOB_GEMM_BF16_N192);
  if (k >= 0) return k == 1;
  const int64_t cus = device_cus();
  const int64_t r256 = ((int64_t)tiles_m * ((N + 255) / 256) + cus - 1) / cus;
  const int64_t r192 = ((int64_t)tiles_m * ((N + 191) / 192) + cus - 1) / cus;
  return r192 * 192 * 100 < r256 * 256 * 97;  // a clear (>3 %) win only: the 192-wide loop is less efficient per flop
}

bool gemm_bf16_supported(int M, int N, int K, int lda, int ldb, int ldc, bool b_kn) {
  // K whole K-steps; 16-B aligned rows for the DMA and the row-piece stores
  return M >= 1 && N >= 8 && K >= TK && K % TK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 8 == 0 && (b_kn ? ldb >= N : ldb >= K) && lda >= K && ldc >= N &&
         (int64_t)M * lda * 2 < (int64_t(1) << 31) && (int64_t)(b_kn ? K : N) * ldb * 2 < (int64_t(1) << 31);
}

void gemm_bf16(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool b_kn,
               int epi, const void* bias, void* aux, int ldaux, hipStream_t stream) {
  GP p;
  p.A = static_cast<const u16*>(A);
  p.B = static_cast<const u16*>(B);
  p.C = static_cast<u16*>(C);
  p.bias = static_cast<const u16*>(bias);
  p.aux = static_cast<u16*>(aux);
  p.gsave = epi == EPI_BIAS_GELU_SAVE_GRAD || epi == EPI_MUL_GRAD;
  if (epi == EPI_BIAS_GELU_SAVE_GRAD) epi = EPI_BIAS_GELU;
  if (epi == EPI_MUL_GRAD) epi = EPI_DGELU;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.ldaux = ldaux;
  p.tiles_m = (M + TM - 1) / TM;
  p.tiles_n = (N + TN - 1) / TN;
  p.nostore = knob(KNOB_GEMM_BF16_NOSTORE) == 1;  // timing probe: pinned to 0 in production builds
  p.ntstore = knob(KNOB_GEMM_NT_STORE) == 1;
  p.group_m = std::max(0, knob(KNOB_GEMM_GROUP_M));
  const dim3 grid(p.tiles_m * p.tiles_n);
#define GB_LAUNCH(BLV, E) hipLaunchKernelGGL((gemm_bf16_kernel<BLV, E>), grid, dim3(GT), 0, stream, p)
#define GB_EPI(BLV)                                       \
  do {                                                    \
    switch (epi) {                                        \
      case EPI_BIAS: GB_LAUNCH(BLV, EPI_BIAS); break;      \
      case EPI_BIAS_GELU: GB_LAUNCH(BLV, EPI_BIAS_GELU); break; \
      case EPI_DGELU: GB_LAUNCH(BLV, EPI_DGELU); break;    \
      default: GB_LAUNCH(BLV, EPI_STORE); break;           \
    }                                                     \
  } while (0)
  const bool nt4 = knob(KNOB_GEMM_BF16_2PHASE) == 0;  // 1: the one-barrier-per-K-step loop (A/B)
  if (!b_kn && knob(KNOB_GEMM_BF16_T2) == 1) {  // 256 x 128 tiles, two workgroups per CU
    p.tiles_m = (M + T2_TM - 1) / T2_TM;
    p.tiles_n = (N + T2_TN - 1) / T2_TN;
    const dim3 g2(p.tiles_m * p.tiles_n);
    switch (epi) {
      case EPI_BIAS: hipLaunchKernelGGL((gemm_bf16_t2_kernel<EPI_BIAS>), g2, dim3(T2_GT), 0, stream, p); break;
      case EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_bf16_t2_kernel<EPI_BIAS_GELU>), g2, dim3(T2_GT), 0, stream, p); break;
      case EPI_DGELU: hipLaunchKernelGGL((gemm_bf16_t2_kernel<EPI_DGELU>), g2, dim3(T2_GT), 0, stream, p); break;
      default: hipLaunchKernelGGL((gemm_bf16_t2_kernel<EPI_STORE>), g2, dim3(T2_GT), 0, stream, p); break;
    }
    return;
  }
  if (b_kn) {
    GB_EPI(1);
  } else if (knob(KNOB_GEMM_BF16_W4) == 1) {  // 4 waves x 128 x 128, one barrier per K-step
    switch (epi) {
      case EPI_BIAS: hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI_BIAS>), grid, dim3(W4_GT), 0, stream, p); break;
      case EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI_BIAS_GELU>), grid, dim3(W4_GT), 0, stream, p); break;
      case EPI_DGELU: hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI_DGELU>), grid, dim3(W4_GT), 0, stream, p); break;
      default: hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI_STORE>), grid, dim3(W4_GT), 0, stream, p); break;
    }
  } else if (nt4) {
    const bool n192 = nt4_use_192(p.tiles_m, N);
    if (n192) p.tiles_n = (N + 191) / 192;
    const dim3 g4(p.tiles_m * p.tiles_n);
    const bool tr = knob(KNOB_GEMM_BF16_TR) != 0;
    // persistent workgroups (knob GEMM_BF16_PERSIST: -1 auto, 0, 1). Auto: where they measured faster at the GPT-2
    // shapes (tools/probes/gemm_persist_ab.py, profiles/r6_gemm_persistent_ab.jsonl): many tiles per CU (the lm_head
    // forward, 49 per CU: 1320 -> 1235 us) or a very long K (its input gradient, 786 K-steps: 1065 -> 1034 us); at 1-3
    // tiles per CU it is level or slower, and the gelu'-multiply epilogue's aux reads stall it (92 -> 108 us)
    const int pk = knob(KNOB_GEMM_BF16_PERSIST);
    const bool persist = pk >= 0 ? pk == 1
                                 : (epi != EPI_DGELU && ((int64_t)p.tiles_m * p.tiles_n >= 8 * (int64_t)device_cus() ||
                                                         K / TK >= 256));
    if (tr && K / TK >= 2 && persist) {
      const dim3 gp((unsigned)std::min<int64_t>((int64_t)p.tiles_m * p.tiles_n, device_cus()));
#define NT4P_LAUNCH(E)                                                                             \
  do {                                                                                             \
    if (n192) hipLaunchKernelGGL((gemm_bf16_nt4p_kernel<E, 3>), gp, dim3(GT), 0, stream, p);        \
    else hipLaunchKernelGGL((gemm_bf16_nt4p_kernel<E, 4>), gp, dim3(GT), 0, stream, p);             \
  } while (0)
      switch (epi) {
        case EPI_BIAS: NT4P_LAUNCH(EPI_BIAS); break;
        case EPI_BIAS_GELU: NT4P_LAUNCH(EPI_BIAS_GELU); break;
        case EPI_DGELU: NT4P_LAUNCH(EPI_DGELU); break;
        default: NT4P_LAUNCH(EPI_STORE); break;
      }
#undef NT4P_LAUNCH
      return;
    }
#define NT4_LAUNCH(E)                                                                                  \
  do {                                                                                                 \
    if (n192 && tr) hipLaunchKernelGGL((gemm_bf16_nt4_kernel<E, 3, true>), g4, dim3(GT), 0, stream, p); \
    else if (n192) hipLaunchKernelGGL((gemm_bf16_nt4_kernel<E, 3>), g4, dim3(GT), 0, stream, p);       \
    else if (tr) hipLaunchKernelGGL((gemm_bf16_nt4_kernel<E, 4, true>), g4, dim3(GT), 0, stream, p);   \
    else hipLaunchKernelGGL((gemm_bf16_nt4_kernel<E, 4>), g4, dim3(GT), 0, stream, p);                 \
  } while (0)
    switch (epi) {
      case EPI_BIAS: NT4_LAUNCH(EPI_BIAS); break;
      case EPI_BIAS_GELU: NT4_LAUNCH(EPI_BIAS_GELU); break;
      case EPI_DGELU: NT4_LAUNCH(EPI_DGELU); break;
      default: NT4_LAUNCH(EPI_STORE); break;
    }
#undef NT4_LAUNCH
  } else {
    GB_EPI(0);
  }
#undef GB_EPI
#undef GB_LAUNCH
}

}  // namespace sdml
