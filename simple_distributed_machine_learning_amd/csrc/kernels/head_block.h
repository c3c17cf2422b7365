// The 784-128-10 MLP's classifier head on a 256-row block of h, on fp16 MFMAs (16x16x32), shared by
// mlp_u8.hip's fused uint8 forward + head (h straight from the forward's accumulators) and head_xent.hip's
// standalone block head (h read from HBM): both feed the same function the same registers, so their logits,
// dl and dW2 are the same operations in the same order (the fused kernel's dl is bit-identical to the
// standalone head's on the same rows).
//
// Reference ops: /root/reference/simple_distributed.py:77-79 (fc2, log_softmax), :111 (nll_loss).
//
// Numerics (fp32-accurate, as the first layer's GEMMs): every fp32 operand is two fp16 planes of v * 2^s,
// hi = fp16(v 2^s), lo = fp16(v 2^s - hi) (u8_planes.h's split: each element to within one fp32 ulp above
// 2^(E-15) when |v| < 2^E, an absolute error below 2^(E-39) under it), and a product is the three exact fp16
// MFMA products hi*lo + lo*hi + hi*hi accumulated in fp32 (lo*lo <= 2^-22 |ab| is dropped). Plane scales, all
// exact powers of two: h by 2^(14 - E) from the block's max |h| (one LDS exchange), W2 by its max |W2| (every
// wave computes the same value from registers), dl by the a-priori bound |dl| <= loss_scale
// (|softmax - onehot| <= 1). The round-4 head ran the same math on fp32 MFMAs (v_mfma_f32_16x16x4_f32, 16x
// slower per product) and cost ~12K of the fused forward's ~27K-cycle epilogue per block.
//
// Block = 8 waves, wave w = (wm = w % 4, wn = w / 4) holding h[64 wm + ..][64 wn + ..] in the 32x32 MFMA C
// layout: y[i][j][r] = h[64 wm + 32 i + 8 (r >> 2) + 4 (lane >> 5) + (r & 3)][64 wn + 32 j + (lane & 31)].
//  1. h planes into an LDS image [plane][hid][row] of 8-byte granules (4 rows of one hidden unit): the C
//     layout gives a lane exactly one granule per register quad, so the image is written with 32
//     ds_write_b64 per lane (round 4: 64 ds_write_b32 of fp32). Granule q of hidden unit h sits at q ^ gswz(h):
//     the writes (16 lanes = 16 hidden units), the logits' transposed reads and the dW2 reads are all
//     bank-conflict-free (checked by enumeration in tests/test_head_block_layout.py).
//  2. logits^T = W2 h^T, 16 classes x 16 rows per 16x16x32 MFMA: A = W2 planes (lane: class), B = the h image
//     read transposed (ds_read_b64_tr_b16: lane = row, 8 consecutive hidden units), 4 k-steps x 3 products;
//     wave w runs the row tiles w and w + 8. The accumulator leaves lane (r, g) with row r's logits of classes
//     4g .. 4g+3, the layout head_tile.h's softmax_dz works on.
//  3. dW2 = dl^T h over the block's 256 rows, 16 hidden units per wave (no cross-wave reduction): A = dl^T
//     planes from a small LDS image (lane: class), B = the h image (lane: hidden unit, 8 consecutive rows).
#pragma once

#include <hip/hip_runtime.h>

#include "head_tile.h"
#include "lds_dma.h"

namespace sdml {
namespace hblk {

typedef float hb_f32x16 __attribute__((ext_vector_type(16)));
typedef float hb_f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 hb_f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 hb_f16x4 __attribute__((ext_vector_type(4)));
typedef short hb_s16x4 __attribute__((ext_vector_type(4)));
typedef float hb_f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 hb_f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned hb_u32x2 __attribute__((ext_vector_type(2)));

constexpr int ROWS = 256, HID = 128, NW = 8, NT = 512;
constexpr int PLANE_B = HID * ROWS * 2;              // bytes per h plane (fp16)
constexpr int DLT_OFF = 2 * PLANE_B;                  // dl planes [2][ROWS][16 classes] fp16 (dl_off)
constexpr int DLT_PLANE_B = 16 * ROWS * 2;
constexpr int RED_OFF = DLT_OFF + 2 * DLT_PLANE_B;    // floats below
// red: [0, 8) wave max |h|, [8, 136) db partials [wave][16], [136, 144) loss, [144, 152) correct, [152, 160) amx,
// [160, 168) wave max |W2|
constexpr int RED_FLOATS = 168;
// W2's fp16 planes, split once per block: [plane][16 classes][W2PP] bytes, rows padded to 288 B so the A-operand
// reads (ds_read_b128 in its 4 lane groups) are conflict-free (tests/test_head_block_layout.py); classes >= C are
// zero rows
constexpr int W2PP = HID * 2 + 32;
constexpr int W2PL = 16 * W2PP;
constexpr int W2_OFF = RED_OFF + RED_FLOATS * 4;
constexpr int LDS_BYTES = W2_OFF + 2 * W2PL;
static_assert(W2_OFF % 16 == 0 && W2PP % 16 == 0, "W2 plane alignment");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

// granule swizzle of hidden unit (or class) h: bits (h2, h3, h0, h1, h3) -> bits 0..4
__device__ __forceinline__ int gswz(int h) {
  return ((h >> 2) & 1) | (((h >> 3) & 1) << 1) | ((h & 1) << 2) | (((h >> 1) & 1) << 3) | (((h >> 3) & 1) << 4);
}
// byte offset of granule q (rows 4q .. 4q+3) of hidden unit h in plane p of the h image: the two planes of a hidden
// unit are adjacent 512-B rows (HPL apart: an immediate offset for the second plane's access; 65536 is not), which
// leaves every access's banks as they were (both offsets are multiples of 256 B)
constexpr int HPL = ROWS * 2;
__device__ __forceinline__ int hoff(int p, int h, int q) { return h * (2 * HPL) + p * HPL + 8 * (q ^ gswz(h)); }
// hoff(0, h, qb) for a granule index qb whose bits 1..3 are zero: hoff(0, h, qb | c) == hid_base(h, qb) ^ 8 c for
// c in [0, 16) with bit 0 clear (tests/test_head_block_layout.py)
__device__ __forceinline__ int hid_base(int h, int qb) { return h * (2 * HPL) + 8 * (qb ^ gswz(h)); }
// byte offset of classes 4s .. 4s+3 of row R in plane p of the dl image: rows of 16 classes (32 B), row R at physical
// row R ^ (bit 3 of R) << 2 and its 8-byte class slots swizzled by that row's bits 2..3, so the 8-byte writes (lane:
// one row's 4 classes) and the dW2 A-operand reads (ds_read_b64_tr_b16: a 16-lane group takes 4 rows x 4 slots and
// hands lane r class r of the 4 rows) are conflict-free (tests/test_head_block_layout.py). Round 4's dl^T image
// [class][row] took 8 ds_write_b16 per lane and row tile.
__device__ __forceinline__ int dl_off(int p, int R, int s) {
  const int P = R ^ (((R >> 3) & 1) << 2);
  return DLT_OFF + p * DLT_PLANE_B + P * 32 + 8 * (s ^ ((P >> 2) & 3));
}

// exponent E with |v| < 2^E for finite v >= 0, clamped so 2^(14 - E) and 2^(E - 14) stay normal floats
__device__ __forceinline__ int bexp(float v) {
  const unsigned b = __float_as_uint(v);
  const int e = (int)((b >> 23) & 0xffu) - 126;
  return (b & 0x7fffffffu) == 0u ? -100 : min(max(e, -100), 120);
}
__device__ __forceinline__ float p2(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }

// two fp16 planes of x (already scaled): hi = fp16(x), lo = fp16(x - hi)
__device__ __forceinline__ void split2(float x, _Float16& hi, _Float16& lo) {
  hi = static_cast<_Float16>(x);
  lo = static_cast<_Float16>(x - static_cast<float>(hi));
}
// the lo planes of a pair: fp16(x - hi) as fma(hi, -1, x) rounded once (x - hi is exact in fp32: the same bits as
// split2). Written out because hipcc turns the scalar form back into conversions and a packed fma (6 instead of 4
// instructions per pair with the hi plane's v_pk_mul_f32 + v_cvt_pk_f16_f32)
__device__ __forceinline__ hb_f16x2 lo_pair(hb_f16x2 h, hb_f32x2 x) {
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo)
      : "v"(__builtin_bit_cast(unsigned, h)), "v"(x[0]), "v"(x[1]));
  return __builtin_bit_cast(hb_f16x2, lo);
}
__device__ __forceinline__ hb_f32x4 mfma16(hb_f16x8 a, hb_f16x8 b, hb_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ hb_s16x4 tr16(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) hb_s16x4*)(p));
}
__device__ __forceinline__ hb_f16x8 cat8(hb_s16x4 a, hb_s16x4 b) {
  return __builtin_bit_cast(hb_f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct Args {
  const float* w2;             // [C][HID]
  const float* b2;             // [C]
  const int64_t* target;       // [M]
  float loss_scale;
  bool train;
  float* dl;                   // optional [M][C]
  float* part;                 // this block's slab row [C * HID + C + 2] (train: dW2, db2; always loss, correct)
  float* bound;                // optional: this block's 2 max_row sum_c |dl_c| * max |W2|
};

// The block's global operands of the head, as loaded (clamped addresses; the masks for classes >= C are applied in
// block_head): one float4 of W2 per thread (flat index tid: the block stages W2 in LDS once - each wave loading all of
// W2 in its A-operand layout cost 8 waves x 8 KB of vector-memory traffic per block, ~2K cycles per round by the
// stamps), the biases of classes 4g .. 4g+3 and the targets of the lane's two row tiles. The fused forward loads them
// inside its K loop (their latency hides there; no value is used before the epilogue - a select on them in the
// prologue made hipcc wait for the loads before the first DMA); the standalone head right before block_head.
struct Operands {
  hb_f32x4 w2c;
  headtile::f32x4m b;
  int tg[2];
};
template <int C>
__device__ __forceinline__ void load_operands(const Args& a, int m0, int M, int wave, int lane, Operands& o) {
  const int r = lane & 15, g = lane >> 4;
  o.w2c = reinterpret_cast<const hb_f32x4*>(a.w2)[min(wave * 64 + lane, C * HID / 4 - 1)];
#pragma unroll
  for (int v = 0; v < 4; ++v) o.b[v] = a.b2[min(4 * g + v, C - 1)];
#pragma unroll
  for (int it = 0; it < 2; ++it)  // the low word of the int64 class index (a dwordx2 load whose dead high half hipcc
                                  // reused as a register made it wait for the load right away)
    o.tg[it] = reinterpret_cast<const int*>(a.target)[2 * (size_t)min(m0 + 16 * (wave + NW * it) + r, M - 1)];
}

// prep(y) fills y: this wave's 64 x 64 tile of h (rows >= M zero), C layout above. smem: LDS_BYTES, free (the caller's
// previous use finished with a barrier or not yet started: the first thing here is a barrier). hook(T, row, valid, dz):
// called per row tile after the softmax with the lane's dz (the standalone head's dx pass; a no-op when fused).
struct NoOp {
  __device__ void operator()() const {}
};
// post_b1(): run right after the first barrier (the fused forward issues its next-block pixel prefetch there)
template <int C, class Prep, class Hook, class PostB1 = NoOp>
__device__ __forceinline__ void block_head(Prep&& prep, unsigned char* smem, const Args& a, const Operands& ops, int m0,
                                           int M, int wave, int lane, Hook&& hook, long long* stamp,
                                           PostB1&& post_b1 = PostB1{}) {
  static_assert(C >= 2 && C <= 16 && C % 2 == 0, "one 16-class tile; dl stored by class pairs");
  auto st = [&](int k) {
    if (stamp && lane == 0) stamp[k] = (long long)__builtin_amdgcn_s_memtime();
  };
  float* red = reinterpret_cast<float*>(smem + RED_OFF);
  const int wm = wave & 3, wn = wave >> 2, h2 = lane >> 5, r32 = lane & 31;
  const int r = lane & 15, g = lane >> 4;
  const int tid = wave * 64 + lane;
  headtile::f32x4m bv;
#pragma unroll
  for (int v = 0; v < 4; ++v) bv[v] = (4 * g + v) < C ? ops.b[v] : 0.f;
  const int tg[2] = {ops.tg[0], ops.tg[1]};

  hb_f32x16 y[2][2];
  prep(y);
  // block max |h| -> plane scale (all waves, after one exchange)
  float hm = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) hm = fmaxf(hm, fabsf(y[i][j][q]));
  hm = wv::max64(hm);
  // max |W2| over the staged chunks (threads past C * HID / 4 hold a clamped duplicate)
  const float wc = fmaxf(fmaxf(fabsf(ops.w2c[0]), fabsf(ops.w2c[1])), fmaxf(fabsf(ops.w2c[2]), fabsf(ops.w2c[3])));
  const float wmw = wv::max64(wc);
  if (lane == 0) {
    red[wave] = hm;
    red[160 + wave] = wmw;
  }
  __syncthreads();  // (B1) the maxima are in LDS; the caller's buffers are free
  st(17);
  post_b1();
  float bm = red[0], wm2 = red[160];
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    bm = fmaxf(bm, red[w]);
    wm2 = fmaxf(wm2, red[160 + w]);
  }
  const int Eh = bexp(bm), Ew = bexp(wm2), Ed = bexp(a.loss_scale);
  const float sh = p2(14 - Eh), sw = p2(14 - Ew), sd = p2(14 - Ed);
  const hb_f32x2 sh2 = {sh, sh}, sd2 = {sd, sd};
  {  // W2's planes, split once per block: thread tid holds W2 row tid / 32, columns 4 (tid % 32) .. +3 (each wave
     // splitting all of W2 for its own A operands took ~120 VALU per lane)
    const bool ok = tid < C * HID / 4;
    const hb_f32x2 sw2 = {sw, sw};
    const hb_f32x2 x01 = hb_f32x2{ok ? ops.w2c[0] : 0.f, ok ? ops.w2c[1] : 0.f} * sw2;
    const hb_f32x2 x23 = hb_f32x2{ok ? ops.w2c[2] : 0.f, ok ? ops.w2c[3] : 0.f} * sw2;
    const hb_f16x2 h01 = __builtin_convertvector(x01, hb_f16x2), h23 = __builtin_convertvector(x23, hb_f16x2);
    const hb_f16x2 l01 = lo_pair(h01, x01), l23 = lo_pair(h23, x23);
    unsigned char* dst = smem + W2_OFF + (tid >> 5) * W2PP + 8 * (tid & 31);
    *reinterpret_cast<hb_f16x4*>(dst) = hb_f16x4{h01[0], h01[1], h23[0], h23[1]};
    *reinterpret_cast<hb_f16x4*>(dst + W2PL) = hb_f16x4{l01[0], l01[1], l23[0], l23[1]};
  }

  // 1. the h image: granule (4 rows) of hidden unit 64 wn + 32 j + r32, rows 64 wm + 32 i + 8 rq + 4 h2 ..
  // granule q = (16 wm + h2) | (8 i + 2 rq): its byte offset hoff(p, hid, q) is a lane base XOR 8 (8 i + 2 rq) (the
  // granule's varying bits 1..3 never carry; the swizzle is lane-constant), one VALU per address
  const int ib0 = hid_base(64 * wn + r32, 16 * wm + h2), ib1 = hid_base(64 * wn + 32 + r32, 16 * wm + h2);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        // split2's operations, the hi planes on pairs (v_pk_mul_f32, v_cvt_pk_f16_f32) and each lo as one mixed
        // fma (v_fma_mix{lo,hi}_f16: fp16(x - hi) from the f32 x and the f16 hi): the same IEEE results as the
        // scalar form in 4 instead of 8 instructions per pair - the epilogue is VALU-bound
        const hb_f32x2 x01 = hb_f32x2{y[i][j][4 * rq], y[i][j][4 * rq + 1]} * sh2;
        const hb_f32x2 x23 = hb_f32x2{y[i][j][4 * rq + 2], y[i][j][4 * rq + 3]} * sh2;
        const hb_f16x2 h01 = __builtin_convertvector(x01, hb_f16x2), h23 = __builtin_convertvector(x23, hb_f16x2);
        const hb_f16x4 hi = {h01[0], h01[1], h23[0], h23[1]};
        const hb_f16x2 l01 = lo_pair(h01, x01), l23 = lo_pair(h23, x23);
        const hb_f16x4 lo = {l01[0], l01[1], l23[0], l23[1]};
        const int o = (j ? ib1 : ib0) ^ (8 * (8 * i + 2 * rq));  // = hoff(0, hid, q)
        *reinterpret_cast<hb_f16x4*>(smem + o) = hi;
        *reinterpret_cast<hb_f16x4*>(smem + HPL + o) = lo;
      }
    }
  __syncthreads();  // (B2) the h image and W2's planes are complete
  st(18);
  // W2 planes (A operands of the logits): lane (class r, k-group g) takes W2[r][32 kk + 8 g .. +7], wp[kk][0] hi, [1] lo
  hb_f16x8 wp[4][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      wp[kk][p] = *reinterpret_cast<const hb_f16x8*>(smem + W2_OFF + p * W2PL + r * W2PP + 2 * (32 * kk + 8 * g));

  // 2. logits of row tiles wave, wave + 8; softmax, NLL, dl (+ its planes into the dl^T image)
  headtile::TileAcc acc;
  acc.zero();
  const float zsc = p2(Eh - 14) * p2(Ew - 14);  // 2^-(sh + sw) as one exact power of two
  hb_f32x4 dbs = {0.f, 0.f, 0.f, 0.f};          // this lane's dz sums of classes 4g .. 4g+3
  const int lb0 = hoff(0, 8 * g + (r >> 2), 4 * wave + (r & 3)), lb1 = hoff(0, 8 * g + 4 + (r >> 2), 4 * wave + (r & 3));
  const __amdgpu_buffer_rsrc_t dlr = dma_rsrc(a.dl, (unsigned)((size_t)M * C * 4));
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int T = wave + NW * it;
    // B operand lanes: row 16 T + (i16 = lane & 15); image rows (hidden) 32 kk + 8 g + (i16 >> 2) (+ 4), granule
    // 4 T + (i16 & 3)
    // hoff(p, 32 kk + hx, 4 T + (r & 3)) = lb[hx] + 32768 kk + 512 p + 256 it (hx = 8 g + (r >> 2) (+ 4) < 32: the
    // swizzle is lane-constant, and 4 wave + (r & 3) < 32 keeps the tile bit 5 of the granule out of it)
    hb_f16x8 hp[4][2];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        hp[kk][p] = cat8(tr16(smem + lb0 + 32768 * kk + HPL * p + 256 * it),
                         tr16(smem + lb1 + 32768 * kk + HPL * p + 256 * it));
    }
    hb_f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      d = mfma16(wp[kk][0], hp[kk][1], d);  // hi * lo
      d = mfma16(wp[kk][1], hp[kk][0], d);  // lo * hi
      d = mfma16(wp[kk][0], hp[kk][0], d);  // hi * hi
    }
    headtile::f32x4m z;
#pragma unroll
    for (int v = 0; v < 4; ++v) z[v] = fmaf(d[v], zsc, bv[v]);
    const int row = m0 + 16 * T + r;
    const bool valid = row < M;
    float dz[4];
    headtile::softmax_dz<C>(z, tg[it], valid, a.train, a.loss_scale, g, acc, dz, a.bound != nullptr);
    if (a.train && a.dl) {  // classes 4g, 4g+1 | 4g+2, 4g+3 as two 8-byte buffer stores; invalid pairs (rows past
                            // M, classes >= C; C is even) get an out-of-range offset, which the store drops -
                            // no exec-mask branches around the stores
      const unsigned o = (unsigned)(((size_t)row * C + 4 * g) * 4);
      const unsigned o0 = valid && 4 * g + 1 < C ? o : 0x80000000u, o1 = valid && 4 * g + 3 < C ? o + 8 : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b64(hb_u32x2{__float_as_uint(dz[0]), __float_as_uint(dz[1])}, dlr, o0, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(hb_u32x2{__float_as_uint(dz[2]), __float_as_uint(dz[3])}, dlr, o1, 0, 0);
    }
    if (a.train) {
#pragma unroll
      for (int v = 0; v < 4; ++v) dbs[v] += dz[v];
      // the planes of dz * sd (split2's bits, as the h image: packed hi, mixed-fma lo)
      const hb_f32x2 x01 = hb_f32x2{dz[0], dz[1]} * sd2, x23 = hb_f32x2{dz[2], dz[3]} * sd2;
      const hb_f16x2 h01 = __builtin_convertvector(x01, hb_f16x2), h23 = __builtin_convertvector(x23, hb_f16x2);
      const hb_f16x2 l01 = lo_pair(h01, x01), l23 = lo_pair(h23, x23);
      *reinterpret_cast<hb_f16x4*>(smem + dl_off(0, 16 * T + r, g)) = hb_f16x4{h01[0], h01[1], h23[0], h23[1]};
      *reinterpret_cast<hb_f16x4*>(smem + dl_off(1, 16 * T + r, g)) = hb_f16x4{l01[0], l01[1], l23[0], l23[1]};
      hook(T, row, valid, dz);
    }
  }
  st(19);
  // per-wave partials: loss, correct, |dl| bound, db (16 rows of each tile summed over the lane's row index)
  acc.loss = wv::sum64(acc.loss);
  acc.corr = wv::sum64(acc.corr);
  acc.amx = wv::max64(acc.amx);
#pragma unroll
  for (int v = 0; v < 4; ++v) dbs[v] = wv::sum16(dbs[v]);
  if (lane == 0) {
    red[136 + wave] = acc.loss;
    red[144 + wave] = acc.corr;
    red[152 + wave] = acc.amx;
  }
  if (r == 0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) red[8 + 16 * wave + 4 * g + v] = dbs[v];
  }
  __syncthreads();  // (B3) the dl image and the wave partials are complete
  st(20);

  // 3. dW2 of hidden units 16 wave .. +15 over the block's rows: lane (class r / hidden r, row group g)
  if (a.train) {
    hb_f32x4 gacc = {0.f, 0.f, 0.f, 0.f};
    const int hid = 16 * wave + r;
    // Lane-constant bases, so each address below is the base plus an immediate or one XOR with a constant:
    // dl_off(p, 32 ks + X, s) = dl_off(p, X, s) + 1024 ks (X < 32), and granule 8 ks + 2 g + e of hidden unit hid sits
    // at byte hid * 512 + 64 (ks ^ (gswz(hid) >> 3)) + 8 ((2 g + e) ^ (gswz(hid) & 7)), whose bits 6..8 are ks's alone
    const int db0 = dl_off(0, 8 * g + (r >> 2), r & 3), db1 = dl_off(0, 8 * g + 4 + (r >> 2), r & 3);
    const int sw = gswz(hid);
    const int hb0 = (hid * (2 * HPL) + 8 * ((2 * g) ^ (sw & 7))) | (64 * (sw >> 3));
    const int hb1 = (hid * (2 * HPL) + 8 * ((2 * g + 1) ^ (sw & 7))) | (64 * (sw >> 3));
    // the lo plane's bases, opaque to hipcc: otherwise it merges each hi/lo pair into one ds_read2st64_b64 and then
    // spends 4 v_mov per k-step regrouping the granules by plane (bit 9, which HPL sets, is clear in hb0 / hb1)
    int hb0l = hb0 + HPL, hb1l = hb1 + HPL;
    asm volatile("" : "+v"(hb0l), "+v"(hb1l));
    // operands of k-step ks into buffer b; the next k-step's reads are issued before this one's MFMAs (left to
    // itself hipcc reused one register set and exposed two LDS round trips per k-step)
    hb_f16x8 dp[2][2], hq[2][2];  // [buffer][plane]
    auto ld = [&](int ks, int b) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        // A = dl^T: lane (class r, g) gets rows 32 ks + 8 g .. +7 of class r through two transposed reads
        const hb_s16x4 d0 = tr16(smem + db0 + p * DLT_PLANE_B + 1024 * ks);
        const hb_s16x4 d1 = tr16(smem + db1 + p * DLT_PLANE_B + 1024 * ks);
        dp[b][p] = cat8(d0, d1);
        // B = h: lane (hidden r, g) gets rows 32 ks + 8 g .. +7 (granules 8 ks + 2 g, + 1)
        const hb_s16x4 h0 = *reinterpret_cast<const hb_s16x4*>(smem + ((p ? hb0l : hb0) ^ (64 * ks)));
        const hb_s16x4 h1 = *reinterpret_cast<const hb_s16x4*>(smem + ((p ? hb1l : hb1) ^ (64 * ks)));
        hq[b][p] = cat8(h0, h1);
      }
    };
    ld(0, 0);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int b = ks & 1;
      if (ks + 1 < 8) ld(ks + 1, b ^ 1);
      __builtin_amdgcn_sched_barrier(0);  // (the scheduler sank those reads below the MFMAs: lgkmcnt(0) per k-step)
      gacc = mfma16(dp[b][0], hq[b][1], gacc);  // hi * lo
      gacc = mfma16(dp[b][1], hq[b][0], gacc);  // lo * hi
      gacc = mfma16(dp[b][0], hq[b][0], gacc);  // hi * hi
    }
    // lane (hidden r, g) holds dW2[class 4 g + v][16 wave + r]
    const float gsc = p2(Ed - 14) * p2(Eh - 14);
#pragma unroll
    for (int v = 0; v < 4; ++v)
      if (4 * g + v < C) a.part[(4 * g + v) * HID + hid] = gacc[v] * gsc;
  }
  auto sumw = [&](int base) {  // the 8 wave partials in wave order (pairwise tree)
    return ((red[base] + red[base + 1]) + (red[base + 2] + red[base + 3])) +
           ((red[base + 4] + red[base + 5]) + (red[base + 6] + red[base + 7]));
  };
  if (a.train && tid < C) {
    const int c = tid;
    a.part[C * HID + c] = ((red[8 + c] + red[8 + 16 + c]) + (red[8 + 32 + c] + red[8 + 48 + c])) +
                          ((red[8 + 64 + c] + red[8 + 80 + c]) + (red[8 + 96 + c] + red[8 + 112 + c]));
  }
  if (tid == 64) a.part[C * HID + C] = sumw(136);
  if (tid == 128) a.part[C * HID + C + 1] = sumw(144);
  if (tid == 192 && a.bound) {
    float am = red[152];
#pragma unroll
    for (int w = 1; w < NW; ++w) am = fmaxf(am, red[152 + w]);
    *a.bound = 2.f * am * wm2;
  }
  st(21);
}

}  // namespace hblk
}  // namespace sdml
