// Host-side launch API of the gfx950 HIP kernels (no torch headers here: kernel TUs compile fast).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "knobs.h"

namespace sdml {

// The head's deferred slab reduction (head_logsoftmax_nll with `defer`): the per-block slabs and where
// they sum to. head_reduce_run launches it alone; u8_wgrad_dl runs it in the same launch as its own
// slab reduction.
struct HeadReduceArgs {
  const float* part = nullptr;  // [nblocks][CK + C + 2]; nullptr: nothing deferred
  int nblocks = 0, CK = 0, C = 0;
  float* gW = nullptr;
  float* gb = nullptr;
  float* stats = nullptr;
  int flags = 0;  // bit 0 = training (accumulate gW/gb), bit 1 = overwrite stats
};
void head_reduce_run(const HeadReduceArgs& a, hipStream_t stream);

// The optimizer step applied by the reduction that produces the last gradients of a step (the one-rank
// MLP step: u8_wgrad_dl's slab + head reduction), instead of a separate SGD launch. p/buf are the
// parameters and momentum aligned with the reduced gradient (p[i] <-> gw[i]), hp/hbuf with the head's
// gW (gb must follow gW). planes: the uint8 forward's fp16 weight planes of the weight at float
// offset pl_off (relative to gw), [rows][K] (SgdPlanes' layout).
struct SgdFuse {
  float* p = nullptr;  // nullptr: no update
  float* buf = nullptr;
  float* hp = nullptr;
  float* hbuf = nullptr;
  float lr = 0.f, mom = 0.f, damp = 0.f, wd = 0.f;
  int nesterov = 0, first = 0, zero_grad = 0;
  unsigned short* planes = nullptr;
  int64_t pl_off4 = 0, pl_n4 = 0, K = 0, Kp = 0, plane_stride = 0;
};

// ---- fp32 MFMA GEMM ------------------------------------------------------------------------
// C[M,N] (op)= sum_k A(m,k) * B(n,k)
//   A(m,k) = A[m*lda + k]        (a_kmajor = false)   or A[k*lda + m]   (a_kmajor = true)
//   B(n,k) = B[n*ldb + k]        (b_kmajor = false)   or B[k*ldb + n]   (b_kmajor = true)
//   if amask: A(m,k) *= (amask(m,k) > 0)   (same layout/ld as A) — fused ReLU backward
// Epilogues: see GemmEpi. Split-K over grid.z requires EPI_ATOMIC.
enum GemmEpi : int {
  EPI_STORE = 0,          // C = acc
  EPI_BIAS = 1,           // C = acc + bias[n]
  EPI_BIAS_RELU = 2,      // C = relu(acc + bias[n])
  EPI_ACCUM = 3,          // C += acc
  EPI_ATOMIC = 4,         // atomicAdd(C, acc)           (split-K capable)
  EPI_BIAS_GELU = 5,      // gemm_bf16 only: U = acc + bias -> aux, C = gelu(U)
  EPI_DGELU = 6,          // gemm_bf16 only: C = acc * gelu'(U), U read from aux
  EPI_BIAS_GELU_SAVE_GRAD = 7,  // gemm_bf16 only: C = gelu(acc + bias), aux = gelu'(acc + bias)
  EPI_MUL_GRAD = 8,             // gemm_bf16 only: C = acc * aux (aux from EPI_BIAS_GELU_SAVE_GRAD)
};

struct GemmArgs {
  const float* A = nullptr;
  const float* amask = nullptr;
  const float* B = nullptr;
  float* C = nullptr;
  const float* bias = nullptr;
  float* rowsum = nullptr;  // if set: rowsum[m] += sum_k A(m,k)  (atomic)   — fused bias-grad
  const float* cmask = nullptr;  // EPI_STORE only: C = acc * (cmask(m,n) > 0), cmask laid out like C
  int M = 0, N = 0, K = 0;
  int lda = 0, ldb = 0, ldc = 0;
  bool a_kmajor = false, b_kmajor = false;
  int epi = EPI_STORE;
  int splits = 1;  // split-K factor (EPI_ATOMIC only)
  // bf16x3 engine only: B already split into bf16 planes [3][N][ldb] (split3_planes of B);
  // k-contiguous B, K % 8 == 0, ldb % 8 == 0 (gemm_f32x3_can_presplit_b)
  const unsigned short* b_split = nullptr;
};

// returns false if the shape/alignment is not supported by the MFMA path
bool gemm_f32_supported(const GemmArgs& g);
void gemm_f32(const GemmArgs& g, hipStream_t stream);
int gemm_f32_pick_splits(int M, int N, int K);
// gemm_f32 internally splits K for few-tile/long-K shapes with non-atomic epilogues
// (bias-init + atomic split-K + ReLU/mask pass); this is its split count, 0 = not used.
int gemm_f32_skinny_splits(int M, int N, int K, int epi);
// small-batch weight gradient (VALU, deterministic): gw[N,K] += (gy*(mask>0))^T[N,M] x[M,K];
// gb[N] += column sums (gb/mask optional); gy/mask are [M,N], x is [M,K], all row-major
constexpr int DW_SMALLK_MAX_M = 128;
// gemm_f32 runs x @ W^T forwards with M <= this many rows on a VALU small-batch kernel
constexpr int FWD_SMALLM_MAX_M = 64;
void dw_smallk(const float* gy, const float* mask, const float* x, float* gw, float* gb, int M, int N, int K,
               hipStream_t stream);
void gemm_f32_set_variant(int v);  // tuning experiments: 0 auto, 16 / 32 = K-step
// fp32 GEMM engine for large shapes: 1 = bf16x3 split on bf16 MFMA (gemm_f32x3.hip, fp32
// accuracy, default), 0 = exact fp32-input MFMA (gemm_f32.hip). Env SDML_F32_GEMM=x3|mfma.
void gemm_f32_set_mode(int mode);
int gemm_f32_mode();
bool gemm_f32x3_eligible(const GemmArgs& g);
int gemm_f32x3_pick_splits(int M, int N, int K, bool a_kmajor);
void gemm_f32x3(const GemmArgs& g, hipStream_t stream);
// true iff gemm_f32 will run this shape on the bf16x3 engine
bool gemm_f32_uses_x3(const GemmArgs& g);
bool gemm_f32x3_can_presplit_b(const GemmArgs& g);
// x[n] fp32 -> out[3][n] bf16 bits (hi, mid, lo; x == hi + mid + lo), n % 4 == 0, 16-B aligned
void split3_planes(const float* x, unsigned short* out, int64_t n, hipStream_t stream);
// transposed split: w [R][C] fp32 -> bf16 planes [3][C][R] (pre-split B = W^T of an input-gradient GEMM)
void split3_planes_t(const float* w, unsigned short* out, int R, int C, hipStream_t stream);
void gemm_f32x3_set_variant(int v);  // pipeline A/B: 0 = early split (default), 1 = split after MFMAs
// uint8-pixel first layer on the bf16x3 engine (the pixel operand is exact in one bf16 plane:
// 3 MFMAs per product, 1 byte per element read). X [M][ldx] uint8.
//   fwd  : C[M,N] = act(scale * X W^T + b), W given pre-split (split3_planes, [3][N][K]);
//          K % 16 == 0, ldx % 16 == 0, X 16-B aligned, ldc >= N
//   wgrad: gw[N,K] += scale * gz^T X, gb[N] += colsum(gz) (gb may be null); gz [M,N] fp32;
//          K % 8 == 0, ldx % 8 == 0, X 8-B aligned, N % 4 == 0
void gemm_u8x3_fwd(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_split, int N,
                   const float* bias, float* C, int ldc, bool relu, float scale, hipStream_t stream);
//          slab: optional [u8x3_wgrad_splits(M, N, K)][N][K] fp32 workspace -> deterministic
//          split-K reduction (nullptr: fp32 atomics); needs (N * K) % 4 == 0 and 16-B aligned gw
int u8x3_wgrad_splits(int M, int N, int K);
void gemm_u8x3_wgrad(const float* gz, const unsigned char* X, int M, int N, int K, int ldx, float* gw, float* gb,
                     float scale, float* slab, hipStream_t stream);
// mlp_u8.hip: LDS-DMA pipelined forward of the uint8-fed first layer (N % 128 == 0). W is given as
// zero-padded fp16 planes [2][N][Kp] of W * 2^8 (u8_planes.h), Kp = u8_fwd_kpad(K), written by
// split_planes_pad or by the fused SGD step.
constexpr int kU8FwdPlanes = 2;
int u8_fwd_kpad(int K);
bool u8_fwd_supported(int M, int N, int K, int ldx, const void* X);
void split_planes_pad(const float* w, unsigned short* out, int N, int K, int Kp, hipStream_t stream);
// mask (optional, relu only): [M][N / 32] words, bit n % 32 of word n / 32 = (y[m][n] > 0), the ReLU
// mask the factored weight gradient (u8_wgrad_dl) reads instead of y itself
void u8_fwd(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_planes, int N, int Kp,
            const float* bias, float* C, int ldc, bool relu, float scale, hipStream_t stream,
            unsigned* mask = nullptr, float* wmax = nullptr);
// wmax slots u8_fwd writes for M x N (per-wave max |output|, a split bound for the next two-plane GEMM)
int u8_fwd_wmax_slots(int M, int N);
// The uint8 first layer and the classifier head in ONE kernel (N = 128 hidden, C in {2, 10, 16}, training):
// h = relu(scale X W^T + b) stays in the workgroup (LDS, from the MFMA accumulators), the head
// (head_tile.h: logits, log_softmax, NLL, argmax, dl = loss_scale (softmax - onehot), dW2^T/db2 partials)
// runs on it, and only dl [M][C], the ReLU bits mask [M][4], one head slab row per block
// ([C*128 dW2 | C db2 | loss, correct], reduced by head_reduce_run / u8_wgrad_dl) and one |dl @ W2|
// bound per block leave the chip. h is never written.
struct U8HeadArgs {
  const float* w2 = nullptr;      // [C][128]
  const float* b2 = nullptr;      // [C]
  const int64_t* target = nullptr;
  int C = 0;
  float loss_scale = 0.f;
  float* dl = nullptr;            // [M][C]
  unsigned* mask = nullptr;       // [M][4]
  float* part = nullptr;          // [u8_fwd_head_blocks(M)][C * 128 + C + 2]
  float* bound = nullptr;         // [u8_fwd_head_blocks(M)]
};
bool u8_fwd_head_supported(int M, int N, int K, int ldx, const void* X, int C);
int u8_fwd_head_blocks(int M);
// experiments builds: the next u8_fwd_head launches write MODE 7 phase stamps into buf ([blocks][8][u8_stamp_slots()]
// int64; nullptr turns them off); production builds return false and ignore it
bool u8_set_stamps(void* buf);
int u8_stamp_slots();
// test probe: ds_read_b64_tr_b8 over a 1-KiB image (img [1024] bytes, addr [64] byte offsets, out [64][2] int32)
void u8_tr8_probe(const unsigned char* img, const int* addr, int* out, hipStream_t stream);
// experiments builds: weight-gradient phase stamps ([blocks][8][16] int64; nullptr off)
bool u8_set_wgrad_stamps(void* buf);
void u8_fwd_head(const unsigned char* X, int M, int K, int ldx, const unsigned short* w_planes, int N, int Kp,
                 const float* bias, float scale, const U8HeadArgs& head, hipStream_t stream);
// mlp_u8.hip: weight + bias gradient of the uint8-fed first layer (K = 784 pixel columns, N % 64 == 0,
// M % 32 == 0): gw[N][784] += scale * dz^T X, gb[N] += colsum(dz), where gb MUST directly follow gw in
// memory (gwb = gw, gwb + N * 784 = gb: the flat gradient buffer's layout). slab: workspace of
// u8_wgrad_slab_floats(M, N) floats; deterministic (fixed-order reduction).
bool u8_wgrad_supported(int M, int N, int K, int ldx, const void* X, const void* dz);
// (blocks > 0: the slab of a hidden-group range launched with that many row splits, WgradGroups)
int64_t u8_wgrad_slab_floats(int M, int N, int blocks = 0);
// dz enters as two fp16 planes scaled by a power of two chosen from a bound: amax [namax] with
// |dz| <= max(amax) (required here: the fused head's per-block maxima or a torch amax).
void u8_wgrad(const float* dz, const unsigned char* X, int M, int N, int ldx, float* slab, float* gwb, float scale,
              const float* amax, int namax, hipStream_t stream);
// the same with the factored boundary gradient: dz = (dl @ w2) * (h > 0) (dl [M][C], w2 [C][N],
// h [M][N]) expanded in the kernel's staging with head_dx_from_dl's exact arithmetic; without amax
// (namax == 0) each workgroup bounds its dz by max_row sum_c |dl| * max |w2|. With the same amax the
// result is bit-identical to head_dx_from_dl + u8_wgrad. The ReLU mask comes from h [M][N] OR from
// its bits (mask [M][N / 32], u8_fwd / u8_fwd_head): exactly one of h / mask is non-null.
bool u8_wgrad_dl_supported(int M, int N, int K, int ldx, const void* X, const void* h, int C);
// A range of 64-unit hidden groups [g_first, g_first + g_count) of the weight gradient, in ~`blocks` row
// splits (the data-parallel step computes the gradient in two such ranges, so that the first range's
// all-reduce overlaps the second range's kernel; parallel/pipeline.py). Deterministic for a given
// (M, blocks); the partition differs from the whole-gradient launch, so the sums round differently.
struct WgradGroups {
  int g_first, g_count, blocks;
};
// head (optional): a deferred head reduction run in the same launch as this one's slab reduction
// grp (optional): only that hidden-group range (reduced with its bias entries; no fused optimizer step)
void u8_wgrad_dl(const float* dl, const float* w2, const float* h, const unsigned* mask, int C,
                 const unsigned char* X, int M, int N, int ldx, float* slab, float* gwb, float scale,
                 const float* amax, int namax, hipStream_t stream, const HeadReduceArgs* head = nullptr,
                 const SgdFuse* sgd = nullptr, const WgradGroups* grp = nullptr);
// out[i] += sum_s slab[s * stride + i] in split order (n % 4 == 0, 16-B aligned)
void slab_reduce(const float* slab, int64_t stride, int splits, float* out, int64_t n, hipStream_t stream);

// ---- fused classifier head: z = x W^T + b; log_softmax; NLL; backward --------------------
// x [M,K] fp32, W [C,K], b [C], target [M] int64. stats[0] += sum loss, stats[1] += #correct.
// If dx != nullptr: dx = scale * (softmax - onehot) @ W ; gW += dz^T x ; gb += sum dz.
// K must be 128 for the fully fused kernel (the 784-128-10 model); head_generic handles others
// (and writes dz for a follow-up GEMM).
// The fused path needs a workspace of head_workspace_floats(M, K, C) floats (per-block
// partial slabs, reduced by a second deterministic pass).
bool head_fused_supported(int K, int C);
// wide-K LDS-staged head (C = 10, K <= 1024): with gW/gb and a workspace it also produces dW/db
bool head_lds_supported(int M, int K, int C);
size_t head_workspace_floats(int M, int K, int C);
// mask_dx: dx *= (x > 0) — the producing stage's ReLU backward, fused (x is its output)
// dl (fused path only, may be null): also/instead write the scaled dlogits dz [M][C] — the rank-C
// factor of dx = dz @ W (with dx == nullptr the dx pass is skipped; gW/gb/stats as usual)
void head_logsoftmax_nll(const float* x, const float* W, const float* b, const int64_t* target, int M, int K,
                         int C, float scale, float* stats, float* dx, float* gW, float* gb, float* dz_out,
                         float* workspace, bool mask_dx, hipStream_t stream, float* dl = nullptr,
                         bool stats_overwrite = false,  // stats_overwrite: stats = this call's totals
                         float* dx_amax = nullptr, int* n_amax = nullptr, HeadReduceArgs* defer = nullptr);
// dx_amax (capacity kHeadAmaxMax floats): where the MFMA head path writes per-block bounds on |dx| and the
// wide-K (LDS) head its per-block max |dx| (*n_amax of them; 0 when another head variant ran) - the uint8
// weight gradient's dz bound, the two-plane split's bound
constexpr int kHeadAmaxMax = 1024;
// dx = (dl @ W) * (x > 0 if mask): the fused head's dx rebuilt bit-identically from its factor dl
// (K == 128, C in {2, 10, 16}: head_fused_supported)
void head_dx_from_dl(const float* dl, const float* W, const float* x, float* dx, int M, int K, int C, bool mask,
                     hipStream_t stream);

// head_pool.hip: global average pool + Linear(K -> C) + log_softmax + NLL + the whole backward (ResNet's last
// layer). x [M][P][K] channels-last, W [C][K], b [C], dx like x, gW / gb accumulated, all bf16 (bf16 = true) or
// fp32; stats [2] (loss sum, correct) added, or overwritten with stats_overwrite. ws:
// head_pool_workspace_floats(M, K, C) floats. Deterministic (fixed-order slab reduction).
bool head_pool_supported(int M, int P, int K, int C);
int64_t head_pool_workspace_floats(int M, int K, int C);
void head_pool_xent(const void* x, const void* W, const void* b, const int64_t* tgt, int M, int P, int K, int C,
                    float scale, void* dx, void* gW, void* gb, float* stats, bool stats_overwrite, float* ws, bool bf16,
                    hipStream_t stream);

// ---- SGD with momentum over a flat buffer ------------------------------------------------
// zero_grad: also writes g = 0 after reading it (fuses the next step's zero_grad)
// optional bf16 weight-plane cache written from the updated weights (see sgd_kernel)
struct SgdPlanes {
  unsigned short* planes = nullptr;  // [2][rows][Kp] (u8_planes.h), plane_stride = rows * Kp
  int64_t off4 = 0, n4 = 0;          // float4 range of the flat buffer holding the [rows][K] weight
  int64_t K = 0, Kp = 0, plane_stride = 0;
};
void sgd_momentum(float* p, float* g, float* buf, int64_t n, float lr, float momentum, float dampening,
                  float wd, bool nesterov, bool first, bool zero_grad, hipStream_t stream,
                  SgdPlanes planes = SgdPlanes());

// bf16 model weights with fp32 master weights: master/buf fp32, p/g bf16 (n % 4 == 0)
void sgd_momentum_mixed(float* master, void* p_bf16, void* g_bf16, float* buf, int64_t n, float lr, float momentum,
                        float dampening, float wd, bool nesterov, bool first, bool zero_grad, hipStream_t stream);

// ---- synthetic MNIST-shape data (counter-based; bit-identical to the host generator) -----
void synth_mnist(uint64_t seed, int64_t start, int64_t n, int H, int W, int mode, float* x, int64_t* y,
                 hipStream_t stream);

// ---- transformer (GPT-2) kernels, bf16 ----------------------------------------------------
// per-row loss / correct (fp32) and, if dlogits != nullptr, dlogits = scale*(softmax-onehot)
void cross_entropy_bf16(const void* logits, const int64_t* target, int rows, int V, int ld, float scale,
                        int ignore_index, float* row_loss, float* row_ok, void* dlogits, hipStream_t stream);
// LayerNorm over the last dim D (D % 8 == 0, D <= 4096); saves fp32 mean/rstd per row
// res/xs non-null: fused residual add, xs = x + res is stored and normalised (one pass)
void layernorm_fwd_bf16(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int rows,
                        int D, float eps, hipStream_t stream, const void* res = nullptr, void* xs = nullptr);
// dx (bf16) and dwdb_acc[0:D] += dw, dwdb_acc[D:2D] += db (fp32); workspace: blocks * 2D floats
int layernorm_bwd_blocks(int rows);
void layernorm_bwd_bf16(const void* x, const void* w, const void* gy, const float* mean, const float* rstd, void* dx,
                        float* workspace, float* dwdb_acc, float* unused, int rows, int D, hipStream_t stream);

// same, but dw/db are added straight into the bf16 parameter gradients gw/gb (no fp32 copy,
// no separate accumulate kernel)
// gadd non-null: dx also gets the residual-path gradient of a fused add + LayerNorm
void layernorm_bwd_bf16_accum(const void* x, const void* w, const void* gy, const float* mean, const float* rstd,
                              void* dx, float* workspace, void* gw, void* gb, int rows, int D, hipStream_t stream,
                              const void* gadd = nullptr);
// bias gradient of a bf16 linear layer: gb[n] (bf16) += sum_m gy[m][n]; workspace fp32
// [bias_grad_blocks(M) * N]. Deterministic (fixed-order partial sums).
int bias_grad_blocks(int M);
void bias_grad_bf16(const void* gy, int M, int N, int ld, void* gb, float* workspace, hipStream_t stream);

// ---- the whole 784-128-10 MLP training step in two launches (mlp_small.hip, B <= 128) ----------------
// x [B][784] fp32 (or uint8 pixels, x_u8: scaled by 1/255), parameters and momentum buffers updated in
// place (torch.optim.SGD), stats = {loss sum, correct}; scratch: h [B][128], snap [10 * 128 + 10].
int mlp_small_step_max_batch();
bool mlp_small_step(const void* x, bool x_u8, const int64_t* target, int B, float scale, float* w1, float* b1,
                    float* w2, float* b2, float* m1, float* mb1, float* m2, float* mb2, float lr, float mom,
                    float damp, float wd, bool nesterov, bool first, float* h_scratch, float* snap_scratch,
                    float* stats, hipStream_t stream);

// ---- GPT-2 elementwise / embedding kernels (gpt2_ops.hip) ------------------------------------
// tanh-GELU (n % 8 == 0, 16-B aligned): y = gelu(x); gx = gy * gelu'(x) (gx may alias gy)
void gelu_fwd_bf16(const void* x, void* y, int64_t n, hipStream_t stream);
// dst[k] = src[k]^T ([R][C] -> [C][R], bf16, R and C multiples of 8) for n <= kTransposeBatchMax matrices, one launch
constexpr int kTransposeBatchMax = 64;
void transpose_batched_bf16(const void* const* src, void* const* dst, const int* R, const int* C, int n,
                            hipStream_t stream);
void gelu_bwd_bf16(const void* gy, const void* x, void* gx, int64_t n, hipStream_t stream);
// out[r] = wte[tok[r]] + wpe[r % S]  (rows = B * S, C % 4 == 0)
void embedding_fwd_bf16(const int64_t* tok, const void* wte, const void* wpe, void* out, int rows, int S, int C, int V,
                        hipStream_t stream);
// gwpe[s] += sum_b g[b][s]; gwte[v] += sum over positions of token v (sorted_tok / perm: the tokens sorted
// stably, with their positions) - deterministic, either gradient may be null
void embedding_bwd_bf16(const void* g, const int64_t* sorted_tok, const int64_t* perm, void* gwte, void* gwpe, int B,
                        int S, int C, int V, hipStream_t stream);

// ---- bf16 GEMM with fused epilogues (gemm_bf16.hip): C[M][N] = A[M][K] . (b_kn ? B[K][N] : B[N][K]^T) ----
// epi: EPI_STORE, EPI_BIAS (bias [N] bf16), EPI_BIAS_GELU (aux = pre-activation out), EPI_DGELU (aux =
// pre-activation in). K % 64 == 0, N % 8 == 0, leading dimensions % 8 == 0 (gemm_bf16_supported).
bool gemm_bf16_supported(int M, int N, int K, int lda, int ldb, int ldc, bool b_kn);
void gemm_bf16(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, bool b_kn,
               int epi, const void* bias, void* aux, int ldaux, hipStream_t stream);

// ---- the reference CNN's whole training step (both stages on one rank) in two launches (ref_cnn.hip) ----
// params / bufs: conv1.w, conv1.b, conv2.w, conv2.b, fc1.w, fc1.b, fc2.w, fc2.b (bufs[i] nullptr: no momentum);
// rec: [B][ref_cnn_step_record_floats()] scratch; stats [2] = (loss sum, correct) (overwritten); *ctr += 1
int ref_cnn_step_record_floats();
// records + the split backward's per-sample workspace (B <= 128)
int ref_cnn_step_workspace_floats(int B);
void ref_cnn_step(const float* x, const int64_t* target, int B, float* const* params, float* const* bufs,
                  unsigned long long seed0, unsigned long long seed1, long long* ctr, float p0, bool drop0, float p1,
                  bool drop1, float scale, float lr, float mom, float damp, float wd, bool nesterov, bool first,
                  float* rec, float* stats, hipStream_t stream, long long* stamps = nullptr);

// ---- fp32-accurate GEMMs from pre-split fp16 planes (gemm_f16x2.hip) ---------------------------
// An fp32 tensor X [rows][cols] becomes planes [2][rows][ldp] (hi, lo of X * 2^(14 - E), |X| < 2^E from
// the max of |amax[0..namax)|); scale_out receives 2^(E - 14). Products use 3 fp16 MFMA products.
void x2_split(const float* X, int rows, int cols, int ldx, const float* amax, int namax, void* planes, int64_t ps,
              int ldp, float* scale_out, hipStream_t stream);
// the same for X^T: planes [2][cols][ldp] of the transpose (the input gradient's NT weight operand)
void x2_split_t(const float* X, int rows, int cols, int ldx, const float* amax, int namax, void* planes, int64_t ps,
                int ldp, float* scale_out, hipStream_t stream);
// C[M][N] (fp32) = sa sb A'[M][K] . (b_kn ? B'[K][N] : B'[N][K]^T) (+ bias[n]) (relu) (* (mask[m][n] > 0));
// A/B: plane 0, plane 1 at + a_ps / b_ps (elements). wmax (optional, x2_gemm_wmax_slots floats): per-wave
// max |C|, a bound source for the next x2_split. K % 64 == 0, N % 8 == 0 (x2_gemm_supported).
bool x2_gemm_supported(int M, int N, int K, int lda, int ldb, int ldc, bool b_kn);
int x2_gemm_wmax_slots(int M, int N);
void x2_gemm(const void* A, int64_t a_ps, const void* B, int64_t b_ps, float* C, int M, int N, int K, int lda, int ldb,
             int ldc, bool b_kn, const float* sa, const float* sb, const float* bias, bool relu, const float* mask,
             int ldm, float* wmax, hipStream_t stream);
// gw[M][N] (fp32, ldc) += sdz sx sum_t dz'[t][m] x'[t][n]; gb (optional) [M] += sdz sum_t dz'[t][m]
bool x2_wgrad_supported(int M, int N, int T, int lda, int ldb);
size_t x2_wgrad_workspace_floats(int M, int N, int T);
void x2_wgrad(const void* dz, int64_t dz_ps, const void* x, int64_t x_ps, const float* sdz, const float* sx, float* gw,
              int ldc, float* gb, float* workspace, int M, int N, int T, int lda, int ldb, hipStream_t stream);

// ---- weight gradient of a bf16 Linear: gw[M,N] (bf16) += gy[T,M]^T x[T,N] -------------------
// fp32 accumulation, token range split over workgroups, deterministic slab reduction.
// workspace: wgrad_bf16_workspace_floats(M, N, T) fp32 (0 = none needed)
bool wgrad_bf16_supported(int M, int N, int T, int lda, int ldb, int ldc);
int wgrad_bf16_splits(int M, int N, int T);
size_t wgrad_bf16_workspace_floats(int M, int N, int T);
// gb (optional, bf16 [M]) += column sums of gy (the bias gradient), fused
void wgrad_bf16(const void* gy, const void* x, void* gw, void* gb, float* workspace, int M, int N, int T, int lda,
                int ldb, int ldc, hipStream_t stream);

// ---- 3x3 stride-1 pad-1 convolution, bf16 NHWC (conv_bf16.hip) ---------------------------
// C (input channels) and Co multiples of 64. Weights in torch layout [Co][C][3][3] are first
// transformed: forward [Co][9][C]; dgrad (flipped, transposed) [C][9][Co] — the dgrad is the
// forward kernel on dy with the dgrad weights.
bool conv3x3_bf16_supported(int C, int Co);
// torch [Co][C][3][3] weight -> forward layout [Co][9][C] and/or dgrad layout [C][9][Co] (flipped taps); either may be null
void conv3x3_weight_transform_bf16(const void* w_torch, void* fwd, void* dgrad, int Co, int C, hipStream_t stream);
// up to kWtBatchMax weights' forward (and, where dgrad[k] is set, dgrad) layouts in one launch
constexpr int kWtBatchMax = 32;
void conv3x3_weight_transform_batched_bf16(const void* const* w, void* const* fwd, void* const* dgrad, const int* Co,
                                           const int* C, int n, hipStream_t stream);
// add (optional, y's layout): y = bf16(conv + add). part (optional): BatchNorm partials of y,
// [conv_part_rows(Nb, OH, OW)][2][Co] fp32 (per 256-pixel tile: sum y, sum y^2), for bn_nhwc_fwd_bf16.
int conv_part_rows(int Nb, int OH, int OW);
// bnb (optional, with part): y is the input gradient dy of a training BatchNorm whose forward input x has y's layout;
// part then receives that BatchNorm backward's per-tile sums of g = dy * mask and g * (x - mean) * rstd (for
// bn_nhwc_bwd_bf16's part) instead of the forward statistics. relu: 0 none, 1 mask y_bn > 0 (y_bn = the
// BatchNorm's saved output), 2 mask recomputed from x, gamma, beta, mean, rstd.
struct ConvBnBack {
  const void* x = nullptr;
  const void* y = nullptr;
  const float* mean = nullptr;
  const float* rstd = nullptr;
  const void* gamma = nullptr;
  const void* beta = nullptr;
  int relu = 0;
};
void conv3x3_fwd_bf16(const void* x, const void* wt, void* y, int Nb, int H, int W, int C, int Co, hipStream_t stream,
                      const void* add = nullptr, float* part = nullptr, const ConvBnBack* bnb = nullptr);
// gw_torch [Co][C][3][3] bf16 += dw; workspace: conv3x3_wgrad_workspace_floats(...) fp32
// general bf16 NHWC convolution on the implicit-GEMM kernels: kernel 3 (pad 1) or 1 (pad 0), stride 1
// or 2, C and Co multiples of 64. Forward (im2col kernel; wt = [Co][ks*ks][C]) and weight gradient
// (accumulated into the bf16 torch-layout [Co][C][ks][ks] gradient). The input gradient of a stride-2
// one: four parity-class GEMMs in one launch (conv_dgrad_s2_bf16) on the packed weights of
// conv_dgrad_s2_weight_bf16 (conv_dgrad_s2_weight_elems bf16 elements); dx [Nb][H][W][C] NHWC is
// written in full.
int conv_out_size(int in, int ks, int stride, int pad);
bool conv_general_supported(int C, int Co, int ks, int stride, int pad);
void conv_fwd_bf16(const void* x, const void* wt, void* y, int Nb, int H, int W, int C, int Co, int ks, int stride,
                   int pad, hipStream_t stream, const void* add = nullptr, float* part = nullptr);
size_t conv_dgrad_s2_weight_elems(int Co, int C, int ks);
void conv_dgrad_s2_weight_bf16(const void* w_torch, void* packed, int Co, int C, int ks, int pad, hipStream_t stream);
// part / bnb: as conv3x3_fwd_bf16's, conv_dgrad_s2_part_rows rows (the parity classes' pixel tiles)
int conv_dgrad_s2_part_rows(int Nb, int H, int W, int ks, int pad);
void conv_dgrad_s2_bf16(const void* dy, const void* packed, void* dx, int Nb, int H, int W, int C, int Co, int ks,
                        int pad, hipStream_t stream, const void* add = nullptr, float* part = nullptr,
                        const ConvBnBack* bnb = nullptr);
size_t conv_wgrad_workspace_floats(int Nb, int H, int W, int C, int Co, int ks, int stride, int pad);
void conv_wgrad_bf16(const void* dy, const void* x, void* gw_torch, float* workspace, int Nb, int H, int W, int C,
                     int Co, int ks, int stride, int pad, hipStream_t stream);
// stem convolution with ONE input channel, 3x3 / stride 1 / pad 1, bf16: x [N][H][W], w [Co][1][3][3],
// y NHWC [N][H][W][Co]; weight gradient accumulated into the bf16 [Co][1][3][3] gradient
bool conv_c1_supported(int Co);
void conv_c1_fwd_bf16(const void* x, const void* w, void* y, int Nb, int H, int W, int Co, hipStream_t stream);
size_t conv_c1_wgrad_workspace_floats(int Nb, int H, int W, int Co);
void conv_c1_wgrad_bf16(const void* dy, const void* x, void* gw, float* workspace, int Nb, int H, int W, int Co,
                        hipStream_t stream);
size_t conv3x3_wgrad_workspace_floats(int Nb, int H, int W, int C, int Co);
void conv3x3_wgrad_bf16(const void* dy, const void* x, void* gw_torch, float* workspace, int Nb, int H, int W, int C,
                        int Co, hipStream_t stream);

// ---- BatchNorm (+ residual) (+ ReLU), channels-last bf16 [M = N*H*W][C] (batchnorm_nhwc.hip) ---
// training forward: batch statistics, optional running-stat update (rmean/rvar may be null),
// y = relu?(bn(x) + res?); mean/rstd (fp32 [C]) saved for the backward.
// workspace: bn_nhwc_workspace_floats(M, C) fp32
bool bn_nhwc_supported(int C);
size_t bn_nhwc_workspace_floats(int M, int C);
void bn_nhwc_fwd_bf16(const void* x, const void* res, const void* gamma, const void* beta, void* rmean, void* rvar,
                      int M, int C, float eps, float momentum, bool relu, void* y, float* mean, float* rstd,
                      float* workspace, hipStream_t stream, int64_t* num_batches_tracked = nullptr,
                      const float* part = nullptr, int part_rows = 0);
// backward: g = dy * (y > 0 if relu); dx, dres = g (optional), ggamma/gbeta (bf16, accumulated; optional)
void bn_nhwc_bwd_bf16(const void* x, const void* dy, const void* y, const float* mean, const float* rstd,
                      const void* gamma, int M, int C, bool relu, void* dx, void* dres, void* ggamma, void* gbeta,
                      float* workspace, hipStream_t stream, const void* beta = nullptr, const float* part = nullptr,
                      int part_rows = 0);
void bn_nhwc_eval_bf16(const void* x, const void* res, const float* scale, const float* shift, int M, int C, bool relu,
                       void* y, hipStream_t stream);

// ---- causal flash attention, bf16, head_dim 64 ------------------------------------------
// q/k/v (and dq/dk/dv) share one strided layout [b][h][s][64] (strides sqb, sqh, sqs; d
// contiguous) — e.g. views into the fused c_attn output; o/dout share another (sob, soh, sos).
// lse/delta: fp32 [B*H*S] scratch (lse written by fwd, read by bwd).
struct AttnShape {
  const void *q = nullptr, *k = nullptr, *v = nullptr, *o = nullptr, *dout = nullptr;
  void *out = nullptr, *dq = nullptr, *dk = nullptr, *dv = nullptr;
  float *lse = nullptr, *delta = nullptr;
  int B = 0, H = 0, S = 0;
  long sqb = 0, sqh = 0, sqs = 0, sob = 0, soh = 0, sos = 0;
  float scale = 1.f;
  int causal = 1;
};
void attention_fwd_bf16(const AttnShape& s, hipStream_t stream);
void attention_set_fwd_kb(int kb);  // tuning: keys per forward tile (0 = default, 64, 128)
void attention_bwd_bf16(const AttnShape& s, hipStream_t stream);

// ---- reference CNN (MNIST), fp32, one launch per stage pass (ref_cnn.hip) ------------------
// Dropout masks: keep iff u(seed_eff, sample0 + n, unit) >= p, scale 1/(1-p) (drop == false: off),
// seed_eff = seed + 0x9E3779B97F4A7C15 * (*ctr) (ctr: optional device step counter).
// Training forwards save z1 [B,1440] f32 and argmax bytes [B,ref_cnn_idx_bytes()] for the backward
// (nullptr: inference, nothing saved). The backward takes the forward's output for the ReLU mask.
int ref_cnn_idx_bytes();
int ref_cnn_z1_floats();
void ref_cnn_stage0_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2, float* out,
                        float* z1_save, unsigned char* idx_save, int B, unsigned long long seed, const long long* ctr,
                        unsigned sample0, float p, bool drop, hipStream_t stream);
void ref_cnn_stage0_bwd(const float* x, const float* w2, const float* out, const float* gout, const float* z1_save,
                        const unsigned char* idx_save, int B, unsigned long long seed, const long long* ctr,
                        unsigned sample0, float p, bool drop, float* gw1, float* gb1, float* gw2, float* gb2,
                        hipStream_t stream);
// stats[0] += sum NLL, stats[1] += correct; train iff dx != nullptr (then all grads accumulate)
void ref_cnn_stage1(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                    const int64_t* target, int B, unsigned long long seed, const long long* ctr, unsigned sample0,
                    float p, bool drop, float scale, float* stats, float* dx, float* gw1, float* gb1, float* gw2,
                    float* gb2, hipStream_t stream);

}  // namespace sdml
