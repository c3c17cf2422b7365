// Kernel-variant switches, read on every launch from one table (no getenv on the hot path).
//
// Two kinds:
//  * variant switches pick between two CORRECT implementations of the same op (e.g. the LDS-DMA
//    weight-gradient loop vs the register-staged one). Tests A/B them through set_knob() (the
//    _kernels.set_knob binding); the value stays until it is set again.
//  * probe switches exist only to time a kernel with part of its work removed (e.g. the bf16 GEMM
//    without its output stores). Their results are WRONG by design, so in production builds they are
//    pinned to their defaults: knob() returns the default and set_knob() refuses them.
//
// Environment variables (SDML_<NAME>) are consulted only in builds compiled with
// -DSDML_KERNEL_EXPERIMENTS (SDML_KERNEL_EXPERIMENTS=1 python -m ..._build kernels), once, at first use.
#pragma once

namespace sdml {

enum KnobId : int {
  KNOB_CONV_FWD_IM2COL = 0,  // 1: the im2col conv forward instead of the halo kernel
  KNOB_CONV_BN128_MIN,       // tiles needed before a conv forward uses 128-wide column tiles
  KNOB_CONV_WG_ROWS64,       // 0: 128-row conv weight-gradient tiles for Cout = 64 too
  KNOB_CONV_WG_BLOCKS,       // conv weight-gradient target workgroups
  KNOB_CONV_WGRAD_DMA,       // 1: LDS-DMA conv weight-gradient loop
  KNOB_CONV_WGRAD_STAGES,    // its ring depth (2 or 3)
  KNOB_GEMM_NT_STORE,        // 1: nontemporal epilogue stores (bf16 / two-plane GEMMs)
  KNOB_GEMM_BF16_2PHASE,     // 1: the one-barrier-per-K-step bf16 NT loop
  KNOB_WGRAD_WAVES,          // bf16 weight-gradient grid waves
  KNOB_WGRAD_DMA,            // 0: register-staged weight-gradient loop (bf16 and two-plane)
  KNOB_X2_2PHASE,            // 1: the one-barrier-per-K-step two-plane NT loop
  KNOB_X3_DEEP,              // -1 auto, 0/1: force the bf16x3 engine's pipelining depth
  KNOB_HEAD_VALU,            // 1: the VALU classifier head instead of the MFMA head
  KNOB_HEAD_MAX_BLOCKS,      // VALU head grid cap
  KNOB_U8_WGRAD_XCD,         // uint8 weight gradient: XCD-aware tile order
  KNOB_U8_FWD_WMT,           // uint8 forward wave-tile rows (0 auto)
  KNOB_U8_FWD_WAVES,         // uint8 forward waves per block (0 auto)
  KNOB_U8_FWD_X3,            // 1: uint8 forward on the older bf16x3 kernel
  KNOB_U8_WGRAD_X3,          // 1: uint8 weight gradient on the older bf16x3 kernel
  KNOB_U8_FH_STAGES,         // LDS ring stages of the fused uint8 forward + head (2 or 3)
  KNOB_U8_FWD_PRIO,          // 1: s_setprio 1 on the younger half of the uint8 forward's waves
  KNOB_U8_WGRAD_PRIO,        // 1: the same in the uint8 weight gradient
  KNOB_CNN_SPLIT_BWD,        // reference CNN step, B <= 128: stage 0's backward over 10 workgroups per sample
  KNOB_U8_WGRAD_ILV,         // 1: uint8 weight gradient with the explicit MFMA / staging interleave
  KNOB_GEMM_BF16_T2,         // 1: bf16 NT GEMM on 256 x 128 tiles, two workgroups per CU
  KNOB_U8_WGRAD_RING,        // 1: uint8 weight gradient (dl + ReLU bits) with its operands on an LDS-DMA ring
  KNOB_U8_WGRAD_BAL,         // 1: the ring form with equal MFMA work per SIMD (last 16 columns on 16x16x32 MFMAs)
  KNOB_U8_FWD_DMA_SPREAD,    // 1: fused uint8 forward + head: the next stage's DMA spread over the first substeps
  KNOB_GEMM_BF16_N192,       // bf16 NT GEMM tile width: -1 auto (256 or 192 by wave quantization), 0 256, 1 192
  KNOB_U8_FWD_PREFETCH,      // 1: fused uint8 forward + head prefetches the next workgroup's first pixels into L2
  KNOB_U8_SLAB_COLS,         // weight-gradient slab reduction: float4 columns per 1024-thread block (64 or 32)
  KNOB_GEMM_BF16_TR,         // 1 (default): bf16 NT GEMM (4-phase) accumulates C^T: 8-byte row pieces in the epilogue
  KNOB_WGRAD_NFAST,          // bf16 weight gradient tile order: -1 auto (N fastest when gy is larger than the MALL), 0, 1
  KNOB_ATTN_DKDV_KT,         // attention dK/dV: 32-key tiles per wave (1: 2 waves per SIMD, 2: 1 wave per SIMD)
  KNOB_U8_FH_ROWS512,        // fused uint8 forward + head: 512-row blocks (two head passes): 0 (default, measured no
                             // faster: profiles/r6_fused_rows512_ab.jsonl), 1, -1 auto (when they cover every CU)
  KNOB_GEMM_GROUP_M,         // bf16 / fp16-plane GEMM tile order: 0 M fastest, g > 0 groups of g m-tiles (tile_order.h)
  KNOB_GEMM_BF16_W4,         // bf16 NT GEMM: 1 = the 4-wave 128 x 128-per-wave kernel (one barrier per K-step)
  KNOB_U8_WGRAD_PAIR,        // ring uint8 weight gradient: pairwise in-kernel combine of splits s and s + S/2
  KNOB_ATTN_FWD_QS,          // attention forward: 32-query sub-blocks per wave (1, or 2: two independent softmax chains; 3: 2 in 2-wave blocks)
  KNOB_SGD_MIXED_V,          // bf16 + fp32-master SGD: 0 one 8-element chunk per loop trip, 1 two chunks in flight, 2 nontemporal stores
  KNOB_ATTN_OCC,
  KNOB_CONV_HALO_1WG,        // (A/B) halo conv kernel padded to one workgroup per CU (wave quantization test)             // attention forward: waves-per-SIMD register bound 2 (default), 3 or 4 (A/B)
  KNOB_GEMM_BF16_PERSIST,    // bf16 NT GEMM (4-phase, C^T accumulators): persistent workgroups, the next tile's DMA under this one's last K-steps (-1 auto, 0, 1)
  // ---- probe switches (pinned in production builds) ----
  KNOB_GEMM_BF16_NOSTORE,    // 1: bf16 GEMM skips its output stores (timing only)
  KNOB_U8_VARIANT,           // bf16x3 uint8 kernels' timing variants
  KNOB_COUNT
};

// current value of a switch
int knob(KnobId id);
// set a switch by name (the enum name without KNOB_); false if unknown or a pinned probe switch
bool set_knob(const char* name, int value);
// reset every switch to its default
void reset_knobs();
// whether probe switches are live in this build
bool kernel_experiments_build();

}  // namespace sdml
