// LDS-DMA through MUBUF (buffer_load_dwordx4 ... offen lds) instead of global_load_lds_dwordx4.
//
// Why: hipcc models global_load_lds as a FLAT-family access that may touch LDS as well as memory, and a
// pending FLAT access forces every later LDS wait to lgkmcnt(0) (the waitcnt pass cannot count it). In a
// K loop that prefetches the next substep's fragments, that turns the intended counted wait (the reads
// of substep s back, those of s + 1 still in flight) into a full drain before every substep's MFMAs -
// the prefetch buys nothing. The buffer form is a plain VMEM access on vmcnt only, so ds_read waits stay
// counted. Same DMA (1 KiB per wave-instruction, lane-linear into LDS at the wave-uniform destination).
//
// The resource covers [base, base + bytes); offsets are per-lane byte offsets (< 2^32) from base.
#pragma once

#include <hip/hip_runtime.h>

namespace sdml {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(const void* base, unsigned bytes) {
  // dword 3 = 0x00020000: the gfx9-family raw-buffer format word (32-bit data, no swizzle)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// 16 B per lane from base + voff into the wave's 1-KiB LDS block (wave-uniform)
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t r, unsigned voff, void* lds_block) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_block, 16, (int)voff, 0,
                                           0, 0);
}

// The same DMA as inline assembly, with a wave-uniform byte offset soff (the K-step advance) added.
// Why: the wait-count pass tracks LDS-DMA writes and, before every later LDS read it cannot prove disjoint from
// them, waits for all of them. Reads through the ds_read_b64_tr_* builtins carry no alias information, so each
// one got s_waitcnt vmcnt(0): a full drain of a multi-stage DMA ring in front of every fragment read. The pass
// does not see an asm DMA; the caller then owns every wait on it (s_waitcnt vmcnt(N) and a barrier before the
// block reads what it wrote). M0 (the LDS destination) is written here and declared clobbered, so compiler-generated
// M0 users (the builtin LDS-DMA forms, ds_*_addtid) reload it after the asm.
typedef int dma_i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ dma_i32x4 dma_rsrc4(const void* base, unsigned bytes) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(base);
  dma_i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32) & 0xffff);
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

__device__ __forceinline__ void bdma16_asm(dma_i32x4 r, unsigned voff, unsigned soff, const void* lds_block) {
  const unsigned a = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long long)(const __attribute__((address_space(3))) void*)lds_block);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(r),
               "s"(__builtin_amdgcn_readfirstlane(soff)), "s"(a)
               : "memory", "m0");
}

}  // namespace sdml
