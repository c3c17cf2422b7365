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

}  // namespace sdml
