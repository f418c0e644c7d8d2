// LDS-DMA (buffer_load ... lds) issued as inline asm.
//
// Why not __builtin_amdgcn_raw_ptr_buffer_load_lds: the compiler's waitcnt
// pass records every builtin LDS-DMA as a pending LDS write and, lacking
// alias-scope information, makes the next ds_read_b64_tr_b16 (the transposed
// fragment read of the MFMA kernels) wait for vmcnt(0) — i.e. for the DMA just
// issued for a LATER pipeline stage, which put the full HBM latency into every
// step of the GEMM, attention and dq pipelines. Every kernel using these
// helpers counts its own DMA with explicit `s_waitcnt vmcnt(N)` before a
// barrier, so that wait was never needed for correctness.
// M0 carries the wave's LDS destination base; it is declared clobbered (the
// compiler loads M0 itself before each of its own M0 users). One wait state
// between the M0 write and the LDS-DMA that reads it (s_nop 0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// 16 B per lane: lane l's bytes land at dst + 16 l (dst wave-uniform)
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rs, const void* dst, uint32_t voff) {
    const uint32_t m =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)dst);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(rs) : "m0");
}
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t rs, const __attribute__((address_space(3))) char* dst,
                                          uint32_t voff) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(rs) : "m0");
}
// 4 B per lane: lane l's word lands at dst + 4 l
__device__ __forceinline__ void lds_dma4(__amdgpu_buffer_rsrc_t rs, const void* dst, uint32_t voff) {
    const uint32_t m =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)dst);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(rs) : "m0");
}
#pragma clang diagnostic pop
