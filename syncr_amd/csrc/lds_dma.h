// lds_dma.h -- gfx950 LDS-DMA helpers shared by the scan and hash kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cdc {

// LDS byte address of a generic pointer into dynamic shared memory.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

template <int N> __device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16 B per lane, HBM -> LDS (M0 = wave-uniform LDS base; lane l lands at +16*l).
// Written as inline asm so hipcc does not drain it with vmcnt(0) before the
// ds_reads of the OTHER buffer; completion is tracked by hand (wait_vmcnt).
template <bool NT>
__device__ __forceinline__ void dma16(const uint8_t *gsrc, uint32_t lds) {
    lds = (uint32_t)__builtin_amdgcn_readfirstlane(lds);     // M0 takes an SGPR (wave-uniform by contract)
    uint32_t keep;
    if constexpr (NT)
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(gsrc), "s"(lds)
            : "memory");
    else
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(gsrc), "s"(lds)
            : "memory");
}

// 4 B per lane from a per-lane address into LDS (M0 = wave-uniform LDS base;
// lane l lands at +4*l).  Completion is tracked by hand (wait_vmcnt).
__device__ __forceinline__ void dma4(const void *gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds)
        : "memory");
}

// 16 B per lane from a wave-uniform SGPR base + per-lane VGPR offset into LDS.
// NT: non-temporal policy (the bytes are read exactly once).
template <bool NT>
__device__ __forceinline__ void dma16_s(uint32_t voff, uint64_t sbase, uint32_t lds) {
    lds = (uint32_t)__builtin_amdgcn_readfirstlane(lds);     // M0 takes an SGPR (wave-uniform by contract)
    // the base too (wave-uniform by contract): the "s" operand must be an SGPR pair
    // even where the compiler cannot prove the value uniform
    sbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sbase >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
    uint32_t keep;
    if constexpr (NT)
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %3\n\t"
            "s_nop 4\n\t"
            "global_load_lds_dwordx4 %1, %2 nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(sbase), "s"(lds)
            : "memory");
    else
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %3\n\t"
            "s_nop 4\n\t"
            "global_load_lds_dwordx4 %1, %2\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(sbase), "s"(lds)
            : "memory");
}

}  // namespace cdc
