// lds_dma.h — global -> LDS DMA helpers shared by the 256 x 256-tile bf16 kernels
// (knn_b16w.hip: the k-NN candidate pass; vit_gemm.hip: the ViT GEMMs).
//
// global_load_lds_dwordx4 is issued from inline asm with M0 set and restored inside the same
// statement: the builtin makes hipcc insert a vmcnt(0) before every later LDS read, which would
// serialise the ring (DESIGN.md "Kernels").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace imgrec {

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// Four one-KiB LDS-DMA pieces under one M0 value (instruction offsets move both the global source
// and the LDS destination; the per-lane offsets are pre-reduced by j KiB).
__device__ __forceinline__ void dma4x(const void* sbase, uint32_t lds0, uint32_t v0, uint32_t v1,
                                      uint32_t v2, uint32_t v3) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %5\n\t"
        "global_load_lds_dwordx4 %2, %5 offset:1024\n\t"
        "global_load_lds_dwordx4 %3, %5 offset:2048\n\t"
        "global_load_lds_dwordx4 %4, %5 offset:3072\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0))
        : "memory");
}

template <int OFF>
__device__ __forceinline__ void dma1(const void* sbase, uint32_t lds0, uint32_t v) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:%4\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0)), "n"(OFF)
        : "memory");
}

// one piece at instruction offset (j & 3) KiB (the dma4x group member j of a partial issue)
__device__ __forceinline__ void dma1_at(int j, const void* sbase, uint32_t lds0, uint32_t v) {
    switch (j & 3) {
        case 0: dma1<0>(sbase, lds0, v); break;
        case 1: dma1<1024>(sbase, lds0, v); break;
        case 2: dma1<2048>(sbase, lds0, v); break;
        default: dma1<3072>(sbase, lds0, v); break;
    }
}

// one dword per lane (the row norms of a tile)
__device__ __forceinline__ void dma4_norm(const float* g, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

__device__ __forceinline__ void barrier_lds() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace imgrec
