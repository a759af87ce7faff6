// wave_ops.h — wave-level helpers shared by the gfx950 kernels (device code only; included by
// the .hip translation units).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace imgrec {

// Order-preserving map of a float key to u32 (ascending floats -> ascending unsigned), so a key
// and a 32-bit row id pack into one u64 whose unsigned order is (key, row).
__device__ __forceinline__ uint32_t key_bits_ordered(float k) {
    const uint32_t u = __float_as_uint(k);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_from_ordered(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Wave-wide minimum of a u64 with DPP row shifts (in-row prefix minimum, lanes shifting in from
// outside the row keep the identity) and four lane reads: the result is uniform (SGPRs).  Replaces
// a 6-step shuffle butterfly whose LDS-crossbar latency dominated the merge rounds.
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    auto step = [&](auto ctrl) __attribute__((always_inline)) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(uint32_t)v,
                                                                  decltype(ctrl)::value, 0xf, 0xf, false);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(uint32_t)(v >> 32),
                                                                  decltype(ctrl)::value, 0xf, 0xf, false);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    };
    step(std::integral_constant<int, 0x111>{});     // row_shr:1
    step(std::integral_constant<int, 0x112>{});     // row_shr:2
    step(std::integral_constant<int, 0x114>{});     // row_shr:4
    step(std::integral_constant<int, 0x118>{});     // row_shr:8 -> lane 15 of a row: its minimum
    uint64_t m = ~0ull;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 16 * r + 15);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 16 * r + 15);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        m = o < m ? o : m;
    }
    return m;
}

// Wave-wide sum (uniform) and exclusive prefix sum of an int: DPP row_shr steps give the in-row
// inclusive prefix, lane reads of the row totals carry it across rows.
__device__ __forceinline__ int row_inclusive_sum(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    return x;
}
__device__ __forceinline__ int wave_sum_i32(int x) {
    const int r = row_inclusive_sum(x);
    return __builtin_amdgcn_readlane(r, 15) + __builtin_amdgcn_readlane(r, 31) +
           __builtin_amdgcn_readlane(r, 47) + __builtin_amdgcn_readlane(r, 63);
}
__device__ __forceinline__ int wave_excl_scan_i32(int x) {
    const int r = row_inclusive_sum(x);
    const int t0 = __builtin_amdgcn_readlane(r, 15), t1 = __builtin_amdgcn_readlane(r, 31);
    const int t2 = __builtin_amdgcn_readlane(r, 47);
    const int row = (int)(threadIdx.x & 63) >> 4;
    return r - x + (row > 0 ? t0 : 0) + (row > 1 ? t1 : 0) + (row > 2 ? t2 : 0);
}

}  // namespace imgrec
