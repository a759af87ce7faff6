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

// The K = min(kout, valid) smallest of a wave's packed entries (order-preserving key bits | row,
// KIN per lane, ~0 = empty; distinct: a row sits in one list; each lane's entries ascending).
// T, the K-th smallest, is found bit by bit (count of entries <= a trial value, summed over the
// wave): the key bits below the highest one where the smallest and largest valid value differ,
// then the 32 row bits only when the K-th key is tied across the cut.  Each lane's entries <= T
// (a prefix of its sorted list) go to LDS slots of `buf` (64 entries, this wave's) from an
// exclusive scan.  Returns K (uniform); lane < K gets its output value `mine` and its `rank`.
template <int KIN>
__device__ __forceinline__ int wave_select_packed(const uint64_t (&v)[KIN], int kout, uint64_t* buf,
                                                  uint64_t& mine, int& rank) {
    constexpr uint64_t kEmpty = ~0ull;
    const int lane = (int)(threadIdx.x & 63);
    auto count_le = [&](uint64_t x) __attribute__((always_inline)) {
        int c = 0;
#pragma unroll
        for (int p = 0; p < KIN; ++p) c += v[p] <= x ? 1 : 0;
        return c;
    };
    int nvl = 0;
    uint64_t vmin = kEmpty, vmax = 0;
#pragma unroll
    for (int p = 0; p < KIN; ++p) {
        const bool val = v[p] != kEmpty;
        nvl += val ? 1 : 0;
        vmin = v[p] < vmin ? v[p] : vmin;
        vmax = (val && v[p] > vmax) ? v[p] : vmax;
    }
    const int K = min(kout, wave_sum_i32(nvl));
    uint64_t T = 0;
    if (K > 0) {
        // T lies in [min, max] of the valid values: the bits above their highest difference are
        // common, so the select starts below them (keys of one query sit in a narrow range)
        vmin = wave_min_u64(vmin);
        vmax = ~wave_min_u64(~vmax);
        const int hb = vmin == vmax ? -1 : 63 - __builtin_clzll(vmin ^ vmax);
        uint64_t prefix = hb < 0 ? vmin : (hb >= 63 ? 0 : vmin & ~((2ull << hb) - 1));
        for (int b = min(hb, 63); b >= 32; --b) {
            const uint64_t lo = prefix | ((1ull << b) - 1);
            if (wave_sum_i32(count_le(lo)) < K) prefix |= 1ull << b;
        }
        T = prefix | 0xffffffffull;
        if (wave_sum_i32(count_le(T)) > K) {                   // the K-th key is tied: rows decide
            for (int b = min(hb, 31); b >= 0; --b) {
                const uint64_t lo = prefix | ((1ull << b) - 1);
                if (wave_sum_i32(count_le(lo)) < K) prefix |= 1ull << b;
            }
            T = prefix;
        }
    }
    const int c = K > 0 ? count_le(T) : 0;
    const int base = wave_excl_scan_i32(c);
#pragma unroll
    for (int p = 0; p < KIN; ++p)
        if (p < c) buf[base + p] = v[p];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    mine = kEmpty;
    rank = 0;
    if (lane < K) {
        mine = buf[lane];
        for (int j = 0; j < K; ++j) rank += buf[j] < mine ? 1 : 0;
    }
    return K;
}

// wave_select_packed for lanes whose KIN entries are each SORTED ascending (empties last): U =
// the kout-th smallest of the lanes' H leading entries bounds the answer (kout distinct entries
// are <= it), so only each lane's prefix <= U competes — typically a few dozen entries for
// kout = 16 with H = 1, ~100 for kout = 64 with H = 2 — ranked against each other by broadcast
// LDS reads instead of the 32+ dependent wave-sum steps of the bit-by-bit select.  buf: this
// wave's LDS, 64 H + CAP entries (>= 64).  Falls back to wave_select_packed when the survivors
// exceed CAP or fewer than kout leading entries are valid.  Same result as wave_select_packed
// (the K smallest, distinct); lane < K: mine = the rank-lane value, rank = lane.
template <int KIN, int H, int CAP>
__device__ __forceinline__ int wave_select_sorted(const uint64_t (&v)[KIN], int kout, uint64_t* buf,
                                                  uint64_t& mine, int& rank) {
    static_assert(H >= 1 && H <= KIN && 64 * H + CAP >= 64, "bound entries");
    constexpr uint64_t kEmpty = ~0ull;
    const int lane = (int)(threadIdx.x & 63);
    uint64_t* const lead = buf;               // 64 H leading entries, later the K sorted outputs
    uint64_t* const surv = buf + 64 * H;      // <= CAP survivors
    int nl = 0;
#pragma unroll
    for (int p = 0; p < H; ++p) nl += v[p] != kEmpty ? 1 : 0;
    const int nlead = wave_sum_i32(nl);
    if (kout <= 0 || nlead < kout) return wave_select_packed<KIN>(v, kout, buf, mine, rank);
#pragma unroll
    for (int p = 0; p < H; ++p) lead[p * 64 + lane] = v[p];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int rl[H];
#pragma unroll
    for (int p = 0; p < H; ++p) rl[p] = 0;
#pragma unroll 8
    for (int j = 0; j < 64 * H; ++j) {
        const uint64_t x = lead[j];
#pragma unroll
        for (int p = 0; p < H; ++p) rl[p] += x < v[p] ? 1 : 0;
    }
    // exactly one valid leading entry has rank kout - 1 (valid entries are distinct)
    int ul = 0, up = 0;
#pragma unroll
    for (int p = 0; p < H; ++p) {
        const uint64_t hit = __ballot(v[p] != kEmpty && rl[p] == kout - 1);
        if (hit) { ul = (int)__builtin_ctzll(hit); up = p; }
    }
    const uint64_t lu = lead[up * 64 + ul];
    const uint64_t U = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lu >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lu);
    int c = 0;
#pragma unroll
    for (int p = 0; p < KIN; ++p) c += v[p] <= U ? 1 : 0;
    const int C = wave_sum_i32(c);
    if (C > CAP) {
        __builtin_amdgcn_wave_barrier();
        return wave_select_packed<KIN>(v, kout, buf, mine, rank);
    }
    const int base = wave_excl_scan_i32(c);
#pragma unroll
    for (int p = 0; p < KIN; ++p)
        if (p < c) surv[base + p] = v[p];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // every survivor is a valid entry (<= U < empty); exactly kout of them rank below kout
    for (int i = lane; i < C; i += 64) {
        const uint64_t x = surv[i];
        int r = 0;
        for (int j = 0; j < C; ++j) r += surv[j] < x ? 1 : 0;
        if (r < kout) lead[r] = x;            // lead[] is no longer read (kout <= 64 <= 64 H)
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    mine = lane < kout ? lead[lane] : kEmpty;
    rank = lane;
    return kout;
}

}  // namespace imgrec
