// Micro-benchmark (round 5): the stage loop of the bf16 candidate kernel with the QUERY operand
// taken straight from global memory into registers instead of through the LDS ring.
//
// In knn_b16w.hip every wave multiplies its own 32 queries against all 256 rows of the tile, so
// the query block in LDS is never shared between waves: the B fragments can be loaded by each
// wave for itself (global_load_dwordx4 of a fragment-native copy of the queries, 1 KiB per
// fragment, fully coalesced), the LDS ring then holds the corpus tile only (half the DMA writes
// into LDS, no B-fragment ds_reads).  Geometries, all 8 waves x 32 queries each:
//   L   the production form: B through LDS, 256-row tile (reference point)
//   G   B from global, 256-row tile, the next stage's 4 B fragments prefetched (32 VGPRs)
//   H   B from global, 128-row tile (8 row blocks: half the accumulators, so two accumulator
//       sets fit where one did — the form that lets a tile's top-k overlap the next tile's MFMAs)
// Each can run with a synthetic "epilogue slice" per stage (S dependent insertions of a packed
// value into a 10-entry register list, v_med3_u32 per slot) placed either in every wave at the
// same point (no stagger) or at the start of the stage in waves 0-3 and at its end in waves 4-7
// (stagger): how much VALU work per stage hides under the partner wave's MFMAs.
// Usage: stage_loop_g [tiles_per_split_256=61] [reps=5]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kDW = 992;                  // 32-bit words per row (1984 bf16)
constexpr int kNst = kDW / 32;            // 31 stages (64 bf16 deep) per tile
constexpr int kRowB = 128;
constexpr int kNSplit = 64, kNQB = 4;

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
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
__device__ __forceinline__ void dma2x(const void* sbase, uint32_t lds0, uint32_t v0, uint32_t v1) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %3\n\t"
        "global_load_lds_dwordx4 %2, %3 offset:1024\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v0), "v"(v1), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0))
        : "memory");
}

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));
}
template <int K>
__device__ __forceinline__ void insert_packed(uint32_t (&kp)[K], uint32_t u) {
#pragma unroll
    for (int p = K - 1; p > 0; --p) kp[p] = umed3(kp[p - 1], u, kp[p]);
    kp[0] = min(kp[0], u);
}
// S dependent insertions (the synthetic epilogue slice)
template <int S>
__device__ __forceinline__ void slice(uint32_t (&kp)[10], uint32_t& seed) {
#pragma unroll 1
    for (int i = 0; i < S; ++i) {
        seed = seed * 1664525u + 1013904223u;
        insert_packed<10>(kp, seed >> 4);
    }
}

// BG: B operand from global (fragment-native query copy); RB: 16-row blocks per tile (16 or 8);
// S: slice insertions per stage; STAG: stagger the slice (waves 0-3 first, waves 4-7 last)
template <bool BG, int RB, int S, bool STAG>
__global__ void __launch_bounds__(512, 2)
stage_loop_g(const uint32_t* __restrict__ xh, const uint32_t* __restrict__ qh,
             const u32x4* __restrict__ qf, int tiles, float* out) {
    constexpr int kTR = RB * 16;                        // tile rows
    constexpr int kSA = kTR * kRowB;                    // corpus stage bytes
    constexpr int kSB = BG ? 0 : 256 * kRowB;           // query stage bytes
    constexpr int kStage = kSA + kSB;
    constexpr int kPieces = (kTR + (BG ? 0 : 256)) / 8; // 1-KiB DMA pieces per stage
    constexpr int kLPW = kPieces / 8;                   // per wave (every wave issues)
    constexpr int NR = RB / 4;                          // row quads per k-step
    constexpr int L = 2 * NR;                           // quads per stage
    static_assert(kLPW == 2 || kLPW % 4 == 0, "pieces per wave");
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];

    const int wg = blockIdx.x;
    const int split = wg % kNSplit, qb = wg / kNSplit;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lc = lane & 15, lq = lane >> 4;
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);

    // every wave issues kLPW pieces: pieces wave*kLPW .. ; piece P < kTR/8 is a corpus piece
    const int pbase = wave * kLPW;
    const int prow = lane / 8, pchk = lane % 8;
    uint32_t voff[kLPW];
    const uint32_t* qblk = qh + (size_t)qb * 256 * kDW;
#pragma unroll
    for (int j = 0; j < kLPW; ++j) {
        const int P = pbase + j, r = P * 8 + prow;          // LDS image row (corpus rows first)
        const int srow = r < kTR ? r : r - kTR;             // source row in its tile
        voff[j] = (uint32_t)srow * (uint32_t)(kDW * 4) + 16u * (uint32_t)(pchk ^ ((r >> 1) & 7));
    }
    const uint32_t smem0 = lds_u32(smem);
    const int total = tiles * kNst;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const int t = g / kNst, s = g - t * kNst;
        const uint32_t dst = smem0 + (uint32_t)((g & 1) * kStage) + (uint32_t)(pbase * 1024);
        const bool corpus = pbase * 8 < kTR;
        const uint32_t* src = (corpus ? xh + (size_t)(t * kNSplit + split) * kTR * kDW : qblk) + s * 32;
        if constexpr (kLPW == 2) {
            dma2x(src, dst, voff[0], voff[1] - 1024u);
        } else {
#pragma unroll
            for (int h = 0; h < kLPW / 4; ++h)
                dma4x(src, dst + 4096u * h, voff[4 * h], voff[4 * h + 1] - 1024u, voff[4 * h + 2] - 2048u,
                      voff[4 * h + 3] - 3072u);
        }
    };

    const int fsw = (lc >> 1) & 7;
    int aoff[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) aoff[c] = lc * kRowB + 16 * ((4 * c + lq) ^ fsw);
    const int boff = kSA + wave * 32 * kRowB;

    auto read_a = [&](const char* sb, int i, u32x4 (&fa)[4]) __attribute__((always_inline)) {
        const int c = i / NR, rq = i % NR;
#pragma unroll
        for (int j = 0; j < 4; ++j) fa[j] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + (4 * rq + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + boff + h * 16 * kRowB);
    };
    // fragment-native query copy: [qb][wave][stage][k-step][h][lane]
    const u32x4* qw = qf + (size_t)(qb * 8 + wave) * kNst * 4 * 64 + lane;
    auto load_b = [&](int g, u32x4 (&fb)[2][2]) __attribute__((always_inline)) {
        const int s = g % kNst;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) fb[c][h] = qw[(s * 4 + c * 2 + h) * 64];
    };

    f32x4 acc[RB][2];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[r][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto mfma_quad = [&](const u32x4 (&fa)[4], const u32x4 (&fb)[2], int i) __attribute__((always_inline)) {
        const int rq = i % NR;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                acc[4 * rq + j][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, fa[j]), __builtin_bit_cast(bf16x8, fb[h]), acc[4 * rq + j][h], 0, 0, 0);
    };

    uint32_t kp[10];
#pragma unroll
    for (int p = 0; p < 10; ++p) kp[p] = ~0u;
    uint32_t seed = threadIdx.x * 7919u + blockIdx.x;

    u32x4 fa[2][4], fb[2][2], fbn[2][2];
    issue(0);
    if constexpr (BG) load_b(0, fb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (total > 1) issue(1);
    if constexpr (BG) { if (total > 1) load_b(1, fbn); }
    read_a(smem, 0, fa[0]);
    if constexpr (!BG) read_b(smem, 0, fb[0]);
    for (int g = 0; g < total; ++g) {
        const char* sb = smem + (g & 1) * kStage;
        if constexpr (S > 0) { if (!STAG || wave < 4) slice<S>(kp, seed); }
#pragma unroll
        for (int i = 0; i + 1 < L; ++i) {
            read_a(sb, i + 1, fa[(i + 1) & 1]);
            if constexpr (!BG) { if (i == NR - 1) read_b(sb, 1, fb[1]); }
            mfma_quad(fa[i & 1], fb[i / NR], i);
            const int nrd = 4 + (!BG && i == NR - 1 ? 2 : 0);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (j < nrd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (S > 0) { if (STAG && wave >= 4) slice<S>(kp, seed); }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        u32x4 fl[2];
        fl[0] = fb[1][0];
        fl[1] = fb[1][1];
        if (g + 1 < total) {
            const char* nb = smem + ((g + 1) & 1) * kStage;
            read_a(nb, 0, fa[0]);
            if constexpr (BG) {
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int h = 0; h < 2; ++h) fb[c][h] = fbn[c][h];
            } else {
                read_b(nb, 0, fb[0]);
            }
        }
        if (g + 2 < total) {
            issue(g + 2);
            if constexpr (BG) load_b(g + 2, fbn);
        }
        mfma_quad(fa[(L - 1) & 1], fl, L - 1);
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int h = 0; h < 2; ++h) s += acc[r][h][0] + acc[r][h][1] + acc[r][h][2] + acc[r][h][3];
#pragma unroll
    for (int p = 0; p < 10; ++p) s += (float)(kp[p] & 1u);
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

__global__ void fill_bf16(uint32_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        const uint32_t a = ((h & 0x8000u) | ((0x77u + ((h >> 8) & 3u)) << 7) | (h & 0x7fu));
        const uint32_t b = (((h >> 16) & 0x8000u) | ((0x77u + ((h >> 24) & 3u)) << 7) | ((h >> 17) & 0x7fu));
        p[i] = a | (b << 16);
    }
}

template <bool BG, int RB, int S, bool STAG>
void run(const char* name, const uint32_t* xh, const uint32_t* qh, const u32x4* qf, float* out, int tiles256, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int tiles = tiles256 * 16 / RB;
    const dim3 grid(kNSplit * kNQB), block(512);
    hipLaunchKernelGGL((stage_loop_g<BG, RB, S, STAG>), grid, block, 0, 0, xh, qh, qf, tiles, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((stage_loop_g<BG, RB, S, STAG>), grid, block, 0, 0, xh, qh, qf, tiles, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double flop = 2.0 * kNSplit * tiles256 * 256.0 * 1024.0 * 32.0 * 2 * kNst;
    printf("{\"variant\": \"%s\", \"b_global\": %d, \"tile_rows\": %d, \"slice\": %d, \"stagger\": %d, "
           "\"best_ms\": %.4f, \"mean_ms\": %.4f, \"tflops\": %.1f, \"frac_bf16_peak\": %.3f}\n",
           name, (int)BG, RB * 16, S, (int)STAG, best, sum / reps, flop / (best * 1e-3) / 1e12,
           flop / (best * 1e-3) / 2516.8e12);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 61;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t nx = (size_t)kNSplit * tiles * 256 * kDW, nqw = (size_t)kNQB * 256 * kDW;
    uint32_t *xh, *qh;
    float* out;
    CK(hipMalloc(&xh, nx * 4));
    CK(hipMalloc(&qh, nqw * 4));
    CK(hipMalloc(&out, (size_t)kNSplit * kNQB * 512 * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, xh, nx, 0x1234u);
    hipLaunchKernelGGL(fill_bf16, dim3(512), dim3(256), 0, 0, qh, nqw, 0x9876u);
    CK(hipDeviceSynchronize());
    const u32x4* qf = reinterpret_cast<const u32x4*>(qh);   // same bytes, fragment-native order
    for (int pass = 0; pass < 2; ++pass) {
        run<false, 16, 0, false>("L lds-B 256r", xh, qh, qf, out, tiles, reps);
        run<true, 16, 0, false>("G global-B 256r", xh, qh, qf, out, tiles, reps);
        run<true, 8, 0, false>("H global-B 128r", xh, qh, qf, out, tiles, reps);
        run<false, 16, 4, false>("L slice4", xh, qh, qf, out, tiles, reps);
        run<false, 16, 4, true>("L slice4 stagger", xh, qh, qf, out, tiles, reps);
        run<true, 16, 4, false>("G slice4", xh, qh, qf, out, tiles, reps);
        run<true, 16, 4, true>("G slice4 stagger", xh, qh, qf, out, tiles, reps);
        run<true, 8, 2, false>("H slice2", xh, qh, qf, out, tiles, reps);
        run<true, 8, 2, true>("H slice2 stagger", xh, qh, qf, out, tiles, reps);
        run<true, 8, 4, true>("H slice4 stagger", xh, qh, qf, out, tiles, reps);
        run<true, 8, 8, true>("H slice8 stagger", xh, qh, qf, out, tiles, reps);
    }
    CK(hipFree(xh));
    CK(hipFree(qh));
    CK(hipFree(out));
    return 0;
}
