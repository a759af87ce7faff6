// Micro-benchmark: the stage loop of the 256 x 256 bf16 candidate kernel (knn_b16w.hip) alone —
// LDS-DMA ring, fragment reads, v_mfma_f32_16x16x32_bf16, one barrier per 64-deep stage, no
// top-k epilogue — for three wave geometries of the same 256-query x 256-row tile:
//   A  8 waves, each 32 queries x 256 rows  (the production kernel: 18 ds_read_b128 per 32 MFMAs)
//   B  8 waves, each 64 queries x 128 rows  (2 x 4 waves: 12 reads per 32 MFMAs)
//   C  4 waves, each 64 queries x 256 rows  (one wave per SIMD, 256 accumulators: 20 per 64)
// The question it answers: is the stage loop's loss against the MFMA floor (2466 vs 2048 cycles
// per stage in profiles/r02/b16w_stamps_packed.txt) set by the LDS traffic of the fragment reads?
// Usage: stage_loop [tiles_per_split=61] [reps=5]   (grid: 4 query blocks x 64 row splits)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kDW = 992;                  // 32-bit words per row (1984 bf16: d = 1968 padded)
constexpr int kNst = kDW / 32;            // 31 stages per tile
constexpr int kRowB = 128, kSA = 256 * kRowB, kStage = 2 * kSA;
constexpr int kNSplit = 64, kNQB = 4;

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
template <bool NT>
__device__ __forceinline__ void dma4x(const void* sbase, uint32_t lds0, uint32_t v0, uint32_t v1,
                                      uint32_t v2, uint32_t v3) {
    unsigned keep;
    if constexpr (NT)
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, %5 nt\n\t"
            "global_load_lds_dwordx4 %2, %5 offset:1024 nt\n\t"
            "global_load_lds_dwordx4 %3, %5 offset:2048 nt\n\t"
            "global_load_lds_dwordx4 %4, %5 offset:3072 nt\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0))
            : "memory");
    else
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

// NW waves; each wave: QB 16-query blocks x RB 16-row blocks of the tile
template <int NW, int QB, int RB, bool NT>
__global__ void __launch_bounds__(NW * 64, 1)
stage_loop(const uint32_t* __restrict__ xh, const uint32_t* __restrict__ qh, int tiles, float* out) {
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];
    constexpr int nWC = 16 / QB;                  // wave columns (query groups)
    constexpr int NQ = RB / 4;                    // row quads per k-step
    constexpr int L = 2 * NQ;                     // quads per stage
    constexpr int kLPW = 64 / NW;                 // 1-KiB DMA pieces per wave per stage
    static_assert(nWC * (16 / RB) == NW && kLPW % 4 == 0, "geometry");
    const int wg = blockIdx.x;
    const int split = wg % kNSplit, qb = wg / kNSplit;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wc = wave % nWC, wr = wave / nWC;
    const int lc = lane & 15, lq = lane >> 4;

    const bool isA = wave < NW / 2;
    const int pbase = (isA ? wave : wave - NW / 2) * kLPW;
    const int prow = lane / 8, pchk = lane % 8;
    uint32_t vpar[2];
    for (int e = 0; e < 2; ++e) {
        const int r = (pbase + e) * 8 + prow;
        vpar[e] = (uint32_t)r * (uint32_t)(kDW * 4) + 16u * (uint32_t)(pchk ^ ((r >> 1) & 7));
    }
    const uint32_t kPS = 8u * kDW * 4;
    auto voff_of = [&](int j) { return vpar[j & 1] + (uint32_t)(j & ~1) * kPS - 1024u * (uint32_t)(j & 3); };
    const uint32_t smem0 = lds_u32(smem);
    const uint32_t pdst = (uint32_t)((isA ? 0 : kSA) + pbase * 1024);
    const uint32_t* qblk = qh + (size_t)qb * 256 * kDW;
    const int total = tiles * kNst;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const int t = g / kNst, s = g - t * kNst;
        const uint32_t* src = (isA ? xh + (size_t)(t * kNSplit + split) * 256 * kDW : qblk) + s * 32;
        const uint32_t dst = smem0 + (uint32_t)((g & 1) * kStage) + pdst;
#pragma unroll
        for (int h = 0; h < kLPW / 4; ++h)
            if (isA) dma4x<NT>(src, dst + 4096u * h, voff_of(4 * h), voff_of(4 * h + 1), voff_of(4 * h + 2), voff_of(4 * h + 3));
            else dma4x<false>(src, dst + 4096u * h, voff_of(4 * h), voff_of(4 * h + 1), voff_of(4 * h + 2), voff_of(4 * h + 3));
    };

    const int fsw = (lc >> 1) & 7;
    int aoff[2];
    for (int c = 0; c < 2; ++c) aoff[c] = lc * kRowB + 16 * ((4 * c + lq) ^ fsw);
    const int arow0 = wr * RB * 16 * kRowB, brow0 = kSA + wc * QB * 16 * kRowB;

    auto read_a = [&](const char* sb, int i, u32x4 (&fa)[4]) __attribute__((always_inline)) {
        const int c = i / NQ, rq = i % NQ;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fa[j] = *reinterpret_cast<const u32x4*>(sb + arow0 + aoff[c] + (4 * rq + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[QB]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < QB; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + brow0 + aoff[c] + h * 16 * kRowB);
    };
    f32x4 acc[RB][QB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int h = 0; h < QB; ++h) acc[r][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto mfma_quad = [&](const u32x4 (&fa)[4], const u32x4 (&fb)[QB], int i) __attribute__((always_inline)) {
        const int rq = i % NQ;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < QB; ++h)
                acc[4 * rq + j][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, fa[j]), __builtin_bit_cast(bf16x8, fb[h]), acc[4 * rq + j][h], 0, 0, 0);
    };

    u32x4 fa[2][4], fb[2][QB];
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (total > 1) issue(1);
    read_a(smem, 0, fa[0]);
    read_b(smem, 0, fb[0]);
    for (int g = 0; g < total; ++g) {
        const char* sb = smem + (g & 1) * kStage;
#pragma unroll
        for (int i = 0; i + 1 < L; ++i) {
            read_a(sb, i + 1, fa[(i + 1) & 1]);
            if (i == NQ - 1) read_b(sb, 1, fb[1]);
            mfma_quad(fa[i & 1], fb[i / NQ], i);
            constexpr int nmf = 4 * QB;
            const int nrd = 4 + (i == NQ - 1 ? QB : 0);
#pragma unroll
            for (int j = 0; j < nmf; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (j < nrd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (g + 1 < total) {
            const char* nb = smem + ((g + 1) & 1) * kStage;
            read_a(nb, 0, fa[0]);
            read_b(nb, 0, fb[0]);
        }
        if (g + 2 < total) issue(g + 2);
        mfma_quad(fa[(L - 1) & 1], fb[1], L - 1);
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int h = 0; h < QB; ++h) s += acc[r][h][0] + acc[r][h][1] + acc[r][h][2] + acc[r][h][3];
    out[blockIdx.x * NW * 64 + threadIdx.x] = s;
}

__global__ void fill_bf16(uint32_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        // two bf16 of magnitude in [2^-8, 2^-5), random sign and mantissa
        const uint32_t a = ((h & 0x8000u) | ((0x77u + ((h >> 8) & 3u)) << 7) | (h & 0x7fu));
        const uint32_t b = (((h >> 16) & 0x8000u) | ((0x77u + ((h >> 24) & 3u)) << 7) | ((h >> 17) & 0x7fu));
        p[i] = a | (b << 16);
    }
}

template <int NW, int QB, int RB, bool NT = false>
void run(const char* name, const uint32_t* xh, const uint32_t* qh, float* out, int tiles, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(kNSplit * kNQB), block(NW * 64);
    hipLaunchKernelGGL((stage_loop<NW, QB, RB, NT>), grid, block, 0, 0, xh, qh, tiles, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((stage_loop<NW, QB, RB, NT>), grid, block, 0, 0, xh, qh, tiles, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double flop = 2.0 * kNSplit * tiles * 256.0 * 1024.0 * 32.0 * 2 * kNst;
    printf("{\"geometry\": \"%s\", \"waves\": %d, \"tiles_per_split\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
           "\"tflops\": %.1f, \"ns_per_stage\": %.1f}\n", name, NW, tiles, best, sum / reps,
           flop / (best * 1e-3) / 1e12, best * 1e6 / (tiles * kNst));
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
    for (int pass = 0; pass < 2; ++pass) {
        run<8, 2, 16>("A 8w 32q x 256r", xh, qh, out, tiles, reps);
        run<8, 2, 16, true>("A 8w 32q x 256r, corpus nt", xh, qh, out, tiles, reps);
        run<8, 4, 8>("B 8w 64q x 128r", xh, qh, out, tiles, reps);
        run<8, 4, 8, true>("B 8w 64q x 128r, corpus nt", xh, qh, out, tiles, reps);
    }
    CK(hipFree(xh));
    CK(hipFree(qh));
    CK(hipFree(out));
    return 0;
}
