// Micro-benchmark (round 6): LDS read bytes per MFMA in the bf16 candidate kernel's stage loop.
//
// knn_b16w.hip gives each of its 8 waves 32 queries x all 256 rows of the tile: per 32-deep
// k-step a wave reads 16 A fragments (one per 16-row block) and 2 B fragments for 32 MFMAs, so a
// stage (2 k-steps) reads 36 KiB of LDS per wave, 288 KiB per workgroup, for 64 KiB staged.  The
// guide ranks "fewer LDS read bytes" among what lowers the energy per MFMA and so raises the clock
// a power-capped MFMA loop holds (cdna_hip_programming.md 5.4 rule 28).
//   L  the production geometry: wave = 32 queries x 256 rows (36 ds_read_b128 per 64 MFMAs)
//   W  wave = 64 queries x 128 rows (2 row halves x 4 query quarters): 8 A + 4 B fragments per
//      k-step, 24 ds_read_b128 per 64 MFMAs (-33 % LDS read bytes), same 128 accumulators
//   V  wave = 128 queries x 64 rows (4 row quarters x 2 query halves): 4 A + 8 B, also 24
// Same LDS image, swizzle, DMA schedule and barrier placement in all three; random bf16 operands.
// Usage: stage_loop_w [tiles_per_split=61] [reps=5] [passes=3]
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
constexpr int kSA = 256 * kRowB, kSB = 256 * kRowB, kStage = kSA + kSB;
constexpr int kLPW = 512 / 8 / 8;         // 1-KiB DMA pieces per wave per stage

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

// RBW: 16-row blocks per wave (16 = L, 8 = W, 4 = V); QBW = 32 / RBW * 2 ... query blocks per
// wave such that RBW * QBW = 32 (128 accumulator registers).  A group = 2 row blocks x QBW query
// blocks; 2 k-steps x RBW / 2 groups per stage.
template <int RBW>
__global__ void __launch_bounds__(512, 2)
stage_loop_w(const uint32_t* __restrict__ xh, const uint32_t* __restrict__ qh, int tiles, float* out) {
    constexpr int QBW = 32 / RBW;             // 16-query blocks per wave
    constexpr int NWR = 16 / RBW;             // waves along the rows
    constexpr int GPK = RBW / 2;              // groups per k-step
    constexpr int NG = 2 * GPK;               // groups per stage
    constexpr int MPG = 2 * QBW;              // MFMAs per group
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];

    const int wg = blockIdx.x;
    const int split = wg % kNSplit, qb = wg / kNSplit;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lc = lane & 15, lq = lane >> 4;
    const int wr = wave % NWR, wq = wave / NWR;
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);

    const int pbase = wave * kLPW;
    const int prow = lane / 8, pchk = lane % 8;
    uint32_t voff[kLPW];
    const uint32_t* qblk = qh + (size_t)qb * 256 * kDW;
#pragma unroll
    for (int j = 0; j < kLPW; ++j) {
        const int P = pbase + j, r = P * 8 + prow;
        const int srow = r < 256 ? r : r - 256;
        voff[j] = (uint32_t)srow * (uint32_t)(kDW * 4) + 16u * (uint32_t)(pchk ^ ((r >> 1) & 7));
    }
    const uint32_t smem0 = lds_u32(smem);
    const int total = tiles * kNst;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const int t = g / kNst, s = g - t * kNst;
        const uint32_t dst = smem0 + (uint32_t)((g & 1) * kStage) + (uint32_t)(pbase * 1024);
        const bool corpus = pbase * 8 < 256;
        const uint32_t* src = (corpus ? xh + (size_t)(t * kNSplit + split) * 256 * kDW : qblk) + s * 32;
#pragma unroll
        for (int h = 0; h < kLPW / 4; ++h)
            dma4x(src, dst + 4096u * h, voff[4 * h], voff[4 * h + 1] - 1024u, voff[4 * h + 2] - 2048u,
                  voff[4 * h + 3] - 3072u);
    };

    const int fsw = (lc >> 1) & 7;
    int aoff[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) aoff[c] = lc * kRowB + 16 * ((4 * c + lq) ^ fsw);
    const int arow0 = wr * RBW;               // first row block of this wave
    const int boff = kSA + wq * QBW * 16 * kRowB;

    // group i: k-step i / GPK, row blocks arow0 + 2 (i % GPK), + 1
    auto read_a = [&](const char* sb, int i, u32x4 (&fa)[2]) __attribute__((always_inline)) {
        const int c = i / GPK, rp = i % GPK;
#pragma unroll
        for (int j = 0; j < 2; ++j) fa[j] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + (arow0 + 2 * rp + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[QBW]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < QBW; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + boff + h * 16 * kRowB);
    };

    f32x4 acc[RBW][QBW];
#pragma unroll
    for (int r = 0; r < RBW; ++r)
#pragma unroll
        for (int h = 0; h < QBW; ++h) acc[r][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto mfma_group = [&](const u32x4 (&fa)[2], const u32x4 (&fb)[QBW], int i) __attribute__((always_inline)) {
        const int rp = i % GPK;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int h = 0; h < QBW; ++h)
                acc[2 * rp + j][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, fa[j]), __builtin_bit_cast(bf16x8, fb[h]), acc[2 * rp + j][h], 0, 0, 0);
    };

    u32x4 fa[2][2], fb[2][QBW];
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (total > 1) issue(1);
    read_a(smem, 0, fa[0]);
    read_b(smem, 0, fb[0]);
    for (int g = 0; g < total; ++g) {
        const char* sb = smem + (g & 1) * kStage;
#pragma unroll
        for (int i = 0; i + 1 < NG; ++i) {
            read_a(sb, i + 1, fa[(i + 1) & 1]);
            const bool nb = (i + 1) % GPK == 0;        // next group starts k-step 1
            if (nb) read_b(sb, 1, fb[1]);
            mfma_group(fa[i & 1], fb[i / GPK], i);
            const int nrd = 2 + (nb ? QBW : 0);
#pragma unroll
            for (int j = 0; j < MPG; ++j) {
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
        u32x4 fl[QBW], fal[2];
#pragma unroll
        for (int h = 0; h < QBW; ++h) fl[h] = fb[1][h];
        fal[0] = fa[(NG - 1) & 1][0];
        fal[1] = fa[(NG - 1) & 1][1];
        if (g + 1 < total) {
            const char* nbp = smem + ((g + 1) & 1) * kStage;
            read_a(nbp, 0, fa[0]);
            read_b(nbp, 0, fb[0]);
        }
        if (g + 2 < total) issue(g + 2);
        mfma_group(fal, fl, NG - 1);
    }
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RBW; ++r)
#pragma unroll
        for (int h = 0; h < QBW; ++h) s += acc[r][h][0] + acc[r][h][1] + acc[r][h][2] + acc[r][h][3];
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

template <int RBW>
void run(const char* name, const uint32_t* xh, const uint32_t* qh, float* out, int tiles, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(kNSplit * kNQB), block(512);
    hipLaunchKernelGGL((stage_loop_w<RBW>), grid, block, 0, 0, xh, qh, tiles, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((stage_loop_w<RBW>), grid, block, 0, 0, xh, qh, tiles, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double flop = 2.0 * kNSplit * tiles * 256.0 * 1024.0 * 32.0 * 2 * kNst;
    printf("{\"variant\": \"%s\", \"rows_per_wave\": %d, \"queries_per_wave\": %d, "
           "\"ds_read_b128_per_64_mfma\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, \"tflops\": %.1f, "
           "\"frac_bf16_peak\": %.3f}\n",
           name, RBW * 16, 512 / RBW, 2 * (RBW + 32 / RBW), best, sum / reps,
           flop / (best * 1e-3) / 1e12, flop / (best * 1e-3) / 2516.8e12);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 61;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int passes = argc > 3 ? atoi(argv[3]) : 3;
    const size_t nx = (size_t)kNSplit * tiles * 256 * kDW, nqw = (size_t)kNQB * 256 * kDW;
    uint32_t *xh, *qh;
    float* out;
    CK(hipMalloc(&xh, nx * 4));
    CK(hipMalloc(&qh, nqw * 4));
    CK(hipMalloc(&out, (size_t)kNSplit * kNQB * 512 * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, xh, nx, 0x1234u);
    hipLaunchKernelGGL(fill_bf16, dim3(512), dim3(256), 0, 0, qh, nqw, 0x9876u);
    CK(hipDeviceSynchronize());
    for (int pass = 0; pass < passes; ++pass) {
        run<16>("L 32q x 256r", xh, qh, out, tiles, reps);
        run<8>("W 64q x 128r", xh, qh, out, tiles, reps);
        run<4>("V 128q x 64r", xh, qh, out, tiles, reps);
    }
    CK(hipFree(xh));
    CK(hipFree(qh));
    CK(hipFree(out));
    return 0;
}
