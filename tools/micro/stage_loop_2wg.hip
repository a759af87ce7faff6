// Micro-benchmark (round 5): can a SECOND workgroup per CU hide the bf16 candidate kernel's
// per-tile top-k epilogue?
//
// knn_b16w.hip runs one 8-wave workgroup per CU (256 rows x 256 queries, 64-deep stages, two-slot
// ring of 64 KiB): at every tile end all eight waves run their epilogue (~12k cycles) while the
// matrix pipes idle — 28 % of the kernel at 1M x 768.  Two independent 4-wave workgroups per CU
// (256 rows x 128 queries each) have separate barriers, so one can run its epilogue while the
// other's stages keep the SIMDs' matrix pipes fed.  The LDS budget forces 32-deep stages for that
// (2 workgroups x 2 slots x (256 + 128 rows) x 64 B = 96 KiB).
//
// Variants, each with a synthetic epilogue of E dependent list insertions per wave per tile
// (E = 0 / 64 / 192; the real epilogue is ~12k cycles, ~12 iterations of a latency-bound loop):
//   L    the production form: 8 waves, 256 x 256, 64-deep stages
//   P    two 4-wave workgroups per CU, 256 x 128 each, 32-deep stages
//   PS   P with the second workgroup of a CU starting half a tile later (a half-depth first tile),
//        so the two workgroups' epilogues alternate
// Usage: stage_loop_2wg [tiles_per_split=61] [reps=5] [dw=992]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kNSplit = 64;

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void dma1(const void* sbase, uint32_t lds0, uint32_t v) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(v), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0)) : "memory");
}
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));
}
__device__ __forceinline__ void insert10(uint32_t (&kp)[10], uint32_t u) {
#pragma unroll
    for (int p = 9; p > 0; --p) kp[p] = umed3(kp[p - 1], u, kp[p]);
    kp[0] = min(kp[0], u);
}
__device__ __forceinline__ void epilogue(int E, uint32_t (&kp)[10], uint32_t& seed, const f32x4& a) {
    seed ^= __float_as_uint(a[0]);
#pragma unroll 1
    for (int i = 0; i < E; ++i) {
        seed = seed * 1664525u + 1013904223u;
        insert10(kp, seed >> 4);
    }
}

// NW waves x 32 queries, 256-row tiles, stages of KW 32-bit words (KW = 32: 64 deep, 16: 32 deep)
// of both operands in a two-slot ring; SHIFT: workgroups of the second dispatch round (blockIdx
// >= 256) start with a half-depth tile.
template <int NW, int KW, bool SHIFT>
__global__ void __launch_bounds__(NW * 64, 2)
loop_kernel(const uint32_t* __restrict__ xh, const uint32_t* __restrict__ qh, int tiles, int dw,
            int E, float* out) {
    constexpr int kBQ = NW * 32, kRowB = KW * 4, kCPR = KW / 4;     // chunks per staged row
    constexpr int kRPP = 64 / kCPR;                                 // rows per 1-KiB piece
    constexpr int kSA = 256 * kRowB, kSB = kBQ * kRowB, kStage = kSA + kSB;
    constexpr int kPieces = (256 + kBQ) / kRPP, kLPW = kPieces / NW;
    constexpr int KS = KW / 16;                                     // 32-deep k-steps per stage
    constexpr int L = 4 * KS;                                       // quads per stage
    static_assert(kPieces % NW == 0, "pieces");
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];

    const int nqb = 1024 / kBQ;
    const int wg = blockIdx.x;
    const int split = wg % kNSplit, qb = wg / kNSplit;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lc = lane & 15, lq = lane >> 4;
    if (NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
    const int nst = dw / KW;
    const bool half = SHIFT && blockIdx.x >= 256;
    const int total = tiles * nst - (half ? nst / 2 : 0);

    // swizzle of a staged row: 64-deep rows (8 chunks) chunk ^ ((r >> 1) & 7) as knn_b16w; 32-deep
    // rows (4 chunks) chunk ^ f((r >> 2) & 3), f = {0, 2, 3, 1}: the ds_read_b128 lane groups of
    // a 16 x 16 x 32 fragment read then hit 16 distinct (r mod 4, chunk) pairs = 64 banks
    auto sw = [](int r) { return KW == 32 ? ((r >> 1) & 7) : ((0x78 >> (2 * ((r >> 2) & 3))) & 3); };
    const int pbase = wave * kLPW;
    const int prow = lane / kCPR, pchk = lane % kCPR;
    const uint32_t smem0 = lds_u32(smem);
    const uint32_t* qblk = qh + (size_t)qb * kBQ * dw;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const int gg = g + (half ? nst / 2 : 0);
        const int t = gg / nst, s = gg - t * nst;
        const uint32_t dst0 = smem0 + (uint32_t)((g & 1) * kStage);
#pragma unroll
        for (int j = 0; j < kLPW; ++j) {
            const int P = pbase + j, r = P * kRPP + prow;               // LDS image row
            const bool corpus = P * kRPP < 256;                          // (uniform: pieces never straddle)
            const int srow = corpus ? r : r - 256;
            const uint32_t* src = (corpus ? xh + (size_t)(t * kNSplit + split) * 256 * dw : qblk) + s * KW;
            const uint32_t v = (uint32_t)srow * (uint32_t)(dw * 4) + 16u * (uint32_t)(pchk ^ sw(r));
            dma1(src, dst0 + P * 1024, v);
        }
    };
    // fragment offsets: k-step c of lane quarter lq reads logical chunk 4c + lq (64 deep) or lq
    // (32 deep) of row lc of a 16-row block
    auto foff = [&](int c) { return lc * kRowB + 16 * ((KW == 32 ? 4 * c + lq : lq) ^ sw(lc)); };
    const int boff = kSA + wave * 32 * kRowB;
    auto read_a = [&](const char* sb, int i, u32x4 (&fa)[4]) __attribute__((always_inline)) {
        const int c = i / 4, rq = i % 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) fa[j] = *reinterpret_cast<const u32x4*>(sb + foff(c) + (4 * rq + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + foff(c) + boff + h * 16 * kRowB);
    };
    f32x4 acc[16][2];
    auto mfma_quad = [&](const u32x4 (&fa)[4], const u32x4 (&fb)[2], int i) __attribute__((always_inline)) {
        const int rq = i % 4;
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

    u32x4 fa[2][4], fb[2][2];
    issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (total > 1) issue(1);
    read_a(smem, 0, fa[0]);
    read_b(smem, 0, fb[0]);
    int g = 0;
    int s_in_tile = half ? nst / 2 : 0;
#pragma unroll
    for (int rb = 0; rb < 16; ++rb)
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[rb][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (; g < total; ++g) {
        const char* sb = smem + (g & 1) * kStage;
#pragma unroll
        for (int i = 0; i + 1 < L; ++i) {
            read_a(sb, i + 1, fa[(i + 1) & 1]);
            if (KS == 2 && i == 3) read_b(sb, 1, fb[1]);
            mfma_quad(fa[i & 1], fb[i / 4], i);
            const int nrd = 4 + (KS == 2 && i == 3 ? 2 : 0);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
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
        u32x4 fl[2];
        fl[0] = fb[KS - 1][0];
        fl[1] = fb[KS - 1][1];
        if (g + 1 < total) {
            const char* nb = smem + ((g + 1) & 1) * kStage;
            read_a(nb, 0, fa[0]);
            read_b(nb, 0, fb[0]);
        }
        if (g + 2 < total) issue(g + 2);
        mfma_quad(fa[(L - 1) & 1], fl, L - 1);
        if (++s_in_tile == nst) {               // tile end: the synthetic epilogue, then reset
            s_in_tile = 0;
            epilogue(E, kp, seed, acc[0][0]);
#pragma unroll
            for (int rb = 0; rb < 16; ++rb)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    seed += __float_as_uint(acc[rb][h][1]);
                    acc[rb][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
                }
        }
    }
    float s = (float)(seed & 1u);
#pragma unroll
    for (int p = 0; p < 10; ++p) s += (float)(kp[p] & 1u);
    out[blockIdx.x * NW * 64 + threadIdx.x] = s;
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

template <int NW, int KW, bool SHIFT>
void run(const char* name, const uint32_t* xh, const uint32_t* qh, float* out, int tiles, int reps, int dw, int E) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(kNSplit * (1024 / (NW * 32))), block(NW * 64);
    hipLaunchKernelGGL((loop_kernel<NW, KW, SHIFT>), grid, block, 0, 0, xh, qh, tiles, dw, E, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((loop_kernel<NW, KW, SHIFT>), grid, block, 0, 0, xh, qh, tiles, dw, E, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double flop = 2.0 * kNSplit * tiles * 256.0 * 1024.0 * 64.0 * (dw / 32);
    printf("{\"variant\": \"%s\", \"epilogue_insertions\": %d, \"dw\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
           "\"tflops\": %.1f, \"frac_bf16_peak\": %.3f}\n", name, E, dw, best, sum / reps,
           flop / (best * 1e-3) / 1e12, flop / (best * 1e-3) / 2516.8e12);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 61;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int dw = argc > 3 ? atoi(argv[3]) : 992;
    const size_t nx = (size_t)kNSplit * tiles * 256 * dw, nqw = (size_t)1024 * dw;
    uint32_t *xh, *qh;
    float* out;
    CK(hipMalloc(&xh, nx * 4));
    CK(hipMalloc(&qh, nqw * 4));
    CK(hipMalloc(&out, (size_t)kNSplit * 8 * 256 * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, xh, nx, 0x1234u);
    hipLaunchKernelGGL(fill_bf16, dim3(512), dim3(256), 0, 0, qh, nqw, 0x9876u);
    CK(hipDeviceSynchronize());
    for (int pass = 0; pass < 2; ++pass)
        for (int E : {0, 64, 192}) {
            run<8, 32, false>("L 8w 256x256 64-deep", xh, qh, out, tiles, reps, dw, E);
            run<4, 16, false>("P 2x4w 256x128 32-deep", xh, qh, out, tiles, reps, dw, E);
            run<4, 16, true>("PS shifted", xh, qh, out, tiles, reps, dw, E);
        }
    CK(hipFree(xh));
    CK(hipFree(qh));
    CK(hipFree(out));
    return 0;
}
