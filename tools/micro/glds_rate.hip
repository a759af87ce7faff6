// Micro-benchmark: sustained global -> LDS rate of global_load_lds_dwordx4 per CU, as used by the
// 256 x 256 bf16 candidate kernel (1-KiB pieces of 8 rows x 128 B, rows `stride` bytes apart,
// four pieces per M0 write), for several numbers of pieces kept in flight per wave.
// One 8-wave workgroup per CU; the LDS ring is overwritten freely (rate only, data unused).
// Usage: glds_rate [span_MiB] [stride_bytes]   (span: bytes each workgroup cycles through)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

template <int INF>
__global__ void __launch_bounds__(512) rate(const char* src, long span_rows, int stride, int iters) {
    __shared__ __attribute__((aligned(16))) char sm[128 * 1024];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int prow = lane / 8, pchk = lane % 8;
    uint32_t v[4];
    for (int j = 0; j < 4; ++j) v[j] = (uint32_t)((j * 8 + prow) * stride + pchk * 16 - 1024 * j);
    const uint32_t lds = lds_u32(sm) + wave * 16384;
    long row = ((long)blockIdx.x * 8 + wave) * 32;
    for (int it = 0; it < iters; ++it) {
        const char* base = src + (row % span_rows) * stride;
        row += 8 * 32;                                   // the workgroup's 8 waves x 32 rows
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, %5\n\t"
            "global_load_lds_dwordx4 %2, %5 offset:1024\n\t"
            "global_load_lds_dwordx4 %3, %5 offset:2048\n\t"
            "global_load_lds_dwordx4 %4, %5 offset:3072\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "s"(base),
              "s"(__builtin_amdgcn_readfirstlane(lds + (it & 3) * 4096))
            : "memory");
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int INF>
void run(const char* d, long span_rows, int stride, int cus) {
    const int iters = 4096;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(rate<INF>, cus, 512, 0, 0, d, span_rows, stride, 64);
    hipEventRecord(a);
    hipLaunchKernelGGL(rate<INF>, cus, 512, 0, 0, d, span_rows, stride, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)cus * 8 * iters * 4096;
    printf("in-flight %2d pieces/wave (%3d KiB/CU): %.3f ms, %.1f GB/s per CU, %.1f TB/s total\n",
           INF + 4, (INF + 4) * 8, ms, bytes / cus / (ms * 1e6), bytes / (ms * 1e9));
}

int main(int argc, char** argv) {
    const long span_mib = argc > 1 ? atol(argv[1]) : 64;
    const int stride = argc > 2 ? atoi(argv[2]) : 3968;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const long span_rows = span_mib * 1024 * 1024 / stride / 256 * 256;
    char* d;
    if (hipMalloc(&d, (size_t)(span_rows + 512) * stride) != hipSuccess) return 1;
    hipMemset(d, 1, (size_t)(span_rows + 512) * stride);
    printf("%d CUs, span %ld MiB (%ld rows of %d B)\n", cus, span_mib, span_rows, stride);
    run<0>(d, span_rows, stride, cus);
    run<4>(d, span_rows, stride, cus);
    run<8>(d, span_rows, stride, cus);
    run<12>(d, span_rows, stride, cus);
    run<20>(d, span_rows, stride, cus);
    run<28>(d, span_rows, stride, cus);
    hipFree(d);
    return 0;
}
