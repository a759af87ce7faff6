// Micro-benchmark: HBM read rate of the colour histogram's access pattern without its counting.
//   per_block  one 256-thread workgroup per 196,608-B block (one 256 x 256 RGB image), three
//              coalesced 16-B loads per thread per iteration, as color_hist16_kernel
//   per_block_4wg_per_cu  per_block held to the colour kernel's 4 workgroups per CU
//   grid       the same bytes swept grid-stride by 2048 workgroups (consecutive workgroups on
//              consecutive 12-KiB chunks: the whole grid walks memory in order)
// Each thread XOR-folds what it loads and writes one word (the loads cannot be dropped).
// Usage: stream_read [images=16384] [reps=10] [random=0]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NT = 256;
constexpr int64_t kImg = 256 * 256 * 3;

__global__ void __launch_bounds__(NT) per_block(const uint4* __restrict__ p, uint32_t* out) {
    const uint4* b = p + (int64_t)blockIdx.x * (kImg / 16);
    const int64_t nvec = kImg / 16;
    uint32_t acc = 0;
    for (int64_t c = threadIdx.x; c + 2 * NT < nvec; c += 3 * NT) {
        const uint4 a = b[c], d = b[c + NT], e = b[c + 2 * NT];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ d.x ^ d.y ^ d.z ^ d.w ^ e.x ^ e.y ^ e.z ^ e.w;
    }
    out[blockIdx.x * NT + threadIdx.x] = acc;
}

// per_block at the colour kernel's occupancy: 36 KiB of LDS per workgroup -> 4 workgroups per CU
__global__ void __launch_bounds__(NT) per_block4(const uint4* __restrict__ p, uint32_t* out) {
    __shared__ uint32_t pad[9216];
    const uint4* b = p + (int64_t)blockIdx.x * (kImg / 16);
    const int64_t nvec = kImg / 16;
    uint32_t acc = 0;
    for (int64_t c = threadIdx.x; c + 2 * NT < nvec; c += 3 * NT) {
        const uint4 a = b[c], d = b[c + NT], e = b[c + 2 * NT];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ d.x ^ d.y ^ d.z ^ d.w ^ e.x ^ e.y ^ e.z ^ e.w;
    }
    pad[threadIdx.x] = acc;
    __syncthreads();
    out[blockIdx.x * NT + threadIdx.x] = pad[(threadIdx.x + 1) % NT];
}

__global__ void fill_random(uint32_t* p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        p[i] = h;
    }
}

__global__ void __launch_bounds__(NT) grid(const uint4* __restrict__ p, int64_t nvec, uint32_t* out) {
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * 3 * NT;
    for (int64_t c = (int64_t)blockIdx.x * 3 * NT + threadIdx.x; c + 2 * NT < nvec; c += stride) {
        const uint4 a = p[c], d = p[c + NT], e = p[c + 2 * NT];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ d.x ^ d.y ^ d.z ^ d.w ^ e.x ^ e.y ^ e.z ^ e.w;
    }
    out[blockIdx.x * NT + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 16384;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int64_t bytes = (int64_t)n * kImg;
    uint4* p;
    uint32_t* out;
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&out, (size_t)n * NT * 4));
    const bool rnd = argc > 3 && atoi(argv[3]) != 0;   // random bytes (the colour benchmark's data)
    if (rnd) hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(p), bytes / 4, 0x1234u);
    else CK(hipMemset(p, 0x5a, bytes));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int pass = 0; pass < 2; ++pass)
        for (int which = 0; which < 4; ++which) {
            const int g = which == 1 ? 2048 : 4096;
            auto launch = [&]() {
                if (which == 0) hipLaunchKernelGGL(per_block, dim3(n), dim3(NT), 0, 0, p, out);
                else if (which == 3) hipLaunchKernelGGL(per_block4, dim3(n), dim3(NT), 0, 0, p, out);
                else hipLaunchKernelGGL(grid, dim3(g), dim3(NT), 0, 0, p, bytes / 16, out);
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("{\"pattern\": \"%s\", \"data\": \"%s\", \"workgroups\": %d, \"ms\": %.4f, \"tbs\": %.3f}\n",
                   which == 0 ? "per_block" : which == 3 ? "per_block_4wg_per_cu" : "grid_stride", rnd ? "random" : "0x5a",
                   which == 0 || which == 3 ? n : g, ms, bytes / ms / 1e9);
            fflush(stdout);
        }
    CK(hipFree(p));
    CK(hipFree(out));
    return 0;
}
