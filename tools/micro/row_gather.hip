// Micro-benchmark (round 6): how fast can 1024 workgroups gather random fp32 corpus rows — the
// rerank's access pattern (rerank_certify_kernel: one 8-wave workgroup per query, its ~20
// candidate rows of 1968 floats = 7.9 KB at random places in the 7.9 GB fp32 corpus, each dotted
// with the query row).  Variants: R rows per workgroup, loaded ROWS_IN_FLIGHT per wave at a time
// (2 = the rerank's "two candidate rows per wave in flight"), or every row a wave owns at once.
// Prints the time and the gathered bytes' rate.
// Usage: row_gather [rows_per_query=20] [reps=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kD = 1984;                  // padded row (floats)
constexpr int kV = kD / 4 / 64;           // float4 per lane per row: 7.75 -> 8 (last partial)

// each wave takes rows w, w + 8, ... of its query's list; IF rows loaded before any is consumed
template <int IF>
__global__ void __launch_bounds__(512)
gather_kernel(const float* __restrict__ xb, const float* __restrict__ q, const int* __restrict__ ids,
              int rows_per_q, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = blockIdx.x;
    float4 qr[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int e = (c * 64 + lane) * 4;
        qr[c] = e < kD ? *reinterpret_cast<const float4*>(q + (size_t)qi * kD + e) : make_float4(0, 0, 0, 0);
    }
    for (int r0 = wave; r0 < rows_per_q; r0 += 8 * IF) {
        float4 v[IF][8];
#pragma unroll
        for (int i = 0; i < IF; ++i) {
            const int r = r0 + 8 * i;
            const int id = r < rows_per_q ? ids[qi * rows_per_q + r] : -1;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int e = (c * 64 + lane) * 4;
                typedef float f4 __attribute__((ext_vector_type(4)));
                f4 w = (f4){0.f, 0.f, 0.f, 0.f};
                if (id >= 0 && e < kD) w = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xb + (size_t)id * kD + e));
                v[i][c] = make_float4(w.x, w.y, w.z, w.w);
            }
        }
#pragma unroll
        for (int i = 0; i < IF; ++i) {
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                s += v[i][c].x * qr[c].x + v[i][c].y * qr[c].y + v[i][c].z * qr[c].z + v[i][c].w * qr[c].w;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            const int r = r0 + 8 * i;
            if (lane == 0 && r < rows_per_q) out[qi * rows_per_q + r] = s;
        }
    }
}

__global__ void fill(float* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (float)((i * 2654435761u) & 1023) * (1.f / 1024.f);
}

template <int IF>
void run(const float* xb, const float* q, const int* ids, int nq, int R, float* out, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((gather_kernel<IF>), dim3(nq), dim3(512), 0, 0, xb, q, ids, R, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((gather_kernel<IF>), dim3(nq), dim3(512), 0, 0, xb, q, ids, R, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    const double bytes = (double)nq * R * 1968 * 4;
    printf("{\"rows_in_flight_per_wave\": %d, \"rows_per_query\": %d, \"queries\": %d, \"best_us\": %.2f, "
           "\"mean_us\": %.2f, \"gathered_TBps_best\": %.2f}\n",
           IF, R, nq, best * 1e3, sum / reps * 1e3, bytes / (best * 1e-3) / 1e12);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 20;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int nq = 1024;
    const size_t nrows = 1000000;
    float *xb, *q, *out;
    int* ids;
    CK(hipMalloc(&xb, nrows * kD * sizeof(float)));
    CK(hipMalloc(&q, (size_t)nq * kD * sizeof(float)));
    CK(hipMalloc(&out, (size_t)nq * 64 * sizeof(float)));
    CK(hipMalloc(&ids, (size_t)nq * 64 * sizeof(int)));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, xb, nrows * kD);
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, q, (size_t)nq * kD);
    int* h = (int*)malloc((size_t)nq * 64 * sizeof(int));
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < nq * 64; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (int)(s % nrows); }
    CK(hipMemcpy(ids, h, (size_t)nq * 64 * sizeof(int), hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    for (int pass = 0; pass < 2; ++pass) {
        run<1>(xb, q, ids, nq, R, out, reps);
        run<2>(xb, q, ids, nq, R, out, reps);
        run<3>(xb, q, ids, nq, R, out, reps);
        run<4>(xb, q, ids, nq, 32, out, reps);
        run<2>(xb, q, ids, nq, 32, out, reps);
        run<2>(xb, q, ids, nq, 64, out, reps);
        run<8>(xb, q, ids, nq, 64, out, reps);
    }
    CK(hipFree(xb));
    CK(hipFree(q));
    CK(hipFree(out));
    CK(hipFree(ids));
    free(h);
    return 0;
}
