// ivfpq.hip — GPU IVF-PQ search kernels (gfx950): per-query distance tables and the ADC list scan.
//
// The reference's default index is faiss IndexIVFPQ(IndexHNSWFlat(d, 32), d, 2048, m, 12) with
// nprobe 1 (/root/reference/main/create_index.py:218-228; searched at
// main/search_from_image.py:247).  These kernels restate faiss's search arithmetic for it
// (by-residual L2 product quantisation, distance-table ADC; oracle/ivfpq.py is the CPU
// statement the tests hold them to):
//
//   ivfpq_lut_kernel   one workgroup per (8 residuals, sub-quantiser): the residual sub-vectors
//                      sit in LDS, each thread scores centroids i, i + 256, ... of the transposed
//                      codebook (coalesced columns, each read serving 8 residuals):
//                      lut[r][j][i] = sum_t (r_jt - c_jit)^2.
//   ivfpq_scan_kernel  one 4-wave workgroup per query: its 256 lanes take the rows of the probed
//                      lists round-robin, a row's distance is the sum over j of lut[j][code_j]
//                      (fp32, j ascending), kept in a per-lane (distance, label) list; each wave
//                      reduces its lanes to k by k rounds of a wave-wide u64 minimum over the lane
//                      heads (order-preserving key bits | label), then the first wave merges the
//                      four lists the same way.
//
// Both are memory-light next to the exact path: the scan reads m codes (2 B each) and m table
// entries per row of the probed lists (~N / nlist rows per probe).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include <math.h>

#include <algorithm>

#include "knn_kernels.h"
#include "wave_ops.h"

namespace imgrec {
namespace {

constexpr int kLutThreads = 256;
constexpr int kMaxDsub = 256;

constexpr int kLutRes = 8;          // residuals per workgroup: each codebook column read serves 8

__global__ void __launch_bounds__(kLutThreads)
ivfpq_lut_kernel(const float* __restrict__ resid, int64_t nr, int d, int m, int ksub,
                 const float* __restrict__ cbt, float* __restrict__ lut) {
    __shared__ float sr[kLutRes][kMaxDsub];
    const int64_t r0 = (int64_t)blockIdx.x * kLutRes;
    const int j = blockIdx.y;
    const int dsub = d / m;
    const int nres = (int)min((int64_t)kLutRes, nr - r0);
    for (int e = threadIdx.x; e < kLutRes * dsub; e += kLutThreads) {
        const int r = e / dsub, t = e - r * dsub;
        sr[r][t] = r < nres ? resid[(r0 + r) * d + (int64_t)j * dsub + t] : 0.f;
    }
    __syncthreads();
    const float* cb = cbt + (size_t)j * dsub * ksub;
    for (int i = threadIdx.x; i < ksub; i += kLutThreads) {
        float acc[kLutRes];
#pragma unroll
        for (int r = 0; r < kLutRes; ++r) acc[r] = 0.f;
        for (int t = 0; t < dsub; ++t) {
            const float c = cb[(size_t)t * ksub + i];
#pragma unroll
            for (int r = 0; r < kLutRes; ++r) {
                const float df = sr[r][t] - c;
                acc[r] = fmaf(df, df, acc[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < kLutRes; ++r)
            if (r < nres) lut[((size_t)(r0 + r) * m + j) * ksub + i] = acc[r];
    }
}

// (d1, i1) before (d2, i2): smaller distance, ties by smaller label; label -1 = empty, last.
__device__ __forceinline__ bool before(float d1, int i1, float d2, int i2) {
    return i2 < 0 || d1 < d2 || (d1 == d2 && i1 < i2);
}

template <int KM>
__device__ __forceinline__ void insert_sorted(float (&kd)[KM], int (&ki)[KM], float d, int id) {
#pragma unroll
    for (int p = KM - 1; p > 0; --p) {
        const bool shift = before(d, id, kd[p - 1], ki[p - 1]);
        const bool here = !shift && before(d, id, kd[p], ki[p]);
        kd[p] = shift ? kd[p - 1] : (here ? d : kd[p]);
        ki[p] = shift ? ki[p - 1] : (here ? id : ki[p]);
    }
    const bool here0 = before(d, id, kd[0], ki[0]);
    kd[0] = here0 ? d : kd[0];
    ki[0] = here0 ? id : ki[0];
}

template <int KM>
__global__ void __launch_bounds__(256)
ivfpq_scan_kernel(const float* __restrict__ lut, const int64_t* __restrict__ probes, int64_t nq,
                  int nprobe, const int64_t* __restrict__ list_off,
                  const uint16_t* __restrict__ codes, const int64_t* __restrict__ ids, int m,
                  int ksub, int k, float* __restrict__ D, int64_t* __restrict__ I) {
    // one 4-wave workgroup per query: the probed rows go round-robin over its 256 lanes
    __shared__ uint64_t best[4][32];                            // each wave's k best, ascending
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t q = blockIdx.x;
    float kd[KM];
    int ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }
    for (int p = 0; p < nprobe; ++p) {
        const int64_t l = probes[q * nprobe + p];
        if (l < 0) continue;
        const float* T = lut + (size_t)(q * nprobe + p) * m * ksub;
        const int64_t r1 = list_off[l + 1];
        for (int64_t row = list_off[l] + threadIdx.x; row < r1; row += 256) {
            const uint16_t* c = codes + row * m;
            float dist = 0.f;
            for (int j = 0; j < m; ++j) dist += T[(size_t)j * ksub + c[j]];
            const int id = (int)ids[row];
            if (before(dist, id, kd[KM - 1], ki[KM - 1])) insert_sorted<KM>(kd, ki, dist, id);
        }
    }
    // per wave: k rounds of the wave minimum over the lane heads
    constexpr uint64_t kEmpty = ~0ull;
    for (int r = 0; r < k; ++r) {
        const uint64_t v = ki[0] < 0 ? kEmpty : ((uint64_t)key_bits_ordered(kd[0]) << 32) | (uint32_t)ki[0];
        const uint64_t b = wave_min_u64(v);
        if (b != kEmpty && v == b) {
#pragma unroll
            for (int p = 0; p < KM - 1; ++p) { kd[p] = kd[p + 1]; ki[p] = ki[p + 1]; }
            kd[KM - 1] = INFINITY;
            ki[KM - 1] = -1;
        }
        if (lane == 0) best[wave][r] = b;
    }
    __syncthreads();
    if (wave != 0) return;
    // the four waves' sorted lists: lane w < 4 holds the head of list w
    int head = 0;
    uint64_t cur = lane < 4 ? best[lane][0] : kEmpty;
    for (int r = 0; r < k; ++r) {
        const uint64_t b = wave_min_u64(cur);
        if (b != kEmpty && cur == b) cur = ++head < k ? best[lane][head] : kEmpty;
        if (lane == 0) {
            D[q * k + r] = b == kEmpty ? FLT_MAX : key_from_ordered((uint32_t)(b >> 32));
            I[q * k + r] = b == kEmpty ? (int64_t)-1 : (int64_t)(uint32_t)b;
        }
    }
}

// Any k (faiss IndexIVFPQ serves every k): the ADC distance of EVERY row of each query's probed
// lists, summed in the scan kernel's order (the same bits), as (ordered key bits << 32 | label) at
// the (query, probe)'s slot probe_off[q * nprobe + p]; a segmented sort per query follows.
__global__ void __launch_bounds__(256)
ivfpq_adc_all_kernel(const float* __restrict__ lut, const int64_t* __restrict__ probes,
                     const int64_t* __restrict__ list_off, const uint16_t* __restrict__ codes,
                     const int64_t* __restrict__ ids, int m, int ksub,
                     const int64_t* __restrict__ probe_off, uint64_t* __restrict__ out) {
    const int64_t qp = blockIdx.x;                              // q * nprobe + p
    const int64_t l = probes[qp];
    if (l < 0) return;
    const float* T = lut + (size_t)qp * m * ksub;
    const int64_t r0 = list_off[l], r1 = list_off[l + 1];
    uint64_t* o = out + probe_off[qp];
    for (int64_t row = r0 + threadIdx.x; row < r1; row += 256) {
        const uint16_t* c = codes + row * m;
        float dist = 0.f;
        for (int j = 0; j < m; ++j) dist += T[(size_t)j * ksub + c[j]];
        o[row - r0] = ((uint64_t)key_bits_ordered(dist) << 32) | (uint32_t)ids[row];
    }
}

// Row q of D / I: the first min(k, segment size) sorted entries of query q, then -1 / FLT_MAX.
__global__ void ivfpq_write_all_kernel(const uint64_t* __restrict__ sorted, const uint32_t* __restrict__ seg_off,
                                       int k, float* __restrict__ D, int64_t* __restrict__ I) {
    const int64_t q = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const int64_t n = (int64_t)seg_off[q + 1] - seg_off[q];
    const uint64_t x = i < n ? sorted[seg_off[q] + i] : ~0ull;
    D[q * k + i] = x == ~0ull ? FLT_MAX : key_from_ordered((uint32_t)(x >> 32));
    I[q * k + i] = x == ~0ull ? (int64_t)-1 : (int64_t)(uint32_t)x;
}

}  // namespace

hipError_t launch_ivfpq_scan_all(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                                 const int64_t* list_off, const uint16_t* codes, const int64_t* ids,
                                 int m, int ksub, const int64_t* probe_off, const uint32_t* seg_off,
                                 int64_t total, int k, float* D, int64_t* I, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    if (k <= 0 || nprobe <= 0 || m <= 0 || ksub <= 0 || ksub > 65536 || total < 0 ||
        total >= ((int64_t)1 << 32) || nq > 0x7fffffff)
        return hipErrorInvalidValue;
    uint64_t *a = nullptr, *b = nullptr;
    void* tmp = nullptr;
    size_t tmp_cap = 0;
    hipError_t e = hipSuccess;
    const size_t nbytes = (size_t)std::max<int64_t>(total, 1) * 8;
    if ((e = hipMallocAsync((void**)&a, nbytes, st)) == hipSuccess &&
        (e = hipMallocAsync((void**)&b, nbytes, st)) == hipSuccess) {
        if (total > 0) {
            hipLaunchKernelGGL(ivfpq_adc_all_kernel, dim3((unsigned)(nq * nprobe)), dim3(256), 0, st, lut,
                               probes, list_off, codes, ids, m, ksub, probe_off, a);
            e = hipGetLastError();
            if (e == hipSuccess)
                e = sort_u64_segments(a, b, total, (int)nq, seg_off, 64u, &tmp, &tmp_cap, true, st);
        }
        // (queries in slices of 65535: the grid's y extent)
        for (int64_t q0 = 0; q0 < nq && e == hipSuccess; q0 += 65535) {
            const int64_t qn = std::min<int64_t>(65535, nq - q0);
            hipLaunchKernelGGL(ivfpq_write_all_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)qn), dim3(256),
                               0, st, b, seg_off + q0, k, D + q0 * k, I + q0 * k);
            e = hipGetLastError();
        }
    }
    for (void* p : {(void*)a, (void*)b, tmp})
        if (p) (void)hipFreeAsync(p, st);
    return e;
}

hipError_t launch_ivfpq_lut(const float* resid, int64_t nr, int d, int m, int ksub,
                            const float* cbt, float* lut, hipStream_t st) {
    if (nr <= 0) return hipSuccess;
    if (m <= 0 || d % m != 0 || d / m > kMaxDsub || ksub <= 0 || nr > 0x7fffffff || m > 65535)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(ivfpq_lut_kernel, dim3((unsigned)((nr + kLutRes - 1) / kLutRes), (unsigned)m),
                       dim3(kLutThreads), 0, st, resid, nr, d, m, ksub, cbt, lut);
    return hipGetLastError();
}

hipError_t launch_ivfpq_scan(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                             const int64_t* list_off, const uint16_t* codes, const int64_t* ids,
                             int m, int ksub, int k, float* D, int64_t* I, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    if (k <= 0 || k > 32 || nprobe <= 0 || m <= 0 || ksub <= 0 || ksub > 65536)
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)nq), block(256);
    if (k <= 16)
        hipLaunchKernelGGL((ivfpq_scan_kernel<16>), grid, block, 0, st, lut, probes, nq, nprobe,
                           list_off, codes, ids, m, ksub, k, D, I);
    else
        hipLaunchKernelGGL((ivfpq_scan_kernel<32>), grid, block, 0, st, lut, probes, nq, nprobe,
                           list_off, codes, ids, m, ksub, k, D, I);
    return hipGetLastError();
}

}  // namespace imgrec
