// knn_hugek.hip — exact search and list merges for k > KNN_MAX_K_LARGE (any k: faiss IndexFlat
// serves every k, padding past ntotal with label -1; the reference passes the CLI's --top-k
// straight to index.search, /root/reference/main/search_from_image.py:27, 247).
//
// The in-LDS large-k route (knn_largek.hip) selects from 32-entry lists and its radix select holds
// at most 8192 values per query.  Past k = 1024 the answer is a large fraction of a list union
// anyway, so this route keys the whole corpus instead:
//   1. hugek_keys_kernel: the exact fp32 key of every (query, row) pair of a query chunk —
//      (|q|^2 + |x|^2) - 2 q.x clamped at 0 (L2) or -q.x (IP / cosine), the same key form as every
//      other path — as a u64 (order-preserving key bits << rb | row, rb = the bits a row index
//      needs), whose unsigned order is faiss's (key, label) order.  A register-tiled VALU GEMM: 64 rows x 64 queries per 256-thread
//      workgroup, 4 x 4 pairs per thread, 16-deep k stages of both operands through LDS.
//   2. a segmented radix sort of each query's N keys (rocPRIM, over the 32 + rb bits they use);
//   3. hugek_write_kernel: the first k of each segment to D / I (label + id_offset), padding.
// The query chunk is sized so a chunk's keys fit kHKEntries u64 (1 GiB, twice for the sort).
// List merges (shards' or ranks' sorted k-lists, k > 1024 and more than 8192 entries per query)
// take the same sort over the gathered lists.
//
// This route exists for coverage of faiss's k range, not speed: it writes N x Q keys (the one
// path that does) and its sort reads them eight times.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>

#include <algorithm>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "knn_index.h"
#include "wave_ops.h"

namespace imgrec {
namespace {

constexpr int kHKT = 64;                       // rows and queries per key tile
constexpr int kHKBK = 16;                      // k depth of one LDS stage
constexpr int64_t kHKEntries = int64_t(1) << 27;   // keys per chunk (1 GiB of u64)
constexpr int64_t kHKMaxQ = 65535;                 // queries per chunk: the write grid's y extent

// keys[qi * nrows + row] for queries [0, nqc) of the padded query block qp (rows of dp floats,
// zero beyond d) and every row of the index.  dp % 16 == 0 (knn_index rows are padded so).
__global__ void __launch_bounds__(256)
hugek_keys_kernel(const float* __restrict__ xb, const float* __restrict__ xn, int64_t nrows, int dp,
                  const float* __restrict__ qp, const float* __restrict__ qn, int nqc, int metric,
                  int rb, uint64_t* __restrict__ keys) {
    __shared__ float sx[kHKBK][kHKT + 4];      // sx[k][row]   (+4: 16-B aligned, rows spread over banks)
    __shared__ float sq[kHKBK][kHKT + 4];      // sq[k][query]
    const int t = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * kHKT;
    const int q0 = blockIdx.y * kHKT;
    const int tr = t & 15, tq = t >> 4;        // this thread's rows r0 + 4 tr .., queries q0 + 4 tq ..
    const int lr = t >> 2, lk = (t & 3) * 4;   // this thread's stage load: row / query lr, k lk .. lk + 3
    const int64_t xrow = r0 + lr;
    const int qrow = q0 + lr;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* xs = reinterpret_cast<const float4*>(xb + (xrow < nrows ? xrow : 0) * (int64_t)dp + lk);
    const float4* qs = reinterpret_cast<const float4*>(qp + (int64_t)(qrow < nqc ? qrow : 0) * dp + lk);
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    float4 a = xrow < nrows ? xs[0] : zero, b = qrow < nqc ? qs[0] : zero;
    for (int k0 = 0; k0 < dp; k0 += kHKBK) {
        __syncthreads();
        sx[lk + 0][lr] = a.x; sx[lk + 1][lr] = a.y; sx[lk + 2][lr] = a.z; sx[lk + 3][lr] = a.w;
        sq[lk + 0][lr] = b.x; sq[lk + 1][lr] = b.y; sq[lk + 2][lr] = b.z; sq[lk + 3][lr] = b.w;
        __syncthreads();
        if (k0 + kHKBK < dp) {                 // the next stage's loads in flight under the FMAs
            const int s = (k0 + kHKBK) / 4;
            a = xrow < nrows ? xs[s] : zero;
            b = qrow < nqc ? qs[s] : zero;
        }
        // two-level sum: a stage's 16 products in their own chain, then added to the total (the
        // error of a 1968-term key grows with ~124 + 16 additions instead of 1968)
        float part[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) part[i][j] = 0.f;
#pragma unroll
        for (int kk = 0; kk < kHKBK; ++kk) {
            const float4 xv = *reinterpret_cast<const float4*>(&sx[kk][tr * 4]);
            const float4 qv = *reinterpret_cast<const float4*>(&sq[kk][tq * 4]);
            const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, qa[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) part[i][j] = fmaf(xa[i], qa[j], part[i][j]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += part[i][j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int qi = q0 + tq * 4 + j;
        if (qi >= nqc) break;
        uint64_t* out = keys + (int64_t)qi * nrows;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t row = r0 + tr * 4 + i;
            if (row < nrows) {
                // L2: (|q|^2 + |x|^2) - 2 q.x, clamped at 0; IP: -q.x
                const float key = metric == 1 ? fmaxf((qn[qi] + xn[row]) - 2.f * acc[i][j], 0.f) : -acc[i][j];
                out[row] = ((uint64_t)key_bits_ordered(key) << rb) | (uint64_t)row;
            }
        }
    }
}

__global__ void hugek_offsets_kernel(unsigned* off, int nseg, int64_t seg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= nseg) off[i] = (unsigned)(i * seg);
}

// Row q of D / I (k entries) from the first min(k, seg) sorted values (key bits << rb | label) of
// segment q.
__global__ void hugek_write_kernel(const uint64_t* __restrict__ sorted, int64_t seg, int k, int metric,
                                   int rb, int64_t id_offset, bool label_is_row, float* __restrict__ D,
                                   int64_t* __restrict__ I) {
    const int64_t q = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const uint64_t x = i < seg ? sorted[q * seg + i] : ~0ull;
    float* d = D + q * k;
    int64_t* l = I + q * k;
    if (x == ~0ull) {
        d[i] = metric == 1 ? FLT_MAX : -FLT_MAX;
        l[i] = -1;
    } else {
        const float key = key_from_ordered((uint32_t)(x >> rb));
        d[i] = metric == 1 ? key : -key;
        l[i] = (int64_t)(x & ((uint64_t(1) << rb) - 1)) + (label_is_row ? id_offset : 0);
    }
}

// Gathered lists -> one u64 per entry (list l of query q at cD[l * sd + q * kin ...]); empty
// (label -1) entries sort last.
__global__ void hugek_pack_lists_kernel(const float* __restrict__ cD, const int64_t* __restrict__ cI,
                                        int nlists, int kin, int64_t sd, int64_t si, int metric,
                                        uint64_t* __restrict__ v) {
    const int64_t q = blockIdx.y;
    const int64_t M = (int64_t)nlists * kin;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= M) return;
    const int64_t l = e / kin, p = e - l * kin;
    const int64_t lab = cI[l * si + q * kin + p];
    const float d = cD[l * sd + q * kin + p];
    v[q * M + e] = lab < 0 ? ~0ull : ((uint64_t)key_bits_ordered(metric == 1 ? d : -d) << 32) | (uint32_t)lab;
}

int bits_for(int64_t n) {                      // bits a row index < n needs
    int b = 0;
    while (b < 32 && (int64_t(1) << b) < n) ++b;
    return b;
}

// Segmented sort of nseg segments of `seg` u64 in `in` -> `out` over bits [0, end_bit).  The
// sort's temporary storage grows in *tmp: by hipMalloc (an index's workspace), or in stream order
// by hipMallocAsync when `async_tmp` (a merge's, freed by the caller with hipFreeAsync).
hipError_t sort_segments(uint64_t* in, uint64_t* out, int nseg, int64_t seg, unsigned end_bit,
                         unsigned* off, void** tmp, size_t* tmp_cap, bool async_tmp, hipStream_t st) {
    hipLaunchKernelGGL(hugek_offsets_kernel, dim3((unsigned)((nseg + 256) / 256)), dim3(256), 0, st, off,
                       nseg, seg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return sort_u64_segments(in, out, (int64_t)nseg * seg, nseg, off, end_bit, tmp, tmp_cap, async_tmp, st);
}

}  // namespace

hipError_t sort_u64_segments(uint64_t* in, uint64_t* out, int64_t total, int nseg, const unsigned* off,
                             unsigned end_bit, void** tmp, size_t* tmp_cap, bool async_tmp, hipStream_t st) {
    hipError_t e;
    size_t need = 0;
    e = rocprim::segmented_radix_sort_keys(nullptr, need, in, out, (unsigned)total, (unsigned)nseg,
                                           off, off + 1, 0u, end_bit, st);
    if (e != hipSuccess) return e;
    if (need > *tmp_cap) {
        if (*tmp) (void)(async_tmp ? hipFreeAsync(*tmp, st) : hipFree(*tmp));
        *tmp = nullptr;
        *tmp_cap = 0;
        if ((e = async_tmp ? hipMallocAsync(tmp, need, st) : hipMalloc(tmp, need)) != hipSuccess) return e;
        *tmp_cap = need;
    }
    size_t have = *tmp_cap;
    return rocprim::segmented_radix_sort_keys(*tmp, have, in, out, (unsigned)total, (unsigned)nseg,
                                              off, off + 1, 0u, end_bit, st);
}

int hugek_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                 hipStream_t st) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int64_t N = ix->ntotal;
    if (N > (int64_t)UINT32_MAX) KNN_FAIL(KNN_EINVAL, "k > %d search: more than 2^32 rows", KNN_MAX_K_LARGE);
    if (N == 0) {
        KNN_HIP(launch_fill_empty(D, I, nq * (int64_t)k, kmetric, st));
        return KNN_OK;
    }
    if (ix->dp % kHKBK) KNN_FAIL(KNN_EINVAL, "row stride %d not a multiple of %d", ix->dp, kHKBK);
    const int64_t per = std::max<int64_t>(1, std::min<int64_t>({nq, kHKEntries / N, kHKMaxQ}));   // queries per chunk
    const int64_t per_pad = round_up(per, kHKT);
    int rc;
    if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)per_pad * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)per_pad)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hk_a, &ix->hk_a_cap, (size_t)(per * N))) != KNN_OK) return rc;
    if ((rc = grow(&ix->hk_b, &ix->hk_b_cap, (size_t)(per * N))) != KNN_OK) return rc;
    if ((rc = grow(&ix->hk_off, &ix->hk_off_cap, (size_t)per + 1)) != KNN_OK) return rc;
    const int rb = std::max(1, bits_for(N));
    const unsigned end_bit = 32u + (unsigned)rb;
    for (int64_t q0 = 0; q0 < nq; q0 += per) {
        const int64_t qc = std::min<int64_t>(per, nq - q0);
        KNN_HIP(launch_rows_ingest(q + q0 * ix->d, qc, ix->d, ix->dp, round_up(qc, kHKT),
                                   ix->metric == KNN_METRIC_COSINE ? 1 : 0, ix->qpad, ix->qnorm, st));
        const dim3 grid((unsigned)((N + kHKT - 1) / kHKT), (unsigned)((qc + kHKT - 1) / kHKT));
        hipLaunchKernelGGL(hugek_keys_kernel, grid, dim3(256), 0, st, ix->xb, ix->xn, N, ix->dp, ix->qpad,
                           ix->qnorm, (int)qc, kmetric, rb, ix->hk_a);
        KNN_HIP(hipGetLastError());
        KNN_HIP(sort_segments(ix->hk_a, ix->hk_b, (int)qc, N, end_bit, ix->hk_off, &ix->hk_tmp,
                              &ix->hk_tmp_cap, false, st));
        hipLaunchKernelGGL(hugek_write_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)qc), dim3(256), 0,
                           st, ix->hk_b, N, k, kmetric, rb, ix->id_offset, true, D + q0 * k, I + q0 * k);
        KNN_HIP(hipGetLastError());
    }
    return KNN_OK;
}

void hugek_free(knn_index* ix) {
    for (void* p : {(void*)ix->hk_a, (void*)ix->hk_b, (void*)ix->hk_off, ix->hk_tmp})
        if (p) (void)hipFree(p);
    ix->hk_a = ix->hk_b = nullptr;
    ix->hk_off = nullptr;
    ix->hk_tmp = nullptr;
    ix->hk_a_cap = ix->hk_b_cap = ix->hk_off_cap = ix->hk_tmp_cap = 0;
}

// Merge of nlists sorted lists of kin entries per query into the top k (any k; labels < 2^32),
// by the same segmented sort; workspace allocated and freed in stream order on `st`.
hipError_t launch_merge_huge(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                             int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                             hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    const int64_t M = (int64_t)nlists * kin;
    const int64_t per = std::max<int64_t>(1, std::min<int64_t>({nq, kHKEntries / std::max<int64_t>(M, 1), kHKMaxQ}));
    uint64_t *a = nullptr, *b = nullptr;
    unsigned* off = nullptr;
    void* tmp = nullptr;
    size_t tmp_cap = 0;
    hipError_t e;
    auto cleanup = [&]() {
        for (void* p : {(void*)a, (void*)b, (void*)off, tmp})
            if (p) (void)hipFreeAsync(p, st);
    };
    if ((e = hipMallocAsync((void**)&a, (size_t)(per * M) * 8, st)) != hipSuccess ||
        (e = hipMallocAsync((void**)&b, (size_t)(per * M) * 8, st)) != hipSuccess ||
        (e = hipMallocAsync((void**)&off, (size_t)(per + 1) * 4, st)) != hipSuccess) {
        cleanup();
        return e;
    }
    for (int64_t q0 = 0; q0 < nq && e == hipSuccess; q0 += per) {
        const int64_t qc = std::min<int64_t>(per, nq - q0);
        hipLaunchKernelGGL(hugek_pack_lists_kernel, dim3((unsigned)((M + 255) / 256), (unsigned)qc), dim3(256), 0,
                           st, cD + q0 * kin, cI + q0 * kin, nlists, kin, sd, si, metric, a);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = sort_segments(a, b, (int)qc, M, 64u, off, &tmp, &tmp_cap, true, st)) != hipSuccess) break;
        hipLaunchKernelGGL(hugek_write_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)qc), dim3(256), 0,
                           st, b, M, k, metric, 32, (int64_t)0, false, D + q0 * k, I + q0 * k);
        e = hipGetLastError();
    }
    cleanup();
    return e;
}

hipError_t launch_merge_any(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                            int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                            hipStream_t st) {
    if (k <= KNN_MAX_K_LARGE && (int64_t)nlists * kin <= 8192)
        return launch_merge_large(cD, cI, nlists, nq, kin, sd, si, k, metric, D, I, st);
    return launch_merge_huge(cD, cI, nlists, nq, kin, sd, si, k, metric, D, I, st);
}

}  // namespace imgrec
