// knn_largek.hip — exact search for KNN_MAX_K < k <= KNN_MAX_K_LARGE (gfx950).
//
// The fused kernels keep register top-k lists (k <= 32).  faiss IndexFlat serves any k
// (main/search_from_image.py:247 passes the CLI's --top-k), so larger k runs faiss's own flat
// algorithm instead (exhaustive_L2sqr_blas): an fp32 GEMM of a query block against a corpus
// block (rocBLAS sgemm, alpha = -2: G = -2 q.x exactly), keys formed with the stored norms in the
// same (|q|^2 + |x|^2) - 2 q.x form as every other path, and per query a running top-k merged
// with each block by an exact radix select in LDS:
//   * a workgroup per query packs the block's keys with their rows into u64 (order-preserving
//     key bits | row: unsigned order = (key, row), faiss's tie rule) next to the running list;
//   * eight 8-bit digit passes of a 256-bin LDS histogram find the k-th smallest value T;
//   * the values < T, then copies of T, fill the new running list (empties = ~0 pad a corpus
//     with fewer than k rows); after the last block a bitonic sort orders it and the workgroup
//     writes D / I.
// Throughput is the GEMM's (the selection reads the block from L2); this path exists for
// completeness of the faiss surface, the k <= 32 paths are the fast ones.

#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdint.h>
#include <float.h>
#include <math.h>

#include <algorithm>

#include "knn_index.h"
#include "wave_ops.h"

namespace imgrec {
namespace {

constexpr int kLKThreads = 256;
constexpr int kLKM = 8192;          // LDS values per query: running list + corpus block
constexpr int kLKSort = 1024;       // KNN_MAX_K_LARGE, a power of two
static_assert(KNN_MAX_K_LARGE <= kLKSort && (kLKSort & (kLKSort - 1)) == 0, "sort width");

// The k smallest of v[0 .. M) (LDS, u64 values, empties = ~0) into sel[0 .. k) — ascending when
// `sort` — by an exact radix select of the k-th smallest T (eight 8-bit digit passes of a 256-bin
// LDS histogram), then the values < T and copies of T; the rest of sel is ~0.  Block-wide.
__device__ void select_k(const uint64_t* v, int M, int k, uint64_t* sel, uint32_t* hist,
                         uint64_t* s_prefix, int* s_rem, int* s_nlt, bool sort) {
    const int t = threadIdx.x;
    const int kk = min(k, M);
    if (t == 0) { *s_prefix = 0; *s_rem = kk; }
    __syncthreads();
    uint64_t mask = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int b = t; b < 256; b += kLKThreads) hist[b] = 0u;
        __syncthreads();
        const uint64_t prefix = *s_prefix;
        for (int i = t; i < M; i += kLKThreads) {
            const uint64_t x = v[i];
            if ((x & mask) == prefix) atomicAdd(&hist[(x >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (t < 64) {                                   // wave 0: the digit where rem is reached
            const uint32_t h0 = hist[4 * t], h1 = hist[4 * t + 1], h2 = hist[4 * t + 2], h3 = hist[4 * t + 3];
            const int mine = (int)(h0 + h1 + h2 + h3);
            const int before = wave_excl_scan_i32(mine);
            const int rem = *s_rem;
            if (before < rem && before + mine >= rem) {
                int c = before, dgt = 4 * t;
                const uint32_t hh[4] = {h0, h1, h2, h3};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (c + (int)hh[e] >= rem) { dgt = 4 * t + e; break; }
                    c += (int)hh[e];
                }
                *s_prefix = prefix | ((uint64_t)dgt << shift);
                *s_rem = rem - c;
            }
        }
        mask |= (uint64_t)255 << shift;
        __syncthreads();
    }
    const uint64_t T = *s_prefix;                       // the kk-th smallest value
    if (t == 0) *s_nlt = 0;
    __syncthreads();
    for (int i = t; i < M; i += kLKThreads)
        if (v[i] < T) sel[atomicAdd(s_nlt, 1)] = v[i];
    __syncthreads();
    const int nlt = *s_nlt;                             // < kk; the rest are copies of T
    for (int i = nlt + t; i < kLKSort; i += kLKThreads) sel[i] = i < kk ? T : ~0ull;
    __syncthreads();
    if (!sort) return;
    for (int size = 2; size <= kLKSort; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = t; i < kLKSort / 2; i += kLKThreads) {
                const int lo = 2 * stride * (i / stride) + (i % stride), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const uint64_t a = sel[lo], b = sel[hi];
                if ((a > b) == up) { sel[lo] = b; sel[hi] = a; }
            }
            __syncthreads();
        }
}

// Workgroup (query qq of the block, stripe s = blockIdx.y): the GEMM columns [s * nrc, (s + 1) *
// nrc) of this round (ldg = the round's rows; global row r0 + s * nrc at column s * nrc) merged
// into stripe s's running list run[(s * nq_all + q) * k ...].  With one stripe the last round
// sorts and writes D / I; with several, largek_final_kernel merges the stripes.
__global__ void __launch_bounds__(kLKThreads)
largek_select_kernel(const float* __restrict__ G, int ldg, int nrc, const float* __restrict__ qnorm,
                     const float* __restrict__ xn, int64_t r0, int k, int metric, int first,
                     int last, int64_t q0, int64_t nq_all, uint64_t* __restrict__ run,
                     float* __restrict__ D, int64_t* __restrict__ I, int64_t id_offset) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    const int t = threadIdx.x;
    const int64_t qq = blockIdx.x, q = q0 + qq;
    const int sidx = blockIdx.y;
    run += (int64_t)sidx * nq_all * k;
    const int c0 = sidx * nrc;
    const int ns = max(0, min(nrc, ldg - c0));          // this stripe's columns in the round
    const int64_t rs = r0 + c0;
    const int nr = first ? 0 : k;
    for (int i = t; i < nr; i += kLKThreads) v[i] = run[q * k + i];
    const float qn = qnorm[q];
    const float* g = G + qq * (int64_t)ldg + c0;
    for (int j = t; j < ns; j += kLKThreads) {
        // L2: (|q|^2 + |x|^2) - 2 q.x, clamped at 0; IP: -q.x (G = -2 q.x, halving is exact)
        const float key = metric == 1 ? fmaxf((qn + xn[rs + j]) + g[j], 0.f) : 0.5f * g[j];
        v[nr + j] = ((uint64_t)key_bits_ordered(key) << 32) | (uint32_t)(rs + j);
    }
    const int M = nr + ns;
    select_k(v, M, k, sel, hist, &s_prefix, &s_rem, &s_nlt, last != 0);
    if (!last) {
        for (int i = t; i < k; i += kLKThreads) run[q * k + i] = sel[i];
        return;
    }
    for (int i = t; i < k; i += kLKThreads) {
        const uint64_t x = sel[i];
        if (x == ~0ull) {
            D[q * k + i] = metric == 1 ? FLT_MAX : -FLT_MAX;
            I[q * k + i] = -1;
        } else {
            const float key = key_from_ordered((uint32_t)(x >> 32));
            D[q * k + i] = metric == 1 ? key : -key;
            I[q * k + i] = (int64_t)(uint32_t)x + id_offset;
        }
    }
}

// The stripes' running lists of one query (S x k local rows) -> the final sorted top-k.
__global__ void __launch_bounds__(kLKThreads)
largek_final_kernel(const uint64_t* __restrict__ run, int S, int64_t nq_all, int k, int64_t q0,
                    int metric, float* __restrict__ D, int64_t* __restrict__ I, int64_t id_offset) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    const int t = threadIdx.x;
    const int64_t q = q0 + blockIdx.x;
    const int M = S * k;
    for (int e = t; e < M; e += kLKThreads) {
        const int sidx = e / k, i = e - sidx * k;
        v[e] = run[((int64_t)sidx * nq_all + q) * k + i];
    }
    __syncthreads();
    select_k(v, M, k, sel, hist, &s_prefix, &s_rem, &s_nlt, true);
    for (int i = t; i < k; i += kLKThreads) {
        const uint64_t x = sel[i];
        if (x == ~0ull) {
            D[q * k + i] = metric == 1 ? FLT_MAX : -FLT_MAX;
            I[q * k + i] = -1;
        } else {
            const float key = key_from_ordered((uint32_t)(x >> 32));
            D[q * k + i] = metric == 1 ? key : -key;
            I[q * k + i] = (int64_t)(uint32_t)x + id_offset;
        }
    }
}

// Merge of nlists sorted per-shard results of kin entries per query (distance-ascending for L2,
// inner-product-descending otherwise; label -1 = empty) into the final top-k for k > KNN_MAX_K:
// list l of query q at cD[l * sd + q * kin], cI[l * si + q * kin].  Labels must be < 2^32 (they
// pack beside the key; ties order by label, faiss's rule).
__global__ void __launch_bounds__(kLKThreads)
largek_merge_kernel(const float* __restrict__ cD, const int64_t* __restrict__ cI, int nlists,
                    int kin, int64_t sd, int64_t si, int k, int metric, float* __restrict__ D,
                    int64_t* __restrict__ I) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    const int t = threadIdx.x;
    const int64_t q = blockIdx.x;
    const int M = nlists * kin;
    for (int e = t; e < M; e += kLKThreads) {
        const int l = e / kin, p = e - l * kin;
        const int64_t lab = cI[l * si + q * kin + p];
        const float d = cD[l * sd + q * kin + p];
        v[e] = lab < 0 ? ~0ull : ((uint64_t)key_bits_ordered(metric == 1 ? d : -d) << 32) | (uint32_t)lab;
    }
    __syncthreads();
    select_k(v, M, k, sel, hist, &s_prefix, &s_rem, &s_nlt, true);
    for (int i = t; i < k; i += kLKThreads) {
        const uint64_t x = sel[i];
        if (x == ~0ull) {
            D[q * k + i] = metric == 1 ? FLT_MAX : -FLT_MAX;
            I[q * k + i] = -1;
        } else {
            const float key = key_from_ordered((uint32_t)(x >> 32));
            D[q * k + i] = metric == 1 ? key : -key;
            I[q * k + i] = (int64_t)(uint32_t)x;
        }
    }
}

}  // namespace

hipError_t launch_merge_large(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                              int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                              hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    if (k > KNN_MAX_K_LARGE || (int64_t)nlists * kin > kLKM) return hipErrorInvalidValue;
    hipLaunchKernelGGL(largek_merge_kernel, dim3((unsigned)nq), dim3(kLKThreads), 0, st, cD, cI,
                       nlists, kin, sd, si, k, metric, D, I);
    return hipGetLastError();
}

void largek_free(knn_index* ix) {
    if (ix->blas) (void)rocblas_destroy_handle((rocblas_handle)ix->blas);
    ix->blas = nullptr;
    for (void* p : {(void*)ix->lk_g, (void*)ix->lk_run})
        if (p) (void)hipFree(p);
    ix->lk_g = nullptr;
    ix->lk_run = nullptr;
}

int largek_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    if (k > KNN_MAX_K_LARGE) KNN_FAIL(KNN_EINVAL, "k must be <= %d (got %d)", KNN_MAX_K_LARGE, k);
    if (ix->ntotal > (int64_t)UINT32_MAX) KNN_FAIL(KNN_EINVAL, "large-k search: more than 2^32 rows");
    if (ix->ntotal == 0) {
        KNN_HIP(launch_fill_empty(D, I, nq * (int64_t)k, kmetric, st));
        return KNN_OK;
    }
    int rc;
    // Small batches: S stripes of running lists per query, so one GEMM round covers S corpus
    // blocks (S x fewer GEMM + select launches, S workgroups per query) and a final kernel merges
    // the S lists (S * k <= kLKM).  Large batches fill the chip with one stripe.
    const int S = nq <= 64 ? (int)std::max<int64_t>(1, std::min<int64_t>(32, kLKM / k)) : 1;
    const int64_t nqc = std::min<int64_t>(nq, 2048);       // queries per GEMM block
    const int nrc_max = kLKM - k;
    const int64_t round_rows = (int64_t)S * nrc_max;
    // workspace sized for ONE query block (queries, norms, GEMM block, running lists), reused
    // by every block: independent of the batch size
    if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)nqc * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)nqc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->lk_g, &ix->lk_g_cap, (size_t)nqc * round_rows)) != KNN_OK) return rc;
    if ((rc = grow(&ix->lk_run, &ix->lk_run_cap, (size_t)S * nqc * k)) != KNN_OK) return rc;
    if (!ix->blas) {
        rocblas_handle h;
        if (rocblas_create_handle(&h) != rocblas_status_success)
            KNN_FAIL(KNN_EHIP, "rocblas_create_handle failed");
        ix->blas = h;
    }
    const rocblas_handle h = (rocblas_handle)ix->blas;
    if (rocblas_set_stream(h, st) != rocblas_status_success) KNN_FAIL(KNN_EHIP, "rocblas_set_stream failed");
    const float alpha = -2.f, beta = 0.f;
    for (int64_t q0 = 0; q0 < nq; q0 += nqc) {
        const int qc = (int)std::min<int64_t>(nqc, nq - q0);
        KNN_HIP(launch_rows_ingest(q + q0 * ix->d, qc, ix->d, ix->dp, qc,
                                   ix->metric == KNN_METRIC_COSINE ? 1 : 0, ix->qpad, ix->qnorm, st));
        float* Db = D + q0 * k;          // the block's outputs; the kernels index it from 0
        int64_t* Ib = I + q0 * k;
        for (int64_t r0 = 0; r0 < ix->ntotal; r0 += round_rows) {
            const int m = (int)std::min<int64_t>(round_rows, ix->ntotal - r0);
            // column-major: G (m x qc, ld m) = X_rows^T (m x dp) * Q_block (dp x qc)
            if (rocblas_sgemm(h, rocblas_operation_transpose, rocblas_operation_none, m, qc, ix->dp,
                              &alpha, ix->xb + r0 * ix->dp, ix->dp, ix->qpad, ix->dp,
                              &beta, ix->lk_g, m) != rocblas_status_success)
                KNN_FAIL(KNN_EHIP, "rocblas_sgemm failed");
            const int last = (S == 1 && r0 + m >= ix->ntotal) ? 1 : 0;
            hipLaunchKernelGGL(largek_select_kernel, dim3((unsigned)qc, (unsigned)S), dim3(kLKThreads), 0, st,
                               ix->lk_g, m, nrc_max, ix->qnorm, ix->xn, r0, k, kmetric, r0 == 0 ? 1 : 0,
                               last, (int64_t)0, nqc, ix->lk_run, Db, Ib, ix->id_offset);
            KNN_HIP(hipGetLastError());
        }
        if (S > 1) {
            hipLaunchKernelGGL(largek_final_kernel, dim3((unsigned)qc), dim3(kLKThreads), 0, st,
                               ix->lk_run, S, nqc, k, (int64_t)0, kmetric, Db, Ib, ix->id_offset);
            KNN_HIP(hipGetLastError());
        }
    }
    return KNN_OK;
}

}  // namespace imgrec
