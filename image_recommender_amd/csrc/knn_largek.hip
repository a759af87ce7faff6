// knn_largek.hip — exact search for KNN_MAX_K < k <= KNN_MAX_K_LARGE (gfx950), hand-written
// end to end (no vendor GEMM, no N x Q key block in HBM).
//
// The fused kernels keep register top-k lists (k <= 32).  faiss IndexFlat serves any k
// (main/search_from_image.py:247 passes the CLI's --top-k), so larger k runs in three steps:
//   1. the exact fp32 tile kernel (knn_tile_topk_kernel, KM = 32) over the whole corpus: per
//      (query, row split, list) the 32 best (key, row) of that list's rows — the key in the same
//      (|q|^2 + |x|^2) - 2 q.x form as every other path;
//   2. largek_union_kernel, a workgroup per query: the k best of the union of all lists by an
//      exact radix select in LDS (running top-k over chunks of the lists), certified against the
//      lists' FLOOR: a row no list kept was screened out by a FULL list (its 32nd key, or its
//      partner lane's, beats the row), so it ranks at or after the smallest 32nd key of any full
//      list; the union's k-th key strictly below that floor proves the union's top-k is the
//      corpus's.  With rows interleaved over the splits in 8-row groups a list holds ~k / lists of
//      the answer (4 at k = 1024 over 256 lists), so the certificate fails only when one list's
//      rows crowd the answer (or k approaches the corpus size);
//   3. the queries it leaves (listed and counted on the device) are re-run by an exact scan: S
//      stripes of the corpus per query, each a workgroup computing its rows' fp32 keys (one wave
//      per row) into LDS and folding them into a running top-k with the same select, then the S
//      lists merged.  The scan's grid is fixed (S stripes x kLKFailWG workgroups that walk the
//      failed queries the device counted), so the host never waits: with every query certified
//      the scan's workgroups read the count and exit (a few us).
// Radix select (select_k): the values are u64 (order-preserving key bits | local row: unsigned
// order = (key, row), faiss's tie rule); eight 8-bit digit passes of a 256-bin LDS histogram find
// the k-th smallest T; the values < T, then copies of T, fill the result (empties = ~0 pad a
// corpus with fewer than k rows); the last round sorts it bitonically.

#include <hip/hip_runtime.h>
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
constexpr int64_t kLKChunk = 1024;  // queries per chunk: bounds the scan's stripe lists (run) to
                                    // kLKChunk x 8192 u64 = 64 MiB
constexpr int kLKFailWG = 64;       // scan / final workgroups walking a chunk's failed queries
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

// Output of a finished top-k list: row q of D / I from sel[0 .. k) (local rows + id_offset).
__device__ void write_topk(const uint64_t* sel, int k, int metric, int64_t id_offset, float* D,
                           int64_t* I) {
    for (int i = threadIdx.x; i < k; i += kLKThreads) {
        const uint64_t x = sel[i];
        if (x == ~0ull) {
            D[i] = metric == 1 ? FLT_MAX : -FLT_MAX;
            I[i] = -1;
        } else {
            const float key = key_from_ordered((uint32_t)(x >> 32));
            D[i] = metric == 1 ? key : -key;
            I[i] = (int64_t)(uint32_t)x + id_offset;
        }
    }
}

// Step 1 for small batches (nq <= 4, d <= 4096): the exact fp32 tile kernel computes 32-query tiles, so one
// query pays for 32 (1M x 1968: 2.9 ms, MFMA-bound on 31 padding queries).  This pass instead
// streams the fp32 corpus once (HBM-bound: 7.9 GB at 1M x 1968) with VALU dot products: one
// 4-wave workgroup per row split (8-row groups s, s + nsplit, ... as the int8 scan), a 16-lane
// group per row, lane j the float4 chunks j, j + 16, ... against the queries' rows in LDS, a DPP
// row sum, lane j (< NQ) of the group keeping query j's list of 32 (insert_mono: rows arrive in
// increasing order per lane, so ties keep the smaller row).  The 16 lists of a split fold to its
// 32 best — the same per-(query, split) lists of exact keys the union certifies (a row a lane
// list dropped has a key >= that list's 32nd >= the folded list's 32nd).  Keys are the exact
// kernel's form, (|q|^2 + |x|^2) - 2 q.x clamped at 0 or -q.x, the dot summed in this kernel's
// own fp32 order.
template <int K>
__device__ __forceinline__ void lk_insert(float (&kd)[K], int (&ki)[K], float d, int id) {
    bool c[K];
#pragma unroll
    for (int p = 0; p < K; ++p) c[p] = d < kd[p];
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        kd[p] = __builtin_amdgcn_fmed3f(kd[p - 1], d, kd[p]);
        const int nx = c[p] ? id : ki[p];
        ki[p] = c[p - 1] ? ki[p - 1] : nx;
    }
    kd[0] = c[0] ? d : kd[0];
    ki[0] = c[0] ? id : ki[0];
}

__device__ __forceinline__ float lk_row16_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
    return v;
}

constexpr int kLKSW = 4;            // waves of the streaming pass
constexpr int kLKSDp = 4096;        // widest padded row of the streaming pass (query rows in LDS)

template <int NQ>
__global__ void __launch_bounds__(kLKSW * 64) __attribute__((amdgpu_waves_per_eu(2)))
largek_stream_kernel(const float* __restrict__ xb, const float* __restrict__ xn, int nrows, int dp,
                     const float* __restrict__ qpad, const float* __restrict__ qnorm, int nq,
                     int nsplit, int metric, int64_t id_offset, float* __restrict__ cand_d,
                     int64_t* __restrict__ cand_i, int ncand) {
    constexpr int KM = KNN_MAX_K;
    __shared__ __attribute__((aligned(16))) float sq[NQ * kLKSDp];
    __shared__ float fd[NQ][16][KM];
    __shared__ int fi[NQ][16][KM];
    const int split = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = lane & 15, g = lane >> 4;
    const int n4 = dp / 4;
    for (int i = tid; i < NQ * n4; i += kLKSW * 64) {
        const int qi = i / n4;
        reinterpret_cast<float4*>(sq)[i] = qi < nq ? reinterpret_cast<const float4*>(qpad)[(int64_t)qi * n4 + (i - qi * n4)]
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float qn[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) qn[q] = (metric == 1 && q < nq) ? qnorm[q] : 0.f;
    __syncthreads();
    float kd[KM];
    int ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }
    const bool owner = j < NQ && j < nq;
    const int ngroups = (nrows + 7) / 8;
    // a wave step: the 4 rows 4 h + g of an 8-row group (two steps per group)
    const int cnt = 2 * (split < ngroups ? (ngroups - split + nsplit - 1) / nsplit : 0);
    const float4* sq4 = reinterpret_cast<const float4*>(sq);
    for (int li = wave; li < cnt; li += kLKSW) {
        const int m = split + (li >> 1) * nsplit;
        const int row = m * 8 + 4 * (li & 1) + g;
        const int rc = min(row, nrows - 1);
        const float4* x4 = reinterpret_cast<const float4*>(xb + (int64_t)rc * dp);
        float acc[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
        // 8 chunks in flight per lane (128 B), then their products
        for (int c0 = j; c0 < n4; c0 += 16 * 8) {
            float4 xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = c0 + 16 * u;
                typedef float f32x4v __attribute__((ext_vector_type(4)));
                if (c < n4) {
                    const f32x4v w = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(x4 + c));
                    xv[u] = make_float4(w.x, w.y, w.z, w.w);
                } else {
                    xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = min(c0 + 16 * u, n4 - 1);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float4 qv = sq4[q * n4 + c];
                    acc[q] = fmaf(xv[u].x, qv.x, acc[q]);
                    acc[q] = fmaf(xv[u].y, qv.y, acc[q]);
                    acc[q] = fmaf(xv[u].z, qv.z, acc[q]);
                    acc[q] = fmaf(xv[u].w, qv.w, acc[q]);
                }
            }
        }
        const float xnr = metric == 1 ? xn[rc] : 0.f;
        float kv = INFINITY;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float dot = lk_row16_sum(acc[q]);
            const float key = metric == 1 ? fmaxf((qn[q] + xnr) - 2.f * dot, 0.f) : -dot;
            kv = j == q ? key : kv;
        }
        kv = (owner && row < nrows && kv < kd[KM - 1]) ? kv : INFINITY;
        if (__any(kv != INFINITY)) lk_insert<KM>(kd, ki, kv, row);
    }
    // fold the split's 16 lists of each query (4 waves x 4 row groups) into its 32 best
    if (owner) {
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            fd[j][wave * 4 + g][p] = kd[p];
            fi[j][wave * 4 + g][p] = ki[p];
        }
    }
    __syncthreads();
    const int fq = wave * 4 + (lane >> 4), fl = lane & 15;
    if (fq >= NQ || fq >= nq) return;                    // (whole 16-lane groups leave together)
    int pos = 0;
    for (int p = 0; p < KM; ++p) {
        float hk = pos < KM ? fd[fq][fl][pos] : INFINITY;
        int hl = pos < KM ? fi[fq][fl][pos] : -1;
        if (hl < 0) hk = INFINITY;
        float bk = hk;
        int bl = hl < 0 ? 0x7fffffff : hl;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
            const float ok = __shfl_xor(bk, o, 16);
            const int ol = __shfl_xor(bl, o, 16);
            if (ok < bk || (ok == bk && ol < bl)) { bk = ok; bl = ol; }
        }
        const bool won = hk == bk && (hl < 0 ? 0x7fffffff : hl) == bl && bk != INFINITY;
        if (won) ++pos;
        if (fl == 0) {
            const int64_t o = (int64_t)fq * ncand + (int64_t)split * KM + p;
            cand_d[o] = bk;
            cand_i[o] = bk == INFINITY ? (int64_t)-1 : (int64_t)bl + id_offset;
        }
    }
}

// Step 2 (module doc): a workgroup per query of the block.  cd / ci: the tile kernel's lists
// (nlists of km ascending keys per query, stride ncand; labels with id_offset, -1 = empty).
// Certified queries are written to D / I; the others go to fail_list (with their union's k-th
// value, the fallback's bound) — fail_cnt counts them.
__global__ void __launch_bounds__(kLKThreads)
largek_union_kernel(const float* __restrict__ cd, const int64_t* __restrict__ ci, int nlists, int km,
                    int ncand, int k, int64_t ntotal, int metric, int64_t id_offset,
                    float* __restrict__ D, int64_t* __restrict__ I, int* __restrict__ fail_list,
                    int* __restrict__ fail_cnt, int* __restrict__ fail_total) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    __shared__ uint32_t s_floor;
    const int t = threadIdx.x;
    const int64_t q = blockIdx.x;
    const float* qd = cd + q * (int64_t)ncand;
    const int64_t* qi = ci + q * (int64_t)ncand;
    if (t == 0) s_floor = ~0u;
    __syncthreads();
    const int M = nlists * km, C = kLKM - k;
    int nr = 0;
    for (int c0 = 0; c0 < M; c0 += C) {
        const int cn = min(C, M - c0);
        for (int i = t; i < nr; i += kLKThreads) v[i] = sel[i];
        for (int e = t; e < cn; e += kLKThreads) {
            const int idx = c0 + e;
            const int64_t lab = qi[idx];
            const uint32_t kb = key_bits_ordered(qd[idx]);
            v[nr + e] = lab < 0 ? ~0ull : ((uint64_t)kb << 32) | (uint32_t)(lab - id_offset);
            // the last entry of a FULL list bounds every row that list (or its partner) dropped
            if (idx % km == km - 1 && lab >= 0) atomicMin(&s_floor, kb);
        }
        __syncthreads();
        select_k(v, nr + cn, k, sel, hist, &s_prefix, &s_rem, &s_nlt, c0 + C >= M);
        nr = k;
    }
    const int kk = (int)min<int64_t>(k, ntotal);
    const uint64_t T = sel[kk - 1];
    const bool ok = s_floor == ~0u || (T != ~0ull && (uint32_t)(T >> 32) < s_floor);
    if (ok) {
        write_topk(sel, k, metric, id_offset, D + q * k, I + q * k);
    } else if (t == 0) {
        fail_list[atomicAdd(fail_cnt, 1)] = (int)q;
        atomicAdd(fail_total, 1);
    }
}

// One (stripe, failed query) item of largek_scan_kernel (workgroup-uniform arguments).
__device__ void largek_scan_one(const float* __restrict__ xb, const float* __restrict__ xn, int64_t ntotal,
                                int dp, const float* __restrict__ qpad, const float* __restrict__ qnorm,
                                int q, int f, int64_t R, int k, int metric, uint64_t* __restrict__ run) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int S = gridDim.x, s = blockIdx.x;
    __syncthreads();                                    // the previous item's LDS reads are done
    const float4* q4 = reinterpret_cast<const float4*>(qpad + (int64_t)q * dp);
    const float qn = qnorm[q];
    const int64_t r0 = (int64_t)s * R, r1 = min(ntotal, r0 + R);
    const int C = kLKM - k;
    const int nv4 = dp / 4;
    int nr = 0;
    for (int64_t c0 = r0; c0 < r1 || (c0 == r0 && nr == 0); c0 += C) {
        const int cn = (int)max<int64_t>(0, min<int64_t>(C, r1 - c0));
        for (int i = t; i < nr; i += kLKThreads) v[i] = sel[i];
        for (int j = wave; j < cn; j += kLKThreads / 64) {
            const int64_t row = c0 + j;
            const float4* x4 = reinterpret_cast<const float4*>(xb + row * dp);
            float acc = 0.f;
            for (int c = lane; c < nv4; c += 64) {
                const float4 a = x4[c], b = q4[c];
                acc = fmaf(a.x, b.x, acc);
                acc = fmaf(a.y, b.y, acc);
                acc = fmaf(a.z, b.z, acc);
                acc = fmaf(a.w, b.w, acc);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
            if (lane == 0) {
                // L2: (|q|^2 + |x|^2) - 2 q.x, clamped at 0; IP: -q.x
                const float key = metric == 1 ? fmaxf((qn + xn[row]) - 2.f * acc, 0.f) : -acc;
                v[nr + j] = ((uint64_t)key_bits_ordered(key) << 32) | (uint32_t)row;
            }
        }
        __syncthreads();
        select_k(v, nr + cn, k, sel, hist, &s_prefix, &s_rem, &s_nlt, false);
        nr = k;
        if (cn == 0) break;
    }
    uint64_t* out = run + ((int64_t)f * S + s) * k;
    for (int i = t; i < k; i += kLKThreads) out[i] = sel[i];
}

// Step 3, a workgroup per (stripe s = blockIdx.x, failed queries f = blockIdx.y, + gridDim.y, ...
// below the device's count): the exact fp32 keys of rows [s R, (s + 1) R) — one wave per row,
// lanes over the row's float4s, a shuffle reduction — folded chunk by chunk into a running top-k
// (select_k), written to run[(f S + s) k ...].  qpad / qnorm: the query block's padded rows and
// norms.
__global__ void __launch_bounds__(kLKThreads)
largek_scan_kernel(const float* __restrict__ xb, const float* __restrict__ xn, int64_t ntotal, int dp,
                   const float* __restrict__ qpad, const float* __restrict__ qnorm,
                   const int* __restrict__ fail_list, const int* __restrict__ fail_cnt, int64_t R,
                   int k, int metric, uint64_t* __restrict__ run) {
    const int nfail = *fail_cnt;                        // written by largek_union_kernel
    for (int f = blockIdx.y; f < nfail; f += gridDim.y)
        largek_scan_one(xb, xn, ntotal, dp, qpad, qnorm, fail_list[f], f, R, k, metric, run);
}

// The S stripe lists of each failed query f (S * k <= kLKM; f = blockIdx.x, + gridDim.x, ...
// below the device's count) -> its final sorted top-k in D / I.
__global__ void __launch_bounds__(kLKThreads)
largek_final_kernel(const uint64_t* __restrict__ run, int S, int k, const int* __restrict__ fail_list,
                    const int* __restrict__ fail_cnt, int metric, int64_t id_offset,
                    float* __restrict__ D, int64_t* __restrict__ I) {
    __shared__ uint64_t v[kLKM];
    __shared__ uint64_t sel[kLKSort];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t s_prefix;
    __shared__ int s_rem, s_nlt;
    const int t = threadIdx.x;
    const int nfail = *fail_cnt;
    const int M = S * k;
    for (int f = blockIdx.x; f < nfail; f += gridDim.x) {
        const int q = fail_list[f];
        __syncthreads();                                // the previous query's LDS reads are done
        for (int e = t; e < M; e += kLKThreads) v[e] = run[(int64_t)f * M + e];
        __syncthreads();
        select_k(v, M, k, sel, hist, &s_prefix, &s_rem, &s_nlt, true);
        write_topk(sel, k, metric, id_offset, D + (int64_t)q * k, I + (int64_t)q * k);
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

// (rows narrower than 128 floats leave most of a row's 16 lanes idle: one query on 1M x 48
// colour rows streams in 0.221 ms against the tile kernel's 0.207 — profiles/r05/stream/)
bool stream_lists_ok(const knn_index* ix, int64_t nq) {
    return ix->stream_lists && nq >= 1 && nq <= 4 && ix->dp >= 128 && ix->dp <= kLKSDp && ix->dp % 4 == 0;
}

int stream_splits(const knn_index* ix) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)ix->cus * 2, (ix->ntotal + 7) / 8));
}

// The streaming list pass (largek_stream_kernel): nq <= 4 padded queries, sp row splits, the
// lists at cd / ci + q * sp * 32 + s * 32.
hipError_t launch_stream_lists(const knn_index* ix, const float* qpad, const float* qnorm, int64_t nq,
                               int metric, int sp, float* cd, int64_t* ci, hipStream_t st) {
    if (nq < 1 || nq > 4 || ix->dp % 4 != 0 || ix->dp > kLKSDp || sp < 1) return hipErrorInvalidValue;
#define IMGREC_LKS(NQV)                                                                            \
    hipLaunchKernelGGL((largek_stream_kernel<NQV>), dim3((unsigned)sp), dim3(kLKSW * 64), 0, st, ix->xb, \
                       ix->xn, (int)ix->ntotal, ix->dp, qpad, qnorm, (int)nq, sp, metric,          \
                       ix->id_offset, cd, ci, sp * KNN_MAX_K)
    if (nq == 1) IMGREC_LKS(1);
    else if (nq == 2) IMGREC_LKS(2);
    else IMGREC_LKS(4);
#undef IMGREC_LKS
    return hipGetLastError();
}

int largek_fallbacks(knn_index* ix, int64_t* n) {
    *n = 0;
    if (!ix->lk_fail) return KNN_OK;
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    int v = 0;
    KNN_HIP(hipMemcpyAsync(&v, ix->lk_fail + kLKChunk + 1, sizeof(int), hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    *n = v;
    return KNN_OK;
}

void largek_free(knn_index* ix) {
    for (void* p : {(void*)ix->lk_run, (void*)ix->lk_fail})
        if (p) (void)hipFree(p);
    ix->lk_run = nullptr;
    ix->lk_fail = nullptr;
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
    // fallback geometry: S stripes per failed query (S k <= kLKM for the final merge); the stripe
    // lists of every query of a chunk have a slot (run), so the device needs no host decision
    const int S = (int)std::max<int64_t>(1, std::min<int64_t>({64, kLKM / k, (ix->ntotal + 1023) / 1024}));
    const int64_t R = (ix->ntotal + S - 1) / S;
    const int64_t chunk = std::min<int64_t>(kLKChunk, nq);
    if ((rc = grow(&ix->lk_run, &ix->lk_run_cap, (size_t)chunk * S * k)) != KNN_OK) return rc;
    // lk_fail: a chunk's failed queries [0, kLKChunk), their count, the search's total
    if ((rc = grow(&ix->lk_fail, &ix->lk_fail_cap, (size_t)kLKChunk + 2)) != KNN_OK) return rc;
    int* cnt = ix->lk_fail + kLKChunk;
    KNN_HIP(hipMemsetAsync(cnt + 1, 0, sizeof(int), st));
    for (int64_t q0 = 0; q0 < nq; q0 += kLKChunk) {
        const int64_t qc = std::min<int64_t>(kLKChunk, nq - q0);
        const Plan p = make_plan(ix->ntotal, qc, KNN_MAX_K, ix->cus);     // KM = 32 lists
        // <= 4 queries whose rows fit the streaming pass's LDS: lists from one fp32 stream of the
        // corpus instead of 32-query tiles (IMGREC_STREAM_LISTS=0 at index creation: tiles)
        const bool stream = stream_lists_ok(ix, qc);
        const int sp = stream_splits(ix);
        const size_t ncap = std::max<size_t>((size_t)p.ncand, (size_t)sp * KNN_MAX_K);
        if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)p.nq_pad * ix->dp)) != KNN_OK) return rc;
        if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)p.nq_pad)) != KNN_OK) return rc;
        if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)qc * ncap)) != KNN_OK) return rc;
        if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)qc * ncap)) != KNN_OK) return rc;
        KNN_HIP(launch_rows_ingest(q + q0 * ix->d, qc, ix->d, ix->dp, p.nq_pad,
                                   ix->metric == KNN_METRIC_COSINE ? 1 : 0, ix->qpad, ix->qnorm, st));
        int nlists = p.ncand / p.km, ncand = p.ncand;
        if (stream) {
            KNN_HIP(launch_stream_lists(ix, ix->qpad, ix->qnorm, qc, kmetric, sp, ix->cand_d, ix->cand_i, st));
            nlists = sp;
            ncand = sp * KNN_MAX_K;
        } else {
            TileArgs a{};
            a.wr = p.wr; a.wq = p.wq; a.km = p.km;
            a.xb = ix->xb; a.xnorm = ix->xn; a.nrows = (int)ix->ntotal; a.dp = ix->dp;
            a.qp = ix->qpad; a.qnorm = ix->qnorm; a.nq = (int)qc; a.metric = kmetric;
            a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb; a.id_offset = ix->id_offset;
            a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand; a.mode = kModeF32;
            KNN_HIP(launch_tile_topk(a, st));
        }
        float* Db = D + q0 * k;
        int64_t* Ib = I + q0 * k;
        KNN_HIP(hipMemsetAsync(cnt, 0, sizeof(int), st));
        hipLaunchKernelGGL(largek_union_kernel, dim3((unsigned)qc), dim3(kLKThreads), 0, st, ix->cand_d,
                           ix->cand_i, nlists, KNN_MAX_K, ncand, k, ix->ntotal, kmetric,
                           ix->id_offset, Db, Ib, ix->lk_fail, cnt, cnt + 1);
        KNN_HIP(hipGetLastError());
        // the certificate's leftovers, as many as the device counted: fixed grids walk them
        const int G = (int)std::min<int64_t>(qc, kLKFailWG);
        hipLaunchKernelGGL(largek_scan_kernel, dim3((unsigned)S, (unsigned)G), dim3(kLKThreads), 0, st,
                           ix->xb, ix->xn, ix->ntotal, ix->dp, ix->qpad, ix->qnorm, ix->lk_fail, cnt, R,
                           k, kmetric, ix->lk_run);
        KNN_HIP(hipGetLastError());
        hipLaunchKernelGGL(largek_final_kernel, dim3((unsigned)G), dim3(kLKThreads), 0, st, ix->lk_run, S,
                           k, ix->lk_fail, cnt, kmetric, ix->id_offset, Db, Ib);
        KNN_HIP(hipGetLastError());
    }
    return KNN_OK;
}

}  // namespace imgrec
