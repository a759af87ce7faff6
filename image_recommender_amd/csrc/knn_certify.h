// knn_certify.h — device code of the candidate paths' certificate shared by the rerank kernel
// (knn_refine.hip) and the certificate tail kernel (knn_kernels.hip): the error bounds of one
// query, the exact fp32 rerank dot products, the second chance over the raw per-split lists, and
// the cross-workgroup hand-off primitives the tail kernel's device-planned exact re-run uses.
// Device code only; included by .hip translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "knn_kernels.h"
#include "wave_ops.h"

namespace imgrec {

template <typename I>
__device__ __forceinline__ bool ranks_before_r(float d1, I i1, float d2, I i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

constexpr int kRerankWaves = 8, kRerankRows = 2, kWideCap = 1024;
// second-chance rows per wave and round (4 measured the same at config 2 and 2 us slower at
// config 3's 1968-element rows: profiles/r05/nq1/direct/)
#ifndef IMGREC_SC_ROWS
#define IMGREC_SC_ROWS 2
#endif
constexpr int kSliceRows = IMGREC_SC_ROWS;
static_assert(kRerankWaves == kRerankWavesHost, "host plans use kRerankWavesHost");

#ifdef IMGREC_TAIL_STAMPS
// diagnostic build only (tools/tail_stamps.py): s_memrealtime (100 MHz, one clock for every
// XCD) per workgroup of the certificate tail
// at fixed points (slot: 0 entry, 1 first claim, 2 slice filtered, 3 slice reranked, 4 slice
// counted, 5 item merged, 6 plan published / seen, 7 exit); 1024 workgroups x 8 slots
__device__ unsigned long long g_tail_stamps[1024 * 8];
#define TAIL_STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < 1024) \
    g_tail_stamps[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// the rerank kernel's workgroup 0 (one-query searches): per wave, slots 0 entry, 1 level-1 lists
// loaded, 2 level-1 selected, 3 level-2 ranked, 4 exit
__device__ unsigned long long g_rr_stamps[8 * 8];
#define RR_STAMP(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) \
    g_rr_stamps[(threadIdx.x >> 6) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TAIL_STAMP(slot) do {} while (0)
#define RR_STAMP(slot) do {} while (0)
#endif

// Error bounds of one query's certificate (DESIGN.md "bf16 path" / "Split path").
struct QueryBounds {
    float qn, xm, nn, e_ip, c_fp, c_trunc;
    int metric;
    static constexpr float u = 1.0f / 8388608.f;   // 2^-23
    __device__ __forceinline__ QueryBounds(const RerankArgs& a, int64_t q) {
        metric = a.metric;
        qn = a.qnorm[q];
        xm = *a.xn_max;
        c_fp = a.c_fp;
        c_trunc = a.c_trunc;
        nn = sqrtf(qn) * sqrtf(xm) * (1.f + 1.0f / 1024.f) + 1e-30f;
        // |approximate q.x - q.x| for every row:
        //   split: c_split |q| max|x|
        //   bf16:  |q.(x - xh) + (q - qh).xh| + accumulation <= |q| R + dq (X + R) + c_acc |qh| |xh|
        //          (Cauchy-Schwarz with the stored residual norms; R = max row residual, X = max
        //          |x|, |qh| <= |q| + dq, |xh| <= X + R), inflated for the bound's fp32 evaluation
        //   i8:    the same with dq = |q - q~| of the two-level int8 query (q8r) and R the int8
        //          copy's residual
        if (a.mode == kModeBF16 || a.mode == kModeI8) {
            const float sq = sqrtf(qn), X = sqrtf(xm), R = *a.xr_max;
            const float dq = a.q_resid ? a.q_resid[q] : 0.f;
            e_ip = (sq * R + dq * (X + R) + a.c_split * (sq + dq) * (X + R)) * (1.f + 1.0f / 256.f) + 1e-30f;
        } else {
            e_ip = a.c_split * nn;
        }
    }
    // |approx key - exact key| bound at key v
    __device__ __forceinline__ float bound_a(float v) const {
        return metric == 1 ? 2.f * e_ip + 2.f * u * (qn + xm + fabsf(v)) : e_ip;
    }
    // |fp32 rerank key - exact key| bound
    __device__ __forceinline__ float bound_f(float v) const {
        return metric == 1 ? 2.f * c_fp * nn + 2.f * u * (qn + xm + fabsf(v)) : c_fp * nn;
    }
    // candidates with approximate key above this cannot reach the top k (the k best by
    // approximate key have exact keys <= a_k + E_a)
    // (a candidate key may sit up to c_trunc |a| below the approximate key it stands for: a
    // lower bound everywhere it bounds rows from below; added where it bounds from above)
    __device__ __forceinline__ float prefix_limit(float a_k) const {
        return a_k + 2.02f * (bound_a(a_k) + bound_f(a_k) + trunc(a_k));
    }
    __device__ __forceinline__ float trunc(float a) const { return c_trunc * fabsf(a); }
};

// Rerank row loads (A/B): IMGREC_RERANK_NT=1 reads the candidate rows non-temporally (each is
// read once per query; the int8 scan's non-temporal stream measured 13-15 % faster than the
// default policy, profiles/r06/nq1_cold/)
#ifndef IMGREC_RERANK_NT
#define IMGREC_RERANK_NT 0
#endif
__device__ __forceinline__ float4 row_load(const float4* p) {
#if IMGREC_RERANK_NT
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(w.x, w.y, w.z, w.w);
#else
    return *p;
#endif
}

// Exact fp32 dot products of one query with R rows (default kRerankRows), one wave,
// lane-strided float4 chunks (x y z w FMAs) then a butterfly: a row's key has the same bits in
// every pass, whatever R.  IT > 0: the query's chunks are in registers (qr); IT = 0: streamed
// with the rows.
template <int IT, int R = kRerankRows>
__device__ __forceinline__ void rerank_dots(const float4* __restrict__ q4, const float4 (&qr)[IT > 0 ? IT : 1],
                                            int n4, int lane, const float4* const (&r4)[R],
                                            float (&acc)[R]) {
    constexpr int kRerankRows = R;
#pragma unroll
    for (int v = 0; v < kRerankRows; ++v) acc[v] = 0.f;
    if constexpr (IT > 0) {
        float4 b[kRerankRows][IT];
#pragma unroll
        for (int v = 0; v < kRerankRows; ++v)
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int i = lane + 64 * it;
                b[v][it] = i < n4 ? row_load(r4[v] + i) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
            for (int v = 0; v < kRerankRows; ++v) {
                acc[v] = fmaf(qr[it].x, b[v][it].x, acc[v]);
                acc[v] = fmaf(qr[it].y, b[v][it].y, acc[v]);
                acc[v] = fmaf(qr[it].z, b[v][it].z, acc[v]);
                acc[v] = fmaf(qr[it].w, b[v][it].w, acc[v]);
            }
    } else {
#pragma unroll 4
        for (int i = lane; i < n4; i += 64) {
            const float4 qa = q4[i];
#pragma unroll
            for (int v = 0; v < kRerankRows; ++v) {
                const float4 bb = row_load(r4[v] + i);
                acc[v] = fmaf(qa.x, bb.x, acc[v]);
                acc[v] = fmaf(qa.y, bb.y, acc[v]);
                acc[v] = fmaf(qa.z, bb.z, acc[v]);
                acc[v] = fmaf(qa.w, bb.w, acc[v]);
            }
        }
    }
#pragma unroll
    for (int v = 0; v < kRerankRows; ++v)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc[v] += __shfl_xor(acc[v], off, 64);
}

__device__ __forceinline__ float rerank_key(float ip, float qn, float xnr, int metric) {
    if (metric == 1) {
        const float kv = fmaf(-2.f, ip, qn + xnr);
        return kv < 0.f ? 0.f : kv;
    }
    return -ip;
}


// ---------------------------------------------------------------------------------------------
// Cross-workgroup hand-off (MI355X_MICROARCH.md "Valid forms"): producer = every storing wave's
// vmcnt(0) wait, the workgroup barrier, then ONE lane's agent-scope release and counter add;
// consumer = that lane's agent-scope acquire after the counter says so, vmcnt(0), then the
// workgroup barrier before any plain load of the handed-off bytes.
__device__ __forceinline__ void wg_release_stores() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Lane 0: release, add 1 to *ctr (agent scope), return the value before the add.
__device__ __forceinline__ int lane0_release_add(int* ctr) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lane0_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Barrier over a grid whose workgroups are all resident (the caller sizes it so): *ctr counts
// arrivals from 0 (zeroed before the launch); every workgroup's stores before it are visible to
// every workgroup after it.  Polls with relaxed agent-scope loads (L2, not L1) and s_sleep.
__device__ __forceinline__ void grid_barrier(int* ctr, int nwg) {
    wg_release_stores();
    if (threadIdx.x == 0) {
        lane0_release_add(ctr);
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nwg)
            __builtin_amdgcn_s_sleep(2);
        lane0_acquire();
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// Second chance for a query the rerank could not certify (item `item` of chance_list): every
// entry of the candidate pass's per-split lists with approximate key <= the prefix limit (those
// above it cannot reach the top k) is reranked, and the certificate is re-run against the list
// floor alone — the smallest last key of a full list, below which no row outside all lists can
// be.  A query it cannot settle goes to the exact re-run list (stats[0]).
//
// The item is cut into a.sc_slices slices (lists slice, slice + S, ...) that different
// workgroups rerank at once — a one-query search's second chance is a few hundred dependent row
// loads, ~350 us in one 2-wave workgroup, ~10 us spread over the grid.  A slice keeps its k best
// exact (key, label) in the item's workspace and folds its list floor into the item's atomic
// minimum; the workgroup that completes the item's last slice ranks the S x k survivors (the
// item's k best are among them), checks the certificate, writes the answer and resets the
// item's counters.  NW waves per workgroup.  Returns 0 (not the item's last slice), 1 (the item
// answered) or 2 (the item queued for the exact re-run).
struct SecondChanceLDS {
    float w_key[kWideCap], w_apx[kWideCap];
    int64_t w_lab[kWideCap];
    float o_key[64];
    int64_t o_lab[64];
    int w_n;
    unsigned w_tau;
    unsigned s_ratio;
    float s_sk;
    int s_last;
    int s_flag;
    unsigned s_heads[64];       // RerankArgs::direct: per lane, the smallest list head (key bits)
    float s_thr;
};

// agent-scope relaxed store (global_store ... sc1): written through to where every XCD reads it
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NW>
__device__ __forceinline__ int second_chance_slice(const RerankArgs& a, int item, int slice,
                                                   SecondChanceLDS& L, int q_item0) {
    constexpr int NT = NW * 64;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int dp = a.dp, k = a.k, metric = a.metric, kc = a.kc, S = a.sc_slices;
    const int n4 = dp / 4;
    const float4 none[1] = {make_float4(0.f, 0.f, 0.f, 0.f)};
    // (item 0's query: loaded at entry; direct: item i is query i)
    const int64_t q = a.direct ? (int64_t)item : item == 0 ? q_item0 : a.chance_list[item];
    const float* rd = a.raw_d + q * a.raw_stride_q;
    const int64_t* ri = a.raw_i + q * a.raw_stride_q;
    const int km = a.raw_km;
    const int nl = (a.raw_lists - slice + S - 1) / S;          // lists slice, slice + S, ...
    const int ne = nl * km;
    auto entry = [&](int j) { return (slice + (j / km) * S) * km + j % km; };
    // the slice's first kPre entries per thread are loaded together with the bounds' inputs (one
    // dependent round trip instead of two; a one-query second chance is a chain of them)
    // (16 measured the same at config 2's 2048 entries per slice of unfolded lists and 0.6 us
    // slower at config 3: profiles/r05/nq1/direct_raw/)
    constexpr int kPre = 8;
    float pv[kPre];
    int64_t pl[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const int j = t + u * NT;
        pl[u] = -1;
        pv[u] = INFINITY;
        if (j < ne) {
            pl[u] = ri[entry(j)];
            pv[u] = rd[entry(j)];
        }
    }
    const QueryBounds B(a, q);
    float thr;
    if (!a.direct) {
        // the same prefix limit as the first pass, from the merged candidates' k-th key
        const int nvalid = (int)__popcll(__ballot(lane < kc && a.ci[q * kc + lane] >= 0));
        thr = nvalid >= k ? B.prefix_limit(a.cd[q * kc + k - 1]) : INFINITY;
    } else {
        // no merge ran: U = the k-th smallest of 64 lane minima of the lists' first keys (lane
        // l: lists l, l + 64, ...; the scan wrote them contiguously, I8Args::heads) is >= the k-th
        // approximate key a_k (k distinct entries are <= U), so prefix_limit(U) >= the first
        // pass's limit and every entry that can reach the top k is still reranked (fewer than k
        // non-empty minima: +inf, every entry)
        if (wave == 0) {
            constexpr int kH = 12;              // lists per lane loaded in one round (<= 768)
            const int nh = a.heads_n > 0 ? a.heads_n : a.raw_lists;
            const float* hd = a.heads + q * nh;
            float hv[kH];
#pragma unroll
            for (int u = 0; u < kH; ++u) {
                const int l = lane + 64 * u;
                hv[u] = l < nh ? hd[l] : INFINITY;
            }
            unsigned m = 0xffffffffu;
#pragma unroll
            for (int u = 0; u < kH; ++u)
                if (hv[u] != INFINITY) m = min(m, key_bits_ordered(hv[u]));
            for (int l = lane + 64 * kH; l < nh; l += 64)
                if (hd[l] != INFINITY) m = min(m, key_bits_ordered(hd[l]));
            L.s_heads[lane] = m;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            int r = 0;                          // rank of (m, lane) among the 64
#pragma unroll 8
            for (int i = 0; i < 64; ++i) {
                const unsigned x = L.s_heads[i];
                r += (x < m || (x == m && i < lane)) ? 1 : 0;
            }
            const uint64_t hit = __ballot(m != 0xffffffffu && r == k - 1);
            if (lane == 0)
                L.s_thr = hit ? B.prefix_limit(key_from_ordered(L.s_heads[__builtin_ctzll(hit)])) : INFINITY;
        }
        __syncthreads();
        thr = L.s_thr;
    }
    if (t == 0) {
        L.w_n = 0;
        L.w_tau = 0xffffffffu;
        L.s_ratio = 0u;
    }
    __syncthreads();
    // a full list (last entry valid) bounds the rows it dropped: its last key is a floor; the
    // entries under the prefix limit are reranked
    auto take = [&](int j, int64_t l, float v) __attribute__((always_inline)) {
        if (j % km == km - 1 && l >= 0) atomicMin(&L.w_tau, key_bits_ordered(v));
        if (l >= 0 && v <= thr) {
            const int s2 = atomicAdd(&L.w_n, 1);
            if (s2 < kWideCap) { L.w_apx[s2] = v; L.w_lab[s2] = l; }
        }
    };
#pragma unroll
    for (int u = 0; u < kPre; ++u)
        if (t + u * NT < ne) take(t + u * NT, pl[u], pv[u]);
    // the rest in batches of kPre loads per thread (the direct route's unfolded lists: up to
    // 2048 entries per slice)
    for (int j0 = t + kPre * NT; j0 < ne; j0 += kPre * NT) {
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
            const int j = j0 + u * NT;
            pl[u] = j < ne ? ri[entry(j)] : -1;
            pv[u] = j < ne ? rd[entry(j)] : INFINITY;
        }
#pragma unroll
        for (int u = 0; u < kPre; ++u)
            if (j0 + u * NT < ne) take(j0 + u * NT, pl[u], pv[u]);
    }
    __syncthreads();
    TAIL_STAMP(2);
    const int n = L.w_n;
    const bool overflow = n > kWideCap;
    float* const ok_ = a.sc_key + ((int64_t)item * S + slice) * k;
    int64_t* const ol_ = a.sc_lab + ((int64_t)item * S + slice) * k;
    if (!overflow) {
        const float4* q4 = reinterpret_cast<const float4*>(a.qp + q * dp);
        // kSliceRows rows per wave and round (the rows' keys have the same bits whatever the count)
        for (int c0 = wave; c0 < n; c0 += NW * kSliceRows) {
            const float4* r4[kSliceRows];
            float acc[kSliceRows], xr[kSliceRows];
#pragma unroll
            for (int v = 0; v < kSliceRows; ++v) {
                const int64_t row = L.w_lab[min(c0 + NW * v, n - 1)] - a.id_offset;
                r4[v] = reinterpret_cast<const float4*>(a.xb + row * dp);
                xr[v] = a.xn[row];                      // loaded with the row, not after it
            }
            rerank_dots<0, kSliceRows>(q4, none, n4, lane, r4, acc);
#pragma unroll
            for (int v = 0; v < kSliceRows; ++v) {
                const int c = c0 + NW * v;
                if (lane == 0 && c < n) L.w_key[c] = rerank_key(acc[v], B.qn, xr[v], metric);
            }
        }
        __syncthreads();
        TAIL_STAMP(3);
        // this slice's k best by (key, label) (labels are distinct: a row sits in one list);
        // the observed error / bound goes to the chunk's maximum once per workgroup (one
        // same-address global atomic per reranked entry serialised the slices: ~100 us)
        float rmax = 0.f;
        for (int s2 = t; s2 < n; s2 += NT) {
            const float kv = L.w_key[s2];
            const int64_t lb = L.w_lab[s2];
            int rank = 0;
            for (int j = 0; j < n && rank < k; ++j)
                rank += ranks_before_r(L.w_key[j], L.w_lab[j], kv, lb) ? 1 : 0;
            if (rank < k) { st_sc1(ok_ + rank, kv); st_sc1(ol_ + rank, lb); }
            rmax = fmaxf(rmax, fabsf(L.w_apx[s2] - kv) /
                                   (B.bound_a(L.w_apx[s2]) + B.bound_f(kv) + B.trunc(L.w_apx[s2])));
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, off, 64));
        if (lane == 0) atomicMax(&L.s_ratio, __float_as_uint(rmax));
    }
    for (int r = t; r < k; r += NT)
        if (overflow || r >= n) { st_sc1(ok_ + r, INFINITY); st_sc1(ol_ + r, (int64_t)-1); }
    __syncthreads();                                    // L.s_ratio complete
    if (t == 0) {                                       // the slice's floor, error ratio, overflow
        unsigned* meta = a.sc_meta + ((int64_t)item * S + slice) * 4;
        st_sc1(meta, L.w_tau);
        st_sc1(meta + 1, L.s_ratio);
        st_sc1(meta + 2, overflow ? 1u : 0u);
    }
    // Hand-off without an L2 write-back (MI355X_MICROARCH.md, valid forms, table row 1): the
    // slice lists are stored sc1, every storing wave waits for its stores, then ONE lane adds to
    // the item's counter; the workgroup whose add comes last reads them with sc1 loads only (an
    // agent release per slice — buffer_wbl2 of the XCD's L2 — made the slices' completions
    // serialise: ~5 us per slice).  ONE same-address atomic per slice: the slice's floor, error
    // ratio and overflow go to its own meta slot (three agent atomics per slice on per-item
    // words — and one more on the chunk's ratio — cost ~2 us per slice, serialised).
    wg_release_stores();
    if (t == 0)
        L.s_last = __hip_atomic_fetch_add(a.sc_done + item, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
    __syncthreads();
    const bool last = L.s_last != 0;
    __syncthreads();                                    // L reused below / by the next slice
    TAIL_STAMP(4);
    if (!last) return 0;

    // ---- the item's last slice: merge the S sorted slice lists (k each) in one wave — k rounds
    // of a wave u64 minimum over the S list heads, (ordered key bits | split-local label)
    // (a quadratic rank of the S x k survivors cost ~80 us at S = 32), certify, answer
    const float* sk_ = a.sc_key + (int64_t)item * S * k;
    const int64_t* sl_ = a.sc_lab + (int64_t)item * S * k;
    // the S x k (<= kWideCap) slice lists staged in LDS by one round of independent sc1 loads:
    // the merge's k rounds then read their heads from LDS (a dependent agent-scope load per
    // round, ~1 us each across XCDs, was most of a one-query second chance)
    // (unrolled: every load in flight before the first LDS store — a rolled loop waited for each
    // iteration's loads in turn, ~7 us of a one-query second chance, tools/tail_stamps.py)
    constexpr int kStg = (kWideCap + NT - 1) / NT;
    int64_t slb[kStg];
    float skv[kStg];
#pragma unroll
    for (int u = 0; u < kStg; ++u) {
        const int e = t + u * NT;
        if (e < S * k) {
            slb[u] = __hip_atomic_load(sl_ + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            skv[u] = __hip_atomic_load(sk_ + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#pragma unroll
    for (int u = 0; u < kStg; ++u) {
        const int e = t + u * NT;
        if (e < S * k) {
            L.w_lab[e] = slb[u];
            L.w_key[e] = skv[u];
        }
    }
    // the slices' floor, error ratio and overflow, loaded in the same round
    unsigned tb = 0xffffffffu, rb = 0u, fb = 0u;
    if (wave == 0 && lane < S) {
        const unsigned* meta = a.sc_meta + ((int64_t)item * S + lane) * 4;
        tb = __hip_atomic_load(meta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rb = __hip_atomic_load(meta + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fb = __hip_atomic_load(meta + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (wave == 0) {
        auto head = [&](int p) -> uint64_t {
            if (lane >= S || p >= k) return ~0ull;
            const int64_t lb = L.w_lab[lane * k + p];
            const float kv = L.w_key[lane * k + p];
            return lb < 0 ? ~0ull : ((uint64_t)key_bits_ordered(kv) << 32) | (uint32_t)(lb - a.id_offset);
        };
        L.o_key[lane] = INFINITY;                       // rounds after an exhausted merge: empty
        L.o_lab[lane] = -1;
        int p = 0;
        uint64_t h = head(0);
        float sk = -INFINITY;
        for (int r = 0; r < k; ++r) {
            const uint64_t m = wave_min_u64(h);
            if (lane == 0) {
                L.o_key[r] = m == ~0ull ? INFINITY : key_from_ordered((uint32_t)(m >> 32));
                L.o_lab[r] = m == ~0ull ? (int64_t)-1 : (int64_t)(uint32_t)m + a.id_offset;
            }
            if (m == ~0ull) break;
            if (r == k - 1) sk = key_from_ordered((uint32_t)(m >> 32));
            if (h == m) h = head(++p);                  // unique: a row sits in one list
        }
        if (lane == 0) L.s_sk = sk;
        // the item's floor (min over slices), error ratio (max) and overflow (any)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            tb = min(tb, (unsigned)__shfl_xor((int)tb, off, 64));
            rb = max(rb, (unsigned)__shfl_xor((int)rb, off, 64));
            fb |= (unsigned)__shfl_xor((int)fb, off, 64);
        }
        if (lane == 0) {
            L.w_tau = tb;
            L.s_flag = (int)fb;
            if (rb) atomicMax(reinterpret_cast<unsigned*>(a.stats + 1), rb);
        }
    }
    __syncthreads();
    const unsigned tbm = L.w_tau;
    const int flag = L.s_flag;
    // +inf floor: no list dropped a row, so every row was a candidate and the slices hold all
    // that can matter
    const float tauL = tbm == 0xffffffffu ? INFINITY : key_from_ordered(tbm);
    const bool ok = flag == 0 && (tauL == INFINITY || (tauL - B.bound_a(tauL)) > (L.s_sk + B.bound_f(L.s_sk)));
    if (ok) {
        if (t < k) {
            const int64_t lb = L.o_lab[t];
            a.D[q * k + t] = lb < 0 ? ((metric == 1) ? FLT_MAX : -FLT_MAX)
                                    : ((metric == 1) ? L.o_key[t] : -L.o_key[t]);
            a.I[q * k + t] = lb;
        }
    } else if (t == 0) {
        a.fail_list[atomicAdd(a.stats, 1)] = (int)q;
    }
    __syncthreads();
    if (t == 0) a.sc_done[item] = 0;                    // ready for the next search's items
    TAIL_STAMP(5);
    return ok ? 1 : 2;
}

}  // namespace imgrec
