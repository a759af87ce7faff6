// knn_refine.hip — candidate paths of the exact k-NN search (gfx950): split-bf16 and bf16.
//
// The fused kernel (knn_kernels.hip, SPLIT=true) scores every corpus row against every query with
// three bf16 MFMAs per 16-deep step (x = hi + lo, both bf16; q.x ~= qh.xh + qh.xl + ql.xh), 5.3x
// fewer matrix cycles than the exact v_mfma_f32_32x32x2_f32 form, and keeps the K' best
// approximate keys per query (K' > k).  This file turns that candidate set into the exact answer:
//
//   split_rows      fp32 rows -> split layout (per BK-deep stage j, lane half h and MFMA k-step
//                   s < BK/16: a 16-B hi chunk and a 16-B lo chunk, logical chunks
//                   h*(BK/8) + 2s and +1, holding depth BK*j + 16s + 8h + 0..7).
//   rerank_certify  one workgroup per query: exact fp32 keys of the K' candidates (the same
//                   faiss exhaustive_L2sqr_blas key form as the exact kernel), top-k by
//                   (key, label), and a certificate that no row outside the candidate set can
//                   rank before a returned row:
//                       tau - E_approx > s_k + E_fp32
//                   tau = K'-th approximate key (every excluded row's approximate key is >= tau),
//                   s_k = k-th exact key, E_* rigorous error bounds (DESIGN.md "Split path").
//                   A query whose certificate fails is listed; the host re-runs it on the exact
//                   fp32 kernel.  So the returned (D, I) always carry the exact path's guarantee.
//   gather_rows / scatter_results   compact the failed queries for that re-run and put back.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "knn_certify.h"
#include "knn_kernels.h"
#include "wave_ops.h"

namespace imgrec {

__device__ __forceinline__ uint32_t bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// one thread per (row, BK-deep stage j, lane half h, k-step s): 8 floats in, 32 B out
__global__ void __launch_bounds__(256)
split_rows_kernel(const float* __restrict__ src, int64_t n, int dp, int bk,
                  uint32_t* __restrict__ dst) {
    const int per_row = dp / 8;                      // (dp/bk) stages x 2 halves x bk/16 k-steps
    const int ks = bk / 16;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * per_row) return;
    const int64_t row = t / per_row;
    const int r = (int)(t - row * per_row);
    const int j = r / (2 * ks), h = (r / ks) & 1, s = r % ks;
    const float* x = src + row * dp + j * bk + 16 * s + 8 * h;
    const float4 v0 = *reinterpret_cast<const float4*>(x);
    const float4 v1 = *reinterpret_cast<const float4*>(x + 4);
    const float e[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t h0 = bf16_rne(e[2 * p]), h1 = bf16_rne(e[2 * p + 1]);
        const uint32_t l0 = bf16_rne(e[2 * p] - __uint_as_float(h0 << 16));
        const uint32_t l1 = bf16_rne(e[2 * p + 1] - __uint_as_float(h1 << 16));
        hi[p] = h0 | (h1 << 16);
        lo[p] = l0 | (l1 << 16);
    }
    // logical chunk h*2ks + 2s (hi) and +1 (lo): 32 contiguous bytes
    uint32_t* o = dst + row * dp + j * bk + (h * 2 * ks + 2 * s) * 4;
    *reinterpret_cast<uint4*>(o) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    *reinterpret_cast<uint4*>(o + 4) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
}

// One wave per row: fp32 row (stride dp words) -> bf16 row (stride dpb elements, RNE, zero
// padded) and the Euclidean norm of the rounding residual x - bf16(x), accumulated in fp32 (the
// certificate inflates it, knn_capi.cpp bf16 bound).
__global__ void __launch_bounds__(256)
bf16_rows_kernel(const float* __restrict__ src, int64_t n, int dp, int dpb,
                 uint16_t* __restrict__ dst, float* __restrict__ resid) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* x = src + row * dp;
    uint16_t* o = dst + row * dpb;
    float acc = 0.f;
    for (int c = lane; c < dpb / 8; c += 64) {         // 8 elements (16 B out) per lane step
        float e[8];
        if (8 * c + 8 <= dp) {
            const float4 v0 = *reinterpret_cast<const float4*>(x + 8 * c);
            const float4 v1 = *reinterpret_cast<const float4*>(x + 8 * c + 4);
            e[0] = v0.x; e[1] = v0.y; e[2] = v0.z; e[3] = v0.w;
            e[4] = v1.x; e[5] = v1.y; e[6] = v1.z; e[7] = v1.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) e[j] = (8 * c + j < dp) ? x[8 * c + j] : 0.f;
        }
        uint32_t w[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t h0 = bf16_rne(e[2 * p]), h1 = bf16_rne(e[2 * p + 1]);
            const float r0 = e[2 * p] - __uint_as_float(h0 << 16);
            const float r1 = e[2 * p + 1] - __uint_as_float(h1 << 16);
            acc = fmaf(r0, r0, acc);
            acc = fmaf(r1, r1, acc);
            w[p] = h0 | (h1 << 16);
        }
        *reinterpret_cast<uint4*>(o + 8 * c) = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) resid[row] = sqrtf(acc);
}

// One wave per query row, the bf16 path's whole query side in one pass: raw row (d floats) ->
// padded fp32 row (dp, zero tail; L2-normalised when `normalize`, faiss fvec_renorm_L2 scale), its
// |q|^2, the bf16 row (dpb, RNE) and |q - bf16(q)|.  Rows n..n_pad-1 are zero.  Each lane holds
// chunks of 8 elements (c = lane + 64 it) in registers; dpb <= 512 * IT.
template <int IT>
__global__ void __launch_bounds__(256)
query_prep_b16_kernel(const float* __restrict__ src, int64_t n, int d, int dp, int dpb,
                      int64_t n_pad, int normalize, float* __restrict__ dst,
                      float* __restrict__ norms, uint16_t* __restrict__ qb,
                      float* __restrict__ resid) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_pad) return;
    const bool real = row < n;
    const float* s = src + row * d;
    float e[IT][8];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int j0 = 8 * (lane + 64 * it);
        if (real && (d & 3) == 0 && j0 + 8 <= d) {
            const float4 v0 = *reinterpret_cast<const float4*>(s + j0);
            const float4 v1 = *reinterpret_cast<const float4*>(s + j0 + 4);
            e[it][0] = v0.x; e[it][1] = v0.y; e[it][2] = v0.z; e[it][3] = v0.w;
            e[it][4] = v1.x; e[it][5] = v1.y; e[it][6] = v1.z; e[it][7] = v1.w;
        } else {
#pragma unroll
            for (int t = 0; t < 8; ++t) e[it][t] = (real && j0 + t < d) ? s[j0 + t] : 0.f;
        }
    }
    float scale = 1.f;
    if (normalize) {
        float acc = 0.f;
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
            for (int t = 0; t < 8; ++t) acc = fmaf(e[it][t], e[it][t], acc);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (acc > 0.f) scale = (float)(1.0 / (double)sqrtf(acc));
    }
    float nacc = 0.f, racc = 0.f;
    float* o = dst + row * dp;
    uint16_t* ob = qb + row * dpb;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = lane + 64 * it;
        if (8 * c >= dpb) continue;
        float v[8];
        uint32_t w[4];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            v[t] = normalize ? e[it][t] * scale : e[it][t];
            nacc = fmaf(v[t], v[t], nacc);
        }
#pragma unroll
        for (int p2 = 0; p2 < 4; ++p2) {
            const uint32_t h0 = bf16_rne(v[2 * p2]), h1 = bf16_rne(v[2 * p2 + 1]);
            const float r0 = v[2 * p2] - __uint_as_float(h0 << 16);
            const float r1 = v[2 * p2 + 1] - __uint_as_float(h1 << 16);
            racc = fmaf(r0, r0, racc);
            racc = fmaf(r1, r1, racc);
            w[p2] = h0 | (h1 << 16);
        }
        *reinterpret_cast<uint4*>(ob + 8 * c) = make_uint4(w[0], w[1], w[2], w[3]);
        if (8 * c < dp) {                                    // dp is a multiple of 16
            *reinterpret_cast<float4*>(o + 8 * c) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4*>(o + 8 * c + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        nacc += __shfl_xor(nacc, off, 64);
        racc += __shfl_xor(racc, off, 64);
    }
    if (lane == 0) {
        norms[row] = nacc;
        resid[row] = sqrtf(racc);
    }
}

// One workgroup of kRerankWaves waves per query.  a.cd/a.ci: the merged approximate candidates,
// nq x kc, ascending raw keys (L2 distance or -ip), empty = label -1.
// IT > 0: the query row sits in registers (IT float4 per lane, dp <= 256 IT) and every wave loads
// its candidates' rows kRerankRows at a time, all loads in flight at once; IT = 0 streams the
// query with the rows (any dp).
// A query whose certificate fails goes to the second-chance queue (a.raw_d set: stats[3] counts
// it) or straight to the exact re-run list (stats[0]).
// NW waves per workgroup: 8, or 4 (RerankArgs::nw, opt-in for large batches; no fused merge
// there): at the register budget of four waves per SIMD a CU then holds four workgroups instead
// of two — measured no faster (profiles/r05/rerank_nw4_ab/).
template <int IT, bool SL, int NW>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(4)))
rerank_certify_kernel(const RerankArgs a) {
    __shared__ float skey[64];
    __shared__ int64_t slab[64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t q = blockIdx.x;
    const int dp = a.dp, kc = a.kc, k = a.k, metric = a.metric;
    const int64_t id_offset = a.id_offset;
    // the certificate tail kernel's grid-barrier counters start from zero (it runs next)
    if (a.tail_ctl && blockIdx.x == 0 && threadIdx.x < 4) a.tail_ctl[threadIdx.x] = 0;
    RR_STAMP(0);
    // exact fp32 keys of the prefix (below): candidate c goes to wave c % kRerankWaves; the query
    // row is loaded first (while wave 0 runs the fused merge level)
    const int n4 = dp / 4;
    const float4* q4 = reinterpret_cast<const float4*>(a.qp + q * dp);
    float4 qr[IT > 0 ? IT : 1];
    if constexpr (IT > 0) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = lane + 64 * it;
            qr[it] = i < n4 ? q4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#ifdef IMGREC_TAIL_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // (diagnostic: the query row's round trip)
    RR_STAMP(5);
#endif
    // the candidate merge's second level (RerankArgs::l1_G): the query's E = 16 l1_G level-1
    // entries (<= one per thread) packed (order-preserving key bits | row) in LDS; each thread
    // ranks its entry against all E (broadcast LDS reads; entries are distinct: a row sits in
    // one list) and the kc smallest land at their ranks — for this kernel (LDS) and the second
    // chance (global).  (The wave threshold select of cand_merge_lane_kernel took ~10 us here:
    // 32 dependent wave-sum steps in one wave while seven waited.)
    const bool fused = NW == kRerankWaves && (a.l1_G > 0 || (SL && a.s_lists > 0));   // (SL: the instance with s_lists)
    __shared__ float s_mkey[64];
    __shared__ int64_t s_mlab[64];
    __shared__ __attribute__((aligned(16))) uint64_t s_ent[kRerankWaves * 64];
    __shared__ float s_floor;
    // RerankArgs::l0_lists: the first level too — wave w selects the 16 best of raw lists
    // 64 w .. 64 w + 63 (wave_select_sorted, as cand_merge_lane_kernel would in its own launch)
    // into s_ent[16 w ..] and the group's floor (the last key of its full lists) into s_gfl[w]
    __shared__ uint64_t s_sel[kRerankWaves][64 + 256];
    __shared__ float s_gfl[kRerankWaves];
    if (SL && fused && a.s_lists > 0) {
        // RerankArgs::s_lists: the single-level merge (<= 64 lists of raw_km <= 16 entries: the
        // large batches' per-split lists) by the whole workgroup.  Thread t holds entries t and
        // t + 512; U = the kc-th smallest of the lists' first two entries bounds the answer (kc
        // distinct entries are <= it), the entries <= U are compacted in LDS and each ranked
        // against the others; the kc best land at their ranks (LDS for the rerank, global for the
        // second chance) and the floor is the smallest last key of the full lists — the same
        // result as cand_merge_lane_kernel's wave select, without its launch or the candidates'
        // round trip through global memory.
        constexpr uint64_t kEmpty = ~0ull;
        constexpr int NT = kRerankWaves * 64;
        const int t = threadIdx.x, KIN = a.raw_km, L = a.s_lists, E = L * KIN;
        const float* rd = a.raw_d + q * a.raw_stride_q;
        const int64_t* ri = a.raw_i + q * a.raw_stride_q;
        uint64_t* lead = &s_sel[0][0];                       // 2 L leading entries
        uint64_t* surv = &s_sel[0][0] + 128;                 // survivors (<= E - 128 + 128)
        __shared__ uint64_t s_U;
        __shared__ int s_cnt;
        uint64_t v[2] = {kEmpty, kEmpty};
        float fl = INFINITY;
        int nlead = 0, nval = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int e = t + NT * h;
            if (e < E) {
                const int64_t lb = ri[e];
                const float kv = rd[e];
                if (lb >= 0) {
                    v[h] = ((uint64_t)key_bits_ordered(kv) << 32) | (uint32_t)(lb - id_offset);
                    ++nval;
                    if (e % KIN == KIN - 1) fl = fminf(fl, kv);  // a full list: its last key
                }
                const int p = e % KIN;
                if (p < 2) {
                    lead[(e / KIN) * 2 + p] = v[h];
                    nlead += v[h] != kEmpty ? 1 : 0;
                }
            }
        }
        if (t == 0) s_cnt = 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
        if (lane == 0) s_gfl[wave] = fl;
        int nlead_all = 0, nval_all = 0;
        {                                                    // (its barrier also publishes lead[])
            __shared__ int s_nl[kRerankWaves], s_nv[kRerankWaves];
            const int wl = wave_sum_i32(nlead), wv = wave_sum_i32(nval);
            if (lane == 0) { s_nl[wave] = wl; s_nv[wave] = wv; }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < kRerankWaves; ++i) { nlead_all += s_nl[i]; nval_all += s_nv[i]; }
        }
        const int K = min(kc, nval_all);
        if (nlead_all >= kc) {
            // exactly one valid leading entry has rank kc - 1 among the 2 L (distinct entries)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = t + NT * h;
                if (e < E && e % KIN < 2 && v[h] != kEmpty) {
                    int r = 0;
                    for (int j = 0; j < 2 * L; ++j) r += lead[j] < v[h] ? 1 : 0;
                    if (r == kc - 1) s_U = v[h];
                }
            }
        } else if (t == 0) {
            s_U = kEmpty - 1;                                // fewer than kc leads: all compete
        }
        __syncthreads();
        const uint64_t U = s_U;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (v[h] <= U) surv[atomicAdd(&s_cnt, 1)] = v[h];
        __syncthreads();
        const int C = s_cnt;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (v[h] <= U) {
                int r = 0;
                for (int j = 0; j < C; ++j) r += surv[j] < v[h] ? 1 : 0;
                if (r < K) {
                    const float kv = key_from_ordered((uint32_t)(v[h] >> 32));
                    const int64_t lb = (int64_t)(uint32_t)v[h] + id_offset;
                    s_mkey[r] = kv; s_mlab[r] = lb;
                    a.cd[q * kc + r] = kv; a.ci[q * kc + r] = lb;
                }
            }
        }
        if (t >= K && t < kc) {
            s_mkey[t] = FLT_MAX; s_mlab[t] = -1;
            a.cd[q * kc + t] = FLT_MAX; a.ci[q * kc + t] = -1;
        }
        if (wave == 0) {
            float f = lane < kRerankWaves ? s_gfl[lane] : INFINITY;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) f = fminf(f, __shfl_xor(f, off, 64));
            if (lane == 0) { s_floor = f; a.floor[q] = f; }
        }
        __syncthreads();
        RR_STAMP(3);
    } else if (fused) {
        constexpr uint64_t kEmpty = ~0ull;
        const int t = threadIdx.x, G = a.l1_G, E = 16 * G;
        uint64_t mine = kEmpty;
        if (a.l0_lists > 0) {
            if (wave < G) {
                const int l = 64 * wave + lane;
                const float* rd = a.raw_d + q * a.raw_stride_q + (int64_t)l * 16;
                const int64_t* ri = a.raw_i + q * a.raw_stride_q + (int64_t)l * 16;
                uint64_t v[16];
                float fl = INFINITY;
                if (l < a.l0_lists) {
#pragma unroll
                    for (int p = 0; p < 16; ++p) {
                        const int64_t lb = ri[p];
                        v[p] = lb < 0 ? kEmpty
                                      : ((uint64_t)key_bits_ordered(rd[p]) << 32) | (uint32_t)(lb - id_offset);
                    }
                    if (ri[15] >= 0) fl = rd[15];       // a full list: its last key
                } else {
#pragma unroll
                    for (int p = 0; p < 16; ++p) v[p] = kEmpty;
                }
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
                RR_STAMP(1);
#ifdef IMGREC_TAIL_STAMPS
                {   // diagnostic: the same lists loaded again (warm caches, warm code): slot 6
                    const int l2_ = 64 * wave + lane;
                    const float* rd2 = a.raw_d + q * a.raw_stride_q + (int64_t)l2_ * 16;
                    const int64_t* ri2 = a.raw_i + q * a.raw_stride_q + (int64_t)l2_ * 16;
                    uint64_t acc2 = 0;
                    if (l2_ < a.l0_lists) {
#pragma unroll
                        for (int p = 0; p < 16; ++p) acc2 += (uint64_t)ri2[p] ^ __float_as_uint(rd2[p]);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" :: "v"(acc2) : "memory");
                    RR_STAMP(6);
                }
#endif
                uint64_t m1;
                int r1;
                const int K1 = wave_select_sorted<16, 1, 256>(v, 16, s_sel[wave], m1, r1);
                if (lane < K1) s_ent[16 * wave + r1] = m1;
                else if (lane < 16) s_ent[16 * wave + lane] = kEmpty;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                // a group that kept 16 bounds the rows it dropped by its 16th key (as level 2
                // folds a full level-1 list's last key)
                const uint64_t last = s_ent[16 * wave + 15];
                if (last != kEmpty) fl = fminf(fl, key_from_ordered((uint32_t)(last >> 32)));
                if (lane == 0) s_gfl[wave] = fl;
                RR_STAMP(2);
            }
            __syncthreads();
            if (t < E) mine = s_ent[t];
            if (wave == 0) {
                float fl = lane < G ? s_gfl[lane] : INFINITY;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
                if (lane == 0) s_floor = fl;
            }
        } else {
            const float* ld = a.l1_d + q * E;
            const int64_t* li = a.l1_i + q * E;
            if (t < E) {
                const int64_t lb = li[t];
                if (lb >= 0) mine = ((uint64_t)key_bits_ordered(ld[t]) << 32) | (uint32_t)(lb - id_offset);
                s_ent[t] = mine;
            }
            if (wave == 0) {                            // floor: the level-1 floors and the last
                float fl = INFINITY;                    // key of every full level-1 list
                if (lane < G) {
                    fl = a.l1_floor[q * G + lane];
                    if (li[16 * lane + 15] >= 0) fl = fminf(fl, ld[16 * lane + 15]);
                }
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
                if (lane == 0) s_floor = fl;
            }
        }
        const int nv = __syncthreads_count(mine != kEmpty);
        const int K = min(kc, nv);
        if (mine != kEmpty) {
            int r = 0;
            const ulonglong2* e2 = reinterpret_cast<const ulonglong2*>(s_ent);
#pragma unroll 4
            for (int j = 0; j < E / 2; ++j) {
                const ulonglong2 p = e2[j];
                r += (p.x < mine ? 1 : 0) + (p.y < mine ? 1 : 0);
            }
            if (r < K) {
                const float kv = key_from_ordered((uint32_t)(mine >> 32));
                const int64_t lb = (int64_t)(uint32_t)mine + id_offset;
                s_mkey[r] = kv; s_mlab[r] = lb;
                a.cd[q * kc + r] = kv; a.ci[q * kc + r] = lb;
            }
        }
        if (t >= K && t < kc) {
            s_mkey[t] = FLT_MAX; s_mlab[t] = -1;
            a.cd[q * kc + t] = FLT_MAX; a.ci[q * kc + t] = -1;
        }
        if (t == 0) a.floor[q] = s_floor;
        __syncthreads();
        RR_STAMP(3);
    }
    const int64_t lab = lane < kc ? (fused ? s_mlab[lane] : a.ci[q * kc + lane]) : (int64_t)-1;
    const float ak = lane < kc ? (fused ? s_mkey[lane] : a.cd[q * kc + lane]) : INFINITY;  // ascending
    const bool valid = lab >= 0;
    const int nvalid = __popcll(__ballot(valid));               // valid candidates come first
    const QueryBounds B(a, q);

    // A query whose K' candidates all sit inside the band this certificate needs (tau - E_a(tau)
    // at most a quarter bound above the k-th approximate key, tau = min(K'-th candidate, floor))
    // would pass only if its exact k-th key fell well below the approximate one — observed errors
    // are ~0.1 of the bound — so it goes to the second chance (a complete procedure of its own)
    // without the first rerank's row reads (RerankArgs::chance_skip; a wrong guess costs time only)
    if (a.chance_skip && a.raw_d && nvalid >= kc && k <= kc) {
        const float a_kk = __shfl(ak, k - 1, 64);
        float tau0 = __shfl(ak, kc - 1, 64);
        if (fused) tau0 = fminf(tau0, s_floor);
        else if (a.floor) tau0 = fminf(tau0, a.floor[q]);
        if (tau0 - B.bound_a(tau0) <= a_kk + 0.25f * B.bound_a(a_kk)) {
            if (threadIdx.x == 0) {
                atomicAdd(a.stats + 2, 1);
                a.chance_list[atomicAdd(a.stats + 3, 1)] = (int)q;
            }
            RR_STAMP(4);
            return;
        }
    }

    // Only a prefix of the (ascending) candidates can hold the answer; the prefix P = {approx <=
    // prefix_limit(a_k)} is reranked and the first candidate left out bounds every excluded
    // candidate's approximate key from below.
    int m = nvalid;
    if (nvalid >= k) {
        const float thr = B.prefix_limit(__shfl(ak, k - 1, 64));
        m = __popcll(__ballot(valid && ak <= thr));
    }

    auto row_of = [&](int c) {
        const int lo32 = __shfl((int)(lab & 0xffffffff), c, 64);
        const int hi32 = __shfl((int)(lab >> 32), c, 64);
        const int64_t l = ((int64_t)hi32 << 32) | (uint32_t)lo32;
        return reinterpret_cast<const float4*>(a.xb + (l - id_offset) * dp);
    };
    // the lane's own candidate's |x|^2, loaded up front (not after each round's dot products)
    const float xn_own = valid ? a.xn[lab - id_offset] : 0.f;
    // candidates [c_begin, c_end), NW * R rows in flight per round
    auto rerank_range = [&](int c_begin, int c_end, auto r_tag) {
        constexpr int R = decltype(r_tag)::value;
        for (int c0 = c_begin + wave; c0 < c_end; c0 += NW * R) {
            const float4* r4[R];
            float acc[R];
#pragma unroll
            for (int v = 0; v < R; ++v)
                r4[v] = row_of(min(c0 + NW * v, c_end - 1));   // clamped: loads unconditional
            rerank_dots<IT, R>(q4, qr, n4, lane, r4, acc);
#pragma unroll
            for (int v = 0; v < R; ++v) {
                const int c = c0 + NW * v;
                if (lane == c && c < c_end) skey[c] = rerank_key(acc[v], B.qn, xn_own, metric);
            }
        }
    };
    if (wave == 0) slab[lane] = lab;
    // Two phases: the first P1 candidates, then — with s1 = the k-th exact key among them (an
    // upper bound of the final k-th) — only the candidates c with a_c - E_a(a_c) <= s1 + E_f(s1)
    // (any other has exact key > s1 + E_f(s1): v - E_a(v) is increasing, and a truncated key is
    // below the approximate key it stands for).  The refined prefix replaces a_k's twice-bounded
    // limit; its first candidate left out passes the certificate by construction.
    // P1 = RerankArgs::p1 (k for large batches: the first k candidates usually ARE the answer
    // and their max exact key already cuts the rest, so the 16 - k extra rows a 16-row first
    // phase reads are bytes a throughput-bound batch pays for; small batches keep 16 — one round
    // of row loads — since a second phase is a dependent round trip there)
    constexpr int P1max = kRerankWaves * kRerankRows;   // (16: one round of loads at NW = 8)
    const int P1 = a.p1 > 0 ? min(a.p1, P1max) : P1max;
    const int m1 = min(m, P1);
    rerank_range(0, m1, std::integral_constant<int, kRerankRows>{});
    __syncthreads();
    if (m > m1) {
        if (m1 >= k) {                                  // (k > P1: the whole prefix, one phase)
            const float key1 = lane < m1 ? skey[lane] : INFINITY;
            int r1 = 0;
            for (int i = 0; i < m1; ++i)
                if (lane < m1 && ranks_before_r(skey[i], slab[i], key1, lab)) ++r1;
            const uint64_t hit = __ballot(lane < m1 && r1 == k - 1);
            const float s1 = __shfl(key1, hit ? (int)__builtin_ctzll(hit) : 0, 64);
            const float lim = s1 + B.bound_f(s1);
            const int m2 = __popcll(__ballot(valid && lane < m && ak - B.bound_a(ak) <= lim));
            m = max(m1, m2);
        }
        // (4 rows per wave in flight here measured no faster at one query: 23.4 vs 22.4 us)
        rerank_range(m1, m, std::integral_constant<int, kRerankRows>{});
        __syncthreads();
    }
    if (wave != 0) return;
    const float key = lane < m ? skey[lane] : INFINITY;

    // rank of this lane's candidate inside the prefix by (key, label)
    const bool inP = lane < m;
    int rank = 0;
    for (int i = 0; i < m; ++i)
        if (inP && ranks_before_r(skey[i], slab[i], key, lab)) ++rank;
    if (inP && rank < k) {
        a.D[q * k + rank] = (metric == 1) ? key : -key;
        a.I[q * k + rank] = lab;
    }
    if (lane >= m && lane < k) {
        a.D[q * k + lane] = (metric == 1) ? FLT_MAX : -FLT_MAX;
        a.I[q * k + lane] = -1;
    }

    // observed |approx - rerank| of every reranked candidate relative to the two bounds (<= 1
    // whenever the bounds hold; reported by knn_search_stats so tests and the bench watch it)
    {   // one same-address atomic per query, not one per reranked candidate
        float r = inP ? fabsf(ak - key) / (B.bound_a(ak) + B.bound_f(key) + B.trunc(ak)) : 0.f;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) r = fmaxf(r, __shfl_xor(r, off, 64));
        if (lane == 0 && m > 0) atomicMax(reinterpret_cast<unsigned*>(a.stats + 1), __float_as_uint(r));
    }

    // certificate: tau = smallest approximate key a row outside the prefix can have — the K'-th
    // candidate's (when the set is full), the merge floor (rows dropped by full lists) and the
    // first candidate left out of the prefix; +inf means every row was reranked
    const int lo_tau = __shfl((int)(lab & 0xffffffff), kc - 1, 64);
    const int hi_tau = __shfl((int)(lab >> 32), kc - 1, 64);
    const int64_t lab_tau = ((int64_t)hi_tau << 32) | (uint32_t)lo_tau;
    float tau = (lab_tau >= 0 && nvalid >= kc) ? __shfl(ak, kc - 1, 64) : INFINITY;
    if (fused) tau = fminf(tau, s_floor);
    else if (a.floor) tau = fminf(tau, a.floor[q]);
    const float a_out = __shfl(ak, min(m, 63), 64);
    if (m < nvalid) tau = fminf(tau, a_out);
    bool failed = false;                            // tau = +inf: every row was reranked
    if (tau != INFINITY) {
        float sk = (inP && rank == k - 1) ? key : -INFINITY;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sk = fmaxf(sk, __shfl_xor(sk, off, 64));
        // fewer than k reranked rows while rows were left out: nothing to certify with
        failed = !(m >= k && (tau - B.bound_a(tau)) > (sk + B.bound_f(sk)));
    }
    if (failed && lane == 0) {
        atomicAdd(a.stats + 2, 1);
        if (a.raw_d) a.chance_list[atomicAdd(a.stats + 3, 1)] = (int)q;
        else a.fail_list[atomicAdd(a.stats, 1)] = (int)q;
    }
}

__global__ void __launch_bounds__(256)
gather_rows_kernel(const float* __restrict__ src, const float* __restrict__ src_norm, int dp,
                   const int* __restrict__ list, int64_t n, int64_t n_pad,
                   float* __restrict__ dst, float* __restrict__ dst_norm) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n_pad) return;
    float* o = dst + row * dp;
    if (row >= n) {
        for (int j = lane; j < dp; j += 64) o[j] = 0.f;
        if (lane == 0) dst_norm[row] = 0.f;
        return;
    }
    const float* s = src + (int64_t)list[row] * dp;
    for (int j = lane; j < dp; j += 64) o[j] = s[j];
    if (lane == 0) dst_norm[row] = src_norm[list[row]];
}

__global__ void __launch_bounds__(256)
scatter_results_kernel(const float* __restrict__ sd, const int64_t* __restrict__ si,
                       const int* __restrict__ list, int64_t n, int k, float* __restrict__ D,
                       int64_t* __restrict__ I) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * k) return;
    const int64_t r = t / k;
    const int j = (int)(t - r * k);
    D[(int64_t)list[r] * k + j] = sd[t];
    I[(int64_t)list[r] * k + j] = si[t];
}

__global__ void max_norm_kernel(const float* __restrict__ xn, int64_t n, float* __restrict__ out) {
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, xn[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    // norms are >= 0: their IEEE bit patterns order like unsigned integers
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned*>(out), __float_as_uint(m));
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_split_rows(const float* src, int64_t n, int dp, int bk, uint32_t* dst,
                             hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if ((bk != 16 && bk != 32) || dp % bk != 0) return hipErrorInvalidValue;
    const int64_t threads = n * (dp / 8);
    hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                       src, n, dp, bk, dst);
    return hipGetLastError();
}

#ifdef IMGREC_TAIL_STAMPS
extern "C" int knn_rerank_stamps_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_rr_stamps), sizeof(imgrec::g_rr_stamps));
}
#endif

hipError_t launch_rerank_certify(const RerankArgs& a, hipStream_t st) {
    if (a.nq <= 0) return hipSuccess;
    if (a.kc > 64 || a.k > a.kc || a.k > 64 || a.dp % 4 != 0 || !a.stats || !a.fail_list)
        return hipErrorInvalidValue;
    if (a.l1_G > 0 && (16 * a.l1_G > kRerankWaves * 64 || !a.floor)) return hipErrorInvalidValue;
    if (a.l1_G > 0 && a.l0_lists == 0 && (!a.l1_d || !a.l1_i || !a.l1_floor)) return hipErrorInvalidValue;
    if (a.l0_lists > 0 && (a.l1_G != (a.l0_lists + 63) / 64 || a.l1_G > kRerankWaves ||
                           a.raw_km != 16 || !a.raw_d || !a.raw_i))
        return hipErrorInvalidValue;
    if (a.raw_d && (!a.raw_i || !a.chance_list || a.raw_km < a.k || a.raw_lists <= 0))
        return hipErrorInvalidValue;
    if (a.s_lists > 0 && (a.s_lists > 64 || a.raw_km > 16 || a.raw_lists != a.s_lists || !a.raw_d ||
                          !a.floor || !a.cd || !a.ci || a.l1_G > 0))
        return hipErrorInvalidValue;
    if (a.nw != 0 && (a.nw != 4 || a.s_lists > 0 || a.l1_G > 0 || a.chance_skip))
        return hipErrorInvalidValue;
    // (the single-level merge has its own instance: its registers stay out of the default one)
#define IMGREC_RERANK(ITV)                                                                          \
    do {                                                                                            \
        if (a.nw == 4)                                                                              \
            hipLaunchKernelGGL((rerank_certify_kernel<ITV, false, 4>), dim3((unsigned)a.nq),         \
                               dim3(4 * 64), 0, st, a);                                             \
        else if (a.s_lists > 0)                                                                     \
            hipLaunchKernelGGL((rerank_certify_kernel<ITV, true, kRerankWaves>), dim3((unsigned)a.nq), \
                               dim3(kRerankWaves * 64), 0, st, a);                                  \
        else                                                                                        \
            hipLaunchKernelGGL((rerank_certify_kernel<ITV, false, kRerankWaves>), dim3((unsigned)a.nq), \
                               dim3(kRerankWaves * 64), 0, st, a);                                  \
    } while (0)
    if (a.dp <= 512) IMGREC_RERANK(2);
    else if (a.dp <= 1024) IMGREC_RERANK(4);
    else if (a.dp <= 2048) IMGREC_RERANK(8);
    else IMGREC_RERANK(0);
#undef IMGREC_RERANK
    return hipGetLastError();
}

hipError_t launch_gather_rows(const float* src, const float* src_norm, int dp, const int* list,
                              int64_t n, int64_t n_pad, float* dst, float* dst_norm, hipStream_t st) {
    if (n_pad <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n_pad + 3) / 4)), dim3(256), 0, st, src,
                       src_norm, dp, list, n, n_pad, dst, dst_norm);
    return hipGetLastError();
}

hipError_t launch_scatter_results(const float* sd, const int64_t* si, const int* list, int64_t n,
                                  int k, float* D, int64_t* I, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_results_kernel, dim3((unsigned)((n * k + 255) / 256)), dim3(256), 0,
                       st, sd, si, list, n, k, D, I);
    return hipGetLastError();
}

hipError_t launch_bf16_rows(const float* src, int64_t n, int dp, int dpb, uint16_t* dst,
                            float* resid, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (dpb % 8 != 0 || dp % 8 != 0 || dpb < dp) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bf16_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, src, n, dp,
                       dpb, dst, resid);
    return hipGetLastError();
}

hipError_t launch_query_prep_b16(const float* src, int64_t n, int d, int dp, int dpb, int64_t n_pad,
                                 int normalize, float* dst, float* norms, uint16_t* qb, float* resid,
                                 hipStream_t st) {
    if (n_pad <= 0) return hipSuccess;
    if (dpb % 8 != 0 || dp % 16 != 0 || dpb < dp || dp < d) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n_pad + 3) / 4)), block(256);
#define IMGREC_QPREP(ITV) hipLaunchKernelGGL((query_prep_b16_kernel<ITV>), grid, block, 0, st, src, n, \
                                             d, dp, dpb, n_pad, normalize, dst, norms, qb, resid)
    if (dpb <= 512) IMGREC_QPREP(1);
    else if (dpb <= 1024) IMGREC_QPREP(2);
    else if (dpb <= 2048) IMGREC_QPREP(4);
    else if (dpb <= 4096) IMGREC_QPREP(8);
    else return hipErrorInvalidValue;
#undef IMGREC_QPREP
    return hipGetLastError();
}

hipError_t launch_max_norm(const float* xn, int64_t n, float* out, hipStream_t st) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float), st);
    if (e != hipSuccess || n <= 0) return e;
    const int64_t blocks = std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(max_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, st, xn, n, out);
    return hipGetLastError();
}

}  // namespace imgrec
