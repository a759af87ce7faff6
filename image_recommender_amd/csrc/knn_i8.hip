// knn_i8.hip — the small-batch candidate pass on a block-scaled int8 copy of the corpus (gfx950).
//
// A search of a few queries (the reference CLI's regime: main/search_from_image.py:247
// searches ONE query vector per call) is HBM-bound: the bf16 candidate pass streams 2 bytes per
// element (3.97 GB at 1M x 1968; 0.646 ms at 6.1 TB/s, profiles/r03/nq1_final.jsonl).  This pass
// streams 1 byte per element plus one fp32 scale per 64 (2.17 GB) and keeps the same contract as
// the bf16 pass: per (query, row split) the KM best APPROXIMATE keys, which the candidate merge,
// the fp32 rerank and the certificate (knn_refine.hip, knn_certify.h kModeI8) turn into the exact
// answer.  The approximation is certified, not trusted:
//
//   x~ = s_b * c   per 64-element block b, s_b = max|x_b| / 127, c = rint(x / s_b) in [-127, 127]
//   q~ = s_hi c_hi + s_lo c_lo   two levels of the same per query block (|q - q~| ~ 2^-14 |q|)
//   |q.x - q~.x~| <= |q| |x - x~| + |q - q~| |x~|     (R = max stored residual norm of the rows)
//
// On the bench rows (1M x 1968, unit-norm parts) R = 0.016 against the bf16 copy's 0.0036; the
// rows within the certificate's band of the 10th approximate key number 21-53 per query (numpy
// over the whole 1M corpus, tools/i8_band_check.py), below the rerank's 64 candidates.
//
// Scan: one workgroup per row split (8-row groups s, s + nsplit, ... as the bf16 kernels, so a
// store with similar images on adjacent rows spreads them over every split), four waves; a wave
// takes one 8-row group at a time, a 16-lane group per row, lane j the 64-element blocks j,
// j + 16, ... of its row (rows stored without padding: knn_kernels.h i8_slot): 16-B code loads
// (two register sets: the next group's loads in flight),
// the query's codes from LDS, exact int32 v_dot4_i32_i8 products of the row's codes with the
// query's hi and lo codes (no int8 -> fp32 conversions: 0.56 VALU instructions per element and
// query, against 2 for an fp32 FMA form that converts every code), one fp32 fold per block
// (acc += s_x (s_hi D_hi + s_lo D_lo)), a DPP row-rotate sum over the 16 lanes.  Lane j (< NQ)
// of each row group keeps query j's list; at the end the 16 lists of a split are merged in LDS
// to one list of KM.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "knn_kernels.h"
#include "wave_ops.h"

namespace imgrec {
namespace {

constexpr int kBlk = 64;       // elements per scale block
constexpr int kWaves = 4;
constexpr int kGroup = 8;      // rows per split group (the bf16 kernels' DMA piece)
#ifndef IMGREC_I8_NT
#define IMGREC_I8_NT 1
#endif
constexpr bool kNtCodes = IMGREC_I8_NT != 0;   // non-temporal code loads in the scan


#ifdef IMGREC_I8_STAMPS
// diagnostic build only (tools/i8_stamps.py): s_memrealtime (100 MHz, one clock for the chip) per
// scan workgroup (< 1024): 0 entry, 1 query side in LDS, 2 first group processed (wave 0),
// 3-6 waves 0-3 leave the row loop, 7 lists written
__device__ unsigned long long g_i8_stamps[1024 * 8];
#define I8_STAMP(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) \
    g_i8_stamps[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define I8_STAMP(slot) do {} while (0)
#endif

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// sum over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1): every lane gets the row's total
__device__ __forceinline__ float row16_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
    return v;
}

// Build: one wave per row, lane b quantises block b (nblk <= 64) into its slots of the compact
// row (i8_slot).  The residual norm is computed against the dequantised value the scan uses
// (s * c) and inflated for its own fp32 evaluation.
__global__ void __launch_bounds__(256)
i8_rows_kernel(const float* __restrict__ xb, int64_t n, int dp, int nblk, int8_t* __restrict__ codes,
               float* __restrict__ scales, float* __restrict__ resid) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= n) return;
    const float* x = xb + row * dp;
    float rsq = 0.f, xsq = 0.f;
    if (lane < nblk) {
        float v[kBlk];
        float mx = 0.f;
#pragma unroll
        for (int e = 0; e < kBlk; ++e) {
            const int i = lane * kBlk + e;
            v[e] = i < dp ? x[i] : 0.f;
            mx = fmaxf(mx, fabsf(v[e]));
        }
        const float s = mx / 127.f;
        const float inv = mx > 0.f ? 127.f / mx : 0.f;
        uint32_t w[kBlk / 4];
#pragma unroll
        for (int e4 = 0; e4 < kBlk / 4; ++e4) {
            uint32_t word = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float ve = v[4 * e4 + t];
                const int c = max(-127, min(127, (int)rintf(ve * inv)));
                const float r = ve - (float)c * s;
                rsq = fmaf(r, r, rsq);
                xsq = fmaf(ve, ve, xsq);
                word |= ((uint32_t)c & 0xffu) << (8 * t);
            }
            w[e4] = word;
        }
        // chunk c of block b at 16-B slot i8_slot(nblk, b, c) of the row (knn_kernels.h)
        uint4* dst = reinterpret_cast<uint4*>(codes + row * (int64_t)i8_row_bytes(nblk));
#pragma unroll
        for (int c = 0; c < 4; ++c)
            dst[i8_slot(nblk, lane, c)] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
        scales[row * nblk + lane] = s;
    }
    rsq = wave_sum(rsq);
    xsq = wave_sum(xsq);
    // |fl(c s) - c s| <= 2^-24 |c s| per element: 2^-22 |x| covers the evaluation of every term
    if (lane == 0) resid[row] = sqrtf(rsq) * (1.f + 1.f / 65536.f) + sqrtf(xsq) * (1.f / 4194304.f);
}

// Two-level int8 codes of one 64-element query block, q~ = s_hi c_hi + s_lo c_lo (c_hi =
// rint(v / s_hi), s_hi = max|v| / 127; c_lo the same of v - s_hi c_hi), on 4 lanes: lanes
// 4g .. 4g + 3 hold one block, quarter q4 = elements 16 q4 .. 16 q4 + 15.  The block maxima meet
// over the four lanes by shuffles (exact in any order).  emit(lev, e4, word) gets the codes of the
// block's elements 4 e4 .. 4 e4 + 3 of level lev (0 = hi) as they are made; sc = (s_hi, s_lo); v
// ends as the residual v - q~; this lane's partial sums xsq += |v|^2, rsq += |v - q~|^2.  The
// one quantiser of i8_query_prep_kernel and the scan's fused prep (bit-identical by construction:
// both walk the blocks 16 per pass).  Round 4-5 ran a block on one lane: a 64-element dependent
// chain, ~3 us of the prep before the scan streams anything.  All four lanes of a group must be
// active.
template <class Emit>
__device__ __forceinline__ void quantize_query_quarter(float (&v)[16], int q4, Emit&& emit,
                                                       float (&sc)[2], float& xsq, float& rsq) {
    float mx = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        mx = fmaxf(mx, fabsf(v[t]));
        xsq = fmaf(v[t], v[t], xsq);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
#pragma unroll
    for (int lev = 0; lev < 2; ++lev) {
        const float sl = mx / 127.f, inv = mx > 0.f ? 127.f / mx : 0.f;
        float mx2 = 0.f;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
            uint32_t word = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int c = max(-127, min(127, (int)rintf(v[4 * e4 + t] * inv)));
                v[4 * e4 + t] -= (float)c * sl;              // the residual, next level's input
                mx2 = fmaxf(mx2, fabsf(v[4 * e4 + t]));
                word |= ((uint32_t)c & 0xffu) << (8 * t);
            }
            emit(lev, 4 * q4 + e4, word);
        }
        sc[lev] = sl;
        mx2 = fmaxf(mx2, __shfl_xor(mx2, 1, 64));
        mx = fmaxf(mx2, __shfl_xor(mx2, 2, 64));
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) rsq = fmaf(v[t], v[t], rsq);
}

// |q - q~| bound from the block sums (inflated for its own fp32 evaluation as the rows' is)
__device__ __forceinline__ float query_resid(float rsq, float xsq) {
    return sqrtf(rsq) * (1.f + 1.f / 65536.f) + sqrtf(xsq) * (1.f / 4194304.f);
}

// The int8 path's whole query side in one pass (one wave per query row): raw row (d floats) ->
// padded fp32 row (dp, zero tail; L2-normalised when `normalize`) and |q|^2 — the same lane
// chunks, order and reductions as query_prep_b16_kernel (knn_refine.hip), so the rows and norms
// are bit-identical to the bf16 path's — then, from a copy of the row in LDS, the two-level int8
// codes per 64-element block, q~ = s_hi c_hi + s_lo c_lo (c_hi = rint(q / s_hi), s_hi =
// max|q_b| / 127; c_lo the same of q - s_hi c_hi), so the scan's products are exact int32 dot4s
// and the query's own rounding |q - q~| (about 2^-14 |q|, inflated for its own fp32 evaluation as
// the rows' is) is the certificate's dq term (q_resid).  Lane b = block b (nblk <= 64); out:
// codes[q][b] = 64 hi | 64 lo, scales[q][b] = (s_hi, s_lo), resid[q].  Rows n .. n_pad-1
// (the exact re-run tile's padding) get zero rows and norms, no codes.  dp <= 512 IT.
template <int IT>
__global__ void __launch_bounds__(64)
i8_query_prep_kernel(const float* __restrict__ src, int64_t n, int d, int dp, int normalize,
                     int nblk, float* __restrict__ dst, float* __restrict__ norms,
                     int8_t* __restrict__ codes, float* __restrict__ scales,
                     float* __restrict__ resid) {
    constexpr int kPitch = kBlk + 1;                     // block b at b * 65: lane b's reads
    __shared__ float srow[64 * kPitch];                  // walk distinct banks
    const int64_t row = blockIdx.x;
    const int lane = threadIdx.x;
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
    float nacc = 0.f;
    float* o = dst + row * dp;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int c = lane + 64 * it;
        if (8 * c >= dp) continue;                       // dp is a multiple of 16
        float v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            v[t] = normalize ? e[it][t] * scale : e[it][t];
            nacc = fmaf(v[t], v[t], nacc);
            const int i = 8 * c + t;
            srow[(i >> 6) * kPitch + (i & 63)] = v[t];
        }
        *reinterpret_cast<float4*>(o + 8 * c) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 8 * c + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nacc += __shfl_xor(nacc, off, 64);
    if (lane == 0) norms[row] = nacc;
    if (!real) return;                                   // (whole wave)
    for (int i = dp + lane; i < nblk * kBlk; i += 64) srow[(i >> 6) * kPitch + (i & 63)] = 0.f;
    __syncthreads();
    float rsq = 0.f, xsq = 0.f;
    // four lanes per block, 16 blocks per pass (quantize_query_quarter; the scan's fused prep
    // walks the blocks the same way, so the sums meet in the same order)
    for (int b0 = 0; b0 < nblk; b0 += 16) {
        const int b = b0 + (lane >> 2), q4 = lane & 3;
        if (b < nblk) {
            uint32_t w[2][4];
            float sc[2];
            float v[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) v[t] = srow[b * kPitch + 16 * q4 + t];
            quantize_query_quarter(v, q4, [&](int lev, int e4, uint32_t word) { w[lev][e4 & 3] = word; },
                                   sc, xsq, rsq);
            uint4* out = reinterpret_cast<uint4*>(codes + (row * nblk + b) * 2 * kBlk);
            out[q4] = make_uint4(w[0][0], w[0][1], w[0][2], w[0][3]);       // words 4 q4 .. + 3
            out[4 + q4] = make_uint4(w[1][0], w[1][1], w[1][2], w[1][3]);
            if (q4 == 0) {
                scales[(row * nblk + b) * 2] = sc[0];
                scales[(row * nblk + b) * 2 + 1] = sc[1];
            }
        }
    }
    rsq = wave_sum(rsq);
    xsq = wave_sum(xsq);
    if (lane == 0) resid[row] = query_resid(rsq, xsq);
}

// Ascending list, labels arriving in increasing order: slot p's key is the median of (kd[p-1], d,
// kd[p]) (ties keep the earlier, smaller label); d = +inf is a no-op.
template <int K>
__device__ __forceinline__ void insert_mono(float (&kd)[K], int (&ki)[K], float d, int id) {
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

template <int NQ, int KM, int NBI, bool DYN>
__global__ void __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(2)))
knn_i8_scan_kernel(const int8_t* __restrict__ codes, const float* __restrict__ scales,
                   const float* __restrict__ xnorm, int nrows, int nblk,
                   const int8_t* __restrict__ qcodes, const float* __restrict__ qscales,
                   const float* __restrict__ qnorm, int nq,
                   int nsplit, int64_t id_offset, int l2, float* __restrict__ cand_d,
                   int64_t* __restrict__ cand_i, int ncand, const float* __restrict__ qsrc, int d,
                   int dp, int normalize, float* __restrict__ qpad, float* __restrict__ qnorm_out,
                   float* __restrict__ qresid, int* __restrict__ zero_ctl,
                   float* __restrict__ heads, int raw16, int half_k, int* __restrict__ dyn,
                   int pool, int pool_ch) {
    // the queries' two-level codes in LDS: block b of query q at sqc[q][b] = 64 hi codes | 64 lo
    // codes | 16-B pad — the pad puts lane j's block (b = j + 16 bi) on 16-B bank slot j, so a
    // ds_read_b128 lane group (16 distinct j) is conflict-free; their scales (s_hi, s_lo) in sqs
    // (the final fold's lists reuse the codes' LDS: 39 KB instead of 55 KB per workgroup at NQ = 8
    // keeps three workgroups on a CU)
    constexpr int kQB = 2 * kBlk + 16;
    union Lds {
        int8_t qc[NQ][16 * NBI][kQB];
        struct { float d[NQ][16][KM]; int i[NQ][16][KM]; } f;
    };
    __shared__ __attribute__((aligned(16))) Lds lds;
    auto& sqc = lds.qc;
    auto& fd = lds.f.d;
    auto& fi = lds.f.i;
    __shared__ float sqs[NQ][16 * NBI][2];

    const int split = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = lane & 15, g = lane >> 4;
    const int64_t rowb = i8_row_bytes(nblk);
    if (wave == 0) I8_STAMP(0);
    // the certificate tail's claim counters, when no rerank launch runs between (I8Args::zero_ctl)
    if (zero_ctl && split == 0 && tid < 4) zero_ctl[tid] = 0;
    float qn[NQ];
    float kd[KM];
    int ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }
    const bool owner = j < NQ && j < nq;

    const int ngroups = (nrows + kGroup - 1) / kGroup;
    // pool > 0 (I8Args::pool): the last `pool` groups are not assigned up front; a wave that has
    // run out of its own groups takes chunks of pool_ch of them from the counter dyn[0], so the
    // workgroups end together instead of the slowest 15-25 us behind the median
    const int sg = DYN ? ngroups - pool : ngroups;               // statically assigned groups
    // H rows per lane and step: a wave step covers 4 H rows (H = 2: a whole 8-row group; H = 1 at
    // NQ = 8, at NQ = 4 with KM = 32 and at d > 2048: half a group, which keeps the queries'
    // dots, the lists and the prefetched codes within the register file — a spill's reload waits
    // for every outstanding load, the prefetch too)
    constexpr int H = (NQ * KM > 64 || NBI > 2) ? 1 : 2;
    constexpr int kSub = 2 / H;                                  // wave steps per 8-row group
    // Groups round-robin over the splits (group m to split m % nsplit).  half_k = K > 0 (two
    // workgroups per CU): in every K-th round a second-half split's group goes to its first-half
    // partner (split - nsplit / 2) — the workgroup dispatched second onto a CU loses issue to the
    // first and ended ~10 us later (profiles/r05/i8_stamps/, loop_end_by_half)
    const int h2 = nsplit / 2;
    const bool first_half = split < h2;
    const int rs = split < sg ? (sg - split + nsplit - 1) / nsplit : 0;    // own rounds
    int ng = rs;
    if (half_k > 0) {
        if (first_half) {
            const int rp = split + h2 < sg ? (sg - split - h2 + nsplit - 1) / nsplit : 0;
            ng = rs + rp / half_k;
        } else {
            ng = rs - rs / half_k;
        }
    }
    const int cnt = kSub * ng;
    // this split's n-th group
    auto group_of = [&](int n) __attribute__((always_inline)) -> int {
        if (half_k <= 0) return split + n * nsplit;
        if (first_half) {
            const int b = n / (half_k + 1), o = n - b * (half_k + 1);
            return split + (o == half_k ? h2 : 0) + (b * half_k + min(o, half_k - 1)) * nsplit;
        }
        const int b = n / (half_k - 1), o = n - b * (half_k - 1);
        return split + (b * half_k + o) * nsplit;
    };
    // One 8-row group per wave step; two register sets, so the next group's loads are in flight
    // while this one's products run (a single set left each wave idle for a whole HBM round trip
    // per group: 4.7 TB/s with three waves per SIMD).
    struct Grp {
        uint4 cw[H][NBI][4];     // H rows x NBI blocks x 64 codes
        float sc[H][NBI];
        float xn[H];
        int row[H];
    };
    // sub-step sub of 8-row group m
    auto load = [&](int m, int sub, Grp& G) __attribute__((always_inline)) {
        const int r0 = m * kGroup + 4 * sub;
#pragma unroll
        for (int h = 0; h < H; ++h) {
            G.row[h] = r0 + 4 * h + g;
            const int rc = min(G.row[h], nrows - 1);
#pragma unroll
            for (int bi = 0; bi < NBI; ++bi) {
                const int b = j + 16 * bi;
                // chunk c of block b: slot 64 bi + m c + j (i8_slot, m = blocks of this group), so
                // the m live lanes of a row read 16 m contiguous bytes per load; lanes past nblk
                // load nothing (zero codes, zero scale)
                const int m = min(16, nblk - 16 * bi);
                const uint4* src = reinterpret_cast<const uint4*>(codes + (int64_t)rc * rowb) + 64 * bi + j;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    G.cw[h][bi][c] = make_uint4(0u, 0u, 0u, 0u);
                    if (b < nblk) {
                        if constexpr (kNtCodes) {    // streamed once per search: non-temporal loads
                            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                            const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + m * c));
                            G.cw[h][bi][c] = make_uint4(w.x, w.y, w.z, w.w);
                        } else {
                            G.cw[h][bi][c] = src[m * c];
                        }
                    }
                }
                G.sc[h][bi] = b < nblk ? scales[(int64_t)rc * nblk + b] : 0.f;
            }
            G.xn[h] = l2 ? xnorm[rc] : 0.f;
        }
    };
    auto process = [&](Grp& G) __attribute__((always_inline)) {
        float acc[H][NQ];
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[h][q] = 0.f;
#pragma unroll
        for (int bi = 0; bi < NBI; ++bi) {
            const int b = j + 16 * bi;
            // exact int32 dots of the row's 64 codes with the query block's hi and lo codes
            // (|sum| <= 64 * 127^2 < 2^24: exact in fp32 too), folded once per block:
            // acc += s_x (s_hi D_hi + s_lo D_lo); queries four at a time (NQ = 8: the dots of
            // four queries live at once, not eight)
            constexpr int QN = NQ < 4 ? NQ : 4;
#pragma unroll
            for (int q0 = 0; q0 < NQ; q0 += QN) {
                int dh[H][QN], dl[H][QN];
#pragma unroll
                for (int h = 0; h < H; ++h)
#pragma unroll
                    for (int t = 0; t < QN; ++t) dh[h][t] = dl[h][t] = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    // chunk by chunk: the laundered offset keeps this chunk's query reads below
                    // the previous chunk's (pinned) dots, so one chunk's query codes are live at
                    // a time
                    int qoff = 16 * c;
                    asm volatile("" : "+v"(qoff));
#pragma unroll
                    for (int t = 0; t < QN; ++t) {
                        const uint4 hi = *reinterpret_cast<const uint4*>(&sqc[q0 + t][b][qoff]);
                        const uint4 lo = *reinterpret_cast<const uint4*>(&sqc[q0 + t][b][kBlk + qoff]);
#pragma unroll
                        for (int h = 0; h < H; ++h) {
                            const uint4 w = G.cw[h][bi][c];
                            dh[h][t] = __builtin_amdgcn_sdot4((int)w.x, (int)hi.x, dh[h][t], false);
                            dh[h][t] = __builtin_amdgcn_sdot4((int)w.y, (int)hi.y, dh[h][t], false);
                            dh[h][t] = __builtin_amdgcn_sdot4((int)w.z, (int)hi.z, dh[h][t], false);
                            dh[h][t] = __builtin_amdgcn_sdot4((int)w.w, (int)hi.w, dh[h][t], false);
                            dl[h][t] = __builtin_amdgcn_sdot4((int)w.x, (int)lo.x, dl[h][t], false);
                            dl[h][t] = __builtin_amdgcn_sdot4((int)w.y, (int)lo.y, dl[h][t], false);
                            dl[h][t] = __builtin_amdgcn_sdot4((int)w.z, (int)lo.z, dl[h][t], false);
                            dl[h][t] = __builtin_amdgcn_sdot4((int)w.w, (int)lo.w, dl[h][t], false);
                        }
                    }
#pragma unroll
                    for (int h = 0; h < H; ++h)
#pragma unroll
                        for (int t = 0; t < QN; ++t) asm volatile("" : "+v"(dh[h][t]), "+v"(dl[h][t]));
                }
#pragma unroll
                for (int t = 0; t < QN; ++t) {
                    const float sh = sqs[q0 + t][b][0], sl = sqs[q0 + t][b][1];
#pragma unroll
                    for (int h = 0; h < H; ++h)
                        acc[h][q0 + t] = fmaf(G.sc[h][bi], fmaf(sl, (float)dl[h][t], sh * (float)dh[h][t]),
                                              acc[h][q0 + t]);
                }
            }
        }
        // keys; lane j (< NQ) of the row's group inserts query j's key (rows increase per lane)
#pragma unroll
        for (int h = 0; h < H; ++h) {
            float kv = INFINITY;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const float dot = row16_sum(acc[h][q]);
                float key = l2 ? fmaxf(fmaf(-2.f, dot, qn[q] + G.xn[h]), 0.f) : -dot;
                kv = j == q ? key : kv;
            }
            kv = (owner && G.row[h] < nrows && kv < kd[KM - 1]) ? kv : INFINITY;
            if (__any(kv != INFINITY)) insert_mono<KM>(kd, ki, kv, G.row[h]);
        }
    };
    Grp A, B;
    int li = wave;
    __shared__ float s_qn[NQ];
    // (the 8-query instance keeps the separate prep: the fused section's registers cost its
    // VALU-bound main loop ~25 %, profiles/r05/modes_nq/)
    if (NQ <= 4 && qsrc) {
        // Fused query prep (I8Args::qsrc): wave w derives queries w, w + 4 from the raw rows with
        // i8_query_prep_kernel's arithmetic — the same lane chunks and reductions for the row, its
        // norm and scale, the same quantiser per block — straight into this workgroup's LDS;
        // workgroup 0 also writes the padded fp32 rows, |q|^2 and |q - q~| for the rerank and
        // the tail.  (One launch and its dependent gap fewer per search; every workgroup repeats
        // ~1 us of quantising that overlaps the other waves' first code loads.)
        for (int i = tid; i < NQ * 16 * NBI * 8; i += kWaves * 64) {      // what no query fills
            const int qi = i / (16 * NBI * 8), r = i - qi * (16 * NBI * 8), b = r >> 3, c = r & 7;
            if (qi >= nq || b >= nblk) *reinterpret_cast<uint4*>(&sqc[qi][b][16 * c]) = make_uint4(0u, 0u, 0u, 0u);
        }
        for (int i = tid; i < NQ * 16 * NBI; i += kWaves * 64) {
            const int qi = i / (16 * NBI), b = i - qi * (16 * NBI);
            if (qi >= nq || b >= nblk) { sqs[qi][b][0] = 0.f; sqs[qi][b][1] = 0.f; }
        }
#pragma unroll 1
        for (int qi = wave; qi < NQ && qi < nq; qi += kWaves) {
            const float* s = qsrc + (int64_t)qi * d;
            // the row in i8_query_prep_kernel's chunks (lane c: elements 8c .. 8c + 7; chunks past
            // dp add exact zeros there, so they are skipped here)
            auto chunk = [&](int c, float (&e)[8]) __attribute__((always_inline)) {
                const int j0 = 8 * c;
                if ((d & 3) == 0 && j0 + 8 <= d) {
                    const float4 v0 = *reinterpret_cast<const float4*>(s + j0);
                    const float4 v1 = *reinterpret_cast<const float4*>(s + j0 + 4);
                    e[0] = v0.x; e[1] = v0.y; e[2] = v0.z; e[3] = v0.w;
                    e[4] = v1.x; e[5] = v1.y; e[6] = v1.z; e[7] = v1.w;
                } else {
#pragma unroll
                    for (int t = 0; t < 8; ++t) e[t] = j0 + t < d ? s[j0 + t] : 0.f;
                }
            };
            float scale = 1.f;
            if (normalize) {
                float acc = 0.f;
                for (int c = lane; 8 * c < dp; c += 64) {
                    float e[8];
                    chunk(c, e);
#pragma unroll
                    for (int t = 0; t < 8; ++t) acc = fmaf(e[t], e[t], acc);
                }
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
                if (acc > 0.f) scale = (float)(1.0 / (double)sqrtf(acc));
            }
            float nacc = 0.f;
            for (int c = lane; 8 * c < dp; c += 64) {
                float e[8];
                chunk(c, e);
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    e[t] = normalize ? e[t] * scale : e[t];
                    nacc = fmaf(e[t], e[t], nacc);
                }
                if (split == 0) {
                    float* o = qpad + (int64_t)qi * dp + 8 * c;
                    *reinterpret_cast<float4*>(o) = make_float4(e[0], e[1], e[2], e[3]);
                    *reinterpret_cast<float4*>(o + 4) = make_float4(e[4], e[5], e[6], e[7]);
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nacc += __shfl_xor(nacc, off, 64);
            float rsq = 0.f, xsq = 0.f;
            for (int b0 = 0; b0 < nblk; b0 += 16) {
                // four lanes per block (quantize_query_quarter): block b's quarter q4 from the raw
                // row (L1 / L2 after the chunk pass), scaled as the chunk pass scaled it (the same
                // product); elements past d are zero
                const int b = b0 + (lane >> 2), q4 = lane & 3;
                if (b >= nblk) continue;                 // (whole four-lane groups)
                const int i0 = b * kBlk + 16 * q4;
                float v[16];
                if ((d & 3) == 0 && i0 + 16 <= d) {
#pragma unroll
                    for (int t4 = 0; t4 < 4; ++t4) {
                        const float4 x4 = *reinterpret_cast<const float4*>(s + i0 + 4 * t4);
                        v[4 * t4] = x4.x; v[4 * t4 + 1] = x4.y; v[4 * t4 + 2] = x4.z; v[4 * t4 + 3] = x4.w;
                    }
                } else {
#pragma unroll
                    for (int t = 0; t < 16; ++t) v[t] = i0 + t < d ? s[i0 + t] : 0.f;
                }
                if (normalize) {
#pragma unroll
                    for (int t = 0; t < 16; ++t) v[t] = v[t] * scale;
                }
                float sc[2];
                uint32_t* qw = reinterpret_cast<uint32_t*>(&sqc[qi][b][0]);
                quantize_query_quarter(v, q4, [&](int lev, int e4, uint32_t word) { qw[lev * (kBlk / 4) + e4] = word; },
                                       sc, xsq, rsq);
                if (q4 == 0) {
                    sqs[qi][b][0] = sc[0];
                    sqs[qi][b][1] = sc[1];
                }
            }
            if (lane == 0) s_qn[qi] = nacc;
            if (split == 0) {
                rsq = wave_sum(rsq);
                xsq = wave_sum(xsq);
                if (lane == 0) { qnorm_out[qi] = nacc; qresid[qi] = query_resid(rsq, xsq); }
            }
        }
    } else {
        for (int i = tid; i < NQ * 16 * NBI * 8; i += kWaves * 64) {          // 16-B chunks
            const int qi = i / (16 * NBI * 8), r = i - qi * (16 * NBI * 8), b = r >> 3, c = r & 7;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (qi < nq && b < nblk) v = reinterpret_cast<const uint4*>(qcodes + ((int64_t)qi * nblk + b) * 2 * kBlk)[c];
            *reinterpret_cast<uint4*>(&sqc[qi][b][16 * c]) = v;
        }
        for (int i = tid; i < NQ * 16 * NBI; i += kWaves * 64) {
            const int qi = i / (16 * NBI), b = i - qi * (16 * NBI);
            const bool in = qi < nq && b < nblk;
            sqs[qi][b][0] = in ? qscales[((int64_t)qi * nblk + b) * 2] : 0.f;
            sqs[qi][b][1] = in ? qscales[((int64_t)qi * nblk + b) * 2 + 1] : 0.f;
        }
        if (tid < NQ) s_qn[tid] = tid < nq ? qnorm[tid] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q)      // (uniform: scalar registers, as the kernel-argument loads were)
        qn[q] = (l2 && q < nq) ? __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s_qn[q]))) : 0.f;

    // (the first group's loads issued before the query prep instead — by every wave, or only by
    // the waves that quantise no query — measured the same: profiles/r05/nq1/preload/)
    if (wave == 0) I8_STAMP(1);
    bool first_done = false;
    if constexpr (!DYN) {
    if (li < cnt) load(group_of(li / kSub), li % kSub, A);
    while (li < cnt) {
        if (li + kWaves < cnt) load(group_of((li + kWaves) / kSub), (li + kWaves) % kSub, B);
        process(A);
        if (wave == 0 && !first_done) { I8_STAMP(2); first_done = true; }
        li += kWaves;
        if (li >= cnt) break;
        if (li + kWaves < cnt) load(group_of((li + kWaves) / kSub), (li + kWaves) % kSub, A);
        process(B);
        li += kWaves;
    }
    } else {
    // The wave's steps in increasing row order (the lists' insert_mono needs it): its own
    // groups' steps li = wave, wave + 4, ..., then the pool's chunks in the order the counter
    // hands them out.  A chunk is 4 pool_ch groups for the whole workgroup (group c of the chunk
    // to wave c % 4): wave 0 takes it with one lane's atomic add — issued a chunk ahead, so its
    // latency hides under the products — and hands it over in LDS between two barriers (device
    // atomics run beyond the XCD's L2: one per wave and group cost more than the imbalance,
    // profiles/r06/i8_pool/).  The last workgroup to find the pool empty resets both counters
    // for the next launch (no host zeroing; safe to replay in a graph).
    __shared__ int s_chunk;
    const int chw = 4 * pool_ch;                                 // groups per chunk
    const int pool_chunks = pool > 0 ? (pool + chw - 1) / chw : 0;
    int pend = 0;                       // wave 0, lane 0: the grab in flight
    bool pend_on = false;
    int pc_base = 0, pc_t = 0, pc_n = 0;    // this wave's share of the current chunk
    auto grab = [&]() __attribute__((always_inline)) {
        if (lane == 0) pend = __hip_atomic_fetch_add(dyn, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend_on = true;
    };
    auto fetch = [&]() __attribute__((always_inline)) -> int {
        // (LDS only: the loads of the group in flight stay in flight)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (wave == 0) {
            if (!pend_on) grab();
            const int p = __builtin_amdgcn_readfirstlane(pend);
            pend_on = false;
            if (lane == 0) s_chunk = p;
            if (p < pool_chunks) {
                grab();
            } else if (lane == 0) {
                const int n = __hip_atomic_fetch_add(dyn + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (n == (int)gridDim.x - 1) {
                    __hip_atomic_store(dyn, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(dyn + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        return __builtin_amdgcn_readfirstlane(s_chunk);
    };
    auto next_step = [&]() __attribute__((always_inline)) -> int {
        if (li < cnt) {
            const int r = group_of(li / kSub) * kSub + li % kSub;
            li += kWaves;
            if (wave == 0 && pool_chunks > 0 && !pend_on && li + kWaves >= cnt) grab();
            return r;
        }
        if (pool_chunks == 0) return -1;
        for (;;) {
            if (pc_t < pc_n) {
                const int t = pc_t++;
                return (pc_base + kWaves * (t / kSub)) * kSub + t % kSub;
            }
            const int p = fetch();                   // every wave of the workgroup, together
            if (p >= pool_chunks) return -1;
            pc_base = sg + p * chw + wave;
            const int left = ngroups - pc_base;      // this wave's groups: pc_base + 4 i < ngroups
            pc_n = kSub * (left <= 0 ? 0 : min(pool_ch, (left + kWaves - 1) / kWaves));
            pc_t = 0;
        }
    };
    int cur = next_step();
    if (cur >= 0) load(cur / kSub, cur % kSub, A);
    while (cur >= 0) {
        const int nx = next_step();
        if (nx >= 0) load(nx / kSub, nx % kSub, B);
        process(A);
        if (wave == 0 && !first_done) { I8_STAMP(2); first_done = true; }
        if (nx < 0) break;
        cur = next_step();
        if (cur >= 0) load(cur / kSub, cur % kSub, A);
        process(B);
    }
    }

    I8_STAMP(3 + wave);
    // fold the split's 16 lists of each query (4 waves x 4 row groups) into one list of KM
    __syncthreads();                                     // (every wave is done with the codes)
    if (owner) {
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            fd[j][wave * 4 + g][p] = kd[p];
            fi[j][wave * 4 + g][p] = ki[p];
        }
    }
    __syncthreads();
    if constexpr (NQ <= 4) {
        if (raw16) {
            // the direct route (I8Args::raw16): the split's 16 sorted lane lists go out unfolded
            // (list l of the split = 16 split + l), and wave q writes the smallest of their first
            // keys as the split's head — the fold's ~5 us at the end of the last workgroup leave
            // the critical path; the second chance filters 16x the entries instead
            for (int i = tid; i < nq * 16 * KM; i += kWaves * 64) {
                const int qi = i / (16 * KM), r = i - qi * (16 * KM);
                const int ll = fi[qi][r / KM][r % KM];
                const size_t o = (size_t)qi * ncand + (size_t)split * 16 * KM + r;
                cand_d[o] = ll < 0 ? INFINITY : fd[qi][r / KM][r % KM];
                cand_i[o] = ll < 0 ? (int64_t)-1 : (int64_t)ll + id_offset;
            }
            if (heads && wave < nq) {
                float h = lane < 16 && fi[wave][lane][0] >= 0 ? fd[wave][lane][0] : INFINITY;
#pragma unroll
                for (int off = 8; off > 0; off >>= 1) h = fminf(h, __shfl_xor(h, off, 64));
                if (lane == 0) heads[(size_t)wave * nsplit + split] = h;
            }
            return;
        }
        // wave q selects query q's KM best of the 16 sorted lists at once (wave_select_sorted:
        // the lists' leading entries bound the answer, the survivors are ranked against each
        // other) — the round-by-round 16-lane minimum took ~5 us of dependent shuffles at the end
        // of every workgroup (profiles/r05/i8_stamps/)
        __shared__ uint64_t s_fold[NQ][(KM == 16 ? 64 : 128) + 192];
        const int fq = wave;
        if (fq >= NQ || fq >= nq) return;                // (whole waves)
        constexpr uint64_t kEmpty = ~0ull;
        uint64_t v[KM];
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            const float kk = lane < 16 ? fd[fq][lane][p] : INFINITY;
            const int ll = lane < 16 ? fi[fq][lane][p] : -1;
            v[p] = (ll < 0 || kk == INFINITY) ? kEmpty : ((uint64_t)key_bits_ordered(kk) << 32) | (uint32_t)ll;
        }
        uint64_t mine;
        int rank;
        const int K = wave_select_sorted<KM, (KM == 16 ? 1 : 2), 192>(v, KM, s_fold[fq], mine, rank);
        const size_t o = (size_t)fq * ncand + (size_t)split * KM;
        if (lane < K) {
            cand_d[o + rank] = key_from_ordered((uint32_t)(mine >> 32));
            cand_i[o + rank] = (int64_t)(uint32_t)mine + id_offset;
            if (heads && rank == 0) heads[(size_t)fq * nsplit + split] = key_from_ordered((uint32_t)(mine >> 32));
        } else if (lane < KM) {
            cand_d[o + lane] = INFINITY;
            cand_i[o + lane] = -1;
        }
        if (heads && K == 0 && lane == 0) heads[(size_t)fq * nsplit + split] = INFINITY;
#ifdef IMGREC_I8_STAMPS
        if (fq == 0 && lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            g_i8_stamps[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        return;
    }
    // wave w merges queries 4w .. 4w + 3, a 16-lane group per query, lane = list
    const int fq = wave * 4 + (lane >> 4), fl = lane & 15;
    if (fq >= NQ || fq >= nq) return;                    // (whole 16-lane groups leave together)
    int pos = 0;
    for (int p = 0; p < KM; ++p) {
        float hk = pos < KM ? fd[fq][fl][pos] : INFINITY;
        int hl = pos < KM ? fi[fq][fl][pos] : -1;
        if (hl < 0) hk = INFINITY;
        // min (key, label) over the group's 16 lanes; empty lists sort last
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
            const size_t o = (size_t)fq * ncand + (size_t)split * KM + p;
            cand_d[o] = bk;
            cand_i[o] = bk == INFINITY ? (int64_t)-1 : (int64_t)bl + id_offset;
            if (heads && p == 0) heads[(size_t)fq * nsplit + split] = bk;
        }
    }
#ifdef IMGREC_I8_STAMPS
    if (fq == 0 && fl == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        g_i8_stamps[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

}  // namespace

hipError_t launch_i8_rows(const float* xb, int64_t n, int dp, int nblk, int8_t* codes, float* scales,
                          float* resid, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (nblk <= 0 || nblk > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(i8_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, xb, n, dp,
                       nblk, codes, scales, resid);
    return hipGetLastError();
}

hipError_t launch_i8_query_prep(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                                int normalize, int nblk, float* dst, float* norms, int8_t* codes,
                                float* scales, float* resid, hipStream_t st) {
    if (n_pad <= 0) return hipSuccess;
    if (nblk <= 0 || nblk > 64 || dp % 16 != 0 || dp < d || dp > nblk * kBlk || n_pad < n)
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)n_pad), block(64);
#define IMGREC_I8QP(ITV) hipLaunchKernelGGL((i8_query_prep_kernel<ITV>), grid, block, 0, st, src, n, d, \
                                            dp, normalize, nblk, dst, norms, codes, scales, resid)
    if (dp <= 512) IMGREC_I8QP(1);
    else if (dp <= 1024) IMGREC_I8QP(2);
    else if (dp <= 2048) IMGREC_I8QP(4);
    else IMGREC_I8QP(8);
#undef IMGREC_I8QP
    return hipGetLastError();
}

hipError_t launch_i8_scan(const I8Args& a, hipStream_t st) {
    if (a.nblk <= 0 || a.nblk > 64 || a.nq < 1 || a.nsplit < 1) return hipErrorInvalidValue;
    if (a.qsrc && (a.dp % 16 != 0 || a.dp < a.d || a.d < 1 || a.dp > a.nblk * kBlk || !a.qpad ||
                   !a.qnorm_out || !a.qresid))
        return hipErrorInvalidValue;
    if (!a.qsrc && (!a.qcodes || !a.qscales || !a.qnorm)) return hipErrorInvalidValue;
    // the in-scan query prep serves at most 4 queries: the 5-8 query instance reads qcodes
    if (a.qsrc && a.nq > 4) return hipErrorInvalidValue;
    if (a.raw16 && (a.nq > 4 || a.ncand < a.nsplit * 16 * a.km)) return hipErrorInvalidValue;
    if (a.half_k != 0 && (a.half_k < 2 || a.nsplit % 2 != 0)) return hipErrorInvalidValue;
    if (a.pool < 0 || a.pool > (a.nrows + kGroup - 1) / kGroup || a.pool_ch < 1 ||
        (a.pool > 0 && (!a.dyn || a.half_k != 0)))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)a.nsplit), block(kWaves * 64);
    const int nbi = (a.nblk + 15) / 16;
    // the run-time pool is built for one or two queries with lists of 16 (the reference CLI's one
    // query per search); other instances keep the static split (their registers have no room)
    const bool dyn = a.pool > 0;
    if (dyn && (a.nq > 2 || a.km != 16)) return hipErrorInvalidValue;
#define IMGREC_I8(NQV, KMV, NBIV)                                                                 \
    if (dyn) IMGREC_I8D(NQV, KMV, NBIV, (NQV <= 2 && KMV == 16));                                    \
    else IMGREC_I8D(NQV, KMV, NBIV, false)
#define IMGREC_I8D(NQV, KMV, NBIV, DYNV)                                                          \
    hipLaunchKernelGGL((knn_i8_scan_kernel<NQV, KMV, NBIV, DYNV>), grid, block, 0, st, a.codes, a.scales, \
                       a.xnorm, a.nrows, a.nblk, a.qcodes, a.qscales, a.qnorm, a.nq, a.nsplit,      \
                       a.id_offset,                                                                 \
                       a.l2, a.cand_d, a.cand_i, a.ncand, a.qsrc, a.d, a.dp, a.normalize, a.qpad,  \
                       a.qnorm_out, a.qresid, a.zero_ctl, a.heads, a.raw16, a.half_k, a.dyn,     \
                       a.pool, a.pool_ch)
#define IMGREC_I8_NBI(NQV, KMV)                                   \
    do {                                                          \
        switch (nbi) {                                            \
            case 1: IMGREC_I8(NQV, KMV, 1); break;                \
            case 2: IMGREC_I8(NQV, KMV, 2); break;                \
            case 3: IMGREC_I8(NQV, KMV, 3); break;                \
            default: IMGREC_I8(NQV, KMV, 4); break;               \
        }                                                         \
    } while (0)
#define IMGREC_I8_KM(NQV)                                         \
    do {                                                          \
        if (a.km == 16) IMGREC_I8_NBI(NQV, 16);                   \
        else if (a.km == 32) IMGREC_I8_NBI(NQV, 32);              \
        else return hipErrorInvalidValue;                         \
    } while (0)
    if (a.nq == 1) IMGREC_I8_KM(1);
    else if (a.nq == 2) IMGREC_I8_KM(2);
    else if (a.nq <= 4) IMGREC_I8_KM(4);
    else if (a.nq <= 8) IMGREC_I8_KM(8);
    else return hipErrorInvalidValue;
#undef IMGREC_I8_KM
#undef IMGREC_I8_NBI
#undef IMGREC_I8
#undef IMGREC_I8D
    return hipGetLastError();
}

}  // namespace imgrec

#ifdef IMGREC_I8_STAMPS
extern "C" int knn_i8_stamps_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_i8_stamps), sizeof(imgrec::g_i8_stamps));
}
extern "C" int knn_i8_stamps_clear() {
    static unsigned long long zero[1024 * 8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(imgrec::g_i8_stamps), zero, sizeof(zero));
}
#endif
