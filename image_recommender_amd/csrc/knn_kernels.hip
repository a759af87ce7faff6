// knn_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the exact k-NN hot path.
//
// Replaces the arithmetic of faiss.IndexFlatL2.search / IndexFlatIP.search that the reference
// reaches from main/search_from_image.py:247 (and Analytics/rt_Search.py:63), and the add-time
// norm computation of IndexFlat.add reached from main/create_index.py:311.
//
// Kernels
//   rows_ingest       copy rows into the HBM layout (row stride dp = d rounded up to 16 floats,
//                     zero padded), optional L2 normalisation (faiss.normalize_L2 semantics,
//                     main/search_from_image.py:322), squared norm of every stored row.
//   knn_tile_topk     fused distance + top-k: an LDS-staged f32 MFMA contraction
//                     (v_mfma_f32_32x32x2_f32, exact fp32) of a BM-row corpus tile against a
//                     BQ-query tile over the full depth, then an epilogue that turns each
//                     accumulator into an L2 / IP key and filters it into a per-lane register
//                     top-K list.  The N x Q distance matrix never reaches HBM.
//   knn_merge         one wave per query: per-lane lists + a 64-lane butterfly argmin, k rounds.
//
// Accumulator layout (v_mfma_f32_32x32x2_f32, C/D map of cdna_hip_programming.md §3):
//   col = lane & 31 -> query,  row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5) -> corpus row.
// So every lane already holds 16 rows x 1 query per 32x32 block: the top-k filter needs no data
// movement.  The K index is permuted so each lane reads 8 contiguous floats per operand per
// 16-deep stage: MFMA sub-step s, lane half h uses depth k = 8h + s (same permutation on both
// operands, so the contraction is unchanged).

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <stdint.h>
#include <float.h>
#include <math.h>

#include "knn_certify.h"
#include "knn_kernels.h"
#include "wave_ops.h"

namespace imgrec {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 16-B fragment chunk c of a per-lane float array, reinterpreted as 8 bf16 (split layout)
template <int N>
__device__ __forceinline__ bf16x8 frag_bf16(const float (&v)[N], int c) {
    const f32x4 f = {v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
    return __builtin_bit_cast(bf16x8, f);
}

// ---------------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------------

// (d1, i1) ranks before (d2, i2): smaller key, exact ties by smaller label.
template <typename I>
__device__ __forceinline__ bool ranks_before(float d1, I i1, float d2, I i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

// Insert (d, id) into an ascending register list of length K (caller checked it beats kd[K-1]).
// Fully unrolled with compile-time indices so the list stays in VGPRs.
template <int K, typename I>
__device__ __forceinline__ void list_insert(float (&kd)[K], I (&ki)[K], float d, I id) {
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        const bool shift = ranks_before(d, id, kd[p - 1], ki[p - 1]);
        const bool here = !shift && ranks_before(d, id, kd[p], ki[p]);
        kd[p] = shift ? kd[p - 1] : (here ? d : kd[p]);
        ki[p] = shift ? ki[p - 1] : (here ? id : ki[p]);
    }
    const bool here0 = ranks_before(d, id, kd[0], ki[0]);
    kd[0] = here0 ? d : kd[0];
    ki[0] = here0 ? id : ki[0];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------------------------------------
// rows_ingest: one wave per destination row.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
rows_ingest_kernel(const float* __restrict__ src, int64_t n, int d, int dp, int64_t n_pad,
                   int normalize, float* __restrict__ dst, float* __restrict__ norms) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_pad) return;
    float* o = dst + row * (int64_t)dp;
    if (row >= n) {
        for (int j = lane; j < dp; j += 64) o[j] = 0.f;
        if (lane == 0) norms[row] = 0.f;
        return;
    }
    const float* s = src + row * (int64_t)d;
    float scale = 1.f;
    if (normalize) {
        float acc = 0.f;
        for (int j = lane; j < d; j += 64) acc = fmaf(s[j], s[j], acc);
        acc = wave_sum(acc);
        // faiss fvec_renorm_L2: nr = 1.0 / sqrtf(nr) (double reciprocal, stored as float)
        if (acc > 0.f) scale = (float)(1.0 / (double)sqrtf(acc));
    }
    float acc2 = 0.f;
    for (int j = lane; j < dp; j += 64) {
        const float v = (j < d) ? (normalize ? s[j] * scale : s[j]) : 0.f;
        o[j] = v;
        acc2 = fmaf(v, v, acc2);
    }
    acc2 = wave_sum(acc2);
    if (lane == 0) norms[row] = acc2;
}

// ---------------------------------------------------------------------------------------------
// knn_tile_topk
//
// Workgroup = WR x WQ waves; wave tile = 32*WB corpus rows (WB MFMA row blocks, 4 or 8) x 32
// queries, so the workgroup tile is BM = 32*WB*WR rows x BQ = 32*WQ queries.  A workgroup owns one query block and a
// contiguous range of row tiles (a "row split") and streams it as one continuous sequence of
// BK-deep K stages: (tile t0, stage 0..nsteps-1), (t0+1, 0..), ...
//
// Staging is LDS-DMA (global_load_lds_dwordx4): each wave instruction moves one 1-KiB piece
// (RPP rows x 4*BK bytes) straight into LDS, no staging VGPRs, into an NS-deep ring; a stage is
// read NS-1 iterations after its loads were issued, behind a counted `s_waitcnt vmcnt` and one raw
// s_barrier per stage (cdna_hip_programming.md §5 "Pipelining across barriers").  The ring runs
// across tile boundaries, so a tile's top-k epilogue overlaps the next tile's loads.
//
// LDS image: rows of BK floats; 16-B chunk c of row r stored at chunk c ^ ((r / RPB) % CPR)
// (RPB = rows per 256-B bank row, CPR = chunks per row).  The XOR is applied to the per-lane
// GLOBAL source address (the DMA destination is lane-linear); the fragment reads apply the same
// XOR, which makes every ds_read_b128 16-lane group hit 16 distinct 16-B bank slots.
// ---------------------------------------------------------------------------------------------
template <int WR, int WQ, int NS, int BK, int WB = 4>
struct TileGeom {
    static constexpr int NW = WR * WQ, NT = NW * 64;
    static constexpr int RW = 32 * WB;                 // corpus rows per wave
    static constexpr int BM = WR * RW, BQ = WQ * 32;
    static constexpr int CPR = BK / 4;                 // 16-B chunks per staged row
    static constexpr int RPP = 64 / CPR;               // rows per 1-KiB DMA piece
    static constexpr int RPB = 64 / BK;                // rows per 256-B bank row
    static constexpr int SA = BM * BK, SB = BQ * BK, STAGE = SA + SB;   // floats
    static constexpr int PA = BM / RPP, PB = BQ / RPP, PIECES = PA + PB;
    static constexpr int LPW = PIECES / NW;            // pieces per wave per stage
    // epilogue key parking in a spent stage: all 16 keys of a block in one round when they fit
    static constexpr int PR = (SA + SB) >= NW * 16 * 64 ? 16 : 8;
    static constexpr int PARK = NW * PR * 64;
    static constexpr int LDS_FLOATS = NS * STAGE + NS * BM;
    static_assert(BK == 16 || BK == 32, "stage depth");
    static_assert(PIECES % NW == 0, "pieces must divide evenly over waves");
    static_assert(BM % 64 == 0, "norm DMA uses whole waves");
    static_assert(STAGE >= PARK, "epilogue parking must fit in one stage");
    static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}

// LDS-DMA issued from inline asm (M0 = wave-uniform LDS destination, set and restored inside the
// statement).  hipcc does not see these as LDS writes, so it inserts no vmcnt(0) in front of the
// fragment ds_reads (it would for __builtin_amdgcn_global_load_lds, serialising the ring); every
// wait on them is the explicit counted wait_vmcnt below.
__device__ __forceinline__ void dma16(const float* g, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
// The same with the non-temporal policy, for bf16 corpus rows that exactly one workgroup reads (a
// launch with one query block): nq = 1 on 1M x 1968 0.695 -> 0.667 ms.  The fp32 corpus of the
// exact kernel runs slower with it (1.94 -> 2.70 ms), so it keeps the default policy.
__device__ __forceinline__ void dma16_nt(const float* g, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ void dma4(const float* g, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

// s_barrier that also orders the compiler's LDS accesses (the intrinsic alone is IntrNoMem).
__device__ __forceinline__ void barrier_raw() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Insert into an ascending list when labels reach this lane in increasing order (true inside
// the fused kernel: a lane visits its rows in increasing row order), so "ranks before" is a plain
// key comparison and an equal key always lands behind the existing entries.
template <int K>
__device__ __forceinline__ void list_insert_mono(float (&kd)[K], int (&ki)[K], float d, int id) {
    // c[p]: d goes before slot p of the old list (monotone); one compare, four selects per slot
    bool c[K];
#pragma unroll
    for (int p = 0; p < K; ++p) c[p] = d < kd[p];
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        // the same select on an ascending list is the median of (kd[p-1], d, kd[p]): one v_med3
        kd[p] = __builtin_amdgcn_fmed3f(kd[p - 1], d, kd[p]);
        ki[p] = c[p - 1] ? ki[p - 1] : (c[p] ? id : ki[p]);
    }
    kd[0] = c[0] ? d : kd[0];
    ki[0] = c[0] ? id : ki[0];
}

// 4-wave workgroups run two per CU (two waves per SIMD): hold them to 256 VGPR+AGPR per lane.
#define IMGREC_MIN_WAVES(nw) ((nw) == 4 ? 2 : 1)
// The work of one (query block, row split) item `wgid` (query block wgid % nqb, split
// wgid / nqb), in the LDS array smem (G::LDS_FLOATS floats).  The kernel below runs one item per
// workgroup; the certificate tail kernel loops over the items of a device-planned exact re-run.
template <int WR, int WQ, int KM, int NS, int BK, int MODE, int WB>
__device__ __forceinline__ void tile_topk_item(
        const float* __restrict__ xb, const float* __restrict__ xnorm, int nrows, int dp,
        const float* __restrict__ qp, const float* __restrict__ qnorm, int nq, int metric,
        int ntiles, int nsplit, int nqb, int64_t id_offset, float* __restrict__ cand_d,
        int64_t* __restrict__ cand_i, int ncand, int wgid, float* __restrict__ smem) {
    using G = TileGeom<WR, WQ, NS, BK, WB>;
    constexpr int RW = G::RW;
    constexpr int NW = G::NW, BM = G::BM, BQ = G::BQ, SA = G::SA, STAGE = G::STAGE;
    constexpr int PA = G::PA, LPW = G::LPW, CPR = G::CPR, RPP = G::RPP, RPB = G::RPB, PR = G::PR;
    constexpr int KH = BK / 2;          // MFMA sub-steps per stage (each covers depth 2)
    float* const norm_base = smem + NS * STAGE;
    const int qb = wgid % nqb;
    const int split = wgid / nqb;
    // this split's tiles, in increasing order: tile(j) for j in [0, t1).  Round-robin (split s
    // takes tiles s, s + nsplit, ...) spreads rows that are adjacent in storage — the reference
    // numbers images folder by folder — over many lists, so one list seldom holds a query's
    // whole neighbourhood (which would pull the certificate's floor down).
    const int t0 = 0;
    const int t1 = split < ntiles ? (ntiles - split + nsplit - 1) / nsplit : 0;
    auto tile = [&](int j) { return split + j * nsplit; };

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WQ;
    const int wq = wave % WQ;
    const int li = lane & 31;
    const int lh = lane >> 5;
    const int qcol = qb * BQ + wq * 32 + li;     // the query this lane owns (< nq_pad)
    const bool qvalid = qcol < nq;
    float qn = (metric == 1) ? qnorm[qcol] : 0.f;
    asm volatile("" : "+v"(qn));   // consume the load here, before the DMA stream starts

    // per-lane DMA source offsets inside a piece (row lane/CPR, logical chunk swizzled); the
    // swizzle of a piece's rows depends on the piece index modulo 64/(RPP*...) -> two variants.
    const int prow = lane / CPR, pchk = lane % CPR;
    const int goff0 = prow * dp + 4 * (pchk ^ (((0 * RPP + prow) / RPB) % CPR));
    const int goff1 = prow * dp + 4 * (pchk ^ (((1 * RPP + prow) / RPB) % CPR));
    // per-lane fragment offsets inside a 32-row block: logical chunks lh*CPR/2 + c of row li
    const int fsw = (li / RPB) % CPR;
    int fo[CPR / 2];
#pragma unroll
    for (int c = 0; c < CPR / 2; ++c) fo[c] = li * BK + 4 * ((lh * (CPR / 2) + c) ^ fsw);

    float kd[KM];
    int ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }

    const int nsteps = dp / BK;
    const float* qbase = qp + (size_t)qb * BQ * dp;

    // ---- DMA issue cursor (runs NS-1 stages ahead of the consumer) -------------------------
    // Piece j of this wave is piece pc = wave*LPW + j of a stage: an A piece (RPP corpus rows of
    // the tile) or a B piece (RPP queries).  Its source is base + tile offset + BK*stage floats.
    int64_t poff[LPW];
    bool pis_a[LPW];
    uint32_t pdst[LPW];
    bool pnt[LPW];                          // corpus piece of a one-query-block launch: read once
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
        const int pc = wave * LPW + j;
        pis_a[j] = pc < PA;
        pnt[j] = MODE == kModeBF16 && pis_a[j] && nqb == 1;   // fp32 rows: 1.94 -> 2.70 ms at nq = 1
        const int prow0 = pis_a[j] ? pc * RPP : (pc - PA) * RPP;
        poff[j] = (int64_t)prow0 * dp + (((prow0 / RPP) & 1) ? goff1 : goff0);
        pdst[j] = (uint32_t)(pis_a[j] ? pc * 256 : SA + (pc - PA) * 256) * 4u;
    }
    const uint32_t smem_u32 = lds_addr(smem);
    const uint32_t norm_u32 = lds_addr(norm_base);
    int it = t0, is = 0, ibuf = 0;
    const float* itile = xb + (size_t)tile(t0) * BM * dp;   // corpus rows of tile `it`
    auto issue_next = [&]() __attribute__((always_inline)) {
        if (it >= t1) return;
        const uint32_t st = smem_u32 + (uint32_t)(ibuf * STAGE) * 4u;
        if (is == 0) {                      // row norms of the tile, one 4-B DMA per lane
            for (int j = wave; j < BM / 64; j += NW)
                dma4(xnorm + (size_t)tile(it) * BM + j * 64 + lane,
                     norm_u32 + (uint32_t)(((it - t0) % NS) * BM + j * 64) * 4u);
        }
        const int k0 = is * BK;
#pragma unroll
        for (int j = 0; j < LPW; ++j) {
            if (pnt[j]) dma16_nt(itile + poff[j] + k0, st + pdst[j]);
            else dma16((pis_a[j] ? itile : qbase) + poff[j] + k0, st + pdst[j]);
        }
        if (++is == nsteps) { is = 0; ++it; itile += (size_t)nsplit * BM * dp; }
        ibuf = (ibuf + 1 == NS) ? 0 : ibuf + 1;
    };

#pragma unroll
    for (int j = 0; j < NS - 1; ++j) issue_next();
    int remaining = (t1 - t0) * nsteps;     // stages not yet consumed
    int cbuf = 0;

    for (int t = t0; t < t1; ++t) {
        const int row0 = tile(t) * BM;
        f32x16 acc[WB];
#pragma unroll
        for (int b = 0; b < WB; ++b) acc[b] = (f32x16){0.f};

        const float* st = smem;
        for (int s = 0; s < nsteps; ++s) {
            // own DMA of this stage landed (later stages may stay in flight)
            --remaining;                             // stages issued after this one: min(NS-2, remaining)
            if (remaining >= NS - 2) wait_vmcnt<LPW * (NS - 2)>();
            else if (NS > 3 && remaining == 1) wait_vmcnt<LPW>();
            else wait_vmcnt<0>();
            barrier_raw();                           // everyone's DMA landed; previous stage read

            st = smem + cbuf * STAGE;
            cbuf = (cbuf + 1 == NS) ? 0 : cbuf + 1;
            float a[WB][KH], bq[KH];
            {
                const float* bp = st + SA + wq * 32 * BK;
#pragma unroll
                for (int c = 0; c < CPR / 2; ++c) {
                    const float4 v = *reinterpret_cast<const float4*>(bp + fo[c]);
                    bq[4 * c] = v.x; bq[4 * c + 1] = v.y; bq[4 * c + 2] = v.z; bq[4 * c + 3] = v.w;
                }
            }
#pragma unroll
            for (int b = 0; b < WB; ++b) {
                const float* ap = st + (wr * RW + b * 32) * BK;
#pragma unroll
                for (int c = 0; c < CPR / 2; ++c) {
                    const float4 v = *reinterpret_cast<const float4*>(ap + fo[c]);
                    a[b][4 * c] = v.x; a[b][4 * c + 1] = v.y; a[b][4 * c + 2] = v.z; a[b][4 * c + 3] = v.w;
                }
            }
            // The stage's DMA pieces go out right after the fragment reads (their address math
            // overlaps the LDS latency), before the MFMAs.  Measured alternatives, all slower:
            // pieces pinned between MFMAs (38.6 ms vs 33.5 at BK=16), staggered per wave (38.8),
            // a 5-deep ring (39.0).
            issue_next();                            // refills the buffer the previous stage used
            if constexpr (MODE == kModeBF16) {
                // bf16 rows (2 elements per 32-bit word): this lane half's chunk c holds the 8
                // elements of MFMA k-step c (depth 32h + 8c + 0..7 of the 64-deep stage, the same
                // permutation on both operands); one bf16 MFMA per product
#pragma unroll
                for (int c = 0; c < CPR / 2; ++c) {
                    const bf16x8 bv = frag_bf16(bq, c);
#pragma unroll
                    for (int b = 0; b < WB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_bf16(a[b], c), bv, acc[b], 0, 0, 0);
                }
            } else if constexpr (MODE == kModeSplit) {
                // split layout: this lane half's chunks 2s / 2s+1 are the hi / lo bf16 planes of
                // MFMA k-step s; dot ~= hi.hi + hi.lo + lo.hi (the lo.lo term is below the bound)
#pragma unroll
                for (int s2 = 0; s2 < CPR / 4; ++s2) {
                    const bf16x8 bh = frag_bf16(bq, 2 * s2), bl = frag_bf16(bq, 2 * s2 + 1);
#pragma unroll
                    for (int b = 0; b < WB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_bf16(a[b], 2 * s2), bh, acc[b], 0, 0, 0);
#pragma unroll
                    for (int b = 0; b < WB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_bf16(a[b], 2 * s2), bl, acc[b], 0, 0, 0);
#pragma unroll
                    for (int b = 0; b < WB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag_bf16(a[b], 2 * s2 + 1), bh, acc[b], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int kk = 0; kk < KH; ++kk) {
#pragma unroll
                    for (int b = 0; b < WB; ++b)
                        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[b][kk], bq[kk], acc[b], 0, 0, 0);
                }
            }
        }

        // ---- epilogue: key = L2 distance (faiss exhaustive_L2sqr_blas form, clamped at 0) or
        // -ip; screened against this lane's K-th key and (<=) its partner lane's K-th key (the
        // partner holds the same query's other rows: a key worse than the partner's K-th cannot
        // reach the union's top K).  Survivors are parked in the stage this tile just consumed
        // (refilled only after the next barrier, which every wave reaches after its epilogue)
        // and inserted one by one.
        // every wave (all lanes: qvalid is per lane) passes this barrier exactly once per tile
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier_raw();                               // all fragment reads of the spent stage done
        if (qvalid) {
            const float* nrm = norm_base + ((t - t0) % NS) * BM;
            float* park = const_cast<float*>(st) + wave * (PR * 64);
#pragma unroll
            for (int b = 0; b < WB; ++b) {
                float key[16];
                unsigned mask = 0;
                const float tau = kd[KM - 1];
                const float tau_p = __shfl_xor(tau, 32, 64);
                const int rb = wr * RW + b * 32 + 4 * lh;      // row of accumulator reg 0
#pragma unroll
                for (int j = 0; j < 4; ++j) {                  // regs 4j..4j+3 = rows rb+8j+0..3
                    float4 n4 = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (metric == 1) n4 = *reinterpret_cast<const float4*>(nrm + rb + 8 * j);
                    const float nv[4] = {n4.x, n4.y, n4.z, n4.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = 4 * j + i;
                        const float ip = acc[b][r];
                        float kv;
                        if (metric == 1) {
                            kv = fmaf(-2.f, ip, qn + nv[i]);
                            kv = kv < 0.f ? 0.f : kv;
                        } else {
                            kv = -ip;
                        }
                        key[r] = kv;
                        const bool pass = (row0 + rb + 8 * j + i < nrows) && kv < tau && kv <= tau_p;
                        mask |= (unsigned)pass << r;
                    }
                }
                // survivors are inserted one per iteration per lane (ctz walk of the lane's own
                // mask): the wave loops max-popcount times, not once per row any lane needs
#pragma unroll
                for (int h = 0; h < 16 / PR; ++h) {
                    unsigned m = (mask >> (PR * h)) & ((1u << PR) - 1u);
                    if (__any(m != 0)) {
#pragma unroll
                        for (int r = 0; r < PR; ++r) park[r * 64 + lane] = key[PR * h + r];
                        while (__any(m != 0)) {
                            if (m) {
                                const int r = __builtin_ctz(m);
                                m &= m - 1u;
                                const float kv = park[r * 64 + lane];
                                const int rr = PR * h + r;
                                const int row = row0 + rb + (rr & 3) + 8 * (rr >> 2);
                                if (kv < kd[KM - 1]) list_insert_mono<KM>(kd, ki, kv, row);
                            }
                        }
                    }
                }
            }
        }
    }

    if (qvalid) {
        const size_t base = (size_t)qcol * ncand + (size_t)((split * WR + wr) * 2 + lh) * KM;
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            cand_d[base + p] = kd[p];
            cand_i[base + p] = ki[p] < 0 ? (int64_t)-1 : (int64_t)ki[p] + id_offset;
        }
    }
}

template <int WR, int WQ, int KM, int NS, int BK, int MODE, int WB>
__global__ void __launch_bounds__(WR * WQ * 64, IMGREC_MIN_WAVES(WR * WQ))
knn_tile_topk_kernel(const float* __restrict__ xb, const float* __restrict__ xnorm, int nrows,
                     int dp, const float* __restrict__ qp, const float* __restrict__ qnorm, int nq,
                     int metric, int ntiles, int nsplit, int nqb, int64_t id_offset,
                     float* __restrict__ cand_d, int64_t* __restrict__ cand_i, int ncand) {
    using G = TileGeom<WR, WQ, NS, BK, WB>;
    __shared__ __attribute__((aligned(16))) float smem[G::LDS_FLOATS];
    // XCD-aware, bijective block -> (query block, row split) map: blocks b and b+8 share an XCD;
    // consecutive remapped ids (same XCD) share a row split, so the corpus stages they stream are
    // served from that XCD's L2 for all query blocks.
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (wg >> 3);
    if (wgid >= nqb * nsplit) return;
    tile_topk_item<WR, WQ, KM, NS, BK, MODE, WB>(xb, xnorm, nrows, dp, qp, qnorm, nq, metric,
                                                 ntiles, nsplit, nqb, id_offset, cand_d, cand_i,
                                                 ncand, wgid, smem);
}

// ---------------------------------------------------------------------------------------------
// knn_merge: WPQ waves per query.  The input is nlists candidate lists per query, each sorted
// best-first (the fused kernel's per-lane lists, or gathered per-shard results); list l of query q
// starts at q*stride_q + l*stride_l and holds kin entries, label -1 marking an empty tail.
// A lane walks whole lists with 8-wide batches of independent loads and stops at the first entry
// that does not beat its running K-th (everything after it in a sorted list is worse); the lanes'
// lists are then reduced by k rounds of a 64-lane (key, label) argmin, per wave and, for WPQ > 1,
// once more over the waves' results through LDS.
// ---------------------------------------------------------------------------------------------
// k rounds of a wave-wide (key, label) argmin over the lanes' sorted lists.  Lane 0 writes round
// r to out_d/out_i[r] (memory, never a private array: a runtime index would go to scratch); with
// final != 0 it writes the faiss output convention (IP sign restored, empty = -1 / +-FLT_MAX).
template <int KM>
__device__ __forceinline__ void wave_select(float (&kd)[KM], int64_t (&ki)[KM], int k, int lane,
                                            float* out_d, int64_t* out_i, int final, int metric) {
    for (int r = 0; r < k; ++r) {
        float bd = kd[0];
        int64_t bi = ki[0];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float od = __shfl_xor(bd, off, 64);
            const int lo = __shfl_xor((int)(bi & 0xffffffff), off, 64);
            const int hi = __shfl_xor((int)(bi >> 32), off, 64);
            const int64_t oi = ((int64_t)hi << 32) | (uint32_t)lo;
            // empty entries (label -1) rank last regardless of their key
            const bool take = (oi >= 0) && (bi < 0 || ranks_before(od, oi, bd, bi));
            bd = take ? od : bd;
            bi = take ? oi : bi;
        }
        if (bi >= 0 && kd[0] == bd && ki[0] == bi) {
#pragma unroll
            for (int p = 0; p < KM - 1; ++p) { kd[p] = kd[p + 1]; ki[p] = ki[p + 1]; }
            kd[KM - 1] = INFINITY;
            ki[KM - 1] = -1;
        }
        if (lane == 0) {
            if (final) {
                out_d[r] = bi < 0 ? ((metric == 1) ? FLT_MAX : -FLT_MAX) : ((metric == 1) ? bd : -bd);
            } else {
                out_d[r] = bi < 0 ? INFINITY : bd;
            }
            out_i[r] = bi;
        }
    }
}

// One query (WPQ = 4) or four (WPQ = 1) of knn_merge_kernel; block-uniform control flow (no
// wave leaves before the block's __syncthreads).
template <int KM, int WPQ>
__device__ __forceinline__ void merge_block(const float* __restrict__ cd, const int64_t* __restrict__ ci,
                                            int64_t blk, int64_t nq, int nlists, int kin,
                                            int64_t stride_q, int64_t stride_l, int64_t stride_li,
                                            int k, int metric, int negate_in, float* __restrict__ D,
                                            int64_t* __restrict__ I, float* __restrict__ floor_out,
                                            const int* __restrict__ out_rows,
                                            float (&sd)[4][KM], int64_t (&si)[4][KM]) {
    constexpr int QPB = 4 / WPQ;                     // queries per 256-thread block
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t q = blk * QPB + wave / WPQ;
    const int sub = wave % WPQ;
    const bool active = q < nq;

    float kd[KM];
    int64_t ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }

    // floor (candidate merges only): the smallest key among rows that no output can contain
    // because a full input list ended before them (its last key) or a lane list dropped them
    float floor_v = INFINITY;
    bool dropped = false;
    if (active) {
        for (int l = sub * 64 + lane; l < nlists; l += 64 * WPQ) {
            const float* lp = cd + q * stride_q + (int64_t)l * stride_l;
            const int64_t* ip = ci + q * stride_q + (int64_t)l * stride_li;
            if (floor_out && ip[kin - 1] >= 0) floor_v = fminf(floor_v, lp[kin - 1]);
            bool stop = false;
            for (int p0 = 0; p0 < kin && !stop; p0 += 8) {
                float d8[8];
                int64_t i8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {         // clamped index: loads are unconditional
                    const int p = min(p0 + j, kin - 1);
                    d8[j] = lp[p];
                    i8[j] = ip[p];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float d = negate_in ? -d8[j] : d8[j];
                    const bool real = !stop && (p0 + j < kin) && i8[j] >= 0;
                    const bool ok = real && ranks_before(d, i8[j], kd[KM - 1], ki[KM - 1]);
                    // a real entry turned away, or one pushed out of a full lane list
                    dropped = dropped || (real && (!ok || ki[KM - 1] >= 0));
                    stop = stop || !ok;
                    if (ok) list_insert<KM, int64_t>(kd, ki, d, i8[j]);
                }
            }
        }
    }

    if (WPQ == 1) {
        if (floor_out) {
            if (dropped) floor_v = fminf(floor_v, kd[KM - 1]);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) floor_v = fminf(floor_v, __shfl_xor(floor_v, off, 64));
            if (active && lane == 0) floor_out[q] = floor_v;
        }
        if (active) {
            const int64_t orow = out_rows ? (int64_t)out_rows[q] : q;
            wave_select<KM>(kd, ki, k, lane, D + orow * k, I + orow * k, 1, metric);
        }
        return;
    }
    // WPQ == 4: one query per block; every wave's top-k to LDS, wave 0 merges the 4k.
    wave_select<KM>(kd, ki, k, lane, sd[wave], si[wave], 0, metric);
    __syncthreads();
    if (wave == 0 && active) {
#pragma unroll
        for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }
        if (lane < 4) {
            for (int r = 0; r < k; ++r) {
                const float d = sd[lane][r];
                const int64_t id = si[lane][r];
                if (id < 0) break;
                list_insert<KM, int64_t>(kd, ki, d, id);
            }
        }
        const int64_t orow = out_rows ? (int64_t)out_rows[q] : q;
        wave_select<KM>(kd, ki, k, lane, D + orow * k, I + orow * k, 1, metric);
    }
}

template <int KM, int WPQ>
__global__ void __launch_bounds__(256)
knn_merge_kernel(const float* __restrict__ cd, const int64_t* __restrict__ ci, int64_t nq,
                 int nlists, int kin, int64_t stride_q, int64_t stride_l, int64_t stride_li, int k,
                 int metric, int negate_in, float* __restrict__ D, int64_t* __restrict__ I,
                 float* __restrict__ floor_out) {
    __shared__ float sd[4][KM];
    __shared__ int64_t si[4][KM];
    merge_block<KM, WPQ>(cd, ci, blockIdx.x, nq, nlists, kin, stride_q, stride_l, stride_li, k,
                         metric, negate_in, D, I, floor_out, nullptr, sd, si);
}

// One wave merges query q's nlists sorted lists of kin entries (list l at q * stride_q + l * kin,
// label -1 = empty) into output row orow of D / I (faiss convention).  The certificate tail's
// exact re-run: a query block's lists are merged by the workgroup that finished its last split.
template <int KM>
__device__ __forceinline__ void merge_query_wave(const float* __restrict__ cd,
                                                 const int64_t* __restrict__ ci, int64_t q,
                                                 int nlists, int kin, int64_t stride_q, int k,
                                                 int metric, float* __restrict__ D,
                                                 int64_t* __restrict__ I, int64_t orow) {
    const int lane = threadIdx.x & 63;
    float kd[KM];
    int64_t ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }
    for (int l = lane; l < nlists; l += 64) {
        const float* lp = cd + q * stride_q + (int64_t)l * kin;
        const int64_t* ip = ci + q * stride_q + (int64_t)l * kin;
        for (int p = 0; p < kin; ++p) {
            const int64_t id = ip[p];
            const float d = lp[p];
            if (id < 0 || !ranks_before(d, id, kd[KM - 1], ki[KM - 1])) break;   // sorted list
            list_insert<KM, int64_t>(kd, ki, d, id);
        }
    }
    wave_select<KM>(kd, ki, k, lane, D + orow * k, I + orow * k, 1, metric);
}

// ---------------------------------------------------------------------------------------------
// cert_tail_kernel<KM>: everything after the rerank of a candidate chunk in ONE launch (it was
// four: second chance, re-run plan, exact tile, merge — each ~4.5 us even when empty, most of it
// the kernel boundary and a dependent load of a device count).  Reads the chunk's counts, which
// the rerank wrote: with nothing queued, workgroup 0 folds the stats and every workgroup exits.
// Otherwise, with no workgroup ever waiting on one that has not yet claimed work (so the launch
// cannot deadlock whatever else shares the GPU — the multi-device index runs shards concurrently
// on one device):
//   1. second-chance units (item, slice) are claimed from ctl[0]; the workgroup that finishes an
//      item's last slice answers it and counts it in ctl[1]; the one that completes the last item
//      (or takes ticket 0 when none was queued) is the planner;
//   2. the planner folds the stats, gathers the uncertified queries (fail_list) into fq / fqn
//      (zero rows up to a multiple of 32), zeroes the per-query-block tickets and publishes
//      ctl[2] = count + 1 (at once when count = 0: nothing to gather); everyone else waits for
//      it (the planner is running: it completed an item).  With one item its finisher is the
//      planner without the ctl[1] count;
//   3. exact (2,1)-tile items (query block, row split) are claimed from ctl[3]; the workgroup
//      that finishes a query block's last split merges that block's lists into the rows
//      fail_list[q] of D / I.
// ctl[0..3] are zeroed by the rerank kernel (the launch before this one on the stream; with
// RerankArgs::direct, by the candidate scan, and every query is a second-chance item).
// ---------------------------------------------------------------------------------------------
constexpr int kTailWR = 2, kTailNS = 3, kTailBK = 16, kTailWB = 4, kTailWaves = kTailWR;

template <int KM>
__global__ void __launch_bounds__(kTailWaves * 64, 1)
cert_tail_kernel(const TailArgs a) {
    using G = TileGeom<kTailWR, 1, kTailNS, kTailBK, kTailWB>;
    constexpr int kFloats = G::LDS_FLOATS > (int)(sizeof(SecondChanceLDS) / 4 + 1)
                                ? G::LDS_FLOATS : (int)(sizeof(SecondChanceLDS) / 4 + 1);
    __shared__ __attribute__((aligned(16))) float smem[kFloats];
    __shared__ int s_val;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int* const sp = a.stat + 4 * a.parity;
    int* const ctl = a.r.tail_ctl;
    TAIL_STAMP(0);
    // final: the rerank kernel has completed (direct: no rerank ran, every query is an item)
    const int n_chance = a.r.direct ? (int)a.r.nq : sp[3];
    const int q_item0 = !a.r.direct && a.r.chance_list ? a.r.chance_list[0] : -1;   // same round trip
    if (n_chance == 0 && sp[0] == 0) {          // the common case: every query certified
        if (blockIdx.x == 0 && t == 0) {
            int* acc = a.stat + 8;
            acc[0] = a.first ? 0 : acc[0];
            acc[1] = a.first ? sp[1] : max(acc[1], sp[1]);   // ratio >= 0: bit order = float order
            acc[2] = a.first ? sp[2] : acc[2] + sp[2];
            int* other = a.stat + 4 * (a.parity ^ 1);
            other[0] = 0; other[1] = 0; other[2] = 0; other[3] = 0;
        }
        return;
    }
    // ---- 1. second chance ----------------------------------------------------------------
    bool planner = false;
    int known = -1;                             // the re-run count, when the planner knows it
    if (n_chance > 0) {
        // units = (item, slice): workgroup b takes unit b, then (only when the units outnumber
        // the grid) claims grid + ctl[0]++ — the grid's first claims all on one address
        // serialised ~3 us of a one-query tail; the workgroup that finishes an item's last slice
        // counts the item in ctl[1]
        const int S = a.r.sc_slices;
        bool first_unit = true;
        for (;;) {
            int unit = (int)blockIdx.x;
            if (!first_unit) {
                if ((int)gridDim.x >= n_chance * S) break;     // every unit was a first one
                if (t == 0)
                    s_val = (int)gridDim.x + __hip_atomic_fetch_add(ctl + 0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __syncthreads();
                unit = s_val;
                __syncthreads();
            }
            first_unit = false;
            TAIL_STAMP(1);
            if (unit >= n_chance * S) break;
            const int res = second_chance_slice<kTailWaves>(a.r, unit / S, unit % S,
                                                            *reinterpret_cast<SecondChanceLDS*>(smem), q_item0);
            if (res == 0) continue;
            if (n_chance == 1) {                // the only item: its finisher plans, no count;
                planner = true;                 // its outcome is the chunk's re-run count (the
                known = res == 2 ? 1 : 0;       // rerank queues every failure for the chance)
                continue;
            }
            wg_release_stores();
            if (t == 0) {
                const int done = lane0_release_add(ctl + 1);
                s_val = done == n_chance - 1;
                if (s_val) lane0_acquire();
            }
            __syncthreads();
            planner = planner || s_val != 0;
            __syncthreads();
        }
    } else {
        if (t == 0) s_val = __hip_atomic_fetch_add(ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
        __syncthreads();
        planner = s_val != 0;
        __syncthreads();
    }
    // ---- 2. plan + query gather (one workgroup) ------------------------------------------
    int count;
    if (planner) {
        count = known >= 0 ? known : __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int nqb = (count + 31) / 32;
        // nothing to re-run: release the waiters at once (they read nothing the planner writes
        // below; ctl[2] = count + 1 carries the count, saving each waiter a reload of sp)
        if (count == 0 && t == 0) __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        TAIL_STAMP(6);
        if (count > 0) wg_release_stores();     // this workgroup's fail_list stores (one item)
        if (t == 0) {
            int* acc = a.stat + 8;
            const int first_fail = a.r.direct ? (int)a.r.nq : sp[2];   // direct: all had no first pass
            acc[0] = a.first ? count : acc[0] + count;
            acc[1] = a.first ? sp[1] : max(acc[1], sp[1]);
            acc[2] = a.first ? first_fail : acc[2] + first_fail;
            int* other = a.stat + 4 * (a.parity ^ 1);
            other[0] = 0; other[1] = 0; other[2] = 0; other[3] = 0;
        }
        for (int i = t; i < nqb; i += kTailWaves * 64) a.ticket[i] = 0;
        for (int row = wave; row < nqb * 32; row += kTailWaves) {
            float* o = a.fq + (int64_t)row * a.dp;
            if (row >= count) {
                for (int j = lane; j < a.dp; j += 64) o[j] = 0.f;
                if (lane == 0) a.fqn[row] = 0.f;
                continue;
            }
            const int src = a.r.fail_list[row];
            const float* s = a.qpad + (int64_t)src * a.dp;
            for (int j = lane; j < a.dp; j += 64) o[j] = s[j];
            if (lane == 0) a.fqn[row] = a.qnorm[src];
        }
        if (count == 0) { TAIL_STAMP(7); return; }
        wg_release_stores();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(ctl + 2, count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lane0_acquire();                    // this CU's L1 holds no stale copy of fq either
        }
        __syncthreads();
    } else {
        if (t == 0) {
            // the planner is running (it completed an item or took ticket 0); the bound only
            // turns a broken invariant into a reported error (stats bit) instead of a hang
            int spins = 0, c2;
            s_val = 0;
            while ((c2 = __hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1 << 26)) break;
            }
            if (c2 == 0) atomicOr(a.stat + 11, 1);
            else if (c2 > 1) lane0_acquire();
            s_val = c2 - 1;                     // -1: timed out
        }
        __syncthreads();
        TAIL_STAMP(6);
        count = s_val;
        if (count <= 0) { TAIL_STAMP(7); return; }
    }
    // ---- 3. exact re-run: (query block, row split) items, merged by each block's last split ----
    const int nqb = (count + 31) / 32;
    const int nsplit = max(1, min((int)gridDim.x / nqb, a.ntiles));
    const int nitems = nqb * nsplit;
    const int ncand = nsplit * a.lists_km;
    for (;;) {
        if (t == 0) s_val = __hip_atomic_fetch_add(ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int item = s_val;
        __syncthreads();
        if (item >= nitems) break;
        tile_topk_item<kTailWR, 1, KM, kTailNS, kTailBK, kModeF32, kTailWB>(
            a.xb, a.xn, a.nrows, a.dp, a.fq, a.fqn, count, a.metric, a.ntiles, nsplit, nqb,
            a.id_offset, a.fcd, a.fci, ncand, item, smem);
        const int qb = item % nqb;
        wg_release_stores();
        if (t == 0) {
            const int done = lane0_release_add(a.ticket + qb);
            s_val = done == nsplit - 1;
            if (s_val) lane0_acquire();
        }
        __syncthreads();
        if (s_val) {
            for (int ql = qb * 32 + wave; ql < min(count, qb * 32 + 32); ql += kTailWaves)
                merge_query_wave<KM>(a.fcd, a.fci, ql, ncand / KM, KM, ncand, a.r.k, a.metric,
                                     a.r.D, a.r.I, a.r.fail_list[ql]);
        }
        __syncthreads();                        // s_val and the LDS ring reused by the next item
    }
}

#ifdef IMGREC_TAIL_STAMPS
extern "C" int knn_tail_stamps_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_tail_stamps), sizeof(imgrec::g_tail_stamps));
}
extern "C" int knn_tail_stamps_clear() {
    static unsigned long long zero[1024 * 8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(imgrec::g_tail_stamps), zero, sizeof(zero));
}
#endif

hipError_t launch_cert_tail(const TailArgs& a, int grid, hipStream_t st) {
    if (grid <= 0 || !a.r.tail_ctl || !a.ticket || a.dp % kTailBK != 0) return hipErrorInvalidValue;
    if (a.lists_km != 2 * kTailWR * a.km) return hipErrorInvalidValue;
#define IMGREC_TAIL(KMV) hipLaunchKernelGGL((cert_tail_kernel<KMV>), dim3((unsigned)grid), \
                                            dim3(kTailWaves * 64), 0, st, a)
    switch (a.km) {
        case 8: IMGREC_TAIL(8); break;
        case 10: IMGREC_TAIL(10); break;
        case 16: IMGREC_TAIL(16); break;
        case 32: IMGREC_TAIL(32); break;
        default: return hipErrorInvalidValue;
    }
#undef IMGREC_TAIL
    return hipGetLastError();
}

__global__ void fill_empty_kernel(float* __restrict__ D, int64_t* __restrict__ I, int64_t n,
                                  int metric) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { D[i] = (metric == 1) ? FLT_MAX : -FLT_MAX; I[i] = -1; }
}

// ---------------------------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------------------------
hipError_t launch_rows_ingest(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                              int normalize, float* dst, float* norms, hipStream_t st) {
    if (n_pad <= 0) return hipSuccess;
    const int64_t blocks = (n_pad + 3) / 4;
    hipLaunchKernelGGL(rows_ingest_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, n, d, dp,
                       n_pad, normalize, dst, norms);
    return hipGetLastError();
}

template <int WR, int WQ, int NS, int BK, int MODE = kModeF32, int WB = 4>
static hipError_t launch_tile_km(int km, const TileArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)(a.nqb * a.nsplit)), block(WR * WQ * 64);
#define IMGREC_LAUNCH_TILE(KMV)                                                                   \
    hipLaunchKernelGGL((knn_tile_topk_kernel<WR, WQ, KMV, NS, BK, MODE, WB>), grid, block, 0, st, a.xb, \
                       a.xnorm, a.nrows, a.dp, a.qp, a.qnorm, a.nq, a.metric, a.ntiles, a.nsplit, \
                       a.nqb, a.id_offset, a.cand_d, a.cand_i, a.ncand)
    switch (km) {
        case 8: IMGREC_LAUNCH_TILE(8); break;
        case 10: IMGREC_LAUNCH_TILE(10); break;
        case 16: IMGREC_LAUNCH_TILE(16); break;
        case 32: IMGREC_LAUNCH_TILE(32); break;
        default: return hipErrorInvalidValue;
    }
#undef IMGREC_LAUNCH_TILE
    return hipGetLastError();
}

// (1,8) exact tile of the ablations kept in DESIGN.md: 32-deep stages, 3-slot ring
constexpr int kBKBig = 32, kNSBig = 3;

hipError_t launch_tile_topk(const TileArgs& a, hipStream_t st) {
    if (a.mode == kModeBF16) {
        // bf16 candidate pass: rows of dp bf16 = dp/2 words, 64-deep (32-word) stages
        if (a.dp % 32 != 0 || (a.km != 16 && a.km != 32)) return hipErrorInvalidValue;
        if (a.wb != kB16WB) return hipErrorInvalidValue;
        if (a.wr == kB16WR && a.wq == kB16WQ)
            return launch_tile_km<kB16WR, kB16WQ, kB16NS, 32, kModeBF16, kB16WB>(a.km, a, st);
        // small batches: 256 rows x 32 queries, two 2-wave workgroups per CU
        if (a.wr == 2 && a.wq == 1) return launch_tile_km<2, 1, 2, 32, kModeBF16, kB16WB>(a.km, a, st);
        return hipErrorInvalidValue;
    }
    if (a.mode == kModeSplit) {
        // split-bf16 candidate pass (knn_refine.hip certifies and reranks its output); the
        // staging depth must be the one the split copy was laid out for (a.sbk)
        if (a.dp % 32 != 0 || (a.km != 16 && a.km != 32)) return hipErrorInvalidValue;
        if (a.sbk != kSplitBK || a.wb != kSplitWB) return hipErrorInvalidValue;
        if (a.wr == 1 && a.wq == 4)
            return launch_tile_km<1, 4, kSplitNS, kSplitBK, kModeSplit, kSplitWB>(a.km, a, st);
        return hipErrorInvalidValue;
    }
    if (a.dp % kBKBig != 0 && a.wr == 1 && a.wq == 8)
        return launch_tile_km<1, 8, 4, 16>(a.km, a, st);
    if (a.wr == 1 && a.wq == 8) return launch_tile_km<1, 8, kNSBig, kBKBig>(a.km, a, st);
    if (a.wr == 1 && a.wq == 4 && a.dp % 32 == 0) return launch_tile_km<1, 4, 2, 32>(a.km, a, st);
    if (a.wr == 1 && a.wq == 4) return launch_tile_km<1, 4, 2, 16>(a.km, a, st);
    if (a.wr == 2 && a.wq == 2) return launch_tile_km<2, 2, 3, 16>(a.km, a, st);
    if (a.wr == 2 && a.wq == 1) return launch_tile_km<2, 1, 3, 16>(a.km, a, st);
    return hipErrorInvalidValue;
}

hipError_t launch_merge(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                        int64_t stride_q, int64_t stride_l, int k, int metric, int negate_in,
                        float* D, int64_t* I, hipStream_t st) {
    return launch_merge_strided(cd, ci, nq, nlists, kin, stride_q, stride_l, stride_l, k, metric,
                                negate_in, D, I, st);
}

hipError_t launch_merge_strided(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                                int64_t stride_q, int64_t stride_l, int64_t stride_li, int k,
                                int metric, int negate_in, float* D, int64_t* I, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    // few queries with many lists: 4 waves per query; otherwise one wave per query
    const bool wide = nq < 1024 && nlists > 256;
    const dim3 block(256);
    const dim3 grid((unsigned)(wide ? nq : (nq + 3) / 4));
#define IMGREC_LAUNCH_MERGE(KMV)                                                                    \
    do {                                                                                            \
        if (wide)                                                                                   \
            hipLaunchKernelGGL((knn_merge_kernel<KMV, 4>), grid, block, 0, st, cd, ci, nq, nlists, \
                               kin, stride_q, stride_l, stride_li, k, metric, negate_in, D, I, nullptr); \
        else                                                                                        \
            hipLaunchKernelGGL((knn_merge_kernel<KMV, 1>), grid, block, 0, st, cd, ci, nq, nlists, \
                               kin, stride_q, stride_l, stride_li, k, metric, negate_in, D, I, nullptr); \
    } while (0)
    if (k <= 8) IMGREC_LAUNCH_MERGE(8);
    else if (k <= 10) IMGREC_LAUNCH_MERGE(10);
    else if (k <= 16) IMGREC_LAUNCH_MERGE(16);
    else if (k <= 32) IMGREC_LAUNCH_MERGE(32);
    else return hipErrorInvalidValue;
#undef IMGREC_LAUNCH_MERGE
    return hipGetLastError();
}

// Candidate merge when every lane holds at most one sorted input list (<= 64 lists per query):
// entries packed into one 64-bit value (order-preserving key bits | local row), the kout
// smallest found by a wave select (wave_ops.h).

// A query's nlists lists may be split into G groups of <= 64 (two-level merge): wave s handles
// group s % G of query s / G; floor_in (optional, G per output row of the previous level) is
// folded into the output floor.
template <int KIN>
__global__ void __launch_bounds__(256)
cand_merge_lane_kernel(const float* __restrict__ cd, const int64_t* __restrict__ ci, int64_t nsub,
                       int nlists, int G, int64_t stride_q, int64_t stride_l, int kout,
                       int64_t id_offset, const float* __restrict__ floor_in, int G_in,
                       float* __restrict__ D, int64_t* __restrict__ I, float* __restrict__ floor_out) {
    const int lane = threadIdx.x & 63;
    const int64_t sq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (sq >= nsub) return;                                     // whole wave
    const int64_t q = sq / G;
    const int grp = (int)(sq - q * G);
    const int nl = min(64, nlists - 64 * grp);                  // lists of this group
    constexpr uint64_t kEmpty = ~0ull;
    uint64_t v[KIN];
    float fl = (floor_in && lane < G_in) ? floor_in[sq * G_in + lane] : INFINITY;
    if (lane < nl) {
        const float* lp = cd + q * stride_q + (int64_t)(64 * grp + lane) * stride_l;
        const int64_t* ip = ci + q * stride_q + (int64_t)(64 * grp + lane) * stride_l;
#pragma unroll
        for (int p = 0; p < KIN; ++p) {
            const float kv = lp[p];
            const int64_t lab = ip[p];
            v[p] = lab < 0 ? kEmpty
                           : ((uint64_t)key_bits_ordered(kv) << 32) | (uint32_t)(lab - id_offset);
        }
        if (ip[KIN - 1] >= 0) fl = fminf(fl, lp[KIN - 1]);      // a full list: its last key
    } else {
#pragma unroll
        for (int p = 0; p < KIN; ++p) v[p] = kEmpty;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
    if (lane == 0) floor_out[sq] = fl;

    // the leading-entry bound + survivor ranks (wave_select_sorted): the list heads for
    // kout <= 16 (level 1 of the two-level merge), the first two entries of every list above
    uint64_t mine = 0;
    int rank = 0;
    __shared__ uint64_t sel[4][128 + 192];
    uint64_t* const buf = sel[threadIdx.x >> 6];
    const int K = kout <= 16 ? wave_select_sorted<KIN, 1, 256>(v, kout, buf, mine, rank)
                             : wave_select_sorted<KIN, 2, 192>(v, kout, buf, mine, rank);
    if (lane < K) {
        D[sq * kout + rank] = key_from_ordered((uint32_t)(mine >> 32));
        I[sq * kout + rank] = (int64_t)(uint32_t)mine + id_offset;
    } else if (lane < kout) {
        D[sq * kout + lane] = FLT_MAX;
        I[sq * kout + lane] = -1;
    }
}

// Block-wide candidate merge (round 3), one NT-thread block per query: the query's M = nlists x kin
// entries (sorted (key, global label) lists, label -1 = empty, at cd / ci + q * stride_q, list l
// at l * kin) are packed as (order-preserving key bits | local row) u64 in registers (PER per
// thread) and the K = min(kout, valid) smallest are found by the same bit-by-bit threshold select
// as cand_merge_lane_kernel, with block-wide counts: 32 steps over the key bits — fewer, from
// the highest bit where the smallest and largest valid value differ — and the row bits only when
// the K-th key is tied.  The K winners are compacted by a block scan and each placed at its rank.
// Floor = min(floor_in of every list, when given; the last key of every full list).
// The second level after cand_merge_lane_kernel (NT 256, G <= 64 lists of <= 64) when level 1
// keeps kout per group (kout <= 16, or IMGREC_MERGE_K1=0), where it replaced a one-wave LDS-queue
// merge (32.5 -> 17.3 us per query at nq = 1); with 16 per group the second level is one more
// lane-kernel wave (16.0 -> ~7 us at nq = 1, round 3).  Measured and
// dropped: the whole merge of a small batch in one 1024-thread block per query (2048 lists x 16
// at nq = 1, 32 entries per thread): 50.1 us against the two levels' 32 us — one CU's VALU
// issue of the counts, where level 1 spreads the lists over 32 waves on as many CUs
// (profiles/r03/nq1_single_level_merge_rejected.csv).
template <int NT>
__device__ __forceinline__ int block_sum_i32(int x, int* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int w = wave_sum_i32(x);
    if (lane == 0) red[wave] = w;
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) tot += red[i];
    __syncthreads();                                  // red reused by the next call
    return tot;
}

template <int NT, int PER>
__global__ void __launch_bounds__(NT)
cand_merge_block_kernel(const float* __restrict__ cd, const int64_t* __restrict__ ci, int64_t nq,
                        int nlists, int kin, int64_t stride_q, int kout, int64_t id_offset,
                        const float* __restrict__ floor_in, float* __restrict__ D,
                        int64_t* __restrict__ I, float* __restrict__ floor_out) {
    constexpr int NW = NT / 64;
    __shared__ int red[NW];
    __shared__ float redf[NW];
    __shared__ uint64_t redm[2][NW];
    __shared__ uint64_t sel[64];
    constexpr uint64_t kEmpty = ~0ull;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t q = blockIdx.x;
    const int M = nlists * kin;
    const float* qd = cd + q * stride_q;
    const int64_t* qi = ci + q * stride_q;
    uint64_t v[PER];
    int nvl = 0;
    uint64_t vmin = kEmpty, vmax = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int e = t + j * NT;
        v[j] = kEmpty;
        if (e < M) {
            const int64_t lab = qi[e];
            if (lab >= 0) {
                v[j] = ((uint64_t)key_bits_ordered(qd[e]) << 32) | (uint32_t)(lab - id_offset);
                ++nvl;
                vmin = v[j] < vmin ? v[j] : vmin;
                vmax = v[j] > vmax ? v[j] : vmax;
            }
        }
    }
    vmin = wave_min_u64(vmin);
    vmax = ~wave_min_u64(~vmax);
    if (lane == 0) { redm[0][wave] = vmin; redm[1][wave] = vmax; }
    float fl = INFINITY;
    for (int l = t; l < nlists; l += NT) {
        if (floor_in) fl = fminf(fl, floor_in[q * nlists + l]);
        const int last = l * kin + kin - 1;
        if (qi[last] >= 0) fl = fminf(fl, qd[last]);       // a full list: its last key
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fl = fminf(fl, __shfl_xor(fl, off, 64));
    if (lane == 0) redf[wave] = fl;
    auto count_le = [&](uint64_t x) __attribute__((always_inline)) {
        int c = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) c += v[j] <= x ? 1 : 0;
        return c;
    };
    const int K = min(kout, block_sum_i32<NT>(nvl, red));   // (its barrier publishes redf, redm)
    if (t == 0) {
        float f = redf[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) f = fminf(f, redf[i]);
        floor_out[q] = f;
    }
    uint64_t T = 0;
    if (K > 0) {
        // bits above the highest difference of the valid values' min and max are common to T
        for (int i = 0; i < NW; ++i) {
            vmin = redm[0][i] < vmin ? redm[0][i] : vmin;
            vmax = redm[1][i] > vmax ? redm[1][i] : vmax;
        }
        const int hb = vmin == vmax ? -1 : 63 - __builtin_clzll(vmin ^ vmax);
        uint64_t prefix = hb < 0 ? vmin : (hb >= 63 ? 0 : vmin & ~((2ull << hb) - 1));
        for (int b = min(hb, 63); b >= 32; --b) {
            const uint64_t lo = prefix | ((1ull << b) - 1);
            if (block_sum_i32<NT>(count_le(lo), red) < K) prefix |= 1ull << b;
        }
        T = prefix | 0xffffffffull;
        if (block_sum_i32<NT>(count_le(T), red) > K) {    // the K-th key is tied: rows decide
            for (int b = min(hb, 31); b >= 0; --b) {
                const uint64_t lo = prefix | ((1ull << b) - 1);
                if (block_sum_i32<NT>(count_le(lo), red) < K) prefix |= 1ull << b;
            }
            T = prefix;
        }
    }
    // compaction of the K winners (values are distinct: a row sits in one list)
    const int c = K > 0 ? count_le(T) : 0;
    const int wex = wave_excl_scan_i32(c);
    if (lane == 63) red[wave] = wex + c;
    __syncthreads();
    int base = wex;
    for (int i = 0; i < wave; ++i) base += red[i];
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if (v[j] <= T && K > 0) sel[base++] = v[j];
    __syncthreads();
    if (t < K) {
        const uint64_t mine = sel[t];
        int rank = 0;
        for (int j = 0; j < K; ++j) rank += sel[j] < mine ? 1 : 0;
        D[q * kout + rank] = key_from_ordered((uint32_t)(mine >> 32));
        I[q * kout + rank] = (int64_t)(uint32_t)mine + id_offset;
    } else if (t < kout) {
        D[q * kout + t] = FLT_MAX;
        I[q * kout + t] = -1;
    }
}

hipError_t launch_merge_candidates(const float* cd, const int64_t* ci, int64_t nq, int nlists,
                                   int kin, int64_t stride_q, int64_t stride_l, int kout,
                                   int64_t id_offset, float* D, int64_t* I, float* floor,
                                   float* ws_d, int64_t* ws_i, float* ws_floor, hipStream_t st,
                                   int* l1_G) {
    if (l1_G) *l1_G = 0;
    if (nq <= 0) return hipSuccess;
    if (kout <= 0 || kout > 64 || !floor) return hipErrorInvalidValue;
    const int G = (nlists + 63) / 64;
    if ((kin == 8 || kin == 10 || kin == 16) && G <= 64 && (G == 1 || (ws_d && ws_i && ws_floor))) {
#define IMGREC_CAND_LANE(KV, NSUB, NL, GG, SQ, SL, KO, FIN, GIN, OD, OI, OF)                      \
        hipLaunchKernelGGL((cand_merge_lane_kernel<KV>), dim3((unsigned)(((NSUB) + 3) / 4)), dim3(256), \
                           0, st, cd_, ci_, NSUB, NL, GG, SQ, SL, KO, id_offset, FIN, GIN, OD, OI, OF)
        const float* cd_ = cd;
        const int64_t* ci_ = ci;
        if (G == 1) {
            if (kin == 8) IMGREC_CAND_LANE(8, nq, nlists, 1, stride_q, stride_l, kout, nullptr, 0, D, I, floor);
            else if (kin == 10) IMGREC_CAND_LANE(10, nq, nlists, 1, stride_q, stride_l, kout, nullptr, 0, D, I, floor);
            else IMGREC_CAND_LANE(16, nq, nlists, 1, stride_q, stride_l, kout, nullptr, 0, D, I, floor);
            return hipGetLastError();
        }
        // level 1: each group of 64 lists -> its k1 best (+ floor: a group that keeps fewer
        // than kout would cap the certificate at that group's last key); level 2: the G lists.
        // k1 = 16 when kout > 16: a group rarely holds more than 16 of the kout best (at G = 12,
        // ~5), and when it does its full list's 16th key is the floor the certificate then
        // uses; level 2 is then one more wave (G lists of 16) instead of a block select over
        // G x kout.  IMGREC_MERGE_K1=0 keeps k1 = kout.
        static const bool k1_16 = [] {
            const char* e = std::getenv("IMGREC_MERGE_K1");
            return !(e && *e == '0');
        }();
        const int64_t nsub = nq * (int64_t)G;
        if (k1_16 && kout > 16) {
            if (kin == 8) IMGREC_CAND_LANE(8, nsub, nlists, G, stride_q, stride_l, 16, nullptr, 0, ws_d, ws_i, ws_floor);
            else if (kin == 10) IMGREC_CAND_LANE(10, nsub, nlists, G, stride_q, stride_l, 16, nullptr, 0, ws_d, ws_i, ws_floor);
            else IMGREC_CAND_LANE(16, nsub, nlists, G, stride_q, stride_l, 16, nullptr, 0, ws_d, ws_i, ws_floor);
            hipError_t e1 = hipGetLastError();
            if (e1 != hipSuccess) return e1;
            if (l1_G && 16 * G <= kRerankWaves * 64) {   // level 2 in the rerank (an entry a thread)
                *l1_G = G;
                return hipSuccess;
            }
            cd_ = ws_d;
            ci_ = ws_i;
            IMGREC_CAND_LANE(16, nq, G, 1, (int64_t)G * 16, 16, kout, ws_floor, G, D, I, floor);
            return hipGetLastError();
        }
        if (kin == 8) IMGREC_CAND_LANE(8, nsub, nlists, G, stride_q, stride_l, kout, nullptr, 0, ws_d, ws_i, ws_floor);
        else if (kin == 10) IMGREC_CAND_LANE(10, nsub, nlists, G, stride_q, stride_l, kout, nullptr, 0, ws_d, ws_i, ws_floor);
        else IMGREC_CAND_LANE(16, nsub, nlists, G, stride_q, stride_l, kout, nullptr, 0, ws_d, ws_i, ws_floor);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        // Level 2 (the G group outputs): the block-wide threshold select above.  Round 2's
        // one-wave LDS-queue merge took 31-32.5 us per query at nq = 1; also measured and
        // dropped then: the threshold select with a group's 64 outputs per lane of ONE wave
        // (cand_merge_lane_kernel<64>, 32.5 us), reading each queue's next entry one pop ahead
        // (32.3 us), and a 256-thread rank form (binary searches of every entry in every other
        // queue, 123 us: dependent LDS reads per thread).
#undef IMGREC_CAND_LANE
        hipLaunchKernelGGL((cand_merge_block_kernel<256, 16>), dim3((unsigned)nq), dim3(256), 0, st,
                           ws_d, ws_i, nq, G, kout, (int64_t)G * kout, kout, id_offset, ws_floor, D, I,
                           floor);
        return hipGetLastError();
    }
    // one wave per query; the lane lists hold 16 entries (what a lane drops beyond that is
    // covered by the floor), the output takes kout rounds of the wave argmin
    hipLaunchKernelGGL((knn_merge_kernel<16, 1>), dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, st,
                       cd, ci, nq, nlists, kin, stride_q, stride_l, stride_l, kout, 1, 0, D, I, floor);
    return hipGetLastError();
}

__global__ void iota64_kernel(int64_t* __restrict__ dst, int64_t n, int64_t start) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = start + i;
}

__global__ void map_labels_kernel(int64_t* __restrict__ I, int64_t n, const int64_t* __restrict__ lmap,
                                  int64_t offset) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && I[i] >= 0) I[i] = lmap[I[i]] + offset;
}

hipError_t launch_iota64(int64_t* dst, int64_t n, int64_t start, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(iota64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, n, start);
    return hipGetLastError();
}

hipError_t launch_map_labels(int64_t* I, int64_t n, const int64_t* lmap, int64_t offset,
                             hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(map_labels_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, I, n,
                       lmap, offset);
    return hipGetLastError();
}

hipError_t launch_fill_empty(float* D, int64_t* I, int64_t n, int metric, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_empty_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, D, I,
                       n, metric);
    return hipGetLastError();
}

}  // namespace imgrec

