// knn_b16w.hip — 256 x 256-tile bf16 candidate kernel on v_mfma_f32_16x16x32_bf16 (gfx950).
//
// Same contract, launch plan, LDS ring and DMA schedule as knn_b16_tile_kernel (knn_b16.hip):
// score every corpus row of the workgroup's row split against a block of 256 queries with one
// bf16 MFMA per product (fp32 accumulation) and keep, per (query, row split), the KM best
// approximate keys; knn_refine.hip reranks and certifies the merged candidates.  It replaces the
// arithmetic of faiss IndexFlat.search reached from main/search_from_image.py:247.
//
// Why a 16 x 16 MFMA form: in a power-limited MFMA loop the chip holds a higher clock on
// v_mfma_f32_16x16x32_bf16 than on v_mfma_f32_32x32x16_bf16 at equal cycles per flop
// (MI355X_MICROARCH.md, DVFS give-back item 7), and the 32 x 32 kernel runs at ~1.67 GHz.
//
// Geometry: 8 waves along the queries; wave w owns queries 32w .. 32w + 31 of the block (two
// 16-query MFMA blocks) against all 256 rows of the tile (sixteen 16-row blocks): 32 MFMAs per
// 32-deep k-step, 128 accumulator registers per lane.  With the 16 x 16 accumulator map (col =
// lane & 15 -> query, row = 4 (lane >> 4) + reg) each lane owns two queries and 64 rows of each,
// so the top-k keeps two register lists per lane as the 32 x 32 kernel does; the four lanes of
// a query (one per lane quarter) hold its four lists, so the screen's shared bound and the final
// fold are wave-local shuffles (no LDS share region, no cross-wave fold).
//
// Stage = 64 bf16 of depth per row (two 32-deep k-steps) for 256 rows + 256 queries, two-slot
// ring, same LDS image and XOR swizzle as knn_b16.hip (row r, 16-B chunk c at c ^ ((r >> 1) & 7)).
// k-step c of lane quarter lq reads logical chunk 4c + lq of row (lane & 15) of a 16-row block:
// the ds_read_b128 lane groups then hit 16 distinct bank slots.  A stage's 64 MFMAs run as 8
// quads (4 row blocks x 2 query blocks each); the next quad's fragments are read under the
// current quad's MFMAs, one read per MFMA gap; the barrier sits before the last quad.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include <type_traits>

#include "knn_kernels.h"
#include "lds_dma.h"

namespace imgrec {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kNW = 8;                    // waves, all along the queries
constexpr int kBM = kB16BigRows;          // 256 corpus rows per tile
constexpr int kBQ = kB16BigQueries;       // 256 queries per workgroup
constexpr int kQW = kBQ / kNW;            // 32 queries per wave
constexpr int kRB = kBM / 16;             // 16-row blocks per tile
constexpr int kBKW = 32;                  // 32-bit words (2 bf16) per staged row
constexpr int kNS = 2;                    // stages in the LDS ring
constexpr int kRowB = kBKW * 4;           // bytes per staged row
constexpr int kCPR = kBKW / 4;            // 16-B chunks per staged row
constexpr int kRPP = 64 / kCPR;           // rows per one-KiB DMA piece
constexpr int kRPB = 64 / kBKW;           // rows per 256-B bank row
constexpr int kGPT = kBM / kRPP;          // row groups (= A pieces) per tile
constexpr int kSA = kBM * kRowB;          // A (corpus) stage bytes
constexpr int kSB = kBQ * kRowB;          // B (query) stage bytes
constexpr int kStage = kSA + kSB;
constexpr int kLPW = (kBM + kBQ) / kRPP / kNW;   // DMA pieces per wave per stage
constexpr int kNormSlots = 4;             // row-norm ring (tiles)
constexpr int kNormOff = kNS * kStage;
constexpr int kParkOff = kNormOff + kNormSlots * kBM * 4;   // per wave: 8 accumulators per lane
constexpr int kLDS = kParkOff + kNW * 64 * 8 * 4;
constexpr int kQuads = 8;                 // MFMA quads per stage (2 k-steps x 4)
// the query-tile waves issue their DMA after this quad of the next stage (the corpus-tile waves
// issue theirs right after the barrier), so each SIMD's other wave feeds the MFMA pipe meanwhile
#ifndef IMGREC_B16W_DEFER_Q
#define IMGREC_B16W_DEFER_Q 3
#endif
constexpr int kDeferQ = IMGREC_B16W_DEFER_Q;
static_assert(kBKW == 32 && kCPR == 8, "stage depth: two 32-deep k-steps per stage");
static_assert(kLDS <= 160 * 1024, "LDS budget");
static_assert(kLPW % 4 == 0, "pieces go out in dma4x groups of four");
static_assert(kDeferQ >= 0 && kDeferQ < kQuads - 1, "deferred DMA inside the stage's first quads");
// Insertion without the LDS park (round 6 default; =0 restores the park for A/B): a passing row's
// accumulator and norm are picked from the registers of its two row blocks by a 3-level
// v_cndmask tree instead of a ds_write / ds_read round trip per row (the norms stay in the
// registers the screen loaded them into).  Bit-identical; cfg2 0.3-1.2 % faster, cfg3 the same
// (profiles/r06/nopark/).
#ifndef IMGREC_B16W_NOPARK
#define IMGREC_B16W_NOPARK 1
#endif
// Measurement builds only (tools/b16w_epi_split.sh; the lists they return are wrong):
// 1 = no per-tile epilogue (the stage loop alone), 2 = the screen without the insertions.  Both
// hand every accumulator (and 2 the screen's masks) to an empty asm at each tile end, so the
// MFMAs and the screen stay live (round 6: without it the compiler dropped every MFMA — PMC
// SQ_INSTS_MFMA = 0, profiles/r06/epi_split/pmc_invalid_variants/).
#ifndef IMGREC_B16W_EPI_EXP
#define IMGREC_B16W_EPI_EXP 0
#endif

// Ascending register list, labels arriving in increasing order per lane: slot p's key is the
// median of (kd[p-1], d, kd[p]); selects stay v_cndmask (no branches); d = +inf is a no-op.
template <int K>
__device__ __forceinline__ void insert_mono(float (&kd)[K], int (&ki)[K], float d, int id) {
    bool c[K];
#pragma unroll
    for (int p = 0; p < K; ++p) c[p] = d < kd[p];
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        kd[p] = __builtin_amdgcn_fmed3f(kd[p - 1], d, kd[p]);
        const int nx = __builtin_unpredictable(c[p]) ? id : ki[p];
        ki[p] = __builtin_unpredictable(c[p - 1]) ? ki[p - 1] : nx;
    }
    kd[0] = __builtin_unpredictable(c[0]) ? d : kd[0];
    ki[0] = __builtin_unpredictable(c[0]) ? id : ki[0];
}

__device__ __forceinline__ bool rank_lt(float d1, int i1, float d2, int i2) {
    return i2 < 0 || d1 < d2 || (d1 == d2 && i1 < i2);
}

template <int K>
__device__ __forceinline__ void insert_any(float (&kd)[K], int (&ki)[K], float d, int id) {
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        const bool shift = rank_lt(d, id, kd[p - 1], ki[p - 1]);
        const bool here = !shift && rank_lt(d, id, kd[p], ki[p]);
        kd[p] = shift ? kd[p - 1] : (here ? d : kd[p]);
        ki[p] = shift ? ki[p - 1] : (here ? id : ki[p]);
    }
    const bool here0 = rank_lt(d, id, kd[0], ki[0]);
    kd[0] = here0 ? d : kd[0];
    ki[0] = here0 ? id : ki[0];
}

// min / max over the four lane quarters of a column (lanes l, l ^ 16, l ^ 32, l ^ 48): a
// v_permlane16_swap then a v_permlane32_swap of the value with itself hands every lane its row
// partner's value in the other output register (no LDS crossbar round trip, unlike ds_bpermute)
__device__ __forceinline__ float quarter_min(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fminf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float quarter_max(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

__device__ __forceinline__ uint32_t quarter_min_u(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    x = min(r[0], r[1]);
    const auto s = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return min(s[0], s[1]);
}
__device__ __forceinline__ uint32_t quarter_max_u(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    x = max(r[0], r[1]);
    const auto s = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return max(s[0], s[1]);
}

// Packed list entries (PACK): the order-preserving bits of the key (ascending floats ->
// ascending u32) with the low ib bits replaced by the split-local row index, so one u32 compare
// orders entries by (key truncated toward -inf, row) and an insertion is one v_med3_u32 per slot.
__device__ __forceinline__ uint32_t ord_bits(float k) {
    const uint32_t u = __float_as_uint(k);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_float(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
// x[r] of eight register values, r in [0, 8) (lane-varying): three levels of v_cndmask
__device__ __forceinline__ float sel8(int r, float x0, float x1, float x2, float x3, float x4, float x5,
                                      float x6, float x7) {
    const bool b0 = r & 1, b1 = r & 2, b2 = r & 4;
    const float a0 = b0 ? x1 : x0, a1 = b0 ? x3 : x2, a2 = b0 ? x5 : x4, a3 = b0 ? x7 : x6;
    const float c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
    return b2 ? c1 : c0;
}
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));          // -> v_med3_u32
}
// ascending packed list, any arrival order (entries are distinct; ~0u = empty, and inserting it
// or anything at or above the last entry changes nothing)
template <int K>
__device__ __forceinline__ void insert_packed(uint32_t (&kp)[K], uint32_t u) {
#pragma unroll
    for (int p = K - 1; p > 0; --p) kp[p] = umed3(kp[p - 1], u, kp[p]);
    kp[0] = min(kp[0], u);
}
// smallest key of the bucket after u's (every key that truncates to u's bucket or below is
// smaller): the screen threshold a packed list entry stands for
__device__ __forceinline__ float bucket_end(uint32_t u, uint32_t lowmask) {
    return u == ~0u ? INFINITY : ord_float((u | lowmask) + 1u);
}

}  // namespace

#ifdef IMGREC_B16_STAMPS
// diagnostic build only (tools/b16_stamps.py): s_memtime per wave at fixed points of one tile
__device__ unsigned long long g_b16w_stamps[8 * 256];
// per workgroup (blockIdx.x < 1024): s_memrealtime (100 MHz) at entry and after its last tile
__device__ unsigned long long g_b16w_wg[2 * 1024];
#define B16W_STAMP(slot) do { if (stamp_on && lane == 0) { \
    unsigned long long v_ = __builtin_amdgcn_s_memtime(); g_b16w_stamps[wave * 256 + (slot)] = v_; } } while (0)
#else
#define B16W_STAMP(slot) do {} while (0)
#endif

// PACK: one u32 per list entry (see ord_bits), ib = index bits (host: every split-local row index
// t * 256 + tile row fits); otherwise separate key / label lists (any corpus size).
template <int KM, int L2, bool PACK>
__global__ void __launch_bounds__(512, 2)
knn_b16w_tile_kernel(const uint32_t* __restrict__ xh, const float* __restrict__ xnorm, int nrows,
                     int dw, const uint32_t* __restrict__ qh, const float* __restrict__ qnorm, int nq,
                     int nsplit, int nqb, int64_t id_offset, float* __restrict__ cand_d,
                     int64_t* __restrict__ cand_i, int ncand, int ib, uint32_t* __restrict__ sync,
                     uint32_t epoch, int lag) {
    __shared__ __attribute__((aligned(16))) char smem[kLDS];

    // XCD-aware bijective block -> (query block, row split) map, as knn_b16_tile_kernel
    const int nwg = gridDim.x, wg = blockIdx.x;
#ifdef IMGREC_B16_STAMPS
    if (threadIdx.x == 0 && wg < 1024) g_b16w_wg[2 * wg] = __builtin_amdgcn_s_memrealtime();
#endif
    const int xcd = wg & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (wg >> 3);
    constexpr int kG = 4;
    const int G = (nqb % kG == 0) ? kG : nqb;
    const int qbg = wgid / (nsplit * G), rem = wgid - qbg * (nsplit * G);
    const int split = rem / G;
    const int qb = qbg * G + rem % G;
    // the G query-block workgroups of this row split: wgids sib0 .. sib0 + G - 1
    const int sib0 = wgid - rem % G;
    bool sync_on = sync != nullptr && G == kG;
    const int ngroups = (nrows + kRPP - 1) / kRPP;
    const int cnt = split < ngroups ? (ngroups - split + nsplit - 1) / nsplit : 0;
    const int t0 = 0, t1 = (cnt + kGPT - 1) / kGPT;
    auto trow = [&](int t, int tr) {
        const int m = t * kGPT + tr / kRPP;
        return (split + (m < cnt ? m : t * kGPT) * nsplit) * kRPP + tr % kRPP;
    };

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lc = lane & 15, lq = lane >> 4;
    int qcol[2];
    qcol[0] = qb * kBQ + wave * kQW + lc;
    qcol[1] = qcol[0] + 16;
    float qn[2] = {0.f, 0.f};
    if (L2) { qn[0] = qnorm[qcol[0]]; qn[1] = qnorm[qcol[1]]; }
    asm volatile("" : "+v"(qn[0]), "+v"(qn[1]));

    // ---- DMA (as knn_b16.hip): waves 0-3 move the corpus tile, 4-7 the query tile
    const bool isA = wave < 4;
    if (!isA) __builtin_amdgcn_s_setprio(1);
    const int pbase = (isA ? wave : wave - 4) * kLPW;
    const int prow = lane / kCPR, pchk = lane % kCPR;
    static_assert(kRPP == 8 && kRPB == 2 && kLPW % 2 == 0, "piece offset form");
    uint32_t vpar[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int P = pbase + e, r = P * kRPP + prow;
        const int srow = isA ? P * nsplit * kRPP + prow : r;
        vpar[e] = (uint32_t)srow * (uint32_t)(dw * 4) + 16u * (uint32_t)(pchk ^ ((r / kRPB) % kCPR));
    }
    const uint32_t kPS = (uint32_t)((isA ? nsplit : 1) * kRPP * dw * 4);
    auto voff_of = [&](int j) {
        return vpar[j & 1] + (uint32_t)(j & ~1) * kPS - 1024u * (uint32_t)(j & 3);
    };
    const uint32_t smem0 = lds_u32(smem);
    const uint32_t pdst = (uint32_t)((isA ? 0 : kSA) + pbase * 1024);

    // fragment read offsets: k-step c of lane quarter lq = logical chunk 4c + lq of row lc of a
    // 16-row block (the swizzle of row lc is the same in every block: (lc >> 1) & 7)
    const int fsw = (lc / kRPB) % kCPR;
    int aoff[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) aoff[c] = lc * kRowB + 16 * ((4 * c + lq) ^ fsw);
    const int boff = kSA + wave * kQW * kRowB;

    float kd[2][KM];
    int ki[2][KM];
    uint32_t kp[2][KM];
    const uint32_t lowm = PACK ? (1u << ib) - 1u : 0u;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            if constexpr (PACK) kp[h][p] = ~0u;
            else { kd[h][p] = INFINITY; ki[h][p] = -1; }
        }

    const int nst = dw / kBKW;
    const int total = (t1 - t0) * nst;
    const uint32_t* qblk = qh + (size_t)qb * kBQ * dw;

    int c_it = t0, c_is = 0;
    const uint32_t* c_tile = isA ? xh + (size_t)trow(t0, 0) * dw : qblk;
    int c_ng = (isA && t0 == t1 - 1) ? cnt - t0 * kGPT : kGPT;
    auto issue = [&](int g) __attribute__((always_inline)) {
        const uint32_t* src = c_tile + c_is * kBKW;
        const uint32_t dst = smem0 + (uint32_t)((g & (kNS - 1)) * kStage) + pdst;
        if (pbase + kLPW <= c_ng || !isA) {
#pragma unroll
            for (int h = 0; h < kLPW / 4; ++h)
                dma4x(src, dst + 4096u * h, voff_of(4 * h), voff_of(4 * h + 1), voff_of(4 * h + 2),
                      voff_of(4 * h + 3));
        } else {
            // the split's last, partial tile: pieces past its groups are skipped
#pragma unroll
            for (int j = 0; j < kLPW; ++j)
                if (pbase + j < c_ng) {
                    const uint32_t d = dst + 4096u * (j / 4);
                    switch (j & 3) {
                        case 0: dma1<0>(src, d, voff_of(j)); break;
                        case 1: dma1<1024>(src, d, voff_of(j)); break;
                        case 2: dma1<2048>(src, d, voff_of(j)); break;
                        default: dma1<3072>(src, d, voff_of(j)); break;
                    }
                }
        }
        if (c_is == 0 && wave < 4)
            dma4_norm(xnorm + trow(c_it, wave * 64 + lane),
                      smem0 + (uint32_t)(kNormOff + ((c_it - t0) & (kNormSlots - 1)) * kBM * 4 + wave * 256));
        if (++c_is == nst) {
            c_is = 0;
            ++c_it;
            if (isA) {
                c_tile = xh + (size_t)trow(c_it, 0) * dw;
                c_ng = c_it == t1 - 1 ? cnt - c_it * kGPT : kGPT;
            }
        }
    };
    static_assert(kNS == 2 && kNormSlots == 4, "power-of-two ring slots");

    constexpr int kJ = (KM + 3) / 4;
    constexpr float kLo = 1.0f / 1048576.f;
    float4* const park = reinterpret_cast<float4*>(smem + kParkOff) + wave * (2 * 64);
    const float* const pk = reinterpret_cast<const float*>(park);

    // quad q of a stage: k-step q >> 2, row blocks 4 (q & 3) .. + 3
    auto read_a = [&](const char* sb, int q, u32x4 (&fa)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            fa[j] = *reinterpret_cast<const u32x4*>(sb + aoff[q >> 2] + (4 * (q & 3) + j) * 16 * kRowB);
    };
    auto read_b = [&](const char* sb, int c, u32x4 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < 2; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + boff + h * 16 * kRowB);
    };
    auto mfma_quad = [&](f32x4 (&acc)[kRB][2], const u32x4 (&fa)[4], const u32x4 (&fb)[2], int q) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                acc[4 * (q & 3) + j][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    __builtin_bit_cast(bf16x8, fa[j]), __builtin_bit_cast(bf16x8, fb[h]), acc[4 * (q & 3) + j][h], 0, 0, 0);
    };

    u32x4 fa[2][4], fb[2][2];
    int g = 0;
    int pend = -1;
    if (total > 0) {
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        if (total > 1) issue(1);
        read_a(smem, 0, fa[0]);
        read_b(smem, 0, fb[0]);
    }
    for (int t = t0; t < t1; ++t) {
#ifdef IMGREC_B16_STAMPS
        const bool stamp_on = blockIdx.x == 100 && t - t0 < 120;
        int nit = 0;
        unsigned long long ins_cyc = 0;      // cycles inside the insertion blocks of this tile
#endif
        f32x4 acc[kRB][2];
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[rb][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
        // live quad rows (64 tile rows each) of this tile: a split's partial last tile runs the
        // MFMAs, fragment reads and screens of its live row blocks only
        const int nlive = (t + 1) * kGPT <= cnt ? 4 : (((cnt - t * kGPT) * kRPP + 63) >> 6);
        // one tile's stages with NR live quad rows: per stage 2 k-steps x NR quads, quad i =
        // (k-step i / NR, quad row i % NR); the next quad's fragments are read under the current
        // one's MFMAs (the second k-step's B fragments under the first k-step's last quad); the
        // barrier sits before the last quad, after which the next stage's first fragments are
        // read and the corpus-tile waves issue the DMA of the stage after it
        auto stage_loop = [&](auto nr_tag) __attribute__((always_inline)) {
            constexpr int NR = decltype(nr_tag)::value, L = 2 * NR;
            for (int s = 0; s < nst; ++s, ++g) {
                const char* sb = smem + (g & 1) * kStage;
#pragma unroll
                for (int i = 0; i + 1 < L; ++i) {
                    read_a(sb, 4 * ((i + 1) / NR) + (i + 1) % NR, fa[(i + 1) & 1]);
                    if (i == NR - 1) read_b(sb, 1, fb[1]);
                    mfma_quad(acc, fa[i & 1], fb[i / NR], 4 * (i / NR) + i % NR);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
                    }
                    if (i == NR - 1) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    } else {
                        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (i == (kDeferQ < L - 2 ? kDeferQ : L - 2) && pend >= 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        issue(pend);
                        pend = -1;
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                barrier_lds();
                __builtin_amdgcn_sched_barrier(0);
                if (s + 1 < nst) {
                    const char* nb = smem + ((g + 1) & 1) * kStage;
                    read_a(nb, 0, fa[0]);
                    read_b(nb, 0, fb[0]);
                }
                if (g + 2 < total) {
                    if (isA) issue(g + 2);
                    else pend = g + 2;
                }
                mfma_quad(acc, fa[1], fb[1], 4 + NR - 1);
            }
        };
        if (nlive >= 4) stage_loop(std::integral_constant<int, 4>{});
        else if (nlive == 3) stage_loop(std::integral_constant<int, 3>{});
        else if (nlive == 2) stage_loop(std::integral_constant<int, 2>{});
        else stage_loop(std::integral_constant<int, 1>{});

        // ---- top-k epilogue of tile t.  Screen: a row matters only if its key beats T = min(the
        // K-th of any of the query's four lane lists, max over them of their J-th best) — four
        // lists holding J >= KM/4 entries each at or below that max give the union KM better
        // entries, and a dropped row ranks behind the folded list's last entry (merge floor).
        // The test runs on the accumulator (see knn_b16.hip): d = (|x|^2 (1/2 - 2^-20) + c) - acc
        // with c = (|q|^2 - T)/2 - 2^-20 (|q|^2 + |T|) is negative iff the row passes.
        B16W_STAMP(2 * (t - t0));
#if IMGREC_B16W_EPI_EXP != 0
#pragma unroll
        for (int rb = 0; rb < kRB; ++rb)
#pragma unroll
            for (int h = 0; h < 2; ++h) asm volatile("" :: "v"(acc[rb][h]));
#endif
        const float* nrm = reinterpret_cast<const float*>(smem + kNormOff + ((t - t0) % kNormSlots) * kBM * 4);
        const bool full = (t + 1) * kGPT <= cnt && trow(t, kBM - 1) < nrows;
        auto row_ok = [&](int tr) { return t * kGPT + tr / kRPP < cnt && trow(t, tr) < nrows; };
        float cth[2];
        auto screen = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float T;
                if constexpr (PACK) T = bucket_end(min(quarter_min_u(kp[h][KM - 1]), quarter_max_u(kp[h][kJ - 1])), lowm);
                else T = fminf(quarter_min(kd[h][KM - 1]), quarter_max(kd[h][kJ - 1]));
                const float c = L2 ? 0.5f * (qn[h] - T) - kLo * (qn[h] + fabsf(T)) : -T;
                cth[h] = qcol[h] < nq ? c : INFINITY;
            }
        };
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            if (rg >= nlive || IMGREC_B16W_EPI_EXP == 1) break;
            // row group rg = row blocks 4 rg .. 4 rg + 3; bit 4 j + i of a mask = accumulator
            // register i of row block 4 rg + j = tile row (4 rg + j) * 16 + 4 lq + i
            screen();
            unsigned live = 0xffffu;
            if (!full) {
                live = 0;
#pragma unroll
                for (int b = 0; b < 16; ++b) live |= (unsigned)row_ok((4 * rg + (b >> 2)) * 16 + 4 * lq + (b & 3)) << b;
            }
            unsigned msk[2] = {0u, 0u};
            float4 nr4[4];                                      // the group's row norms
#pragma unroll
            for (int j = 3; j >= 0; --j) {                      // high bits first
                const int rb = 4 * rg + j;
                float4 n4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (L2) n4 = *reinterpret_cast<const float4*>(nrm + rb * 16 + 4 * lq);
                nr4[j] = n4;
                const f32x2 half2 = (f32x2){0.5f - kLo, 0.5f - kLo};
                const f32x2 hlo = (f32x2){n4.x, n4.y} * half2, hhi = (f32x2){n4.z, n4.w} * half2;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x2 c2 = (f32x2){cth[h], cth[h]};
                    const f32x2 dhi = (L2 ? hhi + c2 : c2) - (f32x2){acc[rb][h][2], acc[rb][h][3]};
                    const f32x2 dlo = (L2 ? hlo + c2 : c2) - (f32x2){acc[rb][h][0], acc[rb][h][1]};
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dhi.y), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dhi.x), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dlo.y), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dlo.x), 31);
                }
            }
#ifdef IMGREC_B16_STAMPS
            const unsigned long long ins0 = __builtin_amdgcn_s_memtime();
#endif
#if IMGREC_B16W_EPI_EXP == 2
            asm volatile("" :: "v"(msk[0] & live), "v"(msk[1] & live));   // the screen, no insertion
            continue;
#endif
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const unsigned m = msk[h] & live;
                if (!__any(m != 0)) continue;
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {                // row blocks 4 rg + 2 hf, + 1
                    unsigned mh = (m >> (8 * hf)) & 0xffu;
                    if (!__any(mh != 0)) continue;
                    const int rb0 = 4 * rg + 2 * hf;
#if !IMGREC_B16W_NOPARK
                    park[lane] = make_float4(acc[rb0][h][0], acc[rb0][h][1], acc[rb0][h][2], acc[rb0][h][3]);
                    park[64 + lane] = make_float4(acc[rb0 + 1][h][0], acc[rb0 + 1][h][1],
                                                  acc[rb0 + 1][h][2], acc[rb0 + 1][h][3]);
#endif
                    while (__any(mh != 0)) {
#ifdef IMGREC_B16_STAMPS
                        ++nit;
#endif
                        const bool act = mh != 0u;
                        const int r8 = act ? __builtin_ctz(mh) : 0;
                        mh &= mh - 1u;
                        const int tr = (rb0 + (r8 >> 2)) * 16 + 4 * lq + (r8 & 3);
#if IMGREC_B16W_NOPARK
                        const float a = sel8(r8, acc[rb0][h][0], acc[rb0][h][1], acc[rb0][h][2], acc[rb0][h][3],
                                             acc[rb0 + 1][h][0], acc[rb0 + 1][h][1], acc[rb0 + 1][h][2],
                                             acc[rb0 + 1][h][3]);
                        const float4 na = nr4[2 * hf], nb = nr4[2 * hf + 1];
                        const float xn = L2 ? sel8(r8, na.x, na.y, na.z, na.w, nb.x, nb.y, nb.z, nb.w) : 0.f;
#else
                        const float a = pk[((r8 >> 2) * 64 + lane) * 4 + (r8 & 3)];
                        const float xn = L2 ? nrm[tr] : 0.f;
#endif
                        float kv = L2 ? fmaf(-2.f, a, qn[h] + xn) : -a;
                        if constexpr (PACK) {
                            // L2: the clamp at 0 and the order map in two integer ops — a key
                            // with the sign bit set (negative or -0) maps to ord(+0) = 2^31, a
                            // non-negative one to its bits | 2^31
                            const uint32_t ob = L2 ? ((uint32_t)max((int)__float_as_uint(kv), 0) | 0x80000000u)
                                                   : ord_bits(kv);
                            const uint32_t u = (ob & ~lowm) | (uint32_t)(t * kBM + tr);
                            insert_packed<KM>(kp[h], __builtin_unpredictable(act) ? u : ~0u);
                        } else {
                            if (L2) kv = kv < 0.f ? 0.f : kv;
                            kv = __builtin_unpredictable(act && kv < kd[h][KM - 1]) ? kv : INFINITY;
                            insert_mono<KM>(kd[h], ki[h], kv, trow(t, tr));
                        }
                    }
                }
            }
#ifdef IMGREC_B16_STAMPS
            ins_cyc += __builtin_amdgcn_s_memtime() - ins0;
#endif
        }
        B16W_STAMP(2 * (t - t0) + 1);
        // sibling lockstep (TileArgs::sync): publish this tile, wait (bounded) until the G
        // workgroups of this row split have all finished it (minus the lag), so they enter the
        // next tile together and its corpus stages are fetched from HBM once, then served from
        // L2 to the other three.  Only lane 0 of wave 0 waits; the other waves run on into the
        // next tile and stop at its first stage barrier.  A sibling that never shows up (not
        // resident) turns the wait off for the rest of the launch.
        if (sync_on && wave == 0 && t + 1 < t1) {
            if (lane == 0) {
                const uint32_t mine = (epoch << 16) + (uint32_t)(t - t0) + 1u;
                __hip_atomic_store(sync + wgid, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t want = mine - (uint32_t)lag;
                for (int spin = 0;; ++spin) {
                    bool ok = true;
#pragma unroll
                    for (int s2 = 0; s2 < kG; ++s2)
                        ok = ok && (int)(__hip_atomic_load(sync + sib0 + s2, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) - want) >= 0;
                    if (ok) break;
                    if (spin >= 4096) { sync_on = false; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        }
#ifdef IMGREC_B16_STAMPS
        if (stamp_on && lane == 0) g_b16w_stamps[wave * 256 + 128 + (t - t0)] = (unsigned long long)nit;
        if (stamp_on && lane == 0 && t - t0 < 64) g_b16w_stamps[wave * 256 + 192 + (t - t0)] = ins_cyc;
#endif
        if (g < total) {
            read_a(smem + (g & 1) * kStage, 0, fa[0]);
            read_b(smem + (g & 1) * kStage, 0, fb[0]);
        }
    }

#ifdef IMGREC_B16_STAMPS
    if (threadIdx.x == 0 && wg < 1024) g_b16w_wg[2 * wg + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    // ---- one list per (query, row split): fold lane quarters 2, 3 into 0, 1 (lane ^ 32), then
    // quarter 1 into 0 (lane ^ 16).  Entries a fold drops rank behind the folded list's last
    // entry, which the merge floor covers.
#pragma unroll
    for (int x = 32; x >= 16; x >>= 1) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (PACK) {
                // every lane merges its partner's list as it was before the fold (both lists
                // change in this step; a list must not take an entry it already holds)
                uint32_t o[KM];
#pragma unroll
                for (int p = 0; p < KM; ++p) o[p] = (uint32_t)__shfl_xor((int)kp[h][p], x, 64);
#pragma unroll
                for (int p = 0; p < KM; ++p) insert_packed<KM>(kp[h], o[p]);
                continue;
            }
#pragma unroll
            for (int p = 0; p < KM; ++p) {
                const float od = __shfl_xor(kd[h][p], x, 64);
                const int oi = __shfl_xor(ki[h][p], x, 64);
                if (lq < x / 16 && oi >= 0 && rank_lt(od, oi, kd[h][KM - 1], ki[h][KM - 1]))
                    insert_any<KM>(kd[h], ki[h], od, oi);
            }
        }
    }
    if (lq != 0) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (qcol[h] >= nq) continue;
        const size_t base = (size_t)qcol[h] * ncand + (size_t)split * KM;
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            if constexpr (PACK) {
                // key truncated toward -inf (a lower bound of the approximate key: the rerank
                // adds the truncation to its bounds, RerankArgs::c_trunc); split-local row ->
                // stored row
                const uint32_t u = kp[h][p];
                const int j = (int)(u & lowm);
                cand_d[base + p] = u == ~0u ? INFINITY : ord_float(u & ~lowm);
                cand_i[base + p] = u == ~0u ? (int64_t)-1
                                            : (int64_t)((split + (j >> 3) * nsplit) * kRPP + (j & 7)) + id_offset;
            } else {
                cand_d[base + p] = kd[h][p];
                cand_i[base + p] = ki[h][p] < 0 ? (int64_t)-1 : (int64_t)ki[h][p] + id_offset;
            }
        }
    }
}

hipError_t launch_b16_wide(const TileArgs& a, hipStream_t st) {
    if (a.wr != 2 || a.wq != 4 || a.dp % kBKW != 0 || a.nsplit < 1) return hipErrorInvalidValue;
    if (((int64_t)(kGPT - 1) * a.nsplit * kRPP + kBQ) * a.dp * 4 + 8192 >= ((int64_t)1 << 32))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)(a.nqb * a.nsplit)), block(kNW * 64);
    const uint32_t* xh = reinterpret_cast<const uint32_t*>(a.xb);
    const uint32_t* qh = reinterpret_cast<const uint32_t*>(a.qp);
    if (a.ib < 0 || a.ib > kB16PackMaxIB) return hipErrorInvalidValue;
#define IMGREC_LAUNCH_B16W(KMV, L2V, PK)                                                             \
    hipLaunchKernelGGL((knn_b16w_tile_kernel<KMV, L2V, PK>), grid, block, 0, st, xh, a.xnorm,      \
                       a.nrows, a.dp, qh, a.qnorm, a.nq, a.nsplit, a.nqb, a.id_offset, a.cand_d,   \
                       a.cand_i, a.ncand, a.ib, a.sync, a.epoch, a.sync_lag)
#define IMGREC_LAUNCH_B16W_K(KMV, PK)                                                               \
    do { if (a.metric == 1) IMGREC_LAUNCH_B16W(KMV, 1, PK); else IMGREC_LAUNCH_B16W(KMV, 0, PK); } while (0)
    if (a.km == 8) {
        if (a.ib > 0) IMGREC_LAUNCH_B16W_K(8, true); else IMGREC_LAUNCH_B16W_K(8, false);
    } else if (a.km == 10) {
        if (a.ib > 0) IMGREC_LAUNCH_B16W_K(10, true); else IMGREC_LAUNCH_B16W_K(10, false);
    } else {
        return hipErrorInvalidValue;
    }
#undef IMGREC_LAUNCH_B16W_K
#undef IMGREC_LAUNCH_B16W
    return hipGetLastError();
}

}  // namespace imgrec


#ifdef IMGREC_B16_STAMPS
extern "C" int knn_b16w_stamps_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_b16w_stamps), sizeof(imgrec::g_b16w_stamps));
}
extern "C" int knn_b16w_wg_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_b16w_wg), sizeof(imgrec::g_b16w_wg));
}
#endif
