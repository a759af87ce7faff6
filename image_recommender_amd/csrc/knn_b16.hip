// knn_b16.hip — 256 x 256-tile bf16 candidate kernel of the k-NN search (gfx950 / MI355X).
//
// Same contract as knn_tile_topk_kernel<..., kModeBF16, ...> (knn_kernels.hip): score every corpus
// row of the workgroup's row split against a block of queries with ONE bf16 MFMA per product
// (v_mfma_f32_32x32x16_bf16, fp32 accumulation) and keep, per (query, list), the KM best
// approximate keys in registers; knn_refine.hip reranks and certifies the merged candidates.  It
// replaces the arithmetic of faiss IndexFlat.search reached from main/search_from_image.py:247.
//
// Why a second kernel: the 128 x 128 tile of the generic kernel stages 2 bytes of LDS-DMA and
// reads 1.25 KiB of LDS per MFMA; at one workgroup per CU a 256 x 256 tile halves the staged bytes
// (2·N·D·Q·(1/BM + 1/BQ)) and a 128-row x 64-query wave tile reads 0.75 KiB per MFMA.
//
// Geometry: 8 waves = 2 (rows) x 4 (queries), wave tile 128 rows x 64 queries = 4 x 2 blocks of
// 32 x 32.  Stage = 64 bf16 of depth per row (128 B): A 256 rows + B 256 queries = 64 KiB, a
// two-slot ring (128 KiB) + row norms, screen bounds and a per-wave park region (150 KiB).  Each
// wave moves 8 one-KiB pieces per stage (waves 0-3 the corpus tile, 4-7 the query tile) with
// global_load_lds_dwordx4 in the saddr form: one per-piece 32-bit lane offset fixed for the
// whole launch, one scalar base per stage, one M0 write per four pieces (instruction offsets).
// Per stage: k-steps 0..2 (fragments of step c+1 read under step c's 8 MFMAs, two reads per MFMA
// gap), wait for the own DMA of the next stage, barrier, read the next stage's first fragments;
// the corpus-tile waves (0-3) then issue the DMA of the stage after it into the slot just read
// while the query-tile waves (4-7, static priority 1) run k-step 3's MFMAs, and the query-tile
// waves issue theirs one k-step later, so each SIMD's MFMA pipe has a feeder during either
// wave's DMA issue.  After a tile's last stage the top-k epilogue runs without barriers (it
// touches no stage memory).
// Measured with per-tile s_memtime stamps (-DIMGREC_B16_STAMPS, tools/b16_stamps.py; profiles/
// r02/b16_stamps.txt) at 1M x 1024 x 1968: a 31-stage tile = ~76k cycles of stage loop (~2450 per
// stage against 2048 of MFMA: the barrier and the corpus-tile waves' DMA issue) + ~14k of
// epilogue (screen ~3.5k, ~12 insertion rounds).

// LDS image: row r of a stage, 16-B chunk c stored at chunk c ^ ((r >> 1) & 7) (two 128-B rows
// per 256-B bank row); the XOR is applied on the DMA's per-lane global source offset, so every
// ds_read_b128 lane group of 16 hits 16 distinct bank slots.
//
// Row splits: the corpus is cut into groups of kRPP rows (one DMA piece each); split s owns the
// global groups s, s + nsplit, s + 2 nsplit, ... and a tile holds kGPT consecutive groups of its
// split.  A stored order that keeps similar rows together (the reference stores images folder by
// folder) is thereby spread over every split, so no split's short list has to hold most of a
// query's neighbours — with contiguous splits the merge floor bound on such corpora and sent a
// quarter of the queries to the exact re-run.  A tile's pieces sit nsplit * kRPP rows apart: the
// per-lane offsets stay fixed, the scalar base moves by kGPT groups per tile.
//
// Accumulator map (v_mfma_f32_32x32x16_bf16): col = lane & 31 -> query, row = (reg & 3) +
// 8 (reg >> 2) + 4 (lane >> 5) -> corpus row: each lane owns two queries (one per query block)
// and 16 rows of each row block, so the top-k needs no data movement.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "knn_kernels.h"

// Stage depth in 32-bit words per staged row (32 = 64 bf16 per row and stage).

namespace imgrec {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kNW = 8;                    // waves: 2 along rows x 4 along queries
constexpr int kBM = kB16BigRows;          // 256 corpus rows per tile
constexpr int kBQ = kB16BigQueries;       // 256 queries per workgroup
constexpr int kBKW = 32;                  // 32-bit words (2 bf16) per staged row
constexpr int kNS = 2;                    // stages in the LDS ring
constexpr int kRowB = kBKW * 4;           // bytes per staged row
constexpr int kCPR = kBKW / 4;            // 16-B chunks per staged row
constexpr int kKS = kCPR / 2;             // 16-deep MFMA k-steps per stage (chunks per lane half)
constexpr int kRPP = 64 / kCPR;           // rows per one-KiB DMA piece
constexpr int kRPB = 64 / kBKW;           // rows per 256-B bank row
constexpr int kGPT = kBM / kRPP;          // row groups (= A pieces) per tile
constexpr int kSA = kBM * kRowB;          // A (corpus) stage bytes
constexpr int kSB = kBQ * kRowB;          // B (query) stage bytes
constexpr int kStage = kSA + kSB;
constexpr int kLPW = (kBM + kBQ) / kRPP / kNW;   // pieces per wave per stage (8 or 4)
constexpr int kNormSlots = 4;             // row-norm ring (tiles)
constexpr int kNormOff = kNS * kStage;
constexpr int kShareOff = kNormOff + kNormSlots * kBM * 4;   // per (wave, query): screen bound
constexpr int kParkOff = kShareOff + kNW * 2 * 32 * 4;     // per wave: 8 accumulators per lane
constexpr int kLDS = kParkOff + kNW * 64 * 8 * 4;
static_assert(kBKW == 32, "stage depth: four 16-deep k-steps per stage");
static_assert(kLDS <= 160 * 1024, "LDS budget");
static_assert(kLPW % 4 == 0, "pieces go out in dma4x groups of four");

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// Four one-KiB LDS-DMA pieces under ONE M0 value: the instruction offset (j KiB) moves both the
// global source and the LDS destination (measured, tools/micro/glds_offset.hip), so the per-lane
// offsets v[j] are pre-reduced by j KiB.
__device__ __forceinline__ void dma4x(const void* sbase, uint32_t lds0, uint32_t v0, uint32_t v1,
                                      uint32_t v2, uint32_t v3) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %5\n\t"
        "global_load_lds_dwordx4 %2, %5 offset:1024\n\t"
        "global_load_lds_dwordx4 %3, %5 offset:2048\n\t"
        "global_load_lds_dwordx4 %4, %5 offset:3072\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0))
        : "memory");
}

// One one-KiB piece (instruction offset OFF, as piece OFF / 1024 of a dma4x group).
template <int OFF>
__device__ __forceinline__ void dma1(const void* sbase, uint32_t lds0, uint32_t v) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 offset:%4\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds0)), "n"(OFF)
        : "memory");
}

// One 4-byte-per-lane LDS-DMA (row norms of a tile).
__device__ __forceinline__ void dma4_norm(const float* g, uint32_t lds) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

__device__ __forceinline__ void barrier_lds() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Ascending register list; labels arrive in increasing order per lane, so an equal key lands
// behind the entries already present (ties by smaller label).  c[p]: d goes before slot p (on the
// old list; monotone in p); slot p takes slot p-1's entry when d goes before p-1, else d when it
// goes before p — on an ascending list that key select is the median of (kd[p-1], d, kd[p]), one
// v_med3.  No control flow: the selects are marked unpredictable so they stay v_cndmask instead
// of exec-mask branches (the branchy form cost ~10 % of the epilogue), and d = +inf is a no-op.
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

// (d1, i1) ranks before (d2, i2): smaller key, ties by smaller label (empty = label -1 last).
__device__ __forceinline__ bool rank_lt(float d1, int i1, float d2, int i2) {
    return i2 < 0 || d1 < d2 || (d1 == d2 && i1 < i2);
}

// Insert into an ascending list when labels arrive in any order (the end-of-kernel folds).
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

}  // namespace

#ifdef IMGREC_B16_STAMPS
// diagnostic build only (tools/b16_stamps.py): s_memtime per wave at fixed points of one tile
__device__ unsigned long long g_b16_stamps[8 * 256];
#define B16_STAMP(slot) do { if (stamp_on && lane == 0) { \
    unsigned long long v_ = __builtin_amdgcn_s_memtime(); g_b16_stamps[wave * 256 + (slot)] = v_; } } while (0)
#else
#define B16_STAMP(slot) do {} while (0)
#endif

template <int KM, int L2>
__global__ void __launch_bounds__(512, 2)
knn_b16_tile_kernel(const uint32_t* __restrict__ xh, const float* __restrict__ xnorm, int nrows,
                    int dw, const uint32_t* __restrict__ qh, const float* __restrict__ qnorm, int nq,
                    int nsplit, int nqb, int64_t id_offset, float* __restrict__ cand_d,
                    int64_t* __restrict__ cand_i, int ncand) {
    __shared__ __attribute__((aligned(16))) char smem[kLDS];

    // XCD-aware bijective block -> (query block, row split) map (as knn_tile_topk_kernel): the
    // query blocks of one row split run on one XCD and share its L2 for the corpus tiles.
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (wg >> 3);
    // G query blocks per row split group on one XCD (G = nqb: all query blocks of a split share
    // its corpus tiles through that XCD's L2; smaller G keeps fewer query blocks per L2)
    constexpr int kG = 4;                   // query blocks per XCD group
    const int G = (nqb % kG == 0) ? kG : nqb;
    const int qbg = wgid / (nsplit * G), rem = wgid - qbg * (nsplit * G);
    const int split = rem / G;
    const int qb = qbg * G + rem % G;
    // this split's rows (header): cnt groups, global group split + m * nsplit for m < cnt, tile t
    // = groups t * kGPT .. + kGPT - 1 of the split (the last tile may hold fewer)
    const int ngroups = (nrows + kRPP - 1) / kRPP;
    const int cnt = split < ngroups ? (ngroups - split + nsplit - 1) / nsplit : 0;
    const int t0 = 0, t1 = (cnt + kGPT - 1) / kGPT;
    // stored row of tile row tr of tile t (groups past the split's end: the tile's first group)
    auto trow = [&](int t, int tr) {
        const int m = t * kGPT + tr / kRPP;
        return (split + (m < cnt ? m : t * kGPT) * nsplit) * kRPP + tr % kRPP;
    };

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave >> 2, wq = wave & 3;
    const int li = lane & 31, lh = lane >> 5;
    int qcol[2];
    qcol[0] = qb * kBQ + wq * 64 + li;
    qcol[1] = qcol[0] + 32;
    float qn[2] = {0.f, 0.f};
    if (L2) { qn[0] = qnorm[qcol[0]]; qn[1] = qnorm[qcol[1]]; }
    asm volatile("" : "+v"(qn[0]), "+v"(qn[1]));   // consume the loads before the DMA stream

    // DMA pieces of this wave: kLPW consecutive pieces of the A tile (waves 0-3) or B tile (4-7);
    // lane -> (row prow of the piece, chunk pchk), source chunk pre-swizzled.
    const bool isA = wave < 4;
    // waves 4-7 (the younger half) lose issue arbitration to 0-3 at every segment start; a static
    // raised priority evens that out (~1 %; per-cluster priority flips measured slower)
    if (!isA) __builtin_amdgcn_s_setprio(1);
    const int pbase = (isA ? wave : wave - 4) * kLPW;          // first piece index in its tile
    const int prow = lane / kCPR, pchk = lane % kCPR;
    // Per-piece lane offsets in bytes from the stage's scalar base (the tile's first row, or the
    // query block), minus the instruction offset dma4x adds to piece j (>= 0: piece j starts at
    // least j KiB in).  Corpus piece P of a tile = the split's group t * kGPT + P.  Pieces are
    // kPS bytes apart and the swizzle of a piece's rows depends only on the piece's parity, so
    // the lane keeps two bases and piece j's offset is vpar[j & 1] + j * kPS - 1024 (j & 3).
    static_assert(kRPP == 8 && kRPB == 2 && kCPR == 8 && kLPW % 2 == 0, "piece offset form");
    uint32_t vpar[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int P = pbase + e, r = P * kRPP + prow;              // r: LDS row of this lane
        const int srow = isA ? P * nsplit * kRPP + prow : r;
        vpar[e] = (uint32_t)srow * (uint32_t)(dw * 4) + 16u * (uint32_t)(pchk ^ ((r / kRPB) % kCPR));
    }
    const uint32_t kPS = (uint32_t)((isA ? nsplit : 1) * kRPP * dw * 4);   // bytes between pieces
    auto voff_of = [&](int j) {
        return vpar[j & 1] + (uint32_t)(j & ~1) * kPS - 1024u * (uint32_t)(j & 3);
    };
    const uint32_t smem0 = lds_u32(smem);
    const uint32_t pdst = (uint32_t)((isA ? 0 : kSA) + pbase * 1024);

    // fragment read offsets (bytes, inside a stage): k-step c of this lane half = logical chunk
    // lh*kKS + c of row li of each 32-row block (the swizzle of row li is the same in every block)
    const int fsw = (li / kRPB) % kCPR;
    int aoff[kKS];
#pragma unroll
    for (int c = 0; c < kKS; ++c) aoff[c] = (wr * 128 + li) * kRowB + 16 * ((lh * kKS + c) ^ fsw);
    const int boff = kSA + (wq * 64 - wr * 128) * kRowB;       // B fragment = A offset + boff

    float kd[2][KM];
    int ki[2][KM];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int p = 0; p < KM; ++p) { kd[h][p] = INFINITY; ki[h][p] = -1; }
    if (lh == 0) {                                              // screen bounds: none yet
        float* share = reinterpret_cast<float*>(smem + kShareOff);
        share[((wr * 4 + wq) * 2) * 32 + li] = INFINITY;
        share[((wr * 4 + wq) * 2 + 1) * 32 + li] = INFINITY;
    }

    const int nst = dw / kBKW;                                  // stages per tile
    const int total = (t1 - t0) * nst;
    const uint32_t* qblk = qh + (size_t)qb * kBQ * dw;

    // DMA of stage g into ring slot g % kNS (+ the tile's row norms with its first stage).  Called
    // for g = 0, 1, 2, ... in order, so the source is a cursor advanced per stage and moved to the
    // next tile's first row once per tile (no per-stage division by the stage count: the scalar
    // address work sits between the barrier and the last k-step's MFMAs).
    int c_it = t0, c_is = 0;
    const uint32_t* c_tile = isA ? xh + (size_t)trow(t0, 0) * dw : qblk;
    int c_ng = (isA && t0 == t1 - 1) ? cnt - t0 * kGPT : kGPT;           // groups in the tile
    auto issue = [&](int g) __attribute__((always_inline)) {
        const uint32_t* src = c_tile + c_is * kBKW;
        const uint32_t dst = smem0 + (uint32_t)((g & (kNS - 1)) * kStage) + pdst;
        if (pbase + kLPW <= c_ng || !isA) {
#pragma unroll
            for (int h = 0; h < kLPW / 4; ++h)
                dma4x(src, dst + 4096u * h, voff_of(4 * h), voff_of(4 * h + 1), voff_of(4 * h + 2),
                      voff_of(4 * h + 3));
        } else {
            // the split's last, partial tile: pieces past its groups are skipped (their LDS rows
            // keep stale data; the epilogue masks those rows)
#pragma unroll
            for (int j = 0; j < kLPW; ++j)
                if (pbase + j < c_ng) {
                    const uint32_t d = dst + 4096u * (j / 4);
                    switch (j & 3) {                            // constant once unrolled
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

    // ---- top-k epilogue of one tile.  Screen: a row can only matter if its key beats T = min(own
    // K-th, the partner lane's K-th, max over the query's four lists of their J-th best) — four
    // lists holding J >= KM/4 entries each at or below that max already give the union KM better
    // entries; a dropped row ranks behind the folded list's last entry (merge floor).  The test
    // runs on the accumulator: d = (|x|^2 (1/2 - 2^-20) + c) - acc with c = (|q|^2 - T)/2 -
    // 2^-20 (|q|^2 + |T|) is negative iff the row passes (the 2^-20 terms keep fp32 rounding from
    // rejecting a row the exact key would keep); two packed adds per pair of rows and one
    // v_alignbit per row shift the sign bits into a 16-bit lane mask.  A lane's passing rows are
    // then visited one per round through the wave's own LDS park region (eight accumulators per
    // lane at a time), keyed and inserted.  Touches no stage memory: needs no barrier of its own.
    constexpr int kJ = (KM + 3) / 4;
    constexpr float kLo = 1.0f / 1048576.f;
    float* const share = reinterpret_cast<float*>(smem + kShareOff);
    float4* const park = reinterpret_cast<float4*>(smem + kParkOff) + wave * (2 * 64);   // own region
    const float* const pk = reinterpret_cast<const float*>(park);

    // fragments of k-step c of a stage (A: 4 row blocks, B: 2 query blocks)
    auto read_frags = [&](const char* sb, int c, u32x4 (&fa)[4], u32x4 (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) fa[rb] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + rb * 32 * kRowB);
#pragma unroll
        for (int h = 0; h < 2; ++h) fb[h] = *reinterpret_cast<const u32x4*>(sb + aoff[c] + boff + h * 32 * kRowB);
    };
    // MFMAs i0 .. i1-1 of a k-step (i = 4 h + rb)
    auto mfma_part = [&](f32x16 (&acc)[4][2], const u32x4 (&fa)[4], const u32x4 (&fb)[2], int i0, int i1) __attribute__((always_inline)) {
#pragma unroll
        for (int i = i0; i < i1; ++i)
            acc[i & 3][i >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf16x8, fa[i & 3]), __builtin_bit_cast(bf16x8, fb[i >> 2]), acc[i & 3][i >> 2], 0, 0, 0);
    };
    auto mfma_step = [&](f32x16 (&acc)[4][2], const u32x4 (&fa)[4], const u32x4 (&fb)[2]) __attribute__((always_inline)) {
        mfma_part(acc, fa, fb, 0, 8);
    };

    u32x4 fa[2][4], fb[2][2];
    int g = 0;
    int pend = -1;                                              // deferred DMA stage
    // ---- main loop.  One barrier per stage, placed before the stage's last k-step: by then every
    // wave has read the whole stage (its slot is refilled with stage g + 2 right after) and waited
    // for its own DMA of stage g + 1, so the next stage's first fragments are read after the
    // barrier while the last k-step's MFMAs run — the MFMA pipe does not drain at the barrier.
    if (total > 0) {
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();
        if (total > 1) issue(1);
        read_frags(smem, 0, fa[0], fb[0]);
    }
    for (int t = t0; t < t1; ++t) {
#ifdef IMGREC_B16_STAMPS
        const bool stamp_on = blockIdx.x == 100 && t - t0 < 120;
#endif
        f32x16 acc[4][2];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[rb][h] = (f32x16){0.f};
        for (int s = 0; s < nst; ++s, ++g) {
            const char* sb = smem + (g & 1) * kStage;
#pragma unroll
            for (int c = 0; c + 1 < kKS; ++c) {
                // the 8 MFMAs with the next k-step's 6 fragment reads placed two per MFMA gap after
                // each of the first three (a third read in one gap saturates the LDS array)
                read_frags(sb, c + 1, fa[(c + 1) & 1], fb[(c + 1) & 1]);
                mfma_step(acc, fa[c & 1], fb[c & 1]);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 5, 0);
                __builtin_amdgcn_sched_barrier(0);
                // the query-tile waves issue their DMA here, one k-step after the corpus-tile
                // waves issued theirs, so each SIMD's other wave keeps the MFMA pipe busy
                if (c == 0 && pend >= 0) {
                    __builtin_amdgcn_sched_barrier(0);
                    issue(pend);
                    pend = -1;
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // (the fences keep the compiler from sinking k-step kKS-2's MFMAs below the wait)
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            barrier_lds();
            __builtin_amdgcn_sched_barrier(0);
            // (after a tile's last stage the next fragments are read after the epilogue instead)
            if (s + 1 < nst) read_frags(smem + ((g + 1) & 1) * kStage, 0, fa[kKS & 1], fb[kKS & 1]);
            if (g + 2 < total) {
                if (isA) issue(g + 2);
                else pend = g + 2;
            }
            mfma_step(acc, fa[(kKS - 1) & 1], fb[(kKS - 1) & 1]);
        }
        // ---- epilogue of tile t (see above)
        B16_STAMP(2 * (t - t0));
#ifdef IMGREC_B16_STAMPS
        int nit = 0;
#endif
        const float* nrm = reinterpret_cast<const float*>(smem + kNormOff + ((t - t0) % kNormSlots) * kBM * 4);
        const bool full = (t + 1) * kGPT <= cnt && trow(t, kBM - 1) < nrows;
        auto row_ok = [&](int tr) { return t * kGPT + tr / kRPP < cnt && trow(t, tr) < nrows; };
        // the other row-half wave's published J-th bounds (read once per tile)
        float other[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            other[h] = share[(((1 - wr) * 4 + wq) * 2 + h) * 32 + li];
        }
        float cth[2];
        auto screen = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float tau = kd[h][KM - 1];
                const float jb = fmaxf(kd[h][kJ - 1], __shfl_xor(kd[h][kJ - 1], 32, 64));
                const float T = fminf(fminf(tau, __shfl_xor(tau, 32, 64)), fmaxf(jb, other[h]));
                const float c = L2 ? 0.5f * (qn[h] - T) - kLo * (qn[h] + fabsf(T)) : -T;
                cth[h] = qcol[h] < nq ? c : INFINITY;
            }
        };
        screen();
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
            // re-tighten after the previous block's insertions (in the first tile the empty lists
            // would otherwise pass every row of all four blocks)
            if (rb > 0) screen();
            const int rbase = wr * 128 + rb * 32 + 4 * lh;      // tile row of accumulator reg 0
            unsigned live = 0xffffu;                            // rows of the block that count
            if (!full) {
                live = 0;
#pragma unroll
                for (int r = 0; r < 16; ++r) live |= (unsigned)row_ok(rbase + (r & 3) + 8 * (r >> 2)) << r;
            }
            unsigned msk[2] = {0u, 0u};
#pragma unroll
            for (int j = 3; j >= 0; --j) {                      // rows 4j+3 .. 4j: high bits first
                float4 n4 = make_float4(0.f, 0.f, 0.f, 0.f);
                if (L2) n4 = *reinterpret_cast<const float4*>(nrm + rbase + 8 * j);
                const f32x2 half2 = (f32x2){0.5f - kLo, 0.5f - kLo};
                const f32x2 hlo = (f32x2){n4.x, n4.y} * half2, hhi = (f32x2){n4.z, n4.w} * half2;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x2 c2 = (f32x2){cth[h], cth[h]};
                    const f32x2 dhi = (L2 ? hhi + c2 : c2) - (f32x2){acc[rb][h][4 * j + 2], acc[rb][h][4 * j + 3]};
                    const f32x2 dlo = (L2 ? hlo + c2 : c2) - (f32x2){acc[rb][h][4 * j], acc[rb][h][4 * j + 1]};
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dhi.y), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dhi.x), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dlo.y), 31);
                    msk[h] = __builtin_amdgcn_alignbit(msk[h], __float_as_uint(dlo.x), 31);
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const unsigned m = msk[h] & live;
                if (!__any(m != 0)) continue;
                auto key_of = [&](float a, int tr) __attribute__((always_inline)) {
                    float kv;
                    if (L2) {
                        kv = fmaf(-2.f, a, qn[h] + nrm[tr]);
                        kv = kv < 0.f ? 0.f : kv;
                    } else {
                        kv = -a;
                    }
                    return kv;
                };
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {                // rows 8hf .. 8hf+7 of the block
                    unsigned mh = (m >> (8 * hf)) & 0xffu;
                    if (!__any(mh != 0)) continue;
                    park[lane] = make_float4(acc[rb][h][8 * hf], acc[rb][h][8 * hf + 1],
                                             acc[rb][h][8 * hf + 2], acc[rb][h][8 * hf + 3]);
                    park[64 + lane] = make_float4(acc[rb][h][8 * hf + 4], acc[rb][h][8 * hf + 5],
                                                  acc[rb][h][8 * hf + 6], acc[rb][h][8 * hf + 7]);
                    while (__any(mh != 0)) {
#ifdef IMGREC_B16_STAMPS
                        ++nit;
#endif
                        // straight-line round: a lane with nothing left inserts +inf (a no-op on
                        // an ascending list), so the round has no divergent branches
                        const bool act = mh != 0u;
                        const int r8 = act ? __builtin_ctz(mh) : 0;
                        mh &= mh - 1u;
                        const float a = pk[((r8 >> 2) * 64 + lane) * 4 + (r8 & 3)];
                        const int r = 8 * hf + r8;
                        const int tr = rbase + (r & 3) + 8 * (r >> 2);
                        float kv = key_of(a, tr);
                        kv = __builtin_unpredictable(act && kv < kd[h][KM - 1]) ? kv : INFINITY;
                        insert_mono<KM>(kd[h], ki[h], kv, trow(t, tr));
                    }
                }
            }
        }
        // publish this wave's J-th bound per query (pair max) for the other row-half wave; a
        // reader sees this or an older (larger) value: both bound the lists
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float jb = fmaxf(kd[h][kJ - 1], __shfl_xor(kd[h][kJ - 1], 32, 64));
            if (lh == 0) share[((wr * 4 + wq) * 2 + h) * 32 + li] = jb;
        }
        B16_STAMP(2 * (t - t0) + 1);
#ifdef IMGREC_B16_STAMPS
        if (stamp_on && lane == 0) g_b16_stamps[wave * 256 + 128 + (t - t0)] = (unsigned long long)nit;
#endif
        if (g < total) read_frags(smem + (g & 1) * kStage, 0, fa[kKS & 1], fb[kKS & 1]);
    }

    // ---- one list per (query, row split): fold the partner lane's list (lane ^ 32, the query's
    // other rows) by shuffles, then wave wr = 1's lists into wave wr = 0's through LDS.  Entries a
    // fold drops rank behind the folded list's last entry, which the merge floor covers.
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            const float od = __shfl_xor(kd[h][p], 32, 64);
            const int oi = __shfl_xor(ki[h][p], 32, 64);
            if (lh == 0 && oi >= 0 && rank_lt(od, oi, kd[h][KM - 1], ki[h][KM - 1]))
                insert_any<KM>(kd[h], ki[h], od, oi);
        }
    }
    float* xd = reinterpret_cast<float*>(smem);                 // [wq][h][li][KM] keys, then labels
    int* xi = reinterpret_cast<int*>(smem) + 4 * 2 * 32 * KM;
    if (wr == 1 && lh == 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int p = 0; p < KM; ++p) {
                xd[((wq * 2 + h) * 32 + li) * KM + p] = kd[h][p];
                xi[((wq * 2 + h) * 32 + li) * KM + p] = ki[h][p];
            }
    }
    __syncthreads();
    if (wr == 1 || lh == 1) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            const float od = xd[((wq * 2 + h) * 32 + li) * KM + p];
            const int oi = xi[((wq * 2 + h) * 32 + li) * KM + p];
            if (oi >= 0 && rank_lt(od, oi, kd[h][KM - 1], ki[h][KM - 1]))
                insert_any<KM>(kd[h], ki[h], od, oi);
        }
        if (qcol[h] >= nq) continue;
        const size_t base = (size_t)qcol[h] * ncand + (size_t)split * KM;
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            cand_d[base + p] = kd[h][p];
            cand_i[base + p] = ki[h][p] < 0 ? (int64_t)-1 : (int64_t)ki[h][p] + id_offset;
        }
    }
}

hipError_t launch_b16_big(const TileArgs& a, hipStream_t st) {
    if (IMGREC_B16_MFMA16) return launch_b16_wide(a, st);
    if (a.wr != 2 || a.wq != 4 || a.dp % kBKW != 0 || a.nsplit < 1) return hipErrorInvalidValue;
    // the lane offsets are 32-bit: a tile's last group sits (kGPT - 1) * nsplit groups past its first
    if (((int64_t)(kGPT - 1) * a.nsplit * kRPP + kBQ) * a.dp * 4 + 8192 >= ((int64_t)1 << 32))
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)(a.nqb * a.nsplit)), block(kNW * 64);
    const uint32_t* xh = reinterpret_cast<const uint32_t*>(a.xb);
    const uint32_t* qh = reinterpret_cast<const uint32_t*>(a.qp);
#define IMGREC_LAUNCH_B16(KMV, L2V)                                                                \
    hipLaunchKernelGGL((knn_b16_tile_kernel<KMV, L2V>), grid, block, 0, st, xh, a.xnorm, a.nrows,  \
                       a.dp, qh, a.qnorm, a.nq, a.nsplit, a.nqb, a.id_offset, a.cand_d,             \
                       a.cand_i, a.ncand)
    if (a.km == 8) {
        if (a.metric == 1) IMGREC_LAUNCH_B16(8, 1); else IMGREC_LAUNCH_B16(8, 0);
    } else if (a.km == 10) {
        if (a.metric == 1) IMGREC_LAUNCH_B16(10, 1); else IMGREC_LAUNCH_B16(10, 0);
    } else {
        return hipErrorInvalidValue;
    }
#undef IMGREC_LAUNCH_B16
    return hipGetLastError();
}

}  // namespace imgrec


#ifdef IMGREC_B16_STAMPS
extern "C" int knn_b16_stamps_read(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(imgrec::g_b16_stamps), sizeof(imgrec::g_b16_stamps));
}
#endif
