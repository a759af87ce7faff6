// knn_kernels.h — internal launch interface between the C ABI (knn_capi.cpp) and the gfx950
// kernels (knn_kernels.hip).  Not part of the public ABI (see include/imgrec_knn.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace imgrec {

// Arithmetic of the fused distance + top-k kernel.
constexpr int kModeF32 = 0;     // exact fp32 rows, v_mfma_f32_32x32x2_f32
constexpr int kModeSplit = 1;   // split-bf16 rows (hi, lo), three bf16 MFMAs per product
constexpr int kModeBF16 = 2;    // bf16 rows, one bf16 MFMA per product (candidate pass)
constexpr int kModeI8 = 3;      // block-scaled int8 rows, fp32 VALU dot (small-batch candidate pass)

// Arguments of one fused distance + top-k launch.
struct TileArgs {
    int wr, wq, km;             // waves along rows / queries, register list length
    int wb = 4;                 // 32-row MFMA blocks per wave (rows per wave = 32*wb)
    int sbk = 0;                // split path: staging depth the split copy is laid out for
    int mode = kModeF32;        // kMode*: layout of xb / qp and the MFMA form
    const float* xb;            // corpus, nrows_cap x dp 32-bit words (rows padded to 256)
    const float* xnorm;         // |x|^2 per stored row
    int nrows, dp;              // dp = row stride in 32-bit words (bf16 rows: elements / 2)
    const float* qp;            // queries, nq_pad x dp
    const float* qnorm;         // |q|^2 per padded query
    int nq;
    int metric;                 // 1 = L2, otherwise inner product
    int ntiles, nsplit, nqb;
    int64_t id_offset;
    float* cand_d;              // nq x ncand keys
    int64_t* cand_i;            // nq x ncand labels
    int ncand;
    int ib = 0;                 // 256 x 256 bf16 kernel: > 0 = packed lists with ib index bits
    // 256 x 256 bf16 kernel, optional: per-workgroup tile progress (one uint32 per workgroup,
    // values (epoch << 16) + tiles done), so the query-block workgroups that share a row split
    // start every tile together and read its corpus stages from L2 once (NULL = off)
    uint32_t* sync = nullptr;
    uint32_t epoch = 0;
    int sync_lag = 0;           // tiles a workgroup may run ahead of its slowest sibling
};

// One rerank + certificate launch over merged candidate-pass candidates (knn_refine.hip).
constexpr int kRerankWavesHost = 8;     // the rerank workgroup's waves (knn_certify.h kRerankWaves)

struct RerankArgs {
    int mode;                   // kModeSplit, kModeBF16 or kModeI8: which error bound certifies
    const float* qp;            // fp32 padded queries, nq x dp
    const float* qnorm;
    int dp;
    const float* xb;            // fp32 corpus
    const float* xn;
    const float* xn_max;        // device scalar: max stored |x|^2
    int64_t id_offset;
    float* cd;                  // nq x kc approximate keys, ascending (written here when l1_G > 0)
    int64_t* ci;                // nq x kc labels (id_offset applied), -1 = empty
    int kc;
    int64_t nq;
    int k, metric;              // metric 1 = L2, otherwise inner product
    float c_trunc = 0.f;        // candidate keys truncated toward -inf by at most c_trunc |key|
                                // (the packed-list candidate kernel); 0 = exact approximate keys
    float c_split, c_fp;        // relative error-bound coefficients (see knn_capi.cpp); for
                                // kModeBF16 c_split is the MFMA accumulation coefficient
    const float* q_resid;       // kModeBF16: |q - bf16(q)| per query (kModeI8: NULL, fp32 query)
    const float* xr_max;        // kModeBF16: device scalar, max over rows of |x - bf16(x)|;
                                // kModeI8: max over rows of |x - s c| (the int8 copy's residual)
    float* floor;               // per query: smallest key any row outside the candidates can
                                // have besides the K'-th candidate's (merge "floor"), or NULL
    // the candidate merge's second level fused into the rerank (launch_merge_candidates with
    // defer_level2; small batches): per query l1_G lists of 16 (key, label) at l1_d / l1_i +
    // q * l1_G * 16 and their floors at l1_floor + q * l1_G; wave 0 selects the kc best and writes
    // them to cd / ci and the floor to floor (the second chance reads them).  0 = cd / ci / floor
    // are the inputs.
    const float* l1_d = nullptr;
    const int64_t* l1_i = nullptr;
    const float* l1_floor = nullptr;
    int l1_G = 0;
    // l0_lists > 0: the merge's first level fused as well — the raw_lists (= l0_lists <= 64 x
    // kRerankWaves) per-split lists of 16 are selected by the rerank's waves (one group of 64 lists
    // a wave, l1_G = groups); no merge launch at all
    int l0_lists = 0;
    // s_lists > 0: ONE merge level, in this kernel — the raw_lists (= s_lists <= 64) per-split
    // lists of raw_km <= 16 entries are selected by the whole workgroup (large batches' single
    // level; no merge launch)
    int s_lists = 0;
    int nw = 0;                 // rerank workgroup waves: 0 = kRerankWaves (8), 4 = large batches
    int p1 = 0;                 // first-phase rerank size (0 = kRerankWaves x kRerankRows = 16);
                                // large batches use k: their rerank is bound by row bytes
    int chance_skip = 0;        // queue a query whose band certainly-ish exceeds K' straight to the
                                // second chance (no first-pass row reads); needs raw_d
    int direct = 0;             // no merge and no rerank launch: the certificate tail gives EVERY
                                // query (item i = query i) the second chance, its prefix limit from
                                // the raw lists' first keys at heads + q * raw_lists (I8Args::heads;
                                // cd / ci / floor / chance_list unused)
    const float* heads = nullptr;
    int heads_n = 0;            // first keys per query at heads (raw_lists when 0)
    float* D;
    int64_t* I;
    int* stats;                 // this chunk's device counters (zero on entry): [0] queries left
                                // for the exact re-run, [1] max observed error / bound (float
                                // bits, atomicMax), [2] queries whose first certificate failed,
                                // [3] of those, queued for the second chance
    int* fail_list;             // nq entries: the queries left for the exact re-run
    int* chance_list = nullptr; // nq entries: the second-chance queue (raw_d set)
    // the candidate pass's raw per-split lists (second chance; NULL = none): raw_lists sorted
    // lists of raw_km entries per query, query q's at q * raw_stride_q (global labels, -1 empty)
    const float* raw_d = nullptr;
    const int64_t* raw_i = nullptr;
    int raw_lists = 0, raw_km = 0;
    int64_t raw_stride_q = 0;
    int* tail_ctl = nullptr;    // the certificate tail's grid-barrier counters (zeroed by the rerank)
    // second chance in slices (cert_tail_kernel): item i's raw lists are cut into sc_slices
    // slices reranked by different workgroups; per slice its k best (key, label) at
    // sc_key / sc_lab[(i * sc_slices + s) * k] and (floor bits, error ratio bits, overflow) at
    // sc_meta[(i * sc_slices + s) * 4]; per item the completed-slice count (reset by the item's
    // last slice; allocated zero)
    int sc_slices = 1;
    float* sc_key = nullptr;
    int64_t* sc_lab = nullptr;
    unsigned* sc_meta = nullptr;
    int* sc_done = nullptr;
};

// The certificate tail of a candidate chunk (knn_kernels.hip cert_tail_kernel), ONE launch after
// the rerank: the second chance over the raw per-split lists, the stats fold, and the exact fp32
// re-run of the queries neither certificate settled (query gather, the (2,1) exact tile over a
// device-planned set of (query block, row split) items, and the per-query-block merge scattered
// into D / I).  With no query queued (the common case) it folds the stats and exits.
struct TailArgs {
    RerankArgs r;               // the rerank's arguments (second chance; stats, lists, D, I)
    int parity, first;          // this chunk's stats parity; first chunk of the search
    int* stat;                  // 12 ints: two chunk parities + the search accumulators
    const float* qpad;          // the chunk's padded fp32 queries and norms (re-run input)
    const float* qnorm;
    int dp, nrows, ntiles, metric;
    const float* xb;            // fp32 corpus + norms
    const float* xn;
    int64_t id_offset;
    float* fq;                  // gathered re-run queries (cap_rows x dp) and norms
    float* fqn;
    float* fcd;                 // re-run candidate lists
    int64_t* fci;
    int* ticket;                // per query block: row splits done (zeroed in the kernel)
    int km, lists_km;           // list length, lists per row split x km
};

constexpr int kTileRowsMax = 256;   // corpus capacity is rounded to this many rows
constexpr int kDepthPad = 16;       // row stride is rounded to this many floats

// Split-path tile: (1,4) workgroups of kSplitWB-block waves, kSplitBK-word stages, kSplitNS ring.
#ifndef IMGREC_SPLIT_BK
#define IMGREC_SPLIT_BK 32
#endif
#ifndef IMGREC_SPLIT_NS
#define IMGREC_SPLIT_NS 2
#endif
#ifndef IMGREC_SPLIT_WB
#define IMGREC_SPLIT_WB 4
#endif
constexpr int kSplitBK = IMGREC_SPLIT_BK, kSplitNS = IMGREC_SPLIT_NS, kSplitWB = IMGREC_SPLIT_WB;

// bf16 candidate-pass tile: (kB16WR, kB16WQ) workgroups of kB16WB-block waves, 64-deep stages
// (32 words), kB16NS ring, kB16WGPCU workgroups per CU; rows of the bf16 copy padded to
// kB16Pad elements.
#ifndef IMGREC_B16_WR
#define IMGREC_B16_WR 1
#endif
#ifndef IMGREC_B16_WQ
#define IMGREC_B16_WQ 4
#endif
#ifndef IMGREC_B16_WB
#define IMGREC_B16_WB 4
#endif
#ifndef IMGREC_B16_NS
#define IMGREC_B16_NS 2
#endif
#ifndef IMGREC_B16_WGPCU
#define IMGREC_B16_WGPCU 2
#endif
constexpr int kB16WR = IMGREC_B16_WR, kB16WQ = IMGREC_B16_WQ, kB16WB = IMGREC_B16_WB;
constexpr int kB16NS = IMGREC_B16_NS, kB16WGPCU = IMGREC_B16_WGPCU, kB16Pad = 64;

// 256 x 256-tile bf16 kernel (knn_b16.hip): one 8-wave workgroup per CU, k <= 10, batches of at
// least kB16BigMinQ queries.
#ifndef IMGREC_B16_BIG_MINQ
#define IMGREC_B16_BIG_MINQ 512
#endif
#ifndef IMGREC_B16_MFMA16
#define IMGREC_B16_MFMA16 1
#endif
// packed candidate lists (knn_b16w.hip) while a split's row index fits this many bits: the
// approximate keys keep 23 - ib mantissa bits (relative truncation <= 2^(ib - 23))
#ifndef IMGREC_B16_PACK_MAXIB
#define IMGREC_B16_PACK_MAXIB 14
#endif
constexpr int kB16PackMaxIB = IMGREC_B16_PACK_MAXIB;
constexpr int kB16BigRows = 256, kB16BigQueries = 256, kB16BigMinQ = IMGREC_B16_BIG_MINQ;

// Small-batch candidate pass on the block-scaled int8 copy (knn_i8.hip): per (query, row split)
// the km best approximate keys, nq <= 8 queries in one launch, nsplit workgroups.
struct I8Args {
    const int8_t* codes;        // cap x nblk*64 codes
    const float* scales;        // cap x nblk block scales
    const float* xnorm;         // |x|^2 per stored row (exact)
    int nrows, nblk;
    const int8_t* qcodes;       // nq x nblk x (64 hi | 64 lo) two-level query codes
    const float* qscales;       // nq x nblk x (s_hi, s_lo)
    const float* qnorm;
    int nq, km, nsplit, l2;
    int64_t id_offset;
    float* cand_d;              // nq x ncand keys, one sorted list of km per split
    int64_t* cand_i;
    int ncand;
    // Fused query prep (qsrc non-NULL; qcodes / qscales / qnorm unused): the raw query rows (nq x
    // d); the scan quantises them itself and workgroup 0 writes what launch_i8_query_prep would
    // for the rerank: the padded fp32 rows (nq x dp, L2-normalised when `normalize`), |q|^2 and
    // |q - q~|.  (The codes themselves are consumed by the scan only.)
    const float* qsrc;
    int d, dp, normalize;
    float* qpad;
    float* qnorm_out;
    float* qresid;
    // non-NULL: workgroup 0 zeroes these 4 ints (the certificate tail's claim counters, which
    // the rerank launch zeroes otherwise — RerankArgs::direct has none)
    int* zero_ctl = nullptr;
    // non-NULL: per (query, split) the first key of the split's list (+inf: empty) at
    // heads[q * nsplit + split] — the direct second chance's prefix-limit bound, 4 B per list
    // instead of a strided read of every list's first entry
    float* heads = nullptr;
    // <= 4 queries: the split's 16 lane lists written unfolded (16 nsplit lists of km per query;
    // ncand >= 16 nsplit km) and heads = the smallest of their first keys — the direct route
    int raw16 = 0;
    // > 1: every half_k-th round of row groups, a second-half split's group goes to split -
    // nsplit / 2 (two workgroups per CU: the one dispatched second gets less work); 0 = even
    int half_k = 0;
    // > 0: the last `pool` 8-row groups are handed out at run time in chunks of pool_ch groups
    // from the counter dyn[0] (dyn[1] counts the waves done; the scan leaves both at 0, so they
    // are zeroed once when allocated); requires half_k = 0, nq <= 2 and km = 16
    int* dyn = nullptr;
    int pool = 0, pool_ch = 1;
};
// Bytes per row of the int8 copy: 64 per block, no padding (round 4; rows were whole 1-KiB
// groups of 16 blocks, 25 % zeros at d = 768).  Blocks sit in groups of 16 (the scan's 16 lanes of
// a row): group g = b / 16 holds m = min(16, nblk - 16 g) blocks at byte 1024 g, chunk c (16 B)
// of its block j = b % 16 at 16-B slot m c + j, so lane j's load c of a row reads 16 m contiguous
// bytes with its group's other lanes (256 B for a full group).
__host__ __device__ inline int64_t i8_row_bytes(int nblk) { return (int64_t)64 * nblk; }
__host__ __device__ inline int i8_slot(int nblk, int b, int c) {
    const int g = b >> 4, m = nblk - 16 * g < 16 ? nblk - 16 * g : 16;
    return 64 * g + m * c + (b & 15);
}
hipError_t launch_i8_rows(const float* xb, int64_t n, int dp, int nblk, int8_t* codes, float* scales,
                          float* resid, hipStream_t st);
hipError_t launch_i8_scan(const I8Args& a, hipStream_t st);
// launch_query_prep_b16's fp32 rows and norms + the int8 query codes in one pass (knn_i8.hip)
hipError_t launch_i8_query_prep(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                                int normalize, int nblk, float* dst, float* norms, int8_t* codes,
                                float* scales, float* resid, hipStream_t st);

hipError_t launch_rows_ingest(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                              int normalize, float* dst, float* norms, hipStream_t st);
hipError_t launch_tile_topk(const TileArgs& a, hipStream_t st);
hipError_t launch_b16_big(const TileArgs& a, hipStream_t st);     // knn_b16.hip
hipError_t launch_b16_wide(const TileArgs& a, hipStream_t st);    // knn_b16w.hip (16x16x32 form)
hipError_t launch_merge(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                        int64_t stride_q, int64_t stride_l, int k, int metric, int negate_in,
                        float* D, int64_t* I, hipStream_t st);
// launch_merge with a separate list stride for the labels (packed key|label buffers)
hipError_t launch_merge_strided(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                                int64_t stride_q, int64_t stride_l, int64_t stride_li, int k,
                                int metric, int negate_in, float* D, int64_t* I, hipStream_t st);
// Candidate merge for the rerank: nq x kout approximate candidates (ascending raw keys, empty =
// label -1) and, per query, the floor: the smallest key a row dropped by any list or by the merge's
// own lane lists can have (+inf when nothing was dropped).
// ws_*: two-level workspace for more than 64 lists per query (nq * ceil(nlists/64) * kout entries,
// nq * ceil(nlists/64) floors), may be NULL when nlists <= 64.
// l1_G (optional): when non-NULL and the merge takes two levels of which the first keeps 16 per
// group, with at most 32 groups (one level-1 entry per rerank thread), only level 1 runs and
// *l1_G = its group count (the rerank then selects the kout best from ws_*: RerankArgs::l1_G);
// otherwise *l1_G = 0 and D / I / floor hold the result.
hipError_t launch_merge_candidates(const float* cd, const int64_t* ci, int64_t nq, int nlists,
                                   int kin, int64_t stride_q, int64_t stride_l, int kout,
                                   int64_t id_offset, float* D, int64_t* I, float* floor,
                                   float* ws_d, int64_t* ws_i, float* ws_floor, hipStream_t st,
                                   int* l1_G = nullptr);
hipError_t launch_fill_empty(float* D, int64_t* I, int64_t n, int metric, hipStream_t st);
// multi-device index: dst[i] = start + i, and labels through a shard's local -> global map
// (I[i] = lmap[I[i]] + offset, -1 kept)
hipError_t launch_iota64(int64_t* dst, int64_t n, int64_t start, hipStream_t st);
hipError_t launch_map_labels(int64_t* I, int64_t n, const int64_t* lmap, int64_t offset,
                             hipStream_t st);

hipError_t launch_split_rows(const float* src, int64_t n, int dp, int bk, uint32_t* dst,
                             hipStream_t st);
hipError_t launch_rerank_certify(const RerankArgs& a, hipStream_t st);
// The certificate tail (TailArgs) on `grid` resident workgroups of the (2,1) exact tile.
hipError_t launch_cert_tail(const TailArgs& a, int grid, hipStream_t st);
constexpr int kTailWGPerCU = 1;     // tail grid = kTailWGPerCU x CUs (work is claimed, never awaited)
hipError_t launch_gather_rows(const float* src, const float* src_norm, int dp, const int* list,
                              int64_t n, int64_t n_pad, float* dst, float* dst_norm, hipStream_t st);
hipError_t launch_scatter_results(const float* sd, const int64_t* si, const int* list, int64_t n,
                                  int k, float* D, int64_t* I, hipStream_t st);
// fp32 rows (stride dp) -> bf16 rows (stride dpb elements, zero padded), |x - bf16(x)| per row
hipError_t launch_bf16_rows(const float* src, int64_t n, int dp, int dpb, uint16_t* dst,
                            float* resid, hipStream_t st);
// bf16 path query side in one pass: padded fp32 rows + |q|^2 + bf16 rows + residual norms
// (dpb <= 4096; hipErrorInvalidValue otherwise, the caller then uses the two kernels above)
hipError_t launch_query_prep_b16(const float* src, int64_t n, int d, int dp, int dpb, int64_t n_pad,
                                 int normalize, float* dst, float* norms, uint16_t* qb, float* resid,
                                 hipStream_t st);
hipError_t launch_max_norm(const float* xn, int64_t n, float* out, hipStream_t st);

// IVF-PQ (ivfpq.hip; layouts in include/imgrec_ivfpq.h)
// segmented radix sort of u64 keys (knn_hugek.hip, rocPRIM): segment i = [off[i], off[i + 1]) of
// `total` (< 2^32) keys over bits [0, end_bit); the temporary storage grows in *tmp (hipMallocAsync
// on st when async_tmp)
hipError_t sort_u64_segments(uint64_t* in, uint64_t* out, int64_t total, int nseg, const unsigned* off,
                             unsigned end_bit, void** tmp, size_t* tmp_cap, bool async_tmp, hipStream_t st);
// IVF-PQ for any k: every probed row's ADC key, a segmented sort per query, the first k
hipError_t launch_ivfpq_scan_all(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                                 const int64_t* list_off, const uint16_t* codes, const int64_t* ids,
                                 int m, int ksub, const int64_t* probe_off, const uint32_t* seg_off,
                                 int64_t total, int k, float* D, int64_t* I, hipStream_t st);
hipError_t launch_ivfpq_lut(const float* resid, int64_t nr, int d, int m, int ksub,
                            const float* cbt, float* lut, hipStream_t st);
hipError_t launch_ivfpq_scan(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                             const int64_t* list_off, const uint16_t* codes, const int64_t* ids,
                             int m, int ksub, int k, float* D, int64_t* I, hipStream_t st);

}  // namespace imgrec
