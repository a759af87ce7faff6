// knn_index.h — internal state of one k-NN index and the helpers the C-ABI translation units
// share (knn_capi.cpp: entry points; knn_plan.cpp: launch geometry and error-bound coefficients;
// knn_search.cpp: the search paths; knn_io.cpp: the faiss file layout; knn_multi.cpp: one index
// over several devices).  Not part of the public ABI (include/imgrec_knn.h).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/imgrec_knn.h"
#include "knn_kernels.h"

namespace imgrec {

void set_err(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
// the value of a test / A-B environment knob, logged once on stderr when set (knn_capi.cpp)
const char* test_knob(const char* name);

#define KNN_FAIL(code, ...)              \
    do {                                 \
        ::imgrec::set_err(__VA_ARGS__);  \
        return (code);                   \
    } while (0)

#define KNN_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::imgrec::set_err("%s failed: %s", #expr, hipGetErrorString(e_));          \
            return e_ == hipErrorOutOfMemory ? KNN_ENOMEM : KNN_EHIP;                  \
        }                                                                              \
    } while (0)

struct DeviceGuard {
    int old = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&old) != hipSuccess) old = -1;
        if (dev >= 0 && dev != old) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (old >= 0 && hipGetDevice(&cur) == hipSuccess && cur != old) (void)hipSetDevice(old);
    }
};

inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Device buffer that only grows (workspace reused across searches).
template <typename T>
int grow(T** p, size_t* cap, size_t need) {
    if (*cap >= need) return KNN_OK;
    const size_t n = std::max(need, *cap * 3 / 2);
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    KNN_HIP(hipMalloc((void**)p, n * sizeof(T)));
    *cap = n;
    return KNN_OK;
}

// ---- launch geometry (knn_plan.cpp; DESIGN.md "Launch plan") ---------------------------------
struct Plan {
    int wr, wq, km, bm, bq;
    int nqb, nq_pad, ntiles, nsplit, ncand, wgs;
    bool big;                    // bf16 path: the 256 x 256-tile kernel (knn_b16.hip)
    int ib;                      // > 0: its packed-list form with ib split-local index bits
};
constexpr int64_t kQueryChunk = 8192;
Plan make_plan(int64_t ntotal, int64_t nq, int k, int cus);
Plan make_split_plan(int64_t ntotal, int64_t nq, int kc, int cus);
Plan make_b16_plan(int64_t ntotal, int64_t nq, int k, int cus, int dpb);
// The exact re-run of uncertified queries (inside the certificate tail kernel): the (2,1) tile
// of make_plan (256 rows x 32 queries), planned on device for whatever count the certificate
// leaves.
constexpr int kFallbackWR = 2;                 // lists per row split = 2 * kFallbackWR
int fallback_km(int k);
int split_kc(int k);
float split_coef(int dp);
float rerank_coef(int dp);
float b16_acc_coef(int dpb);
// int8 small-batch pass (knn_i8.hip): batches of at most kI8MaxQ queries, K' = kB16Cand
constexpr int kI8MaxQ = 8;
float i8_acc_coef(int nblk);
// wgpcu: int8 scan workgroups per CU (the split count is CUs x wgpcu); 0 = by batch size
Plan make_i8_plan(int64_t ntotal, int64_t nq, int k, int cus, int wgpcu, int nblk);
constexpr int kI8WGPCUDefault = 0;
constexpr int kB16Cand = 64;                   // K': candidates the bf16 pass hands to the rerank
int b16_km(int k);

}  // namespace imgrec

struct knn_index {
    int d = 0, dp = 0, metric = KNN_METRIC_L2, device = 0, cus = 256;
    // launch knobs read from the environment at creation (A/B and tests): the int8 scan's
    // workgroups per CU (IMGREC_I8_WGPCU) and the merge's second level inside the rerank
    // (IMGREC_MERGE_FUSE=0: off)
    int i8_wgpcu = imgrec::kI8WGPCUDefault;
    bool merge_fuse = true;
    bool chance_skip = true;    // IMGREC_CHANCE_SKIP=0: every query takes the first rerank
    // int8 batches of at most this many queries skip the merge and the first rerank: the
    // certificate tail's second chance answers every query (RerankArgs::direct);
    // IMGREC_CHANCE_DIRECT=N sets it, 0 = off.  4: two queries 10 / 5.5 us faster at config 2 / 3,
    // four queries 9-18 us faster at config 2 and the same at config 3
    // (profiles/r05/nq1/direct_nq24/)
    int chance_direct_max = 4;
    // ... over the scan's lane lists unfolded: 1 = while <= 4096 per query, 2 = always, 0 = never
    // (IMGREC_DIRECT_RAW)
    int direct_raw = 1;
    // int8 scan at two workgroups per CU: every K-th round the second-dispatched half's groups go
    // to the first half (I8Args::half_k; IMGREC_I8_HALF_K=K, 0 = even split).  12: config 2 one
    // query 0.1517 -> 0.1503 ms; 6-8 and 24-32 measured worse (profiles/r05/nq1/half_k/)
    int i8_half_k = 12;
    // int8 scan: the last i8_pool64 / 64 of the row groups handed out at run time in chunks of
    // 4 i8_pool_ch groups (I8Args::pool).  Default: one query on one workgroup per CU (rows of
    // >= 24 blocks), where 4/64 in chunks of 8 groups took the config-3 search from 0.3258 to
    // 0.3210 ms; config 2's two workgroups per CU lost 4-30 us with any pool (profiles/r06/i8_pool/).
    // IMGREC_I8_POOL=<64ths> (0 = off) applies it to every one- or two-query scan with lists of 16.
    int i8_pool64 = 4;
    int i8_pool_ch = 2;
    bool i8_pool_forced = false;
    int* i8_dyn = nullptr;      // the pool's two counters (zeroed once; the scan leaves them at 0)
    bool stream_lists = true;   // exact lists of <= 4 queries from one fp32 stream (IMGREC_STREAM_LISTS=0: tiles)
    bool merge_single = false;  // IMGREC_MERGE_SINGLE=1: the single-level merge in the rerank
    bool rerank_nw4 = false;    // IMGREC_RERANK_NW4=1: large batches rerank on 4-wave workgroups
    bool rerank_p1k = true;     // large batches rerank k rows first (IMGREC_RERANK_P1=0: 16)
    bool i8_fused_prep = true;  // int8 query prep inside the scan (IMGREC_I8_FUSED_PREP=0: own launch)
    bool merge_fuse1 = true;    // IMGREC_MERGE_FUSE=1: only level 2 in the rerank (0: neither)
    int64_t ntotal = 0, cap = 0, id_offset = 0;
    bool trained = true;
    float* xb = nullptr;     // cap x dp
    float* xn = nullptr;     // cap
    uint32_t* xs = nullptr;  // cap x dp split-bf16 copy (built by the first split search)
    uint16_t* xh = nullptr;  // cap x dpb bf16 copy (b16_ok only)
    float* xr = nullptr;     // cap: |x - bf16(x)| per row (b16_ok only)
    int8_t* x8 = nullptr;    // cap x nblk8*64 block-scaled int8 copy (built by the first i8 search)
    float* x8s = nullptr;    // cap x nblk8 block scales
    float* x8r = nullptr;    // cap: |x - s c| per row
    float* x8r_max = nullptr; size_t x8r_max_cap = 0;   // device scalar, max of x8r
    int nblk8 = 0;           // 64-element blocks per row (d <= 4096)
    int8_t* q8 = nullptr; size_t q8_cap = 0;        // a search's two-level query codes
    float* q8s = nullptr; size_t q8s_cap = 0;       //   their scales
    float* q8r = nullptr; size_t q8r_cap = 0;       //   |q - q~| per query
    float* xn_max = nullptr; // device scalar, max |x|^2 (refreshed when rows change)
    float* xr_max = nullptr; // device scalar, max |x - bf16(x)|
    int dpb = 0;             // bf16 row stride (elements)
    bool split_ok = false, b16_ok = false, xn_max_stale = true;
    int mode = KNN_SEARCH_AUTO;
    int last_path = 0;       // knn_last_path
    int64_t last_split_queries = 0;   // queries of the last search on a candidate path
    hipStream_t stream = nullptr;     // the index's own stream (host-pointer entry points)
    std::mutex mu;
    // Cross-stream ordering: an asynchronous operation records `fence` on its stream when it ends
    // (KNN_FENCE_EAGER, the default) or only remembers the stream and records the event there
    // when a later operation arrives on a different stream (KNN_FENCE_LAZY, opt-in); an operation
    // on a different stream waits for the event (adds before searches, one search's workspace use
    // before the next's, ...).  Host-synchronous operations leave no fence.
    hipEvent_t fence = nullptr;
    hipStream_t fence_stream = nullptr;
    bool fence_set = false;        // an operation on fence_stream may still run
    bool fence_recorded = false;   // `fence` already marks its end
    bool fence_lazy = false;
    // search workspace
    float* qpad = nullptr; size_t qpad_cap = 0;
    float* qnorm = nullptr; size_t qnorm_cap = 0;
    size_t xn_max_cap = 0;
    float* cand_d = nullptr; size_t cand_d_cap = 0;
    int64_t* cand_i = nullptr; size_t cand_i_cap = 0;
    uint32_t* qsplit = nullptr; size_t qsplit_cap = 0;
    float* cand2_d = nullptr; size_t cand2_d_cap = 0;
    int64_t* cand2_i = nullptr; size_t cand2_i_cap = 0;
    int* fail = nullptr; size_t fail_cap = 0;          // the uncertified queries of a chunk
    int* chance = nullptr; size_t chance_cap = 0;      // the second-chance queue of a chunk
    float* sc_key = nullptr; size_t sc_key_cap = 0;    // sliced second chance (RerankArgs::sc_*)
    int64_t* sc_lab = nullptr; size_t sc_lab_cap = 0;
    unsigned* sc_meta = nullptr; size_t sc_meta_cap = 0;
    int* sc_done = nullptr; size_t sc_done_cap = 0;
    int* stat = nullptr;                               // 12 ints: two chunk parities + totals
    int stat_seq = 0;                                  // chunks run (parity = seq & 1)
    bool stat_valid = false;                           // the last search ran a candidate path
    uint16_t* qb16 = nullptr; size_t qb16_cap = 0;
    float* q_resid = nullptr; size_t q_resid_cap = 0;
    float* floor = nullptr; size_t floor_cap = 0;
    float* heads = nullptr; size_t heads_cap = 0;       // int8 lists' first keys (direct route)
    float* mws_d = nullptr; size_t mws_d_cap = 0;          // two-level candidate merge workspace
    int64_t* mws_i = nullptr; size_t mws_i_cap = 0;
    float* mws_f = nullptr; size_t mws_f_cap = 0;
    uint32_t* b16_sync = nullptr; size_t b16_sync_cap = 0;   // 256 x 256 kernel sibling progress
    uint32_t b16_epoch = 0;
    size_t xr_max_cap = 0;
    // exact re-run workspace (device-planned: queries, candidate lists, plan)
    float* fb_q = nullptr; size_t fb_q_cap = 0;
    float* fb_qn = nullptr; size_t fb_qn_cap = 0;
    float* fb_cd = nullptr; size_t fb_cd_cap = 0;
    int64_t* fb_ci = nullptr; size_t fb_ci_cap = 0;
    int* tail_ctl = nullptr; size_t tail_ctl_cap = 0;   // tail claim counters + block tickets
    // host-path staging (device side), and page-locked host buffers for small searches
    float* pq = nullptr; size_t pq_cap = 0;        // hipHostMalloc'ed (caps in bytes)
    float* pd = nullptr; size_t pd_cap = 0;
    int64_t* pi = nullptr; size_t pi_cap = 0;
    float* hq = nullptr; size_t hq_cap = 0;
    float* hd = nullptr; size_t hd_cap = 0;
    int64_t* hi = nullptr; size_t hi_cap = 0;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev;   // pairs
    size_t ev_used = 0;
    // one index over several devices (knn_multi.cpp); NULL for a single-device index
    struct knn_multi* multi = nullptr;
    // k > KNN_MAX_K (knn_largek.hip): the fallback's stripe lists, the uncertified queries (+ count)
    uint64_t* lk_run = nullptr; size_t lk_run_cap = 0;
    // a chunk's failed queries, then their count and the last large-k search's total (device)
    int* lk_fail = nullptr; size_t lk_fail_cap = 0;
    // k > KNN_MAX_K_LARGE (knn_hugek.hip): a query chunk's keys, sorted keys, segment offsets, and
    // the sort's temporary storage (bytes)
    uint64_t* hk_a = nullptr; size_t hk_a_cap = 0;
    uint64_t* hk_b = nullptr; size_t hk_b_cap = 0;
    unsigned* hk_off = nullptr; size_t hk_off_cap = 0;
    void* hk_tmp = nullptr; size_t hk_tmp_cap = 0;
};

namespace imgrec {

// knn_capi.cpp
const char* last_error();
int set_metric(knn_index* ix, int metric);
int set_trained(knn_index* ix, bool trained);
int fence_begin(knn_index* ix, hipStream_t st);
int fence_end(knn_index* ix, hipStream_t st);
int fence_end_synced(knn_index* ix);
int reserve_rows(knn_index* ix, int64_t need, hipStream_t st);
int add_device_locked(knn_index* ix, const float* x, int64_t n, hipStream_t st);
int ensure_split(knn_index* ix, hipStream_t st);
int ensure_i8(knn_index* ix, hipStream_t st);
int create_single(int d, int metric, int device, knn_index** out);
void free_single(knn_index* ix);
// knn_search.cpp
int search_locked(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st);
int read_search_stats(knn_index* ix, int64_t* split_q, int64_t* fallback_q, int64_t* first_fail,
                      float* ratio);
bool use_b16(const knn_index* ix, int64_t nq, int k);
bool use_i8(const knn_index* ix, int64_t nq, int k);
// knn_largek.hip
int largek_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st);
// Exact per-(query, row split) top-32 lists of <= 4 queries from one fp32 stream of the corpus
// (csrc/knn_largek.hip largek_stream_kernel): the large-k route's lists and the exact route for
// small batches; lists at cd / ci + q * sp * 32 + s * 32 (labels with id_offset, -1 = empty).
bool stream_lists_ok(const knn_index* ix, int64_t nq);
int stream_splits(const knn_index* ix);
hipError_t launch_stream_lists(const knn_index* ix, const float* qpad, const float* qnorm, int64_t nq,
                               int metric, int sp, float* cd, int64_t* ci, hipStream_t st);
void largek_free(knn_index* ix);
// queries the last large-k search sent to the exact scan (a device count; waits for the index)
int largek_fallbacks(knn_index* ix, int64_t* n);
// merge of nlists sorted per-shard lists for KNN_MAX_K < k (nlists * kin <= 8192; labels < 2^32)
hipError_t launch_merge_large(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                              int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                              hipStream_t st);
bool use_split(const knn_index* ix, int64_t nq, int k);
// knn_hugek.hip: k > KNN_MAX_K_LARGE — every (query, row) key, a segmented sort per query
int hugek_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                 hipStream_t st);
void hugek_free(knn_index* ix);
// merge of nlists sorted lists of kin entries per query for any k (labels < 2^32)
hipError_t launch_merge_huge(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                             int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                             hipStream_t st);
// the large-k list merge when it fits the in-LDS select (nlists * kin <= 8192), else the sort
hipError_t launch_merge_any(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin,
                            int64_t sd, int64_t si, int k, int metric, float* D, int64_t* I,
                            hipStream_t st);

}  // namespace imgrec
