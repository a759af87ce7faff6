// knn_capi.cpp — the C ABI of include/imgrec_knn.h: index object, HBM corpus buffer, query
// workspace, launch planning and the faiss IndexFlat file layout.
//
// Reference call sites each entry point replaces are listed in include/imgrec_knn.h.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/imgrec_knn.h"
#include "../../include/imgrec_ivfpq.h"
#include "knn_kernels.h"

using imgrec::TileArgs;

namespace {

thread_local std::string g_err;

void set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define KNN_FAIL(code, ...)      \
    do {                         \
        set_err(__VA_ARGS__);    \
        return (code);           \
    } while (0)

#define KNN_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            set_err("%s failed: %s", #expr, hipGetErrorString(e_));                    \
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

struct Plan {
    int wr, wq, km, bm, bq;
    int nqb, nq_pad, ntiles, nsplit, ncand, wgs;
    bool big;                    // bf16 path: the 256 x 256-tile kernel (knn_b16.hip)
};

// Fused-kernel geometry for one query chunk (see DESIGN.md "Launch plan").
Plan make_plan(int64_t ntotal, int64_t nq, int k, int cus) {
    Plan p{};
    p.km = k <= 8 ? 8 : (k <= 10 ? 10 : (k <= 16 ? 16 : 32));
    int wg_per_cu;
    if (nq <= 32) { p.wr = 2; p.wq = 1; wg_per_cu = 3; }
    else if (nq <= 128) { p.wr = 2; p.wq = 2; wg_per_cu = 2; }
#ifdef IMGREC_BIG_TILE_18
    else { p.wr = 1; p.wq = 8; wg_per_cu = 1; }   // one 8-wave workgroup per CU (32.2 ms, ablation)
#else
    // Two independent 4-wave workgroups per CU: their barriers do not line up, so one
    // workgroup's stage bubble is filled by the other's MFMAs (31.4 vs 32.2 ms, bench config).
    else { p.wr = 1; p.wq = 4; wg_per_cu = 2; }
#endif
    p.bm = p.wr * 128;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
    const int target = cus * wg_per_cu;
    int ns = (target + p.nqb - 1) / p.nqb;
    ns = std::max(1, std::min(ns, p.ntiles));
    p.nsplit = ns;
    p.ncand = ns * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

constexpr int64_t kQueryChunk = 8192;

// Split-path geometry: one tile shape for every batch size ((1,4) workgroups, two per CU,
// kSplitWB row blocks per wave).
Plan make_split_plan(int64_t ntotal, int64_t nq, int kc, int cus) {
    Plan p{};
    p.km = kc;
    p.wr = 1;
    p.wq = 4;
    p.bm = p.wr * 32 * imgrec::kSplitWB;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
#ifndef IMGREC_SPLIT_WGPCU
#define IMGREC_SPLIT_WGPCU 2
#endif
    const int target = cus * IMGREC_SPLIT_WGPCU;
    p.nsplit = std::max(1, std::min((target + p.nqb - 1) / p.nqb, p.ntiles));
    p.ncand = p.nsplit * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

// Split-bf16 candidate path (knn_refine.hip): used for batches the (1,4) plan covers, k <= 16,
// rows padded to 32 floats.  K' = candidates kept per query for the exact rerank.
inline int split_kc(int k) { return k <= 10 ? 16 : (k <= 16 ? 32 : 0); }

// Relative error-bound coefficients of the certificate (DESIGN.md "Split path"), multiplied by
// |q| * max|x| in the kernel:
//   split dot:  3.1 * 2^-16 (dropped lo.lo / residual terms of x = hi + lo + r, |r| <= 2^-16 |x|)
//               + 1.02 * gamma_n, n = 3 MFMAs x (dp/16) steps x 5 (a 16-term tree inside each),
//               with unit roundoff 2^-23 (allows truncating accumulation);
//   rerank dot: 1.02 * gamma_n, n = 4*ceil(dp/256) + 8 fp32 FMAs + butterfly levels, u = 2^-24.
inline float split_coef(int dp) {
    return (float)(3.1 * std::ldexp(1.0, -16) + 1.02 * (15.0 * (dp / 16) + 16.0) * std::ldexp(1.0, -23));
}
inline float rerank_coef(int dp) {
    return (float)(1.02 * (4.0 * ((dp + 255) / 256) + 8.0) * std::ldexp(1.0, -24));
}

// bf16 candidate pass (one bf16 MFMA per product): the products of two bf16 values are exact in
// fp32, so the only arithmetic error besides the operand rounding (bounded in the rerank kernel
// from the stored residual norms) is the fp32 accumulation: 1.02 * gamma_n, n = (dpb/16) MFMAs x 5
// (a 16-term tree inside each) + 16, with unit roundoff 2^-23 (allows truncating accumulation),
// relative to |qh| |xh|.
inline float b16_acc_coef(int dpb) {
    return (float)(1.02 * (5.0 * (dpb / 16) + 16.0) * std::ldexp(1.0, -23));
}
// Candidates the bf16 pass hands to the rerank (K'), and the per-lane list length of its fused
// kernel (the merge floor covers what a lane list drops).
constexpr int kB16Cand = 64;
inline int b16_km(int k) { return k <= 16 ? 16 : 32; }
#ifndef IMGREC_B16_NARROW_Q
#define IMGREC_B16_NARROW_Q 32
#endif
constexpr int kB16NarrowQ = IMGREC_B16_NARROW_Q;   // batches up to this use the 32-query tile

// bf16-path geometry: large batches with k <= 10 on the 256 x 256-tile kernel (one workgroup
// per CU, lane lists of 8 / 10); otherwise (kB16WR, kB16WQ) workgroups, kB16WGPCU per CU.
Plan make_b16_plan(int64_t ntotal, int64_t nq, int k, int cus, int dpb) {
    Plan p{};
    // (dpb bound: the 256 x 256 kernel's 32-bit lane offsets, see launch_b16_big)
    if (nq >= imgrec::kB16BigMinQ && k <= 10 && dpb <= 16384) {
        p.big = true;
        p.km = k <= 8 ? 8 : 10;
        p.wr = 2;
        p.wq = 4;
        p.bm = imgrec::kB16BigRows;
        p.bq = imgrec::kB16BigQueries;
        p.nqb = (int)((nq + p.bq - 1) / p.bq);
        p.nq_pad = p.nqb * p.bq;
        p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
        p.nsplit = std::max(1, std::min((cus + p.nqb - 1) / p.nqb, p.ntiles));
        p.ncand = p.nsplit * p.km;               // lists folded to one per (query, split)
        p.wgs = p.nqb * p.nsplit;
        return p;
    }
    p.km = b16_km(k);
    // batches of <= 32 queries: a 32-query tile (the (1,4) tile would pad them to 128 and spend
    // four times the matrix work of an HBM-bound search)
    const bool narrow = nq <= kB16NarrowQ;
    p.wr = narrow ? 2 : imgrec::kB16WR;
    p.wq = narrow ? 1 : imgrec::kB16WQ;
    p.bm = p.wr * 32 * imgrec::kB16WB;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
    const int target = cus * imgrec::kB16WGPCU;
    p.nsplit = std::max(1, std::min((target + p.nqb - 1) / p.nqb, p.ntiles));
    p.ncand = p.nsplit * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

}  // namespace

struct knn_index {
    int d = 0, dp = 0, metric = KNN_METRIC_L2, device = 0, cus = 256;
    int64_t ntotal = 0, cap = 0, id_offset = 0;
    bool trained = true;
    float* xb = nullptr;     // cap x dp
    float* xn = nullptr;     // cap
    uint32_t* xs = nullptr;  // cap x dp split-bf16 copy (split_ok only)
    uint16_t* xh = nullptr;  // cap x dpb bf16 copy (b16_ok only)
    float* xr = nullptr;     // cap: |x - bf16(x)| per row (b16_ok only)
    float* xn_max = nullptr; // device scalar, max |x|^2 (refreshed when rows change)
    float* xr_max = nullptr; // device scalar, max |x - bf16(x)|
    int dpb = 0;             // bf16 row stride (elements)
    bool split_ok = false, b16_ok = false, xn_max_stale = true;
    int mode = KNN_SEARCH_AUTO;
    int last_path = 0;       // knn_last_path
    int64_t last_fallback = 0, last_split_queries = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // search workspace
    float* qpad = nullptr; size_t qpad_cap = 0;
    float* qnorm = nullptr; size_t qnorm_cap = 0;
    size_t xn_max_cap = 0;
    float* cand_d = nullptr; size_t cand_d_cap = 0;
    int64_t* cand_i = nullptr; size_t cand_i_cap = 0;
    uint32_t* qsplit = nullptr; size_t qsplit_cap = 0;
    float* cand2_d = nullptr; size_t cand2_d_cap = 0;
    int64_t* cand2_i = nullptr; size_t cand2_i_cap = 0;
    // [0] = uncertified count, [1] = max observed error / bound (float bits), [2] unused,
    // [3..] = the uncertified queries; [0..1] are zero between searches
    int* fail = nullptr; size_t fail_cap = 0;
    int* mail = nullptr;                                // pinned, mapped: [seq, count, ratio bits]
    int* mail_dev = nullptr;                            // its device address
    int mail_seq = 0;
    float last_err_ratio = 0.f;
    uint16_t* qb16 = nullptr; size_t qb16_cap = 0;
    float* q_resid = nullptr; size_t q_resid_cap = 0;
    float* floor = nullptr; size_t floor_cap = 0;
    float* mws_d = nullptr; size_t mws_d_cap = 0;          // two-level candidate merge workspace
    int64_t* mws_i = nullptr; size_t mws_i_cap = 0;
    float* mws_f = nullptr; size_t mws_f_cap = 0;
    size_t xr_max_cap = 0;
    // cascade workspace (queries a candidate pass could not certify, re-run by the next path)
    float* cs_q = nullptr; size_t cs_q_cap = 0;
    float* cs_qn = nullptr; size_t cs_qn_cap = 0;
    float* cs_d = nullptr; size_t cs_d_cap = 0;
    int64_t* cs_i = nullptr; size_t cs_i_cap = 0;
    int* cs_list = nullptr; size_t cs_list_cap = 0;
    float* fb_q = nullptr; size_t fb_q_cap = 0;
    float* fb_qn = nullptr; size_t fb_qn_cap = 0;
    float* fb_d = nullptr; size_t fb_d_cap = 0;
    int64_t* fb_i = nullptr; size_t fb_i_cap = 0;
    // host-path staging
    float* hq = nullptr; size_t hq_cap = 0;
    float* hd = nullptr; size_t hd_cap = 0;
    int64_t* hi = nullptr; size_t hi_cap = 0;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev;   // pairs
    size_t ev_used = 0;
};

namespace {

int reserve_rows(knn_index* ix, int64_t need) {
    if (need <= ix->cap) return KNN_OK;
    int64_t ncap = round_up(std::max(need, ix->cap + ix->cap / 2), imgrec::kTileRowsMax);
    float* nxb = nullptr;
    float* nxn = nullptr;
    KNN_HIP(hipMalloc((void**)&nxb, (size_t)ncap * ix->dp * sizeof(float)));
    hipError_t e = hipMalloc((void**)&nxn, (size_t)ncap * sizeof(float));
    if (e != hipSuccess) {
        (void)hipFree(nxb);
        KNN_FAIL(KNN_ENOMEM, "hipMalloc of %lld row norms failed", (long long)ncap);
    }
    uint32_t* nxs = nullptr;
    if (ix->split_ok) {
        e = hipMalloc((void**)&nxs, (size_t)ncap * ix->dp * sizeof(uint32_t));
        if (e != hipSuccess) {
            (void)hipFree(nxb);
            (void)hipFree(nxn);
            KNN_FAIL(KNN_ENOMEM, "hipMalloc of the %lld-row split copy failed", (long long)ncap);
        }
        KNN_HIP(hipMemsetAsync(nxs, 0, (size_t)ncap * ix->dp * sizeof(uint32_t), ix->stream));
    }
    uint16_t* nxh = nullptr;
    float* nxr = nullptr;
    if (ix->b16_ok) {
        e = hipMalloc((void**)&nxh, (size_t)ncap * ix->dpb * sizeof(uint16_t));
        if (e == hipSuccess) e = hipMalloc((void**)&nxr, (size_t)ncap * sizeof(float));
        if (e != hipSuccess) {
            for (void* p : {(void*)nxb, (void*)nxn, (void*)nxs, (void*)nxh})
                if (p) (void)hipFree(p);
            KNN_FAIL(KNN_ENOMEM, "hipMalloc of the %lld-row bf16 copy failed", (long long)ncap);
        }
        KNN_HIP(hipMemsetAsync(nxh, 0, (size_t)ncap * ix->dpb * sizeof(uint16_t), ix->stream));
        KNN_HIP(hipMemsetAsync(nxr, 0, (size_t)ncap * sizeof(float), ix->stream));
    }
    KNN_HIP(hipMemsetAsync(nxb, 0, (size_t)ncap * ix->dp * sizeof(float), ix->stream));
    KNN_HIP(hipMemsetAsync(nxn, 0, (size_t)ncap * sizeof(float), ix->stream));
    if (ix->ntotal > 0) {
        KNN_HIP(hipMemcpyAsync(nxb, ix->xb, (size_t)ix->ntotal * ix->dp * sizeof(float),
                               hipMemcpyDeviceToDevice, ix->stream));
        KNN_HIP(hipMemcpyAsync(nxn, ix->xn, (size_t)ix->ntotal * sizeof(float),
                               hipMemcpyDeviceToDevice, ix->stream));
        if (nxs)
            KNN_HIP(hipMemcpyAsync(nxs, ix->xs, (size_t)ix->ntotal * ix->dp * sizeof(uint32_t),
                                   hipMemcpyDeviceToDevice, ix->stream));
        if (nxh) {
            KNN_HIP(hipMemcpyAsync(nxh, ix->xh, (size_t)ix->ntotal * ix->dpb * sizeof(uint16_t),
                                   hipMemcpyDeviceToDevice, ix->stream));
            KNN_HIP(hipMemcpyAsync(nxr, ix->xr, (size_t)ix->ntotal * sizeof(float),
                                   hipMemcpyDeviceToDevice, ix->stream));
        }
    }
    KNN_HIP(hipStreamSynchronize(ix->stream));
    if (ix->xb) (void)hipFree(ix->xb);
    if (ix->xn) (void)hipFree(ix->xn);
    if (ix->xs) (void)hipFree(ix->xs);
    if (ix->xh) (void)hipFree(ix->xh);
    if (ix->xr) (void)hipFree(ix->xr);
    ix->xb = nxb;
    ix->xn = nxn;
    ix->xs = nxs;
    ix->xh = nxh;
    ix->xr = nxr;
    ix->cap = ncap;
    return KNN_OK;
}

// *_device entry points run on the caller's stream; NULL is the HIP null (default) stream, as in
// every HIP API (torch's default stream has handle 0).
hipStream_t pick(knn_index* ix, void* s) {
    (void)ix;
    return (hipStream_t)s;
}

// Timing events around the dominant (fused) kernel launch of a chunk.
int timed_begin(knn_index* ix, hipStream_t st, hipEvent_t* e1) {
    *e1 = nullptr;
    if (!ix->timing) return KNN_OK;
    if (ix->ev_used + 2 > ix->ev.size()) {
        for (int i = 0; i < 64; ++i) {
            hipEvent_t e;
            KNN_HIP(hipEventCreate(&e));
            ix->ev.push_back(e);
        }
    }
    KNN_HIP(hipEventRecord(ix->ev[ix->ev_used], st));
    *e1 = ix->ev[ix->ev_used + 1];
    ix->ev_used += 2;
    return KNN_OK;
}

// Exact fp32 path over nq padded queries (qpad holds make_plan(nq).nq_pad zero-padded rows).
int exact_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
                int64_t* I, hipStream_t st, bool timed) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const Plan p = make_plan(ix->ntotal, nq, k, ix->cus);
    int rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = p.km;
    a.xb = ix->xb; a.xnorm = ix->xn; a.nrows = (int)ix->ntotal; a.dp = ix->dp;
    a.qp = qpad; a.qnorm = qnorm; a.nq = (int)nq; a.metric = kmetric;
    a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb; a.id_offset = ix->id_offset;
    a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand; a.mode = imgrec::kModeF32;
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    KNN_HIP(imgrec::launch_merge(ix->cand_d, ix->cand_i, nq, p.ncand / p.km, p.km, p.ncand, p.km, k,
                                 kmetric, 0, D, I, st));
    return KNN_OK;
}

// max |x|^2 (and max bf16 residual) over the stored rows, recomputed after rows change
int refresh_maxima(knn_index* ix, hipStream_t st) {
    if (!ix->xn_max_stale) return KNN_OK;
    int rc;
    if ((rc = grow(&ix->xn_max, &ix->xn_max_cap, 1)) != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_max_norm(ix->xn, ix->ntotal, ix->xn_max, st));
    if (ix->b16_ok) {
        if ((rc = grow(&ix->xr_max, &ix->xr_max_cap, 1)) != KNN_OK) return rc;
        KNN_HIP(imgrec::launch_max_norm(ix->xr, ix->ntotal, ix->xr_max, st));
    }
    ix->xn_max_stale = false;
    return KNN_OK;
}

// AUTO: large batches are matrix-bound (bf16 MFMA vs fp32 MFMA) once the corpus amortises the
// rerank; small batches are HBM-bound (the bf16 copy streams half the bytes) once the corpus is
// large enough to repay the candidate path's fixed cost (~0.1-0.2 ms).
constexpr int64_t kB16MinRowsLarge = 16384, kB16MinRowsSmall = 131072;
bool use_b16(const knn_index* ix, int64_t nq, int k) {
    if (!ix->b16_ok || k > KNN_MAX_K) return false;
    if (ix->mode == KNN_SEARCH_BF16) return true;
    if (ix->mode != KNN_SEARCH_AUTO) return false;
    return ix->ntotal >= (nq > 128 ? kB16MinRowsLarge : kB16MinRowsSmall);
}

bool use_split(const knn_index* ix, int64_t nq, int k) {
    if (!ix->split_ok || ix->mode == KNN_SEARCH_EXACT || split_kc(k) == 0) return false;
    if (ix->mode == KNN_SEARCH_SPLIT) return true;
    // auto (when the bf16 path is unavailable): batches the (1,4) plan covers, corpora with
    // enough rows to amortise the rerank
    return ix->mode == KNN_SEARCH_AUTO && nq > 128 && ix->ntotal >= 16384;
}

int split_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
                int64_t* I, hipStream_t st, bool timed);

// Workspace for the rerank's stats: counters zeroed once here (the publish kernel after every
// rerank zeroes them again) and the pinned host mailbox it publishes to.
int grow_fail(knn_index* ix, int64_t nq, hipStream_t st) {
    if (!ix->mail) {
        KNN_HIP(hipHostMalloc((void**)&ix->mail, 4 * sizeof(int),
                              hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(ix->mail, 0, 4 * sizeof(int));
        KNN_HIP(hipHostGetDevicePointer((void**)&ix->mail_dev, ix->mail, 0));
    }
    if (ix->fail_cap >= (size_t)nq + 3) return KNN_OK;
    int rc = grow(&ix->fail, &ix->fail_cap, (size_t)nq + 3);
    if (rc != KNN_OK) return rc;
    KNN_HIP(hipMemsetAsync(ix->fail, 0, 3 * sizeof(int), st));
    return KNN_OK;
}

// Point a rerank at the stats workspace; the next mailbox sequence number goes with it.
void bind_stats(knn_index* ix, imgrec::RerankArgs* r) {
    r->fail_count = ix->fail;
    r->err_ratio = reinterpret_cast<float*>(ix->fail + 1);
    r->fail_list = ix->fail + 3;
    r->mail = ix->mail_dev;
    r->seq = ++ix->mail_seq;
    if (r->seq <= 0) r->seq = ix->mail_seq = 1;          // 0 is the mailbox's initial value
}

// Uncertified count and max error ratio of the last rerank: spin on the host mailbox the publish
// kernel writes (no copy, no stream synchronisation), with a stream query now and then so
// that a failed or drained stream ends the wait.
int read_stats(knn_index* ix, hipStream_t st, int* nfail, float* ratio) {
    const int seq = ix->mail_seq;
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(&ix->mail[0], __ATOMIC_ACQUIRE) == seq) break;
        if ((it & 255u) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {
                if (__atomic_load_n(&ix->mail[0], __ATOMIC_ACQUIRE) == seq) break;
                set_err("rerank finished without publishing its stats (seq %d)", seq);
                return KNN_EHIP;
            }
            if (e != hipErrorNotReady) KNN_HIP(e);
        }
        __builtin_ia32_pause();
    }
    *nfail = __atomic_load_n(&ix->mail[1], __ATOMIC_ACQUIRE);
    const int bits = __atomic_load_n(&ix->mail[2], __ATOMIC_ACQUIRE);
    std::memcpy(ratio, &bits, sizeof(float));
    return KNN_OK;
}

// Re-run the nfail queries listed in `list` (device, indices into qpad) on the next, more precise
// path — the split path when enough of them fail and it is available, else the exact kernel —
// and scatter the results back into D, I.  Own workspace: the nested path may use every other.
int cascade(knn_index* ix, const float* qpad, const float* qnorm, const int* list, int nfail, int k,
            float* D, int64_t* I, hipStream_t st) {
    const bool to_split = ix->split_ok && split_kc(k) != 0 && nfail > 128;
    const int64_t pad = to_split ? make_split_plan(ix->ntotal, nfail, split_kc(k), ix->cus).nq_pad
                                 : make_plan(ix->ntotal, nfail, k, ix->cus).nq_pad;
    int rc;
    if ((rc = grow(&ix->cs_q, &ix->cs_q_cap, (size_t)pad * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cs_qn, &ix->cs_qn_cap, (size_t)pad)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cs_d, &ix->cs_d_cap, (size_t)nfail * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cs_i, &ix->cs_i_cap, (size_t)nfail * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cs_list, &ix->cs_list_cap, (size_t)nfail)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpyAsync(ix->cs_list, list, (size_t)nfail * sizeof(int), hipMemcpyDeviceToDevice, st));
    KNN_HIP(imgrec::launch_gather_rows(qpad, qnorm, ix->dp, ix->cs_list, nfail, pad, ix->cs_q,
                                       ix->cs_qn, st));
    const int64_t keep_q = ix->last_split_queries, keep_fb = ix->last_fallback;
    rc = to_split ? split_chunk(ix, ix->cs_q, ix->cs_qn, nfail, k, ix->cs_d, ix->cs_i, st, false)
                  : exact_chunk(ix, ix->cs_q, ix->cs_qn, nfail, k, ix->cs_d, ix->cs_i, st, false);
    ix->last_split_queries = keep_q;
    ix->last_fallback = keep_fb;
    if (rc != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_scatter_results(ix->cs_d, ix->cs_i, ix->cs_list, nfail, k, D, I, st));
    return KNN_OK;
}

// bf16 candidates (one bf16 MFMA per product) + exact fp32 rerank of K' = 64 + certificate;
// uncertified queries cascade to the split path / exact kernel.
int b16_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
              int64_t* I, hipStream_t st, bool timed, bool q_ready) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int kc = kB16Cand;
    const Plan p = make_b16_plan(ix->ntotal, nq, k, ix->cus, ix->dpb);
    const int km = p.km;
    int rc;
    if ((rc = refresh_maxima(ix, st)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qb16, &ix->qb16_cap, (size_t)p.nq_pad * ix->dpb)) != KNN_OK) return rc;
    if ((rc = grow(&ix->q_resid, &ix->q_resid_cap, (size_t)p.nq_pad)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_d, &ix->cand2_d_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_i, &ix->cand2_i_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->floor, &ix->floor_cap, (size_t)nq)) != KNN_OK) return rc;
    if ((rc = grow_fail(ix, nq, st)) != KNN_OK) return rc;
    if (!q_ready)   // else search_locked's fused query prep already wrote qb16 / q_resid
        KNN_HIP(imgrec::launch_bf16_rows(qpad, p.nq_pad, ix->dp, ix->dpb, ix->qb16, ix->q_resid, st));
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = km; a.wb = imgrec::kB16WB; a.mode = imgrec::kModeBF16;
    a.xb = reinterpret_cast<const float*>(ix->xh); a.xnorm = ix->xn; a.nrows = (int)ix->ntotal;
    a.dp = ix->dpb / 2; a.qp = reinterpret_cast<const float*>(ix->qb16); a.qnorm = qnorm;
    a.nq = (int)nq; a.metric = kmetric; a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb;
    a.id_offset = ix->id_offset; a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand;
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(p.big ? imgrec::launch_b16_big(a, st) : imgrec::launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    const int nlists = p.ncand / km, ngrp = (nlists + 63) / 64;
    if (ngrp > 1) {
        if ((rc = grow(&ix->mws_d, &ix->mws_d_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_i, &ix->mws_i_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_f, &ix->mws_f_cap, (size_t)nq * ngrp)) != KNN_OK) return rc;
    }
    KNN_HIP(imgrec::launch_merge_candidates(ix->cand_d, ix->cand_i, nq, nlists, km, p.ncand, km, kc,
                                            ix->id_offset, ix->cand2_d, ix->cand2_i, ix->floor,
                                            ix->mws_d, ix->mws_i, ix->mws_f, st));
    imgrec::RerankArgs r{};
    r.mode = imgrec::kModeBF16;
    r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
    r.xn_max = ix->xn_max; r.id_offset = ix->id_offset; r.cd = ix->cand2_d; r.ci = ix->cand2_i;
    r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = b16_acc_coef(ix->dpb);
    r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
    bind_stats(ix, &r);
    r.q_resid = ix->q_resid; r.xr_max = ix->xr_max; r.floor = ix->floor;
    KNN_HIP(imgrec::launch_rerank_certify(r, st));
    int nfail = 0;
    float ratio = 0.f;
    if ((rc = read_stats(ix, st, &nfail, &ratio)) != KNN_OK) return rc;
    ix->last_err_ratio = std::max(ix->last_err_ratio, ratio);
    ix->last_split_queries += nq;
    if (nfail <= 0) return KNN_OK;
    ix->last_fallback += nfail;
    return cascade(ix, qpad, qnorm, ix->fail + 3, nfail, k, D, I, st);
}

// Split-bf16 candidates + exact rerank + certificate; uncertified queries re-run exactly.
int split_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
                int64_t* I, hipStream_t st, bool timed) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int kc = split_kc(k);
    const Plan p = make_split_plan(ix->ntotal, nq, kc, ix->cus);
    int rc;
    if ((rc = refresh_maxima(ix, st)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qsplit, &ix->qsplit_cap, (size_t)p.nq_pad * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_d, &ix->cand2_d_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_i, &ix->cand2_i_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow_fail(ix, nq, st)) != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_split_rows(qpad, p.nq_pad, ix->dp, imgrec::kSplitBK, ix->qsplit, st));
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = kc;
    a.xb = reinterpret_cast<const float*>(ix->xs); a.xnorm = ix->xn; a.nrows = (int)ix->ntotal;
    a.dp = ix->dp; a.qp = reinterpret_cast<const float*>(ix->qsplit); a.qnorm = qnorm;
    a.nq = (int)nq; a.metric = kmetric; a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb;
    a.id_offset = ix->id_offset; a.cand_d = ix->cand_d; a.cand_i = ix->cand_i;
    a.ncand = p.nsplit * p.wr * 2 * kc; a.mode = imgrec::kModeSplit;
    a.wb = imgrec::kSplitWB; a.sbk = imgrec::kSplitBK;
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    // global top-K' approximate candidates, raw ascending keys (merge in its L2 convention)
    KNN_HIP(imgrec::launch_merge(ix->cand_d, ix->cand_i, nq, a.ncand / kc, kc, a.ncand, kc, kc, 1,
                                 0, ix->cand2_d, ix->cand2_i, st));
    imgrec::RerankArgs r{};
    r.mode = imgrec::kModeSplit;
    r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
    r.xn_max = ix->xn_max; r.id_offset = ix->id_offset; r.cd = ix->cand2_d; r.ci = ix->cand2_i;
    r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = split_coef(ix->dp);
    r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
    bind_stats(ix, &r);
    KNN_HIP(imgrec::launch_rerank_certify(r, st));
    int nfail = 0;
    float ratio = 0.f;
    if ((rc = read_stats(ix, st, &nfail, &ratio)) != KNN_OK) return rc;
    ix->last_err_ratio = std::max(ix->last_err_ratio, ratio);
    ix->last_split_queries += nq;
    if (nfail <= 0) return KNN_OK;
    ix->last_fallback += nfail;
    const Plan pf = make_plan(ix->ntotal, nfail, k, ix->cus);
    if ((rc = grow(&ix->fb_q, &ix->fb_q_cap, (size_t)pf.nq_pad * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_qn, &ix->fb_qn_cap, (size_t)pf.nq_pad)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_d, &ix->fb_d_cap, (size_t)nfail * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_i, &ix->fb_i_cap, (size_t)nfail * k)) != KNN_OK) return rc;
    KNN_HIP(imgrec::launch_gather_rows(qpad, qnorm, ix->dp, ix->fail + 3, nfail, pf.nq_pad, ix->fb_q,
                                       ix->fb_qn, st));
    if ((rc = exact_chunk(ix, ix->fb_q, ix->fb_qn, nfail, k, ix->fb_d, ix->fb_i, st, false)) != KNN_OK)
        return rc;
    KNN_HIP(imgrec::launch_scatter_results(ix->fb_d, ix->fb_i, ix->fail + 3, nfail, k, D, I, st));
    return KNN_OK;
}

int search_locked(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st) {
    const int normalize = ix->metric == KNN_METRIC_COSINE;
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    ix->last_fallback = 0;
    ix->last_split_queries = 0;
    ix->last_err_ratio = 0.f;
    if (ix->ntotal == 0) {
        KNN_HIP(imgrec::launch_fill_empty(D, I, nq * (int64_t)k, kmetric, st));
        return KNN_OK;
    }
    for (int64_t c0 = 0; c0 < nq; c0 += kQueryChunk) {
        const int64_t cn = std::min(kQueryChunk, nq - c0);
        const bool b16 = use_b16(ix, cn, k);
        const bool split = !b16 && use_split(ix, cn, k);
        // padding: the query tile of the plan this chunk will run
        const Plan p = b16 ? make_b16_plan(ix->ntotal, cn, k, ix->cus, ix->dpb)
                     : split ? make_split_plan(ix->ntotal, cn, split_kc(k), ix->cus)
                             : make_plan(ix->ntotal, cn, k, ix->cus);
        const int64_t nq_pad = p.nq_pad;
        int rc;
        if (c0 == 0) ix->last_path = b16 ? 2 : (split ? 1 : 0);
        if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)nq_pad * ix->dp)) != KNN_OK) return rc;
        if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)nq_pad)) != KNN_OK) return rc;
        bool q_ready = false;
        if (b16 && ix->dpb <= 4096) {   // fused query prep: fp32 padded rows + norms + bf16 + residuals
            if ((rc = grow(&ix->qb16, &ix->qb16_cap, (size_t)nq_pad * ix->dpb)) != KNN_OK) return rc;
            if ((rc = grow(&ix->q_resid, &ix->q_resid_cap, (size_t)nq_pad)) != KNN_OK) return rc;
            KNN_HIP(imgrec::launch_query_prep_b16(q + c0 * ix->d, cn, ix->d, ix->dp, ix->dpb, nq_pad,
                                                  normalize, ix->qpad, ix->qnorm, ix->qb16,
                                                  ix->q_resid, st));
            q_ready = true;
        } else {
            KNN_HIP(imgrec::launch_rows_ingest(q + c0 * ix->d, cn, ix->d, ix->dp, nq_pad, normalize,
                                               ix->qpad, ix->qnorm, st));
        }
        rc = b16 ? b16_chunk(ix, ix->qpad, ix->qnorm, cn, k, D + c0 * k, I + c0 * k, st, true, q_ready)
             : split ? split_chunk(ix, ix->qpad, ix->qnorm, cn, k, D + c0 * k, I + c0 * k, st, true)
                     : exact_chunk(ix, ix->qpad, ix->qnorm, cn, k, D + c0 * k, I + c0 * k, st, true);
        if (rc != KNN_OK) return rc;
    }
    return KNN_OK;
}

int add_device_locked(knn_index* ix, const float* x, int64_t n, hipStream_t st) {
    int rc = reserve_rows(ix, ix->ntotal + n);
    if (rc != KNN_OK) return rc;
    if ((int64_t)(ix->ntotal + n) > (int64_t)INT32_MAX)
        KNN_FAIL(KNN_EINVAL, "a single index shard holds at most 2^31-1 rows");
    KNN_HIP(imgrec::launch_rows_ingest(x, n, ix->d, ix->dp, n,
                                       ix->metric == KNN_METRIC_COSINE ? 1 : 0,
                                       ix->xb + (size_t)ix->ntotal * ix->dp, ix->xn + ix->ntotal, st));
    if (ix->split_ok)
        KNN_HIP(imgrec::launch_split_rows(ix->xb + (size_t)ix->ntotal * ix->dp, n, ix->dp,
                                          imgrec::kSplitBK, ix->xs + (size_t)ix->ntotal * ix->dp, st));
    if (ix->b16_ok)
        KNN_HIP(imgrec::launch_bf16_rows(ix->xb + (size_t)ix->ntotal * ix->dp, n, ix->dp, ix->dpb,
                                         ix->xh + (size_t)ix->ntotal * ix->dpb, ix->xr + ix->ntotal, st));
    ix->ntotal += n;
    ix->xn_max_stale = true;
    return KNN_OK;
}

}  // namespace

extern "C" {

const char* knn_last_error(void) { return g_err.c_str(); }
const char* knn_version(void) { return "imgrec-knn 0.1 (gfx950, f32 MFMA 32x32x2, fused top-k)"; }

int knn_create(int d, int metric, int device, knn_index_t** out) {
    if (!out) KNN_FAIL(KNN_EINVAL, "out is NULL");
    *out = nullptr;
    if (d <= 0) KNN_FAIL(KNN_EINVAL, "d must be positive (got %d)", d);
    if (metric != KNN_METRIC_L2 && metric != KNN_METRIC_IP && metric != KNN_METRIC_COSINE)
        KNN_FAIL(KNN_EINVAL, "unknown metric %d", metric);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        KNN_FAIL(KNN_ENOSYS, "no HIP device visible");
    if (device < 0) KNN_HIP(hipGetDevice(&device));
    if (device >= ndev) KNN_FAIL(KNN_EINVAL, "device %d out of range (%d visible)", device, ndev);
    DeviceGuard g(device);
    knn_index* ix = new knn_index();
    ix->d = d;
    // rows padded to 16 floats; from d >= 512 to 32 so the 32-deep staging path applies
    ix->dp = (int)round_up(d, d >= 512 ? 2 * imgrec::kDepthPad : imgrec::kDepthPad);
    ix->metric = metric;
    ix->device = device;
    ix->split_ok = ix->dp % 32 == 0 && d >= 256;
    ix->b16_ok = d >= 64;
    ix->dpb = (int)round_up(d, imgrec::kB16Pad);
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        ix->cus = cus;
    if (hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ix;
        KNN_FAIL(KNN_EHIP, "hipStreamCreate failed");
    }
    *out = ix;
    return KNN_OK;
}

int knn_free(knn_index_t* ix) {
    if (!ix) return KNN_OK;
    DeviceGuard g(ix->device);
    (void)hipStreamSynchronize(ix->stream);
    for (void* p : {(void*)ix->xh, (void*)ix->xr, (void*)ix->xr_max, (void*)ix->qb16,
                    (void*)ix->q_resid, (void*)ix->floor, (void*)ix->cs_q, (void*)ix->cs_qn,
                    (void*)ix->cs_d, (void*)ix->cs_i, (void*)ix->cs_list, (void*)ix->mws_d,
                    (void*)ix->mws_i, (void*)ix->mws_f})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)ix->xb, (void*)ix->xn, (void*)ix->xs, (void*)ix->xn_max,
                    (void*)ix->qpad, (void*)ix->qnorm, (void*)ix->cand_d, (void*)ix->cand_i,
                    (void*)ix->qsplit, (void*)ix->cand2_d, (void*)ix->cand2_i, (void*)ix->fail,
                    (void*)ix->fb_q, (void*)ix->fb_qn, (void*)ix->fb_d, (void*)ix->fb_i,
                    (void*)ix->hq, (void*)ix->hd, (void*)ix->hi})
        if (p) (void)hipFree(p);
    if (ix->mail) (void)hipHostFree(ix->mail);
    for (hipEvent_t e : ix->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(ix->stream);
    delete ix;
    return KNN_OK;
}

int knn_dim(const knn_index_t* ix) { return ix ? ix->d : KNN_EINVAL; }
int knn_metric(const knn_index_t* ix) { return ix ? ix->metric : KNN_EINVAL; }
int64_t knn_ntotal(const knn_index_t* ix) { return ix ? ix->ntotal : KNN_EINVAL; }
int knn_is_trained(const knn_index_t* ix) { return ix ? (ix->trained ? 1 : 0) : KNN_EINVAL; }

int knn_set_id_offset(knn_index_t* ix, int64_t off) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    ix->id_offset = off;
    return KNN_OK;
}

int knn_train(knn_index_t* ix, const float* x, int64_t n) {
    (void)x;
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0) KNN_FAIL(KNN_EINVAL, "n must be >= 0");
    ix->trained = true;
    return KNN_OK;
}

int knn_reserve(knn_index_t* ix, int64_t n) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    return reserve_rows(ix, n);
}

int knn_add_device(knn_index_t* ix, const float* x, int64_t n, void* stream) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0 || (n > 0 && !x)) KNN_FAIL(KNN_EINVAL, "bad rows (n=%lld)", (long long)n);
    if (n == 0) return KNN_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    return add_device_locked(ix, x, n, pick(ix, stream));
}

int knn_add(knn_index_t* ix, const float* x, int64_t n) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0 || (n > 0 && !x)) KNN_FAIL(KNN_EINVAL, "bad rows (n=%lld)", (long long)n);
    if (n == 0) return KNN_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc = reserve_rows(ix, ix->ntotal + n);
    if (rc != KNN_OK) return rc;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64 << 20) / ((int64_t)ix->d * 4));
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int64_t cn = std::min(chunk, n - r0);
        if ((rc = grow(&ix->hq, &ix->hq_cap, (size_t)cn * ix->d)) != KNN_OK) return rc;
        KNN_HIP(hipMemcpyAsync(ix->hq, x + r0 * ix->d, (size_t)cn * ix->d * sizeof(float),
                               hipMemcpyHostToDevice, ix->stream));
        if ((rc = add_device_locked(ix, ix->hq, cn, ix->stream)) != KNN_OK) return rc;
        KNN_HIP(hipStreamSynchronize(ix->stream));
    }
    return KNN_OK;
}

int knn_reset(knn_index_t* ix) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    std::lock_guard<std::mutex> lk(ix->mu);
    ix->ntotal = 0;
    ix->xn_max_stale = true;
    return KNN_OK;
}

int knn_reconstruct_n(const knn_index_t* cix, int64_t i0, int64_t n, float* x) {
    knn_index* ix = const_cast<knn_index*>(cix);
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (i0 < 0 || n < 0 || i0 + n > ix->ntotal || (n > 0 && !x))
        KNN_FAIL(KNN_EINVAL, "reconstruct range [%lld, %lld) outside [0, %lld)", (long long)i0,
                 (long long)(i0 + n), (long long)ix->ntotal);
    if (n == 0) return KNN_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    KNN_HIP(hipMemcpy2DAsync(x, (size_t)ix->d * 4, ix->xb + (size_t)i0 * ix->dp, (size_t)ix->dp * 4,
                             (size_t)ix->d * 4, (size_t)n, hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    return KNN_OK;
}

int knn_search_device(knn_index_t* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                      void* stream) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (k <= 0 || k > KNN_MAX_K) KNN_FAIL(KNN_EINVAL, "k must be in [1, %d] (got %d)", KNN_MAX_K, k);
    if (nq < 0 || (nq > 0 && (!q || !D || !I))) KNN_FAIL(KNN_EINVAL, "bad query/output pointers");
    if (nq == 0) return KNN_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    return search_locked(ix, q, nq, k, D, I, pick(ix, stream));
}

int knn_search(knn_index_t* ix, const float* q, int64_t nq, int k, float* D, int64_t* I) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (k <= 0 || k > KNN_MAX_K) KNN_FAIL(KNN_EINVAL, "k must be in [1, %d] (got %d)", KNN_MAX_K, k);
    if (nq < 0 || (nq > 0 && (!q || !D || !I))) KNN_FAIL(KNN_EINVAL, "bad query/output pointers");
    if (nq == 0) return KNN_OK;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = grow(&ix->hq, &ix->hq_cap, (size_t)nq * ix->d)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hd, &ix->hd_cap, (size_t)nq * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hi, &ix->hi_cap, (size_t)nq * k)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpyAsync(ix->hq, q, (size_t)nq * ix->d * sizeof(float), hipMemcpyHostToDevice,
                           ix->stream));
    if ((rc = search_locked(ix, ix->hq, nq, k, ix->hd, ix->hi, ix->stream)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpyAsync(D, ix->hd, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost,
                           ix->stream));
    KNN_HIP(hipMemcpyAsync(I, ix->hi, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost,
                           ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    return KNN_OK;
}

int knn_merge_device(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin, int k,
                     int metric, float* D, int64_t* I, void* stream) {
    if (nlists <= 0 || kin <= 0 || nq < 0) KNN_FAIL(KNN_EINVAL, "bad merge shape");
    if (k <= 0 || k > KNN_MAX_K) KNN_FAIL(KNN_EINVAL, "k must be in [1, %d] (got %d)", KNN_MAX_K, k);
    if (nq == 0) return KNN_OK;
    if (!cD || !cI || !D || !I) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    const int kmetric = metric == KNN_METRIC_L2 ? 1 : 0;
    KNN_HIP(imgrec::launch_merge(cD, cI, nq, nlists, kin, kin, nq * (int64_t)kin, k, kmetric,
                                 kmetric ? 0 : 1, D, I, (hipStream_t)stream));
    return KNN_OK;
}

int64_t knn_packed_bytes(int64_t nq, int k) {
    if (nq < 0 || k <= 0) return KNN_EINVAL;
    const int64_t n = nq * k;
    return (n + (n & 1)) * 4 + n * 8;
}

int knn_merge_packed_device(const void* packed, int nlists, int64_t nq, int kin, int k, int metric,
                            float* D, int64_t* I, void* stream) {
    if (nlists <= 0 || kin <= 0 || nq < 0) KNN_FAIL(KNN_EINVAL, "bad merge shape");
    if (k <= 0 || k > KNN_MAX_K) KNN_FAIL(KNN_EINVAL, "k must be in [1, %d] (got %d)", KNN_MAX_K, k);
    if (nq == 0) return KNN_OK;
    if (!packed || !D || !I) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    const int64_t n = nq * kin, nf = n + (n & 1);
    const float* cD = static_cast<const float*>(packed);
    const int64_t* cI = reinterpret_cast<const int64_t*>(static_cast<const char*>(packed) + nf * 4);
    const int kmetric = metric == KNN_METRIC_L2 ? 1 : 0;
    // chunk = nf floats + n int64: nf + 2n floats, nf / 2 + n int64
    KNN_HIP(imgrec::launch_merge_strided(cD, cI, nq, nlists, kin, kin, nf + 2 * n, nf / 2 + n, k,
                                         kmetric, kmetric ? 0 : 1, D, I, (hipStream_t)stream));
    return KNN_OK;
}

int ivfpq_lut_device(const float* residuals, int64_t nr, int d, int m, int ksub,
                     const float* codebooks_t, float* lut, void* stream) {
    if (nr < 0 || d <= 0 || m <= 0 || ksub <= 0) KNN_FAIL(KNN_EINVAL, "bad IVF-PQ table shape");
    if (d % m != 0 || d / m > 256) KNN_FAIL(KNN_EINVAL, "d=%d must be m=%d x dsub with dsub <= 256", d, m);
    if (nr == 0) return KNN_OK;
    if (!residuals || !codebooks_t || !lut) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    KNN_HIP(imgrec::launch_ivfpq_lut(residuals, nr, d, m, ksub, codebooks_t, lut, (hipStream_t)stream));
    return KNN_OK;
}

int ivfpq_scan_device(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                      const int64_t* list_off, const uint16_t* codes, const int64_t* ids, int m,
                      int ksub, int k, float* D, int64_t* I, void* stream) {
    if (nq < 0 || nprobe <= 0 || m <= 0 || ksub <= 0 || ksub > 65536)
        KNN_FAIL(KNN_EINVAL, "bad IVF-PQ scan shape");
    if (k <= 0 || k > KNN_MAX_K) KNN_FAIL(KNN_EINVAL, "k must be in [1, %d] (got %d)", KNN_MAX_K, k);
    if (nq == 0) return KNN_OK;
    if (!lut || !probes || !list_off || !codes || !ids || !D || !I) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    KNN_HIP(imgrec::launch_ivfpq_scan(lut, probes, nq, nprobe, list_off, codes, ids, m, ksub, k, D, I,
                                      (hipStream_t)stream));
    return KNN_OK;
}

int knn_normalize_L2(float* x, int64_t n, int d) {
    if (n < 0 || d <= 0 || (n > 0 && !x)) KNN_FAIL(KNN_EINVAL, "bad array");
    // faiss fvec_renorm_L2: per row, nr = |x|^2; if nr > 0: x *= 1 / sqrt(nr).  The norm is
    // accumulated in double here (faiss sums in float SIMD lanes), so the scale is the correctly
    // rounded reciprocal norm and each output is within ~1 ulp of x / |x|.
    for (int64_t i = 0; i < n; ++i) {
        float* r = x + i * (int64_t)d;
        double nr = 0.0;
        for (int j = 0; j < d; ++j) nr += (double)r[j] * (double)r[j];
        if (nr > 0.0) {
            const float s = (float)(1.0 / sqrt(nr));
            for (int j = 0; j < d; ++j) r[j] *= s;
        }
    }
    return KNN_OK;
}

int knn_set_timing(knn_index_t* ix, int enable) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    std::lock_guard<std::mutex> lk(ix->mu);
    ix->timing = enable != 0;
    ix->ev_used = 0;
    return KNN_OK;
}

int knn_kernel_time(knn_index_t* ix, double* total_ms, int* launches) {
    if (!ix || !total_ms || !launches) KNN_FAIL(KNN_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    double tot = 0.0;
    for (size_t i = 0; i + 1 < ix->ev_used; i += 2) {
        KNN_HIP(hipEventSynchronize(ix->ev[i + 1]));
        float ms = 0.f;
        KNN_HIP(hipEventElapsedTime(&ms, ix->ev[i], ix->ev[i + 1]));
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int)(ix->ev_used / 2);
    ix->ev_used = 0;
    return KNN_OK;
}

int knn_set_search_mode(knn_index_t* ix, int mode) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (mode != KNN_SEARCH_AUTO && mode != KNN_SEARCH_EXACT && mode != KNN_SEARCH_SPLIT &&
        mode != KNN_SEARCH_BF16)
        KNN_FAIL(KNN_EINVAL, "unknown search mode %d", mode);
    std::lock_guard<std::mutex> lk(ix->mu);
    if (mode == KNN_SEARCH_SPLIT && !ix->split_ok)
        KNN_FAIL(KNN_EINVAL, "split search needs d >= 256 (rows padded to 32 floats); d = %d", ix->d);
    if (mode == KNN_SEARCH_BF16 && !ix->b16_ok)
        KNN_FAIL(KNN_EINVAL, "bf16 search needs d >= 64; d = %d", ix->d);
    ix->mode = mode;
    return KNN_OK;
}

int knn_search_stats(knn_index_t* ix, int64_t* split_queries, int64_t* fallback_queries,
                     float* max_err_ratio) {
    if (!ix || !split_queries || !fallback_queries) KNN_FAIL(KNN_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(ix->mu);
    *split_queries = ix->last_split_queries;
    *fallback_queries = ix->last_fallback;
    if (max_err_ratio) *max_err_ratio = ix->last_err_ratio;
    return KNN_OK;
}

int knn_last_path(const knn_index_t* ix) { return ix ? ix->last_path : KNN_EINVAL; }

int knn_plan(const knn_index_t* ix, int64_t nq, int k, int* tr, int* tq, int* splits, int* wgs) {
    if (!ix || !tr || !tq || !splits || !wgs) KNN_FAIL(KNN_EINVAL, "NULL argument");
    const int64_t cn = std::min(nq, kQueryChunk);
    const Plan p = use_b16(ix, cn, k) ? make_b16_plan(ix->ntotal, cn, k, ix->cus, ix->dpb)
                 : use_split(ix, cn, k) ? make_split_plan(ix->ntotal, cn, split_kc(k), ix->cus)
                                        : make_plan(ix->ntotal, cn, k, ix->cus);
    *tr = p.bm;
    *tq = p.bq;
    *splits = p.nsplit;
    *wgs = p.wgs;
    return KNN_OK;
}

// ----------------------------------------------------------------------------------------------
// faiss IndexFlat file layout (faiss/impl/index_write.cpp, write_index_header + WRITEXBVECTOR):
//   u32 fourcc ("IxF2" L2 / "IxFI" IP) | i32 d | i64 ntotal | i64 1<<20 | i64 1<<20 |
//   u8 is_trained | i32 metric_type (0 IP, 1 L2) | u64 ntotal*d | f32[ntotal*d]
// followed by an optional 8-byte trailer "IRGM" + i32 metric that faiss ignores and that marks
// a COSINE index (rows stored normalised, queries normalised on search).
// ----------------------------------------------------------------------------------------------
int knn_write(const knn_index_t* cix, const char* path) {
    knn_index* ix = const_cast<knn_index*>(cix);
    if (!ix || !path) KNN_FAIL(KNN_EINVAL, "NULL argument");
    FILE* f = fopen(path, "wb");
    if (!f) KNN_FAIL(KNN_EIO, "cannot open %s for writing", path);
    const char* cc = ix->metric == KNN_METRIC_L2 ? "IxF2" : "IxFI";
    uint32_t h = (uint32_t)(uint8_t)cc[0] | ((uint32_t)(uint8_t)cc[1] << 8) |
                 ((uint32_t)(uint8_t)cc[2] << 16) | ((uint32_t)(uint8_t)cc[3] << 24);
    int32_t d = ix->d;
    int64_t nt = ix->ntotal, dummy = 1 << 20;
    uint8_t tr = 1;
    int32_t mt = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    uint64_t nfl = (uint64_t)nt * (uint64_t)d;
    bool ok = fwrite(&h, 4, 1, f) == 1 && fwrite(&d, 4, 1, f) == 1 && fwrite(&nt, 8, 1, f) == 1 &&
              fwrite(&dummy, 8, 1, f) == 1 && fwrite(&dummy, 8, 1, f) == 1 &&
              fwrite(&tr, 1, 1, f) == 1 && fwrite(&mt, 4, 1, f) == 1 && fwrite(&nfl, 8, 1, f) == 1;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64 << 20) / ((int64_t)d * 4));
    std::vector<float> buf;
    for (int64_t r0 = 0; ok && r0 < nt; r0 += chunk) {
        const int64_t cn = std::min(chunk, nt - r0);
        buf.resize((size_t)cn * d);
        int rc = knn_reconstruct_n(ix, r0, cn, buf.data());
        if (rc != KNN_OK) { fclose(f); return rc; }
        ok = fwrite(buf.data(), sizeof(float), buf.size(), f) == buf.size();
    }
    if (ok && ix->metric == KNN_METRIC_COSINE) {
        int32_t m = KNN_METRIC_COSINE;
        ok = fwrite("IRGM", 1, 4, f) == 4 && fwrite(&m, 4, 1, f) == 1;
    }
    if (fclose(f) != 0) ok = false;
    if (!ok) KNN_FAIL(KNN_EIO, "write to %s failed", path);
    return KNN_OK;
}

int knn_read(const char* path, int device, knn_index_t** out) {
    if (!path || !out) KNN_FAIL(KNN_EINVAL, "NULL argument");
    *out = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) KNN_FAIL(KNN_EIO, "cannot open %s", path);
    uint32_t h = 0;
    int32_t d = 0, mt = 0;
    int64_t nt = 0, dm1 = 0, dm2 = 0;
    uint8_t tr = 0;
    uint64_t nfl = 0;
    bool ok = fread(&h, 4, 1, f) == 1 && fread(&d, 4, 1, f) == 1 && fread(&nt, 8, 1, f) == 1 &&
              fread(&dm1, 8, 1, f) == 1 && fread(&dm2, 8, 1, f) == 1 && fread(&tr, 1, 1, f) == 1 &&
              fread(&mt, 4, 1, f) == 1;
    char cc[5] = {(char)(h & 0xff), (char)((h >> 8) & 0xff), (char)((h >> 16) & 0xff),
                  (char)((h >> 24) & 0xff), 0};
    if (!ok || (strcmp(cc, "IxF2") != 0 && strcmp(cc, "IxFI") != 0)) {
        fclose(f);
        KNN_FAIL(KNN_EIO, "%s is not a faiss IndexFlatL2/IndexFlatIP file (fourcc '%s')", path, cc);
    }
    if (mt > 1) {  // metric_arg present for metrics > 1 (never written by us)
        float marg;
        ok = fread(&marg, 4, 1, f) == 1;
    }
    ok = ok && fread(&nfl, 8, 1, f) == 1;
    if (!ok || d <= 0 || nt < 0 || nfl != (uint64_t)nt * (uint64_t)d) {
        fclose(f);
        KNN_FAIL(KNN_EIO, "%s: corrupt IndexFlat header (d=%d ntotal=%lld)", path, d, (long long)nt);
    }
    // trailer check (COSINE marker)
    int metric = mt == 1 ? KNN_METRIC_L2 : KNN_METRIC_IP;
    long data_pos = ftell(f);
    if (fseek(f, 0, SEEK_END) == 0) {
        long end = ftell(f);
        long want = data_pos + (long)(nfl * 4);
        if (end == want + 8) {
            char tag[4];
            int32_t m = 0;
            fseek(f, want, SEEK_SET);
            if (fread(tag, 1, 4, f) == 4 && fread(&m, 4, 1, f) == 1 && memcmp(tag, "IRGM", 4) == 0 &&
                m == KNN_METRIC_COSINE)
                metric = KNN_METRIC_COSINE;
        } else if (end < want) {
            fclose(f);
            KNN_FAIL(KNN_EIO, "%s: truncated (%ld of %ld bytes)", path, end, want);
        }
    }
    fseek(f, data_pos, SEEK_SET);
    knn_index_t* ix = nullptr;
    int rc = knn_create(d, metric, device, &ix);
    if (rc != KNN_OK) { fclose(f); return rc; }
    if ((rc = knn_reserve(ix, nt)) != KNN_OK) { fclose(f); knn_free(ix); return rc; }
    // COSINE rows are already normalised; re-normalising a unit row is idempotent up to rounding,
    // so load them through the IP path and restore the metric afterwards.
    ix->metric = metric == KNN_METRIC_COSINE ? KNN_METRIC_IP : metric;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64 << 20) / ((int64_t)d * 4));
    std::vector<float> buf;
    for (int64_t r0 = 0; r0 < nt; r0 += chunk) {
        const int64_t cn = std::min(chunk, nt - r0);
        buf.resize((size_t)cn * d);
        if (fread(buf.data(), sizeof(float), buf.size(), f) != buf.size()) {
            fclose(f);
            knn_free(ix);
            KNN_FAIL(KNN_EIO, "%s: short read", path);
        }
        if ((rc = knn_add(ix, buf.data(), cn)) != KNN_OK) { fclose(f); knn_free(ix); return rc; }
    }
    fclose(f);
    ix->metric = metric;
    ix->trained = tr != 0;
    *out = ix;
    return KNN_OK;
}

}  // extern "C"
