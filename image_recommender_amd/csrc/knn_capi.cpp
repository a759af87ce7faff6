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

}  // namespace

struct knn_index {
    int d = 0, dp = 0, metric = KNN_METRIC_L2, device = 0, cus = 256;
    int64_t ntotal = 0, cap = 0, id_offset = 0;
    bool trained = true;
    float* xb = nullptr;     // cap x dp
    float* xn = nullptr;     // cap
    hipStream_t stream = nullptr;
    std::mutex mu;
    // search workspace
    float* qpad = nullptr; size_t qpad_cap = 0;
    float* qnorm = nullptr; size_t qnorm_cap = 0;
    float* cand_d = nullptr; size_t cand_d_cap = 0;
    int64_t* cand_i = nullptr; size_t cand_i_cap = 0;
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
    KNN_HIP(hipMemsetAsync(nxb, 0, (size_t)ncap * ix->dp * sizeof(float), ix->stream));
    KNN_HIP(hipMemsetAsync(nxn, 0, (size_t)ncap * sizeof(float), ix->stream));
    if (ix->ntotal > 0) {
        KNN_HIP(hipMemcpyAsync(nxb, ix->xb, (size_t)ix->ntotal * ix->dp * sizeof(float),
                               hipMemcpyDeviceToDevice, ix->stream));
        KNN_HIP(hipMemcpyAsync(nxn, ix->xn, (size_t)ix->ntotal * sizeof(float),
                               hipMemcpyDeviceToDevice, ix->stream));
    }
    KNN_HIP(hipStreamSynchronize(ix->stream));
    if (ix->xb) (void)hipFree(ix->xb);
    if (ix->xn) (void)hipFree(ix->xn);
    ix->xb = nxb;
    ix->xn = nxn;
    ix->cap = ncap;
    return KNN_OK;
}

// *_device entry points run on the caller's stream; NULL is the HIP null (default) stream, as in
// every HIP API (torch's default stream has handle 0).
hipStream_t pick(knn_index* ix, void* s) {
    (void)ix;
    return (hipStream_t)s;
}

int search_locked(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st) {
    const int normalize = ix->metric == KNN_METRIC_COSINE;
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    if (ix->ntotal == 0) {
        KNN_HIP(imgrec::launch_fill_empty(D, I, nq * (int64_t)k, kmetric, st));
        return KNN_OK;
    }
    for (int64_t c0 = 0; c0 < nq; c0 += kQueryChunk) {
        const int64_t cn = std::min(kQueryChunk, nq - c0);
        const Plan p = make_plan(ix->ntotal, cn, k, ix->cus);
        int rc;
        if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)p.nq_pad * ix->dp)) != KNN_OK) return rc;
        if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)p.nq_pad)) != KNN_OK) return rc;
        if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)cn * p.ncand)) != KNN_OK) return rc;
        if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)cn * p.ncand)) != KNN_OK) return rc;
        KNN_HIP(imgrec::launch_rows_ingest(q + c0 * ix->d, cn, ix->d, ix->dp, p.nq_pad, normalize,
                                           ix->qpad, ix->qnorm, st));
        TileArgs a{};
        a.wr = p.wr; a.wq = p.wq; a.km = p.km;
        a.xb = ix->xb; a.xnorm = ix->xn; a.nrows = (int)ix->ntotal; a.dp = ix->dp;
        a.qp = ix->qpad; a.qnorm = ix->qnorm; a.nq = (int)cn; a.metric = kmetric;
        a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb; a.id_offset = ix->id_offset;
        a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (ix->timing) {
            if (ix->ev_used + 2 > ix->ev.size()) {
                for (int i = 0; i < 64; ++i) {
                    hipEvent_t e;
                    KNN_HIP(hipEventCreate(&e));
                    ix->ev.push_back(e);
                }
            }
            e0 = ix->ev[ix->ev_used];
            e1 = ix->ev[ix->ev_used + 1];
            ix->ev_used += 2;
            KNN_HIP(hipEventRecord(e0, st));
        }
        KNN_HIP(imgrec::launch_tile_topk(a, st));
        if (e1) KNN_HIP(hipEventRecord(e1, st));
        const int nlists = p.ncand / p.km;
        KNN_HIP(imgrec::launch_merge(ix->cand_d, ix->cand_i, cn, nlists, p.km, p.ncand, p.km, k,
                                     kmetric, 0, D + c0 * k, I + c0 * k, st));
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
    ix->ntotal += n;
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
    for (void* p : {(void*)ix->xb, (void*)ix->xn, (void*)ix->qpad, (void*)ix->qnorm,
                    (void*)ix->cand_d, (void*)ix->cand_i, (void*)ix->hq, (void*)ix->hd,
                    (void*)ix->hi})
        if (p) (void)hipFree(p);
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

int knn_plan(const knn_index_t* ix, int64_t nq, int k, int* tr, int* tq, int* splits, int* wgs) {
    if (!ix || !tr || !tq || !splits || !wgs) KNN_FAIL(KNN_EINVAL, "NULL argument");
    const Plan p = make_plan(ix->ntotal, std::min(nq, kQueryChunk), k, ix->cus);
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
