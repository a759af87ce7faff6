// knn_capi.cpp — the C ABI of include/imgrec_knn.h: index lifetime, the HBM corpus buffer, adds,
// searches, merges, timing and stats.  The search paths live in knn_search.cpp, the launch
// geometry in knn_plan.cpp, the file layout in knn_io.cpp, the multi-device index in
// knn_multi.cpp.
//
// Reference call sites each entry point replaces are listed in include/imgrec_knn.h.
//
// Stream semantics: *_device entry points enqueue on the caller's stream and return without
// waiting for the GPU; host-pointer entry points run on the index's own stream and synchronise.
// An operation on another stream than the previous one first waits for the previous one's stream
// (fence_begin), so mixing streams (or host and device calls) is always ordered.

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "knn_index.h"
#include "knn_multi.h"

namespace imgrec {

namespace {
thread_local std::string g_err;
}  // namespace

// The A/B and test knobs read at index creation (IMGREC_CUS, IMGREC_I8_WGPCU, IMGREC_MERGE_FUSE,
// IMGREC_CHANCE_SKIP, IMGREC_B16W_SYNC_LAG; INTEGRATION.md "A/B switches"): not product settings.
// An inherited one silently re-plans every launch, so the first read of each that is set says so
// once on stderr.
const char* test_knob(const char* name) {
    const char* e = std::getenv(name);
    if (e && *e) {
        static std::mutex mu;
        static std::string seen;
        std::lock_guard<std::mutex> lk(mu);
        const std::string tag = std::string("|") + name + "|";
        if (seen.find(tag) == std::string::npos) {
            seen += tag;
            std::fprintf(stderr, "[imgrec] %s=%s overrides a launch default (test / A-B knob, "
                                 "INTEGRATION.md)\n", name, e);
        }
    }
    return e && *e ? e : nullptr;
}

void set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

const char* last_error() { return g_err.c_str(); }

// Fences.  By default (KNN_FENCE_EAGER) an asynchronous operation records the index's fence
// event on its stream as its last enqueued step, and the next operation on ANOTHER stream waits
// for that event: nothing depends on the old stream afterwards (it may be destroyed, and work the
// caller queues on it later is not waited for).  KNN_FENCE_LAZY (opt-in, knn_set_fence_mode)
// records nothing while the stream stays the same and records the event on the remembered stream
// only when a different stream arrives: back-to-back operations on one stream then pay no event
// record (each costs ~5.7 us of idle GPU between the kernels around it on MI355X,
// profiles/r03/), but the remembered stream must stay valid until that next operation, and the
// wait covers whatever the caller queued on it meanwhile.  A lazy record that reports an error
// falls back to a device-wide synchronisation instead of wedging the index — best effort only:
// recording on a stream the caller has destroyed is a use after free, not a guaranteed error
// return, so in lazy mode the stream MUST outlive the next call on the index (imgrec_knn.h).
// Host-pointer operations synchronise their stream before returning and leave no fence.
int fence_begin(knn_index* ix, hipStream_t st) {
    if (!ix->fence_set || ix->fence_stream == st) return KNN_OK;
    if (!ix->fence_recorded) {
        if (hipEventRecord(ix->fence, ix->fence_stream) != hipSuccess) {
            (void)hipGetLastError();
            ix->fence_set = false;
            KNN_HIP(hipDeviceSynchronize());
            return KNN_OK;
        }
        ix->fence_recorded = true;
    }
    KNN_HIP(hipStreamWaitEvent(st, ix->fence, 0));
    return KNN_OK;
}

int fence_end(knn_index* ix, hipStream_t st) {
    ix->fence_stream = st;
    ix->fence_set = true;
    ix->fence_recorded = false;
    if (!ix->fence_lazy) {
        KNN_HIP(hipEventRecord(ix->fence, st));
        ix->fence_recorded = true;
    }
    return KNN_OK;
}

// After a host-synchronous operation (its stream drained before returning): nothing to wait for.
int fence_end_synced(knn_index* ix) {
    ix->fence_set = false;
    ix->fence_recorded = false;
    return KNN_OK;
}

// Grow the corpus buffers (fp32 rows, norms, split / bf16 copies) to hold `need` rows; the
// copies of the existing rows run on `st` (ordered after the adds that wrote them), which is
// synchronised before the old buffers are released.
int reserve_rows(knn_index* ix, int64_t need, hipStream_t st) {
    if (need <= ix->cap) return KNN_OK;
    const int64_t ncap = round_up(std::max(need, ix->cap + ix->cap / 2), kTileRowsMax);
    float* nxb = nullptr;
    float* nxn = nullptr;
    uint32_t* nxs = nullptr;
    uint16_t* nxh = nullptr;
    float* nxr = nullptr;
    int8_t* nx8 = nullptr;
    float* nx8s = nullptr;
    float* nx8r = nullptr;
    auto release = [&]() {
        for (void* p : {(void*)nxb, (void*)nxn, (void*)nxs, (void*)nxh, (void*)nxr, (void*)nx8,
                        (void*)nx8s, (void*)nx8r})
            if (p) (void)hipFree(p);
    };
    hipError_t e = hipMalloc((void**)&nxb, (size_t)ncap * ix->dp * sizeof(float));
    if (e == hipSuccess) e = hipMalloc((void**)&nxn, (size_t)ncap * sizeof(float));
    // the split copy exists only once a split-mode search has materialised it (ensure_split)
    if (e == hipSuccess && ix->xs) e = hipMalloc((void**)&nxs, (size_t)ncap * ix->dp * sizeof(uint32_t));
    if (e == hipSuccess && ix->b16_ok) e = hipMalloc((void**)&nxh, (size_t)ncap * ix->dpb * sizeof(uint16_t));
    if (e == hipSuccess && ix->b16_ok) e = hipMalloc((void**)&nxr, (size_t)ncap * sizeof(float));
    // the int8 copy exists only once a small-batch search has materialised it (ensure_i8)
    const size_t row8 = (size_t)i8_row_bytes(ix->nblk8);
    if (e == hipSuccess && ix->x8) e = hipMalloc((void**)&nx8, (size_t)ncap * row8);
    if (e == hipSuccess && ix->x8) e = hipMalloc((void**)&nx8s, (size_t)ncap * ix->nblk8 * sizeof(float));
    if (e == hipSuccess && ix->x8) e = hipMalloc((void**)&nx8r, (size_t)ncap * sizeof(float));
    if (e != hipSuccess) {
        release();
        (void)hipGetLastError();
        KNN_FAIL(KNN_ENOMEM, "hipMalloc of the %lld-row corpus buffers failed", (long long)ncap);
    }
    const size_t old = (size_t)ix->ntotal;
    auto copy_tail = [&](void* dst, const void* src, size_t row_bytes, size_t rows_cap) -> hipError_t {
        hipError_t r = hipSuccess;
        if (old && src) r = hipMemcpyAsync(dst, src, old * row_bytes, hipMemcpyDeviceToDevice, st);
        if (r == hipSuccess)
            r = hipMemsetAsync((char*)dst + old * row_bytes, 0, (rows_cap - old) * row_bytes, st);
        return r;
    };
    e = copy_tail(nxb, ix->xb, (size_t)ix->dp * sizeof(float), (size_t)ncap);
    if (e == hipSuccess) e = copy_tail(nxn, ix->xn, sizeof(float), (size_t)ncap);
    if (e == hipSuccess && nxs) e = copy_tail(nxs, ix->xs, (size_t)ix->dp * sizeof(uint32_t), (size_t)ncap);
    if (e == hipSuccess && nxh) e = copy_tail(nxh, ix->xh, (size_t)ix->dpb * sizeof(uint16_t), (size_t)ncap);
    if (e == hipSuccess && nxr) e = copy_tail(nxr, ix->xr, sizeof(float), (size_t)ncap);
    if (e == hipSuccess && nx8) e = copy_tail(nx8, ix->x8, row8, (size_t)ncap);
    if (e == hipSuccess && nx8s) e = copy_tail(nx8s, ix->x8s, (size_t)ix->nblk8 * sizeof(float), (size_t)ncap);
    if (e == hipSuccess && nx8r) e = copy_tail(nx8r, ix->x8r, sizeof(float), (size_t)ncap);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);
        release();
        KNN_FAIL(KNN_EHIP, "corpus regrowth failed: %s", hipGetErrorString(e));
    }
    for (void* p : {(void*)ix->xb, (void*)ix->xn, (void*)ix->xs, (void*)ix->xh, (void*)ix->xr,
                    (void*)ix->x8, (void*)ix->x8s, (void*)ix->x8r})
        if (p) (void)hipFree(p);
    ix->x8 = nx8;
    ix->x8s = nx8s;
    ix->x8r = nx8r;
    ix->xb = nxb;
    ix->xn = nxn;
    ix->xs = nxs;
    ix->xh = nxh;
    ix->xr = nxr;
    ix->cap = ncap;
    return KNN_OK;
}

int add_device_locked(knn_index* ix, const float* x, int64_t n, hipStream_t st) {
    if ((int64_t)(ix->ntotal + n) > (int64_t)INT32_MAX)
        KNN_FAIL(KNN_EINVAL, "a single index shard holds at most 2^31-1 rows");
    int rc = reserve_rows(ix, ix->ntotal + n, st);
    if (rc != KNN_OK) return rc;
    KNN_HIP(launch_rows_ingest(x, n, ix->d, ix->dp, n, ix->metric == KNN_METRIC_COSINE ? 1 : 0,
                               ix->xb + (size_t)ix->ntotal * ix->dp, ix->xn + ix->ntotal, st));
    if (ix->xs)
        KNN_HIP(launch_split_rows(ix->xb + (size_t)ix->ntotal * ix->dp, n, ix->dp, kSplitBK,
                                  ix->xs + (size_t)ix->ntotal * ix->dp, st));
    if (ix->b16_ok)
        KNN_HIP(launch_bf16_rows(ix->xb + (size_t)ix->ntotal * ix->dp, n, ix->dp, ix->dpb,
                                 ix->xh + (size_t)ix->ntotal * ix->dpb, ix->xr + ix->ntotal, st));
    if (ix->x8)
        KNN_HIP(launch_i8_rows(ix->xb + (size_t)ix->ntotal * ix->dp, n, ix->dp, ix->nblk8,
                               ix->x8 + (size_t)ix->ntotal * i8_row_bytes(ix->nblk8),
                               ix->x8s + (size_t)ix->ntotal * ix->nblk8, ix->x8r + ix->ntotal, st));
    ix->ntotal += n;
    ix->xn_max_stale = true;
    return KNN_OK;
}

// The split-bf16 copy (cap x dp words, as many bytes as the fp32 rows) is built on the first
// search that runs the split path, from the stored fp32 rows, and kept up to date by later adds.
// AUTO never takes the split path while the bf16 copy exists (every d >= 64), so a default index
// holds only the fp32 rows, norms and the bf16 copy: 12 GB instead of 20 GB per 1M x 1968 rows.
int ensure_split(knn_index* ix, hipStream_t st) {
    if (ix->xs) return KNN_OK;
    if (!ix->split_ok) KNN_FAIL(KNN_EINVAL, "split search needs d >= 256; d = %d", ix->d);
    uint32_t* xs = nullptr;
    if (hipMalloc((void**)&xs, (size_t)std::max<int64_t>(ix->cap, 1) * ix->dp * sizeof(uint32_t)) != hipSuccess) {
        (void)hipGetLastError();
        KNN_FAIL(KNN_ENOMEM, "hipMalloc of the %lld-row split copy failed", (long long)ix->cap);
    }
    ix->xs = xs;
    if (ix->ntotal > 0)
        KNN_HIP(launch_split_rows(ix->xb, ix->ntotal, ix->dp, kSplitBK, ix->xs, st));
    return KNN_OK;
}

// The block-scaled int8 copy (i8_row_bytes(nblk8) + nblk8 scales + one residual per row, about half
// the bf16 copy) is built on the first search that runs the int8 small-batch path, from the stored
// fp32 rows, and kept up to date by later adds (the split copy's pattern).
int ensure_i8(knn_index* ix, hipStream_t st) {
    if (ix->x8) return KNN_OK;
    if (ix->nblk8 <= 0) KNN_FAIL(KNN_EINVAL, "int8 search needs 64 <= d <= 4096; d = %d", ix->d);
    const size_t cap = (size_t)std::max<int64_t>(ix->cap, 1);
    int8_t* x8 = nullptr;
    float* x8s = nullptr;
    float* x8r = nullptr;
    hipError_t e = hipMalloc((void**)&x8, cap * (size_t)i8_row_bytes(ix->nblk8));
    if (e == hipSuccess) e = hipMalloc((void**)&x8s, cap * ix->nblk8 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc((void**)&x8r, cap * sizeof(float));
    if (e != hipSuccess) {
        for (void* p : {(void*)x8, (void*)x8s, (void*)x8r})
            if (p) (void)hipFree(p);
        (void)hipGetLastError();
        KNN_FAIL(KNN_ENOMEM, "hipMalloc of the %lld-row int8 copy failed", (long long)ix->cap);
    }
    ix->x8 = x8;
    ix->x8s = x8s;
    ix->x8r = x8r;
    ix->xn_max_stale = true;             // refresh_maxima computes the int8 residual maximum
    if (ix->ntotal > 0)
        KNN_HIP(launch_i8_rows(ix->xb, ix->ntotal, ix->dp, ix->nblk8, ix->x8, ix->x8s, ix->x8r, st));
    return KNN_OK;
}

int create_single(int d, int metric, int device, knn_index** out) {
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        KNN_FAIL(KNN_ENOSYS, "no HIP device visible");
    if (device < 0) KNN_HIP(hipGetDevice(&device));
    if (device >= ndev) KNN_FAIL(KNN_EINVAL, "device %d out of range (%d visible)", device, ndev);
    DeviceGuard g(device);
    knn_index* ix = new knn_index();
    ix->d = d;
    // rows padded to 16 floats; from d >= 256 to 32, so the 32-deep staging path and the split
    // copy (32-float stages) serve every d the split path takes
    ix->dp = (int)round_up(d, d >= 256 ? 2 * kDepthPad : kDepthPad);
    ix->metric = metric;
    ix->device = device;
    ix->split_ok = ix->dp % 32 == 0 && d >= 256;
    ix->b16_ok = d >= 64;
    ix->dpb = (int)round_up(d, kB16Pad);
    ix->nblk8 = d >= 64 && d <= 4096 ? (d + 63) / 64 : 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        ix->cus = cus;
    // IMGREC_CUS=n (tests): plan launches for n CUs, as on a partitioned device (CPX mode)
    if (const char* e = test_knob("IMGREC_CUS")) {
        const int v = std::atoi(e);
        if (v > 0 && v < ix->cus) ix->cus = v;
    }
    if (const char* e = test_knob("IMGREC_I8_WGPCU")) {
        const int v = std::atoi(e);
        if (v > 0 && v <= 16) ix->i8_wgpcu = v;
    }
    if (const char* e = test_knob("IMGREC_MERGE_FUSE")) {
        ix->merge_fuse = *e != '0';
        ix->merge_fuse1 = *e != '0' && *e != '1';
    }
    if (const char* e = test_knob("IMGREC_CHANCE_SKIP")) ix->chance_skip = *e != '0';
    if (const char* e = test_knob("IMGREC_CHANCE_DIRECT")) ix->chance_direct_max = std::max(0, std::atoi(e));
    if (const char* e = test_knob("IMGREC_I8_HALF_K")) {
        const int v = std::atoi(e);
        ix->i8_half_k = v >= 2 ? v : 0;
    }
    if (const char* e = test_knob("IMGREC_I8_POOL")) {
        ix->i8_pool64 = std::min(64, std::max(0, std::atoi(e)));
        ix->i8_pool_forced = true;
    }
    if (const char* e = test_knob("IMGREC_I8_POOL_CH")) ix->i8_pool_ch = std::min(64, std::max(1, std::atoi(e)));
    if (const char* e = test_knob("IMGREC_DIRECT_RAW")) ix->direct_raw = std::min(2, std::max(0, std::atoi(e)));
    if (const char* e = test_knob("IMGREC_I8_FUSED_PREP")) ix->i8_fused_prep = *e != '0';
    if (const char* e = test_knob("IMGREC_RERANK_P1")) ix->rerank_p1k = *e != '0';
    if (const char* e = test_knob("IMGREC_RERANK_NW4")) ix->rerank_nw4 = *e != '0';
    if (const char* e = test_knob("IMGREC_MERGE_SINGLE")) ix->merge_single = *e != '0';
    if (const char* e = test_knob("IMGREC_STREAM_LISTS")) ix->stream_lists = *e != '0';
    if (hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ix->fence, hipEventDisableTiming) != hipSuccess) {
        if (ix->stream) (void)hipStreamDestroy(ix->stream);
        delete ix;
        KNN_FAIL(KNN_EHIP, "hipStreamCreate / hipEventCreate failed");
    }
    *out = ix;
    return KNN_OK;
}

void free_single(knn_index* ix) {
    DeviceGuard g(ix->device);
    (void)hipDeviceSynchronize();       // searches on other streams may still use the buffers
    for (void* p : {(void*)ix->x8, (void*)ix->x8s, (void*)ix->x8r, (void*)ix->x8r_max,
                    (void*)ix->q8, (void*)ix->q8s, (void*)ix->q8r})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)ix->pq, (void*)ix->pd, (void*)ix->pi})
        if (p) (void)hipHostFree(p);
    for (void* p : {(void*)ix->xh, (void*)ix->xr, (void*)ix->xr_max, (void*)ix->qb16,
                    (void*)ix->q_resid, (void*)ix->floor, (void*)ix->mws_d, (void*)ix->mws_i,
                    (void*)ix->mws_f, (void*)ix->stat, (void*)ix->fb_cd, (void*)ix->fb_ci,
                    (void*)ix->b16_sync,
                    (void*)ix->tail_ctl, (void*)ix->chance, (void*)ix->sc_key, (void*)ix->sc_lab,
                    (void*)ix->sc_meta, (void*)ix->sc_done, (void*)ix->heads, (void*)ix->i8_dyn})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)ix->xb, (void*)ix->xn, (void*)ix->xs, (void*)ix->xn_max,
                    (void*)ix->qpad, (void*)ix->qnorm, (void*)ix->cand_d, (void*)ix->cand_i,
                    (void*)ix->qsplit, (void*)ix->cand2_d, (void*)ix->cand2_i, (void*)ix->fail,
                    (void*)ix->fb_q, (void*)ix->fb_qn, (void*)ix->hq, (void*)ix->hd, (void*)ix->hi})
        if (p) (void)hipFree(p);
    largek_free(ix);
    hugek_free(ix);
    for (hipEvent_t e : ix->ev) (void)hipEventDestroy(e);
    if (ix->fence) (void)hipEventDestroy(ix->fence);
    (void)hipStreamDestroy(ix->stream);
    delete ix;
}

int set_metric(knn_index* ix, int metric) {
    if (ix->multi) return multi_set_metric(ix, metric);
    ix->metric = metric;
    return KNN_OK;
}

int set_trained(knn_index* ix, bool trained) {
    ix->trained = trained;
    if (ix->multi) return multi_set_trained(ix, trained);
    return KNN_OK;
}

}  // namespace imgrec

using namespace imgrec;

extern "C" {

const char* knn_last_error(void) { return imgrec::last_error(); }
const char* knn_version(void) {
    return "imgrec-knn 0.2 (gfx950: bf16 / split-bf16 / f32 MFMA candidates, fused top-k, "
           "device-side certificate)";
}

int knn_create(int d, int metric, int device, knn_index_t** out) {
    if (!out) KNN_FAIL(KNN_EINVAL, "out is NULL");
    *out = nullptr;
    if (d <= 0) KNN_FAIL(KNN_EINVAL, "d must be positive (got %d)", d);
    if (metric != KNN_METRIC_L2 && metric != KNN_METRIC_IP && metric != KNN_METRIC_COSINE)
        KNN_FAIL(KNN_EINVAL, "unknown metric %d", metric);
    return create_single(d, metric, device, out);
}

int knn_free(knn_index_t* ix) {
    if (!ix) return KNN_OK;
    if (ix->multi) return multi_free(ix);
    free_single(ix);
    return KNN_OK;
}

int knn_dim(const knn_index_t* ix) { return ix ? ix->d : KNN_EINVAL; }
int knn_metric(const knn_index_t* ix) { return ix ? ix->metric : KNN_EINVAL; }
int64_t knn_ntotal(const knn_index_t* ix) { return ix ? ix->ntotal : KNN_EINVAL; }
int knn_is_trained(const knn_index_t* ix) { return ix ? (ix->trained ? 1 : 0) : KNN_EINVAL; }

int knn_set_id_offset(knn_index_t* ix, int64_t off) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    std::lock_guard<std::mutex> lk(ix->mu);
    ix->id_offset = off;
    return KNN_OK;
}

int knn_train(knn_index_t* ix, const float* x, int64_t n) {
    (void)x;
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0) KNN_FAIL(KNN_EINVAL, "n must be >= 0");
    return set_trained(ix, true);
}

int knn_reserve(knn_index_t* ix, int64_t n) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (ix->multi) return multi_reserve(ix, n);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    if ((rc = reserve_rows(ix, n, ix->stream)) != KNN_OK) return rc;
    return fence_end(ix, ix->stream);
}

int knn_add_device(knn_index_t* ix, const float* x, int64_t n, void* stream) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0 || (n > 0 && !x)) KNN_FAIL(KNN_EINVAL, "bad rows (n=%lld)", (long long)n);
    if (n == 0) return KNN_OK;
    if (ix->multi) return multi_add_device(ix, x, n, (hipStream_t)stream);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    const hipStream_t st = (hipStream_t)stream;
    int rc;
    if ((rc = fence_begin(ix, st)) != KNN_OK) return rc;
    if ((rc = add_device_locked(ix, x, n, st)) != KNN_OK) return rc;
    return fence_end(ix, st);
}

int knn_add(knn_index_t* ix, const float* x, int64_t n) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (n < 0 || (n > 0 && !x)) KNN_FAIL(KNN_EINVAL, "bad rows (n=%lld)", (long long)n);
    if (n == 0) return KNN_OK;
    if (ix->multi) return multi_add(ix, x, n);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    if ((rc = reserve_rows(ix, ix->ntotal + n, ix->stream)) != KNN_OK) return rc;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64 << 20) / ((int64_t)ix->d * 4));
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
        const int64_t cn = std::min(chunk, n - r0);
        if ((rc = grow(&ix->hq, &ix->hq_cap, (size_t)cn * ix->d)) != KNN_OK) return rc;
        KNN_HIP(hipMemcpyAsync(ix->hq, x + r0 * ix->d, (size_t)cn * ix->d * sizeof(float),
                               hipMemcpyHostToDevice, ix->stream));
        if ((rc = add_device_locked(ix, ix->hq, cn, ix->stream)) != KNN_OK) return rc;
        KNN_HIP(hipStreamSynchronize(ix->stream));
    }
    return fence_end_synced(ix);
}

int knn_reset(knn_index_t* ix) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (ix->multi) return multi_reset(ix);
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
    if (ix->multi) return multi_reconstruct_n(ix, i0, n, x);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpy2DAsync(x, (size_t)ix->d * 4, ix->xb + (size_t)i0 * ix->dp, (size_t)ix->dp * 4,
                             (size_t)ix->d * 4, (size_t)n, hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    return fence_end_synced(ix);
}

int knn_search_device(knn_index_t* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                      void* stream) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (k <= 0) KNN_FAIL(KNN_EINVAL, "k must be >= 1 (got %d)", k);
    if (nq < 0 || (nq > 0 && (!q || !D || !I))) KNN_FAIL(KNN_EINVAL, "bad query/output pointers");
    if (nq == 0) return KNN_OK;
    if (ix->multi) return multi_search_device(ix, q, nq, k, D, I, (hipStream_t)stream);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    const hipStream_t st = (hipStream_t)stream;
    int rc;
    if ((rc = fence_begin(ix, st)) != KNN_OK) return rc;
    if ((rc = search_locked(ix, q, nq, k, D, I, st)) != KNN_OK) return rc;
    return fence_end(ix, st);
}

// Page-locked host buffer that only grows (the host-pointer search's staging for small batches).
static int grow_pinned(void** p, size_t* cap, size_t need_bytes) {
    if (*cap >= need_bytes) return KNN_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    KNN_HIP(hipHostMalloc(p, need_bytes, hipHostMallocDefault));
    *cap = need_bytes;
    return KNN_OK;
}

// Batches whose query rows fit this many bytes go through page-locked staging: a pageable copy
// is a driver-staged, host-synchronous transfer on each side of a one-query search (round 1
// measured 47 us of PCIe-side overhead per one-query search), while a memcpy of a few KB into a
// pinned buffer and one DMA each way are a few us.  Larger batches copy pageable memory directly.
constexpr size_t kPinnedSearchBytes = 1 << 20;

int knn_search(knn_index_t* ix, const float* q, int64_t nq, int k, float* D, int64_t* I) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (k <= 0) KNN_FAIL(KNN_EINVAL, "k must be >= 1 (got %d)", k);
    if (nq < 0 || (nq > 0 && (!q || !D || !I))) KNN_FAIL(KNN_EINVAL, "bad query/output pointers");
    if (nq == 0) return KNN_OK;
    if (ix->multi) return multi_search(ix, q, nq, k, D, I);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hq, &ix->hq_cap, (size_t)nq * ix->d)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hd, &ix->hd_cap, (size_t)nq * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hi, &ix->hi_cap, (size_t)nq * k)) != KNN_OK) return rc;
    const size_t qbytes = (size_t)nq * ix->d * sizeof(float);
    const bool pinned = qbytes <= kPinnedSearchBytes;
    if (pinned) {
        if ((rc = grow_pinned((void**)&ix->pq, &ix->pq_cap, qbytes)) != KNN_OK) return rc;
        if ((rc = grow_pinned((void**)&ix->pd, &ix->pd_cap, (size_t)nq * k * sizeof(float))) != KNN_OK) return rc;
        if ((rc = grow_pinned((void**)&ix->pi, &ix->pi_cap, (size_t)nq * k * sizeof(int64_t))) != KNN_OK) return rc;
        // (the previous host-pointer search synchronised before returning: the buffers are free)
        std::memcpy(ix->pq, q, qbytes);
    }
    KNN_HIP(hipMemcpyAsync(ix->hq, pinned ? ix->pq : q, qbytes, hipMemcpyHostToDevice, ix->stream));
    if ((rc = search_locked(ix, ix->hq, nq, k, ix->hd, ix->hi, ix->stream)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpyAsync(pinned ? ix->pd : D, ix->hd, (size_t)nq * k * sizeof(float),
                           hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipMemcpyAsync(pinned ? ix->pi : I, ix->hi, (size_t)nq * k * sizeof(int64_t),
                           hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    if ((rc = fence_end_synced(ix)) != KNN_OK) return rc;
    if (pinned) {
        std::memcpy(D, ix->pd, (size_t)nq * k * sizeof(float));
        std::memcpy(I, ix->pi, (size_t)nq * k * sizeof(int64_t));
    }
    return KNN_OK;
}

int knn_merge_device(const float* cD, const int64_t* cI, int nlists, int64_t nq, int kin, int k,
                     int metric, float* D, int64_t* I, void* stream) {
    if (nlists <= 0 || kin <= 0 || nq < 0) KNN_FAIL(KNN_EINVAL, "bad merge shape");
    if (k <= 0) KNN_FAIL(KNN_EINVAL, "k must be >= 1 (got %d)", k);
    if (nq == 0) return KNN_OK;
    if (!cD || !cI || !D || !I) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    const int kmetric = metric == KNN_METRIC_L2 ? 1 : 0;
    if (k > KNN_MAX_K) {
        KNN_HIP(launch_merge_any(cD, cI, nlists, nq, kin, nq * (int64_t)kin, nq * (int64_t)kin, k,
                                 kmetric, D, I, (hipStream_t)stream));
        return KNN_OK;
    }
    KNN_HIP(launch_merge(cD, cI, nq, nlists, kin, kin, nq * (int64_t)kin, k, kmetric,
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
    if (k <= 0) KNN_FAIL(KNN_EINVAL, "k must be >= 1 (got %d)", k);
    if (nq == 0) return KNN_OK;
    if (!packed || !D || !I) KNN_FAIL(KNN_EINVAL, "NULL pointer");
    const int64_t n = nq * kin, nf = n + (n & 1);
    const float* cD = static_cast<const float*>(packed);
    const int64_t* cI = reinterpret_cast<const int64_t*>(static_cast<const char*>(packed) + nf * 4);
    const int kmetric = metric == KNN_METRIC_L2 ? 1 : 0;
    if (k > KNN_MAX_K) {
        KNN_HIP(launch_merge_any(cD, cI, nlists, nq, kin, nf + 2 * n, nf / 2 + n, k, kmetric, D, I,
                                 (hipStream_t)stream));
        return KNN_OK;
    }
    // chunk = nf floats + n int64: nf + 2n floats, nf / 2 + n int64
    KNN_HIP(launch_merge_strided(cD, cI, nq, nlists, kin, kin, nf + 2 * n, nf / 2 + n, k, kmetric,
                                 kmetric ? 0 : 1, D, I, (hipStream_t)stream));
    return KNN_OK;
}

int knn_set_timing(knn_index_t* ix, int enable) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (ix->multi) return multi_set_timing(ix, enable);
    std::lock_guard<std::mutex> lk(ix->mu);
    ix->timing = enable != 0;
    ix->ev_used = 0;
    return KNN_OK;
}

int knn_set_fence_mode(knn_index_t* ix, int mode) {
    if (!ix) KNN_FAIL(KNN_EINVAL, "index is NULL");
    if (mode != KNN_FENCE_EAGER && mode != KNN_FENCE_LAZY) KNN_FAIL(KNN_EINVAL, "unknown fence mode %d", mode);
    std::lock_guard<std::mutex> lk(ix->mu);
    if (ix->multi) {
        int rc = multi_set_fence_mode(ix, mode);
        if (rc != KNN_OK) return rc;
    }
    ix->fence_lazy = mode == KNN_FENCE_LAZY;
    return KNN_OK;
}

int knn_kernel_time(knn_index_t* ix, double* total_ms, int* launches) {
    if (!ix || !total_ms || !launches) KNN_FAIL(KNN_EINVAL, "NULL argument");
    if (ix->multi) return multi_kernel_time(ix, total_ms, launches);
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
        mode != KNN_SEARCH_BF16 && mode != KNN_SEARCH_I8)
        KNN_FAIL(KNN_EINVAL, "unknown search mode %d", mode);
    if (ix->multi) return multi_set_search_mode(ix, mode);
    std::lock_guard<std::mutex> lk(ix->mu);
    if (mode == KNN_SEARCH_SPLIT && !ix->split_ok)
        KNN_FAIL(KNN_EINVAL, "split search needs d >= 256; d = %d", ix->d);
    if (mode == KNN_SEARCH_BF16 && !ix->b16_ok)
        KNN_FAIL(KNN_EINVAL, "bf16 search needs d >= 64; d = %d", ix->d);
    if (mode == KNN_SEARCH_I8 && ix->nblk8 <= 0)
        KNN_FAIL(KNN_EINVAL, "int8 search needs 64 <= d <= 4096; d = %d", ix->d);
    ix->mode = mode;
    return KNN_OK;
}

int knn_search_stats(knn_index_t* ix, int64_t* split_queries, int64_t* fallback_queries,
                     float* max_err_ratio) {
    return knn_search_stats2(ix, split_queries, fallback_queries, nullptr, max_err_ratio);
}

int knn_search_stats2(knn_index_t* ix, int64_t* split_queries, int64_t* fallback_queries,
                      int64_t* second_chance_queries, float* max_err_ratio) {
    if (!ix || !split_queries || !fallback_queries) KNN_FAIL(KNN_EINVAL, "NULL argument");
    if (ix->multi)
        return multi_search_stats(ix, split_queries, fallback_queries, second_chance_queries,
                                  max_err_ratio);
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int64_t first_fail = 0;
    const int rc = read_search_stats(ix, split_queries, fallback_queries, &first_fail, max_err_ratio);
    if (second_chance_queries) *second_chance_queries = first_fail - *fallback_queries;
    return rc;
}

int knn_last_path(const knn_index_t* ix) {
    if (!ix) return KNN_EINVAL;
    return ix->multi ? multi_last_path(ix) : ix->last_path;
}

// The count lives on the device (the large-k search never waits for the GPU): reading it waits
// for the index's last operation.
static int large_k_fallbacks_one(knn_index* ix, int64_t* n) {
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    const int rc = largek_fallbacks(ix, n);
    if (rc != KNN_OK) return rc;
    return fence_end_synced(ix);
}

int knn_large_k_fallbacks(const knn_index_t* cix, int64_t* n) {
    if (!cix || !n) KNN_FAIL(KNN_EINVAL, "NULL argument");
    knn_index* ix = const_cast<knn_index*>(cix);     // (only the fence state changes)
    if (!ix->multi) return large_k_fallbacks_one(ix, n);
    *n = 0;
    for (int s = 0; s < multi_num_shards(ix); ++s) {
        int64_t v = 0;
        const int rc = large_k_fallbacks_one(const_cast<knn_index*>(multi_shard(ix, s)), &v);
        if (rc != KNN_OK) return rc;
        *n += v;
    }
    return KNN_OK;
}

int knn_plan(const knn_index_t* cix, int64_t nq, int k, int* tr, int* tq, int* splits, int* wgs) {
    if (!cix || !tr || !tq || !splits || !wgs) KNN_FAIL(KNN_EINVAL, "NULL argument");
    const knn_index* ix = cix->multi ? multi_shard(cix, 0) : cix;
    const int64_t cn = std::min(nq, kQueryChunk);
    const Plan p = use_i8(ix, cn, k) ? make_i8_plan(ix->ntotal, cn, k, ix->cus, ix->i8_wgpcu, ix->nblk8)
                 : use_b16(ix, cn, k) ? make_b16_plan(ix->ntotal, cn, k, ix->cus, ix->dpb)
                 : use_split(ix, cn, k) ? make_split_plan(ix->ntotal, cn, split_kc(k), ix->cus)
                                        : make_plan(ix->ntotal, cn, k, ix->cus);
    *tr = p.bm;
    *tq = p.bq;
    *splits = p.nsplit;
    *wgs = p.wgs;
    return KNN_OK;
}

int knn_plan_kernel(const knn_index_t* cix, int64_t nq, int k, char* name, int cap) {
    if (!cix || !name || cap < 1) KNN_FAIL(KNN_EINVAL, "NULL argument");
    const knn_index* ix = cix->multi ? multi_shard(cix, 0) : cix;
    const int64_t cn = std::min(nq, kQueryChunk);
    const int l2 = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    if (use_i8(ix, cn, k)) {
        const Plan p = make_i8_plan(ix->ntotal, cn, k, ix->cus, ix->i8_wgpcu, ix->nblk8);
        std::snprintf(name, cap, "knn_i8_scan_kernel<%d, %d, %d>", cn <= 2 ? (int)cn : (cn <= 4 ? 4 : 8), p.km,
                      (ix->nblk8 + 15) / 16);
    } else if (use_b16(ix, cn, k)) {
        const Plan p = make_b16_plan(ix->ntotal, cn, k, ix->cus, ix->dpb);
        if (p.big && IMGREC_B16_MFMA16)
            std::snprintf(name, cap, "knn_b16w_tile_kernel<%d, %d, %s>", p.km, l2, p.ib > 0 ? "true" : "false");
        else if (p.big)
            std::snprintf(name, cap, "knn_b16_tile_kernel<%d, %d>", p.km, l2);
        else
            std::snprintf(name, cap, "knn_tile_topk_kernel<%d, %d, ..., %d, ...>", p.wr, p.wq, kModeBF16);
    } else if (use_split(ix, cn, k)) {
        const Plan p = make_split_plan(ix->ntotal, cn, split_kc(k), ix->cus);
        std::snprintf(name, cap, "knn_tile_topk_kernel<%d, %d, ..., %d, ...>", p.wr, p.wq, kModeSplit);
    } else {
        const Plan p = make_plan(ix->ntotal, cn, k, ix->cus);
        std::snprintf(name, cap, "knn_tile_topk_kernel<%d, %d, ..., %d, ...>", p.wr, p.wq, kModeF32);
    }
    return KNN_OK;
}

}  // extern "C"
