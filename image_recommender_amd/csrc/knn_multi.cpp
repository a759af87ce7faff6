// knn_multi.cpp — one k-NN index over several HIP devices of one process (include/imgrec_knn.h
// knn_create_multi).  The reference's CLI is single-process (/root/reference/main/
// search_from_image.py:430-441, main/create_index.py:327-341), so this is how its own entry
// points use every GPU of a node without torchrun: the faiss-compatible index object is the same,
// its corpus lives in per-device row shards.
//
// Layout: every add of n rows is cut into ndev contiguous pieces, piece s appended to shard s;
// a shard keeps, per local row, its global label (device array `lmap`), so labels stay the
// reference's dense offsets whatever the add sizes.  Within a shard global labels grow with local
// rows, so a shard's (key, local row) order is the (key, label) order of the whole index.
//
// Search: the query batch reaches every shard's device (peer copy; none when the shard shares the
// first device), each shard runs the single-device search on its own stream concurrently, maps
// its labels, and its (nq, k) result lands in a [ndev][nq][k] gather buffer on the first device
// (peer copy over xGMI), where knn_merge's kernel produces the final rows.  The same shard merge as
// the torchrun path (sharded.py), with device-to-device copies instead of an RCCL all-gather.
#include <cstdlib>
#include <cstring>

#include "knn_multi.h"

struct knn_multi {
    std::vector<knn_index*> shards;
    std::vector<int> devices;
    struct Run { int64_t g0; int shard; int64_t l0; int64_t n; };
    std::vector<Run> runs;                       // global row ranges in increasing order
    std::vector<int64_t*> lmap;                  // per shard (its device): local row -> label
    std::vector<size_t> lmap_cap;
    std::vector<float*> sq;                      // per shard: query copy (other devices only)
    std::vector<size_t> sq_cap;
    std::vector<float*> sd;                      // per shard: results (other devices only)
    std::vector<size_t> sd_cap;
    std::vector<int64_t*> si;
    std::vector<size_t> si_cap;
    std::vector<float*> sx;                      // per shard: row staging for add_device
    std::vector<size_t> sx_cap;
    std::vector<hipEvent_t> done;                // per shard (its device)
    hipEvent_t ready = nullptr;                  // inputs ready on the first device
    // IMGREC_MULTI_FORCE_REMOTE=1 (tests): shards on the first device take the other devices'
    // staging + peer-copy path too, so one GPU exercises it
    bool force_remote = false;
    float* gD = nullptr; size_t gD_cap = 0;      // [ndev][nq][k] on the first device
    int64_t* gI = nullptr; size_t gI_cap = 0;
};

namespace imgrec {

namespace {

knn_multi* M(const knn_index* ix) { return ix->multi; }

// shard s's piece of an add of n rows
inline int64_t piece0(int64_t n, int s, int ndev) { return n * s / ndev; }

// a label map that keeps its entries when it grows
int grow_keep(int64_t** p, size_t* cap, size_t need, hipStream_t st) {
    if (*cap >= need) return KNN_OK;
    const size_t n = std::max(need, *cap * 3 / 2);
    int64_t* np = nullptr;
    KNN_HIP(hipMalloc((void**)&np, n * sizeof(int64_t)));
    if (*p) {
        const hipError_t e = hipMemcpyAsync(np, *p, *cap * sizeof(int64_t), hipMemcpyDeviceToDevice, st);
        const hipError_t e2 = e == hipSuccess ? hipStreamSynchronize(st) : e;
        if (e2 != hipSuccess) {
            (void)hipFree(np);
            KNN_FAIL(KNN_EHIP, "label map regrowth failed: %s", hipGetErrorString(e2));
        }
        (void)hipFree(*p);
    }
    *p = np;
    *cap = n;
    return KNN_OK;
}

int append_runs(knn_index* ix, const std::vector<int64_t>& before, int64_t n) {
    knn_multi* m = M(ix);
    const int ndev = (int)m->shards.size();
    for (int s = 0; s < ndev; ++s) {
        const int64_t r0 = piece0(n, s, ndev), r1 = piece0(n, s + 1, ndev);
        if (r1 <= r0) continue;
        m->runs.push_back({ix->ntotal + r0, s, before[s], r1 - r0});
        knn_index* sh = m->shards[s];
        DeviceGuard g(sh->device);
        int rc;
        // lmap grows with the shard's capacity; rows already mapped keep their labels
        if ((rc = grow_keep(&m->lmap[s], &m->lmap_cap[s], (size_t)sh->cap, sh->stream)) != KNN_OK)
            return rc;
        KNN_HIP(launch_iota64(m->lmap[s] + before[s], r1 - r0, ix->ntotal + r0, sh->stream));
        KNN_HIP(hipStreamSynchronize(sh->stream));
    }
    ix->ntotal += n;
    return KNN_OK;
}

}  // namespace

int multi_create(int d, int metric, const int* devices, int ndev, knn_index** out) {
    *out = nullptr;
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible <= 0)
        KNN_FAIL(KNN_ENOSYS, "no HIP device visible");
    for (int s = 0; s < ndev; ++s)
        if (devices[s] < 0 || devices[s] >= visible)
            KNN_FAIL(KNN_EINVAL, "device %d out of range (%d visible)", devices[s], visible);
    knn_index* ix = nullptr;
    int rc = create_single(d, metric, devices[0], &ix);
    if (rc != KNN_OK) return rc;
    knn_multi* m = new knn_multi();
    ix->multi = m;
    m->devices.assign(devices, devices + ndev);
    if (const char* e = std::getenv("IMGREC_MULTI_FORCE_REMOTE")) m->force_remote = std::atoi(e) != 0;
    m->lmap.assign(ndev, nullptr);
    m->lmap_cap.assign(ndev, 0);
    m->sq.assign(ndev, nullptr);
    m->sq_cap.assign(ndev, 0);
    m->sd.assign(ndev, nullptr);
    m->sd_cap.assign(ndev, 0);
    m->si.assign(ndev, nullptr);
    m->si_cap.assign(ndev, 0);
    m->sx.assign(ndev, nullptr);
    m->sx_cap.assign(ndev, 0);
    m->done.assign(ndev, nullptr);
    {
        DeviceGuard g(ix->device);
        if (hipEventCreateWithFlags(&m->ready, hipEventDisableTiming) != hipSuccess) {
            multi_free(ix);
            KNN_FAIL(KNN_EHIP, "hipEventCreate failed");
        }
    }
    for (int s = 0; s < ndev; ++s) {
        knn_index* sh = nullptr;
        if ((rc = create_single(d, metric, devices[s], &sh)) != KNN_OK) {
            multi_free(ix);
            return rc;
        }
        m->shards.push_back(sh);
        DeviceGuard g(devices[s]);
        if (hipEventCreateWithFlags(&m->done[s], hipEventDisableTiming) != hipSuccess) {
            multi_free(ix);
            KNN_FAIL(KNN_EHIP, "hipEventCreate failed");
        }
        // peer access between the first device and every other (xGMI); already enabled or
        // unsupported is not an error here: peer copies then stage through the runtime
        if (devices[s] != devices[0]) {
            (void)hipDeviceEnablePeerAccess(devices[0], 0);
            DeviceGuard g0(devices[0]);
            (void)hipDeviceEnablePeerAccess(devices[s], 0);
            (void)hipGetLastError();
        }
    }
    *out = ix;
    return KNN_OK;
}

int multi_free(knn_index* ix) {
    knn_multi* m = M(ix);
    for (size_t s = 0; s < m->devices.size(); ++s) {
        DeviceGuard g(m->devices[s]);
        (void)hipDeviceSynchronize();
        for (void* p : {(void*)m->lmap[s], (void*)m->sq[s], (void*)m->sd[s], (void*)m->si[s],
                        (void*)m->sx[s]})
            if (p) (void)hipFree(p);
        if (m->done[s]) (void)hipEventDestroy(m->done[s]);
    }
    for (knn_index* sh : m->shards) free_single(sh);
    {
        DeviceGuard g(ix->device);
        if (m->gD) (void)hipFree(m->gD);
        if (m->gI) (void)hipFree(m->gI);
        if (m->ready) (void)hipEventDestroy(m->ready);
    }
    delete m;
    ix->multi = nullptr;
    free_single(ix);
    return KNN_OK;
}

int multi_reserve(knn_index* ix, int64_t n) {
    knn_multi* m = M(ix);
    std::lock_guard<std::mutex> lk(ix->mu);
    const int ndev = (int)m->shards.size();
    for (int s = 0; s < ndev; ++s) {
        // later adds are cut evenly: shard s ends up with about n / ndev rows
        int rc = knn_reserve(m->shards[s], (n + ndev - 1) / ndev + 1);
        if (rc != KNN_OK) return rc;
    }
    return KNN_OK;
}

int multi_add(knn_index* ix, const float* x, int64_t n) {
    knn_multi* m = M(ix);
    std::lock_guard<std::mutex> lk(ix->mu);
    const int ndev = (int)m->shards.size();
    std::vector<int64_t> before(ndev);
    for (int s = 0; s < ndev; ++s) {
        before[s] = m->shards[s]->ntotal;
        const int64_t r0 = piece0(n, s, ndev), r1 = piece0(n, s + 1, ndev);
        if (r1 <= r0) continue;
        int rc = knn_add(m->shards[s], x + r0 * ix->d, r1 - r0);
        if (rc != KNN_OK) return rc;
    }
    return append_runs(ix, before, n);
}

int multi_add_device(knn_index* ix, const float* x, int64_t n, hipStream_t st) {
    knn_multi* m = M(ix);
    std::lock_guard<std::mutex> lk(ix->mu);
    const int ndev = (int)m->shards.size();
    int rc;
    {
        DeviceGuard g(ix->device);
        KNN_HIP(hipEventRecord(m->ready, st));       // the rows are written on the caller's stream
    }
    std::vector<int64_t> before(ndev);
    for (int s = 0; s < ndev; ++s) {
        knn_index* sh = m->shards[s];
        before[s] = sh->ntotal;
        const int64_t r0 = piece0(n, s, ndev), r1 = piece0(n, s + 1, ndev);
        if (r1 <= r0) continue;
        const float* src = x + r0 * ix->d;
        if (sh->device == ix->device && !m->force_remote) {
            if ((rc = knn_add_device(sh, src, r1 - r0, st)) != KNN_OK) return rc;
            continue;
        }
        DeviceGuard g(sh->device);
        const size_t bytes = (size_t)(r1 - r0) * ix->d * sizeof(float);
        if ((rc = grow(&m->sx[s], &m->sx_cap[s], (size_t)(r1 - r0) * ix->d)) != KNN_OK) return rc;
        KNN_HIP(hipStreamWaitEvent(sh->stream, m->ready, 0));
        KNN_HIP(hipMemcpyPeerAsync(m->sx[s], sh->device, src, ix->device, bytes, sh->stream));
        if ((rc = knn_add_device(sh, m->sx[s], r1 - r0, sh->stream)) != KNN_OK) return rc;
        // the caller may reuse x once its stream passes this point
        KNN_HIP(hipEventRecord(m->done[s], sh->stream));
        KNN_HIP(hipStreamWaitEvent(st, m->done[s], 0));
    }
    return append_runs(ix, before, n);
}

int multi_reset(knn_index* ix) {
    knn_multi* m = M(ix);
    std::lock_guard<std::mutex> lk(ix->mu);
    for (knn_index* sh : m->shards) {
        int rc = knn_reset(sh);
        if (rc != KNN_OK) return rc;
    }
    m->runs.clear();
    ix->ntotal = 0;
    return KNN_OK;
}

int multi_reconstruct_n(knn_index* ix, int64_t i0, int64_t n, float* x) {
    knn_multi* m = M(ix);
    std::lock_guard<std::mutex> lk(ix->mu);
    const int64_t i1 = i0 + n;
    for (const auto& r : m->runs) {
        const int64_t a = std::max(i0, r.g0), b = std::min(i1, r.g0 + r.n);
        if (a >= b) continue;
        int rc = knn_reconstruct_n(m->shards[r.shard], r.l0 + (a - r.g0), b - a, x + (a - i0) * ix->d);
        if (rc != KNN_OK) return rc;
    }
    return KNN_OK;
}

namespace {

// Every shard searches q (device pointer on the first device, ready when m->ready fires) into the
// gather buffer; the first device's stream `st` then merges into D, I.
int fan_out_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                   hipStream_t st) {
    knn_multi* m = M(ix);
    const int ndev = (int)m->shards.size();
    const size_t nk = (size_t)nq * k;
    int rc;
    {
        DeviceGuard g(ix->device);
        if ((rc = grow(&m->gD, &m->gD_cap, nk * ndev)) != KNN_OK) return rc;
        if ((rc = grow(&m->gI, &m->gI_cap, nk * ndev)) != KNN_OK) return rc;
        KNN_HIP(hipEventRecord(m->ready, st));
    }
    for (int s = 0; s < ndev; ++s) {
        knn_index* sh = m->shards[s];
        const bool local = sh->device == ix->device && !m->force_remote;
        DeviceGuard g(sh->device);
        std::lock_guard<std::mutex> lk(sh->mu);
        const hipStream_t ss = sh->stream;
        KNN_HIP(hipStreamWaitEvent(ss, m->ready, 0));
        if ((rc = fence_begin(sh, ss)) != KNN_OK) return rc;
        const float* qs = q;
        float* ds = m->gD + s * nk;
        int64_t* is = m->gI + s * nk;
        if (!local) {
            if ((rc = grow(&m->sq[s], &m->sq_cap[s], (size_t)nq * ix->d)) != KNN_OK) return rc;
            if ((rc = grow(&m->sd[s], &m->sd_cap[s], nk)) != KNN_OK) return rc;
            if ((rc = grow(&m->si[s], &m->si_cap[s], nk)) != KNN_OK) return rc;
            KNN_HIP(hipMemcpyPeerAsync(m->sq[s], sh->device, q, ix->device,
                                       (size_t)nq * ix->d * sizeof(float), ss));
            qs = m->sq[s];
            ds = m->sd[s];
            is = m->si[s];
        }
        if ((rc = search_locked(sh, qs, nq, k, ds, is, ss)) != KNN_OK) return rc;
        KNN_HIP(launch_map_labels(is, (int64_t)nk, m->lmap[s], ix->id_offset, ss));
        if (!local) {
            KNN_HIP(hipMemcpyPeerAsync(m->gD + s * nk, ix->device, ds, sh->device,
                                       nk * sizeof(float), ss));
            KNN_HIP(hipMemcpyPeerAsync(m->gI + s * nk, ix->device, is, sh->device,
                                       nk * sizeof(int64_t), ss));
        }
        if ((rc = fence_end(sh, ss)) != KNN_OK) return rc;
        KNN_HIP(hipEventRecord(m->done[s], ss));
    }
    DeviceGuard g(ix->device);
    for (int s = 0; s < ndev; ++s) KNN_HIP(hipStreamWaitEvent(st, m->done[s], 0));
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    if (k > KNN_MAX_K) {
        KNN_HIP(launch_merge_any(m->gD, m->gI, ndev, nq, k, (int64_t)nk, (int64_t)nk, k, kmetric, D, I, st));
        return KNN_OK;
    }
    KNN_HIP(launch_merge(m->gD, m->gI, nq, ndev, k, k, (int64_t)nk, k, kmetric, kmetric ? 0 : 1, D, I,
                         st));
    return KNN_OK;
}

}  // namespace

int multi_search_device(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                        hipStream_t st) {
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, st)) != KNN_OK) return rc;
    if (ix->ntotal == 0) {
        KNN_HIP(launch_fill_empty(D, I, nq * (int64_t)k, ix->metric == KNN_METRIC_L2 ? 1 : 0, st));
        return fence_end(ix, st);
    }
    if ((rc = fan_out_search(ix, q, nq, k, D, I, st)) != KNN_OK) return rc;
    return fence_end(ix, st);
}

int multi_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I) {
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hq, &ix->hq_cap, (size_t)nq * ix->d)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hd, &ix->hd_cap, (size_t)nq * k)) != KNN_OK) return rc;
    if ((rc = grow(&ix->hi, &ix->hi_cap, (size_t)nq * k)) != KNN_OK) return rc;
    KNN_HIP(hipMemcpyAsync(ix->hq, q, (size_t)nq * ix->d * sizeof(float), hipMemcpyHostToDevice,
                           ix->stream));
    if (ix->ntotal == 0) {
        KNN_HIP(launch_fill_empty(ix->hd, ix->hi, nq * (int64_t)k,
                                  ix->metric == KNN_METRIC_L2 ? 1 : 0, ix->stream));
    } else if ((rc = fan_out_search(ix, ix->hq, nq, k, ix->hd, ix->hi, ix->stream)) != KNN_OK) {
        return rc;
    }
    KNN_HIP(hipMemcpyAsync(D, ix->hd, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost,
                           ix->stream));
    KNN_HIP(hipMemcpyAsync(I, ix->hi, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost,
                           ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    return fence_end_synced(ix);
}

int multi_set_metric(knn_index* ix, int metric) {
    ix->metric = metric;
    for (knn_index* sh : M(ix)->shards) sh->metric = metric;
    return KNN_OK;
}

int multi_set_trained(knn_index* ix, bool trained) {
    for (knn_index* sh : M(ix)->shards) sh->trained = trained;
    ix->trained = trained;
    return KNN_OK;
}

int multi_set_timing(knn_index* ix, int enable) {
    for (knn_index* sh : M(ix)->shards) {
        int rc = knn_set_timing(sh, enable);
        if (rc != KNN_OK) return rc;
    }
    return KNN_OK;
}

int multi_kernel_time(knn_index* ix, double* total_ms, int* launches) {
    double tot = 0.0;
    int n = 0;
    for (knn_index* sh : M(ix)->shards) {
        double t = 0.0;
        int l = 0;
        int rc = knn_kernel_time(sh, &t, &l);
        if (rc != KNN_OK) return rc;
        tot += t;
        n += l;
    }
    *total_ms = tot;
    *launches = n;
    return KNN_OK;
}

int multi_set_fence_mode(knn_index* ix, int mode) {
    for (knn_index* sh : M(ix)->shards) {
        std::lock_guard<std::mutex> lk(sh->mu);
        sh->fence_lazy = mode == KNN_FENCE_LAZY;
    }
    return KNN_OK;
}

int multi_set_search_mode(knn_index* ix, int mode) {
    for (knn_index* sh : M(ix)->shards) {
        int rc = knn_set_search_mode(sh, mode);
        if (rc != KNN_OK) return rc;
    }
    ix->mode = mode;
    return KNN_OK;
}

// queries on a candidate path: every query runs on every shard, so the largest shard count;
// re-runs and second chances: summed over shards (one query can count once per shard)
int multi_search_stats(knn_index* ix, int64_t* split_q, int64_t* fallback_q, int64_t* second_q,
                       float* ratio) {
    *split_q = 0;
    *fallback_q = 0;
    if (second_q) *second_q = 0;
    if (ratio) *ratio = 0.f;
    for (knn_index* sh : M(ix)->shards) {
        int64_t a = 0, b = 0, c = 0;
        float r = 0.f;
        int rc = knn_search_stats2(sh, &a, &b, &c, &r);
        if (rc != KNN_OK) return rc;
        *split_q = std::max(*split_q, a);
        *fallback_q += b;
        if (second_q) *second_q += c;
        if (ratio) *ratio = std::max(*ratio, r);
    }
    return KNN_OK;
}

int multi_last_path(const knn_index* ix) { return M(ix)->shards[0]->last_path; }

const knn_index* multi_shard(const knn_index* ix, int s) { return M(ix)->shards[s]; }

int multi_num_shards(const knn_index* ix) { return (int)M(ix)->shards.size(); }

}  // namespace imgrec

extern "C" {

int knn_create_multi(int d, int metric, const int* devices, int ndev, knn_index_t** out) {
    if (!out) KNN_FAIL(KNN_EINVAL, "out is NULL");
    *out = nullptr;
    if (d <= 0) KNN_FAIL(KNN_EINVAL, "d must be positive (got %d)", d);
    if (metric != KNN_METRIC_L2 && metric != KNN_METRIC_IP && metric != KNN_METRIC_COSINE)
        KNN_FAIL(KNN_EINVAL, "unknown metric %d", metric);
    if (!devices || ndev <= 0 || ndev > 64) KNN_FAIL(KNN_EINVAL, "need 1..64 devices (got %d)", ndev);
    return imgrec::multi_create(d, metric, devices, ndev, out);
}

int knn_num_shards(const knn_index_t* ix) {
    if (!ix) return KNN_EINVAL;
    return ix->multi ? imgrec::multi_num_shards(ix) : 1;
}

}  // extern "C"
