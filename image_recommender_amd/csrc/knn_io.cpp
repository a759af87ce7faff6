// knn_io.cpp — faiss's IndexFlat file layout (write_index / read_index, the reference's
// /root/reference/main/create_index.py:320 and main/search_from_image.py:339) and
// normalize_L2 (main/search_from_image.py:322).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "knn_index.h"

using imgrec::set_err;

namespace {

struct FlatHeader {
    int32_t d = 0;
    int64_t ntotal = 0;
    int metric = KNN_METRIC_L2;
    bool trained = true;
    long data_pos = 0;
};

}  // namespace

extern "C" {

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

}  // extern "C"

namespace {

// Parse the IndexFlat header of `path`; on success f is positioned at the first row.
int read_header(const char* path, FILE** fp, FlatHeader* h) {
    *fp = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) KNN_FAIL(KNN_EIO, "cannot open %s", path);
    uint32_t fourcc = 0;
    int32_t d = 0, mt = 0;
    int64_t nt = 0, dm1 = 0, dm2 = 0;
    uint8_t tr = 0;
    uint64_t nfl = 0;
    bool ok = fread(&fourcc, 4, 1, f) == 1 && fread(&d, 4, 1, f) == 1 && fread(&nt, 8, 1, f) == 1 &&
              fread(&dm1, 8, 1, f) == 1 && fread(&dm2, 8, 1, f) == 1 && fread(&tr, 1, 1, f) == 1 &&
              fread(&mt, 4, 1, f) == 1;
    char cc[5] = {(char)(fourcc & 0xff), (char)((fourcc >> 8) & 0xff), (char)((fourcc >> 16) & 0xff),
                  (char)((fourcc >> 24) & 0xff), 0};
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
    const long data_pos = ftell(f);
    if (fseek(f, 0, SEEK_END) == 0) {
        const long end = ftell(f);
        const long want = data_pos + (long)(nfl * 4);
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
    h->d = d;
    h->ntotal = nt;
    h->metric = metric;
    h->trained = tr != 0;
    h->data_pos = data_pos;
    *fp = f;
    return KNN_OK;
}

// Rows of an opened file into a created index (single or multi-device), in 64 MiB chunks.
// COSINE rows are already normalised; re-normalising a unit row is idempotent only up to
// rounding, so they go in through the IP path and the metric is restored afterwards.
int load_rows(FILE* f, const FlatHeader& h, const char* path, knn_index_t* ix) {
    int rc;
    if ((rc = knn_reserve(ix, h.ntotal)) != KNN_OK) return rc;
    if (h.metric == KNN_METRIC_COSINE && (rc = imgrec::set_metric(ix, KNN_METRIC_IP)) != KNN_OK)
        return rc;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64 << 20) / ((int64_t)h.d * 4));
    std::vector<float> buf;
    for (int64_t r0 = 0; r0 < h.ntotal; r0 += chunk) {
        const int64_t cn = std::min(chunk, h.ntotal - r0);
        buf.resize((size_t)cn * h.d);
        if (fread(buf.data(), sizeof(float), buf.size(), f) != buf.size())
            KNN_FAIL(KNN_EIO, "%s: short read", path);
        if ((rc = knn_add(ix, buf.data(), cn)) != KNN_OK) return rc;
    }
    if ((rc = imgrec::set_metric(ix, h.metric)) != KNN_OK) return rc;
    return imgrec::set_trained(ix, h.trained);
}

}  // namespace

extern "C" {

int knn_read(const char* path, int device, knn_index_t** out) {
    if (!path || !out) KNN_FAIL(KNN_EINVAL, "NULL argument");
    *out = nullptr;
    FILE* f = nullptr;
    FlatHeader h;
    int rc = read_header(path, &f, &h);
    if (rc != KNN_OK) return rc;
    knn_index_t* ix = nullptr;
    if ((rc = knn_create(h.d, h.metric, device, &ix)) == KNN_OK) rc = load_rows(f, h, path, ix);
    fclose(f);
    if (rc != KNN_OK) {
        if (ix) knn_free(ix);
        return rc;
    }
    *out = ix;
    return KNN_OK;
}

int knn_read_multi(const char* path, const int* devices, int ndev, knn_index_t** out) {
    if (!path || !out) KNN_FAIL(KNN_EINVAL, "NULL argument");
    *out = nullptr;
    FILE* f = nullptr;
    FlatHeader h;
    int rc = read_header(path, &f, &h);
    if (rc != KNN_OK) return rc;
    knn_index_t* ix = nullptr;
    if ((rc = knn_create_multi(h.d, h.metric, devices, ndev, &ix)) == KNN_OK)
        rc = load_rows(f, h, path, ix);
    fclose(f);
    if (rc != KNN_OK) {
        if (ix) knn_free(ix);
        return rc;
    }
    *out = ix;
    return KNN_OK;
}

}  // extern "C"
