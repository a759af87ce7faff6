// ivfpq_capi.cpp — C ABI of the IVF-PQ kernels (include/imgrec_ivfpq.h; reference default index
// IndexIVFPQ(IndexHNSWFlat(d,32), d, 2048, m, 12), /root/reference/main/create_index.py:218-228).
#include "../../include/imgrec_ivfpq.h"
#include "knn_index.h"

using imgrec::set_err;

extern "C" {

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

int ivfpq_scan_all_device(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                          const int64_t* list_off, const uint16_t* codes, const int64_t* ids, int m,
                          int ksub, const int64_t* probe_off, const uint32_t* seg_off, int64_t total,
                          int k, float* D, int64_t* I, void* stream) {
    if (nq < 0 || nprobe <= 0 || m <= 0 || ksub <= 0 || ksub > 65536)
        KNN_FAIL(KNN_EINVAL, "bad IVF-PQ scan shape");
    if (k <= 0) KNN_FAIL(KNN_EINVAL, "k must be >= 1 (got %d)", k);
    if (total < 0 || total >= ((int64_t)1 << 32)) KNN_FAIL(KNN_EINVAL, "total entries %lld out of range", (long long)total);
    if (nq == 0) return KNN_OK;
    if (!lut || !probes || !list_off || !codes || !ids || !probe_off || !seg_off || !D || !I)
        KNN_FAIL(KNN_EINVAL, "NULL pointer");
    KNN_HIP(imgrec::launch_ivfpq_scan_all(lut, probes, nq, nprobe, list_off, codes, ids, m, ksub, probe_off,
                                          seg_off, total, k, D, I, (hipStream_t)stream));
    return KNN_OK;
}

}  // extern "C"
