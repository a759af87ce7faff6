/*
 * TEST INFRASTRUCTURE ONLY — plain-C restatements of the hot path (the checker and the scalar
 * CPU port; never linked into the product).
 *
 * oracle_flat_search: exact flat k-NN with faiss IndexFlat semantics (faiss-cpu 1.10.0, the library
 *   behind index.search at /root/reference/main/search_from_image.py:247): squared L2 ascending or
 *   inner product descending, accumulated in double; ties by the smaller label; k > n padded with
 *   label -1 and +-FLT_MAX.  OpenMP over queries.
 * oracle_color_counts: cv2.calcHist(bins, [0,256)) per RGB channel
 *   (/root/reference/vector_scripts/create_color_vector.py:46-47), integer counts.
 */
#include <float.h>
#include <stdint.h>
#include <stdlib.h>

static int before(double d1, int64_t i1, double d2, int64_t i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

int oracle_flat_search(const float* xb, int64_t n, const float* xq, int64_t nq, int d, int k,
                       int metric_l2, double* D, int64_t* I) {
    if (k <= 0 || d <= 0 || n < 0 || nq < 0) return -1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t q = 0; q < nq; ++q) {
        double* kd = D + q * k;
        int64_t* ki = I + q * k;
        for (int p = 0; p < k; ++p) { kd[p] = 1e308; ki[p] = -1; }
        const float* qv = xq + q * d;
        for (int64_t i = 0; i < n; ++i) {
            const float* x = xb + i * d;
            double s = 0.0;
            if (metric_l2) {
                for (int j = 0; j < d; ++j) { double t = (double)qv[j] - (double)x[j]; s += t * t; }
            } else {
                for (int j = 0; j < d; ++j) s += (double)qv[j] * (double)x[j];
                s = -s;
            }
            if (!before(s, i, kd[k - 1], ki[k - 1])) continue;
            int p = k - 1;
            while (p > 0 && before(s, i, kd[p - 1], ki[p - 1])) { kd[p] = kd[p - 1]; ki[p] = ki[p - 1]; --p; }
            kd[p] = s; ki[p] = i;
        }
        for (int p = 0; p < k; ++p) {
            if (ki[p] < 0) kd[p] = metric_l2 ? FLT_MAX : -FLT_MAX;
            else if (!metric_l2) kd[p] = -kd[p];
        }
    }
    return 0;
}

int oracle_color_counts(const uint8_t* rgb, int64_t npix, int bins, int64_t* counts) {
    if (bins < 1 || bins > 256 || npix < 0) return -1;
    for (int b = 0; b < 3 * bins; ++b) counts[b] = 0;
    for (int64_t p = 0; p < npix; ++p)
        for (int c = 0; c < 3; ++c) counts[c * bins + ((rgb[3 * p + c] * bins) >> 8)] += 1;
    return 0;
}
