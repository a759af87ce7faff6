/*
 * imgrec_ivfpq.h — C ABI of the GPU IVF-PQ search kernels.
 *
 * The reference's default index is faiss IndexIVFPQ(IndexHNSWFlat(d, 32), d, nlist = 2048, m,
 * nbits = 12) searched with nprobe = 1 (/root/reference/main/create_index.py:218-228,
 * main/search_from_image.py:247).  The exact index (imgrec_knn.h) is the parity target; these
 * entry points are the approximate alternative with the reference's index structure: residual
 * product quantisation over coarse inverted lists, asymmetric-distance (ADC) search.  Training,
 * coarse assignment and encoding run on the exact k-NN kernels (image_recommender_amd/ivfpq.py);
 * the per-query distance tables and the list scan are these kernels.
 *
 * Layouts (device memory, row-major):
 *   residuals   nr x d float32           query minus the probed list's centroid
 *   codebooks_t m x dsub x ksub float32  sub-quantiser j, dimension t, centroid i (transposed so a
 *                                        thread per centroid reads coalesced); dsub = d / m
 *   lut         nr x m x ksub float32    squared L2 of residual sub-vector j to centroid i
 *   probes      nq x nprobe int64        list ids to scan per query (-1 = none)
 *   lut rows    query q, probe p uses lut row q * nprobe + p
 *   list_off    nlist + 1 int64          rows of list l: [list_off[l], list_off[l+1])
 *   codes       ntotal x m uint16        codes of the rows in list order (nbits <= 16)
 *   ids         ntotal int64             label of each row in list order
 * Results: D, I nq x k, ascending distance, ties by smaller label, -1 / FLT_MAX padding — the
 * conventions of knn_search.  Return codes and knn_last_error() as in imgrec_knn.h.
 */
#ifndef IMGREC_IVFPQ_H
#define IMGREC_IVFPQ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Distance tables: lut[r][j][i] = sum_t (residuals[r][j*dsub + t] - codebooks_t[j][t][i])^2. */
int ivfpq_lut_device(const float* residuals, int64_t nr, int d, int m, int ksub,
                     const float* codebooks_t, float* lut, void* stream);

/* ADC scan of each query's probed lists: distance of a row = sum_j lut[q*nprobe+p][j][code_j];
 * the k best per query over all its probes.  k <= 32. */
int ivfpq_scan_device(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                      const int64_t* list_off, const uint16_t* codes, const int64_t* ids, int m,
                      int ksub, int k, float* D, int64_t* I, void* stream);

/* Any k (faiss IndexIVFPQ's range): the ADC distance of every row of each query's probed lists
 * (summed as ivfpq_scan_device sums it), sorted per query by (distance, label), the first k, then
 * label -1 / FLT_MAX.  probe_off (nq x nprobe int64): the first slot of (query q, probe p) in a
 * buffer of `total` entries, the rows of that probe's list in list order (0 rows for a -1 probe);
 * seg_off (nq + 1 uint32): query q's entries are [seg_off[q], seg_off[q + 1]), seg_off[nq] =
 * total < 2^32.  Labels < 2^32.  Work space (2 x total x 8 B + the sort's) is allocated and freed
 * in stream order on `stream`. */
int ivfpq_scan_all_device(const float* lut, const int64_t* probes, int64_t nq, int nprobe,
                          const int64_t* list_off, const uint16_t* codes, const int64_t* ids, int m,
                          int ksub, const int64_t* probe_off, const uint32_t* seg_off, int64_t total,
                          int k, float* D, int64_t* I, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* IMGREC_IVFPQ_H */
