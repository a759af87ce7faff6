/*
 * imgrec_knn.h — C ABI of the MI355X exact k-NN index (the image_recommender hot path).
 *
 * This is the drop-in boundary for the faiss calls the reference makes on its search/index path
 * (SURVEY.md §8b).  Every entry point below replaces one faiss call site of the reference:
 *
 *   knn_create(d, KNN_METRIC_L2, ...)   faiss.IndexFlatL2(d) — the parity target named by north_star; the
 *                                        reference default IndexIVFPQ(IndexHNSWFlat(d,32),d,2048,m,12) is
 *                                        built at /root/reference/main/create_index.py:218-228
 *   knn_train                            index.train(train_vecs)       main/create_index.py:296-299
 *   knn_add / knn_add_device             index.add(arr)                main/create_index.py:311
 *   knn_search / knn_search_device       index.search(query_vec, k)    main/search_from_image.py:247,
 *                                                                      Analytics/rt_Search.py:63
 *   knn_ntotal / knn_dim                 index.ntotal / index.d        main/search_from_image.py:340,
 *                                                                      main/create_index.py:321
 *   knn_write                            faiss.write_index(index, f)   main/create_index.py:320
 *   knn_read                             faiss.read_index(f)           main/search_from_image.py:339
 *   knn_normalize_L2                     faiss.normalize_L2(x)         main/search_from_image.py:322
 *   knn_merge_device                     (new) per-shard top-k merge after the RCCL all-gather (§8e)
 *   knn_packed_bytes / knn_merge_packed_device  (new) the same over one packed key|label buffer,
 *                                        so the all-gather is a single collective
 *   knn_create_multi / knn_read_multi    (new) one index over several devices of one process, so
 *                                        the reference's single-process CLI
 *                                        (main/search_from_image.py:430-441) can use every GPU
 *
 * Conventions
 *   - All functions return 0 on success and a negative KNN_E* code on failure; the message of the
 *     last failure on the calling thread is returned by knn_last_error().
 *   - Host-pointer functions (knn_add, knn_search, knn_write, ...) synchronise before returning.
 *     *_device functions take device pointers and a hipStream_t (passed as void*; NULL = the
 *     HIP null stream, like any HIP API), enqueue asynchronously and never wait for the GPU: the
 *     candidate paths' certificate, its second chance and the exact re-run of the queries it
 *     cannot settle are all decided on the device.  They allocate only when the workspace must
 *     grow.
 *   - Operations on one index may come from different streams and threads: an operation on
 *     another stream than the previous operation's first waits for that operation (an add on
 *     stream A is complete before a search on stream B reads the rows; two searches never share
 *     the workspace concurrently).  A call on the index's host entry points is ordered after
 *     earlier device-stream calls the same way.  By default (KNN_FENCE_EAGER) every *_device call
 *     records an event on its stream as its last step and the next call on another stream waits
 *     for it, so a stream may be destroyed as soon as the call returns.  knn_set_fence_mode
 *     (KNN_FENCE_LAZY) records the event only when the stream changes: one stream used back to
 *     back then records none (~6 us of GPU time per call saved on MI355X), but the previous
 *     call's stream must stay valid until the next call on the index, and the wait then also
 *     covers work the caller queued on that stream in between.
 *   - Vectors are row-major float32, n rows × d.  Labels are int64.  Result rows are sorted by
 *     ascending distance (L2) or descending inner product (IP/COSINE); exact ties are broken by the
 *     smaller label.  When fewer than k vectors exist, the tail of a result row holds label -1 and
 *     distance FLT_MAX (L2) or -FLT_MAX (IP/COSINE), as faiss's heaps do.
 *   - L2 distances are squared L2, evaluated as (|q|^2 + |x|^2) - 2 q.x and clamped at 0, as in
 *     faiss's exhaustive_L2sqr_blas.
 */
#ifndef IMGREC_KNN_H
#define IMGREC_KNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct knn_index knn_index_t;

enum knn_metric {
    KNN_METRIC_IP = 0,     /* faiss METRIC_INNER_PRODUCT (IndexFlatIP) */
    KNN_METRIC_L2 = 1,     /* faiss METRIC_L2 (IndexFlatL2) */
    KNN_METRIC_COSINE = 2  /* rows and queries L2-normalised on entry, then IP */
};

enum knn_error {
    KNN_OK = 0,
    KNN_EINVAL = -1,   /* bad argument (d <= 0, k <= 0, NULL pointer, unsupported k, ...) */
    KNN_EHIP = -2,     /* HIP runtime error */
    KNN_ENOMEM = -3,   /* device allocation failed */
    KNN_EIO = -4,      /* file could not be read/written or has a bad layout */
    KNN_ENOSYS = -5    /* not supported (e.g. no GPU visible) */
};

/* Search arithmetic.  Every mode returns the exact search's result up to the fp32 tie window:
 * a candidate pass proposes K' rows per query, an fp32 rerank computes their exact keys and a
 * per-query error-bound certificate proves that no row outside the candidates can rank before a
 * returned one.  The returned labels are those of the fp32 keys of the rerank.  Tie windows, as
 * tested (tests/knn_check.py):
 *   - rigorous (every parity test): every returned distance is within the worst-case fp32 bound
 *     gamma_D (|q|^2 + |x|^2 + 2 sum|q_i x_i|) + rounding of the norm terms (gamma_D = D u /
 *     (1 - D u), u = 2^-24: about 1e-4 relative at D = 1968) of its row's exact distance, and
 *     labels equal the float64 oracle's at every rank separated from both neighbours by twice it;
 *   - empirical (check_knn_tight: the full-size configs 2-4 and the int8 path at d >= 1024):
 *     labels equal BOTH the float64 oracle's and faiss IndexFlatL2's fp32 result (its
 *     exhaustive_L2sqr_blas restated, oracle.flat_knn.search_blas_fp32_blocked) at every rank
 *     separated from both neighbours by more than w = max(8 x the measured max |fp32 key -
 *     float64 key| of both, 1e-6 x the query's key scale) — about 1e-6 relative on the bench
 *     data — and the top-k label SETS are equal wherever the k-th / (k+1)-th gap exceeds w; at
 *     least 95 % of ranks are so checked at the full-size configurations.
 * Inside the window modes may order near-equal rows differently.  A query whose certificate fails gets a second chance (every
 * per-split list entry reranked, certified against the list floor); if that fails too it is
 * re-run on the exact fp32 kernel, planned on the device.
 * AUTO: the bf16 path (d >= 64; one bf16 MFMA per product, K' = 64) for every batch at every
 *       corpus size (large batches: bf16 MFMA; small ones: the bf16 copy streams half the
 *       bytes; small corpora: the exact kernel's latency floor of ~0.16 ms per search); the
 *       split path when bf16 is unavailable and the batch is large; everything else (d < 64,
 *       k > KNN_MAX_K) the exact fp32 kernel.
 *       Batches of <= 8 queries (the reference CLI's one-query searches) take the int8 path
 *       instead (64 <= d <= 4096; at d <= 512, where an int8 row's 1-KiB group is wider than
 *       its bf16 row, only while the int8 copy is <= 64 MB): a block-scaled int8 copy of the rows (one fp32 scale per 64
 *       elements, about half the bf16 copy's bytes, built on the first such search), a
 *       two-level int8 query and exact int32 dot4 products, K' = 64, the same certificate with
 *       the int8 copy's and the query's residual bounds (csrc/knn_i8.hip).
 * EXACT: always the fp32 kernel.  SPLIT: the split path (bf16 hi/lo, three MFMAs per product,
 *       K' = 16/32) whenever k <= 16 and d >= 256.  BF16: the bf16 path for every batch (tests).
 * I8:   the int8 path for batches of <= 8 queries (64 <= d <= 4096; tests), else as AUTO. */
enum knn_search_mode {
    KNN_SEARCH_AUTO = 0,
    KNN_SEARCH_EXACT = 1,
    KNN_SEARCH_SPLIT = 2,
    KNN_SEARCH_BF16 = 3,
    KNN_SEARCH_I8 = 4
};

/* Largest k the fused top-k kernels serve (they keep per-lane lists of this length). */
#define KNN_MAX_K 32
/* Every k >= 1 is served (faiss IndexFlat's range; past ntotal the tail is label -1, distance
 * +-FLT_MAX).  KNN_MAX_K < k <= KNN_MAX_K_LARGE runs the exact fp32 fused kernel with 32-entry
 * lists, the k best of their union by an exact per-query radix select, certified against the
 * lists' floor; the queries the certificate cannot settle are re-run by an exact corpus scan whose
 * fixed grid walks the failed queries the device counted (csrc/knn_largek.hip: no key block
 * reaches HBM, the host never waits).  k > KNN_MAX_K_LARGE keys every (query, row) pair in fp32
 * and sorts each query's keys (csrc/knn_hugek.hip: coverage of faiss's k range, not a fast path).
 * Merges of k-lists (multi-device shards, knn_merge_*_device) use the in-LDS select up to 8192
 * gathered entries per query and the sort beyond. */
#define KNN_MAX_K_LARGE 1024

/* Create an empty index of dimension d on HIP device `device` (-1 = current device). */
int knn_create(int d, int metric, int device, knn_index_t** out);
/* Create an empty index whose rows are split over ndev devices (entries may repeat: several
 * shards on one device).  Every add is cut into ndev contiguous pieces, one per shard; labels are
 * the dense row offsets as for one device.  A search runs all shards concurrently (each on its own
 * device and stream) and merges their top-k on devices[0]; *_device pointers live on devices[0].
 * Every other entry point works unchanged on the returned handle. */
int knn_create_multi(int d, int metric, const int* devices, int ndev, knn_index_t** out);
/* Row shards of an index (1 for knn_create). */
int knn_num_shards(const knn_index_t* index);
int knn_free(knn_index_t* index);

int knn_dim(const knn_index_t* index);
int knn_metric(const knn_index_t* index);
int64_t knn_ntotal(const knn_index_t* index);
int knn_is_trained(const knn_index_t* index);

/* Labels returned by search are (row offset + id_offset); a row shard sets its global base here. */
int knn_set_id_offset(knn_index_t* index, int64_t id_offset);

/* Flat index: training only marks the index trained (faiss IndexFlat is always trained). */
int knn_train(knn_index_t* index, const float* x, int64_t n);

/* Append n rows; ids are implicitly ntotal .. ntotal+n-1 (faiss Index::add). */
int knn_add(knn_index_t* index, const float* x_host, int64_t n);
int knn_add_device(knn_index_t* index, const float* x_dev, int64_t n, void* stream);
/* Pre-size the corpus buffer for n rows (avoids regrowth copies during streamed adds). */
int knn_reserve(knn_index_t* index, int64_t n);
int knn_reset(knn_index_t* index);

/* Copy rows [i0, i0+n) back to the host as stored (normalised for COSINE). */
int knn_reconstruct_n(const knn_index_t* index, int64_t i0, int64_t n, float* x_host);

/* k nearest neighbours of nq queries.  D, I: nq*k, row-major. */
int knn_search(knn_index_t* index, const float* q_host, int64_t nq, int k,
               float* D_host, int64_t* I_host);
int knn_search_device(knn_index_t* index, const float* q_dev, int64_t nq, int k,
                      float* D_dev, int64_t* I_dev, void* stream);

/* Merge nlists candidate lists per query into the top k.  cand_D/cand_I are laid out
 * [nlists][nq][kin] (the layout of an all-gather of per-shard [nq][kin] results); entries with
 * label -1 are ignored.  Output nq*k, same ordering/padding rules as knn_search. */
int knn_merge_device(const float* cand_D, const int64_t* cand_I, int nlists, int64_t nq, int kin,
                     int k, int metric, float* D_dev, int64_t* I_dev, void* stream);

/* Packed per-shard results: one chunk of knn_packed_bytes(nq, k) bytes per shard holding the nq*k
 * float keys (padded to an even count), then the nq*k int64 labels (8-byte aligned).  A shard
 * searches straight into its chunk (D = chunk, I = chunk + 4 * (nq*k rounded up to even)); one
 * all-gather of the chunks gives knn_merge_packed_device its [nlists] chunks. */
int64_t knn_packed_bytes(int64_t nq, int k);
int knn_merge_packed_device(const void* packed, int nlists, int64_t nq, int kin, int k, int metric,
                            float* D_dev, int64_t* I_dev, void* stream);

/* faiss IndexFlat on-disk layout ("IxF2" for L2, "IxFI" for IP/COSINE). */
int knn_write(const knn_index_t* index, const char* path);
int knn_read(const char* path, int device, knn_index_t** out);
int knn_read_multi(const char* path, const int* devices, int ndev, knn_index_t** out);

/* In-place row normalisation of a host array (faiss.normalize_L2: rows with norm 0 unchanged). */
int knn_normalize_L2(float* x_host, int64_t n, int d);

/* Kernel timing for the live roofline figure in bench.py.  While enabled, every search records a
 * HIP event pair around its fused distance+top-k launch, on the stream that launch uses.
 * knn_kernel_time waits for the recorded events, returns the summed duration (ms) and launch
 * count since the last call, and clears them. */
int knn_set_timing(knn_index_t* index, int enable);

/* Cross-stream fence of the *_device entry points (Conventions above). */
enum knn_fence_mode { KNN_FENCE_EAGER = 0, KNN_FENCE_LAZY = 1 };
int knn_set_fence_mode(knn_index_t* index, int mode);
int knn_kernel_time(knn_index_t* index, double* total_ms, int* launches);

int knn_set_search_mode(knn_index_t* index, int mode);
/* Queries of the last search that took a candidate path (split or bf16), how many of them were
 * re-run on the exact kernel because neither certificate held, and (may be NULL) the largest
 * observed |approximate key - fp32 key| / (error bound of both) over all reranked candidates:
 * <= 1 whenever the certificate's bounds hold, in practice far below.  Waits for that search.
 * knn_search_stats2 also returns the queries whose first certificate failed and whose second
 * chance certified them (may be NULL).  A multi-device index sums re-runs over its shards. */
int knn_search_stats(knn_index_t* index, int64_t* split_queries, int64_t* fallback_queries,
                     float* max_err_ratio);
int knn_search_stats2(knn_index_t* index, int64_t* split_queries, int64_t* fallback_queries,
                      int64_t* second_chance_queries, float* max_err_ratio);

/* Arithmetic the last search's first query chunk ran: 0 = exact fp32 kernel, 1 = split path,
 * 2 = bf16 path, 3 = int8 path (the candidate paths' fallbacks are counted by knn_search_stats). */
int knn_last_path(const knn_index_t* index);

/* Queries of the last k > KNN_MAX_K search that its certificate could not settle from the fused
 * kernel's 32-entry lists and that were re-run by the exact corpus scan (csrc/knn_largek.hip);
 * summed over the shards of a multi-device index. */
int knn_large_k_fallbacks(const knn_index_t* index, int64_t* queries);

/* Launch geometry chosen for a search of nq queries (for reports): workgroup tile rows/queries,
 * row splits and workgroup count. */
int knn_plan(const knn_index_t* index, int64_t nq, int k, int* tile_rows, int* tile_queries,
             int* splits, int* workgroups);

/* Name of the fused candidate/distance kernel a search of nq queries launches, as profilers print
 * it (e.g. "knn_b16w_tile_kernel<10, 1, true>"), NUL-terminated into name[cap]. */
int knn_plan_kernel(const knn_index_t* index, int64_t nq, int k, char* name, int cap);

const char* knn_last_error(void);
const char* knn_version(void);

#ifdef __cplusplus
}
#endif

#endif /* IMGREC_KNN_H */
