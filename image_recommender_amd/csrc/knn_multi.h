// knn_multi.h — one k-NN index over several HIP devices in one process (knn_create_multi):
// the corpus is split into per-device row shards, a search runs every shard concurrently on its
// own device and stream and merges the per-shard top-k on the first device.  Internal to the C
// ABI (knn_capi.cpp dispatches here when knn_index::multi is set).
#pragma once

#include "knn_index.h"

namespace imgrec {

int multi_create(int d, int metric, const int* devices, int ndev, knn_index** out);
int multi_free(knn_index* ix);
int multi_reserve(knn_index* ix, int64_t n);
int multi_add(knn_index* ix, const float* x, int64_t n);
int multi_add_device(knn_index* ix, const float* x, int64_t n, hipStream_t st);
int multi_reset(knn_index* ix);
int multi_reconstruct_n(knn_index* ix, int64_t i0, int64_t n, float* x);
int multi_search(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I);
int multi_search_device(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                        hipStream_t st);
int multi_set_metric(knn_index* ix, int metric);
int multi_set_trained(knn_index* ix, bool trained);
int multi_set_timing(knn_index* ix, int enable);
int multi_kernel_time(knn_index* ix, double* total_ms, int* launches);
int multi_set_search_mode(knn_index* ix, int mode);
int multi_set_fence_mode(knn_index* ix, int mode);
int multi_search_stats(knn_index* ix, int64_t* split_q, int64_t* fallback_q, int64_t* second_q,
                       float* ratio);
int multi_last_path(const knn_index* ix);
const knn_index* multi_shard(const knn_index* ix, int s);
int multi_num_shards(const knn_index* ix);

}  // namespace imgrec
