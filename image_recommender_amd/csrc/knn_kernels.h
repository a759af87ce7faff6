// knn_kernels.h — internal launch interface between the C ABI (knn_capi.cpp) and the gfx950
// kernels (knn_kernels.hip).  Not part of the public ABI (see include/imgrec_knn.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace imgrec {

// Arguments of one fused distance + top-k launch.
struct TileArgs {
    int wr, wq, km;             // waves along rows / queries, register list length
    const float* xb;            // corpus, nrows_cap x dp (rows padded to 256, columns to 16)
    const float* xnorm;         // |x|^2 per stored row
    int nrows, dp;
    const float* qp;            // queries, nq_pad x dp
    const float* qnorm;         // |q|^2 per padded query
    int nq;
    int metric;                 // 1 = L2, otherwise inner product
    int ntiles, nsplit, nqb;
    int64_t id_offset;
    float* cand_d;              // nq x ncand keys
    int64_t* cand_i;            // nq x ncand labels
    int ncand;
};

constexpr int kTileRowsMax = 256;   // corpus capacity is rounded to this many rows
constexpr int kDepthPad = 16;       // row stride is rounded to this many floats

hipError_t launch_rows_ingest(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                              int normalize, float* dst, float* norms, hipStream_t st);
hipError_t launch_tile_topk(const TileArgs& a, hipStream_t st);
hipError_t launch_merge(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                        int64_t stride_q, int64_t stride_l, int k, int metric, int negate_in,
                        float* D, int64_t* I, hipStream_t st);
hipError_t launch_fill_empty(float* D, int64_t* I, int64_t n, int metric, hipStream_t st);

}  // namespace imgrec
