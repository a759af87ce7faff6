// knn_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the exact k-NN hot path.
//
// Replaces the arithmetic of faiss.IndexFlatL2.search / IndexFlatIP.search that the reference
// reaches from main/search_from_image.py:247 (and Analytics/rt_Search.py:63), and the add-time
// norm computation of IndexFlat.add reached from main/create_index.py:311.
//
// Kernels
//   rows_ingest       copy rows into the HBM layout (row stride dp = d rounded up to 16 floats,
//                     zero padded), optional L2 normalisation (faiss.normalize_L2 semantics,
//                     main/search_from_image.py:322), squared norm of every stored row.
//   knn_tile_topk     fused distance + top-k: an LDS-staged f32 MFMA contraction
//                     (v_mfma_f32_32x32x2_f32, exact fp32) of a BM-row corpus tile against a
//                     BQ-query tile over the full depth, then an epilogue that turns each
//                     accumulator into an L2 / IP key and filters it into a per-lane register
//                     top-K list.  The N x Q distance matrix never reaches HBM.
//   knn_merge         one wave per query: per-lane lists + a 64-lane butterfly argmin, k rounds.
//
// Accumulator layout (v_mfma_f32_32x32x2_f32, C/D map of cdna_hip_programming.md §3):
//   col = lane & 31 -> query,  row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5) -> corpus row.
// So every lane already holds 16 rows x 1 query per 32x32 block: the top-k filter needs no data
// movement.  The K index is permuted so each lane reads 8 contiguous floats per operand per
// 16-deep stage: MFMA sub-step s, lane half h uses depth k = 8h + s (same permutation on both
// operands, so the contraction is unchanged).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include <math.h>

#include "knn_kernels.h"

namespace imgrec {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------------

// (d1, i1) ranks before (d2, i2): smaller key, exact ties by smaller label.
template <typename I>
__device__ __forceinline__ bool ranks_before(float d1, I i1, float d2, I i2) {
    return d1 < d2 || (d1 == d2 && i1 < i2);
}

// Insert (d, id) into an ascending register list of length K (caller checked it beats kd[K-1]).
// Fully unrolled with compile-time indices so the list stays in VGPRs.
template <int K, typename I>
__device__ __forceinline__ void list_insert(float (&kd)[K], I (&ki)[K], float d, I id) {
#pragma unroll
    for (int p = K - 1; p > 0; --p) {
        const bool shift = ranks_before(d, id, kd[p - 1], ki[p - 1]);
        const bool here = !shift && ranks_before(d, id, kd[p], ki[p]);
        kd[p] = shift ? kd[p - 1] : (here ? d : kd[p]);
        ki[p] = shift ? ki[p - 1] : (here ? id : ki[p]);
    }
    const bool here0 = ranks_before(d, id, kd[0], ki[0]);
    kd[0] = here0 ? d : kd[0];
    ki[0] = here0 ? id : ki[0];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------------------------------------
// rows_ingest: one wave per destination row.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
rows_ingest_kernel(const float* __restrict__ src, int64_t n, int d, int dp, int64_t n_pad,
                   int normalize, float* __restrict__ dst, float* __restrict__ norms) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_pad) return;
    float* o = dst + row * (int64_t)dp;
    if (row >= n) {
        for (int j = lane; j < dp; j += 64) o[j] = 0.f;
        if (lane == 0) norms[row] = 0.f;
        return;
    }
    const float* s = src + row * (int64_t)d;
    float scale = 1.f;
    if (normalize) {
        float acc = 0.f;
        for (int j = lane; j < d; j += 64) acc = fmaf(s[j], s[j], acc);
        acc = wave_sum(acc);
        // faiss fvec_renorm_L2: nr = 1.0 / sqrtf(nr) (double reciprocal, stored as float)
        if (acc > 0.f) scale = (float)(1.0 / (double)sqrtf(acc));
    }
    float acc2 = 0.f;
    for (int j = lane; j < dp; j += 64) {
        const float v = (j < d) ? (normalize ? s[j] * scale : s[j]) : 0.f;
        o[j] = v;
        acc2 = fmaf(v, v, acc2);
    }
    acc2 = wave_sum(acc2);
    if (lane == 0) norms[row] = acc2;
}

// ---------------------------------------------------------------------------------------------
// knn_tile_topk
// ---------------------------------------------------------------------------------------------
constexpr int BK = 16;     // depth of one LDS stage
constexpr int LROW = 20;   // floats per staged row: 16 + 4 pad -> 80-B stride, conflict-free b128

template <int WR, int WQ, int KM>
__global__ void __launch_bounds__(WR * WQ * 64)
knn_tile_topk_kernel(const float* __restrict__ xb, const float* __restrict__ xnorm, int nrows,
                     int dp, const float* __restrict__ qp, const float* __restrict__ qnorm, int nq,
                     int metric, int ntiles, int nsplit, int nqb, int64_t id_offset,
                     float* __restrict__ cand_d, int64_t* __restrict__ cand_i, int ncand) {
    constexpr int NT = WR * WQ * 64;
    constexpr int BM = WR * 128;   // corpus rows per tile (wave tile: 128 rows = 4 row blocks)
    constexpr int BQ = WQ * 32;    // queries per tile   (wave tile: 32 queries)
    constexpr int A4 = BM * 4;     // float4 per A stage (BM rows x 16 floats)
    constexpr int B4 = BQ * 4;
    constexpr int AP = (A4 + NT - 1) / NT;
    constexpr int BP = (B4 + NT - 1) / NT;

    // One LDS allocation: [A stage 0 | A stage 1 | B stage 0 | B stage 1 | row norms].  The
    // stage region doubles as the epilogue's per-wave key parking (16 x 64 floats per wave).
    constexpr int SA = BM * LROW, SB = BQ * LROW;
    static_assert(2 * (SA + SB) >= WR * WQ * 16 * 64, "parking area exceeds stage buffers");
    __shared__ __attribute__((aligned(16))) float smem[2 * SA + 2 * SB + BM];
    float* const Ns = smem + 2 * SA + 2 * SB;

    // XCD-aware, bijective block -> (query block, row split) map: blocks b and b+8 share an XCD;
    // consecutive remapped ids (same XCD) share a row split so the corpus tile they stream is
    // served from that XCD's L2 for all query blocks.
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, qq = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (wg >> 3);
    const int qb = wgid % nqb;
    const int split = wgid / nqb;
    const int t0 = (int)((int64_t)split * ntiles / nsplit);
    const int t1 = (int)((int64_t)(split + 1) * ntiles / nsplit);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave / WQ;
    const int wq = wave % WQ;
    const int li = lane & 31;
    const int lh = lane >> 5;
    const int qcol = qb * BQ + wq * 32 + li;     // the query this lane owns (< nq_pad)
    const bool qvalid = qcol < nq;
    const float qn = (metric == 1) ? qnorm[qcol] : 0.f;

    float kd[KM];
    int ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }

    const int nsteps = dp / BK;
    const float* qbase = qp + (size_t)qb * BQ * dp;

    for (int t = t0; t < t1; ++t) {
        const int row0 = t * BM;
        const float* abase = xb + (size_t)row0 * dp;

        f32x16 acc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[b] = (f32x16){0.f};

        float4 ra[AP], rb[BP];
        auto load_stage = [&](int k0) {
#pragma unroll
            for (int p = 0; p < AP; ++p) {
                const int f = tid + p * NT;
                if (A4 % NT == 0 || f < A4)
                    ra[p] = *reinterpret_cast<const float4*>(abase + (size_t)(f >> 2) * dp + k0 + (f & 3) * 4);
            }
#pragma unroll
            for (int p = 0; p < BP; ++p) {
                const int f = tid + p * NT;
                if (B4 % NT == 0 || f < B4)
                    rb[p] = *reinterpret_cast<const float4*>(qbase + (size_t)(f >> 2) * dp + k0 + (f & 3) * 4);
            }
        };
        auto store_stage = [&](int buf) {
#pragma unroll
            for (int p = 0; p < AP; ++p) {
                const int f = tid + p * NT;
                if (A4 % NT == 0 || f < A4)
                    *reinterpret_cast<float4*>(&smem[buf * SA + (f >> 2) * LROW + (f & 3) * 4]) = ra[p];
            }
#pragma unroll
            for (int p = 0; p < BP; ++p) {
                const int f = tid + p * NT;
                if (B4 % NT == 0 || f < B4)
                    *reinterpret_cast<float4*>(&smem[2 * SA + buf * SB + (f >> 2) * LROW + (f & 3) * 4]) = rb[p];
            }
        };

        load_stage(0);
        for (int r = tid; r < BM; r += NT) Ns[r] = xnorm[row0 + r];
        store_stage(0);
        __syncthreads();

        int cur = 0;
        for (int s = 0; s < nsteps; ++s) {
            const bool more = (s + 1) < nsteps;
            if (more) load_stage((s + 1) * BK);

            float a[4][8], bq[8];
            {
                const float* bp = &smem[2 * SA + cur * SB + (wq * 32 + li) * LROW + lh * 8];
                const float4 b0 = *reinterpret_cast<const float4*>(bp);
                const float4 b1 = *reinterpret_cast<const float4*>(bp + 4);
                bq[0] = b0.x; bq[1] = b0.y; bq[2] = b0.z; bq[3] = b0.w;
                bq[4] = b1.x; bq[5] = b1.y; bq[6] = b1.z; bq[7] = b1.w;
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const float* ap = &smem[cur * SA + (wr * 128 + b * 32 + li) * LROW + lh * 8];
                const float4 a0 = *reinterpret_cast<const float4*>(ap);
                const float4 a1 = *reinterpret_cast<const float4*>(ap + 4);
                a[b][0] = a0.x; a[b][1] = a0.y; a[b][2] = a0.z; a[b][3] = a0.w;
                a[b][4] = a1.x; a[b][5] = a1.y; a[b][6] = a1.z; a[b][7] = a1.w;
            }
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[b][kk], bq[kk], acc[b], 0, 0, 0);
            }

            if (more) store_stage(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }

        // Epilogue: key = L2 distance (faiss exhaustive_L2sqr_blas form, clamped at 0) or -ip.
        // Keys of one 32x32 block are screened against the lane's current K-th key; only when a
        // lane of the wave has a survivor are the 16 keys parked in (now idle) stage LDS and
        // inserted one by one, so the list insert is emitted once per block, not per register.
        if (qvalid) {
            float* park = smem + wave * (16 * 64);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                float key[16];
                unsigned mask = 0;
                const float tau_d = kd[KM - 1];
                const int tau_i = ki[KM - 1];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rl = wr * 128 + b * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float ip = acc[b][r];
                    float kv;
                    if (metric == 1) {
                        kv = fmaf(-2.f, ip, qn + Ns[rl]);
                        kv = kv < 0.f ? 0.f : kv;
                    } else {
                        kv = -ip;
                    }
                    key[r] = kv;
                    const bool pass = (row0 + rl < nrows) && ranks_before(kv, row0 + rl, tau_d, tau_i);
                    mask |= (unsigned)pass << r;
                }
                if (__any(mask != 0)) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) park[r * 64 + lane] = key[r];
#pragma unroll 1
                    for (int r = 0; r < 16; ++r) {
                        if ((mask >> r) & 1u) {
                            const float kv = park[r * 64 + lane];
                            const int row = row0 + wr * 128 + b * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                            if (ranks_before(kv, row, kd[KM - 1], ki[KM - 1]))
                                list_insert<KM, int>(kd, ki, kv, row);
                        }
                    }
                }
            }
        }
        __syncthreads();   // Ns / stage buffers are rewritten by the next tile's prologue
    }

    if (qvalid) {
        const size_t base = (size_t)qcol * ncand + (size_t)((split * WR + wr) * 2 + lh) * KM;
#pragma unroll
        for (int p = 0; p < KM; ++p) {
            cand_d[base + p] = kd[p];
            cand_i[base + p] = ki[p] < 0 ? (int64_t)-1 : (int64_t)ki[p] + id_offset;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// knn_merge: one wave per query.  Candidate (q, l, p) lives at q*stride_q + l*stride_l + p.
// ---------------------------------------------------------------------------------------------
template <int KM>
__global__ void __launch_bounds__(256)
knn_merge_kernel(const float* __restrict__ cd, const int64_t* __restrict__ ci, int64_t nq,
                 int nlists, int kin, int64_t stride_q, int64_t stride_l, int k, int metric,
                 int negate_in, float* __restrict__ D, int64_t* __restrict__ I) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (q >= nq) return;

    float kd[KM];
    int64_t ki[KM];
#pragma unroll
    for (int p = 0; p < KM; ++p) { kd[p] = INFINITY; ki[p] = -1; }

    const int total = nlists * kin;
    for (int c = lane; c < total; c += 64) {
        const int l = c / kin, p = c - l * kin;
        const int64_t off = q * stride_q + (int64_t)l * stride_l + p;
        const int64_t id = ci[off];
        if (id < 0) continue;
        // gathered search results carry output-convention values (IP: larger first): re-key
        const float d = negate_in ? -cd[off] : cd[off];
        if (ranks_before(d, id, kd[KM - 1], ki[KM - 1])) list_insert<KM, int64_t>(kd, ki, d, id);
    }

    for (int r = 0; r < k; ++r) {
        float bd = kd[0];
        int64_t bi = ki[0];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float od = __shfl_xor(bd, off, 64);
            const int lo = __shfl_xor((int)(bi & 0xffffffff), off, 64);
            const int hi = __shfl_xor((int)(bi >> 32), off, 64);
            const int64_t oi = ((int64_t)hi << 32) | (uint32_t)lo;
            // empty entries (label -1) rank last regardless of their key
            const bool take = (oi >= 0) && (bi < 0 || ranks_before(od, oi, bd, bi));
            bd = take ? od : bd;
            bi = take ? oi : bi;
        }
        if (bi >= 0 && kd[0] == bd && ki[0] == bi) {
#pragma unroll
            for (int p = 0; p < KM - 1; ++p) { kd[p] = kd[p + 1]; ki[p] = ki[p + 1]; }
            kd[KM - 1] = INFINITY;
            ki[KM - 1] = -1;
        }
        if (lane == 0) {
            float out;
            if (bi < 0) out = (metric == 1) ? FLT_MAX : -FLT_MAX;
            else out = (metric == 1) ? bd : -bd;
            D[q * k + r] = out;
            I[q * k + r] = bi;
        }
    }
}

__global__ void fill_empty_kernel(float* __restrict__ D, int64_t* __restrict__ I, int64_t n,
                                  int metric) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { D[i] = (metric == 1) ? FLT_MAX : -FLT_MAX; I[i] = -1; }
}

// ---------------------------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------------------------
hipError_t launch_rows_ingest(const float* src, int64_t n, int d, int dp, int64_t n_pad,
                              int normalize, float* dst, float* norms, hipStream_t st) {
    if (n_pad <= 0) return hipSuccess;
    const int64_t blocks = (n_pad + 3) / 4;
    hipLaunchKernelGGL(rows_ingest_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, n, d, dp,
                       n_pad, normalize, dst, norms);
    return hipGetLastError();
}

template <int WR, int WQ>
static hipError_t launch_tile_km(int km, const TileArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)(a.nqb * a.nsplit)), block(WR * WQ * 64);
#define IMGREC_LAUNCH_TILE(KMV)                                                                   \
    hipLaunchKernelGGL((knn_tile_topk_kernel<WR, WQ, KMV>), grid, block, 0, st, a.xb, a.xnorm,     \
                       a.nrows, a.dp, a.qp, a.qnorm, a.nq, a.metric, a.ntiles, a.nsplit, a.nqb,    \
                       a.id_offset, a.cand_d, a.cand_i, a.ncand)
    switch (km) {
        case 8: IMGREC_LAUNCH_TILE(8); break;
        case 16: IMGREC_LAUNCH_TILE(16); break;
        case 32: IMGREC_LAUNCH_TILE(32); break;
        default: return hipErrorInvalidValue;
    }
#undef IMGREC_LAUNCH_TILE
    return hipGetLastError();
}

hipError_t launch_tile_topk(const TileArgs& a, hipStream_t st) {
    if (a.wr == 1 && a.wq == 8) return launch_tile_km<1, 8>(a.km, a, st);
    if (a.wr == 2 && a.wq == 2) return launch_tile_km<2, 2>(a.km, a, st);
    if (a.wr == 2 && a.wq == 1) return launch_tile_km<2, 1>(a.km, a, st);
    return hipErrorInvalidValue;
}

hipError_t launch_merge(const float* cd, const int64_t* ci, int64_t nq, int nlists, int kin,
                        int64_t stride_q, int64_t stride_l, int k, int metric, int negate_in,
                        float* D, int64_t* I, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nq + 3) / 4)), block(256);
    if (k <= 8)
        hipLaunchKernelGGL(knn_merge_kernel<8>, grid, block, 0, st, cd, ci, nq, nlists, kin, stride_q,
                           stride_l, k, metric, negate_in, D, I);
    else if (k <= 16)
        hipLaunchKernelGGL(knn_merge_kernel<16>, grid, block, 0, st, cd, ci, nq, nlists, kin,
                           stride_q, stride_l, k, metric, negate_in, D, I);
    else if (k <= 32)
        hipLaunchKernelGGL(knn_merge_kernel<32>, grid, block, 0, st, cd, ci, nq, nlists, kin,
                           stride_q, stride_l, k, metric, negate_in, D, I);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_fill_empty(float* D, int64_t* I, int64_t n, int metric, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_empty_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, D, I,
                       n, metric);
    return hipGetLastError();
}

}  // namespace imgrec
