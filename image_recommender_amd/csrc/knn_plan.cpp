// knn_plan.cpp — launch geometry of the fused distance + top-k kernels and the relative
// error-bound coefficients of the candidate paths' certificate (DESIGN.md "Launch plan",
// "bf16 path", "Split path").
#include <cmath>
#include <cstdlib>

#include "knn_index.h"

namespace imgrec {

// Fused-kernel geometry for one query chunk of the exact fp32 path.
Plan make_plan(int64_t ntotal, int64_t nq, int k, int cus) {
    Plan p{};
    p.km = k <= 8 ? 8 : (k <= 10 ? 10 : (k <= 16 ? 16 : 32));
    int wg_per_cu;
    if (nq <= 32) { p.wr = 2; p.wq = 1; wg_per_cu = 3; }
    else if (nq <= 128) { p.wr = 2; p.wq = 2; wg_per_cu = 2; }
    // Two independent 4-wave workgroups per CU: their barriers do not line up, so one
    // workgroup's stage bubble is filled by the other's MFMAs (31.4 vs 32.2 ms for one 8-wave
    // (1,8) workgroup, bench config).
    else { p.wr = 1; p.wq = 4; wg_per_cu = 2; }
    p.bm = p.wr * 128;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
    const int target = cus * wg_per_cu;
    int ns = (target + p.nqb - 1) / p.nqb;
    ns = std::max(1, std::min(ns, p.ntiles));
    p.nsplit = ns;
    p.ncand = ns * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

int fallback_km(int k) { return k <= 8 ? 8 : (k <= 10 ? 10 : (k <= 16 ? 16 : 32)); }

// Split-path geometry: one tile shape for every batch size ((1,4) workgroups, two per CU,
// kSplitWB row blocks per wave).
Plan make_split_plan(int64_t ntotal, int64_t nq, int kc, int cus) {
    Plan p{};
    p.km = kc;
    p.wr = 1;
    p.wq = 4;
    p.bm = p.wr * 32 * kSplitWB;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
    const int target = cus * 2;
    p.nsplit = std::max(1, std::min((target + p.nqb - 1) / p.nqb, p.ntiles));
    p.ncand = p.nsplit * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

// Split-bf16 candidate path (knn_refine.hip): used for batches the (1,4) plan covers, k <= 16,
// rows padded to 32 floats.  K' = candidates kept per query for the exact rerank.
int split_kc(int k) { return k <= 10 ? 16 : (k <= 16 ? 32 : 0); }

// Relative error-bound coefficients of the certificate (DESIGN.md "Split path"), multiplied by
// |q| * max|x| in the kernel:
//   split dot:  3.1 * 2^-16 (dropped lo.lo / residual terms of x = hi + lo + r, |r| <= 2^-16 |x|)
//               + 1.02 * gamma_n, n = 3 MFMAs x (dp/16) steps x 5 (a 16-term tree inside each),
//               with unit roundoff 2^-23 (allows truncating accumulation);
//   rerank dot: 1.02 * gamma_n, n = 4*ceil(dp/256) + 8 fp32 FMAs + butterfly levels, u = 2^-24.
float split_coef(int dp) {
    return (float)(3.1 * std::ldexp(1.0, -16) + 1.02 * (15.0 * (dp / 16) + 16.0) * std::ldexp(1.0, -23));
}
float rerank_coef(int dp) {
    return (float)(1.02 * (4.0 * ((dp + 255) / 256) + 8.0) * std::ldexp(1.0, -24));
}

// bf16 candidate pass (one bf16 MFMA per product): the products of two bf16 values are exact in
// fp32, so the only arithmetic error besides the operand rounding (bounded in the rerank kernel
// from the stored residual norms) is the fp32 accumulation: 1.02 * gamma_n, n = (dpb/16) MFMAs x 5
// (a 16-term tree inside each) + 16, with unit roundoff 2^-23 (allows truncating accumulation),
// relative to |qh| |xh|.
float b16_acc_coef(int dpb) {
    return (float)(1.02 * (5.0 * (dpb / 16) + 16.0) * std::ldexp(1.0, -23));
}
// int8 small-batch pass (knn_i8.hip): per block an exact int32 dot of the row's and the query's
// codes per level (exact in fp32 as well, |D| < 2^24), the fold s_x (s_hi D_hi + s_lo D_lo) into
// the lane's accumulator (three roundings), ceil(nblk/16) blocks per lane, then the 16-lane DPP
// sum: gamma_n with n = 3 + ceil(nblk/16) + 4 — bounded here, generously, by
// 1.02 * (16 + 4 ceil(nblk/16)) u, u = 2^-23, relative to (|q| + dq)(|x~|) as the bf16 one.
float i8_acc_coef(int nblk) {
    return (float)(1.02 * (16.0 + 4.0 * ((nblk + 15) / 16)) * std::ldexp(1.0, -23));
}

// int8-path geometry: one workgroup per row split, kI8WGPCU per CU, all of the batch's queries
// in each; one folded list of km per (query, split)
// (two 4-wave workgroups per CU are resident at the kernel's 222 VGPRs; three per CU, i.e. a
// second partial round, measured faster at nq = 1 / 2: 0.366 / 0.375 vs 0.386 / 0.399 ms kernel,
// profiles/r03/i8_small_batch/sweep.jsonl; IMGREC_I8_WGPCU overrides for measurements)
// Workgroups per CU of the int8 scan: 2 for one or two queries (fewer lists for the merge, and
// the scan itself no slower: cfg2 one query 0.187 -> 0.182 ms), 3 from four queries on (cfg2 at
// nq = 8: 0.406 ms with 2, 0.358 with 3) — profiles/r04/i8_wgpcu/.
// Workgroups per CU of the int8 scan: 3 from three queries, 2 for one or two (fewer lists for the
// merge, no slower a scan: profiles/r04/i8_wgpcu/), 1 for ONE query on rows of >= 24 blocks (the
// 1M x 1968 scan 0.311 -> 0.308 ms and the search 3 us shorter on two boxes, while 1M x 768 rows
// lose 28 us with one: sweep_nq1_b.txt).  IMGREC_I8_WGPCU overrides.
Plan make_i8_plan(int64_t ntotal, int64_t nq, int k, int cus, int wgpcu, int nblk) {
    const int kI8WGPCU = wgpcu > 0 ? wgpcu : (nq == 1 && nblk >= 24 ? 1 : nq <= 2 ? 2 : 3);
    Plan p{};
    p.km = b16_km(k);
    p.wr = 1;
    p.wq = 1;
    p.bm = 8;
    p.bq = (int)nq;
    p.nqb = 1;
    p.nq_pad = (int)nq;
    const int64_t groups = (ntotal + 7) / 8;
    p.ntiles = (int)groups;
    p.nsplit = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * kI8WGPCU, groups));
    p.ncand = p.nsplit * p.km;
    p.wgs = p.nsplit;
    return p;
}

// per-lane list length of the generic bf16 tile (the merge floor covers what a lane list drops)
int b16_km(int k) { return k <= 16 ? 16 : 32; }

constexpr int kB16NarrowQ = 32;   // batches up to this use the 32-query tile

// bf16-path geometry: large batches with k <= 10 on the 256 x 256-tile kernel (one workgroup
// per CU, lane lists of 8 / 10); otherwise (kB16WR, kB16WQ) workgroups, kB16WGPCU per CU.
Plan make_b16_plan(int64_t ntotal, int64_t nq, int k, int cus, int dpb) {
    Plan p{};
    // (dpb bound: the 256 x 256 kernel's 32-bit lane offsets, see launch_b16_big)
    if (nq >= kB16BigMinQ && k <= 10 && dpb <= 16384) {
        p.big = true;
        p.km = k <= 8 ? 8 : 10;
        p.wr = 2;
        p.wq = 4;
        p.bm = kB16BigRows;
        p.bq = kB16BigQueries;
        p.nqb = (int)((nq + p.bq - 1) / p.bq);
        p.nq_pad = p.nqb * p.bq;
        p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
        p.nsplit = std::max(1, std::min((cus + p.nqb - 1) / p.nqb, p.ntiles));
        p.ncand = p.nsplit * p.km;               // lists folded to one per (query, split)
        p.wgs = p.nqb * p.nsplit;
        // packed lists (16x16 kernel): split-local row index t * 256 + tile row of every tile of
        // the largest split must fit ib bits
        p.ib = 0;
        if (IMGREC_B16_MFMA16) {
            const int64_t groups = (ntotal + 7) / 8, cnt = (groups + p.nsplit - 1) / p.nsplit;
            const int64_t idx_max = (cnt + 31) / 32 * 256 - 1;
            int ib = 1;
            while ((int64_t{1} << ib) <= idx_max) ++ib;
            if (ib <= kB16PackMaxIB) p.ib = ib;
        }
        return p;
    }
    p.km = b16_km(k);
    // batches of <= 32 queries: a 32-query tile (the (1,4) tile would pad them to 128 and spend
    // four times the matrix work of an HBM-bound search)
    const bool narrow = nq <= kB16NarrowQ;
    p.wr = narrow ? 2 : kB16WR;
    p.wq = narrow ? 1 : kB16WQ;
    p.bm = p.wr * 32 * kB16WB;
    p.bq = p.wq * 32;
    p.nqb = (int)((nq + p.bq - 1) / p.bq);
    p.nq_pad = p.nqb * p.bq;
    p.ntiles = (int)((ntotal + p.bm - 1) / p.bm);
    const int target = cus * kB16WGPCU;
    p.nsplit = std::max(1, std::min((target + p.nqb - 1) / p.nqb, p.ntiles));
    p.ncand = p.nsplit * p.wr * 2 * p.km;
    p.wgs = p.nqb * p.nsplit;
    return p;
}

}  // namespace imgrec
