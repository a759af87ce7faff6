// knn_search.cpp — the three search arithmetics of one k-NN index and their device-side
// certificate handling (DESIGN.md "Kernels"):
//
//   exact   the fused fp32 MFMA distance + top-k kernel, then the list merge;
//   bf16    bf16 candidate pass (one bf16 MFMA per product) -> candidate merge (top K' = 64 +
//           list floor) -> fp32 rerank + certificate, with a second chance over every per-split
//           list entry for queries the first certificate cannot settle;
//   split   split-bf16 candidate pass (three bf16 MFMAs per product) -> merge -> rerank +
//           certificate (+ second chance).
//
// Queries no certificate settles are re-run exactly inside the certificate tail kernel, planned on
// the device: the count never travels to the host, so knn_search_device enqueues a whole search
// without waiting for the GPU.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "knn_index.h"

namespace imgrec {

namespace {

// Timing events around the dominant (fused) kernel launch of a chunk.
int timed_begin(knn_index* ix, hipStream_t st, hipEvent_t* e1) {
    *e1 = nullptr;
    if (!ix->timing) return KNN_OK;
    if (ix->ev_used + 2 > ix->ev.size()) {
        for (int i = 0; i < 64; ++i) {
            hipEvent_t e;
            KNN_HIP(hipEventCreate(&e));
            ix->ev.push_back(e);
        }
    }
    KNN_HIP(hipEventRecord(ix->ev[ix->ev_used], st));
    *e1 = ix->ev[ix->ev_used + 1];
    ix->ev_used += 2;
    return KNN_OK;
}

// Exact fp32 path over nq padded queries (qpad holds make_plan(nq).nq_pad zero-padded rows).
int exact_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
                int64_t* I, hipStream_t st, bool timed) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    int rc;
    if (stream_lists_ok(ix, nq)) {
        // <= 4 queries: the corpus streamed once (HBM-bound) into exact lists of 32 per row
        // split, merged — instead of 32-query fp32 MFMA tiles that compute 28-31 padding queries
        // (d = 48 colour-only or d = 1968 exact mode, one query on 1M rows; profiles/r05/stream/)
        const int sp = stream_splits(ix);
        const size_t nc = (size_t)sp * KNN_MAX_K;
        if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * nc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * nc)) != KNN_OK) return rc;
        hipEvent_t e1 = nullptr;
        if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
        KNN_HIP(launch_stream_lists(ix, qpad, qnorm, nq, kmetric, sp, ix->cand_d, ix->cand_i, st));
        if (e1) KNN_HIP(hipEventRecord(e1, st));
        KNN_HIP(launch_merge(ix->cand_d, ix->cand_i, nq, sp, KNN_MAX_K, (int64_t)nc, KNN_MAX_K, k,
                             kmetric, 0, D, I, st));
        return KNN_OK;
    }
    const Plan p = make_plan(ix->ntotal, nq, k, ix->cus);
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = p.km;
    a.xb = ix->xb; a.xnorm = ix->xn; a.nrows = (int)ix->ntotal; a.dp = ix->dp;
    a.qp = qpad; a.qnorm = qnorm; a.nq = (int)nq; a.metric = kmetric;
    a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb; a.id_offset = ix->id_offset;
    a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand; a.mode = kModeF32;
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    KNN_HIP(launch_merge(ix->cand_d, ix->cand_i, nq, p.ncand / p.km, p.km, p.ncand, p.km, k,
                         kmetric, 0, D, I, st));
    return KNN_OK;
}

// max |x|^2 (and max bf16 residual) over the stored rows, recomputed after rows change
int refresh_maxima(knn_index* ix, hipStream_t st) {
    if (!ix->xn_max_stale) return KNN_OK;
    int rc;
    if ((rc = grow(&ix->xn_max, &ix->xn_max_cap, 1)) != KNN_OK) return rc;
    KNN_HIP(launch_max_norm(ix->xn, ix->ntotal, ix->xn_max, st));
    if (ix->b16_ok) {
        if ((rc = grow(&ix->xr_max, &ix->xr_max_cap, 1)) != KNN_OK) return rc;
        KNN_HIP(launch_max_norm(ix->xr, ix->ntotal, ix->xr_max, st));
    }
    if (ix->x8) {
        if ((rc = grow(&ix->x8r_max, &ix->x8r_max_cap, 1)) != KNN_OK) return rc;
        KNN_HIP(launch_max_norm(ix->x8r, ix->ntotal, ix->x8r_max, st));
    }
    ix->xn_max_stale = false;
    return KNN_OK;
}

// Certificate counters (two chunk parities + per-search totals, zeroed once here; the fallback
// prep kernel folds and re-zeroes them) and the uncertified-query list.
int grow_stats(knn_index* ix, int64_t nq, hipStream_t st) {
    if (!ix->stat) {
        KNN_HIP(hipMalloc((void**)&ix->stat, 12 * sizeof(int)));
        KNN_HIP(hipMemsetAsync(ix->stat, 0, 12 * sizeof(int), st));
        ix->stat_seq = 0;
    }
    int rc = grow(&ix->fail, &ix->fail_cap, (size_t)nq);
    if (rc != KNN_OK) return rc;
    return grow(&ix->chance, &ix->chance_cap, (size_t)nq);
}

// The rerank + certificate of a candidate chunk, then its whole tail in ONE launch
// (cert_tail_kernel: second chance, stats fold, and the exact fp32 re-run of the queries neither
// certificate settles — planned on the device, so the host never waits).  With every query
// certified the tail is one near-empty launch.
int certify_chunk(knn_index* ix, RerankArgs& r, const float* qpad, const float* qnorm, int64_t nq,
                  int k, float* D, int64_t* I, hipStream_t st, bool first) {
    const int parity = ix->stat_seq & 1;
    const int km = fallback_km(k);
    const int grid = kTailWGPerCU * ix->cus;
    const int64_t cap_rows = round_up(nq, 32);
    const int bm = 128 * kFallbackWR;
    const int lists_km = 2 * kFallbackWR * km;
    // candidate lists of the exact re-run: nqb query blocks x nsplit = max(1, grid / nqb) row
    // splits, lists_km entries per (query, split).  nqb * nsplit <= grid while nqb <= grid; past
    // that (more than 32 x grid uncertified queries: a device with fewer CUs) nsplit = 1 and the
    // lists need cap_rows x lists_km (sizing by the grid alone overflowed there)
    const size_t ncap = (size_t)std::max<int64_t>(grid, cap_rows / 32) * 32 * lists_km;
    int rc;
    if ((rc = grow(&ix->fb_q, &ix->fb_q_cap, (size_t)cap_rows * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_qn, &ix->fb_qn_cap, (size_t)cap_rows)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_cd, &ix->fb_cd_cap, ncap)) != KNN_OK) return rc;
    if ((rc = grow(&ix->fb_ci, &ix->fb_ci_cap, ncap)) != KNN_OK) return rc;
    if ((rc = grow(&ix->tail_ctl, &ix->tail_ctl_cap, (size_t)4 + cap_rows / 32)) != KNN_OK) return rc;
    r.stats = ix->stat + 4 * parity;
    r.fail_list = ix->fail;
    r.chance_list = ix->chance;
    if (r.raw_d) {
        // sliced second chance: up to 64 slices per item (profiles/r03/second_chance/)
        static const int kSlices = [] {           // IMGREC_SC_SLICES overrides (measurements)
            const char* e = std::getenv("IMGREC_SC_SLICES");
            const int v = e ? std::atoi(e) : 0;
            return v > 0 ? v : 64;
        }();
        // (<= 64: the last slice's merge reads the slice heads from the lanes of one wave;
        // S k <= 1024 = kWideCap, knn_certify.h: it stages the S lists of k in LDS)
        r.sc_slices = std::max(1, std::min({kSlices, 64, r.raw_lists, 1024 / k}));
        const size_t ns = (size_t)nq * r.sc_slices * k;
        if ((rc = grow(&ix->sc_key, &ix->sc_key_cap, ns)) != KNN_OK) return rc;
        if ((rc = grow(&ix->sc_lab, &ix->sc_lab_cap, ns)) != KNN_OK) return rc;
        if ((rc = grow(&ix->sc_meta, &ix->sc_meta_cap, (size_t)nq * r.sc_slices * 4)) != KNN_OK) return rc;
        const size_t c0 = ix->sc_done_cap;
        if ((rc = grow(&ix->sc_done, &ix->sc_done_cap, (size_t)nq)) != KNN_OK) return rc;
        if (ix->sc_done_cap != c0)      // (re)allocated: the self-resetting counters start at 0
            KNN_HIP(hipMemsetAsync(ix->sc_done, 0, ix->sc_done_cap * sizeof(int), st));
        r.sc_key = ix->sc_key; r.sc_lab = ix->sc_lab; r.sc_meta = ix->sc_meta; r.sc_done = ix->sc_done;
    }
    r.tail_ctl = ix->tail_ctl;
    // (small batches only: a large batch's rerank is throughput-bound and its second chances
    // queue up in the tail; at 1024 queries the A/B was within the +-15 us noise of the step,
    // profiles/r04/chance_skip/ab_env_nq1024*.txt, so large batches keep the round-3 route)
    r.chance_skip = ix->chance_skip && r.raw_d && nq <= ix->cus ? 1 : 0;
    // first rerank phase of k rows for batches past one rerank workgroup per CU
    // (IMGREC_RERANK_P1: 0 keeps 16 everywhere, for A/B)
    r.p1 = ix->rerank_p1k && nq > ix->cus ? k : 0;
    // 4-wave rerank workgroups past one per CU (four resident per CU, one round for 1024 queries):
    // opt-in (IMGREC_RERANK_NW4=1) — measured 3-4 us slower per 125k-row step than 8 waves, the
    // rerank is not residency-bound (profiles/r05/rerank_nw4_ab/)
    r.nw = ix->rerank_nw4 && nq > ix->cus && r.l1_G == 0 && r.s_lists == 0 && !r.chance_skip ? 4 : 0;
    if (!r.direct) KNN_HIP(launch_rerank_certify(r, st));
    TailArgs t{};
    t.r = r;
    t.parity = parity;
    t.first = first ? 1 : 0;
    t.stat = ix->stat;
    t.qpad = qpad;
    t.qnorm = qnorm;
    t.dp = ix->dp;
    t.nrows = (int)ix->ntotal;
    t.ntiles = (int)((ix->ntotal + bm - 1) / bm);
    t.metric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    t.xb = ix->xb;
    t.xn = ix->xn;
    t.id_offset = ix->id_offset;
    t.fq = ix->fb_q;
    t.fqn = ix->fb_qn;
    t.fcd = ix->fb_cd;
    t.fci = ix->fb_ci;
    t.ticket = ix->tail_ctl + 4;
    t.km = km;
    t.lists_km = lists_km;
    const hipError_t e = launch_cert_tail(t, grid, st);
    if (e != hipSuccess) {        // the parities may hold this chunk's counts: start clean
        (void)hipMemsetAsync(ix->stat, 0, 12 * sizeof(int), st);
        ix->stat_seq = 0;
        KNN_FAIL(KNN_EHIP, "certificate tail launch failed: %s", hipGetErrorString(e));
    }
    ++ix->stat_seq;
    ix->stat_valid = true;
    ix->last_split_queries += nq;
    return KNN_OK;
}

// The candidate merge's second level inside the rerank kernel (one launch fewer: ~10 us at
// nq = 1, where it is one wave's select behind a kernel boundary) while the batch leaves the rerank
// at most one workgroup per CU; larger batches keep the separate level-2 launch (its 4-wave blocks
// do not idle seven waves of each rerank workgroup behind the select).  IMGREC_MERGE_FUSE=0 at
// index creation: off.
bool fuse_merge_level2(const knn_index* ix, int64_t nq) {
    return ix->merge_fuse && nq <= ix->cus;
}

// Both merge levels inside the rerank (RerankArgs::l0_lists): small batches whose merge would
// take two levels of 16-entry lists with at most one group of 64 lists per rerank wave — no merge
// launch at all (the level-1 launch was ~9 us of a one-query search).
bool fuse_merge_level1(const knn_index* ix, int64_t nq, int nlists, int km) {
    return fuse_merge_level2(ix, nq) && ix->merge_fuse1 && km == 16 && nlists > 64 &&
           nlists <= 64 * kRerankWavesHost;
}

// A single-level merge (<= 64 per-split lists of <= 16: the 256 x 256 kernel's 64 lists of 8 / 10)
// inside the rerank workgroup (RerankArgs::s_lists): no merge launch and no round trip of the K'
// candidates through global memory.  Measured at 1024 queries it saves nothing — the 10.8-us
// launch comes back as rerank workgroups that hold their CU longer (125k rows 0.4815 vs 0.4846 ms
// per step, cfg3 3.181 vs 3.189, two runs each on one box: profiles/r05/merge_rerank_ab/) — so it
// is opt-in: IMGREC_MERGE_SINGLE=1 at index creation.
bool fuse_merge_single(const knn_index* ix, int nlists, int km) {
    return ix->merge_single && nlists <= 64 && km <= 16;
}

// Sibling lockstep of the 256 x 256 bf16 kernel (TileArgs::sync): IMGREC_B16W_SYNC_LAG = the
// tiles a workgroup may run ahead of the slowest workgroup of its row split; unset or negative =
// off.
int b16_sync_lag() {
    static const int v = [] {
        const char* e = test_knob("IMGREC_B16W_SYNC_LAG");
        return e && *e ? std::atoi(e) : -1;
    }();
    return v;
}

// bf16 candidates (one bf16 MFMA per product) + exact fp32 rerank of K' = 64 + certificate.
int b16_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
              int64_t* I, hipStream_t st, bool timed, bool q_ready, bool first) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int kc = kB16Cand;
    const Plan p = make_b16_plan(ix->ntotal, nq, k, ix->cus, ix->dpb);
    const int km = p.km;
    int rc;
    if ((rc = refresh_maxima(ix, st)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qb16, &ix->qb16_cap, (size_t)p.nq_pad * ix->dpb)) != KNN_OK) return rc;
    if ((rc = grow(&ix->q_resid, &ix->q_resid_cap, (size_t)p.nq_pad)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_d, &ix->cand2_d_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_i, &ix->cand2_i_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->floor, &ix->floor_cap, (size_t)nq)) != KNN_OK) return rc;
    if ((rc = grow_stats(ix, nq, st)) != KNN_OK) return rc;
    if (!q_ready)   // else search_locked's fused query prep already wrote qb16 / q_resid
        KNN_HIP(launch_bf16_rows(qpad, p.nq_pad, ix->dp, ix->dpb, ix->qb16, ix->q_resid, st));
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = km; a.wb = kB16WB; a.mode = kModeBF16;
    a.xb = reinterpret_cast<const float*>(ix->xh); a.xnorm = ix->xn; a.nrows = (int)ix->ntotal;
    a.dp = ix->dpb / 2; a.qp = reinterpret_cast<const float*>(ix->qb16); a.qnorm = qnorm;
    a.nq = (int)nq; a.metric = kmetric; a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb;
    a.id_offset = ix->id_offset; a.cand_d = ix->cand_d; a.cand_i = ix->cand_i; a.ncand = p.ncand;
    a.ib = p.big ? p.ib : 0;
    if (p.big && b16_sync_lag() >= 0) {
        // sibling lockstep of the 256 x 256 kernel: progress slots zeroed once, a new epoch per
        // launch (values of earlier launches compare as "not yet")
        const size_t cap0 = ix->b16_sync_cap;
        if ((rc = grow(&ix->b16_sync, &ix->b16_sync_cap, (size_t)p.wgs)) != KNN_OK) return rc;
        if (ix->b16_sync_cap != cap0)
            KNN_HIP(hipMemsetAsync(ix->b16_sync, 0, ix->b16_sync_cap * sizeof(uint32_t), st));
        ix->b16_epoch = (ix->b16_epoch + 1) & 0xffffu;
        a.sync = ix->b16_sync;
        a.epoch = ix->b16_epoch;
        a.sync_lag = b16_sync_lag();
    }
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(p.big ? launch_b16_big(a, st) : launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    const int nlists = p.ncand / km, ngrp = (nlists + 63) / 64;
    if (ngrp > 1) {
        if ((rc = grow(&ix->mws_d, &ix->mws_d_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_i, &ix->mws_i_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_f, &ix->mws_f_cap, (size_t)nq * ngrp)) != KNN_OK) return rc;
    }
    int l1G = 0;
    const bool single = fuse_merge_single(ix, nlists, km);
    const bool l0 = !single && fuse_merge_level1(ix, nq, nlists, km);
    if (l0) l1G = (nlists + 63) / 64;
    else if (!single)
        KNN_HIP(launch_merge_candidates(ix->cand_d, ix->cand_i, nq, nlists, km, p.ncand, km, kc,
                                        ix->id_offset, ix->cand2_d, ix->cand2_i, ix->floor,
                                        ix->mws_d, ix->mws_i, ix->mws_f, st,
                                        fuse_merge_level2(ix, nq) ? &l1G : nullptr));
    RerankArgs r{};
    r.mode = kModeBF16;
    if (single) r.s_lists = nlists;
    r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
    r.xn_max = ix->xn_max; r.id_offset = ix->id_offset; r.cd = ix->cand2_d; r.ci = ix->cand2_i;
    r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = b16_acc_coef(ix->dpb);
    r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
    r.c_trunc = a.ib > 0 ? (float)std::ldexp(1.0, a.ib - 23) : 0.f;
    r.q_resid = ix->q_resid; r.xr_max = ix->xr_max; r.floor = ix->floor;
    if (l1G > 0) { r.l1_d = ix->mws_d; r.l1_i = ix->mws_i; r.l1_floor = ix->mws_f; r.l1_G = l1G; }
    if (l0) r.l0_lists = nlists;
    r.raw_d = ix->cand_d; r.raw_i = ix->cand_i; r.raw_lists = nlists; r.raw_km = km;
    r.raw_stride_q = p.ncand;
    return certify_chunk(ix, r, qpad, qnorm, nq, k, D, I, st, first);
}

// Block-scaled int8 candidates (int8 dot4 products, batches of <= kI8MaxQ queries) + exact fp32
// rerank of K' = 64 + certificate: the bf16 path's chain with the int8 copy's bound.
int i8_chunk(knn_index* ix, const float* qraw, const float* qpad, const float* qnorm, int64_t nq,
             int k, float* D, int64_t* I, hipStream_t st, bool timed, bool first) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int kc = kB16Cand;
    const Plan p = make_i8_plan(ix->ntotal, nq, k, ix->cus, ix->i8_wgpcu, ix->nblk8);
    // direct: no merge, no rerank launch — the certificate tail reranks every query's list entries
    // under its prefix limit (RerankArgs::direct); the scan zeroes the tail's claim counters and
    // (raw: <= 4 queries) writes its 16 lane lists per split unfolded
    const bool direct = ix->chance_direct_max > 0 && nq <= ix->chance_direct_max && k <= 64;
    // (unfolded while they make <= 4096 lists per query, i.e. <= 1024 entries per second-chance
    // slice: config 3's 256 splits 2 us faster, config 2's 512 splits 1 us slower than folded,
    // profiles/r05/nq1/direct_raw/; IMGREC_DIRECT_RAW=2: unfolded at any split count)
    const bool raw = direct && nq <= 4 &&
                     (ix->direct_raw == 2 || (ix->direct_raw == 1 && 16 * p.nsplit <= 4096));
    const int ncand = raw ? p.nsplit * 16 * p.km : p.ncand;
    int rc;
    if ((rc = ensure_i8(ix, st)) != KNN_OK) return rc;
    if ((rc = refresh_maxima(ix, st)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_d, &ix->cand2_d_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_i, &ix->cand2_i_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->floor, &ix->floor_cap, (size_t)nq)) != KNN_OK) return rc;
    if ((rc = grow_stats(ix, nq, st)) != KNN_OK) return rc;
    // qraw non-NULL: the scan quantises the raw query rows itself and writes qpad / qnorm /
    // q8r (I8Args::qsrc); otherwise the codes ix->q8 / q8s / q8r came with qpad from
    // launch_i8_query_prep
    I8Args a{};
    a.codes = ix->x8; a.scales = ix->x8s; a.xnorm = ix->xn; a.nrows = (int)ix->ntotal;
    a.nblk = ix->nblk8; a.nq = (int)nq;
    if (qraw) {
        a.qsrc = qraw; a.d = ix->d; a.dp = ix->dp;
        a.normalize = ix->metric == KNN_METRIC_COSINE ? 1 : 0;
        a.qpad = const_cast<float*>(qpad); a.qnorm_out = const_cast<float*>(qnorm); a.qresid = ix->q8r;
    } else {
        a.qcodes = ix->q8; a.qscales = ix->q8s; a.qnorm = qnorm;
    }
    a.km = p.km;
    a.nsplit = p.nsplit; a.l2 = kmetric; a.id_offset = ix->id_offset; a.cand_d = ix->cand_d;
    a.cand_i = ix->cand_i; a.ncand = ncand; a.raw16 = raw ? 1 : 0;
    if (p.nsplit == 2 * ix->cus) a.half_k = ix->i8_half_k;     // two workgroups per CU
    if (ix->i8_pool64 > 0 && nq <= 2 && p.km == 16 &&
        (ix->i8_pool_forced || (nq == 1 && p.nsplit == ix->cus))) {
        // run-time pool of the last row groups (I8Args::pool): replaces the half_k shift
        if (!ix->i8_dyn) {
            KNN_HIP(hipMalloc((void**)&ix->i8_dyn, 2 * sizeof(int)));
            KNN_HIP(hipMemsetAsync(ix->i8_dyn, 0, 2 * sizeof(int), st));
        }
        a.dyn = ix->i8_dyn;
        a.pool = (int)((ix->ntotal + 7) / 8 * ix->i8_pool64 / 64);
        a.pool_ch = ix->i8_pool_ch;
        a.half_k = 0;
    }
    if (direct) {
        if ((rc = grow(&ix->tail_ctl, &ix->tail_ctl_cap, (size_t)4 + round_up(nq, 32) / 32)) != KNN_OK)
            return rc;
        a.zero_ctl = ix->tail_ctl;
        if ((rc = grow(&ix->heads, &ix->heads_cap, (size_t)nq * p.nsplit)) != KNN_OK) return rc;
        a.heads = ix->heads;
    }
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(launch_i8_scan(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    const int nlists = p.nsplit, ngrp = (nlists + 63) / 64;
    if (direct) {
        RerankArgs r{};
        r.mode = kModeI8;
        r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
        r.xn_max = ix->xn_max; r.id_offset = ix->id_offset;
        r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = i8_acc_coef(ix->nblk8);
        r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
        r.q_resid = ix->q8r; r.xr_max = ix->x8r_max;
        r.raw_d = ix->cand_d; r.raw_i = ix->cand_i; r.raw_lists = raw ? 16 * nlists : nlists;
        r.raw_km = p.km;
        r.raw_stride_q = ncand;
        r.direct = 1;
        r.heads = ix->heads;
        r.heads_n = nlists;
        return certify_chunk(ix, r, qpad, qnorm, nq, k, D, I, st, first);
    }
    if (ngrp > 1) {
        if ((rc = grow(&ix->mws_d, &ix->mws_d_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_i, &ix->mws_i_cap, (size_t)nq * ngrp * kc)) != KNN_OK) return rc;
        if ((rc = grow(&ix->mws_f, &ix->mws_f_cap, (size_t)nq * ngrp)) != KNN_OK) return rc;
    }
    int l1G = 0;
    const bool l0 = fuse_merge_level1(ix, nq, nlists, p.km);
    if (l0) l1G = (nlists + 63) / 64;
    else
        KNN_HIP(launch_merge_candidates(ix->cand_d, ix->cand_i, nq, nlists, p.km, p.ncand, p.km, kc,
                                        ix->id_offset, ix->cand2_d, ix->cand2_i, ix->floor,
                                        ix->mws_d, ix->mws_i, ix->mws_f, st,
                                        fuse_merge_level2(ix, nq) ? &l1G : nullptr));
    RerankArgs r{};
    r.mode = kModeI8;
    r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
    r.xn_max = ix->xn_max; r.id_offset = ix->id_offset; r.cd = ix->cand2_d; r.ci = ix->cand2_i;
    r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = i8_acc_coef(ix->nblk8);
    r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
    r.c_trunc = 0.f;
    r.q_resid = ix->q8r; r.xr_max = ix->x8r_max; r.floor = ix->floor;
    if (l1G > 0) { r.l1_d = ix->mws_d; r.l1_i = ix->mws_i; r.l1_floor = ix->mws_f; r.l1_G = l1G; }
    if (l0) r.l0_lists = nlists;
    r.raw_d = ix->cand_d; r.raw_i = ix->cand_i; r.raw_lists = nlists; r.raw_km = p.km;
    r.raw_stride_q = p.ncand;
    return certify_chunk(ix, r, qpad, qnorm, nq, k, D, I, st, first);
}

// Split-bf16 candidates + exact rerank + certificate.
int split_chunk(knn_index* ix, const float* qpad, const float* qnorm, int64_t nq, int k, float* D,
                int64_t* I, hipStream_t st, bool timed, bool first) {
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    const int kc = split_kc(k);
    const Plan p = make_split_plan(ix->ntotal, nq, kc, ix->cus);
    int rc;
    if ((rc = ensure_split(ix, st)) != KNN_OK) return rc;
    if ((rc = refresh_maxima(ix, st)) != KNN_OK) return rc;
    if ((rc = grow(&ix->qsplit, &ix->qsplit_cap, (size_t)p.nq_pad * ix->dp)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_d, &ix->cand_d_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand_i, &ix->cand_i_cap, (size_t)nq * p.ncand)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_d, &ix->cand2_d_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow(&ix->cand2_i, &ix->cand2_i_cap, (size_t)nq * kc)) != KNN_OK) return rc;
    if ((rc = grow_stats(ix, nq, st)) != KNN_OK) return rc;
    KNN_HIP(launch_split_rows(qpad, p.nq_pad, ix->dp, kSplitBK, ix->qsplit, st));
    TileArgs a{};
    a.wr = p.wr; a.wq = p.wq; a.km = kc;
    a.xb = reinterpret_cast<const float*>(ix->xs); a.xnorm = ix->xn; a.nrows = (int)ix->ntotal;
    a.dp = ix->dp; a.qp = reinterpret_cast<const float*>(ix->qsplit); a.qnorm = qnorm;
    a.nq = (int)nq; a.metric = kmetric; a.ntiles = p.ntiles; a.nsplit = p.nsplit; a.nqb = p.nqb;
    a.id_offset = ix->id_offset; a.cand_d = ix->cand_d; a.cand_i = ix->cand_i;
    a.ncand = p.ncand; a.mode = kModeSplit;
    a.wb = kSplitWB; a.sbk = kSplitBK;
    hipEvent_t e1 = nullptr;
    if (timed && (rc = timed_begin(ix, st, &e1)) != KNN_OK) return rc;
    KNN_HIP(launch_tile_topk(a, st));
    if (e1) KNN_HIP(hipEventRecord(e1, st));
    // global top-K' approximate candidates, raw ascending keys (merge in its L2 convention)
    KNN_HIP(launch_merge(ix->cand_d, ix->cand_i, nq, p.ncand / kc, kc, p.ncand, kc, kc, 1, 0,
                         ix->cand2_d, ix->cand2_i, st));
    RerankArgs r{};
    r.mode = kModeSplit;
    r.qp = qpad; r.qnorm = qnorm; r.dp = ix->dp; r.xb = ix->xb; r.xn = ix->xn;
    r.xn_max = ix->xn_max; r.id_offset = ix->id_offset; r.cd = ix->cand2_d; r.ci = ix->cand2_i;
    r.kc = kc; r.nq = nq; r.k = k; r.metric = kmetric; r.c_split = split_coef(ix->dp);
    r.c_fp = rerank_coef(ix->dp); r.D = D; r.I = I;
    r.raw_d = ix->cand_d; r.raw_i = ix->cand_i; r.raw_lists = p.ncand / kc; r.raw_km = kc;
    r.raw_stride_q = p.ncand;
    return certify_chunk(ix, r, qpad, qnorm, nq, k, D, I, st, first);
}

}  // namespace

// AUTO: the bf16 path at every corpus size.  Large batches are matrix-bound (bf16 MFMA vs fp32
// MFMA), small ones HBM-bound (the bf16 copy streams half the bytes), and on small corpora the
// exact kernel has a latency floor of its own: one 256-row tile's whole depth of fp32 MFMAs per
// workgroup, ~0.16 ms from 1000 rows up, against the candidate path's ~0.05-0.1 ms
// (profiles/r03/small_corpora/: 1000-131072 rows x nq 9-1024, bf16 1.8-2.8x faster).
bool use_b16(const knn_index* ix, int64_t nq, int k) {
    if (!ix->b16_ok || k > KNN_MAX_K) return false;
    if (ix->mode == KNN_SEARCH_BF16) return true;
    // (I8 mode: batches the int8 path does not take are served as AUTO serves them)
    return ix->mode == KNN_SEARCH_AUTO || ix->mode == KNN_SEARCH_I8;
}

// AUTO: batches of <= kI8AutoQ queries at every corpus size (the int8 copy streams about half of
// the bf16 copy's bytes; its dot products grow with the batch: nq <= 4 is HBM-bound, nq = 5-8
// VALU-bound and still faster than the bf16 pass; one query on 1000-65536 rows 0.05-0.075 ms
// against the exact kernel's 0.18-0.22, profiles/r03/small_corpora/)
// A row's 16-lane group in the scan has one lane per 64-element block, so narrow rows leave most
// lanes idle (d = 128: 2 of 16).  One or two queries stay HBM-bound at every width since the
// rows are compact (round 4): one query on 1M rows, int8 against bf16, 0.133 / 0.143 ms at
// d = 64, 0.134 / 0.154 at 128, 0.137 / 0.183 at 256, 0.140 / 0.221 at 384, 0.140 / 0.247 at 512
// (profiles/r05/small_d/), so they take the int8 path at any width.  Larger batches multiply the
// dot products per byte: below kI8MinBlocks blocks they take it only while the copy is small
// enough (<= 64 MB, ~10 us of streaming) for the fixed costs to decide.
constexpr int kI8AutoQ = 8;
constexpr int kI8MinBlocks = 8;
// 5-8 queries run the scan's 8-query instance, VALU-bound: its time steps with the blocks per
// lane (NBI = ceil(blocks / 16)), the bf16 pass's grows with d.  One box, 1M rows
// (profiles/r05/modes_nq/, small_d/): 8 queries int8 / bf16 0.355 / 0.326 ms at 12 blocks,
// 0.339 / 0.397 at 16, 0.530 / 0.496 at 20, 0.585 / 0.679 at 31 — the int8 route at 14-16 blocks
// and from 23
bool i8_wins_8q(int nblk) { return (nblk >= 14 && nblk <= 16) || nblk >= 23; }
constexpr int64_t kI8SmallCopyBytes = 64ll << 20;
bool use_i8(const knn_index* ix, int64_t nq, int k) {
    if (ix->nblk8 <= 0 || k > KNN_MAX_K || nq > kI8MaxQ) return false;
    if (ix->mode == KNN_SEARCH_I8) return true;
    if (ix->mode != KNN_SEARCH_AUTO || nq > kI8AutoQ) return false;
    const int64_t i8_row = i8_row_bytes(ix->nblk8) + 4 * ix->nblk8;
    const bool wide_enough = nq <= 2 ? true : nq <= 4 ? ix->nblk8 >= kI8MinBlocks : i8_wins_8q(ix->nblk8);
    return !ix->b16_ok || wide_enough || ix->ntotal * i8_row <= kI8SmallCopyBytes;
}

bool use_split(const knn_index* ix, int64_t nq, int k) {
    if (!ix->split_ok || ix->mode == KNN_SEARCH_EXACT || split_kc(k) == 0) return false;
    if (ix->mode == KNN_SEARCH_SPLIT) return true;
    // auto (when the bf16 path is unavailable): batches the (1,4) plan covers, corpora with
    // enough rows to amortise the rerank
    return (ix->mode == KNN_SEARCH_AUTO || ix->mode == KNN_SEARCH_I8) && nq > 128 && ix->ntotal >= 16384;
}

int search_locked(knn_index* ix, const float* q, int64_t nq, int k, float* D, int64_t* I,
                  hipStream_t st) {
    const int normalize = ix->metric == KNN_METRIC_COSINE;
    const int kmetric = ix->metric == KNN_METRIC_L2 ? 1 : 0;
    ix->last_split_queries = 0;
    ix->stat_valid = false;
    if (k > KNN_MAX_K) {               // register top-k lists end at 32: faiss's GEMM + select form
        ix->last_path = 0;
        return k > KNN_MAX_K_LARGE ? hugek_search(ix, q, nq, k, D, I, st)
                                   : largek_search(ix, q, nq, k, D, I, st);
    }
    if (ix->ntotal == 0) {
        KNN_HIP(launch_fill_empty(D, I, nq * (int64_t)k, kmetric, st));
        return KNN_OK;
    }
    bool first_cand = true;
    for (int64_t c0 = 0; c0 < nq; c0 += kQueryChunk) {
        const int64_t cn = std::min(kQueryChunk, nq - c0);
        const bool i8 = use_i8(ix, cn, k);
        const bool b16 = !i8 && use_b16(ix, cn, k);
        const bool split = !i8 && !b16 && use_split(ix, cn, k);
        // padding: the query tile of the plan this chunk will run (and the exact re-run's 32)
        const Plan p = i8 ? make_i8_plan(ix->ntotal, cn, k, ix->cus, ix->i8_wgpcu, ix->nblk8)
                     : b16 ? make_b16_plan(ix->ntotal, cn, k, ix->cus, ix->dpb)
                     : split ? make_split_plan(ix->ntotal, cn, split_kc(k), ix->cus)
                             : make_plan(ix->ntotal, cn, k, ix->cus);
        const int64_t nq_pad = p.nq_pad;
        int rc;
        if (c0 == 0) ix->last_path = i8 ? 3 : (b16 ? 2 : (split ? 1 : 0));
        if ((rc = grow(&ix->qpad, &ix->qpad_cap, (size_t)nq_pad * ix->dp)) != KNN_OK) return rc;
        if ((rc = grow(&ix->qnorm, &ix->qnorm_cap, (size_t)nq_pad)) != KNN_OK) return rc;
        bool q_ready = false;
        // fused query prep: fp32 padded rows + norms + bf16 + residuals, or for the int8 path
        // the same rows and norms + the two-level int8 codes (one short pass instead of
        // rows_ingest's latency-bound row loop and a second launch)
        // (the int8 path's prep runs inside its scan unless IMGREC_I8_FUSED_PREP=0: nq_pad = cn)
        const bool i8_fused = i8 && ix->i8_fused_prep && nq_pad == cn && cn <= 4;
        if (i8) {
            if ((rc = grow(&ix->q8r, &ix->q8r_cap, (size_t)cn)) != KNN_OK) return rc;
        }
        if (i8_fused) {
            q_ready = true;
        } else if (i8) {
            if ((rc = grow(&ix->q8, &ix->q8_cap, (size_t)cn * ix->nblk8 * 128)) != KNN_OK) return rc;
            if ((rc = grow(&ix->q8s, &ix->q8s_cap, (size_t)cn * ix->nblk8 * 2)) != KNN_OK) return rc;
            KNN_HIP(launch_i8_query_prep(q + c0 * ix->d, cn, ix->d, ix->dp, nq_pad, normalize,
                                         ix->nblk8, ix->qpad, ix->qnorm, ix->q8, ix->q8s, ix->q8r, st));
            q_ready = true;
        } else if (b16 && ix->dpb <= 4096) {
            if ((rc = grow(&ix->qb16, &ix->qb16_cap, (size_t)nq_pad * ix->dpb)) != KNN_OK) return rc;
            if ((rc = grow(&ix->q_resid, &ix->q_resid_cap, (size_t)nq_pad)) != KNN_OK) return rc;
            KNN_HIP(launch_query_prep_b16(q + c0 * ix->d, cn, ix->d, ix->dp, ix->dpb, nq_pad,
                                          normalize, ix->qpad, ix->qnorm, ix->qb16, ix->q_resid, st));
            q_ready = true;
        } else {
            KNN_HIP(launch_rows_ingest(q + c0 * ix->d, cn, ix->d, ix->dp, nq_pad, normalize,
                                       ix->qpad, ix->qnorm, st));
        }
        float* Dc = D + c0 * k;
        int64_t* Ic = I + c0 * k;
        if (i8 || b16 || split) {
            rc = i8 ? i8_chunk(ix, i8_fused ? q + c0 * ix->d : nullptr, ix->qpad, ix->qnorm, cn, k,
                               Dc, Ic, st, true, first_cand)
               : b16 ? b16_chunk(ix, ix->qpad, ix->qnorm, cn, k, Dc, Ic, st, true, q_ready, first_cand)
                     : split_chunk(ix, ix->qpad, ix->qnorm, cn, k, Dc, Ic, st, true, first_cand);
            first_cand = false;
        } else {
            rc = exact_chunk(ix, ix->qpad, ix->qnorm, cn, k, Dc, Ic, st, true);
        }
        if (rc != KNN_OK) return rc;
    }
    return KNN_OK;
}

// Totals of the last search's candidate chunks (waits for that search to finish).
int read_search_stats(knn_index* ix, int64_t* split_q, int64_t* fallback_q, int64_t* first_fail,
                      float* ratio) {
    *split_q = ix->last_split_queries;
    *fallback_q = 0;
    if (first_fail) *first_fail = 0;
    if (ratio) *ratio = 0.f;
    if (!ix->stat_valid) return KNN_OK;
    int rc;
    if ((rc = fence_begin(ix, ix->stream)) != KNN_OK) return rc;
    int acc[4] = {0, 0, 0, 0};
    KNN_HIP(hipMemcpyAsync(acc, ix->stat + 8, sizeof(acc), hipMemcpyDeviceToHost, ix->stream));
    KNN_HIP(hipStreamSynchronize(ix->stream));
    if (acc[3] != 0) {        // cert_tail_kernel's bounded wait for its planner ran out
        // reported once: clear the bit so later clean searches read their stats again
        const int zero = 0;
        KNN_HIP(hipMemcpyAsync(ix->stat + 11, &zero, sizeof(int), hipMemcpyHostToDevice, ix->stream));
        KNN_HIP(hipStreamSynchronize(ix->stream));
        KNN_FAIL(KNN_EHIP, "certificate tail: a workgroup gave up waiting for the re-run plan "
                           "(error bits 0x%x); results of that search are not certified", acc[3]);
    }
    *fallback_q = acc[0];
    if (first_fail) *first_fail = acc[2];
    if (ratio) std::memcpy(ratio, &acc[1], sizeof(float));
    return KNN_OK;
}

}  // namespace imgrec
