"""Parity at the shapes of BASELINE.json's configurations, through the C ABI.

The other GPU tests hold the kernels to the float64 oracle on corpora of up to 60k rows.  These
run the regimes only the full sizes reach — at 1M rows each of the 64 row splits of the bf16
256 x 256-tile kernel walks ~61 tiles, so the in-kernel screen re-tightening, the merge floor and
the 64-candidate certificate operate as in the bench — and check EVERY query of the 1024-query
batches against a float64 scan of the same rows on the device
(tests/device_oracle.py; the host oracle oracle.flat_knn.search_exact takes ~1 s per query at this
size and is kept for the one-query searches and, with the plain-C oracle, for spread samples):

* cfg3: 1M x 1968 concat (48 colour | 128 SIFT | 1792 DreamSim, every part unit-norm: the
  reference's stored layout, /root/reference/main/create_index.py:171-188), AUTO arithmetic
  (the bf16 candidate kernel), 1024 queries normalised after concatenation
  (/root/reference/main/search_from_image.py:305-322), k = 10.
* cfg4's per-rank shapes: the same corpus as 8 row shards of 125k rows (the bench's N = 8 strong-
  scaling shard) searched into packed chunks and merged by knn_merge_packed_device (the all-gather
  layout), and one 1.25M-row shard of the 10M corpus with the last rank's id offset.
* cfg5: a small run of bench_pipeline (HIP colour histogram -> DreamSim-architecture forward ->
  index -> search): integer histogram counts equal oracle.color_hist, every query image finds
  itself at rank 0.

Data come from bench.py's own block-seeded device generators, so they are the bench's rows.

Every full-size check also runs tests/knn_check.check_knn_tight: labels
integer-exact against the float64 oracle AND against faiss IndexFlatL2's fp32 arithmetic restated
(oracle.flat_knn.search_blas_fp32_blocked, exhaustive_L2sqr_blas) at every rank separated by more
than an empirical window (8x the measured max |fp32 - float64| key error, ~1e-6 of the key scale),
and top-k label sets equal wherever the k-th / (k+1)-th gap exceeds it; the checked fractions are
printed and held to stated minimums.
"""
import numpy as np
import pytest

from tests.knn_check import check_knn, check_knn_tight

pytestmark = pytest.mark.gpu

NQ, K, NSAMPLE = 1024, 10, 32   # every query checked; NSAMPLE for one-at-a-time searches
RANK_FRAC, SET_FRAC = 0.95, 0.9      # minimum fractions of ranks / top-k sets label-checked


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _generate(torch, cfg_id, r0, r1, nq):
    """Rows [r0, r1) of bench config cfg_id on the device (list of blocks), a host float32 copy,
    and the config's 1024 normalised queries."""
    import bench
    cfg = dict(bench.CONFIGS[cfg_id])
    dev = torch.device("cuda", 0)
    centres = bench.make_centres(torch, cfg, dev, cfg_id)
    d = sum(cfg["parts"])
    host = np.empty((r1 - r0, d), np.float32)
    blocks, pos = [], 0
    for blk in bench.gen_rows(torch, cfg, centres, r0, r1, dev, cfg_id):
        host[pos:pos + blk.shape[0]] = blk.cpu().numpy()
        blocks.append(blk)
        pos += blk.shape[0]
    q = bench.gen_queries(torch, cfg, centres, nq, dev, cfg_id)
    return blocks, host, q


@pytest.fixture(scope="module")
def cfg3(faiss):
    """The cfg3 corpus resident in one index + the oracle of EVERY query (computed once on the
    device, tests/device_oracle.py: float64 and faiss's fp32 form); `sel` = all 1024 queries,
    `sample` = 32 spread queries for the one-query and exact-kernel tests."""
    import torch
    from tests.device_oracle import device_topk
    blocks, xb, q = _generate(torch, 3, 0, 1_000_000, NQ)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.reserve(xb.shape[0])
    st = torch.cuda.current_stream().cuda_stream
    for blk in blocks:
        idx.add_device(blk.data_ptr(), blk.shape[0], st)
    torch.cuda.synchronize()
    Dg, Ig, _, blas = device_topk(torch, blocks, q, K + 1)
    del blocks
    sel = np.arange(NQ)
    sample = np.linspace(0, NQ - 1, NSAMPLE).astype(int)
    xq = q.cpu().numpy()
    return dict(idx=idx, xb=xb, q=q, xq=xq, sel=sel, sample=sample, oracle=(Dg, Ig), blas=blas)


def test_cfg3_full_size_auto_bf16(faiss, cfg3):
    """1M x 1968, 1024 queries, AUTO: the 256 x 256-tile bf16 kernel + rerank + certificate."""
    import ctypes as C
    import torch
    from image_recommender_amd import _lib
    idx, q, sel = cfg3["idx"], cfg3["q"], cfg3["sel"]
    tr, tq, sp, wg = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    _lib.check(_lib.load().knn_plan(idx.handle, NQ, K, C.byref(tr), C.byref(tq), C.byref(sp),
                                    C.byref(wg)), "knn_plan")
    assert (tr.value, tq.value) == (256, 256) and sp.value == 64
    D = torch.empty((NQ, K), dtype=torch.float32, device="cuda")
    I = torch.empty((NQ, K), dtype=torch.int64, device="cuda")
    idx.search_device(q.data_ptr(), NQ, K, D.data_ptr(), I.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert _lib.load().knn_last_path(idx.handle) == 2
    ncand, nfb, ratio = idx.search_stats(with_error=True)
    assert ncand == NQ and 0.0 <= ratio < 1.0, (ncand, ratio)
    print(f"cfg3: {nfb} of {NQ} queries failed the certificate, error/bound {ratio:.3g}")
    Dh, Ih = D.cpu().numpy(), I.cpu().numpy()
    check_knn(Dh[sel], Ih[sel], cfg3["xb"], cfg3["xq"][sel], K, "l2", min_exact_frac=0.5,
              oracle=cfg3["oracle"], tight=False)
    check_knn_tight(Dh[sel], Ih[sel], cfg3["xb"], cfg3["xq"][sel], K, "l2", oracle=cfg3["oracle"],
                    blas=cfg3["blas"], min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC,
                    tag="cfg3 bf16 nq=1024, all queries")
    # the host entry point (the faiss call the reference makes) returns the same result
    D2, I2 = idx.search(cfg3["xq"], K)
    np.testing.assert_array_equal(I2, Ih)
    np.testing.assert_array_equal(D2, Dh)


def test_cfg3_full_size_single_queries_int8(faiss, cfg3):
    """The reference CLI's regime at full size: one query, and two, per search through AUTO on the
    1M x 1968 corpus take the int8 small-batch path (knn_i8.hip); 16 sampled queries searched one
    at a time and 8 pairs, against the float64 oracle, every query certified on the first pass."""
    from image_recommender_amd import _lib
    idx, xq = cfg3["idx"], cfg3["xq"]
    Dg, Ig = cfg3["oracle"]
    Db, Ib = cfg3["blas"]
    rows, Ds, Is = [], [], []
    smp = cfg3["sample"]
    for r in range(0, len(smp), 2):
        s = smp[r]
        D, I = idx.search(xq[s:s + 1], K)
        assert _lib.load().knn_last_path(idx.handle) == 3
        st = idx.certificate_stats()
        assert st["candidate_queries"] == 1 and st["exact_reruns"] == 0
        assert 0.0 <= st["max_err_over_bound"] < 1.0
        check_knn(D, I, cfg3["xb"], xq[s:s + 1], K, "l2", min_exact_frac=0.5,
                  oracle=(Dg[s:s + 1], Ig[s:s + 1]))
        rows.append(s), Ds.append(D), Is.append(I)
    for r in range(0, len(smp) - 1, 4):
        pair = smp[[r, r + 1]]
        D, I = idx.search(xq[pair], K)
        assert _lib.load().knn_last_path(idx.handle) == 3
        check_knn(D, I, cfg3["xb"], xq[pair], K, "l2", min_exact_frac=0.5,
                  oracle=(Dg[pair], Ig[pair]))
        rows += pair.tolist()
        Ds.append(D), Is.append(I)
    rows = np.array(rows)
    check_knn_tight(np.concatenate(Ds), np.concatenate(Is), cfg3["xb"], xq[rows], K,
                    "l2", oracle=(Dg[rows], Ig[rows]), blas=(Db[rows], Ib[rows]),
                    min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC, tag="cfg3 int8 nq=1,2")


def test_cfg3_full_size_exact_kernel(faiss, cfg3):
    """The fp32 exact kernel on the same corpus (128 queries: the (1,4) tile), sampled queries."""
    idx, xq = cfg3["idx"], cfg3["xq"]
    sel = cfg3["sample"][:8]
    idx.search_mode = "exact"
    try:
        D, I = idx.search(xq[sel], K)
    finally:
        idx.search_mode = "auto"
    Dg, Ig = cfg3["oracle"]
    rows = sel
    check_knn(D, I, cfg3["xb"], xq[sel], K, "l2", min_exact_frac=0.5, oracle=(Dg[rows], Ig[rows]))
    Db, Ib = cfg3["blas"]
    check_knn_tight(D, I, cfg3["xb"], xq[sel], K, "l2", oracle=(Dg[rows], Ig[rows]),
                    blas=(Db[rows], Ib[rows]), min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC,
                    tag="cfg3 exact fp32")


def test_cfg4_rank_shape_eight_shards_packed_merge(faiss, cfg3):
    """8 row shards of 125k rows (the N = 8 shard of the 1M bench corpus) with global id offsets,
    each searching the 1024-query batch into its packed chunk; knn_merge_packed_device over the 8
    chunks (the RCCL all-gather layout, include/imgrec_knn.h) equals the oracle and the one-index
    result."""
    import torch
    from image_recommender_amd.sharded import merge_packed_device, packed_layout, packed_views, shard_range
    xb, q, sel = cfg3["xb"], cfg3["q"], cfg3["sel"]
    n, d = xb.shape
    shards = 8
    g = torch.zeros((shards, packed_layout(NQ, K)[0]), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    fallbacks = 0
    for r in range(shards):
        r0, r1 = shard_range(n, r, shards)
        sh = faiss.IndexFlatL2(d)
        sh.set_id_offset(r0)
        x = torch.from_numpy(xb[r0:r1]).cuda()
        sh.add_device(x.data_ptr(), r1 - r0, st)
        pD, pI = packed_views(g[r], NQ, K)
        sh.search_device(q.data_ptr(), NQ, K, pD.data_ptr(), pI.data_ptr(), st)
        torch.cuda.synchronize()
        ncand, nfb, ratio = sh.search_stats(with_error=True)
        assert ncand == NQ and ratio < 1.0
        fallbacks += nfb
        del sh, x
    D, I = merge_packed_device(g, NQ, K, K)
    torch.cuda.synchronize()
    Dh, Ih = D.cpu().numpy(), I.cpu().numpy()
    check_knn(Dh[sel], Ih[sel], xb, cfg3["xq"][sel], K, "l2", min_exact_frac=0.5,
              oracle=cfg3["oracle"], tight=False)
    check_knn_tight(Dh[sel], Ih[sel], xb, cfg3["xq"][sel], K, "l2", oracle=cfg3["oracle"],
                    blas=cfg3["blas"], min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC,
                    tag="cfg4 8 x 125k packed merge, all queries")
    D1, I1 = cfg3["idx"].search(cfg3["xq"], K)
    print(f"8 shards: {fallbacks} certificate fallbacks; labels equal to one index: "
          f"{(Ih == I1).mean():.5f}")
    if fallbacks == 0 and cfg3["idx"].search_stats()[1] == 0:
        np.testing.assert_array_equal(Ih, I1)
        np.testing.assert_array_equal(Dh, D1)
    else:   # a query re-run on the fp32 kernel on one side only: last-bit key differences
        assert (Ih == I1).mean() > 0.999


def test_cfg4_last_rank_shard_full_size(faiss):
    """One 1.25M-row shard of the 10M x 1968 corpus (rank 7 of 8: rows 8.75M..10M, labels offset
    by 8.75M), 1024 queries on AUTO; every query against the device float64 oracle of that shard."""
    import torch
    from tests.device_oracle import device_topk
    r0, r1 = 8_750_000, 10_000_000
    blocks, xb, q = _generate(torch, 4, r0, r1, NQ)
    sh = faiss.IndexFlatL2(xb.shape[1])
    sh.set_id_offset(r0)
    sh.reserve(r1 - r0)
    st = torch.cuda.current_stream().cuda_stream
    for blk in blocks:
        sh.add_device(blk.data_ptr(), blk.shape[0], st)
    torch.cuda.synchronize()
    Dg, Ig, _, blas = device_topk(torch, blocks, q, K + 1)        # local labels (row0 = 0)
    del blocks
    D = torch.empty((NQ, K), dtype=torch.float32, device="cuda")
    I = torch.empty((NQ, K), dtype=torch.int64, device="cuda")
    sh.search_device(q.data_ptr(), NQ, K, D.data_ptr(), I.data_ptr(), st)
    torch.cuda.synchronize()
    ncand, nfb, ratio = sh.search_stats(with_error=True)
    assert ncand == NQ and 0.0 <= ratio < 1.0
    xq = q.cpu().numpy()
    Ih = I.cpu().numpy()
    assert (Ih >= r0).all() and (Ih < r1).all()
    check_knn(D.cpu().numpy(), Ih - r0, xb, xq, K, "l2", min_exact_frac=0.5, oracle=(Dg, Ig),
              tight=False)
    check_knn_tight(D.cpu().numpy(), Ih - r0, xb, xq, K, "l2", oracle=(Dg, Ig), blas=blas,
                    min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC,
                    tag="cfg4 1.25M-row shard, all queries")


def test_cfg5_pipeline_smoke(gpu):
    """bench_pipeline on 2048 images: colour counts equal the oracle's, the DreamSim-architecture
    forward and index add run, and every query image (the first 256) is its own nearest row."""
    import ctypes as C
    import torch
    import bench_pipeline as bp
    from image_recommender_amd import _lib
    from oracle.color_hist import color_counts
    out = bp.run(bp.parse(["--images", "2048", "--model-batch", "128", "--nq", "256",
                           "--search-reps", "2"]))
    assert out["stages"]["search"]["self_match_at_rank0"] == 1.0
    assert out["config"]["dim"] == 48 + 1792
    # the histogram stage's counts on a sample of the same images, against the integer oracle
    dev = torch.device("cuda", 0)
    imgs = bp.gen_images(torch, 100, 16, dev)
    n = imgs.shape[0]
    offs = torch.arange(n, dtype=torch.int64, device=dev) * (bp.IMG * bp.IMG * 3)
    npix = torch.full((n,), bp.IMG * bp.IMG, dtype=torch.int64, device=dev)
    hist = torch.empty((n, 48), dtype=torch.float32, device=dev)
    counts = torch.empty((n, 48), dtype=torch.int32, device=dev)
    rc = _lib.load().color_hist_device(C.c_void_p(imgs.data_ptr()), C.c_void_p(offs.data_ptr()),
                                       C.c_void_p(npix.data_ptr()), n, 16,
                                       C.c_void_p(hist.data_ptr()), C.c_void_p(counts.data_ptr()),
                                       None)
    assert rc == 0
    torch.cuda.synchronize()
    host = imgs.cpu().numpy()
    got = counts.cpu().numpy()
    for i in range(n):
        np.testing.assert_array_equal(got[i], color_counts(host[i], 16))


def test_cfg5_pipeline_full_size_one_gpu(gpu):
    """BASELINE.json configs[4] at its stated 100,000 images (on one GPU; the 8-GPU form is the
    driver's scaling run): the HIP colour histogram, the DreamSim-architecture forward (every GEMM
    on vit_linear_bf16), the index add and 1024 searches; every query image finds itself at rank 0
    and the colour counts of images spread over the whole range equal the integer oracle's
    (/root/reference/vector_scripts/create_color_vector.py:18-52, create_dreamsim_vector.py:51-93)."""
    import ctypes as C
    import torch
    import bench_pipeline as bp
    from image_recommender_amd import _lib
    from oracle.color_hist import color_counts
    out = bp.run(bp.parse(["--images", "100000", "--model-batch", "512", "--nq", "1024",
                           "--search-reps", "2"]))
    print(f"cfg5 100k: {out['value']:.0f} images/s, dreamsim {out['stages']['dreamsim']['images_per_s']:.0f}")
    assert out["config"]["images"] == 100_000
    assert out["stages"]["search"]["self_match_at_rank0"] == 1.0
    dev = torch.device("cuda", 0)
    for g0 in (0, 31_337, 65_535, 99_936):
        imgs = bp.gen_images(torch, g0, 64, dev)
        offs = torch.arange(64, dtype=torch.int64, device=dev) * (bp.IMG * bp.IMG * 3)
        npix = torch.full((64,), bp.IMG * bp.IMG, dtype=torch.int64, device=dev)
        hist = torch.empty((64, 48), dtype=torch.float32, device=dev)
        counts = torch.empty((64, 48), dtype=torch.int32, device=dev)
        assert _lib.load().color_hist_device(C.c_void_p(imgs.data_ptr()), C.c_void_p(offs.data_ptr()),
                                             C.c_void_p(npix.data_ptr()), 64, 16,
                                             C.c_void_p(hist.data_ptr()), C.c_void_p(counts.data_ptr()),
                                             None) == 0
        torch.cuda.synchronize()
        host, got = imgs.cpu().numpy(), counts.cpu().numpy()
        for i in range(0, 64, 9):
            np.testing.assert_array_equal(got[i], color_counts(host[i], 16))


# --------------------------------------------------------------------------------------------
# cfg2 at its full size
# --------------------------------------------------------------------------------------------
_DUP_SRC, _DUP_ROWS = 100_000, [24 + 512 * j for j in range(16)]


def test_cfg2_full_size_auto_with_forced_rerun(faiss):
    """cfg2 (BASELINE.json configs[1]): 1M x 768 DreamSim-only rows, L2, k = 10, 1024 queries on
    AUTO (the 256 x 256-tile bf16 kernel at d = 768), /root/reference/main/search_from_image.py:247.

    Query 0 is made to need the device-planned exact re-run AT 1M ROWS: it equals corpus row
    100000, and 16 rows that all sit in ONE row split of the candidate kernel (8-row groups 3,
    67, 131, ... of the 64 splits) are copies of that row.  Their split's list then holds 10 keys
    equal to the answer, so the list floor equals the 10th key and neither the first certificate
    nor the second chance can settle the query: it is re-run on the fp32 kernel, and its answer
    is the 10 smallest labels among the 17 copies (exact ties by the smaller label).  Every query
    is checked against the device float64 oracle of the same (patched) corpus
    (tests/device_oracle.py) and eight spread queries also against the independent plain-C oracle
    (oracle/c/oracle_ref.c)."""
    import torch
    from image_recommender_amd import _lib
    from oracle import c_oracle
    from tests.device_oracle import device_topk
    blocks, xb, q = _generate(torch, 2, 0, 1_000_000, NQ)
    assert xb.shape == (1_000_000, 768)
    src = xb[_DUP_SRC].copy()
    xb[_DUP_ROWS] = src
    blocks[0][_DUP_ROWS] = torch.from_numpy(src).to(blocks[0].device)   # rows < 16384: block 0
    q[0] = torch.from_numpy(src).to(q.device)
    idx = faiss.IndexFlatL2(768)
    idx.reserve(xb.shape[0])
    st = torch.cuda.current_stream().cuda_stream
    for blk in blocks:
        idx.add_device(blk.data_ptr(), blk.shape[0], st)
    torch.cuda.synchronize()
    Dg, Ig, _, blas = device_topk(torch, blocks, q, K + 1)
    del blocks
    import ctypes as C
    tr, tq, sp, wg = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    _lib.check(_lib.load().knn_plan(idx.handle, NQ, K, C.byref(tr), C.byref(tq), C.byref(sp),
                                    C.byref(wg)), "knn_plan")
    assert (tr.value, tq.value, sp.value) == (256, 256, 64)      # the split layout the dups assume
    D = torch.empty((NQ, K), dtype=torch.float32, device="cuda")
    I = torch.empty((NQ, K), dtype=torch.int64, device="cuda")
    idx.search_device(q.data_ptr(), NQ, K, D.data_ptr(), I.data_ptr(), st)
    torch.cuda.synchronize()
    assert _lib.load().knn_last_path(idx.handle) == 2
    stats = idx.certificate_stats()
    print(f"cfg2: {stats}")
    assert stats["candidate_queries"] == NQ and 0.0 <= stats["max_err_over_bound"] < 1.0
    assert stats["exact_reruns"] >= 1                            # query 0, at least
    Dh, Ih = D.cpu().numpy(), I.cpu().numpy()
    np.testing.assert_array_equal(Ih[0], _DUP_ROWS[:K])
    assert (Dh[0] == 0.0).all()
    xq = q.cpu().numpy()
    np.testing.assert_array_equal(Ig[0, :K], _DUP_ROWS[:K])      # the oracle sees the patch too
    check_knn(Dh, Ih, xb, xq, K, "l2", min_exact_frac=0.5, oracle=(Dg, Ig), tight=False)
    # (query 0's ten answers are exact copies, tied at 0: inside any window by construction)
    check_knn_tight(Dh, Ih, xb, xq, K, "l2", oracle=(Dg, Ig), blas=blas,
                    min_rank_frac=RANK_FRAC * (NQ - 1) / NQ,
                    min_set_frac=SET_FRAC * (NQ - 1) / NQ, tag="cfg2 bf16 nq=1024, all queries")
    sel = np.linspace(0, NQ - 1, 8).astype(int)
    Dc, Ic = c_oracle.flat_search(xb, xq[sel], K + 1, "l2")
    check_knn(Dh[sel], Ih[sel], xb, xq[sel], K, "l2", min_exact_frac=0.5, oracle=(Dc, Ic))


# --------------------------------------------------------------------------------------------
# cfg4's whole answer: 10M x 1968 in one index over 8 row shards
# --------------------------------------------------------------------------------------------
def _device_oracle(torch, cfg_id, nrows, qs, k, need):
    """tests/device_oracle.device_topk over rows [0, nrows) of bench config cfg_id, regenerated
    block by block on the device (bench.gen_rows: the same rows the index holds), keeping the row
    vectors of the answers and of every label in `need` (no host copy of a 10M corpus)."""
    import bench
    from tests.device_oracle import device_topk
    cfg = dict(bench.CONFIGS[cfg_id])
    centres = bench.make_centres(torch, cfg, qs.device, cfg_id)
    return device_topk(torch, bench.gen_rows(torch, cfg, centres, 0, nrows, qs.device, cfg_id),
                       qs, k, need=need, collect_rows=True)


def test_cfg4_whole_10m_corpus_eight_shards(faiss):
    """cfg4's whole corpus: 10M x 1968 concat rows in ONE IndexFlatL2 over 8 row shards
    (knn_create_multi, devices [0]*8: fp32 + bf16 copies of every shard, ~120 GB of the 288 GB),
    1024 queries on AUTO, the shards' top-k merged by knn_merge_kernel.  Every query against a
    float64 scan of the same 10M rows regenerated on the device.  (One GPU here: the
    shards share device 0, so the cross-device peer copies of knn_multi.cpp do not run.)"""
    import torch
    import bench
    from oracle.flat_knn import fp32_error_bound  # noqa: F401  (check_knn's bound)
    cfg = dict(bench.CONFIGS[4])
    n, d = cfg["rows"], sum(cfg["parts"])
    dev = torch.device("cuda", 0)
    centres = bench.make_centres(torch, cfg, dev, 4)
    idx = faiss.IndexFlatL2(d, devices=[0] * 8)
    assert idx.num_shards == 8
    idx.reserve(n)
    st = torch.cuda.current_stream().cuda_stream
    for blk in bench.gen_rows(torch, cfg, centres, 0, n, dev, 4):
        idx.add_device(blk.data_ptr(), blk.shape[0], st)
    assert idx.ntotal == n
    q = bench.gen_queries(torch, cfg, centres, NQ, dev, 4)
    D = torch.empty((NQ, K), dtype=torch.float32, device="cuda")
    I = torch.empty((NQ, K), dtype=torch.int64, device="cuda")
    idx.search_device(q.data_ptr(), NQ, K, D.data_ptr(), I.data_ptr(), st)
    torch.cuda.synchronize()
    stats = idx.certificate_stats()
    print(f"cfg4 10M: {stats}")
    assert stats["candidate_queries"] == NQ and stats["max_err_over_bound"] < 1.0
    sel = np.arange(NQ)
    Dh, Ih = D.cpu().numpy()[sel], I.cpu().numpy()[sel]
    assert (Ih >= 0).all() and (Ih < n).all()
    Dg, Ig, rows, (Db, Ib) = _device_oracle(torch, 4, n, q[sel], K + 1, set(Ih.ravel().tolist()))
    labels = np.array(sorted(rows))
    xb = np.stack([rows[int(l)] for l in labels])
    remap = lambda a: np.searchsorted(labels, a)                 # noqa: E731
    check_knn(Dh, remap(Ih), xb, q.cpu().numpy()[sel], K, "l2", min_exact_frac=0.5,
              oracle=(Dg, remap(Ig)), tight=False)
    check_knn_tight(Dh, remap(Ih), xb, q.cpu().numpy()[sel], K, "l2", oracle=(Dg, remap(Ig)),
                    blas=(Db, remap(Ib)), min_rank_frac=RANK_FRAC, min_set_frac=SET_FRAC,
                    tag="cfg4 whole 10M, 8 shards, all queries")
    hits = sum(len(set(a.tolist()) & set(b[:K].tolist())) for a, b in zip(Ih, Ig))
    assert hits / (K * len(sel)) == 1.0, hits                    # recall@10, every query
    del idx
    torch.cuda.synchronize()


def test_cfg3_full_size_any_k(faiss, cfg3):
    """k = 2048 (> KNN_MAX_K_LARGE: csrc/knn_hugek.hip, every key + a segmented sort) on the whole
    1M x 1968 cfg3 corpus for 4 queries, against the device float64 oracle of the same rows:
    labels integer-exact at every rank separated by more than the empirical window.
    /root/reference/main/search_from_image.py:27 (top_k), :247 (index.search)."""
    import torch
    from tests.device_oracle import device_topk
    k, sel = 2048, np.array([0, 333, 700, 1023])
    idx, xb = cfg3["idx"], cfg3["xb"]
    D, I = idx.search(cfg3["xq"][sel], k)
    assert D.shape == (len(sel), k) and (I >= 0).all() and (np.diff(D, axis=1) >= 0).all()
    blocks = (torch.from_numpy(xb[i:i + 16384]).cuda() for i in range(0, xb.shape[0], 16384))
    Dg, Ig, _, blas = device_topk(torch, blocks, cfg3["q"][sel].contiguous(), k + 1)
    check_knn(D, I, xb, cfg3["xq"][sel], k, "l2", min_exact_frac=0.0, oracle=(Dg, Ig), tight=False)
    # (2,048 deep among 1M rows the neighbours' keys are packed within a few 1e-6 of each other,
    # the window of this route's fp32 dot products (16-term stage sums added to a running total),
    # so only part of the ranks are separated by more (measured 0.69); every one of those must
    # carry the oracle's label)
    check_knn_tight(D, I, xb, cfg3["xq"][sel], k, "l2", oracle=(Dg, Ig), blas=blas,
                    min_rank_frac=0.5, min_set_frac=0.0, tag="cfg3 k=2048, 1M rows")
