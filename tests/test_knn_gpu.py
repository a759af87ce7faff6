"""HIP parity tests of the exact k-NN index (faiss IndexFlatL2 / IndexFlatIP semantics).

The reference reaches this arithmetic through index.search (main/search_from_image.py:247) on
vectors added at main/create_index.py:311.  Every result is checked against the float64 oracle
(oracle/flat_knn.py) with the fp32 error bound stated in tests/knn_check.py.
"""
import struct

import numpy as np
import pytest

from tests.datagen import concat_rows, mixture
from tests.knn_check import check_knn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


@pytest.mark.parametrize("d", [48, 64, 100, 512, 768])
@pytest.mark.parametrize("nq", [1, 17, 33, 130, 300])
def test_l2_shapes(faiss, d, nq):
    xb = mixture(3000, d, centres=40, seed=d)
    xq = mixture(nq, d, centres=40, seed=d + 1)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    assert idx.ntotal == 3000
    D, I = idx.search(xq, 10)
    assert D.dtype == np.float32 and I.dtype == np.int64
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("k", [1, 5, 8, 9, 16, 17, 32])
def test_l2_k_values(faiss, k):
    xb = mixture(5000, 128, centres=60, seed=k)
    xq = mixture(40, 128, centres=60, seed=k + 100)
    idx = faiss.IndexFlatL2(128)
    idx.add(xb)
    D, I = idx.search(xq, k)
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("metric", ["ip", "cosine"])
@pytest.mark.parametrize("nq", [3, 200])
def test_ip_and_cosine(faiss, metric, nq):
    xb = mixture(4000, 96, centres=30, seed=7)
    xq = mixture(nq, 96, centres=30, seed=8)
    idx = faiss.IndexFlatIP(96) if metric == "ip" else faiss.IndexFlat(96, faiss.METRIC_COSINE)
    idx.add(xb)
    D, I = idx.search(xq, 10)
    check_knn(D, I, xb, xq, 10, metric, min_exact_frac=0.5)
    assert np.all(np.diff(D, axis=1) <= 0)   # IP results descending


def test_self_query_concat_layout(faiss):
    """Config-3 layout (48|128|1792 unit parts, |x|^2 = 3) with normalised queries: the reference
    pipeline's L2 value 3 + 1 - 2 q.x and a self-match at rank 0."""
    xb = concat_rows(2048, seed=3)
    q = xb[:64].copy()
    faiss.normalize_L2(q)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.add(xb)
    D, I = idx.search(q, 10)
    check_knn(D, I, xb, q, 10, "l2", min_exact_frac=0.5)
    assert (I[:, 0] == np.arange(64)).all()
    np.testing.assert_allclose(D[:, 0], 4 - 2 * np.sqrt(3), rtol=0, atol=1e-5)


def test_k_exceeds_ntotal_and_empty(faiss):
    xb = mixture(7, 32, seed=1)
    idx = faiss.IndexFlatL2(32)
    D, I = idx.search(xb[:2], 5)
    assert (I == -1).all() and (D == np.finfo(np.float32).max).all()
    idx.add(xb)
    D, I = idx.search(xb[:3], 10)
    check_knn(D, I, xb, xb[:3], 10, "l2")
    assert (I[:, 7:] == -1).all()
    ip = faiss.IndexFlatIP(32)
    ip.add(xb)
    D, I = ip.search(xb[:2], 9)
    assert (I[:, 7:] == -1).all() and (D[:, 7:] == -np.finfo(np.float32).max).all()


def test_duplicate_rows_tie_by_smaller_label(faiss):
    rng = np.random.default_rng(5)
    base = rng.standard_normal((50, 64)).astype(np.float32)
    xb = np.concatenate([base, base, base])          # every vector 3 times: labels i, i+50, i+100
    perm = rng.permutation(len(xb))
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    D, I = idx.search(base[:20], 6)
    for q in range(20):
        assert list(I[q, :3]) == [q, q + 50, q + 100], I[q]
        assert D[q, 0] == D[q, 1] == D[q, 2]
    del perm


def test_incremental_add_matches_single_add(faiss):
    xb = mixture(6000, 200, seed=11)
    xq = mixture(50, 200, seed=12)
    a = faiss.IndexFlatL2(200)
    a.add(xb)
    b = faiss.IndexFlatL2(200)
    for s in range(0, 6000, 777):
        b.add(xb[s:s + 777])
    Da, Ia = a.search(xq, 10)
    Db, Ib = b.search(xq, 10)
    np.testing.assert_array_equal(Ia, Ib)
    np.testing.assert_array_equal(Da, Db)
    np.testing.assert_array_equal(b.reconstruct_n(0, 6000), xb)


def test_write_read_roundtrip_faiss_layout(faiss, tmp_path):
    xb = mixture(1000, 40, seed=2)
    idx = faiss.IndexFlatL2(40)
    idx.add(xb)
    f = tmp_path / "index_hnsw_color.faiss"
    faiss.write_index(idx, str(f))
    raw = f.read_bytes()
    assert raw[:4] == b"IxF2"
    d, nt, dm1, dm2 = struct.unpack_from("<iqqq", raw, 4)
    assert (d, nt, dm1, dm2) == (40, 1000, 1 << 20, 1 << 20)
    tr, mt, nfl = struct.unpack_from("<BiQ", raw, 32)
    assert (tr, mt, nfl) == (1, 1, 40000)
    np.testing.assert_array_equal(np.frombuffer(raw, np.float32, 40000, 45).reshape(1000, 40), xb)
    idx2 = faiss.read_index(str(f))
    assert idx2.ntotal == 1000 and idx2.d == 40
    q = xb[:5]
    np.testing.assert_array_equal(idx.search(q, 7)[1], idx2.search(q, 7)[1])


def test_hnsw_and_ivfpq_constructors_search_exactly(faiss):
    """The reference's default constructor chain (main/create_index.py:218-228) runs unchanged."""
    d = 96
    xb = mixture(3000, d, seed=21)
    q = faiss.IndexHNSWFlat(d, 32)
    q.hnsw.efConstruction = 200
    q.hnsw.efSearch = 64
    ivf = faiss.IndexIVFPQ(q, d, 2048, 48, 12)
    assert not ivf.is_trained
    ivf.train(xb)
    assert ivf.is_trained
    ivf.add(xb)
    D, I = ivf.search(xb[:30], 5)
    check_knn(D, I, xb, xb[:30], 5, "l2")


def test_normalize_L2_semantics(faiss):
    x = mixture(10, 33, seed=3)
    x[4] = 0
    y = x.copy()
    faiss.normalize_L2(y)
    n = np.linalg.norm(x, axis=1)
    np.testing.assert_allclose(y[n > 0], x[n > 0] / n[n > 0, None], rtol=2e-6, atol=1e-7)
    assert (y[4] == 0).all()
    with pytest.raises(TypeError):
        faiss.normalize_L2(x.astype(np.float64))


def test_search_larger_batch_chunks(faiss):
    xb = mixture(20000, 64, seed=31)
    xq = mixture(9000, 64, seed=32)       # > one 8192-query chunk
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    D, I = idx.search(xq, 4)
    sel = np.r_[0:40, 8180:8200, 8990:9000]
    check_knn(D[sel], I[sel], xb, xq[sel], 4, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("n,d,nq", [(100_000, 256, 300), (400_000, 64, 5), (150_000, 128, 100)])
def test_many_row_tiles_per_workgroup(faiss, n, d, nq):
    """Corpora large enough that every workgroup walks several row tiles (the bench regime)."""
    xb = mixture(n, d, centres=200, seed=n % 97)
    xq = mixture(nq, d, centres=200, seed=n % 89)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(xq, 10)
    sel = np.arange(min(nq, 24))
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("d", [48, 1968])
def test_many_row_tiles_odd_depth_steps(faiss, d):
    """Odd number of 16-deep stages (48 -> 3, 1968 -> 123) with several tiles per workgroup."""
    n = 120_000 if d == 48 else 60_000
    xb = concat_rows(n, seed=5) if d == 1968 else mixture(n, d, centres=100, seed=9)
    xq = xb[:300].copy() + 0.01
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(xq, 10)
    sel = np.arange(16)
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("mode", ["exact", "bf16"])
@pytest.mark.parametrize("metric", ["l2", "ip"])
@pytest.mark.parametrize("shards,nq,k", [(2, 7, 10), (4, 300, 5), (8, 1, 10), (3, 1100, 16)])
def test_sharded_merge_is_bit_identical(faiss, mode, metric, shards, nq, k):
    """Row shards with global id offsets + the all-gather layout merge (knn_merge_device) give
    exactly the single-index result: same distances, same labels — for one search
    arithmetic on both sides (the exact kernel, or the bf16 path whose reranked keys do not depend
    on which shard holds a row)."""
    import torch
    from image_recommender_amd.sharded import merge_gathered_device, shard_range
    n, d = 20000, 160
    xb = mixture(n, d, centres=80, seed=shards * 7 + nq)
    xq = mixture(nq, d, centres=80, seed=nq + 1)
    M = faiss.METRIC_L2 if metric == "l2" else faiss.METRIC_INNER_PRODUCT
    full = faiss.IndexFlat(d, M)
    full.add(xb)
    full.search_mode = mode
    Df, If = full.search(xq, k)
    fallbacks = full.search_stats()[1]
    gD = torch.empty((shards, nq, k), dtype=torch.float32, device="cuda")
    gI = torch.empty((shards, nq, k), dtype=torch.int64, device="cuda")
    q = torch.from_numpy(xq).cuda()
    for r in range(shards):
        r0, r1 = shard_range(n, r, shards)
        sh = faiss.IndexFlat(d, M)
        sh.set_id_offset(r0)
        sh.add(xb[r0:r1])
        sh.search_mode = mode
        sh.search_device(q.data_ptr(), nq, k, gD[r].data_ptr(), gI[r].data_ptr(), 0)
        torch.cuda.synchronize()
        fallbacks += sh.search_stats()[1]
    D, I = merge_gathered_device(gD, gI, k, M)
    torch.cuda.synchronize()
    if fallbacks:      # a query re-run exactly on one side only: keys of two summation orders
        check_knn(D.cpu().numpy(), I.cpu().numpy(), xb, xq, k, metric, min_exact_frac=0.5)
        return
    np.testing.assert_array_equal(I.cpu().numpy(), If)
    np.testing.assert_array_equal(D.cpu().numpy(), Df)


@pytest.mark.parametrize("metric", ["l2", "ip"])
@pytest.mark.parametrize("shards,nq,k", [(2, 7, 10), (4, 301, 5), (3, 1024, 10), (8, 1, 3)])
def test_packed_merge_matches_gathered(faiss, metric, shards, nq, k):
    """ShardedIndex.search's single-collective layout: each shard searches into its packed chunk
    (keys, padding when nq*k is odd, labels) and knn_merge_packed_device gives exactly what
    knn_merge_device gives on the separate [shards][nq][k] arrays."""
    import torch
    from image_recommender_amd.sharded import (merge_gathered_device, merge_packed_device,
                                               packed_layout, packed_views, shard_range)
    n, d = 6000, 96
    xb = mixture(n, d, centres=40, seed=shards + nq)
    xq = mixture(nq, d, centres=40, seed=nq + 3)
    M = faiss.METRIC_L2 if metric == "l2" else faiss.METRIC_INNER_PRODUCT
    nbytes = packed_layout(nq, k)[0]
    g = torch.zeros((shards, nbytes), dtype=torch.uint8, device="cuda")
    gD = torch.empty((shards, nq, k), dtype=torch.float32, device="cuda")
    gI = torch.empty((shards, nq, k), dtype=torch.int64, device="cuda")
    q = torch.from_numpy(xq).cuda()
    for r in range(shards):
        r0, r1 = shard_range(n, r, shards)
        sh = faiss.IndexFlat(d, M)
        sh.set_id_offset(r0)
        sh.add(xb[r0:r1])
        sh.search_mode = "exact"
        pD, pI = packed_views(g[r], nq, k)
        sh.search_device(q.data_ptr(), nq, k, pD.data_ptr(), pI.data_ptr(), 0)
        sh.search_device(q.data_ptr(), nq, k, gD[r].data_ptr(), gI[r].data_ptr(), 0)
        torch.cuda.synchronize()
    D1, I1 = merge_gathered_device(gD, gI, k, M)
    D2, I2 = merge_packed_device(g, nq, k, k, M)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(I2.cpu().numpy(), I1.cpu().numpy())
    np.testing.assert_array_equal(D2.cpu().numpy(), D1.cpu().numpy())
    check_knn(D2.cpu().numpy(), I2.cpu().numpy(), xb, xq, k, metric)


def test_merge_device_padding_and_partial_lists(faiss):
    """Shards smaller than k: -1 tails in the gathered lists are skipped, output padded."""
    import torch
    from image_recommender_amd.sharded import merge_gathered_device
    xb = mixture(9, 16, seed=4)
    gD = torch.empty((3, 2, 6), dtype=torch.float32, device="cuda")
    gI = torch.empty((3, 2, 6), dtype=torch.int64, device="cuda")
    q = torch.from_numpy(xb[:2].copy()).cuda()
    for r in range(3):
        sh = faiss.IndexFlatL2(16)
        sh.set_id_offset(3 * r)
        sh.add(xb[3 * r:3 * r + 3])
        sh.search_device(q.data_ptr(), 2, 6, gD[r].data_ptr(), gI[r].data_ptr(), 0)
    D, I = merge_gathered_device(gD, gI, 12, faiss.METRIC_L2)
    I = I.cpu().numpy()
    assert (I[:, 9:] == -1).all() and sorted(I[0, :9].tolist()) == list(range(9))
    assert (D.cpu().numpy()[:, 9:] == np.finfo(np.float32).max).all()
    check_knn(D.cpu().numpy()[:, :9], I[:, :9], xb, xb[:2], 9, "l2")
