"""The device-side certificate path and the multi-device index, through the C ABI.

* Second chance (csrc/knn_refine.hip rerank_certify_kernel): a query whose first certificate
  fails because more than K' = 64 rows crowd its k-th distance is settled by reranking every
  per-split list entry that can still rank, certified against the list floor — no exact re-run.
* Device-planned exact re-run (knn_search.cpp run_fallback): queries no certificate settles are
  re-run on the fp32 kernel with a launch planned on the GPU from the uncertified count (1, 32+,
  hundreds of queries: one and several query blocks), results scattered into place.
* Streams: adds on one stream (with buffer regrowth) followed by a search on another are ordered
  by the index's fence (reserve_rows / refresh_maxima ordering).
* knn_create_multi: 4 row shards on the one test GPU ([0, 0, 0, 0]) equal one index and the
  oracle, through the host and device entry points, reconstruct, write/read and IMGREC_DEVICES
  (the reference's single-process CLI, /root/reference/main/search_from_image.py:430-441).
"""
import numpy as np
import pytest

from tests.datagen import mixture
from tests.knn_check import check_knn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _crowded(n, d, nq, crowd, seed):
    """A corpus where the first `nq // 20` queries each have `crowd` rows at nearly the same
    distance (a shell of radius ~0.1 around the query), spread over the corpus."""
    rng = np.random.default_rng(seed)
    xb = mixture(n, d, centres=60, seed=seed, normalize=True)
    xq = mixture(nq, d, centres=60, seed=seed + 1, normalize=True)
    nc = max(1, nq // 20)
    rows = rng.permutation(n)[:nc * crowd].reshape(nc, crowd)
    for i in range(nc):
        u = rng.standard_normal((crowd, d))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        xb[rows[i]] = (xq[i] + 0.1 * (1 + 1e-5 * rng.random((crowd, 1))) * u).astype(np.float32)
    return xb, xq, nc


@pytest.mark.parametrize("nq,k", [(600, 10), (300, 16)])
def test_second_chance_settles_crowded_queries(faiss, nq, k):
    """100 rows within ~1e-6 of each other around 5 % of the queries: the K' = 64 candidates
    cannot certify them; the second chance over all list entries does (no exact re-run)."""
    xb, xq, nc = _crowded(40000, 256, nq, 100, seed=nq + k)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, k)
    st = idx.certificate_stats()
    print(st)
    assert st["candidate_queries"] == nq and st["max_err_over_bound"] < 1.0
    assert st["second_chance"] >= nc and st["exact_reruns"] == 0
    sel = np.r_[0:nc, nc:nq:13]
    check_knn(D[sel], I[sel], xb, xq[sel], k, "l2", min_exact_frac=0.3)


@pytest.mark.parametrize("nq", [1, 40, 600, 1100])
def test_device_planned_exact_rerun(faiss, nq):
    """Every row duplicated 1100 times (more than K' and than any per-split list can hold, so
    full lists end in duplicates): neither certificate holds, every query is re-run exactly by
    the device-planned launch (1, 2, 19 and 35 query blocks of 32); ties break by the smaller
    label."""
    dup = 1100
    base = mixture(150, 256, centres=20, seed=9)
    xb = np.repeat(base, dup, axis=0)
    src = np.arange(nq) % 150
    xq = base[src] + np.float32(1e-3)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    assert st["candidate_queries"] == nq and st["exact_reruns"] == nq
    assert (I == src[:, None] * dup + np.arange(10)[None, :]).all()
    sel = np.arange(min(nq, 40))
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2")
    # the same index and queries on the split path (its own rerank, same device re-run)
    idx.search_mode = "split"
    D2, I2 = idx.search(xq, 10)
    assert idx.search_stats()[1] == nq
    np.testing.assert_array_equal(I2, I)


def test_rerun_mixed_with_certified_and_chunks(faiss):
    """9000 queries (two 8192-query chunks) where 1 in 10 fails its first certificate (70
    duplicates of its nearest row): each chunk's second chance / device re-run and the per-search
    totals add up; certified rows are untouched."""
    base = mixture(300, 128, centres=30, seed=3, normalize=True)
    xb = np.concatenate([np.repeat(base, 70, axis=0),
                         mixture(30000, 128, centres=30, seed=4, normalize=True)])
    rng = np.random.default_rng(5)
    xq = mixture(9000, 128, centres=30, seed=6, normalize=True)
    dup = rng.permutation(9000)[:900]
    xq[dup] = base[dup % 300] + np.float32(1e-3)
    idx = faiss.IndexFlatL2(128)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    first_fail = st["second_chance"] + st["exact_reruns"]
    print(st)
    # the 900 planted queries fail their first certificate (others may too: a query of the
    # mixture can land next to one of the 70-fold rows)
    assert st["candidate_queries"] == 9000 and first_fail >= 900
    assert (I[dup] == (dup % 300)[:, None] * 70 + np.arange(10)[None, :]).all()
    sel = np.r_[dup[:20], 8185:8200]       # (all-tied rows: the label rule is asserted above)
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2")


def test_adds_and_search_on_different_streams(faiss):
    """Streamed device adds without a reserve (every add regrows the buffers, copying rows the
    previous add wrote on the same stream) and a search on another stream: the fence orders them."""
    import torch
    d = 768
    xb = mixture(12000, d, centres=50, seed=44)
    xq = mixture(300, d, centres=50, seed=45)
    idx = faiss.IndexFlatL2(d)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    parts = []
    with torch.cuda.stream(sa):
        for part in np.array_split(xb, 6):
            t = torch.from_numpy(part).to("cuda", non_blocking=False)
            idx.add_device(t.data_ptr(), t.shape[0], sa.cuda_stream)
            parts.append(t)                                       # keep alive until sa drains
    q = torch.from_numpy(xq).cuda()
    torch.cuda.synchronize()
    with torch.cuda.stream(sb):
        D = torch.empty((300, 10), dtype=torch.float32, device="cuda")
        I = torch.empty((300, 10), dtype=torch.int64, device="cuda")
        idx.search_device(q.data_ptr(), 300, 10, D.data_ptr(), I.data_ptr(), sb.cuda_stream)
    sb.synchronize()
    sa.synchronize()
    np.testing.assert_array_equal(idx.reconstruct_n(0, 12000), xb)
    check_knn(D.cpu().numpy(), I.cpu().numpy(), xb, xq, 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("mode", ["bf16", "exact"])
def test_multi_device_index_four_shards(faiss, mode, tmp_path, monkeypatch):
    """knn_create_multi with devices [0, 0, 0, 0]: three uneven adds cut into 4 shards each;
    host and device searches equal one index (bit for bit when no re-run happened) and the
    oracle; reconstruct, write/read (also through IMGREC_DEVICES), id offsets.  (AUTO decides
    per shard from the shard's rows, so the comparison pins one arithmetic on both sides.)"""
    import torch
    d, k = 384, 10
    xb = mixture(30001, d, centres=80, seed=71)
    xq = mixture(520, d, centres=80, seed=72)
    multi = faiss.IndexFlatL2(d, devices=[0, 0, 0, 0])
    assert multi.num_shards == 4
    for a, b in ((0, 7), (7, 20000), (20000, 30001)):
        multi.add(xb[a:b])
    assert multi.ntotal == 30001
    multi.search_mode = mode
    one = faiss.IndexFlatL2(d)
    one.add(xb)
    one.search_mode = mode
    D, I = multi.search(xq, k)
    D1, I1 = one.search(xq, k)
    reruns = multi.search_stats()[1] + one.search_stats()[1]
    check_knn(D[::7], I[::7], xb, xq[::7], k, "l2", min_exact_frac=0.5)
    if reruns == 0:
        np.testing.assert_array_equal(I, I1)
        np.testing.assert_array_equal(D, D1)
    else:
        assert (I == I1).mean() > 0.99
    # device entry point on a torch stream, id offset applied after the shard merge
    multi.set_id_offset(1000)
    q = torch.from_numpy(xq).cuda()
    Dd = torch.empty((520, k), dtype=torch.float32, device="cuda")
    Id = torch.empty((520, k), dtype=torch.int64, device="cuda")
    multi.search_device(q.data_ptr(), 520, k, Dd.data_ptr(), Id.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(Id.cpu().numpy(), I + 1000)
    np.testing.assert_array_equal(Dd.cpu().numpy(), D)
    multi.set_id_offset(0)
    np.testing.assert_array_equal(multi.reconstruct_n(0, 30001), xb)
    np.testing.assert_array_equal(multi.reconstruct_n(19990, 20), xb[19990:20010])
    f = tmp_path / "multi.faiss"
    faiss.write_index(multi, f)
    monkeypatch.setenv("IMGREC_DEVICES", "0,0,0")
    back = faiss.read_index(f)
    assert back.num_shards == 3 and back.ntotal == 30001
    back.search_mode = mode
    D3, I3 = back.search(xq, k)
    check_knn(D3[::7], I3[::7], xb, xq[::7], k, "l2", min_exact_frac=0.5)
    one2 = faiss.IndexFlatL2(d, device=0)
    assert one2.num_shards == 1


def test_multi_device_add_device_and_reset(faiss):
    """Device-pointer adds into a 3-shard index (rows on the first device), reset, re-add."""
    import torch
    d = 128
    xb = mixture(5000, d, centres=30, seed=81)
    xq = mixture(40, d, centres=30, seed=82)
    multi = faiss.IndexFlatL2(d, devices=[0, 0, 0])
    t = torch.from_numpy(xb).cuda()
    st = torch.cuda.current_stream().cuda_stream
    multi.add_device(t[:1234].data_ptr(), 1234, st)
    multi.add_device(t[1234:].data_ptr(), 5000 - 1234, st)
    D, I = multi.search(xq, 5)
    check_knn(D, I, xb, xq, 5, "l2", min_exact_frac=0.5)
    multi.reset()
    assert multi.ntotal == 0
    D, I = multi.search(xq, 5)
    assert (I == -1).all()
    multi.add(xb[:100])
    D, I = multi.search(xq, 5)
    check_knn(D, I, xb[:100], xq, 5, "l2")


# --------------------------------------------------------------------------------------------
# round 4: the cross-device branches of knn_multi.cpp on one GPU, the
# exact re-run workspace on a device with few CUs and the fence on destroyed streams
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["auto", "exact"])
def test_multi_device_forced_remote_staging(faiss, mode, monkeypatch):
    """IMGREC_MULTI_FORCE_REMOTE=1: shards on the first device take the other devices' path —
    rows staged by a peer copy into the shard's buffer before its add, queries peer-copied to
    each shard, per-shard results peer-copied back into the gather buffer on devices[0] — so one
    GPU runs the code an 8-GPU process runs.  Device adds, searches of 1 and 1024 queries at
    k = 10 and k = 200 (the k > 32 merge), reset and re-add, against the oracle and one index."""
    import torch
    monkeypatch.setenv("IMGREC_MULTI_FORCE_REMOTE", "1")
    d = 320
    xb = mixture(24001, d, centres=60, seed=91)
    xq = mixture(1024, d, centres=60, seed=92)
    multi = faiss.IndexFlatL2(d, devices=[0, 0, 0])
    monkeypatch.delenv("IMGREC_MULTI_FORCE_REMOTE")      # read at creation: this index keeps it
    multi.search_mode = mode
    t = torch.from_numpy(xb).cuda()
    st = torch.cuda.current_stream().cuda_stream
    multi.add_device(t[:10001].data_ptr(), 10001, st)
    multi.add_device(t[10001:].data_ptr(), 24001 - 10001, st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(multi.reconstruct_n(0, 24001), xb)
    one = faiss.IndexFlatL2(d)
    one.add(xb)
    one.search_mode = mode
    from oracle.flat_knn import search_exact
    for nq, k in ((1, 10), (1024, 10), (1, 200), (1024, 200)):
        q = torch.from_numpy(xq[:nq]).cuda()
        D = torch.empty((nq, k), dtype=torch.float32, device="cuda")
        I = torch.empty((nq, k), dtype=torch.int64, device="cuda")
        multi.search_device(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), st)
        torch.cuda.synchronize()
        Dh, Ih = D.cpu().numpy(), I.cpu().numpy()
        sel = np.arange(0, nq, 41)
        check_knn(Dh[sel], Ih[sel], xb, xq[sel], k, "l2", min_exact_frac=0.5,
                  oracle=search_exact(xb, xq[sel], k + 1, "l2"))
        D2, I2 = multi.search(xq[:nq], k)                            # host entry point
        np.testing.assert_array_equal(I2, Ih)
        D1, I1 = one.search(xq[:nq], k)
        assert (I1 == Ih).mean() > 0.99, (nq, k)    # (k > 32: GEMM blocking differs per shard)
    multi.reset()
    assert multi.ntotal == 0
    multi.add_device(t[:500].data_ptr(), 500, st)
    D, I = multi.search(xq[:7], 5)
    check_knn(D, I, xb[:500], xq[:7], 5, "l2")


def test_exact_rerun_with_few_cus(faiss, monkeypatch):
    """IMGREC_CUS=8 plans every launch for 8 CUs (a partitioned device): the certificate tail's
    grid is 8 workgroups, and 1100 all-tied queries (35 query blocks of 32 > 8) need the exact
    re-run's lists sized by the query count, not by the grid (the grid-sized buffer
    overflowed there)."""
    monkeypatch.setenv("IMGREC_CUS", "8")
    dup, nq = 1100, 1100
    base = mixture(150, 256, centres=20, seed=9)
    xb = np.repeat(base, dup, axis=0)
    src = np.arange(nq) % 150
    xq = base[src] + np.float32(1e-3)
    idx = faiss.IndexFlatL2(256)
    monkeypatch.delenv("IMGREC_CUS")
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    assert st["candidate_queries"] == nq and st["exact_reruns"] == nq
    assert (I == src[:, None] * dup + np.arange(10)[None, :]).all()
    check_knn(D[:40], I[:40], xb, xq[:40], 10, "l2")


def _hip():
    import ctypes as C
    import torch  # noqa: F401  (its HIP runtime is the one libimgrec.so binds)
    return C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)   # by SONAME: the runtime already loaded


@pytest.mark.parametrize("lazy", [False, True])
def test_fence_across_destroyed_and_switched_streams(faiss, lazy):
    """Default (eager) fence: a search on a stream the caller destroys right after the call, then
    a search on another stream and the stats read — ordered, no error (the lazy record
    on a destroyed stream wedged the index).  Lazy fence: back-to-back searches on one stream,
    then a switch to a live stream, equal the eager results."""
    import ctypes as C
    import torch
    hip = _hip()
    d = 256
    xb = mixture(20000, d, centres=40, seed=31)
    xq = mixture(300, d, centres=40, seed=32)
    idx = faiss.IndexFlatL2(d)
    idx.set_fence_mode(lazy)
    idx.add(xb)
    q = torch.from_numpy(xq).cuda()
    outs = []
    for _ in range(3):
        D = torch.empty((300, 10), dtype=torch.float32, device="cuda")
        I = torch.empty((300, 10), dtype=torch.int64, device="cuda")
        outs.append((D, I))
    torch.cuda.synchronize()
    if not lazy:
        s = C.c_void_p()
        assert hip.hipStreamCreate(C.byref(s)) == 0
        idx.search_device(q.data_ptr(), 300, 10, outs[0][0].data_ptr(), outs[0][1].data_ptr(), s.value)
        assert hip.hipStreamDestroy(s) == 0
    else:
        st = torch.cuda.current_stream().cuda_stream
        idx.search_device(q.data_ptr(), 300, 10, outs[0][0].data_ptr(), outs[0][1].data_ptr(), st)
        idx.search_device(q.data_ptr(), 300, 10, outs[1][0].data_ptr(), outs[1][1].data_ptr(), st)
    other = torch.cuda.Stream()
    idx.search_device(q.data_ptr(), 300, 10, outs[2][0].data_ptr(), outs[2][1].data_ptr(),
                      other.cuda_stream)
    other.synchronize()
    idx.certificate_stats()                                  # host read after the switch
    torch.cuda.synchronize()
    I0, I2 = outs[0][1].cpu().numpy(), outs[2][1].cpu().numpy()
    np.testing.assert_array_equal(I0, I2)
    np.testing.assert_array_equal(outs[0][0].cpu().numpy(), outs[2][0].cpu().numpy())
    check_knn(outs[2][0].cpu().numpy()[::10], I2[::10], xb, xq[::10], 10, "l2", min_exact_frac=0.5)
