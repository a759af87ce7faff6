"""IVF-PQ oracle (oracle/ivfpq.py) on the CPU: its ADC distances are the distances to the
reconstructed vectors, and on data the quantisers represent exactly, with every list probed, it
is the exact flat search (reference index: main/create_index.py:218-228)."""
import numpy as np

from oracle import ivfpq
from oracle.flat_knn import search_exact


def _params(rng, nlist, m, ksub, dsub):
    return (rng.standard_normal((nlist, m * dsub)).astype(np.float32),
            rng.standard_normal((m, ksub, dsub)).astype(np.float32))


def test_adc_distance_is_distance_to_reconstruction():
    rng = np.random.default_rng(3)
    nlist, m, ksub, dsub = 5, 4, 16, 3
    cen, cb = _params(rng, nlist, m, ksub, dsub)
    x = rng.standard_normal((200, m * dsub)).astype(np.float32)
    lists, codes = ivfpq.encode(x, cen, cb)
    q = rng.standard_normal((7, m * dsub)).astype(np.float32)
    ids = np.arange(200)
    D, I = ivfpq.search(q, cen, cb, lists, codes, ids, k=10, nprobe=nlist)
    recon = cen[lists].astype(np.float64) + np.concatenate([cb[j][codes[:, j]] for j in range(m)], 1)
    for i in range(7):
        dd = ((recon[I[i]] - q[i].astype(np.float64)) ** 2).sum(1)
        np.testing.assert_allclose(D[i], dd, rtol=1e-12, atol=1e-12)
        assert np.all(np.diff(D[i]) >= 0)


def test_exactly_representable_data_gives_the_flat_search():
    rng = np.random.default_rng(4)
    nlist, m, ksub, dsub = 6, 3, 8, 4
    cen, cb = _params(rng, nlist, m, ksub, dsub)
    lists = rng.integers(0, nlist, 300)
    codes = rng.integers(0, ksub, (300, m))
    x = cen[lists].astype(np.float64) + np.concatenate([cb[j][codes[:, j]] for j in range(m)], 1)
    q = rng.standard_normal((9, m * dsub))
    D, I = ivfpq.search(q, cen, cb, lists, codes, np.arange(300), k=12, nprobe=nlist)
    De, Ie = search_exact(x, q, 12, "l2")
    np.testing.assert_array_equal(I, Ie)
    np.testing.assert_allclose(D, De, rtol=1e-9, atol=1e-9)


def test_encode_picks_the_nearest_codeword_and_list():
    rng = np.random.default_rng(5)
    cen, cb = _params(rng, 4, 2, 32, 5)
    x = rng.standard_normal((50, 10)).astype(np.float32)
    lists, codes = ivfpq.encode(x, cen, cb)
    for i in range(50):
        dl = ((cen.astype(np.float64) - x[i]) ** 2).sum(1)
        assert dl[lists[i]] == dl.min()
        r = x[i].astype(np.float64) - cen[lists[i]]
        for j in range(2):
            dj = ((cb[j].astype(np.float64) - r[j * 5:(j + 1) * 5]) ** 2).sum(1)
            assert dj[codes[i, j]] == dj.min()


def test_padding_when_the_probed_lists_hold_fewer_than_k():
    rng = np.random.default_rng(6)
    cen, cb = _params(rng, 3, 2, 4, 2)
    lists = np.array([0, 0, 1])
    codes = rng.integers(0, 4, (3, 2))
    D, I = ivfpq.search(cen[:1] + 0.01, cen, cb, lists, codes, np.array([10, 11, 12]), k=5, nprobe=1)
    assert sorted(I[0, :2].tolist()) == [10, 11] and (I[0, 2:] == -1).all()
    assert (D[0, 2:] == ivfpq.FLT_MAX).all()
