"""The candidate paths' launch knobs must not change a single returned bit.

Round 4 gave the candidate merge two selects (the list-head bound of level 1, the two-entry bound of
the K' = 64 single level; wave_ops.h) and moved both levels into the rerank workgroup for small
batches (RerankArgs::l0_lists, l1_G); the int8 scan's split count depends on the batch size.  Whatever the
merge route and however many per-split lists the scan writes, the certified top-k is the same rows
with the same exact fp32 keys (the rerank's key form does not depend on the route), so these
tests compare the default index against indexes created with IMGREC_MERGE_FUSE=0 (both levels
as their own launches) and =1 (level 1 launched, level 2 in the rerank), IMGREC_I8_WGPCU=1 / 5 (256 / 1280 lists per query against the default 512 or
768: 4 / 20 level-1 groups), IMGREC_CHANCE_SKIP=0 (every query through the first rerank, none
sent straight to the second chance by its band) and IMGREC_I8_FUSED_PREP=0 (the int8 query codes
from their own launch instead of inside the scan) and IMGREC_RERANK_P1=0 (a 16-row first rerank
phase for every batch instead of k rows past one rerank workgroup per CU) and
IMGREC_MERGE_SINGLE=1 (the single-level merge of <= 64 lists inside the rerank workgroup) and
IMGREC_RERANK_NW4=1 (4-wave rerank workgroups for large batches) and IMGREC_CHANCE_DIRECT=0 (one-query
int8 searches through the merge and the first rerank instead of straight to the second chance) and
IMGREC_DIRECT_RAW=2 (that second chance over the scan's 16 unfolded lane lists per split, which the
default uses only up to 256 splits)
bit for bit, and the default against the float64 oracle (tests/knn_check.py).  The config-2
distribution (bench.py's 1M x 768 rows) makes most single queries take the second
chance, so the tail's hand-offs run under every route.
"""
import numpy as np
import pytest

from tests.knn_check import check_knn

pytestmark = pytest.mark.gpu

ROWS, K = 1_000_000, 10


@pytest.fixture(scope="module")
def corpus(gpu):
    import torch

    import bench
    cfg = dict(bench.CONFIGS[2])
    dev = torch.device("cuda", 0)
    centres = bench.make_centres(torch, cfg, dev, 2)
    blocks = list(bench.gen_rows(torch, cfg, centres, 0, ROWS, dev, 2))
    xb = torch.cat(blocks).cpu().numpy()
    q = bench.gen_queries(torch, cfg, centres, 300, dev, 2).cpu().numpy()
    return xb, q


def _index(xb, env, monkeypatch):
    from image_recommender_amd import faiss_compat as faiss
    for k_, v in env.items():
        monkeypatch.setenv(k_, v)
    idx = faiss.IndexFlatL2(xb.shape[1])          # the knobs are read at index creation
    for k_ in env:
        monkeypatch.delenv(k_)
    idx.add(xb)
    return idx


VARIANTS = {"unfused": {"IMGREC_MERGE_FUSE": "0"}, "level2only": {"IMGREC_MERGE_FUSE": "1"},
            "wgpcu1": {"IMGREC_I8_WGPCU": "1"},
            "wgpcu5": {"IMGREC_I8_WGPCU": "5"}, "noskip": {"IMGREC_CHANCE_SKIP": "0"},
            "separate_prep": {"IMGREC_I8_FUSED_PREP": "0"}, "rerank_p1_16": {"IMGREC_RERANK_P1": "0"},
            "single_fused": {"IMGREC_MERGE_SINGLE": "1"}, "rerank_nw4": {"IMGREC_RERANK_NW4": "1"},
            "first_pass": {"IMGREC_CHANCE_DIRECT": "0"}, "direct_raw": {"IMGREC_DIRECT_RAW": "2"}}


@pytest.mark.parametrize("nq", [1, 2, 5, 8, 16, 256, 257, 1024])
def test_routes_return_identical_bits(corpus, monkeypatch, nq):
    """nq 1-2: the int8 path (split counts 1-5 per CU, fused or separate level 2); 5 and 8 at
    d = 768 the bf16 small-batch tile (the int8 route's 8-query instance loses at 12 blocks); 16: the
    bf16 path's small-batch tile with the fused or separate level 2; 256 / 257: the last batch
    that fuses (one rerank workgroup per CU) and the first that does not.  The float64 oracle
    checks the default route on up to 16 of the queries."""
    xb, q = corpus
    xq = np.ascontiguousarray(q[:nq])
    base = _index(xb, {}, monkeypatch)
    D0, I0 = base.search(xq, K)
    _, reruns, ratio = base.search_stats(with_error=True)
    assert 0.0 <= ratio < 1.0, ratio
    check_knn(D0[:16], I0[:16], xb, xq[:16], K, "l2", min_exact_frac=0.5)
    for name, env in VARIANTS.items():
        idx = _index(xb, env, monkeypatch)
        D, I = idx.search(xq, K)
        assert np.array_equal(I, I0), (name, np.argwhere(I != I0)[:5])
        assert np.array_equal(D, D0), (name, float(np.abs(D - D0).max()))
        del idx


def test_second_chance_taken_on_this_distribution(corpus, monkeypatch):
    """The premise of the bit-identity test: on the config-2 distribution single queries do take
    the second chance (their int8 band is wider than K' = 64), so the tail's sliced path ran."""
    xb, q = corpus
    idx = _index(xb, {}, monkeypatch)
    taken = 0
    for i in range(16):
        idx.search(np.ascontiguousarray(q[i:i + 1]), K)
        taken += idx.certificate_stats()["second_chance"]
    assert taken >= 4, taken
