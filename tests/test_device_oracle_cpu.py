"""tests/device_oracle.device_topk (the full-batch checker of the full-size GPU tests) against the
host float64 oracle (oracle.flat_knn.search_exact) — run here on CPU tensors: same labels in
(key, label) order, exact duplicates tied exactly, and the fp32 form equal to faiss's restated
exhaustive_L2sqr_blas (oracle.flat_knn.search_blas_fp32_blocked)."""
import numpy as np
import torch

from oracle.flat_knn import search_blas_fp32_blocked, search_exact
from tests.device_oracle import compact, device_topk


def test_device_topk_matches_host_oracle():
    rng = np.random.default_rng(3)
    xb = rng.standard_normal((6000, 96)).astype(np.float32)
    xb[[10, 700, 3000, 5999]] = xb[1234]                  # exact duplicates across blocks
    xq = rng.standard_normal((33, 96)).astype(np.float32)
    xq[0] = xb[1234]
    blocks = [torch.from_numpy(xb[i:i + 1024]) for i in range(0, len(xb), 1024)]
    Dg, Ig, rows, (Db, Ib) = device_topk(torch, iter(blocks), torch.from_numpy(xq), 11,
                                         need={5, 17}, collect_rows=True)
    D2, I2 = search_exact(xb, xq, 11, "l2")
    np.testing.assert_array_equal(Ig, I2)
    np.testing.assert_allclose(Dg, D2, rtol=0, atol=1e-9)
    np.testing.assert_array_equal(Ig[0, :5], [10, 700, 1234, 3000, 5999])
    assert (Dg[0, :5] == 0.0).all()
    D3, I3 = search_blas_fp32_blocked(xb, xq, 10)
    assert (Ib[1:] == I3[1:]).mean() > 0.99       # fp32 near-ties may swap (query 0: five exact ties)
    labels, sub, remap = compact(rows)
    assert {5, 17} <= set(labels.tolist())
    np.testing.assert_array_equal(sub[remap(Ig[3])], xb[Ig[3]])


def test_device_topk_row_offset():
    rng = np.random.default_rng(4)
    xb = rng.standard_normal((3000, 32)).astype(np.float32)
    xq = rng.standard_normal((5, 32)).astype(np.float32)
    Dg, Ig, _, _ = device_topk(torch, [torch.from_numpy(xb)], torch.from_numpy(xq), 4, row0=1000)
    np.testing.assert_array_equal(Ig - 1000, search_exact(xb, xq, 4, "l2")[1])
