"""CPU tests of the C-ABI library: it loads, exports exactly what include/*.h declares, and the
host-only entry points (BLOB decoder, argument validation, normalize_L2) behave.  No GPU compute.
"""
import ctypes as C
import pickle
import re
from pathlib import Path

import numpy as np
import pytest

from image_recommender_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
HEADERS = sorted((ROOT / "include").glob("*.h"))


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w]*\s*\**\s+\**([A-Za-z_]\w*)\s*\(",
                             text, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_the_expected_surface():
    names = declared_functions()
    for must in ("knn_create", "knn_add", "knn_search", "knn_search_device", "knn_merge_device",
                 "knn_write", "knn_read", "knn_normalize_L2", "color_hist_device",
                 "ingest_parse_f32"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert names == set(_lib.SIGNATURES), (names ^ set(_lib.SIGNATURES))
    assert b"gfx950" in lib.knn_version()


def test_no_gpu_entry_points_fail_cleanly():
    lib = _lib.load()
    h = C.c_void_p()
    rc = lib.knn_create(0, _lib.KNN_METRIC_L2, -1, C.byref(h))
    assert rc == _lib.KNN_EINVAL and b"d must be positive" in lib.knn_last_error()
    rc = lib.knn_create(16, 7, -1, C.byref(h))
    assert rc == _lib.KNN_EINVAL


def _blob(a):
    return pickle.dumps(a, protocol=pickle.HIGHEST_PROTOCOL)


@pytest.mark.parametrize("d", [1, 48, 128, 255, 256, 1792, 32768])
def test_ingest_parse_matches_pickle(d):
    lib = _lib.load()
    a = np.random.default_rng(d).standard_normal(d).astype(np.float32)
    b = _blob(a)
    out = np.empty(d, np.float32)
    n = lib.ingest_parse_f32(b, len(b), out.ctypes.data, d)
    assert n == d
    np.testing.assert_array_equal(out, pickle.loads(b))


@pytest.mark.parametrize("obj", [
    np.arange(5, dtype=np.float64), np.arange(5, dtype=np.int32), [1.0, 2.0], "x",
    np.arange(6, dtype=np.float32).reshape(2, 3).T.copy(order="F")])
def test_ingest_rejects_other_layouts(obj):
    lib = _lib.load()
    b = _blob(obj)
    out = np.empty(64, np.float32)
    assert lib.ingest_parse_f32(b, len(b), out.ctypes.data, 64) == _lib.INGEST_NOT_FAST


def test_ingest_accepts_row_vector_and_capacity():
    lib = _lib.load()
    a = np.arange(8, dtype=np.float32).reshape(1, 8)
    b = _blob(a)
    out = np.empty(8, np.float32)
    assert lib.ingest_parse_f32(b, len(b), out.ctypes.data, 8) == 8
    np.testing.assert_array_equal(out, a.ravel())
    assert lib.ingest_parse_f32(b, len(b), out.ctypes.data, 4) == _lib.INGEST_TOO_SMALL
    assert lib.ingest_parse_f32(b[:-1], len(b) - 1, out.ctypes.data, 8) == _lib.INGEST_NOT_FAST


def test_ingest_concat_rows_status():
    lib = _lib.load()
    rng = np.random.default_rng(0)
    dims = [3, 4]
    rows = [[rng.standard_normal(3).astype(np.float32), rng.standard_normal(4).astype(np.float32)]
            for _ in range(4)]
    blobs = [[_blob(p) for p in r] for r in rows]
    blobs[1][1] = _blob(rows[1][1].astype(np.float64))   # needs pickle fallback
    blobs[2][0] = _blob(np.zeros(5, np.float32))          # wrong dim
    flat = [b for r in blobs for b in r]
    keep = [C.c_char_p(b) for b in flat]
    ptrs = (C.c_void_p * len(flat))(*[C.cast(k, C.c_void_p) for k in keep])
    lens = (C.c_int64 * len(flat))(*[len(b) for b in flat])
    pd = (C.c_int64 * 2)(*dims)
    out = np.zeros((4, 7), np.float32)
    st = np.zeros(4, np.int8)
    good = lib.ingest_concat_rows(ptrs, lens, 4, 2, pd, out.ctypes.data, st.ctypes.data)
    assert good == 2 and list(st) == [0, 1, 2, 0]
    for r in (0, 3):
        np.testing.assert_array_equal(out[r], np.concatenate(rows[r]))


def test_normalize_L2_host_entry():
    from image_recommender_amd import faiss_compat as faiss
    x = np.random.default_rng(1).standard_normal((6, 19)).astype(np.float32)
    x[2] = 0
    y = x.copy()
    faiss.normalize_L2(y)
    n = np.linalg.norm(x, axis=1)
    np.testing.assert_allclose(y[n > 0], x[n > 0] / n[n > 0, None], rtol=3e-7, atol=1e-7)
    assert (y[2] == 0).all()
    v = x[0].copy()
    faiss.normalize_L2(v)
    np.testing.assert_allclose(v, x[0] / n[0], rtol=3e-7)


def test_packed_layout_matches_library():
    """sharded.packed_layout (the Python views) and knn_packed_bytes (the merge's reading of the
    chunk) agree, odd nq*k included; bad shapes are rejected."""
    from image_recommender_amd.sharded import packed_layout
    lib = _lib.load()
    for nq, k in [(1, 1), (3, 3), (7, 10), (1024, 10), (5, 32)]:
        nbytes, off = packed_layout(nq, k)
        assert lib.knn_packed_bytes(nq, k) == nbytes
        assert off % 8 == 0 and off >= 4 * nq * k and nbytes - off == 8 * nq * k
    assert lib.knn_packed_bytes(-1, 3) < 0 and lib.knn_packed_bytes(3, 0) < 0
