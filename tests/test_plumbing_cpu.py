"""CPU tests of the build/search plumbing against fixtures captured from the REFERENCE's own
modules (tests/golden/plumbing.json, made by tests/golden/make_golden.py under import stubs).

Covers: canonical type order (search_from_image.py:256-273), the builder's SQL + BLOB decoding +
concatenation order + batching + offsets (create_index.py:115-189, 236-249, 301-317) through the
native decoder, and query assembly before normalisation (search_from_image.py:275-322).
"""
import hashlib
import json
import pickle
import sqlite3
from pathlib import Path

import numpy as np
import pytest

from oracle import plumbing
from tests.golden.make_golden import build_db

GOLDEN = json.loads((Path(__file__).parent / "golden" / "plumbing.json").read_text())


@pytest.fixture()
def golden_db(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    recipe = build_db(tmp_path / "images.db")
    assert recipe["paths"] == GOLDEN["recipe"]["paths"]
    return tmp_path / "images.db"


def test_oracle_canonical_order_matches_reference():
    for s, want in GOLDEN["ordered_types"].items():
        assert plumbing.ordered_index_types(s) == want


def test_package_canonical_order_matches_reference():
    from image_recommender_amd.main.search_from_image import ImageRecommender
    rec = ImageRecommender.__new__(ImageRecommender)
    for s, want in GOLDEN["ordered_types"].items():
        assert ImageRecommender._get_ordered_index_types(rec, s) == want


def test_find_valid_m():
    assert [plumbing.find_valid_m(d) for d in (512, 768, 1968, 48, 1840, 7)] == [64, 64, 48, 48, 16, 1]


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("combo", list(GOLDEN["builds"]))
def test_oracle_build_rows_match_reference(golden_db, combo):
    g = GOLDEN["builds"][combo]
    types = g["index_file"][len("index_hnsw_"):-len(".faiss")].split("_")
    ids, mat = plumbing.build_rows(str(golden_db), types)
    assert [[i, k] for k, i in enumerate(ids)] == g["offsets"]
    assert mat.shape == (g["ntotal"], g["dim"])
    assert _digest(mat) == g["matrix_sha256"]


@pytest.mark.parametrize("combo", list(GOLDEN["builds"]))
def test_builder_decode_and_offsets_match_reference(golden_db, combo, tmp_path):
    """FAISSIndexBuilderDB's scan through the native BLOB decoder, batch size 7 as in the fixture."""
    from image_recommender_amd.main.create_index import FAISSIndexBuilderDB
    g = GOLDEN["builds"][combo]
    types = g["index_file"][len("index_hnsw_"):-len(".faiss")].split("_")
    b = FAISSIndexBuilderDB(db_path=str(golden_db), vector_types=types, batch_size=7,
                            log_dir=str(tmp_path / "logs"))
    assert b.index_file.name == g["index_file"] and b.offset_table == g["offset_table"]
    ids_all, mats, batches, dims = [], [], [], None
    for rows in b._batch_records():
        ids, arr, dims = b._process_batch(rows, dims)
        if ids:
            batches.append(len(ids))
            ids_all += ids
            mats.append(arr)
    mat = np.concatenate(mats)
    assert batches == g["add_batches"]
    assert [[i, k] for k, i in enumerate(ids_all)] == g["offsets"]
    assert _digest(mat) == g["matrix_sha256"]
    assert mat[0, :4].tolist() == pytest.approx(g["first_row_head"], rel=0, abs=0)


def test_decode_rows_fallbacks(tmp_path):
    """Non-fast-layout BLOBs take the reference's pickle path; broken ones are skipped."""
    from image_recommender_amd.ingest import decode_rows
    rng = np.random.default_rng(0)
    a = [rng.standard_normal(4).astype(np.float32) for _ in range(4)]
    b = [rng.standard_normal(3).astype(np.float32) for _ in range(4)]
    rows = [(1, pickle.dumps(a[0], 5), pickle.dumps(b[0], 5)),
            (2, pickle.dumps(a[1].astype(np.float64), 5), pickle.dumps(b[1], 5)),   # fallback
            (3, b"garbage", pickle.dumps(b[2], 5)),                                   # skipped
            (4, pickle.dumps(a[3].tolist(), 5), pickle.dumps(b[3].reshape(1, 3), 5))]
    logs = []
    ids, mat, dims = decode_rows(rows, ["x", "y"], None, log=lambda m, lvl="warning": logs.append(m))
    assert ids == [1, 2, 4] and dims == [4, 3]
    np.testing.assert_array_equal(mat[0], np.concatenate([a[0], b[0]]))
    np.testing.assert_array_equal(mat[1], np.concatenate([a[1], b[1]]))
    np.testing.assert_array_equal(mat[2], np.concatenate([a[3], b[3]]))
    assert any("ID 3: error loading x" in m for m in logs)


def test_query_assembly_matches_reference(golden_db, monkeypatch):
    """The pre-normalisation query vector equals the one the reference passed to normalize_L2."""
    import image_recommender_amd.main.search_from_image as sfi
    seen = []
    real = sfi.faiss.normalize_L2
    monkeypatch.setattr(sfi.faiss, "normalize_L2", lambda x: (seen.append(x.copy()), real(x)))
    rec = sfi.ImageRecommender(images_root=".", db_path=str(golden_db), top_k=5)
    for s in GOLDEN["searches"]:
        if s["query_vector"] is None:
            continue
        seen.clear()
        ordered = rec._get_ordered_index_types(s["index_type"])
        q = rec._extract_query_vector(s["paths"], ordered)
        assert q is not None and len(seen) == 1
        np.testing.assert_array_equal(seen[0], np.asarray(s["query_vector"], np.float32))
        n = np.linalg.norm(seen[0])
        np.testing.assert_allclose(q, seen[0] / n, rtol=1e-6, atol=1e-9)


def test_offsets_table_schema(golden_db, tmp_path):
    from image_recommender_amd.main.create_index import FAISSIndexBuilderDB
    FAISSIndexBuilderDB(db_path=str(golden_db), vector_types=["color"], log_dir=str(tmp_path / "l"))
    con = sqlite3.connect(golden_db)
    cols = con.execute("PRAGMA table_info(faiss_index_offsets_color)").fetchall()
    assert [(c[1], c[2], c[5]) for c in cols] == [("image_id", "INTEGER", 1), ("offset", "INTEGER", 0)]
