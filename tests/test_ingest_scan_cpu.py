"""The native scan of the index build (include/imgrec_ingest.h ingest_scan_*; CPU, no GPU needed).

ingest.scan_native steps the builder's own SELECT from C through the system SQLite library and
parses the protocol-5 BLOBs in place.  It must yield exactly what the reference-shaped Python
loop yields (_batch_records + _process_batch, /root/reference/main/create_index.py:136-189):
same ids in the same order, the same float32 rows, with BLOBs in other layouts (float64 arrays,
lists) going through the pickle fallback and undecodable rows skipped with the reference's
warning."""
import pickle
import sqlite3

import numpy as np
import pytest

from image_recommender_amd import ingest
from image_recommender_amd.main.create_db import create_schema

TYPES = ["color", "sift"]
DIMS = [48, 128]


def _make_db(path, n=3000, seed=0):
    rng = np.random.default_rng(seed)
    con = sqlite3.connect(path)
    create_schema(con, TYPES)
    special = {}
    for i in range(1, n + 1):
        con.execute("INSERT INTO images (id, path) VALUES (?, ?)", (i, f"img/{i}.jpg"))
        for t, d in zip(TYPES, DIMS):
            v = rng.standard_normal(d).astype(np.float32)
            blob = pickle.dumps(v, protocol=5)
            if t == "sift" and i % 997 == 0:          # another layout: the pickle fallback
                blob = pickle.dumps(v.astype(np.float64), protocol=4)
                special[i] = "float64"
            if t == "color" and i % 1201 == 0:        # undecodable: skipped with a warning
                blob = b"not a pickle"
                special[i] = "corrupt"
            if t == "sift" and i % 1499 == 0:         # wrong dimension: skipped
                blob = pickle.dumps(rng.standard_normal(d + 1).astype(np.float32), protocol=5)
                special[i] = "dim"
            con.execute(f"INSERT INTO {t}_vectors (image_id, {t}_vector_blob) VALUES (?, ?)",
                        (i, sqlite3.Binary(blob)))
    # an image with only one part is excluded by the JOIN
    con.execute("INSERT INTO images (id, path) VALUES (?, ?)", (n + 1, "img/lonely.jpg"))
    con.execute("INSERT INTO color_vectors (image_id, color_vector_blob) VALUES (?, ?)",
                (n + 1, sqlite3.Binary(pickle.dumps(np.zeros(48, np.float32), protocol=5))))
    con.commit()
    con.close()
    return special


def _sql():
    sel = ", ".join(["i.id"] + [f"v{k}.{t}_vector_blob" for k, t in enumerate(TYPES)])
    joins = " ".join(f"JOIN {t}_vectors v{k} ON i.id = v{k}.image_id" for k, t in enumerate(TYPES))
    return f"SELECT {sel} FROM images i {joins}"


@pytest.mark.parametrize("batch", [1, 512, 8192])
def test_native_scan_equals_python_scan(tmp_path, batch):
    db = tmp_path / "images.db"
    special = _make_db(db)
    con = sqlite3.connect(db)
    py_ids, py_rows, logs_py = [], [], []
    cur = con.execute(_sql())
    while True:
        rows = cur.fetchmany(batch)
        if not rows:
            break
        ids, arr, _ = ingest.decode_rows(rows, TYPES, DIMS, log=lambda m, lv="warning": logs_py.append(m))
        py_ids += list(ids)
        py_rows.append(arr)

    def refetch(ids):
        return con.execute(_sql() + f" WHERE i.id IN ({','.join('?' * len(ids))})", ids).fetchall()

    nat_ids, nat_rows, logs_nat = [], [], []
    for ids, arr in ingest.scan_native(str(db), _sql(), TYPES, DIMS, batch, refetch,
                                       log=lambda m, lv="warning": logs_nat.append(m)):
        assert len(ids) == arr.shape[0] <= batch
        nat_ids += list(ids)
        nat_rows.append(arr)
    con.close()
    assert nat_ids == py_ids
    np.testing.assert_array_equal(np.concatenate(nat_rows), np.concatenate(py_rows))
    assert sorted(logs_nat) == sorted(logs_py)
    # float64 BLOBs came through the fallback; corrupt and wrong-dimension rows were skipped
    for i, kind in special.items():
        assert (i in nat_ids) == (kind == "float64"), (i, kind)
    assert 3001 not in nat_ids


def test_native_scan_reports_sql_errors(tmp_path):
    db = tmp_path / "images.db"
    _make_db(db, n=10)
    with pytest.raises(RuntimeError, match="sqlite3_prepare_v2"):
        list(ingest.scan_native(str(db), "SELECT nope FROM nowhere", TYPES, DIMS, 8, lambda ids: []))


def test_builder_decoded_batches_native_equals_reference_loop(tmp_path, monkeypatch):
    """FAISSIndexBuilderDB._decoded_batches (native scan on a producer thread, refetch of the
    rows it cannot parse on that thread's own connection) yields what the reference-shaped loop
    (_batch_records + _process_batch) yields."""
    from image_recommender_amd.main.create_index import FAISSIndexBuilderDB
    db = tmp_path / "images.db"
    _make_db(db, n=2500)
    monkeypatch.chdir(tmp_path)
    b = FAISSIndexBuilderDB(db_path=str(db), vector_types=TYPES, batch_size=700,
                            log_dir=str(tmp_path / "logs"))
    got = [(list(ids), arr) for ids, arr, _ in b._decoded_batches()]
    ref = []
    dims = None
    for rows in b._batch_records():
        ids, arr, dims = b._process_batch(rows, dims)
        ref.append((list(ids), arr))
    assert [i for ids, _ in got for i in ids] == [i for ids, _ in ref for i in ids]
    np.testing.assert_array_equal(np.concatenate([a for _, a in got]), np.concatenate([a for _, a in ref]))
