#!/usr/bin/env python3
"""Bulk-ingest throughput of the index build.

The reference builds its index from SQLite BLOB tables with TWO full scans, each unpickling every
BLOB row by row (/root/reference/main/create_index.py:160-189 _process_batch, :283-317 the
training pass and the add pass).  Here FAISSIndexBuilderDB.build_index makes one scan, decodes a
whole batch per native call (csrc/ingest.cpp) and adds it to the HBM-resident index.

This tool writes an images.db of N rows with the three BLOB tables of config 3 (color 48 |
sift 128 | dreamsim 1792 float32, pickled protocol 5 as vector_scripts/create_vector_base.py:144
writes them), then times, on the same host:
  native      ingest.scan_native: the builder's SELECT stepped from C (system SQLite), BLOBs
              parsed in place (the build's default path)
  scan        the Python sqlite3 SELECT ... JOIN fetchmany loop alone (no decode)
  decode      ingest.decode_rows on every batch of that scan (native BLOB parser)
  add         index.add of the decoded batches (H2D + HBM layout + bf16 copy) — GPU only
  build       FAISSIndexBuilderDB(...).build_index() end to end (scan + decode + add + offsets
              table + faiss.write_index of the index file) — GPU only
  reference   the reference's decode shape: two scans, pickle.loads per BLOB, np.concatenate
              per row, np.stack per batch (oracle/plumbing.py's restatement), no faiss
One JSON line with rows/s per phase.  Usage: bench_ingest.py [--rows N] [--db PATH] [--keep]
"""
from __future__ import annotations

import argparse
import json
import os
import pickle
import sqlite3
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

PARTS = (("color", 48), ("sift", 128), ("dreamsim", 1792))


def make_db(path: Path, n: int, batch: int = 20000, seed: int = 0) -> float:
    from image_recommender_amd.main.create_db import create_schema
    t0 = time.perf_counter()
    con = sqlite3.connect(path)
    con.execute("PRAGMA journal_mode=WAL;")
    con.execute("PRAGMA synchronous=OFF;")
    create_schema(con, [p for p, _ in PARTS])
    rng = np.random.default_rng(seed)
    for r0 in range(0, n, batch):
        m = min(batch, n - r0)
        ids = range(r0 + 1, r0 + m + 1)
        con.executemany("INSERT INTO images (id, path) VALUES (?, ?)",
                        [(i, f"image_data/img_{i:08d}.jpg") for i in ids])
        for name, d in PARTS:
            x = rng.standard_normal((m, d), dtype=np.float32)
            x /= np.linalg.norm(x, axis=1, keepdims=True)
            con.executemany(f"INSERT INTO {name}_vectors (image_id, {name}_vector_blob) VALUES (?, ?)",
                            [(i, sqlite3.Binary(pickle.dumps(x[j], protocol=pickle.HIGHEST_PROTOCOL)))
                             for j, i in enumerate(ids)])
        con.commit()
    con.close()
    return time.perf_counter() - t0


def scan_batches(path: Path, types, batch: int):
    con = sqlite3.connect(path)
    sel = ", ".join(["i.id"] + [f"v{k}.{t}_vector_blob" for k, t in enumerate(types)])
    joins = " ".join(f"JOIN {t}_vectors v{k} ON i.id = v{k}.image_id" for k, t in enumerate(types))
    cur = con.execute(f"SELECT {sel} FROM images i {joins}")
    while True:
        rows = cur.fetchmany(batch)
        if not rows:
            break
        yield rows
    con.close()


def reference_pass(path: Path, types, batch: int) -> int:
    """One reference-shaped scan: create_index.py:170-189 per row, then np.stack per batch."""
    n = 0
    for rows in scan_batches(path, types, batch):
        embs = []
        for rec_id, *blobs in rows:
            parts = []
            for blob in blobs:
                vec = pickle.loads(blob)
                if hasattr(vec, "cpu"):
                    vec = vec.cpu().numpy()
                parts.append(np.asarray(vec, dtype="float32").ravel())
            embs.append(np.concatenate(parts))
        arr = np.stack(embs).astype("float32")
        n += arr.shape[0]
    return n


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--db", default=None)
    ap.add_argument("--batch", type=int, default=8192, help="the builder's batch_size")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    types = [p for p, _ in PARTS]
    tmp = Path(a.db).parent if a.db else Path(os.environ.get("TMPDIR", tempfile.gettempdir()))
    db = Path(a.db) if a.db else tmp / f"ingest_{a.rows}.db"
    out = {"rows": a.rows, "dim": sum(d for _, d in PARTS), "batch": a.batch,
           "parts": {p: d for p, d in PARTS}, "db": str(db)}
    if not db.exists():
        out["generate_s"] = make_db(db, a.rows)
    out["db_bytes"] = db.stat().st_size
    from image_recommender_amd import _lib
    from image_recommender_amd.ingest import decode_rows
    _lib.load()                               # library load (HIP runtime init) outside the timing

    # scan alone, then scan + native decode (decode time measured around each call)
    t0 = time.perf_counter()
    n = sum(len(r) for r in scan_batches(db, types, a.batch))
    t_scan = time.perf_counter() - t0
    t_dec, nd, mats = 0.0, 0, []
    t0 = time.perf_counter()
    dims = None
    for rows in scan_batches(db, types, a.batch):
        t1 = time.perf_counter()
        ids, arr, dims = decode_rows(rows, types, dims)
        t_dec += time.perf_counter() - t1
        nd += len(ids)
        if not a.no_gpu:
            mats.append(arr)
    t_scan_dec = time.perf_counter() - t0
    assert n == a.rows and nd == a.rows, (n, nd)
    # the builder's default path: the same SELECT stepped from C, BLOBs parsed in place
    from image_recommender_amd.ingest import scan_native
    sel = ", ".join(["i.id"] + [f"v{k}.{t}_vector_blob" for k, t in enumerate(types)])
    joins = " ".join(f"JOIN {t}_vectors v{k} ON i.id = v{k}.image_id" for k, t in enumerate(types))
    t0 = time.perf_counter()
    nn = sum(len(ids) for ids, _ in scan_native(str(db), f"SELECT {sel} FROM images i {joins}",
                                                 types, dims, a.batch, lambda ids: []))
    t_nat = time.perf_counter() - t0
    assert nn == a.rows
    out["native_scan_decode"] = {"s": t_nat, "rows_per_s": nn / t_nat,
                                 "GB_per_s": nn * out["dim"] * 4 / t_nat / 1e9,
                                 "note": "ingest.scan_native (C: sqlite3_step + in-place BLOB parse)"}
    out["scan"] = {"s": t_scan, "rows_per_s": n / t_scan}
    out["decode"] = {"s": t_dec, "rows_per_s": nd / t_dec, "GB_per_s": nd * out["dim"] * 4 / t_dec / 1e9}
    out["scan_plus_decode"] = {"s": t_scan_dec, "rows_per_s": nd / t_scan_dec}

    if not a.no_gpu:
        import torch
        from image_recommender_amd import faiss_compat as faiss
        from image_recommender_amd.main.create_index import FAISSIndexBuilderDB
        idx = faiss.IndexFlatL2(out["dim"])
        idx.reserve(nd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for arr in mats:
            idx.add(arr)
        torch.cuda.synchronize()
        t_add = time.perf_counter() - t0
        out["add"] = {"s": t_add, "rows_per_s": nd / t_add, "GB_per_s": nd * out["dim"] * 4 / t_add / 1e9}
        del idx, mats
        index_file = tmp / f"ingest_{a.rows}.faiss"
        logdir = tmp / "ingest_logs"
        t0 = time.perf_counter()
        b = FAISSIndexBuilderDB(db_path=str(db), vector_types=types, batch_size=a.batch,
                                index_file=str(index_file), log_dir=str(logdir))
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            index = b.build_index()
        t_build = time.perf_counter() - t0
        out["build"] = {"s": t_build, "rows_per_s": index.ntotal / t_build,
                        "index_file_bytes": index_file.stat().st_size,
                        "note": "FAISSIndexBuilderDB.build_index end to end: one scan, native decode, "
                                "add, offsets table, faiss.write_index"}
        del index
        index_file.unlink(missing_ok=True)

    t0 = time.perf_counter()
    nr1 = reference_pass(db, types, a.batch)      # the training pass (create_index.py:283-291)
    t_r1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    nr2 = reference_pass(db, types, a.batch)      # the add pass (create_index.py:300-317)
    t_r2 = time.perf_counter() - t0
    out["reference_two_pass_decode"] = {
        "s": t_r1 + t_r2, "pass_s": [t_r1, t_r2], "rows_per_s": nr2 / (t_r1 + t_r2),
        "note": "two scans of pickle.loads per BLOB + np.concatenate per row + np.stack per batch "
                "(create_index.py:160-189 x 2), no faiss train/add (faiss absent)"}
    out["speedup_python_scan_decode"] = out["reference_two_pass_decode"]["s"] / t_scan_dec
    out["speedup_native_scan_decode"] = out["reference_two_pass_decode"]["s"] / t_nat
    out["host"] = {"cpu_model": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                                      if l.startswith("model name")), "?"),
                   "python_threads": 1}
    if not a.keep and not a.db:
        for suf in ("", "-wal", "-shm"):
            Path(str(db) + suf).unlink(missing_ok=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
