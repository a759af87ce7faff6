"""Index build over the SQLite embedding tables — drop-in for the reference's main.create_index.

Mirrors /root/reference/main/create_index.py (FAISSIndexBuilderDB, :13-325): same constructor
arguments and defaults (:14-24), same index file name ``index_hnsw_<types>.faiss`` (:36-37), same
offsets table ``faiss_index_offsets_<types>(image_id INTEGER PRIMARY KEY, offset INTEGER)``
(:99-113, :236-249), same SQL join over the per-type vector tables (:115-158), same log lines.
What changes is underneath:

* the index is this package's exact MI355X flat index (``faiss_compat``), resident in HBM, written
  in faiss's IndexFlat file layout;
* BLOBs are decoded natively in batches (``ingest.decode_rows``) and the table is scanned ONCE
  (the reference scans and unpickles everything twice: a training pass :283-292 and an add pass
  :304-317; a flat index needs no training pass, ``train`` is still called on the first batch);
* the build order of the vector types is recorded in ``<index_file>.meta.json`` so the searcher
  can concatenate queries in the order the index was built with (fixes SURVEY Appendix C.1: the
  reference builds ``color_sift_dreamsim`` but searches ``color_dreamsim_sift``).

Reproduced on purpose: ``update_index=True`` still re-adds every row without clearing the file or
the offsets (:269-320, Appendix C.2); rows missing any part are skipped (inner JOIN); a row whose
BLOB fails to decode is skipped with a warning (:181-185).
CLI: ``python -m image_recommender_amd.main.create_index --db-path images.db --vector-types color
sift dreamsim`` — the flags the reference README documents (README.md:101-110) but never parses.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import queue
import sqlite3
import threading
from pathlib import Path
from types import SimpleNamespace

import numpy as np

from .. import faiss_compat as faiss
from ..ingest import decode_rows, scan_native

os.environ.setdefault("KMP_DUPLICATE_LIB_OK", "TRUE")


class FAISSIndexBuilderDB:
    def __init__(
        self,
        db_path: str = "images.db",
        vector_types: list = None,
        batch_size: int = 8192,
        index_file: str = None,
        hnsw_M: int = 32,
        efConstruction: int = 200,
        efSearch: int = 64,
        log_file: str = "faiss_builder.log",
        log_dir: str = "logs",
        device: int = -1,
    ):
        self.log_dir = log_dir
        self.log_file = log_file
        self._setup_logging()

        self.db_path = db_path
        self.vector_types = list(vector_types or ["color"])
        self.vector_cols = [f"{t}_vector_blob" for t in self.vector_types]
        self.batch_size = batch_size

        name = "_".join(self.vector_types)
        self.index_file = Path(index_file) if index_file else Path(f"index_hnsw_{name}.faiss")
        self.hnsw_M = hnsw_M
        self.efConstruction = efConstruction
        self.efSearch = efSearch
        self.device = device
        self.offset_table = f"faiss_index_offsets_{name}"

        self.read_conn = sqlite3.connect(self.db_path)
        self._configure_db(self.read_conn)
        self.read_cur = self.read_conn.cursor()
        self.write_conn = sqlite3.connect(self.db_path)
        self._configure_db(self.write_conn)
        self.write_cur = self.write_conn.cursor()
        self._prepare_offset_table()

    # ---- logging / DB setup (create_index.py:55-113) -----------------------------------------
    def _setup_logging(self):
        Path(self.log_dir).mkdir(parents=True, exist_ok=True)
        full_path = Path(self.log_dir) / self.log_file
        logging.basicConfig(level=logging.INFO, filename=str(full_path), filemode="a",
                            format="%(asctime)s - %(levelname)s - %(message)s", encoding="utf-8")
        self._log(f"Logging initialized (file={full_path})", level="info")

    def _log(self, message: str, level: str = "info"):
        print(message)
        getattr(logging, level.lower() if level.lower() in ("info", "warning", "error") else "debug")(message)

    def _configure_db(self, conn):
        conn.execute("PRAGMA journal_mode=WAL;")
        conn.execute("PRAGMA synchronous=OFF;")

    def _prepare_offset_table(self):
        self.write_cur.execute(
            f"CREATE TABLE IF NOT EXISTS {self.offset_table} ("
            f"image_id INTEGER PRIMARY KEY, offset INTEGER);")
        self.write_conn.commit()
        self._log(f"Offset table '{self.offset_table}' is ready.", level="info")

    # ---- SQL (create_index.py:115-158) ---------------------------------------------------------
    def _make_select_and_joins(self):
        select_cols = ["i.id"]
        join_strs = []
        for k, vtype in enumerate(self.vector_types):
            alias = f"v{k}"   # the reference uses vtype[0], which collides for equal initials
            select_cols.append(f"{alias}.{vtype}_vector_blob")
            join_strs.append(f"JOIN {vtype}_vectors {alias} ON i.id = {alias}.image_id")
        return ", ".join(select_cols), " ".join(join_strs)

    def _count_records(self):
        _, join_strs = self._make_select_and_joins()
        return self.read_cur.execute(f"SELECT COUNT(*) FROM images i {join_strs}").fetchone()[0]

    def _batch_records(self):
        select_cols, join_strs = self._make_select_and_joins()
        self.read_cur.execute(f"SELECT {select_cols} FROM images i {join_strs}")
        while True:
            rows = self.read_cur.fetchmany(self.batch_size)
            if not rows:
                break
            yield rows

    def _process_batch(self, rows, part_dims=None):
        """(ids, float32 matrix, part_dims) of the decodable rows, parts in caller order."""
        return decode_rows(rows, self.vector_types, part_dims, log=self._log)

    # ---- the build's scan: native when the system SQLite library loads (§8f row 1) ------------
    def _probe_part_dims(self, probe_rows=64):
        select_cols, join_strs = self._make_select_and_joins()
        rows = self.read_cur.execute(
            f"SELECT {select_cols} FROM images i {join_strs} LIMIT {int(probe_rows)}").fetchall()
        return decode_rows(rows, self.vector_types, None, log=lambda *a, **k: None)[2]

    def _refetch(self, ids):
        """The (id, blob...) rows of `ids` (rows the native scan could not parse), on a
        connection of the calling thread (the scan's producer thread)."""
        select_cols, join_strs = self._make_select_and_joins()
        out = []
        con = sqlite3.connect(self.db_path)
        try:
            for i in range(0, len(ids), 900):            # SQLite's bound-variable limit
                chunk = ids[i:i + 900]
                out += con.execute(
                    f"SELECT {select_cols} FROM images i {join_strs} WHERE i.id IN "
                    f"({','.join('?' * len(chunk))})", chunk).fetchall()
        finally:
            con.close()
        return out

    def _decoded_batches(self):
        """(ids, float32 matrix, part_dims) per batch of the scan, in the query's row order.

        Native path (ingest.scan_native: the same SELECT stepped from C, BLOBs parsed in place)
        on a producer thread, so the scan of batch i+1 overlaps the index add of batch i (both
        release the GIL); rows it cannot parse are re-read and decoded by _process_batch's pickle
        fallback.  Without the native scan: _batch_records + _process_batch (the reference's
        loop, create_index.py:136-189, with the batch decode in C)."""
        part_dims = self._probe_part_dims()
        if part_dims is not None:
            select_cols, join_strs = self._make_select_and_joins()
            sql = f"SELECT {select_cols} FROM images i {join_strs}"
            try:
                gen = scan_native(self.db_path, sql, self.vector_types, part_dims, self.batch_size,
                                  self._refetch, log=self._log)
                first = next(gen, None)
            except NotImplementedError as e:
                self._log(f"native scan unavailable ({e}); scanning in Python", level="warning")
                gen = None
            if gen is not None:
                if first is None:
                    return
                q: queue.Queue = queue.Queue(maxsize=2)

                def produce():
                    try:
                        for item in gen:
                            q.put(item)
                        q.put(None)
                    except BaseException as e:   # noqa: BLE001 - re-raised on the consumer side
                        q.put(e)
                t = threading.Thread(target=produce, daemon=True)
                t.start()
                yield first[0], first[1], part_dims
                while True:
                    item = q.get()
                    if item is None:
                        break
                    if isinstance(item, BaseException):
                        raise item
                    yield item[0], item[1], part_dims
                t.join()
                return
        for batch in self._batch_records():
            ids, arr, part_dims = self._process_batch(batch, part_dims)
            yield ids, arr, part_dims

    # ---- index (create_index.py:191-234) -------------------------------------------------------
    def find_valid_m(self, dim, candidates=(64, 56, 48, 32, 28, 24, 16, 12, 8)):
        for m in candidates:
            if dim % m == 0:
                return m
        return 1

    def _initialize_index(self, dim, use_pq=True):
        if use_pq:
            # the reference's IndexHNSWFlat(dim, 32) coarse quantiser (create_index.py:219-221) is
            # recorded as parameters only: the exact index never consults it, so no second device
            # index is created for it
            coarse = SimpleNamespace(d=dim, hnsw=SimpleNamespace(
                M=self.hnsw_M, efConstruction=self.efConstruction, efSearch=self.efSearch))
            nlist, m, nbits = 2048, self.find_valid_m(dim), 12
            index = faiss.IndexIVFPQ(coarse, dim, nlist, m, nbits, device=self.device)
            self._log(f"Created exact MI355X flat index behind the IVFPQ interface "
                      f"(dim={dim}, nlist={nlist}, m={m}, nbits={nbits}: recorded, search is exact)",
                      level="info")
            return index
        index = faiss.IndexHNSWFlat(dim, self.hnsw_M, device=self.device)
        index.hnsw.efConstruction = self.efConstruction
        index.hnsw.efSearch = self.efSearch
        self._log(f"Created exact MI355X flat index (dim={dim}, M={self.hnsw_M} recorded)", level="info")
        return index

    def _store_offsets(self, ids, start_offset):
        pairs = [(rid, start_offset + i) for i, rid in enumerate(ids)]
        self.write_cur.executemany(
            f"INSERT OR REPLACE INTO {self.offset_table} (image_id, offset) VALUES (?, ?)", pairs)
        self.write_conn.commit()

    def _write_meta(self, dim, part_dims):
        meta = {"vector_types": self.vector_types, "part_dims": part_dims, "dim": dim,
                "offset_table": self.offset_table, "metric": "L2"}
        Path(str(self.index_file) + ".meta.json").write_text(json.dumps(meta))

    # ---- build (create_index.py:251-325) -------------------------------------------------------
    def build_index(self, update_index: bool = False):
        combo = "_".join(self.vector_types)
        self._log(f"Starting FAISS index build for [{combo}]…", level="info")
        if not update_index:
            if self.index_file.exists():
                self._log(f"Removing existing index {self.index_file}", level="info")
                self.index_file.unlink()
            self._log(f"Clearing offset table {self.offset_table}", level="info")
            self.write_cur.execute(f"DELETE FROM {self.offset_table}")
            self.write_conn.commit()

        total = self._count_records()
        self._log(f"{total} complete records found.", level="info")
        if total == 0:
            self._log("No complete embeddings found; aborting.", level="error")
            return None

        index = None
        part_dims = None
        offset_counter = 0
        batch_num = 0
        for ids, arr, part_dims in self._decoded_batches():
            batch_num += 1
            if len(ids) == 0:
                continue
            if index is None:
                index = self._initialize_index(arr.shape[1])
                index.reserve(total)
                if not index.is_trained:
                    index.train(arr)
            index.add(arr)
            self._store_offsets(ids, offset_counter)
            offset_counter += len(ids)
            self._log(f"Batch {batch_num}: added {len(ids)} vectors (total {offset_counter}).",
                      level="info")
        if index is None:
            self._log("No decodable embeddings found; aborting.", level="error")
            return None
        self._log(f"Writing FAISS index to {self.index_file.resolve()}", level="info")
        faiss.write_index(index, str(self.index_file))
        self._write_meta(int(index.d), part_dims)
        self._log(f"Index saved ({index.ntotal} vectors).", level="info")
        self.read_conn.close()
        self.write_conn.close()
        self._log("Done.", level="info")
        return index


def main(argv=None):
    ap = argparse.ArgumentParser(description="Build the exact MI355X k-NN index from images.db")
    ap.add_argument("--db-path", default="images.db")
    ap.add_argument("--vector-types", nargs="+", default=["color"])
    ap.add_argument("--output", default=None, help="index file (default index_hnsw_<types>.faiss)")
    ap.add_argument("--batch-size", type=int, default=8192)
    ap.add_argument("--hnsw_M", type=int, default=32)
    ap.add_argument("--efConstruction", type=int, default=200)
    ap.add_argument("--efSearch", type=int, default=64)
    ap.add_argument("--update-index", action="store_true")
    ap.add_argument("--device", type=int, default=-1)
    a = ap.parse_args(argv)
    types = [t for v in a.vector_types for t in v.split(",") if t]
    FAISSIndexBuilderDB(db_path=a.db_path, vector_types=types, batch_size=a.batch_size,
                        index_file=a.output, hnsw_M=a.hnsw_M, efConstruction=a.efConstruction,
                        efSearch=a.efSearch, device=a.device).build_index(update_index=a.update_index)


if __name__ == "__main__":
    main()
