"""Resumable batch feature extraction into the SQLite vector tables.

Mirrors /root/reference/vector_scripts/create_vector_base.py (BaseVectorIndexer, :11-207): rows of
``images`` without a vector in ``<table>`` are fetched in id order (``LEFT JOIN ... IS NULL AND
i.id > last``, :98-115), ``compute_vectors`` runs on their paths, and the results are upserted as
``pickle.dumps(vec, HIGHEST_PROTOCOL)`` BLOBs in one transaction per batch (:131-162) — the exact
BLOB format the index builder decodes.  SIGINT exits cleanly (:75-84).
``load_image`` (:212-274) decodes with PIL (OpenCV is not part of this path): RGB, optional resize
(LANCZOS), optional [0, 1] scaling.
"""
from __future__ import annotations

import logging
import pickle
import signal
import sqlite3
import sys
from pathlib import Path

import numpy as np


class BaseVectorIndexer:
    vector_column: str = None
    batch_size: int = 1024
    table_name: str = None
    path_column: str = "path"
    id_column: str = "image_id"

    def __init__(self, db_path: str, base_dir: str, batch_size: int = None,
                 log_file: str = "vector_indexer.log", log_dir: str = "logs",
                 install_sigint: bool = True):
        self.db_path = db_path
        self.base_dir = Path(base_dir)
        if batch_size is not None:
            self.batch_size = batch_size
        self._setup_logging(log_file, log_dir)
        self._init_db()
        if install_sigint:
            try:
                signal.signal(signal.SIGINT, self._handle_sigint)
            except ValueError:       # not the main thread
                pass

    def _setup_logging(self, log_file: str, log_dir: str):
        Path(log_dir).mkdir(parents=True, exist_ok=True)
        full_path = Path(log_dir) / log_file
        logging.basicConfig(level=logging.INFO, filename=str(full_path), filemode="a",
                            format="%(asctime)s - %(levelname)s - %(message)s", encoding="utf-8")
        self._log_and_print(f"Logging initialized at {full_path}", level="info")

    def _log_and_print(self, message: str, level: str = "info"):
        print(message)
        lvl = level.lower()
        getattr(logging, lvl if lvl in ("info", "warning", "error") else "debug")(message)

    def _handle_sigint(self, signum, frame):
        self._log_and_print("Aborted by user.", level="info")
        sys.exit(0)

    def _init_db(self):
        self.read_conn = sqlite3.connect(self.db_path, timeout=30, isolation_level=None)
        self.read_conn.execute("PRAGMA journal_mode=WAL;")
        self.write_conn = sqlite3.connect(self.db_path, timeout=30, isolation_level=None)
        self.write_conn.execute("PRAGMA journal_mode=WAL;")
        self.write_conn.execute("PRAGMA synchronous=OFF;")
        self.write_conn.execute("PRAGMA temp_store=MEMORY;")
        self._log_and_print(f"Connected to DB: {self.db_path}", level="info")

    def get_pending_rows(self, last_id: int):
        sql = (f"SELECT i.id, i.path FROM images i "
               f"LEFT JOIN {self.table_name} v ON i.id = v.image_id "
               f"WHERE v.{self.vector_column} IS NULL AND i.id > ? "
               f"ORDER BY i.id ASC LIMIT ?")
        return self.read_conn.cursor().execute(sql, (last_id, self.batch_size)).fetchall()

    def compute_vectors(self, paths: list[str]):
        raise NotImplementedError

    def write_updates(self, id_vec_pairs):
        if not id_vec_pairs:
            self._log_and_print("No vectors to write for this batch.", level="warning")
            return
        blobs = [(rid, sqlite3.Binary(pickle.dumps(vec, protocol=pickle.HIGHEST_PROTOCOL)))
                 for rid, vec in id_vec_pairs]
        cur = self.write_conn.cursor()
        sql = (f"INSERT INTO {self.table_name} (image_id, {self.vector_column}) VALUES (?, ?) "
               f"ON CONFLICT(image_id) DO UPDATE SET {self.vector_column}=excluded.{self.vector_column}")
        try:
            self._log_and_print(f"Writing {len(blobs)} vectors to DB...", level="info")
            cur.execute("BEGIN TRANSACTION;")
            cur.executemany(sql, blobs)
            self.write_conn.commit()
            self._log_and_print(f"Wrote {len(blobs)} vectors to DB.", level="info")
        except Exception as e:   # noqa: BLE001 - reference rolls back and logs
            self.write_conn.rollback()
            self._log_and_print(f"Write failed, rolled back: {e}", level="error")

    def batch_iterator(self):
        last_id = 0
        while True:
            rows = self.get_pending_rows(last_id)
            if not rows:
                break
            ids, paths = zip(*rows)
            yield ids, paths
            last_id = ids[-1]

    def run(self):
        total = self.read_conn.cursor().execute(
            f"SELECT COUNT(*) FROM images i LEFT JOIN {self.table_name} v ON i.id = v.image_id "
            f"WHERE v.{self.vector_column} IS NULL").fetchone()[0]
        self._log_and_print(f"Starting indexing for {total} images…", level="info")
        processed = 0
        for ids, paths in self.batch_iterator():
            self._log_and_print(f"Batch: IDs {ids[0]}–{ids[-1]}, {len(ids)} images", level="info")
            vectors = self.compute_vectors(list(paths))
            self.write_updates([(rid, vec) for rid, vec in zip(ids, vectors) if vec is not None])
            processed += len(ids)
            self._log_and_print(f"Progress: {processed}/{total}", level="info")
        self._log_and_print("Indexing finished.", level="info")
        self.read_conn.close()
        self.write_conn.close()


def load_image(img_path, img_size=None, gray=False, normalize=True, antialias=True,
               as_array=False):
    """PIL decode (create_vector_base.py:212-274, PIL branch).

    Returns a PIL image, or with as_array=True an HxWx3 (HxW for gray) uint8 array (float32,
    scaled to [0, 1] when normalize=True); None when the file is missing or unreadable."""
    from PIL import Image
    img_path = Path(img_path)
    if not img_path.exists():
        print(f"Image not found: {img_path}")
        return None
    try:
        img = Image.open(img_path)
        if img.mode == "P":
            img = img.convert("RGBA" if "transparency" in img.info else "RGB")
        img = img.convert("L" if gray else "RGB")
        if img_size is not None:
            img = img.resize(img_size, resample=Image.Resampling.LANCZOS if antialias
                             else Image.Resampling.NEAREST)
        if not as_array:
            return img
        arr = np.asarray(img)
        if normalize:
            return arr.astype(np.float32) / 255.0
        return np.ascontiguousarray(arr)
    except Exception as e:   # noqa: BLE001
        print(f"Error reading {img_path}: {e}")
        return None
