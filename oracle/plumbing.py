"""TEST INFRASTRUCTURE ONLY — the reference's index/search plumbing restated.

Pinned by tests/golden/plumbing.json (captured from the reference's own modules by
tests/golden/make_golden.py).
"""
from __future__ import annotations

import pickle
import sqlite3

import numpy as np

# /root/reference/main/search_from_image.py:267
CANONICAL = ["color", "hog", "lpips", "dreamsim", "sift", "color_sift", "sift_dreamsim"]


def ordered_index_types(index_type: str) -> list[str]:
    """main/search_from_image.py:256-273."""
    requested = [x.strip() for x in index_type.lower().split(",")]
    return [v for v in CANONICAL if v in requested]


def find_valid_m(dim: int, candidates=(64, 56, 48, 32, 28, 24, 16, 12, 8)) -> int:
    """main/create_index.py:191-205."""
    for m in candidates:
        if dim % m == 0:
            return m
    return 1


def index_names(vector_types) -> tuple[str, str]:
    """main/create_index.py:36-37, 43: (index file, offsets table)."""
    name = "_".join(vector_types)
    return f"index_hnsw_{name}.faiss", f"faiss_index_offsets_{name}"


def build_rows(db_path: str, vector_types):
    """The builder's scan (main/create_index.py:115-189): (ids, matrix) of rows that have every
    part and whose BLOBs unpickle, parts concatenated in caller order, ascending image id."""
    con = sqlite3.connect(db_path)
    sel = ", ".join(["i.id"] + [f"t{k}.{t}_vector_blob" for k, t in enumerate(vector_types)])
    joins = " ".join(f"JOIN {t}_vectors t{k} ON i.id = t{k}.image_id"
                     for k, t in enumerate(vector_types))
    ids, rows = [], []
    for rec_id, *blobs in con.execute(f"SELECT {sel} FROM images i {joins} ORDER BY i.id"):
        try:
            parts = [np.asarray(pickle.loads(b), dtype="float32").ravel() for b in blobs]
        except Exception:   # noqa: BLE001 - skipped row, as the reference
            continue
        ids.append(rec_id)
        rows.append(np.concatenate(parts))
    con.close()
    return ids, (np.stack(rows) if rows else np.zeros((0, 0), np.float32))


def assemble_query(per_image_parts) -> np.ndarray:
    """main/search_from_image.py:286-317 before normalize_L2: per image the (1, d_i) parts in
    canonical order concatenated; images with a missing part skipped; mean over images."""
    vecs = []
    for parts in per_image_parts:
        if any(p is None for p in parts):
            continue
        parts = [np.asarray(p).reshape(1, -1) for p in parts]
        vecs.append(np.concatenate(parts, axis=1).astype("float32") if len(parts) > 1
                    else parts[0].astype("float32"))
    if not vecs:
        return None
    q = np.mean(vecs, axis=0)
    return q.reshape(1, -1) if q.ndim == 1 else q
