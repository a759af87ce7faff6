"""Generate tests/golden/plumbing.json by running the REFERENCE's own index/search plumbing.

Runs only in the build container, where /root/reference exists: the
reference's main/create_index.py and main/search_from_image.py are imported with stub modules for
the packages the image lacks (faiss, seaborn, cv2, dreamsim).  The faiss stub is an exact float64
flat index (oracle.flat_knn.search_exact) that also records every matrix passed to add(), so the
fixture pins the reference's plumbing — SQL joins, BLOB decoding, part concatenation order, offset
bookkeeping, canonical search order, query averaging + normalisation, result mapping and sorting —
independently of faiss's approximate arithmetic.  Nothing of the reference is copied: the fixture
holds only inputs (a seeded DB recipe) and the outputs the reference produced.

Usage (from the repo root):  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import pickle
import sqlite3
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "plumbing.json"

from oracle.flat_knn import search_exact  # noqa: E402

# ---- the seeded DB recipe (tests rebuild exactly this DB) -----------------------------------
DIMS = {"color": 48, "sift": 128, "dreamsim": 1792}
N_IMAGES = 40
SEED = 1234


def build_db(db_path: Path) -> dict:
    """Schema of main/create_db.py:49-86; pickled float32 BLOBs as create_vector_base.py:144."""
    rng = np.random.default_rng(SEED)
    con = sqlite3.connect(db_path)
    c = con.cursor()
    c.execute("CREATE TABLE images (id INTEGER PRIMARY KEY AUTOINCREMENT, path TEXT UNIQUE)")
    for t in DIMS:
        c.execute(f"CREATE TABLE {t}_vectors (image_id INTEGER PRIMARY KEY, {t}_vector_blob BLOB, "
                  f"FOREIGN KEY(image_id) REFERENCES images(id) ON DELETE CASCADE)")
    paths = [f"image_data/set{i % 3}/{i:04d}.png" for i in range(N_IMAGES)]
    c.executemany("INSERT INTO images (path) VALUES (?)", [(p,) for p in paths])
    missing = {"color": {5}, "sift": {7, 21}, "dreamsim": {13}}
    broken = {"dreamsim": {30}}
    vectors = {}
    for t, d in DIMS.items():
        centres = rng.standard_normal((4, d))
        rows = []
        for i in range(N_IMAGES):
            v = centres[i % 4] + 0.3 * rng.standard_normal(d)
            v = (np.abs(v) if t == "color" else v)
            v = (v / np.linalg.norm(v)).astype(np.float32)
            vectors.setdefault(t, {})[i + 1] = v
            if i in missing[t]:
                continue
            blob = pickle.dumps(v, protocol=pickle.HIGHEST_PROTOCOL)
            if i in broken.get(t, ()):
                blob = b"not a pickle"
            rows.append((i + 1, sqlite3.Binary(blob)))
        c.executemany(f"INSERT INTO {t}_vectors (image_id, {t}_vector_blob) VALUES (?, ?)", rows)
    con.commit()
    con.close()
    return {"paths": paths, "missing": {k: sorted(v) for k, v in missing.items()},
            "broken": {k: sorted(v) for k, v in broken.items()}}


# ---- stubs -----------------------------------------------------------------------------------
class _StubIndex:
    """Exact float64 flat L2 index standing in for faiss.IndexHNSWFlat / IndexIVFPQ."""

    def __init__(self, d, *a, **kw):
        self.d = d
        self.hnsw = types.SimpleNamespace(efConstruction=None, efSearch=None)
        self.is_trained = False
        self.xb = np.zeros((0, d), np.float32)
        self.added = []

    def train(self, x):
        self.is_trained = True

    def add(self, x):
        x = np.asarray(x, np.float32)
        self.added.append(x.copy())
        self.xb = np.concatenate([self.xb, x])

    @property
    def ntotal(self):
        return self.xb.shape[0]

    def search(self, q, k):
        D, I = search_exact(self.xb, np.asarray(q, np.float32), k, "l2")
        return D.astype(np.float32), I


_FILES: dict = {}
_LOG: dict = {"normalize_calls": []}


def _install_stubs():
    faiss = types.ModuleType("faiss")
    faiss.IndexHNSWFlat = lambda d, M: _StubIndex(d)
    faiss.IndexIVFPQ = lambda q, d, nlist, m, nbits: _StubIndex(d)

    def write_index(index, fname):
        _FILES[os.path.basename(fname)] = index
        Path(fname).write_bytes(b"stub")

    def read_index(fname):
        if os.path.basename(fname) not in _FILES:
            raise RuntimeError(f"read_index: {fname} not found")
        return _FILES[os.path.basename(fname)]

    def normalize_L2(x):
        _LOG["normalize_calls"].append(np.array(x, copy=True).tolist())
        n = np.linalg.norm(x, axis=1, keepdims=True)
        np.divide(x, n, out=x, where=n > 0)

    faiss.write_index, faiss.read_index, faiss.normalize_L2 = write_index, read_index, normalize_L2
    sys.modules["faiss"] = faiss
    for name in ("seaborn", "cv2", "dreamsim"):
        sys.modules[name] = types.ModuleType(name)

    def _no_dreamsim(*a, **kw):
        raise RuntimeError("dreamsim weights are not available offline")

    sys.modules["dreamsim"].dreamsim = _no_dreamsim
    sys.path.insert(0, str(REF))


def _digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def main():
    if not REF.exists():
        sys.exit("the reference checkout is only available in the build container")
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    _install_stubs()
    work = Path(tempfile.mkdtemp(prefix="golden_"))
    os.chdir(work)
    recipe = build_db(work / "images.db")
    from main.create_index import FAISSIndexBuilderDB          # the reference's module
    from main.search_from_image import ImageRecommender        # the reference's module

    fixture = {"recipe": {"dims": DIMS, "n_images": N_IMAGES, "seed": SEED, **recipe},
               "builds": {}, "searches": [], "ordered_types": {}}
    combos = [["color"], ["dreamsim"], ["color", "dreamsim"], ["color", "sift", "dreamsim"],
              ["color", "dreamsim", "sift"]]
    for combo in combos:
        b = FAISSIndexBuilderDB(db_path="images.db", vector_types=list(combo), batch_size=7,
                                log_dir=str(work / "logs"))
        b.build_index(update_index=False)
        name = "_".join(combo)
        con = sqlite3.connect("images.db")
        offs = con.execute(f"SELECT image_id, offset FROM faiss_index_offsets_{name} "
                           f"ORDER BY image_id").fetchall()
        con.close()
        idx = _FILES[f"index_hnsw_{name}.faiss"]
        fixture["builds"][name] = {
            "index_file": f"index_hnsw_{name}.faiss", "offset_table": f"faiss_index_offsets_{name}",
            "offsets": offs, "ntotal": idx.ntotal, "dim": idx.d,
            "add_batches": [a.shape[0] for a in idx.added], "matrix_sha256": _digest(idx.xb),
            "first_row_head": idx.xb[0, :4].tolist(),
        }
    rec = ImageRecommender(images_root=".", db_path="images.db", top_k=5)
    captured = {}
    rec._plot_results = lambda paths, results: captured.__setitem__("r", results)
    for s in ["color", "dreamsim", "color,dreamsim", "dreamsim,color", "sift,color,dreamsim",
              "COLOR, Dreamsim", "bogus"]:
        fixture["ordered_types"][s] = rec._get_ordered_index_types(s)
    queries = [(["image_data/set0/0000.png"], "color"),
               (["image_data/set1/0001.png"], "dreamsim"),
               (["image_data/set2/0002.png", "image_data/set0/0003.png"], "color,dreamsim"),
               (["image_data/set1/0004.png"], "color,dreamsim"),
               (["image_data/set2/0005.png"], "color"),                  # image lacking colour
               (["image_data/set1/0013.png", "image_data/set0/0009.png"], "color,dreamsim"),
               (["image_data/set0/0006.png"], "color,sift,dreamsim")]   # canonical-order file
    for paths, itype in queries:
        captured.clear()
        _LOG["normalize_calls"].clear()
        err = None
        try:
            rec.search_similar_images([str(work / p) for p in paths], index_type=itype)
        except Exception as e:          # e.g. a DreamSim cache miss without the model
            err = type(e).__name__
        res = captured.get("r")
        fixture["searches"].append({
            "paths": paths, "index_type": itype,
            "query_vector": _LOG["normalize_calls"][0] if _LOG["normalize_calls"] else None,
            "results": None if res is None else [[str(Path(p).relative_to(work)), float(d)] for p, d in res],
            "error": err,
        })
    OUT.write_text(json.dumps(fixture, indent=1))
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


if __name__ == "__main__":
    main()
