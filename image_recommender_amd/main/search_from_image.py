"""Similarity search — drop-in for the reference's main.search_from_image.

Mirrors /root/reference/main/search_from_image.py (ImageRecommender, :17-428): same constructor
arguments (:18-28), the same per-type feature lookup with DB cache and raw-float32 fallback
(:50-125), canonical type order (:256-273), query assembly — parts concatenated per image, averaged
over query images, faiss.normalize_L2 (:275-324) — index file / offsets table naming (:326-344),
result mapping and distance sort (:346-379), and the reference's error convention (log and
return None, never raise, :235-252, :342-344).  The search itself runs on the exact MI355X index.

Deliberate changes:
* the index and its offset->image_id map are loaded once per process and kept resident
  (the reference re-reads the index file on every search, :339, and does k full-table scans of
  the offsets table per query, :361-376);
* when ``index_hnsw_<canonical>.faiss`` is absent, an index built from the same types in another
  order is used, with the query concatenated in that build order (read from the builder's
  ``.meta.json``), fixing the build/search order mismatch of Appendix C.1;
* ``search_similar_images`` also returns the result list it plots.
Colour features missing from the DB are computed by the HIP histogram kernel
(vector_scripts.create_color_vector); SIFT-VLAD and DreamSim features come from the DB cache (their
extractors need trained artefacts / pretrained weights that are not part of this path).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import pickle
import sqlite3
import sys
from pathlib import Path

import numpy as np

from .. import faiss_compat as faiss

os.environ.setdefault("KMP_DUPLICATE_LIB_OK", "TRUE")

CANONICAL_TYPES = ["color", "hog", "lpips", "dreamsim", "sift", "color_sift", "sift_dreamsim"]


class ImageRecommender:
    def __init__(
        self,
        images_root="image_data",
        db_path="images.db",
        use_gpu=True,
        sift_codebook_path="sift_codebook.npy",
        sift_pca_path="sift_vlad_pca.joblib",
        sift_n_clusters=256,
        sift_desc_dim=128,
        top_k=5,
        device=-1,
        index_dir=None,
    ):
        self.base_dir = Path().expanduser().resolve()
        self.images_root = (self.base_dir / images_root).resolve()
        self.db_path = Path(db_path).expanduser().resolve()
        self.use_gpu = use_gpu
        self.device = device
        self.index_dir = Path(index_dir) if index_dir else None
        self.sift_codebook_path = Path(sift_codebook_path).expanduser().resolve()
        self.sift_pca_path = Path(sift_pca_path).expanduser().resolve()
        self.sift_n_clusters = sift_n_clusters
        self.sift_desc_dim = sift_desc_dim
        self.top_k = top_k
        self._indexes: dict = {}       # canonical -> (index, offset_table, build_order, id_map)
        logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(message)s")

    # ---- DB cache (search_from_image.py:50-125) ------------------------------------------------
    def _get_db_vector(self, path_rel: str, vector_table: str, vector_column: str):
        conn = sqlite3.connect(self.db_path)
        cur = conn.cursor()
        cur.execute("SELECT id FROM images WHERE path = ?", (path_rel,))
        row = cur.fetchone()
        if not row:
            conn.close()
            return None
        cur.execute(f"SELECT {vector_column} FROM {vector_table} WHERE image_id = ?", (row[0],))
        vrow = cur.fetchone()
        conn.close()
        if vrow and vrow[0] is not None:
            blob = vrow[0]
            try:
                arr = pickle.loads(blob)
                if isinstance(arr, np.ndarray):
                    logging.info(f"Loaded '{vector_column}' from DB for '{path_rel}' "
                                 f"(shape: {arr.shape}) via pickle.")
                    return arr.reshape(1, -1) if arr.ndim == 1 else arr
            except Exception:   # noqa: BLE001 - reference falls back to raw float32 bytes
                pass
            if len(blob) % 4 != 0:
                logging.warning(f"Invalid BLOB size {len(blob)} bytes for '{vector_column}' at "
                                f"'{path_rel}', skipping cache.")
                return None
            arr = np.frombuffer(blob, dtype="float32").reshape(1, -1)
            logging.info(f"Loaded '{vector_column}' from DB for '{path_rel}' "
                         f"(shape: {arr.shape}) via raw bytes.")
            return arr
        return None

    def get_or_compute_vector(self, path_rel, vector_table, vector_column, compute_func,
                              reshape=None, print_vectors=False):
        cached = self._get_db_vector(path_rel, vector_table, vector_column)
        if cached is not None:
            if print_vectors:
                print(f"[DB-Vector]: {cached}")
            return cached
        vec = compute_func()
        if vec is None:
            logging.error(f"Failed to compute {vector_column} for '{path_rel}'.")
            return None
        if reshape is not None:
            vec = vec.reshape(*reshape)
        return vec

    def extract_color_features(self, path_rel: str):
        def compute():
            from ..vector_scripts.create_color_vector import ColorVectorIndexer
            return ColorVectorIndexer.compute_paths([path_rel], self.images_root)[0]
        return self.get_or_compute_vector(path_rel, "color_vectors", "color_vector_blob", compute,
                                          reshape=(1, -1))

    def extract_sift_vlad_features(self, path_rel: str):
        def compute():
            logging.error("SIFT-VLAD extraction needs the trained codebook/encoder of the "
                          "reference's vector_scripts/create_sift_vector.py; only DB-cached "
                          "SIFT vectors are served by this search path.")
            return None
        return self.get_or_compute_vector(path_rel, "sift_vectors", "sift_vector_blob", compute)

    def extract_dreamsim_features(self, path_rel: str):
        def compute():
            from ..vector_scripts.create_dreamsim_vector import DreamSimVectorIndexer
            if not hasattr(self, "_dreamsim_indexer"):
                self._dreamsim_indexer = DreamSimVectorIndexer(
                    db_path=str(self.db_path), base_dir=str(self.images_root), batch_size=4096,
                    model_batch=128, log_file="dreamsim_indexer.log", log_dir="logs")
            emb, valid = self._dreamsim_indexer._batch_image_to_vector([path_rel])
            if len(valid) == 1 and emb.shape[0] == 1:
                return emb[0].numpy().reshape(1, -1)
            return None
        return self.get_or_compute_vector(path_rel, "dreamsim_vectors", "dreamsim_vector_blob",
                                          compute)

    # ---- search (search_from_image.py:219-254) -------------------------------------------------
    def search_similar_images(self, query_image_paths, index_type: str = "color"):
        if isinstance(query_image_paths, (str, Path)):
            query_image_paths = [query_image_paths]
        paths_rel = [Path(p).resolve().relative_to(self.images_root).as_posix()
                     for p in query_image_paths]
        ordered = self._get_ordered_index_types(index_type)
        if not ordered:
            return None
        canonical = "_".join(ordered)
        loaded = self._load_faiss_index(canonical, ordered)
        if loaded is None:
            return None
        index, offset_table, build_order, id_map = loaded
        query_vec = self._extract_query_vector(paths_rel, build_order)
        if query_vec is None:
            return None
        distances, indices = index.search(query_vec, self.top_k)
        results = self._fetch_results(indices, distances, offset_table, id_map)
        if not results:
            logging.error("No similar images found.")
            return None
        self._plot_results(query_image_paths, results)
        return results

    def _get_ordered_index_types(self, index_type: str):
        requested = [x.strip() for x in index_type.lower().split(",")]
        ordered = [v for v in CANONICAL_TYPES if v in requested]
        if not ordered:
            logging.error(f"Unknown index_type '{index_type}'. Choose from {CANONICAL_TYPES}.")
            return []
        logging.info(f"Extracting features in order: {ordered}")
        return ordered

    def _extract_query_vector(self, paths_rel, ordered):
        all_query_vectors = []
        for path_rel in paths_rel:
            logging.info(f"Extracting vector for query image: '{path_rel}'")
            parts = []
            for vec_type in ordered:
                if vec_type == "color":
                    parts.append(self.extract_color_features(path_rel))
                elif vec_type == "sift":
                    parts.append(self.extract_sift_vlad_features(path_rel))
                elif vec_type == "dreamsim":
                    parts.append(self.extract_dreamsim_features(path_rel))
                else:
                    logging.error(f"Unknown vector type '{vec_type}' for '{path_rel}'.")
                    return None
            if any(p is None for p in parts):
                logging.error(f"Could not compute all vector features for '{path_rel}', "
                              f"skipping this image.")
                continue
            if len(parts) == 1:
                full_vec = parts[0].astype("float32")
            else:
                parts = [x.reshape(1, -1) if x.ndim == 1 else x for x in parts]
                full_vec = np.concatenate(parts, axis=1).astype("float32")
            all_query_vectors.append(full_vec)
        if not all_query_vectors:
            logging.error("Could not extract a vector for any of the query images.")
            return None
        combined = np.mean(all_query_vectors, axis=0)
        if combined.ndim == 1:
            combined = combined.reshape(1, -1)
        combined = np.ascontiguousarray(combined, dtype=np.float32)
        faiss.normalize_L2(combined)
        return combined

    def _index_path(self, name: str) -> Path:
        return (self.index_dir / name) if self.index_dir else Path(name)

    def _load_faiss_index(self, canonical, ordered=None):
        """Resident index for a canonical type combination (loaded once per process).

        Returns (index, offset_table, build_order, offset->image_id array) or None."""
        if canonical in self._indexes:
            return self._indexes[canonical]
        types = list(ordered) if ordered else [canonical]
        candidates = [canonical]
        if len(types) > 1:       # an index built in another order of the same types
            import itertools
            candidates += ["_".join(p) for p in itertools.permutations(types) if list(p) != types]
        for name in candidates:
            f = self._index_path(f"index_hnsw_{name}.faiss")
            if not f.exists():
                continue
            try:
                index = faiss.read_index(str(f), device=self.device)
            except Exception as e:   # noqa: BLE001 - reference logs and returns None
                logging.error(f"Error loading index '{f}': {e}")
                return None
            meta_f = Path(str(f) + ".meta.json")
            build_order = list(types)
            if name != canonical:     # a permutation: which one
                import itertools
                for p in itertools.permutations(types):
                    if "_".join(p) == name:
                        build_order = list(p)
                        break
            if meta_f.exists():
                build_order = json.loads(meta_f.read_text()).get("vector_types", build_order)
            offset_table = f"faiss_index_offsets_{name}"
            id_map = self._load_offsets(offset_table, index.ntotal)
            logging.info(f"Loaded index '{f}' with {index.ntotal} vectors (build order "
                         f"{build_order}).")
            self._indexes[canonical] = (index, offset_table, build_order, id_map)
            return self._indexes[canonical]
        logging.error(f"Error loading index 'index_hnsw_{canonical}.faiss': file not found")
        return None

    def _load_offsets(self, offset_table, ntotal):
        """offset -> image_id as one int64 array (-1 where the table has no entry)."""
        id_map = np.full(ntotal, -1, np.int64)
        try:
            conn = sqlite3.connect(self.db_path)
            for image_id, off in conn.execute(f"SELECT image_id, offset FROM {offset_table}"):
                if off is not None and 0 <= off < ntotal:
                    id_map[off] = image_id
            conn.close()
        except sqlite3.Error as e:
            logging.error(f"Could not read {offset_table}: {e}")
        return id_map

    def _fetch_results(self, indices, distances, offset_table, id_map=None):
        if id_map is None:
            id_map = self._load_offsets(offset_table, int(np.max(indices)) + 1)
        conn = sqlite3.connect(self.db_path)
        cur = conn.cursor()
        results = []
        for rank, offset in enumerate(indices[0]):
            offset = int(offset)
            img_id = int(id_map[offset]) if 0 <= offset < len(id_map) else -1
            if img_id < 0:
                logging.warning(f"No entry found for offset={offset} in {offset_table}")
                continue
            cur.execute("SELECT path FROM images WHERE id = ?", (img_id,))
            fp_row = cur.fetchone()
            if not fp_row:
                logging.warning(f"No path found for id={img_id}")
                continue
            results.append((Path(self.base_dir) / fp_row[0], float(distances[0, rank])))
        conn.close()
        results.sort(key=lambda x: x[1])
        return results

    def _plot_results(self, query_image_paths, results):
        """Display query and results (main/search_from_image.py:381-428); needs matplotlib."""
        try:
            import matplotlib.pyplot as plt
            from PIL import Image
        except Exception as e:   # noqa: BLE001
            logging.error(f"Plotting unavailable: {e}")
            return
        n_q = len(query_image_paths)
        total = n_q + len(results)
        ncols = max(4, n_q)
        nrows = int(np.ceil(total / ncols))
        fig, axes = plt.subplots(nrows, ncols, figsize=(5 * ncols, 5 * nrows))
        axes = np.asarray(axes).reshape(-1)
        items = [(p, f"Query: {Path(p).name}") for p in query_image_paths] + \
                [(fp, f"{Path(fp).name}\nDist: {d:.4f}") for fp, d in results]
        for ax, (p, title) in zip(axes, items):
            try:
                ax.imshow(Image.open(p).convert("RGB"))
                ax.set_title(title)
            except Exception as e:   # noqa: BLE001
                logging.error(f"Error rendering {p}: {e}")
            ax.axis("off")
        for ax in axes[total:]:
            ax.axis("off")
        plt.tight_layout(pad=2.0, h_pad=3.0)
        plt.show()


def main(argv=None):
    ap = argparse.ArgumentParser(description="Search similar images on the MI355X index")
    ap.add_argument("--db-path", default="images.db")
    ap.add_argument("--images-root", default="image_data")
    ap.add_argument("--query", nargs="+", required=True)
    ap.add_argument("--index", default="color", help="comma-separated types, e.g. color,dreamsim")
    ap.add_argument("--top-k", type=int, default=5)
    ap.add_argument("--no-plot", action="store_true")
    a = ap.parse_args(argv)
    idx = a.index[len("combo_"):] if a.index.startswith("combo_") else a.index
    rec = ImageRecommender(images_root=a.images_root, db_path=a.db_path, top_k=a.top_k)
    if a.no_plot:
        rec._plot_results = lambda *args, **kw: None
    res = rec.search_similar_images(a.query, index_type=idx.replace("_", ","))
    for p, d in res or []:
        print(f"{d:.6f}\t{p}")
    return 0 if res else 1


if __name__ == "__main__":
    sys.exit(main())
