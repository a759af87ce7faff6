"""End-to-end GPU tests of the drop-in modules against outputs of the REFERENCE's own plumbing
(tests/golden/plumbing.json): index build (offsets table, stored matrix) and search results
(paths, order, distances within the fp32 bound), plus the colour-histogram kernel vs the oracle.
"""
import hashlib
import json
import sqlite3
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import build_db

pytestmark = pytest.mark.gpu
GOLDEN = json.loads((Path(__file__).parent / "golden" / "plumbing.json").read_text())


@pytest.fixture()
def built(gpu, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    build_db(tmp_path / "images.db")
    from image_recommender_amd.main.create_index import FAISSIndexBuilderDB
    idx = {}
    for name, g in GOLDEN["builds"].items():
        types = g["index_file"][len("index_hnsw_"):-len(".faiss")].split("_")
        b = FAISSIndexBuilderDB(db_path="images.db", vector_types=types, batch_size=7,
                                log_dir=str(tmp_path / "logs"))
        idx[name] = b.build_index()
    return tmp_path, idx


def test_build_matches_reference(built):
    tmp, idx = built
    con = sqlite3.connect(tmp / "images.db")
    for name, g in GOLDEN["builds"].items():
        offs = con.execute(f"SELECT image_id, offset FROM {g['offset_table']} ORDER BY image_id").fetchall()
        assert [list(o) for o in offs] == g["offsets"]
        assert (tmp / g["index_file"]).exists()
        assert idx[name].ntotal == g["ntotal"] and idx[name].d == g["dim"]
        mat = idx[name].reconstruct_n(0, g["ntotal"])
        assert hashlib.sha256(mat.tobytes()).hexdigest() == g["matrix_sha256"]
        meta = json.loads((tmp / (g["index_file"] + ".meta.json")).read_text())
        assert "_".join(meta["vector_types"]) == name


def test_search_matches_reference(built):
    tmp, _ = built
    from image_recommender_amd.main.search_from_image import ImageRecommender
    rec = ImageRecommender(images_root=".", db_path=str(tmp / "images.db"), top_k=5)
    rec._plot_results = lambda *a, **k: None
    for s in GOLDEN["searches"]:
        paths = [str(tmp / p) for p in s["paths"]]
        if s["error"]:
            with pytest.raises(RuntimeError):
                rec.search_similar_images(paths, index_type=s["index_type"])
            continue
        res = rec.search_similar_images(paths, index_type=s["index_type"])
        if s["results"] is None:
            assert res is None
            continue
        got = [(str(Path(p).relative_to(tmp)), d) for p, d in res]
        want = s["results"]
        assert len(got) == len(want)
        gd = np.array([d for _, d in got])
        wd = np.array([d for _, d in want])
        # the empirical window of tests/knn_check.check_knn_tight: 8 x this build's measured
        # |fp32 - float64| distance error, at least 1e-6 of the key scale, with that error first
        # held below 32 unit roundoffs of the key's term scale (|q|^2 + |x|^2 <= 1 + 3: the query
        # is normalised, a stored row has at most three unit-norm parts)
        err = float(np.abs(gd - wd).max())
        assert err <= 32 * 2.0 ** -24 * 4.0, (s["paths"], err)
        w = max(8.0 * err, 1e-6 * float(np.abs(wd).max()))
        for j, ((gp, g_d), (wp, w_d)) in enumerate(zip(got, want)):
            lo = j == 0 or abs(wd[j] - wd[j - 1]) > w
            hi = j + 1 >= len(wd) or abs(wd[j + 1] - wd[j]) > w
            if lo and hi:
                assert gp == wp, (s["paths"], j, got, want, w)      # integer-exact label
            else:            # inside a tie window: the label is one of the window's labels
                assert any(abs(w_d - d2) <= w and p2 == gp for p2, d2 in want), (gp, wp, w)


def test_index_resident_across_searches(built):
    tmp, _ = built
    from image_recommender_amd.main.search_from_image import ImageRecommender
    rec = ImageRecommender(images_root=".", db_path=str(tmp / "images.db"), top_k=3)
    rec._plot_results = lambda *a, **k: None
    r1 = rec.search_similar_images([str(tmp / "image_data/set0/0000.png")], "color")
    loaded = rec._indexes["color"][0]
    r2 = rec.search_similar_images([str(tmp / "image_data/set0/0000.png")], "color")
    assert rec._indexes["color"][0] is loaded and r1 == r2


def test_build_order_mismatch_fixed(built):
    """Appendix C.1: an index built as color,sift,dreamsim is searched with the query
    concatenated in THAT order when only that file exists."""
    tmp, _ = built
    (tmp / "index_hnsw_color_dreamsim_sift.faiss").unlink()
    (tmp / "index_hnsw_color_dreamsim_sift.faiss.meta.json").unlink()
    from image_recommender_amd.main.search_from_image import ImageRecommender
    rec = ImageRecommender(images_root=".", db_path=str(tmp / "images.db"), top_k=3)
    rec._plot_results = lambda *a, **k: None
    res = rec.search_similar_images([str(tmp / "image_data/set0/0006.png")], "sift,dreamsim,color")
    assert res is not None and Path(res[0][0]).name == "0006.png"
    assert rec._indexes["color_dreamsim_sift"][2] == ["color", "sift", "dreamsim"]
    assert res[0][1] == pytest.approx(4 - 2 * np.sqrt(3), abs=2e-5)   # self match, P = 3


# ---- colour histogram (vector_scripts/create_color_vector.py:46-51) ---------------------------
@pytest.mark.parametrize("bins", [16, 8, 32, 1, 7])
def test_color_histogram_kernel(gpu, bins):
    from image_recommender_amd.vector_scripts.create_color_vector import color_histograms
    from oracle.color_hist import color_counts, color_hist_reference
    rng = np.random.default_rng(bins)
    shapes = [(1, 1), (3, 5), (17, 33), (256, 256), (480, 640), (31, 7), (2, 2)]
    imgs = [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in shapes]
    imgs.append(np.full((100, 120, 3), 200, np.uint8))             # one bin per channel
    imgs.append(np.zeros((0, 4, 3), np.uint8))                      # empty image
    grad = np.linspace(0, 255, 300 * 400).reshape(300, 400).astype(np.uint8)
    imgs.append(np.stack([grad, grad[::-1], 255 - grad], -1))
    out, counts = color_histograms(imgs, bins=bins, return_counts=True)
    for im, h, c in zip(imgs, out, counts):
        np.testing.assert_array_equal(c, color_counts(im, bins))
        np.testing.assert_allclose(h, color_hist_reference(im, bins), rtol=1e-6, atol=1e-9)


def test_color_indexer_on_png_files(gpu, tmp_path, monkeypatch):
    from PIL import Image
    monkeypatch.chdir(tmp_path)
    from image_recommender_amd.main.create_db import ImageDBCreator
    from image_recommender_amd.vector_scripts.create_color_vector import ColorVectorIndexer
    from oracle.color_hist import color_hist_reference
    rng = np.random.default_rng(3)
    folder = tmp_path / "image_data" / "a"
    folder.mkdir(parents=True)
    arrays = {}
    for i in range(6):
        a = rng.integers(0, 256, (20 + i, 30 + 2 * i, 3), dtype=np.uint8)
        Image.fromarray(a).save(folder / f"{i}.png")
        arrays[f"image_data/a/{i}.png"] = a
    (folder / "broken.png").write_bytes(b"not an image")
    ImageDBCreator("images.db", "image_data").process_batches()
    ColorVectorIndexer("images.db", tmp_path, log_dir=str(tmp_path / "logs"), install_sigint=False).run()
    con = sqlite3.connect("images.db")
    import pickle
    rows = con.execute("SELECT i.path, c.color_vector_blob FROM images i JOIN color_vectors c "
                       "ON i.id = c.image_id").fetchall()
    assert sorted(p for p, _ in rows) == sorted(arrays)
    for p, blob in rows:
        np.testing.assert_allclose(pickle.loads(blob), color_hist_reference(arrays[p]), rtol=1e-6)


def test_dreamsim_ensemble_shapes(gpu, tmp_path):
    from image_recommender_amd.vector_scripts import create_dreamsim_vector as ds
    import sqlite3 as sq
    db = tmp_path / "x.db"
    from image_recommender_amd.main.create_db import create_schema
    create_schema(sq.connect(db))
    with pytest.raises(RuntimeError):
        ds.DreamSimVectorIndexer(str(db), str(tmp_path), log_dir=str(tmp_path / "l"))
    ix = ds.DreamSimVectorIndexer(str(db), str(tmp_path), log_dir=str(tmp_path / "l"),
                                  allow_random_init=True)
    import torch
    x = torch.rand(3, 3, 224, 224, device=ix.device)
    e = ix.embed_tensor(x)
    assert e.shape == (3, 1792)
    torch.testing.assert_close(e.norm(dim=1), torch.ones(3, device=e.device), rtol=1e-5, atol=1e-5)


def test_color_histogram_fixed_bins_alignments(gpu):
    """bins = 16 (cv2's default here) runs the 48-byte-granule kernel: images packed back to back
    so their first bytes take every 16-B alignment and every channel phase of the granules, plus
    images shorter than one granule; counts exact against the oracle."""
    from image_recommender_amd.vector_scripts.create_color_vector import color_histograms
    from oracle.color_hist import color_counts, color_hist_reference
    rng = np.random.default_rng(77)
    imgs = [rng.integers(0, 256, (37 + (w % 5), w, 3), dtype=np.uint8) for w in range(1, 49)]
    imgs += [rng.integers(0, 256, (1, w, 3), dtype=np.uint8) for w in range(1, 20)]
    skew = rng.integers(0, 256, (512, 517, 3), dtype=np.uint8)
    skew[..., 1] = 17                                                 # one channel in one bin
    imgs.append(skew)
    out, counts = color_histograms(imgs, bins=16, return_counts=True)
    for im, h, c in zip(imgs, out, counts):
        np.testing.assert_array_equal(c, color_counts(im, 16))
        np.testing.assert_allclose(h, color_hist_reference(im, 16), rtol=1e-6, atol=1e-9)


def test_color_histogram_large_image(gpu):
    """An 18 MB image: more bytes per thread than a 16-bit counter holds (the fixed-bin kernel
    built with 16-bit counters folds its columns between chunks); counts exact."""
    from image_recommender_amd.vector_scripts.create_color_vector import color_histograms
    from oracle.color_hist import color_counts
    rng = np.random.default_rng(78)
    big = rng.integers(0, 256, (2500, 2400, 3), dtype=np.uint8)
    big[:1200, :, 0] = 3                                              # a heavily skewed channel
    out, counts = color_histograms([big, big[:1, :5]], bins=16, return_counts=True)
    np.testing.assert_array_equal(counts[0], color_counts(big, 16))
    np.testing.assert_array_equal(counts[1], color_counts(big[:1, :5], 16))


@pytest.mark.gpu
def test_color_histogram_constant_images(gpu):
    """Register (SWAR) counting of the 16-bin kernel: every byte of a channel in ONE bin (the
    4-bit and 8-bit packed counters at their limits, bin 15 = the top nibble of the u64, bin 0)
    over many flushes, and a gradient through every bin; counts exact against the oracle."""
    from image_recommender_amd.vector_scripts.create_color_vector import color_histograms
    from oracle.color_hist import color_counts
    imgs = []
    for rgb in ((255, 0, 128), (0, 255, 15), (16, 31, 240)):
        im = np.empty((700, 701, 3), dtype=np.uint8)
        im[...] = np.array(rgb, dtype=np.uint8)
        imgs.append(im)
    grad = np.arange(300 * 256 * 3, dtype=np.int64).reshape(300, 256, 3) % 256
    imgs.append(grad.astype(np.uint8))
    out, counts = color_histograms(imgs, bins=16, return_counts=True)
    for im, c in zip(imgs, counts):
        np.testing.assert_array_equal(c, color_counts(im, 16))
