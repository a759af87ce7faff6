"""The colour feature from image FILES: decode workers -> page-locked
shared-memory ring -> async DMA -> HIP histogram (vector_scripts/decode_pipeline.py).

Checked against the integer oracle (oracle/color_hist.py, the restatement of
/root/reference/vector_scripts/create_color_vector.py:46-51) on the same decoder's pixels: JPEG and
PNG files, a grayscale file (converted to RGB like cv2.IMREAD_COLOR), an unreadable file (None, as
the reference's worker returns), odd sizes, and an image larger than a ring slot (host spill).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(path):
    from image_recommender_amd.vector_scripts.create_vector_base import load_image
    from oracle.color_hist import color_counts, color_hist_reference
    img = load_image(path, normalize=False, as_array=True)
    return color_counts(img, 16), color_hist_reference(img, 16)


def test_pipeline_counts_equal_oracle(gpu, tmp_path):
    from PIL import Image
    from image_recommender_amd.vector_scripts.decode_pipeline import (ColorDecodePipeline,
                                                                      write_synthetic_images)
    paths = write_synthetic_images(tmp_path / "jpg", 300, size=256, fmt="jpg", workers=4)
    paths += write_synthetic_images(tmp_path / "png", 40, size=97, fmt="png", seed=7, workers=4)
    rng = np.random.default_rng(3)
    gray = tmp_path / "gray.png"
    Image.fromarray(rng.integers(0, 256, (33, 45), dtype=np.uint8), "L").save(gray)
    bad = tmp_path / "broken.jpg"
    bad.write_bytes(b"\xff\xd8\xff not really a jpeg")
    big = tmp_path / "big.png"                        # 2600 x 2600 x 3 = 20 MB > one 16 MB slot
    Image.fromarray(rng.integers(0, 256, (2600, 2600, 3), dtype=np.uint8), "RGB").save(big)
    paths = paths[:150] + [gray, bad] + paths[150:] + [big, tmp_path / "missing.png"]
    with ColorDecodePipeline(workers=4, chunk=32) as pipe:
        vecs, counts = pipe.histograms(paths, return_counts=True)
        again = pipe.histograms(paths[:70])           # the ring is reusable
    assert vecs[150] is not None and vecs[151] is None and vecs[-1] is None
    for i, p in enumerate(paths):
        if vecs[i] is None:
            continue
        c_ref, v_ref = _oracle(p)
        np.testing.assert_array_equal(counts[i], c_ref)
        np.testing.assert_allclose(vecs[i], v_ref, rtol=1e-6, atol=1e-7)
    for a, b in zip(again, vecs[:70]):
        np.testing.assert_array_equal(a, b)


def test_color_indexer_batch_path_uses_pipeline(gpu, tmp_path):
    """ColorVectorIndexer.compute_vectors (the reference's batch entry point,
    create_color_vector.py:54-78) returns the oracle's vectors for relative paths."""
    from image_recommender_amd.vector_scripts.create_color_vector import ColorVectorIndexer
    from image_recommender_amd.vector_scripts.decode_pipeline import write_synthetic_images
    paths = write_synthetic_images(tmp_path / "image_data", 50, size=64, fmt="jpg", workers=2)
    idx = ColorVectorIndexer.__new__(ColorVectorIndexer)        # no DB needed for this call
    idx.base_dir = tmp_path
    idx.bins = 16
    rel = [str(p.relative_to(tmp_path)) for p in paths]
    vecs = idx.compute_vectors(rel)
    idx._pipeline.close()
    for p, v in zip(paths, vecs):
        np.testing.assert_allclose(v, _oracle(p)[1], rtol=1e-6, atol=1e-7)
