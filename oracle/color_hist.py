"""TEST INFRASTRUCTURE ONLY — the reference's colour feature restated in numpy.

/root/reference/vector_scripts/create_color_vector.py:46-51 (opencv-python 4.11.0.86, not
installed — parity against cv2 itself is unpinned): the image is RGB (BGR->RGB in load_image,
vector_scripts/create_vector_base.py:246-247) as float32 0..255 (normalize=False, :67-72);
per channel cv2.calcHist([c], [0], None, [bins], [0, 256]) -> a uniform histogram whose bin of an
integer value v is floor(v * bins / 256); channels concatenated R|G|B as float32; divided by
np.linalg.norm when that norm is non-zero.
"""
import numpy as np


def color_counts(img: np.ndarray, bins: int = 16) -> np.ndarray:
    """Integer bin counts, shape (3*bins,), for an HxWx3 uint8 RGB image."""
    img = np.asarray(img)
    assert img.ndim == 3 and img.shape[2] == 3 and img.dtype == np.uint8
    out = []
    for c in range(3):
        v = img[..., c].astype(np.int64).ravel()
        out.append(np.bincount((v * bins) >> 8, minlength=bins))
    return np.concatenate(out)


def color_hist_reference(img: np.ndarray, bins: int = 16) -> np.ndarray:
    vec = color_counts(img, bins).astype(np.float32)
    l2 = np.linalg.norm(vec)
    if l2 != 0:
        vec /= l2
    return vec
