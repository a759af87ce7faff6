"""Seeded synthetic embeddings shaped like the reference's vector tables (test helper).

Rows are Gaussian-mixture samples (clustered, so neighbour sets are meaningful rather than the
distance concentration of iid high-dimensional noise).  `concat_rows` builds the
(color 48 | SIFT 128 | DreamSim 1792) layout of SURVEY.md §8d config 3, each part unit-norm.
"""
import numpy as np


def mixture(n, d, centres=50, sigma=0.5, seed=0, normalize=False, dtype=np.float32):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((centres, d))
    x = c[rng.integers(0, centres, n)] + sigma * rng.standard_normal((n, d))
    if normalize:
        x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(dtype)


def concat_rows(n, seed=3, dims=(48, 128, 1792), centres=64):
    rng = np.random.default_rng(seed)
    parts = []
    for i, d in enumerate(dims):
        if i == 0:
            p = np.abs(rng.standard_normal((n, d)))
        else:
            c = rng.standard_normal((centres, d))
            p = c[rng.integers(0, centres, n)] + 0.5 * rng.standard_normal((n, d))
        p /= np.linalg.norm(p, axis=1, keepdims=True)
        parts.append(p)
    return np.concatenate(parts, 1).astype(np.float32)
