"""TEST INFRASTRUCTURE ONLY — ctypes binding of the plain-C oracle (oracle/c/oracle_ref.c).

The C restatement is a second, independently written checker: a direct double-precision
sum((q - x)^2) scan with an insertion top-k (no BLAS, no |q|^2 + |x|^2 - 2 q.x expansion), where
oracle/flat_knn.py is a blocked numpy float64 GEMM form.  tests/test_oracle_c_cpu.py holds the two
against each other; the full-size cfg2 GPU test (tests/test_configs_gpu.py) checks its sampled
queries against both.  Built by oracle/c/Makefile into oracle/_build/liboracle.so (git-ignored;
__graft_entry__.build() runs the Makefile, and load() runs it when the library is missing).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB = _HERE / "_build" / "liboracle.so"
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(_HERE / "c")], check=True)
        lib = C.CDLL(str(LIB))
        lib.oracle_flat_search.restype = C.c_int
        lib.oracle_flat_search.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int,
                                           C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.oracle_color_counts.restype = C.c_int
        lib.oracle_color_counts.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
        _lib = lib
    return _lib


def flat_search(xb: np.ndarray, xq: np.ndarray, k: int, metric: str = "l2"):
    """Exact k-NN (faiss IndexFlat conventions, ties by smaller label) -> (D float64, I int64)."""
    if metric not in ("l2", "ip"):
        raise ValueError("the C oracle serves l2 and ip")
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), np.float64)
    I = np.empty((nq, k), np.int64)
    rc = load().oracle_flat_search(xb.ctypes.data, xb.shape[0], xq.ctypes.data, nq, d, int(k),
                                   1 if metric == "l2" else 0, D.ctypes.data, I.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_flat_search rc={rc}")
    return D, I


def color_counts(img: np.ndarray, bins: int = 16) -> np.ndarray:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    assert img.ndim == 3 and img.shape[2] == 3
    out = np.empty(3 * bins, np.int64)
    rc = load().oracle_color_counts(img.ctypes.data, img.shape[0] * img.shape[1], int(bins),
                                    out.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_color_counts rc={rc}")
    return out
