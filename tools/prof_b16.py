"""Epilogue breakdown of the 256 x 256 bf16 kernel from an -DIMGREC_B16_PROF build
(libimgrec_b16prof.so): cycles in the first tile's epilogue, the other tiles' epilogues, the
stage loops and the whole tile loop; insertion-loop iterations; blocks with a passing lane.
Usage: python tools/prof_b16.py [rows].  Debug tool, not part of the product.
"""
import ctypes as C
import os
import sys

os.environ.setdefault("IMGREC_LIB_NAME", "libimgrec_b16prof.so")
rows = sys.argv[1] if len(sys.argv) > 1 else "1000000"
sys.argv = [sys.argv[0], "--profile-only", "--steps", "1", "--warmup", "0", "--rows", rows]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from image_recommender_amd import _lib  # noqa: E402

lib = _lib.load()
lib.knn_debug_b16prof.restype = C.c_int
buf = (C.c_ulonglong * 8)()
lib.knn_debug_b16prof(buf)          # clear what loading/warm-up left
bench.main()
assert lib.knn_debug_b16prof(buf) == 0
tiles = buf[7] or 1
waves = 256 * 8
names = ["epilogue first tile", "epilogue other tiles", "kernel tile loop", "insert iters first",
         "insert iters other", "stage loops", "blocks with a pass", "tiles (x waves)"]
for n, v in zip(names, buf):
    print(f"{n:22s} {v:16d}  per wave {v / waves:12.1f}")
