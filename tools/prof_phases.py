"""Phase breakdown of the fused kernel from an -DIMGREC_PROF build (libimgrec_prof.so).

Runs the bench workload (1M x 1968, 1024 queries) in the given mode and prints, per wave, the
s_memtime cycles spent in: DMA wait, stage barrier, fragment reads + DMA issue, MFMA issue,
epilogue barrier, epilogue work, and the whole tile loop.  Debug tool, not part of the product.
"""
import ctypes as C
import os
import sys

os.environ["IMGREC_LIB_NAME"] = "libimgrec_prof.so"
sys.argv = [sys.argv[0], "--profile-only", "--steps", "2", "--warmup", "1", "--mode",
            sys.argv[1] if len(sys.argv) > 1 else "split"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from image_recommender_amd import _lib  # noqa: E402

bench.main()
lib = _lib.load()
lib.knn_debug_prof.restype = C.c_int
buf = (C.c_ulonglong * 8)()
assert lib.knn_debug_prof(buf) == 0
names = ["dma_wait", "stage_barrier", "reads+dma_issue", "mfma_issue", "epi_barrier", "epilogue",
         "tile_loop_total", "-"]
tot = buf[6] or 1
for n, v in zip(names, buf):
    print(f"{n:18s} {v:16d}  {100.0 * v / tot:6.2f} %")
