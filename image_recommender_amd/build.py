"""Build the native library ``image_recommender_amd/lib/libimgrec.so`` for gfx950.

One C-ABI shared library holds every native piece of the hot path (no torch types anywhere in its
signatures):

* ``csrc/knn_*.hip`` + ``csrc/knn_{capi,plan,search,multi,io}.cpp`` — the exact k-NN index
  (include/imgrec_knn.h), ``csrc/ivfpq.hip`` + ``ivfpq_capi.cpp`` — IVF-PQ (include/imgrec_ivfpq.h)
* ``csrc/color_hist.hip`` — the per-image colour histogram (include/imgrec_color.h)
* ``csrc/ingest.cpp`` — the SQLite pickle-BLOB fast path (include/imgrec_ingest.h)

The library is built in-tree so that it travels to the GPU box with the repository snapshot.
Usage: ``python -m image_recommender_amd.build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = PKG.parent / "build" / ("obj" + os.environ.get("IMGREC_OBJ_SUFFIX", ""))
LIB = LIBDIR / os.environ.get("IMGREC_LIB_NAME", "libimgrec.so")
EXTRA_FLAGS = os.environ.get("IMGREC_EXTRA_FLAGS", "").split()
ARCH = os.environ.get("IMGREC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["knn_kernels.hip", "knn_b16.hip", "knn_b16w.hip", "knn_refine.hip", "knn_capi.cpp", "knn_plan.cpp",
           "knn_search.cpp", "knn_multi.cpp", "knn_io.cpp", "ivfpq_capi.cpp", "color_hist.hip",
           "ingest.cpp", "ivfpq.hip", "knn_largek.hip", "knn_hugek.hip", "vit_fused.hip", "vit_attn.hip", "knn_i8.hip", "vit_gemm.hip"]
HEADERS = ["knn_kernels.h", "knn_index.h", "knn_multi.h", "wave_ops.h", "knn_certify.h", "lds_dma.h", "../../include/imgrec_ivfpq.h",
           "../../include/imgrec_knn.h", "../../include/imgrec_color.h", "../../include/imgrec_ingest.h",
           "../../include/imgrec_vit.h"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the ROCm toolchain is required to build libimgrec.so")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.exists() and d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path, force: bool) -> str:
    deps = [src] + [(CSRC / h).resolve() for h in HEADERS]
    if not force and not _stale(obj, deps):
        return f"up to date: {obj.name}"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
           "-Wno-unused-function", *EXTRA_FLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return f"compiled {src.name}"


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    srcs = [CSRC / s for s in SOURCES]
    objs = [OBJDIR / (s.rsplit(".", 1)[0] + ".o") for s in SOURCES]
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for msg in ex.map(lambda so: _compile(so[0], so[1], force), zip(srcs, objs)):
            if verbose:
                print(f"[imgrec build] {msg}", file=sys.stderr)
    if force or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + \
              [str(o) for o in objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[imgrec build] linked {LIB}", file=sys.stderr)
    return LIB


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    main()
