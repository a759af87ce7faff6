"""ctypes binding of ``lib/libimgrec.so`` (the C ABI declared in ``include/*.h``).

The product path has no fallback: if the library is missing or cannot load, every call raises
``NativeLibraryError``.  There is deliberately no NumPy / PyTorch re-implementation of any kernel
in this package (the CPU restatements live in ``oracle/`` and are test infrastructure only).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / os.environ.get("IMGREC_LIB_NAME", "libimgrec.so")

# Error codes of include/imgrec_knn.h
KNN_OK, KNN_EINVAL, KNN_EHIP, KNN_ENOMEM, KNN_EIO, KNN_ENOSYS = 0, -1, -2, -3, -4, -5
KNN_METRIC_IP, KNN_METRIC_L2, KNN_METRIC_COSINE = 0, 1, 2
KNN_MAX_K = 32          # fused top-k kernels (include/imgrec_knn.h)
KNN_MAX_K_LARGE = 1024  # largest k of the in-LDS large-k route; beyond it the sort route (any k)
KNN_SEARCH_AUTO, KNN_SEARCH_EXACT, KNN_SEARCH_SPLIT, KNN_SEARCH_BF16, KNN_SEARCH_I8 = 0, 1, 2, 3, 4
KNN_FENCE_EAGER, KNN_FENCE_LAZY = 0, 1
COLOR_HIST_MAX_BINS = 32
INGEST_NOT_FAST, INGEST_TOO_SMALL = -1, -2

# (name, restype, argtypes) of every exported symbol — also the list the CPU test checks against
# the headers.
_vp, _i, _i64, _f, _d = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_double
_pi64, _pf, _pi, _pd = C.POINTER(C.c_int64), C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_double)
SIGNATURES = {
    # imgrec_knn.h
    "knn_create": (_i, [_i, _i, _i, C.POINTER(_vp)]),
    "knn_create_multi": (_i, [_i, _i, _pi, _i, C.POINTER(_vp)]),
    "knn_num_shards": (_i, [_vp]),
    "knn_free": (_i, [_vp]),
    "knn_dim": (_i, [_vp]),
    "knn_metric": (_i, [_vp]),
    "knn_ntotal": (_i64, [_vp]),
    "knn_is_trained": (_i, [_vp]),
    "knn_set_id_offset": (_i, [_vp, _i64]),
    "knn_train": (_i, [_vp, _vp, _i64]),
    "knn_add": (_i, [_vp, _vp, _i64]),
    "knn_add_device": (_i, [_vp, _vp, _i64, _vp]),
    "knn_reserve": (_i, [_vp, _i64]),
    "knn_reset": (_i, [_vp]),
    "knn_reconstruct_n": (_i, [_vp, _i64, _i64, _vp]),
    "knn_search": (_i, [_vp, _vp, _i64, _i, _vp, _vp]),
    "knn_search_device": (_i, [_vp, _vp, _i64, _i, _vp, _vp, _vp]),
    "knn_merge_device": (_i, [_vp, _vp, _i, _i64, _i, _i, _i, _vp, _vp, _vp]),
    "knn_packed_bytes": (_i64, [_i64, _i]),
    "knn_merge_packed_device": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _vp, _vp]),
    # imgrec_ivfpq.h
    "ivfpq_lut_device": (_i, [_vp, _i64, _i, _i, _i, _vp, _vp, _vp]),
    "ivfpq_scan_device": (_i, [_vp, _vp, _i64, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "ivfpq_scan_all_device": (_i, [_vp, _vp, _i64, _i, _vp, _vp, _vp, _i, _i, _vp, _vp, _i64, _i, _vp,
                                   _vp, _vp]),
    "knn_write": (_i, [_vp, C.c_char_p]),
    "knn_read": (_i, [C.c_char_p, _i, C.POINTER(_vp)]),
    "knn_read_multi": (_i, [C.c_char_p, _pi, _i, C.POINTER(_vp)]),
    "knn_normalize_L2": (_i, [_vp, _i64, _i]),
    "knn_set_timing": (_i, [_vp, _i]),
    "knn_set_fence_mode": (_i, [_vp, _i]),
    "knn_kernel_time": (_i, [_vp, _pd, _pi]),
    "knn_plan": (_i, [_vp, _i64, _i, _pi, _pi, _pi, _pi]),
    "knn_plan_kernel": (_i, [_vp, _i64, _i, C.c_char_p, _i]),
    "knn_set_search_mode": (_i, [_vp, _i]),
    "knn_search_stats": (_i, [_vp, _pi64, _pi64, _pf]),
    "knn_search_stats2": (_i, [_vp, _pi64, _pi64, _pi64, _pf]),
    "knn_last_path": (_i, [_vp]),
    "knn_large_k_fallbacks": (_i, [_vp, C.POINTER(_i64)]),
    "knn_last_error": (C.c_char_p, []),
    "knn_version": (C.c_char_p, []),
    # imgrec_color.h
    "color_hist_device": (_i, [_vp, _vp, _vp, _i64, _i, _vp, _vp, _vp]),
    "color_hist_host": (_i, [_vp, _i64, _vp, _vp, _i64, _i, _i, _vp, _vp]),
    "color_hist_last_error": (C.c_char_p, []),
    "color_host_register": (_i, [_vp, _i64]),
    "color_host_unregister": (_i, [_vp]),
    "vit_add_layernorm_bf16": (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _i, C.c_float, _vp]),
    "vit_quick_gelu_bf16": (_i, [_vp, _i64, _vp]),
    "vit_gelu_bf16": (_i, [_vp, _i64, _vp]),
    "vit_patchify_bf16": (_i, [_vp, _i64, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "vit_tokens_f32": (_i, [_vp, _vp, _vp, _i64, _i, _i, _vp, _vp]),
    "vit_attention_bf16": (_i, [_vp, _i64, _i, _i, _i, C.c_float, _vp, _vp]),
    "vit_linear_bf16": (_i, [_vp, _vp, _vp, _i64, _i, _i, _i, _vp, _vp]),
    "color_hist_batch_async": (_i, [_vp, _i64, _vp, _i64, _i, _vp, _vp, _vp, _vp, _vp]),
    # imgrec_ingest.h
    "ingest_parse_f32": (_i64, [_vp, _i64, _vp, _i64]),
    "ingest_concat_rows": (_i64, [C.POINTER(_vp), _pi64, _i64, _i, _pi64, _vp, _vp]),
    "ingest_concat_packed": (_i64, [_vp, _vp, _vp, _i64, _i, _vp, _vp, _vp]),
    "ingest_scan_open": (_i, [C.c_char_p, C.c_char_p, _i, _pi64, C.POINTER(_vp)]),
    "ingest_scan_next": (_i64, [_vp, _i64, _vp, _vp, _vp]),
    "ingest_scan_close": (_i, [_vp]),
    "ingest_scan_error": (C.c_char_p, []),
}


class NativeLibraryError(RuntimeError):
    """libimgrec.so is missing or failed to load — the HIP path is mandatory."""


class KnnError(RuntimeError):
    """A C-ABI call returned an error code (the message is knn_last_error())."""


_lock = threading.Lock()
_lib = None


def load() -> C.CDLL:
    """Load libimgrec.so once.

    torch (if installed) is imported first so that its bundled HIP runtime (SONAME
    libamdhip64.so.7) is the one the library binds to: one HIP runtime per process.
    """
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise NativeLibraryError(
                f"{LIB_PATH} not found: build it with `python -m image_recommender_amd.build` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        if os.environ.get("IMGREC_NO_TORCH_PRELOAD") != "1":
            try:
                import torch  # noqa: F401
            except Exception:  # pragma: no cover - torch is optional for the C ABI itself
                pass
        try:
            lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    msg = load().knn_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise KnnError(f"{what} failed (code {rc}): {last_error()}")
    return rc
