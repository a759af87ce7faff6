#!/usr/bin/env python3
"""Per-tile cost of vit_linear_bf16 (csrc/vit_gemm.hip): the GEMM at M = 197 x batch tokens for
K = 768 / 1536 / 3072 at fixed N (so the tile count is fixed), HIP events over `iters` launches.
A line fit of ms against K gives the per-stage and the per-tile fixed cost (epilogue + tile
turnaround).  LIBS (comma-separated lib/ names) compares builds, e.g. the measurement builds of
IMGREC_VIT_EPI_EXP=1 (stores skipped) and =2 (no epilogue).  One JSON line per (lib, shape)."""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

PEAK = 2516.8
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
M = 197 * a.batch
dev = torch.device("cuda", 0)
libdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "image_recommender_amd", "lib")
libs = os.environ.get("LIBS", "libimgrec.so").split(",")
ACT = {"none": 0, "gelu_tanh": 2}
shapes = [(k, n, "none") for n in (768, 2304) for k in (768, 1536, 3072)] + [(768, 3072, "gelu_tanh"), (768, 3072, "none")]
for libname in libs:
    lib = C.CDLL(os.path.join(libdir, libname))
    lib.vit_linear_bf16.restype = C.c_int
    lib.vit_linear_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int,
                                    C.c_int, C.c_void_p, C.c_void_p]
    for k, n, act in shapes:
        x = torch.randn(M, k, device=dev).bfloat16()
        w = (torch.randn(n, k, device=dev) / k ** 0.5).bfloat16()
        b = torch.randn(n, device=dev)
        y = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
        st = torch.cuda.current_stream(dev).cuda_stream

        def run():
            rc = lib.vit_linear_bf16(x.data_ptr(), w.data_ptr(), b.data_ptr(), M, k, n, ACT[act], y.data_ptr(), st)
            assert rc == 0
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tf = 2.0 * M * k * n / (ms * 1e-3) / 1e12
        print(json.dumps({"lib": libname, "m": M, "k": k, "n": n, "act": act, "ms": round(ms, 4),
                          "tflops": round(tf, 1), "frac": round(tf / PEAK, 4)}), flush=True)
        del x, w, b, y
