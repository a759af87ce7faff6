#!/usr/bin/env python3
"""Independent ceiling for the bf16 candidate kernel.

Times the vendor library's bf16 GEMM (torch.matmul -> hipBLASLt) at the candidate kernel's shape:
Q = 1024 queries x D = 1968 against N = 1M corpus rows, bf16 inputs, bf16 output, fp32
accumulation, in both output orientations (q . x^T -> 1024 x N and x . q^T -> N x 1024), with HIP
events on the launch stream.  The fused kernel does the same 2*N*D*Q flop plus a top-k epilogue
and writes no N x Q matrix, so the GEMM's TFLOP/s at the same held clock is the practical MFMA
ceiling for this shape on this chip.

Prints one JSON line per orientation: {"shape", "ms", "tflops", "frac_of_dense_peak"}.
`--profile-only` runs only the timed launches (for the rocprofv3 --pmc clock/busy pass).
"""
from __future__ import annotations

import argparse
import json

PEAK = 2516.8   # dense bf16 MFMA TFLOP/s (MI355X_MICROARCH.md)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=1968)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--orient", choices=("both", "qx", "xq"), default="both")
    ap.add_argument("--profile-only", action="store_true")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.rows, a.dim, generator=g, device=dev).to(torch.bfloat16)
    q = torch.randn(a.nq, a.dim, generator=g, device=dev).to(torch.bfloat16)
    flop = 2.0 * a.rows * a.dim * a.nq
    orients = ("qx", "xq") if a.orient == "both" else (a.orient,)
    for o in orients:
        out = torch.empty((a.nq, a.rows) if o == "qx" else (a.rows, a.nq), dtype=torch.bfloat16,
                          device=dev)

        def run():
            if o == "qx":
                torch.matmul(q, x.T, out=out)
            else:
                torch.matmul(x, q.T, out=out)
        for _ in range(a.warmup):
            run()
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        tf = flop / (ms * 1e-3) / 1e12
        if not a.profile_only:
            print(json.dumps({"shape": f"{o}: ({a.nq} x {a.dim}) . ({a.dim} x {a.rows}) bf16 -> bf16"
                              if o == "qx" else f"{o}: ({a.rows} x {a.dim}) . ({a.dim} x {a.nq}) bf16 -> bf16",
                              "orient": o, "ms": ms, "tflops": tf, "frac_of_dense_peak": tf / PEAK,
                              "out_bytes": out.numel() * 2}), flush=True)
        del out


if __name__ == "__main__":
    main()
