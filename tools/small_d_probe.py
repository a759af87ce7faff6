#!/usr/bin/env python3
"""One-query search time on 1M-row corpora of small widths (colour-only d = 48, SIFT-only 128;
WIDTHS=48,128,512 adds d = 512, the int8 gate's 8-block boundary):
device-resident queries through search_device, median of 200 searches; the path AUTO takes
(knn_last_path: 0 exact, 2 bf16, 3 int8).  NQS=1,8 adds batch sizes (default 1).  Measurement
tool, one JSON line per (width, batch, mode)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from image_recommender_amd import _lib, faiss_compat as faiss  # noqa: E402

torch.cuda.set_device(0)
n = int(os.environ.get("ROWS", 1_000_000))
for d in [int(w) for w in os.environ.get("WIDTHS", "48,128").split(",")]:
    g = torch.Generator(device="cuda").manual_seed(d)
    xb = torch.randn((n, d), device="cuda", generator=g)
    idx = faiss.IndexFlatL2(d)
    idx.reserve(n)
    st = torch.cuda.current_stream().cuda_stream
    idx.add_device(xb.data_ptr(), n, st)
    for nq in [int(v) for v in os.environ.get("NQS", "1").split(",")]:
      q = torch.randn((nq, d), device="cuda", generator=g)
      D = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
      I = torch.empty((nq, 10), dtype=torch.int64, device="cuda")
      for modes in (("auto", "exact") if d < 64 else ("auto", "exact", "bf16", "i8")):
        idx.search_mode = modes
        ts = []
        for i in range(250):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.search_device(q.data_ptr(), nq, 10, D.data_ptr(), I.data_ptr(), st)
            torch.cuda.synchronize()
            if i >= 50:
                ts.append(time.perf_counter() - t0)
        ts.sort()
        print(json.dumps({"d": d, "rows": n, "nq": nq, "mode": modes,
                          "path": _lib.load().knn_last_path(idx.handle),
                          "median_ms": 1e3 * ts[len(ts) // 2]}), flush=True)
    del idx, xb
