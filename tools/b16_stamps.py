"""Diagnostic: per-wave s_memtime at each tile's epilogue begin/end in one workgroup of the bf16
candidate kernel (a build with -DIMGREC_B16_STAMPS, lib/libimgrec_stamps.so): stage-loop and
epilogue cycles per tile, with two stamps per tile (negligible perturbation)."""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("IMGREC_LIB_NAME", "libimgrec_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
from image_recommender_amd import _lib
from image_recommender_amd.faiss_compat import METRIC_L2
from image_recommender_amd.sharded import ShardedIndex

CFG = int(os.environ.get("IMGREC_STAMPS_CFG", "3"))    # bench config (2: 1M x 768)
cfg = dict(bench.CONFIGS[CFG])
if os.environ.get("IMGREC_STAMPS_ROWS"):       # e.g. 125000: the N = 8 shard
    cfg["rows"] = int(os.environ["IMGREC_STAMPS_ROWS"])
dev = torch.device("cuda", 0)
D = int(sum(cfg["parts"]))
centres = bench.make_centres(torch, cfg, dev, CFG)
q = bench.gen_queries(torch, cfg, centres, 1024, dev, CFG)
shard = ShardedIndex(D, cfg["rows"], METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, centres, shard.row0, shard.row1, dev, CFG):
    shard.add_local(blk)
shard.index.search_mode = "bf16"
for _ in range(4):
    shard.search(q, 10)
torch.cuda.synchronize()
lib = _lib.load()
buf = (C.c_ulonglong * (8 * 256))()
assert getattr(lib, os.environ.get("IMGREC_STAMPS_FN", "knn_b16_stamps_read"))(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(8, 256).astype(np.int64)
nst = -(-D // 64)
ntile = int((a[0, :128] != 0).sum() // 2)
epi_s, epi_e = a[:, 0:2 * ntile:2], a[:, 1:2 * ntile:2]
loop = epi_s[:, 1:] - epi_e[:, :-1]                 # stage loop of tile t (from the previous epilogue end)
epi = epi_e - epi_s
out = {"nst": nst, "tiles": ntile, "stage_loop_per_tile": loop.tolist(), "epilogue_per_tile": epi.tolist(),
       "wg_cycles": int(epi_e.max() - epi_s.min())}
print(f"tiles {ntile}, stages/tile {nst}", file=sys.stderr)
for w in range(8):
    print(f"wave {w}: loop/tile median {np.median(loop[w]):.0f} (per stage {np.median(loop[w]) / nst:.0f}); "
          f"epilogue first {epi[w, 0]} median {np.median(epi[w, 1:]):.0f} mean {epi[w, 1:].mean():.0f}", file=sys.stderr)
nit = a[:, 128:128 + ntile]
print("insert-loop iterations per tile (wave 0): first", nit[0, :4].tolist(), "median", float(np.median(nit[0, 1:])),
      "mean", float(nit[0, 1:].mean()), "(all waves mean", float(nit[:, 1:].mean()), ")", file=sys.stderr)
out["insert_iterations"] = nit.tolist()
ins = a[:, 192:192 + min(ntile, 64)]
out["insert_cycles"] = ins.tolist()
print("cycles in the insertion blocks per tile: median per wave", [float(np.median(ins[w, 1:])) for w in range(8)],
      "(epilogue median per wave", [float(np.median(epi[w, 1:])) for w in range(8)], ")", file=sys.stderr)
tile = np.median(loop[0]) + np.median(epi.max(0)[1:])
print(f"tile period ~{tile:.0f}; ideal MFMA {nst * 2048}", file=sys.stderr)
print(json.dumps(out))
