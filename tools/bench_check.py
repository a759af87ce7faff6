"""Diagnostic: bench.py's data path at reduced size, checked against the numpy oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from oracle.flat_knn import search_exact
from image_recommender_amd.sharded import ShardedIndex
from image_recommender_amd.faiss_compat import METRIC_L2, IndexFlatL2

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
cfg = dict(bench.CONFIGS[3]); cfg["rows"] = rows
dev = torch.device("cuda", 0)
cen = bench.make_centres(torch, cfg, dev, 3)
q = bench.gen_queries(torch, cfg, cen, 1024, dev, 3)
sh = ShardedIndex(1968, rows, METRIC_L2, device=0)
blocks = []
for blk in bench.gen_rows(torch, cfg, cen, 0, rows, dev, 3):
    sh.add_local(blk); blocks.append(blk.cpu().numpy())
xb = np.concatenate(blocks)
D, I = sh.search(q, 10)
torch.cuda.synchronize()
D, I = D.cpu().numpy(), I.cpu().numpy()
qn = q.cpu().numpy()
Dg, Ig = search_exact(xb, qn[:16], 10, "l2")
print("dev add  : D", D[:2], "\nI", I[:2]); print("oracle   : D", Dg[:2], "\nI", Ig[:2])
h = IndexFlatL2(1968); h.add(xb); Dh, Ih = h.search(qn[:16], 10)
print("host add : I", Ih[:2])
rec = np.back = sum(len(set(a) & set(b)) for a, b in zip(I[:16], Ig)) / 160
print("recall dev-add", rec, " host-add", sum(len(set(a) & set(b)) for a, b in zip(Ih, Ig)) / 160)
gd, gi = bench.exact_ground_truth(torch, None, 1, cfg, cen, 0, rows, q[:16], 10, dev, 3)
print("bench GT : I", gi[:2], "\nrecall bench-GT vs oracle", sum(len(set(a) & set(b)) for a, b in zip(gi, Ig)) / 160)
