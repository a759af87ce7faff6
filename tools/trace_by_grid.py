#!/usr/bin/env python3
"""Average duration per (kernel, grid size) from a rocprofv3 kernel_trace.csv — separates the
shapes one kernel template runs at (e.g. the four ViT GEMMs).  Usage: trace_by_grid.py trace.csv"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    key = (name[:70], grid)
    acc[key][0] += 1
    acc[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in acc.values())
for (name, grid), (n, us) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{us / n:9.1f} us  x{n:5d}  {100 * us / tot:5.1f} %  grid {grid:>8}  {name}")
