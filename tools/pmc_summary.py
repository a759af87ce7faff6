"""Summarise rocprofv3 --pmc CSVs of the fused kernel (per-dispatch averages)."""
import collections, csv, glob, sys
out = sys.argv[1]
for f in sorted(glob.glob(f"{out}/*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append((float(r["Counter_Value"]), t))
    for (k, c), v in sorted(agg.items()):
        print(f"{f.split('/')[-2]:5s} {k:40s} {c:28s} n={len(v):3d} avg={sum(x for x, _ in v) / len(v):.4g} dur_ms={sum(t for _, t in v) / len(v):.3f}")
