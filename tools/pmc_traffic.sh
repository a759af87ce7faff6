#!/bin/bash
# HBM traffic of the fused k-NN kernel from rocprofv3 PMC counters, one counter per pass
# (MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads,
# including LDS-DMA; WRITE_SIZE is exact for these stores).  Writes gpurun_out/traffic_<tag>/<tag>_traffic.json (copy into profiles/).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-r01}; OUT=gpurun_out/traffic_$TAG; mkdir -p $OUT
B="python3 bench.py --profile-only --steps 3 --warmup 1 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex 'knn_tile|knn_b16' --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- $B > $OUT/f.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex 'knn_tile|knn_b16' --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- $B > $OUT/w.log 2>&1 || exit 2
python3 - "$OUT" "$TAG" <<'PY'
import csv, json, sys, collections
out, tag = sys.argv[1], sys.argv[2]
def read(f, name):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == name:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals
fs = read(f"{out}/f/run_counter_collection.csv", "FETCH_SIZE")
ws = read(f"{out}/w/run_counter_collection.csv", "WRITE_SIZE")
res = {}
for k in fs:
    f = sum(fs[k]) / len(fs[k]); w = sum(ws.get(k, [0])) / max(len(ws.get(k, [0])), 1)
    res[k] = {"launches": len(fs[k]), "fetch_size_kb_raw": f, "write_size_kb": w,
              "hbm_read_bytes": 2 * f * 1024, "hbm_write_bytes": w * 1024,
              "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
              "note": "read = FETCH_SIZE x 1024 x 2 (gfx950 half-count of 16-B/lane streaming reads)"}
json.dump(res, open(f"{out}/{tag}_traffic.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
