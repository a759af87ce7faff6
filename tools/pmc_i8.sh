#!/bin/bash
# Issue profile of the int8 small-batch scan (knn_i8_scan_kernel) at nq = NQ (default 1): instruction counts
# and wave-cycle split (one --pmc pass, SQ counters only), plus the clock.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmci8}; mkdir -p $OUT
R="--kernel-trace --kernel-include-regex knn_i8_scan --output-format csv"
timeout -s KILL 120 rocprofv3 $R --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $OUT/a -o run -- python3 bench.py --nq ${NQ:-1} --mode i8 --profile-only --steps 20 --warmup 5 > $OUT/a.log 2>&1 || { tail -5 $OUT/a.log; exit 2; }
timeout -s KILL 120 rocprofv3 $R --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY -d $OUT/b -o run -- python3 bench.py --nq ${NQ:-1} --mode i8 --profile-only --steps 20 --warmup 5 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
python3 - $OUT <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
agg = collections.defaultdict(list); dur = []
for sub in ("a", "b"):
    f = glob.glob(f"{out}/{sub}/*/run_counter_collection.csv") + glob.glob(f"{out}/{sub}/run_counter_collection.csv")
    for r in csv.DictReader(open(f[0])):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if sub == "a":
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
t = sum(dur) / len(dur)
m = {k: sum(v) / len(v) for k, v in agg.items()}
clk = m["GRBM_GUI_ACTIVE"] / 8 / t
print(f"dur {t*1e6:.1f} us  clock {clk/1e9:.2f} GHz")
for k in sorted(m):
    print(f"{k:28s} {m[k]:.4g}")
PY
