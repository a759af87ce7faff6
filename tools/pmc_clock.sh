#!/bin/bash
# Clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA-pipe busy fraction of the bf16 candidate
# kernel for each library variant in LIBS (one --pmc pass per variant).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmcclk}; mkdir -p $OUT
R="--kernel-trace --kernel-include-regex knn_b16 --output-format csv"
for v in ${LIBS:-libimgrec.so}; do
  IMGREC_LIB_NAME=$v timeout -s KILL 120 rocprofv3 $R --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $OUT/$v -o run -- python3 bench.py --profile-only --steps 3 --warmup 1 ${BENCH_ARGS:-} > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.log; exit 2; }
  python3 - $OUT/$v <<'PY'
import collections, csv, glob, sys
d = sys.argv[1]
f = glob.glob(d + "/*/run_counter_collection.csv") + glob.glob(d + "/run_counter_collection.csv")
agg = collections.defaultdict(list); dur = []
for r in csv.DictReader(open(f[0])):
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg[r["Counter_Name"]].append(float(r["Counter_Value"])); dur.append(t)
t = sum(dur) / len(dur)
g = sum(agg["GRBM_GUI_ACTIVE"]) / len(agg["GRBM_GUI_ACTIVE"])
clk = g / 8 / t
m = sum(agg["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(agg["SQ_VALU_MFMA_BUSY_CYCLES"])
print(f"{d.split('/')[-1]:24s} dur {t*1e3:.3f} ms  clock {clk/1e9:.2f} GHz  MFMA busy {m / (256*4*clk*t):.1%}  "
      f"MFMA insts {sum(agg['SQ_INSTS_MFMA'])/len(agg['SQ_INSTS_MFMA']):.4g}")
import json, os
kern = next(csv.DictReader(open(f[0])))["Kernel_Name"].split("(")[0]
json.dump({kern: {"clock_ghz": clk / 1e9, "mfma_busy": m / (256 * 4 * clk * t), "dur_ms_under_pmc": t * 1e3,
                  "note": "clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; busy = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x cycles)"}},
          open(os.path.join(os.path.dirname(d), os.path.basename(d) + "_clock.json"), "w"), indent=1)
PY
done
