#!/bin/bash
# Sibling lockstep of the 256 x 256 bf16 kernel (IMGREC_B16W_SYNC_LAG): kernel time, HBM fetch
# (FETCH_SIZE x 2) and clock / MFMA busy per lag setting, default bench workload (1M x 1968, 1024
# queries).  "off" = the round-3 kernel.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03r}; mkdir -p $OUT
R="--kernel-trace --kernel-include-regex knn_b16w --output-format csv"
B="python3 bench.py --profile-only --steps 5 --warmup 2"
for lag in ${LAGS:-off 0 1 2}; do
  if [ "$lag" = off ]; then unset IMGREC_B16W_SYNC_LAG; else export IMGREC_B16W_SYNC_LAG=$lag; fi
  for i in 1 2; do
    timeout -k 10 120 python bench.py --profile-only --steps 30 --warmup 10 > $OUT/lag_$lag.$i.json 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
    echo "lag $lag: $(cat $OUT/lag_$lag.$i.json)"
  done
  timeout -s KILL 120 rocprofv3 $R --pmc FETCH_SIZE -d $OUT/f_$lag -o run -- $B > $OUT/f_$lag.log 2>&1 || { tail -5 $OUT/f_$lag.log; exit 2; }
  timeout -s KILL 120 rocprofv3 $R --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/c_$lag -o run -- $B > $OUT/c_$lag.log 2>&1 || { tail -5 $OUT/c_$lag.log; exit 3; }
  python3 - $OUT $lag <<'PY'
import collections, csv, glob, sys
out, lag = sys.argv[1], sys.argv[2]
def rd(sub):
    f = glob.glob(f"{out}/{sub}/*/run_counter_collection.csv") + glob.glob(f"{out}/{sub}/run_counter_collection.csv")
    agg = collections.defaultdict(list); dur = []
    for r in csv.DictReader(open(f[0])):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: sum(v) / len(v) for k, v in agg.items()}, sum(dur) / len(dur)
f, tf = rd(f"f_{lag}")
c, tc = rd(f"c_{lag}")
clk = c["GRBM_GUI_ACTIVE"] / 8 / tc
print(f"lag {lag}: fetch {f['FETCH_SIZE']*2048/1e9:.3f} GB/launch  clock {clk/1e9:.3f} GHz  "
      f"mfma busy {c['SQ_VALU_MFMA_BUSY_CYCLES']/(256*4*clk*tc):.3f}  dur(pmc) {tc*1e3:.3f} ms")
PY
done
