#!/bin/bash
# DreamSim-architecture forward: per-op probes, variant timings at batch 512, and a rocprofv3
# kernel split of the fused forward alone.  Writes under gpurun_out/$1.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ds}; mkdir -p $OUT
if [ -n "${PYTEST_SEL:-}" ]; then
timeout -k 10 600 python -u -m pytest $PYTEST_SEL -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
fi
if [ -z "${SKIP_PROBE:-}" ]; then
timeout -k 10 300 python tools/dreamsim_probe.py 512 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
fi
timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --variants ${VARIANTS:-fused,fused_gelu_lt,fused_gelu_lt@efficient} --iters 6 > $OUT/variants.jsonl 2> $OUT/variants.err || { tail $OUT/variants.err; exit 2; }
cat $OUT/variants.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/dreamsim_variants.py --batches 512 --variants fused_gelu_lt --iters 4 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
python3 - $OUT/prof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{float(r['TotalDurationNs'])/tot*100:5.1f}% {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_nq1 -o run --output-format csv -- python3 bench.py --nq 1 --profile-only --steps 200 --warmup 20 > $OUT/prof_nq1.log 2>&1 || { tail $OUT/prof_nq1.log; exit 4; }
grep elapsed $OUT/prof_nq1.log
for i in 1 2; do timeout -k 10 120 python bench.py --nq 1 --profile-only --steps 300 --warmup 50 >> $OUT/nq1.jsonl 2>>$OUT/nq1.err || exit 5; done
cat $OUT/nq1.jsonl
