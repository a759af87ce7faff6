#!/bin/bash
# Round-6 final evidence: every -m gpu test, the smoke, the default bench (live PMC), config 2,
# the 125k-row (N = 8 shard) step, and a rocprofv3 kernel-stats profile of the bench command.
# Each GPU step under its own time limit; stop at the first failure.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06/final}; mkdir -p $O
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $O/gpu_tests.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 $O/gpu_tests.log
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 2; }
[ -n "${SKIP_TESTS:-}" ] || tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 3; }
timeout -k 10 600 python bench.py --config 2 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo "cfg2 bench failed"; tail -20 $O/bench_cfg2.err; exit 4; }
timeout -k 10 300 python bench.py --rows 125000 --no-cpu-baseline --pmc off > $O/rows125k.json 2> $O/rows125k.err || { echo "125k failed"; exit 5; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --pmc off > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 6; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bench_under_rocprof.csv \;
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench.json", "bench_cfg2.json", "rows125k.json"):
    d = json.load(open(f"{o}/{f}"))
    r = d["roofline"]
    print(f, "value %.0f" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel %.4f" % r["kernel_ms"],
          "frac %.4f" % r["frac"], "traffic", r["traffic"], "busy", r["mfma_busy"], "clk", r["clock_ghz"],
          "recall", d["recall_at_10"], d["recall_queries"], "sq", {k: d["single_query"][k] for k in ("kernel_ms", "kernel_ms_cold", "hbm_frac", "hbm_frac_warm", "ms_per_query_cold")})
PY
head -4 $O/kernel_stats_bench_under_rocprof.csv | cut -c1-220
