#!/bin/bash
# Round-3 closing box: the whole GPU suite, smoke, the driver's bench command, the same bench
# under rocprofv3 --kernel-trace --stats, single-query / small-batch steps (nq 1, 2, 4, 8), the
# 125k-row (N = 8 shard) step and the config-2 single-query probe.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 2; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 4; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:6]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:90])"
for nq in 1 2 4 8; do timeout -k 10 120 python bench.py --nq $nq --profile-only --steps 300 --warmup 100 >> $OUT/small_batch.jsonl 2>>$OUT/err.log || exit 5; done
for i in 1 2; do timeout -k 10 120 python bench.py --rows 125000 --profile-only --steps 200 --warmup 60 >> $OUT/rows125k.jsonl 2>>$OUT/err.log || exit 6; done
CFG=2 timeout -k 10 300 python tools/i8_cfg2_probe.py > $OUT/probe_cfg2.jsonl 2>> $OUT/err.log || exit 7
cat $OUT/small_batch.jsonl $OUT/rows125k.jsonl $OUT/probe_cfg2.jsonl
