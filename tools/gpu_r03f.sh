#!/bin/bash
# Round-3 final validation: the whole GPU suite, the nq = 1 and 125k-row profile-only steps
# (one-launch small-batch merge), then the records of gpu_r03e.sh.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do timeout -k 10 120 python bench.py --nq 1 --profile-only --steps 300 --warmup 100 >> $OUT/nq1.jsonl 2>>$OUT/nq1.err || exit 2; done
cat $OUT/nq1.jsonl
for i in 1 2; do timeout -k 10 120 python bench.py --rows 125000 --profile-only --steps 200 --warmup 60 >> $OUT/rows125k.jsonl 2>>$OUT/rows125k.err || exit 3; done
cat $OUT/rows125k.jsonl
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_nq1 -o run --output-format csv -- python3 bench.py --nq 1 --profile-only --steps 300 --warmup 100 > $OUT/prof_nq1.log 2>&1 || exit 4
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_nq1/run_kernel_stats.csv')):
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:90])"
bash tools/gpu_r03e.sh ${1:-r03f}
