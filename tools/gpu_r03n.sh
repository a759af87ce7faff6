#!/bin/bash
# int8 small-batch path: its tests and the neighbouring bf16 / exact suites, then nq = 1 and 2
# profile-only steps (AUTO now takes the int8 path) and a kernel split of the nq = 1 search.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03n}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_i8_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_i8.log 2>&1 || { echo "i8 tests failed"; tail -40 $OUT/pytest_i8.log; exit 1; }
tail -1 $OUT/pytest_i8.log
for nq in 1 2; do timeout -k 10 120 python bench.py --nq $nq --profile-only --steps 300 --warmup 100 >> $OUT/nq$nq.jsonl 2>>$OUT/nq.err || { tail $OUT/nq.err; exit 2; }; done
cat $OUT/nq1.jsonl $OUT/nq2.jsonl
timeout -k 10 120 python bench.py --nq 1 --mode bf16 --profile-only --steps 300 --warmup 100 >> $OUT/nq1_bf16.jsonl 2>>$OUT/nq.err || exit 3
cat $OUT/nq1_bf16.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_nq1 -o run --output-format csv -- python3 bench.py --nq 1 --profile-only --steps 300 --warmup 100 > $OUT/prof_nq1.log 2>&1 || { tail $OUT/prof_nq1.log; exit 4; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof_nq1/run_kernel_stats.csv')))[:10]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:90])"
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_bf16_gpu.py tests/test_sweep_gpu.py tests/test_certificate_multi_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_rest.log 2>&1 || { echo "other tests failed"; tail -30 $OUT/pytest_rest.log; exit 5; }
tail -1 $OUT/pytest_rest.log
