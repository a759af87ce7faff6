#!/bin/bash
# one-query cold/warm kernel times (two libraries x two configs), the launcher GPU tests, the bench
set -o pipefail
O=gpurun_out/r06/cold; mkdir -p $O
for v in libimgrec.so libimgrec_nont.so; do
  for c in 3 2; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/nq1_cold.py $c 64 >> $O/nq1_cold.jsonl 2>> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  done
done
cat $O/nq1_cold.jsonl
timeout -k 10 600 python -u -m pytest tests/test_launch_gpu.py -x -v --timeout 400 --timeout-method thread > $O/launch_tests.log 2>&1 || { tail -30 $O/launch_tests.log; exit 2; }
tail -1 $O/launch_tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['single_query'])"
