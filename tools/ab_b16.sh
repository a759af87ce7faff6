#!/bin/bash
# A/B of bf16-kernel variants: the bf16 parity tests on the default library, then timing of each
# library in LIBS (bench --profile-only; ablated variants produce wrong results).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest_b16.log 2>&1 || { echo "bf16 pytest failed"; tail -40 $OUT/pytest_b16.log; exit 1; }
grep -E "passed|failed|cluster-sorted" $OUT/pytest_b16.log | tail -4
for v in ${LIBS:-libimgrec.so}; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python3 bench.py --profile-only --steps 10 --warmup 2 ${BENCH_ARGS:-} > $OUT/$v.json 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.json; exit 1; }
  echo "$v $(tail -1 $OUT/$v.json)"
done
