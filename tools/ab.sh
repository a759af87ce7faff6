#!/bin/bash
# A/B timing of library variants on the bench workload (profile-only runs), then correctness of
# each variant on the k-NN GPU tests.  Usage: bash tools/ab.sh TAG lib1.so lib2.so ...
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python3 bench.py --profile-only --steps 5 --warmup 1 ${BENCH_ARGS:-} > $OUT/ab_${v}_$rep.json 2>&1 || { echo "$v failed"; tail -5 $OUT/ab_${v}_$rep.json; exit 1; }
    echo "$rep $v $(tail -1 $OUT/ab_${v}_$rep.json)"
  done
done
for v in "$@"; do
  IMGREC_LIB_NAME=$v timeout -k 10 600 python -m pytest ${TESTS:-tests/test_knn_gpu.py} -x -q -m gpu > $OUT/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $OUT/pytest_$v.log; exit 2; }
  echo "$v $(tail -1 $OUT/pytest_$v.log)"
done
