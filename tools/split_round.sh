#!/bin/bash
# split-path GPU round: parity tests (split + exact), then profile-only timings of both modes
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-split}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_split_gpu.py tests/test_knn_gpu.py -x -q -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for lib in ${LIBS:-libimgrec.so}; do
  for mode in split exact; do
    IMGREC_LIB_NAME=$lib timeout -k 10 300 python3 bench.py --profile-only --steps 5 --warmup 1 --mode $mode > $OUT/b_${lib}_$mode.json 2>&1 || { echo "bench $lib $mode failed"; tail -20 $OUT/b_${lib}_$mode.json; exit 2; }
    echo "$lib $mode $(tail -1 $OUT/b_${lib}_$mode.json)"
  done
done
