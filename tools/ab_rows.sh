#!/bin/bash
# Interleaved kernel timing of library variants (TIME_LIBS) at several corpus sizes (ROWS), two
# rounds; the bf16 parity tests on TEST_LIBS first.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in ${TEST_LIBS:-}; do IMGREC_LIB_NAME=$v timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -30 gpurun_out/ab/pytest_$v.log; exit 1; }; echo "$v $(tail -1 gpurun_out/ab/pytest_$v.log)"; done
for r in 1 2; do for R in ${ROWS:-1000000}; do for v in $TIME_LIBS; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python3 bench.py --rows $R --profile-only --steps ${STEPS:-20} --warmup 3 2>/dev/null | tail -1 | sed "s/^/$R $v /" || exit 1
done; done; done
