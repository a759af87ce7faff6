#!/bin/bash
# bf16 kernel ablations (timing only; ablated variants produce wrong results) + phase profile
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-abl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in ${LIBS:-libimgrec.so libimgrec_noepi.so libimgrec_nodma.so libimgrec_nowait.so}; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python3 bench.py --profile-only --steps 5 --warmup 1 ${BENCH_ARGS:-} > $OUT/$v.json 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.json; exit 1; }
  echo "$v $(tail -1 $OUT/$v.json)"
done
timeout -k 10 200 python3 tools/prof_phases.py ${PHASE_MODE:-bf16} > $OUT/phases.txt 2>&1 || { echo "phases failed"; tail -5 $OUT/phases.txt; exit 2; }
cat $OUT/phases.txt
