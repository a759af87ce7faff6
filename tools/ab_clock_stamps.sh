#!/bin/bash
# Per-variant clock / MFMA busy (tools/pmc_clock.sh) and per-tile stamps (tools/b16_stamps.py) of
# the bf16 candidate kernels: LIBS (timed builds), STAMPS ("lib:reader_fn" pairs).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abcs}; mkdir -p $OUT
LIBS="${LIBS:-libimgrec.so}" bash tools/pmc_clock.sh ${1:-abcs}/pmc || exit 1
for p in ${STAMPS:-}; do
  v=${p%%:*}; fn=${p##*:}
  IMGREC_LIB_NAME=$v IMGREC_STAMPS_FN=$fn timeout -k 10 300 python3 tools/b16_stamps.py > $OUT/$v.json 2> $OUT/$v.txt || { tail -5 $OUT/$v.txt; exit 1; }
  echo "== $v"; cat $OUT/$v.txt
done
