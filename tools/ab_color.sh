#!/bin/bash
# colour-histogram parity tests + rate for each library variant in LIBS (default lib first)
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_color; mkdir -p $OUT
LIBS=${LIBS:-libimgrec.so}
for v in $(echo $LIBS | tr ' ' '\n' | sort -u); do
  IMGREC_LIB_NAME=$v timeout -k 10 300 python -m pytest tests/test_dropin_gpu.py -x -q -k color > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
for v in $LIBS; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/color_hist_rate.py >> $OUT/rate.jsonl 2> $OUT/rate.err || { tail -20 $OUT/rate.err; exit 2; }
done
cat $OUT/rate.jsonl
