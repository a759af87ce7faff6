#!/bin/bash
# colour-histogram parity tests + A/B of the fixed-bin kernel (default lib) vs the generic one
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_color; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_dropin_gpu.py -x -q -k color > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${LIBS:-libimgrec.so libimgrec_colgen.so libimgrec.so}; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/color_hist_rate.py >> $OUT/rate.jsonl 2> $OUT/rate.err || { tail -20 $OUT/rate.err; exit 2; }
done
cat $OUT/rate.jsonl
