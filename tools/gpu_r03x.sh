#!/bin/bash
# int8 scan: workgroups per CU (row splits = 256 x W) at nq = 1, cfg3.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03x}; mkdir -p $OUT
for w in 3 4 6 8 2 3; do
  IMGREC_I8_WGPCU=$w timeout -k 10 120 python bench.py --nq 1 --profile-only --steps 300 --warmup 100 > $OUT/w$w.json 2>>$OUT/err.log || exit 1
  echo "wgpcu $w $(cat $OUT/w$w.json)"
done
