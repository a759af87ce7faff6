#!/bin/bash
# A/B of several environment switches read at index creation (one run each, "default" = none):
#   tools/ab_envs.sh TAG "IMGREC_MERGE_FUSE=0" "IMGREC_RERANK_P1=0" ...
# bench.py --profile-only --no-phases on each of $CFGS (default "r125k 3"; r125k = --rows 125000,
# a number = --config N) at --nq $NQ (default 1024), twice alternating -> gpurun_out/TAG/ab_envs.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for e in "" "$@"; do
    for c in ${CFGS:-r125k 3}; do
      ca="--config $c"; [ $c = r125k ] && ca="--rows 125000"
      env $e timeout -k 10 200 python bench.py $ca --nq ${NQ:-1024} --profile-only --no-phases --steps 100 --warmup 30 > $OUT/ab.json 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$rep [${e:-default}] cfg$c nq ${NQ:-1024} step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/ab_envs.txt
    done
  done
done
