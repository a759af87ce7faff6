#!/bin/bash
# A/B of an environment switch read at index creation: bench.py --profile-only on configs 2 and 3
# at --nq $NQ (default 1024) with and without "$2" (e.g. IMGREC_CHANCE_SKIP=0), twice alternating
# -> gpurun_out/$1/ab_env.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
  for e in "" "$2"; do
    for c in 2 3; do
      env $e timeout -k 10 200 python bench.py --config $c --nq ${NQ:-1024} --profile-only --steps 60 --warmup 20 > $OUT/ab.json 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$rep [${e:-default}] cfg$c nq ${NQ:-1024} step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/ab_env.txt
    done
  done
done
