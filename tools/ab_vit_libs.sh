#!/bin/bash
# DreamSim-architecture forward (batch 512, hip_gemm_tanh) on several builds of the library,
# twice alternating: tools/ab_vit_libs.sh TAG libimgrec.so libimgrec_X.so ... -> gpurun_out/TAG/ab_vit.jsonl
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    IMGREC_LIB_NAME=$lib timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --iters 6 --variants hip_gemm_tanh \
      > $OUT/v.jsonl 2>> $OUT/ab_vit.err || { tail -5 $OUT/ab_vit.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/v.jsonl').read().splitlines()[-1]);d['lib']='$lib';d['rep']=$rep;print(json.dumps(d))" | tee -a $OUT/ab_vit.jsonl
  done
done
