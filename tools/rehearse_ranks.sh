#!/bin/bash
# Rehearsal of the N-rank bench protocol on ONE GPU (gloo, every rank on device 0; the timing is
# meaningless, the point is that the partition, gather, merge, recall and JSON line all run).
# The measured multi-GPU runs are the driver's (RCCL, one rank per GPU).  Usage: rehearse_ranks.sh N [extra bench args]
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
N=${1:-2}; shift
OUT=gpurun_out/rehearse; mkdir -p $OUT
IMGREC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 3 --warmup 1 --single-query-steps 3 "$@" \
  > $OUT/n$N.json 2> $OUT/n$N.err || { tail -30 $OUT/n$N.err; exit 1; }
cat $OUT/n$N.json
