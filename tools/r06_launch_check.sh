#!/bin/bash
# VERDICT r05 item 1 on a one-GPU box: `bench.py --gpus 2` without torchrun
#  (a) RCCL (default): exits non-zero before any work (one GPU visible);
#  (b) IMGREC_DIST_BACKEND=gloo: the launcher starts 2 ranks sharing the GPU, world_size 2.
set -o pipefail
out=gpurun_out/r06/launch
mkdir -p $out
timeout -k 10 120 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    > $out/nccl_one_gpu.stdout 2> $out/nccl_one_gpu.stderr
rc=$?
echo "rccl --gpus 2 on one GPU: exit $rc" | tee $out/nccl_one_gpu.rc
[ $rc -eq 2 ] || exit 1
IMGREC_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --single-query-steps 5 > $out/gloo_two_ranks.json 2> $out/gloo_two_ranks.stderr
rc=$?
echo "gloo --gpus 2: exit $rc"
tail -3 $out/gloo_two_ranks.stderr
exit $rc
