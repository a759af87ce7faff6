#!/bin/bash
# Per-rank step of the row partition (1024 queries x 1M/N rows) vs the query x row partition
# (512 queries x 2M/N rows) at N = 2, 4, 8, on one GPU (profile-only bench: step wall + kernel).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for r in 1 2; do for n in 2 4 8; do
  R=$((1000000 / n)); R2=$((2000000 / n))
  a=$(timeout -k 10 200 python3 bench.py --rows $R --nq 1024 --profile-only --steps 50 --warmup 5 2>/dev/null | tail -1) || exit 1
  b=$(timeout -k 10 200 python3 bench.py --rows $R2 --nq 512 --profile-only --steps 50 --warmup 5 2>/dev/null | tail -1) || exit 1
  echo "{\"N\": $n, \"row_partition_1024q_x_${R}\": $a, \"query_row_512q_x_${R2}\": $b}"
done; done
