#!/bin/bash
# Per-tile stage-loop / epilogue cycles and insertion iterations of one workgroup (stamps build)
set -o pipefail
O=gpurun_out/r06/stamps; mkdir -p $O
for c in 2 3; do
  IMGREC_STAMPS_CFG=$c IMGREC_STAMPS_FN=knn_b16w_stamps_read timeout -k 10 300 python tools/b16_stamps.py \
      > $O/cfg$c.json 2> $O/cfg$c.txt || { tail -5 $O/cfg$c.txt; exit 1; }
  grep -v Warn $O/cfg$c.txt | tail -14
done
