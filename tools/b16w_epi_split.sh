#!/bin/bash
# Split the bf16 candidate kernel's time into its stage loop and its per-tile epilogue at one
# workload: the production library, the stage loop alone
# (IMGREC_B16W_EPI_EXP=1) and the screen without insertions (=2), each timed by the bench's own
# HIP events (--profile-only).  Build the variants first:
#   bash tools/build_variants.sh noepi "-DIMGREC_B16W_EPI_EXP=1" scronly "-DIMGREC_B16W_EPI_EXP=2"
# Usage: tools/b16w_epi_split.sh <out dir> [bench args...]
set -u
OUT=$1; shift
mkdir -p $OUT
for v in ${LIBS:-libimgrec.so libimgrec_noepi.so libimgrec_scronly.so}; do
  IMGREC_LIB_NAME=$v timeout -k 10 300 python3 bench.py --profile-only --steps 20 --warmup 3 --no-phases "$@" \
      > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -5 $OUT/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$v.json')); print('$v', 'kernel_ms %.4f' % d['kernel_ms'], 'ms_per_step %.4f' % d['ms_per_step'])"
done
