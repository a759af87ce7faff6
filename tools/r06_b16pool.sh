#!/bin/bash
# A/B of the bf16 kernel's tile pool (IMGREC_B16W_POOL) at cfg3, cfg2 and the 125k shard, and the
# pool-off code against the previous commit's library (libimgrec_base.so).
set -o pipefail
O=gpurun_out/r06/b16pool; mkdir -p $O
timeout -k 10 400 python tools/b16_pool_ab.py 3 20 3 0,1,2,3 > $O/cfg3.jsonl 2> $O/cfg3.err || exit 1
timeout -k 10 300 python tools/b16_pool_ab.py 2 20 3 0,1,2,3 > $O/cfg2.jsonl 2> $O/cfg2.err || exit 2
timeout -k 10 300 python tools/b16_pool_ab.py 3 40 3 0,1,2 125000 > $O/cfg3_125k.jsonl 2> $O/cfg3_125k.err || exit 3
for r in 1 2; do
  LIBS="libimgrec_base.so libimgrec.so" bash tools/b16w_epi_split.sh $O/base_cfg3_r$r --config 3 || exit 4
done
