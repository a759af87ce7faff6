#!/bin/bash
# A/B: non-temporal rerank row loads (libimgrec_rrnt.so) vs production — result hashes, the cfg3
# bench (steps and the one-query leg), the 125k-row step
set -o pipefail
O=gpurun_out/r06/rrnt; mkdir -p $O
for v in libimgrec.so libimgrec_rrnt.so; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/ab_result_hash.py 3 1024 >> $O/hash.txt 2>> $O/err.txt || exit 1
done
cat $O/hash.txt
for r in 1 2; do
  for v in libimgrec.so libimgrec_rrnt.so; do
    IMGREC_LIB_NAME=$v timeout -k 10 300 python bench.py --no-cpu-baseline --pmc off --single-query-steps 200 > $O/cfg3_${v}_$r.json 2>> $O/err.txt || exit 2
    IMGREC_LIB_NAME=$v timeout -k 10 300 python bench.py --rows 125000 --steps 200 --warmup 20 --profile-only --no-phases > $O/r125k_${v}_$r.json 2>> $O/err.txt || exit 3
    python3 -c "
import json; a=json.load(open('$O/cfg3_${v}_$r.json')); b=json.load(open('$O/r125k_${v}_$r.json'))
print('$v', 'cfg3 ms/step %.4f' % a['ms_per_step'], 'nq1 ms %.4f' % (1e3/a['single_query']['queries_per_s']), '125k ms/step %.4f kernel %.4f' % (b['ms_per_step'], b['kernel_ms']))"
  done
done
