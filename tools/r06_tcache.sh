#!/bin/bash
# A/B: screen-threshold cache (libimgrec_tcache.so) vs production — result hashes, kernel times
set -o pipefail
O=gpurun_out/r06/tcache; mkdir -p $O
for v in libimgrec.so libimgrec_tcache.so; do
  for c in 2 3; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/ab_result_hash.py $c 1024 >> $O/hash.txt 2>> $O/err.txt || exit 1
  done
done
cat $O/hash.txt
for r in 1 2 3; do
  LIBS="libimgrec.so libimgrec_tcache.so" bash tools/b16w_epi_split.sh $O/cfg2_r$r --config 2 || exit 2
  LIBS="libimgrec.so libimgrec_tcache.so" bash tools/b16w_epi_split.sh $O/cfg3_r$r --config 3 || exit 3
done
