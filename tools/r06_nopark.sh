#!/bin/bash
# A/B of the no-park insertion: bit-identity (result hashes) and kernel time at cfg2 / cfg3
set -o pipefail
O=gpurun_out/r06/nopark; mkdir -p $O
for v in libimgrec.so libimgrec_nopark.so; do
  for c in 2 3; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/ab_result_hash.py $c 1024 >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
for r in 1 2; do
  LIBS="libimgrec.so libimgrec_nopark.so" bash tools/b16w_epi_split.sh $O/cfg2_r$r --config 2 || exit 2
  LIBS="libimgrec.so libimgrec_nopark.so" bash tools/b16w_epi_split.sh $O/cfg3_r$r --config 3 || exit 3
done
