#!/bin/bash
# A/B: non-temporal corpus DMA in the bf16 candidate kernel (libimgrec_cnt.so, IMGREC_B16W_CORPUS_NT=1)
# vs production: result hashes, kernel times (3 alternating rounds), traffic and clock under PMC.
set -o pipefail
O=gpurun_out/r06/cnt; mkdir -p $O
for v in libimgrec.so libimgrec_cnt.so; do
  for c in 2 3; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/ab_result_hash.py $c 1024 >> $O/hash.txt 2>> $O/err.txt || exit 1
  done
done
cat $O/hash.txt
for r in 1 2 3; do
  LIBS="libimgrec.so libimgrec_cnt.so" bash tools/b16w_epi_split.sh $O/cfg3_r$r --config 3 || exit 3
  LIBS="libimgrec.so libimgrec_cnt.so" bash tools/b16w_epi_split.sh $O/cfg2_r$r --config 2 || exit 2
done
for v in libimgrec.so libimgrec_cnt.so; do
  IMGREC_LIB_NAME=$v LIBS=$v BENCH_ARGS="--config 3" bash tools/pmc_traffic.sh cnt_${v%.so} > /dev/null || exit 4
done
LIBS="libimgrec.so libimgrec_cnt.so" BENCH_ARGS="--config 3" bash tools/pmc_clock.sh r06/cnt/clk || exit 5
cat gpurun_out/traffic_cnt_*/*_traffic.json
