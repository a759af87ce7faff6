#!/bin/bash
# Clock / MFMA busy of the epilogue variants at cfg3 and cfg2 (tools/pmc_clock.sh per library),
# and the cfg2 traffic record of the production library (profiles/*_cfg2_traffic.json).
set -o pipefail
export LIBS="libimgrec.so libimgrec_noepi.so libimgrec_scronly.so libimgrec_scrmin.so"
BENCH_ARGS="--config 3" bash tools/pmc_clock.sh r06/clk_cfg3 || exit 1
BENCH_ARGS="--config 2" bash tools/pmc_clock.sh r06/clk_cfg2 || exit 2
LIBS=libimgrec.so BENCH_ARGS="--config 2" bash tools/pmc_traffic.sh r06_v1_cfg2 > /dev/null || exit 3
cat gpurun_out/traffic_r06_v1_cfg2/r06_v1_cfg2_traffic.json
