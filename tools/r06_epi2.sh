#!/bin/bash
# The epilogue split again with the MFMAs kept live in the variants, plus their PMC clock / busy
set -o pipefail
bash tools/b16w_epi_split.sh gpurun_out/r06/epi2_cfg2 --config 2 || exit 1
bash tools/b16w_epi_split.sh gpurun_out/r06/epi2_cfg3 --config 3 || exit 2
export LIBS="libimgrec.so libimgrec_noepi.so libimgrec_scronly.so"
BENCH_ARGS="--config 3" bash tools/pmc_clock.sh r06/clk2_cfg3 || exit 3
BENCH_ARGS="--config 2" bash tools/pmc_clock.sh r06/clk2_cfg2 || exit 4
