#!/bin/bash
# Fresh PMC records for the bench kernel: HBM traffic (FETCH/WRITE passes) and clock / MFMA busy
set -u
TAG=${1:-r01_v16}
bash tools/pmc_traffic.sh $TAG && bash tools/pmc_clock.sh pmcclk_$TAG
