#!/bin/bash
# A/B of the v_med3 list insertion (default lib) vs the select form (nomed3), at 1M and 125k rows
set -u
L="${L:-libimgrec.so libimgrec_nomed3.so libimgrec.so libimgrec_nomed3.so}"
LIBS="$L" bash tools/ab_b16.sh ab_med3_1m && LIBS="$L" BENCH_ARGS="--rows 125000 --steps 50 --warmup 5" bash tools/ab_b16.sh ab_med3_125k
