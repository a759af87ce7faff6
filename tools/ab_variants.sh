# A/B of library variants (tools/build_variants.sh): bf16 parity tests on TEST_LIBS, per-tile
# stamps (tools/b16_stamps.py) of STAMP_LIBS, two interleaved timing rounds of TIME_LIBS.
set -u
mkdir -p gpurun_out/ab
for v in $TEST_LIBS; do IMGREC_LIB_NAME=$v timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -30 gpurun_out/ab/pytest_$v.log; exit 1; }; echo "$v $(tail -1 gpurun_out/ab/pytest_$v.log)"; done
for v in $STAMP_LIBS; do IMGREC_LIB_NAME=$v timeout -k 10 300 python3 tools/b16_stamps.py > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.txt || exit 1; done
for r in 1 2; do for v in $TIME_LIBS; do IMGREC_LIB_NAME=$v timeout -k 10 200 python3 bench.py --profile-only --steps 10 --warmup 2 2>/dev/null | tail -1 | sed "s/^/$v /" || exit 1; done; done
