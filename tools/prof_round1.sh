#!/bin/bash
# Counter + ablation pass for the fused k-NN kernel (round 1).  Run on the GPU box via gpurun.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1prof; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
B="python3 bench.py --profile-only --steps 3 --warmup 1"
for v in libimgrec.so libimgrec_NO_GLOBAL.so libimgrec_NO_EPILOGUE.so; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 $B > $OUT/abl_$v.json 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc FETCH_SIZE -d $OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc3 -o run --output-format csv -- $B > $OUT/pmc3.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $OUT/pmc4 -o run --output-format csv -- $B > $OUT/pmc4.log 2>&1 || exit 5
echo done
