#!/bin/bash
# Ablation + counter pass of the fused k-NN kernel.  Run on the GPU box via gpurun.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-abl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
B="python3 bench.py --profile-only --steps 5 --warmup 1 ${BENCH_ARGS:-}"
for v in libimgrec.so libimgrec_NO_DMA.so libimgrec_NO_EPILOGUE.so ${EXTRA_LIBS:-}; do
  IMGREC_LIB_NAME=$v timeout -k 10 200 $B > $OUT/abl_$v.json 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/abl_$v.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc FETCH_SIZE -d $OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex knn_tile --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL -d $OUT/pmc4 -o run --output-format csv -- $B > $OUT/pmc4.log 2>&1 || exit 5
python3 tools/pmc_summary.py $OUT
