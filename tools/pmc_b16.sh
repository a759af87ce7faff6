#!/bin/bash
# PMC passes on the fused kernel in a given mode (default bf16), one pass per counter group.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmcb16}; mkdir -p $OUT
B="python3 bench.py --profile-only --steps 3 --warmup 1 --mode ${MODE:-bf16}"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
R="--kernel-trace --kernel-include-regex knn_b16|knn_tile --output-format csv"
timeout -s KILL 120 rocprofv3 $R --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 $R --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 $R --pmc FETCH_SIZE -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 $R --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/p4 -o run -- $B > $OUT/p4.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 $R --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p5 -o run -- $B > $OUT/p5.log 2>&1 || exit 6
python3 tools/pmc_summary.py $OUT
