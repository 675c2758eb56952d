#!/bin/bash
# PMC passes over tools/dbg/gemm_pmc_drive.py -> gpurun_out/gemm_pmc/
set -u
export TMPDIR=/tmp
OUT=gpurun_out/gemm_pmc
mkdir -p $OUT
D="python3 tools/dbg/gemm_pmc_drive.py"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $D > $OUT/kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $OUT/p1 -o pmc --output-format csv -- $D > $OUT/p1.log 2>&1
echo rc=$?
