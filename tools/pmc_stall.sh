#!/bin/bash
# Where a kernel waits: one PMC pass of issue / L1-miss-queue counters over a
# command (default: bench.py).  Usage on the GPU box:
#   bash tools/pmc_stall.sh <out_name> [python args...]
set -u
export TMPDIR=/tmp
name=${1:-bench}; shift || true
args=${*:-bench.py --steps 5 --warmup 2 --no-cpu-baseline}
O=gpurun_out/stall_$name; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr -d $O -o pmc --output-format csv -- python3 $args > $O/run.log 2>&1
