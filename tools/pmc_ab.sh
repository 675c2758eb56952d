#!/bin/bash
# PMC passes over an in-process A/B (tools/ab_tune.py): every configuration's
# main kernel gets the same counters in one process.  Usage (GPU box):
#   AB_ARGS='--configs "base;pair:flat_pair=1"' bash tools/pmc_ab.sh <tag>
set -u
export TMPDIR=/tmp
TAG=${1:-ab}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
AB="tools/ab_tune.py --rounds 1 --reps 3 ${AB_ARGS:-}"
pass() {  # name counters...
  local name=$1; shift
  echo "== $name"; date +%T
  eval timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_agg_" -d $OUT/$name -o pmc \
      --output-format csv -- python3 $AB > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
pass l2 TCC_HIT_sum TCC_MISS_sum
pass stall GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr
pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS
pass fetch FETCH_SIZE
find $OUT -name "*counter_collection.csv"
