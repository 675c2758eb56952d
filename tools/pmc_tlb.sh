#!/bin/bash
# Address-translation (UTCL1 / UTCL2) counters of the main kernel, one PMC pass
# per group (each group within the TCP block's 4-counter limit).  Usage on the GPU box:
#   bash tools/pmc_tlb.sh <out_name> [python args...]
# then: python tools/tlb_summary.py gpurun_out/tlb_<out_name>
set -u
export TMPDIR=/tmp
name=${1:-bench}; shift || true
args=${*:-bench.py --steps 5 --warmup 2 --no-cpu-baseline}
O=gpurun_out/tlb_$name; mkdir -p $O
pass() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $O/$tag -o pmc --output-format csv -- python3 $args > $O/$tag.log 2>&1
  local rc=$?
  echo "tlb pass $tag rc=$rc"
  return $rc
}
pass p1 GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum &&
pass p2 GRBM_GUI_ACTIVE TCP_UTCL1_SERIALIZATION_STALL TCP_UTCL1_STALL_INFLIGHT_MAX TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS &&
pass p3 GRBM_GUI_ACTIVE TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS TCP_CLIENT_UTCL1_INFLIGHT TCP_UTCL1_THRASHING_STALL TCP_UTCL1_LFIFO_FULL
