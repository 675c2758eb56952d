#!/bin/bash
# rocprofv3 on the GPU box: kernel-trace stats of bench.py, then separate PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) restricted
# to the dominant kernel.  Outputs under $PROF_OUT (default gpurun_out/prof/);
# BENCH_ARGS is appended to the bench command (e.g. --workload products);
# NO_CALIB=1 skips the FETCH_SIZE calibration pass.
set -u
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
}
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref-paths ${BENCH_ARGS:-}"
run kt 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $B
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 $B
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_write -o pmc --output-format csv -- python3 $B
run pmc_stall 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_stall -o pmc --output-format csv -- python3 $B
run pmc_l2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_l2 -o pmc --output-format csv -- python3 $B
# memory-side requests: DRAM-targeted reads (Infinity-Cache hits still counted), DRAM credit
# stalls (fabric back-pressure), accumulated L2 read latency
run pmc_ea 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_READ_REQ_LATENCY_sum --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_ea -o pmc --output-format csv -- python3 $B
run pmc_lat 600 rocprofv3 --pmc TCC_READ_REQ_sum TCC_TAG_STALL_sum TCC_LATENCY_FIFO_FULL_sum TCC_BUSY_sum --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_lat -o pmc --output-format csv -- python3 $B

[ -z "${NO_CALIB:-}" ] && run pmc_calib 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_agg_(main|flat)" -d $OUT/pmc_calib -o pmc --output-format csv -- python3 tools/pmc_calibrate.py
find $OUT -name "*.csv"
