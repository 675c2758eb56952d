#!/bin/bash
# rocprofv3 of the GATConv(256, 32, heads=8) training step on the config-3
# graph (tools/bench_configs.py c3train): kernel-trace stats, then one PMC
# pass per counter group restricted to the fused forward / backward main
# kernels (k_agg_main<GatRed..> / k_agg_main<GatBwdRed..>).  Outputs under
# gpurun_out/prof_gat/; summarise with tools/pmc_gat_summary.py.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof_gat
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
}
C="tools/bench_configs.py --configs ${GAT_CONFIG:-c3train}"
RX="k_agg_main<mp::Gat(Bwd)?Red"
run kt 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $C
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 $C
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $OUT/pmc_write -o pmc --output-format csv -- python3 $C
run pmc_l2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" -d $OUT/pmc_l2 -o pmc --output-format csv -- python3 $C
run pmc_stall 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --kernel-include-regex "$RX" -d $OUT/pmc_stall -o pmc --output-format csv -- python3 $C
find $OUT -name "*.csv" | head -20
