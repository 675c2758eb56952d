#!/bin/bash
# One GPU call, round 4: the GPU suite + smoke + default bench (tools/gpu_check.sh),
# then the other bench workloads at N = 1 (config 5 products, config 3 GAT, config 4 max), the
# config-5 workload as bench.py's own 2-rank launch (gloo ranks sharing the GPU,
# --verify), and every other config / layer (tools/bench_configs.py) -- the
# inputs of DESIGN.md section 2.  Each step under its own time limit; a
# crash-type exit ends the call.
set -u
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
cp gpurun_out/bench.log gpurun_out/bench_rmat21.log
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "$name rc=$rc"; grep '^{' "gpurun_out/$name.json" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$name.err"; echo "STOP after $name"; exit $rc; fi
}
step bench_products_n1 300 python -u bench.py --workload products --steps 20 --warmup 5 --verify
step bench_gat_n1 300 python -u bench.py --workload gat --steps 20 --warmup 5 --verify
step bench_reddit_n1 300 python -u bench.py --workload reddit --steps 20 --warmup 5 --verify
MP_BENCH_BACKEND=gloo step bench_products_gloo2 400 python -u bench.py --gpus 2 --workload products --steps 5 \
  --warmup 2 --no-cpu-baseline --no-ref-paths --verify
echo "== bench_configs"; date +%T
timeout -k 10 700 python tools/bench_configs.py --cpu-baseline > gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_configs.err
rc=$?
echo "bench_configs rc=$rc"; cut -c1-300 gpurun_out/bench_configs.jsonl
exit $rc
