#!/bin/bash
# One GPU call: parity suite + smoke + bench (tools/gpu_check.sh), then every
# other config's benchmark with CPU baselines -> gpurun_out/bench_configs.jsonl
set -u
bash tools/gpu_check.sh || exit $?
echo "== bench_configs"; date +%T
timeout -k 10 900 python tools/bench_configs.py --cpu-baseline > gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_configs.err
rc=$?
echo "bench_configs rc=$rc"; tail -c 1500 gpurun_out/bench_configs.jsonl
exit $rc
