#!/bin/bash
# One GPU-box session of the round's measurements; every step under its own
# time limit, the session stops at the first failing step.  Outputs under
# gpurun_out/ (copied into profiles/ as rNN_* when they are kept):
#   STEPS="tests bench rccl gloo2 gat_gloo2 prof train" R=r05 bash tools/gpu_round.sh
#   tests     pytest -m gpu                           -> $R_pytest_gpu.txt
#   bench     python bench.py (the driver's N=1 line)  -> $R_bench_rmat21.json
#   bench_gat / bench_products / bench_reddit  the other workloads at N=1 (--verify)
#   configs   tools/bench_configs.py (configs 3 / 4 / 5, layer steps, Cora graph) -> $R_bench_configs.jsonl
#   rccl      one RCCL rank, --sharded --emulate-peers 8,4,2 (RCCL beside the aggregation),
#             rocprofv3 kernel trace of the same command -> $R_bench_sharded_rccl_one_rank.json,
#             $R_rccl_kernel_trace/ (+ tools/kernel_overlap.py summary)
#   rccl_products  the same for config 5 (P = 8, 4, 2) -> $R_bench_sharded_rccl_one_rank_products.json
#   gloo2     bench.py --gpus 2, gloo ranks sharing the GPU (--verify) -> $R_bench_rmat21_gloo2_rehearsal.json
#   gloo8 / gloo4  bench.py --gpus 8 / 4 as gloo ranks sharing the GPU (per-rank compute_in_turn:
#             each rank's compute with the GPU to itself) -> $R_bench_rmat21_gloo{8,4}_rehearsal.json;
#             one hardware queue per process (GPU_MAX_HW_QUEUES=1): 4 x 4 queues oversubscribe the
#             GPU's queue slots and stretch a 1 s build to 60 s
#   products_gloo2 / products_gloo4 / products_gloo8  config 5 (--workload products) as 4 / 8 gloo ranks sharing the GPU (--verify)
#   gat_gloo2 the same for --workload gat                -> $R_bench_gat_gloo2_rehearsal.json
#   gat_drop_gloo2  the same with attention dropout 0.3 over the cover (--verify with the keep mask)
#   prof      tools/profile.sh (kernel trace + PMC of the default bench); prof_gat / prof_products /
#             prof_reddit the same for the other bench workloads (summarise with tools/pmc_summary.py)
#   diag      tools/gat_shard_diag.py (sharded vs single-GPU vs float64 GAT gradients, per seed)
#   train     kernel trace of the GCNConv / GATConv layer training steps (tools/bench_configs.py)
set -u
export TMPDIR=/tmp
R=${R:-r06}
O=gpurun_out
mkdir -p $O
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in ${STEPS:-tests bench}; do
  case $s in
    tests) run tests 900 bash -c "python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/${R}_pytest_gpu.txt 2>&1"; tail -3 $O/${R}_pytest_gpu.txt ;;
    bench) run bench 400 bash -c "python bench.py > $O/${R}_bench_rmat21.json 2> $O/${R}_bench_rmat21.err"; cut -c1-400 $O/${R}_bench_rmat21.json ;;
    bench_gat) run bench_gat 400 bash -c "python bench.py --workload gat --verify > $O/${R}_bench_gat_n1.json 2> $O/${R}_bench_gat_n1.err"; cut -c1-300 $O/${R}_bench_gat_n1.json ;;
    bench_products) run bench_products 500 bash -c "python bench.py --workload products --verify > $O/${R}_bench_products_n1.json 2> $O/${R}_bench_products_n1.err"; cut -c1-300 $O/${R}_bench_products_n1.json ;;
    bench_reddit) run bench_reddit 500 bash -c "python bench.py --workload reddit --verify > $O/${R}_bench_reddit_n1.json 2> $O/${R}_bench_reddit_n1.err"; cut -c1-300 $O/${R}_bench_reddit_n1.json ;;
    configs) run configs 700 bash -c "python tools/bench_configs.py --cpu-baseline > $O/${R}_bench_configs.jsonl 2> $O/${R}_bench_configs.err"; cut -c1-200 $O/${R}_bench_configs.jsonl ;;
    rccl) run rccl 500 bash -c "python bench.py --sharded --emulate-peers 8,4,2 --steps 10 --warmup 3 --verify > $O/${R}_bench_sharded_rccl_one_rank.json 2> $O/${R}_bench_sharded_rccl_one_rank.err"
          run rccl_trace 500 rocprofv3 --kernel-trace --stats -d $O/${R}_rccl_kt -o kt --output-format csv -- python3 bench.py --sharded --emulate-peers 8,4,2 --steps 5 --warmup 2 --no-cpu-baseline --no-ref-paths --no-build-split
          python3 tools/kernel_overlap.py $O/${R}_rccl_kt > $O/${R}_rccl_kernel_overlap.json; cat $O/${R}_rccl_kernel_overlap.json | head -40 ;;
    rccl_products) run rccl_products 500 bash -c "python bench.py --workload products --sharded --emulate-peers 8,4,2 --steps 10 --warmup 3 --verify > $O/${R}_bench_sharded_rccl_one_rank_products.json 2> $O/${R}_bench_sharded_rccl_one_rank_products.err" ;;
    gloo2) run gloo2 600 bash -c "MP_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 --verify > $O/${R}_bench_rmat21_gloo2_rehearsal.json 2> $O/${R}_bench_rmat21_gloo2_rehearsal.err"; cut -c1-300 $O/${R}_bench_rmat21_gloo2_rehearsal.json ;;
    gloo8) run gloo8 1100 bash -c "GPU_MAX_HW_QUEUES=1 MP_BENCH_BACKEND=gloo python bench.py --gpus 8 --steps 3 --warmup 1 > $O/${R}_bench_rmat21_gloo8_rehearsal.json 2> $O/${R}_bench_rmat21_gloo8_rehearsal.err"; cut -c1-300 $O/${R}_bench_rmat21_gloo8_rehearsal.json ;;
    gloo4) run gloo4 900 bash -c "GPU_MAX_HW_QUEUES=1 MP_BENCH_BACKEND=gloo python bench.py --gpus 4 --steps 3 --warmup 1 > $O/${R}_bench_rmat21_gloo4_rehearsal.json 2> $O/${R}_bench_rmat21_gloo4_rehearsal.err"; cut -c1-300 $O/${R}_bench_rmat21_gloo4_rehearsal.json ;;
    products_gloo4) run products_gloo4 1100 bash -c "GPU_MAX_HW_QUEUES=1 MP_BENCH_BACKEND=gloo python bench.py --workload products --gpus 4 --steps 3 --warmup 1 --verify > $O/${R}_bench_products_gloo4_rehearsal.json 2> $O/${R}_bench_products_gloo4_rehearsal.err"; cut -c1-300 $O/${R}_bench_products_gloo4_rehearsal.json ;;
    products_gloo2) run products_gloo2 900 bash -c "MP_BENCH_BACKEND=gloo python bench.py --workload products --gpus 2 --steps 3 --warmup 1 --verify > $O/${R}_bench_products_gloo2_rehearsal.json 2> $O/${R}_bench_products_gloo2_rehearsal.err"; cut -c1-300 $O/${R}_bench_products_gloo2_rehearsal.json ;;
    products_gloo8) run products_gloo8 1150 bash -c "GPU_MAX_HW_QUEUES=1 MP_BENCH_BACKEND=gloo python bench.py --workload products --gpus 8 --steps 3 --warmup 1 --verify > $O/${R}_bench_products_gloo8_rehearsal.json 2> $O/${R}_bench_products_gloo8_rehearsal.err"; cut -c1-300 $O/${R}_bench_products_gloo8_rehearsal.json ;;
    gat_gloo2) run gat_gloo2 600 bash -c "MP_BENCH_BACKEND=gloo python bench.py --gpus 2 --workload gat --steps 3 --warmup 1 --verify > $O/${R}_bench_gat_gloo2_rehearsal.json 2> $O/${R}_bench_gat_gloo2_rehearsal.err"; cut -c1-300 $O/${R}_bench_gat_gloo2_rehearsal.json ;;
    gat_drop_gloo2) run gat_drop_gloo2 600 bash -c "MP_BENCH_BACKEND=gloo python bench.py --gpus 2 --workload gat --gat-dropout 0.3 --steps 3 --warmup 1 --verify > $O/${R}_bench_gat_dropout_gloo2_rehearsal.json 2> $O/${R}_bench_gat_dropout_gloo2_rehearsal.err"; cut -c1-300 $O/${R}_bench_gat_dropout_gloo2_rehearsal.json ;;
    gat_drop_gloo4) run gat_drop_gloo4 900 bash -c "GPU_MAX_HW_QUEUES=1 MP_BENCH_BACKEND=gloo python bench.py --gpus 4 --workload gat --gat-dropout 0.3 --steps 3 --warmup 1 --verify > $O/${R}_bench_gat_dropout_gloo4_rehearsal.json 2> $O/${R}_bench_gat_dropout_gloo4_rehearsal.err"; cut -c1-300 $O/${R}_bench_gat_dropout_gloo4_rehearsal.json ;;
    diag) run diag 500 bash -c "python tools/gat_shard_diag.py > $O/${R}_gat_shard_diag.jsonl 2> $O/${R}_gat_shard_diag.err"; cat $O/${R}_gat_shard_diag.jsonl ;;
    prof) PROF_OUT=$O/${R}_prof run prof 1100 bash tools/profile.sh ;;
    prof_gat) PROF_OUT=$O/${R}_prof_gat NO_CALIB=1 BENCH_ARGS="--workload gat" run prof_gat 1100 bash tools/profile.sh ;;
    prof_products) PROF_OUT=$O/${R}_prof_products NO_CALIB=1 BENCH_ARGS="--workload products" run prof_products 1100 bash tools/profile.sh ;;
    prof_reddit) PROF_OUT=$O/${R}_prof_reddit NO_CALIB=1 BENCH_ARGS="--workload reddit" run prof_reddit 1100 bash tools/profile.sh ;;
    train) run train 500 rocprofv3 --kernel-trace --stats -d $O/${R}_train_kt -o kt --output-format csv -- python3 tools/bench_configs.py --configs c2train,c3train ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
