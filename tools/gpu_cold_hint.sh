mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for g in products rmat21_flat rmat21 rmat21_deg15; do timeout -k 10 200 python tools/bench_graph.py --graph $g > gpurun_out/bg_$g.log 2>&1 || exit 1; grep '^{' gpurun_out/bg_$g.log; done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
cut -c1-600 gpurun_out/bench.log | tail -n 1
timeout -k 10 600 python tools/bench_configs.py --configs c5 > gpurun_out/c5.jsonl 2>gpurun_out/c5.err || exit 1
cut -c1-500 gpurun_out/c5.jsonl
