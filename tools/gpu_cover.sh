set -u
mkdir -p gpurun_out
[ -n "${NO_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "cover or bench_multi_rank or overlapped" > gpurun_out/cover_tests.log 2>&1
rc=$?; [ -n "${NO_TESTS:-}" ] || tail -8 gpurun_out/cover_tests.log; [ $rc -eq 0 ] || exit $rc
for P in ${PARTS:-2 4 8}; do
  timeout -k 10 400 python -u tools/exp_halo_cover_gpu.py --parts $P > gpurun_out/cover_p$P.jsonl 2> gpurun_out/cover_p$P.err || { echo "P=$P failed"; tail -20 gpurun_out/cover_p$P.err; exit 1; }
  cat gpurun_out/cover_p$P.jsonl
done
