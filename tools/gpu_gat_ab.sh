set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gat or GAT" -p no:cacheprovider > gpurun_out/pytest_gat.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gat.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gat -o run -- python -u tools/bench_configs.py --configs c3train > gpurun_out/c3train.jsonl 2>&1
rc=$?; grep '^{' gpurun_out/c3train.jsonl | cut -c1-400; exit $rc
