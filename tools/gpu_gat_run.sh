set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gat or GAT" -p no:cacheprovider > gpurun_out/pytest_gat.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gat.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_gat_tile.py --vecs 0,4,2 > gpurun_out/ab_gat_tile.log 2>&1
rc=$?; cat gpurun_out/ab_gat_tile.log | grep -v amdgpu.ids; exit $rc
