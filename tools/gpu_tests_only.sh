#!/bin/bash
# GPU-box run: the GPU test suite only (optionally -k filtered by PYTEST_K)
set -u
mkdir -p gpurun_out
PT="python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25"
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 1000 $PT -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 1000 $PT > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25; exit $rc
