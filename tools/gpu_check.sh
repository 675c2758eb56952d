#!/bin/bash
# GPU-box run: parity tests, smoke, bench.  Stops at the first crash-type
# exit (abort / segfault / timeout); plain test failures (rc 1) continue.
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
{ nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > gpurun_out/host_probe.log 2>&1
PT="python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread --durations=25"
if [ -n "${PYTEST_K:-}" ]; then
  step pytest_gpu 1100 $PT -k "$PYTEST_K"
else
  step pytest_gpu 1100 $PT
fi
if [ -z "${NO_BENCH:-}" ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 600 python bench.py --steps 20 --warmup 5
fi
