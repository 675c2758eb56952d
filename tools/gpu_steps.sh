#!/bin/bash
# GPU-box helper: run named steps, each under its own time limit, stop at the
# first crash-type exit.  Usage: bash tools/gpu_steps.sh "<name>|<timeout>|<cmd>" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($t s)"; date +%T
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
