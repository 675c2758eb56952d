#!/bin/bash
# Merge-path task size sweep of the default kernel (RMAT21, products-scale).
set -u
mkdir -p gpurun_out
o=gpurun_out/ab_chunk.log; : > $o
for C in 256 512 1024 2048; do
  timeout -k 10 300 python tools/ab_tune.py --chunk $C --configs "base" --rounds 3 >> $o 2>&1 || exit 1
done
for C in 512 1024 2048; do
  timeout -k 10 300 python tools/ab_tune.py --graph products --chunk $C --configs "base" --rounds 3 >> $o 2>&1 || exit 1
done
grep config $o | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['graph'], d['chunk'], d['median_ms'], d['fixup_ms'])
"
