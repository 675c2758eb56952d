#!/bin/bash
# Flat-kernel shape A/Bs over mid-width rows: lane width
# (VEC 1/2/4) and flat vs k_agg_main for sum and max/min.  GPU box:
#   bash tools/ab_advice.sh  -> gpurun_out/ab_advice.log (one JSON line per config)
set -u
mkdir -p gpurun_out
o=gpurun_out/ab_advice.log; : > $o
BIG=1000000000000000
for F in 130 200 250; do
  timeout -k 10 200 python tools/ab_tune.py --reduce max --F $F --rounds 5 \
    --configs "base;v1:flat_vec_arg=1;v4:flat_vec_arg=4;main:flat_min_f_arg=512" >> $o 2>&1 || exit $?
  timeout -k 10 200 python tools/ab_tune.py --reduce sum --F $F --rounds 5 \
    --configs "base;v2:flat_vec1_min_bytes=$BIG;v4:flat_vec=4,flat_vec1_min_bytes=$BIG;main:flat_min_f=512" >> $o 2>&1 || exit $?
done
grep config $o | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['graph'], d['reduce'], d['F'], d['config'], d['median_ms'], d['fixup_ms'], d['bitwise_equal_to_base'], d['kernel'][:60])
"
