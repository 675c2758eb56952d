#!/bin/bash
# A/B: scalar slot batches for max/min (flat_smem_arg) at VEC 1/2, and the
# sum/mean VEC=1 default (flat_vec1_min_bytes 0 vs 1 GiB), RMAT21 and Reddit.
set -u
mkdir -p gpurun_out
o=gpurun_out/ab_smem_arg.log; : > $o
for G in reddit rmat21; do
  timeout -k 10 300 python tools/ab_tune.py --graph $G --reduce max --rounds 5 \
    --configs "base;sm2:flat_smem_arg=1;sm1:flat_smem_arg=1,flat_vec_arg=1" >> $o 2>&1 || exit $?
  timeout -k 10 300 python tools/ab_tune.py --graph $G --reduce sum --rounds 5 \
    --configs "base;old:flat_vec1_min_bytes=1073741824" >> $o 2>&1 || exit $?
done
timeout -k 10 300 python tools/ab_tune.py --graph products --reduce sum --rounds 3 \
    --configs "base;old:flat_vec1_min_bytes=1073741824" >> $o 2>&1 || exit $?
grep config $o | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['graph'], d['reduce'], d['F'], d['config'], d['median_ms'], d['fixup_ms'], d['bitwise_equal_to_base'], d['kernel'][:70])
"
