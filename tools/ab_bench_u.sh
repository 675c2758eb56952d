#!/bin/bash
# Batch depth U of the far-x sum kernel swapped by library
# (tools/variants/lib_far<U>.so: make variant NAME=far<U> DEFS=-DMP_U_VEC1_FAR=<U>),
# every measurement its own process (bench.py's setup: tools/bench_graph.py),
# rounds interleaved:   bash tools/ab_bench_u.sh "6 8" "rmat21 products"
set -e
L=pytorch_geometric-1_amd/mi355_mp/libmi355_mp.so
cp $L /tmp/lib_default.so
for r in 1 2; do
  for g in ${2:-rmat21 products}; do
    for u in ${1:-6 8}; do
      cp tools/variants/lib_far$u.so $L
      timeout -k 10 200 python tools/bench_graph.py --graph $g > gpurun_out/bg_${g}_u$u.log 2>&1
      python -c "import json; d=json.loads([l for l in open('gpurun_out/bg_${g}_u$u.log') if l.startswith('{')][0]); print('round $r %-13s deg %5.1f U=$u main %.3f ms fixup %.3f' % (d['graph'], d['avg_degree'], d['main_ms'], d['fixup_ms']))"
    done
  done
done
cp /tmp/lib_default.so $L
