#!/bin/bash
# Cold-sources hint check on more graphs: each graph with the far-x
# batch depth pinned to 6 and to 8 (tools/bench_graph.py --force-u), every
# measurement its own process, two interleaved rounds.
set -e
for r in 1 2; do
  for g in ${GRAPHS:-products_deg25 rmat22 rmat22_deg30 products rmat21}; do
    for u in 6 8; do
      timeout -k 10 200 python tools/bench_graph.py --graph $g --force-u $u > gpurun_out/hg_${g}_$u.log 2>&1
      python -c "import json; d=json.loads([l for l in open('gpurun_out/hg_${g}_$u.log') if l.startswith('{')][0]); print('round $r %-15s deg %5.1f hot %.3f U=$u main %.3f ms' % (d['graph'], d['avg_degree'], d['hot_share'], d['main_ms']), flush=True)"
    done
  done
done
