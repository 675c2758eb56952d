#!/bin/bash
# Cold-source cache-policy A/B: tools/variants/lib_cold<v>.so
# (make variant NAME=coldnt DEFS=-DMP_COLD_TAG_AUX=2; sc1 = 16, nt+sc1 = 18)
# with the sources of out-degree <= T sign-tagged by tools/bench_graph.py
# (MP_COLD_TAG_T), every measurement its own process, rounds interleaved.
set -e
L=pytorch_geometric-1_amd/mi355_mp/libmi355_mp.so
cp $L /tmp/lib_default.so
G=${G:-rmat21}
for r in 1 2; do
  timeout -k 10 200 python tools/bench_graph.py --graph $G > gpurun_out/ct_base.log 2>&1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ct_base.log') if l.startswith('{')][0]); print('round $r $G base main %.3f ms' % d['main_ms'])"
  for v in ${V:-nt sc1 ntsc1}; do
    for t in ${T:-32 128}; do
      cp tools/variants/lib_cold$v.so $L
      MP_COLD_TAG_T=$t timeout -k 10 200 python tools/bench_graph.py --graph $G > gpurun_out/ct_${v}_$t.log 2>&1 || { cp /tmp/lib_default.so $L; exit 1; }
      python -c "import json; d=json.loads([l for l in open('gpurun_out/ct_${v}_$t.log') if l.startswith('{')][0]); print('round $r $G cold<=$t aux=$v main %.3f ms' % d['main_ms'])"
      grep "cold tag" gpurun_out/ct_${v}_$t.log || true
    done
  done
  cp /tmp/lib_default.so $L
done
