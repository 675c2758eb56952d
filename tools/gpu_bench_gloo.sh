#!/bin/bash
# bench.py's multi-rank path at full config-2 size as gloo ranks sharing the one GPU
# (halo rows staged through the host: the exchange time is not xGMI's; the per-rank
# send / interior / boundary HIP events and the cover's row counts are the point)
set -u
mkdir -p gpurun_out
for P in ${PARTS:-2 4}; do
  echo "== P=$P"; date +%T
  MP_BENCH_BACKEND=gloo timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $P \
    --master-addr 127.0.0.1 --master-port $((29500 + P)) bench.py --gpus $P --steps 5 --warmup 2 \
    > gpurun_out/bench_gloo$P.jsonl 2> gpurun_out/bench_gloo$P.err
  rc=$?; echo "P=$P rc=$rc"; grep '^{' gpurun_out/bench_gloo$P.jsonl | cut -c1-300
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_gloo$P.err; exit $rc; }
done
