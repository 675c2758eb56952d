mkdir -p gpurun_out
timeout -k 10 120 env GPU_MAX_HW_QUEUES=1 python tools/exp_interior.py > gpurun_out/r06_exp_interior_q1.jsonl 2> gpurun_out/r06_exp_interior_q1.err
pids=""
for i in 1 2 3 4 5 6 7; do
  timeout -k 5 90 env GPU_MAX_HW_QUEUES=1 python -c "import torch,time; t=torch.empty(1<<28, device='cuda'); t.fill_(1); torch.cuda.synchronize(); time.sleep(45)" &
  pids="$pids $!"
done
sleep 20
timeout -k 10 120 env GPU_MAX_HW_QUEUES=1 python tools/exp_interior.py > gpurun_out/r06_exp_interior_q1_siblings.jsonl 2> gpurun_out/r06_exp_interior_q1_siblings.err
rc=$?
wait $pids
exit $rc
