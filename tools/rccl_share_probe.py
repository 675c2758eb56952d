"""Probe: can two ranks on ONE GPU form an RCCL communicator?  (The GPU box has
one device; bench.py --gpus N uses RCCL all_to_all_single for the halo.)
Run: python tools/rccl_share_probe.py  -> prints one line per rank."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    x = torch.arange(4 * world, dtype=torch.float32, device="cuda") + 100 * rank
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x)
    torch.cuda.synchronize()
    print("rank", rank, "ok", y.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.spawn(_worker, args=(world, port), nprocs=world, join=True)
