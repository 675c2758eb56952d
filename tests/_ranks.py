"""Multi-process rank runner for the distributed tests (gloo on the CPU, or
ranks sharing one GPU).

run_ranks() fails the CALLING TEST by name, with its own deadline, before
pytest-timeout's global backstop (pytest.ini) would fire: the first rank to
exit non-zero, or the deadline, terminates every rank still alive (a rank
stuck in a collective whose peer died would otherwise sit until the process
group's timeout), then kills what ignores the terminate.  No rank outlives
the test, so no orphan holds the GPU or a port."""
import socket
import time

import torch.multiprocessing as mp

# below pytest.ini's 600 s per-test backstop, which aborts the whole session
DEFAULT_TIMEOUT = 420


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(target, world=2, timeout=DEFAULT_TIMEOUT, args=()):
    """Run target(rank, world, port, q, *args) in `world` spawned processes and
    return the sorted items each rank put on q (one per rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + tuple(args)) for r in range(world)]
    for p in procs:
        p.start()
    deadline = time.monotonic() + timeout
    try:
        while any(p.is_alive() for p in procs):
            bad = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not bad, "a rank exited with %s" % bad
            assert time.monotonic() < deadline, "ranks still running after %d s" % timeout
            time.sleep(0.1)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        return sorted(q.get(timeout=10) for _ in range(world))
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join(5)
