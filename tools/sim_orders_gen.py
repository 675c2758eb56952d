"""Destination-row processing orders for tools/sim_orders.c,
from the config-2 CSR written by tools/sim_l2_gen.py (/tmp/sim/col.bin,
rowptr.bin).  Each order is an int32 permutation of the rows -> /tmp/sim/order_<name>.bin:

  natural      CSR row order (what the kernel runs today)
  random       a random permutation (control)
  degree       in-degree descending
  rcm          reverse Cuthill-McKee of the symmetric adjacency (scipy): a
               bandwidth-reducing relabel computed once at CSR build
  minhash      rows sorted by two min-hashes of their source sets (rows sharing
               their minimum-hash source cluster together)
  hubkey       rows sorted by their most popular source, then the second
  srcsort      rows sorted by their smallest source id (a cheap locality key)
"""
import os
import sys
import time

import numpy as np

D = "/tmp/sim"
col = np.fromfile(os.path.join(D, "col.bin"), dtype=np.int32)
rowptr = np.fromfile(os.path.join(D, "rowptr.bin"), dtype=np.int32).astype(np.int64)
N = rowptr.size - 1
E = col.size
deg_in = np.diff(rowptr)
outdeg = np.bincount(col, minlength=N)


def save(name, perm):
    perm = np.asarray(perm, dtype=np.int32)
    assert perm.size == N and np.array_equal(np.sort(perm), np.arange(N, dtype=np.int32))
    perm.tofile(os.path.join(D, "order_%s.bin" % name))
    print("order", name, "written", flush=True)


def seg_min(vals):
    """per-row minimum of a per-slot int64 array (rows with no slot -> max)."""
    out = np.full(N, np.iinfo(np.int64).max, dtype=np.int64)
    # np.minimum.reduceat over the non-empty rows
    nz = deg_in > 0
    starts = rowptr[:-1][nz]
    out[nz] = np.minimum.reduceat(vals, starts)
    return out


names = sys.argv[1:] or ["natural", "random", "degree", "srcsort", "hubkey", "minhash", "rcm"]
for name in names:
    t0 = time.time()
    if name == "natural":
        save(name, np.arange(N))
    elif name == "random":
        save(name, np.random.default_rng(0).permutation(N))
    elif name == "degree":
        save(name, np.argsort(-deg_in, kind="stable"))
    elif name == "srcsort":
        save(name, np.argsort(seg_min(col.astype(np.int64)), kind="stable"))
    elif name == "hubkey":
        # most popular source of each row (ties: smaller id), then the row's second key
        pop = outdeg[col].astype(np.int64) * (1 << 22) + (np.int64(1 << 22) - 1 - col)
        best = -seg_min(-pop)                              # max popularity key per row
        hub = (np.int64(1 << 22) - 1) - (best & ((1 << 22) - 1))
        hub[deg_in == 0] = N
        save(name, np.lexsort((np.arange(N), hub)))
    elif name == "minhash":
        h1 = (col.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(20)
        h2 = (col.astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)) >> np.uint64(20)
        m1 = seg_min(h1.astype(np.int64))
        m2 = seg_min(h2.astype(np.int64))
        save(name, np.lexsort((m2, m1)))
    elif name == "rcm":
        import scipy.sparse as sp
        from scipy.sparse.csgraph import reverse_cuthill_mckee
        A = sp.csr_matrix((np.ones(E, dtype=np.int8), col, rowptr), shape=(N, N))
        save(name, reverse_cuthill_mckee(A, symmetric_mode=True))
    print("  %.1f s" % (time.time() - t0), flush=True)
