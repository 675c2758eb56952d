"""Model of the halo exchange volume of the destination-range shards
against a hybrid exchange: for every ordered rank pair (q -> p), the cross
edges (source owned by q, destination owned by p) must be covered either by
shipping x_j of the source (pull, today) or by shipping q's partial sum of the
destination row (push).  The fewest rows = a minimum vertex cover of the
bipartite cross-edge graph (Konig: = maximum matching, scipy Hopcroft-Karp).

CPU only; prints rows per pair for pull-only, push-only, the
higher-degree-endpoint heuristic and the exact minimum cover.

  python tools/exp_halo_cover.py --scale 21 --samples 30000000 --parts 2 4 8
"""
import argparse
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import maximum_bipartite_matching

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pytorch_geometric-1_amd"))


def cuts_of(deg, parts):
    cs = np.cumsum(deg)
    tot = cs[-1]
    cuts = [0]
    for p in range(1, parts):
        c = int(np.searchsorted(cs, tot * p / parts, side="left")) + 1
        cuts.append(max(c, cuts[-1]))
    cuts.append(len(deg))
    return cuts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=21)
    ap.add_argument("--samples", type=int, default=30_000_000)
    ap.add_argument("--parts", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--row-bytes", type=int, default=1024)
    ap.add_argument("--exact", action="store_true", help="also the exact minimum cover (slow at P=2)")
    a = ap.parse_args()
    import torch
    from mi355_mp.graphgen import rmat_edge_index
    t = time.time()
    ei = rmat_edge_index(scale=a.scale, n_samples=a.samples, seed=1).numpy()
    N = 1 << a.scale
    src, dst = ei[0], ei[1]
    keep = src != dst
    src, dst = src[keep], dst[keep]
    print("# RMAT scale %d, %d edges without loops (%.1f s)" % (a.scale, src.size, time.time() - t), flush=True)
    deg = np.bincount(dst, minlength=N) + 1
    for P in a.parts:
        cuts = np.array(cuts_of(deg, P))
        own_s = np.searchsorted(cuts[1:], src, side="right")
        own_d = np.searchsorted(cuts[1:], dst, side="right")
        tot = {"pull": 0, "push": 0, "heur": 0, "exact": 0}
        worst = {"pull": 0, "push": 0, "heur": 0, "exact": 0}
        for p in range(P):
            into = (own_d == p) & (own_s != p)
            for k in ("pull", "push", "heur", "exact"):
                per_rank = 0
                for q in range(P):
                    if q == p:
                        continue
                    m = into & (own_s == q)
                    s, d = src[m], dst[m]
                    if s.size == 0:
                        continue
                    us, si = np.unique(s, return_inverse=True)
                    ud, di = np.unique(d, return_inverse=True)
                    if k == "pull":
                        r = us.size
                    elif k == "push":
                        r = ud.size
                    elif k == "heur":
                        # higher cross-degree endpoint covers the edge; ties -> source
                        ds = np.bincount(si)[si]
                        dd = np.bincount(di)[di]
                        pick_s = ds >= dd
                        # refinement 1: an edge whose source is pulled anyway is pulled
                        in_s = np.zeros(us.size, bool)
                        in_s[si[pick_s]] = True
                        push = ~in_s[si]
                        # refinement 2: an edge whose destination is pushed anyway is pushed
                        in_d = np.zeros(ud.size, bool)
                        in_d[di[push]] = True
                        pull = ~in_d[di]
                        r = np.unique(si[pull]).size + int(in_d.sum())
                    else:
                        if not a.exact:
                            continue
                        g = sp.csr_matrix((np.ones(si.size, np.int8), (si, di)), shape=(us.size, ud.size))
                        g.sum_duplicates()
                        mt = maximum_bipartite_matching(g, perm_type="column")
                        r = int((mt >= 0).sum())
                    per_rank += r
                    worst[k] = max(worst[k], r)
                tot[k] = max(tot[k], per_rank)
        gb = a.row_bytes / 1e9
        print("P=%d  max rows in per rank: pull %d (%.3f GB)  push %d  heuristic %d (%.3f GB, %.2fx pull)%s   "
              "largest pair: pull %.3f GB heuristic %.3f GB" % (
                  P, tot["pull"], tot["pull"] * gb, tot["push"], tot["heur"], tot["heur"] * gb,
                  tot["heur"] / max(1, tot["pull"]),
                  ("  exact cover %d (%.2fx)" % (tot["exact"], tot["exact"] / max(1, tot["pull"]))) if a.exact else "",
                  worst["pull"] * gb, worst["heur"] * gb), flush=True)


if __name__ == "__main__":
    main()
