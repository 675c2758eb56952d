"""Seeded synthetic graphs for the BASELINE.md configs (no datasets offline).

  rmat_edge_index     RMAT (Graph500-style) -- config 2/3: scale 21,
                      (a,b,c,d) = (.57,.19,.19,.05), 30M samples symmetrised
  powerlaw_edge_index RMAT mapped into [0, N) -- configs 4/5 (Reddit- and
                      ogbn-products-scale node counts)
  cora_like           Cora-shaped planetoid stand-in -- config 1

Generation runs with torch ops on the requested device (GPU for the bench
sizes; the CPU gives the same edges for the same seed only when generated
on the CPU -- tests generate on the CPU and copy).
"""
import math

import torch


def _rmat_pairs(scale, n_samples, a, b, c, gen, device, chunk=1 << 24):
    srcs, dsts = [], []
    ab, abc = a + b, a + b + c
    done = 0
    while done < n_samples:
        n = min(chunk, n_samples - done)
        src = torch.zeros(n, dtype=torch.int64, device=device)
        dst = torch.zeros(n, dtype=torch.int64, device=device)
        for _ in range(scale):
            r = torch.rand(n, generator=gen, device=device)
            sbit = (r >= ab).to(torch.int64)
            dbit = ((r >= a) & (r < ab)) | (r >= abc)
            src = src * 2 + sbit
            dst = dst * 2 + dbit.to(torch.int64)
        srcs.append(src)
        dsts.append(dst)
        done += n
    return torch.cat(srcs), torch.cat(dsts)


def rmat_edge_index(scale=21, n_samples=30_000_000, abcd=(0.57, 0.19, 0.19, 0.05), seed=1, device="cpu",
                    symmetric=True, permute=True, num_nodes=None):
    """[2, E] int64 edge_index; E = 2*n_samples when symmetric (duplicates kept,
    RMAT self loops kept -- GCNConv's add_remaining_self_loops removes them)."""
    a, b, c, _ = abcd
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    src, dst = _rmat_pairs(scale, n_samples, a, b, c, gen, device)
    N = 1 << scale
    if num_nodes is not None and num_nodes < N:
        src = src % num_nodes
        dst = dst % num_nodes
        N = num_nodes
    if permute:
        perm = torch.randperm(N, generator=gen, device=device)
        src = perm[src]
        dst = perm[dst]
    if symmetric:
        ei = torch.stack([torch.cat([src, dst]), torch.cat([dst, src])], dim=0)
    else:
        ei = torch.stack([src, dst], dim=0)
    return ei


def powerlaw_edge_index(num_nodes, num_edges, seed=3, device="cpu", symmetric=True):
    """RMAT-like power-law graph on exactly `num_nodes` nodes with `num_edges`
    directed edges (num_edges even when symmetric)."""
    scale = max(1, int(math.ceil(math.log2(num_nodes))))
    n_samples = num_edges // 2 if symmetric else num_edges
    return rmat_edge_index(scale, n_samples, seed=seed, device=device, symmetric=symmetric,
                           num_nodes=num_nodes)


def cora_like(seed=0, num_nodes=2708, num_pairs=5278, num_features=1433, num_classes=7, p=0.0127):
    """Cora-shaped stand-in: E = 2*num_pairs directed edges (no loops, no
    duplicates), Bernoulli(p) bag-of-words rows normalised to sum 1
    (T.NormalizeFeatures), labels, and the planetoid split sizes 140/500/1000."""
    gen = torch.Generator()
    gen.manual_seed(seed)
    pairs = set()
    while len(pairs) < num_pairs:
        u = torch.randint(num_nodes, (num_pairs,), generator=gen).tolist()
        v = torch.randint(num_nodes, (num_pairs,), generator=gen).tolist()
        for s, t in zip(u, v):
            if s != t:
                pairs.add((min(s, t), max(s, t)))
            if len(pairs) == num_pairs:
                break
    pr = torch.tensor(sorted(pairs), dtype=torch.long)
    edge_index = torch.cat([pr.t(), pr.t().flip(0)], dim=1)
    x = (torch.rand((num_nodes, num_features), generator=gen) < p).to(torch.float32)
    x[x.sum(1) == 0, 0] = 1.0
    x = x / x.sum(1, keepdim=True)
    y = torch.randint(num_classes, (num_nodes,), generator=gen)
    idx = torch.randperm(num_nodes, generator=gen)
    train_mask = torch.zeros(num_nodes, dtype=torch.bool)
    val_mask = torch.zeros(num_nodes, dtype=torch.bool)
    test_mask = torch.zeros(num_nodes, dtype=torch.bool)
    train_mask[idx[:140]] = True
    val_mask[idx[140:640]] = True
    test_mask[idx[640:1640]] = True
    return dict(x=x, edge_index=edge_index, y=y, train_mask=train_mask, val_mask=val_mask,
                test_mask=test_mask, num_classes=num_classes)
