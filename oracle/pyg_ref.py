"""PyG 1.4.3 hot-path semantics on the CPU -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Plain torch CPU restatements of the torch_geometric 1.4.3 functions on the
aggregation path (all [U]); callers in the reference tree:
examples/gcn.py:18-27 (GCNConv cached), ConvexPruning.py:180-224 (GCN/GAT
stacks), examples/ppi.py:22-28 (multi-head GAT), README.md:35-49 (custom
MessagePassing with aggr='max').  Works in float32 (parity) or float64
(ground truth for tolerance analysis).
"""
import torch
import torch.nn.functional as F

from . import scatter_ref as S


# --- utils.loop [U4] --------------------------------------------------------

def remove_self_loops(edge_index, edge_attr=None):
    row, col = edge_index
    mask = row != col
    return edge_index[:, mask], (None if edge_attr is None else edge_attr[mask])


def add_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    N = num_nodes
    loops = torch.arange(N, dtype=torch.long).unsqueeze(0).repeat(2, 1)
    if edge_weight is not None:
        edge_weight = torch.cat([edge_weight, edge_weight.new_full((N,), fill_value)])
    return torch.cat([edge_index, loops], dim=1), edge_weight


def add_remaining_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    """kept non-loop edges (original order), then loops 0..N-1; a loop keeps the
    weight of the node's last pre-existing loop, else fill_value."""
    N = num_nodes
    row, col = edge_index
    mask = row != col
    loop_weight = torch.full((N,), fill_value, dtype=None if edge_weight is None else edge_weight.dtype)
    if edge_weight is not None:
        rem = edge_weight[~mask]
        rrows = row[~mask]
        for k in range(rrows.numel()):  # sequential: last one wins (CPU index_put_)
            loop_weight[rrows[k]] = rem[k]
        edge_weight = torch.cat([edge_weight[mask], loop_weight])
    loops = torch.arange(N, dtype=row.dtype).unsqueeze(0).repeat(2, 1)
    return torch.cat([edge_index[:, mask], loops], dim=1), edge_weight


# --- utils.scatter_ [U2] / utils.softmax [U3] ------------------------------

def scatter_(name, src, index, dim_size):
    if name == "add":
        out = S.scatter_sum(src, index, dim_size)
    elif name == "mean":
        out = S.scatter_mean(src, index, dim_size)
    elif name == "max":
        out = S.scatter_max(src, index, dim_size)[0]
        out[out < -10000] = 0
    elif name == "min":
        out = S.scatter_min(src, index, dim_size)[0]
        out[out > 10000] = 0
    else:
        raise ValueError(name)
    return out


def _seg_max(src, index, N):
    if src.dtype == torch.float32:
        return S.scatter_max(src, index, N)[0]
    out = torch.full((N,) + tuple(src.shape[1:]), float("-inf"), dtype=src.dtype)
    out = out.scatter_reduce(0, index.view((-1,) + (1,) * (src.dim() - 1)).expand_as(src), src, "amax")
    return torch.where(torch.isinf(out), torch.zeros_like(out), out)


def softmax(src, index, num_nodes):
    out = src - _seg_max(src, index, num_nodes)[index]
    out = out.exp()
    out = out / (S.scatter_sum(out, index, num_nodes)[index] + 1e-16)
    return out


# --- GCNConv [U5] -----------------------------------------------------------

def gcn_norm(edge_index, num_nodes, edge_weight=None, improved=False, dtype=torch.float32):
    if edge_weight is None:
        edge_weight = torch.ones((edge_index.size(1),), dtype=dtype)
    fill_value = 1 if not improved else 2
    edge_index, edge_weight = add_remaining_self_loops(edge_index, edge_weight, fill_value, num_nodes)
    row, col = edge_index
    deg = S.scatter_sum(edge_weight, row, num_nodes)
    deg_inv_sqrt = deg.pow(-0.5)
    deg_inv_sqrt[deg_inv_sqrt == float("inf")] = 0
    return edge_index, deg_inv_sqrt[row] * edge_weight * deg_inv_sqrt[col]


def gcn_aggregate(x, edge_index, norm, num_nodes):
    """propagate(edge_index, x=x, norm=norm): message norm*x_j, scatter add."""
    x_j = x.index_select(0, edge_index[0])
    msg = norm.view(-1, 1) * x_j
    return S.scatter_sum(msg, edge_index[1], num_nodes)


def gcn_conv(x, edge_index, weight, bias=None, edge_weight=None, improved=False):
    N = x.size(0)
    h = torch.matmul(x, weight)
    ei, norm = gcn_norm(edge_index, N, edge_weight, improved, h.dtype)
    out = gcn_aggregate(h, ei, norm, N)
    return out + bias if bias is not None else out


# --- GATConv [U6] -----------------------------------------------------------

def gat_dropout_keep_slots(seed, p, H, n_slots, start=0):
    """The fused kernels' attention-dropout keep mask (csrc/mp_aggregate.hip
    drop_hash / drop_bits), restated in numpy: bool [n_slots, H], slot s of the
    destination CSR (s from `start`), head h kept iff hash(seed, s*H + h) >= floor(p * 2^32).
    The reference draws its mask from torch's RNG (GATConv.message:
    F.dropout(alpha, p)); parity is checked for a given mask, not a given draw."""
    import numpy as np
    M = np.uint64(0xFFFFFFFF)

    def mix(h):
        h = h ^ (h >> np.uint64(16))
        h = (h * np.uint64(0x85EBCA6B)) & M
        h = h ^ (h >> np.uint64(13))
        h = (h * np.uint64(0xC2B2AE35)) & M
        return h ^ (h >> np.uint64(16))

    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    idx = np.arange(start * H, (start + n_slots) * H, dtype=np.uint64)  # slots [start, start + n_slots)
    a = mix((idx & M) ^ np.uint64(seed & 0xFFFFFFFF))
    hi = (idx >> np.uint64(32)) ^ np.uint64(seed >> 32)
    b = mix((a + ((np.uint64(0x9E3779B9) * hi) & M) + np.uint64(0x632BE5AB)) & M)
    thr = min(int(np.floor(float(np.float32(p)) * 4294967296.0)), 0xFFFFFFFF)
    return torch.from_numpy((b >= np.uint64(thr)).reshape(n_slots, H))


def gat_conv(x, edge_index, weight, att, bias, heads, out_channels, concat=True, negative_slope=0.2,
             return_alpha=False, drop_keep=None, drop_p=0.0):
    """drop_keep (bool [E', H] over the layer's edges incl. its self loops) and
    drop_p: training-mode attention dropout, alpha * keep / (1 - p) on the
    messages (F.dropout's scale); the returned alpha is the undropped one."""
    N = x.size(0)
    ei, _ = remove_self_loops(edge_index)
    ei, _ = add_self_loops(ei, num_nodes=N)
    h = torch.matmul(x, weight)
    x_i = h.index_select(0, ei[1]).view(-1, heads, out_channels)
    x_j = h.index_select(0, ei[0]).view(-1, heads, out_channels)
    alpha = (torch.cat([x_i, x_j], dim=-1) * att).sum(dim=-1)
    alpha = F.leaky_relu(alpha, negative_slope)
    alpha = softmax(alpha, ei[1], N)
    a_msg = alpha
    if drop_keep is not None:
        scale = float(1.0 / (1.0 - float(torch.tensor(drop_p, dtype=torch.float32))))
        a_msg = alpha * drop_keep.to(alpha.dtype) * scale
    msg = x_j * a_msg.view(-1, heads, 1)
    out = S.scatter_sum(msg, ei[1], N)
    out = out.view(-1, heads * out_channels) if concat else out.mean(dim=1)
    if bias is not None:
        out = out + bias
    return (out, ei, alpha) if return_alpha else out


# --- aggr='max' MessagePassing / GraphConv [U7] -----------------------------

def max_aggregate(h, edge_index, num_nodes, pyg_mask=True):
    """propagate with message h_j and aggr='max' -> (scatter_ output, arg)."""
    msg = h.index_select(0, edge_index[0])
    out, arg = S.scatter_max(msg, edge_index[1], num_nodes)
    if pyg_mask:
        out[out < -10000] = 0
    return out, arg


def graph_conv_max(x, edge_index, weight, lin_w, lin_b):
    h = torch.matmul(x, weight)
    out, _ = max_aggregate(h, edge_index, x.size(0))
    return out + F.linear(x, lin_w, lin_b)


def edge_conv_max(x, edge_index, mlp):
    """README.md:35-49 EdgeConv: message mlp(cat[x_i, x_j - x_i]), aggr='max'."""
    x_i = x.index_select(0, edge_index[1])
    x_j = x.index_select(0, edge_index[0])
    msg = mlp(torch.cat([x_i, x_j - x_i], dim=1))
    out, _ = S.scatter_max(msg, edge_index[1], x.size(0))
    out[out < -10000] = 0
    return out


# --- utils.get_laplacian / ChebConv / AGNNConv [U] ---------------------------
# callers: ConvexPruning.py:259-264 (ChebConv(..., K=1)), :236-237 (AGNNConv)

def get_laplacian(edge_index, edge_weight=None, normalization=None, dtype=torch.float32, num_nodes=None):
    edge_index, edge_weight = remove_self_loops(edge_index, edge_weight)
    if edge_weight is None:
        edge_weight = torch.ones((edge_index.size(1),), dtype=dtype)
    row, col = edge_index
    deg = S.scatter_sum(edge_weight, row, num_nodes)
    if normalization is None:
        edge_index, _ = add_self_loops(edge_index, num_nodes=num_nodes)
        return edge_index, torch.cat([-edge_weight, deg], dim=0)
    if normalization == "sym":
        dinv = deg.pow(-0.5)
        dinv[dinv == float("inf")] = 0
        edge_weight = dinv[row] * edge_weight * dinv[col]
    else:
        dinv = 1.0 / deg
        dinv[dinv == float("inf")] = 0
        edge_weight = dinv[row] * edge_weight
    return add_self_loops(edge_index, -edge_weight, fill_value=1, num_nodes=num_nodes)


def cheb_norm(edge_index, num_nodes, edge_weight=None, normalization="sym", lambda_max=2.0,
              dtype=torch.float32):
    edge_index, edge_weight = remove_self_loops(edge_index, edge_weight)
    edge_index, edge_weight = get_laplacian(edge_index, edge_weight, normalization, dtype, num_nodes)
    edge_weight = (2.0 * edge_weight) / lambda_max
    edge_weight.masked_fill_(edge_weight == float("inf"), 0)
    return add_self_loops(edge_index, edge_weight, fill_value=-1, num_nodes=num_nodes)


def cheb_conv(x, edge_index, weight, bias=None, edge_weight=None, normalization="sym", lambda_max=None):
    """ChebConv.forward: weight [K, F_in, F_out]."""
    N = x.size(0)
    lambda_max = 2.0 if lambda_max is None else lambda_max
    ei, norm = cheb_norm(edge_index, N, edge_weight, normalization, lambda_max, x.dtype)
    Tx_0 = x
    out = torch.matmul(Tx_0, weight[0])
    if weight.size(0) > 1:
        Tx_1 = gcn_aggregate(x, ei, norm, N)
        out = out + torch.matmul(Tx_1, weight[1])
    for k in range(2, weight.size(0)):
        Tx_2 = 2 * gcn_aggregate(Tx_1, ei, norm, N) - Tx_0
        out = out + torch.matmul(Tx_2, weight[k])
        Tx_0, Tx_1 = Tx_1, Tx_2
    return out + bias if bias is not None else out


def agnn_conv(x, edge_index, beta):
    """AGNNConv.forward: softmax over N(i) u {i} of beta * cos(x_i, x_j), sum of alpha * x_j."""
    N = x.size(0)
    ei, _ = remove_self_loops(edge_index)
    ei, _ = add_self_loops(ei, num_nodes=N)
    x_norm = F.normalize(x, p=2, dim=-1)
    x_j = x.index_select(0, ei[0])
    alpha = beta * (x_norm.index_select(0, ei[1]) * x_norm.index_select(0, ei[0])).sum(dim=-1)
    alpha = softmax(alpha, ei[1], N)
    return S.scatter_sum(x_j * alpha.view(-1, 1), ei[1], N)


# --- SGConv / GINConv [U] (upstream examples/sgc.py, examples/mutag_gin.py) ---

def sg_conv(x, edge_index, K, lin_w, lin_b=None, edge_weight=None):
    N = x.size(0)
    ei, norm = gcn_norm(edge_index, N, edge_weight, False, x.dtype)
    for _ in range(K):
        x = gcn_aggregate(x, ei, norm, N)
    return F.linear(x, lin_w, lin_b)


def gin_conv(x, edge_index, mlp, eps):
    ei, _ = remove_self_loops(edge_index)
    x_j = x.index_select(0, ei[0])
    return mlp((1 + eps) * x + S.scatter_sum(x_j, ei[1], x.size(0)))
