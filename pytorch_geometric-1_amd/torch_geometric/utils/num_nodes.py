def maybe_num_nodes(index, num_nodes=None):
    """Number of nodes implied by an index tensor (PyG 1.4.3 utils.num_nodes)."""
    if num_nodes is not None:
        return num_nodes
    return int(index.max()) + 1 if index.numel() > 0 else 0
