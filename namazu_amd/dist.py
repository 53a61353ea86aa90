"""Multi-GPU sharding of the sweeps and the search (one process per GPU).

Seed sweeps shard by contiguous seed range with no data-path collective; the
only exchange is the failure-candidate merge: each rank's top-k (k x 24 B) is
all_gathered (RCCL over xGMI with backend "nccl", gloo on CPU) and merged
deterministically by (n_fault desc, sum_delay desc, seed asc). The all-pairs
search deals 32-wave tile groups round-robin over ranks (equal cells per
group) and all_gathers the partial k-NN key lists (N x k x 8 B) for a per-trace
merge (nmz_knn_merge_dev on the GPU, merge_knn_keys on the host).
"""
import numpy as np

from ._lib import TOPK_DTYPE


def shard_range(total, world, rank):
    """Contiguous [lo, hi) slice of `total` units for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def merge_topk(entries, k):
    """Deterministic merge of top-k candidate arrays (TOPK_DTYPE)."""
    a = np.concatenate([np.frombuffer(np.ascontiguousarray(e).tobytes(), TOPK_DTYPE) for e in entries])
    rows = sorted(a.tolist(), key=lambda t: (-t[2], -t[1], t[0]))  # exact integer keys
    return np.array(rows[:k], TOPK_DTYPE)


def merge_knn_keys(parts, k):
    """parts: [n_parts][N][k] sorted uint64 keys -> [N][k] (k smallest per trace)."""
    p = np.asarray(parts, np.uint64)
    allk = np.concatenate(list(p), axis=1)
    return np.sort(allk, axis=1)[:, :k]


def all_gather_bytes(dist, tensor):
    """all_gather a byte tensor (same size on every rank) -> list of tensors."""
    out = [tensor.new_empty(tensor.shape) for _ in range(dist.get_world_size())]
    dist.all_gather(out, tensor)
    return out


def gather_topk(dist, topk_np, k, device="cpu"):
    """All ranks contribute their top-k; every rank returns the merged global top-k."""
    import torch
    t = torch.from_numpy(np.frombuffer(np.ascontiguousarray(topk_np).tobytes(), np.uint8).copy()).to(device)
    parts = all_gather_bytes(dist, t)
    return merge_topk([p.cpu().numpy() for p in parts], k)
