"""Multi-GPU sharding of the sweeps and the search (one process per GPU).

Seed sweeps shard by contiguous seed range with no data-path collective; the
only exchange is the failure-candidate merge: each rank's top-k (k x 24 B) is
all_gathered (RCCL over xGMI with backend "nccl", gloo on CPU) and merged
deterministically by (n_fault desc, sum_delay desc, seed asc). The all-pairs
search deals its work chunks round-robin over ranks and
all_gathers the partial k-NN key lists (N x k x 8 B) for a per-trace merge
(nmz_knn_merge_dev on the GPU, merge_knn_keys on the host). On a bit-parallel
plan a shard lists only its pairs within the band; the merged lists are then
completed with (band + 1, smallest unlisted ids) (nmz_ed_knn_fill_dev on the
GPU, fill_knn_keys on the host).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import TOPK_DTYPE


def shard_range(total, world, rank):
    """Contiguous [lo, hi) slice of `total` units for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def ed_block_shard(qb, world):
    """Shard owning query block qb (queries 64 qb .. 64 qb + 63) of the two-phase all-pairs search
    (nmz_ed_allpairs_knn_shard_dev; csrc/ed.hip ed_block_shard): in each period of 2 world blocks, block r and
    its mirror 2 world - 1 - r form a pair (the falling work per block inside the upper triangle and inside each
    family of near-duplicates cancels between them), and pair p of period g goes to shard (p + g) mod world, so
    every shard takes every position. Whole query blocks, so a query pair's DP entries stay in one shard. A fixed
    rule (no environment knob): every process of a job must deal the same way."""
    if world <= 1:
        return 0
    r = qb % (2 * world)
    pr = r if r < world else 2 * world - 1 - r
    return (pr + qb // (2 * world)) % world


def ed_pair_shard(i, j, world):
    """Shard owning the pair (i, j): the block of the smaller index (the filter runs every j > q of query q)."""
    return ed_block_shard(min(i, j) // 64, world)


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


def fill_knn_keys(keys, n_cand, fill_d, self_exclude=True):
    """Host restatement of nmz_ed_knn_fill_dev (csrc/ed.hip k_knn_fill): keep each list's keys with distance
    < fill_d, then append (fill_d, j) for the smallest ids j < n_cand not listed (j != i), up to k keys."""
    keys = np.array(keys, np.uint64, copy=True)
    none = np.iinfo(np.uint64).max
    for i, row in enumerate(keys):
        kept = [int(x) for x in row if x != none and (int(x) >> 32) < fill_d]
        listed = {x & 0xFFFFFFFF for x in kept}
        out, j = list(kept), 0
        while len(out) < len(row):
            while j < n_cand and ((self_exclude and j == i) or j in listed):
                j += 1
            out.append((fill_d << 32) | j if j < n_cand else none)
            j += 1
        keys[i] = np.array(out, np.uint64)
    return keys


def all_gather_bytes(dist, tensor):
    """all_gather a byte tensor (same size on every rank) -> list of tensors."""
    out = [tensor.new_empty(tensor.shape) for _ in range(dist.get_world_size())]
    dist.all_gather(out, tensor)
    return out


def check_ed_plans(dist, L, plan, device="cpu"):
    """Every rank's edit-distance plan fingerprint (nmz_ed_plan_fingerprint: kernel kind, band, store shape, search
    options) to every rank; raises ValueError on every rank when any rank's differs from rank 0's. Ranks whose plans
    took different kernels or hold different stores would not search the same pairs, and their merged k-NN would be
    wrong without an error (the device groups make the same check inside nmz_ed_group_plan_create)."""
    import ctypes

    import torch

    from namazu_amd import _lib
    fp = np.zeros(_lib.NMZ_ED_FP_WORDS, np.uint64)
    _lib.check(L.nmz_ed_plan_fingerprint(plan, ctypes.c_void_p(fp.ctypes.data)))
    t = torch.from_numpy(fp.view(np.uint8).copy()).to(device)
    parts = [p.cpu().numpy().view(np.uint64) for p in all_gather_bytes(dist, t)]
    bad = [r for r, p in enumerate(parts) if not np.array_equal(p, parts[0])]
    if bad:
        raise ValueError(f"ranks {bad} built edit-distance plans whose fingerprint differs from rank 0's "
                         f"(kernel, band, store or search options disagree): {[p.tolist() for p in parts]}")
    return fp


def gather_topk(dist, topk_np, k, device="cpu"):
    """All ranks contribute their top-k; every rank returns the merged global top-k."""
    import torch
    t = torch.from_numpy(np.frombuffer(np.ascontiguousarray(topk_np).tobytes(), np.uint8).copy()).to(device)
    parts = all_gather_bytes(dist, t)
    return merge_topk([p.cpu().numpy() for p in parts], k)


class RandomShardSweep:
    """One rank's share of a random-policy fault sweep (BASELINE configs[3]): seeds
    [seed0 + lo, seed0 + hi) of `n_total` (shard_range), swept on this rank's GPU with the
    top-k selected on the device (nmz_random_sweep_dev + nmz_topk_select_dev, randompolicy.go:300-346).
    The per-event tables are built once (the plan); step() enqueues one sweep of the share on
    `stream` and leaves the rank's top-k (k x 24 B, TOPK_DTYPE) in the device buffer `d_topk`,
    which the caller all_gathers (RCCL) and merges with merge_topk."""

    def __init__(self, ctx, torch, device, evhash, evclass, params, seed0, n_total, world, rank, k=64):
        self.L = _lib.load()
        self.ctx = ctx
        self.lo, self.hi = shard_range(n_total, world, rank)
        self.seed0 = (seed0 + self.lo) % (1 << 64)
        self.n = self.hi - self.lo
        self.k = k
        evhash = np.ascontiguousarray(evhash, np.uint64)
        evclass = np.ascontiguousarray(evclass, np.uint8)
        self.plan = ctypes.c_void_p()
        _lib.check(self.L.nmz_random_plan_create(ctx.handle, _lib.ptr(evhash), _lib.ptr(evclass), len(evhash),
                                                 ctypes.byref(params), max(self.n, 1), ctypes.byref(self.plan)))
        self.d_stats = torch.empty(max(self.n, 1) * 32, dtype=torch.uint8, device=device)
        self.d_topk = torch.empty(k * 24, dtype=torch.uint8, device=device)

    def step(self, stream):
        _lib.check(self.L.nmz_random_sweep_dev(self.plan, self.seed0, self.n,
                                               ctypes.c_void_p(self.d_stats.data_ptr()), stream))
        _lib.check(self.L.nmz_topk_select_dev(self.ctx.handle, ctypes.c_void_p(self.d_stats.data_ptr()), self.n,
                                              self.seed0, self.k, ctypes.c_void_p(self.d_topk.data_ptr()), stream))

    def stats(self):
        return np.frombuffer(self.d_stats.cpu().numpy().tobytes(), _lib.SCHED_STATS_DTYPE)[:self.n]

    def topk(self):
        return np.frombuffer(self.d_topk.cpu().numpy().tobytes(), TOPK_DTYPE)

    def close(self):
        if self.plan:
            self.L.nmz_random_plan_destroy(self.plan)
            self.plan = None
