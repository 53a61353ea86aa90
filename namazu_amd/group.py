"""Device groups: several GPUs behind one call of the C ABI (csrc/group.hip, include/nmz_gpu.h).

The reference's callers are single processes (cli/run.go:123-136 initPolicy, cli/tools/visualize.go:138-172);
a group lets one process drive every GPU of a node: one context + worker thread per device and one RCCL
communicator, created once. `n_shards` may exceed the device count (virtual shards: one GPU runs the sharding
and merge logic of any shard count). Results equal one unsharded call (deterministic merges).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import SCHED_STATS_DTYPE, TOPK_DTYPE

GROUP_ID_BYTES = 128


def _u8(a):
    return np.ascontiguousarray(a, np.uint8)


class Group:
    """nmz_open_group(dev_mask, n_shards) or, with `unique_id`, nmz_open_group_rank (one process per device)."""

    def __init__(self, devices=(0,), n_shards=0, unique_id=None, n_ranks=None, rank=None):
        self.L = _lib.load()
        h = ctypes.c_void_p()
        if unique_id is None:
            mask = 0
            for d in devices:
                mask |= 1 << int(d)
            _lib.check(self.L.nmz_open_group(mask, int(n_shards), ctypes.byref(h)))
        else:
            uid = _u8(np.frombuffer(bytes(unique_id), np.uint8))
            assert uid.size == GROUP_ID_BYTES
            _lib.check(self.L.nmz_open_group_rank(_lib.ptr(uid), int(n_ranks), int(rank), int(devices[0]),
                                                  int(n_shards), ctypes.byref(h)))
        self.handle = h
        nr, nl, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint32()
        _lib.check(self.L.nmz_group_info(h, ctypes.byref(nr), ctypes.byref(nl), ctypes.byref(ns)))
        self.n_ranks, self.n_local, self.n_shards = nr.value, nl.value, ns.value

    @staticmethod
    def unique_id():
        b = np.zeros(GROUP_ID_BYTES, np.uint8)
        _lib.check(_lib.load().nmz_group_unique_id(_lib.ptr(b)))
        return b.tobytes()

    def close(self):
        """nmz_close_group: fails (NmzError, NMZ_EINVAL) while plans made on the group are alive."""
        if self.handle:
            _lib.check(self.L.nmz_close_group(self.handle))
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- one-call forms --------------------------------------------------------------------------
    def replayable_sweep(self, seed_off, seed_bytes, hint_off, hint_bytes, max_interval_ns, k=0, stats=True):
        seed_off = np.ascontiguousarray(seed_off, np.uint32)
        hint_off = np.ascontiguousarray(hint_off, np.uint32)
        n, e = len(seed_off) - 1, len(hint_off) - 1
        st = np.zeros(n, SCHED_STATS_DTYPE) if stats else None
        tk = np.zeros(k, TOPK_DTYPE)
        _lib.check(self.L.nmz_replayable_sweep_topk_group(
            self.handle, _lib.ptr(seed_off), _lib.ptr(_u8(seed_bytes)), n, _lib.ptr(hint_off),
            _lib.ptr(_u8(hint_bytes)), e, int(max_interval_ns), k, _lib.ptr(st), _lib.ptr(tk) if k else None))
        return st, tk

    def random_sweep(self, seed0, n_seeds, evhash, evclass, params, k=0, stats=True):
        evhash = np.ascontiguousarray(evhash, np.uint64)
        evclass = np.ascontiguousarray(evclass, np.uint8)
        st = np.zeros(n_seeds, SCHED_STATS_DTYPE) if stats else None
        tk = np.zeros(k, TOPK_DTYPE)
        _lib.check(self.L.nmz_random_sweep_topk_group(
            self.handle, int(seed0) % (1 << 64), int(n_seeds), _lib.ptr(evhash), _lib.ptr(evclass), len(evhash),
            ctypes.byref(params), k, _lib.ptr(st), _lib.ptr(tk) if k else None))
        return st, tk

    def ed_allpairs_knn(self, ts, band, k):
        n = len(ts)
        ids = np.zeros(n * k, np.uint32)
        ds = np.zeros(n * k, np.uint32)
        _lib.check(self.L.nmz_ed_allpairs_knn_group(self.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), n, band, k,
                                                    _lib.ptr(ids), _lib.ptr(ds)))
        return ids.reshape(n, k), ds.reshape(n, k)


class ReplayableGroupPlan:
    """A replayable plan on every device of a group, for repeated sweeps (nmz_replayable_group_plan_*)."""

    def __init__(self, group, hint_off, hint_bytes, max_interval_ns, max_seeds_per_shard):
        self.g, self.L = group, group.L
        hint_off = np.ascontiguousarray(hint_off, np.uint32)
        self.h = ctypes.c_void_p()
        _lib.check(self.L.nmz_replayable_group_plan_create(group.handle, _lib.ptr(hint_off), _lib.ptr(_u8(hint_bytes)),
                                                           len(hint_off) - 1, int(max_interval_ns),
                                                           int(max_seeds_per_shard), ctypes.byref(self.h)))

    def sweep(self, seed_off, seed_bytes, k=0, stats=True):
        seed_off = np.ascontiguousarray(seed_off, np.uint32)
        n = len(seed_off) - 1
        st = np.zeros(n, SCHED_STATS_DTYPE) if stats else None
        tk = np.zeros(k, TOPK_DTYPE)
        _lib.check(self.L.nmz_replayable_group_sweep(self.h, _lib.ptr(seed_off), _lib.ptr(_u8(seed_bytes)), n, k,
                                                     _lib.ptr(st), _lib.ptr(tk) if k else None))
        return st, tk

    def sweep_decimal(self, seed_lo, n_seeds, k=0, stats=True):
        st = np.zeros(n_seeds, SCHED_STATS_DTYPE) if stats else None
        tk = np.zeros(k, TOPK_DTYPE)
        _lib.check(self.L.nmz_replayable_group_sweep_decimal(self.h, int(seed_lo) % (1 << 64), int(n_seeds), k,
                                                             _lib.ptr(st), _lib.ptr(tk) if k else None))
        return st, tk

    def close(self):
        if self.h:
            self.L.nmz_replayable_group_plan_destroy(self.h)
            self.h = None


class RandomGroupPlan:
    def __init__(self, group, evhash, evclass, params, max_seeds_per_shard):
        self.g, self.L = group, group.L
        evhash = np.ascontiguousarray(evhash, np.uint64)
        evclass = np.ascontiguousarray(evclass, np.uint8)
        self.h = ctypes.c_void_p()
        _lib.check(self.L.nmz_random_group_plan_create(group.handle, _lib.ptr(evhash), _lib.ptr(evclass), len(evhash),
                                                       ctypes.byref(params), int(max_seeds_per_shard),
                                                       ctypes.byref(self.h)))

    def sweep(self, seed0, n_seeds, k=0, stats=True):
        st = np.zeros(n_seeds, SCHED_STATS_DTYPE) if stats else None
        tk = np.zeros(k, TOPK_DTYPE)
        _lib.check(self.L.nmz_random_group_sweep(self.h, int(seed0) % (1 << 64), int(n_seeds), k, _lib.ptr(st),
                                                 _lib.ptr(tk) if k else None))
        return st, tk

    def close(self):
        if self.h:
            self.L.nmz_random_group_plan_destroy(self.h)
            self.h = None


class EdGroupPlan:
    def __init__(self, group, ts, band):
        self.g, self.L, self.n = group, group.L, len(ts)
        self.h = ctypes.c_void_p()
        _lib.check(self.L.nmz_ed_group_plan_create(group.handle, _lib.ptr(ts.off), _lib.ptr(ts.sym), len(ts), band,
                                                   ctypes.byref(self.h)))

    def knn(self, k):
        ids = np.zeros(self.n * k, np.uint32)
        ds = np.zeros(self.n * k, np.uint32)
        _lib.check(self.L.nmz_ed_group_allpairs_knn(self.h, k, _lib.ptr(ids), _lib.ptr(ds)))
        return ids.reshape(self.n, k), ds.reshape(self.n, k)

    def timing(self):
        """Per local device: (share upload, RCCL all_gather, device plan build) in ms (nmz_ed_group_plan_timing)."""
        up, ga, bu = (np.zeros(self.g.n_local, np.float64) for _ in range(3))
        _lib.check(self.L.nmz_ed_group_plan_timing(self.h, _lib.ptr(up), _lib.ptr(ga), _lib.ptr(bu)))
        return dict(upload_ms=up.tolist(), gather_ms=ga.tolist(), build_ms=bu.tolist())

    def close(self):
        if self.h:
            self.L.nmz_ed_group_plan_destroy(self.h)
            self.h = None


for _cls in (ReplayableGroupPlan, RandomGroupPlan, EdGroupPlan):
    def _del(self):
        try:
            self.close()
        except Exception:
            pass
    _cls.__del__ = _del
