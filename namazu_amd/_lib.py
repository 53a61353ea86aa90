"""ctypes binding of libnmz_gpu.so (the C ABI declared in include/nmz_gpu.h).

The HIP library is the only compute path: if it is missing this module raises
NmzLibraryError instead of falling back to anything on the CPU.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NMZ_LIB_PATH: an alternative in-tree build of the same library (tuning variants)
DEFAULT_LIB_PATH = os.path.join(HERE, "libnmz_gpu.so")
LIB_PATH = os.environ.get("NMZ_LIB_PATH") or DEFAULT_LIB_PATH

NMZ_OK = 0
NMZ_EINVAL = -1
NMZ_EHIP = -2
NMZ_ENOMEM = -3
NMZ_ERANGE = -4
NMZ_EAGAIN = -5

NMZ_EV_PRIORITIZED = 0x01
NMZ_EV_FAULTABLE = 0x02
NMZ_STAT_RNG_OVERFLOW = 0x01
NMZ_NONE = 0xFFFFFFFF
NMZ_ED_NCOUNTERS = 6
NMZ_ED_OPT_SINGLE_KERNEL, NMZ_ED_OPT_NO_QGRAM, NMZ_ED_OPT_COMPACT, NMZ_ED_OPT_HOST_BUILD = 1, 2, 4, 8
NMZ_ED_FP_WORDS = 8

SCHED_STATS_DTYPE = np.dtype([
    ("sum_delay_ns", "<u8"), ("max_delay_ns", "<i8"), ("argmax_event", "<u4"),
    ("n_fault", "<u4"), ("first_fault", "<u4"), ("flags", "<u4")])
assert SCHED_STATS_DTYPE.itemsize == 32
TOPK_DTYPE = np.dtype([("seed", "<u8"), ("sum_delay_ns", "<i8"), ("n_fault", "<u4"),
                       ("first_fault", "<u4")])
assert TOPK_DTYPE.itemsize == 24


class NmzLibraryError(RuntimeError):
    """libnmz_gpu.so is missing or failed to load (no CPU fallback exists)."""


class NmzError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"nmz error {code}: {msg}")
        self.code = code


class NmzInvalidArgument(NmzError, ValueError):
    pass


class RandomParams(ctypes.Structure):
    _fields_ = [("min_ns", ctypes.c_int64 * 2), ("max_ns", ctypes.c_int64 * 2),
                ("fault_threshold", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


# every entry point declared in include/nmz_gpu.h: name -> (restype, argtypes)
_P = ctypes.c_void_p
_u64, _i64, _u32, _i32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32
_int = ctypes.c_int
SIGNATURES = {
    "nmz_open": (_int, [_int, ctypes.POINTER(_P)]),
    "nmz_close": (_int, [_P]),
    "nmz_last_error": (ctypes.c_char_p, []),
    "nmz_abi_version": (_int, []),
    "nmz_device_count": (_int, [ctypes.POINTER(_int)]),
    "nmz_ctx_stream": (_int, [_P, ctypes.POINTER(_P)]),
    "nmz_random_params_resolve": (_int, [_i64, _i64, ctypes.c_double, _P]),
    "nmz_fnv1a64_batch": (_int, [_P, _P, _P, _u64, _P]),
    "nmz_replayable_sweep": (_int, [_P, _P, _P, _u64, _P, _P, _u32, _i64, _P, _P, _u64, _u32, _P]),
    "nmz_replayable_plan_create": (_int, [_P, _P, _P, _u32, _i64, _u64, ctypes.POINTER(_P)]),
    "nmz_replayable_plan_create_async": (_int, [_P, _P, _P, _u32, _i64, _u64, ctypes.POINTER(_P)]),
    "nmz_replayable_seeds_create": (_int, [_P, _P, _P, _u64, _u64, ctypes.POINTER(_P)]),
    "nmz_replayable_seeds_destroy": (_int, [_P]),
    "nmz_replayable_sweep_seeds_topk_dev": (_int, [_P, _P, _u64, _u32, _P, _P, _P]),
    "nmz_replayable_sweep_traces": (_int, [_P, _u32, _P, _P, _P, _i64, _u64, _u64, _u32, _P]),
    "nmz_replayable_plan_destroy": (_int, [_P]),
    "nmz_replayable_plan_kernel": (_int, [_P]),
    "nmz_replayable_sweep_dev": (_int, [_P, _P, _P, _u64, _P, _P]),
    "nmz_replayable_sweep_topk_dev": (_int, [_P, _P, _P, _u64, _u64, _u32, _P, _P, _P]),
    "nmz_replayable_decide": (_int, [_P, _P, _u32, _P, _P, _u32, _i64, _P]),
    "nmz_random_decide": (_int, [_P, _u64, _P, _P, _u32, _P, _P, _P]),
    "nmz_random_sweep": (_int, [_P, _u64, _u64, _P, _P, _u32, _P, _P, _P, _P, _u64, _u32, _P]),
    "nmz_random_plan_create": (_int, [_P, _P, _P, _u32, _P, _u64, ctypes.POINTER(_P)]),
    "nmz_random_plan_destroy": (_int, [_P]),
    "nmz_random_sweep_dev": (_int, [_P, _u64, _u64, _P, _P]),
    "nmz_ed_pairs": (_int, [_P, _P, _P, _u32, _P, _u64, _u32, _P]),
    "nmz_ed_allpairs_knn": (_int, [_P, _P, _P, _u32, _u32, _u32, _P, _P]),
    "nmz_ed_plan_create": (_int, [_P, _P, _P, _u32, _u32, ctypes.POINTER(_P)]),
    "nmz_ed_plan_destroy": (_int, [_P]),
    "nmz_ed_plan_create_dev": (_int, [_P, _P, _P, _u32, _u32, ctypes.POINTER(_P)]),
    "nmz_ed_plan_create_opts": (_int, [_P, _P, _P, _P, _u32, _u32, _u32, ctypes.POINTER(_P)]),
    "nmz_ed_plan_fingerprint": (_int, [_P, _P]),
    "nmz_ed_plan_is_fast": (_int, [_P]),
    "nmz_ed_block_shard": (_u32, [_u32, _u32]),
    "nmz_ed_allpairs_knn_dev": (_int, [_P, _u32, _P, _P]),
    "nmz_ed_allpairs_knn_shard_dev": (_int, [_P, _u32, _u32, _u32, _P, _P]),
    "nmz_knn_merge_dev": (_int, [_P, _P, _u32, _u32, _u32, _P, _P]),
    "nmz_ed_knn_fill_dev": (_int, [_P, _u32, _P, _P]),
    "nmz_ed_plan_counters": (_int, [_P, _P, _P]),
    "nmz_debug_tp_offsets": (_int, [_P, _P, _u32, _u32, _P, _P, _P, _P]),
    "nmz_ed_plan_query_knn": (_int, [_P, _P, _P, _u32, _u32, _P, _P]),
    "nmz_trace_signatures": (_int, [_P, _P, _P, _P, _u32, _P]),
    "nmz_unique_traces": (_int, [_P, _P, _P, _P, _u32, _P]),
    "nmz_unique_traces_dev": (_int, [_P, _P, _P, _P, _u32, _u32, _P, _P, _P]),
    "nmz_topk_select_dev": (_int, [_P, _P, _u64, _u64, _u32, _P, _P]),
    "nmz_replayable_sweep_decimal_topk_dev": (_int, [_P, _u64, _u64, _u32, _P, _P, _P]),
    "nmz_random_decide_host": (_int, [_u64, _P, _P, _u32, _P, _P, _P]),
    "nmz_replayable_decide_host": (_int, [_P, _u32, _P, _P, _u32, _i64, _P]),
    "nmz_fnv1a64_batch_host": (_int, [_P, _P, _u64, _P]),
    "nmz_tbqueue_create": (_int, [ctypes.POINTER(_P)]),
    "nmz_tbqueue_close": (_int, [_P]),
    "nmz_tbqueue_destroy": (_int, [_P]),
    "nmz_monotonic_ns": (_i64, []),
    "nmz_tbqueue_enqueue": (_int, [_P, _u64, _i64]),
    "nmz_tbqueue_enqueue_fixed": (_int, [_P, _u64, _i64, _i64]),
    "nmz_tbqueue_dequeue": (_int, [_P, _i64, ctypes.POINTER(_u64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "nmz_tbqueue_stats": (_int, [_P, ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    # device groups (multi-GPU inside the C ABI, csrc/group.hip)
    "nmz_open_group": (_int, [_u32, _u32, ctypes.POINTER(_P)]),
    "nmz_group_unique_id": (_int, [_P]),
    "nmz_open_group_rank": (_int, [_P, _int, _int, _int, _u32, ctypes.POINTER(_P)]),
    "nmz_close_group": (_int, [_P]),
    "nmz_group_info": (_int, [_P, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_u32)]),
    "nmz_group_collectives": (_int, [_P, ctypes.POINTER(_u64)]),
    "nmz_topk_merge_dev": (_int, [_P, _P, _u64, _u32, _P, _P, _P]),
    "nmz_replayable_group_plan_create": (_int, [_P, _P, _P, _u32, _i64, _u64, ctypes.POINTER(_P)]),
    "nmz_replayable_group_plan_destroy": (_int, [_P]),
    "nmz_replayable_group_sweep": (_int, [_P, _P, _P, _u64, _u32, _P, _P]),
    "nmz_replayable_group_sweep_decimal": (_int, [_P, _u64, _u64, _u32, _P, _P]),
    "nmz_replayable_sweep_topk_group": (_int, [_P, _P, _P, _u64, _P, _P, _u32, _i64, _u32, _P, _P]),
    "nmz_random_group_plan_create": (_int, [_P, _P, _P, _u32, _P, _u64, ctypes.POINTER(_P)]),
    "nmz_random_group_plan_destroy": (_int, [_P]),
    "nmz_random_group_sweep": (_int, [_P, _u64, _u64, _u32, _P, _P]),
    "nmz_random_sweep_topk_group": (_int, [_P, _u64, _u64, _P, _P, _u32, _P, _u32, _P, _P]),
    "nmz_ed_group_plan_create": (_int, [_P, _P, _P, _u32, _u32, ctypes.POINTER(_P)]),
    "nmz_ed_group_plan_create_opts": (_int, [_P, _P, _P, _u32, _u32, _u32, ctypes.POINTER(_P)]),
    "nmz_ed_group_plan_destroy": (_int, [_P]),
    "nmz_ed_group_plan_timing": (_int, [_P, _P, _P, _P]),
    "nmz_ed_group_allpairs_knn": (_int, [_P, _u32, _P, _P]),
    "nmz_ed_allpairs_knn_group": (_int, [_P, _P, _P, _u32, _u32, _u32, _P, _P]),
    "nmz_timing_enable": (_int, [_P, _int]),
    "nmz_timing_read": (_int, [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_u64), _int]),
    "nmz_timing_read_span": (_int, [_P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_u64), _int]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load libnmz_gpu.so (fails loudly; there is no CPU fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NmzLibraryError(
                f"{LIB_PATH} not found: build it with `make -C namazu_amd/csrc` "
                "(or __graft_entry__.build()); the engine has no CPU fallback")
        try:
            import torch  # noqa: F401  (pin one HIP runtime per process when torch is present)
        except Exception:
            pass
        try:
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise NmzLibraryError(f"failed to load {LIB_PATH}: {e}") from e
        variant = LIB_PATH != DEFAULT_LIB_PATH  # an A/B build (NMZ_LIB_PATH) may predate newer entry points
        for name, (res, args) in SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L


def last_error():
    return load().nmz_last_error().decode(errors="replace")


def check(rc):
    if rc != NMZ_OK:
        msg = last_error()
        if rc == NMZ_EINVAL:
            raise NmzInvalidArgument(rc, msg)
        raise NmzError(rc, msg)


def ptr(a):
    """Data pointer of a numpy array (None for None)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


def resolve_random_params(min_ns, max_ns, probability):
    p = RandomParams()
    check(load().nmz_random_params_resolve(int(min_ns), int(max_ns), float(probability),
                                           ctypes.byref(p)))
    return p


class Context:
    """One device context (libnmz_gpu nmz_ctx). Use as a context manager."""

    def __init__(self, device=0):
        self._lib = load()
        h = ctypes.c_void_p()
        check(self._lib.nmz_open(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device

    def stream(self):
        """The context's own HIP stream handle (int): what a NULL stream argument means."""
        s = ctypes.c_void_p()
        check(self._lib.nmz_ctx_stream(self.handle, ctypes.byref(s)))
        return s.value

    def close(self):
        if self.handle:
            self._lib.nmz_close(self.handle)
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


def device_count():
    n = ctypes.c_int()
    check(load().nmz_device_count(ctypes.byref(n)))
    return n.value


_default_ctx = {}


def default_context(device=0):
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = _default_ctx[device] = Context(device)
    return ctx
