"""Time nmz_replayable_plan_create / destroy for the configs[1] trace (host wall clock, GPU box)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402
from namazu_amd.synth import splitmix64  # noqa: E402

L = _lib.load()
ctx = _lib.Context(0)
for rep in range(12):
    hints = [str(int(x)) for x in splitmix64(0x5EED + rep, 4096).view(np.int64)]
    ho, hb = to_csr(hints)
    plan = ctypes.c_void_p()
    t0 = time.perf_counter()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), 4096, 100_000_000, 1 << 20,
                                            ctypes.byref(plan)))
    t1 = time.perf_counter()
    L.nmz_replayable_plan_destroy(plan)
    t2 = time.perf_counter()
    print(f"create {1e3 * (t1 - t0):.3f} ms  destroy {1e3 * (t2 - t1):.3f} ms")
ctx.close()
