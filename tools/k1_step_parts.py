"""configs[1] step with and without the top-k (pipelined over 3 plans/streams as bench.py does): how much of the
step the top-k kernels cost once they overlap the neighbouring steps' sweeps. usage: python tools/k1_step_parts.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from bench import decimal_csr, host_ptr, zk_hints  # noqa: E402
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402

L = _lib.load()
ctx = _lib.Context(0)
S, E, NP = 1 << 20, 4096, 3
hoff, hb = to_csr(zk_hints(E))
plans = []
for _ in range(NP):
    p = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, host_ptr(hoff), host_ptr(hb), E, 100_000_000, S, ctypes.byref(p)))
    plans.append(p)
dev = torch.device("cuda", 0)
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(NP - 1)]
csr = [decimal_csr(sp * S, S) for sp in range(NP)]
d_soff = [torch.from_numpy(so.view(np.int32)).to(dev) for so, _ in csr]
d_sb = [torch.from_numpy(sb).to(dev) for _, sb in csr]
d_stats = [torch.empty(S * 32, dtype=torch.uint8, device=dev) for _ in range(NP)]
d_topk = [torch.empty(64 * 24, dtype=torch.uint8, device=dev) for _ in range(NP)]
out = {}
for k in (64, 0):
    for mode in ("csr", "decimal"):
        def step(i):
            sp = i % NP
            with torch.cuda.stream(streams[sp]):
                st = ctypes.c_void_p(streams[sp].cuda_stream)
                if mode == "csr":
                    _lib.check(L.nmz_replayable_sweep_topk_dev(plans[sp], ctypes.c_void_p(d_soff[sp].data_ptr()),
                                                               ctypes.c_void_p(d_sb[sp].data_ptr()), S, sp * S, k,
                                                               ctypes.c_void_p(d_stats[sp].data_ptr()),
                                                               ctypes.c_void_p(d_topk[sp].data_ptr()), st))
                else:
                    _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plans[sp], sp * S, S, k,
                                                                       ctypes.c_void_p(d_stats[sp].data_ptr()),
                                                                       ctypes.c_void_p(d_topk[sp].data_ptr()), st))
        for i in range(6):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 60
        for i in range(n):
            step(i)
        torch.cuda.synchronize()
        out[f"k{k}_{mode}"] = (time.perf_counter() - t0) / n * 1e3
print(json.dumps({"ms_per_step": out}))
