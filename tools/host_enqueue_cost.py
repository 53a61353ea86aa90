"""Host time to enqueue configs[1] steps (nmz_replayable_sweep_topk_dev + timing) vs the GPU time of the same
steps (GPU box). If enqueueing a step takes about as long as the GPU runs it, the host bounds the step rate."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from namazu_amd import _lib  # noqa: E402
from namazu_amd.explorepolicy import to_csr  # noqa: E402
from namazu_amd.synth import splitmix64  # noqa: E402

L = _lib.load()
ctx = _lib.Context(0)
dev = torch.device("cuda", 0)
E, S, NP = 4096, 1 << 20, 3
hints = [str(int(x)) for x in splitmix64(0x5EED, E).view(np.int64)]
ho, hb = to_csr(hints)
plans, so, sb, st, tk = [], [], [], [], []
streams = [torch.cuda.Stream(dev) for _ in range(NP)]
for sp in range(NP):
    p = ctypes.c_void_p()
    _lib.check(L.nmz_replayable_plan_create(ctx.handle, _lib.ptr(ho), _lib.ptr(hb), E, 100_000_000, S, ctypes.byref(p)))
    plans.append(p)
    o, b = to_csr([str(i) for i in range(sp * S, (sp + 1) * S)])
    so.append(torch.from_numpy(o.view(np.int32)).to(dev))
    sb.append(torch.from_numpy(b).to(dev))
    st.append(torch.empty(S * 32, dtype=torch.uint8, device=dev))
    tk.append(torch.empty(64 * 24, dtype=torch.uint8, device=dev))


def step(i):
    sp = i % NP
    _lib.check(L.nmz_replayable_sweep_topk_dev(plans[sp], ctypes.c_void_p(so[sp].data_ptr()),
                                               ctypes.c_void_p(sb[sp].data_ptr()), S, sp * S, 64,
                                               ctypes.c_void_p(st[sp].data_ptr()), ctypes.c_void_p(tk[sp].data_ptr()),
                                               ctypes.c_void_p(streams[sp].cuda_stream)))


for timing in (0, 1):
    _lib.check(L.nmz_timing_enable(ctx.handle, timing))
    for i in range(6):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        step(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"timing={timing}: host enqueue {1e6 * (t1 - t0) / 200:.1f} us per step, "
          f"wall {1e6 * (t2 - t0) / 200:.1f} us per step", flush=True)
ctx.close()
