#!/usr/bin/env python3
"""Host read cost of a small device-to-host result (measurement tooling, GPU box): 1,536 bytes copied by
hipMemcpyAsync into pinned memory from torch's pin_memory() and from hipHostMalloc with several flags, then read by
numpy; the median over 100 rounds of the read alone.

usage: python tools/pinned_read.py
"""
import ctypes
import time

import numpy as np
import torch

FLAGS = {"default": 0x0, "coherent": 0x40000000, "noncoherent": 0x80000000, "portable": 0x1}


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    n = 1536
    src = torch.arange(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    bufs = {"torch_pin": torch.empty(n, dtype=torch.uint8).pin_memory(), "pageable": torch.empty(n, dtype=torch.uint8)}
    ptrs = {k: v.data_ptr() for k, v in bufs.items()}
    for name, fl in FLAGS.items():
        p = ctypes.c_void_p()
        if hip.hipHostMalloc(ctypes.byref(p), n, fl) == 0:
            ptrs[name] = p.value
    for name, ptr in ptrs.items():
        view = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr))
        reads, copies = [], []
        for _ in range(100):
            t = time.perf_counter()
            assert hip.hipMemcpyAsync(ptr, src.data_ptr(), n, 2, st.cuda_stream) == 0
            hip.hipStreamSynchronize(st.cuda_stream)
            t1 = time.perf_counter()
            out = view.copy()
            t2 = time.perf_counter()
            copies.append(t1 - t)
            reads.append(t2 - t1)
            assert out[5] == 5
        print(f"{name:12s} copy+sync median {np.median(copies) * 1e6:6.1f} us   read median {np.median(reads) * 1e6:6.2f} us"
              f"  max {np.max(reads) * 1e6:6.2f} us")


if __name__ == "__main__":
    main()
