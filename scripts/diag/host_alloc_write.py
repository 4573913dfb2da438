#!/usr/bin/env python3
"""Host-side write and read speed of pinned memory by hipHostMalloc flag
(default vs coherent / fine-grained): the batcher writes every chunk's
descriptor into such a buffer on the submitting thread.  Prints one JSON
object (GB/s, best of 5, 64 MiB)."""
import ctypes
import json
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
N = 64 << 20
res = {}
for name, flag in (("default", 0x0), ("coherent", 0x40000000), ("noncoherent", 0x80000000)):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), N, flag) == 0, name
    a = np.ctypeslib.as_array((ctypes.c_uint8 * N).from_address(p.value))
    src = np.random.default_rng(1).integers(0, 255, N, dtype=np.uint8)
    w, r, s = [], [], []
    for _ in range(5):
        t = time.perf_counter(); a[:] = src; w.append(time.perf_counter() - t)
        t = time.perf_counter(); x = a.sum(dtype=np.uint64); r.append(time.perf_counter() - t)
        u = a.view(np.uint64)
        t = time.perf_counter()
        for i in range(0, 1 << 16):         # scattered 8-B stores, as the reserve loop makes
            u[i] = i
        s.append(time.perf_counter() - t)
    res[name] = {"write_gb_s": round(N / min(w) / 1e9, 2), "read_gb_s": round(N / min(r) / 1e9, 2),
                 "scalar_store_ns": round(min(s) / (1 << 16) * 1e9, 1)}
    hip.hipHostFree(p)
print(json.dumps(res))
