"""Kernel timing source for the chunk-parallel wkv6 (run under rocprofv3 --kernel-trace --stats):
serial k_wkv6_s64 and k_wkv6c_prep + k_wkv6c_scan at the v6-1B6 head count (H = 32) for T = 1024 and
4096 through rwkv_mi355x_selftest_wkv6, 5 runs each; prints each form's error against the float64
recurrence for the first run."""
import ctypes
import os
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
from rwkv_lib import library  # noqa: E402

P = ctypes.POINTER(ctypes.c_float)
f = library().library.rwkv_mi355x_selftest_wkv6
f.argtypes = [ctypes.c_int] * 4 + [P] * 8
f.restype = ctypes.c_bool
H = 32
for T in (1024, 4096):
    rng = np.random.default_rng(T)
    C = H * 64
    r = rng.standard_normal((T, C)).astype(np.float32)
    k = (rng.standard_normal((T, C)) * 0.5).astype(np.float32)
    v = rng.standard_normal((T, C)).astype(np.float32)
    u = (rng.standard_normal(C) * 0.5).astype(np.float32)
    w = np.exp(-np.exp(rng.uniform(-7, 1.8, (T, C)))).astype(np.float32)
    s0 = rng.standard_normal((H, 64, 64)).astype(np.float32)
    outs = {}
    for chunked in (0, 1):
        for rep in range(5):
            y = np.zeros((T, C), np.float32)
            so = np.zeros((H, 64, 64), np.float32)
            assert f(T, H, chunked, 1, *[a.ctypes.data_as(P) for a in (k, v, r, u, w, s0, so, y)])
        outs[chunked] = (y, so)
    d = np.abs(outs[1][0] - outs[0][0]).max() / np.abs(outs[0][0]).max()
    print(f'T={T} H={H}: chunked vs serial relative max |dy| {d:.2e}', flush=True)
