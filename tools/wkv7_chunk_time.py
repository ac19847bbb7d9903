"""Kernel timing source for the chunk-parallel WKV-7 (run under rocprofv3 --kernel-trace --stats):
serial k_wkv7_s64 and k_wkv7c_prep + carry + out at the v7-2.9B head count (H = 40) for T = 1024 and
4096 through rwkv_mi355x_selftest_wkv7, 5 runs each; prints the chunked form's distance from the
serial one for the last run."""
import ctypes
import os
import sys

import numpy as np
import torch  # noqa: F401

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
from rwkv_lib import library  # noqa: E402
from test_gpu_wkv_chunk import operands7  # noqa: E402

P = ctypes.POINTER(ctypes.c_float)
f = library().library.rwkv_mi355x_selftest_wkv7
f.argtypes = [ctypes.c_int] * 3 + [P] * 9
f.restype = ctypes.c_bool
H = 40
for T in (1024, 4096):
    ops = [np.ascontiguousarray(x) for x in operands7(T, H, seed=T)]
    outs = {}
    for chunked in (0, 1):
        for rep in range(5):
            y = np.zeros((T, H * 64), np.float32)
            so = np.zeros((H, 64, 64), np.float32)
            assert f(T, H, chunked, *[a.ctypes.data_as(P) for a in ops], so.ctypes.data_as(P), y.ctypes.data_as(P))
        outs[chunked] = (y, so)
    d = np.abs(outs[1][0] - outs[0][0]).max() / np.abs(outs[0][0]).max()
    print(f'T={T} H={H}: chunked vs serial relative max |dy| {d:.2e}', flush=True)
