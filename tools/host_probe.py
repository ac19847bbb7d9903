"""Host-side cost of one decode token's graph launch (tools/, GPU box): times each
rwkv_mi355x_eval_device(sync=False) call (host enqueue) against the steady-state rate.
Usage: python tools/host_probe.py [config] [steps]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import rwkv_cpp  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'v6-1b6-q4_0'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
lib = rwkv_cpp.RWKVSharedLibrary(os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'))
L = lib.library
arch, V, C, NL, F, fmt, label = bench.CONFIGS[cfg]
path = f'/tmp/rwkv_bench/{cfg}-seed1.bin'
os.makedirs('/tmp/rwkv_bench', exist_ok=True)
if not os.path.isfile(path):
    assert L.rwkv_mi355x_write_synthetic_model(path.encode(), arch, V, C, NL, F, fmt.encode(), 1)
ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
toks = [np.array([(i * 7919) % V], np.int32) for i in range(steps + 20)]
P = ctypes.POINTER(ctypes.c_int32)
for i in range(20):
    assert L.rwkv_mi355x_eval_device(ctx.ptr, toks[i].ctypes.data_as(P), 1, True, None, False)
L.rwkv_mi355x_sync(ctx.ptr)
enq = []
t0 = time.perf_counter()
for i in range(20, 20 + steps):
    a = time.perf_counter()
    assert L.rwkv_mi355x_eval_device(ctx.ptr, toks[i].ctypes.data_as(P), 1, True, None, False)
    enq.append(time.perf_counter() - a)
t1 = time.perf_counter()
L.rwkv_mi355x_sync(ctx.ptr)
t2 = time.perf_counter()
enq = np.array(enq) * 1e6
print(f'{cfg}: {steps} tokens in {(t2 - t0) * 1e3:.1f} ms = {(t2 - t0) / steps * 1e6:.1f} us/token; '
      f'host enqueue p50 {np.median(enq):.1f} us p90 {np.percentile(enq, 90):.1f} us mean {enq.mean():.1f} us; '
      f'enqueue loop {(t1 - t0) / steps * 1e6:.1f} us/token, drain after loop {(t2 - t1) * 1e3:.2f} ms')
# one token at a time, synchronous: enqueue + GPU time with an idle queue
sy = []
for i in range(20):
    a = time.perf_counter()
    assert L.rwkv_mi355x_eval_device(ctx.ptr, toks[i].ctypes.data_as(P), 1, True, None, True)
    sy.append(time.perf_counter() - a)
print(f'synchronous single token: p50 {np.median(sy) * 1e6:.1f} us')
lib.rwkv_free(ctx)
