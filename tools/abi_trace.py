"""ABI decode (rwkv_eval with host state, the reference contract rwkv_eval.inc:2-22) in a loop, for a
rocprofv3 --memory-copy-trace --kernel-trace run (tools/, GPU box).
Usage: python tools/abi_trace.py pageable|pinned [steps]
Prints the steady-state rate; the trace shows where each token's copies and kernels sit."""
import ctypes
import os
import sys
import time

import numpy as np
import torch  # before librwkv initialises HIP (torch's HIP runtime must come up first)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import rwkv_cpp  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'pageable'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = os.environ.get('CFG', 'v6-1b6-q4_0')
lib = rwkv_cpp.RWKVSharedLibrary(os.environ.get('RWKV_MI355X_BENCH_LIB') or
                                 os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'))
L = lib.library
arch, V, C, NL, F, fmt, label = bench.CONFIGS[cfg]
path = f'/tmp/rwkv_bench/{cfg}-seed1.bin'
os.makedirs('/tmp/rwkv_bench', exist_ok=True)
if not os.path.isfile(path):
    assert L.rwkv_mi355x_write_synthetic_model(path.encode(), arch, V, C, NL, F, fmt.encode(), 1)
ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
n_state, n_vocab = L.rwkv_get_state_len(ctx.ptr), L.rwkv_get_n_vocab(ctx.ptr)
PF = ctypes.POINTER(ctypes.c_float)
if kind == 'pinned':
    st_t = torch.zeros(n_state, dtype=torch.float32).pin_memory()
    lg_t = torch.zeros(n_vocab, dtype=torch.float32).pin_memory()
    st, lg = ctypes.cast(st_t.data_ptr(), PF), ctypes.cast(lg_t.data_ptr(), PF)
else:
    st_a = np.zeros(n_state, np.float32)
    lg_a = np.zeros(n_vocab, np.float32)
    st, lg = st_a.ctypes.data_as(PF), lg_a.ctypes.data_as(PF)
L.rwkv_init_state(ctx.ptr, st)
for i in range(8):
    assert L.rwkv_eval(ctx.ptr, (i * 7919) % V, st, st, lg)
t0 = time.perf_counter()
for i in range(steps):
    assert L.rwkv_eval(ctx.ptr, (i * 104729) % V, st, st, lg)
dt = time.perf_counter() - t0
print(f'{kind}: {steps / dt:.1f} tok/s ({dt / steps * 1e6:.0f} us/token)', flush=True)
