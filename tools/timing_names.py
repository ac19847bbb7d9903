"""Diagnostic: kernel-timing stats names/launches recorded for a few decode steps of a model."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
import rwkv_cpp  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, 'tests', 'golden', 'tiny-rwkv-6v0-3m-Q5_0.bin')
lib = rwkv_cpp.RWKVSharedLibrary(os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'))
L = lib.library
ctx = lib.rwkv_init_from_file(path, 1, 99)
L.rwkv_mi355x_set_kernel_timing(ctx.ptr, True)
assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
for t in (34, 105, 110):
    arr = (ctypes.c_int32 * 1)(t)
    assert L.rwkv_mi355x_eval_device(ctx.ptr, arr, 1, True, None, True)
n = L.rwkv_mi355x_kernel_stats(ctx.ptr, -1, None, 0, None, None, None, None)
for i in range(n):
    name = ctypes.create_string_buffer(128)
    la, ms, by, fl = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    L.rwkv_mi355x_kernel_stats(ctx.ptr, i, name, 128, ctypes.byref(la), ctypes.byref(ms), ctypes.byref(by), ctypes.byref(fl))
    print(repr(name.value), la.value, round(ms.value, 4), by.value)
L.rwkv_mi355x_set_kernel_timing(ctx.ptr, False)
lib.rwkv_free(ctx)
