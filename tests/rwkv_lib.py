"""Locates and loads the product library (rwkv.cppy_amd/build/librwkv.so) through the
package's own ctypes mirror of the reference wrapper."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'rwkv.cppy_amd')
LIB_PATH = os.path.join(PKG, 'build', 'librwkv.so')
sys.path.insert(0, os.path.join(PKG, 'python'))

from rwkv_cpp import RWKVModel, RWKVSharedLibrary  # noqa: E402

_lib = None


def build_library():
    subprocess.check_call(['make', '-s', '-C', PKG, '-j8'])


def library() -> RWKVSharedLibrary:
    global _lib
    if _lib is None:
        if not os.path.isfile(LIB_PATH):
            build_library()
        _lib = RWKVSharedLibrary(LIB_PATH)
    return _lib


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False
