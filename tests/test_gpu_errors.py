"""Error paths of the loader and the engine on the GPU (the reference's error contract,
rwkv.h:38-62, rwkv_file_format.inc:115-197, rwkv_model_loading.inc:128-419): malformed files are
rejected with the right flags and a NULL context -- never a fault or an exception across the ABI --
and a failed workspace allocation leaves the context usable."""
import ctypes
import os
import struct

import numpy as np
import pytest

from rwkv_lib import library

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
BB = {2: 18, 3: 20, 7: 22, 8: 24, 9: 34}

# rwkv.h:38-62 (flags = category << 8 | code)
E_FILE, E_MODEL_PARAMS = 2 << 8, 4 << 8
E_FILE_READ, E_SHAPE, E_DIMENSION, E_DATA_TYPE = 4, 10, 11, 8


def records(path):
    out = []
    with open(path, 'rb') as f:
        hdr = f.read(24)
        while True:
            h = f.read(12)
            if len(h) < 12:
                break
            nd, kl, ty = struct.unpack('<3I', h)
            ne = list(struct.unpack(f'<{nd}I', f.read(4 * nd)))
            key = f.read(kl)
            n = int(np.prod(ne))
            nb = n * 4 if ty == 0 else n * 2 if ty == 1 else n // 32 * BB[ty]
            out.append([ty, ne, key, f.read(nb)])
    return hdr, out


def write(path, hdr, recs):
    with open(path, 'wb') as f:
        f.write(hdr)
        for ty, ne, key, data in recs:
            f.write(struct.pack('<3I', len(ne), len(key), ty))
            f.write(struct.pack(f'<{len(ne)}I', *ne))
            f.write(key)
            f.write(data)


def load_flags(path):
    L = library()
    lib = L.library
    lib.rwkv_set_print_errors(None, False)
    try:
        ctx = lib.rwkv_init_from_file(path.encode(), 1, 99)
        err = lib.rwkv_get_last_error(None)
        if ctx:
            lib.rwkv_free(ctx)
        return ctx, err
    finally:
        lib.rwkv_set_print_errors(None, True)


def mutate(tmp_path, name, fn, src='tiny-rwkv-6v0-3m-Q5_0.bin'):
    hdr, recs = records(os.path.join(GOLD, src))
    fn(recs)
    p = str(tmp_path / name)
    write(p, hdr, recs)
    return p


def find(recs, key):
    return next(r for r in recs if r[2] == key.encode())


def test_truncated_file(tmp_path):
    data = open(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'), 'rb').read()
    p = str(tmp_path / 'trunc.bin')
    open(p, 'wb').write(data[: len(data) // 2])
    ctx, err = load_flags(p)
    assert not ctx and err & 0xff == E_FILE_READ


def test_huge_key_length(tmp_path):
    hdr, recs = records(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'))
    p = str(tmp_path / 'key.bin')
    with open(p, 'wb') as f:
        f.write(hdr)
        f.write(struct.pack('<4I', 1, 0x7fffffff, 0, 4))  # dims 1, key_len 2^31-1, FP32, ne0 4
    ctx, err = load_flags(p)
    assert not ctx and err & 0xff == E_FILE_READ


def test_matrix_with_wrong_shape(tmp_path):
    def fn(recs):
        r = find(recs, 'blocks.3.att.key.weight')
        r[1] = [r[1][0] // 2, r[1][1] * 2]  # K halved, M doubled: same bytes, wrong shape
    ctx, err = load_flags(mutate(tmp_path, 'shape.bin', fn))
    assert not ctx and err == E_MODEL_PARAMS | E_SHAPE


def test_vector_with_wrong_length(tmp_path):
    def fn(recs):
        r = find(recs, 'blocks.1.att.time_maa_k')
        r[1] = [r[1][0] // 2]
        r[3] = r[3][: len(r[3]) // 2]
    ctx, err = load_flags(mutate(tmp_path, 'vec.bin', fn))
    assert not ctx and err == E_MODEL_PARAMS | E_SHAPE


def test_maa_w2_shape(tmp_path):
    def fn(recs):
        r = find(recs, 'blocks.0.att.time_maa_w2')
        r[1] = [r[1][0], r[1][1] * 5]  # right element count, 2-D instead of [D, C, 5]
    ctx, err = load_flags(mutate(tmp_path, 'w2.bin', fn))
    assert not ctx and err & 0xff == E_SHAPE


def test_quantized_embedding_rejected(tmp_path):
    def fn(recs):
        e = find(recs, 'emb.weight')
        q = find(recs, 'blocks.0.att.key.weight')  # borrow a Q5_0 payload of the right byte count
        n = int(np.prod(e[1]))
        e[0] = q[0]
        e[3] = (q[3] * (n // 32 * BB[q[0]] // len(q[3]) + 1))[: n // 32 * BB[q[0]]]
    ctx, err = load_flags(mutate(tmp_path, 'emb.bin', fn))
    assert not ctx and err == E_MODEL_PARAMS | E_DATA_TYPE


def test_workspace_allocation_failure_recovers():
    """A sequence chunk whose workspace cannot be allocated fails cleanly (false, no fault), and the
    same context then evaluates normally (engine.hip ensure_workspace commits its capacity only
    after every allocation succeeded)."""
    L = library()
    lib = L.library
    ctx = L.rwkv_init_from_file(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'), 1, 99)
    lib.rwkv_set_print_errors(ctx.ptr, False)
    n = lib.rwkv_get_state_len(ctx.ptr)
    V = lib.rwkv_get_logits_len(ctx.ptr)
    st = np.zeros(n, np.float32)
    lg = np.zeros(V, np.float32)
    P = ctypes.POINTER(ctypes.c_float)
    assert lib.rwkv_eval(ctx.ptr, 34, None, st.ctypes.data_as(P), lg.ctypes.data_as(P))
    ref = lg.copy()
    dummy = ctypes.c_void_p(16)  # never dereferenced: the workspace allocation fails first
    assert not lib.rwkv_mi355x_eval_layers(ctx.ptr, None, 1 << 30, 1, 2, dummy, None, False, None)
    lib.rwkv_get_last_error(ctx.ptr)
    st2 = np.zeros(n, np.float32)
    assert lib.rwkv_eval(ctx.ptr, 34, None, st2.ctypes.data_as(P), lg.ctypes.data_as(P))
    assert np.array_equal(lg, ref) and np.array_equal(st2, st)
    L.rwkv_free(ctx)
