"""Clones on a chosen GPU (rwkv_mi355x_clone_context_on, SURVEY.md §8 F4 / §8e decode replicas) and
per-layer state slices (rwkv_mi355x_state_{upload,download}_layers).  The one-GPU box places every
replica on GPU 0 (the same code path as other GPUs: the model is shared per device); with two or
more GPUs the replicas also run on GPU 1.  Every result is bit-exact to the single-context path."""
import ctypes
import os

import numpy as np
import pytest
import torch

from rwkv_lib import RWKVModel, library

pytestmark = pytest.mark.gpu

FP = ctypes.POINTER(ctypes.c_float)
GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def _synthetic(tmp_path, arch=6, fmt='Q4_0', n_layer=4, C=1024):
    L = library()
    p = str(tmp_path / f'rep{arch}{fmt}.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, C, n_layer, 0, fmt.encode(), 3)
    return p


def _seq(L, ctx, toks, state_in=None):
    n = L.library.rwkv_get_state_len(ctx.ptr)
    st = np.empty(n, np.float32)
    lg = np.empty(L.library.rwkv_get_n_vocab(ctx.ptr), np.float32)
    t = (ctypes.c_int32 * len(toks))(*toks)
    assert L.library.rwkv_eval_sequence(ctx.ptr, t, len(toks), None if state_in is None else state_in.ctypes.data_as(FP),
                                        st.ctypes.data_as(FP), lg.ctypes.data_as(FP))
    return lg, st


def _bits(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


@pytest.mark.parametrize('path', ['tiny-rwkv-6v0-3m-Q5_0.bin', 'tiny-rwkv-7v0-834K-FP32.bin'])
def test_clone_on_device_bit_exact(path):
    L = library()
    ctx = L.rwkv_init_from_file(os.path.join(GOLD, path), 1, 99)
    toks = [3, 17, 99, 4, 250, 8]
    ref = _seq(L, ctx, toks)
    ndev = torch.cuda.device_count()
    for d in sorted({0, min(1, ndev - 1)}):
        c = L.rwkv_mi355x_clone_context_on(ctx, 1, d)
        assert L.library.rwkv_mi355x_context_device(c.ptr) == d
        got = _seq(L, c, toks)
        assert _bits(got[0], ref[0]) and _bits(got[1], ref[1]), d
        # the clone keeps its own state: serial decode from the clone == sequence of the parent
        st = np.empty_like(ref[1])
        lg = np.empty_like(ref[0])
        for i, t in enumerate(toks):
            assert L.library.rwkv_eval(c.ptr, t, None if i == 0 else st.ctypes.data_as(FP), st.ctypes.data_as(FP),
                                       lg.ctypes.data_as(FP))
        assert _bits(lg, ref[0]) and _bits(st, ref[1]), d
        L.rwkv_free(c)
    L.rwkv_free(ctx)


def test_clone_on_bad_device_fails_with_args_flag():
    L = library()
    ctx = L.rwkv_init_from_file(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'), 1, 99)
    L.library.rwkv_set_print_errors(ctx.ptr, False)
    for bad in (-1, torch.cuda.device_count(), 1000):
        assert not L.library.rwkv_mi355x_clone_context_on(ctx.ptr, 1, bad)
        assert L.library.rwkv_get_last_error(ctx.ptr) & 256  # RWKV_ERROR_ARGS
    # the parent is untouched
    _seq(L, ctx, [1, 2, 3])
    L.rwkv_free(ctx)


def test_replica_pool_runs_sequences_concurrently_bit_exact(tmp_path):
    """Two replicas per available GPU (up to 4), 7 independent sequences dealt round-robin and
    evaluated from host threads at once: each equals its single-context evaluation."""
    from rwkv_cpp.replicas import ReplicaPool
    L = library()
    p = _synthetic(tmp_path)
    ctx = L.rwkv_init_from_file(p, 1, 99)
    rng = np.random.default_rng(5)
    seqs = [[int(t) for t in rng.integers(0, 1024, n)] for n in (5, 17, 33, 2, 9, 64, 12)]
    refs = [_seq(L, ctx, s) for s in seqs]
    ndev = torch.cuda.device_count()
    devices = [d % ndev for d in range(min(4, 2 * ndev))] if ndev > 1 else [0, 0]
    pool = ReplicaPool(L, ctx, devices)
    assert pool.devices() == devices
    out = pool.eval_sequences(seqs)
    for k, ((lg, st), (rl, rs)) in enumerate(zip(out, refs)):
        assert _bits(lg, rl) and _bits(st, rs), k
    # continuing every sequence from its returned state on the pool == one longer sequence
    more = [[7, 8, 9]] * len(seqs)
    out2 = pool.eval_sequences(more, states=[st for _, st in out])
    for k in range(len(seqs)):
        rl, rs = _seq(L, ctx, seqs[k] + more[k])
        assert _bits(out2[k][0], rl) and _bits(out2[k][1], rs), k
    pool.free()
    L.rwkv_free(ctx)


@pytest.mark.parametrize('arch,fmt', [(6, 'Q4_0'), (4, 'Q8_0'), (7, 'Q5_1')])
def test_state_slices_move_only_their_layers(tmp_path, arch, fmt):
    """Uploading a state as two layer slices (and downloading it the same way) equals the whole-state
    calls bit for bit, and each call moves exactly its slice's bytes."""
    L = library()
    lib = L.library
    p = _synthetic(tmp_path, arch, fmt, n_layer=5)
    ctx = L.rwkv_init_from_file(p, 1, 99)
    toks = [5, 6, 7, 300, 12]
    _, mid = _seq(L, ctx, toks)
    ref_lg, ref_st = _seq(L, ctx, [9, 10, 11], mid)
    n_layer, per = lib.rwkv_get_n_layer(ctx.ptr), lib.rwkv_mi355x_layer_state_len(ctx.ptr)
    assert per * n_layer == len(mid)
    h0, d0 = L.rwkv_mi355x_state_io_bytes(ctx)
    assert lib.rwkv_mi355x_state_upload_layers(ctx.ptr, mid[:2 * per].ctypes.data, 0, 2)
    part = np.ascontiguousarray(mid[2 * per:])
    assert lib.rwkv_mi355x_state_upload_layers(ctx.ptr, part.ctypes.data, 2, n_layer)
    h1, _ = L.rwkv_mi355x_state_io_bytes(ctx)
    assert h1 - h0 == len(mid) * 4
    t = np.array([9, 10, 11], np.uint32)
    assert lib.rwkv_mi355x_eval_device(ctx.ptr, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 3, False, None, True)
    a = np.empty(3 * per, np.float32)
    assert lib.rwkv_mi355x_state_download_layers(ctx.ptr, a.ctypes.data, 1, 4)
    _, d1 = L.rwkv_mi355x_state_io_bytes(ctx)
    assert d1 - d0 == 3 * per * 4
    assert _bits(a, ref_st[per:4 * per])
    # a fresh slice resets only its layers
    assert lib.rwkv_mi355x_state_upload_layers(ctx.ptr, None, 1, 2)
    full = np.empty(len(mid), np.float32)
    assert lib.rwkv_mi355x_state_download(ctx.ptr, full.ctypes.data_as(FP))
    fresh = np.zeros(per, np.float32)
    if arch == 4:
        C = lib.rwkv_get_n_embed(ctx.ptr)
        fresh[4 * C:] = -1e30
    assert _bits(full[per:2 * per], fresh)
    assert _bits(full[:per], ref_st[:per]) and _bits(full[2 * per:], ref_st[2 * per:])
    # bad ranges are refused with RWKV_ERROR_ARGS, never a fault
    lib.rwkv_set_print_errors(ctx.ptr, False)
    assert not lib.rwkv_mi355x_state_upload_layers(ctx.ptr, None, 3, 3)
    assert lib.rwkv_get_last_error(ctx.ptr) & 256
    assert not lib.rwkv_mi355x_state_download_layers(ctx.ptr, a.ctypes.data, 2, n_layer + 1)
    assert lib.rwkv_get_last_error(ctx.ptr) & 256
    L.rwkv_free(ctx)
