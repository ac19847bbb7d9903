"""rwkv_eval with host state buffers runs the decode as layer-chunk graphs with the state copies
overlapped (engine.hip eval_host_chunked).  It must return exactly what the one-graph path with
whole-state copies returns (RWKV_MI355X_STATE_PIPELINE=0), for pageable and page-locked buffers,
under the reference ABI contract (rwkv_eval.inc:2-22: NULL state_in = fresh state, state_in ==
state_out allowed, NULL outputs skipped), bit for bit."""
import ctypes
import os

import numpy as np
import pytest
import torch  # before librwkv initialises HIP

from oracle_ctypes import assert_bits_equal
from rwkv_lib import library

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden')
P_F = ctypes.POINTER(ctypes.c_float)


def run(L, ctx, tokens, n_state, n_vocab, pinned, in_place):
    alloc = (lambda n: torch.zeros(n, dtype=torch.float32).pin_memory()) if pinned else \
        (lambda n: torch.zeros(n, dtype=torch.float32))
    s0, s1, lg = alloc(n_state), alloc(n_state), alloc(n_vocab)
    ptr = lambda t: ctypes.cast(t.data_ptr(), P_F)  # noqa: E731
    outs = []
    for i, t in enumerate(tokens):
        sin = None if i == 0 else (s0 if in_place or i % 2 else s1)
        sout = s0 if in_place or i % 2 == 0 else s1
        logits = None if i == 2 else lg  # one step without logits
        assert L.rwkv_eval(ctx, t, ptr(sin) if sin is not None else None, ptr(sout),
                           ptr(logits) if logits is not None else None)
        outs.append((sout.numpy().copy(), lg.numpy().copy()))
    # state_out NULL: logits only
    assert L.rwkv_eval(ctx, 7, ptr(s0), None, ptr(lg))
    outs.append((None, lg.numpy().copy()))
    return outs


@pytest.mark.parametrize('name', ['tiny-rwkv-6v0-3m-Q5_1.bin', 'tiny-rwkv-7v0-834K-FP32.bin',
                                  'tiny-rwkv-4v0-660K-FP16.bin', 'tiny-rwkv-5v2-730K-FP32.bin'])
@pytest.mark.parametrize('in_place', [True, False])
def test_pinned_host_state_bit_exact(name, in_place):
    check(os.path.join(GOLD, name), [34, 105, 110, 32, 77, 12], in_place)


def one_graph_context(lib, path):
    os.environ['RWKV_MI355X_STATE_PIPELINE'] = '0'
    try:
        return lib.rwkv_init_from_file(path, 1, 99)
    finally:
        del os.environ['RWKV_MI355X_STATE_PIPELINE']


def check(path, toks, in_place, chunk=None):
    lib = library()
    L = lib.library
    if chunk:
        os.environ['RWKV_MI355X_IO_CHUNK'] = str(chunk)
    try:
        ctx = lib.rwkv_init_from_file(path, 1, 99)
    finally:
        os.environ.pop('RWKV_MI355X_IO_CHUNK', None)
    ref = one_graph_context(lib, path)
    n_state, n_vocab = L.rwkv_get_state_len(ctx.ptr), L.rwkv_get_n_vocab(ctx.ptr)
    r = run(L, ref.ptr, toks, n_state, n_vocab, False, in_place)
    for pinned in (False, True):
        a = run(L, ctx.ptr, toks, n_state, n_vocab, pinned, in_place)
        for i, ((sa, la), (sr, lr)) in enumerate(zip(a, r)):
            if sr is not None:
                assert_bits_equal(sa, sr, f'pinned={pinned} step {i} state')
            assert_bits_equal(la, lr, f'pinned={pinned} step {i} logits')
    lib.rwkv_free(ctx)
    lib.rwkv_free(ref)


def test_pinned_real_width():
    """v6 at the 1B6 width (2 layers): the per-layer slices are real-sized."""
    lib = library()
    p = '/tmp/rwkv_pinned_v6.bin'
    assert lib.library.rwkv_mi355x_write_synthetic_model(p.encode(), 6, 4096, 2048, 2, 0, b'Q4_0', 3)
    check(p, [1, 2, 3, 400, 5], True)


@pytest.mark.parametrize('chunk', [1, 4])
def test_chunk_sizes(chunk):
    """Layer chunks of 1 (every layer its own graph) and uneven chunks (the last one shorter)."""
    lib = library()
    p = '/tmp/rwkv_pinned_v5.bin'
    assert lib.library.rwkv_mi355x_write_synthetic_model(p.encode(), 5, 1024, 512, 6, 0, b'Q5_1', 4)
    check(p, [9, 8, 7], False, chunk=chunk)


def test_host_state_after_async_device_eval():
    """rwkv_eval with a host state_in right after rwkv_mi355x_eval_device(sync = false): the chunked
    upload must wait for the decode steps still queued on the context's stream (they write the
    buffer the upload fills).  Equal to a fresh context given the same host state, bit for bit."""
    lib = library()
    L = lib.library
    p = '/tmp/rwkv_async_v6.bin'
    assert L.rwkv_mi355x_write_synthetic_model(p.encode(), 6, 4096, 2048, 4, 0, b'Q4_0', 6)
    ctx = lib.rwkv_init_from_file(p, 1, 99)
    ref = lib.rwkv_init_from_file(p, 1, 99)
    n_state, n_vocab = L.rwkv_get_state_len(ctx.ptr), L.rwkv_get_n_vocab(ctx.ptr)
    host = np.random.default_rng(5).standard_normal(n_state).astype(np.float32) * 0.1
    out_a, out_r = np.zeros(n_state, np.float32), np.zeros(n_state, np.float32)
    lg_a, lg_r = np.zeros(n_vocab, np.float32), np.zeros(n_vocab, np.float32)
    assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
    for t in range(12):   # queued, not waited for
        tok = np.array([t + 1], np.uint32)
        assert L.rwkv_mi355x_eval_device(ctx.ptr, tok.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 1, True,
                                         None, False)
    assert L.rwkv_eval(ctx.ptr, 77, host.ctypes.data_as(P_F), out_a.ctypes.data_as(P_F), lg_a.ctypes.data_as(P_F))
    assert L.rwkv_eval(ref.ptr, 77, host.ctypes.data_as(P_F), out_r.ctypes.data_as(P_F), lg_r.ctypes.data_as(P_F))
    assert_bits_equal(out_a, out_r, 'state after async device steps')
    assert_bits_equal(lg_a, lg_r, 'logits after async device steps')
    lib.rwkv_free(ctx)
    lib.rwkv_free(ref)
