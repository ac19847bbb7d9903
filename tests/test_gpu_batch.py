"""Batched multi-context decode (rwkv_mi355x_eval_batch) on the GPU.

B independent contexts of one model advance one token each in one pass over the weights.  The
gate is bit-exactness: context i's logits and new state equal rwkv_eval(tokens[i], state_i) --
the reference's single-context call -- bit for bit, and hence the oracle's GPU-association
variant (checked directly on the tiny models).  The reference runs such contexts as clones side
by side (rwkv.h:93-99, rwkv.cpp:123-139; bit-identical clones: test_context_cloning.c:48).
"""
import ctypes
import os

import numpy as np
import pytest
import torch  # before librwkv initialises HIP (torch's own HIP runtime must come up first)

from oracle_ctypes import assert_bits_equal, gpu_variant
from rwkv_lib import RWKVModel, library

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
TEXT = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')


def prefixes(B, vocab):
    """B distinct token histories (lengths 0..) so every context starts from its own state."""
    return [[(TEXT[(7 * i + j) % len(TEXT)] + i) % vocab for j in range(i % 4)] for i in range(B)]


def contexts(model, hist):
    """Per-context states after each history (fresh state for an empty one), via rwkv_eval."""
    n = model._state_buffer_element_count
    states = np.zeros((len(hist), n), np.float32)
    fresh = np.zeros(n, np.float32)
    model._library.library.rwkv_init_state(model._ctx.ptr, fresh.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    for i, h in enumerate(hist):
        st = None
        for t in h:
            _, st = model.eval(t, st, st, None, use_numpy=True) if st is not None else \
                model.eval(t, None, None, None, use_numpy=True)
        states[i] = fresh if st is None else st
    return states


def check_batch(path, B, vocab=None, oracle=False):
    m = RWKVModel(library(), path)
    vocab = vocab or m.n_vocab
    hist = prefixes(B, vocab)
    states = contexts(m, hist)
    toks = [(97 + 13 * i) % vocab for i in range(B)]
    blg, bst = m.eval_batch(toks, states)
    for i in range(B):
        lg, st = m.eval(toks[i], states[i].copy(), None, None, use_numpy=True)
        assert_bits_equal(blg[i], lg, f'context {i} logits')
        assert_bits_equal(bst[i], st, f'context {i} state')
        if oracle and i < 3:
            glg, gst = gpu_variant(path, hist[i] + [toks[i]])
            assert_bits_equal(blg[i], glg, f'context {i} logits vs oracle')
            assert_bits_equal(bst[i], gst, f'context {i} state vs oracle')
    m.free()


TINY = ['tiny-rwkv-4v0-660K-FP32.bin', 'tiny-rwkv-5v1-730K-FP16.bin', 'tiny-rwkv-5v2-730K-FP32.bin',
        'tiny-rwkv-6v0-3m-Q5_0.bin', 'tiny-rwkv-6v0-3m-FP32-to-Q4_0.bin', 'tiny-rwkv-6v0-3m-FP16-to-Q5_1.bin',
        'tiny-rwkv-7v0-834K-FP32.bin', 'tiny-rwkv-7v0-834K-FP16.bin']


@pytest.mark.parametrize('name', TINY)
def test_batch_tiny_bit_exact(name):
    check_batch(os.path.join(GOLD, name), 5, oracle=True)


def test_batch_fresh_states_and_sizes():
    """state_in NULL (fresh contexts), B = 1, and B past the k_mm token pass (not a multiple of 4)."""
    path = os.path.join(GOLD, 'tiny-rwkv-6v0-3m-Q5_1.bin')
    m = RWKVModel(library(), path)
    toks = [3, 50, 97, 200, 7, 11, 13]
    blg, bst = m.eval_batch(toks, None)
    for i, t in enumerate(toks):
        lg, st = m.eval(t, None, None, None, use_numpy=True)
        assert_bits_equal(blg[i], lg, f'fresh context {i} logits')
        assert_bits_equal(bst[i], st, f'fresh context {i} state')
    one_lg, one_st = m.eval_batch([toks[0]], None)
    assert_bits_equal(one_lg[0], blg[0], 'B=1')
    m.free()
    check_batch(path, 37)


def test_batch_decode_loop_matches_serial():
    """Several batched steps in a row (graph replay with alternating buffers) == per-context serial."""
    path = os.path.join(GOLD, 'tiny-rwkv-7v0-834K-FP32.bin')
    m = RWKVModel(library(), path)
    B, steps = 4, 6
    seqs = [[(TEXT[(5 * i + j) % len(TEXT)]) for j in range(steps)] for i in range(B)]
    st = None
    for j in range(steps):
        lg, st = m.eval_batch([s[j] for s in seqs], st)
    for i in range(B):
        slg, sst = None, None
        for t in seqs[i]:
            slg, sst = m.eval(t, sst, sst, None, use_numpy=True) if sst is not None else \
                m.eval(t, None, None, None, use_numpy=True)
        assert_bits_equal(lg[i], slg, f'context {i} logits after {steps} steps')
        assert_bits_equal(st[i], sst, f'context {i} state after {steps} steps')
    m.free()


CONFIGS = {
    'v4-169m-q8_0': (4, 768, 0, 'Q8_0'),
    'v6-1b6-q4_0': (6, 2048, 0, 'Q4_0'),
    'v7-2b9-q5_1': (7, 2560, 0, 'Q5_1'),
    'v5-7b-q4_1': (5, 4096, 14336, 'Q4_1'),
}


@pytest.fixture(scope='module')
def cfg_dir(tmp_path_factory):
    return tmp_path_factory.mktemp('bcfg')


@pytest.mark.parametrize('name', sorted(CONFIGS))
@pytest.mark.parametrize('B', [8, 56])
def test_batch_real_width_bit_exact(cfg_dir, name, B):
    """BASELINE widths (2 layers, 4096-token vocabulary); B = 8 (decode matvec over the contexts)
    and B = 56 (past batch_gemm_min_ = 48: the int8-MFMA GEMM on token tiles)."""
    arch, C, F, fmt = CONFIGS[name]
    p = os.path.join(str(cfg_dir), f'{name}.bin')
    if not os.path.isfile(p):
        assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 4096, C, 2, F, fmt.encode(), 5)
    check_batch(p, B)


def test_batch_device_api_matches_host():
    """rwkv_mi355x_eval_batch_device on HBM buffers == the host-buffer call."""
    path = os.path.join(GOLD, 'tiny-rwkv-6v0-3m-FP32-to-Q4_0.bin')
    m = RWKVModel(library(), path)
    B = 6
    states = contexts(m, prefixes(B, m.n_vocab))
    toks = [5 * i + 1 for i in range(B)]
    hlg, hst = m.eval_batch(toks, states)
    L = library().library
    sin = torch.from_numpy(states).cuda()
    sout = torch.zeros_like(sin)
    lout = torch.zeros((B, m.n_vocab), dtype=torch.float32, device='cuda')
    arr = (np.array(toks, dtype=np.uint32))
    torch.cuda.synchronize()
    assert L.rwkv_mi355x_eval_batch_device(m._ctx.ptr, arr.ctypes.data, B, sin.data_ptr(), sout.data_ptr(),
                                           lout.data_ptr())
    assert L.rwkv_mi355x_sync(m._ctx.ptr)
    assert_bits_equal(lout.cpu().numpy(), hlg, 'device logits')
    assert_bits_equal(sout.cpu().numpy(), hst, 'device states')
    # same buffers for in and out are refused
    library().library.rwkv_set_print_errors(m._ctx.ptr, False)
    assert not L.rwkv_mi355x_eval_batch_device(m._ctx.ptr, arr.ctypes.data, B, sin.data_ptr(), sin.data_ptr(), None)
    m.free()
