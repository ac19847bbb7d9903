"""The layer pipeline behind the C ABI (include/rwkv_mi355x.h rwkv_mi355x_init_pipeline,
RWKV_MI355X_PIPELINE): one process, P stage contexts, chunk c's residual stream forwarded stage to
stage by peer copies while the previous stage starts chunk c + 1.  On the one-GPU box every stage sits
on device 0 (the same code path; the peer copy is then a device-local copy).  rwkv_eval_sequence /
rwkv_eval on the pipeline context must equal a single-GPU context bit for bit -- logits and state,
fresh and carried state -- at the BASELINE config-4 width (v7-2.9B: C 2560, H 40, Q5_1) over several
256-token chunks, at BASELINE config 5's partition (v5-7B width, 8 stages, 4096 tokens in chunks of
1024), and on the tiny v6 checkpoint through the environment switch."""
import ctypes
import os

import numpy as np
import pytest
import torch  # noqa: F401  (torch's HIP runtime before the library's)

from oracle_ctypes import assert_bits_equal, gpu_variant
from rwkv_lib import library

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
P_F = ctypes.POINTER(ctypes.c_float)


def _seq(L, ctx, toks, state_in=None):
    n_vocab, n_state = L.rwkv_get_n_vocab(ctx), L.rwkv_get_state_len(ctx)
    t = np.ascontiguousarray(np.asarray(toks, np.int32))
    lg = np.zeros(n_vocab, np.float32)
    st = np.zeros(n_state, np.float32)
    sin = None if state_in is None else np.ascontiguousarray(state_in, np.float32).ctypes.data_as(P_F)
    assert L.rwkv_eval_sequence(ctx, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(t), sin,
                                st.ctypes.data_as(P_F), lg.ctypes.data_as(P_F))
    return lg, st


def _decode(L, ctx, toks, state):
    n_vocab = L.rwkv_get_n_vocab(ctx)
    st = np.array(state, np.float32, copy=True)
    lg = np.zeros(n_vocab, np.float32)
    for t in toks:
        assert L.rwkv_eval(ctx, int(t), st.ctypes.data_as(P_F), st.ctypes.data_as(P_F), lg.ctypes.data_as(P_F))
    return lg, st


@pytest.fixture(scope='module')
def v7_model(tmp_path_factory):
    p = str(tmp_path_factory.mktemp('pipeabi') / 'v7-2b9-q5_1-L4.bin')
    assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), 7, 4096, 2560, 4, 0, b'Q5_1', 31)
    return p


def test_pipeline_v7_width_four_stages(v7_model):
    """BASELINE config 4's partition: 4 stages of one layer each at the v7-2.9B width, 600 tokens
    (chunks of 256, 256, 88: the steady state and a ragged tail), then a carried-state second call."""
    L = library().library
    toks = [int(t) for t in np.random.default_rng(41).integers(0, 4096, 600)]
    single = L.rwkv_init_from_file(v7_model.encode(), 1, 99)
    assert single
    lg, st = _seq(L, single, toks)
    lg2, st2 = _seq(L, single, toks[:300], st)
    devs = (ctypes.c_int * 4)(0, 0, 0, 0)
    pipe = L.rwkv_mi355x_init_pipeline(v7_model.encode(), 1, 4, devs)
    assert pipe
    assert L.rwkv_mi355x_pipeline_stages(pipe) == 4
    assert L.rwkv_get_state_len(pipe) == L.rwkv_get_state_len(single)
    plg, pst = _seq(L, pipe, toks)
    assert_bits_equal(plg, lg, 'pipeline logits')
    assert_bits_equal(pst, st, 'pipeline state')
    plg2, pst2 = _seq(L, pipe, toks[:300], pst)
    assert_bits_equal(plg2, lg2, 'pipeline logits, carried state')
    assert_bits_equal(pst2, st2, 'pipeline state, carried state')
    # rwkv_eval through the pipeline (every stage in turn, one token)
    dlg, dst = _decode(L, single, toks[:3], st)
    pdlg, pdst = _decode(L, pipe, toks[:3], st)
    assert_bits_equal(pdlg, dlg, 'pipeline decode logits')
    assert_bits_equal(pdst, dst, 'pipeline decode state')
    # device-resident entry points refuse a pipeline context (it holds a layer range)
    arr = (ctypes.c_int32 * 1)(5)
    L.rwkv_set_print_errors(pipe, False)
    assert not L.rwkv_mi355x_eval_device(pipe, arr, 1, True, None, True)
    L.rwkv_free(pipe)
    L.rwkv_free(single)


def test_pipeline_env_switch_and_clone(monkeypatch):
    """RWKV_MI355X_PIPELINE=3 turns rwkv_init_from_file into a 3-stage pipeline (tiny v6, 12 layers);
    rwkv_clone_context of it is a pipeline with a fresh state; both equal a single context."""
    L = library().library
    path = os.path.join(GOLD, 'tiny-rwkv-6v0-3m-Q5_1.bin').encode()
    toks = [int(t) for t in np.random.default_rng(42).integers(0, 256, 300)]
    single = L.rwkv_init_from_file(path, 1, 99)
    lg, st = _seq(L, single, toks)
    monkeypatch.setenv('RWKV_MI355X_PIPELINE', '3')
    monkeypatch.setenv('RWKV_MI355X_PIPELINE_DEVICES', '0,0,0')
    pipe = L.rwkv_init_from_file(path, 1, 99)
    monkeypatch.delenv('RWKV_MI355X_PIPELINE')
    assert pipe and L.rwkv_mi355x_pipeline_stages(pipe) == 3
    plg, pst = _seq(L, pipe, toks)
    assert_bits_equal(plg, lg, 'env pipeline logits')
    assert_bits_equal(pst, st, 'env pipeline state')
    clone = L.rwkv_clone_context(pipe, 1)
    assert clone and L.rwkv_mi355x_pipeline_stages(clone) == 3
    clg, cst = _seq(L, clone, toks)
    assert_bits_equal(clg, lg, 'cloned pipeline logits')
    assert_bits_equal(cst, st, 'cloned pipeline state')
    L.rwkv_free(clone)
    L.rwkv_free(pipe)
    L.rwkv_free(single)


def _seq_chunks(L, ctx, toks, chunk):
    n_vocab, n_state = L.rwkv_get_n_vocab(ctx), L.rwkv_get_state_len(ctx)
    t = np.ascontiguousarray(np.asarray(toks, np.int32))
    lg = np.zeros(n_vocab, np.float32)
    st = np.zeros(n_state, np.float32)
    assert L.rwkv_eval_sequence_in_chunks(ctx, t.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(t), chunk, None,
                                          st.ctypes.data_as(P_F), lg.ctypes.data_as(P_F))
    return lg, st


def test_pipeline_v5_width_eight_stages(tmp_path):
    """BASELINE config 5's partition: 8 stages at the v5-7B width (C 4096, FFN 14336, 64 heads, Q4_1),
    one layer per stage, 4096 tokens through rwkv_eval_sequence_in_chunks(chunk_size = 1024), which a
    pipeline context takes as its chunk: equal to one single-GPU context bit for bit.  The oracle
    (GPU association) pins the same 8-stage pipeline on 160 tokens in chunks of 64 (64, 64, 32:
    ragged), the CPU-affordable length at this width.  Every stage sits on device 0 of the one-GPU
    test box; init reports no peer pairs then."""
    L = library().library
    p = str(tmp_path / 'v5-7b-q4_1-L8.bin')
    assert L.rwkv_mi355x_write_synthetic_model(p.encode(), 5, 4096, 4096, 8, 14336, b'Q4_1', 33)
    toks = [int(t) for t in np.random.default_rng(43).integers(0, 4096, 4096)]
    devs = (ctypes.c_int * 8)(*([0] * 8))
    pipe = L.rwkv_mi355x_init_pipeline(p.encode(), 1, 8, devs)
    assert pipe and L.rwkv_mi355x_pipeline_stages(pipe) == 8
    assert L.rwkv_mi355x_pipeline_peer_pairs(pipe) == 0
    plg, pst = _seq_chunks(L, pipe, toks, 1024)
    single = L.rwkv_init_from_file(p.encode(), 1, 99)
    assert single
    slg, sst = _seq_chunks(L, single, toks, 1024)
    L.rwkv_free(single)
    assert_bits_equal(plg, slg, '8-stage pipeline logits, T = 4096')
    assert_bits_equal(pst, sst, '8-stage pipeline state, T = 4096')
    short = toks[:160]
    olg, ost = gpu_variant(p, short, sequence=True)
    plg, pst = _seq_chunks(L, pipe, short, 64)
    assert_bits_equal(plg, olg, '8-stage pipeline logits vs oracle')
    assert_bits_equal(pst, ost, '8-stage pipeline state vs oracle')
    # the whole-state entry points act on every stage
    st = np.zeros(L.rwkv_get_state_len(pipe), np.float32)
    assert L.rwkv_mi355x_state_download(pipe, st.ctypes.data_as(P_F))
    assert_bits_equal(st, ost, 'pipeline rwkv_mi355x_state_download')
    assert L.rwkv_mi355x_sync(pipe)
    L.rwkv_set_print_errors(pipe, False)
    assert not L.rwkv_mi355x_stream(pipe)
    assert not L.rwkv_mi355x_device_state(pipe)
    assert not L.rwkv_mi355x_clone_context_on(pipe, 1, 0)
    L.rwkv_free(pipe)
