"""Layer pipeline on the GPU: rwkv_mi355x_eval_layers stages composed over layer
ranges and T-chunks give the whole-sequence result bit for bit, and the multi-process driver
(rwkv_cpp.pipeline) does too.  The one-GPU box runs the 2-rank driver with gloo as the wire
(both ranks on cuda:0; RCCL needs one GPU per rank) -- the nccl path is the same code with
device-resident messages, exercised by bench.py --gpus N."""
import os
import socket

import numpy as np
import pytest
import torch

from rwkv_lib import LIB_PATH, RWKVModel, library

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def _ctx_eval_layers(L, ctx, toks, l0, l1, x, want_logits, n_vocab):
    import ctypes
    lg = np.zeros(n_vocab, np.float32) if want_logits else None
    t = np.ascontiguousarray(np.asarray(toks, np.uint32))
    ok = L.library.rwkv_mi355x_eval_layers(ctx.ptr, t.ctypes.data, len(t), l0, l1, x[0].data_ptr(),
                                           x[1].data_ptr() if x.shape[0] > 1 else None, want_logits,
                                           lg.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None)
    assert ok
    return lg


def _synthetic(tmp_path, arch, fmt, n_layer=5, C=2048):
    L = library()
    p = str(tmp_path / f'pipe{arch}{fmt}C{C}L{n_layer}.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, C, n_layer, 0, fmt.encode(), 5)
    return p


@pytest.mark.parametrize('arch,fmt', [(6, 'Q4_0'), (7, 'Q5_1'), (5, 'Q4_1'), (4, 'Q8_0')])
def test_stage_composition_bit_exact(tmp_path, arch, fmt):
    """[0, a) then [a, b) then [b, L) per chunk of 24 tokens == one rwkv_eval_sequence of 70."""
    L = library()
    p = _synthetic(tmp_path, arch, fmt)
    m = RWKVModel(L, p)
    toks = [int(t) for t in np.random.default_rng(9).integers(0, 1024, 70)]
    ref_lg, ref_st = m.eval_sequence(toks, None, use_numpy=True)
    m.free()
    ctx = L.rwkv_init_from_file(p, 1, 99)
    n_layer, C, n_vocab = L.rwkv_get_n_layer(ctx), L.rwkv_get_n_embed(ctx), L.rwkv_get_n_vocab(ctx)
    assert L.library.rwkv_mi355x_state_upload(ctx.ptr, None)
    planes = 2 if arch == 7 else 1
    cuts = [(0, 2), (2, 3), (3, n_layer)]
    lg = None
    for a in range(0, len(toks), 24):
        ch = toks[a:a + 24]
        x = torch.zeros((planes, len(ch), C), dtype=torch.float32, device='cuda')
        for l0, l1 in cuts:
            lg = _ctx_eval_layers(L, ctx, ch, l0, l1, x, l1 == n_layer, n_vocab)
    st = np.zeros(L.rwkv_get_state_buffer_element_count(ctx), np.float32)
    assert L.library.rwkv_mi355x_state_download(ctx.ptr, st.ctypes.data_as(
        __import__('ctypes').POINTER(__import__('ctypes').c_float)))
    L.rwkv_free(ctx)
    assert np.array_equal(lg.view(np.uint32), ref_lg.view(np.uint32))
    assert np.array_equal(st.view(np.uint32), ref_st.view(np.uint32))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, path, toks, chunk, out_dir, async_):
    import ctypes
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(LIB_PATH), '..', 'python'))
    from rwkv_cpp import RWKVSharedLibrary
    from rwkv_cpp.pipeline import LibraryStage, model_n_layer, pipeline_eval_sequence, stage_layers
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        L = RWKVSharedLibrary(LIB_PATH)
        stage = LibraryStage.from_file(L, path, rank, world, async_=async_)   # this stage's layers only
        ctx = stage.ctx
        stage.reset_state()
        n_layer, C = model_n_layer(path), L.rwkv_get_n_embed(ctx)
        lg = pipeline_eval_sequence(stage, toks, chunk, n_layer, C, stage.planes, rank, world,
                                    torch.device('cuda', 0), wire_device=torch.device('cpu'))
        st = np.zeros(L.rwkv_get_state_buffer_element_count(ctx), np.float32)
        assert L.library.rwkv_mi355x_state_download(ctx.ptr, st.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        l0, l1 = stage_layers(n_layer, world, rank)
        per = len(st) // n_layer
        np.save(os.path.join(out_dir, f'state{rank}.npy'), st[l0 * per:l1 * per])
        np.save(os.path.join(out_dir, f'bytes{rank}.npy'),
                np.array([L.library.rwkv_mi355x_weight_bytes(ctx.ptr, False),
                          L.library.rwkv_mi355x_weight_bytes(ctx.ptr, True)]))
        if lg is not None:
            np.save(os.path.join(out_dir, 'logits.npy'), lg)
        L.rwkv_free(ctx)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('arch,fmt,chunk,world,async_,C,n_layer', [
    (6, 'Q4_0', 16, 2, False, 2048, 5), (7, 'Q5_1', 33, 2, True, 2048, 5), (5, 'Q4_1', 20, 3, True, 2048, 5),
    (7, 'Q5_1', 24, 4, True, 2560, 4)])   # the last: BASELINE config 4's four stages at the v7-2.9B width
def test_multi_process_pipeline_bit_exact(tmp_path, arch, fmt, chunk, world, async_, C, n_layer):
    """Stage contexts loaded with rwkv_mi355x_init_from_file_layers hold only their layers (HBM weight
    bytes ~1/world of the model's; the head only on the last stage) and the pipelined result equals
    one rwkv_eval_sequence bit for bit, synchronous and stream-ordered (async) stages alike."""
    import torch.multiprocessing as mp
    L = library()
    p = _synthetic(tmp_path, arch, fmt, n_layer, C)
    toks = [int(t) for t in np.random.default_rng(4).integers(0, 1024, 70)]
    m = RWKVModel(L, p)
    ref_lg, ref_st = m.eval_sequence(toks, None, use_numpy=True)
    n_layer = L.rwkv_get_n_layer(m._ctx)
    full_layers = L.library.rwkv_mi355x_weight_bytes(m._ctx.ptr, False)
    full_head = L.library.rwkv_mi355x_weight_bytes(m._ctx.ptr, True) - full_layers
    m.free()
    mp.start_processes(_rank_main, args=(world, _free_port(), p, toks, chunk, str(tmp_path), async_), nprocs=world,
                       start_method='spawn', join=True)
    assert np.array_equal(np.load(tmp_path / 'logits.npy').view(np.uint32), ref_lg.view(np.uint32))
    per = len(ref_st) // n_layer
    from rwkv_cpp.pipeline import stage_layers
    total = 0.0
    for r in range(world):
        l0, l1 = stage_layers(n_layer, world, r)
        got = np.load(tmp_path / f'state{r}.npy')
        assert np.array_equal(got.view(np.uint32), ref_st[l0 * per:l1 * per].view(np.uint32)), r
        lb, tb = np.load(tmp_path / f'bytes{r}.npy')
        # layers are near-equal in size (v7's layer 0 lacks the value-residual LoRA)
        assert lb <= full_layers * (l1 - l0) / n_layer * 1.05, (r, lb, full_layers)
        assert (tb - lb) == pytest.approx(full_head if r == world - 1 else 0.0, rel=1e-6, abs=1.0), r
        total += lb
    assert total == pytest.approx(full_layers, rel=1e-9)   # the stages partition the layer weights


def test_stage_context_rejects_whole_model_calls(tmp_path):
    """A stage context (layers [l0, l1) only) refuses rwkv_eval / rwkv_eval_sequence and layer ranges it
    does not hold, with the context's error flags set -- never a fault."""
    import ctypes
    L = library()
    lib = L.library
    p = _synthetic(tmp_path, 6, 'Q4_0')
    ptr = lib.rwkv_mi355x_init_from_file_layers(p.encode(), 1, 1, 3)
    assert ptr
    lib.rwkv_set_print_errors(ptr, False)
    C, n_vocab = lib.rwkv_get_n_embed(ptr), lib.rwkv_get_n_vocab(ptr)
    st = np.zeros(lib.rwkv_get_state_buffer_element_count(ptr), np.float32)
    lg = np.zeros(n_vocab, np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    assert not lib.rwkv_eval(ptr, 1, None, st.ctypes.data_as(fp), lg.ctypes.data_as(fp))
    assert lib.rwkv_get_last_error(ptr) != 0
    toks = (ctypes.c_int32 * 3)(1, 2, 3)
    assert not lib.rwkv_eval_sequence(ptr, toks, 3, None, st.ctypes.data_as(fp), lg.ctypes.data_as(fp))
    assert lib.rwkv_get_last_error(ptr) != 0
    x = torch.zeros((1, 3, C), dtype=torch.float32, device='cuda')
    t = np.array([1, 2, 3], np.uint32)
    assert lib.rwkv_mi355x_state_upload(ptr, None)
    assert not lib.rwkv_mi355x_eval_layers(ptr, t.ctypes.data, 3, 0, 2, x.data_ptr(), None, False, None)
    assert lib.rwkv_get_last_error(ptr) != 0
    assert lib.rwkv_mi355x_eval_layers(ptr, t.ctypes.data, 3, 1, 3, x.data_ptr(), None, False, None)
    assert lib.rwkv_get_last_error(ptr) == 0
    lib.rwkv_free(ptr)


def _slice_rank_main(rank, world, port, path, toks, chunk, out_dir, mid_path):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(LIB_PATH), '..', 'python'))
    from rwkv_cpp import RWKVSharedLibrary
    from rwkv_cpp.pipeline import (LibraryStage, gather_state, model_n_layer, pipeline_eval_sequence, scatter_state,
                                   stage_layers)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        L = RWKVSharedLibrary(LIB_PATH)
        stage = LibraryStage.from_file(L, path, rank, world, async_=True)
        n_layer, C = model_n_layer(path), L.rwkv_get_n_embed(stage.ctx)
        per = L.library.rwkv_mi355x_layer_state_len(stage.ctx.ptr)
        l0, l1 = stage_layers(n_layer, world, rank)
        mid = np.load(mid_path) if rank == 0 else None
        part = scatter_state(mid, n_layer, per, rank, world)
        stage.upload_state_slice(part, l0, l1)
        lg = pipeline_eval_sequence(stage, toks, chunk, n_layer, C, stage.planes, rank, world,
                                    torch.device('cuda', 0), wire_device=torch.device('cpu'))
        whole = gather_state(stage.download_state_slice(l0, l1), n_layer, per, rank, world)
        np.save(os.path.join(out_dir, f'io{rank}.npy'), np.array(L.rwkv_mi355x_state_io_bytes(stage.ctx)))
        if whole is not None:
            np.save(os.path.join(out_dir, 'state.npy'), whole)
        if lg is not None:
            np.save(os.path.join(out_dir, 'logits.npy'), lg)
        L.rwkv_free(stage.ctx)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('arch,fmt,world', [(6, 'Q4_0', 2), (7, 'Q5_1', 3)])
def test_pipeline_stages_move_only_their_state_slice(tmp_path, arch, fmt, world):
    """starting from a mid-sequence host state held by rank 0, each stage receives,
    uploads and downloads ONLY its layers' state slice (rwkv_mi355x_state_{upload,download}_layers;
    the context's PCIe byte counters equal the slice size), and the gathered final state and the
    logits equal one rwkv_eval_sequence from that state bit for bit."""
    import torch.multiprocessing as mp
    L = library()
    p = _synthetic(tmp_path, arch, fmt, 5, 2048)
    rng = np.random.default_rng(12)
    pre = [int(t) for t in rng.integers(0, 1024, 9)]
    toks = [int(t) for t in rng.integers(0, 1024, 40)]
    m = RWKVModel(L, p)
    _, mid = m.eval_sequence(pre, None, use_numpy=True)
    ref_lg, ref_st = m.eval_sequence(toks, mid, use_numpy=True)
    n_layer = L.rwkv_get_n_layer(m._ctx)
    per = L.library.rwkv_mi355x_layer_state_len(m._ctx.ptr)
    assert per * n_layer == len(mid)
    m.free()
    mid_path = str(tmp_path / 'mid.npy')
    np.save(mid_path, mid)
    mp.start_processes(_slice_rank_main, args=(world, _free_port(), p, toks, 16, str(tmp_path), mid_path),
                       nprocs=world, start_method='spawn', join=True)
    assert np.array_equal(np.load(tmp_path / 'logits.npy').view(np.uint32), ref_lg.view(np.uint32))
    assert np.array_equal(np.load(tmp_path / 'state.npy').view(np.uint32), ref_st.view(np.uint32))
    from rwkv_cpp.pipeline import stage_layers
    for r in range(world):
        l0, l1 = stage_layers(n_layer, world, r)
        h2d, d2h = np.load(tmp_path / f'io{r}.npy')
        assert h2d == d2h == (l1 - l0) * per * 4, (r, h2d, d2h)
