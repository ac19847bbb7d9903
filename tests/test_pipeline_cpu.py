"""Layer pipeline on the CPU: the stage split, the layer-range restatement in the
oracle, and the multi-process driver (rwkv.cppy_amd/python/rwkv_cpp/pipeline.py) over gloo with
2 and 3 ranks, the oracle as every stage's computation.  The pipelined result must equal one
whole-sequence evaluation bit for bit (logits and every state slice)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle_ctypes import OracleModel

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
from rwkv_cpp.pipeline import (gather_state, layer_state_len, pipeline_eval_sequence, scatter_state,  # noqa: E402
                               stage_layers)

GOLD = os.path.join(REPO, 'tests', 'golden')
MODELS = ['tiny-rwkv-4v0-660K-FP32.bin', 'tiny-rwkv-5v2-730K-FP32.bin', 'tiny-rwkv-6v0-3m-Q5_0.bin',
          'tiny-rwkv-7v0-834K-FP32.bin']
TOKENS = [int(t) for t in np.random.default_rng(7).integers(0, 256, 23)]


def _layer_slices(m):
    per = m.n_embed * (2 + m.head_size) if m.arch_major >= 5 else 5 * m.n_embed
    return lambda l0, l1: slice(l0 * per, l1 * per)


@pytest.mark.parametrize('n_layer', [1, 4, 12, 24, 32])
@pytest.mark.parametrize('world', [1, 2, 3, 4, 8])
def test_stage_layers_partition(n_layer, world):
    if world > n_layer:
        with pytest.raises(ValueError):
            stage_layers(n_layer, world, 0)
        return
    ranges = [stage_layers(n_layer, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n_layer
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1


class OracleStage:
    """stage_fn on the oracle, keeping this stage's state across chunks."""

    def __init__(self, path):
        self.m = OracleModel(path)
        self.state = self.m.init_state()

    def __call__(self, tokens, l0, l1, x, want_logits):
        xs = x.numpy()
        lg, self.state = self.m.eval_layers(tokens, l0, l1, x=xs[0], vfirst=xs[1] if xs.shape[0] > 1 else None,
                                            state_in=self.state, want_logits=want_logits)
        return lg


@pytest.mark.parametrize('model', MODELS)
def test_oracle_layer_ranges_compose(model):
    """eval_layers over consecutive ranges and chunks == eval_sequence (the oracle's own check)."""
    path = os.path.join(GOLD, model)
    m = OracleModel(path)
    ref_lg, ref_st = m.eval_sequence(TOKENS)
    cut = m.n_layer // 2 + 1
    st = m.init_state()
    planes = 2 if m.arch_major == 7 else 1
    for a in range(0, len(TOKENS), 5):
        toks = TOKENS[a:a + 5]
        x = np.zeros((planes, len(toks), m.n_embed), np.float32)
        _, st = m.eval_layers(toks, 0, cut, x=x[0], vfirst=x[1] if planes == 2 else None, state_in=st)
        lg, st = m.eval_layers(toks, cut, m.n_layer, x=x[0], vfirst=x[1] if planes == 2 else None, state_in=st,
                               want_logits=True)
    assert np.array_equal(lg.view(np.uint32), ref_lg.view(np.uint32))
    assert np.array_equal(st.view(np.uint32), ref_st.view(np.uint32))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, path, chunk, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        stage = OracleStage(path)
        m = stage.m
        planes = 2 if m.arch_major == 7 else 1
        lg = pipeline_eval_sequence(stage, TOKENS, chunk, m.n_layer, m.n_embed, planes, rank, world,
                                    torch.device('cpu'))
        l0, l1 = stage_layers(m.n_layer, world, rank)
        sl = _layer_slices(m)(l0, l1)
        np.save(os.path.join(out_dir, f'state{rank}.npy'), stage.state[sl])
        if lg is not None:
            np.save(os.path.join(out_dir, 'logits.npy'), lg)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('model,world,chunk', [(MODELS[1], 2, 4), (MODELS[2], 2, 23), (MODELS[3], 3, 5),
                                               (MODELS[0], 2, 1)])
def test_pipeline_gloo_matches_whole_sequence(model, world, chunk, tmp_path):
    path = os.path.join(GOLD, model)
    mp.start_processes(_rank_main, args=(world, _free_port(), path, chunk, str(tmp_path)), nprocs=world,
                       start_method='spawn', join=True)
    m = OracleModel(path)
    ref_lg, ref_st = m.eval_sequence(TOKENS)
    lg = np.load(tmp_path / 'logits.npy')
    assert np.array_equal(lg.view(np.uint32), ref_lg.view(np.uint32))
    sl = _layer_slices(m)
    for r in range(world):
        l0, l1 = stage_layers(m.n_layer, world, r)
        got = np.load(tmp_path / f'state{r}.npy')
        assert np.array_equal(got.view(np.uint32), ref_st[sl(l0, l1)].view(np.uint32)), f'rank {r} state slice'


def _slice_rank_main(rank, world, port, path, chunk, out_dir):
    """Rank 0 owns a whole (non-fresh) state; each stage receives only its slice, runs the pipeline
    from it, and the final slices are gathered back on rank 0."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        stage = OracleStage(path)
        m = stage.m
        per = layer_state_len(m.n_embed, m.arch_major, m.head_size)
        full = None
        if rank == 0:
            _, full = m.eval_sequence(TOKENS[:7])  # a real mid-sequence state
        part = scatter_state(full, m.n_layer, per, rank, world)
        l0, l1 = stage_layers(m.n_layer, world, rank)
        np.save(os.path.join(out_dir, f'recv{rank}.npy'), part)
        stage.state[l0 * per:l1 * per] = part  # only this stage's layers are ever read
        planes = 2 if m.arch_major == 7 else 1
        lg = pipeline_eval_sequence(stage, TOKENS[7:], chunk, m.n_layer, m.n_embed, planes, rank, world,
                                    torch.device('cpu'))
        whole = gather_state(stage.state[l0 * per:l1 * per], m.n_layer, per, rank, world)
        if rank == 0:
            np.save(os.path.join(out_dir, 'state.npy'), whole)
        if lg is not None:
            np.save(os.path.join(out_dir, 'logits.npy'), lg)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('model,world,chunk', [(MODELS[2], 2, 4), (MODELS[3], 3, 6), (MODELS[0], 2, 16)])
def test_pipeline_state_slices_scatter_gather(model, world, chunk, tmp_path):
    """Each stage moves exactly its own state slice (stage_layers), and a pipeline started from a
    scattered mid-sequence state and gathered back equals one whole-sequence evaluation."""
    path = os.path.join(GOLD, model)
    mp.start_processes(_slice_rank_main, args=(world, _free_port(), path, chunk, str(tmp_path)), nprocs=world,
                       start_method='spawn', join=True)
    m = OracleModel(path)
    _, mid = m.eval_sequence(TOKENS[:7])
    ref_lg, ref_st = m.eval_sequence(TOKENS[7:], state_in=mid)
    per = layer_state_len(m.n_embed, m.arch_major, m.head_size)
    for r in range(world):
        l0, l1 = stage_layers(m.n_layer, world, r)
        got = np.load(tmp_path / f'recv{r}.npy')
        assert got.size == (l1 - l0) * per, f'rank {r} received {got.size} floats'
        assert np.array_equal(got.view(np.uint32), mid[l0 * per:l1 * per].view(np.uint32))
    assert np.array_equal(np.load(tmp_path / 'state.npy').view(np.uint32), ref_st.view(np.uint32))
    assert np.array_equal(np.load(tmp_path / 'logits.npy').view(np.uint32), ref_lg.view(np.uint32))
