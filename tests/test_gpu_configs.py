"""BASELINE.json configurations at their real shapes on the GPU, bit-exact against the oracle.

Each configuration is a synthetic rwkv.cpp file (rwkv_mi355x_write_synthetic_model: seeded weights,
quantized by our KAT-exact quantizer) with the checkpoint's real widths -- n_embed, FFN width, head
count/size (reference rwkv_model_loading.inc:403-409), LoRA widths -- but 2 layers and a 4096-token
vocabulary so the CPU oracle finishes in seconds.  Decode (serial rwkv_eval) and sequence evaluation
must equal the oracle's GPU-association variant bit for bit, logits and state; serial == sequence on
the GPU.  These shapes select code paths the tiny models never reach: the K = 2560 two-unit decode
prologue (v7-2.9B), the register LayerNorm prologue at its n_embed 4096 edge with F = 14336 (v5-7B),
H = 40 heads (v7-2.9B), C = 768 (v4-169M).

test_v6_1b6_width_1024_tokens runs the headline workload's sequence length (T = 1024, one chunk)
at the v6-1B6 width, bit-exact against the oracle.
"""
import os

import numpy as np
import pytest

from oracle_ctypes import assert_bits_equal, gpu_variant
from rwkv_lib import RWKVModel, library

pytestmark = pytest.mark.gpu

# name: arch, n_embed, ffn (0 = arch default), format -- BASELINE.json configs 2..5
CONFIGS = {
    'v4-169m-q8_0': (4, 768, 0, 'Q8_0'),
    'v6-1b6-q4_0': (6, 2048, 0, 'Q4_0'),
    'v7-2b9-q5_1': (7, 2560, 0, 'Q5_1'),
    'v5-7b-q4_1': (5, 4096, 14336, 'Q4_1'),
}
VOCAB = 4096
LAYERS = 2


@pytest.fixture(scope='module')
def cfg_dir(tmp_path_factory):
    return tmp_path_factory.mktemp('cfg')


def cfg_model(cfg_dir, name, layers=LAYERS):
    arch, C, F, fmt = CONFIGS[name]
    p = os.path.join(str(cfg_dir), f'{name}-L{layers}.bin')
    if not os.path.isfile(p):
        assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, VOCAB, C, layers, F,
                                                                   fmt.encode(), 21)
    return p


def gpu_serial(model, tokens):
    logits, state = None, None
    for t in tokens:
        logits, state = model.eval(t, state, state, None, use_numpy=True) if state is not None else \
            model.eval(t, None, None, None, use_numpy=True)
    return logits, state


@pytest.mark.parametrize('name', sorted(CONFIGS))
def test_config_decode_bit_exact(cfg_dir, name):
    path = cfg_model(cfg_dir, name)
    toks = [int(t) for t in np.random.default_rng(7).integers(0, VOCAB, 6)]
    m = RWKVModel(library(), path)
    lg, st = gpu_serial(m, toks)
    glg, gst = gpu_variant(path, toks)
    assert_bits_equal(lg, glg, f'{name} decode logits')
    assert_bits_equal(st, gst, f'{name} decode state')
    m.free()


@pytest.mark.parametrize('name', sorted(CONFIGS))
def test_config_sequence_bit_exact(cfg_dir, name):
    path = cfg_model(cfg_dir, name)
    toks = [int(t) for t in np.random.default_rng(8).integers(0, VOCAB, 70)]
    m = RWKVModel(library(), path)
    lg, st = m.eval_sequence(toks, None, use_numpy=True)
    glg, gst = gpu_variant(path, toks, sequence=True)
    assert_bits_equal(lg, glg, f'{name} sequence logits')
    assert_bits_equal(st, gst, f'{name} sequence state')
    # chunked (the rwkv_eval_sequence_in_chunks driver) equals one call
    lg2, st2 = m.eval_sequence_in_chunks(toks, None, chunk_size=32, use_numpy=True)
    assert_bits_equal(lg2, lg, 'chunked logits')
    assert_bits_equal(st2, st, 'chunked state')
    m.free()


def test_v6_1b6_width_1024_tokens(cfg_dir):
    """The headline sequence length: 1024 tokens in one rwkv_eval_sequence at the v6-1B6 width."""
    path = cfg_model(cfg_dir, 'v6-1b6-q4_0')
    toks = [int(t) for t in np.random.default_rng(9).integers(0, VOCAB, 1024)]
    m = RWKVModel(library(), path)
    lg, st = m.eval_sequence(toks, None, use_numpy=True)
    glg, gst = gpu_variant(path, toks, sequence=True)
    assert_bits_equal(lg, glg, 'T=1024 logits')
    assert_bits_equal(st, gst, 'T=1024 state')
    m.free()
