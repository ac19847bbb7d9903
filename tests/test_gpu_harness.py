"""The Python harness on the GPU library: the reference's perplexity loop
(measure_pexplexity.py:73-109) and greedy generation (sampling at temperature 0, generate_completions
style) through the unchanged RWKVModel interface give exactly the oracle's numbers -- the logits
are bit-identical to the GPU-association oracle, so the losses and the chosen tokens are too."""
import os

import numpy as np
import pytest

from oracle_ctypes import VARIANT_GPU, OracleModel, set_variant
from rwkv_lib import RWKVModel, library
from rwkv_cpp import perplexity, sampling

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden')
TEXT = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')


class OracleAsModel:
    def __init__(self, path):
        self.m = OracleModel(path)

    def eval(self, token, state_in, state_out=None, logits_out=None, use_numpy=True):
        return self.m.eval_sequence([token], state_in)


@pytest.mark.parametrize('name', ['tiny-rwkv-6v0-3m-Q5_1.bin', 'tiny-rwkv-7v0-834K-FP16.bin'])
def test_perplexity_and_greedy_generation_match_oracle(name):
    path = os.path.join(GOLD, name)
    m = RWKVModel(library(), path)
    loss, ppl, n = perplexity.measure(m, TEXT, ignore_first_n=8)
    set_variant(VARIANT_GPU)
    try:
        o = OracleAsModel(path)
        oloss, oppl, on = perplexity.measure(o, TEXT, ignore_first_n=8)
        # greedy continuation of the prompt, 16 tokens
        def greedy(model):
            logits, state = None, None
            for t in TEXT[:20]:
                logits, state = model.eval(t, state, state, logits, use_numpy=True)
            out = []
            for _ in range(16):
                t = sampling.sample_logits(logits, temperature=0.0)
                out.append(t)
                logits, state = model.eval(t, state, state, logits, use_numpy=True)
            return out
        gen_o = greedy(o)
    finally:
        set_variant(0)
    assert (loss, ppl, n) == (oloss, oppl, on)
    assert greedy(m) == gen_o
    m.free()
