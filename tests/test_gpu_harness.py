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


def test_world_tokenizer_generation_on_gpu(tmp_path):
    """The whole World-model harness on the GPU box: the reference's tokenizer vector text is
    tokenized with the World vocabulary (the reference's data file, tests/golden), a synthetic
    World-vocabulary v6 model (n_vocab 65536) evaluates the prompt and generates 12 tokens greedily
    through the unchanged RWKVModel interface, and every logit and chosen token equals the
    GPU-association oracle's; the generated ids decode back to text."""
    from rwkv_cpp.world_tokenizer import WorldTokenizer
    tok = WorldTokenizer(os.path.join(GOLD, 'rwkv_vocab_v20230424.txt'))
    text = 'I\'ll \'d test блабла 以下は、]) -> <|endoftext|><|padding|> int'
    ids = tok.encode(text)
    assert ids[:4] == [74, 5229, 274, 101]
    L = library()
    p = str(tmp_path / 'world-v6.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), 6, 65536, 256, 3, 0, b'Q5_1', 11)
    m = RWKVModel(L, p)
    set_variant(VARIANT_GPU)
    try:
        o = OracleAsModel(p)

        def run(model):
            logits, state = model.eval(ids[0], None, None, None, use_numpy=True)
            for t in ids[1:]:
                logits, state = model.eval(t, state, state, logits, use_numpy=True)
            out, lgs = [], [logits.copy()]
            for _ in range(12):
                t = sampling.sample_logits(logits, temperature=0.0)
                out.append(t)
                logits, state = model.eval(t, state, state, logits, use_numpy=True)
                lgs.append(logits.copy())
            return out, np.stack(lgs)

        gen_o, lg_o = run(o)
    finally:
        set_variant(0)
    gen, lg = run(m)
    m.free()
    assert gen == gen_o
    assert np.array_equal(lg.view(np.uint32), lg_o.view(np.uint32))
    assert isinstance(tok.decode([t for t in gen if t in tok.index_to_token]), str)
