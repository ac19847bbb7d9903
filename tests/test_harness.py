"""Harness around the eval path on CPU: the World tokenizer, sampling and the
perplexity loop (rwkv.cppy_amd/python/rwkv_cpp/{world_tokenizer,sampling,perplexity}.py).

Pins: the reference's tokenizer test vector (python/rwkv_cpp/rwkv_world_tokenizer.test.py:4-17,
restated; the vocabulary is the reference's data file, copied to tests/golden by
golden/fetch_fixtures.sh); the perplexity loop over the CPU oracle, against a direct restatement of
measure_pexplexity.py:73-109's arithmetic.
"""
import os

import numpy as np
import pytest

from oracle_ctypes import OracleModel, gpu_variant  # noqa: F401
from rwkv_lib import PKG  # noqa: F401
from rwkv_cpp import perplexity, sampling
from rwkv_cpp.world_tokenizer import WorldTokenizer

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
VOCAB = os.environ.get('RWKV_WORLD_VOCAB', os.path.join(GOLD, 'rwkv_vocab_v20230424.txt'))


def test_world_tokenizer_reference_vector():
    t = WorldTokenizer(VOCAB)
    text = 'I\'ll \'d test блабла 以下は、]) -> <|endoftext|><|padding|> int'
    expected = [74, 5229, 274, 101, 32223, 5092, 27980, 2795, 27980, 33, 10399, 10258, 10139, 10079, 1682, 3463,
                295, 125, 25258, 7588, 2318, 125, 790, 125, 49520, 125, 63, 21888]
    assert t.encode(text) == expected
    assert t.decode(expected) == text
    # partial UTF-8 decodes with U+FFFD (the streaming contract of the reference)
    assert '�' in t.decode(t.encode('блабла')[:1] + [0x80 + 1])


def test_world_tokenizer_longest_match(tmp_path):
    p = tmp_path / 'v.txt'
    p.write_text("1 'a' 1\n2 'ab' 2\n3 'abc' 3\n4 'b' 1\n5 b'\\xff' 1\n6 'c' 1\n", encoding='utf-8')
    t = WorldTokenizer(str(p))
    assert t.encode('abcab') == [3, 2]
    assert t.encode('abbc') == [2, 4, 6]
    assert t.encode_bytes(b'a\xffc') == [1, 5, 6]
    with pytest.raises(ValueError):
        t.encode('z')


def test_sampling_semantics():
    rng = np.random.default_rng(0)
    logits = np.array([0.0, 3.0, 1.0, 2.0], np.float32)
    assert sampling.sample_logits(logits, temperature=0.0) == 1
    assert sampling.sample_logits(logits, temperature=0.0, logit_bias={0: 10.0}) == 0
    # top_p below the top probability keeps only the top token
    p = sampling.softmax(logits.astype(np.float64))
    assert all(sampling.sample_probs(p, 1.0, float(p.max()) * 0.9, rng=rng) == 1 for _ in range(50))
    # top_p 1 and temperature 1: the softmax distribution itself
    draws = np.bincount([sampling.sample_logits(logits, 1.0, 1.0, rng=rng) for _ in range(20000)], minlength=4)
    np.testing.assert_allclose(draws / draws.sum(), p, atol=0.015)
    with pytest.raises(ValueError):
        sampling.sample_probs(p, temperature=-1.0)


class OracleAsModel:
    """The RWKVModel.eval interface over the CPU oracle (GPU-association variant)."""

    def __init__(self, path):
        self.m = OracleModel(path)

    def eval(self, token, state_in, state_out=None, logits_out=None, use_numpy=True):
        return self.m.eval_sequence([token], state_in)


def test_perplexity_loop_on_oracle():
    path = os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin')
    toks = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')
    loss, ppl, n = perplexity.measure(OracleAsModel(path), toks, ignore_first_n=4)
    # restated reference arithmetic: serial eval, cross-entropy of the next token, exp(mean)
    m = OracleModel(path)
    st, losses = None, []
    for i in range(len(toks) - 1):
        lg, st = m.eval_sequence([toks[i]], st)
        if i + 1 >= 4:
            x = lg.astype(np.float64)
            losses.append(np.log(np.exp(x - x.max()).sum()) + x.max() - x[toks[i + 1]])
    assert n == len(losses)
    assert abs(loss - np.mean(losses)) < 1e-9 and abs(ppl - np.exp(np.mean(losses))) < 1e-6
    assert 1.0 < ppl < 256.0
