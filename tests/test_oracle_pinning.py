"""Pins the CPU oracle to the reference's own fixtures (CPU only).

- FP32 tiny models vs tests/expected-logits-*.bin (reference tests/, same prompt as
  logit_difference_validator.inc:48-83), max |dlogit| <= 1e-5.
- Quantizer byte-exact vs the reference's tiny-rwkv-*-to-Q*.bin (sha256 fixture).
- Quantized/FP16 signed sums within the reference's 1.05*|bound| rule, and the
  'pinned' (current-ggml) constants reproduced to 1e-4 relative (or 1e-5 absolute).
- Serial == sequence == chunked state, bit-exact (test_eval_sequence_in_chunks.c:45-55).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_ctypes import OracleModel, quantize_file

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
PROMPT = [34, 105, 110]
CONST = json.load(open(os.path.join(GOLD, 'reference_constants.json')))
FULL_VERSIONS = ['4v0-660K', '5v1-730K', '5v2-730K', '7v0-834K']


def expected(v):
    return np.fromfile(os.path.join(GOLD, f'expected-logits-{v}.bin'), np.float32)


@pytest.mark.parametrize('v', FULL_VERSIONS)
def test_fp32_expected_logits(v):
    m = OracleModel(os.path.join(GOLD, f'tiny-rwkv-{v}-FP32.bin'))
    lg, _ = m.eval_serial(PROMPT)
    d = lg - expected(v)
    assert np.abs(d).max() <= 1e-5
    assert abs(d.sum()) <= abs(CONST['full'][v]['FP32']) * 1.05
    lg2, _ = m.eval_sequence(PROMPT)
    assert np.abs(lg2 - expected(v)).max() <= 1e-5


@pytest.mark.parametrize('v', FULL_VERSIONS)
def test_fp16_signed_sum(v):
    m = OracleModel(os.path.join(GOLD, f'tiny-rwkv-{v}-FP16.bin'))
    lg, _ = m.eval_serial(PROMPT)
    s = float((lg - expected(v)).sum())
    bound = CONST['full'][v]['FP16']
    # 5v1 FP16 is one of the stale constants; bound still holds.
    assert abs(s) <= abs(bound) * 1.05


@pytest.mark.parametrize('v', FULL_VERSIONS)
@pytest.mark.parametrize('src', ['FP32', 'FP16'])
@pytest.mark.parametrize('q', ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
def test_quantizer_kat_and_signed_sum(v, src, q, tmp_path):
    kat = json.load(open(os.path.join(GOLD, 'quantizer_kat_sha256.json')))
    name = f'tiny-rwkv-{v}-{src}-to-{q}.bin'
    out = str(tmp_path / name)
    quantize_file(os.path.join(GOLD, f'tiny-rwkv-{v}-{src}.bin'), out, q)
    assert hashlib.sha256(open(out, 'rb').read()).hexdigest() == kat[name]
    m = OracleModel(out)
    lg, _ = m.eval_serial(PROMPT)
    s = float((lg - expected(v)).sum())
    bound = CONST[f'quantized_{src}'][v][q]
    if [v, f'{src}-to-{q}'] in CONST['pinned']:
        assert abs(s - bound) <= max(1e-4 * abs(bound), 1e-5), (s, bound)
    # the reference's own acceptance rule (logit_difference_validator.inc:68,83)
    assert abs(s) <= abs(bound) * 1.05, (s, bound)


@pytest.mark.parametrize('q', ['Q5_0', 'Q5_1'])
def test_v6_compat_files(q):
    m = OracleModel(os.path.join(GOLD, f'tiny-rwkv-6v0-3m-{q}.bin'))
    assert (m.arch_major, m.head_count, m.head_size) == (6, 16, 8)
    lg, _ = m.eval_serial(PROMPT)
    s = float((lg - expected('6v0-3m')).sum())
    bound = CONST['compat']['6v0-3m'][q]
    if q == 'Q5_0':
        assert abs(s - bound) <= 1e-4 * abs(bound)
    assert abs(s) <= abs(bound) * 1.05


def test_serial_sequence_chunked_bit_exact():
    # test_eval_sequence_in_chunks.c:69: 70-char prompt, chunk sizes 1, 2, 8, 10
    prompt = b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM'
    toks = list(prompt)
    m = OracleModel(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'))
    _, ref = m.eval_serial(toks)
    for chunk in (1, 2, 8, 10):
        st = None
        for i in range(0, len(toks), chunk):
            _, st = m.eval_sequence(toks[i:i + chunk], st)
        assert np.array_equal(st, ref)


def test_init_state_v4():
    m = OracleModel(os.path.join(GOLD, 'tiny-rwkv-4v0-660K-FP32.bin'))
    s = m.init_state()
    C = m.n_embed
    per = s.reshape(m.n_layer, 5, C)
    assert np.all(per[:, :4] == 0) and np.all(per[:, 4] == np.float32(-1e30))
