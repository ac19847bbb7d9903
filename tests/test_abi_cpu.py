"""C-ABI checks that need no GPU: the library loads, exports every symbol include/*.h
declares, the host-side tooling (quantizer, synthetic writer) is byte-exact, and the
error convention of the reference (rwkv_error_handling.inc) holds."""
import ctypes
import hashlib
import json
import os
import re

import numpy as np
import pytest

from rwkv_lib import LIB_PATH, REPO, library
from oracle_ctypes import OracleModel, quantize_file as oracle_quantize

GOLD = os.path.join(os.path.dirname(__file__), 'golden')

RWKV_ERROR_ARGS = 1 << 8
RWKV_ERROR_FILE = 2 << 8
RWKV_ERROR_CTX = 6 << 8
RWKV_ERROR_FILE_OPEN = 2
RWKV_ERROR_FILE_MAGIC = 6
RWKV_ERROR_DATA_TYPE = 8
RWKV_ERROR_UNSUPPORTED = 9


def declared_symbols():
    names = set()
    for h in ('rwkv.h', 'rwkv_mi355x.h'):
        src = open(os.path.join(REPO, 'include', h)).read()
        for m in re.finditer(r'RWKV_API\s+[^;(]*?\b(rwkv_\w+)\s*\(', src):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB_PATH)
    names = declared_symbols()
    # the reference ABI (rwkv.h:70-224 + legacy rwkv.cpp:145-153)
    ref = {'rwkv_set_print_errors', 'rwkv_get_print_errors', 'rwkv_get_last_error', 'rwkv_init_from_file',
           'rwkv_clone_context', 'rwkv_eval', 'rwkv_eval_sequence', 'rwkv_eval_sequence_in_chunks',
           'rwkv_get_n_vocab', 'rwkv_get_n_embed', 'rwkv_get_n_layer', 'rwkv_get_state_len',
           'rwkv_get_logits_len', 'rwkv_init_state', 'rwkv_free', 'rwkv_quantize_model_file',
           'rwkv_get_system_info_string', 'rwkv_get_state_buffer_element_count',
           'rwkv_get_logits_buffer_element_count'}
    assert ref <= names
    for n in names:
        assert hasattr(lib, n), n


def test_quantizer_byte_exact_via_abi(tmp_path):
    kat = json.load(open(os.path.join(GOLD, 'quantizer_kat_sha256.json')))
    lib = library()
    n = 0
    for v in ['4v0-660K', '5v1-730K', '5v2-730K', '7v0-834K']:
        for src in ['FP32', 'FP16']:
            for q in ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0']:
                name = f'tiny-rwkv-{v}-{src}-to-{q}.bin'
                out = str(tmp_path / name)
                lib.rwkv_quantize_model_file(os.path.join(GOLD, f'tiny-rwkv-{v}-{src}.bin'), out, q)
                assert hashlib.sha256(open(out, 'rb').read()).hexdigest() == kat[name], name
                n += 1
    assert n == 40


def test_quantizer_errors(tmp_path):
    lib = library()
    L = lib.library
    L.rwkv_set_print_errors(None, False)
    assert not L.rwkv_quantize_model_file(b'/nonexistent.bin', str(tmp_path / 'o.bin').encode(), b'Q4_0')
    assert L.rwkv_get_last_error(None) == RWKV_ERROR_FILE | RWKV_ERROR_FILE_OPEN
    assert L.rwkv_get_last_error(None) == 0  # read-and-clear
    src = os.path.join(GOLD, 'tiny-rwkv-4v0-660K-FP32.bin').encode()
    assert not L.rwkv_quantize_model_file(src, str(tmp_path / 'o.bin').encode(), b'Q4_K')
    assert L.rwkv_get_last_error(None) == RWKV_ERROR_ARGS | RWKV_ERROR_DATA_TYPE
    # quantized input is rejected (must be FP32/FP16)
    qf = str(tmp_path / 'q.bin')
    lib.rwkv_quantize_model_file(src.decode(), qf, 'Q8_0')
    assert not L.rwkv_quantize_model_file(qf.encode(), str(tmp_path / 'o2.bin').encode(), b'Q4_0')
    assert L.rwkv_get_last_error(None) & RWKV_ERROR_FILE
    L.rwkv_set_print_errors(None, True)


def test_print_errors_flag():
    L = library().library
    assert L.rwkv_get_print_errors(None)
    L.rwkv_set_print_errors(None, False)
    assert not L.rwkv_get_print_errors(None)
    L.rwkv_set_print_errors(None, True)


@pytest.mark.skipif(os.path.exists('/dev/kfd') and os.access('/dev/kfd', os.R_OK), reason='GPU present')
def test_init_fails_loudly_without_gpu():
    L = library().library
    L.rwkv_set_print_errors(None, False)
    ptr = L.rwkv_init_from_file(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin').encode(), 2, 0)
    assert ptr is None
    assert L.rwkv_get_last_error(None) == RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED
    L.rwkv_set_print_errors(None, True)
    assert 'CPU_PATH=0' in library().rwkv_get_system_info_string()


@pytest.mark.parametrize('arch,fmt', [(4, 'Q8_0'), (5, 'Q4_1'), (6, 'Q4_0'), (7, 'Q5_1'), (6, 'FP16'), (7, 'FP32')])
def test_synthetic_model_loads_in_oracle(tmp_path, arch, fmt):
    """The synthetic checkpoints bench.py uses have the reference's tensor layout: the oracle
    (which follows rwkv_model_loading.inc's parameter table) loads and evaluates them."""
    L = library().library
    p = str(tmp_path / f'syn{arch}{fmt}.bin')
    assert L.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 512, 128, 2, 0, fmt.encode(), 42)
    m = OracleModel(p)
    assert m.arch_major == arch and m.n_embed == 128 and m.n_layer == 2 and m.n_vocab == 512
    if arch >= 5:
        assert m.head_size == 64
    lg, st = m.eval_serial([1, 2, 3])
    assert np.all(np.isfinite(lg)) and np.all(np.isfinite(st))
    # the writer's quantizer agrees with the oracle quantizer: re-quantizing an FP32 synthetic
    # file with the oracle gives the same bytes as the library's writer for that format
    if fmt not in ('FP16', 'FP32'):
        f32 = str(tmp_path / 'f32.bin')
        assert L.rwkv_mi355x_write_synthetic_model(f32.encode(), arch, 512, 128, 2, 0, b'FP32', 42)
        q1 = str(tmp_path / 'q1.bin')
        oracle_quantize(f32, q1, fmt)
        q2 = str(tmp_path / 'q2.bin')
        library().rwkv_quantize_model_file(f32, q2, fmt)
        assert open(q1, 'rb').read() == open(q2, 'rb').read()
