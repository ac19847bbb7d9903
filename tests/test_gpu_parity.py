"""GPU parity: librwkv.so on the MI355X vs the CPU oracle and the reference's fixtures.

The gate is BIT-EXACTNESS: every tiny model x format (the reference's fixtures and our KAT-exact
quantizations of them), serial decode and sequence evaluation, must equal the oracle's
GPU-association variant (oracle.c, variant bit 8: the same ggml semantics evaluated in the
kernels' documented association and with their exp/tanh) bit for bit, logits and state.

Beside it, bounds against the reference semantics (written here, see DESIGN.md "Parity"):
  * FP32 weights: |logit_gpu - logit_oracle_v0| <= 1e-3 (north-star bound), state <= 1e-3,
    and FP32 logits vs the reference's expected-logits <= 1e-3.
  * FP16 / quantized weights: activations are rounded to fp16 / re-quantized to Q8 blocks at
    every matmul (ggml numerics), so a last-bit difference of association can flip one rounding
    step, and some tiny checkpoints (5v1/5v2) amplify that chaotically.  The distance to the
    ggml-order oracle (variant 0) is therefore bounded by max(1e-3, 1.5 * noise), noise = the
    largest deviation among the oracle's own 7 re-associated restatements; it documents that
    the GPU association is one more valid restatement -- the bit-exact gate above is the check.
  * the reference's signed-sum rule |sum(logits - expected)| <= 1.05*|bound| exactly as written
    (logit_difference_validator.inc:68,83: fp32 sum in index order), no widening.
  * Layout/bookkeeping properties are bit-exact: serial == sequence == chunked state,
    NULL-logits state, cloned contexts (reference tests/test_eval_sequence_in_chunks.c,
    test_logit_calculation_skipping.c, test_context_cloning.c).
"""
import json
import os

import numpy as np
import pytest

from oracle_ctypes import OracleModel, assert_bits_equal, gpu_variant, noise_band
from rwkv_lib import RWKVModel, library

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
PROMPT = [34, 105, 110]
CONST = json.load(open(os.path.join(GOLD, 'reference_constants.json')))
VERSIONS = ['4v0-660K', '5v1-730K', '5v2-730K', '7v0-834K']
LONG = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')


def expected(v):
    return np.fromfile(os.path.join(GOLD, f'expected-logits-{v}.bin'), np.float32)


def diff_sum_f32(lg, ref):
    """The reference's difference sum: one float accumulator over the vocabulary in index order
    (logit_difference_validator.inc:60-66)."""
    d = np.asarray(lg, np.float32) - np.asarray(ref, np.float32)
    return float(np.cumsum(d, dtype=np.float32)[-1])


def assert_signed_sum(lg, v, bound, variants=None):
    """The reference rule as written: |sum(logits - expected)| <= 1.05 * |bound|
    (logit_difference_validator.inc:68,83).  Every case of this file meets it without any widening
    (round 6: each of the 48 tiny-model cases computed on the oracle's GPU-association variant, which
    the GPU equals bit for bit); `variants` is unused and kept for the callers' signature."""
    s = diff_sum_f32(lg, expected(v))
    assert abs(s) <= abs(bound) * 1.05, (s, bound)


def gpu_serial(model, tokens, state=None):
    logits = None
    for t in tokens:
        logits, state = model.eval(t, state, state, None, use_numpy=True) if state is not None else \
            model.eval(t, None, None, None, use_numpy=True)
    return logits, state


@pytest.fixture(scope='module')
def quantized_dir(tmp_path_factory):
    return tmp_path_factory.mktemp('q')


def model_path(v, fmt, qdir):
    if fmt in ('FP32', 'FP16'):
        return os.path.join(GOLD, f'tiny-rwkv-{v}-{fmt}.bin')
    src, q = fmt.split('-to-')
    out = os.path.join(str(qdir), f'tiny-rwkv-{v}-{fmt}.bin')
    if not os.path.isfile(out):
        library().rwkv_quantize_model_file(os.path.join(GOLD, f'tiny-rwkv-{v}-{src}.bin'), out, q)
    return out


@pytest.mark.parametrize('v', VERSIONS)
@pytest.mark.parametrize('fmt', ['FP32', 'FP16'])
def test_float_models_match_oracle(v, fmt, quantized_dir):
    path = model_path(v, fmt, quantized_dir)
    m = RWKVModel(library(), path, gpu_layer_count=99)
    lg, st = gpu_serial(m, PROMPT)
    glg, gst = gpu_variant(path, PROMPT)
    assert_bits_equal(lg, glg, 'logits')
    assert_bits_equal(st, gst, 'state')
    olg, ost, noise, variants = noise_band(path, PROMPT)
    tol = 1e-3 if fmt == 'FP32' else max(1e-3, 1.5 * noise)
    assert np.abs(lg - olg).max() <= tol, (np.abs(lg - olg).max(), noise)
    assert np.abs(st - ost).max() <= max(tol, 1e-3)
    if fmt == 'FP32':
        assert np.abs(lg - expected(v)).max() <= 1e-3
    assert_signed_sum(lg, v, CONST['full'][v][fmt], variants)
    m.free()


@pytest.mark.parametrize('v', VERSIONS)
@pytest.mark.parametrize('q', ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
@pytest.mark.parametrize('src', ['FP32', 'FP16'])
def test_quantized_models_match_oracle(v, q, src, quantized_dir):
    fmt = f'{src}-to-{q}'
    path = model_path(v, fmt, quantized_dir)
    m = RWKVModel(library(), path)
    lg, st = gpu_serial(m, PROMPT)
    glg, gst = gpu_variant(path, PROMPT)
    assert_bits_equal(lg, glg, 'logits')
    assert_bits_equal(st, gst, 'state')
    olg, _, noise, variants = noise_band(path, PROMPT)
    assert np.abs(lg - olg).max() <= max(1e-3, 1.5 * noise), (np.abs(lg - olg).max(), noise)
    assert_signed_sum(lg, v, CONST[f'quantized_{src}'][v][q], variants)
    m.free()


DUP_V6 = {'FP32-to-Q5_0': 'Q5_0', 'FP32-to-Q5_1': 'Q5_1'}
V6_FIXTURES = ['Q5_0', 'Q5_1'] + [f'{s}-to-{q}' for s in ('FP32', 'FP16') for q in ('Q4_0', 'Q4_1', 'Q5_0', 'Q5_1')]


@pytest.mark.parametrize('fmt', V6_FIXTURES)
def test_v6_reference_fixtures(fmt):
    """Every v6 tiny model the reference ships (tests/tiny-rwkv-6v0-3m-*.bin; the FP32/FP16 sources
    are missing, .MISSING_LARGE_BLOBS): bit-exact to the GPU-association oracle, serial and sequence,
    and the reference's signed-sum rule (test_tiny_rwkv.c:163-227 / compat :295-308)."""
    # the reference's FP32-to-Q5_0 / -Q5_1 files are byte-identical to its -Q5_0 / -Q5_1 files (same
    # sha256): one copy is kept, checked against both sets of bounds
    path = os.path.join(GOLD, f"tiny-rwkv-6v0-3m-{DUP_V6.get(fmt, fmt)}.bin")
    m = RWKVModel(library(), path)
    lg, st = gpu_serial(m, PROMPT)
    glg, gst = gpu_variant(path, PROMPT)
    assert_bits_equal(lg, glg, 'logits')
    assert_bits_equal(st, gst, 'state')
    slg, sst = m.eval_sequence(LONG, None, use_numpy=True)
    oslg, osst = gpu_variant(path, LONG, sequence=True)
    assert_bits_equal(slg, oslg, 'sequence logits')
    assert_bits_equal(sst, osst, 'sequence state')
    olg, _, noise, variants = noise_band(path, PROMPT)
    assert np.abs(lg - olg).max() <= max(1e-3, 1.5 * noise), (np.abs(lg - olg).max(), noise)
    if '-to-' in fmt:
        s, q = fmt.split('-to-')
        bound = CONST[f'quantized_{s}']['6v0-3m'][q]
    else:
        bound = CONST['compat']['6v0-3m'][fmt]
    assert_signed_sum(lg, '6v0-3m', bound, variants)
    m.free()


@pytest.mark.parametrize('path', [f'tiny-rwkv-{v}-FP32.bin' for v in VERSIONS] + ['tiny-rwkv-6v0-3m-Q5_1.bin'])
def test_sequence_equals_serial_bit_exact(path):
    """test_eval_sequence_in_chunks.c:45-55 on every architecture."""
    m = RWKVModel(library(), os.path.join(GOLD, path))
    lg_ser, st_ser = gpu_serial(m, LONG)
    for chunk in (1, 2, 8, 10):
        lg, st = m.eval_sequence_in_chunks(LONG, None, chunk_size=chunk, use_numpy=True)
        assert np.array_equal(st, st_ser), chunk
        assert np.array_equal(lg, lg_ser), chunk
    lg, st = m.eval_sequence(LONG, None, use_numpy=True)
    assert np.array_equal(st, st_ser)
    # chunk by hand through eval_sequence with host state in between
    st = None
    for i in range(0, len(LONG), 7):
        lg, st = m.eval_sequence(LONG[i:i + 7], st, st if st is not None else None, use_numpy=True)
    assert np.array_equal(st, st_ser)
    m.free()


@pytest.mark.parametrize('v', VERSIONS)
@pytest.mark.parametrize('fmt', ['FP32', 'FP16', 'FP32-to-Q4_0', 'FP16-to-Q5_1', 'FP32-to-Q8_0', 'FP16-to-Q4_1',
                                 'FP32-to-Q5_0'])
def test_sequence_matches_oracle_bit_exact(v, fmt, quantized_dir):
    """70-token rwkv_eval_sequence (sequence kernels: MFMA GEMM, chunked wkv) equals the
    GPU-association oracle's sequence evaluation bit for bit; FP32 also within 1e-3 of variant 0."""
    path = model_path(v, fmt, quantized_dir)
    m = RWKVModel(library(), path)
    lg, st = m.eval_sequence(LONG, None, use_numpy=True)
    glg, gst = gpu_variant(path, LONG, sequence=True)
    assert_bits_equal(lg, glg, 'logits')
    assert_bits_equal(st, gst, 'state')
    if fmt == 'FP32':
        olg, ost = OracleModel(path).eval_sequence(LONG)
        assert np.abs(lg - olg).max() <= 1e-3
        assert np.abs(st - ost).max() <= 1e-3
    m.free()


def test_logit_skipping_keeps_state():
    """test_logit_calculation_skipping.c:90-166"""
    L = library()
    path = os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin')
    m = RWKVModel(L, path)
    prompt = list(b'hello world')
    _, st_a = gpu_serial(m, prompt)
    n = m._state_buffer_element_count
    st_b = np.zeros(n, np.float32)
    import ctypes
    P = ctypes.POINTER(ctypes.c_float)
    lib = L.library
    assert lib.rwkv_eval(m._ctx.ptr, prompt[0], None, st_b.ctypes.data_as(P), None)
    for t in prompt[1:]:
        assert lib.rwkv_eval(m._ctx.ptr, t, st_b.ctypes.data_as(P), st_b.ctypes.data_as(P), None)
    assert np.array_equal(st_a, st_b)
    arr = (ctypes.c_int32 * len(prompt))(*prompt)
    st_c = np.zeros(n, np.float32)
    st_d = np.zeros(n, np.float32)
    lg = np.zeros(m._logits_buffer_element_count, np.float32)
    assert lib.rwkv_eval_sequence(m._ctx.ptr, ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32)), len(prompt), None,
                                  st_c.ctypes.data_as(P), lg.ctypes.data_as(P))
    assert lib.rwkv_eval_sequence(m._ctx.ptr, ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32)), len(prompt), None,
                                  st_d.ctypes.data_as(P), None)
    assert np.array_equal(st_c, st_d)
    m.free()


def test_context_cloning():
    """test_context_cloning.c:10-56: a clone gives identical logits after the original is freed."""
    L = library()
    lib = L.library
    ctx = L.rwkv_init_from_file(os.path.join(GOLD, 'tiny-rwkv-5v2-730K-FP32.bin'), 2, 0)
    n = lib.rwkv_get_state_len(ctx.ptr)
    V = lib.rwkv_get_logits_len(ctx.ptr)
    prompt = list(b'hello world')
    st = np.zeros(n, np.float32)
    lg = np.zeros(V, np.float32)
    L.rwkv_eval(ctx, prompt[0], None, st.ctypes.data, lg.ctypes.data)
    for t in prompt[1:]:
        L.rwkv_eval(ctx, t, st.ctypes.data, st.ctypes.data, lg.ctypes.data)
    expected_lg = lg.copy()
    ctx2 = lib.rwkv_clone_context(ctx.ptr, 2)
    assert ctx2 and ctx2 != ctx.ptr
    L.rwkv_free(ctx)
    from rwkv_cpp.rwkv_cpp_shared_library import RWKVContext
    c2 = RWKVContext(ctx2)
    lg2 = np.zeros(V, np.float32)
    L.rwkv_eval(c2, prompt[0], None, st.ctypes.data, lg2.ctypes.data)
    for t in prompt[1:]:
        L.rwkv_eval(c2, t, st.ctypes.data, st.ctypes.data, lg2.ctypes.data)
    assert np.array_equal(expected_lg, lg2)
    L.rwkv_free(c2)


def test_error_flags_on_gpu():
    L = library()
    lib = L.library
    ctx = L.rwkv_init_from_file(os.path.join(GOLD, 'tiny-rwkv-4v0-660K-FP32.bin'), 1, 0)
    lib.rwkv_set_print_errors(ctx.ptr, False)
    n = lib.rwkv_get_state_len(ctx.ptr)
    st = np.zeros(n, np.float32)
    import ctypes
    P = ctypes.POINTER(ctypes.c_float)
    assert not lib.rwkv_eval(ctx.ptr, 256, None, st.ctypes.data_as(P), None)
    assert lib.rwkv_get_last_error(ctx.ptr) == (1 << 8)
    assert lib.rwkv_get_last_error(ctx.ptr) == 0
    assert not lib.rwkv_eval_sequence(ctx.ptr, None, 0, None, None, None)
    assert lib.rwkv_get_last_error(ctx.ptr) == (1 << 8)
    assert lib.rwkv_eval_sequence(ctx.ptr, None, 5, None, None, None)  # build-only
    # rwkv_init_state: v4 pp = -1e30
    lib.rwkv_init_state(ctx.ptr, st.ctypes.data_as(P))
    C = lib.rwkv_get_n_embed(ctx.ptr)
    assert np.all(st.reshape(-1, 5, C)[:, 4] == np.float32(-1e30))
    L.rwkv_free(ctx)
    lib.rwkv_set_print_errors(None, False)
    assert L.library.rwkv_init_from_file(b'/nonexistent', 1, 0) is None
    assert lib.rwkv_get_last_error(None) == (2 << 8) | 2
    lib.rwkv_set_print_errors(None, True)


def test_device_resident_matches_abi():
    L = library()
    lib = L.library
    path = os.path.join(GOLD, 'tiny-rwkv-6v0-3m-Q5_0.bin')
    m = RWKVModel(L, path)
    lg_abi, st_abi = gpu_serial(m, LONG[:20])
    import ctypes
    P = ctypes.POINTER(ctypes.c_float)
    assert lib.rwkv_mi355x_state_upload(m._ctx.ptr, None)
    lg = np.zeros(m._logits_buffer_element_count, np.float32)
    for t in LONG[:19]:
        arr = (ctypes.c_int32 * 1)(t)
        assert lib.rwkv_mi355x_eval_device(m._ctx.ptr, ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32)), 1, False, None, False)
    arr = (ctypes.c_int32 * 1)(LONG[19])
    assert lib.rwkv_mi355x_eval_device(m._ctx.ptr, ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32)), 1, True,
                                       lg.ctypes.data_as(P), True)
    st = np.zeros(m._state_buffer_element_count, np.float32)
    assert lib.rwkv_mi355x_state_download(m._ctx.ptr, st.ctypes.data_as(P))
    assert np.array_equal(st, st_abi)
    assert np.array_equal(lg, lg_abi)
    m.free()


@pytest.mark.parametrize('arch,fmt', [(6, 'Q4_0'), (7, 'Q5_1'), (5, 'Q4_1'), (4, 'Q8_0'), (6, 'FP16')])
def test_synthetic_real_width_matches_oracle(tmp_path, arch, fmt):
    """Real widths (C=2048, S=64 heads, LoRA dims of the checkpoints), 2 layers, vs oracle."""
    L = library()
    p = str(tmp_path / f'syn{arch}.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 4096, 2048, 2, 0, fmt.encode(), 7)
    m = RWKVModel(L, p)
    toks = [5, 77, 1023, 4000, 9, 2048]
    lg, st = m.eval_sequence(toks, None, use_numpy=True)
    glg, gst = gpu_variant(p, toks, sequence=True)
    assert_bits_equal(lg, glg, 'logits')
    assert_bits_equal(st, gst, 'state')
    olg, ost, noise, _ = noise_band(p, toks, sequence=True)
    assert np.abs(lg - olg).max() <= max(1e-3, 1.5 * noise), (np.abs(lg - olg).max(), noise)
    lg2, st2 = gpu_serial(m, toks)
    assert np.array_equal(st, st2) and np.array_equal(lg, lg2)
    m.free()


@pytest.mark.parametrize('arch,fmt', [(6, 'Q4_0'), (5, 'Q4_1'), (7, 'Q5_1'), (6, 'Q8_0'), (6, 'Q5_1'), (6, 'Q5_0')])
def test_real_width_long_sequence_bit_exact(tmp_path, arch, fmt):
    """70 tokens through the sequence kernels (MFMA GEMM, chunk-staged wkv: 32+32+6) equal 70
    serial decode steps bit for bit, and chunked evaluation equals both."""
    L = library()
    p = str(tmp_path / f'long{arch}{fmt}.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, 2048, 2, 0, fmt.encode(), 11)
    m = RWKVModel(L, p)
    toks = [int(t) for t in np.random.default_rng(3).integers(0, 1024, 70)]
    lg, st = m.eval_sequence(toks, None, use_numpy=True)
    lg2, st2 = gpu_serial(m, toks)
    assert np.array_equal(st, st2) and np.array_equal(lg, lg2)
    lg3, st3 = m.eval_sequence_in_chunks(toks, None, chunk_size=16, use_numpy=True)
    assert np.array_equal(st, st3) and np.array_equal(lg, lg3)
    m.free()


def test_kernel_timing_mode_is_transparent():
    """Kernel timing (bench.py's roofline source) runs the same graph path: results bit-identical to
    the untimed path, and every decode matvec launch reports a duration."""
    import ctypes
    L = library()
    lib = L.library
    path = os.path.join(GOLD, 'tiny-rwkv-6v0-3m-Q5_0.bin')
    m = RWKVModel(L, path)
    P = ctypes.POINTER(ctypes.c_float)
    PI = ctypes.POINTER(ctypes.c_int32)
    outs = []
    for timing in (False, True):
        lib.rwkv_mi355x_set_kernel_timing(m._ctx.ptr, timing)
        assert lib.rwkv_mi355x_state_upload(m._ctx.ptr, None)
        lg = np.zeros(m._logits_buffer_element_count, np.float32)
        for i, t in enumerate(LONG[:12]):
            arr = (ctypes.c_int32 * 1)(t)
            assert lib.rwkv_mi355x_eval_device(m._ctx.ptr, ctypes.cast(arr, PI), 1, True, lg.ctypes.data_as(P), True)
        st = np.zeros(m._state_buffer_element_count, np.float32)
        assert lib.rwkv_mi355x_state_download(m._ctx.ptr, st.ctypes.data_as(P))
        outs.append((lg.copy(), st))
    n = lib.rwkv_mi355x_kernel_stats(m._ctx.ptr, -1, None, 0, None, None, None, None)
    found = False
    for i in range(n):
        name = ctypes.create_string_buffer(128)
        la, ms, by, fl = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        lib.rwkv_mi355x_kernel_stats(m._ctx.ptr, i, name, 128, ctypes.byref(la), ctypes.byref(ms), ctypes.byref(by),
                                     ctypes.byref(fl))
        if name.value == b'k_mv':
            found = True
            assert la.value > 0 and ms.value > 0 and by.value > 0
    assert found
    lib.rwkv_mi355x_set_kernel_timing(m._ctx.ptr, False)
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    m.free()


@pytest.mark.parametrize('fmt', ['Q4_0', 'Q5_1', 'FP16'])
def test_v6_fused_maa_decode_equals_split(tmp_path, fmt):
    """The one-launch v6 maa LoRA (mv_maa.hip) reproduces the W1 matvec + mix launch pair bit for bit."""
    L = library()
    p = str(tmp_path / f'maa{fmt}.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), 6, 1024, 2048, 2, 0, fmt.encode(), 13)
    toks = [int(t) for t in np.random.default_rng(5).integers(0, 1024, 12)]
    outs = []
    for split in ('1', '0'):
        os.environ['RWKV_MI355X_SPLIT_MAA'] = split
        try:
            m = RWKVModel(L, p)
        finally:
            os.environ.pop('RWKV_MI355X_SPLIT_MAA', None)
        outs.append(gpu_serial(m, toks))
        m.free()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_v6_1b6_width_token1_vs_ggml_order(tmp_path):
    """At the headline width (v6-1B6: C 2048, H 32, FFN 7168, Q4_0; 2 layers, 4096-token vocabulary),
    the FIRST token -- before any Q8 re-quantization flip can be amplified by the recurrence -- must
    sit within 1e-4 of the ggml-order oracle (variant 0): max|dlogit| <= 1e-4 and max|dstate| <= 1e-4
    relative to max|state|.  This is where a systematic error of the GPU association would show;
    later tokens are bounded by the oracle's noise band (bench.py's parity reports the growth).
    Measured on the oracle's GPU-association variant (which the GPU equals bit for bit): 1.7e-5 and
    3.6e-7 relative."""
    L = library()
    p = str(tmp_path / 'v6-1b6-width.bin')
    assert L.library.rwkv_mi355x_write_synthetic_model(p.encode(), 6, 4096, 2048, 2, 0, b'Q4_0', 21)
    tok = [int(np.random.default_rng(31).integers(0, 4096))]
    m = RWKVModel(L, p)
    lg, st = gpu_serial(m, tok)
    m.free()
    glg, gst = gpu_variant(p, tok)
    assert_bits_equal(lg, glg, 'token-1 logits vs GPU-association oracle')
    assert_bits_equal(st, gst, 'token-1 state vs GPU-association oracle')
    o = OracleModel(p)
    olg, ost = o.eval_serial(tok)
    o.close()
    assert np.abs(lg - olg).max() <= 1e-4, np.abs(lg - olg).max()
    assert np.abs(st - ost).max() <= 1e-4 * np.abs(ost).max(), (np.abs(st - ost).max(), np.abs(ost).max())
