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
import torch  # before librwkv initialises HIP (torch's own HIP runtime must come up first)

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


def test_v5_7b_width_4096_tokens_in_chunks(cfg_dir):
    """BASELINE config 5's workload: 4096 tokens through rwkv_eval_sequence_in_chunks with chunk 1024
    (reference rwkv_eval.inc:158-221) at the v5-7B width (C 4096, FFN 14336, 64 heads), one layer so
    the CPU oracle finishes in seconds.  Bit-exact against the oracle's GPU-association variant over
    the whole sequence, and equal to one rwkv_eval_sequence call (which splits at 1024 itself)."""
    path = cfg_model(cfg_dir, 'v5-7b-q4_1', layers=1)
    toks = [int(t) for t in np.random.default_rng(10).integers(0, VOCAB, 4096)]
    m = RWKVModel(library(), path)
    lg, st = m.eval_sequence_in_chunks(toks, None, chunk_size=1024, use_numpy=True)
    lg1, st1 = m.eval_sequence(toks, None, use_numpy=True)
    m.free()
    assert_bits_equal(lg1, lg, 'one call vs chunks of 1024: logits')
    assert_bits_equal(st1, st, 'one call vs chunks of 1024: state')
    glg, gst = gpu_variant(path, toks, sequence=True)
    assert_bits_equal(lg, glg, 'T=4096 chunked logits')
    assert_bits_equal(st, gst, 'T=4096 chunked state')


def test_v7_2b9_width_four_stages(cfg_dir):
    """BASELINE config 4's partition: four pipeline stages (one layer each) at the v7-2.9B width
    (C 2560, H 40, Q5_1), composed over T-chunks through rwkv_mi355x_eval_layers on stage contexts
    that hold only their own layers (rwkv_mi355x_init_from_file_layers), carrying x and v_first
    between stages.  Equals one rwkv_eval_sequence of the whole model and the oracle, bit for bit."""
    import ctypes
    import torch
    path = cfg_model(cfg_dir, 'v7-2b9-q5_1', layers=4)
    toks = [int(t) for t in np.random.default_rng(11).integers(0, VOCAB, 70)]
    L = library()
    lib = L.library
    m = RWKVModel(L, path)
    ref_lg, ref_st = m.eval_sequence(toks, None, use_numpy=True)
    m.free()
    glg, gst = gpu_variant(path, toks, sequence=True)
    assert_bits_equal(ref_lg, glg, 'whole-model logits vs oracle')
    assert_bits_equal(ref_st, gst, 'whole-model state vs oracle')
    fp = ctypes.POINTER(ctypes.c_float)
    stages = []
    for s in range(4):
        ptr = lib.rwkv_mi355x_init_from_file_layers(path.encode(), 1, s, s + 1)
        assert ptr, s
        assert lib.rwkv_mi355x_state_upload(ptr, None)
        stages.append(ptr)
    C, n_vocab = lib.rwkv_get_n_embed(stages[0]), lib.rwkv_get_n_vocab(stages[0])
    lg = np.zeros(n_vocab, np.float32)
    for a in range(0, len(toks), 24):
        ch = np.ascontiguousarray(np.asarray(toks[a:a + 24], np.uint32))
        x = torch.zeros((2, len(ch), C), dtype=torch.float32, device='cuda')
        for s, ptr in enumerate(stages):
            last = s == 3
            assert lib.rwkv_mi355x_eval_layers(ptr, ch.ctypes.data, len(ch), s, s + 1, x[0].data_ptr(),
                                               x[1].data_ptr(), last, lg.ctypes.data_as(fp) if last else None)
    n = lib.rwkv_get_state_buffer_element_count(stages[0])
    per = n // 4
    for s, ptr in enumerate(stages):
        st = np.zeros(n, np.float32)
        assert lib.rwkv_mi355x_state_download(ptr, st.ctypes.data_as(fp))
        assert_bits_equal(st[s * per:(s + 1) * per], ref_st[s * per:(s + 1) * per], f'stage {s} state slice')
        lib.rwkv_free(ptr)
    assert_bits_equal(lg, ref_lg, 'four-stage logits')


FUSION_MASKS = [0, 1023 ^ 2, 1023 ^ 8, 1023 ^ 16, 1023 ^ 32, 1023 ^ 1, 1023 ^ 64, 1023 ^ 96, 1023 ^ 128, 1023 ^ 256,
                1023 ^ 512, 1023 ^ 192, 511, 255, 63]


@pytest.mark.parametrize('name', sorted(CONFIGS))
def test_decode_fusion_arms_bit_exact(cfg_dir, name):
    """Every decode fusion has an unfused arm (Engine::FUSE_*: 1 v6 attention launch, 2 its Wo, 4 v4
    attention launch, 8 its Wo, 16 v7 LoRA + attention, 32 FFN value + receptance, 64 the whole channel
    mix in one launch, 128 its co-resident form while the context has the device alone, 256 the v6
    channel mix's value rows with the next layer's maa, co-resident, 512 the v6 embedding LayerNorm
    inside layer 0's maa launch).  Each mask,
    switched per context (rwkv_mi355x_debug_set "decode_fusion") and at creation
    (RWKV_MI355X_DECODE_FUSION), decodes bit-exactly against the oracle; switching back and forth on
    one context (the fused Wo's granules cleared at each switch) too."""
    path = cfg_model(cfg_dir, name)
    toks = [int(t) for t in np.random.default_rng(7).integers(0, VOCAB, 6)]
    glg, gst = gpu_variant(path, toks)
    L = library()
    m = RWKVModel(L, path)
    for mask in FUSION_MASKS + [1023]:
        assert L.library.rwkv_mi355x_debug_set(m._ctx.ptr, b'decode_fusion', mask)
        lg, st = gpu_serial(m, toks)
        assert_bits_equal(lg, glg, f'{name} decode logits, fusion mask {mask}')
        assert_bits_equal(st, gst, f'{name} decode state, fusion mask {mask}')
    m.free()
    os.environ['RWKV_MI355X_DECODE_FUSION'] = '0'
    try:
        m = RWKVModel(L, path)
    finally:
        os.environ.pop('RWKV_MI355X_DECODE_FUSION', None)
    lg, st = gpu_serial(m, toks)
    assert_bits_equal(lg, glg, f'{name} decode logits, RWKV_MI355X_DECODE_FUSION=0')
    assert_bits_equal(st, gst, f'{name} decode state, RWKV_MI355X_DECODE_FUSION=0')
    m.free()


@pytest.mark.parametrize('arch,fmt', [(4, 'Q8_0'), (6, 'Q4_0')])
def test_width_above_4096_generic_path(cfg_dir, arch, fmt):
    """n_embed 4608 (> the 4096 that the register LayerNorm prologues hold; RWKV-4 14B is 5120): the
    engine routes decode through the sequence kernels and the embedding LayerNorm through its wide
    form.  Serial decode, sequence evaluation and the oracle agree bit for bit."""
    p = os.path.join(str(cfg_dir), f'wide-v{arch}.bin')
    if not os.path.isfile(p):
        assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, 4608, 1, 0, fmt.encode(), 23)
    toks = [int(t) for t in np.random.default_rng(14).integers(0, 1024, 5)]
    m = RWKVModel(library(), p)
    lg, st = gpu_serial(m, toks)
    slg, sst = m.eval_sequence(toks, None, use_numpy=True)
    m.free()
    assert_bits_equal(lg, slg, 'wide decode vs sequence logits')
    assert_bits_equal(st, sst, 'wide decode vs sequence state')
    glg, gst = gpu_variant(p, toks)
    assert_bits_equal(lg, glg, 'wide decode logits vs oracle')
    assert_bits_equal(st, gst, 'wide decode state vs oracle')


@pytest.mark.parametrize('arch,C,fmt', [(4, 4096, 'Q8_0'), (6, 2560, 'Q4_0'), (6, 4096, 'Q4_0')])
def test_wide_fused_decode_bit_exact(cfg_dir, arch, C, fmt):
    """The fused decode launches at the widest shapes they take (v4-7B's C = 4096; v6 at
    40 and 64 heads, where the co-resident attention layout does not fit at one workgroup per CU and
    the ordered layout runs): serial decode, sequence evaluation and the oracle agree bit for bit, with
    the default rule and with each attention layout forced."""
    p = os.path.join(str(cfg_dir), f'wide-fused-v{arch}-{C}.bin')
    if not os.path.isfile(p):
        assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, C, 1, 0, fmt.encode(), 29)
    toks = [int(t) for t in np.random.default_rng(C).integers(0, 1024, 5)]
    glg, gst = gpu_variant(p, toks)
    L = library()
    m = RWKVModel(L, p)
    slg, sst = m.eval_sequence(toks, None, use_numpy=True)
    assert_bits_equal(slg, glg, f'v{arch} C={C} sequence logits vs oracle')
    for co in (-1, 0, 1):
        assert L.library.rwkv_mi355x_debug_set(m._ctx.ptr, b'co_mode', co)
        lg, st = gpu_serial(m, toks)
        assert_bits_equal(lg, glg, f'v{arch} C={C} co_mode {co} decode logits vs oracle')
        assert_bits_equal(st, gst, f'v{arch} C={C} co_mode {co} decode state vs oracle')
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


def test_v6_decode_handoff_many_tokens(cfg_dir):
    """The fused v6 decode launch (mv_att6f.hip: r, k, v, g and decay-LoRA rows + per-head attention,
    an in-launch granule hand-off per head) at the v6-1B6 width over many tokens: serial decode equals
    one sequence evaluation bit for bit (the sequence path has no hand-off), every rwkv_eval
    succeeded (no hand-off timed out) and afterwards every granule is cleared."""
    import ctypes
    path = cfg_model(cfg_dir, 'v6-1b6-q4_0')
    toks = [int(t) for t in np.random.default_rng(12).integers(0, VOCAB, 48)]
    m = RWKVModel(library(), path)
    lg, st = gpu_serial(m, toks)
    slg, sst = m.eval_sequence(toks, None, use_numpy=True)
    assert_bits_equal(lg, slg, 'decode vs sequence logits')
    assert_bits_equal(st, sst, 'decode vs sequence state')
    C = 2048
    gran = np.ones(6 * C, np.uint64)  # r, k, v, g rows + one decay-LoRA copy per head
    n = library().library.rwkv_mi355x_debug_buffer(m._ctx.ptr, b'granules', gran.ctypes.data_as(ctypes.c_void_p),
                                                   gran.nbytes)
    assert n == gran.nbytes
    assert not gran.any(), f'hand-off granules not cleared: {np.nonzero(gran)[0][:8]}'
    m.free()


@pytest.mark.parametrize('co_mode', [-1, 0, 1])
@pytest.mark.parametrize('skip_wg', [9, 8 * 31 + 7])
def test_v6_decode_handoff_timeout_fails_the_call(cfg_dir, skip_wg, co_mode):
    """A hand-off that times out must fail the evaluation, never return garbage with success
    (reference error convention: false + RWKV_ERROR_CTX, rwkv_error_handling.inc:1-54).  The test hook
    makes one producer workgroup of k_v6_att_fused publish nothing (9: head 9's first 32 rows and
    decay-LoRA row 9; 255: head 31's last 32 rows) with a short sweep bound.  rwkv_eval (host
    state, the chunked graphs) and rwkv_mi355x_eval_device + rwkv_mi355x_sync both fail with
    RWKV_ERROR_CTX; with the hook off the same context then decodes bit-exactly again (the granules
    were cleared and the flag re-armed).  co_mode: the attention layout rule (-1: co-resident while
    alone, the call re-run in the ordered layout after a co-resident timeout -- which times out
    again here; 0: ordered; 1: co-resident)."""
    import ctypes
    L = library().library
    path = cfg_model(cfg_dir, 'v6-1b6-q4_0')
    toks = [int(t) for t in np.random.default_rng(13).integers(0, VOCAB, 4)]
    ctx = L.rwkv_init_from_file(path.encode(), 1, 99)
    assert ctx
    L.rwkv_set_print_errors(ctx, False)
    n_state, n_vocab = L.rwkv_get_state_len(ctx), L.rwkv_get_n_vocab(ctx)
    fp = ctypes.POINTER(ctypes.c_float)
    ref_lg, ref_st = gpu_variant(path, toks)
    E_CTX = 6 << 8  # RWKV_ERROR_CTX (reference rwkv.h:50; flags = category | code)
    assert L.rwkv_mi355x_debug_set(ctx, b'co_mode', co_mode)
    assert L.rwkv_mi355x_debug_set(ctx, b'spin_max', 2048)
    assert L.rwkv_mi355x_debug_set(ctx, b'skip_granule', skip_wg)
    st = np.zeros(n_state, np.float32)
    lg = np.zeros(n_vocab, np.float32)
    L.rwkv_init_state(ctx, st.ctypes.data_as(fp))
    assert not L.rwkv_eval(ctx, toks[0], st.ctypes.data_as(fp), st.ctypes.data_as(fp), lg.ctypes.data_as(fp))
    assert (L.rwkv_get_last_error(ctx) & 0xff00) == E_CTX
    # the device-resident path: enqueue without waiting, the synchronising call reports it
    arr = (ctypes.c_int32 * 1)(toks[0])
    assert L.rwkv_mi355x_state_upload(ctx, None)
    assert L.rwkv_mi355x_eval_device(ctx, arr, 1, True, None, False)
    assert not L.rwkv_mi355x_sync(ctx)
    assert (L.rwkv_get_last_error(ctx) & 0xff00) == E_CTX
    # hook off: the context decodes correctly again
    assert L.rwkv_mi355x_debug_set(ctx, b'skip_granule', -1)
    assert L.rwkv_mi355x_debug_set(ctx, b'spin_max', 0)
    L.rwkv_init_state(ctx, st.ctypes.data_as(fp))
    for t in toks:
        assert L.rwkv_eval(ctx, t, st.ctypes.data_as(fp), st.ctypes.data_as(fp), lg.ctypes.data_as(fp))
    assert_bits_equal(lg, ref_lg, 'logits after a timed-out hand-off')
    assert_bits_equal(st, ref_st, 'state after a timed-out hand-off')
    L.rwkv_free(ctx)
