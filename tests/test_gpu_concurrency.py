"""Clone contexts decoding at the same time on ONE GPU (the reference's parallel pattern: contexts from
rwkv_clone_context evaluated from several host threads, rwkv.h:93-99, rwkv.cpp:123-139).

The fused decode launches hand values between workgroups inside one launch (k_v6_att_fused: the
r/k/v/g and decay-LoRA rows to the per-head reducers, the head outputs to the Wo workgroups;
k_v4_att_fused: every channel's output to the Wo workgroups).  Several contexts decoding at once put
several such launches on the GPU together, so no launch can count on all of its workgroups being
resident.  Each waiting workgroup therefore waits only on workgroups with a LOWER index (mv_att6f.hip,
mv_att4f.hip), which are dispatched before it.  These tests run 2, 4 and 8 clones from their own
threads -- through rwkv_eval (host state) and through rwkv_mi355x_eval_device (each clone's own
stream) -- at the BASELINE widths where the fused launches are on (v6 C = 2048, v4 C = 768): every
call must succeed and every context must equal its own serial run bit for bit.

The v6 attention launch has two layouts with the same bits: the ordered one above, and a
co-resident one (mv_att6c.hip) that needs all its workgroups resident and that a context uses only
while it is the process's only context with decode work queued on the device.  The serial
reference runs here use the co-resident layout (one context), the concurrent clones mostly the
ordered one: bit-equality covers both.

test_decode_after_sequence_* (ADVICE round 5): the Wo hand-off tags carry (layer, state parity); a
sequence evaluation flips the parity without writing them, so a later decode must never accept a
value left by the decode before the sequence.  One-layer models make that the only layer: decode,
sequence, decode must equal the serial decode of the same tokens bit for bit.
"""
import ctypes
import os
import threading

import numpy as np
import pytest
import torch  # noqa: F401  (torch's HIP runtime first)

from rwkv_lib import library

pytestmark = pytest.mark.gpu

FP = ctypes.POINTER(ctypes.c_float)
VOCAB = 1024
WIDTHS = {6: (2048, 'Q4_0'), 4: (768, 'Q8_0')}


def _model(tmp_path, arch, n_layer):
    C, fmt = WIDTHS[arch]
    p = str(tmp_path / f'conc-v{arch}-L{n_layer}.bin')
    if not os.path.isfile(p):
        assert library().library.rwkv_mi355x_write_synthetic_model(p.encode(), arch, VOCAB, C, n_layer, 0,
                                                                   fmt.encode(), 41)
    return p


def _bits(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def _serial(lib, ctx, toks):
    n, v = lib.rwkv_get_state_len(ctx), lib.rwkv_get_n_vocab(ctx)
    st, lg = np.zeros(n, np.float32), np.zeros(v, np.float32)
    for i, t in enumerate(toks):
        assert lib.rwkv_eval(ctx, t, None if i == 0 else st.ctypes.data_as(FP), st.ctypes.data_as(FP),
                             lg.ctypes.data_as(FP))
    return lg, st


def _device_serial(lib, ctx, toks):
    n, v = lib.rwkv_get_state_len(ctx), lib.rwkv_get_n_vocab(ctx)
    lg, st = np.zeros(v, np.float32), np.zeros(n, np.float32)
    assert lib.rwkv_mi355x_state_upload(ctx, None)
    for t in toks:
        arr = (ctypes.c_int32 * 1)(t)
        assert lib.rwkv_mi355x_eval_device(ctx, arr, 1, True, lg.ctypes.data_as(FP), True)
    assert lib.rwkv_mi355x_state_download(ctx, st.ctypes.data_as(FP))
    return lg, st


@pytest.mark.parametrize('path_kind', ['abi', 'device'])
@pytest.mark.parametrize('n', [2, 4, 8])
@pytest.mark.parametrize('arch', [6, 4])
def test_concurrent_clone_decode_bit_exact(tmp_path, arch, n, path_kind):
    L = library()
    lib = L.library
    p = _model(tmp_path, arch, 3)
    ctx = lib.rwkv_init_from_file(p.encode(), 1, 99)
    assert ctx
    rng = np.random.default_rng(100 + n)
    streams = [[int(t) for t in rng.integers(0, VOCAB, 24)] for _ in range(n)]
    run = _serial if path_kind == 'abi' else _device_serial
    refs = [run(lib, ctx, s) for s in streams]
    clones = [lib.rwkv_clone_context(ctx, 1) for _ in range(n)]
    assert all(clones)
    out = [None] * n
    errs = [None] * n
    go = threading.Barrier(n)

    def worker(i):
        try:
            go.wait()
            out[i] = run(lib, clones[i], streams[i])
        except BaseException as e:  # noqa: BLE001 -- reported by the main thread
            errs[i] = e

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), 'a decoding thread did not finish'
    for i in range(n):
        assert errs[i] is None, f'context {i}: {errs[i]!r} (error flags {lib.rwkv_get_last_error(clones[i])})'
        assert _bits(out[i][0], refs[i][0]), f'context {i}: logits differ from its serial run'
        assert _bits(out[i][1], refs[i][1]), f'context {i}: state differs from its serial run'
    for c in clones:
        lib.rwkv_free(c)
    lib.rwkv_free(ctx)


@pytest.mark.parametrize('n_layer', [1, 2])
@pytest.mark.parametrize('arch', [6, 4])
def test_decode_after_sequence_bit_exact(tmp_path, arch, n_layer):
    L = library()
    lib = L.library
    p = _model(tmp_path, arch, n_layer)
    toks = [int(t) for t in np.random.default_rng(7).integers(0, VOCAB, 11)]
    a, b = toks[:3], toks[3:7]
    c = toks[7:]
    ctx = lib.rwkv_init_from_file(p.encode(), 1, 99)
    ref_lg, ref_st = _serial(lib, ctx, toks)
    n, v = lib.rwkv_get_state_len(ctx), lib.rwkv_get_n_vocab(ctx)
    # host-state ABI: decode, sequence, decode (odd sequence lengths too: the parity lands either way)
    for seq_len in (len(b), len(b) - 1):
        bb = b[:seq_len]
        cc = b[seq_len:] + c
        st, lg = np.zeros(n, np.float32), np.zeros(v, np.float32)
        for i, t in enumerate(a):
            assert lib.rwkv_eval(ctx, t, None if i == 0 else st.ctypes.data_as(FP), st.ctypes.data_as(FP),
                                 lg.ctypes.data_as(FP))
        arr = (ctypes.c_int32 * len(bb))(*bb)
        assert lib.rwkv_eval_sequence(ctx, arr, len(bb), st.ctypes.data_as(FP), st.ctypes.data_as(FP),
                                      lg.ctypes.data_as(FP))
        for t in cc:
            assert lib.rwkv_eval(ctx, t, st.ctypes.data_as(FP), st.ctypes.data_as(FP), lg.ctypes.data_as(FP))
        assert _bits(lg, ref_lg), f'abi decode after a {seq_len}-token sequence: logits'
        assert _bits(st, ref_st), f'abi decode after a {seq_len}-token sequence: state'
    # device-resident: the same
    for seq_len in (len(b), len(b) - 1):
        bb = b[:seq_len]
        cc = b[seq_len:] + c
        lg = np.zeros(v, np.float32)
        assert lib.rwkv_mi355x_state_upload(ctx, None)
        for t in a:
            assert lib.rwkv_mi355x_eval_device(ctx, (ctypes.c_int32 * 1)(t), 1, False, None, False)
        assert lib.rwkv_mi355x_eval_device(ctx, (ctypes.c_int32 * len(bb))(*bb), len(bb), False, None, False)
        for t in cc:
            assert lib.rwkv_mi355x_eval_device(ctx, (ctypes.c_int32 * 1)(t), 1, True, lg.ctypes.data_as(FP), False)
        st = np.zeros(n, np.float32)
        assert lib.rwkv_mi355x_state_download(ctx, st.ctypes.data_as(FP))
        assert _bits(lg, ref_lg), f'device decode after a {seq_len}-token sequence: logits'
        assert _bits(st, ref_st), f'device decode after a {seq_len}-token sequence: state'
    lib.rwkv_free(ctx)


@pytest.mark.parametrize('knobs', [{'wo_rows': 4}, {'wo_prepoll': 0}, {'graphs': 0}, {'wo_rows': 4, 'wo_prepoll': 0},
                                   {'co_mode': 0}, {'co_mode': 1}, {'co_mode': 0, 'wo_rows': 4},
                                   {'decode_fusion': 127}, {'decode_fusion': 127, 'ffn_wdelay': 0},
                                   {'decode_fusion': 127, 'ffn_prepoll': 0}])
def test_decode_knob_arms_bit_exact(tmp_path, knobs):
    """The non-default arms of the per-context decode knobs (Switches): the fused-Wo
    workgroup shape (4 rows per wave), the gather without the per-head pre-poll, eager decode
    launches without graphs, and the v6 attention layout forced (co_mode 0: the ordered layout of
    mv_att6f.hip; 1: the co-resident one of mv_att6c.hip; default: co-resident while the context is
    alone on the device), and the one-launch channel mix (decode_fusion 127, off by default) with its
    consumer weight delay off and without its pre-poll -- each decodes the v6-1B6-width model
    bit-exactly like the defaults,
    through both the host-state ABI and the device-resident path."""
    lib = library().library
    p = _model(tmp_path, 6, 2)
    toks = [int(t) for t in np.random.default_rng(8).integers(0, VOCAB, 9)]
    ctx = lib.rwkv_init_from_file(p.encode(), 1, 99)
    ref = _serial(lib, ctx, toks)
    dref = _device_serial(lib, ctx, toks)
    assert _bits(ref[0], dref[0]) and _bits(ref[1], dref[1])
    for k, v in knobs.items():
        assert lib.rwkv_mi355x_debug_set(ctx, k.encode(), v), k
    for run in (_serial, _device_serial):
        lg, st = run(lib, ctx, toks)
        assert _bits(lg, ref[0]), f'{knobs} {run.__name__}: logits'
        assert _bits(st, ref[1]), f'{knobs} {run.__name__}: state'
    lib.rwkv_free(ctx)
