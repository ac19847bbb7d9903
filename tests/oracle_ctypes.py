"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product library never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, 'oracle')
ORACLE_SO = os.path.join(ORACLE_DIR, 'build', 'liboracle.so')

_lib = None


def build_oracle():
    subprocess.check_call(['make', '-s', '-C', ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(ORACLE_SO):
            build_oracle()
        L = ctypes.CDLL(ORACLE_SO)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.oracle_load.restype = vp
        L.oracle_load.argtypes = [ctypes.c_char_p]
        L.oracle_free.argtypes = [vp]
        L.oracle_info.argtypes = [vp, vp]
        L.oracle_init_state.argtypes = [vp, vp]
        L.oracle_eval.argtypes = [vp, vp, sz, vp, vp, vp]
        L.oracle_eval.restype = ctypes.c_int
        L.oracle_eval_layers.argtypes = [vp, vp, sz, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, vp]
        L.oracle_eval_layers.restype = ctypes.c_int
        L.oracle_quantize_file.argtypes = [ctypes.c_char_p] * 3
        L.oracle_quantize_file.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_get_threads.restype = ctypes.c_int
        L.oracle_block_bytes.argtypes = [ctypes.c_int]
        L.oracle_block_bytes.restype = sz
        L.oracle_quantize_row.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int64]
        L.oracle_quantize_act.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int64]
        L.oracle_dequantize_row.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int64]
        L.oracle_matmul.argtypes = [ctypes.c_int, vp, ctypes.c_int64, ctypes.c_int64, vp, ctypes.c_int64, vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class OracleModel:
    """Mirror of the rwkv.h eval semantics on the CPU restatement."""

    def __init__(self, path):
        self.ptr = lib().oracle_load(path.encode())
        if not self.ptr:
            raise ValueError(f'oracle failed to load {path}')
        info = np.zeros(8, np.int64)
        lib().oracle_info(self.ptr, _p(info))
        (self.n_vocab, self.n_embed, self.n_layer, self.arch_major, self.arch_minor,
         self.head_count, self.head_size, self.state_len) = [int(v) for v in info]

    def init_state(self):
        s = np.zeros(self.state_len, np.float32)
        lib().oracle_init_state(self.ptr, _p(s))
        return s

    def eval_sequence(self, tokens, state_in=None, want_logits=True):
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint32))
        st = np.zeros(self.state_len, np.float32)
        lg = np.zeros(self.n_vocab, np.float32) if want_logits else None
        rc = lib().oracle_eval(self.ptr, _p(toks), len(toks), _p(state_in), _p(st), _p(lg))
        if rc:
            raise ValueError(f'oracle_eval failed rc={rc}')
        return lg, st

    def eval_layers(self, tokens, l0, l1, x=None, vfirst=None, state_in=None, want_logits=False):
        """Layers [l0, l1) over len(tokens) tokens (a pipeline stage).  x / vfirst: [T, C] float32
        arrays updated in place (required when l0 > 0; vfirst for v7 only).  Returns
        (logits or None, full state with only this range's slices updated)."""
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint32))
        st = np.zeros(self.state_len, np.float32)
        lg = np.zeros(self.n_vocab, np.float32) if want_logits and l1 == self.n_layer else None
        rc = lib().oracle_eval_layers(self.ptr, _p(toks), len(toks), l0, l1, _p(x), _p(vfirst), _p(state_in),
                                      _p(st), _p(lg))
        if rc:
            raise ValueError(f'oracle_eval_layers failed rc={rc}')
        return lg, st

    def eval_serial(self, tokens, state_in=None):
        st = state_in
        lg = None
        for t in tokens:
            lg, st = self.eval_sequence([t], st)
        return lg, st

    def close(self):
        if self.ptr:
            lib().oracle_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def quantize_file(src, dst, fmt):
    rc = lib().oracle_quantize_file(src.encode(), dst.encode(), fmt.encode())
    if rc:
        raise ValueError(f'oracle_quantize_file rc={rc}')


TYPE_IDS = {'FP32': 0, 'FP16': 1, 'Q4_0': 2, 'Q4_1': 3, 'Q5_0': 7, 'Q5_1': 8, 'Q8_0': 9, 'Q8_1': 10}


def quantize_rows(fmt, x):
    """File quantizer on a [M, K] float32 matrix -> raw block bytes (FP32 / FP16: the raw rows, as the
    converter writes them)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    if fmt == 'FP32':
        return x.reshape(-1).view(np.uint8).copy()
    if fmt == 'FP16':
        return x.astype(np.float16).reshape(-1).view(np.uint8).copy()
    t = TYPE_IDS[fmt]
    M, K = x.shape
    bb = lib().oracle_block_bytes(t)
    out = np.zeros(M * (K // 32) * bb, np.uint8)
    for m in range(M):
        lib().oracle_quantize_row(t, _p(x[m]), out.ctypes.data + m * (K // 32) * bb, K)
    return out


def matmul(fmt, w_bytes, K, M, x):
    """ggml-numerics matmul: x [T, K] float32 -> y [T, M]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    T = x.shape[0]
    y = np.zeros((T, M), np.float32)
    w_bytes = np.ascontiguousarray(w_bytes)
    lib().oracle_matmul(TYPE_IDS[fmt], _p(w_bytes), K, M, _p(x), T, _p(y))
    return y


def set_variant(v):
    L = lib()
    L.oracle_set_variant.argtypes = [ctypes.c_int]
    L.oracle_set_variant(v)


# Variant bit 8: the GPU kernels' association (oracle.c "GPU-association variant") -- the variant the
# MI355X path must reproduce bit for bit.
VARIANT_GPU = 8


def gpu_variant(path, tokens, sequence=False, state_in=None):
    """(logits, state) of the oracle's GPU-association variant: serial single-token evals, or one
    eval_sequence call when sequence=True."""
    set_variant(VARIANT_GPU)
    try:
        m = OracleModel(path)
        out = m.eval_sequence(tokens, state_in) if sequence else m.eval_serial(tokens, state_in)
        m.close()
    finally:
        set_variant(0)
    return out


def assert_bits_equal(a, b, what=''):
    """Bit-for-bit equality of two float32 arrays (a -0.0 / +0.0 difference counts)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    ne = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
    if ne.size:
        i = int(ne[0])
        raise AssertionError(f'{what}: {ne.size} of {a.size} values differ; first at {i}: {a[i]!r} vs {b[i]!r}, '
                             f'max|d| {float(np.nanmax(np.abs(a - b))):.3g}')


def noise_band(path, tokens, sequence=False):
    """Oracle logits/state (variant 0) plus the largest deviation any re-associated variant
    (1..7: reversed order / scalar ggml dot / fp32 accumulators) produces: how strongly this
    model amplifies last-bit differences.  Returns (logits, state, noise_logits, variants)."""
    outs = []
    try:
        for v in range(8):
            set_variant(v)
            m = OracleModel(path)
            outs.append(m.eval_sequence(tokens) if sequence else m.eval_serial(tokens))
            m.close()
    finally:
        set_variant(0)
    lg0, st0 = outs[0]
    noise = max(float(np.abs(o[0] - lg0).max()) for o in outs[1:])
    return lg0, st0, noise, [o[0] for o in outs]


def dequantize(fmt, w_bytes, K, M):
    L = lib()
    t = TYPE_IDS[fmt]
    out = np.zeros((M, K), np.float32)
    bpr = (K // 32) * L.oracle_block_bytes(t) if t not in (0, 1) else K * (4 if t == 0 else 2)
    w_bytes = np.ascontiguousarray(w_bytes)
    for m in range(M):
        L.oracle_dequantize_row(t, w_bytes.ctypes.data + m * bpr, out[m].ctypes.data, K)
    return out


def quantize_act(fmt, x):
    """ggml activation quantizer (Q8_0 / Q8_1) on one row: returns (q int8 [K], d [K/32], s [K/32])."""
    L = lib()
    t = TYPE_IDS[fmt]
    K = x.shape[0]
    bb = 36 if fmt == 'Q8_1' else 34
    buf = np.zeros((K // 32) * bb, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    L.oracle_quantize_act(t, x.ctypes.data, buf.ctypes.data, K)
    blk = buf.reshape(-1, bb)
    d = blk[:, 0:2].copy().view(np.float16).astype(np.float32).ravel()
    off = 4 if fmt == 'Q8_1' else 2
    s = blk[:, 2:4].copy().view(np.float16).astype(np.float32).ravel() if fmt == 'Q8_1' else None
    q = blk[:, off:off + 32].copy().view(np.int8).ravel()
    return q, d, s
