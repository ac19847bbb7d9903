"""Chunk-parallel WKV-6 (csrc/wkv_chunk.hip; RWKV_MI355X_WKV_CHUNK=1 or
rwkv_mi355x_debug_set(ctx, "wkv_chunk", 1)) -- the long-sequence form of the v5/v6 time-mixing
recurrence (reference: ggml_rwkv_wkv6 via rwkv_graph.inc:363-371).

It re-associates the recurrence's sums (chunk-local decay products as 2^(la_t - la_s), intra-chunk
matrix, carried state), so it is NOT bit-exact with the serial kernel (k_wkv6_s64, decode's
association) and stays off by default.  The bar it is held to instead:

* kernel level, against a float64 restatement of the recurrence (y_t = r_t (S + u k_t v_t^T),
  S <- w_t S + k_t v_t^T): max |y - y64| <= 5e-6 * max |y64| and the same for the final state, over
  T = 2 .. 4096 (ragged chunk tails) with decays from 1 down to exact 0; for comparison the serial
  kernel's own fp32 error is printed beside it;
* model level, v5 and v6 sequence evaluation with the switch on: logits within the oracle's noise
  band, max(1e-3, 1.5 x the spread of the oracle's re-associated variants) -- the rule
  test_oracle_variants.py applies to the GPU-association variant -- and the switch really changes
  the arithmetic (results differ from the serial path's bits), switching it off restores them.
"""
import ctypes

import numpy as np
import pytest
import torch  # noqa: F401  (before librwkv initialises HIP)

from oracle_ctypes import gpu_variant, noise_band, assert_bits_equal
from rwkv_lib import RWKVModel, library

pytestmark = pytest.mark.gpu

TOL = 5e-6
P = ctypes.POINTER(ctypes.c_float)


def selftest():
    L = library().library
    f = L.rwkv_mi355x_selftest_wkv6
    f.argtypes = [ctypes.c_int] * 4 + [P] * 8
    f.restype = ctypes.c_bool
    return f


def operands(T, H, wpt, seed):
    rng = np.random.default_rng(seed)
    C = H * 64
    r = rng.standard_normal((T, C)).astype(np.float32)
    k = (rng.standard_normal((T, C)) * 0.5).astype(np.float32)
    v = rng.standard_normal((T, C)).astype(np.float32)
    u = (rng.standard_normal(C) * 0.5).astype(np.float32)
    d = rng.uniform(-7.0, 1.8, (T, C) if wpt else (C,))
    w = np.exp(-np.exp(d)).astype(np.float32)
    # edge channels: no decay (w = 1) and full decay (w = 0, exp(-exp(5)) underflows)
    if wpt:
        w[:, 3] = 1.0
        w[:, 5] = 0.0
        w[T // 2:, 7] = 0.0
    else:
        w[3], w[5] = 1.0, 0.0
    s0 = rng.standard_normal((H, 64, 64)).astype(np.float32)
    return k, v, r, u, w, s0


def recurrence64(k, v, r, u, w, s0, wpt):
    """float64 restatement of the wkv6 recurrence; state [h][i key][j value]."""
    T, C = k.shape
    H = C // 64
    S = s0.astype(np.float64).copy()
    uh = u.astype(np.float64).reshape(H, 64)
    y = np.zeros((T, C))
    for t in range(T):
        kt = k[t].astype(np.float64).reshape(H, 64)
        vt = v[t].astype(np.float64).reshape(H, 64)
        rt = r[t].astype(np.float64).reshape(H, 64)
        wt = (w[t] if wpt else w).astype(np.float64).reshape(H, 64)
        kv = kt[:, :, None] * vt[:, None, :]
        y[t] = np.einsum('hi,hij->hj', rt, S + uh[:, :, None] * kv).ravel()
        S = wt[:, :, None] * S + kv
    return y, S


def run(T, H, chunked, wpt, ops):
    k, v, r, u, w, s0 = ops
    y = np.zeros((T, H * 64), np.float32)
    so = np.zeros((H, 64, 64), np.float32)
    args = [np.ascontiguousarray(a) for a in (k, v, r, u, w, s0)]
    ok = selftest()(T, H, chunked, int(wpt), *[a.ctypes.data_as(P) for a in args], so.ctypes.data_as(P),
                    y.ctypes.data_as(P))
    return ok, y, so


@pytest.mark.parametrize('T,H,wpt', [(2, 1, True), (15, 2, True), (16, 1, True), (17, 2, True), (100, 2, False),
                                     (1024, 2, True), (1024, 2, False), (4096, 1, True), (1024, 32, True)])
def test_chunked_wkv6_against_float64(T, H, wpt):
    ops = operands(T, H, wpt, seed=T * 7 + H)
    y64, s64 = recurrence64(*ops, wpt)
    ok, yc, sc = run(T, H, 1, wpt, ops)
    assert ok
    ok, ys, ss = run(T, H, 0, wpt, ops)
    assert ok
    ys_err = np.abs(ys - y64).max() / np.abs(y64).max()
    yc_err = np.abs(yc - y64).max() / np.abs(y64).max()
    sc_err = np.abs(sc - s64).max() / np.abs(s64).max()
    print(f'T={T} H={H} wpt={wpt}: relative max error y serial {ys_err:.2e}, chunked {yc_err:.2e}; '
          f'state chunked {sc_err:.2e}')
    assert np.all(np.isfinite(yc)) and np.all(np.isfinite(sc))
    assert yc_err <= TOL, yc_err
    assert sc_err <= TOL, sc_err


def test_chunked_wkv6_refuses_a_single_token():
    ops = operands(1, 1, True, seed=1)
    ok, _, _ = run(1, 1, 1, True, ops)
    assert not ok
    ok, _, _ = run(1, 1, 0, True, ops)
    assert ok


@pytest.mark.parametrize('arch,fmt', [(6, 'Q4_0'), (6, 'FP16'), (5, 'Q4_1')])
def test_chunked_wkv6_model_within_noise_band(tmp_path, arch, fmt):
    lib = library()
    L = lib.library
    p = str(tmp_path / f'wkvc{arch}{fmt}.bin')
    # 512 wide (8 heads of 64), 2 layers, 1024-token vocabulary: the oracle's 8 variants finish fast
    assert L.rwkv_mi355x_write_synthetic_model(p.encode(), arch, 1024, 512, 2, 0, fmt.encode(), 17)
    toks = [int(t) for t in np.random.default_rng(arch).integers(0, 1024, 90)]  # 5 chunks + 10
    m = RWKVModel(lib, p)
    slg, sst = m.eval_sequence(toks, None, use_numpy=True)
    glg, gst = gpu_variant(p, toks, sequence=True)
    assert_bits_equal(slg, glg, 'serial wkv (default) logits')
    assert L.rwkv_mi355x_debug_set(m._ctx.ptr, b'wkv_chunk', 1)
    clg, cst = m.eval_sequence(toks, None, use_numpy=True)
    assert not np.array_equal(clg, slg), 'the switch did not change the wkv arithmetic'
    olg, _, noise, _ = noise_band(p, toks, sequence=True)
    d = float(np.abs(clg - olg).max())
    print(f'v{arch} {fmt}: chunked max|dlogit| vs ggml-order oracle {d:.3g}, serial '
          f'{float(np.abs(slg - olg).max()):.3g}, noise band {noise:.3g}')
    assert d <= max(1e-3, 1.5 * noise), (d, noise)
    assert np.all(np.isfinite(cst))
    assert L.rwkv_mi355x_debug_set(m._ctx.ptr, b'wkv_chunk', 0)
    lg2, st2 = m.eval_sequence(toks, None, use_numpy=True)
    assert_bits_equal(lg2, slg, 'switch off again: logits')
    assert_bits_equal(st2, sst, 'switch off again: state')
    m.free()


# ---------------------------------------------------------------------------------------------------
# Chunk-parallel WKV-7 (csrc/wkv7_chunk.hip, the same switch) -- the v7 time-mixing recurrence
# (reference rwkv_operators_wkv_v7.inc:37-107): the
# transition diag(w) + a b^T is solved per 16-token chunk in its triangular (WY-like) form, so the sums
# are re-associated; held to the same kind of bar as WKV-6 above, against a float64 recurrence.

TOL7 = 2e-5


def selftest7():
    L = library().library
    f = L.rwkv_mi355x_selftest_wkv7
    f.argtypes = [ctypes.c_int] * 3 + [P] * 9
    f.restype = ctypes.c_bool
    return f


def operands7(T, H, seed):
    """v7's operand ranges: w = exp(-0.606531 sigmoid(.)) in [0.545, 1); kk unit rows per head,
    a = -kk, b = kk * iclr with iclr in (0, 1) (rwkv_graph.inc:430-460)."""
    rng = np.random.default_rng(seed)
    C = H * 64
    r = rng.standard_normal((T, C)).astype(np.float32)
    k = (rng.standard_normal((T, C)) * 0.5).astype(np.float32)
    v = rng.standard_normal((T, C)).astype(np.float32)
    w = np.exp(-0.606531 / (1.0 + np.exp(-rng.standard_normal((T, C)) * 2.0))).astype(np.float32)
    kk = rng.standard_normal((T, H, 64))
    kk /= np.linalg.norm(kk, axis=-1, keepdims=True)
    iclr = 1.0 / (1.0 + np.exp(-rng.standard_normal((T, H, 64))))
    a = (-kk).reshape(T, C).astype(np.float32)
    b = (kk * iclr).reshape(T, C).astype(np.float32)
    s0 = (rng.standard_normal((H, 64, 64)) * 0.5).astype(np.float32)
    return r, w, k, v, a, b, s0


def recurrence7_64(r, w, k, v, a, b, s0):
    """float64 restatement: state [h][i value][j key]; sa = S a, S <- S diag(w) + sa b^T + v k^T, y = S r."""
    T, C = r.shape
    H = C // 64
    S = s0.astype(np.float64).copy()
    y = np.zeros((T, C))
    for t in range(T):
        rt, wt, kt, vt, at, bt = (x[t].astype(np.float64).reshape(H, 64) for x in (r, w, k, v, a, b))
        sa = np.einsum('hij,hj->hi', S, at)
        S = S * wt[:, None, :] + sa[:, :, None] * bt[:, None, :] + vt[:, :, None] * kt[:, None, :]
        y[t] = np.einsum('hij,hj->hi', S, rt).ravel()
    return y, S


def run7(T, H, chunked, ops):
    args = [np.ascontiguousarray(x) for x in ops]
    y = np.zeros((T, H * 64), np.float32)
    so = np.zeros((H, 64, 64), np.float32)
    ok = selftest7()(T, H, chunked, *[x.ctypes.data_as(P) for x in args], so.ctypes.data_as(P), y.ctypes.data_as(P))
    return ok, y, so


@pytest.mark.parametrize('T,H', [(2, 1), (15, 2), (16, 1), (17, 2), (100, 3), (1024, 2), (4096, 1), (1024, 40)])
def test_chunked_wkv7_against_float64(T, H):
    ops = operands7(T, H, seed=T * 5 + H)
    y64, s64 = recurrence7_64(*ops)
    ok, yc, sc = run7(T, H, 1, ops)
    assert ok
    ok, ys, ss = run7(T, H, 0, ops)
    assert ok
    ys_err = np.abs(ys - y64).max() / np.abs(y64).max()
    yc_err = np.abs(yc - y64).max() / np.abs(y64).max()
    sc_err = np.abs(sc - s64).max() / np.abs(s64).max()
    ss_err = np.abs(ss - s64).max() / np.abs(s64).max()
    print(f'T={T} H={H}: relative max error y serial {ys_err:.2e}, chunked {yc_err:.2e}; '
          f'state serial {ss_err:.2e}, chunked {sc_err:.2e}')
    assert np.all(np.isfinite(yc)) and np.all(np.isfinite(sc))
    assert yc_err <= TOL7, yc_err
    assert sc_err <= TOL7, sc_err


def test_chunked_wkv7_refuses_a_single_token():
    ops = operands7(1, 1, seed=2)
    ok, _, _ = run7(1, 1, 1, ops)
    assert not ok
    ok, _, _ = run7(1, 1, 0, ops)
    assert ok


def test_chunked_wkv7_model_within_noise_band(tmp_path):
    lib = library()
    L = lib.library
    p = str(tmp_path / 'wkvc7.bin')
    assert L.rwkv_mi355x_write_synthetic_model(p.encode(), 7, 1024, 512, 2, 0, b'Q5_1', 19)
    toks = [int(t) for t in np.random.default_rng(7).integers(0, 1024, 90)]
    m = RWKVModel(lib, p)
    slg, sst = m.eval_sequence(toks, None, use_numpy=True)
    glg, gst = gpu_variant(p, toks, sequence=True)
    assert_bits_equal(slg, glg, 'serial wkv7 (default) logits')
    assert L.rwkv_mi355x_debug_set(m._ctx.ptr, b'wkv_chunk', 1)
    clg, cst = m.eval_sequence(toks, None, use_numpy=True)
    # (the state, not the logits: WKV-7's ~1e-7 relative differences usually vanish in the Q8
    # quantization of Wo's input, so the logits can come out bit-identical)
    assert not np.array_equal(cst, sst), 'the switch did not change the wkv7 arithmetic'
    olg, _, noise, _ = noise_band(p, toks, sequence=True)
    d = float(np.abs(clg - olg).max())
    print(f'v7 Q5_1: chunked max|dlogit| vs ggml-order oracle {d:.3g}, serial '
          f'{float(np.abs(slg - olg).max()):.3g}, noise band {noise:.3g}')
    assert d <= max(1e-3, 1.5 * noise), (d, noise)
    assert np.all(np.isfinite(cst))
    assert L.rwkv_mi355x_debug_set(m._ctx.ptr, b'wkv_chunk', 0)
    lg2, st2 = m.eval_sequence(toks, None, use_numpy=True)
    assert_bits_equal(lg2, slg, 'switch off again: logits')
    assert_bits_equal(st2, sst, 'switch off again: state')
    m.free()
