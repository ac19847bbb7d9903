"""The oracle's GPU-association variant (oracle.c, variant bit 8) is one more valid restatement of
the reference arithmetic: CPU-only checks (no GPU needed).

* its exp / tanh (the kernels' rk_expf / rk_tanhf, restated) are within 1 ulp of the exact values;
* on every tiny model it agrees with the ggml-order oracle (variant 0) as closely as the oracle's
  other re-associated variants agree with it: FP32 models within 1e-5 of the reference's own
  expected-logits, quantized/FP16 models within max(1e-3, 1.5 x the variants' spread).
The GPU path is then held bit-exact to this variant (tests/test_gpu_parity.py, -m gpu).
"""
import ctypes
import glob
import os

import numpy as np
import pytest

import oracle_ctypes as oc

GOLD = os.path.join(os.path.dirname(__file__), 'golden')
PROMPT = [34, 105, 110]


def _ulps(got, ref):
    got = np.asarray(got, np.float64)
    return np.abs(got - ref) / np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)


def test_gpu_exp_tanh_within_one_ulp():
    L = oc.lib()
    L.oracle_gpu_expf.restype = ctypes.c_float
    L.oracle_gpu_expf.argtypes = [ctypes.c_float]
    L.oracle_gpu_tanhf.restype = ctypes.c_float
    L.oracle_gpu_tanhf.argtypes = [ctypes.c_float]
    rng = np.random.default_rng(0)
    xe = np.concatenate([rng.uniform(-87, 88, 4000), rng.uniform(-1, 1, 2000)]).astype(np.float32)
    e = np.array([L.oracle_gpu_expf(float(x)) for x in xe], np.float32)
    assert _ulps(e, np.exp(xe.astype(np.float64))).max() <= 1.0
    xt = np.concatenate([rng.uniform(-10, 10, 4000), rng.uniform(-0.7, 0.7, 2000)]).astype(np.float32)
    t = np.array([L.oracle_gpu_tanhf(float(x)) for x in xt], np.float32)
    assert _ulps(t, np.tanh(xt.astype(np.float64))).max() <= 1.5
    # edges: overflow, underflow, NaN
    assert L.oracle_gpu_expf(100.0) == float('inf') and L.oracle_gpu_expf(-120.0) == 0.0
    assert np.isnan(L.oracle_gpu_expf(float('nan'))) and np.isnan(L.oracle_gpu_tanhf(float('nan')))
    assert L.oracle_gpu_tanhf(20.0) == 1.0 and L.oracle_gpu_tanhf(-20.0) == -1.0


def _eval(path, v):
    oc.set_variant(v)
    try:
        m = oc.OracleModel(path)
        out = m.eval_serial(PROMPT)
        m.close()
    finally:
        oc.set_variant(0)
    return out


@pytest.mark.parametrize('path', sorted(glob.glob(os.path.join(GOLD, 'tiny-rwkv-*.bin'))),
                         ids=lambda p: os.path.basename(p)[10:-4])
def test_gpu_variant_is_a_valid_restatement(path):
    lg8, st8 = _eval(path, oc.VARIANT_GPU)
    lg0, _, noise, _ = oc.noise_band(path, PROMPT)
    name = os.path.basename(path)
    if name.endswith('-FP32.bin'):
        v = name[len('tiny-rwkv-'):-len('-FP32.bin')]
        ref = np.fromfile(os.path.join(GOLD, f'expected-logits-{v}.bin'), np.float32)
        assert np.abs(lg8 - ref).max() <= 1e-5
    assert np.abs(lg8 - lg0).max() <= max(1e-3, 1.5 * noise), (np.abs(lg8 - lg0).max(), noise)
    assert np.all(np.isfinite(st8))
