"""Per-kernel parity on the MI355X through the library's self-test entry points
(include/rwkv_mi355x.h), against the oracle primitive of the same name.

- activation quantizer (emit stage of every producer kernel) vs oracle_quantize_act:
  bit-exact int8 codes and fp16 scales (ggml quantize_row_q8_0/q8_1 x86 semantics).
- matmul kernel (every weight format, decode T=1 and batched T>1, ragged M/K) vs
  oracle_matmul: identical integer block dots, so only the fp32 summation order differs:
  |y_gpu - y_oracle| <= 1e-5 * (|W| |x|) + 1e-6 elementwise.
- int8-MFMA sequence GEMM vs the matvec/matmul kernel: bit-exact (same block dots, same fp32
  association), across formats, ragged M/T and K spanning 1..7 lane classes per row.
"""
import ctypes

import numpy as np
import pytest

from oracle_ctypes import TYPE_IDS, dequantize, matmul as oracle_matmul, quantize_act, quantize_rows
from rwkv_lib import library

pytestmark = pytest.mark.gpu

P_F = ctypes.POINTER(ctypes.c_float)


def lib():
    L = library().library
    L.rwkv_mi355x_selftest_quantize_act.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.rwkv_mi355x_selftest_quantize_act.restype = ctypes.c_bool
    L.rwkv_mi355x_selftest_matmul.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.rwkv_mi355x_selftest_matmul.restype = ctypes.c_bool
    L.rwkv_mi355x_selftest_gemm.argtypes = L.rwkv_mi355x_selftest_matmul.argtypes
    L.rwkv_mi355x_selftest_gemm.restype = ctypes.c_bool
    return L


@pytest.mark.parametrize('wfmt,afmt', [('Q4_0', 'Q8_0'), ('Q4_1', 'Q8_1')])
def test_activation_quantizer_bit_exact(wfmt, afmt):
    rng = np.random.default_rng(1)
    T, K = 4, 2048
    x = rng.standard_normal((T, K)).astype(np.float32) * 3
    x[0, :32] = 0.0                              # all-zero block -> d = 0, q = 0
    x[1, :32] = np.arange(32, dtype=np.float32)  # ties: x*127/31 not integral -> rint path
    x[2, 64:96] = np.float32(0.5)                # every element exactly at amax
    q = np.zeros((T, K), np.int8)
    d = np.zeros(T * K // 32, np.float32)
    s = np.zeros(T * K // 32, np.float32)
    assert lib().rwkv_mi355x_selftest_quantize_act(TYPE_IDS[wfmt], x.ctypes.data, T, K, q.ctypes.data,
                                                   d.ctypes.data, s.ctypes.data)
    for t in range(T):
        rq, rd, rs = quantize_act(afmt, x[t])
        assert np.array_equal(q[t], rq)
        assert np.array_equal(d[t * K // 32:(t + 1) * K // 32], rd)
        if afmt == 'Q8_1':
            assert np.array_equal(s[t * K // 32:(t + 1) * K // 32], rs)


@pytest.mark.parametrize('fmt', ['FP32', 'FP16', 'Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
@pytest.mark.parametrize('M,K,T', [(2048, 2048, 1), (100, 96, 1), (64, 7168, 1), (160, 2048, 5), (72, 320, 9)])
def test_matmul_kernel(fmt, M, K, T):
    rng = np.random.default_rng(M * 7 + K + T)
    w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
    x = rng.standard_normal((T, K)).astype(np.float32)
    if fmt == 'FP32':
        wb = w.view(np.uint8).ravel()
    elif fmt == 'FP16':
        wb = w.astype(np.float16).view(np.uint8).ravel()
    else:
        wb = quantize_rows(fmt, w)
    y = np.zeros((T, M), np.float32)
    assert lib().rwkv_mi355x_selftest_matmul(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y.ctypes.data)
    ref = oracle_matmul(fmt, wb, K, M, x)
    bound = np.abs(x.astype(np.float64)) @ np.abs(dequantize(fmt, wb, K, M).astype(np.float64)).T
    err = np.abs(y.astype(np.float64) - ref)
    assert np.all(err <= 1e-5 * bound + 1e-6), float((err / (bound + 1e-12)).max())


@pytest.mark.parametrize('fmt', ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
@pytest.mark.parametrize('M,K,T', [(2048, 2048, 70), (100, 96, 3), (64, 7168, 33), (160, 2048, 64), (72, 320, 9),
                                   (2048, 64, 17), (40, 4096, 2)])
def test_mfma_gemm_matches_matmul_bit_exact(fmt, M, K, T):
    rng = np.random.default_rng(M * 3 + K * 5 + T)
    w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
    x = rng.standard_normal((T, K)).astype(np.float32)
    wb = quantize_rows(fmt, w)
    y_mm = np.zeros((T, M), np.float32)
    y_g = np.zeros((T, M), np.float32)
    L = lib()
    assert L.rwkv_mi355x_selftest_matmul(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_mm.ctypes.data)
    assert L.rwkv_mi355x_selftest_gemm(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_g.ctypes.data)
    assert np.array_equal(y_g.view(np.uint32), y_mm.view(np.uint32)), float(np.abs(y_g - y_mm).max())
