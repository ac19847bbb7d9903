"""Per-kernel parity on the MI355X through the library's self-test entry points
(include/rwkv_mi355x.h), against the oracle primitive of the same name.

- activation quantizer (emit stage of every producer kernel) vs oracle_quantize_act:
  bit-exact int8 codes and fp16 scales (ggml quantize_row_q8_0/q8_1 x86 semantics).
- matmul kernel (every weight format, decode T=1 and batched T>1, ragged M/K) vs
  oracle_matmul: bit-exact against the oracle's GPU-association variant (same block dots, same
  fp32 association); against the ggml-order oracle only the fp32 summation order differs:
  |y_gpu - y_oracle| <= 1e-5 * (|W| |x|) + 1e-6 elementwise.
- int8-MFMA sequence GEMM vs the matvec/matmul kernel: bit-exact (same block dots, same fp32
  association), across formats, ragged M/T and K spanning 1..7 lane classes per row.
"""
import ctypes

import numpy as np
import pytest

from oracle_ctypes import (TYPE_IDS, VARIANT_GPU, assert_bits_equal, dequantize, matmul as oracle_matmul,
                           quantize_act, quantize_rows, set_variant)
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
    L.rwkv_mi355x_selftest_gemm_split.argtypes = L.rwkv_mi355x_selftest_matmul.argtypes + [ctypes.c_int]
    L.rwkv_mi355x_selftest_gemm_split.restype = ctypes.c_bool
    return L


def double_rounding_blocks(n, seed=5):
    """n 32-element blocks whose Q8_1 s = fp16(fp32(d * sum)) differs from a single rounding of the
    exact product d * sum (the case a fused fp32->fp16 multiply gets wrong)."""
    rng = np.random.default_rng(seed)
    found = []
    while len(found) < n:
        x = (rng.standard_normal((200000, 32)) * rng.uniform(0.01, 4, (200000, 1))).astype(np.float32)
        am = np.abs(x).max(1)
        d = (am / np.float32(127)).astype(np.float32)
        q = np.rint(x * (np.float32(127) / am)[:, None]).astype(np.int64)
        exact = d.astype(np.float64) * q.sum(1)
        two = exact.astype(np.float32).astype(np.float16)
        one = exact.astype(np.float16)
        found.extend(x[two != one][: n - len(found)])
    return np.array(found, np.float32)


@pytest.mark.parametrize('wfmt,afmt', [('Q4_0', 'Q8_0'), ('Q4_1', 'Q8_1')])
def test_activation_quantizer_bit_exact(wfmt, afmt):
    rng = np.random.default_rng(1)
    T, K = 4, 2048
    x = rng.standard_normal((T, K)).astype(np.float32) * 3
    x[0, :32] = 0.0                              # all-zero block -> d = 0, q = 0
    x[1, :32] = np.arange(32, dtype=np.float32)  # ties: x*127/31 not integral -> rint path
    x[2, 64:96] = np.float32(0.5)                # every element exactly at amax
    x[3, :32] *= np.float32(1e-5)                # d and d*sum in the fp16 subnormal range
    x[3, 32:64] = np.float32(3e-7)               # amax/127 below the smallest fp16 subnormal
    x[3, 64:64 + 8 * 32] = double_rounding_blocks(8).ravel()  # fp16(fp32(d*sum)) != fp16(d*sum)
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
@pytest.mark.parametrize('M,K,T', [(2048, 2048, 1), (100, 96, 1), (64, 7168, 1), (160, 2048, 5), (72, 320, 9),
                                   (96, 2560, 16), (2560, 64, 40), (200, 2048, 64), (64, 160, 33),
                                   (4096, 2048, 128), (512, 7168, 80)])
def test_matmul_kernel(fmt, M, K, T):
    """The sequence / batched matmul vs the GPU-association oracle, bit for bit; from T = 16 the FP16 and
    FP32 weights run on the f32 MFMA (mv_fmfma.hip)."""
    rng = np.random.default_rng(M * 7 + K + T)
    w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
    x = rng.standard_normal((T, K)).astype(np.float32)
    x[0, :64] *= np.float32(1e-5)  # Q8 scales (and Q8_1 sums) in the fp16 subnormal range
    if fmt == 'FP32':
        wb = w.view(np.uint8).ravel()
    elif fmt == 'FP16':
        wb = w.astype(np.float16).view(np.uint8).ravel()
    else:
        wb = quantize_rows(fmt, w)
    y = np.zeros((T, M), np.float32)
    assert lib().rwkv_mi355x_selftest_matmul(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y.ctypes.data)
    set_variant(VARIANT_GPU)
    try:
        ref8 = oracle_matmul(fmt, wb, K, M, x)
    finally:
        set_variant(0)
    assert_bits_equal(y, ref8, f'{fmt} matmul vs GPU-association oracle')
    ref = oracle_matmul(fmt, wb, K, M, x)
    bound = np.abs(x.astype(np.float64)) @ np.abs(dequantize(fmt, wb, K, M).astype(np.float64)).T
    err = np.abs(y.astype(np.float64) - ref)
    assert np.all(err <= 1e-5 * bound + 1e-6), float((err / (bound + 1e-12)).max())


@pytest.mark.parametrize('fmt', ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
@pytest.mark.parametrize('M,K,T', [(2048, 2048, 70), (100, 96, 3), (64, 7168, 33), (160, 2048, 64), (72, 320, 9),
                                   (2048, 64, 17), (40, 4096, 2), (64, 20480, 40), (96, 14336, 70)])
def test_mfma_gemm_matches_matmul_bit_exact(fmt, M, K, T):
    """K up to 20480 (a 14B-class FFN value width): the _1 formats' m*s pass at 9-16 blocks per class."""
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


@pytest.mark.parametrize('fmt', ['FP32', 'FP16'])
@pytest.mark.parametrize('M,K,T', [(576, 2560, 64), (128, 2048, 100), (96, 4096, 33), (64, 512, 16)])
@pytest.mark.parametrize('split', [4, 8])
def test_fmm_split_k_bit_exact(fmt, M, K, T, split):
    """Float matmuls on the f32 MFMA with the class tree split into 4 or 8 subtrees (k_fmm<WF, SPLIT> +
    k_qg_combine) == the unsplit k_fmm (itself == the oracle, test_matmul_kernel), bit for bit."""
    rng = np.random.default_rng(M * 5 + K + T * 3 + split)
    w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
    x = rng.standard_normal((T, K)).astype(np.float32)
    wb = quantize_rows(fmt, w)
    y_mm = np.zeros((T, M), np.float32)
    y_s = np.zeros((T, M), np.float32)
    L = lib()
    assert L.rwkv_mi355x_selftest_matmul(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_mm.ctypes.data)
    assert L.rwkv_mi355x_selftest_gemm_split(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_s.ctypes.data,
                                             split)
    assert np.array_equal(y_s.view(np.uint32), y_mm.view(np.uint32)), float(np.abs(y_s - y_mm).max())


@pytest.mark.parametrize('fmt', ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0'])
@pytest.mark.parametrize('M,K,T', [(2048, 2048, 64), (96, 7168, 40), (160, 2048, 128), (64, 768, 7), (2048, 64, 17),
                                   (64, 20480, 16)])
@pytest.mark.parametrize('split', [1, 2, 4, 8])
def test_mfma_gemm_split_k_bit_exact(fmt, M, K, T, split):
    """Split-K GEMM (the class tree in 4 or 8 subtrees on as many workgroups, k_qg_combine adding the
    top levels) == the decode matvec association, bit for bit, for every format and K % 2048 != 0
    (classes of unequal block counts, empty classes at K < 2048)."""
    rng = np.random.default_rng(M * 7 + K * 3 + T + split)
    w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
    x = rng.standard_normal((T, K)).astype(np.float32)
    wb = quantize_rows(fmt, w)
    y_mm = np.zeros((T, M), np.float32)
    y_g = np.zeros((T, M), np.float32)
    L = lib()
    assert L.rwkv_mi355x_selftest_matmul(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_mm.ctypes.data)
    assert L.rwkv_mi355x_selftest_gemm_split(TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y_g.ctypes.data,
                                             split)
    assert np.array_equal(y_g.view(np.uint32), y_mm.view(np.uint32)), float(np.abs(y_g - y_mm).max())
