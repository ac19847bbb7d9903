"""Which float-matmul shapes give NaN outputs (tools/, GPU box): selftest_matmul over a few shapes."""
import sys
sys.path.insert(0, 'tests')
import numpy as np
import test_gpu_kernels as tk

L = tk.lib()
for fmt in ('FP32', 'FP16'):
    for (M, K, T) in [(576, 2560, 64), (512, 2560, 64), (576, 2048, 64), (576, 2560, 32), (64, 2560, 64),
                      (576, 2560, 100), (128, 2048, 100), (96, 4096, 33), (64, 512, 16)]:
        rng = np.random.default_rng(M * 5 + K + T * 3 + 4)
        w = (rng.standard_normal((M, K)) / np.sqrt(K)).astype(np.float32)
        x = rng.standard_normal((T, K)).astype(np.float32)
        wb = tk.quantize_rows(fmt, w)
        y = np.zeros((T, M), np.float32)
        ok = L.rwkv_mi355x_selftest_matmul(tk.TYPE_IDS[fmt], wb.ctypes.data, K, M, x.ctypes.data, T, y.ctypes.data)
        ref = x.astype(np.float64) @ w.astype(np.float64).T if fmt == 'FP32' else None
        nan = int(np.isnan(y).sum())
        err = float(np.abs(y - ref).max()) if ref is not None and nan == 0 else -1
        print(fmt, M, K, T, 'ok' if ok else 'FAIL', 'nan', nan, 'maxerr', err, flush=True)
