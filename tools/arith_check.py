"""Offline check of tools/arith_probe.hip's output (gpurun_out/arith_probe.bin): which rounding
v_dot2_f32_f16 performs, and whether f32 sqrt / division are correctly rounded."""
import sys
import numpy as np
from fractions import Fraction

p = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/arith_probe.bin'
n = 1 << 20
raw = np.fromfile(p, np.uint32)
a, b, c, x, y, dot, sq, dv, rc = [raw[i * n:(i + 1) * n] for i in range(9)]
f = lambda u: u.view(np.float32)
ah = a.view(np.float16).reshape(-1, 2).astype(np.float64)
bh = b.view(np.float16).reshape(-1, 2).astype(np.float64)
p0 = ah[:, 0] * bh[:, 0]
p1 = ah[:, 1] * bh[:, 1]
cc = f(c).astype(np.float64)
# one rounding of the exact sum (products exact in f64, the sum of three such values exact in f64
# whenever their exponents are within 53 bits; flag the others)
fused = (p0 + p1 + cc).astype(np.float32)
two = (np.float32(p0 + p1) + np.float32(cc)).astype(np.float32)  # round(p0+p1) then + c
seq = (np.float32(np.float32(cc + p0)) + np.float32(p1)).astype(np.float32)  # (c + p0) + p1
fma2 = np.float32(np.float32(p0 + cc) + p1)
g = f(dot)
for name, e in [('fused single rounding', fused), ('round(p0+p1)+c', two), ('(c+p0)+p1', seq)]:
    print(f'fdot2 vs {name}: {np.mean(g.view(np.uint32) == e.view(np.uint32)) * 100:.4f}% equal')
xs, ys = f(x).astype(np.float64), f(y).astype(np.float64)
print('sqrt correctly rounded:', np.mean(np.sqrt(np.abs(xs)).astype(np.float32).view(np.uint32) == sq) * 100, '%')
print('div  correctly rounded:', np.mean((xs / ys).astype(np.float32).view(np.uint32) == dv) * 100, '%')
print('rcp  correctly rounded:', np.mean((1.0 / ys).astype(np.float32).view(np.uint32) == rc) * 100, '%')
