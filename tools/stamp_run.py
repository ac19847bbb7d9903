"""Decode a few tokens of the bench model with the stamp build (rwkv.cppy_amd/build_stamp) and
summarize the per-launch phase stamps of one decode token (csrc/stamp.hpp).
Usage: python tools/stamp_run.py [config] [out.bin] [knob=value,...]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (CONFIGS)

cfg = sys.argv[1] if len(sys.argv) > 1 else 'v6-1b6-q4_0'
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, 'gpurun_out', f'stamps_{cfg}.bin')
os.environ['RWKV_STAMP_OUT'] = out
import rwkv_cpp  # noqa: E402
lib = rwkv_cpp.RWKVSharedLibrary(os.path.join(REPO, 'rwkv.cppy_amd', 'build_stamp', 'librwkv.so'))
L = lib.library
arch, V, C, NL, F, fmt, label = bench.CONFIGS[cfg]
path = f'/tmp/rwkv_bench/{cfg}-seed1.bin'
os.makedirs('/tmp/rwkv_bench', exist_ok=True)
if not os.path.isfile(path):
    assert L.rwkv_mi355x_write_synthetic_model(path.encode(), arch, V, C, NL, F, fmt.encode(), 1)
ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
# optional per-context knobs (rwkv_mi355x_debug_set), e.g. "decode_fusion=127,wo_prepoll=0"
for kv in [s for s in (sys.argv[3] if len(sys.argv) > 3 else '').split(',') if s]:
    k, v = kv.split('=')
    assert L.rwkv_mi355x_debug_set(ctx.ptr, k.encode(), int(v, 0)), k
assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
tok = (ctypes.c_int32 * 1)(7)
for i in range(12):
    tok[0] = (i * 7919) % V
    assert L.rwkv_mi355x_eval_device(ctx.ptr, tok, 1, True, None, False)
L.rwkv_mi355x_sync(ctx.ptr)
lib.rwkv_free(ctx)

r = np.fromfile(out, dtype=np.uint64).reshape(-1, 8)
r = r[np.argsort(r[:, 0], kind='stable')]
kid = ((r[:, 3] >> 32) & 15).astype(np.int64)  # kid bits 32..43, cycles 44..63
names = {1: 'k_mva', 2: 'k_mv', 3: 'att6', 5: 'embed', 6: 'att6f/co', 7: 'mvsig', 8: 'att4f', 9: 'ffnf', 10: 'sigmaa'}
# launches: runs of equal kernel id in start order
cuts = np.flatnonzero(np.diff(kid) != 0) + 1
segs = np.split(np.arange(len(r)), cuts)
emb = [i for i, s in enumerate(segs) if kid[s[0]] == 5]
a, b = emb[-3], emb[-2]  # one whole token, away from the ends
print(f'{cfg}: {len(segs)} launches recorded; token span {(r[segs[b][0], 0] - r[segs[a][0], 0]) / 100:.1f} us, '
      f'{b - a} launches')
print(f"{'kernel':10s} {'WGs':>5s} {'gap':>6s} {'spread':>6s} {'mid50':>6s} {'mid90':>6s} {'dur50':>6s} {'dur90':>6s} "
      f"{'span':>6s}   (us; gap = first start - previous launch's last end; mid = inputs ready after own start)")
prev_end = None
tot = 0.0
for s in segs[a:b]:
    t0, t1, t2 = r[s, 0].astype(np.float64), r[s, 1].astype(np.float64), r[s, 2].astype(np.float64)
    k = int(kid[s[0]])
    nm = names.get(k & 15, 'maa' if (k & 15) == 4 else str(k))
    first, last = t0.min(), t2.max()
    gap = (first - prev_end) / 100 if prev_end is not None else float('nan')
    mid = (t1[t1 > 0] - t0[t1 > 0]) / 100 if (t1 > 0).any() else np.array([np.nan])
    dur = (t2 - t0) / 100
    span = (last - first) / 100
    tot += span + (gap if gap == gap else 0)
    xs = ''
    for q in range(4):
        xq = r[s, 4 + q].astype(np.float64)
        ok = xq > 0
        if ok.any():
            xs += f'  x{q} {np.percentile((xq[ok] - t0[ok]) / 100, 50):5.2f}'
    cyc = (r[s, 3] >> 44).astype(np.float64)
    ghz = np.percentile(cyc / np.maximum(dur * 1e3, 1e-9), 50)  # cycles per ns
    print(f'{nm:10s} {len(s):5d} {gap:6.2f} {(t0.max() - first) / 100:6.2f} {np.percentile(mid, 50):6.2f} '
          f'{np.percentile(mid, 90):6.2f} {np.percentile(dur, 50):6.2f} {np.percentile(dur, 90):6.2f} {span:6.2f}'
          f'  {ghz:4.2f}GHz{xs}')
    prev_end = last
