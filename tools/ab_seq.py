"""A/B of per-context / GEMM knobs (rwkv_mi355x_debug_set) on the sequence path, interleaved on ONE
loaded model.

    python tools/ab_seq.py --config v6-1b6-q4_0 --arm "" --arm "wkv_chunk=1" --reps 5

Each arm: knobs applied (defaults first), then one T-token rwkv_mi355x_eval_device from a fresh
state whose logits must equal arm 0's bit for bit (else BROKEN), then REPS timed sequences.
Prints the median ms per sequence and tokens/s per arm.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))

from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='v6-1b6-q4_0', choices=sorted(CONFIGS))
    ap.add_argument('--arm', action='append', default=[])
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--seq-len', type=int, default=1024)
    ap.add_argument('--model-dir', default=os.environ.get('RWKV_BENCH_DIR', '/tmp/rwkv_bench'))
    ap.add_argument('--lib', default=os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'),
                    help='the library to load (another build, for a build-vs-build comparison)')
    args = ap.parse_args()
    arms = args.arm or ['']
    import torch  # noqa: F401
    import rwkv_cpp
    lib = rwkv_cpp.RWKVSharedLibrary(args.lib)
    L = lib.library
    arch, V, C, NL, F, fmt, label = CONFIGS[args.config]
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f'{args.config}-seed1.bin')
    if not os.path.isfile(path):
        assert L.rwkv_mi355x_write_synthetic_model((path + '.tmp').encode(), arch, V, C, NL, F, fmt.encode(), 1)
        os.replace(path + '.tmp', path)
    ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
    n_vocab = L.rwkv_get_n_vocab(ctx.ptr)
    P_F = ctypes.POINTER(ctypes.c_float)
    toks = np.ascontiguousarray(np.random.default_rng(3).integers(0, n_vocab, args.seq_len).astype(np.int32))
    tp = toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))

    def knobs(spec):
        for kv in [s for s in spec.split(',') if s]:
            k, v = kv.split('=')
            if not L.rwkv_mi355x_debug_set(ctx.ptr, k.encode(), int(v, 0)):
                raise SystemExit(f'unknown knob {k}')

    ref = None
    res = {a: [] for a in arms}
    broken = set()
    for rep in range(args.reps):
        for a in arms:
            knobs('wkv_chunk=0')
            knobs(a)
            lg = np.zeros(n_vocab, np.float32)
            assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
            assert L.rwkv_mi355x_eval_device(ctx.ptr, tp, len(toks), True, lg.ctypes.data_as(P_F), True)
            if ref is None:
                ref = lg.copy()
            elif not np.array_equal(lg.view(np.uint32), ref.view(np.uint32)):
                broken.add(a)
            assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
            assert L.rwkv_mi355x_sync(ctx.ptr)
            t0 = time.perf_counter()
            assert L.rwkv_mi355x_eval_device(ctx.ptr, tp, len(toks), True, None, True)
            res[a].append((time.perf_counter() - t0) * 1e3)
    print(f'{label}: T = {args.seq_len} sequence x {args.reps} reps, ms (median [min, max])')
    for a in arms:
        v = np.array(res[a])
        flag = '  BROKEN (bits differ from arm 0)' if a in broken else ''
        print(f'  {a or "(defaults)":40s} {np.median(v):8.2f} [{v.min():.2f}, {v.max():.2f}]  '
              f'{args.seq_len / np.median(v) * 1e3:9.0f} tok/s{flag}')
    lib.rwkv_free(ctx)
    return 1 if broken else 0


if __name__ == '__main__':
    sys.exit(main())
