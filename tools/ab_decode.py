"""A/B of per-context decode knobs (rwkv_mi355x_debug_set) on ONE loaded model, interleaved.

    python tools/ab_decode.py --config v6-1b6-q4_0 --arm "" --arm "decode_fusion=61" --reps 5

Each arm is a comma list of name=value knobs applied to the same context (debug_set drops the
captured graphs; every arm re-captures), then: the bits of 8 fixed decode tokens from a fresh state
(must equal arm 0's, or the arm is reported BROKEN), W warmup tokens and K timed device-resident
decode tokens (graph replays, logits on).  Arms run round-robin REPS times; the median us/token
per arm is printed, with its spread.  Knobs a context does not know make the run fail.
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
    ap.add_argument('--steps', type=int, default=256)
    ap.add_argument('--warmup', type=int, default=16)
    ap.add_argument('--model-dir', default=os.environ.get('RWKV_BENCH_DIR', '/tmp/rwkv_bench'))
    args = ap.parse_args()
    arms = args.arm or ['']
    import torch  # noqa: F401  (torch's HIP runtime first)
    import rwkv_cpp
    lib = rwkv_cpp.RWKVSharedLibrary(os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'))
    L = lib.library
    arch, V, C, NL, F, fmt, label = CONFIGS[args.config]
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f'{args.config}-seed1.bin')
    if not os.path.isfile(path):
        assert L.rwkv_mi355x_write_synthetic_model((path + '.tmp').encode(), arch, V, C, NL, F, fmt.encode(), 1)
        os.replace(path + '.tmp', path)
    ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
    n_vocab = L.rwkv_get_n_vocab(ctx.ptr)
    P_INT = ctypes.POINTER(ctypes.c_int32)
    P_F = ctypes.POINTER(ctypes.c_float)
    rng = np.random.default_rng(5)
    toks = [int(t) for t in rng.integers(0, n_vocab, args.warmup + args.steps)]
    check = [int(t) for t in rng.integers(0, n_vocab, 8)]

    def knobs(spec):
        for kv in [s for s in spec.split(',') if s]:
            k, v = kv.split('=')
            if not L.rwkv_mi355x_debug_set(ctx.ptr, k.encode(), int(v, 0)):
                raise SystemExit(f'unknown knob {k}')

    def one(t, lg=None):
        a = (ctypes.c_int32 * 1)(t)
        return L.rwkv_mi355x_eval_device(ctx.ptr, ctypes.cast(a, P_INT), 1, True, lg, False)

    ref = None
    res = {a: [] for a in arms}
    broken = set()
    for rep in range(args.reps):
        for a in arms:
            knobs('decode_fusion=-1,wkv_chunk=0,wo_rows=8,wo_prepoll=1,ffn_wdelay=-1,ffn_prepoll=1,co_mode=-1')  # defaults first, then the arm
            knobs(a)
            assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
            lg = np.zeros(n_vocab, np.float32)
            for t in check:
                assert one(t)
            assert L.rwkv_mi355x_eval_device(ctx.ptr, ctypes.cast((ctypes.c_int32 * 1)(check[0]), P_INT), 1, True,
                                             lg.ctypes.data_as(P_F), True)
            if ref is None:
                ref = lg.copy()
            elif not np.array_equal(lg.view(np.uint32), ref.view(np.uint32)):
                broken.add(a)
            for t in toks[:args.warmup]:
                assert one(t)
            assert L.rwkv_mi355x_sync(ctx.ptr)
            t0 = time.perf_counter()
            for t in toks[args.warmup:]:
                assert one(t)
            assert L.rwkv_mi355x_sync(ctx.ptr)
            res[a].append((time.perf_counter() - t0) / args.steps * 1e6)
    print(f'{label}: {args.steps} decode tokens x {args.reps} reps, us/token (median [min, max])')
    for a in arms:
        v = np.array(res[a])
        flag = '  BROKEN (bits differ from arm 0)' if a in broken else ''
        print(f'  {a or "(defaults)":40s} {np.median(v):8.1f} [{v.min():.1f}, {v.max():.1f}]  '
              f'{1e6 / np.median(v):7.1f} tok/s{flag}')
    lib.rwkv_free(ctx)
    return 1 if broken else 0


if __name__ == '__main__':
    sys.exit(main())
