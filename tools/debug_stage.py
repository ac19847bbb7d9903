"""Stage-by-stage comparison of one layer's channel mixing (v6 FFN) between the GPU and the oracle's
GPU-association variant, from identical inputs: the matvec inputs (Q8 activations), ffn_r's
output, the emitted relu^2 activations and the layer output.  Usage (GPU box):
  python tools/debug_stage.py MODEL LAYER TOKEN_INDEX"""
import ctypes
import os
import struct
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tests'))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))

import oracle_ctypes as oc  # noqa: E402
from rwkv_lib import RWKVModel, library  # noqa: E402

LONG = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')
TYPES = {0: 'FP32', 1: 'FP16', 2: 'Q4_0', 3: 'Q4_1', 7: 'Q5_0', 8: 'Q5_1', 9: 'Q8_0'}
BB = {2: 18, 3: 20, 7: 22, 8: 24, 9: 34}


def read_tensors(path):
    out = {}
    with open(path, 'rb') as f:
        f.read(24)
        while True:
            h = f.read(12)
            if len(h) < 12:
                break
            nd, kl, ty = struct.unpack('<3I', h)
            ne = struct.unpack(f'<{nd}I', f.read(4 * nd))
            key = f.read(kl).decode()
            n = int(np.prod(ne))
            nb = n * 4 if ty == 0 else n * 2 if ty == 1 else n // 32 * BB[ty]
            out[key] = (ty, ne, np.frombuffer(f.read(nb), np.uint8).copy())
    return out


def f32(t):
    ty, ne, b = t
    return b.view(np.float32) if ty == 0 else b.view(np.float16).astype(np.float32)


def neq(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return int(np.count_nonzero(a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint8) !=
                                b.view(np.uint32 if b.dtype.itemsize == 4 else np.uint8)))


def main():
    import torch
    path, layer, ti = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    tens = read_tensors(path)
    L = library()
    lib = L.library
    lib.rwkv_mi355x_debug_buffer.restype = ctypes.c_longlong
    lib.rwkv_mi355x_debug_buffer.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t]
    m = RWKVModel(L, path)
    oc.set_variant(oc.VARIANT_GPU)
    om = oc.OracleModel(path)
    C, S = om.n_embed, om.head_size
    per = C * (2 + S)
    _, st_prev = om.eval_serial(LONG[:ti]) if ti else (None, om.init_state())
    t = LONG[ti]
    x = np.zeros((1, C), np.float32)
    om.eval_layers([t], 0, layer, x, None, st_prev)     # stream entering `layer`
    xo = x.copy()
    _, st_o = om.eval_layers([t], layer, layer + 1, xo, None, st_prev)
    xd = torch.from_numpy(x.copy()).cuda()
    assert lib.rwkv_mi355x_state_upload(m._ctx.ptr, st_prev.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    assert lib.rwkv_mi355x_eval_layers(m._ctx.ptr, np.array([t], np.uint32).ctypes.data, 1, layer, layer + 1,
                                       xd.data_ptr(), None, False, None)
    torch.cuda.synchronize()
    xg = xd.cpu().numpy()

    def dump(name, n, dt=np.float32):
        a = np.zeros(n, dt)
        assert lib.rwkv_mi355x_debug_buffer(m._ctx.ptr, name.encode(), a.ctypes.data, a.nbytes) == a.nbytes
        return a

    p = f'blocks.{layer}.'
    xp = st_prev[layer * per: layer * per + C]          # old ffn_xx
    xa = st_o[layer * per: layer * per + C]             # new ffn_xx = LN2(x after attention)
    mk, mr = f32(tens[p + 'ffn.time_maa_k']), f32(tens[p + 'ffn.time_maa_r'])
    xk = (xp - xa) * mk + xa
    xr = (xp - xa) * mr + xa
    wr, wk, wv = tens[p + 'ffn.receptance.weight'], tens[p + 'ffn.key.weight'], tens[p + 'ffn.value.weight']
    af = 'Q8_1' if TYPES[wr[0]] in ('Q4_1', 'Q5_1') else 'Q8_0'
    F = wk[1][1]
    for name, slot, vec in (('xk', 0, xk), ('xr', 1, xr)):
        q, d, s = oc.quantize_act(af, vec.astype(np.float32))
        gq, gd, gs = dump(f'slot{slot}.q', C, np.int8), dump(f'slot{slot}.d', C // 32), dump(f'slot{slot}.s', C // 32)
        print(f'{name}: q diff {neq(q, gq)}, d diff {neq(d, gd)}' + (f', s diff {neq(s, gs)}' if af == 'Q8_1' else ''))
    r = oc.matmul(TYPES[wr[0]], wr[2], C, C, xr[None].astype(np.float32))[0]
    print(f'ffn_r out: diff {neq(r, dump("fr", C))}')
    k = oc.matmul(TYPES[wk[0]], wk[2], C, F, xk[None].astype(np.float32))[0]
    k = np.maximum(k, 0) ** 2
    q, d, s = oc.quantize_act(af, k.astype(np.float32))
    gq, gd, gs = dump('slot2.q', F, np.int8), dump('slot2.d', F // 32), dump('slot2.s', F // 32)
    print(f'relu^2 k: q diff {neq(q, gq)}, d diff {neq(d, gd)}' + (f', s diff {neq(s, gs)}' if af == 'Q8_1' else ''))
    if neq(q, gq) or neq(d, gd):
        i = np.flatnonzero((q != gq))[:4]
        print('   first q diffs at', i, q[i], gq[i], 'k', k[i])
    v = oc.matmul(TYPES[wv[0]], wv[2], F, C, k[None].astype(np.float32))[0]
    print(f'layer out x: diff {neq(xg[0], xo[0])} (max {np.abs(xg - xo).max():.3g})')
    oc.set_variant(0)


if __name__ == '__main__':
    main()
