"""Locates the first bit-level difference between the GPU path and the oracle's GPU-association
variant: the first decode token whose logits/state differ, then, at that token, the first layer
whose output differs when both sides start the layer from identical inputs (rwkv_mi355x_eval_layers
vs oracle_eval_layers), and which part of that layer's state slice differs.
Usage (GPU box): python tools/debug_bitexact.py MODEL [n_tokens]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tests'))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))

import oracle_ctypes as oc  # noqa: E402
from rwkv_lib import RWKVModel, library  # noqa: E402

LONG = list(b'This is a port of [BlinkDL/RWKV-LM](https://github.com/BlinkDL/RWKV-LM')


def neq(a, b):
    return np.flatnonzero(np.ascontiguousarray(a, np.float32).view(np.uint32) !=
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def main():
    import torch
    path = sys.argv[1]
    ntok = int(sys.argv[2]) if len(sys.argv) > 2 else len(LONG)
    toks = [int(t) for t in (LONG * 20)[:ntok]]
    L = library()
    m = RWKVModel(L, path)
    lib = L.library
    oc.set_variant(oc.VARIANT_GPU)
    om = oc.OracleModel(path)
    C, NL, S = om.n_embed, om.n_layer, om.head_size
    per = C * (2 + S) if om.arch_major >= 5 else 5 * C
    st_g = st_o = None
    bad = None
    for i, t in enumerate(toks):
        st_prev = st_o
        lg_g, st_g = m.eval(t, st_g, st_g, None, use_numpy=True) if st_g is not None else m.eval(t, None, None, None, use_numpy=True)
        lg_o, st_o = om.eval_sequence([t], st_o)
        dl, ds = neq(lg_g, lg_o), neq(st_g, st_o)
        if dl.size or ds.size:
            print(f'token {i}: {dl.size} logits, {ds.size} state values differ; max|dlogit| {np.abs(lg_g - lg_o).max():.3g}')
            if ds.size:
                j = int(ds[0])
                lay, off = divmod(j, per)
                part = 'ffn_xx' if off < C else 'att_xx' if off < 2 * C else 'att state'
                print(f'  first state diff: layer {lay} {part} offset {off}: {st_g[j]!r} vs {st_o[j]!r}')
            bad = (i, t, st_prev)
            break
    else:
        print(f'all {len(toks)} tokens bit-exact')
        return
    i, t, st_prev = bad
    if st_prev is None:
        st_prev = om.init_state()
    # layer by layer from identical inputs
    dev = torch.device('cuda', 0)
    planes = 2 if om.arch_major == 7 else 1
    x = np.zeros((planes, 1, C), np.float32)
    for l in range(NL):
        # oracle: layers [0, l) give the stream entering l
        xin = x.copy()
        xo = xin.copy()
        _, st_ol = om.eval_layers([t], l, l + 1, xo[0], xo[1] if planes == 2 else None, st_prev, want_logits=False)
        xd = torch.from_numpy(xin.copy()).to(dev)
        assert lib.rwkv_mi355x_state_upload(m._ctx.ptr, st_prev.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        ok = lib.rwkv_mi355x_eval_layers(m._ctx.ptr, np.array([t], np.uint32).ctypes.data, 1, l, l + 1,
                                         xd[0].data_ptr(), xd[1].data_ptr() if planes == 2 else None, False, None)
        assert ok
        torch.cuda.synchronize()
        sg = np.zeros(om.state_len, np.float32)
        assert lib.rwkv_mi355x_state_download(m._ctx.ptr, sg.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        xg = xd.cpu().numpy()
        sl = slice(l * per, (l + 1) * per)
        dsl = neq(sg[sl], st_ol[sl])
        dx = neq(xg, xo)
        print(f'layer {l}: x diff {dx.size}, state-slice diff {dsl.size}')
        if dsl.size or dx.size:
            if dsl.size:
                off = int(dsl[0])
                part = 'ffn_xx' if off < C else 'att_xx' if off < 2 * C else 'att state'
                print(f'  first: {part} offset {off}: gpu {sg[sl][off]!r} oracle {st_ol[sl][off]!r}')
                for name, a, b in (('ffn_xx', 0, C), ('att_xx', C, 2 * C), ('att state', 2 * C, per)):
                    print(f'  {name}: {neq(sg[sl][a:b], st_ol[sl][a:b]).size} differ')
            if dx.size:
                k = int(dx[0])
                print(f'  first x diff at {k}: gpu {xg.ravel()[k]!r} oracle {xo.ravel()[k]!r}, max {np.abs(xg - xo).max():.3g}')
            break
        x = xo
    oc.set_variant(0)


if __name__ == '__main__':
    main()
