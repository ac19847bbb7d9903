"""Model-file tooling: the PyTorch -> rwkv.cpp converter and the LoRA merge
(rwkv.cppy_amd/python/rwkv_cpp/convert.py), on CPU.

Pins: the reference converter's own byte-exact writer test (convert_pytorch_to_ggml.test.py:7-51),
and the reference's tiny FP32/FP16 fixtures: each fixture is taken back to PyTorch form (inverse of
the stored-tensor transforms), converted forward again, and must reproduce the fixture's key order,
shapes and storage types exactly, every untransformed tensor byte for byte, and the transformed
time tensors (exp / log round trip) to float32 rounding.
"""
import os
import struct

import numpy as np
import pytest

from rwkv_lib import PKG  # noqa: F401  (puts the package on sys.path)
from rwkv_cpp import convert

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


def test_reference_writer_bytes(tmp_path):
    """convert_pytorch_to_ggml.test.py:7-51, restated."""
    sd = {'emb.weight': np.array([[1, 2], [3, 4], [5, 6]], np.float32),
          'blocks.0.ln1.weight': np.array([1], np.float32)}
    out = tmp_path / 'x.bin'
    convert.write_state_dict(sd, str(out), 'FP32', log=lambda *a: None)
    expected = struct.pack('=iiiiii' + 'iiiii10sffffff' + 'iiii19sf',
                           0x67676d66, 101, 3, 2, 1, 0,
                           2, 10, 0, 2, 3, b'emb.weight', 1.0, 2.0, 3.0, 4.0, 5.0, 6.0,
                           1, 19, 0, 1, b'blocks.0.ln1.weight', 1.0)
    assert out.read_bytes() == expected


def to_pytorch(tensors, version):
    """Inverse of convert.transform over a fixture's tensors (PyTorch keys, order and shapes)."""
    sd = {}
    for key, t in tensors:
        t = t.astype(np.float32) if t.dtype == np.float16 and '.time_' in key else t
        if version == '7.0':
            if key.endswith('att.x_rwkvag'):
                layer = key.split('.')[1]
                for i, n in enumerate('rwkvag'):
                    sd[f'blocks.{layer}.att.x_{n}'] = t[i:i + 1] if t.ndim == 3 else t.reshape(6, -1)[i]
                continue
            if any(s in key for s in convert._V7_LORA):
                t = t.T
        elif version in ('5.1', '5.2'):
            if '.time_decay' in key:
                t = np.log(-np.log(t.astype(np.float32))).reshape(-1) if version == '5.1' else \
                    np.log(-np.log(t[..., 0].astype(np.float32)))
            elif '.time_first' in key:
                t = np.log(t.astype(np.float32)).reshape(-1)
            elif '.time_faaaa' in key:
                t = t[..., 0]
        elif version == '4':
            if '.time_decay' in key:
                t = np.log(-t.astype(np.float32))
        sd[key] = np.ascontiguousarray(t)
    return sd


FIXTURES = [('4v0-660K', '4'), ('5v1-730K', '5.1'), ('5v2-730K', '5.2'), ('7v0-834K', '7.0')]


@pytest.mark.parametrize('name,version', FIXTURES)
@pytest.mark.parametrize('fmt', ['FP32', 'FP16'])
def test_converter_reproduces_reference_fixtures(tmp_path, name, version, fmt):
    src = os.path.join(GOLD, f'tiny-rwkv-{name}-{fmt}.bin')
    header, tensors = convert.read_model_file(src)
    sd = to_pytorch(tensors, version)
    assert convert.detect_version(sd) == version
    out = tmp_path / 'y.bin'
    convert.write_state_dict(sd, str(out), fmt, log=lambda *a: None)
    h2, t2 = convert.read_model_file(str(out))
    # the fixtures carry file version 100 (an older converter); the current writer emits 101
    assert h2[0] == header[0] and h2[1] == 101 and h2[2:] == header[2:]
    assert [k for k, _ in t2] == [k for k, _ in tensors]
    for (k, a), (_, b) in zip(tensors, t2):
        assert a.shape == b.shape and a.dtype == b.dtype, (k, a.shape, b.shape, a.dtype, b.dtype)
        transformed = (version == '4' and '.time_decay' in k) or \
                      (version in ('5.1', '5.2') and ('.time_decay' in k or '.time_first' in k))
        if transformed:
            np.testing.assert_allclose(b, a, rtol=4e-7, atol=1e-30, err_msg=k)
        else:
            assert a.tobytes() == b.tobytes(), k
    if not any(('.time_decay' in k or '.time_first' in k) for k, _ in tensors) or version == '7.0':
        ref = bytearray(open(src, 'rb').read())
        ref[4:8] = struct.pack('=i', 101)
        assert out.read_bytes() == bytes(ref)


def test_lora_merge(tmp_path):
    """W + B @ A * (alpha / r) into one matrix, a full replacement of another parameter, every other
    tensor byte-identical (merge_lora_into_ggml.py:45-181)."""
    torch = pytest.importorskip('torch')
    src = os.path.join(GOLD, 'tiny-rwkv-4v0-660K-FP32.bin')
    _, tensors = convert.read_model_file(src)
    w = dict(tensors)['blocks.0.att.key.weight']
    g = torch.Generator().manual_seed(5)
    r, alpha = 4, 8
    a = torch.randn(r, w.shape[1], generator=g)
    b = torch.randn(w.shape[0], r, generator=g)
    ln = torch.randn(w.shape[1], generator=g)
    lora = {'blocks.0.att.key.lora_A': a, 'blocks.0.att.key.lora_B': b, 'blocks.0.ln1.weight': ln,
            'blocks.9.unused.lora_A': a}
    out = tmp_path / 'm.bin'
    unused = convert.merge_lora(src, 'v4', lora, alpha, str(out), log=lambda *a: None)
    assert unused == ['blocks.9.unused.lora_A']
    _, merged = convert.read_model_file(str(out))
    assert [k for k, _ in merged] == [k for k, _ in tensors]
    m = dict(merged)
    expect = (torch.from_numpy(w.copy()) + b @ a * (alpha / r)).numpy()
    assert m['blocks.0.att.key.weight'].tobytes() == expect.tobytes()
    assert m['blocks.0.ln1.weight'].tobytes() == ln.numpy().tobytes()
    for k, t in tensors:
        if k not in ('blocks.0.att.key.weight', 'blocks.0.ln1.weight'):
            assert m[k].tobytes() == t.tobytes(), k
