"""rwkv.cpp model-file tooling around the eval path.

* ``write_state_dict`` / ``main``: a PyTorch RWKV checkpoint (v4, v5.1, v5.2, v6.0, v7.0) to the
  rwkv.cpp file format the MI355X library loads -- the stored-tensor semantics of the reference
  converter (python/convert_pytorch_to_ggml.py:28-161): version detection from the key set,
  the per-version parameter transforms (v4 decay -exp(d); v5 decay exp(-exp(d)) and first exp(f);
  v6 LoRA transposes and per-head decay reshape; v7 x_r..x_g concatenated into x_rwkvag and LoRA
  transposes), FP16 storage of matrices except the small / time tensors, ggml (reversed) shapes.
* ``merge_lora``: merges a LoRA checkpoint (RWKV-LM-LoRA format) into an FP32/FP16 rwkv.cpp file
  (python/merge_lora_into_ggml.py:45-181): ``W + B @ A * (alpha / r)``, plus full-parameter
  replacements run through the same transforms.

File layout (docs/FILE_FORMAT.md): header ``=iiiiii`` (magic 0x67676d66 'ggmf', version 101,
n_vocab, n_embed, n_layer, data type), then per tensor ``=iii`` (dims, key length, type 0/1), the
dims in ggml order, the UTF-8 key, the raw little-endian data.  Tensors are numpy arrays here;
torch is needed only to read .pth files (``torch.load(..., weights_only=True)``) and for the LoRA
product (the reference's torch arithmetic, so merged bytes match it).
"""
import argparse
import struct
from typing import Callable, Dict, List, Tuple

import numpy as np

MAGIC = 0x67676D66
VERSION = 101

# tensors kept in FP32 in an FP16 file (besides 1-dim vectors): convert_pytorch_to_ggml.py:131-139
_FP32_KEEP = ('.time_', '.k_k', '.k_a', '.r_k', '.x_rwkvag', '.x_k', '.w0', '.a0', '.v0')
_V7_LORA = ('.w1', '.w2', '.a1', '.a2', '.v1', '.v2', '.g1', '.g2')


def _np(t) -> np.ndarray:
    """float32 numpy copy of a tensor-like (torch tensors included, any float dtype)."""
    if hasattr(t, 'detach'):
        t = t.detach().float().cpu().numpy()
    return np.asarray(t, dtype=np.float32)


def layer_count(sd: Dict) -> int:
    n = 0
    while f'blocks.{n}.ln1.weight' in sd:
        n += 1
    if n == 0:
        raise ValueError('no blocks.N.ln1.weight keys: not an RWKV checkpoint')
    return n


def detect_version(sd: Dict) -> str:
    """'7.0', '6.0', '5.2', '5.1' or '4' from the key set (convert_pytorch_to_ggml.py:37-52)."""
    if 'blocks.0.att.k_k' in sd:
        return '7.0'
    if 'blocks.0.att.time_maa_x' in sd:
        return '6.0'
    if 'blocks.0.att.gate.weight' in sd:
        return '5.2'
    if 'blocks.0.att.ln_x.weight' in sd:
        return '5.1'
    return '4'


def _squeeze_time(key: str, t: np.ndarray) -> np.ndarray:
    return np.squeeze(t) if '.time_' in key else t


def transform(key: str, t: np.ndarray, version: str, n_head: int = 0) -> np.ndarray:
    """The stored form of one parameter (float32 in, float32 out; PyTorch axis order)."""
    t = _squeeze_time(key, t)
    if version == '7.0':
        if any(s in key for s in _V7_LORA):
            t = t.T
    elif version == '6.0':
        if '.time_faaaa' in key:
            t = t[..., None]
        if '.time_maa_w1' in key or '.time_decay_w' in key:
            t = t.T
        if '.time_maa_w2' in key:
            t = np.swapaxes(t, 1, 2)
        if '.time_decay' in key and '_w' not in key:
            t = t.reshape(n_head, -1, 1)
    elif version in ('5.1', '5.2'):
        if '.time_decay' in key:
            # torch float32 arithmetic: exp(-exp(d))
            t = _torch_f32(lambda x: x.exp().neg().exp(), t)
            t = t[..., None] if version == '5.2' else t.reshape(-1, 1, 1)
        if '.time_first' in key:
            t = _torch_f32(lambda x: x.exp(), t).reshape(-1, 1, 1)
        if '.time_faaaa' in key:
            t = t[..., None]
    else:
        if '.time_decay' in key:
            t = _torch_f32(lambda x: x.exp().neg(), t)
    return np.ascontiguousarray(t, dtype=np.float32)


def _torch_f32(fn: Callable, t: np.ndarray) -> np.ndarray:
    """Elementwise math as the reference does it (torch float32); numpy float32 otherwise."""
    try:
        import torch
        return fn(torch.from_numpy(np.ascontiguousarray(t, dtype=np.float32))).numpy()
    except ImportError:
        class _N:
            def __init__(self, a):
                self.a = a

            def exp(self):
                return _N(np.exp(self.a))

            def neg(self):
                return _N(-self.a)
        return fn(_N(np.asarray(t, np.float32))).a.astype(np.float32)


def _v7_concat(sd: Dict) -> Dict:
    """v7: att.x_r .. att.x_g of each layer concatenated (in key order) into att.x_rwkvag; the
    layer-0 v LoRA (v0/v1/v2, unused in layer 0) dropped (convert_pytorch_to_ggml.py:54-70)."""
    out: Dict = {}
    for k, v in sd.items():
        if 'att.x_' in k:
            layer = int(k.split('.')[1])
            nk = f'blocks.{layer}.att.x_rwkvag'
            out[nk] = np.concatenate([out[nk], _np(v)], axis=0) if nk in out else _np(v)
        elif any(s in k for s in ('blocks.0.att.v0', 'blocks.0.att.v1', 'blocks.0.att.v2')):
            continue
        else:
            out[k] = v
    return out


def tensor_record(key: str, t: np.ndarray) -> bytes:
    """One tensor record: =iii header, ggml-order dims, key, data (float32 or float16)."""
    k = key.encode('utf-8')
    ftype = 1 if t.dtype == np.float16 else 0
    head = struct.pack('=iii', t.ndim, len(k), ftype) + struct.pack('=' + 'i' * t.ndim, *reversed(t.shape))
    return head + k + np.ascontiguousarray(t).tobytes()


def write_state_dict(state_dict: Dict, dest_path: str, data_type: str, log: Callable = print) -> None:
    """PyTorch state dict -> rwkv.cpp file (data_type 'FP16'/'float16' or 'FP32'/'float32')."""
    emb = _np(state_dict['emb.weight'])
    n_layer = layer_count(state_dict)
    n_vocab, n_embed = emb.shape
    version = detect_version(state_dict)
    log(f'Detected RWKV v{version}')
    sd = _v7_concat(state_dict) if version == '7.0' else state_dict
    fp16 = data_type in ('FP16', 'float16')
    n_head = _np(sd['blocks.0.att.time_faaaa']).shape[0] if version == '6.0' else 0
    with open(dest_path, 'wb') as f:
        f.write(struct.pack('=iiiiii', MAGIC, VERSION, n_vocab, n_embed, n_layer, 1 if fp16 else 0))
        for key in sd.keys():
            t = transform(key, _np(sd[key]), version, n_head)
            if fp16 and t.ndim > 1 and not any(s in key for s in _FP32_KEEP):
                t = t.astype(np.float16)
            log(f'Writing {key}, shape {tuple(t.shape)}, type {t.dtype}')
            f.write(tensor_record(key, t))


# ---------------------------------------------------------------------------------------- reader
def read_model_file(path: str) -> Tuple[Tuple[int, ...], List[Tuple[str, np.ndarray]]]:
    """(header, [(key, array in PyTorch axis order)]) of an FP32/FP16 rwkv.cpp file."""
    with open(path, 'rb') as f:
        header = struct.unpack('=iiiiii', f.read(24))
        if header[0] != MAGIC:
            raise ValueError(f'Invalid magic value {header[0]:x}')
        if not 100 <= header[1] <= 101:
            raise ValueError(f'Invalid version number {header[1]}')
        tensors = []
        while True:
            h = f.read(12)
            if not h:
                break
            dims, klen, ftype = struct.unpack('=iii', h)
            shape = list(reversed(struct.unpack('=' + 'i' * dims, f.read(4 * dims))))
            key = f.read(klen).decode('utf-8')
            if ftype not in (0, 1):
                raise ValueError(f'{key}: only FP32 and FP16 tensors are supported (type {ftype})')
            dt = np.float16 if ftype == 1 else np.float32
            n = int(np.prod(shape)) if shape else 1
            tensors.append((key, np.frombuffer(f.read(n * np.dtype(dt).itemsize), dtype=dt).reshape(shape)))
    return header, tensors


# ------------------------------------------------------------------------------------ LoRA merge
def merge_lora(src_path: str, arch_version: str, lora_state_dict: Dict, lora_alpha: int, dest_path: str,
               log: Callable = print) -> List[str]:
    """Merge a LoRA checkpoint into an FP32/FP16 rwkv.cpp file.  arch_version: 'v4', 'v5.1',
    'v5.2', 'v6.0'.  Returns the LoRA keys left unused (the reference prints them as warnings).
    The reference's v6.0 replacement branch reads an undefined name (`k`); here it uses the key."""
    import torch
    versions = {'v4': '4', 'v5.1': '5.1', 'v5.2': '5.2', 'v6.0': '6.0'}
    if arch_version not in versions:
        raise ValueError(f'Invalid RWKV architecture version {arch_version}')
    version = versions[arch_version]
    lora = dict(lora_state_dict)
    header, tensors = read_model_file(src_path)
    if header[5] not in (0, 1):
        raise ValueError('Only FP32 and FP16 models are supported')
    with open(dest_path, 'wb') as out:
        out.write(struct.pack('=iiiiii', *header))
        for key, arr in tensors:
            p = torch.from_numpy(arr.copy())
            if key in lora:
                rep = lora.pop(key).float()
                # v6 per-head decay: the head count is the stored tensor's first axis
                rep = torch.from_numpy(transform(key, rep.numpy(), version, int(p.shape[0]) if p.dim() else 0))
                if p.dtype == torch.float16:
                    rep = rep.half()
                if tuple(rep.shape) != tuple(p.shape):
                    raise ValueError(f'Parameter {key} has shape {tuple(p.shape)} in model file '
                                     f'and shape {tuple(rep.shape)} in LoRA file')
                p = rep
                log(f'Replaced parameter {key}')
            for suffix in ('.weight', ''):
                ka = key.replace('.weight', '') + '.lora_A' + suffix
                kb = key.replace('.weight', '') + '.lora_B' + suffix
                if ka in lora:
                    a, b = lora.pop(ka), lora.pop(kb)
                    if b.shape[1] != a.shape[0]:
                        raise ValueError(f'Invalid shape of LoRA matrices for {key}: {tuple(a.shape)}, {tuple(b.shape)}')
                    r = b.shape[1]
                    merged = p + b @ a * (lora_alpha / r)
                    p = merged.half() if p.dtype == torch.float16 else merged
                    log(f'Merged LoRA into parameter {key}, lora_r = {r}')
                    break
            t = p.numpy()
            if t.dtype not in (np.float16, np.float32):
                raise ValueError(f'{key}: merged dtype {t.dtype}')
            out.write(tensor_record(key, t))
    for k in lora:
        log(f'WARNING: Unused parameter in LoRA state dict {k}')
    return list(lora)


def load_checkpoint(path: str) -> Dict:
    """A .pth state dict, loaded without executing anything from the file."""
    import torch
    return torch.load(path, map_location='cpu', weights_only=True)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description='Convert an RWKV PyTorch checkpoint to an rwkv.cpp model file')
    ap.add_argument('src_path')
    ap.add_argument('dest_path')
    ap.add_argument('data_type', choices=['FP16', 'FP32', 'float16', 'float32'], default='FP16')
    a = ap.parse_args(argv)
    write_state_dict(load_checkpoint(a.src_path), a.dest_path, a.data_type)


if __name__ == '__main__':
    main()
