"""Layer pipeline for sequence evaluation across the GPUs of one node.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).  Stage s owns the
contiguous layers stage_layers(n_layer, world, s) and its slice of the recurrent state; stage 0
embeds the tokens, the last stage runs the head.  A sequence is cut into chunks along T; each
chunk's residual stream x [T_chunk, C] (plus, for v7, the layer-0 values v_first, rwkv_graph.inc
:440-453) is the only message, sent point-to-point to the next stage over xGMI.  Stages work on
different chunks at the same time; chunk c reaches layer l only after chunk c-1 left it (every
stage handles its chunks in order), which is the order the recurrence needs, so the results are
bit-identical to one rwkv_eval_sequence over the whole sequence (chunking along T is exact in
this library: tests/test_gpu_parity.py).

The per-stage computation is injected (`stage_fn`), so the same driver runs the library
(LibraryStage, GPU) and, in the CPU tests, the oracle.
"""
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def stage_layers(n_layer: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced layer range [l0, l1) of stage `rank` (earlier stages get the extra
    layers: the last stage also runs the head)."""
    if not 0 <= rank < world or world > n_layer:
        raise ValueError(f'cannot split {n_layer} layers over {world} stages')
    base, extra = divmod(n_layer, world)
    l0 = rank * base + min(rank, extra)
    return l0, l0 + base + (1 if rank < extra else 0)


# stage_fn(tokens, l0, l1, x, want_logits) -> logits or None.  x: float32 tensor [planes, T, C]
# (planes = 2 for v7: x and v_first) holding the stream entering l0 (ignored when l0 == 0) and,
# on return, the stream leaving l1 - 1.
StageFn = Callable[[np.ndarray, int, int, torch.Tensor, bool], Optional[np.ndarray]]


def pipeline_eval_sequence(stage_fn: StageFn, tokens: Sequence[int], chunk: int, n_layer: int, n_embed: int,
                           planes: int, rank: int, world: int, device: torch.device,
                           wire_device: Optional[torch.device] = None, group=None,
                           want_logits: bool = True) -> Optional[np.ndarray]:
    """Runs this rank's stage over every chunk of `tokens`; returns the logits of the last token on
    the last stage (None elsewhere).  wire_device: where messages live for the backend (the GPU for
    nccl, the CPU for gloo); defaults to `device`."""
    if chunk <= 0 or len(tokens) == 0:
        raise ValueError('empty sequence or chunk size 0')
    wire = wire_device or device
    toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint32))
    bounds = [(i, min(i + chunk, len(toks))) for i in range(0, len(toks), chunk)]
    l0, l1 = stage_layers(n_layer, world, rank)
    prev, nxt = rank - 1, rank + 1

    def post_recv(c: int):
        a, b = bounds[c]
        buf = torch.empty((planes, b - a, n_embed), dtype=torch.float32, device=wire)
        return dist.irecv(buf, src=prev, group=group), buf

    pending = post_recv(0) if rank > 0 else None
    sends: List = []
    logits = None
    for c, (a, b) in enumerate(bounds):
        if rank > 0:
            work, buf = pending
            work.wait()
            if wire.type == 'cuda':
                torch.cuda.current_stream(wire).synchronize()  # the stage runs on its own stream
            pending = post_recv(c + 1) if c + 1 < len(bounds) else None
            x = buf if buf.device == device else buf.to(device)
        else:
            x = torch.empty((planes, b - a, n_embed), dtype=torch.float32, device=device)
        last = c == len(bounds) - 1
        lg = stage_fn(toks[a:b], l0, l1, x, want_logits and last and rank == world - 1)
        if last and rank == world - 1:
            logits = lg
        if rank < world - 1:
            out = x if x.device == wire else x.to(wire)
            sends.append((dist.isend(out, dst=nxt, group=group), out))  # keep `out` alive until sent
    for work, _ in sends:
        work.wait()
    return logits


class LibraryStage:
    """stage_fn over librwkv.so's rwkv_mi355x_eval_layers on this process's GPU.  The context keeps
    its stage's state slice resident in HBM across calls (reset with reset_state)."""

    def __init__(self, library, ctx, n_vocab: int, arch_major: int):
        self.lib = library
        self.ctx = ctx
        self.n_vocab = n_vocab
        self.v7 = arch_major == 7
        self.planes = 2 if self.v7 else 1

    def reset_state(self, state: Optional[np.ndarray] = None) -> None:
        ptr = None if state is None else state.ctypes.data
        if not self.lib.library.rwkv_mi355x_state_upload(self.ctx.ptr, ptr):
            raise ValueError('state upload failed')

    def __call__(self, tokens: np.ndarray, l0: int, l1: int, x: torch.Tensor, want_logits: bool):
        import ctypes
        if x.device.type != 'cuda' or not x.is_contiguous():
            raise ValueError('stage buffers must be contiguous device tensors')
        logits = np.zeros(self.n_vocab, np.float32) if want_logits else None
        xp = x.data_ptr()
        vp = x[1].data_ptr() if self.v7 else None
        lg = logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None
        ok = self.lib.library.rwkv_mi355x_eval_layers(self.ctx.ptr, tokens.ctypes.data, len(tokens), l0, l1, xp, vp,
                                                      want_logits, lg)
        if not ok:
            raise ValueError(f'rwkv_mi355x_eval_layers failed on layers [{l0}, {l1})')
        return logits
