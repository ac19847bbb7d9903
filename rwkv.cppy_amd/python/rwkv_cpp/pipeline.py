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
import contextlib
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


def _run_chunks(stage_fn, toks, bounds, l0, l1, post_recv, planes, n_embed, rank, world, device, wire, group,
                want_logits, host_sync):
    nxt = rank + 1
    pending = post_recv(0) if rank > 0 else None
    sends: List = []
    logits = None
    for c, (a, b) in enumerate(bounds):
        if rank > 0:
            work, buf = pending
            work.wait()
            if host_sync and wire.type == 'cuda':
                torch.cuda.current_stream(wire).synchronize()  # a synchronous stage runs on its own stream
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
    prev = rank - 1

    def post_recv(c: int):
        a, b = bounds[c]
        buf = torch.empty((planes, b - a, n_embed), dtype=torch.float32, device=wire)
        return dist.irecv(buf, src=prev, group=group), buf

    # an asynchronous stage (LibraryStage(async_=True)) computes on its own HIP stream: make it
    # current so the receive, the compute and the send of each chunk are stream-ordered with no
    # host wait; a synchronous stage returns with its output complete
    stream = getattr(stage_fn, 'stream', None)
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        logits = _run_chunks(stage_fn, toks, bounds, l0, l1, post_recv, planes, n_embed, rank, world, device, wire,
                             group, want_logits, host_sync=stream is None)
        if stream is not None:
            stream.synchronize()
    return logits


def layer_state_len(n_embed: int, arch_major: int, head_size: int) -> int:
    """Floats of one layer's state in the host layout (rwkv_graph.inc:545-606): v4 five [C] vectors,
    v5+ token shifts [2][C] plus the heads' [H][S][S] wkv state.  For a library context use
    LibraryStage.layer_len (rwkv_mi355x_layer_state_len), the layout the library actually uses."""
    return 5 * n_embed if arch_major == 4 else n_embed * (2 + head_size)


def scatter_state(full: Optional[np.ndarray], n_layer: int, layer_len: int, rank: int, world: int,
                  group=None, wire_device: Optional[torch.device] = None) -> Optional[np.ndarray]:
    """Rank 0 holds a whole host state (None: fresh states everywhere, nothing is sent); every rank
    returns only its stage's slice, layers stage_layers(n_layer, world, rank) -- rank r receives
    (l1 - l0) * layer_len floats and nothing else.  Returns None for a fresh state."""
    wire = wire_device or torch.device('cpu')
    fresh = torch.tensor([1 if full is None else 0], dtype=torch.int32, device=wire)
    dist.broadcast(fresh, src=0, group=group)
    if int(fresh.item()):
        return None
    l0, l1 = stage_layers(n_layer, world, rank)
    if rank == 0:
        if full.size != n_layer * layer_len:
            raise ValueError(f'state has {full.size} floats, expected {n_layer * layer_len}')
        sends = []
        for r in range(1, world):
            a, b = stage_layers(n_layer, world, r)
            t = torch.from_numpy(np.ascontiguousarray(full[a * layer_len:b * layer_len])).to(wire)
            sends.append((dist.isend(t, dst=r, group=group), t))
        for w, _ in sends:
            w.wait()
        return np.ascontiguousarray(full[l0 * layer_len:l1 * layer_len])
    buf = torch.empty((l1 - l0) * layer_len, dtype=torch.float32, device=wire)
    dist.recv(buf, src=0, group=group)
    return buf.cpu().numpy()


def gather_state(part: np.ndarray, n_layer: int, layer_len: int, rank: int, world: int, group=None,
                 wire_device: Optional[torch.device] = None) -> Optional[np.ndarray]:
    """Inverse of scatter_state: every rank sends its stage's slice to rank 0, which returns the
    whole state (None elsewhere)."""
    wire = wire_device or torch.device('cpu')
    l0, l1 = stage_layers(n_layer, world, rank)
    if part.size != (l1 - l0) * layer_len:
        raise ValueError(f'rank {rank}: slice has {part.size} floats, expected {(l1 - l0) * layer_len}')
    if rank != 0:
        dist.send(torch.from_numpy(np.ascontiguousarray(part, dtype=np.float32)).to(wire), dst=0, group=group)
        return None
    full = np.empty(n_layer * layer_len, np.float32)
    full[l0 * layer_len:l1 * layer_len] = part
    for r in range(1, world):
        a, b = stage_layers(n_layer, world, r)
        buf = torch.empty((b - a) * layer_len, dtype=torch.float32, device=wire)
        dist.recv(buf, src=r, group=group)
        full[a * layer_len:b * layer_len] = buf.cpu().numpy()
    return full


def model_n_layer(path: str) -> int:
    """n_layer from an rwkv.cpp file header (docs/FILE_FORMAT.md: magic, version, n_vocab, n_embed,
    n_layer, data_type as uint32)."""
    hdr = np.fromfile(path, dtype=np.uint32, count=6)
    if hdr.size != 6 or hdr[0] != 0x67676d66:
        raise ValueError(f'{path}: not an rwkv.cpp model file')
    return int(hdr[4])


class LibraryStage:
    """stage_fn over librwkv.so's rwkv_mi355x_eval_layers on this process's GPU.  The context keeps
    its stage's state slice resident in HBM across calls (reset with reset_state).

    async_=True enqueues each stage call on the context's HIP stream without a host wait
    (rwkv_mi355x_eval_layers_async); `stream` is that stream as a torch ExternalStream, which
    pipeline_eval_sequence makes current so the RCCL send of a chunk is ordered behind its compute
    and the next chunk's compute overlaps the send."""

    def __init__(self, library, ctx, n_vocab: int, arch_major: int, async_: bool = False):
        self.lib = library
        self.ctx = ctx
        self.n_vocab = n_vocab
        self.v7 = arch_major == 7
        self.planes = 2 if self.v7 else 1
        self.async_ = async_
        self.stream = None
        if async_:
            self.stream = torch.cuda.ExternalStream(int(library.library.rwkv_mi355x_stream(ctx.ptr)))

    @classmethod
    def from_file(cls, library, path: str, rank: int, world: int, async_: bool = False):
        """The stage context of `rank`: only its layers' weights are uploaded
        (rwkv_mi355x_init_from_file_layers), so a stage's HBM holds ~1/world of the model."""
        import ctypes
        from .rwkv_cpp_shared_library import RWKVContext
        n_layer = model_n_layer(path)
        l0, l1 = stage_layers(n_layer, world, rank)
        ptr = library.library.rwkv_mi355x_init_from_file_layers(path.encode(), 1, l0, l1)
        if not ptr:
            raise ValueError(f'failed to load layers [{l0}, {l1}) of {path}')
        ctx = RWKVContext(ptr)
        arch = (ctypes.c_int64 * 4)()
        library.library.rwkv_mi355x_arch(ctx.ptr, arch)
        return cls(library, ctx, library.library.rwkv_get_n_vocab(ctx.ptr), int(arch[0]), async_=async_)

    @property
    def layer_len(self) -> int:
        """Floats of one layer's state slice, from the library (Engine::layer_state_len)."""
        return int(self.lib.library.rwkv_mi355x_layer_state_len(self.ctx.ptr))

    def reset_state(self, state: Optional[np.ndarray] = None) -> None:
        ptr = None if state is None else state.ctypes.data
        if not self.lib.library.rwkv_mi355x_state_upload(self.ctx.ptr, ptr):
            raise ValueError('state upload failed')

    def layer_range(self, world: int, rank: int) -> Tuple[int, int]:
        return stage_layers(self.lib.library.rwkv_get_n_layer(self.ctx.ptr), world, rank)

    def upload_state_slice(self, part: Optional[np.ndarray], l0: int, l1: int) -> None:
        """Only layers [l0, l1) of the state cross PCIe (part = those layers, host layout; None =
        fresh), rwkv_mi355x_state_upload_layers."""
        if part is not None:
            part = np.ascontiguousarray(part, dtype=np.float32)
            n = (l1 - l0) * self.layer_len
            if part.size != n:
                raise ValueError(f'slice has {part.size} floats, expected {n}')
        ok = self.lib.library.rwkv_mi355x_state_upload_layers(self.ctx.ptr, None if part is None else part.ctypes.data,
                                                             l0, l1)
        if not ok:
            raise ValueError(f'state upload of layers [{l0}, {l1}) failed')

    def download_state_slice(self, l0: int, l1: int) -> np.ndarray:
        n = (l1 - l0) * self.layer_len
        out = np.empty(n, np.float32)
        if not self.lib.library.rwkv_mi355x_state_download_layers(self.ctx.ptr, out.ctypes.data, l0, l1):
            raise ValueError(f'state download of layers [{l0}, {l1}) failed')
        return out

    def __call__(self, tokens: np.ndarray, l0: int, l1: int, x: torch.Tensor, want_logits: bool):
        import ctypes
        if x.device.type != 'cuda' or not x.is_contiguous():
            raise ValueError('stage buffers must be contiguous device tensors')
        xp = x.data_ptr()
        vp = x[1].data_ptr() if self.v7 else None
        if self.async_ and not want_logits:
            # enqueued on the context stream; the caller's RCCL ops on the same stream follow it
            ok = self.lib.library.rwkv_mi355x_eval_layers_async(self.ctx.ptr, tokens.ctypes.data, len(tokens), l0, l1,
                                                                xp, vp, False)
            if not ok:
                raise ValueError(f'rwkv_mi355x_eval_layers_async failed on layers [{l0}, {l1})')
            return None
        logits = np.zeros(self.n_vocab, np.float32) if want_logits else None
        lg = logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None
        ok = self.lib.library.rwkv_mi355x_eval_layers(self.ctx.ptr, tokens.ctypes.data, len(tokens), l0, l1, xp, vp,
                                                      want_logits, lg)
        if not ok:
            raise ValueError(f'rwkv_mi355x_eval_layers failed on layers [{l0}, {l1})')
        return logits
