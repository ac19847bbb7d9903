"""Decode replicas across the GPUs of one node from ONE process (SURVEY.md §8e "replicas only" for
decode, §8 F4 multi-context serving).

The reference serves parallel streams by cloning a context (rwkv_clone_context, rwkv.h:93-99,
rwkv.cpp:123-139): the clones share the model and each keeps its own state.  Here a clone can be
placed on another GPU (rwkv_mi355x_clone_context_on); the model is uploaded once per GPU and every
context on that GPU shares it.  Each replica evaluates its own sequences on its own GPU; the calls
release the GIL (ctypes), so one host thread per replica keeps every GPU busy.

The product path is librwkv.so; this module only places contexts and deals sequences to them.
"""
import ctypes
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .rwkv_cpp_shared_library import RWKVContext, RWKVSharedLibrary

P_FLOAT = ctypes.POINTER(ctypes.c_float)


class ReplicaPool:
    """One context per listed GPU over the model `ctx` was loaded from (the parent context stays
    the caller's; replica i is a clone on devices[i])."""

    def __init__(self, library: RWKVSharedLibrary, ctx: RWKVContext, devices: Sequence[int]):
        self.lib = library
        self.parent = ctx
        self.replicas: List[RWKVContext] = []
        try:
            for d in devices:
                self.replicas.append(library.rwkv_mi355x_clone_context_on(ctx, 1, int(d)))
        except Exception:
            self.free()
            raise
        L = library.library
        self.n_vocab = L.rwkv_get_n_vocab(ctx.ptr)
        self.state_len = L.rwkv_get_state_len(ctx.ptr)

    def devices(self) -> List[int]:
        return [self.lib.library.rwkv_mi355x_context_device(c.ptr) for c in self.replicas]

    def _run(self, i: int, tokens: Sequence[int], state_in: Optional[np.ndarray], out: list, slot: int) -> None:
        L = self.lib.library
        c = self.replicas[i]
        toks = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint32))
        state = np.empty(self.state_len, np.float32)
        logits = np.empty(self.n_vocab, np.float32)
        sin = None if state_in is None else np.ascontiguousarray(state_in, dtype=np.float32)
        ok = L.rwkv_eval_sequence(c.ptr, toks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(toks),
                                  None if sin is None else sin.ctypes.data_as(P_FLOAT), state.ctypes.data_as(P_FLOAT),
                                  logits.ctypes.data_as(P_FLOAT))
        out[slot] = (logits, state) if ok else RuntimeError(f'replica {i} (GPU {L.rwkv_mi355x_context_device(c.ptr)}) failed')

    def eval_sequences(self, sequences: Sequence[Sequence[int]],
                       states: Optional[Sequence[Optional[np.ndarray]]] = None) -> List[Tuple[np.ndarray, np.ndarray]]:
        """Evaluates independent sequences (rwkv_eval_sequence each, from states[k] or a fresh
        state), sequence k on replica k % len(replicas); replicas run concurrently, the sequences
        of one replica in order.  Returns (logits of the last token, state) per sequence."""
        n = len(self.replicas)
        out: list = [None] * len(sequences)

        def worker(i: int) -> None:
            for k in range(i, len(sequences), n):
                self._run(i, sequences[k], None if states is None else states[k], out, k)

        threads = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        for r in out:
            if isinstance(r, Exception):
                raise r
        return out

    def free(self) -> None:
        for c in self.replicas:
            if c.ptr:
                self.lib.rwkv_free(c)
        self.replicas = []
