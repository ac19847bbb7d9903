"""RWKVModel over librwkv.so (MI355X build).

Same constructor, properties, eval / eval_sequence / eval_sequence_in_chunks / free
methods, buffer validation and return convention as the reference's
python/rwkv_cpp/rwkv_cpp_model.py:22-364: buffers are float32, contiguous, on the CPU,
shape (state_len,) / (n_vocab,); missing outputs are allocated (numpy or torch, by the
type of the inputs given); returns (logits, state).
"""
import multiprocessing
import os
from typing import List, Optional, Tuple, Any

try:
    from . import rwkv_cpp_shared_library
except ImportError:  # imported as a top-level module
    import rwkv_cpp_shared_library

Tensor = Any  # numpy.ndarray or torch.Tensor


def _is_torch(t) -> bool:
    return type(t).__module__.startswith('torch')


class RWKVModel:
    def __init__(self, shared_library: 'rwkv_cpp_shared_library.RWKVSharedLibrary', model_path: str,
                 thread_count: int = max(1, multiprocessing.cpu_count() // 2), gpu_layer_count: int = 0,
                 **kwargs) -> None:
        if 'gpu_layers_count' in kwargs:
            gpu_layer_count = kwargs['gpu_layers_count']
        if not os.path.isfile(model_path):
            raise ValueError(f'{model_path} is not a file')
        if not thread_count > 0:
            raise ValueError('Thread count must be > 0')
        if not gpu_layer_count >= 0:
            raise ValueError('GPU layer count must be >= 0')
        self._library = shared_library
        self._ctx = self._library.rwkv_init_from_file(model_path, thread_count, gpu_layer_count)
        self._state_buffer_element_count = self._library.rwkv_get_state_buffer_element_count(self._ctx)
        self._logits_buffer_element_count = self._library.rwkv_get_logits_buffer_element_count(self._ctx)
        self._valid = True

    @property
    def n_vocab(self) -> int:
        return self._library.rwkv_get_n_vocab(self._ctx)

    @property
    def n_embed(self) -> int:
        return self._library.rwkv_get_n_embed(self._ctx)

    @property
    def n_layer(self) -> int:
        return self._library.rwkv_get_n_layer(self._ctx)

    # ---- buffer handling --------------------------------------------------------------
    def _prepare(self, state_in, state_out, logits_out, use_numpy):
        if not self._valid:
            raise ValueError('Model was freed')
        for t in (state_in, state_out, logits_out):
            if t is not None:
                use_numpy = not _is_torch(t)
                break
        if state_in is not None:
            self._validate(state_in, 'state_in', self._state_buffer_element_count)
            state_in_ptr = self._ptr(state_in)
        else:
            state_in_ptr = 0
        if state_out is not None:
            self._validate(state_out, 'state_out', self._state_buffer_element_count)
        else:
            state_out = self._zeros(self._state_buffer_element_count, use_numpy)
        if logits_out is not None:
            self._validate(logits_out, 'logits_out', self._logits_buffer_element_count)
        else:
            logits_out = self._zeros(self._logits_buffer_element_count, use_numpy)
        return state_in_ptr, state_out, logits_out

    @staticmethod
    def _validate(t, name: str, size: int) -> None:
        if _is_torch(t):
            import torch
            if t.device != torch.device('cpu'):
                raise ValueError(f'{name} is not on CPU')
            if t.dtype != torch.float32:
                raise ValueError(f'{name} is not of type float32')
            if tuple(t.shape) != (size,):
                raise ValueError(f'{name} has invalid shape {tuple(t.shape)}, expected ({size})')
            if not t.is_contiguous():
                raise ValueError(f'{name} is not contiguous')
        else:
            import numpy as np
            if t.dtype != np.float32:
                raise ValueError(f'{name} is not of type float32')
            if t.shape != (size,):
                raise ValueError(f'{name} has invalid shape {t.shape}, expected ({size})')
            if not t.flags['C_CONTIGUOUS']:
                raise ValueError(f'{name} is not contiguous')

    @staticmethod
    def _ptr(t) -> int:
        return t.data_ptr() if _is_torch(t) else t.ctypes.data

    @staticmethod
    def _zeros(n: int, use_numpy: bool):
        if use_numpy:
            import numpy as np
            return np.zeros(n, dtype=np.float32)
        import torch
        return torch.zeros(n, dtype=torch.float32, device='cpu')

    # ---- evaluation -------------------------------------------------------------------
    def eval(self, token: int, state_in: Optional[Tensor], state_out: Optional[Tensor] = None,
             logits_out: Optional[Tensor] = None, use_numpy: bool = False) -> Tuple[Tensor, Tensor]:
        sin, state_out, logits_out = self._prepare(state_in, state_out, logits_out, use_numpy)
        self._library.rwkv_eval(self._ctx, token, sin, self._ptr(state_out), self._ptr(logits_out))
        return logits_out, state_out

    def eval_sequence(self, tokens: List[int], state_in: Optional[Tensor], state_out: Optional[Tensor] = None,
                      logits_out: Optional[Tensor] = None, use_numpy: bool = False) -> Tuple[Tensor, Tensor]:
        sin, state_out, logits_out = self._prepare(state_in, state_out, logits_out, use_numpy)
        self._library.rwkv_eval_sequence(self._ctx, tokens, sin, self._ptr(state_out), self._ptr(logits_out))
        return logits_out, state_out

    def eval_sequence_in_chunks(self, tokens: List[int], state_in: Optional[Tensor], state_out: Optional[Tensor] = None,
                                logits_out: Optional[Tensor] = None, chunk_size: int = 16,
                                use_numpy: bool = False) -> Tuple[Tensor, Tensor]:
        sin, state_out, logits_out = self._prepare(state_in, state_out, logits_out, use_numpy)
        self._library.rwkv_eval_sequence_in_chunks(self._ctx, tokens, chunk_size, sin, self._ptr(state_out),
                                                   self._ptr(logits_out))
        return logits_out, state_out

    def eval_batch(self, tokens: List[int], states_in=None):
        """MI355X extension (rwkv_mi355x_eval_batch): len(tokens) independent contexts advance one token
        each in one pass over the weights.  states_in: float32 [n, state_len] numpy array, or None for
        fresh states.  Returns (logits [n, n_vocab], states [n, state_len]); row i equals
        eval(tokens[i], states_in[i]) bit for bit."""
        import numpy as np
        if not self._valid:
            raise ValueError('Model was freed')
        n = len(tokens)
        if states_in is not None:
            states_in = np.ascontiguousarray(states_in, dtype=np.float32)
            if states_in.shape != (n, self._state_buffer_element_count):
                raise ValueError(f'states_in must be [{n}, {self._state_buffer_element_count}]')
        states = np.zeros((n, self._state_buffer_element_count), np.float32)
        logits = np.zeros((n, self._logits_buffer_element_count), np.float32)
        self._library.rwkv_mi355x_eval_batch(self._ctx, list(tokens), None if states_in is None else states_in.ctypes.data,
                                             states.ctypes.data, logits.ctypes.data)
        return logits, states

    def free(self) -> None:
        if not self._valid:
            raise ValueError('Already freed')
        self._valid = False
        self._library.rwkv_free(self._ctx)

    def __del__(self) -> None:
        if getattr(self, '_valid', False):
            self.free()
