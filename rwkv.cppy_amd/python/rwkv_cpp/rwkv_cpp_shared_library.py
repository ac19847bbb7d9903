"""ctypes binding of librwkv.so (the MI355X build).

Mirrors the reference's python/rwkv_cpp/rwkv_cpp_shared_library.py interface
(RWKVSharedLibrary, RWKVContext, load_rwkv_shared_library) -- same method names,
argument meaning and error behaviour (ValueError on failure) -- so callers written
against the reference run unchanged.  Argument types match the reference bindings
(rwkv_cpp_shared_library.py:49-107): tokens are passed as int32 (same bits as uint32).
The additive rwkv_mi355x_* entry points (include/rwkv_mi355x.h) are bound too.
"""
import ctypes
import os
import pathlib
import sys
from typing import Tuple, List, Optional

QUANTIZED_FORMAT_NAMES = ('Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0')

P_FLOAT = ctypes.POINTER(ctypes.c_float)
P_INT = ctypes.POINTER(ctypes.c_int32)


class RWKVContext:
    def __init__(self, ptr):
        self.ptr = ptr


class RWKVSharedLibrary:
    """Python wrapper around librwkv.so."""

    def __init__(self, shared_library_path: str) -> None:
        self.library = ctypes.cdll.LoadLibrary(shared_library_path)
        L = self.library
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32

        L.rwkv_init_from_file.argtypes = [ctypes.c_char_p, u32, u32]
        L.rwkv_init_from_file.restype = vp
        L.rwkv_clone_context.argtypes = [vp, u32]
        L.rwkv_clone_context.restype = vp
        L.rwkv_eval.argtypes = [vp, ctypes.c_int32, P_FLOAT, P_FLOAT, P_FLOAT]
        L.rwkv_eval.restype = ctypes.c_bool
        L.rwkv_eval_sequence.argtypes = [vp, P_INT, sz, P_FLOAT, P_FLOAT, P_FLOAT]
        L.rwkv_eval_sequence.restype = ctypes.c_bool
        L.rwkv_eval_sequence_in_chunks.argtypes = [vp, P_INT, sz, sz, P_FLOAT, P_FLOAT, P_FLOAT]
        L.rwkv_eval_sequence_in_chunks.restype = ctypes.c_bool
        for name in ('rwkv_get_n_vocab', 'rwkv_get_n_embed', 'rwkv_get_n_layer', 'rwkv_get_state_len',
                     'rwkv_get_logits_len'):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = sz
        L.rwkv_get_state_buffer_element_count.argtypes = [vp]
        L.rwkv_get_state_buffer_element_count.restype = u32
        L.rwkv_get_logits_buffer_element_count.argtypes = [vp]
        L.rwkv_get_logits_buffer_element_count.restype = u32
        L.rwkv_init_state.argtypes = [vp, P_FLOAT]
        L.rwkv_init_state.restype = None
        L.rwkv_free.argtypes = [vp]
        L.rwkv_free.restype = None
        L.rwkv_quantize_model_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.rwkv_quantize_model_file.restype = ctypes.c_bool
        L.rwkv_get_system_info_string.argtypes = []
        L.rwkv_get_system_info_string.restype = ctypes.c_char_p
        L.rwkv_set_print_errors.argtypes = [vp, ctypes.c_bool]
        L.rwkv_set_print_errors.restype = None
        L.rwkv_get_print_errors.argtypes = [vp]
        L.rwkv_get_print_errors.restype = ctypes.c_bool
        L.rwkv_get_last_error.argtypes = [vp]
        L.rwkv_get_last_error.restype = ctypes.c_int

        # additive MI355X extensions
        L.rwkv_mi355x_state_upload.argtypes = [vp, P_FLOAT]
        L.rwkv_mi355x_state_upload.restype = ctypes.c_bool
        L.rwkv_mi355x_state_download.argtypes = [vp, P_FLOAT]
        L.rwkv_mi355x_state_download.restype = ctypes.c_bool
        L.rwkv_mi355x_eval_device.argtypes = [vp, P_INT, sz, ctypes.c_bool, P_FLOAT, ctypes.c_bool]
        L.rwkv_mi355x_eval_device.restype = ctypes.c_bool
        L.rwkv_mi355x_eval_layers.argtypes = [vp, vp, sz, u32, u32, vp, vp, ctypes.c_bool, P_FLOAT]
        L.rwkv_mi355x_eval_layers.restype = ctypes.c_bool
        L.rwkv_mi355x_eval_layers_async.argtypes = [vp, vp, sz, u32, u32, vp, vp, ctypes.c_bool]
        L.rwkv_mi355x_eval_layers_async.restype = ctypes.c_bool
        L.rwkv_mi355x_logits_device.argtypes = [vp]
        L.rwkv_mi355x_logits_device.restype = vp
        L.rwkv_mi355x_init_from_file_layers.argtypes = [ctypes.c_char_p, u32, u32, u32]
        L.rwkv_mi355x_init_from_file_layers.restype = vp
        L.rwkv_mi355x_debug_buffer.argtypes = [vp, ctypes.c_char_p, vp, sz]
        L.rwkv_mi355x_debug_buffer.restype = ctypes.c_longlong
        L.rwkv_mi355x_sync.argtypes = [vp]
        L.rwkv_mi355x_sync.restype = ctypes.c_bool
        L.rwkv_mi355x_stream.argtypes = [vp]
        L.rwkv_mi355x_stream.restype = vp
        L.rwkv_mi355x_device_state.argtypes = [vp]
        L.rwkv_mi355x_device_state.restype = vp
        L.rwkv_mi355x_decode_bytes.argtypes = [vp, ctypes.c_bool]
        L.rwkv_mi355x_decode_bytes.restype = ctypes.c_double
        L.rwkv_mi355x_weight_bytes.argtypes = [vp, ctypes.c_bool]
        L.rwkv_mi355x_weight_bytes.restype = ctypes.c_double
        L.rwkv_mi355x_matmul_flops_per_token.argtypes = [vp, ctypes.c_bool]
        L.rwkv_mi355x_matmul_flops_per_token.restype = ctypes.c_double
        L.rwkv_mi355x_arch.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
        L.rwkv_mi355x_arch.restype = None
        L.rwkv_mi355x_write_synthetic_model.argtypes = [ctypes.c_char_p, ctypes.c_int, u32, u32, u32, u32,
                                                        ctypes.c_char_p, ctypes.c_uint64]
        L.rwkv_mi355x_write_synthetic_model.restype = ctypes.c_bool
        L.rwkv_mi355x_eval_batch.argtypes = [vp, vp, sz, vp, vp, vp]
        L.rwkv_mi355x_eval_batch.restype = ctypes.c_bool
        L.rwkv_mi355x_eval_batch_device.argtypes = [vp, vp, sz, vp, vp, vp]
        L.rwkv_mi355x_eval_batch_device.restype = ctypes.c_bool
        L.rwkv_mi355x_set_kernel_timing.argtypes = [vp, ctypes.c_bool]
        L.rwkv_mi355x_set_kernel_timing.restype = None
        L.rwkv_mi355x_kernel_stats.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_longlong),
                                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_double)]
        L.rwkv_mi355x_kernel_stats.restype = ctypes.c_int
        L.rwkv_mi355x_layer_state_len.argtypes = [vp]
        L.rwkv_mi355x_layer_state_len.restype = sz
        L.rwkv_mi355x_state_upload_layers.argtypes = [vp, vp, u32, u32]
        L.rwkv_mi355x_state_upload_layers.restype = ctypes.c_bool
        L.rwkv_mi355x_state_download_layers.argtypes = [vp, vp, u32, u32]
        L.rwkv_mi355x_state_download_layers.restype = ctypes.c_bool
        L.rwkv_mi355x_state_io_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.rwkv_mi355x_state_io_bytes.restype = None
        L.rwkv_mi355x_clone_context_on.argtypes = [vp, u32, ctypes.c_int]
        L.rwkv_mi355x_clone_context_on.restype = vp
        L.rwkv_mi355x_context_device.argtypes = [vp]
        L.rwkv_mi355x_context_device.restype = ctypes.c_int
        L.rwkv_mi355x_init_pipeline.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.rwkv_mi355x_init_pipeline.restype = vp
        L.rwkv_mi355x_pipeline_stages.argtypes = [vp]
        L.rwkv_mi355x_pipeline_stages.restype = ctypes.c_int
        L.rwkv_mi355x_pipeline_peer_pairs.argtypes = [vp]
        L.rwkv_mi355x_pipeline_peer_pairs.restype = ctypes.c_int
        L.rwkv_mi355x_debug_set.argtypes = [vp, ctypes.c_char_p, ctypes.c_longlong]
        L.rwkv_mi355x_debug_set.restype = ctypes.c_bool

        self.nullptr = ctypes.cast(0, ctypes.c_void_p)

    # ---- reference interface ----------------------------------------------------------
    def rwkv_init_from_file(self, model_file_path: str, thread_count: int, offload_layers: int) -> RWKVContext:
        ptr = self.library.rwkv_init_from_file(model_file_path.encode('utf-8'), ctypes.c_uint32(thread_count),
                                               ctypes.c_uint32(offload_layers))
        if ptr is None:
            raise ValueError('rwkv_init_from_file failed, check stderr')
        return RWKVContext(ptr)

    def rwkv_eval(self, ctx: RWKVContext, token: int, state_in_address: Optional[int], state_out_address: int,
                  logits_out_address: int) -> None:
        if not self.library.rwkv_eval(ctx.ptr, ctypes.c_int32(token),
                                      ctypes.cast(0 if state_in_address is None else state_in_address, P_FLOAT),
                                      ctypes.cast(state_out_address, P_FLOAT),
                                      ctypes.cast(logits_out_address, P_FLOAT)):
            raise ValueError('rwkv_eval failed, check stderr')

    def rwkv_eval_sequence(self, ctx: RWKVContext, tokens: List[int], state_in_address: Optional[int],
                           state_out_address: int, logits_out_address: int) -> None:
        arr = (ctypes.c_int32 * len(tokens))(*tokens)
        if not self.library.rwkv_eval_sequence(ctx.ptr, ctypes.cast(arr, P_INT), ctypes.c_size_t(len(tokens)),
                                               ctypes.cast(0 if state_in_address is None else state_in_address, P_FLOAT),
                                               ctypes.cast(state_out_address, P_FLOAT),
                                               ctypes.cast(logits_out_address, P_FLOAT)):
            raise ValueError('rwkv_eval_sequence failed, check stderr')

    def rwkv_eval_sequence_in_chunks(self, ctx: RWKVContext, tokens: List[int], chunk_size: int,
                                     state_in_address: Optional[int], state_out_address: int,
                                     logits_out_address: int) -> None:
        arr = (ctypes.c_int32 * len(tokens))(*tokens)
        if not self.library.rwkv_eval_sequence_in_chunks(
                ctx.ptr, ctypes.cast(arr, P_INT), ctypes.c_size_t(len(tokens)), ctypes.c_size_t(chunk_size),
                ctypes.cast(0 if state_in_address is None else state_in_address, P_FLOAT),
                ctypes.cast(state_out_address, P_FLOAT), ctypes.cast(logits_out_address, P_FLOAT)):
            raise ValueError('rwkv_eval_sequence_in_chunks failed, check stderr')

    def rwkv_get_n_vocab(self, ctx: RWKVContext) -> int:
        return self.library.rwkv_get_n_vocab(ctx.ptr)

    def rwkv_get_n_embed(self, ctx: RWKVContext) -> int:
        return self.library.rwkv_get_n_embed(ctx.ptr)

    def rwkv_get_n_layer(self, ctx: RWKVContext) -> int:
        return self.library.rwkv_get_n_layer(ctx.ptr)

    def rwkv_get_state_buffer_element_count(self, ctx: RWKVContext) -> int:
        return self.library.rwkv_get_state_buffer_element_count(ctx.ptr)

    def rwkv_get_logits_buffer_element_count(self, ctx: RWKVContext) -> int:
        return self.library.rwkv_get_logits_buffer_element_count(ctx.ptr)

    def rwkv_free(self, ctx: RWKVContext) -> None:
        self.library.rwkv_free(ctx.ptr)
        ctx.ptr = self.nullptr

    def rwkv_quantize_model_file(self, model_file_path_in: str, model_file_path_out: str, format_name: str) -> None:
        if format_name not in QUANTIZED_FORMAT_NAMES:
            raise ValueError(f'Unknown format name {format_name}, use one of {QUANTIZED_FORMAT_NAMES}')
        if not self.library.rwkv_quantize_model_file(model_file_path_in.encode('utf-8'),
                                                     model_file_path_out.encode('utf-8'),
                                                     format_name.encode('utf-8')):
            raise ValueError('rwkv_quantize_model_file failed, check stderr')

    # ---- additive: batched decode (include/rwkv_mi355x.h) ------------------------------------
    def rwkv_mi355x_eval_batch(self, ctx: RWKVContext, tokens: List[int], state_in_address: Optional[int],
                               state_out_address: Optional[int], logits_out_address: Optional[int]) -> None:
        """len(tokens) contexts advance one token each; states [n][state_len], logits [n][n_vocab]
        (host addresses, None = fresh states / not returned).  Bit-identical to rwkv_eval per context."""
        arr = (ctypes.c_uint32 * len(tokens))(*tokens)
        if not self.library.rwkv_mi355x_eval_batch(ctx.ptr, ctypes.cast(arr, ctypes.c_void_p), len(tokens),
                                                   state_in_address, state_out_address, logits_out_address):
            raise ValueError('rwkv_mi355x_eval_batch failed, check stderr')

    # ---- additive: replicas on other GPUs and per-layer state slices ------------------------
    def rwkv_mi355x_clone_context_on(self, ctx: RWKVContext, thread_count: int, device: int) -> RWKVContext:
        """rwkv_clone_context onto GPU `device` (the model is uploaded once per GPU)."""
        ptr = self.library.rwkv_mi355x_clone_context_on(ctx.ptr, thread_count, device)
        if ptr is None:
            raise ValueError(f'rwkv_mi355x_clone_context_on(device={device}) failed, check stderr')
        return RWKVContext(ptr)

    def rwkv_mi355x_state_io_bytes(self, ctx: RWKVContext) -> Tuple[float, float]:
        """State bytes this context moved so far: (host->device, device->host)."""
        out = (ctypes.c_double * 2)()
        self.library.rwkv_mi355x_state_io_bytes(ctx.ptr, out)
        return out[0], out[1]

    def rwkv_get_system_info_string(self) -> str:
        return self.library.rwkv_get_system_info_string().decode('utf-8')


def load_rwkv_shared_library() -> RWKVSharedLibrary:
    """Finds librwkv.so: $RWKV_CPP_SHARED_LIBRARY, then <repo>/{bin,build,...}/librwkv.so
    relative to the working directory and to this file (reference search order,
    rwkv_cpp_shared_library.py:375-426), plus rwkv.cppy_amd/build/."""
    env = os.environ.get('RWKV_CPP_SHARED_LIBRARY')
    if env and os.path.isfile(env):
        return RWKVSharedLibrary(env)
    file_name = 'librwkv.so'
    children = [
        lambda p: p / 'bin' / 'Release' / file_name,
        lambda p: p / 'bin' / file_name,
        lambda p: p / 'build' / 'bin' / 'Release' / file_name,
        lambda p: p / 'build' / 'bin' / file_name,
        lambda p: p / 'build' / file_name,
        lambda p: p / file_name,
    ]
    here = pathlib.Path(os.path.abspath(__file__)).parent
    cwd = pathlib.Path(os.path.abspath(os.getcwd()))
    parents = [cwd.parent.parent, cwd.parent, cwd, here.parent.parent, here.parent.parent / 'rwkv.cppy_amd']
    for parent in parents:
        for child in children:
            full = child(parent)
            if os.path.isfile(full):
                return RWKVSharedLibrary(str(full))
    raise ValueError(f'Failed to find {file_name} automatically; '
                     f'you need to find the library and create RWKVSharedLibrary specifying the path to it')
