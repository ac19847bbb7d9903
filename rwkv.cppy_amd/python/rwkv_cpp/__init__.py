"""Python mirror of the reference's python/rwkv_cpp package for the MI355X librwkv.so.

Only the eval-path classes are provided (RWKVModel, RWKVSharedLibrary); the reference's
reservoir / ESN / tokenizer modules are callers of this path and out of scope.
"""
from .rwkv_cpp_model import RWKVModel
from .rwkv_cpp_shared_library import RWKVSharedLibrary, load_rwkv_shared_library

__all__ = ['RWKVModel', 'RWKVSharedLibrary', 'load_rwkv_shared_library']
