"""Python mirror of the reference's python/rwkv_cpp package for the MI355X librwkv.so.

The eval-path classes (RWKVModel, RWKVSharedLibrary) and the harness around them (SURVEY.md 8
rows F2/F3): world_tokenizer, sampling, perplexity, convert (PyTorch -> rwkv.cpp, LoRA merge) and
pipeline (multi-GPU sequence evaluation).  The reference's reservoir / ESN modules are out of
scope.
"""
from .rwkv_cpp_model import RWKVModel
from .rwkv_cpp_shared_library import RWKVSharedLibrary, load_rwkv_shared_library

__all__ = ['RWKVModel', 'RWKVSharedLibrary', 'load_rwkv_shared_library']
