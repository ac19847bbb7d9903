"""RWKV World tokenizer (vocabulary rwkv_vocab_v20230424): greedy longest byte match, the
semantics of the reference's python/rwkv_cpp/rwkv_world_tokenizer.py:55-113.

The vocabulary file has one token per line: ``<id> <python literal of the token (str or bytes)>
<byte length>``.  Literals are parsed with ast.literal_eval (the reference eval()s them).
Encoding walks a byte trie from each position and takes the longest token that matches;
decoding joins the tokens' bytes (invalid UTF-8 becomes U+FFFD, as in the reference).
The vocabulary is not shipped here: pass its path, or set RWKV_WORLD_VOCAB.
"""
import ast
import os
from typing import Callable, Dict, List, Tuple


class WorldTokenizer:
    def __init__(self, vocab_path: str) -> None:
        self.index_to_token: Dict[int, bytes] = {}
        with open(vocab_path, 'r', encoding='utf-8') as f:
            for line in f:
                if not line.strip():
                    continue
                a, b = line.index(' '), line.rindex(' ')
                tok = ast.literal_eval(line[a:b].strip())
                tok = tok.encode('utf-8') if isinstance(tok, str) else tok
                if not isinstance(tok, bytes) or len(tok) != int(line[b:]):
                    raise ValueError(f'bad vocabulary line: {line!r}')
                self.index_to_token[int(line[:a])] = tok
        # byte trie: node = dict byte -> child; the token id of a node under key -1
        self.root: Dict = {}
        for idx, tok in self.index_to_token.items():
            node = self.root
            for ch in tok:
                node = node.setdefault(ch, {})
            node[-1] = idx

    def encode_bytes(self, src: bytes) -> List[int]:
        out: List[int] = []
        i, n = 0, len(src)
        while i < n:
            node, j, best, best_end = self.root, i, None, i
            while j < n and src[j] in node:
                node = node[src[j]]
                j += 1
                if -1 in node:
                    best, best_end = node[-1], j
            if best is None:
                raise ValueError(f'no token matches the bytes at offset {i}')
            out.append(best)
            i = best_end
        return out

    def decode_bytes(self, tokens: List[int]) -> bytes:
        return b''.join(self.index_to_token[t] for t in tokens)

    def encode(self, text: str) -> List[int]:
        return self.encode_bytes(text.encode('utf-8'))

    def decode(self, tokens: List[int]) -> str:
        return self.decode_bytes(tokens).decode('utf-8', errors='replace')


def get_world_tokenizer(vocab_path: str = None) -> Tuple[Callable[[List[int]], str], Callable[[str], List[int]]]:
    """(decode, encode) of the World v20230424 tokenizer (rwkv_world_tokenizer.py:116-125)."""
    path = vocab_path or os.environ.get('RWKV_WORLD_VOCAB')
    if not path:
        raise ValueError('World tokenizer vocabulary: pass vocab_path or set RWKV_WORLD_VOCAB')
    t = WorldTokenizer(path)
    return t.decode, t.encode
