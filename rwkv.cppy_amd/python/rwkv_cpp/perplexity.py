"""Perplexity of a model over a token sequence through the rwkv_eval ABI: the reference's
python/measure_pexplexity.py:73-109 loop (serial rwkv_eval, the cross-entropy of each next token,
perplexity = exp(mean loss)).

    python -m rwkv_cpp.perplexity model.bin text.txt ignore_first_n [token_limit] --vocab vocab.txt
"""
import argparse
import math
import time
from typing import List, Tuple

import numpy as np


def cross_entropy(logits: np.ndarray, target: int) -> float:
    """-log softmax(logits)[target] in float64 (torch.nn.functional.cross_entropy's value)."""
    x = np.asarray(logits, dtype=np.float64)
    m = x.max()
    return float(m + math.log(np.exp(x - m).sum()) - x[target])


def measure(model, tokens: List[int], ignore_first_n: int = 0) -> Tuple[float, float, int]:
    """(mean loss, perplexity, tokens scored) over tokens[1:], skipping the first ignore_first_n."""
    if len(tokens) - ignore_first_n <= 1:
        raise ValueError('Need at least 2 tokens for evaluation')
    logits, state = None, None
    loss_sum, count = 0.0, 0
    for i in range(len(tokens) - 1):
        logits, state = model.eval(tokens[i], state, state, logits, use_numpy=True)
        if ignore_first_n == 0 or i + 1 >= ignore_first_n:
            loss_sum += cross_entropy(logits, tokens[i + 1])
            count += 1
    mean = loss_sum / count
    return mean, math.exp(mean), count


def main(argv=None) -> None:
    from . import RWKVModel, load_rwkv_shared_library
    from .world_tokenizer import get_world_tokenizer
    ap = argparse.ArgumentParser(description='Perplexity of an RWKV model on a UTF-8 text file')
    ap.add_argument('model_path')
    ap.add_argument('text_path')
    ap.add_argument('ignore_first_n_tokens', type=int)
    ap.add_argument('token_limit', nargs='?', type=int, default=-1)
    ap.add_argument('--vocab', default=None, help='World tokenizer vocabulary file (or RWKV_WORLD_VOCAB)')
    a = ap.parse_args(argv)
    model = RWKVModel(load_rwkv_shared_library(), a.model_path)
    _, encode = get_world_tokenizer(a.vocab)
    tokens = encode(open(a.text_path, encoding='utf-8').read())
    if a.token_limit > 0:
        tokens = tokens[:a.token_limit]
    t0 = time.time()
    loss, ppl, n = measure(model, tokens, a.ignore_first_n_tokens)
    dt = time.time() - t0
    print(f'{len(tokens)} tokens, {n} scored: loss {loss:.3f}, perplexity {ppl:.3f}, '
          f'latency {dt * 1000 / (len(tokens) - 1):.2f} ms per token')


if __name__ == '__main__':
    main()
