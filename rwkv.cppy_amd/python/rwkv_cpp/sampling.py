"""Token sampling over the logits rwkv_eval returns: the semantics of the reference's
python/sampling.py:6-52 (softmax, logit bias, greedy at temperature 0, top-p cutoff, temperature),
numpy only.  rng: an optional numpy Generator (the reference draws from np.random's global state)."""
from typing import Dict, Optional

import numpy as np


def softmax(x: np.ndarray, axis: int = -1) -> np.ndarray:
    x = x - x.max(axis=axis, keepdims=True)
    e = np.exp(x)
    return e / e.sum(axis=axis, keepdims=True)


def sample_logits(out, temperature: float = 1.0, top_p: float = 0.8, logit_bias: Optional[Dict[int, float]] = None,
                  rng: Optional[np.random.Generator] = None) -> int:
    if hasattr(out, 'detach'):
        out = out.detach().cpu().numpy()
    return sample_probs(softmax(np.asarray(out, dtype=np.float32), axis=-1), temperature, top_p, logit_bias, rng)


def sample_probs(probs: np.ndarray, temperature: float = 1.0, top_p: float = 0.8,
                 logit_bias: Optional[Dict[int, float]] = None, rng: Optional[np.random.Generator] = None) -> int:
    if not 0.0 <= temperature:
        raise ValueError('temperature')
    if not 0.0 <= top_p <= 1.0:
        raise ValueError('top_p')
    probs = np.array(probs, copy=True)
    if top_p == 0.0:
        top_p = 1.0
    if logit_bias:
        logits = np.log(probs)
        ids, values = zip(*logit_bias.items())
        logits[list(ids)] += values
        logits -= logits.max(axis=-1, keepdims=True)
        probs = np.exp(logits) / np.sum(np.exp(logits))
    if temperature == 0.0:
        return int(np.argmax(probs))
    if top_p < 1.0:
        sorted_probs = np.sort(probs)[::-1]
        cumulative = np.cumsum(sorted_probs)
        cutoff = float(sorted_probs[np.argmax(cumulative > top_p)])
        probs[probs < cutoff] = 0
    if temperature != 1.0:
        probs = np.power(probs, 1.0 / temperature)
    probs = probs / np.sum(probs)
    choice = rng.choice if rng is not None else np.random.choice
    return int(choice(a=len(probs), p=probs))
