"""Seeded parameter stream shared by the golden generator and the tests.

The goldens do not store parameter values: both sides regenerate them from
``(seed, parameter index)`` with numpy's PCG64 stream, and the fixture stores a
checksum (``pcheck.<name>`` = [sum, sum|.|]) so a drift in the stream fails loudly.

Scales are chosen so that candidate scores spread by O(1) (the reference init spreads
them by ~1e-4, SURVEY.md §7 "Hard parts").
"""
import numpy as np


def param_std(name, shape):
    if "bert_word_embedding" in name:
        return 0.5
    if "userEmbedding" in name:
        return 0.3
    if "query" in name:
        return 1.0
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return 1.5 / np.sqrt(fan_in)
    return 0.1


def regen_params(names_shapes, seed):
    """names_shapes: ordered [(name, shape)] -> {name: float32 array}."""
    out = {}
    for i, (name, shape) in enumerate(names_shapes):
        rng = np.random.default_rng([int(seed), i])
        z = rng.standard_normal(shape, dtype=np.float32)
        if "layerNorm.weight" in name or "LayerNorm.weight" in name:
            v = 1.0 + 0.1 * z
        else:
            v = z * np.float32(param_std(name, shape))
        if "userEmbedding" in name:
            v[0] = 0.0          # RNN.py:82 zero-initialises the "unknown user" row
        out[name] = v.astype(np.float32)
    return out
