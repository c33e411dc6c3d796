"""Deterministic parameter / input generation shared by the golden capture script
and the tests, so fixtures need not store weights: a tensor is a pure function of
(seed, name, shape).  numpy's PCG64 stream is platform independent."""
import zlib

import numpy as np


def _rng(seed, name):
    return np.random.default_rng([int(seed), zlib.crc32(name.encode())])


def param_value(name, shape, seed=0):
    shape = tuple(int(s) for s in shape)
    r = _rng(seed, name)
    if name.endswith("action_query"):
        return r.standard_normal(shape)
    if len(shape) == 1:
        if name.endswith("weight"):           # every 1-D weight in FACT is a LayerNorm gain
            return 1.0 + 0.1 * r.standard_normal(shape)
        return 0.1 * r.standard_normal(shape)
    fan_in = int(np.prod(shape[1:]))
    return r.standard_normal(shape) / np.sqrt(fan_in)


def fill_state(named_shapes, seed=0):
    """named_shapes: iterable of (name, shape) -> dict name -> float64 ndarray."""
    return {n: param_value(n, s, seed) for n, s in named_shapes}


def randn(name, shape, seed=0, scale=1.0):
    return scale * _rng(seed, name).standard_normal(tuple(shape))


def text_embeddings(n, dim=512, seed=0):
    e = randn("text_embeddings", (n, dim), seed)
    return e / np.linalg.norm(e, axis=1, keepdims=True)


def segmented_video(T, D, classes, nseg, seed=0, noise=0.1):
    """Piecewise-constant features (one prototype per segment) + noise, with labels.
    Boundaries are sorted distinct cut points; label of segment i = classes[(7i+3) % len]."""
    r = _rng(seed, "video")
    cuts = np.sort(r.permutation(np.arange(1, T))[: nseg - 1])
    bounds = np.concatenate([[0], cuts, [T]])
    feats = np.empty((T, D))
    label = np.empty(T, dtype=np.int64)
    for i in range(nseg):
        s, e = bounds[i], bounds[i + 1]
        feats[s:e] = r.standard_normal(D)
        label[s:e] = classes[(7 * i + 3) % len(classes)]
    feats += noise * r.standard_normal((T, D))
    return feats, label


def sample_index(n, k=2048, seed=0):
    """Fixed sample of flat indices used to store large gradients compactly."""
    if n <= k:
        return np.arange(n)
    return np.sort(np.random.default_rng([seed, n]).choice(n, size=k, replace=False))
