"""Deterministic synthetic inputs (counter-based splitmix64), identical on every
machine and numpy version — used by bench.py, the tests and the golden-vector
script so large tables never need to be stored.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF)
        return splitmix64(base + np.arange(n, dtype=np.uint64))


def uniform(seed: int, shape, lo: float, hi: float) -> np.ndarray:
    """float32 uniform in [lo, hi) from 24 random bits per element."""
    n = int(np.prod(shape))
    u = (_stream(seed, n) >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def randint(seed: int, shape, high: int) -> np.ndarray:
    n = int(np.prod(shape))
    return (_stream(seed, n) % np.uint64(high)).astype(np.int64).reshape(shape)


def kge_tables(seed: int, nentity: int, nrelation: int, entity_dim: int, relation_dim: int, embedding_range: float):
    """Entity / relation tables ~ U(-range, range) like model.py:45-57's init."""
    ent = uniform(seed * 2 + 1, (nentity, entity_dim), -embedding_range, embedding_range)
    rel = uniform(seed * 2 + 2, (nrelation, relation_dim), -embedding_range, embedding_range)
    return ent, rel


def kge_batch(seed: int, batch: int, nneg: int, nentity: int, nrelation: int):
    """(positive [B,3] int64, negative [B,n] int64, subsampling weight [B] f32 in [0.1, 0.4))."""
    h = randint(seed * 4 + 1, (batch,), nentity)
    r = randint(seed * 4 + 2, (batch,), nrelation)
    t = randint(seed * 4 + 3, (batch,), nentity)
    pos = np.stack([h, r, t], 1)
    neg = randint(seed * 4 + 4, (batch, nneg), nentity)
    w = uniform(seed * 4 + 5, (batch,), 0.1, 0.4)
    return pos, neg, w
