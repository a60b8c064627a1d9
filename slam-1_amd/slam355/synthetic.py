"""Seeded synthetic inputs (no datasets are reachable): descriptor sets, stereo
image sequences and BA problems of the BASELINE.json config shapes.
See SURVEY.md §8d for the definitions."""
from __future__ import annotations

import numpy as np


def descriptor_set(rng, nq, nt, frac_planted=0.6, flip_p=0.08):
    """Nt uniform random 32-byte rows; Nq rows of which `frac_planted` are
    copies of random train rows with each bit flipped w.p. flip_p (d ~ 20)."""
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    if nt:
        pick = rng.random(nq) < frac_planted
        src = rng.integers(0, nt, nq)
        bits = np.unpackbits(t[src], axis=1) ^ (rng.random((nq, 256)) < flip_p).astype(np.uint8)
        q[pick] = np.packbits(bits, axis=1)[pick]
    return q, t


def descriptor_batch(B, nq, nt, seed=0):
    rng = np.random.default_rng(seed)
    q = np.empty((B, nq, 32), np.uint8)
    t = np.empty((B, nt, 32), np.uint8)
    for b in range(B):
        q[b], t[b] = descriptor_set(rng, nq, nt)
    return q, np.full(B, nq, np.int32), t, np.full(B, nt, np.int32)
