"""Result digests used to check sharded / partitioned runs against the committed golden hashes
(tests/golden/fullsize.json) without moving the values themselves.

sha256_values(x)          sha256 of the value bytes (little-endian, the config dtype)
instance_digests(x)       [B, 32] uint8: sha256 of every instance row of x[B, N]
combine_digests(d)        sha256 over instance digests concatenated in global instance order
instances_digest(x)       combine_digests(instance_digests(x)): a checksum of checksums, so a run
                          sharded over any number of ranks reproduces it from the per-rank digests
"""
from __future__ import annotations

import hashlib

import numpy as np


def sha256_values(x: np.ndarray) -> str:
    x = np.ascontiguousarray(x)
    return hashlib.sha256(x.astype(x.dtype.newbyteorder("<"), copy=False).tobytes()).hexdigest()


def instance_digests(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x)
    if x.ndim == 1:
        x = x[None, :]
    out = np.empty((x.shape[0], 32), dtype=np.uint8)
    for b in range(x.shape[0]):
        out[b] = np.frombuffer(hashlib.sha256(x[b].tobytes()).digest(), dtype=np.uint8)
    return out


def combine_digests(d: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(d, dtype=np.uint8).tobytes()).hexdigest()


def instances_digest(x: np.ndarray) -> str:
    return combine_digests(instance_digests(x))
