"""Synthetic user graphs in CSR form for the ACS_TOPO_CSR topology:
``(rowptr uint64[N+1], colidx uint32[nnz])`` as ``acsim.Simulator(cfg, csr=...)`` takes them.
Used by the CSR benchmarks and tests; any CSR the caller builds works the same way."""
from __future__ import annotations

import numpy as np


def random_csr(n: int, dmin: int, dmax: int, seed: int):
    """Uniform degrees in [dmin, dmax], uniformly random senders."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(dmin, dmax + 1, size=n)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
    colidx = rng.integers(0, n, size=int(rowptr[-1])).astype(np.uint32)
    return rowptr, colidx


def skewed_csr(n: int, dmin: int, dmax: int, seed: int, alpha: float = 2.0):
    """Power-law degrees in [dmin, dmax] (most rows near dmin, a tail up to dmax); senders half
    uniform, half from a hub set of n/100 nodes (skewed in-degree too)."""
    rng = np.random.default_rng(seed)
    u = rng.random(n)
    deg = np.floor(dmin * (1 - u * (1 - (dmin / (dmax + 1)) ** (alpha - 1))) ** (-1 / (alpha - 1))).astype(np.int64)
    deg = np.clip(deg, dmin, dmax)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
    nnz = int(rowptr[-1])
    hubs = rng.integers(0, n, size=max(1, n // 100))
    col = np.where(rng.random(nnz) < 0.5, rng.integers(0, n, size=nnz), hubs[rng.integers(0, hubs.size, size=nnz)])
    return rowptr, col.astype(np.uint32)
