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


# ---------------------------------------------------------------------------- .npz graph files
# user graphs arrive as `.npz` files.  Two layouts are read:
#   acsim's own      rowptr (uint64 [N+1]), colidx (uint32 [nnz])   (save_csr writes this)
#   scipy.sparse     indptr, indices, shape, format = "csr"          (scipy.sparse.save_npz of a CSR
#                    matrix whose row i lists receiver i's senders; `data` is ignored)
# Receiver i's senders are colidx[rowptr[i] : rowptr[i+1]] in slot order (slot = rowptr[i] + t,
# SURVEY §A.3).  Files are loaded with allow_pickle=False: a graph file executes nothing.

def save_csr(path: str, rowptr, colidx) -> None:
    """Write a CSR graph in acsim's `.npz` layout (validated first)."""
    rp, ci = check_csr(rowptr, colidx)
    np.savez(path, rowptr=rp, colidx=ci, format=np.array("acsim-csr-v1"))


def load_csr(path: str):
    """Read a CSR graph file (acsim or scipy.sparse layout) -> (rowptr uint64[N+1], colidx uint32[nnz])."""
    with np.load(path, allow_pickle=False) as z:
        keys = set(z.files)
        if {"rowptr", "colidx"} <= keys:
            rp, ci = z["rowptr"], z["colidx"]
        elif {"indptr", "indices"} <= keys:
            if "format" in keys and str(z["format"].astype(str)) != "csr":
                raise ValueError(f"{path}: scipy.sparse matrix in {z['format']!s} format; CSR expected")
            rp, ci = z["indptr"], z["indices"]
            if "shape" in keys:
                shape = tuple(int(v) for v in z["shape"])
                if shape[0] != shape[1] or shape[0] != rp.size - 1:
                    raise ValueError(f"{path}: adjacency must be N x N with N = len(indptr) - 1, got {shape}")
        else:
            raise ValueError(f"{path}: no CSR arrays (rowptr/colidx or indptr/indices) in {sorted(keys)}")
    return check_csr(rp, ci)


def check_csr(rowptr, colidx):
    """The ACS_TOPO_CSR admission rules that need no config (acs_create_csr re-checks them and the
    per-config m_i > 2t rule): rowptr[0] = 0, non-decreasing, rowptr[N] = nnz, sender ids < N."""
    rp = np.asarray(rowptr)
    ci = np.asarray(colidx)
    if rp.ndim != 1 or rp.size < 2 or ci.ndim != 1:
        raise ValueError("rowptr must be 1-D with N + 1 >= 2 entries, colidx 1-D")
    if not (np.issubdtype(rp.dtype, np.integer) and np.issubdtype(ci.dtype, np.integer)):
        raise ValueError("rowptr and colidx must be integer arrays")
    if rp[0] != 0 or np.any(np.diff(rp.astype(np.int64)) < 0) or int(rp[-1]) != ci.size:
        raise ValueError("rowptr must start at 0, be non-decreasing and end at len(colidx)")
    n = rp.size - 1
    if ci.size and (int(ci.min()) < 0 or int(ci.max()) >= n):
        raise ValueError(f"sender ids must lie in [0, {n})")
    if n >= 1 << 31:
        raise ValueError("at most 2^31 - 1 nodes")
    return rp.astype(np.uint64), ci.astype(np.uint32)
