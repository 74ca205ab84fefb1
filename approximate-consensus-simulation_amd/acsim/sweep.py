"""Parameter sweeps: run the cartesian product of config overrides, one
simulation handle at a time on one GPU, and summarise each run (rounds, convergence, rate).

    from acsim.sweep import sweep
    rows = sweep(preset("cfg3", n_instances=10000), {"loss_p": [0.1, 0.2, 0.3], "seed": [0, 1]})

For multi-GPU sweeps, give each rank its own slice of `points(grid)` (one process per GPU).
"""
from __future__ import annotations

import itertools
import json
import os
from typing import Callable, Dict, Iterable, List, Optional

import numpy as np

from .config import Config
from .io import save_result


def points(grid: Dict[str, Iterable]) -> List[Dict]:
    keys = list(grid)
    return [dict(zip(keys, vals)) for vals in itertools.product(*(list(grid[k]) for k in keys))]


def summarize(cfg: Config, res) -> Dict:
    rounds = np.asarray(res.rounds)
    return {
        "n_instances": int(rounds.size),
        "rounds_min": int(rounds.min()), "rounds_mean": float(rounds.mean()),
        "rounds_max": int(rounds.max()),
        "converged": int(np.asarray(res.converged).sum()),
        "final_spread_max": float(np.asarray(res.spread).max()),
        "node_rounds": int(res.node_rounds), "wall_seconds": float(res.wall_seconds),
        "node_rounds_per_s": float(res.node_rounds / res.wall_seconds) if res.wall_seconds > 0 else None,
    }


def sweep(base: Config, grid: Dict[str, Iterable], out_dir: Optional[str] = None, device: int = 0,
          run: Optional[Callable] = None, keep_values: bool = False, csr=None) -> List[Dict]:
    """run(cfg) -> Result (default: acsim.simulate on `device`; csr: a user graph for
    topology="csr" configs, shared by every point)."""
    if run is None:
        from .sim import simulate
        run = lambda c: simulate(c, device=device, return_values=keep_values or out_dir is not None,  # noqa: E731
                                 csr=csr)
    rows = []
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
    for k, over in enumerate(points(grid)):
        cfg = base.replace(**over)
        res = run(cfg)
        row = {"point": k, **over, **summarize(cfg, res)}
        if out_dir:
            path = os.path.join(out_dir, f"run_{k:04d}.npz")
            save_result(path, res, cfg)
            row["file"] = path
        rows.append(row)
    if out_dir:
        with open(os.path.join(out_dir, "summary.json"), "w") as f:
            json.dump(rows, f, indent=1)
    return rows
