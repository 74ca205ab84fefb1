"""Result file format (SURVEY §8(f) row 3, §5 checkpoint/resume): one ``.npz`` per run.

Arrays: ``rounds`` (u32 [B]), ``converged`` (bool [B]), ``spread`` (f64 [B]), ``x_final``
(f64 [N] or [B, N], optional), ``spread_trace`` (f64 [R+1], optional), ``node_rounds``,
``wall_seconds``; ``config`` is the Config as a JSON string.  Written and read without pickle
(``np.load(allow_pickle=False)``), so a result file never executes anything on load.  A file
with ``x_final`` is also a resume point: ``resume_from(path)`` rebuilds a Simulator at that round.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Any, Dict

import numpy as np

from .config import Config


def config_to_json(cfg: Config) -> str:
    return json.dumps(dataclasses.asdict(cfg), sort_keys=True)


def config_from_json(s: str) -> Config:
    return Config(**json.loads(s))


def save_result(path: str, result, cfg: Config) -> None:
    arrays: Dict[str, Any] = {
        "rounds": np.asarray(result.rounds, dtype=np.uint32),
        "converged": np.asarray(result.converged, dtype=bool),
        "spread": np.asarray(result.spread, dtype=np.float64),
        "node_rounds": np.asarray(int(result.node_rounds), dtype=np.int64),
        "wall_seconds": np.asarray(float(result.wall_seconds), dtype=np.float64),
        "config": np.asarray(config_to_json(cfg)),
        "format": np.asarray("acsim-result-v1"),
    }
    if getattr(result, "x_final", None) is not None:
        arrays["x_final"] = np.asarray(result.x_final, dtype=np.float64)
    if getattr(result, "spread_trace", None) is not None:
        arrays["spread_trace"] = np.asarray(result.spread_trace, dtype=np.float64)
    np.savez(path, **arrays)


def load_result(path: str) -> Dict[str, Any]:
    with np.load(path, allow_pickle=False) as z:
        if str(z["format"]) != "acsim-result-v1":
            raise ValueError(f"{path}: not an acsim result file")
        out = {k: z[k] for k in z.files if k not in ("config", "format")}
        out["config"] = config_from_json(str(z["config"]))
    out["node_rounds"] = int(out["node_rounds"])
    out["wall_seconds"] = float(out["wall_seconds"])
    return out


def resume_from(path: str, device: int = 0, **overrides):
    """A Simulator positioned at the saved round with the saved values (§A.9 resume is exact)."""
    from .sim import Simulator
    r = load_result(path)
    if "x_final" not in r:
        raise ValueError(f"{path} has no x_final; cannot resume")
    cfg = r["config"].replace(**overrides)
    rounds = np.asarray(r["rounds"])
    if rounds.size and not np.all(rounds == rounds[0]):
        raise ValueError("instances stopped at different rounds; resume needs a common round")
    sim = Simulator(cfg, device=device)
    sim.set_state(int(rounds[0]) if rounds.size else 0, np.asarray(r["x_final"]).reshape(-1))
    return sim
