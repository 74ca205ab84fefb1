"""Golden hashes of the FULL-SIZE sharded configs (run: python tests/golden/make_golden_fullsize.py).

Written by the CPU oracle (oracle/acs_oracle.c, OpenMP over receivers; results do not depend on
the thread count) into tests/golden/fullsize.json.  The reference mount holds no code or vectors
(README.md:1), so these are spec-derived like golden.json; the oracle that makes them is pinned by
the Random123 KATs and by bit-for-bit agreement with the independent numpy restatement at reduced
sizes (make_golden.py) — and here again on a sample of cfg3's instances, which are independent.

What is hashed (the GPU tests and bench.py's multi-GPU legs recompute exactly these):
  cfg5  (N = 2^26, random 16-regular, trimmed t = 5, FIXED): sha256 of x after 3 and 10 rounds,
        the spread trace, the first values.
  cfg3  (10^5 instances x 64 nodes, p = 0.2, AVERAGE, eps = 1e-6): instances_digest = sha256 over
        the concatenated per-instance sha256(x_b) digests in global instance order (composable
        over any instance sharding: a checksum of checksums), and sha256 of the rounds array.
  cfg4  (N = 2^20, the bench workload): sha256 of x after 100 FIXED rounds in fp64 and in fp32 mode
        (DESIGN.md §9); cfg4_eps rounds + sha.

`python tests/golden/make_golden_fullsize.py cfg4` regenerates only the named sections and keeps
the others.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "approximate-consensus-simulation_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import oracle as O  # noqa: E402
import spec_np as S  # noqa: E402
from acsim.config import preset  # noqa: E402
from acsim.digest import instances_digest, sha256_values  # noqa: E402

THREADS = max(1, min(16, os.cpu_count() or 1))


def hexd(a) -> list:
    return [float(v).hex() for v in np.asarray(a, dtype=np.float64).ravel()]


def cfg5_golden() -> dict:
    cfg = preset("cfg5", max_rounds=10, trace_spread=True)
    t0 = time.time()
    out = {"config": "preset('cfg5', max_rounds=10)", "n_nodes": int(cfg.n_nodes)}
    with O.OracleSimulator(cfg, threads=THREADS) as o:
        print(f"cfg5 oracle built in {time.time() - t0:.1f} s", flush=True)
        x0 = o.values(0)
        out["x0_sha256"] = sha256_values(x0)
        for r_to in (3, 10):
            o.round(r_to - int(o.rounds()[0]))
            x = o.values(0)
            out[f"x{r_to}_sha256"] = sha256_values(x)
            out[f"x{r_to}_head"] = hexd(x[:8])
            out[f"x{r_to}_minmax"] = [float(x.min()).hex(), float(x.max()).hex()]
            print(f"cfg5 round {r_to}: {out[f'x{r_to}_sha256'][:16]} ({time.time() - t0:.1f} s)", flush=True)
        out["trace"] = hexd(o.spread_trace(0))
    return out


def cfg3_golden() -> dict:
    cfg = preset("cfg3")
    t0 = time.time()
    with O.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        x = o.all_values()
        rounds = o.rounds()
        conv = o.converged()
    print(f"cfg3 oracle: {time.time() - t0:.1f} s, rounds max {int(rounds.max())}", flush=True)
    # independent cross-check on a sample of instances (instances are independent; the numpy
    # restatement runs the sample with the same global instance ids)
    for off in (0, 54321, 99000):
        sub = cfg.replace(n_instances=1000, instance_offset=off)
        n = S.NpSim(sub)
        n.run()
        assert np.array_equal(n.rounds, rounds[off:off + 1000]), off
        assert np.array_equal(n.x.view(np.uint64), x[off:off + 1000].view(np.uint64)), off
    print("cfg3 numpy cross-check on 3 x 1000 instances: ok", flush=True)
    return {"config": "preset('cfg3')", "n_instances": int(cfg.n_instances),
            "instances_digest": instances_digest(x),
            "rounds_sha256": hashlib.sha256(rounds.astype("<u4").tobytes()).hexdigest(),
            "rounds_hist": np.bincount(rounds.astype(np.int64)).tolist(),
            "n_converged": int(conv.sum()),
            "node_rounds": int(cfg.n_nodes) * int(rounds.astype(np.int64).sum())}


def cfg4_golden() -> dict:
    out = {}
    cfg = preset("cfg4", max_rounds=100)
    with O.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        out["fixed100_x_sha256"] = sha256_values(o.values(0))
    cfg = preset("cfg4", max_rounds=100, dtype="f32")
    with O.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        out["f32_fixed100_x_sha256"] = sha256_values(o.values(0))
    cfg = preset("cfg4_eps")
    with O.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        out["eps_rounds"] = int(o.rounds()[0])
        out["eps_x_sha256"] = sha256_values(o.values(0))
    return out


def main() -> None:
    O.build()
    path = os.path.join(HERE, "fullsize.json")
    makers = {"cfg3": cfg3_golden, "cfg4": cfg4_golden, "cfg5": cfg5_golden}
    names = sys.argv[1:] or list(makers)
    out = json.load(open(path)) if sys.argv[1:] and os.path.exists(path) else {}
    out["generator"] = "tests/golden/make_golden_fullsize.py (oracle/acs_oracle.c)"
    for nm in names:
        out[nm] = makers[nm]()
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
