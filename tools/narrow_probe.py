"""Narrow stage A/B: whole run() of cfg4-shaped workloads with the default plan and
with ACSIM_BIN_NARROW=1, alternating fresh handles inside one process, plus the rounds each run
took and a golden-free cross-check (the two plans' final values must be bit-identical).

usage: python tools/narrow_probe.py [reps]
One JSON line per run: workload, plan, rounds, wall µs per round of the whole run() (state on the
device), kernel name.  Workloads: cfg4 FIXED 100 rounds (the bench workload), the driver's shape
(FIXED 25 rounds: its timed rounds 5-25 sit inside), and cfg4 to ε = 1e-12 (EPS).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402

WORKLOADS = {
    "cfg4_fixed100": dict(max_rounds=100, termination="fixed"),
    "cfg4_fixed25": dict(max_rounds=25, termination="fixed"),
    "cfg4_eps1e-12": dict(max_rounds=200, termination="eps", eps=1e-12),
}


def one(name, narrow):
    if narrow:
        os.environ["ACSIM_BIN_NARROW"] = "1"
    else:
        os.environ.pop("ACSIM_BIN_NARROW", None)
    cfg = acsim.preset("cfg4", **WORKLOADS[name])
    with acsim.Simulator(cfg, device=0) as s:
        s.sync()
        t0 = time.perf_counter()
        s.run()
        s.sync()
        dt = time.perf_counter() - t0
        r = int(s.rounds()[0])
        x = s.values(0).copy()
        return {"workload": name, "plan": "narrow" if narrow else "default", "rounds": r,
                "us_per_round": dt / r * 1e6, "node_rounds_per_s": cfg.n_nodes * r / dt,
                "kernel": s.kernel_name()}, x


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for name in WORKLOADS:
        for rep in range(reps):
            xs = {}
            for narrow in ((False, True) if rep % 2 == 0 else (True, False)):
                rec, x = one(name, narrow)
                xs[narrow] = x
                rec["rep"] = rep
                print(json.dumps(rec), flush=True)
            assert np.array_equal(xs[False].view(np.uint64), xs[True].view(np.uint64)), name


if __name__ == "__main__":
    main()
