"""Fixed host-side cost of a timed `round(k)` region on cfg4 (bench.py's bracket: sync, t0,
round(k), sync): wall time for k = 1 ... 40 after convergence, fitted as a + b k; plus a bare
sync.   usage: python tools/fixed_cost_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ks = (1, 2, 5, 10, 20, 40)
    cfg = acsim.preset("cfg4", max_rounds=200 + reps * sum(ks) + 10)
    with acsim.Simulator(cfg) as s:
        s.round(200)   # past the data-dependent slow rounds
        s.sync()
        bare = []
        for _ in range(20):
            t0 = time.perf_counter()
            s.sync()
            bare.append(time.perf_counter() - t0)
        pts = []
        for _ in range(reps):
            for k in ks:
                s.sync()
                t0 = time.perf_counter()
                s.round(k)
                s.sync()
                pts.append((k, time.perf_counter() - t0))
    k = np.array([p[0] for p in pts], dtype=float)
    t = np.array([p[1] for p in pts]) * 1e6
    b, a = np.polyfit(k, t, 1)
    print(json.dumps({"fixed_us": a, "per_round_us": b, "bare_sync_us_median": float(np.median(bare)) * 1e6,
                      "points_us": {int(kk): float(np.median(t[k == kk])) for kk in ks}}))


if __name__ == "__main__":
    main()
