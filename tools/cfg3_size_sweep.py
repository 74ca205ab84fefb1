"""cfg3 batched kernel time against the instance count (one GPU): separates the per-call fixed
cost and the last-generation tail from the per-instance work (DESIGN.md §6, cfg3 scaling).

usage: python tools/cfg3_size_sweep.py [--reps 5] [--sizes 2048,...] [--timing 0|1]
One JSON line per size: median kernel ms (HIP events; only with --timing 1), median run() wall ms
and acs_run's own clock, both with the kernel events off unless --timing 1.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sizes", default="1024,2048,4096,8192,12500,16384,25000,50000,100000")
    ap.add_argument("--timing", type=int, default=1)
    a = ap.parse_args()
    import acsim
    cfg = acsim.preset("cfg3")
    with acsim.Simulator(cfg.replace(n_instances=256), device=0) as w:
        w.run()
    for B in (int(v) for v in a.sizes.split(",")):
        ks, ws, cs = [], [], []
        for _ in range(a.reps):
            sim = acsim.Simulator(cfg.replace(n_instances=B), device=0)
            if a.timing:
                sim.set_kernel_timing(True)
            sim.sync()
            t0 = time.perf_counter()
            res = sim.run()
            dt = time.perf_counter() - t0
            if a.timing:
                ks.append(sim.kernel_timing()[0])
            ws.append(dt * 1e3)
            cs.append(res.wall_seconds * 1e3)
            sim.close()
        print(json.dumps({"instances": B, "kernel_ms": statistics.median(ks) if ks else None,
                          "wall_ms": statistics.median(ws), "c_wall_ms": statistics.median(cs),
                          "timing": a.timing}), flush=True)


if __name__ == "__main__":
    main()
