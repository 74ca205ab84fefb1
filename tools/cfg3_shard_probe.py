"""cfg3 strong-scaling probe on one GPU: the per-rank shard of the 10^5-instance batch at
world sizes 1, 2, 4, 8 (shard_range), timed as bench.py's cfg3_sharded leg times it (wall time of
run() between two syncs, and up to run()'s return without the closing sync) beside the kernel's
own HIP-event time.  --no-events: without kernel events (the bench leg's `single` figure).  The gap is the fixed cost per
rank that bounds the 1 -> 8 GPU scaling of the batched-instance config.

usage: python tools/cfg3_shard_probe.py [--reps 3]   (one JSON line per shard size)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--preset", default="cfg3")
    ap.add_argument("--no-events", action="store_true")
    a = ap.parse_args()
    import acsim
    from acsim.distributed import shard_range
    cfg = acsim.preset(a.preset)
    with acsim.Simulator(cfg.replace(n_instances=256), device=0) as w:
        w.run()
    for world in (1, 2, 4, 8):
        off, cnt = shard_range(cfg.n_instances, world, 0)
        local = cfg.replace(n_instances=cnt, instance_offset=off)
        for rep in range(a.reps):
            t_create = time.perf_counter()
            sim = acsim.Simulator(local, device=0)
            t_create = time.perf_counter() - t_create
            sim.set_kernel_timing(not a.no_events)
            sim.sync()
            t0 = time.perf_counter()
            res = sim.run()
            t_ret = time.perf_counter() - t0   # run() returns once the mapped summary has landed
            sim.sync()
            dt = time.perf_counter() - t0
            k_ms, k_n, kname = sim.kernel_timing()
            nr = int(res.node_rounds)
            sim.close()
            print(json.dumps({"world": world, "instances": cnt, "rep": rep, "wall_ms": dt * 1e3, "run_return_ms": t_ret * 1e3,
                              "kernel_ms": k_ms, "c_wall_ms": res.wall_seconds * 1e3,
                              "create_ms": t_create * 1e3, "node_rounds": nr,
                              "rounds_max": int(res.rounds_max), "kernel": kname}), flush=True)


if __name__ == "__main__":
    main()
