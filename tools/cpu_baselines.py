"""CPU baseline per preset: the oracle (oracle/acs_oracle.c, -O2, OpenMP over
receivers) timed on the host cores on a bounded sample of each workload, 1 thread and T threads.
Prints one JSON line per (config, threads).  usage: python tools/cpu_baselines.py [T] [seconds]

Test/measurement infrastructure: the oracle is the CPU restatement of the spec, never the product.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import acsim  # noqa: E402
import oracle as O  # noqa: E402

CASES = ["cfg1", "cfg1_avg", "cfg2", "cfg3", "cfg4", "cfg5"]


def time_case(name, threads, seconds):
    kw = dict(omp_threads=threads)
    if name in ("cfg4", "cfg5"):
        kw["max_rounds"] = 100000
    if name == "cfg3":
        kw["n_instances"] = 2000 if threads == 1 else 10000   # bounded sample of the 1e5 instances
    cfg = acsim.preset(name, **kw)
    t0 = time.perf_counter()
    o = O.OracleSimulator(cfg, threads=threads)
    setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    if name in ("cfg4", "cfg5"):   # FIXED-round workloads: as many rounds as fit the budget
        o.round(1)
        one = time.perf_counter() - t0
        k = int(max(1, min(1000, seconds / max(one, 1e-6)))) - 1
        if k > 0:
            o.round(k)
        rounds_done = k + 1
        node_rounds = cfg.n_nodes * rounds_done
    else:                           # ε-terminated workloads: run to convergence
        res = o.run()
        node_rounds = int(res.node_rounds)
        rounds_done = int(res.rounds_max)
    dt = time.perf_counter() - t0
    o.close()
    return {"config": name, "threads": threads, "n_nodes": cfg.n_nodes, "n_instances": cfg.n_instances,
            "rounds": rounds_done, "node_rounds": node_rounds, "seconds": dt, "setup_s": setup,
            "node_rounds_per_s": node_rounds / dt}


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    names = sys.argv[3:] or CASES
    for name in names:
        for th in ((T,) if name == "cfg5" else (1, T)):   # cfg5's 1-thread graph build alone takes minutes
            print(json.dumps(time_case(name, th, seconds)), flush=True)


if __name__ == "__main__":
    main()
