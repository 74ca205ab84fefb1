"""Round time against position in the process: does the first handle's first rounds run slower
(clock ramp, first-touch of fresh allocations) than later ones?  Diagnostic for the driver's short
bench run (`--steps 20 --warmup 5`).

usage: python tools/ramp_probe.py [handles] [chunks] [chunk_rounds]
One JSON line per (handle, chunk): the HIP-event device time per round over `chunk_rounds`
consecutive rounds, and the wall time of the chunk.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402


def main():
    handles = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    cr = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    t_proc = time.perf_counter()
    for h in range(handles):
        t0 = time.perf_counter()
        cfg = acsim.preset("cfg4", max_rounds=chunks * cr)
        with acsim.Simulator(cfg) as s:
            s.sync()
            t_create = time.perf_counter() - t0
            for c in range(chunks):
                s.set_kernel_timing(True, every=cr, runs=True)
                s.sync()
                t1 = time.perf_counter()
                s.round(cr)
                s.sync()
                wall = time.perf_counter() - t1
                k_ms, k_n, _ = s.kernel_timing()
                print(json.dumps({"handle": h, "chunk": c, "first_round": c * cr, "create_s": t_create,
                                  "since_process_start_s": time.perf_counter() - t_proc,
                                  "kernel_us_per_round": k_ms / max(1, k_n) * 1e3,
                                  "wall_us_per_round": wall / cr * 1e6}), flush=True)


if __name__ == "__main__":
    main()
