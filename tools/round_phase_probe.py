"""Per-chunk round time of cfg4 across a run, to tell a warm-up effect from a data effect
(the driver's rounds 5-25 run 3-4 % slower than later ones).

usage: python tools/round_phase_probe.py [chunk] [chunks]
One handle, max_rounds large enough for three legs of `chunks` chunks of `chunk` FIXED rounds:
  leg "fresh":  from x^0 right after the handle is built (the driver's shape: its rounds 5-25);
  leg "reset":  x set back to x^0 (acs_set_state) on the same, now warm, handle;
  leg "const":  every x_i set to one value (consensus reached: the values stop changing).
One JSON line per chunk: wall and HIP-event kernel ms per round.  If "reset" repeats "fresh"'s
early slowness the cause is the data; if it does not, it is the handle's or the GPU's warm-up.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402


def leg(s, name, chunk, chunks, r0):
    for c in range(chunks):
        s.set_kernel_timing(True, every=chunk, runs=True)
        s.sync()
        t0 = time.perf_counter()
        s.round(chunk)
        s.sync()
        dt = time.perf_counter() - t0
        k_ms, k_n, _ = s.kernel_timing()
        s.set_kernel_timing(False)
        print(json.dumps({"leg": name, "chunk": c, "first_round": r0 + c * chunk, "rounds": chunk,
                          "wall_us_per_round": dt / chunk * 1e6,
                          "kernel_us_per_round": k_ms * 1e3 / max(1, k_n)}), flush=True)
    return r0 + chunks * chunk


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    chunks = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfg = acsim.preset("cfg4", max_rounds=3 * chunk * chunks + 10)
    with acsim.Simulator(cfg) as s:
        x0 = s.values(0).copy()
        r = leg(s, "fresh", chunk, chunks, 0)
        s.set_state(r, x0)
        r = leg(s, "reset", chunk, chunks, r)
        s.set_state(r, np.full_like(x0, 0.375))
        leg(s, "const", chunk, chunks, r)


if __name__ == "__main__":
    main()
