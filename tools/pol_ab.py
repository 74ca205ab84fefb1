"""A/B of binned-exchange cache policies (ACSIM_BIN_POL) inside ONE library build, alternating, so
code layout and box drift do not bias the comparison.

usage: python tools/pol_ab.py <preset> <rounds> <pol,pol,...> [reps]
One JSON line per (rep, pol): wall ms per round over `rounds` timed FIXED rounds after 2 warm-up
rounds, and the HIP-event time of the round kernels (every round bracketed).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402


def main():
    preset, rounds, pols = sys.argv[1], int(sys.argv[2]), [int(v, 0) for v in sys.argv[3].split(",")]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    # "<preset>_f32": the preset in fp32 mode; pol 0x10000 = the library's default policy
    base, f32 = (preset[:-4], True) if preset.endswith("_f32") else (preset, False)
    cfg = acsim.preset(base, max_rounds=rounds + 2, **({"dtype": "f32"} if f32 else {}))
    for rep in range(reps):
        for pol in pols:
            if pol == 0x10000:
                os.environ.pop("ACSIM_BIN_POL", None)
            else:
                os.environ["ACSIM_BIN_POL"] = str(pol)
            with acsim.Simulator(cfg) as s:
                s.round(2)
                s.set_kernel_timing(True, every=1)
                s.sync()
                t0 = time.perf_counter()
                s.round(rounds)
                s.sync()
                dt = time.perf_counter() - t0
                k_ms, k_n, kname = s.kernel_timing()
            print(json.dumps({"preset": preset, "pol": pol, "rep": rep, "rounds": rounds,
                              "wall_ms_per_round": dt / rounds * 1e3,
                              "kernel_ms_per_round": k_ms / max(1, k_n), "kernel": kname}), flush=True)


if __name__ == "__main__":
    main()
