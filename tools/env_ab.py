"""A/B of plan switches (ACSIM_* environment variables) inside ONE library build, alternating, so
code layout and box drift do not bias the comparison.

usage: python tools/env_ab.py <preset> <rounds> <reps> "<variant>;<variant>;..."
A variant is a comma-separated list NAME=VALUE, or "-" for the library defaults.  One JSON line per
(rep, variant): wall ms per round over `rounds` timed FIXED rounds after 2 warm-up rounds, and the
HIP-event time of the round kernels over runs of 25 consecutive rounds (bench.py's bracket).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402


def parse(variant):
    if variant.strip() in ("", "-"):
        return {}
    return dict(kv.split("=", 1) for kv in variant.split(","))


def main():
    preset, rounds, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    variants = [parse(v) for v in sys.argv[4].split(";")]
    names = sorted({k for v in variants for k in v})
    base, f32 = (preset[:-4], True) if preset.endswith("_f32") else (preset, False)
    cfg = acsim.preset(base, max_rounds=rounds + 2, **({"dtype": "f32"} if f32 else {}))
    for rep in range(reps):
        for v in variants:
            for k in names:
                os.environ.pop(k, None)
            os.environ.update(v)
            with acsim.Simulator(cfg) as s:
                s.round(2)
                s.set_kernel_timing(True, every=25, runs=True)
                s.sync()
                t0 = time.perf_counter()
                s.round(rounds)
                s.sync()
                dt = time.perf_counter() - t0
                k_ms, k_n, kname = s.kernel_timing()
            print(json.dumps({"preset": preset, "env": v, "rep": rep, "rounds": rounds,
                              "wall_ms_per_round": dt / rounds * 1e3,
                              "kernel_ms_per_round": k_ms / max(1, k_n), "kernel": kname}), flush=True)
    for k in names:
        os.environ.pop(k, None)


if __name__ == "__main__":
    main()
