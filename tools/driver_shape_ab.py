"""A/B of plan switches in the driver's bench shape (`bench.py --steps 20 --warmup 5`: rounds 5-25,
the slow part of a run), one bench.py process per (rep, variant), alternating.

usage: python tools/driver_shape_ab.py <reps> "<variant>;<variant>;..."
A variant is a comma-separated list NAME=VALUE, or "-" for the library defaults.  One JSON line per
run: the line's value, frac and average round time.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(variant):
    if variant.strip() in ("", "-"):
        return {}
    return dict(kv.split("=", 1) for kv in variant.split(","))


def main():
    reps = int(sys.argv[1])
    variants = [parse(v) for v in sys.argv[2].split(";")]
    for rep in range(reps):
        for v in variants:
            env = dict(os.environ, **v)
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                                "--legs=", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                               timeout=240, check=True)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(json.dumps({"env": v, "rep": rep, "value": d["value"], "frac": d["roofline"]["frac"],
                              "avg_launch_us": d["roofline"]["avg_launch_us"],
                              "ms_per_step": d["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
