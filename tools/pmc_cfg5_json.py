"""cfg5 per-phase HBM traffic (tools/pmc_cfg5.sh output) -> profiles/pmc_cfg5.json, keyed by the
kernel sources' sha256 like profiles/pmc_cfg4.json (bench.py's cfg5_partitioned leg reports it only
when it was taken on these sources).

usage: python tools/pmc_cfg5_json.py <pmc_cfg5 dir>
FETCH_SIZE is doubled (MI355X_MICROARCH.md §HBM, gfx950), WRITE_SIZE as reported; averages over the
dispatches of each phase kernel (k_bin_scatter / k_bin_regroup / k_bin_gather, fp64).
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import src_sha256  # noqa: E402

E = (1 << 26) * 16   # deliveries per cfg5 round
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "<float" in k or "float," in k:
            continue
        if any(p in k for p in ("k_bin_scatter", "k_bin_regroup", "k_bin_gather")):
            acc[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
phases, tot = {}, 0.0
for k, cs in acc.items():
    fb = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
    wb = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
    phases[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes_per_delivery": (fb + wb) / E,
                 "dispatches": len(cs["FETCH_SIZE"])}
    tot += fb + wb
lib = os.path.join(ROOT, "approximate-consensus-simulation_amd", "acsim", "_lib", "libacsim.so")
rec = {"source": "tools/pmc_cfg5.sh (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each) over "
                 "tools/bench_configs.py cfg5 (20 FIXED rounds, run twice)",
       "correction": "FETCH_SIZE x 2 (MI355X_MICROARCH.md §HBM, gfx950); WRITE_SIZE as reported",
       "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "src_sha256": src_sha256(),
       "deliveries_per_round": E, "bytes_per_round": tot, "bytes_per_delivery": tot / E,
       "unit_bytes_per_round": 208 * (1 << 26), "phases": phases}
json.dump(rec, open(os.path.join(ROOT, "profiles", "pmc_cfg5.json"), "w"), indent=1)
print(f"{tot / 1e9:.2f} GB per round, {tot / E:.2f} B per delivery")
