"""cfg3 roofline counters from tools/pmc_cfg3.sh output -> profiles/<out>.json.

usage: python tools/pmc_cfg3_json.py <pmc_cfg3 dir> <out name>

valu_busy_frac = SQ_ACTIVE_INST_VALU (quad-cycles summed over SIMDs) x 4 / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8); mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x GRBM_GUI_ACTIVE / 8)
(rocprofv3 MfmaUtil); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Counters are averaged over the
dispatches of each kernel (bench_configs.py runs each preset twice).  valu_insts_per_node_round
divides the wave-instruction count by the node-rounds.  valu_insts_per_launch is the count for one
dispatch of the cfg3 workload (10^5 instances, bench_configs.py: 63 323 840 node-rounds); bench.py's
cfg3_sharded leg scales it by its own node-rounds and divides by its own HIP-event kernel time.
The record is keyed by the sha256 of the kernel sources (bench.py src_sha256), as pmc_cfg4.json.
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
NODE_ROUNDS = {"k_batched_split": 63323840, "k_batched_small": 63323840,
               "k_batched_mfma": 63321472}   # cfg3 / cfg3_g16 (bench_configs)
d, out = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_batched" in r["Kernel_Name"]:
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    m["dispatch_cycles_per_xcd"] = cyc
    m["valu_busy_frac"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc)
    m["mfma_busy_frac"] = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * cyc)
    nr = next(v for p, v in NODE_ROUNDS.items() if p in k)
    m["valu_insts_per_node_round"] = m["SQ_INSTS_VALU"] / nr
    m["valu_insts_per_launch"] = m["SQ_INSTS_VALU"]
    m["node_rounds_per_launch"] = nr
    kern[k] = m
lib = os.path.join(ROOT, "approximate-consensus-simulation_amd", "acsim", "_lib", "libacsim.so")
rec = {"source": "tools/pmc_cfg3.sh (rocprofv3 --pmc, 3 passes) over tools/bench_configs.py cfg3 cfg3_g16",
       "derivation": " ".join(__doc__.split("\n\n")[2].split()),
       "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
       "src_sha256": __import__("bench").src_sha256(),
       "kernels": kern}
json.dump(rec, open(os.path.join(ROOT, "profiles", f"{out}.json"), "w"), indent=1)
for k, m in kern.items():
    print(f"{k[:60]:60s} valu_busy {m['valu_busy_frac']:.3f}  mfma_busy {m['mfma_busy_frac']:.3f}  "
          f"valu/node-round {m['valu_insts_per_node_round']:.1f}")
