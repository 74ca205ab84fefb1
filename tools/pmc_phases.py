"""Per-kernel averages of rocprofv3 counter CSVs (tools/pmc.sh output) as one JSON object.
FETCH_SIZE is doubled (MI355X_MICROARCH.md §HBM, gfx950 tallies a 128-B request at 64 B);
WRITE_SIZE as reported.  usage: python tools/pmc_phases.py <dir> [kernel substring ...]"""
import collections
import csv
import glob
import json
import os
import sys

d, pats = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    if pats and not any(p in k for p in pats):
        continue
    rec = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in rec:
        rec["fetch_bytes"] = rec["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in rec:
        rec["write_bytes"] = rec["WRITE_SIZE"] * 1024
    rec["dispatches"] = max(len(v) for v in cs.values())
    out[k.split("(")[0]] = rec
print(json.dumps(out, indent=1))
