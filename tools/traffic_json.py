"""Per-round HBM traffic of the headline round kernels from tools/pmc.sh output -> profiles/.

usage: python tools/traffic_json.py <pmc dir glob> <tag> <bench kernel name> <out> <pattern> [<pattern> ...]
(<pmc dir glob>: directories holding rocprofv3 counter_collection.csv, e.g. gpurun_out/s38/pmc_f64_*;
 <out>: profiles/<out>.json, e.g. pmc_cfg4 (read by bench.py) or pmc_cfg4_f32)

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
tallies each 128-B read request at 64 B, so it is doubled; WRITE_SIZE is taken as reported.  The
per-round traffic sums every kernel matching a pattern (the binned round is two launches).
"""
import collections, csv, glob, hashlib, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d, tag, bench_name, outname, pats = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {}
fetch = write = 0.0
for k, cs in acc.items():
    if not any(p in k for p in pats):
        continue
    f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
    w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
    per[k] = {"fetch_bytes_corrected": f, "write_bytes": w, "dispatches": len(cs["FETCH_SIZE"])}
    fetch += f
    write += w
lib = os.path.join(ROOT, "approximate-consensus-simulation_amd", "acsim", "_lib", "libacsim.so")
sys.path.insert(0, ROOT)
from bench import src_sha256  # noqa: E402  (the kernel sources this measurement belongs to)
rec = {"kernel": bench_name, "n_nodes": 1 << 20, "hbm_bytes_per_launch": fetch + write,
       "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
       "src_sha256": src_sha256(),
       "fetch_bytes_corrected": fetch, "write_bytes": write, "per_kernel": per,
       "source": f"profiles/{tag}_pmc.json",
       "correction": "FETCH_SIZE x 2 (MI355X_MICROARCH.md §HBM, gfx950); WRITE_SIZE as reported"}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump({"tag": tag, "kernels": {k: dict(v) for k, v in acc.items()}}, open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w"), indent=1)
json.dump(rec, open(os.path.join(ROOT, "profiles", f"{outname}.json"), "w"), indent=1)
print(json.dumps(rec, indent=1))
