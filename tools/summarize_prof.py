"""Summarise rocprofv3 CSV output into profiles/ (kernel stats + PMC traffic per launch).

usage: python tools/summarize_prof.py <tag> <kernel_stats.csv> [--pmc DIR ...] [--n-nodes N]

HBM/fabric bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE tallies each 128-B memory-side read request at 64 B (TCC_EA0_RDREQ × 64 B),
so it is doubled before comparing with a byte count; WRITE_SIZE is taken as reported.
Writes profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_pmc.json and, for the cfg4 round
kernel, profiles/pmc_cfg4.json (read by bench.py for roofline.traffic).
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("stats")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--n-nodes", type=int, default=1 << 20)
    ap.add_argument("--kernel", default="k_round_regular<32, 5, true>")
    ap.add_argument("--bench-name", default="k_round_regular<32,5,clean>")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(a.stats, os.path.join(prof, f"{a.tag}_kernel_stats.csv"))
    avg = collections.defaultdict(dict)
    for d in a.pmc:
        for fn in os.listdir(d):
            if not fn.endswith("counter_collection.csv"):
                continue
            acc = collections.defaultdict(list)
            for r in csv.DictReader(open(os.path.join(d, fn))):
                acc[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
            for (k, c), v in acc.items():
                avg[k][c] = sum(v) / len(v)
    out = {"tag": a.tag, "kernels": avg,
           "note": "per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB as reported by rocprofv3"}
    json.dump(out, open(os.path.join(prof, f"{a.tag}_pmc.json"), "w"), indent=1)
    for k, c in avg.items():
        if a.kernel in k and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fetch = c["FETCH_SIZE"] * 1024 * 2      # gfx950: 128-B requests tallied at 64 B
            write = c["WRITE_SIZE"] * 1024
            rec = {"kernel": a.bench_name, "rocprof_kernel": k, "n_nodes": a.n_nodes,
                   "hbm_bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch,
                   "write_bytes": write, "fetch_size_kib_raw": c["FETCH_SIZE"],
                   "write_size_kib_raw": c["WRITE_SIZE"],
                   "tcc_hit": c.get("TCC_HIT_sum"), "tcc_miss": c.get("TCC_MISS_sum"),
                   "source": f"profiles/{a.tag}_pmc.json",
                   "correction": "FETCH_SIZE x 2 (MI355X_MICROARCH.md §HBM, gfx950)"}
            json.dump(rec, open(os.path.join(prof, "pmc_cfg4.json"), "w"), indent=1)
            print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
