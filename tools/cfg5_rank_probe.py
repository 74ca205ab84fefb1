"""cfg5 per-rank compute bound on ONE GPU.

A real G-rank run gives each rank the receiver rows [g·N/G, (g+1)·N/G) and a full replicated x.
Here the G partitions run as virtual partitions on one device (acs_create_partitioned with no
RCCL id: private x copies, device-copy all-gather), with the unchunked sequence
(ACSIM_XCHUNKS=1), so the HIP-event bracket of each round covers exactly the G partitions' round
kernels one after the other, each alone on the whole GPU — the compute a rank runs on its own
GPU.  Per-rank compute = bracketed time / G (partitions are equal: 2^26 / G rows, whole source
blocks).  The exchange (here device copies) is skipped from the figure.

Per-rank bytes (model, from the measured unpartitioned per-delivery traffic of
profiles/r02_fin_pmc_cfg5.json and its re-measure): the rank's deliveries are 1/G of the graph's,
but its phase A still stages every source block of x, the full 512 MiB, each round.

usage: python tools/cfg5_rank_probe.py [--rounds 6] [--warm 2] [--groups 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))

N = 1 << 26
D = 16
XBYTES = N * 8                     # the replicated x a rank's phase A stages each round
X_EXCH_RX = lambda g: (g - 1) / g * XBYTES   # bytes each rank receives per round in the all-gather


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--groups", default="1,2,4,8")
    a = ap.parse_args()
    os.environ["ACSIM_XCHUNKS"] = "1"
    import acsim
    cfg = acsim.preset("cfg5", max_rounds=a.warm + a.rounds)
    for g in (int(v) for v in a.groups.split(",")):
        t0 = time.perf_counter()
        sim = acsim.Simulator(cfg) if g == 1 else acsim.Simulator(cfg, partitions=g)
        t_create = time.perf_counter() - t0
        sim.round(a.warm)
        sim.set_kernel_timing(True)
        sim.sync()
        t0 = time.perf_counter()
        sim.round(a.rounds)
        sim.sync()
        wall = time.perf_counter() - t0
        k_ms, k_n, kname = sim.kernel_timing()
        sim.close()
        per_round = k_ms / max(1, k_n)
        print(json.dumps({
            "G": g, "kernel": kname, "rounds": a.rounds, "create_s": t_create,
            "round_kernels_ms_all_partitions": per_round,
            "per_rank_compute_ms": per_round / g,
            "wall_ms_per_round_one_gpu": wall / a.rounds * 1e3,
            "per_rank_x_staging_bytes": XBYTES,
            "per_rank_allgather_rx_bytes": X_EXCH_RX(g),
            "per_rank_deliveries": N * D // g}), flush=True)


if __name__ == "__main__":
    main()
