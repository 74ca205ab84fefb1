"""Headline benchmark (BASELINE.json metric): node-rounds/s + % HBM roofline on cfg4
(N = 2^20 random 32-regular graph, trimmed mean t = 5, no faults, p = 0), FIXED rounds.

A "step" is one synchronous round of all N nodes (round kernel + ε-spread finalize) with the
state resident in HBM.  `python bench.py --gpus N --steps K --warmup W`; for N > 1 the driver
launches one rank per GPU with torch.distributed.run: cfg4 does not shard (replicas
only), so each rank runs its own independent instance (global instance id = rank; same graph)
and `value` is the whole-node aggregate: N·n_nodes·K ÷ max-over-ranks time ("scaling": "weak").

The roofline object prices the dominant kernel at SURVEY §8(d)'s algorithmic 400 B/node-round
(32·4 B column ids + 32·8 B neighbour values + 8 B own value + 8 B store) times the N nodes one
launch processes, divided by its average device duration measured with HIP events on the
handle's stream over the timed region.  On cfg4 the round is the binned exchange
(csrc/round_binned.hip): two launches, k_bin_scatter then k_bin_gather, bracketed together by
one event pair, so "one launch" here means that pair.  The ε-spread fold of the previous round runs
inside k_bin_scatter (deferred finalize) and is therefore included; the one
standalone k_finalize per 16-round chunk is not.  Every
--event-every-th timed round (default 10) is bracketed: an event pair idles the stream for
~5 µs, which would otherwise inflate ms_per_step by ~7 %.
`traffic` is the pair's measured HBM bytes per round (profiles/pmc_cfg4.json, FETCH_SIZE x 2 +
WRITE_SIZE, tools/traffic_json.py).  cpu_baseline times the CPU oracle (this
repo's spec restatement, oracle/) on rank 0 on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "approximate-consensus-simulation_amd")
sys.path.insert(0, PKG)

METRIC = "node-rounds/sec (whole node) + % HBM roofline, trimmed-mean N=1M sparse"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_NODE_ROUND = 400  # 32*4 + 32*8 + 8 + 8
BYTES_PER_NODE_ROUND_F32 = 264  # SURVEY §8(d) fp32 mode: 32*4 + 32*4 + 4 + 4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n-nodes", type=int, default=1 << 20)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"],
                   help="value type; the headline is fp64, fp32 mode (DESIGN.md §9) is reported separately")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU work for the bounded cpu_baseline sample")
    p.add_argument("--no-event-timing", action="store_true",
                   help="skip per-launch HIP events (roofline then uses ms_per_step)")
    p.add_argument("--event-every", type=int, default=10,
                   help="bracket every k-th timed round with HIP events (each pair idles the "
                        "stream ~5 us, so sampling keeps the timed region representative)")
    return p.parse_args()


def cpu_baseline(n_nodes: int, seconds: float, dtype: str = "f64") -> dict:
    """Time the oracle (oracle/acs_oracle.c, -O2, OpenMP over receivers) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from acsim import preset
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    cfg = preset("cfg4", n_nodes=n_nodes, max_rounds=10000, omp_threads=threads, dtype=dtype)
    with O.OracleSimulator(cfg, threads=threads) as o:
        t0 = time.perf_counter()
        o.round(1)   # warm-up round (page faults, thread spin-up)
        one = time.perf_counter() - t0
        rounds = int(max(1, min(1000, seconds / max(one, 1e-3))))
        t0 = time.perf_counter()
        o.round(rounds)
        dt = time.perf_counter() - t0
    return {"value": n_nodes * rounds / dt, "unit": "node-rounds/s", "cores": threads,
            "kind": "port",
            "sample": f"cfg4 (N={n_nodes}, d=32, t=5, FIXED) — {rounds} rounds after 1 warm-up "
                      f"round, {dt:.1f} s, oracle/acs_oracle.c with {threads} OpenMP threads"}


def load_pmc(kernel: str, n_nodes: int, dtype: str = "f64"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_cfg4.json" if dtype == "f64" else "pmc_cfg4_f32.json")
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if d.get("kernel") == kernel and d.get("n_nodes") == n_nodes:
        return d.get("hbm_bytes_per_launch")
    return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch  # imported before libacsim so both share one HIP runtime
        import torch.distributed as dist
        dist.init_process_group("gloo")
    import acsim

    n = a.n_nodes
    cfg = acsim.preset("cfg4", n_nodes=n, max_rounds=a.warmup + a.steps, instance_offset=rank,
                         dtype=a.dtype)
    dev = 0
    if world > 1:
        import torch
        # device_count() does not initialise the GPU; modulo lets a rehearsal share one card
        dev = local_rank % max(1, torch.cuda.device_count())
    sim = acsim.Simulator(cfg, device=dev)

    def barrier_sync():
        sim.sync()
        if dist is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dist.barrier()

    if a.warmup:
        sim.round(a.warmup)
    sim.set_kernel_timing(not a.no_event_timing, every=a.event_every)
    barrier_sync()
    t0 = time.perf_counter()
    sim.round(a.steps)
    barrier_sync()
    dt = time.perf_counter() - t0
    k_ms, k_n, kname = sim.kernel_timing()
    sim.set_kernel_timing(False)
    rounds = int(sim.rounds()[0])
    assert rounds == a.warmup + a.steps, (rounds, a.warmup, a.steps)

    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank != 0:
        sim.close()
        dist.destroy_process_group()
        return

    value = world * n * a.steps / dt
    avg_launch_s = (k_ms / 1e3 / k_n) if k_n else dt / a.steps
    unit_b = BYTES_PER_NODE_ROUND_F32 if a.dtype == "f32" else BYTES_PER_NODE_ROUND
    achieved = unit_b * n / avg_launch_s / 1e9
    traffic = load_pmc(kname, n, a.dtype)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "node-rounds/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (Philox-seeded x^0 and Feistel graph, SURVEY §A.2/§A.3)",
        "config": {"workload": "cfg4: N=2^20 random 32-regular graph, trimmed mean t=5, no faults, "
                               "no loss, FIXED rounds (SURVEY §A.10)",
                   "n_nodes": n, "degree": 32, "trim": 5, "instances_per_gpu": 1,
                   "parallelism": "replicas" if world > 1 else "single-gpu"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "avg_launch_us": avg_launch_s * 1e6,
                     "bytes_per_node_round": unit_b},
        "hbm_roofline_pct_wall": 100.0 * unit_b * value / world / 1e9 / HBM_PEAK_GBS,
    }
    sim.close()
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, a.cpu_seconds, a.dtype)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
