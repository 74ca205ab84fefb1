"""Time every preset on one GPU: node-rounds/s, rounds, and the round kernel's
average device time.  Prints one JSON line per config.  usage: python tools/bench_configs.py [names]

cfg1/cfg2/cfg3 run to ε-convergence (their natural workload); cfg4/cfg5 run FIXED rounds.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))

import acsim  # noqa: E402

CASES = {
    "cfg1": dict(),
    "cfg1_avg": dict(),
    "cfg2": dict(),
    "cfg3": dict(),
    "cfg3_g16": dict(),
    "cfg4": dict(max_rounds=100),
    "cfg4_eps": dict(),
    "cfg4_byz": dict(),
    "cfg5": dict(max_rounds=20),
    "cfg4_f32": dict(max_rounds=100),   # fp32 mode
    "cfg3_f32": dict(),
    "cfg5_f32": dict(max_rounds=20),   # fp32 two-level plan
    "cfg4_byz_f32": dict(),            # fp32 tagged binned exchange
    "cfg4_fixed14": dict(max_rounds=14),   # the FIXED twin of cfg4_eps's 14 rounds (EPS overhead check)
    # user graph (§8(f) row 1): 2^20 nodes, power-law degrees 11..32, hub-skewed senders, trimmed t=5
    "csr_2e20": dict(max_rounds=20),
    "csr_2e20_generic": dict(max_rounds=20),   # the same graph on the one-workgroup-per-receiver kernel
    # power-law user graph with hubs: degrees 11..20000 (about 19 % of the rows above 32): fast path +
    # hub rows on the generic / big-m kernels, and the same graph on the generic kernel alone
    "csr_2e20_hubs": dict(max_rounds=10),
    "csr_2e20_hubs_generic": dict(max_rounds=10),
    # size probes of the headline shape (stage 64 / 128 / 512 MiB against the 256 MiB MALL)
    "cfg4_n18": dict(max_rounds=100, n_nodes=1 << 18),
    "cfg4_n19": dict(max_rounds=100, n_nodes=1 << 19),
    "cfg4_n21": dict(max_rounds=100, n_nodes=1 << 21),
    # big-m generic path: complete graph above 8192 nodes with loss (segmented radix sort per receiver)
    "complete_16k_loss": dict(max_rounds=3),
    # generic LDS kernel: complete graph with loss (4096 entries per receiver)
    "complete_4k_loss": dict(max_rounds=10),
}


def run(name, **kw):
    csr = None
    if name.startswith("csr_2e20"):
        from acsim.graphs import skewed_csr
        csr = skewed_csr(1 << 20, 11, 20000, 13, alpha=2.5) if "hubs" in name else skewed_csr(1 << 20, 11, 32, 11)
        cfg = acsim.Config(n_nodes=1 << 20, topology="csr", rule="trimmed", trim=5, termination="fixed", **kw)
        os.environ["ACSIM_CSR_FAST"] = "0" if name.endswith("_generic") else "1"
    elif name in ("complete_16k_loss", "complete_4k_loss"):
        cfg = acsim.Config(n_nodes=16384 if name.startswith("complete_16k") else 4096, topology="complete",
                           rule="trimmed", trim=100, loss_p=0.2, termination="fixed", **kw)
    elif name == "cfg4_fixed14" or name.startswith("cfg4_n"):
        cfg = acsim.preset("cfg4", **kw)
    elif name.endswith("_f32"):
        cfg = acsim.preset(name[:-4], dtype="f32", **kw)
    else:
        cfg = acsim.preset(name, **kw)
    t0 = time.perf_counter()
    sim = acsim.Simulator(cfg, csr=csr)
    t_setup = time.perf_counter() - t0
    sim.set_kernel_timing(True, every=10)
    t0 = time.perf_counter()
    res = sim.run()
    wall = time.perf_counter() - t0
    ms, n, kname = sim.kernel_timing()
    rounds = sim.rounds()
    out = {"config": name, "n_nodes": cfg.n_nodes, "n_instances": cfg.n_instances,
           "rounds_max": int(res.rounds_max), "rounds_mean": float(rounds.mean()),
           "n_converged": int(res.n_converged), "node_rounds": int(res.node_rounds),
           "wall_s": wall, "node_rounds_per_s": res.node_rounds / wall,
           "kernel": kname, "kernel_launches": n, "kernel_ms_total": ms,
           "kernel_avg_us": (ms / n * 1e3) if n else None, "setup_s": t_setup}
    sim.close()
    return out


def main():
    names = sys.argv[1:] or list(CASES)
    for nm in names:
        run(nm, **CASES.get(nm, {}))          # warm-up (code objects, allocations)
        print(json.dumps(run(nm, **CASES.get(nm, {}))), flush=True)


if __name__ == "__main__":
    main()
