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
(csrc/round_binned.hip): two launches, k_bin_scatter then k_bin_gather, so "one launch" here means
that pair, i.e. one round.  The events bracket runs of --event-run consecutive timed rounds (default
25: four runs in a 100-step region), one pair per run, so a round's device time includes the
boundary between its two kernels and the one to the next round, and no event-induced idle (a pair
around every 10th single round, rounds 1-3, idled the stream for ~5 µs and inflated the bracketed
round by ~2 µs).  The ε-spread fold of the previous round runs inside k_bin_scatter (deferred
finalize); the one standalone k_finalize per 16-round chunk falls inside a run.
`traffic` is the pair's measured HBM bytes per round from the committed rocprofv3 PMC summary
(profiles/pmc_cfg4.json, FETCH_SIZE x 2 + WRITE_SIZE, tools/traffic_json.py); it is reported only
when that summary was taken on this build (same library sha256, or the same sha256 of the kernel
sources: a rebuild of unchanged sources is not byte-identical), else null.
cpu_baseline times the CPU oracle (this repo's spec restatement, oracle/) on rank 0 on a bounded
sample of the same workload.

Extra legs (every N, each guarded: a failing leg is reported as an error string and never costs
the headline line; each result, and at N > 1 each cfg5 sub-leg, enters the line as soon as it
exists, and a watchdog prints the line — naming the stage that hung — if a leg hangs).  Exit code:
0 when every leg ran and matched its golden hash, 4 when one failed or mismatched (`legs_failed`
names them; at N > 1 the cfg5 leg fails with its default all-gather sequence, while the opt-in
chunked sequence is reported as `opt_in_ok`), 3 when the watchdog fired; the line is printed in
every case and nothing is retried or re-launched:
  cfg4_f32          the headline workload in fp32 mode (north_star: "fp32 mode stated
                    separately"), timed and roofline-priced like the headline at 264 B/node-round,
                    100 FIXED rounds of a fresh handle checked against the oracle's hash.
  cfg3_sharded      10^5 instances x 64 nodes (BASELINE configs[2]) sharded over the ranks by
                    contiguous global instance blocks, no data-path collective; node-rounds/s
                    of the whole job (the batch run 8 times back to back per rank, so the
                    fixed per-rank cost is amortised alike at every N; `single` times one
                    unamortised run), and the checksum of per-instance checksums gathered on
                    rank 0 compared with tests/golden/fullsize.json (every repetition must agree).
  cfg4_narrow       the headline workload (rounds 10-110) on the opt-in narrow plan
                    (ACSIM_BIN_NARROW=1), priced at the same 400 B unit, with the
                    100-round golden check; reported beside the headline, never as it.
  cfg5_partitioned  N = 2^26 random 16-regular (BASELINE configs[4]); one plain handle at N = 1,
                    node-partitioned over the ranks at N > 1, where BOTH exchange sequences run on
                    their own handles (the per-round RCCL all-gather, the default, and the chunked
                    send / receive with ACSIM_XCHUNKS=4); W warm-up + R timed FIXED rounds,
                    ms/round, the exchange share, and sha256(x) after the 10 rounds against the
                    golden hash, per sequence.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "approximate-consensus-simulation_amd")
sys.path.insert(0, PKG)

METRIC = "node-rounds/sec (whole node) + % HBM roofline, trimmed-mean N=1M sparse"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 vector (= fp64 matrix) peak, vendor datasheet
BYTES_PER_NODE_ROUND = 400  # 32*4 + 32*8 + 8 + 8
BYTES_PER_NODE_ROUND_F32 = 264  # SURVEY §8(d) fp32 mode: 32*4 + 32*4 + 4 + 4
CFG5_BYTES_PER_NODE_ROUND = 208  # 16*4 + 16*8 + 16
CFG3_FLOP_PER_NODE_ROUND = 128   # 2*64
# MI355X VALU capacity: 1024 SIMDs x 2.4 GHz SIMD-cycles/s (MI355X_MICROARCH.md chip-level parameters);
# SQ_ACTIVE_INST_VALU counts quad-cycles, so x 4 gives the SIMD-cycles the VALU pipe was busy
VALU_PEAK_SIMD_CYCLES_PER_S = 1024 * 2.4e9
GOLDEN = os.path.join(ROOT, "tests", "golden", "fullsize.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n-nodes", type=int, default=1 << 20)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"],
                   help="value type; the headline is fp64, fp32 mode (DESIGN.md §9) is reported separately")
    p.add_argument("--cpu-seconds", type=float, default=20.0,
                   help="target CPU time of the two bounded cpu_baseline samples together (1 thread, all cores)")
    p.add_argument("--no-event-timing", action="store_true",
                   help="skip per-launch HIP events (roofline then uses ms_per_step)")
    p.add_argument("--event-run", type=int, default=25,
                   help="bracket runs of k consecutive timed rounds with one HIP event pair each "
                        "(per-round device time with no event-induced idle inside a run)")
    p.add_argument("--legs", default="f32,cfg3,cfg5,narrow",
                   help="comma-separated extra legs (f32, cfg3, cfg5, narrow); empty for none")
    p.add_argument("--leg-timeout", type=float, default=180.0,
                   help="watchdog: print the line without the unfinished legs after this many seconds")
    p.add_argument("--allow-shared-device", action="store_true",
                   help="rehearsal only: run more ranks than GPUs (n_gpus then counts distinct devices "
                        "and the line is marked shared_device)")
    return p.parse_args()


def host_facts() -> dict:
    """nproc, the CPUs this process may run on, and the CPU model (the CPU timing
    records the host it ran on)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": model,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def all_core_threads() -> tuple:
    """The all-core thread count and why: OMP_NUM_THREADS when set (the GPU box sets it to the
    job's CPU share, 16 threads per GPU, while nproc there counts the whole machine), else the
    CPUs this process may run on."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env, "OMP_NUM_THREADS (the job's CPU share on the GPU box)"
    try:
        return max(1, len(os.sched_getaffinity(0))), "sched_getaffinity"
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1), "os.cpu_count()"


def time_oracle(n_nodes: int, seconds: float, dtype: str, threads: int) -> dict:
    """One bounded sample of the oracle on the cfg4 workload: a warm-up round, then as many FIXED
    rounds as fit in about `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from acsim import preset
    cfg = preset("cfg4", n_nodes=n_nodes, max_rounds=10000, omp_threads=threads, dtype=dtype)
    with O.OracleSimulator(cfg, threads=threads) as o:
        t0 = time.perf_counter()
        o.round(1)   # warm-up round (page faults, thread spin-up)
        one = time.perf_counter() - t0
        rounds = int(max(1, min(1000, seconds / max(one, 1e-3))))
        t0 = time.perf_counter()
        o.round(rounds)
        dt = time.perf_counter() - t0
    return {"value": n_nodes * rounds / dt, "threads": threads, "rounds": rounds, "seconds": dt}


def cpu_baseline(n_nodes: int, seconds: float, dtype: str = "f64") -> dict:
    """Time the oracle (oracle/acs_oracle.c, -O2, OpenMP over receivers) on the host, single-threaded
    and on all the job's cores, each on a bounded sample of the same workload.
    `value` / `cores` are the all-core figure."""
    t_all, why = all_core_threads()
    one = time_oracle(n_nodes, seconds / 2, dtype, 1)
    allc = time_oracle(n_nodes, seconds / 2, dtype, t_all)
    return {"value": allc["value"], "unit": "node-rounds/s", "cores": t_all,
            "kind": "port",
            "sample": f"cfg4 (N={n_nodes}, d=32, t=5, FIXED, {dtype}) — oracle/acs_oracle.c: "
                      f"{one['rounds']} rounds on 1 thread ({one['seconds']:.1f} s) and {allc['rounds']} rounds "
                      f"on {t_all} OpenMP threads ({allc['seconds']:.1f} s), each after 1 warm-up round",
            "threads_1": one, "threads_all": dict(allc, source=why),
            "host": host_facts()}


def lib_sha256() -> str:
    from acsim import _abi
    path = _abi.library_path()
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def src_sha256() -> str:
    """sha256 over the HIP library's sources (csrc/*.hip, *.hpp, the Makefile, include/acsim.h):
    a rebuild of unchanged sources keeps it, while the library's own hash may change (the
    toolchain's output is not byte-reproducible across build directories)."""
    csrc = os.path.join(PKG, "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".hpp")) or f == "Makefile")
    h = hashlib.sha256()
    for f in files + ["../../include/acsim.h"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def load_pmc_cfg3(kernel: str):
    """cfg3's VALU counters (profiles/pmc_cfg3.json, tools/pmc_cfg3.sh + pmc_cfg3_json.py) for the
    given batched kernel, if they were taken on these kernel sources (same src_sha256 / lib sha256),
    else None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_cfg3.json")))
    except Exception:
        return None
    if d.get("src_sha256") != src_sha256() and d.get("lib_sha256") != lib_sha256():
        return None
    for name, m in d.get("kernels", {}).items():
        if kernel and kernel.split("<")[0] in name and (("<2" in kernel) == ("<2" in name)):
            return m
    return None


def load_pmc_cfg5():
    """cfg5's per-phase HBM traffic (profiles/pmc_cfg5.json, tools/pmc_cfg5_json.py), if it was
    taken on these kernel sources, else None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_cfg5.json")))
    except Exception:
        return None
    if d.get("src_sha256") != src_sha256() and d.get("lib_sha256") != lib_sha256():
        return None
    return {"bytes_per_round": d["bytes_per_round"], "bytes_per_delivery": d["bytes_per_delivery"],
            "phases_bytes_per_delivery": {k.split("::")[-1].split("<")[0]: v["bytes_per_delivery"]
                                          for k, v in d["phases"].items()},
            "source": "profiles/pmc_cfg5.json"}


def load_pmc(kernel: str, n_nodes: int, dtype: str = "f64"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if it was taken on this
    build of libacsim.so — same kernel name and size, and the same library sha256 or the same
    sha256 of the kernel sources — else None."""
    path = os.path.join(ROOT, "profiles", "pmc_cfg4.json" if dtype == "f64" else "pmc_cfg4_f32.json")
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if d.get("kernel") != kernel or d.get("n_nodes") != n_nodes:
        return None
    if d.get("lib_sha256") == lib_sha256() or d.get("src_sha256") == src_sha256():
        return d.get("hbm_bytes_per_launch")
    return None


class Ctx:
    """Rank / device / control-plane plumbing shared by the headline and the legs.  `group` is an
    acsim.rendezvous.Group (plain sockets, no torch in the rank process: every rank maps only the
    HIP runtime and RCCL libacsim.so was built against), None at N = 1."""

    def __init__(self, world, rank, local_rank, dev, group):
        self.world, self.rank, self.local_rank, self.dev, self.group = world, rank, local_rank, dev, group
        self.stage = "headline"   # what is running (the watchdog's note names it)
        self.partial = {}         # rank 0: the running leg's results so far (in the printed line)

    def enter(self, stage: str) -> None:
        """Mark the start of a (sub-)leg.  Fault injection for rehearsals (tools/):
        ACSIM_BENCH_HANG=<stage> makes that stage hang on every rank, so the watchdog path can be
        exercised on one box without a real hang."""
        self.stage = stage
        if os.environ.get("ACSIM_BENCH_HANG") == stage:
            time.sleep(1e9)

    def barrier(self, sim=None):
        if sim is not None:
            sim.sync()
        if self.group is not None:
            self.group.barrier()

    def max(self, v: float) -> float:
        return float(v) if self.group is None else self.group.max(v)

    def all_ok(self, ok: bool) -> bool:
        return ok if self.group is None else self.group.min(1.0 if ok else 0.0) > 0.5

    def gather(self, obj):
        return [obj] if self.group is None else self.group.all_gather(obj)


def golden():
    try:
        return json.load(open(GOLDEN))
    except Exception:
        return {}


def leg_cfg3(ctx: Ctx, reps: int = 8) -> dict:
    """BASELINE configs[2]: instance sharding, no data-path collective.  Two timed
    regions, each from a common start barrier to the slowest rank's last run() return:
      - `single`: ONE run() of the rank's shard on a fresh handle — the unamortised makespan of the
        job, fixed per-rank cost (launch, summary, wake-up) included;
      - the main figure: the shard run `reps` times back to back (one handle each, all created
        before it), so the per-rank fixed cost is amortised the same way at every N.
    Every handle's checksum of per-instance checksums is checked.  `value` is the amortised
    makespan rate: all node-rounds over the slowest rank's time (the closing barrier over the
    socket control plane — tens of µs per collective at N = 8, none at N = 1 — only aligns the
    ranks; `seconds` keeps the time through it)."""
    import numpy as np
    import acsim
    from acsim.digest import instance_digests, combine_digests
    from acsim.distributed import shard_range
    cfg = acsim.preset("cfg3")
    off, cnt = shard_range(cfg.n_instances, ctx.world, ctx.rank)
    local = cfg.replace(n_instances=max(cnt, 1), instance_offset=off)
    sims = []
    one = None
    err = None
    try:
        with acsim.Simulator(local.replace(n_instances=min(256, max(cnt, 1))), device=ctx.dev) as w:
            w.run()   # code-object load and first launch outside the timed region
        one = acsim.Simulator(local, device=ctx.dev)   # the single-run figure: no kernel events
        for _ in range(reps):
            sims.append(acsim.Simulator(local, device=ctx.dev))
            sims[-1].set_kernel_timing(True)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    if not ctx.all_ok(err is None):
        # release whatever this rank did create before raising (its device buffers would stay
        # allocated while the remaining legs run)
        for sim in ([one] if one is not None else []) + sims:
            try:
                sim.close()
            except Exception:  # noqa: BLE001
                pass
        raise RuntimeError(err or "another rank failed to create its cfg3 shard")
    ctx.barrier(one)
    t0 = time.perf_counter()
    one.run()
    t_one = ctx.max(time.perf_counter() - t0)
    one_rounds = one.rounds()
    one_dig = instance_digests(one.all_values())
    one.close()
    ctx.barrier(sims[0])
    t0 = time.perf_counter()
    for sim in sims:
        sim.run()
    t_local = time.perf_counter() - t0
    ctx.barrier(sims[0])
    dt = ctx.max(time.perf_counter() - t0)
    t_local = ctx.max(t_local)
    k_ms = sum(sim.kernel_timing()[0] for sim in sims)
    kname = sims[0].kernel_timing()[2]
    rounds = sims[0].rounds()
    digs = [instance_digests(sim.all_values()) for sim in sims]
    same = all(np.array_equal(d, digs[0]) and np.array_equal(sim.rounds(), rounds) for d, sim in zip(digs, sims))
    same = same and np.array_equal(one_dig, digs[0]) and np.array_equal(one_rounds, rounds)
    dig = digs[0]
    for sim in sims:
        sim.close()
    if cnt == 0:
        rounds, dig = rounds[:0], dig[:0]
    parts = ctx.gather((off, rounds.astype(np.uint32).tobytes(), dig.tobytes(), k_ms, same))
    if ctx.rank != 0:
        return {}
    parts.sort(key=lambda p: p[0])
    all_rounds = np.concatenate([np.frombuffer(p[1], dtype=np.uint32) for p in parts])
    all_dig = np.concatenate([np.frombuffer(p[2], dtype=np.uint8) for p in parts])
    node_rounds_one = int(cfg.n_nodes) * int(all_rounds.astype(np.int64).sum())
    node_rounds = node_rounds_one * reps
    g = golden().get("cfg3", {})
    digest = combine_digests(all_dig)
    kmax = max(p[3] for p in parts) / 1e3
    flops = CFG3_FLOP_PER_NODE_ROUND * node_rounds
    # cfg3's true bound is integer VALU (Philox).  VALU wave-instructions per node-round
    # from the committed counters (taken on these sources), times this leg's node-rounds, over the
    # leg's own HIP-event kernel time, against the VALU issue peak per GPU
    pmc = load_pmc_cfg3(kname)
    valu = None
    if pmc and kmax > 0:
        nr = pmc["node_rounds_per_launch"]
        busy_per_nr = pmc["SQ_ACTIVE_INST_VALU"] * 4 / nr
        ach = busy_per_nr * node_rounds / kmax / ctx.world
        valu = {"bound": "valu", "unit": "VALU busy SIMD-cycles/s per GPU", "achieved": ach,
                "peak": VALU_PEAK_SIMD_CYCLES_PER_S, "frac": ach / VALU_PEAK_SIMD_CYCLES_PER_S,
                "valu_busy_cycles_per_node_round": busy_per_nr,
                "valu_insts_per_node_round": pmc["SQ_INSTS_VALU"] / nr,
                "valu_insts_per_s": pmc["SQ_INSTS_VALU"] / nr * node_rounds / kmax / ctx.world,
                "int64_insts_share": pmc.get("SQ_INSTS_VALU_INT64", 0.0) / pmc["SQ_INSTS_VALU"],
                "busy_frac_pmc": pmc.get("valu_busy_frac"),
                "counters": "profiles/pmc_cfg3.json (tools/pmc_cfg3.sh: rocprofv3 --pmc over the same 10^5-instance "
                            "batch, keyed by the kernel sources' sha256); achieved = SQ_ACTIVE_INST_VALU x 4 per "
                            "node-round x this leg's node-rounds / this leg's HIP-event kernel time; busy_frac_pmc "
                            "is the same busy fraction at the profiled run's own clock (GRBM_GUI_ACTIVE)"}
    return {"workload": f"cfg3: 1e5 instances x 64 nodes, complete graph, p=0.2, AVERAGE, eps=1e-6 "
                        f"(SURVEY §A.10), sharded by global instance blocks; the batch run {reps} times "
                        f"back to back (one handle each) inside the timed region",
            "value": node_rounds / t_local, "unit": "node-rounds/s", "seconds": dt,
            "single": {"what": "one run() of the batch on a fresh handle (no kernel events): the job's "
                               "unamortised makespan, from the start barrier to the slowest rank's return",
                       "value": node_rounds_one / t_one, "seconds": t_one},
            "seconds_before_closing_barrier": t_local, "value_through_closing_barrier": node_rounds / dt,
            "reps": reps,
            "node_rounds": node_rounds, "rounds_max": int(all_rounds.max()),
            "instances_per_rank": [len(np.frombuffer(p[1], dtype=np.uint32)) for p in parts],
            "kernel": kname, "kernel_ms_max_rank": kmax * 1e3,
            "fp64_tflops_kernel": flops / kmax / 1e12 if kmax > 0 else None,
            "fp64_frac_of_peak": flops / kmax / 1e12 / FP64_PEAK_TFLOPS / ctx.world if kmax > 0 else None,
            "roofline": valu,
            "instances_digest": digest,
            "golden_match": bool(g) and all(p[4] for p in parts) and digest == g.get("instances_digest") and
                            hashlib.sha256(all_rounds.astype("<u4").tobytes()).hexdigest() == g.get("rounds_sha256")}


def _cfg5_handle(ctx: Ctx, cfg, xchunks):
    """One cfg5 handle: the plain one-GPU handle at N = 1, else this rank's node partition over a
    fresh RCCL communicator, with ACSIM_XCHUNKS set to `xchunks` while it is created (None: the
    library's default sequence, the per-round all-gather for real ranks)."""
    import acsim
    if ctx.world == 1:
        return acsim.Simulator(cfg, device=ctx.dev)
    from acsim.distributed import partitioned_simulator
    old = os.environ.get("ACSIM_XCHUNKS")
    if xchunks is None:
        os.environ.pop("ACSIM_XCHUNKS", None)
    else:
        os.environ["ACSIM_XCHUNKS"] = str(xchunks)
    try:
        return partitioned_simulator(cfg, ctx.rank, ctx.world, ctx.dev, group=ctx.group)
    finally:
        if old is None:
            os.environ.pop("ACSIM_XCHUNKS", None)
        else:
            os.environ["ACSIM_XCHUNKS"] = old


def _cfg5_sub(ctx: Ctx, warm: int, timed: int, xchunks, stage: str = "cfg5_partitioned") -> dict:
    """Time one cfg5 exchange sequence on its own handle: `warm` + `timed` FIXED rounds, ms/round,
    the exchange share (the part of a round outside the rank's own round kernels) and sha256(x^10)
    against the golden hash."""
    import acsim
    from acsim.digest import sha256_values
    ctx.enter(stage)
    cfg = acsim.preset("cfg5", max_rounds=warm + timed)
    sim = None
    err = None
    try:
        sim = _cfg5_handle(ctx, cfg, xchunks)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    if not ctx.all_ok(err is None):
        if sim is not None:
            sim.close()
        return {"error": err or "another rank failed to create its cfg5 partition"}
    kname = sim.kernel_name()
    sim.round(warm)
    sim.set_kernel_timing(True)
    ctx.barrier(sim)
    t0 = time.perf_counter()
    sim.round(timed)
    ctx.barrier(sim)
    dt = ctx.max(time.perf_counter() - t0)
    k_ms, k_n, _ = sim.kernel_timing()
    k_ms = ctx.max(k_ms)
    rounds = int(sim.rounds()[0])
    out = {}
    if ctx.rank == 0:
        x = sim.values(0)
        h = sha256_values(x)
        g = golden().get("cfg5", {})
        n = int(cfg.n_nodes)
        out = {"value": n * timed / dt, "unit": "node-rounds/s", "ms_per_round": dt / timed * 1e3,
               "kernel": kname, "round_kernel_ms_per_round": k_ms / max(1, k_n),
               "exchange_share": max(0.0, 1.0 - (k_ms / max(1, k_n)) / (dt / timed * 1e3)) if ctx.world > 1 else 0.0,
               "hbm_frac_unit": CFG5_BYTES_PER_NODE_ROUND * n * timed / dt / 1e9 / (HBM_PEAK_GBS * ctx.world),
               "rounds": rounds, "x_sha256": h,
               "golden_match": rounds == warm + timed and h == g.get("x10_sha256")}
    sim.close()
    return out


def leg_cfg5(ctx: Ctx, warm: int = 2, timed: int = 8) -> dict:
    """BASELINE configs[4]: node partition over RCCL.  N = 1: one plain handle.  N > 1:
    BOTH exchange sequences, each on its own handle and golden-checked: the default
    per-round in-place all-gather, and the chunked grouped send / receive overlapping phase B and
    the next round's phase A (ACSIM_XCHUNKS=4).  The leg's headline fields are the default
    sequence's; `sequences` holds both."""
    if ctx.world == 1:
        out = _cfg5_sub(ctx, warm, timed, None)
        if ctx.rank == 0 and "error" not in out:
            out["workload"] = (f"cfg5: N=2^26 random 16-regular, trimmed t=5, FIXED; {warm} warm-up + {timed} "
                               f"timed rounds on one GPU (two-level binned exchange)")
            out["traffic"] = load_pmc_cfg5()
        return out
    # N > 1: the library's default sequence first (the all-gather), then the chunked one.  Each
    # result lands in the printed line as soon as it exists (ctx.partial), so a later sub-leg that
    # fails, mismatches the golden hash or hangs (the watchdog then prints the line and the process
    # exits non-zero) never hides an earlier one; nothing is retried or re-launched.
    seqs = ctx.partial.setdefault("sequences", {}) if ctx.rank == 0 else {}
    for name, xc in (("allgather", None), ("chunked", 4)):
        try:
            res = _cfg5_sub(ctx, warm, timed, xc, stage=f"cfg5_partitioned.{name}")
        except Exception as e:  # noqa: BLE001
            res = {"error": f"{type(e).__name__}: {e}"}
        if ctx.rank == 0:
            seqs[name] = res
    if ctx.rank != 0:
        return {}
    # headline fields: the first sequence that ran and matched the golden hash (the default first)
    ok = [n for n in ("allgather", "chunked") if seqs.get(n, {}).get("golden_match")]
    out = dict(seqs[ok[0]]) if ok else {"error": "no cfg5 exchange sequence matched the golden hash"}
    out["headline_sequence"] = ok[0] if ok else None
    out["workload"] = (f"cfg5: N=2^26 random 16-regular, trimmed t=5, FIXED; {warm} warm-up + {timed} timed "
                       f"rounds, node-partitioned over {ctx.world} ranks; headline fields: the first golden-"
                       f"matching sequence of the per-round RCCL all-gather (the library default) and the "
                       f"chunked send / receive exchange; `sequences` holds both")
    out["traffic"] = None
    out["sequences"] = seqs
    # the leg fails (non-zero exit) when the library's default sequence (the all-gather) fails or
    # mismatches; the opt-in chunked sequence's result is reported beside it (`opt_in_ok`) without
    # failing the run, so a problem on the opt-in path never costs the default path's scaling data
    out["ok"] = "allgather" in ok
    out["opt_in_ok"] = "chunked" in ok
    return out


def leg_cfg4_f32(ctx: Ctx, warm: int = 10, timed: int = 100) -> dict:
    """fp32 mode of the headline workload (BASELINE.json north_star: "fp32 mode stated separately",
    DESIGN.md §9): cfg4 in binary32, timed and roofline-priced like the headline (264 B/node-round,
    SURVEY §8(d)); a fresh handle's 100 FIXED rounds are checked against the oracle's hash."""
    import acsim
    from acsim.digest import sha256_values
    cfg = acsim.preset("cfg4", max_rounds=warm + timed, instance_offset=ctx.rank, dtype="f32")
    with acsim.Simulator(cfg, device=ctx.dev) as sim:
        sim.round(warm)
        sim.set_kernel_timing(True, every=25, runs=True)
        ctx.barrier(sim)
        t0 = time.perf_counter()
        sim.round(timed)
        ctx.barrier(sim)
        dt = ctx.max(time.perf_counter() - t0)
        k_ms, k_n, kname = sim.kernel_timing()
    n = int(cfg.n_nodes)
    avg_s = (k_ms / 1e3 / k_n) if k_n else dt / timed
    out = {}
    if ctx.rank == 0:
        with acsim.Simulator(acsim.preset("cfg4", max_rounds=100, dtype="f32"), device=ctx.dev) as chk:
            chk.run()
            ok = sha256_values(chk.values(0)) == golden().get("cfg4", {}).get("f32_fixed100_x_sha256")
        achieved = BYTES_PER_NODE_ROUND_F32 * n / avg_s / 1e9
        out = {"workload": "cfg4 in fp32 mode (binary32 values, DESIGN.md §9), FIXED rounds",
               "value": ctx.world * n * timed / dt, "unit": "node-rounds/s", "ms_per_step": dt / timed * 1e3,
               "dtype": "f32", "kernel": kname, "avg_launch_us": avg_s * 1e6,
               "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": achieved / HBM_PEAK_GBS, "bytes_per_node_round": BYTES_PER_NODE_ROUND_F32,
                            "traffic": load_pmc(kname, n, "f32")},
               "golden_match": ok}
    return out


def leg_cfg4_narrow(ctx: Ctx, warm: int = 10, timed: int = 100) -> dict:
    """The headline workload on the opt-in narrow plan (ACSIM_BIN_NARROW=1): rounds
    whose values lie within 2^32 ulps of each other stage u32 offsets instead of 8-byte values.  Not
    the headline: cfg4's own ε = 1e-6 run ends at round 14, before any round narrows, so the gain is
    a property of long FIXED or tight-ε runs.  Timed like the headline (rounds 10-110; the spread
    falls below 2^32 ulps after about round 15), priced at the same 400 B unit, and a fresh narrow
    handle's 100 FIXED rounds are checked against the oracle's hash."""
    import acsim
    from acsim.digest import sha256_values
    old = os.environ.get("ACSIM_BIN_NARROW")
    os.environ["ACSIM_BIN_NARROW"] = "1"
    try:
        cfg = acsim.preset("cfg4", max_rounds=warm + timed, instance_offset=ctx.rank)
        with acsim.Simulator(cfg, device=ctx.dev) as sim:
            sim.round(warm)
            sim.set_kernel_timing(True, every=25, runs=True)
            ctx.barrier(sim)
            t0 = time.perf_counter()
            sim.round(timed)
            ctx.barrier(sim)
            dt = ctx.max(time.perf_counter() - t0)
            k_ms, k_n, kname = sim.kernel_timing()
        n = int(cfg.n_nodes)
        avg_s = (k_ms / 1e3 / k_n) if k_n else dt / timed
        out = {}
        if ctx.rank == 0:
            with acsim.Simulator(acsim.preset("cfg4", max_rounds=100), device=ctx.dev) as chk:
                chk.run()
                ok = sha256_values(chk.values(0)) == golden().get("cfg4", {}).get("fixed100_x_sha256")
            achieved = BYTES_PER_NODE_ROUND * n / avg_s / 1e9
            out = {"workload": "cfg4 (the headline workload, rounds 10-110) on the opt-in narrow plan "
                               "(ACSIM_BIN_NARROW=1, DESIGN.md §5.15): not the headline",
                   "value": ctx.world * n * timed / dt, "unit": "node-rounds/s", "ms_per_step": dt / timed * 1e3,
                   "dtype": "f64", "kernel": kname, "avg_launch_us": avg_s * 1e6,
                   "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": achieved / HBM_PEAK_GBS, "bytes_per_node_round": BYTES_PER_NODE_ROUND,
                                "note": "priced at the spec's 400 B unit; the 4-byte rounds move fewer bytes "
                                        "than the unit (DESIGN.md §5.15)"},
                   "golden_match": ok}
        return out
    finally:
        if old is None:
            os.environ.pop("ACSIM_BIN_NARROW", None)
        else:
            os.environ["ACSIM_BIN_NARROW"] = old


LEGS = {"cfg3": ("cfg3_sharded", leg_cfg3), "cfg5": ("cfg5_partitioned", leg_cfg5),
        "f32": ("cfg4_f32", leg_cfg4_f32), "narrow": ("cfg4_narrow", leg_cfg4_narrow)}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    group = None
    ndev = 1
    import acsim
    if world > 1:
        # torch-free control plane (acsim/rendezvous.py): importing torch here would map torch's
        # own HIP runtime and RCCL before libacsim.so and bind the library to them
        from acsim.rendezvous import Group
        group = Group.from_env()
        ndev = max(1, acsim._abi.device_count())
        if world > ndev and not a.allow_shared_device:
            raise SystemExit(f"{world} ranks but {ndev} GPU(s): one rank per GPU (--allow-shared-device "
                             f"for a rehearsal that is not a scaling result)")

    dev = local_rank % ndev
    ctx = Ctx(world, rank, local_rank, dev, group)
    n = a.n_nodes
    cfg = acsim.preset("cfg4", n_nodes=n, max_rounds=a.warmup + a.steps, instance_offset=rank,
                       dtype=a.dtype)
    sim = acsim.Simulator(cfg, device=dev)

    if a.warmup:
        sim.round(a.warmup)
    sim.set_kernel_timing(not a.no_event_timing, every=a.event_run, runs=True)
    ctx.barrier(sim)
    t0 = time.perf_counter()
    sim.round(a.steps)
    ctx.barrier(sim)
    dt = time.perf_counter() - t0
    dt_local = dt
    k_ms, k_n, kname = sim.kernel_timing()
    sim.set_kernel_timing(False)
    rounds = int(sim.rounds()[0])
    assert rounds == a.warmup + a.steps, (rounds, a.warmup, a.steps)
    dt = ctx.max(dt)
    sim.close()
    headline_check = None
    if rank == 0 and a.dtype == "f64" and n == 1 << 20:
        # the bench workload's kernels, run for exactly 100 rounds on a fresh handle (untimed),
        # against the oracle's result (tests/golden/fullsize.json)
        from acsim.digest import sha256_values
        with acsim.Simulator(acsim.preset("cfg4", max_rounds=100), device=dev) as chk:
            chk.run()
            headline_check = sha256_values(chk.values(0)) == golden().get("cfg4", {}).get("fixed100_x_sha256")

    value = world * n * a.steps / dt
    avg_launch_s = (k_ms / 1e3 / k_n) if k_n else dt / a.steps
    unit_b = BYTES_PER_NODE_ROUND_F32 if a.dtype == "f32" else BYTES_PER_NODE_ROUND
    achieved = unit_b * n / avg_launch_s / 1e9
    n_gpus = min(world, ndev)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "node-rounds/s",
        "n_gpus": n_gpus,
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
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": kname, "avg_launch_us": avg_launch_s * 1e6,
                     "launch": "one round (k_bin_scatter + k_bin_gather and their boundaries), device "
                               f"time over runs of {a.event_run} consecutive rounds",
                     "bytes_per_node_round": unit_b},
        "hbm_roofline_pct_wall": 100.0 * unit_b * value / n_gpus / 1e9 / HBM_PEAK_GBS,
        "cpu_baseline": None,
        "parity": {"golden_match": headline_check,
                   "what": "cfg4 run for 100 FIXED rounds on a fresh handle after the timed region: "
                           "sha256(x) equals the oracle's (tests/golden/fullsize.json "
                           "cfg4.fixed100_x_sha256); null for other shapes (--dtype f32, --n-nodes)"},
    }
    if world > ndev:
        # rehearsal: several ranks time replicas on one card; no aggregate is a throughput result
        out["shared_device"] = True
        out["ranks"] = world
        out["rank_values"] = ctx.gather(n * a.steps / dt_local)
        out["value"] = None
        out["hbm_roofline_pct_wall"] = None
    # which HIP runtime / RCCL each rank runs on (the N = 1 line records the same for comparison)
    rt = ctx.gather(acsim._abi.runtime_info())
    out["runtime"] = {"rank0": rt[0], "all_ranks_same": all(r == rt[0] for r in rt)}
    if rank == 0:
        out["roofline"]["traffic"] = load_pmc(kname, n, a.dtype)

    # --- extra legs, guarded; the watchdog prints the line if one hangs (another rank died in a
    # collective, a communicator never forms ...)
    lock = threading.Lock()
    printed = [False]

    def emit(note=None):
        with lock:
            if printed[0] or rank != 0:
                return
            if note:
                out["legs_note"] = note
            print(json.dumps(out), flush=True)
            printed[0] = True

    legs = [s for s in a.legs.split(",") if s]
    failed = []
    if legs:
        def watchdog():
            # the headline line is printed (with every leg and sub-leg finished so far), but the run
            # must not look clean: exit non-zero
            out["legs_failed"] = failed + [ctx.stage]
            emit(f"watchdog: {ctx.stage} unfinished after {a.leg_timeout:.0f} s")
            os._exit(3)
        timer = threading.Timer(a.leg_timeout, watchdog)
        timer.daemon = True
        timer.start()
        for name in legs:
            key, fn = LEGS[name]
            ctx.enter(key)
            ctx.partial = {"running": True}
            if rank == 0:
                out[key] = ctx.partial   # (replaced by the result; a hang prints what exists)
            try:
                res = fn(ctx)
            except Exception as e:  # noqa: BLE001
                res = {"error": f"{type(e).__name__}: {e}"}
            if rank == 0:
                out[key] = res
                if "error" in res or res.get("golden_match") is False or res.get("ok") is False:
                    failed.append(key)
        timer.cancel()
        ctx.stage = "cpu_baseline"
    if rank == 0:
        out["legs_failed"] = failed
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(n, a.cpu_seconds, a.dtype)
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = None
            out["cpu_baseline_error"] = f"{type(e).__name__}: {e}"
    emit()
    if group is not None:
        group.barrier()
        group.close()
    if failed:   # reported in the line above; the process must not look clean (no retry, no re-launch)
        sys.exit(4)


if __name__ == "__main__":
    main()
