"""Property-based differential tests over the whole configuration space (SURVEY §4 rows L0 and L2,
hypothesis).  The fixed-case tests pin chosen corners; these draw random small configurations —
topology, degree, rule and trim, fault model and strategy, loss, delay, missing policy, instances,
dtype, termination, seeds — and check:

  CPU  the C oracle against the independent numpy restatement, bit for bit (rounds, every value,
       every spread trace), and two semantic properties of the rules:
         validity     without Byzantine senders every value stays inside the hull of x^0 (up to
                      the rounding of one mean: a few ulps),
         contraction  without faults and delays the honest spread never grows (same tolerance;
                      with delays only the hull of the last D+1 rounds contracts);
  GPU  the HIP path (libacsim.so, through the C ABI) against the oracle on the same draws, bit for
       bit (every draw avoids the MFMA path, whose bar is 1e-12).

Draws are derandomized (a fixed example sequence), so a failure reproduces; the failing Config is
printed by hypothesis.  Parity is against the frozen spec (no upstream code exists).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import spec_np as S
from acsim.config import Config


@st.composite
def configs(draw, max_n=160):
    """A valid small Config (acs_create's admission rules, include/acsim.h)."""
    topo = draw(st.sampled_from(["complete", "random_regular"]))
    if topo == "complete":
        # batched (N <= 64), dense persistent (Byzantine SPLIT / CONSTANT or clean) and generic
        # (loss / crash / RANDOM above 64 nodes) kernels
        n = draw(st.one_of(st.integers(3, 40), st.integers(41, 300)))
        d = 0
        m = n
    else:
        n = draw(st.integers(8, max_n))
        d = draw(st.sampled_from([2, 4, 6, 8, 12, 16]))
        m = d + 1
    rule = draw(st.sampled_from(["average", "trimmed", "midpoint", "dlpsw", "wmsr"]))
    tmax = (m - 1) // 2
    if rule == "average":
        t = 0
    elif rule == "dlpsw":
        if tmax < 1:
            rule, t = "trimmed", 0
        else:
            t = draw(st.integers(1, tmax))
    else:
        t = draw(st.integers(0, tmax))
    fault = draw(st.sampled_from(["none", "none", "crash", "byzantine"]))
    kw = {}
    if fault != "none":
        kw["n_faulty"] = draw(st.integers(1, max(1, n // 4)))
    if fault == "crash":
        kw["crash_window"] = draw(st.integers(1, 6))
    if fault == "byzantine":
        kw["byz_strategy"] = draw(st.sampled_from(["split", "random", "constant"]))
        kw["byz_delta"] = draw(st.sampled_from([0.0, 0.05, 0.5]))
        kw["byz_const"] = draw(st.sampled_from([0.0, -2.0, 7.5]))
    dtype = draw(st.sampled_from(["f64", "f64", "f32"]))
    term = draw(st.sampled_from(["eps", "fixed"]))
    return Config(
        n_nodes=n, n_instances=draw(st.integers(1, 3)), topology=topo, degree=d, rule=rule, trim=t,
        fault_model=fault, loss_p=draw(st.sampled_from([0.0, 0.0, 0.1, 0.35])),
        mask_group=draw(st.sampled_from([1, 1, 2])), eps=draw(st.sampled_from([1e-4, 1e-7, 1e-10])),
        max_rounds=draw(st.integers(1, 60)), termination=term, dtype=dtype,
        seed=draw(st.integers(0, 2 ** 40)), graph_seed=draw(st.sampled_from([0, 0, 5])),
        trace_spread=True, instance_offset=draw(st.sampled_from([0, 0, 1000])),
        delay_max=draw(st.sampled_from([0, 0, 0, 1, 3])),
        missing_policy=draw(st.sampled_from(["self", "self", "omit"])), **kw)


@st.composite
def csr_configs(draw, max_n=300):
    """A user graph (ACS_TOPO_CSR, §8(f) row 1) with random degrees and senders, and a valid
    Config for it: (cfg, (rowptr, colidx))."""
    n = draw(st.integers(8, max_n))
    dmin = draw(st.integers(0, 12))   # 0: rows without senders (m_i = 1)
    dmax = dmin + draw(st.sampled_from([0, 3, 20, 60]))
    rng = np.random.default_rng(draw(st.integers(0, 2 ** 32)))
    deg = rng.integers(dmin, dmax + 1, size=n)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
    colidx = rng.integers(0, n, size=int(rowptr[-1])).astype(np.uint32)
    base = draw(configs())
    tmax = dmin // 2   # m_i = deg(i) + 1 > 2t for every row
    rule = base.rule
    t = 0 if rule == "average" else draw(st.integers(1 if rule == "dlpsw" else 0, max(tmax, 1)))
    if t > tmax:
        rule, t = "average", 0
    cfg = base.replace(topology="csr", n_nodes=n, degree=0, rule=rule, trim=t,
                       n_faulty=min(base.n_faulty, n - 1))
    return cfg, (rowptr, colidx)


def _run_oracle(oracle_mod, cfg, csr=None):
    with oracle_mod.OracleSimulator(cfg, csr=csr) as o:
        o.run()
        return dict(rounds=o.rounds(), x=o.all_values(), status=o.fault_status(),
                    trace=[o.spread_trace(b) for b in range(cfg.n_instances)])


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32 if a.dtype == np.float32 else np.uint64)


CPU_SETTINGS = settings(max_examples=150, deadline=None, derandomize=True, database=None,
                        suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


@CPU_SETTINGS
@given(cfg=configs())
def test_oracle_matches_numpy_random_configs(oracle_mod, cfg):
    o = _run_oracle(oracle_mod, cfg)
    n = S.NpSim(cfg)
    n.run()
    assert np.array_equal(o["rounds"], n.rounds), cfg
    assert np.array_equal(_bits(o["x"]), _bits(n.x)), cfg
    for b in range(cfg.n_instances):
        assert np.array_equal(_bits(o["trace"][b]), _bits(np.array(n.trace[b]))), (cfg, b)


@settings(CPU_SETTINGS, max_examples=25)   # the numpy CSR restatement loops per row
@given(case=csr_configs(max_n=120))
def test_oracle_matches_numpy_random_csr(oracle_mod, case):
    cfg, csr = case
    o = _run_oracle(oracle_mod, cfg, csr)
    n = S.NpSim(cfg, csr=csr)
    n.run()
    assert np.array_equal(o["rounds"], n.rounds), cfg
    assert np.array_equal(_bits(o["x"]), _bits(n.x)), cfg
    for b in range(cfg.n_instances):
        assert np.array_equal(_bits(o["trace"][b]), _bits(np.array(n.trace[b]))), (cfg, b)


def _x0(oracle_mod, cfg):
    with oracle_mod.OracleSimulator(cfg.replace(max_rounds=1, termination="fixed")) as o:
        o.round(0)
        return o.all_values()


@CPU_SETTINGS
@given(cfg=configs())
def test_validity_and_contraction(oracle_mod, cfg):
    if cfg.fault_model == "byzantine":
        return   # Byzantine values may lie outside the hull by design (§A.4)
    x0 = _x0(oracle_mod, cfg).astype(np.float64)
    o = _run_oracle(oracle_mod, cfg)
    ulp = np.float64(np.finfo(np.float32 if cfg.dtype == "f32" else np.float64).eps)
    for b in range(cfg.n_instances):
        lo, hi = x0[b].min(), x0[b].max()
        tol = 8 * ulp * max(abs(lo), abs(hi), 1.0)
        xb = o["x"][b].astype(np.float64)
        assert xb.min() >= lo - tol and xb.max() <= hi + tol, (cfg, b)
        if cfg.fault_model == "none" and cfg.delay_max == 0:
            tr = np.asarray(o["trace"][b], dtype=np.float64)
            assert np.all(np.diff(tr) <= tol), (cfg, b, tr)


@pytest.mark.gpu
@settings(max_examples=300, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=configs(max_n=400))
def test_gpu_matches_oracle_random_configs(oracle_mod, cfg):
    import acsim
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        gr, gx, gs = g.rounds(), g.all_values(), g.fault_status()
        gt = [g.spread_trace(b) for b in range(cfg.n_instances)]
    o = _run_oracle(oracle_mod, cfg)
    assert np.array_equal(gr, o["rounds"]), cfg
    assert np.array_equal(gs, o["status"]), cfg
    assert np.array_equal(_bits(gx), _bits(o["x"])), cfg
    for b in range(cfg.n_instances):
        assert np.array_equal(_bits(gt[b]), _bits(o["trace"][b])), (cfg, b)


@pytest.mark.gpu
@settings(max_examples=200, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(case=csr_configs(max_n=600))
def test_gpu_matches_oracle_random_csr(oracle_mod, case):
    import acsim
    cfg, csr = case
    with acsim.Simulator(cfg, device=0, csr=csr) as g:
        g.run()
        gr, gx = g.rounds(), g.all_values()
        gt = [g.spread_trace(b) for b in range(cfg.n_instances)]
    o = _run_oracle(oracle_mod, cfg, csr)
    assert np.array_equal(gr, o["rounds"]), cfg
    assert np.array_equal(_bits(gx), _bits(o["x"])), cfg
    for b in range(cfg.n_instances):
        assert np.array_equal(_bits(gt[b]), _bits(o["trace"][b])), (cfg, b)


@st.composite
def binned_configs(draw):
    """One-instance RANDOM_REGULAR configs the binned exchange serves (compiled (d, t) pairs, no
    delays), at sizes that span many source blocks when ACSIM_BIN_SA shrinks them: one-level and
    two-level (phase-M) plans, ragged last blocks, clean / lossy / crash / Byzantine senders, every
    sort-based rule and AVERAGE, fp64 and fp32, SELF and OMIT.  -> (cfg, source block size)"""
    d, t = draw(st.sampled_from([(8, 0), (8, 2), (16, 0), (16, 5), (32, 0), (32, 5)]))
    rule = draw(st.sampled_from(["trimmed", "midpoint", "wmsr", "dlpsw"] if t else
                                ["average", "trimmed", "midpoint"]))
    fault = draw(st.sampled_from(["none", "none", "crash", "byzantine"]))
    n = draw(st.integers(3000, 120000))
    kw = {}
    if fault != "none":
        kw["n_faulty"] = draw(st.integers(1, n // 50))
    if fault == "crash":
        kw["crash_window"] = draw(st.integers(1, 6))
    if fault == "byzantine":
        kw["byz_strategy"] = draw(st.sampled_from(["split", "random", "constant"]))
        kw["byz_delta"] = draw(st.sampled_from([0.0, 0.05]))
        kw["byz_const"] = draw(st.sampled_from([0.0, 3.0]))
    cfg = Config(n_nodes=n, topology="random_regular", degree=d, rule=rule, trim=t, fault_model=fault,
                 loss_p=draw(st.sampled_from([0.0, 0.0, 0.1])), eps=draw(st.sampled_from([1e-7, 1e-10])),
                 max_rounds=draw(st.integers(1, 40)), termination=draw(st.sampled_from(["eps", "fixed"])),
                 dtype=draw(st.sampled_from(["f64", "f64", "f32"])), seed=draw(st.integers(0, 2 ** 40)),
                 trace_spread=True, missing_policy=draw(st.sampled_from(["self", "self", "omit"])), **kw)
    return cfg, draw(st.sampled_from([256, 512, 1024, 4096]))


@st.composite
def dense_configs(draw, max_n=600):
    """Complete graphs the persistent dense kernel serves (round_dense.hip: 65 .. 4096 nodes, clean
    or Byzantine SPLIT / CONSTANT, no loss, no crash, no delays; the sort-based rules): windows of
    64 .. 512 slots, one or two Byzantine classes, fp64 and fp32."""
    base = draw(configs())
    n = draw(st.integers(65, max_n))
    rule = draw(st.sampled_from(["trimmed", "midpoint", "dlpsw"]))   # (AVERAGE / W-MSR: other kernels)
    tmax = (n - 1) // 2
    t = draw(st.integers(1 if rule == "dlpsw" else 0, tmax))
    fault = draw(st.sampled_from(["none", "byzantine", "byzantine"]))
    kw = dict(fault_model=fault, n_faulty=0)
    if fault == "byzantine":
        kw.update(n_faulty=draw(st.integers(1, max(1, n // 3))),
                  byz_strategy=draw(st.sampled_from(["split", "constant"])))
    return base.replace(topology="complete", n_nodes=n, degree=0, rule=rule, trim=t, loss_p=0.0,
                        delay_max=0, missing_policy="self", n_instances=draw(st.integers(1, 2)),
                        max_rounds=min(base.max_rounds, 40), **kw)


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=dense_configs())
def test_gpu_dense_random_configs(oracle_mod, cfg):
    """The persistent dense kernel (one workgroup per instance, class windows with permlane / DPP
    tree sums) against the oracle."""
    import acsim
    with acsim.Simulator(cfg, device=0) as g:
        name = g.kernel_name()
        g.run()
        gr, gx = g.rounds(), g.all_values()
        gt = [g.spread_trace(b) for b in range(cfg.n_instances)]
    assert "k_dense_persist" in name, (cfg, name)   # the draw must land on the dense kernel
    o = _run_oracle(oracle_mod, cfg.replace(omp_threads=16))
    assert np.array_equal(gr, o["rounds"]), (cfg, name)
    assert np.array_equal(_bits(gx), _bits(o["x"])), (cfg, name)
    for b in range(cfg.n_instances):
        assert np.array_equal(_bits(gt[b]), _bits(o["trace"][b])), (cfg, b)


@pytest.mark.gpu
@settings(max_examples=120, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(case=binned_configs())
def test_gpu_binned_exchange_random_configs(oracle_mod, case):
    """The binned exchange (round_binned.hip) with small source blocks against the oracle."""
    import os
    import acsim
    cfg, sa = case
    old = os.environ.get("ACSIM_BIN_SA")
    os.environ["ACSIM_BIN_SA"] = str(sa)
    try:
        with acsim.Simulator(cfg, device=0) as g:
            name = g.kernel_name()
            g.run()
            gr, gx, gt = g.rounds(), g.values(0), g.spread_trace(0)
    finally:
        if old is None:
            os.environ.pop("ACSIM_BIN_SA", None)
        else:
            os.environ["ACSIM_BIN_SA"] = old
    assert "k_bin_" in name, (cfg, sa, name)   # the draw must land on the binned exchange
    o = _run_oracle(oracle_mod, cfg.replace(omp_threads=16))
    assert np.array_equal(gr, o["rounds"]), (cfg, sa, name)
    assert np.array_equal(_bits(gx), _bits(o["x"][0])), (cfg, sa, name)
    assert np.array_equal(_bits(gt), _bits(o["trace"][0])), (cfg, sa, name)


@st.composite
def block_size_cases(draw):
    """Clean binned plans on a phase-B receiver block other than 256 (round 6):
    t = 5, d = 16 / 32, the sort-based rules that take it, fp64 / fp32, one or two passes, one-
    and two-level plans, and sometimes 2-4 virtual partitions with or without the chunked
    exchange.  -> (cfg, source block size, receiver block, passes, partitions, chunks)"""
    d = draw(st.sampled_from([16, 32]))
    sb = draw(st.sampled_from([128, 512] if d == 16 else [128]))
    cfg = Config(n_nodes=draw(st.integers(3000, 120000)), topology="random_regular", degree=d,
                 rule=draw(st.sampled_from(["trimmed", "midpoint", "dlpsw"])), trim=5,
                 eps=draw(st.sampled_from([1e-7, 1e-10])), max_rounds=draw(st.integers(1, 40)),
                 termination=draw(st.sampled_from(["eps", "fixed"])),
                 dtype=draw(st.sampled_from(["f64", "f64", "f32"])), seed=draw(st.integers(0, 2 ** 40)),
                 trace_spread=True)
    parts = draw(st.sampled_from([1, 1, 2, 3, 4]))
    return (cfg, draw(st.sampled_from([512, 1024, 4096])), sb, draw(st.sampled_from(["", "1", "2"])), parts,
            draw(st.sampled_from(["0", "2", "4"])))


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(case=block_size_cases())
def test_gpu_binned_block_size_random_configs(oracle_mod, case):
    """The binned exchange on 128 / 512-receiver phase-B blocks, whole and node-partitioned,
    against the oracle bit for bit (every private copy of x under partitions)."""
    import os
    import acsim
    cfg, sa, sb, split, parts, xchunks = case
    env = {"ACSIM_BIN_SA": str(sa), "ACSIM_BIN_SB": str(sb), "ACSIM_BIN_SPLIT": split, "ACSIM_XCHUNKS": xchunks}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    try:
        with acsim.Simulator(cfg, device=0, partitions=parts) as g:
            name = g.kernel_name()
            g.run()
            gr, gt = g.rounds(), g.spread_trace(0)
            copies = [g.partition_values(q) for q in range(parts)] if parts > 1 else [g.values(0)]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert "k_bin_" in name and f" sb{sb}" in name, (cfg, sa, sb, name)
    o = _run_oracle(oracle_mod, cfg.replace(omp_threads=16))
    assert np.array_equal(gr, o["rounds"]), (cfg, sa, sb, split, parts, name)
    assert np.array_equal(_bits(gt), _bits(o["trace"][0])), (cfg, sa, sb, split, parts, name)
    for q, x in enumerate(copies):
        assert np.array_equal(_bits(x), _bits(o["x"][0])), (cfg, sa, sb, split, parts, q, name)


@st.composite
def narrow_cases(draw):
    """Opt-in narrow plans (ACSIM_BIN_NARROW=1): clean one-level fp64 plans of
    d = 16 / 32 and every rule with a compiled (d, t) pair, FIXED runs long enough to reach the
    4-byte rounds or EPS to a tight ε, one or two phase-B passes in the 8-byte rounds, initial
    values shifted by draw (positive, negative, straddling zero, tiny).  -> (cfg, SA, passes, shift)"""
    d = draw(st.sampled_from([16, 32]))
    t = draw(st.sampled_from([5, 0]))
    rule = draw(st.sampled_from(["trimmed", "midpoint", "dlpsw", "wmsr"] if t else ["average", "midpoint"]))
    term = draw(st.sampled_from(["fixed", "fixed", "eps"]))
    cfg = Config(n_nodes=draw(st.integers(3000, 90000)), topology="random_regular", degree=d, rule=rule, trim=t,
                 eps=draw(st.sampled_from([1e-11, 1e-13])), max_rounds=draw(st.integers(30, 70)),
                 termination=term, seed=draw(st.integers(0, 2 ** 40)), trace_spread=True)
    return (cfg, draw(st.sampled_from([512, 1024, 2048, 4096, 16384])), draw(st.sampled_from(["", "1", "2"])),
            draw(st.sampled_from(["none", "none", "negative", "straddle", "tiny"])))


@pytest.mark.gpu
@settings(max_examples=120, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(case=narrow_cases())
def test_gpu_narrow_random_configs(oracle_mod, case):
    """Narrow plans against the oracle bit for bit: rounds, spread trace, final values (every
    round, whatever stage width it took)."""
    import os
    import acsim
    cfg, sa, split, shift = case
    env = {"ACSIM_BIN_NARROW": "1", "ACSIM_BIN_SA": str(sa), "ACSIM_BIN_SPLIT": split}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    try:
        with acsim.Simulator(cfg, device=0) as g:
            name = g.kernel_name()
            x0 = g.values(0).copy()
            state = None
            if shift != "none":
                x = {"negative": -1.5 - x0, "straddle": x0 - 0.5, "tiny": x0 * 1e-300}[shift]
                state = (0, x[None, :])
                g.set_state(*state)
            g.run()
            gr, gt, gx = g.rounds(), g.spread_trace(0), g.values(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert "k_bin_" in name, (cfg, sa, name)
    with oracle_mod.OracleSimulator(cfg.replace(omp_threads=16)) as o:
        if state is not None:
            o.set_state(*state)
        o.run()
        orr, ot, ox = o.rounds(), o.spread_trace(0), o.values(0)
    assert np.array_equal(gr, orr), (cfg, sa, split, shift, name)
    assert np.array_equal(_bits(gt), _bits(ot)), (cfg, sa, split, shift, name)
    assert np.array_equal(_bits(gx), _bits(ox)), (cfg, sa, split, shift, name)


@st.composite
def partition_cases(draw):
    """Node-partitioned runs (SURVEY §8(e), cfg5's data flow) on virtual partitions: a binned or
    per-lane config, 2-8 row blocks, the chunked or the all-gather exchange, small source blocks."""
    cfg, sa = draw(binned_configs())
    if draw(st.booleans()):   # also the per-lane kernel's partitioned path: (4, 0) / (4, 1) have
        t = draw(st.sampled_from([0, 1]))   # compiled register variants but no binned plan
        rule = draw(st.sampled_from(["trimmed", "midpoint", "wmsr", "dlpsw"] if t else
                                    ["average", "trimmed", "midpoint"]))
        cfg = cfg.replace(degree=4, trim=t, rule=rule)
    return cfg, sa, draw(st.integers(2, 8)), draw(st.sampled_from(["0", "2", "4"]))


@pytest.mark.gpu
@settings(max_examples=100, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(case=partition_cases())
def test_gpu_virtual_partitions_random_configs(oracle_mod, case):
    """Every private copy of x equals the oracle's unpartitioned run, bit for bit."""
    import os
    import acsim
    cfg, sa, parts, xchunks = case
    old = {k: os.environ.get(k) for k in ("ACSIM_BIN_SA", "ACSIM_XCHUNKS")}
    os.environ["ACSIM_BIN_SA"] = str(sa)
    os.environ["ACSIM_XCHUNKS"] = xchunks
    try:
        with acsim.Simulator(cfg, partitions=parts) as p:
            p.run()
            pr, pt = p.rounds(), p.spread_trace(0)
            copies = [p.partition_values(q) for q in range(parts)]
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    o = _run_oracle(oracle_mod, cfg.replace(omp_threads=16))
    assert np.array_equal(pr, o["rounds"]), (cfg, sa, parts, xchunks)
    assert np.array_equal(_bits(pt), _bits(o["trace"][0])), (cfg, sa, parts, xchunks)
    for q, x in enumerate(copies):
        assert np.array_equal(_bits(x), _bits(o["x"][0])), (cfg, sa, parts, xchunks, q)


@pytest.mark.gpu
@settings(max_examples=150, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=configs(max_n=300), frac=st.floats(0.0, 1.0))
def test_gpu_resume_random_configs(oracle_mod, cfg, frac):
    """Checkpoint / resume: rounds stopped at r0, the values read back and set into a
    fresh handle with acs_set_state(r0, x^r0), then run to the end, equal the oracle's straight
    run bit for bit (synchronous rounds: with delays set_state restarts the history by design)."""
    import acsim
    cfg = cfg.replace(delay_max=0)
    o = _run_oracle(oracle_mod, cfg)
    r0 = int(frac * int(o["rounds"].min()))
    with acsim.Simulator(cfg, device=0) as a:
        a.round(r0)
        xr = a.all_values()
    with acsim.Simulator(cfg, device=0) as b:
        b.set_state(r0, xr)
        b.run()
        br, bx = b.rounds(), b.all_values()
    assert np.array_equal(br, o["rounds"]), (cfg, r0)
    assert np.array_equal(_bits(bx), _bits(o["x"])), (cfg, r0)


@pytest.mark.gpu
@settings(max_examples=100, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=configs(max_n=300), steps=st.lists(st.integers(1, 17), min_size=1, max_size=6))
def test_gpu_round_steps_equal_run(cfg, steps):
    """Simulator.round(k) in arbitrary steps (the chunked enqueue loop, EPS polling, deferred
    finalize across calls) ends exactly where one run() does."""
    import acsim
    with acsim.Simulator(cfg, device=0) as a:
        a.run()
        ar, ax = a.rounds(), a.all_values()
        at = [a.spread_trace(b) for b in range(cfg.n_instances)]
    with acsim.Simulator(cfg, device=0) as b:
        k = 0
        while True:
            info = b.round(steps[k % len(steps)])
            k += 1
            if info.done or k > 10_000:
                break
        br, bx = b.rounds(), b.all_values()
        bt = [b.spread_trace(i) for i in range(cfg.n_instances)]
    assert np.array_equal(br, ar), (cfg, steps)
    assert np.array_equal(_bits(bx), _bits(ax)), (cfg, steps)
    for i in range(cfg.n_instances):
        assert np.array_equal(_bits(bt[i]), _bits(at[i])), (cfg, steps, i)


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(cfg=configs(max_n=200), cut=st.integers(1, 7))
def test_gpu_instance_shards_equal_batch(cfg, cut):
    """instances are seeded by their global id, so any split of a batch into
    instance_offset windows (one per rank) reproduces the batch exactly."""
    import acsim
    B = 8
    cfg = cfg.replace(n_instances=B)
    with acsim.Simulator(cfg, device=0) as a:
        a.run()
        ar, ax = a.rounds(), a.all_values()
    parts = [(0, cut), (cut, B - cut)]
    for off, cnt in parts:
        sub = cfg.replace(n_instances=cnt, instance_offset=int(cfg.instance_offset) + off)
        with acsim.Simulator(sub, device=0) as s:
            s.run()
            assert np.array_equal(s.rounds(), ar[off:off + cnt]), (cfg, cut)
            assert np.array_equal(_bits(s.all_values()), _bits(ax[off:off + cnt])), (cfg, cut)
