"""Size limits lifted in round 3.

- Fault schedules of any B·N: the segmented sort of the §A.4 fault keys runs in instance batches
  (setup.hip build_fault_status).  The forced multi-batch schedule against the oracle, and a
  B·N > 2^31 batch whose sampled instances (fault set, x after two rounds) match the oracle run of
  that instance alone (instance_offset = its global id, SURVEY §A.1 counters).
- Receivers with more than 8192 entries (complete graphs above 8192 nodes, CSR hubs): the big-m
  generic path (round_generic.hip: global scratch, segmented radix sort, global stride-halving
  sums), bit-exact against the oracle for every rule, OMIT, fp32, delay and several instances, with
  forced small batches (ACSIM_BIG_CAP) as well.
"""
import contextlib
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config


@contextlib.contextmanager
def env(**kw):
    old = {k: os.environ.get(k) for k in kw}
    os.environ.update({k: str(v) for k, v in kw.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3, 7])
def test_fault_schedule_batches_match_oracle(oracle_mod, batch):
    cfg = Config(n_nodes=1000, n_instances=10, topology="regular", degree=8, rule="trimmed", trim=2,
                 fault_model="crash", n_faulty=120, crash_window=4, loss_p=0.1, eps=1e-9, max_rounds=40,
                 seed=23, instance_offset=5)
    with env(ACSIM_FAULT_BATCH=batch), acsim.Simulator(cfg, device=0) as g:
        g.run()
        st, r, x = g.fault_status(), g.rounds(), g.all_values()
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.fault_status(), st)
        assert np.array_equal(o.rounds(), r)
        assert np.array_equal(bits(o.all_values()), bits(x))


@pytest.mark.gpu
def test_fault_schedule_above_2e31(oracle_mod):
    """B·N = 32 769 · 2^16 > 2^31 (34 GiB of values on the device): byzantine + crash-free RANDOM
    senders on a 4-regular graph, two FIXED rounds on the per-lane kernel."""
    N, B = 1 << 16, 32769
    assert B * N > 2 ** 31
    cfg = Config(n_nodes=N, n_instances=B, topology="regular", degree=4, rule="trimmed", trim=1,
                 fault_model="byzantine", n_faulty=300, byz_strategy="random", byz_delta=0.05,
                 termination="fixed", max_rounds=2, seed=29)
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        assert int(g.rounds().min()) == 2
        st = g.fault_status()
        assert st.shape == (B, N)
        samples = [0, 1, 20000, B - 1]
        got = {b: (st[b].copy(), g.values(b)) for b in samples}
        # every instance has exactly n_faulty Byzantine nodes
        nbyz = (st == 0xFFFFFFFE).sum(axis=1)
        assert np.all(nbyz == 300)
        del st
    for b in samples:
        one = cfg.replace(n_instances=1, instance_offset=b)
        with oracle_mod.OracleSimulator(one, threads=8) as o:
            o.run()
            assert np.array_equal(o.fault_status().reshape(-1), got[b][0]), b
            assert np.array_equal(bits(o.values(0)), bits(got[b][1])), b


def gpu_vs_oracle(oracle_mod, cfg, csr=None, **envs):
    with env(**envs), acsim.Simulator(cfg, device=0, csr=csr) as g:
        kname = g.kernel_name()
        g.run()
        r, x = g.rounds(), g.all_values()
    with oracle_mod.OracleSimulator(cfg, threads=8, csr=csr) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        xo = o.all_values()
    xv = np.ascontiguousarray(x)
    view = np.uint64 if xv.dtype == np.float64 else np.uint32
    assert np.array_equal(np.ascontiguousarray(xo).view(view), xv.view(view))
    return kname


BIG = dict(n_nodes=8300, topology="complete", termination="fixed", max_rounds=2, seed=31)
BIG_CASES = {
    "avg_loss": dict(rule="average", trim=0, loss_p=0.3),
    "trimmed_crash_loss": dict(rule="trimmed", trim=100, loss_p=0.3, fault_model="crash", n_faulty=400, crash_window=2),
    "midpoint_byz_random": dict(rule="midpoint", trim=300, fault_model="byzantine", n_faulty=300,
                                byz_strategy="random", byz_delta=0.2),
    "dlpsw_loss": dict(rule="dlpsw", trim=7, loss_p=0.25),
    "wmsr_crash": dict(rule="wmsr", trim=50, fault_model="crash", n_faulty=200, crash_window=3, loss_p=0.1),
    "trimmed_omit": dict(rule="trimmed", trim=40, loss_p=0.4, fault_model="crash", n_faulty=300, crash_window=2,
                         missing_policy="omit"),
    "avg_omit": dict(rule="average", trim=0, loss_p=0.4, missing_policy="omit"),
    "f32_trimmed": dict(rule="trimmed", trim=60, loss_p=0.2, dtype="f32"),
    "delay_trimmed": dict(rule="trimmed", trim=30, loss_p=0.1, delay_max=2, max_rounds=4),
    "instances_avg": dict(rule="average", trim=0, loss_p=0.3, n_instances=3, instance_offset=2),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(BIG_CASES))
def test_big_m_complete_matches_oracle(oracle_mod, name):
    cfg = Config(**{**BIG, **BIG_CASES[name]})
    kname = gpu_vs_oracle(oracle_mod, cfg)
    assert kname.startswith("k_big_resolve"), kname


@pytest.mark.gpu
def test_big_m_forced_batches(oracle_mod):
    cfg = Config(**{**BIG, **BIG_CASES["trimmed_crash_loss"]})
    gpu_vs_oracle(oracle_mod, cfg, ACSIM_BIG_CAP=3 * 8300 + 17)   # 3 receivers per batch


def hub_csr(n, hubs, seed):
    """A CSR graph whose rows have 6..20 entries, except `hubs` rows of 8500..12000 entries."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(6, 21, size=n)
    hub_rows = rng.choice(n, size=hubs, replace=False)
    deg[hub_rows] = rng.integers(8500, 12001, size=hubs)
    rowptr = np.zeros(n + 1, dtype=np.uint64)
    rowptr[1:] = np.cumsum(deg)
    colidx = rng.integers(0, n, size=int(rowptr[-1])).astype(np.uint32)
    return rowptr, colidx


@pytest.mark.gpu
@pytest.mark.parametrize("rule,t", [("trimmed", 2), ("average", 0), ("wmsr", 3), ("midpoint", 2)])
def test_big_m_csr_hubs_match_oracle(oracle_mod, rule, t):
    """Hubs on the big-m path beside ordinary rows on the LDS kernel, in one round."""
    rowptr, colidx = hub_csr(20000, 7, 37)
    cfg = Config(n_nodes=20000, topology="csr", rule=rule, trim=t, loss_p=0.2, termination="fixed", max_rounds=3,
                 seed=41)
    kname = gpu_vs_oracle(oracle_mod, cfg, csr=(rowptr, colidx), ACSIM_CSR_FAST=0)
    assert "k_big_resolve" in kname and kname.startswith("k_round_generic"), kname
