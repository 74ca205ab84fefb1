"""Persistent binned rounds (csrc/round_persist.hip): the clean one-level fp64
binned exchange of one unpartitioned instance as ONE launch per round(k) call, A-workers streaming
phase A and B-workers gathering receiver blocks concurrently, hand-offs through progress words.

Bar: bit-exact rounds, final values and spread traces against the CPU oracle and against the
two-kernel round (ACSIM_PERSIST=0), across EPS stops, FIXED runs, stepped round(k) calls, resume,
segment counts and ragged graphs.
"""
import contextlib
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def persist_on(monkeypatch):
    """The persistent round is opt-in (ACSIM_PERSIST=1) while it is slower than the two-kernel one."""
    monkeypatch.setenv("ACSIM_PERSIST", "1")


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
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def run_gpu(cfg, steps=None):
    with acsim.Simulator(cfg, device=0) as g:
        name = g.kernel_name()
        if steps:
            for k in steps:
                g.round(k)
        g.run()
        return name, g.rounds(), bits(g.values(0)), bits(g.spread_trace(0))


CASES = {
    "cfg4_2e18_eps": preset("cfg4_eps", n_nodes=1 << 18, trace_spread=True),
    "d32_t5_mid_ragged_100003": Config(n_nodes=100003, topology="regular", degree=32, rule="midpoint", trim=5,
                                       eps=1e-10, max_rounds=300, seed=23, trace_spread=True),
    "d32_t5_dlpsw_200000": Config(n_nodes=200000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                  eps=1e-10, max_rounds=300, seed=24, trace_spread=True),
    "d16_t5_trim_2e19_fixed": Config(n_nodes=1 << 19, topology="regular", degree=16, rule="trimmed", trim=5,
                                     termination="fixed", max_rounds=20, seed=25, trace_spread=True),
    "d16_t0_avg_150001": Config(n_nodes=150001, topology="regular", degree=16, rule="average",
                                eps=1e-10, max_rounds=300, seed=26, trace_spread=True),
    "d16_t0_mid_130000": Config(n_nodes=130000, topology="regular", degree=16, rule="midpoint", trim=0,
                                eps=1e-10, max_rounds=300, seed=27, trace_spread=True),
    "d16_wmsr_120000": Config(n_nodes=120000, topology="regular", degree=16, rule="wmsr", trim=5,
                              eps=1e-10, max_rounds=300, seed=28, trace_spread=True),
}


@pytest.mark.parametrize("name", list(CASES))
def test_persist_matches_oracle_and_two_kernel_round(oracle_mod, name):
    cfg = CASES[name]
    kp, rp, xp, tp = run_gpu(cfg)
    assert kp.startswith("k_bin_persist"), kp
    with env(ACSIM_PERSIST=0):
        kt, rt, xt, tt = run_gpu(cfg)
    assert kt.startswith("k_bin_scatter"), kt
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), bits(o.values(0)), bits(o.spread_trace(0))
    assert np.array_equal(rp, ro) and np.array_equal(rt, ro)
    assert np.array_equal(xp, xo), "persistent rounds: final values differ from the oracle"
    assert np.array_equal(xt, xo)
    assert np.array_equal(tp, to) and np.array_equal(tt, to)


def test_persist_full_cfg4_fixed_matches_two_kernel_round():
    """The headline workload (N = 2^20, d = 32, t = 5): 40 FIXED rounds in one launch, bit for bit
    against the two-kernel round (which tests/test_gpu_fullsize.py pins to the oracle)."""
    cfg = preset("cfg4", max_rounds=40, trace_spread=True)
    kp, rp, xp, tp = run_gpu(cfg)
    assert kp.startswith("k_bin_persist<32,5>"), kp
    with env(ACSIM_PERSIST=0):
        kt, rt, xt, tt = run_gpu(cfg)
    assert kt.startswith("k_bin_scatter"), kt
    assert np.array_equal(rp, rt) and np.array_equal(xp, xt) and np.array_equal(tp, tt)


@pytest.mark.parametrize("segs", [1, 3, 5])
def test_persist_segment_counts(oracle_mod, segs):
    """ACSIM_PERSIST_S sets the phase-A segments per source block (A-workers = P * S, the rest
    B-workers); 3 and 5 give unequal segments.  Same results."""
    cfg = CASES["cfg4_2e18_eps"]
    with env(ACSIM_PERSIST_S=segs):
        kp, rp, xp, tp = run_gpu(cfg)
    assert f" S{segs} " in kp, kp
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rp, o.rounds()) and np.array_equal(xp, bits(o.values(0)))
        assert np.array_equal(tp, bits(o.spread_trace(0)))


def test_persist_stepped_rounds_and_resume(oracle_mod):
    """round(k) in uneven steps (one launch each, EPS stopping inside a step) and a resume from a
    mid-run state equal one straight run and the oracle."""
    cfg = preset("cfg4_eps", n_nodes=1 << 18, eps=1e-12, trace_spread=True)
    _, r0, x0, t0 = run_gpu(cfg)
    _, r1, x1, t1 = run_gpu(cfg, steps=[1, 2, 5, 3])
    assert np.array_equal(r0, r1) and np.array_equal(x0, x1) and np.array_equal(t0, t1)
    with acsim.Simulator(cfg, device=0) as g:
        g.round(6)
        mid = g.values(0).copy()
    with acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name().startswith("k_bin_persist")
        g.set_state(6, mid[None, :])
        g.run()
        assert np.array_equal(g.rounds(), r0) and np.array_equal(bits(g.values(0)), x0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), r0) and np.array_equal(bits(o.values(0)), x0)


def test_persist_kernel_timing_counts_rounds():
    """Kernel timing brackets the one launch and reports the rounds it covered."""
    cfg = preset("cfg4", n_nodes=1 << 18, max_rounds=30)
    with acsim.Simulator(cfg, device=0) as g:
        g.round(5)
        g.set_kernel_timing(True, every=1)
        g.round(20)
        ms, n, name = g.kernel_timing()
    assert name.startswith("k_bin_persist") and n == 20 and ms > 0, (ms, n, name)


def test_persist_not_used_where_it_does_not_fit():
    """Graphs too small for the segment scheme, d = 32 W-MSR and t = 0 (full sorts above the
    128 VGPRs of a 16-wave workgroup), and faulty configs keep the two-kernel round."""
    for cfg in (preset("cfg4_eps", n_nodes=4096),
                Config(n_nodes=100000, topology="regular", degree=32, rule="wmsr", trim=5, max_rounds=5),
                Config(n_nodes=100000, topology="regular", degree=32, rule="midpoint", trim=0, max_rounds=5),
                preset("cfg4_byz", n_nodes=1 << 18, max_rounds=5)):
        with acsim.Simulator(cfg, device=0) as g:
            assert not g.kernel_name().startswith("k_bin_persist"), g.kernel_name()


def test_persist_watchdog_drains_and_reports():
    """A watchdog far below one round's time makes the first waits give up: the abort word stops
    every worker (the grid drains instead of hanging) and the call raises a device error."""
    cfg = preset("cfg4", n_nodes=1 << 18, max_rounds=5)
    with env(ACSIM_PERSIST_TMO="1e-7"), acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name().startswith("k_bin_persist")
        with pytest.raises(acsim.AcsError, match="watchdog"):
            g.round(5)
