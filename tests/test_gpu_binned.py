"""Binned-exchange round (csrc/round_binned.hip) against the CPU oracle and the per-lane kernel.

The binned path serves clean RANDOM_REGULAR configs with a sort-based rule (TRIMMED / MIDPOINT /
DLPSW) on one instance.  Bar: bit-exact final values, spread traces and rounds (the rule depends
only on the multiset of received values, so the slot a value lands in cannot change the result).
ACSIM_BIN_SA shrinks the source block so that small graphs still span many blocks and ragged
last blocks; ACSIM_BINNED=0 forces the per-lane kernel for the cross-check.
"""
import contextlib
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu


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


def run_gpu(cfg):
    with acsim.Simulator(cfg, device=0) as g:
        name = g.kernel_name()
        g.run()
        return name, g.rounds(), bits(g.values(0)), bits(g.spread_trace(0))


CASES = {
    "d32_t5_eps_n50000_sa1024": (Config(n_nodes=50000, topology="regular", degree=32, rule="trimmed",
                                        trim=5, eps=1e-9, max_rounds=100, seed=5, trace_spread=True), 1024),
    "d32_t5_eps_n50000_sa1024_c3": (Config(n_nodes=50000, topology="regular", degree=32, rule="trimmed",
                                           trim=5, eps=1e-9, max_rounds=100, seed=5, trace_spread=True), (1024, 3)),
    "d16_t5_n70001_sa2048_c5": (Config(n_nodes=70001, topology="regular", degree=16, rule="trimmed", trim=5,
                                       eps=1e-9, max_rounds=100, seed=21, trace_spread=True), (2048, 5)),
    "d16_t5_fixed_odd_sa512": (Config(n_nodes=30011, topology="regular", degree=16, rule="trimmed", trim=5,
                                      termination="fixed", max_rounds=25, seed=9, trace_spread=True), 512),
    "d8_t2_midpoint_sa256": (Config(n_nodes=12345, topology="regular", degree=8, rule="midpoint", trim=2,
                                    eps=1e-10, max_rounds=300, seed=3, trace_spread=True), 256),
    "d32_t0_midpoint": (Config(n_nodes=20000, topology="regular", degree=32, rule="midpoint", trim=0,
                               eps=1e-10, max_rounds=300, seed=2, trace_spread=True), 8192),
    "d32_t5_dlpsw_sa2048": (Config(n_nodes=40000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                   eps=1e-10, max_rounds=300, seed=7, trace_spread=True), 2048),
    "cfg4_shape_2e17": (preset("cfg4_eps", n_nodes=1 << 17, trace_spread=True), 8192),
}


@pytest.mark.parametrize("name", list(CASES))
def test_binned_matches_oracle_and_per_lane(oracle_mod, name):
    cfg, sa = CASES[name]
    sa, chunks = sa if isinstance(sa, tuple) else (sa, 1)
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_CHUNKS=chunks):
        kb, rb, xb, tb = run_gpu(cfg)
    assert kb.startswith("k_bin_scatter"), kb
    with env(ACSIM_BINNED=0):
        kr, rr, xr, tr = run_gpu(cfg)
    assert kr.startswith("k_round_regular"), kr
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), bits(o.values(0)), bits(o.spread_trace(0))
    assert np.array_equal(rb, ro) and np.array_equal(rr, ro)
    assert np.array_equal(xb, xo), "binned final values differ from the oracle"
    assert np.array_equal(xr, xo)
    assert np.array_equal(tb, to) and np.array_equal(tr, to)


@pytest.mark.parametrize("chunks", [1, 4])
def test_binned_full_cfg4_fixed_matches_per_lane(chunks):
    """Full-size headline graph (N = 2^20): 30 FIXED rounds, binned vs per-lane bit for bit."""
    cfg = preset("cfg4", max_rounds=30, trace_spread=True)
    with env(ACSIM_BIN_CHUNKS=chunks):
        kb, rb, xb, tb = run_gpu(cfg)
    assert kb.startswith("k_bin_scatter"), kb
    with env(ACSIM_BINNED=0):
        _, rr, xr, tr = run_gpu(cfg)
    assert np.array_equal(rb, rr) and np.array_equal(xb, xr) and np.array_equal(tb, tr)


def test_binned_round_chunks_and_resume():
    cfg = Config(n_nodes=33333, topology="regular", degree=16, rule="trimmed", trim=5, eps=1e-12,
                 max_rounds=60, seed=11, trace_spread=True)
    with env(ACSIM_BIN_SA=1024):
        with acsim.Simulator(cfg, device=0) as g:
            g.run()
            ref = bits(g.values(0))
            rounds = int(g.rounds()[0])
        with acsim.Simulator(cfg, device=0) as g:
            g.round(7)
            mid = g.values(0).copy()
            g.round(5)
            g.run()
            assert int(g.rounds()[0]) == rounds
            assert np.array_equal(bits(g.values(0)), ref)
        with acsim.Simulator(cfg, device=0) as g:
            g.set_state(7, mid[None, :])
            g.run()
            assert np.array_equal(bits(g.values(0)), ref)
