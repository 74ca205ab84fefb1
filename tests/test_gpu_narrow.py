"""Narrow stage (ACSIM_BIN_NARROW=1): once a round's values lie within 2^32 ulps of
each other on one side of zero, the binned exchange stages u32 offsets from their base instead of
8-byte values.  The width is chosen on the device from the (min, max) the previous phase B
published, so every round of these runs is bit-exact against the oracle whatever width it took:
8-byte rounds before the spread narrows, 4-byte ones after (each test runs past that point), the
first round of every call (nothing published yet), resumed states, negative values and ranges that
straddle zero.  Bar: bit-exact (values, rounds, spread traces) against the oracle or its golden
hashes.
"""
import contextlib
import json
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset
from acsim.digest import sha256_values

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))
GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")))


@contextlib.contextmanager
def env(**kw):
    old = {k: os.environ.get(k) for k in kw}
    for k, v in kw.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = str(v)
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


def run_oracle(oracle_mod, cfg, state=None):
    with oracle_mod.OracleSimulator(cfg, threads=THREADS) as o:
        if state is not None:
            o.set_state(*state)
        o.run()
        return o.rounds(), bits(o.values(0)).copy(), bits(o.spread_trace(0)).copy()


def run_gpu(cfg, state=None, **kw):
    with env(ACSIM_BIN_NARROW=1, **kw):
        with acsim.Simulator(cfg, device=0) as g:
            name = g.kernel_name()
            if state is not None:
                g.set_state(*state)
            g.run()
            return name, g.rounds(), bits(g.values(0)).copy(), bits(g.spread_trace(0)).copy()


def regular(n, d, rule, trim, rounds, seed, **kw):
    return Config(n_nodes=n, topology="regular", degree=d, rule=rule, trim=trim, termination="fixed",
                  max_rounds=rounds, seed=seed, trace_spread=True, **kw)


# (config, ACSIM_BIN_SA): FIXED runs long enough to reach the 4-byte rounds (the spread falls below
# 2^32 ulps after 15-25 rounds at these sizes) and, for the fast-contracting rules, the rounds where
# every value is equal
CASES = {
    "d32_t5_n50001": (regular(50001, 32, "trimmed", 5, 60, 5), 1024),
    "d32_t5_n65536_sa16k": (regular(65536, 32, "trimmed", 5, 45, 6), None),
    "d16_t5_n40000": (regular(40000, 16, "trimmed", 5, 60, 7), 1024),
    "d32_mid_n30011": (regular(30011, 32, "midpoint", 5, 60, 8), 1024),
    "d32_dlpsw_n30011": (regular(30011, 32, "dlpsw", 5, 60, 9), 1024),
    "d32_wmsr_n30011": (regular(30011, 32, "wmsr", 5, 60, 10), 1024),
    "d16_avg_n30011": (regular(30011, 16, "average", 0, 80, 11), 1024),
    "d32_mid_t0_n20000": (regular(20000, 32, "midpoint", 0, 60, 12), 2048),
}


@pytest.mark.parametrize("name", list(CASES))
def test_narrow_matches_oracle(oracle_mod, name):
    cfg, sa = CASES[name]
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    k, r, x, t = run_gpu(cfg, ACSIM_BIN_SA=sa)
    assert " narrow" in k, k
    assert np.array_equal(r, orr)
    assert np.array_equal(t, ot), "spread traces differ"
    assert np.array_equal(x, ox), "final values differ from the oracle"
    # the run did reach the 4-byte rounds: the last recorded spread is below 2^32 ulps
    tr = t.view(np.float64)
    assert tr[-1] < 2.0 ** 32 * np.spacing(np.abs(x.view(np.float64)).max())


def test_narrow_one_pass_8byte_rounds(oracle_mod):
    """ACSIM_BIN_SPLIT=1: the one-pass 8-byte rounds of a d = 32 narrow plan."""
    cfg, sa = CASES["d32_t5_n50001"]
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    k, r, x, t = run_gpu(cfg, ACSIM_BIN_SA=sa, ACSIM_BIN_SPLIT=1)
    assert " narrow" in k and " split" not in k, k
    assert np.array_equal(r, orr) and np.array_equal(x, ox) and np.array_equal(t, ot)


def test_narrow_eps_tight(oracle_mod):
    """EPS termination at ε = 1e-13: the verdict and the width come from the same published pair."""
    cfg = Config(n_nodes=50001, topology="regular", degree=32, rule="trimmed", trim=5, eps=1e-13,
                 max_rounds=200, seed=13, trace_spread=True)
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    k, r, x, t = run_gpu(cfg, ACSIM_BIN_SA=1024)
    assert " narrow" in k
    assert np.array_equal(r, orr) and np.array_equal(x, ox) and np.array_equal(t, ot)


def test_narrow_round_chunks_and_resume(oracle_mod):
    """Stepped round(k) calls (each call's first round has no published pair: 8 bytes) and set_state
    onto a later round (the header of the earlier run must not leak into the resumed one)."""
    cfg, sa = CASES["d32_t5_n50001"]
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    with env(ACSIM_BIN_NARROW=1, ACSIM_BIN_SA=sa):
        with acsim.Simulator(cfg, device=0) as g:
            assert " narrow" in g.kernel_name()
            for k in (7, 9, 16, 1, 3, 2):
                g.round(k)
            mid_r = int(g.rounds()[0])
            mid = g.values(0).copy()
            g.run()
            assert np.array_equal(g.rounds(), orr)
            assert np.array_equal(bits(g.values(0)), ox)
            assert np.array_equal(bits(g.spread_trace(0)), ot)
            # the same handle, back to the middle of the run (its header still holds a 4-byte round)
            g.set_state(mid_r, mid[None, :])
            g.run()
            assert np.array_equal(bits(g.values(0)), ox)
    with env(ACSIM_BIN_NARROW=1, ACSIM_BIN_SA=sa):
        with acsim.Simulator(cfg, device=0) as g:
            g.set_state(mid_r, mid[None, :])
            g.run()
            assert np.array_equal(g.rounds(), orr) and np.array_equal(bits(g.values(0)), ox)


@pytest.mark.parametrize("shift", ["negative", "straddle", "near_zero"])
def test_narrow_signs(oracle_mod, shift):
    """Values below zero (the base is the max's pattern), a range around zero (full width until
    it leaves zero's neighbourhood, if ever) and tiny positive values (denormal-adjacent bits)."""
    cfg, sa = CASES["d32_t5_n50001"]
    cfg = cfg.replace(max_rounds=50)
    with acsim.Simulator(cfg.replace(max_rounds=1), device=0) as g0:
        x0 = g0.values(0).copy()
    if shift == "negative":
        x = -1.5 - x0
    elif shift == "straddle":
        x = x0 - 0.5
    else:
        x = x0 * 1e-300
    state = (0, x[None, :])
    orr, ox, ot = run_oracle(oracle_mod, cfg, state)
    k, r, xg, t = run_gpu(cfg, state, ACSIM_BIN_SA=sa)
    assert " narrow" in k
    assert np.array_equal(r, orr) and np.array_equal(xg, ox) and np.array_equal(t, ot)


def test_cfg4_narrow_matches_golden():
    """The bench workload (cfg4, 100 FIXED rounds: 8-byte rounds to about round 15, 4-byte after)."""
    k, r, x, _ = run_gpu(preset("cfg4", max_rounds=100, trace_spread=True))
    assert " narrow" in k and " pk14A" in k, k
    assert int(r[0]) == 100
    assert sha256_values(x.view(np.float64)) == GOLDEN["cfg4"]["fixed100_x_sha256"]


def test_cfg4_eps_narrow_matches_golden():
    k, r, x, _ = run_gpu(preset("cfg4_eps", trace_spread=True))
    assert " narrow" in k
    assert int(r[0]) == GOLDEN["cfg4"]["eps_rounds"]
    assert sha256_values(x.view(np.float64)) == GOLDEN["cfg4"]["eps_x_sha256"]


def test_narrow_not_taken_where_unsupported():
    """fp32, faulty, partitioned and two-level plans ignore ACSIM_BIN_NARROW (no ' narrow' tag)."""
    cases = [
        Config(n_nodes=30000, topology="regular", degree=32, rule="trimmed", trim=5, max_rounds=5,
               termination="fixed", seed=1, dtype="f32"),
        Config(n_nodes=30000, topology="regular", degree=32, rule="trimmed", trim=5, max_rounds=5,
               termination="fixed", seed=1, loss_p=0.1),
        Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed", trim=5, max_rounds=5,
               termination="fixed", seed=1),
    ]
    sas = [1024, 1024, 256]
    for cfg, sa in zip(cases, sas):
        with env(ACSIM_BIN_NARROW=1, ACSIM_BIN_SA=sa):
            with acsim.Simulator(cfg, device=0) as g:
                assert " narrow" not in g.kernel_name(), g.kernel_name()
                g.run()
    with env(ACSIM_BIN_NARROW=1, ACSIM_BIN_SA=1024):
        with acsim.Simulator(CASES["d32_t5_n50001"][0], partitions=2) as p:
            assert " narrow" not in p.kernel_name()
