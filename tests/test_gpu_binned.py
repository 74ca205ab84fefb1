"""Binned-exchange round (csrc/round_binned.hip) against the CPU oracle and the per-lane kernel.

The binned path serves one-instance RANDOM_REGULAR configs with synchronous rounds: clean ones
with any rule, and lossy / crash / Byzantine ones, whose per-slot decisions phase B makes from the
slot-ordered values and the tag k_bin_tag puts on non-normal senders.  Bar: bit-exact final
values, spread traces and rounds against the oracle and the per-lane kernel.
ACSIM_BIN_SA shrinks the source block so that small graphs still span many blocks and ragged
last blocks, and (below a mean of 64 deliveries per (source block, receiver block) tile) take the
two-level plan with the phase-M regroup; ACSIM_BINNED=0 forces the per-lane kernel for the
cross-check.
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
    "two_level_d16_t5_n100000_sa256": (Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed",
                                              trim=5, eps=1e-9, max_rounds=100, seed=21, trace_spread=True), 256),
    "two_level_d32_mid_n150001_sa512": (Config(n_nodes=150001, topology="regular", degree=32, rule="midpoint",
                                               trim=5, eps=1e-10, max_rounds=200, seed=22, trace_spread=True), 512),
    "d16_t5_fixed_odd_sa512": (Config(n_nodes=30011, topology="regular", degree=16, rule="trimmed", trim=5,
                                      termination="fixed", max_rounds=25, seed=9, trace_spread=True), 512),
    "d8_t2_midpoint_sa256": (Config(n_nodes=12345, topology="regular", degree=8, rule="midpoint", trim=2,
                                    eps=1e-10, max_rounds=300, seed=3, trace_spread=True), 256),
    "d32_t0_midpoint": (Config(n_nodes=20000, topology="regular", degree=32, rule="midpoint", trim=0,
                               eps=1e-10, max_rounds=300, seed=2, trace_spread=True), 8192),
    "d32_t5_dlpsw_sa2048": (Config(n_nodes=40000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                   eps=1e-10, max_rounds=300, seed=7, trace_spread=True), 2048),
    "cfg4_shape_2e17": (preset("cfg4_eps", n_nodes=1 << 17, trace_spread=True), 8192),
    "d32_avg_clean_sa1024": (Config(n_nodes=30000, topology="regular", degree=32, rule="average", eps=1e-10,
                                    max_rounds=300, seed=41, trace_spread=True), 1024),
    # slot-dependent configs: loss, crash (partial + silent rounds), Byzantine strategies
    "faulty_d32_t5_byzrandom_drop_sa1024": (Config(n_nodes=50000, topology="regular", degree=32, rule="trimmed",
                                                   trim=5, fault_model="byzantine", n_faulty=1500,
                                                   byz_strategy="random", byz_delta=0.2, loss_p=0.1, eps=1e-8,
                                                   max_rounds=300, seed=42, trace_spread=True), 1024),
    "faulty_two_level_d16_t5_crash_drop_sa256": (Config(n_nodes=100000, topology="regular", degree=16,
                                                        rule="trimmed", trim=5, fault_model="crash",
                                                        n_faulty=3000, crash_window=6, loss_p=0.15, eps=1e-8,
                                                        max_rounds=300, seed=43, trace_spread=True), 256),
    "faulty_d16_avg_drop_sa512": (Config(n_nodes=40000, topology="regular", degree=16, rule="average",
                                         loss_p=0.2, eps=1e-9, max_rounds=300, seed=44, trace_spread=True), 512),
    "faulty_d8_mid_byzconst_sa256": (Config(n_nodes=30001, topology="regular", degree=8, rule="midpoint", trim=2,
                                            fault_model="byzantine", n_faulty=300, byz_strategy="constant",
                                            byz_const=-3.0, eps=1e-7, max_rounds=400, seed=45,
                                            trace_spread=True), 256),
    "faulty_d32_dlpsw_split_sa2048": (Config(n_nodes=40000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                             fault_model="byzantine", n_faulty=1000, byz_strategy="split",
                                             byz_delta=0.1, loss_p=0.05, eps=1e-9, max_rounds=300, seed=46,
                                             trace_spread=True), 2048),
    "faulty_wmsr_d16_t5_crash_sa1024": (Config(n_nodes=30000, topology="regular", degree=16, rule="wmsr", trim=5,
                                               fault_model="crash", n_faulty=600, crash_window=4, loss_p=0.1,
                                               eps=1e-8, max_rounds=300, seed=47, trace_spread=True), 1024),
    "faulty_cfg4_byz_shape_2e17": (preset("cfg4_byz", n_nodes=1 << 17, trace_spread=True), 16384),
    # 65-128 runs per receiver block in two passes (per-part descriptor sets: the N > 2^20 shape)
    "runs98_d32_t5_split_sa2048": (Config(n_nodes=200000, topology="regular", degree=32, rule="trimmed", trim=5,
                                          eps=1e-9, max_rounds=100, seed=48, trace_spread=True), 2048),
    "faulty_runs79_d32_t5_drop_split_sa2048": (Config(n_nodes=160000, topology="regular", degree=32,
                                                      rule="trimmed", trim=5, loss_p=0.1, eps=1e-8,
                                                      max_rounds=200, seed=49, trace_spread=True), 2048),
}


@pytest.mark.parametrize("name", list(CASES))
def test_binned_matches_oracle_and_per_lane(oracle_mod, name):
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa):
        kb, rb, xb, tb = run_gpu(cfg)
    assert kb.startswith("k_bin_scatter"), kb
    if "two_level" in name:
        assert "k_bin_regroup" in kb, kb
    if name.startswith("faulty"):
        assert ",faulty>" in kb, kb
    if "split" in name:
        assert " split2" in kb, kb
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


@pytest.mark.parametrize("name", [n for n in CASES if n.startswith("faulty")])
def test_faulty_fixup_and_tagged_paths_match_oracle(oracle_mod, name):
    """Fault schedules run on the fix-up list by default (k_bin_fixup: the faulty senders'
    deliveries resolved into the stage) and on tagged senders (k_bin_tag) with
    ACSIM_BIN_NOFIX=1 or under OMIT; both bit-exact against the oracle."""
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa):
        kf, rf, xf, tf = run_gpu(cfg)
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_NOFIX=1):
        kt, rt, xt, tt = run_gpu(cfg)
    if cfg.fault_model != "none":
        assert "k_bin_fixup" in kf, kf
        assert "k_bin_tag" in kt, kt
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), bits(o.values(0)), bits(o.spread_trace(0))
    for r_, x_, t_ in ((rf, xf, tf), (rt, xt, tt)):
        assert np.array_equal(r_, ro)
        assert np.array_equal(x_, xo)
        assert np.array_equal(t_, to)


def test_binned_full_cfg4_fixed_matches_per_lane():
    """Full-size headline graph (N = 2^20): 30 FIXED rounds, binned vs per-lane bit for bit."""
    cfg = preset("cfg4", max_rounds=30, trace_spread=True)
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


def test_two_level_full_cfg5_matches_per_lane():
    """Full-size cfg5 graph (N = 2^26, d = 16): the two-level plan, 3 FIXED rounds, bit for bit
    against the per-lane kernel (which the oracle pins at smaller sizes)."""
    cfg = preset("cfg5", max_rounds=3, trace_spread=True)
    kb, rb, xb, tb = run_gpu(cfg)
    assert "k_bin_regroup" in kb, kb
    with env(ACSIM_BINNED=0):
        _, rr, xr, tr = run_gpu(cfg)
    assert np.array_equal(rb, rr) and np.array_equal(tb, tr)
    assert np.array_equal(xb, xr)


@pytest.mark.parametrize("parts", [3, 8])
def test_two_level_virtual_partitions(oracle_mod, parts):
    """Node partitions (each with its own local-row plan) against the oracle."""
    cfg = Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed", trim=5, eps=1e-9,
                 max_rounds=100, seed=23, trace_spread=True)
    with env(ACSIM_BIN_SA=256):
        with acsim.Simulator(cfg, partitions=parts) as p:
            assert "k_bin_regroup" in p.kernel_name(), p.kernel_name()
            p.run()
            pr, px = p.rounds(), bits(p.values(0))
            for q in range(parts):
                assert np.array_equal(bits(p.partition_values(q)), px), f"copy {q} differs"
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), pr)
        assert np.array_equal(bits(o.values(0)), px)


def test_faulty_full_cfg4_byz_matches_per_lane():
    """Full-size cfg4_byz (N = 2^20, 1048 Byzantine RANDOM senders): binned vs per-lane bit for bit."""
    cfg = preset("cfg4_byz", max_rounds=25, trace_spread=True)
    kb, rb, xb, tb = run_gpu(cfg)
    assert kb.startswith("k_bin_scatter") and "+k_bin_fixup" in kb, kb
    with env(ACSIM_BIN_NOFIX=1):   # the tagged-sender path
        kt, rt, xt, tt = run_gpu(cfg)
    assert "+k_bin_tag" in kt, kt
    with env(ACSIM_BINNED=0):
        _, rr, xr, tr = run_gpu(cfg)
    assert np.array_equal(rb, rr) and np.array_equal(xb, xr) and np.array_equal(tb, tr)
    assert np.array_equal(rt, rr) and np.array_equal(xt, xr) and np.array_equal(tt, tr)


def test_faulty_chunks_resume_and_partitions(oracle_mod):
    """Crash + loss: stepped rounds, set_state resume and 3 virtual partitions against one run."""
    cfg = Config(n_nodes=45000, topology="regular", degree=16, rule="trimmed", trim=5, fault_model="crash",
                 n_faulty=900, crash_window=8, loss_p=0.1, eps=1e-9, max_rounds=200, seed=48, trace_spread=True)
    with env(ACSIM_BIN_SA=512):
        with acsim.Simulator(cfg, device=0) as g:
            assert ",faulty>" in g.kernel_name()
            g.run()
            ref, rounds = bits(g.values(0)), int(g.rounds()[0])
        with acsim.Simulator(cfg, device=0) as g:
            g.round(3)
            mid = g.values(0).copy()
            g.round(4)
            g.run()
            assert int(g.rounds()[0]) == rounds and np.array_equal(bits(g.values(0)), ref)
        with acsim.Simulator(cfg, device=0) as g:
            g.set_state(3, mid[None, :])
            g.run()
            assert np.array_equal(bits(g.values(0)), ref)
        with acsim.Simulator(cfg, partitions=3) as p:
            assert ",faulty>" in p.kernel_name(), p.kernel_name()
            p.run()
            assert int(p.rounds()[0]) == rounds and np.array_equal(bits(p.values(0)), ref)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert int(o.rounds()[0]) == rounds and np.array_equal(bits(o.values(0)), ref)


@pytest.mark.parametrize("name,pol", [("d32_t5_eps_n50000_sa1024", p) for p in (0, 2, 64, 32, 608, 1120, 1024, 7)] +
                         [("two_level_d16_t5_n100000_sa256", p) for p in (0, 2, 128, 130, 256, 322)])
def test_cache_policy_switches_bit_exact(oracle_mod, name, pol):
    """ACSIM_BIN_POL only changes cache policies (phase-A and phase-M stage stores, plain /
    nontemporal / write-through; write-through x stores) and pick-up forms.  Bits retired in round 6
    (1, 4, 8, 16: nontemporal runs, plain invpos loads, RevB, NoPf) are ignored (pol 7)."""
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_POL=pol):
        kb, rb, xb, tb = run_gpu(cfg)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))


@pytest.mark.parametrize("name,pol", [
    ("two_level_d16_t5_n100000_sa256", 16384), ("two_level_d16_t5_n100000_sa256", 16384 | 130),
    ("two_level_d32_mid_n150001_sa512", 16384), ("faulty_two_level_d16_t5_crash_drop_sa256", 16384),
    ("d16_t5_fixed_odd_sa512", 16384), ("d8_t2_midpoint_sa256", 16384),
    ("d32_t5_eps_n50000_sa1024", 16384), ("faulty_d16_avg_drop_sa512", 16384),
    ("d32_t5_eps_n50000_sa1024", 32)])   # (the compiler's copies)
def test_asm_run_copies_phase_m_and_one_pass_bit_exact(oracle_mod, name, pol):
    """Run copies by asm saddr LDS-DMA in phase M and in the one-pass phase B (ACSIM_BIN_POL bit
    16384, bin_dma_runs_asm_tb), on one- and two-level, clean and faulty plans, against the oracle
    bit for bit."""
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_POL=pol, ACSIM_BIN_SPLIT=1):
        kb, rb, xb, tb = run_gpu(cfg)
    assert " split2" not in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))


@pytest.mark.parametrize("name,pol,pack", [
    ("d32_t5_eps_n50000_sa1024", 1124, 1), ("d32_t5_eps_n50000_sa1024", 1060, 1),
    # the packed 16-bit pick-up (4096, the default since round 5); the faulty plan
    # keeps the OR-merged pick-up with the switch set
    ("d32_t5_eps_n50000_sa1024", 1124 | 4096, 1), ("d32_t5_dlpsw_sa2048", 1124 | 4096, 1),
    ("cfg4_shape_2e17", 1124 | 4096, 1), ("d32_avg_clean_sa1024", 1124 | 4096, 1),
    ("faulty_d32_t5_byzrandom_drop_sa1024", 1124 | 4096, 1), ("d32_t5_eps_n50000_sa1024", 1124 | 4096, 0),
    # run copies by asm saddr LDS-DMA (8192, the default since round 5), with either pick-up; 5220
    # keeps the compiler's copies
    ("cfg4_shape_2e17", 5220, 1), ("d32_t5_dlpsw_sa2048", 5220, 1),
    ("d32_t5_eps_n50000_sa1024", 1124 | 8192, 1), ("d32_t5_eps_n50000_sa1024", 5220 | 8192, 1),
    ("d32_t5_dlpsw_sa2048", 5220 | 8192, 1), ("cfg4_shape_2e17", 5220 | 8192, 1),
    ("d32_avg_clean_sa1024", 5220 | 8192, 1), ("faulty_d32_t5_byzrandom_drop_sa1024", 5220 | 8192, 1),
    ("d32_t5_dlpsw_sa2048", 1124, 1), ("cfg4_shape_2e17", 1124, 1),
    ("faulty_d32_t5_byzrandom_drop_sa1024", 1124, 1), ("d32_avg_clean_sa1024", 1124, 1)])
def test_clamped_pickup_bit_exact(oracle_mod, name, pol, pack):
    """Clamped two-pass pick-up (ACSIM_BIN_POL bit 1024): part 0 end-aligned in the
    buffer, part 1 start-aligned, every slot reads its part at an index clamped to a zero slot and
    the two reads are OR-merged.  Clean, DLPSW, AVERAGE (entry order) and the fault
    fix-up kernel, across round(k) calls that end mid-chunk, against the oracle bit for bit."""
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_POL=pol, ACSIM_BIN_PACK=pack):
        with acsim.Simulator(cfg, device=0) as g:
            kb = g.kernel_name()
            g.round(3)
            g.round(17)
            g.run()
            rb, xb, tb = g.rounds(), bits(g.values(0)), bits(g.spread_trace(0))
    assert " split2" in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))
        assert np.array_equal(tb, bits(o.spread_trace(0)))


@pytest.mark.parametrize("term", ["eps", "fixed"])
def test_deferred_finalize_matches_standalone(oracle_mod, term):
    """The default folds a round's spread inside the next round's phase A (ACSIM_DEFER_FIN=0:
    a k_finalize launch per round), and under EPS phase B publishes its verdict for the other
    phase-A workgroups (ACSIM_EPS_PUB=0: they stream one last round).  Rounds, traces and values
    must agree with each other and the oracle, across round(k) calls that end mid-chunk."""
    cfg = Config(n_nodes=40000, topology="regular", degree=32, rule="trimmed", trim=5, eps=1e-9,
                 termination=term, max_rounds=37, seed=12, trace_spread=True)
    out = {}
    for d, pub in ((1, 1), (1, 0), (0, 1)):
        with env(ACSIM_BIN_SA=2048, ACSIM_DEFER_FIN=d, ACSIM_EPS_PUB=pub):
            with acsim.Simulator(cfg, device=0) as g:
                g.round(5)
                g.round(19)
                g.run()
                out[d, pub] = (g.rounds(), bits(g.values(0)), bits(g.spread_trace(0)))
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ref = (o.rounds(), bits(o.values(0)), bits(o.spread_trace(0)))
    for key, got3 in out.items():
        for got, want in zip(got3, ref):
            assert np.array_equal(got, want), key


def _pub_variant(variant):
    """(config, csr, env, kernel-name fragment) of one phase-B family that writes the block partials
    of an EPS binned round, and so must also publish into the verdict slots (round_binned.hip)."""
    base = dict(topology="regular", degree=32, rule="trimmed", trim=5, eps=1e-9, max_rounds=60,
                seed=31, trace_spread=True)
    if variant == "split2":
        return Config(n_nodes=40000, **base), None, dict(ACSIM_BIN_SA=2048, ACSIM_BIN_SPLIT=2), " split2"
    if variant == "sb128":   # a receiver block other than the default (round 6)
        return Config(n_nodes=40000, **base), None, dict(ACSIM_BIN_SA=2048, ACSIM_BIN_SB=128), " sb128"
    if variant == "fixup":
        cfg = Config(n_nodes=40000, fault_model="byzantine", n_faulty=300, byz_strategy="random",
                     byz_delta=0.1, loss_p=0.05, **base)
        return cfg, None, dict(ACSIM_BIN_SA=2048), "k_bin_fixup"
    from acsim.graphs import skewed_csr
    rowptr, colidx = skewed_csr(20000, 11, 32, 5)
    cfg = Config(n_nodes=20000, topology="csr", rule="trimmed", trim=5, eps=1e-9, max_rounds=60, seed=31,
                 trace_spread=True)
    return cfg, (rowptr, colidx), dict(ACSIM_BIN_SA=1024), "k_bin"


@pytest.mark.parametrize("pack", [0, 1])
def test_packed_index_streams_bit_exact(oracle_mod, pack):
    """14-bit packed phase-A indices (ACSIM_BIN_PACK bit 0) against the u16 stream and the oracle:
    one- and two-level plans, ragged source blocks.  (Packed phase-B positions,
    bit 1, measured slower and were removed in round 5.)"""
    frag = {0: None, 1: " pk14A"}[pack]
    for name, sa in (("d32_t5_eps_n50000_sa1024", None), ("two_level_d16_t5_n100000_sa256", None),
                     ("d32_t5_dlpsw_sa2048", None)):
        cfg, sa0 = CASES[name]
        with env(ACSIM_BIN_SA=sa or sa0, ACSIM_BIN_PACK=pack, ACSIM_BIN_SPLIT=2 if "d32" in name else 1):
            kb, rb, xb, tb = run_gpu(cfg)
        if frag and "d32" in name:
            assert frag in kb, kb
        if pack == 0:
            assert "pk14" not in kb, kb
        with oracle_mod.OracleSimulator(cfg, threads=8) as o:
            o.run()
            assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))
            assert np.array_equal(tb, bits(o.spread_trace(0)))


@pytest.mark.parametrize("variant", ["split2", "sb128", "fixup", "var"])
def test_eps_publication_in_every_gather_variant(oracle_mod, variant):
    """Every phase-B kernel that writes a binned round's partials publishes its (min, max) for the
    next phase A's other workgroups (ACSIM_EPS_PUB): the two-pass, 128-receiver,
    fault fix-up and variable-degree (CSR) gathers, with publication on and off, across round(k)
    calls that end mid-chunk, bit for bit against the oracle."""
    cfg, csr, envs, frag = _pub_variant(variant)
    got = {}
    for pub in (1, 0):
        with env(ACSIM_EPS_PUB=pub, **envs):
            with acsim.Simulator(cfg, device=0, csr=csr) as g:
                assert frag in g.kernel_name(), g.kernel_name()
                g.round(3)
                g.round(17)
                g.run()
                got[pub] = (g.rounds(), bits(g.values(0)), bits(g.spread_trace(0)))
    kw = dict(csr=csr) if csr is not None else {}
    with oracle_mod.OracleSimulator(cfg, threads=8, **kw) as o:
        o.run()
        ref = (o.rounds(), bits(o.values(0)), bits(o.spread_trace(0)))
    assert 0 < int(ref[0][0]) < cfg.max_rounds   # converged under EPS, so the verdict decided the stop
    for pub, got3 in got.items():
        for a_, b_ in zip(got3, ref):
            assert np.array_equal(a_, b_), pub


SPLIT_CASES = ["d32_t5_eps_n50000_sa1024", "d16_t5_fixed_odd_sa512", "d8_t2_midpoint_sa256",
               "d32_t5_dlpsw_sa2048", "cfg4_shape_2e17"]


@pytest.mark.parametrize("name", SPLIT_CASES)
def test_split_phase_b_matches_oracle(oracle_mod, name):
    """Two-pass phase B (ACSIM_BIN_SPLIT=2: half images in LDS) against the oracle, bit for bit."""
    cfg, sa = CASES[name]
    if name == "d8_t2_midpoint_sa256":
        sa = 1024   # a one-level plan (at 256 this graph takes two levels, whose few runs do not halve)
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_SPLIT=2):
        kb, rb, xb, tb = run_gpu(cfg)
    assert " split2" in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))
        assert np.array_equal(tb, bits(o.spread_trace(0)))


def test_split_phase_b_f32_wmsr_matches_oracle(oracle_mod):
    cfg = Config(n_nodes=30011, topology="regular", degree=16, rule="wmsr", trim=5, eps=1e-6, max_rounds=300,
                 seed=31, trace_spread=True, dtype="f32")
    with env(ACSIM_BIN_SA=512, ACSIM_BIN_SPLIT=2), acsim.Simulator(cfg, device=0) as g:
        assert " split2" in g.kernel_name(), g.kernel_name()
        g.run()
        gr, gx = g.rounds(), g.values(0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(gr, o.rounds())
        assert np.array_equal(gx.view(np.uint32), o.values(0).view(np.uint32))


def test_split_off_matches_oracle(oracle_mod):
    """ACSIM_BIN_SPLIT=0 keeps the one-pass phase B on a d = 32 fp64 graph (the split default)."""
    cfg, sa = CASES["cfg4_shape_2e17"]
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_SPLIT=0):
        kb, rb, xb, tb = run_gpu(cfg)
    assert " split" not in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))


@pytest.mark.parametrize("np_", [3, 4])
def test_split_more_passes_match_oracle(oracle_mod, np_):
    cfg, sa = CASES["d32_t5_eps_n50000_sa1024"]
    with env(ACSIM_BIN_SA=sa, ACSIM_BIN_SPLIT=np_):
        kb, rb, xb, tb = run_gpu(cfg)
    assert f" split{np_}" in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))
        assert np.array_equal(tb, bits(o.spread_trace(0)))


@pytest.mark.parametrize("name", ["faulty_d32_t5_byzrandom_drop_sa1024", "faulty_d32_dlpsw_split_sa2048",
                                  "faulty_cfg4_byz_shape_2e17"])
def test_split_faulty_matches_oracle(oracle_mod, name):
    """Two-pass phase B on tagged / lossy fp64 d = 32 plans (the default there) against the oracle."""
    cfg, sa = CASES[name]
    with env(ACSIM_BIN_SA=sa):
        kb, rb, xb, tb = run_gpu(cfg)
    assert ",faulty>" in kb and " split2" in kb, kb
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(rb, o.rounds()) and np.array_equal(xb, bits(o.values(0)))
        assert np.array_equal(tb, bits(o.spread_trace(0)))


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_set_state_rejects_nonfinite_on_tagged_plan(oracle_mod, dtype):
    """a NaN handed to set_state would be read by the tagged phase B as a sender tag
    (an out-of-range x index).  The ABI rejects NaN / inf / |x| too large and canonicalises -0.0;
    a crash-fault binned run resumed from a state holding -0.0 still matches the oracle."""
    cfg = Config(n_nodes=30000, topology="regular", degree=16, rule="trimmed", trim=5, fault_model="crash",
                 n_faulty=600, crash_window=4, eps=1e-8, max_rounds=300, seed=48, trace_spread=True, dtype=dtype)
    with env(ACSIM_BIN_SA=1024), acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name().startswith("k_bin_scatter") and ",faulty>" in g.kernel_name()
        g.round(2)
        x = g.values(0).copy()
        for bad in (np.nan, np.inf, -np.inf, 1e301 if dtype == "f64" else 2e30):
            y = x.copy()
            y[123] = bad
            with pytest.raises(acsim.AcsError):
                g.set_state(2, y[None, :])
        y = x.copy()
        y[7] = -0.0
        y[8] = -0.0
        g.set_state(2, y[None, :])
        got = g.values(0)
        assert got[7] == 0 and not np.signbit(got[7])
        g.run()
        rg, xg = g.rounds(), g.values(0).copy()
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.set_state(2, y.astype(np.float64)[None, :])
        o.run()
        assert np.array_equal(o.rounds(), rg)
        assert np.array_equal(o.values(0).view(np.uint64 if dtype == "f64" else np.uint32),
                              xg.view(np.uint64 if dtype == "f64" else np.uint32))
