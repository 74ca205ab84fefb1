"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the same seeds.

Bar (BASELINE.json north_star): identical rounds-to-convergence, bit-exact drop masks / fault
schedules, final values — here every path is VALU fp64 without FMA, so the bar applied is
bit-exact equality of the final values and of the spread trace (stricter than 1e-12 relative).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def run_both(oracle_mod, cfg, threads=8):
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        gres = dict(rounds=g.rounds(), conv=g.converged(), x=g.all_values(), spread=g.spread(),
                    status=g.fault_status(),
                    trace=[g.spread_trace(b) for b in range(min(cfg.n_instances, 4))] if cfg.trace_spread else None)
    with oracle_mod.OracleSimulator(cfg, threads=threads) as o:
        o.run()
        ores = dict(rounds=o.rounds(), conv=o.converged(), x=o.all_values(), spread=o.spread(),
                    status=o.fault_status(),
                    trace=[o.spread_trace(b) for b in range(min(cfg.n_instances, 4))] if cfg.trace_spread else None)
    return gres, ores


def assert_same(g, o):
    assert np.array_equal(g["rounds"], o["rounds"]), (g["rounds"][:8], o["rounds"][:8])
    assert np.array_equal(g["conv"], o["conv"])
    assert np.array_equal(g["status"], o["status"]), "fault schedules differ"
    assert np.array_equal(bits(g["x"]), bits(o["x"])), "final values differ"
    assert np.array_equal(bits(g["spread"]), bits(o["spread"]))
    if g["trace"] is not None:
        for a, b in zip(g["trace"], o["trace"]):
            assert np.array_equal(bits(a), bits(b)), "spread traces differ"


@pytest.mark.parametrize("name", sorted(GOLDEN["sims"]))
def test_gpu_matches_golden_and_oracle(oracle_mod, name):
    g = GOLDEN["sims"][name]
    cfg = Config(**g["config"])
    with acsim.Simulator(cfg, device=0) as s:
        s.run()
        assert s.rounds().tolist() == g["rounds"]
        assert s.converged().tolist() == g["converged"]
        for b in range(cfg.n_instances):
            x = s.values(b)
            assert hashlib.sha256(x.tobytes()).hexdigest() == g["x_sha256"][b], f"instance {b}"
        for b, tr in enumerate(g["trace"]):
            assert [float(v).hex() for v in s.spread_trace(b)] == tr
        st = s.fault_status()
        for b, fl in enumerate(g["faulty"]):
            assert np.nonzero(st[b] != 0xFFFFFFFF)[0].tolist() == fl


CASES = {
    # headline kernel, clean, full size EPS (≈ 14 rounds) — every value bit-exact
    "cfg4_full_eps": preset("cfg4_eps", trace_spread=True),
    "cfg4_full_fixed20": preset("cfg4", max_rounds=20, trace_spread=True),
    "cfg4_byz_full": preset("cfg4_byz", trace_spread=True),
    "cfg4_drop_crash": preset("cfg4_eps", n_nodes=100000, loss_p=0.2, fault_model="crash",
                              n_faulty=1000, crash_window=4, trace_spread=True),
    "cfg5_shape_n2e18": preset("cfg5", n_nodes=1 << 18, max_rounds=12, trace_spread=True),
    "reg16_t5_byzsplit_drop": Config(n_nodes=50000, topology="regular", degree=16, rule="trimmed",
                                     trim=5, fault_model="byzantine", n_faulty=2000,
                                     byz_strategy="split", byz_delta=0.2, loss_p=0.1, eps=1e-7,
                                     max_rounds=400, seed=17, trace_spread=True),
    "reg8_mid_byzconst": Config(n_nodes=30001, topology="regular", degree=8, rule="midpoint", trim=2,
                                fault_model="byzantine", n_faulty=300, byz_strategy="constant",
                                byz_const=-3.0, eps=1e-7, max_rounds=400, seed=4, trace_spread=True),
    "reg32_avg": Config(n_nodes=20000, topology="regular", degree=32, rule="average", eps=1e-9,
                        max_rounds=200, seed=8, trace_spread=True),
    "reg32_dlpsw": Config(n_nodes=20000, topology="regular", degree=32, rule="dlpsw", trim=5,
                          loss_p=0.05, eps=1e-9, max_rounds=200, seed=8, trace_spread=True),
    "reg4_t1_multi_instance": Config(n_nodes=5000, n_instances=5, topology="regular", degree=4,
                                     rule="trimmed", trim=1, loss_p=0.1, mask_group=2, eps=1e-6,
                                     max_rounds=3000, seed=12, instance_offset=9, trace_spread=True),
    # W-MSR through every kernel family
    "wmsr_reg16_t5_byzrandom_drop": Config(n_nodes=30000, topology="regular", degree=16, rule="wmsr",
                                           trim=5, fault_model="byzantine", n_faulty=900,
                                           byz_strategy="random", byz_delta=0.2, loss_p=0.1,
                                           eps=1e-8, max_rounds=300, seed=51, trace_spread=True),
    "wmsr_reg32_t5_clean_binned": Config(n_nodes=60000, topology="regular", degree=32, rule="wmsr", trim=5,
                                         eps=1e-10, max_rounds=300, seed=52, trace_spread=True),
    "wmsr_generic_reg12_t3_crash": Config(n_nodes=5000, topology="regular", degree=12, rule="wmsr", trim=3,
                                          fault_model="crash", n_faulty=80, crash_window=5, eps=1e-8,
                                          max_rounds=400, seed=53, trace_spread=True),
    "wmsr_complete200_split": Config(n_nodes=200, topology="complete", rule="wmsr", trim=30,
                                     fault_model="byzantine", n_faulty=30, byz_strategy="split",
                                     byz_delta=0.1, eps=1e-9, max_rounds=500, seed=54, trace_spread=True),
    "wmsr_batched40_crash_drop": Config(n_nodes=40, n_instances=20, topology="complete", rule="wmsr",
                                        trim=6, fault_model="crash", n_faulty=5, crash_window=4,
                                        loss_p=0.2, eps=1e-10, max_rounds=300, seed=55, trace_spread=True),
    # bounded-delay rounds: per-lane regular kernel and the generic kernel
    "delay4_reg16_t5_clean": Config(n_nodes=40000, topology="regular", degree=16, rule="trimmed", trim=5,
                                    delay_max=4, eps=1e-9, max_rounds=300, seed=61, trace_spread=True),
    "delay2_reg32_t5_byz_drop": Config(n_nodes=20000, topology="regular", degree=32, rule="trimmed", trim=5,
                                       fault_model="byzantine", n_faulty=400, byz_strategy="random",
                                       byz_delta=0.1, loss_p=0.1, delay_max=2, eps=1e-8, max_rounds=300,
                                       seed=62, trace_spread=True),
    "delay3_complete60_avg_batched_shape": Config(n_nodes=60, n_instances=6, topology="complete",
                                                  rule="average", loss_p=0.2, delay_max=3, eps=1e-10,
                                                  max_rounds=400, seed=63, trace_spread=True),
    "delay1_complete300_split": Config(n_nodes=300, topology="complete", rule="midpoint", trim=50,
                                       fault_model="byzantine", n_faulty=50, byz_strategy="split",
                                       byz_delta=0.05, delay_max=1, eps=1e-9, max_rounds=500, seed=64,
                                       trace_spread=True),
    # generic kernel (odd d / t, dense complete graphs)
    "generic_reg10_t3": Config(n_nodes=7000, topology="regular", degree=10, rule="trimmed", trim=3,
                               fault_model="crash", n_faulty=100, crash_window=6, loss_p=0.05,
                               eps=1e-8, max_rounds=500, seed=1, trace_spread=True),
    "generic_complete200_byzrand": Config(n_nodes=200, topology="complete", rule="trimmed", trim=20,
                                          fault_model="byzantine", n_faulty=20,
                                          byz_strategy="random", byz_delta=0.3, loss_p=0.1,
                                          eps=1e-8, max_rounds=500, seed=6, trace_spread=True),
    "generic_complete65_avg": Config(n_nodes=65, n_instances=3, topology="complete", rule="average",
                                     loss_p=0.2, eps=1e-9, max_rounds=300, seed=2, trace_spread=True),
    "cfg2_full": preset("cfg2", trace_spread=True),
    # dense shared-sort kernels (complete, no loss, no crash, Byzantine SPLIT/CONSTANT)
    "dense65_split_mid": Config(n_nodes=65, topology="complete", rule="midpoint", trim=3,
                                fault_model="byzantine", n_faulty=20, byz_strategy="split",
                                byz_delta=0.25, eps=1e-9, max_rounds=3000, seed=31, trace_spread=True),
    "dense300_clean_trim": Config(n_nodes=300, topology="complete", rule="trimmed", trim=37,
                                  eps=1e-12, max_rounds=100, seed=32, trace_spread=True),
    "dense500_const_dlpsw": Config(n_nodes=500, topology="complete", rule="dlpsw", trim=40,
                                   fault_model="byzantine", n_faulty=100, byz_strategy="constant",
                                   byz_const=-2.5, eps=1e-9, max_rounds=500, seed=33,
                                   trace_spread=True),
    "dense3000_split_bigwindow": Config(n_nodes=3000, topology="complete", rule="trimmed",
                                        trim=900, fault_model="byzantine", n_faulty=900,
                                        byz_strategy="split", byz_delta=0.0, eps=1e-6,
                                        max_rounds=60, termination="fixed", seed=34,
                                        trace_spread=True),
    # batched persistent kernel (complete, N <= 64)
    "cfg1": preset("cfg1", trace_spread=True),
    "cfg1_avg": preset("cfg1_avg", trace_spread=True),
    "cfg3_b4096": preset("cfg3", n_instances=4096, trace_spread=True),
    "batched13_crash_mid": Config(n_nodes=13, n_instances=50, topology="complete", rule="midpoint",
                                  trim=2, fault_model="crash", n_faulty=3, crash_window=3,
                                  loss_p=0.3, eps=1e-9, max_rounds=300, seed=5, trace_spread=True),
    "batched64_trim_byz": Config(n_nodes=64, n_instances=40, topology="complete", rule="trimmed",
                                 trim=10, fault_model="byzantine", n_faulty=10,
                                 byz_strategy="random", byz_delta=0.05, loss_p=0.1, eps=1e-9,
                                 max_rounds=300, seed=14, trace_spread=True),
    "batched32_dlpsw_fixed": Config(n_nodes=32, n_instances=33, topology="complete", rule="dlpsw",
                                    trim=4, eps=0.0, max_rounds=40, termination="fixed",
                                    loss_p=0.3, mask_group=8, seed=3, trace_spread=True),
}


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_matches_oracle(oracle_mod, name):
    g, o = run_both(oracle_mod, CASES[name])
    assert_same(g, o)


@pytest.mark.parametrize("cfg", [
    preset("cfg3", n_instances=5000, max_rounds=8),                       # some instances hit the cap
    preset("cfg3", n_instances=70000),
    Config(n_nodes=512, topology="random_regular", degree=8, rule="trimmed_mean", trim=2, n_instances=37,
           loss_p=0.2, eps=1e-9, max_rounds=300, seed=11),
], ids=["cfg3_capped", "cfg3_70k", "regular_multi"])
def test_run_summary_folded_on_device(cfg):
    """acs_run's result (rounds_max, converged count, node-rounds, max final spread) is folded on
    the device; it must equal the fold of the per-instance states."""
    with acsim.Simulator(cfg, device=0) as g:
        res = g.run()
        rounds, conv, spread = g.rounds(), g.converged(), g.spread()
    assert res.n_instances == cfg.n_instances
    assert res.rounds_max == int(rounds.max())
    assert res.n_converged == int(conv.sum())
    assert res.node_rounds == int(cfg.n_nodes) * int(rounds.astype(np.int64).sum())
    assert bits(np.array([res.final_spread_max]))[0] == bits(np.array([spread.max()]))[0]


def test_cfg3_full_batch_sampled(oracle_mod):
    """1e5 instances on the GPU; a sample of instance windows re-run on the oracle through
    instance_offset (instances are independent and seeded by their global id)."""
    cfg = preset("cfg3")
    with acsim.Simulator(cfg, device=0) as g:
        res = g.run()
        rounds = g.rounds()
        assert res.n_converged == cfg.n_instances
        samples = {b0: [g.values(b) for b in range(b0, b0 + 8)] for b0 in (0, 31337, 99992)}
    for b0, xs in samples.items():
        sub = cfg.replace(n_instances=8, instance_offset=b0)
        with oracle_mod.OracleSimulator(sub) as o:
            o.run()
            assert np.array_equal(o.rounds(), rounds[b0:b0 + 8])
            for k in range(8):
                assert np.array_equal(bits(o.values(k)), bits(xs[k]))


def test_neighbors_and_status_match(oracle_mod):
    cfg = preset("cfg4_byz", n_nodes=10007, n_faulty=77)
    with acsim.Simulator(cfg, device=0) as g, oracle_mod.OracleSimulator(cfg) as o:
        assert np.array_equal(g.neighbors(), o.neighbors())
        assert np.array_equal(g.fault_status(), o.fault_status())
        assert np.array_equal(bits(g.values(0)), bits(o.values(0)))   # x^0


def test_round_chunks_equal_run(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=50000, loss_p=0.05, trace_spread=True)
    with acsim.Simulator(cfg) as a, acsim.Simulator(cfg) as b:
        a.run()
        steps = 0
        while not b.round(3).done:
            steps += 1
            assert steps < 1000
        assert a.rounds().tolist() == b.rounds().tolist()
        assert np.array_equal(bits(a.values(0)), bits(b.values(0)))
        assert np.array_equal(bits(a.spread_trace(0)), bits(b.spread_trace(0)))


def test_resume_exact():
    cfg = preset("cfg4_eps", n_nodes=50000, fault_model="byzantine", n_faulty=500,
                 byz_strategy="random", byz_delta=0.01)
    with acsim.Simulator(cfg) as a:
        a.round(5)
        x5 = a.values(0)
        a.run()
        ra, xa = a.rounds().tolist(), a.values(0)
    with acsim.Simulator(cfg) as b:
        b.set_state(5, x5)
        b.run()
        assert b.rounds().tolist() == ra
        assert np.array_equal(bits(b.values(0)), bits(xa))


def test_deterministic_across_runs():
    cfg = preset("cfg4", max_rounds=10)
    outs = []
    for _ in range(2):
        with acsim.Simulator(cfg) as s:
            s.run()
            outs.append(s.values(0).tobytes())
    assert outs[0] == outs[1]


def test_fixed_mode_runs_exactly_R():
    cfg = preset("cfg4", n_nodes=1 << 16, max_rounds=37)
    r = acsim.simulate(cfg)
    assert r.rounds.tolist() == [37]
    assert r.node_rounds == 37 * (1 << 16)


def test_kernel_timing_counts_round_launches():
    cfg = preset("cfg4", n_nodes=1 << 16, max_rounds=12)
    with acsim.Simulator(cfg) as s:
        s.set_kernel_timing(True)
        s.run()
        ms, n, name = s.kernel_timing()
        assert n == 12 and ms > 0 and (name.startswith("k_round_regular<32,5") or name.startswith("k_bin_scatter+k_bin_gather<32,5>"))


def test_kernel_timing_runs_count_every_round():
    """Run mode (bench.py): one event pair per run of k consecutive rounds, runs closed at the end
    of each round(k) call, every round counted; the summed device time matches the sampled mode's
    per-round time within a few percent and the results are untouched."""
    cfg = preset("cfg4", n_nodes=1 << 16, max_rounds=60, termination="fixed")
    with acsim.Simulator(cfg) as s:
        s.set_kernel_timing(True, every=8, runs=True)
        s.round(20)   # runs of 8, 8, 4
        s.round(10)   # 8, 2
        ms_r, n_r, _ = s.kernel_timing()
        assert n_r == 30 and ms_r > 0
        s.set_kernel_timing(True, every=1)
        s.round(30)
        ms_1, n_1, _ = s.kernel_timing()
        assert n_1 == 30
        x = s.values(0)
    with acsim.Simulator(cfg) as s2:
        s2.run()
        assert np.array_equal(s2.values(0).view(np.uint64), x.view(np.uint64))
    assert ms_r / n_r < 1.5 * ms_1 / n_1


@pytest.mark.parametrize("name", ["cfg2_full", "dense300_clean_trim", "dense500_const_dlpsw"])
def test_dense_two_kernel_path_still_exact(oracle_mod, name, monkeypatch):
    """The per-round dense kernels (k_dense_sort + k_dense_recv, used above 4096 nodes) on the
    configs the persistent kernel now serves."""
    monkeypatch.setenv("ACSIM_DENSE_PERSIST", "0")
    cfg = CASES[name]
    with acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name() == "k_dense_sort+k_dense_recv"
    g, o = run_both(oracle_mod, cfg)
    assert_same(g, o)


def test_dense_persistent_multi_instance(oracle_mod):
    cfg = Config(n_nodes=700, n_instances=5, topology="complete", rule="trimmed", trim=200,
                 fault_model="byzantine", n_faulty=200, byz_strategy="split", byz_delta=0.01,
                 eps=1e-9, max_rounds=2000, seed=41, instance_offset=3, trace_spread=True)
    with acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name() == "k_dense_persist"
    g, o = run_both(oracle_mod, cfg)
    assert_same(g, o)


def test_delay_resume_matches_oracle(oracle_mod):
    """set_state with delays restarts the history from x on both sides."""
    cfg = CASES["delay4_reg16_t5_clean"]
    with acsim.Simulator(cfg, device=0) as g, oracle_mod.OracleSimulator(cfg, threads=8) as o:
        g.round(6)
        o.round(6)
        mid = g.values(0).copy()
        assert np.array_equal(bits(mid), bits(o.values(0)))
        g.set_state(3, mid[None, :])
        o.set_state(3, mid[None, :])
        g.run()
        o.run()
        assert np.array_equal(g.rounds(), o.rounds())
        assert np.array_equal(bits(g.values(0)), bits(o.values(0)))
