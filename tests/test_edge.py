"""Degenerate and boundary inputs (SURVEY §4's edge cases): one node, two nodes, graphs around
the kernel-selection boundaries, CSR rows with no senders and a graph with no edges at all,
several instances of a one-node graph, runs already converged at round 0, fp32.

CPU part: the C oracle against the independent numpy restatement.  GPU part (marked gpu): the HIP
engine against the oracle, bit for bit (rounds, values, spread trace).
"""
import numpy as np
import pytest

import acsim
import spec_np as S
from acsim.config import Config

E = dict(eps=1e-9, max_rounds=40, seed=5, trace_spread=True)
CASES = {
    "complete_n1_avg": Config(n_nodes=1, topology="complete", rule="average", **E),
    "complete_n1_mid_b3": Config(n_nodes=1, n_instances=3, topology="complete", rule="midpoint", trim=0, **E),
    "complete_n2_avg_loss": Config(n_nodes=2, topology="complete", rule="average", loss_p=0.5, **E),
    "complete_n3_trim1_crash": Config(n_nodes=3, topology="complete", rule="trimmed", trim=1, fault_model="crash",
                                      n_faulty=1, crash_window=2, **E),
    "complete_n64_trim_loss": Config(n_nodes=64, topology="complete", rule="trimmed", trim=10, loss_p=0.3, **E),
    "complete_n65_trim_loss": Config(n_nodes=65, topology="complete", rule="trimmed", trim=10, loss_p=0.3, **E),
    "regular_n3_d2": Config(n_nodes=3, topology="regular", degree=2, rule="trimmed", trim=0, **E),
    "regular_n5_d4_t1": Config(n_nodes=5, topology="regular", degree=4, rule="trimmed", trim=1, **E),
    "regular_n7_d6_wmsr_loss": Config(n_nodes=7, topology="regular", degree=6, rule="wmsr", trim=2, loss_p=0.2, **E),
    "regular_n257_d32_t5": Config(n_nodes=257, topology="regular", degree=32, rule="trimmed", trim=5, **E),
    "complete_n1_fixed": Config(n_nodes=1, topology="complete", rule="average", termination="fixed", max_rounds=3,
                                seed=5, trace_spread=True),
    "complete_n2_f32": Config(n_nodes=2, topology="complete", rule="average", loss_p=0.3, dtype="f32", eps=1e-6,
                              max_rounds=40, seed=5, trace_spread=True),
    "regular_n5_d4_f32": Config(n_nodes=5, topology="regular", degree=4, rule="midpoint", trim=1, dtype="f32",
                                eps=1e-6, max_rounds=40, seed=5, trace_spread=True),
}

# CSR graphs: rows without senders (m_i = 1: only the node itself), and a graph with no edges
CSR = {
    "csr_some_empty_rows": (np.array([0, 0, 2, 2, 5, 5, 6], dtype=np.uint64),
                            np.array([0, 3, 1, 2, 5, 4], dtype=np.uint32)),
    "csr_no_edges": (np.zeros(5, dtype=np.uint64), np.zeros(0, dtype=np.uint32)),
}


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.float64 else np.uint32)


def csr_cfg(name, rule="average"):
    rowptr, _ = CSR[name]
    return Config(n_nodes=len(rowptr) - 1, topology="csr", rule=rule, trim=0, loss_p=0.2, **E)


@pytest.mark.parametrize("name", list(CASES))
def test_edge_oracle_matches_numpy(oracle_mod, name):
    cfg = CASES[name]
    with oracle_mod.OracleSimulator(cfg) as o:
        o.run()
        n = S.NpSim(cfg)
        n.run()
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(bits(o.all_values()), bits(n.x))
        assert np.array_equal(bits(o.spread_trace(0)), bits(np.array(n.trace[0], dtype=np.float64)))


@pytest.mark.parametrize("name", list(CSR))
@pytest.mark.parametrize("rule", ["average", "midpoint", "trimmed"])
def test_edge_csr_oracle_matches_numpy(oracle_mod, name, rule):
    cfg = csr_cfg(name, rule)
    with oracle_mod.OracleSimulator(cfg, csr=CSR[name]) as o:
        o.run()
        n = S.NpSim(cfg, csr=CSR[name])
        n.run()
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(bits(o.values(0)), bits(n.x[0]))


def test_one_node_converges_at_round_zero(oracle_mod):
    """A single node has spread 0 before any round: an EPS run stops at round 0."""
    with oracle_mod.OracleSimulator(CASES["complete_n1_avg"]) as o:
        o.run()
        assert int(o.rounds()[0]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_edge_gpu_matches_oracle(oracle_mod, name):
    cfg = CASES[name]
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        r, x, tr = g.rounds(), g.all_values(), [g.spread_trace(b) for b in range(cfg.n_instances)]
    with oracle_mod.OracleSimulator(cfg) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        assert np.array_equal(bits(o.all_values()), bits(x))
        for b in range(cfg.n_instances):
            assert np.array_equal(bits(o.spread_trace(b)), bits(tr[b]))


@pytest.mark.gpu
@pytest.mark.parametrize("fast", ["0", "1"])
@pytest.mark.parametrize("name", list(CSR))
@pytest.mark.parametrize("rule", ["average", "midpoint", "trimmed"])
def test_edge_csr_gpu_matches_oracle(oracle_mod, monkeypatch, name, rule, fast):
    monkeypatch.setenv("ACSIM_CSR_FAST", fast)
    cfg = csr_cfg(name, rule)
    with acsim.Simulator(cfg, device=0, csr=CSR[name]) as g:
        g.run()
        r, x = g.rounds(), g.values(0)
    with oracle_mod.OracleSimulator(cfg, csr=CSR[name]) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        assert np.array_equal(bits(o.values(0)), bits(x))
