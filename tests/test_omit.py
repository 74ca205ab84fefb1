"""missing_policy = OMIT: a crashed-silent or dropped message is
removed from S_i instead of being replaced by x_i.

CPU part: the C oracle and the independent numpy restatement agree bit for bit on every rule,
topology and fault family (plus fp32), and OMIT differs from SELF wherever messages go missing.
GPU part (marked gpu): every kernel family against the oracle, bit for bit (the MFMA variant
within 1e-12 and with identical rounds).
"""
import contextlib
import os

import numpy as np
import pytest

import acsim
import spec_np as S
from acsim.config import Config, preset

from test_csr import random_csr

CASES = {
    "complete_mid_crash_drop": Config(n_nodes=40, topology="complete", rule="midpoint", trim=3,
                                      fault_model="crash", n_faulty=5, crash_window=4, loss_p=0.3,
                                      eps=1e-7, max_rounds=300, seed=3),
    "complete_avg_crash": Config(n_nodes=16, topology="complete", rule="average", fault_model="crash",
                                 n_faulty=3, crash_window=3, loss_p=0.2, eps=1e-6, max_rounds=300, seed=1),
    "batched_avg_loss": Config(n_nodes=64, n_instances=24, topology="complete", rule="average",
                               loss_p=0.4, eps=1e-8, max_rounds=200, seed=5, instance_offset=11),
    "batched_trim_loss": Config(n_nodes=48, n_instances=6, topology="complete", rule="trimmed", trim=6,
                                loss_p=0.5, eps=1e-8, max_rounds=300, seed=6),
    "regular_d8_trim_heavy_loss": Config(n_nodes=3000, topology="regular", degree=8, rule="trimmed", trim=2,
                                         loss_p=0.45, eps=1e-8, max_rounds=300, seed=7),
    "regular_d16_wmsr_crash": Config(n_nodes=2000, topology="regular", degree=16, rule="wmsr", trim=5,
                                     fault_model="crash", n_faulty=200, crash_window=5, loss_p=0.2,
                                     eps=1e-8, max_rounds=300, seed=8),
    "regular_d32_dlpsw_byz_drop": Config(n_nodes=4000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                         fault_model="byzantine", n_faulty=100, byz_strategy="random",
                                         byz_delta=0.1, loss_p=0.35, eps=1e-8, max_rounds=300, seed=9),
    "regular_d16_mid_crash": Config(n_nodes=3000, topology="regular", degree=16, rule="midpoint", trim=5,
                                    fault_model="crash", n_faulty=300, crash_window=3, loss_p=0.3,
                                    eps=1e-8, max_rounds=300, seed=10),
    "regular_d32_avg_drop": Config(n_nodes=3000, topology="regular", degree=32, rule="average", loss_p=0.25,
                                   eps=1e-9, max_rounds=300, seed=12),
    "regular_d6_generic_trim": Config(n_nodes=1500, topology="regular", degree=6, rule="trimmed", trim=1,
                                      fault_model="crash", n_faulty=100, crash_window=4, loss_p=0.3,
                                      eps=1e-8, max_rounds=300, seed=13),
    "regular_d8_delay_trim": Config(n_nodes=1000, topology="regular", degree=8, rule="trimmed", trim=2,
                                    loss_p=0.3, delay_max=2, eps=1e-8, max_rounds=300, seed=14),
    "f32_regular_d16_trim_crash": Config(n_nodes=2000, topology="regular", degree=16, rule="trimmed", trim=5,
                                         fault_model="crash", n_faulty=150, crash_window=4, loss_p=0.3,
                                         eps=1e-6, max_rounds=300, seed=15, dtype="f32"),
}
for _c in CASES.values():
    _c.missing_policy = "omit"
    _c.trace_spread = True


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.float64 else np.uint32)


@pytest.mark.parametrize("name", list(CASES))
def test_omit_oracle_matches_numpy(oracle_mod, name):
    cfg = CASES[name]
    with oracle_mod.OracleSimulator(cfg, threads=4) as o:
        o.run()
        n = S.NpSim(cfg)
        n.run()
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(bits(o.all_values()), bits(n.x))
        for b in range(min(cfg.n_instances, 3)):
            assert np.array_equal(bits(o.spread_trace(b)), bits(np.array(n.trace[b])))
    # the policy is live: with SELF the run differs
    with oracle_mod.OracleSimulator(cfg.replace(missing_policy="self"), threads=4) as o2:
        o2.run()
        assert not np.array_equal(bits(o2.all_values()), bits(n.x))


def test_omit_csr_oracle_matches_numpy(oracle_mod):
    """Variable degree with heavy loss: some receivers fall to m' <= 2t and keep x_i."""
    rowptr, colidx = random_csr(400, 5, 14, 3)
    for rule, t in (("trimmed", 2), ("midpoint", 2), ("average", 0), ("wmsr", 2)):
        cfg = Config(n_nodes=400, topology="csr", rule=rule, trim=t, loss_p=0.5, eps=1e-9, max_rounds=200,
                     seed=17, trace_spread=True, missing_policy="omit")
        with oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx)) as o:
            o.run()
            n = S.NpSim(cfg, csr=(rowptr, colidx))
            n.run()
            assert np.array_equal(o.rounds(), n.rounds), rule
            assert np.array_equal(bits(o.values(0)), bits(n.x[0])), rule


def test_omit_rejects_unknown_policy(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=100)
    c = cfg.to_c()
    c.missing_policy = 7
    import ctypes as C
    assert oracle_mod.load().acso_validate(C.byref(c)) != 0


# ----------------------------------------------------------------------------------------- GPU
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


def gpu_run(cfg, **envs):
    with env(**envs), acsim.Simulator(cfg, device=0) as g:
        name = g.kernel_name()
        g.run()
        return name, g.rounds(), g.all_values(), g.spread_trace(0) if cfg.trace_spread else None


GPU_CASES = [
    ("complete_mid_crash_drop", {}, "k_batched_small"),
    ("complete_avg_crash", {}, "k_batched_small"),
    ("batched_avg_loss", {}, "k_batched_small"),
    ("batched_trim_loss", {}, "k_batched_small"),
    ("regular_d8_trim_heavy_loss", {"ACSIM_BINNED": 0}, "k_round_regular"),
    ("regular_d8_trim_heavy_loss", {"ACSIM_BIN_SA": 256}, "k_bin_scatter"),
    ("regular_d16_wmsr_crash", {"ACSIM_BINNED": 0}, "k_round_regular"),
    ("regular_d16_wmsr_crash", {"ACSIM_BIN_SA": 256}, "k_bin_scatter"),
    ("regular_d32_dlpsw_byz_drop", {"ACSIM_BINNED": 0}, "k_round_regular"),
    ("regular_d32_dlpsw_byz_drop", {"ACSIM_BIN_SA": 512}, "k_bin_scatter"),
    ("regular_d16_mid_crash", {"ACSIM_BIN_SA": 256}, "k_bin_scatter"),
    ("regular_d32_avg_drop", {"ACSIM_BINNED": 0}, "k_round_regular"),
    ("regular_d32_avg_drop", {"ACSIM_BIN_SA": 512}, "k_bin_scatter"),
    ("regular_d6_generic_trim", {}, "k_round_generic"),
    ("regular_d8_delay_trim", {}, "k_round_regular"),
    ("f32_regular_d16_trim_crash", {"ACSIM_BINNED": 0}, "k_round_regular"),
    ("f32_regular_d16_trim_crash", {"ACSIM_BIN_SA": 512}, "k_bin_scatter"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,envs,kernel", GPU_CASES,
                         ids=[f"{n}-{k}" for n, _, k in GPU_CASES])
def test_omit_gpu_matches_oracle(oracle_mod, name, envs, kernel):
    cfg = CASES[name]
    kname, r, x, tr = gpu_run(cfg, **envs)
    # (clean 64-node AVERAGE batches take the split form of the batched kernel)
    assert kname.startswith(kernel) or (kernel == "k_batched_small" and kname.startswith("k_batched_split")), kname
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        assert np.array_equal(bits(o.all_values()), bits(x))
        assert np.array_equal(bits(o.spread_trace(0)), bits(tr))


@pytest.mark.gpu
def test_omit_generic_complete_graph(oracle_mod):
    """A complete graph above the batched kernel's 64 nodes, with crash + loss: the generic kernel."""
    cfg = Config(n_nodes=300, topology="complete", rule="trimmed", trim=40, fault_model="crash", n_faulty=30,
                 crash_window=3, loss_p=0.4, eps=1e-8, max_rounds=300, seed=19, trace_spread=True,
                 missing_policy="omit")
    kname, r, x, _ = gpu_run(cfg)
    assert kname.startswith("k_round_generic"), kname
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), r) and np.array_equal(bits(o.values(0)), bits(x[0]))


@pytest.mark.gpu
def test_omit_mfma_group_within_1e12(oracle_mod):
    cfg = preset("cfg3_g16", n_instances=512, missing_policy="omit")
    kname, r, x, _ = gpu_run(cfg)
    assert "mfma" in kname, kname
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        xo = o.all_values()
        assert np.max(np.abs(x - xo) / np.abs(xo)) <= 1e-12


@pytest.mark.gpu
def test_omit_csr_gpu_matches_oracle(oracle_mod):
    rowptr, colidx = random_csr(3000, 5, 30, 4)
    for rule, t, faults in (("trimmed", 2, {}), ("average", 0, {}),
                            ("midpoint", 2, dict(fault_model="crash", n_faulty=200, crash_window=4))):
        cfg = Config(n_nodes=3000, topology="csr", rule=rule, trim=t, loss_p=0.4, eps=1e-9, max_rounds=300,
                     seed=21, trace_spread=True, missing_policy="omit", **faults)
        with acsim.Simulator(cfg, device=0, csr=(rowptr, colidx)) as g, \
                oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx), threads=8) as o:
            g.run()
            o.run()
            assert np.array_equal(g.rounds(), o.rounds()), rule
            assert np.array_equal(bits(g.values(0)), bits(o.values(0))), rule
