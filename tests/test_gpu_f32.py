"""fp32 mode on the GPU against the oracle: binary32 values and arithmetic, same
seeds.  Bar: bit-exact final values, spread traces and rounds-to-convergence (every kernel does
IEEE binary32 adds / divides without FMA in the spec's order, so there is nothing to tolerate).
"""
import numpy as np
import pytest

import acsim
from acsim.config import Config, preset
from test_gpu_parity import assert_same, run_both

pytestmark = pytest.mark.gpu

CASES = {
    # per-lane register kernel, clean (the cfg4 shape in binary32)
    "cfg4_shaped": preset("cfg4_eps", n_nodes=8192, dtype="f32", eps=1e-6, trace_spread=True),
    # register kernel, Byzantine RANDOM + loss
    "regular_byzrandom_drop": Config(n_nodes=3000, topology="regular", degree=16, rule="trimmed", trim=5,
                                     fault_model="byzantine", n_faulty=60, byz_strategy="random",
                                     byz_delta=0.05, loss_p=0.1, eps=1e-6, max_rounds=300, seed=3,
                                     trace_spread=True, dtype="f32"),
    # register kernel, W-MSR + crash
    "regular_wmsr_crash": Config(n_nodes=2000, topology="regular", degree=8, rule="wmsr", trim=2,
                                 fault_model="crash", n_faulty=40, crash_window=4, eps=1e-6,
                                 max_rounds=300, seed=5, trace_spread=True, dtype="f32"),
    # register kernel, bounded delay + Byzantine CONSTANT + loss
    "regular_delay_const": Config(n_nodes=1500, topology="regular", degree=8, rule="trimmed", trim=2,
                                  fault_model="byzantine", n_faulty=10, byz_strategy="constant",
                                  byz_const=0.7, loss_p=0.05, delay_max=3, eps=1e-6, max_rounds=300,
                                  seed=16, trace_spread=True, dtype="f32"),
    # batched wavefront kernel (N <= 64): complete graph, midpoint, crash + loss (cfg1-like)
    "complete_mid_crash_drop": Config(n_nodes=50, topology="complete", rule="midpoint", trim=4,
                                      fault_model="crash", n_faulty=6, crash_window=3, loss_p=0.15,
                                      eps=1e-6, max_rounds=200, seed=21, trace_spread=True, dtype="f32"),
    # batched wavefront kernel: averaging instances with grouped drop masks (cfg3-like)
    "complete_avg_batched": Config(n_nodes=64, n_instances=40, topology="complete", rule="average",
                                   loss_p=0.2, mask_group=4, eps=1e-6, max_rounds=100, seed=2,
                                   dtype="f32"),
    # batched wavefront kernel: the cfg1 presets and a cfg3 slice in binary32
    "cfg1_f32": preset("cfg1", dtype="f32", trace_spread=True),
    "cfg1_avg_f32": preset("cfg1_avg", dtype="f32", trace_spread=True),
    "cfg3_slice_f32": preset("cfg3", n_instances=3000, dtype="f32", trace_spread=True),
    # batched wavefront kernel: Byzantine RANDOM, DLPSW and W-MSR on small complete graphs
    "complete_byzrandom_dlpsw": Config(n_nodes=40, n_instances=16, topology="complete", rule="dlpsw", trim=6,
                                       fault_model="byzantine", n_faulty=6, byz_strategy="random",
                                       byz_delta=0.1, loss_p=0.1, eps=1e-6, max_rounds=300, seed=31,
                                       trace_spread=True, dtype="f32"),
    "complete_wmsr_split": Config(n_nodes=33, n_instances=8, topology="complete", rule="wmsr", trim=5,
                                  fault_model="byzantine", n_faulty=5, byz_strategy="split", byz_delta=0.2,
                                  eps=1e-6, max_rounds=300, seed=32, trace_spread=True, dtype="f32"),
    # persistent dense kernel: Byzantine SPLIT trimmed mean on a complete graph (cfg2-like, smaller)
    "complete_trimmed_split": Config(n_nodes=256, topology="complete", rule="trimmed", trim=85,
                                     fault_model="byzantine", n_faulty=85, byz_strategy="split",
                                     eps=1e-6, max_rounds=2000, seed=0, trace_spread=True, dtype="f32"),
    # persistent dense kernel: CONSTANT Byzantine DLPSW, SPLIT midpoint with Δ, several instances
    "dense_const_dlpsw": Config(n_nodes=300, n_instances=3, topology="complete", rule="dlpsw", trim=40,
                                fault_model="byzantine", n_faulty=40, byz_strategy="constant", byz_const=-2.5,
                                eps=1e-6, max_rounds=2000, seed=33, trace_spread=True, dtype="f32"),
    "dense_split_mid_delta": Config(n_nodes=513, topology="complete", rule="midpoint", trim=100,
                                    fault_model="byzantine", n_faulty=100, byz_strategy="split", byz_delta=0.01,
                                    eps=1e-6, max_rounds=2000, seed=34, trace_spread=True, dtype="f32"),
    # odd (d, t): generic kernel on a random-regular graph, DLPSW
    "regular_generic_dlpsw": Config(n_nodes=1000, topology="regular", degree=10, rule="dlpsw", trim=3,
                                    eps=1e-6, max_rounds=300, seed=9, trace_spread=True, dtype="f32"),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_f32_matches_oracle(oracle_mod, name):
    cfg = CASES[name]
    g, o = run_both(oracle_mod, cfg)
    assert g["x"].dtype == np.float32 and o["x"].dtype == np.float32
    assert_same(g, o)
    # cfg1 MIDPOINT, and CONSTANT Byzantine values on a complete graph (every honest receiver holds
    # the same multiset), agree after one round
    assert int(g["rounds"].max()) > (0 if name.startswith(("cfg1", "dense_const")) else 1)


def test_f32_small_complete_graphs_take_the_batched_kernel():
    for name in ("cfg1_f32", "cfg1_avg_f32", "cfg3_slice_f32", "complete_avg_batched"):
        with acsim.Simulator(CASES[name], device=0) as g:
            assert g.kernel_name().startswith(("k_batched_small<", "k_batched_split<")), (name, g.kernel_name())
            assert g.kernel_name().endswith("[f32]")


def test_f32_complete_graphs_take_the_dense_kernel():
    for name in ("complete_trimmed_split", "dense_const_dlpsw", "dense_split_mid_delta"):
        with acsim.Simulator(CASES[name], device=0) as g:
            assert g.kernel_name() == "k_dense_persist [f32]", (name, g.kernel_name())


# fp32 on the two-kernel dense path (k_dense_sort + k_dense_recv, complete graphs above the
# persistent kernel's 4096 nodes, up to 8192; round 6): Byzantine SPLIT with Δ, CONSTANT DLPSW and a
# clean midpoint, a few FIXED rounds each (the oracle sorts 6-8 K entries per receiver per round)
F32_DENSE_BIG = {
    "dense6000_split_trim": Config(n_nodes=6000, topology="complete", rule="trimmed", trim=2000,
                                   fault_model="byzantine", n_faulty=2000, byz_strategy="split", byz_delta=0.01,
                                   termination="fixed", max_rounds=5, seed=51, trace_spread=True, dtype="f32"),
    "dense4500_const_dlpsw": Config(n_nodes=4500, topology="complete", rule="dlpsw", trim=600,
                                    fault_model="byzantine", n_faulty=600, byz_strategy="constant", byz_const=0.25,
                                    termination="fixed", max_rounds=4, seed=52, trace_spread=True, dtype="f32"),
    "dense8192_clean_mid": Config(n_nodes=8192, topology="complete", rule="midpoint", trim=1000,
                                  termination="fixed", max_rounds=3, seed=53, trace_spread=True, dtype="f32"),
}


@pytest.mark.parametrize("name", list(F32_DENSE_BIG))
def test_f32_dense_two_kernel_above_4096_matches_oracle(oracle_mod, name):
    cfg = F32_DENSE_BIG[name]
    with acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name() == "k_dense_sort+k_dense_recv [f32]", g.kernel_name()
    g, o = run_both(oracle_mod, cfg)
    assert g["x"].dtype == np.float32
    assert_same(g, o)


@pytest.mark.parametrize("name", ["complete_trimmed_split", "dense_split_mid_delta"])
def test_f32_dense_two_kernel_small_matches_oracle(oracle_mod, name, monkeypatch):
    """The fp32 two-kernel dense path on the configs the persistent kernel serves, run to ε."""
    monkeypatch.setenv("ACSIM_DENSE_PERSIST", "0")
    cfg = CASES[name]
    with acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name() == "k_dense_sort+k_dense_recv [f32]", g.kernel_name()
    g, o = run_both(oracle_mod, cfg)
    assert_same(g, o)


def test_f32_resume_and_chunks(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=4096, loss_p=0.1, dtype="f32", eps=1e-6)
    with acsim.Simulator(cfg, device=0) as g, oracle_mod.OracleSimulator(cfg, threads=8) as o:
        g.round(3)
        o.round(3)
        x3 = g.values(0)
        assert np.array_equal(x3.view(np.uint32), o.values(0).view(np.uint32))
        g.run()
        o.run()
        final = g.values(0)
        assert np.array_equal(final.view(np.uint32), o.values(0).view(np.uint32))
    with acsim.Simulator(cfg, device=0) as h:
        h.set_state(3, x3)
        h.run()
        assert np.array_equal(h.values(0).view(np.uint32), final.view(np.uint32))


@pytest.mark.parametrize("parts", [2, 3])
def test_f32_virtual_partitions(oracle_mod, parts):
    cfg = preset("cfg4_eps", n_nodes=6000, dtype="f32", eps=1e-6)
    with acsim.Simulator(cfg, device=0) as ref, acsim.Simulator(cfg, partitions=parts) as p:
        ref.run()
        p.run()
        assert np.array_equal(ref.rounds(), p.rounds())
        assert np.array_equal(ref.values(0).view(np.uint32), p.values(0).view(np.uint32))


@pytest.mark.parametrize("n,d,t,rule,sa", [(8192, 32, 5, "trimmed", 1024), (5000, 16, 5, "midpoint", 512),
                                           (3001, 8, 2, "wmsr", 256), (1 << 20, 32, 5, "trimmed", 16384)])
def test_f32_binned_matches_per_lane(oracle_mod, n, d, t, rule, sa):
    """The fp32 binned exchange (float stage, runs padded to 16 B) against the fp32 per-lane kernel
    and, at oracle-friendly sizes, the oracle."""
    import os
    cfg = Config(n_nodes=n, topology="regular", degree=d, rule=rule, trim=t, eps=1e-6,
                 max_rounds=8 if n > 100000 else 300, termination="fixed" if n > 100000 else "eps",
                 seed=4, dtype="f32")
    old = {k: os.environ.get(k) for k in ("ACSIM_BIN_SA", "ACSIM_BINNED")}
    try:
        os.environ["ACSIM_BIN_SA"] = str(sa)
        with acsim.Simulator(cfg, device=0) as g:
            assert "k_bin_gather" in g.kernel_name() and "f32" in g.kernel_name(), g.kernel_name()
            g.run()
            xb, rb = g.values(0), g.rounds()
        os.environ["ACSIM_BINNED"] = "0"
        with acsim.Simulator(cfg, device=0) as g:
            assert "k_round_regular" in g.kernel_name()
            g.run()
            xl, rl = g.values(0), g.rounds()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert np.array_equal(rb, rl)
    assert np.array_equal(xb.view(np.uint32), xl.view(np.uint32))
    if n <= 10000:
        with oracle_mod.OracleSimulator(cfg, threads=8) as o:
            o.run()
            assert np.array_equal(o.rounds(), rb)
            assert np.array_equal(o.values(0).view(np.uint32), xb.view(np.uint32))


def test_f32_rccl_single_rank_path():
    """fp32 node partition with a real RCCL communicator (1 rank): ncclFloat32 all-gather."""
    import ctypes as C
    lib = acsim._abi.load_library()
    n = lib.acs_comm_id_size()
    buf = C.create_string_buffer(n)
    acsim._abi.check(lib, lib.acs_get_comm_id(buf, n))
    cfg = preset("cfg5", n_nodes=1 << 17, max_rounds=10, trace_spread=True, dtype="f32")
    with acsim.Simulator(cfg) as ref, acsim.Simulator(cfg, partitions=1, rank=0, comm_id=buf.raw) as p:
        ref.run()
        p.run()
        assert np.array_equal(p.rounds(), ref.rounds())
        assert np.array_equal(p.values(0).view(np.uint32), ref.values(0).view(np.uint32))
        assert np.array_equal(p.spread_trace(0), ref.spread_trace(0))


def test_f32_csr_matches_oracle(oracle_mod):
    from test_csr import random_csr
    rowptr, colidx = random_csr(500, 6, 20, 1)
    cfg = Config(n_nodes=500, topology="csr", rule="trimmed", trim=2, fault_model="byzantine", n_faulty=20,
                 byz_strategy="random", byz_delta=0.1, loss_p=0.05, eps=1e-6, seed=4, max_rounds=300,
                 trace_spread=True, dtype="f32")
    with acsim.Simulator(cfg, device=0, csr=(rowptr, colidx)) as g, \
            oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx)) as o:
        g.run()
        o.run()
        assert np.array_equal(g.rounds(), o.rounds())
        assert np.array_equal(g.values(0).view(np.uint32), o.values(0).view(np.uint32))
        assert np.array_equal(g.spread_trace(0), o.spread_trace(0))


def _with_env(**kw):
    import contextlib
    import os

    @contextlib.contextmanager
    def cm():
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
    return cm()


F32_TWO_LEVEL = {
    # (config, ACSIM_BIN_SA): small source blocks make these graphs two-level plans
    "d16_t5_n100000_sa256": (Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed", trim=5,
                                    eps=1e-6, max_rounds=100, seed=21, trace_spread=True, dtype="f32"), 256),
    "d32_mid_n150001_sa512": (Config(n_nodes=150001, topology="regular", degree=32, rule="midpoint", trim=5,
                                     eps=1e-6, max_rounds=200, seed=22, trace_spread=True, dtype="f32"), 512),
    "d8_t2_wmsr_n60001_sa128": (Config(n_nodes=60001, topology="regular", degree=8, rule="wmsr", trim=2,
                                       eps=1e-6, max_rounds=300, seed=24, trace_spread=True, dtype="f32"), 128),
}


@pytest.mark.parametrize("name", list(F32_TWO_LEVEL))
def test_f32_two_level_matches_oracle(oracle_mod, name):
    """fp32 two-level binned plans (float stage1 / phase-M image / stage2, runs padded to 4
    elements) against the oracle and the fp32 per-lane kernel, bit for bit."""
    cfg, sa = F32_TWO_LEVEL[name]
    with _with_env(ACSIM_BIN_SA=sa), acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert "k_bin_regroup" in kb and "f32" in kb, kb
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with _with_env(ACSIM_BINNED=0), acsim.Simulator(cfg, device=0) as g:
        assert "k_round_regular" in g.kernel_name()
        g.run()
        rl, xl = g.rounds(), g.values(0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), o.values(0), o.spread_trace(0)
    assert np.array_equal(rb, ro) and np.array_equal(rl, ro)
    assert np.array_equal(xb.view(np.uint32), xo.view(np.uint32)), "two-level fp32 values differ from the oracle"
    assert np.array_equal(xl.view(np.uint32), xo.view(np.uint32))
    assert np.array_equal(tb, to)


F32_PACKED = {
    # (config, ACSIM_BIN_SA): one-level, two-level, tagged (Byzantine + loss), ragged source blocks
    "d32_t5_n50000_sa1024": (Config(n_nodes=50000, topology="regular", degree=32, rule="trimmed", trim=5,
                                    eps=1e-6, max_rounds=100, seed=5, trace_spread=True, dtype="f32"), 1024),
    "d16_t5_n100000_sa256": F32_TWO_LEVEL["d16_t5_n100000_sa256"],
    "d32_byz_n40000_sa2048": (Config(n_nodes=40000, topology="regular", degree=32, rule="trimmed", trim=5,
                                     fault_model="byzantine", n_faulty=400, byz_strategy="random", byz_delta=0.1,
                                     loss_p=0.05, eps=1e-6, max_rounds=100, seed=9, trace_spread=True,
                                     dtype="f32"), 2048),
}


@pytest.mark.parametrize("name", list(F32_PACKED))
def test_f32_packed_phase_a_indices_match_oracle(oracle_mod, name):
    """14-bit packed phase-A indices on fp32 plans (ACSIM_BIN_PACK bit 2 with bit 0):
    float pairs streamed from the packed stream, write-through and nontemporal stage stores, against
    the oracle bit for bit, across round(k) calls that end mid-chunk."""
    cfg, sa = F32_PACKED[name]
    with _with_env(ACSIM_BIN_SA=sa, ACSIM_BIN_PACK=5), acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert "f32" in kb and "pk14A" in kb, kb
        g.round(3)
        g.round(17)
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), o.values(0), o.spread_trace(0)
    assert np.array_equal(rb, ro)
    assert np.array_equal(xb.view(np.uint32), xo.view(np.uint32)), "packed fp32 values differ from the oracle"
    assert np.array_equal(tb, to)


@pytest.mark.parametrize("parts", [3])
def test_f32_two_level_virtual_partitions(oracle_mod, parts):
    cfg = Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed", trim=5, eps=1e-6,
                 max_rounds=100, seed=23, dtype="f32")
    with _with_env(ACSIM_BIN_SA=256), acsim.Simulator(cfg, partitions=parts) as p:
        assert "k_bin_regroup" in p.kernel_name(), p.kernel_name()
        p.run()
        pr, px = p.rounds(), p.values(0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), pr)
        assert np.array_equal(o.values(0).view(np.uint32), px.view(np.uint32))


def test_f32_two_level_full_cfg5_matches_per_lane():
    """Full-size cfg5 graph (N = 2^26, d = 16) in fp32: the two-level plan, 3 FIXED rounds, bit for
    bit against the fp32 per-lane kernel."""
    cfg = preset("cfg5", max_rounds=3, trace_spread=True, dtype="f32")
    with acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert "k_bin_regroup" in kb and "f32" in kb, kb
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with _with_env(ACSIM_BINNED=0), acsim.Simulator(cfg, device=0) as g:
        g.run()
        assert np.array_equal(g.rounds(), rb) and np.array_equal(g.spread_trace(0), tb)
        assert np.array_equal(g.values(0).view(np.uint32), xb.view(np.uint32))


F32_TAGGED = {
    # fault schedules and loss through the fp32 binned exchange (binary32 NaN tags, N <= 2^20)
    "byzrandom_drop_d32_t5_sa1024": (Config(n_nodes=50000, topology="regular", degree=32, rule="trimmed", trim=5,
                                            fault_model="byzantine", n_faulty=1500, byz_strategy="random",
                                            byz_delta=0.2, loss_p=0.1, eps=1e-5, max_rounds=300, seed=42,
                                            trace_spread=True, dtype="f32"), 1024),
    "two_level_crash_drop_d16_t5_sa256": (Config(n_nodes=100000, topology="regular", degree=16, rule="trimmed",
                                                 trim=5, fault_model="crash", n_faulty=3000, crash_window=6,
                                                 loss_p=0.15, eps=1e-5, max_rounds=300, seed=43, trace_spread=True,
                                                 dtype="f32"), 256),
    "avg_drop_d16_sa512": (Config(n_nodes=40000, topology="regular", degree=16, rule="average", loss_p=0.2,
                                  eps=1e-5, max_rounds=300, seed=44, trace_spread=True, dtype="f32"), 512),
    "byzconst_mid_d8_sa256": (Config(n_nodes=30001, topology="regular", degree=8, rule="midpoint", trim=2,
                                     fault_model="byzantine", n_faulty=300, byz_strategy="constant", byz_const=-3.0,
                                     eps=1e-5, max_rounds=400, seed=45, trace_spread=True, dtype="f32"), 256),
    "split_dlpsw_d32_sa2048": (Config(n_nodes=40000, topology="regular", degree=32, rule="dlpsw", trim=5,
                                      fault_model="byzantine", n_faulty=1000, byz_strategy="split", byz_delta=0.1,
                                      loss_p=0.05, eps=1e-5, max_rounds=300, seed=46, trace_spread=True,
                                      dtype="f32"), 2048),
    "wmsr_crash_d16_t5_sa1024": (Config(n_nodes=30000, topology="regular", degree=16, rule="wmsr", trim=5,
                                        fault_model="crash", n_faulty=600, crash_window=4, loss_p=0.1, eps=1e-5,
                                        max_rounds=300, seed=47, trace_spread=True, dtype="f32"), 1024),
}


@pytest.mark.parametrize("name", list(F32_TAGGED))
def test_f32_tagged_binned_matches_oracle(oracle_mod, name):
    cfg, sa = F32_TAGGED[name]
    with _with_env(ACSIM_BIN_SA=sa), acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert kb.startswith("k_bin_scatter") and ",faulty>" in kb and "f32" in kb, kb
        if name.startswith("two_level"):
            assert "k_bin_regroup" in kb, kb
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with _with_env(ACSIM_BINNED=0), acsim.Simulator(cfg, device=0) as g:
        assert "k_round_regular" in g.kernel_name()
        g.run()
        rl, xl = g.rounds(), g.values(0)
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ro, xo, to = o.rounds(), o.values(0), o.spread_trace(0)
    assert np.array_equal(rb, ro) and np.array_equal(rl, ro)
    assert np.array_equal(xb.view(np.uint32), xo.view(np.uint32)), "tagged fp32 binned values differ from the oracle"
    assert np.array_equal(xl.view(np.uint32), xo.view(np.uint32))
    assert np.array_equal(tb, to)


def test_f32_tagged_full_cfg4_byz_matches_per_lane():
    """cfg4_byz at full size (N = 2^20, the largest N the binary32 tag holds) in fp32: 20 FIXED
    rounds, binned vs per-lane bit for bit."""
    cfg = preset("cfg4_byz", termination="fixed", max_rounds=20, trace_spread=True, dtype="f32")
    with acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert ",faulty>" in kb and "f32" in kb, kb
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with _with_env(ACSIM_BINNED=0), acsim.Simulator(cfg, device=0) as g:
        g.run()
        assert np.array_equal(g.rounds(), rb) and np.array_equal(g.spread_trace(0), tb)
        assert np.array_equal(g.values(0).view(np.uint32), xb.view(np.uint32))


F32_TAGGED_BIG = {
    # above 2^20 nodes: crash senders carry their crash rank in the tag's 20-bit field
    "crash_trim_d16_2e21": Config(n_nodes=(1 << 21) + 4096, topology="regular", degree=16, rule="trimmed", trim=5,
                                  fault_model="crash", n_faulty=30000, crash_window=3, loss_p=0.1,
                                  termination="fixed", max_rounds=6, seed=48, trace_spread=True, dtype="f32"),
    "byz_random_d32_2e21": Config(n_nodes=1 << 21, topology="regular", degree=32, rule="trimmed", trim=5,
                                  fault_model="byzantine", n_faulty=20000, byz_strategy="random", byz_delta=0.1,
                                  termination="fixed", max_rounds=5, seed=49, trace_spread=True, dtype="f32"),
}


@pytest.mark.parametrize("name", list(F32_TAGGED_BIG))
def test_f32_tagged_above_2e20_matches_oracle(oracle_mod, name):
    """The fp32 tagged binned exchange above 2^20 nodes (round 3): bit-exact vs the oracle."""
    cfg = F32_TAGGED_BIG[name]
    with acsim.Simulator(cfg, device=0) as g:
        kb = g.kernel_name()
        assert kb.startswith("k_bin_scatter") and ",faulty>" in kb and "f32" in kb, kb
        g.run()
        rb, xb, tb = g.rounds(), g.values(0), g.spread_trace(0)
    with oracle_mod.OracleSimulator(cfg, threads=16) as o:
        o.run()
        assert np.array_equal(rb, o.rounds())
        assert np.array_equal(xb.view(np.uint32), o.values(0).view(np.uint32))
        assert np.array_equal(tb, o.spread_trace(0))
