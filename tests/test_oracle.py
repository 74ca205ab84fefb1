"""CPU tests of the oracle: known-answer vectors, the independent numpy
restatement, the committed golden fixtures, and graph / RNG invariants."""
import json
import os

import numpy as np
import pytest

import spec_np as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from acsim.config import Config, preset

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


@pytest.mark.parametrize("ctr,key,expect", GOLDEN["philox_kat"])
def test_philox_random123_kat(oracle_mod, ctr, key, expect):
    assert list(oracle_mod.philox(ctr, key)) == expect
    assert [int(v) for v in S.philox(*ctr, *key)] == expect


def test_draws_golden(oracle_mod):
    for seed, stream, b, r, s, v in GOLDEN["draws"]:
        assert oracle_mod.draw(seed, stream, b, r, s) == v
        assert int(S.draw(seed, stream, b, r, s)) == v


def test_u53_exact_and_range(oracle_mod):
    lib = oracle_mod.load()
    assert lib.acso_u53(0, 0) == 0.0
    assert lib.acso_u53(0xFFFFFFFF, 0xFFFFFFFF) == (2.0 ** 53 - 1) * 2.0 ** -53
    rng = np.random.default_rng(0)
    w = rng.integers(0, 2 ** 32, size=(1000, 2), dtype=np.uint64)
    for a, b in w[:50]:
        assert lib.acso_u53(int(a), int(b)) == float(S.u53(a, b))


def test_drop_threshold(oracle_mod):
    for p, thr in GOLDEN["drop_threshold"].items():
        assert oracle_mod.drop_threshold(float(p)) == thr == S.drop_threshold(float(p))
    assert oracle_mod.drop_threshold(0.2) == 858993459   # SURVEY §A.5 worked value


def test_drop_rate_within_4_sigma():
    p = 0.2
    n = 200000
    thr = S.drop_threshold(p)
    d = S.draw(0, S.DROP, 0, 3, np.arange(n, dtype=np.uint64)) < thr
    sigma = np.sqrt(n * p * (1 - p))
    assert abs(d.sum() - n * p) < 4 * sigma


def test_tree_sum_order(oracle_mod):
    # pad to 8 with +0.0, stride halving: ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7))
    a = np.array([1e16, 1.0, -1e16, 1.0, 1.0, 3.0], dtype=np.float64)
    w = list(a) + [0.0, 0.0]
    expect = ((w[0] + w[4]) + (w[2] + w[6])) + ((w[1] + w[5]) + (w[3] + w[7]))
    assert oracle_mod.tree_sum(a) == expect == float(S.tree_sum_rows(a[None])[0])


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 1 << 10, 1000003])
def test_feistel_bijection(oracle_mod, n):
    v = np.arange(min(n, 1 << 16), dtype=np.uint64) if n > (1 << 16) else np.arange(n, dtype=np.uint64)
    for k in (0, 5):
        p = S.feistel(n, 0, k, v)
        assert (p < n).all()
        assert (S.feistel(n, 0, k, p, inverse=True) == v).all()
        if v.size == n:
            assert np.unique(p).size == n
        for i in range(0, v.size, max(1, v.size // 16)):
            assert oracle_mod.feistel(n, 0, k, i) == int(p[i])


def test_feistel_golden(oracle_mod):
    for k, vals in GOLDEN["feistel_n1000"].items():
        assert [oracle_mod.feistel(1000, 0, int(k), i) for i in range(64)] == vals


def test_graph_regular_symmetric(oracle_mod):
    cfg = Config(n_nodes=777, topology="regular", degree=10, rule="average", max_rounds=1)
    with oracle_mod.OracleSimulator(cfg) as o:
        nb = o.neighbors().astype(np.int64)
    assert nb.shape == (777, 10)
    # j in nbr(i) <=> i in nbr(j), with multiplicity: the multiset of (i, j) pairs is symmetric
    pairs = np.stack([np.repeat(np.arange(777), 10), nb.ravel()], 1)
    a = np.sort(pairs[:, 0] * 1000 + pairs[:, 1])
    b = np.sort(pairs[:, 1] * 1000 + pairs[:, 0])
    assert np.array_equal(a, b)


@pytest.mark.parametrize("name", sorted(GOLDEN["sims"]))
def test_oracle_reproduces_golden(oracle_mod, name):
    import hashlib
    g = GOLDEN["sims"][name]
    cfg = Config(**g["config"])
    with oracle_mod.OracleSimulator(cfg, threads=4) as o:
        o.run()
        assert o.rounds().tolist() == g["rounds"]
        assert o.converged().tolist() == g["converged"]
        for b in range(cfg.n_instances):
            x = o.values(b)
            assert hashlib.sha256(x.tobytes()).hexdigest() == g["x_sha256"][b]
            assert [float(v).hex() for v in x[:16]] == g["x_head"][b]
        for b, tr in enumerate(g["trace"]):
            assert [float(v).hex() for v in o.spread_trace(b)] == tr
        st = o.fault_status()
        for b, fl in enumerate(g["faulty"]):
            assert np.nonzero(st[b] != 0xFFFFFFFF)[0].tolist() == fl


@pytest.mark.parametrize("cfg", [
    Config(n_nodes=50, topology="complete", rule="midpoint", trim=4, fault_model="crash", n_faulty=6,
           crash_window=3, loss_p=0.15, eps=1e-9, max_rounds=200, seed=21, trace_spread=True),
    Config(n_nodes=300, topology="regular", degree=12, rule="dlpsw", trim=3, fault_model="byzantine",
           n_faulty=20, byz_strategy="split", byz_delta=0.5, eps=1e-9, max_rounds=300, seed=9,
           trace_spread=True),
    Config(n_nodes=10, n_instances=7, topology="complete", rule="average", loss_p=0.4, mask_group=3,
           eps=0.0, max_rounds=25, termination="fixed", seed=2, trace_spread=True),
    Config(n_nodes=400, topology="regular", degree=16, rule="wmsr", trim=4, fault_model="byzantine",
           n_faulty=30, byz_strategy="random", byz_delta=0.3, loss_p=0.1, eps=1e-9, max_rounds=300,
           seed=13, trace_spread=True),
    Config(n_nodes=40, topology="complete", rule="wmsr", trim=6, fault_model="crash", n_faulty=5,
           crash_window=4, eps=1e-10, max_rounds=300, seed=14, trace_spread=True),
    Config(n_nodes=300, topology="regular", degree=8, rule="trimmed", trim=2, fault_model="byzantine",
           n_faulty=10, byz_strategy="split", byz_delta=0.1, loss_p=0.05, delay_max=3, eps=1e-9,
           max_rounds=300, seed=16, trace_spread=True),
    Config(n_nodes=30, n_instances=3, topology="complete", rule="average", fault_model="crash", n_faulty=3,
           crash_window=5, delay_max=2, eps=1e-10, max_rounds=300, seed=17, instance_offset=4,
           trace_spread=True),
], ids=["complete_mid_crash_drop", "regular_dlpsw_split", "batched_avg_fixed_grouped",
        "regular_wmsr_byzrandom_drop", "complete_wmsr_crash", "regular_delay3_split_drop",
        "complete_avg_delay2_crash"])
def test_oracle_matches_numpy(oracle_mod, cfg):
    with oracle_mod.OracleSimulator(cfg) as o:
        o.run()
        n = S.NpSim(cfg)
        n.run()
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(o.all_values().view(np.uint64), n.x.view(np.uint64))
        for b in range(cfg.n_instances):
            assert np.array_equal(o.spread_trace(b).view(np.uint64), np.array(n.trace[b]).view(np.uint64))


def test_oracle_thread_count_invariance(oracle_mod):
    cfg = preset("cfg4_byz", n_nodes=5000, n_faulty=50, loss_p=0.05)
    res = []
    for th in (1, 3, 8):
        with oracle_mod.OracleSimulator(cfg.replace(omp_threads=th)) as o:
            o.run()
            res.append((o.rounds().tolist(), o.values(0).tobytes()))
    assert res[0] == res[1] == res[2]


def test_oracle_round_chunks_equal_run(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=3000, trace_spread=True)
    with oracle_mod.OracleSimulator(cfg) as a, oracle_mod.OracleSimulator(cfg) as b:
        a.run()
        while not b.round(3).done:
            pass
        assert a.rounds().tolist() == b.rounds().tolist()
        assert a.values(0).tobytes() == b.values(0).tobytes()


def test_oracle_resume_exact(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=3000, loss_p=0.1)
    with oracle_mod.OracleSimulator(cfg) as a:
        a.round(4)
        x4 = a.values(0)
        a.run()
        final = a.values(0).tobytes()
        ra = a.rounds().tolist()
    with oracle_mod.OracleSimulator(cfg) as b:
        b.set_state(4, x4)
        b.run()
        assert b.rounds().tolist() == ra
        assert b.values(0).tobytes() == final


# fp32 mode: binary32 values and arithmetic; the C oracle rounds every step of its
# double arithmetic to binary32, numpy runs float32 arrays — they must agree bit for bit.
F32_CFGS = [
    Config(n_nodes=50, topology="complete", rule="midpoint", trim=4, fault_model="crash", n_faulty=6,
           crash_window=3, loss_p=0.15, eps=1e-6, max_rounds=200, seed=21, trace_spread=True, dtype="f32"),
    Config(n_nodes=300, topology="regular", degree=12, rule="dlpsw", trim=3, fault_model="byzantine",
           n_faulty=20, byz_strategy="split", byz_delta=0.5, eps=1e-6, max_rounds=300, seed=9,
           trace_spread=True, dtype="f32"),
    Config(n_nodes=10, n_instances=7, topology="complete", rule="average", loss_p=0.4, mask_group=3,
           eps=0.0, max_rounds=25, termination="fixed", seed=2, trace_spread=True, dtype="f32"),
    Config(n_nodes=400, topology="regular", degree=16, rule="wmsr", trim=4, fault_model="byzantine",
           n_faulty=30, byz_strategy="random", byz_delta=0.3, loss_p=0.1, eps=1e-6, max_rounds=300,
           seed=13, trace_spread=True, dtype="f32"),
    Config(n_nodes=2000, topology="regular", degree=32, rule="trimmed", trim=5, eps=1e-6,
           max_rounds=300, seed=0, trace_spread=True, dtype="f32"),
    Config(n_nodes=300, topology="regular", degree=8, rule="trimmed", trim=2, fault_model="byzantine",
           n_faulty=10, byz_strategy="constant", byz_const=0.7, loss_p=0.05, delay_max=3, eps=1e-6,
           max_rounds=300, seed=16, trace_spread=True, dtype="f32"),
]


@pytest.mark.parametrize("cfg", F32_CFGS, ids=["complete_mid_crash_drop", "regular_dlpsw_split",
                                              "batched_avg_fixed_grouped", "regular_wmsr_byzrandom_drop",
                                              "cfg4_shaped", "regular_delay3_const_drop"])
def test_oracle_matches_numpy_f32(oracle_mod, cfg):
    with oracle_mod.OracleSimulator(cfg) as o:
        o.run()
        n = S.NpSim(cfg)
        n.run()
        assert n.x.dtype == np.float32
        xo = o.all_values()
        assert xo.dtype == np.float32
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(xo.view(np.uint32), n.x.view(np.uint32))
        for b in range(cfg.n_instances):
            assert np.array_equal(o.spread_trace(b).view(np.uint64), np.array(n.trace[b]).view(np.uint64))
        assert int(o.rounds().max()) > 2


def test_oracle_f32_init_and_resume(oracle_mod):
    cfg = preset("cfg4_eps", n_nodes=3000, loss_p=0.1, dtype="f32", eps=1e-6)
    with oracle_mod.OracleSimulator(cfg) as a:
        x0 = a.values(0)
        w = np.array([oracle_mod.draw(0, 0, 0, 0, 2 * i) for i in range(8)], dtype=np.uint64)
        assert np.array_equal(x0[:8], ((w >> 8).astype(np.float64) * 2.0 ** -24).astype(np.float32))
        a.round(4)
        x4 = a.values(0)
        a.run()
        final, ra = a.values(0).tobytes(), a.rounds().tolist()
    with oracle_mod.OracleSimulator(cfg) as b:
        b.set_state(4, x4)
        b.run()
        assert b.rounds().tolist() == ra and b.values(0).tobytes() == final


def test_oracle_set_state_admission(oracle_mod):
    """set_state rejects NaN / inf / out-of-range values and canonicalises -0.0: the
    tagged binned phase B reads any quiet NaN in x as a sender tag, so none may ever enter."""
    cfg = preset("cfg4_eps", n_nodes=1000)
    with oracle_mod.OracleSimulator(cfg) as o:
        x = o.values(0)
        for bad in (np.nan, np.inf, -np.inf, 1e301):
            y = x.copy()
            y[17] = bad
            with pytest.raises(Exception):
                o.set_state(2, y)
        y = x.copy()
        y[5] = -0.0
        o.set_state(2, y)
        got = o.values(0)
        assert got[5] == 0.0 and not np.signbit(got[5])
    f = preset("cfg4_eps", n_nodes=1000, dtype="f32")
    with oracle_mod.OracleSimulator(f) as o:
        y = o.values(0).astype(np.float64)
        y[3] = 2e30
        with pytest.raises(Exception):
            o.set_state(0, y)


def test_oracle_under_address_and_ub_sanitizers():
    """the CPU reference built with -fsanitize=address,undefined runs every config
    family (complete / regular / CSR, crash / Byzantine / loss / delays, fp32, resume) clean."""
    import subprocess
    here = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", here, "asan"], check=True)
    r = subprocess.run([os.path.join(here, "build", "selftest_asan")], capture_output=True, text=True,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"), timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout
