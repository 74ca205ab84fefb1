"""User-supplied CSR topology.

Spec extension: receiver i's entries are itself then colidx[rowptr[i] + t] on slot
rowptr[i] + t; m_i = deg(i) + 1.  Parity unpinned upstream (no reference code) — pinned here by
oracle/numpy agreement; the GPU must match the oracle bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

import acsim
import spec_np as S
from acsim import _abi
from acsim.config import Config


from acsim.graphs import random_csr, skewed_csr  # noqa: E402


CASES = [
    dict(rule="trimmed", trim=3),
    dict(rule="midpoint", trim=2, fault_model="byzantine", n_faulty=30, byz_strategy="random",
         byz_delta=0.1, loss_p=0.2, max_rounds=120),
    dict(rule="average", fault_model="crash", n_faulty=40, crash_window=5, loss_p=0.1),
    dict(rule="dlpsw", trim=2, fault_model="byzantine", n_faulty=20, byz_strategy="split", byz_delta=0.3),
]


@pytest.mark.parametrize("kw", CASES, ids=[c["rule"] for c in CASES])
def test_csr_oracle_matches_numpy(oracle_mod, kw):
    rowptr, colidx = random_csr(500, 6, 20, 1)
    cfg = Config(n_nodes=500, topology="csr", eps=1e-9, seed=4, trace_spread=True,
                 **{"max_rounds": 300, **kw})
    with oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx)) as o:
        o.run()
        n = S.NpSim(cfg, csr=(rowptr, colidx))
        n.run()
        assert np.array_equal(o.rounds(), n.rounds)
        assert np.array_equal(o.values(0).view(np.uint64), n.x[0].view(np.uint64))
        assert np.array_equal(o.spread_trace(0), np.array(n.trace[0]))


BAD = [
    ("rowptr0", lambda rp, ci: (np.concatenate([[1], rp[1:]]), ci)),
    ("decreasing", lambda rp, ci: (np.concatenate([rp[:5], [rp[5] - 100], rp[6:]]), ci)),
    ("colidx_range", lambda rp, ci: (rp, np.where(np.arange(ci.size) == 7, 10 ** 6, ci))),
]


@pytest.mark.parametrize("name,mut", BAD, ids=[b[0] for b in BAD])
def test_csr_bad_arrays_rejected(acsim_lib, oracle_mod, name, mut):
    rowptr, colidx = random_csr(100, 4, 8, 2)
    rp, ci = mut(rowptr.astype(np.int64), colidx.astype(np.int64))
    rp = np.asarray(rp, dtype=np.uint64)
    ci = np.asarray(ci, dtype=np.uint32)
    cfg = Config(n_nodes=100, topology="csr", rule="trimmed", trim=1)
    c = cfg.to_c()
    h = C.c_void_p()
    rc = acsim_lib.acs_create_csr(C.byref(c), rp.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  ci.ctypes.data_as(C.POINTER(C.c_uint32)), 0, C.byref(h))
    assert rc == _abi.EINVAL, acsim_lib.acs_last_error()
    with pytest.raises(acsim.AcsError):
        oracle_mod.OracleSimulator(cfg, csr=(rp, ci))


def test_csr_trim_too_large_rejected(acsim_lib):
    rowptr, colidx = random_csr(100, 4, 8, 3)
    cfg = Config(n_nodes=100, topology="csr", rule="trimmed", trim=3)   # some m_i = 5 <= 6
    c = cfg.to_c()
    h = C.c_void_p()
    rc = acsim_lib.acs_create_csr(C.byref(c), rowptr.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  colidx.ctypes.data_as(C.POINTER(C.c_uint32)), 0, C.byref(h))
    assert rc == _abi.EINVAL
    c2 = Config(n_nodes=100, topology="csr").to_c()
    assert acsim_lib.acs_create(C.byref(c2), _abi.BACKEND_HIP, (C.c_int * 1)(0), 1, C.byref(h)) == _abi.EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("kw", CASES, ids=[c["rule"] for c in CASES])
def test_csr_gpu_matches_oracle(oracle_mod, kw):
    rowptr, colidx = random_csr(3000, 6, 40, 5)
    cfg = Config(n_nodes=3000, topology="csr", eps=1e-9, seed=6, trace_spread=True,
                 **{"max_rounds": 300, **kw})
    with acsim.Simulator(cfg, csr=(rowptr, colidx)) as g, \
            oracle_mod.OracleSimulator(cfg, threads=8, csr=(rowptr, colidx)) as o:
        g.run()
        o.run()
        assert np.array_equal(g.rounds(), o.rounds())
        assert np.array_equal(g.values(0).view(np.uint64), o.values(0).view(np.uint64))
        assert np.array_equal(g.spread_trace(0).view(np.uint64), o.spread_trace(0).view(np.uint64))
        assert np.array_equal(g.fault_status(), o.fault_status())


# --------------------------------------------------------------------------- CSR fast path
# Rows padded to the smallest compiled degree D >= max deg(i) (SELL-64 slices on the per-lane
# register kernel; variable-degree phase B on the binned exchange): bit-exact vs the oracle.
import contextlib  # noqa: E402
import os  # noqa: E402


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


FAST = [
    ("trim5_clean", dict(rule="trimmed", trim=5), (11, 32)),
    ("mid2_byz_drop", dict(rule="midpoint", trim=2, fault_model="byzantine", n_faulty=60, byz_strategy="random",
                           byz_delta=0.1, loss_p=0.2), (5, 8)),
    ("avg_crash_drop", dict(rule="average", fault_model="crash", n_faulty=80, crash_window=5, loss_p=0.15), (3, 16)),
    ("dlpsw5_split", dict(rule="dlpsw", trim=5, fault_model="byzantine", n_faulty=40, byz_strategy="split",
                          byz_delta=0.2), (12, 32)),
    ("wmsr5_clean", dict(rule="wmsr", trim=5), (11, 16)),
    ("trim2_omit_loss", dict(rule="trimmed", trim=2, loss_p=0.4, missing_policy="omit"), (5, 8)),
    ("avg_clean", dict(rule="average"), (2, 32)),
]


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["per_lane", "binned"])
@pytest.mark.parametrize("name,kw,degs", FAST, ids=[f[0] for f in FAST])
def test_csr_fast_path_matches_oracle(oracle_mod, name, kw, degs, path):
    N = 20000
    rowptr, colidx = skewed_csr(N, degs[0], degs[1], 7)
    cfg = Config(n_nodes=N, topology="csr", eps=1e-9, seed=8, trace_spread=True, **{"max_rounds": 300, **kw})
    envs = {"ACSIM_BINNED": 0} if path == "per_lane" else {"ACSIM_BIN_SA": 1024}
    with env(**envs), acsim.Simulator(cfg, csr=(rowptr, colidx)) as g:
        kname = g.kernel_name()
        g.run()
        gr, gx, gt = g.rounds(), g.values(0), g.spread_trace(0)
    assert ("k_round_regular" if path == "per_lane" else "k_bin_scatter") in kname and "csr" in kname, kname
    with oracle_mod.OracleSimulator(cfg, threads=8, csr=(rowptr, colidx)) as o:
        o.run()
        assert np.array_equal(gr, o.rounds())
        assert np.array_equal(gx.view(np.uint64), o.values(0).view(np.uint64))
        assert np.array_equal(gt.view(np.uint64), o.spread_trace(0).view(np.uint64))


@pytest.mark.gpu
def test_csr_fast_path_multi_instance_delay_f32(oracle_mod):
    """The per-lane CSR kernel with 3 instances and bounded delays, and in fp32."""
    rowptr, colidx = skewed_csr(5000, 11, 16, 9)
    for kw in (dict(n_instances=3, rule="trimmed", trim=5, loss_p=0.1, delay_max=2),
               dict(rule="trimmed", trim=5, fault_model="crash", n_faulty=100, crash_window=3, loss_p=0.1,
                    dtype="f32")):
        cfg = Config(n_nodes=5000, topology="csr", eps=1e-7, seed=10, max_rounds=300, **kw)
        with acsim.Simulator(cfg, csr=(rowptr, colidx)) as g, \
                oracle_mod.OracleSimulator(cfg, threads=8, csr=(rowptr, colidx)) as o:
            assert "csr" in g.kernel_name(), g.kernel_name()
            g.run()
            o.run()
            assert np.array_equal(g.rounds(), o.rounds())
            bt = np.uint64 if cfg.dtype == "f64" else np.uint32
            assert np.array_equal(g.all_values().view(bt), o.all_values().view(bt))


@pytest.mark.gpu
def test_csr_full_size_skewed_2e20(oracle_mod):
    """2^20 nodes, power-law degrees 11..32 and hub-skewed senders, trimmed t = 5 (the headline
    rule on a user graph): the binned CSR path, 12 FIXED rounds, bit-exact vs the oracle."""
    N = 1 << 20
    rowptr, colidx = skewed_csr(N, 11, 32, 11)
    cfg = Config(n_nodes=N, topology="csr", rule="trimmed", trim=5, termination="fixed", max_rounds=12, seed=12,
                 trace_spread=True)
    with acsim.Simulator(cfg, csr=(rowptr, colidx)) as g:
        kname = g.kernel_name()
        g.run()
        gx, gt = g.values(0), g.spread_trace(0)
    assert kname.startswith("k_bin_scatter") and "csr" in kname, kname
    with oracle_mod.OracleSimulator(cfg, threads=16, csr=(rowptr, colidx)) as o:
        o.run()
        assert np.array_equal(gx.view(np.uint64), o.values(0).view(np.uint64))
        assert np.array_equal(gt.view(np.uint64), o.spread_trace(0).view(np.uint64))


def hub_graph(n, seed):
    """Power-law rows (10..12000 entries, about 15 % above 32) plus two rows above the generic
    kernel's 8192 entries: the fast path for most rows, hub rows on the generic / big-m path."""
    from acsim.graphs import skewed_csr
    rowptr, colidx = skewed_csr(n, 10, 12000, seed, alpha=2.6)
    deg = np.diff(rowptr.astype(np.int64))
    deg[[7, n // 2]] = [9000, 8200]
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
    rng = np.random.default_rng(seed + 1)
    colidx = rng.integers(0, n, size=int(rowptr[-1])).astype(np.uint32)
    return rowptr, colidx


HUB = [
    ("trimmed_clean", dict(rule="trimmed", trim=5), {}),
    ("trimmed_clean_binned", dict(rule="trimmed", trim=5), {"ACSIM_BIN_SA": 1024}),
    ("wmsr_clean_binned", dict(rule="wmsr", trim=5), {"ACSIM_BIN_SA": 1024}),
    ("midpoint_loss_crash", dict(rule="midpoint", trim=5, loss_p=0.2, fault_model="crash", n_faulty=900,
                                 crash_window=3), {}),
    ("average_loss", dict(rule="average", trim=0, loss_p=0.3), {}),
    ("trimmed_omit_loss", dict(rule="trimmed", trim=5, loss_p=0.3, missing_policy="omit"), {}),
    ("trimmed_f32", dict(rule="trimmed", trim=5, dtype="f32"), {"ACSIM_BINNED": 0}),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,envs", HUB, ids=[h[0] for h in HUB])
def test_csr_hub_rows_match_oracle(oracle_mod, name, kw, envs):
    """Power-law CSR: rows up to the compiled degree on the register / binned path, hub rows (and
    two rows above 8192 entries) on the generic and big-m kernels in the same round."""
    n = 20000
    rowptr, colidx = hub_graph(n, 43)
    deg = np.diff(rowptr.astype(np.int64))
    assert 0 < (deg > 32).sum() <= n // 4 and deg.max() > 8192
    cfg = Config(n_nodes=n, topology="csr", eps=1e-9, max_rounds=60, seed=47, trace_spread=True, **kw)
    with env(**envs), acsim.Simulator(cfg, device=0, csr=(rowptr, colidx)) as g:
        kname = g.kernel_name()
        assert "csr" in kname and "hubs" in kname, kname
        g.run()
        r, x, tr = g.rounds(), g.values(0), g.spread_trace(0)
    with oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx), threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), r)
        view = np.uint32 if x.dtype == np.float32 else np.uint64
        assert np.array_equal(np.ascontiguousarray(o.values(0)).view(view), np.ascontiguousarray(x).view(view))
        assert np.array_equal(o.spread_trace(0).view(np.uint64), tr.view(np.uint64))


@pytest.mark.gpu
def test_csr_full_size_power_law_hubs_2e20(oracle_mod):
    """2^20 nodes, power-law degrees 11..20000 (about 19 % of the rows above 32 entries), trimmed
    t = 5: binned CSR path for the rows up to 32, generic / big-m kernels for the hubs, 6 FIXED
    rounds bit-exact vs the oracle."""
    N = 1 << 20
    rowptr, colidx = skewed_csr(N, 11, 20000, 13, alpha=2.5)
    cfg = Config(n_nodes=N, topology="csr", rule="trimmed", trim=5, termination="fixed", max_rounds=6, seed=14,
                 trace_spread=True)
    with acsim.Simulator(cfg, csr=(rowptr, colidx)) as g:
        kname = g.kernel_name()
        g.run()
        gx, gt = g.values(0), g.spread_trace(0)
    assert kname.startswith("k_bin_scatter") and "hubs" in kname, kname
    with oracle_mod.OracleSimulator(cfg, threads=16, csr=(rowptr, colidx)) as o:
        o.run()
        assert np.array_equal(gx.view(np.uint64), o.values(0).view(np.uint64))
        assert np.array_equal(gt.view(np.uint64), o.spread_trace(0).view(np.uint64))


# ---------------------------------------------------------------------------- .npz graph files
def test_csr_npz_roundtrip_and_scipy_layout(tmp_path):
    from acsim.graphs import check_csr, load_csr, save_csr
    rowptr, colidx = skewed_csr(3000, 3, 40, 5)
    save_csr(str(tmp_path / "g.npz"), rowptr, colidx)
    rp, ci = load_csr(str(tmp_path / "g.npz"))
    assert rp.dtype == np.uint64 and ci.dtype == np.uint32
    assert np.array_equal(rp, rowptr) and np.array_equal(ci, colidx)
    # scipy.sparse.save_npz layout of the same adjacency (row i = receiver i's senders, slot order)
    import scipy.sparse as sp
    m = sp.csr_matrix((np.ones(colidx.size), colidx.astype(np.int32), rowptr.astype(np.int32)), shape=(3000, 3000))
    sp.save_npz(str(tmp_path / "s.npz"), m, compressed=True)
    rp2, ci2 = load_csr(str(tmp_path / "s.npz"))
    assert np.array_equal(rp2, rowptr) and np.array_equal(ci2, colidx)
    # non-square or non-CSR scipy matrices and malformed arrays are refused
    sp.save_npz(str(tmp_path / "rect.npz"), sp.csr_matrix(np.ones((3, 4))))
    with pytest.raises(ValueError):
        load_csr(str(tmp_path / "rect.npz"))
    sp.save_npz(str(tmp_path / "coo.npz"), sp.coo_matrix(np.eye(4)))
    with pytest.raises(ValueError):
        load_csr(str(tmp_path / "coo.npz"))
    for name, mut in BAD:
        rp3, ci3 = mut(rowptr.astype(np.int64), colidx.astype(np.int64))
        with pytest.raises(ValueError):
            check_csr(rp3, ci3)
    np.savez(str(tmp_path / "none.npz"), a=np.zeros(3))
    with pytest.raises(ValueError):
        load_csr(str(tmp_path / "none.npz"))


def _cli(*args):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, "-m", "acsim", *args], capture_output=True, text=True,
                          cwd=root + "/approximate-consensus-simulation_amd")


def test_cli_validate_with_graph_file(tmp_path):
    from acsim.graphs import save_csr
    rowptr, colidx = random_csr(400, 4, 12, 9)
    save_csr(str(tmp_path / "g.npz"), rowptr, colidx)
    r = _cli("validate", "--preset", "cfg4", "--graph", str(tmp_path / "g.npz"), "--set", "trim=1")
    assert r.returncode == 0, r.stderr
    r = _cli("validate", "--preset", "cfg4", "--graph", str(tmp_path / "g.npz"), "--set", "trim=3")
    assert r.returncode == 1 and "invalid" in r.stderr   # rows of degree 4: m_i = 5 <= 2t


@pytest.mark.gpu
def test_cli_run_with_graph_file_matches_oracle(tmp_path, oracle_mod):
    from acsim import io as aio
    from acsim.graphs import save_csr
    rowptr, colidx = skewed_csr(20000, 11, 60, 4)
    save_csr(str(tmp_path / "g.npz"), rowptr, colidx)
    out = tmp_path / "r.npz"
    r = _cli("run", "--preset", "cfg4_eps", "--graph", str(tmp_path / "g.npz"), "--set", "trim=5",
             "--out", str(out))
    assert r.returncode == 0, r.stderr
    saved = aio.load_result(str(out))
    cfg = saved["config"]
    assert cfg.topology in ("csr", _abi.TOPO_CSR) and int(cfg.n_nodes) == 20000
    with oracle_mod.OracleSimulator(cfg, csr=(rowptr, colidx)) as o:
        o.run()
        assert saved["rounds"].tolist() == o.rounds().tolist()
        assert np.array_equal(saved["x_final"].view(np.uint64), o.values(0).view(np.uint64))
