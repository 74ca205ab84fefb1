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


def random_csr(N, dmin, dmax, seed):
    rng = np.random.default_rng(seed)
    deg = rng.integers(dmin, dmax + 1, size=N)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
    colidx = rng.integers(0, N, size=int(rowptr[-1])).astype(np.uint32)
    return rowptr, colidx


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
