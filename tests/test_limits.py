"""Size limits lifted in round 3: fault schedules of any B·N (the segmented sort
of the §A.4 fault keys runs in instance batches, setup.hip build_fault_status).

GPU only: the forced multi-batch schedule against the oracle, and a B·N > 2^31 batch whose
sampled instances (fault set, crash rounds, x after two rounds) match the oracle run of that
instance alone (instance_offset = its global id, SURVEY §A.1 counters).
"""
import contextlib
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config


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
    return np.ascontiguousarray(a).view(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3, 7])
def test_fault_schedule_batches_match_oracle(oracle_mod, batch):
    cfg = Config(n_nodes=1000, n_instances=10, topology="regular", degree=8, rule="trimmed", trim=2,
                 fault_model="crash", n_faulty=120, crash_window=4, loss_p=0.1, eps=1e-9, max_rounds=40,
                 seed=23, instance_offset=5)
    with env(ACSIM_FAULT_BATCH=batch), acsim.Simulator(cfg, device=0) as g:
        g.run()
        st, r, x = g.fault_status(), g.rounds(), g.all_values()
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.fault_status(), st)
        assert np.array_equal(o.rounds(), r)
        assert np.array_equal(bits(o.all_values()), bits(x))


@pytest.mark.gpu
def test_fault_schedule_above_2e31(oracle_mod):
    """B·N = 32 769 · 2^16 > 2^31 (34 GiB of values on the device): byzantine + crash-free RANDOM
    senders on a 4-regular graph, two FIXED rounds on the per-lane kernel."""
    N, B = 1 << 16, 32769
    assert B * N > 2 ** 31
    cfg = Config(n_nodes=N, n_instances=B, topology="regular", degree=4, rule="trimmed", trim=1,
                 fault_model="byzantine", n_faulty=300, byz_strategy="random", byz_delta=0.05,
                 termination="fixed", max_rounds=2, seed=29)
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        assert int(g.rounds().min()) == 2
        st = g.fault_status()
        assert st.shape == (B, N)
        samples = [0, 1, 20000, B - 1]
        got = {b: (st[b].copy(), g.values(b)) for b in samples}
        # every instance has exactly n_faulty Byzantine nodes
        nbyz = (st == 0xFFFFFFFE).sum(axis=1)
        assert np.all(nbyz == 300)
        del st
    for b in samples:
        one = cfg.replace(n_instances=1, instance_offset=b)
        with oracle_mod.OracleSimulator(one, threads=8) as o:
            o.run()
            assert np.array_equal(o.fault_status().reshape(-1), got[b][0]), b
            assert np.array_equal(bits(o.values(0)), bits(got[b][1])), b
