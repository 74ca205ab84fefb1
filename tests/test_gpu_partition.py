"""Node-partitioned rounds on one GPU.

Virtual partitions run the exact multi-GPU data flow (each partition reads only its private copy
of x, writes its own row block, then every copy receives every block — the all-gather) on a
single device; results must be identical to the unpartitioned run and to the oracle, and all
private copies must agree.  The RCCL path is exercised with a real communicator of one rank.
"""
import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


CASES = {
    "cfg5_shape_2e18": preset("cfg5", n_nodes=1 << 18, max_rounds=12, trace_spread=True),
    "cfg4_eps_odd_n": preset("cfg4_eps", n_nodes=100003, trace_spread=True),
    "cfg4_faulty_lossy": preset("cfg4_eps", n_nodes=70001, loss_p=0.1, fault_model="byzantine",
                                n_faulty=700, byz_strategy="random", byz_delta=0.02,
                                trace_spread=True),
    "reg8_mid_crash": Config(n_nodes=33333, topology="regular", degree=8, rule="midpoint", trim=2,
                             fault_model="crash", n_faulty=300, crash_window=4, eps=1e-8,
                             max_rounds=300, seed=21, trace_spread=True),
}


@pytest.mark.parametrize("parts", [2, 3, 8])
@pytest.mark.parametrize("name", list(CASES))
def test_virtual_partitions_match_unpartitioned(oracle_mod, name, parts):
    cfg = CASES[name]
    with acsim.Simulator(cfg) as ref:
        ref.run()
        rr, rx, rt = ref.rounds(), ref.values(0), ref.spread_trace(0)
        rnb = ref.neighbors() if cfg.n_nodes <= 100003 else None
    with acsim.Simulator(cfg, partitions=parts) as p:
        p.run()
        assert np.array_equal(p.rounds(), rr)
        assert np.array_equal(bits(p.values(0)), bits(rx))
        assert np.array_equal(bits(p.spread_trace(0)), bits(rt))
        for q in range(parts):
            assert np.array_equal(bits(p.partition_values(q)), bits(rx)), f"copy {q} differs"
        if rnb is not None:
            assert np.array_equal(p.neighbors(), rnb)
    if parts == 3:
        with oracle_mod.OracleSimulator(cfg, threads=8) as o:
            o.run()
            assert np.array_equal(o.rounds(), rr)
            assert np.array_equal(bits(o.values(0)), bits(rx))


def test_rccl_single_rank_path():
    """acs_create_partitioned with a real RCCL communicator (1 rank): the in-place all-gather and
    the (-min, max) all-reduce run every round; results equal the plain run."""
    import ctypes as C
    lib = acsim._abi.load_library()
    n = lib.acs_comm_id_size()
    buf = C.create_string_buffer(n)
    acsim._abi.check(lib, lib.acs_get_comm_id(buf, n))
    cfg = preset("cfg5", n_nodes=1 << 17, max_rounds=10, trace_spread=True)
    with acsim.Simulator(cfg) as ref, acsim.Simulator(cfg, partitions=1, rank=0, comm_id=buf.raw) as p:
        ref.run()
        p.run()
        assert np.array_equal(p.rounds(), ref.rounds())
        assert np.array_equal(bits(p.values(0)), bits(ref.values(0)))
        assert np.array_equal(bits(p.spread_trace(0)), bits(ref.spread_trace(0)))


def test_partition_rejects_unsupported():
    with pytest.raises(acsim.AcsError):
        acsim.Simulator(preset("cfg2"), partitions=2)       # complete graph
    with pytest.raises(acsim.AcsError):
        acsim.Simulator(preset("cfg4", n_instances=2), partitions=2)
