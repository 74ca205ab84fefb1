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


def test_partitioned_simulator_through_rendezvous_group():
    """bench.py's N > 1 code path up to the communicator: acsim.distributed.partitioned_simulator
    with the torch-free control plane (acsim.rendezvous.Group, world 1): the RCCL id is made on
    rank 0 and broadcast over the group, the communicator forms, and the run equals the plain one.
    The process maps one HIP runtime and one RCCL, the ones libacsim.so was built against."""
    from acsim.distributed import partitioned_simulator
    from acsim.rendezvous import Group
    cfg = preset("cfg5", n_nodes=1 << 17, max_rounds=10, trace_spread=True)
    with Group(0, 1) as g:
        with acsim.Simulator(cfg) as ref, partitioned_simulator(cfg, 0, 1, 0, group=g) as p:
            ref.run()
            p.run()
            assert np.array_equal(p.rounds(), ref.rounds())
            assert np.array_equal(bits(p.values(0)), bits(ref.values(0)))
            assert np.array_equal(bits(p.spread_trace(0)), bits(ref.spread_trace(0)))
    info = acsim._abi.runtime_info()
    assert len(info["libamdhip64"]) == 1 and len(info["librccl"]) == 1, info
    assert info["libamdhip64"][0].startswith("/opt/rocm"), info


def test_partition_rejects_unsupported():
    with pytest.raises(acsim.AcsError):
        acsim.Simulator(preset("cfg2"), partitions=2)       # complete graph
    with pytest.raises(acsim.AcsError):
        acsim.Simulator(preset("cfg4", n_instances=2), partitions=2)


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


@pytest.mark.parametrize("parts,sa,chunks", [(2, 1024, 4), (4, 1024, 2), (8, 512, 4), (4, 2048, 8)])
@pytest.mark.parametrize("mode", ["eps", "fixed", "stepped"])
def test_chunked_exchange_matches_unpartitioned(oracle_mod, parts, sa, chunks, mode):
    """The chunked exchange: phase A by source-block chunk after each chunk's
    exchange, phase B by receiver-block chunk, verdicts on the comm stream, phase A/M running one
    round ahead of the verdict.  EPS runs stop mid round-chunk; stepped runs cross round(k) calls.
    Everything must equal the unpartitioned run bit for bit, in every partition's copy."""
    base = preset("cfg5", n_nodes=1 << 18, trace_spread=True)
    cfg = base.replace(termination="eps", eps=1e-7, max_rounds=200) if mode != "fixed" else base.replace(max_rounds=13)
    with env(ACSIM_BIN_SA=sa):
        with acsim.Simulator(cfg) as ref:
            ref.run()
            rr, rx, rt = ref.rounds(), ref.values(0), ref.spread_trace(0)
        with env(ACSIM_XCHUNKS=chunks), acsim.Simulator(cfg, partitions=parts) as p:
            assert f"xchunks{chunks}" in p.kernel_name(), p.kernel_name()
            if mode == "stepped":
                while not p.round(5).done:
                    pass
            else:
                p.run()
            assert np.array_equal(p.rounds(), rr)
            assert np.array_equal(bits(p.values(0)), bits(rx))
            assert np.array_equal(bits(p.spread_trace(0)), bits(rt))
            for q in range(parts):
                assert np.array_equal(bits(p.partition_values(q)), bits(rx)), f"copy {q} differs"


@pytest.mark.parametrize("n,chunked", [(3000, False), (6144, True)])
def test_chunked_exchange_small_source_blocks(oracle_mod, n, chunked):
    """Source blocks of 64 senders (ACSIM_BIN_SA=64): the chunks must still be whole phase-B
    receiver blocks (256 rows), else a chunk's exchange could be recorded before all of its rows
    ran phase B.  N = 3000 over 2 partitions gives 384-row chunks (refused: the unchunked sequence
    runs); N = 6144 gives 768-row chunks (chunked).  Both equal the unpartitioned run."""
    cfg = preset("cfg5", n_nodes=n, termination="eps", eps=1e-7, max_rounds=200, trace_spread=True)
    with env(ACSIM_BIN_SA=64):
        with acsim.Simulator(cfg) as ref:
            ref.run()
            rr, rx, rt = ref.rounds(), ref.values(0), ref.spread_trace(0)
        with env(ACSIM_XCHUNKS=4), acsim.Simulator(cfg, partitions=2) as p:
            assert ("xchunks4" in p.kernel_name()) == chunked, p.kernel_name()
            p.run()
            assert np.array_equal(p.rounds(), rr)
            assert np.array_equal(bits(p.values(0)), bits(rx))
            assert np.array_equal(bits(p.spread_trace(0)), bits(rt))
            for q in range(2):
                assert np.array_equal(bits(p.partition_values(q)), bits(rx)), f"copy {q} differs"
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(o.rounds(), rr)
        assert np.array_equal(bits(o.values(0)), bits(rx))


def test_chunked_exchange_single_rank_rccl():
    """The chunked sequence over a real RCCL communicator of one rank (no peers: the exchange
    group is empty, the all-reduce is skipped) equals the plain run."""
    import ctypes as C
    lib = acsim._abi.load_library()
    n = lib.acs_comm_id_size()
    buf = C.create_string_buffer(n)
    acsim._abi.check(lib, lib.acs_get_comm_id(buf, n))
    cfg = preset("cfg5", n_nodes=1 << 17, max_rounds=10, trace_spread=True)
    with env(ACSIM_BIN_SA=1024, ACSIM_XCHUNKS=4):
        with acsim.Simulator(cfg) as ref, acsim.Simulator(cfg, partitions=1, rank=0, comm_id=buf.raw) as p:
            assert "xchunks4" in p.kernel_name(), p.kernel_name()
            ref.run()
            p.run()
            assert np.array_equal(bits(p.values(0)), bits(ref.values(0)))
            assert np.array_equal(bits(p.spread_trace(0)), bits(ref.spread_trace(0)))


def test_refused_binned_plan_falls_back_to_per_lane(oracle_mod):
    """A partition whose binned plan is refused once laid out (found by tools/fuzz_gpu.py: 46 081
    nodes, 8-regular, source blocks of 256, 3 partitions — a two-level plan whose phase-M image
    outgrows the LDS) must not fail acs_create: every partition runs the per-lane kernel instead,
    bit-exact against the oracle."""
    import os
    cfg = Config(n_nodes=46081, topology="regular", degree=8, rule="average", eps=1e-7, max_rounds=20,
                 seed=3, trace_spread=True)
    old = os.environ.get("ACSIM_BIN_SA")
    os.environ["ACSIM_BIN_SA"] = "256"
    try:
        with acsim.Simulator(cfg, partitions=3) as p:
            name = p.kernel_name()
            p.run()
            pr, px = p.rounds(), p.values(0)
            copies = [p.partition_values(q) for q in range(3)]
    finally:
        if old is None:
            os.environ.pop("ACSIM_BIN_SA", None)
        else:
            os.environ["ACSIM_BIN_SA"] = old
    assert name.startswith("k_round_regular"), name
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        assert np.array_equal(pr, o.rounds())
        assert np.array_equal(bits(px), bits(o.values(0)))
        for x in copies:
            assert np.array_equal(bits(x), bits(o.values(0)))
