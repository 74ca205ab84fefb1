"""cfg3 with F lanes per receiver (csrc/batched_small.hip k_batched_split<F>): one
64-node instance per F-wave workgroup, drop bits computed in F parts and all-gathered, the §A.7
tree split into its residue-class subtrees and recombined by shuffles.  Bar: bit-exact against the
oracle (values, rounds, spread traces), the full 10^5-instance batch against the golden hashes.
"""
import contextlib
import hashlib
import json
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


CASES = {
    "cfg3_small_batch": preset("cfg3", n_instances=300, trace_spread=True),
    "cfg3_offset_group3": preset("cfg3", n_instances=101, instance_offset=7777, mask_group=3, trace_spread=True),
    "omit_p30": Config(n_nodes=64, n_instances=64, topology="complete", rule="average", loss_p=0.3,
                       missing_policy="omit", eps=1e-8, max_rounds=200, seed=9, trace_spread=True),
    "no_loss_fixed": Config(n_nodes=64, n_instances=40, topology="complete", rule="average", loss_p=0.0,
                            termination="fixed", max_rounds=7, seed=4, trace_spread=True),
    "f32_p20": preset("cfg3", n_instances=128, dtype="f32", eps=1e-5, trace_spread=True),
}


@pytest.mark.parametrize("F", [2, 4])
@pytest.mark.parametrize("name", list(CASES))
def test_split_matches_oracle(oracle_mod, name, F):
    cfg = CASES[name]
    with env(ACSIM_BATCH_SPLIT=F), acsim.Simulator(cfg, device=0) as g:
        assert g.kernel_name().startswith(f"k_batched_split<{F}>"), g.kernel_name()
        g.run()
        gx, gr = g.all_values(), g.rounds()
        gt = [g.spread_trace(b) for b in range(min(cfg.n_instances, 8))]
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        ox, orr = o.all_values(), o.rounds()
        ot = [o.spread_trace(b) for b in range(min(cfg.n_instances, 8))]
    u = np.uint32 if cfg.dtype == "f32" else np.uint64
    assert np.array_equal(gr, orr)
    assert np.array_equal(np.ascontiguousarray(gx).view(u), np.ascontiguousarray(ox).view(u))
    for a, b in zip(gt, ot):   # (instances stop at different rounds: traces differ in length)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


@pytest.mark.parametrize("F", [2, 4])
def test_split_stepped_rounds(F):
    """round(k) in steps (instances stop independently inside a step) equals one run()."""
    cfg = CASES["cfg3_small_batch"]
    with env(ACSIM_BATCH_SPLIT=F):
        with acsim.Simulator(cfg, device=0) as g:
            g.run()
            ref, rr = g.all_values(), g.rounds()
        with acsim.Simulator(cfg, device=0) as g:
            for k in (1, 3, 2, 5):
                g.round(k)
            g.run()
            assert np.array_equal(g.rounds(), rr)
            assert np.array_equal(g.all_values().view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("F", [2, 4])
def test_split_full_batch_matches_golden(F):
    """The full 10^5-instance batch (BASELINE configs[2]) and an 8-way shard of it reproduce the
    oracle's checksum of per-instance checksums and rounds (tests/golden/fullsize.json)."""
    from acsim.digest import combine_digests, instance_digests
    from acsim.distributed import shard_range
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))["cfg3"]
    cfg = preset("cfg3")
    with env(ACSIM_BATCH_SPLIT=F):
        with acsim.Simulator(cfg, device=0) as s:
            s.run()
            x, r = s.all_values(), s.rounds()
        assert combine_digests(instance_digests(x)) == g["instances_digest"]
        assert hashlib.sha256(r.astype("<u4").tobytes()).hexdigest() == g["rounds_sha256"]
        off, cnt = shard_range(cfg.n_instances, 8, 5)
        with acsim.Simulator(cfg.replace(n_instances=cnt, instance_offset=off), device=0) as s:
            s.run()
            assert np.array_equal(s.rounds(), r[off:off + cnt])
            assert np.array_equal(s.all_values().view(np.uint64), x[off:off + cnt].view(np.uint64))
