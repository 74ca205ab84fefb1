"""MFMA group kernel (csrc/batched_mfma.hip): cfg3's batched W·X averaging for 16-instance groups
that share drop masks (mask_group a multiple of 16).

Bar (BASELINE.json north star): identical rounds-to-convergence and converged flags, final values
within 1e-12 relative of the oracle (the MFMA sums in hardware order, not the §A.7 tree order).
ACSIM_MFMA=0 runs the same configs on the bit-exact VALU kernel as a cross-check.
"""
import os

import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu

RTOL = 1e-12

CASES = {
    "cfg3_g16_b4096": preset("cfg3", n_instances=4096, mask_group=16, trace_spread=True),
    "n40_g32_b1000_off32": Config(n_nodes=40, n_instances=1000, topology="complete", rule="average",
                                  loss_p=0.3, mask_group=32, eps=1e-9, max_rounds=500, seed=9,
                                  instance_offset=32, trace_spread=True),
    "n37_g16_b77_fixed": Config(n_nodes=37, n_instances=77, topology="complete", rule="average",
                                loss_p=0.1, mask_group=16, eps=1e-9, max_rounds=25, termination="fixed",
                                seed=4, trace_spread=True),
    "n64_noloss_g16": Config(n_nodes=64, n_instances=48, topology="complete", rule="average",
                             mask_group=16, eps=1e-12, max_rounds=50, seed=2, trace_spread=True),
}


def run(cfg, mfma=True):
    old = os.environ.get("ACSIM_MFMA")
    os.environ["ACSIM_MFMA"] = "1" if mfma else "0"
    try:
        with acsim.Simulator(cfg, device=0) as g:
            name = g.kernel_name()
            g.run()
            return name, g.rounds(), g.converged(), g.all_values(), g.spread_trace(0)
    finally:
        if old is None:
            os.environ.pop("ACSIM_MFMA")
        else:
            os.environ["ACSIM_MFMA"] = old


@pytest.mark.parametrize("name", list(CASES))
def test_mfma_matches_oracle_within_1e12(oracle_mod, name):
    cfg = CASES[name]
    kname, r, c, x, tr = run(cfg)
    assert kname.startswith("k_batched_mfma"), kname
    with oracle_mod.OracleSimulator(cfg, threads=8) as o:
        o.run()
        orr, oc, ox, otr = o.rounds(), o.converged(), o.all_values(), o.spread_trace(0)
    assert np.array_equal(r, orr), "rounds-to-convergence differ"
    assert np.array_equal(c, oc)
    np.testing.assert_allclose(x, ox, rtol=RTOL, atol=0)
    assert len(tr) == len(otr)
    np.testing.assert_allclose(tr, otr, rtol=1e-9, atol=1e-15)   # spreads are differences of ~equal values
    # the bit-exact VALU kernel on the same config
    kv, rv, cv, xv, _ = run(cfg, mfma=False)
    assert kv.startswith(("k_batched_small", "k_batched_split")), kv
    assert np.array_equal(rv, orr)
    assert np.array_equal(xv.view(np.uint64), ox.view(np.uint64))


def test_mfma_round_chunks_equal_run():
    cfg = CASES["n40_g32_b1000_off32"]
    _, r, _, x, _ = run(cfg)
    with acsim.Simulator(cfg, device=0) as g:
        for _ in range(200):
            info = g.round(3)
            if info.done:
                break
        assert np.array_equal(g.rounds(), r)
        assert np.array_equal(g.all_values().view(np.uint64), x.view(np.uint64))
