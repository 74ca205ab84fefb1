"""Full-size parity of the headline path (BASELINE.json configs[3], SURVEY §A.10 cfg4: N = 2^20,
random 32-regular, trimmed mean t = 5) against the CPU oracle, bit for bit, plus the
size-independent properties of the rule at that size.

These are the exact shapes bench.py times: FIXED 100 rounds (the bench workload), the ε-terminated
run, the 0.1 % Byzantine RANDOM variant and fp32 mode.  The oracle (oracle/acs_oracle.c, OpenMP
over receivers) finishes each in a few seconds on the GPU box's 16 host threads.
"""
import os

import numpy as np
import pytest

import acsim
from acsim.config import preset

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64 if a.dtype == np.float64 else np.uint32)


def run_gpu(cfg):
    with acsim.Simulator(cfg, device=0) as g:
        kname = g.kernel_name()
        g.run()
        return kname, g.rounds(), g.values(0).copy(), g.spread_trace(0).copy()


def run_oracle(oracle_mod, cfg):
    with oracle_mod.OracleSimulator(cfg, threads=THREADS) as o:
        o.run()
        return o.rounds(), o.values(0).copy(), o.spread_trace(0).copy()


@pytest.mark.parametrize("name,over", [
    ("cfg4", dict(max_rounds=100)),            # the bench workload (FIXED)
    ("cfg4_eps", dict()),                      # ε-terminated
    ("cfg4_byz", dict()),                      # 0.1 % Byzantine RANDOM senders
    ("cfg4", dict(max_rounds=40, dtype="f32")),
])
def test_cfg4_full_size_bit_exact(oracle_mod, name, over):
    cfg = preset(name, trace_spread=True, **over)
    kname, gr, gx, gt = run_gpu(cfg)
    assert kname.startswith("k_bin_scatter"), kname   # the headline kernels, not a fallback
    orr, ox, ot = run_oracle(oracle_mod, cfg)
    assert np.array_equal(gr, orr), (gr, orr)
    assert np.array_equal(bits(gx), bits(ox)), "final values differ"
    assert np.array_equal(bits(gt), bits(ot)), "spread traces differ"


def test_cfg4_full_size_properties():
    """Validity and contraction of the trimmed mean without faults: every value stays inside the
    hull of x^0, and the honest spread never grows from one round to the next."""
    cfg = preset("cfg4", max_rounds=100, trace_spread=True)
    with acsim.Simulator(cfg, device=0) as g:
        x0 = g.values(0).copy()
        g.run()
        x = g.values(0)
        tr = g.spread_trace(0)
    assert x.min() >= x0.min() and x.max() <= x0.max()
    assert np.all(np.diff(tr) <= 0), "spread increased"
    assert tr[-1] < tr[0] * 1e-6
