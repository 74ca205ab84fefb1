"""round(k)'s info and the per-instance state getters against the oracle after every call.

Handles of at most 16 instances read their states back through host-mapped memory (one small
launch and a polled sequence number, `read_states` in api.hip); larger ones by a
device-to-host copy.  Both paths, on the binned, per-lane, batched and persistent dense kernels,
EPS and FIXED: round, done, instances done, spread / lo / hi, and the rounds / converged / spread
getters, bit for bit after each call of a ragged step sequence.
"""
import numpy as np
import pytest

import acsim
from acsim.config import Config, preset

pytestmark = pytest.mark.gpu

CASES = {
    # binned exchange, one instance, EPS (the cfg4 shape at 2^17 nodes)
    "binned_eps_b1": preset("cfg4_eps", n_nodes=1 << 17),
    # binned, FIXED (the bench workload's shape): the closing finalize of every call
    "binned_fixed_b1": preset("cfg4", n_nodes=1 << 17, max_rounds=40),
    # per-lane register kernel, 3 and 16 instances (mapped), 17 (copied), with loss
    "regular_b3": Config(n_nodes=3000, topology="random_regular", degree=8, rule="trimmed_mean", trim=2,
                         n_instances=3, eps=1e-9, max_rounds=300, seed=3),
    "regular_b16_loss": Config(n_nodes=2000, topology="random_regular", degree=16, rule="trimmed_mean", trim=3,
                               n_instances=16, loss_p=0.1, eps=1e-8, max_rounds=300, seed=4),
    "regular_b17_loss": Config(n_nodes=2000, topology="random_regular", degree=16, rule="trimmed_mean", trim=3,
                               n_instances=17, loss_p=0.1, eps=1e-8, max_rounds=300, seed=4),
    # batched complete graphs (cfg1 shape), 12 and 40 instances
    "batched_b12": preset("cfg1", n_instances=12),
    "batched_b40": preset("cfg1", n_instances=40),
    # persistent dense kernel (cfg2 shape, smaller)
    "dense_b2": preset("cfg2", n_nodes=256, trim=85, n_faulty=85, n_instances=2),
}

STEPS = [1, 3, 16, 5, 17, 2]


def bits(v):
    return np.float64(v).view(np.uint64)


@pytest.mark.parametrize("name", list(CASES))
def test_round_info_and_getters_match_oracle_every_call(oracle_mod, name):
    cfg = CASES[name]
    with acsim.Simulator(cfg, device=0) as g, oracle_mod.OracleSimulator(cfg, threads=8) as o:
        for call in range(200):
            k = STEPS[call % len(STEPS)]
            gi, oi = g.round(k), o.round(k)
            where = (name, call, k)
            assert gi.round == oi.round, where
            assert gi.done == bool(oi.done), where
            assert gi.instances_done == oi.instances_done, where
            assert bits(gi.spread) == bits(oi.spread), where
            assert bits(gi.lo) == bits(oi.lo) and bits(gi.hi) == bits(oi.hi), where
            assert np.array_equal(g.rounds(), o.rounds()), where
            assert np.array_equal(g.converged(), o.converged()), where
            assert np.array_equal(g.spread().view(np.uint64), o.spread().view(np.uint64)), where
            if gi.done:
                break
        assert gi.done
