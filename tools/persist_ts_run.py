"""Record an ACSIM_PERSIST_TS timeline: cfg4-shaped run, 5 warm-up rounds, then one timed launch of
K rounds.  usage: python tools/persist_ts_run.py OUT.csv [n_nodes] [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
k = int(sys.argv[3]) if len(sys.argv) > 3 else 10
with acsim.Simulator(acsim.preset("cfg4", n_nodes=n, max_rounds=5 + k), device=0) as g:
    g.round(5)
    os.environ["ACSIM_PERSIST_TS"] = out
    g.round(k)
    print(g.kernel_name(), int(g.rounds()[0]))
