import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim
from acsim.config import Config

def run(cfg, binned):
    os.environ["ACSIM_BINNED"] = "1" if binned else "0"
    with acsim.Simulator(cfg, device=0) as g:
        g.run()
        return g.values(0).copy(), g.fault_status()[0].copy(), g.neighbors().copy()

for R in (1, 2, 3, 4):
    cfg = Config(n_nodes=20000, topology="regular", degree=16, rule="trimmed", trim=5, fault_model="crash",
                 n_faulty=3000, crash_window=6, termination="fixed", max_rounds=R, seed=43)
    xb, st, nb = run(cfg, True)
    xr, _, _ = run(cfg, False)
    diff = np.nonzero(xb.view(np.uint64) != xr.view(np.uint64))[0]
    print(f"R={R}: {len(diff)} receivers differ", flush=True)
    if R == 1 or R == 2:
        nbr = nb.reshape(cfg.n_nodes, 16)
        for i in diff[:6]:
            sts = st[nbr[i]]
            print(f"  i={i} st_i={st[i]:#x} xb={xb[i]!r} xr={xr[i]!r} nbr st={[hex(v) for v in sts]}")
        # receivers with a sender crashing at round R-1 (partial) vs diffs
        r = R - 1
        cr = np.isin(st, [r])
        part = np.nonzero(cr[nbr].any(axis=1))[0]
        sil = np.nonzero(((st < r) & (st != 0xFFFFFFFF) & (st != 0xFFFFFFFE))[nbr].any(axis=1))[0]
        print(f"  receivers with a partial sender: {len(part)}, with a silent sender: {len(sil)}, "
              f"diff within partial: {np.isin(diff, part).sum()}, within silent: {np.isin(diff, sil).sum()}, "
              f"diff crashed receivers: {(st[diff] != 0xFFFFFFFF).sum()}")
