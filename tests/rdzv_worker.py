"""Worker for tests/test_distributed.py: the torch-free control plane (acsim/rendezvous.py) that
bench.py's ranks use.  Launched by torch.distributed.run (which sets RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT); the worker itself never imports torch.  It runs every collective,
then the sharded cfg3-style run with the CPU oracle as the per-rank simulator, and rank 0 writes a
JSON verdict against the unsharded run.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "approximate-consensus-simulation_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from acsim import distributed as D  # noqa: E402
from acsim.config import Config  # noqa: E402
from acsim.rendezvous import Group  # noqa: E402


def main():
    out = sys.argv[1]
    g = Group.from_env(timeout=120)
    rank, world = g.rank, g.world
    gathered = g.all_gather({"rank": rank, "blob": bytes([rank]) * 3, "v": [rank, 0.5]})
    g.barrier()
    bc = g.broadcast(b"id-from-0" if rank == 0 else None)
    mx, mn = g.max(float(rank)), g.min(float(rank))
    sm = g.sum(np.arange(4, dtype=np.int64) * (rank + 1))
    cfg = Config(n_nodes=24, n_instances=37, topology="complete", rule="average", loss_p=0.2,
                 mask_group=3, eps=1e-7, max_rounds=200, seed=5)
    stats, rounds, values = D.run_sharded(cfg, rank, world, device=0, group=g,
                                          sim_factory=lambda c, d: O.OracleSimulator(c),
                                          return_values=True)
    tmax = D.max_over_ranks(float(rank), group=g)
    parts = g.all_gather([rank, rounds.astype(np.uint32).tobytes(), values.tobytes()])
    if rank == 0:
        all_rounds = np.concatenate([np.frombuffer(p[1], dtype=np.uint32) for p in sorted(parts)])
        all_vals = np.concatenate([np.frombuffer(p[2], dtype=np.float64) for p in sorted(parts)])
        with O.OracleSimulator(cfg) as ref:
            ref.run()
            ref_rounds = ref.rounds()
            verdict = {
                "world": world,
                "gather_ok": [x["rank"] for x in gathered] == list(range(world))
                             and all(x["blob"] == bytes([x["rank"]]) * 3 for x in gathered),
                "broadcast_ok": bc == b"id-from-0",
                "max": mx, "min": mn, "sum": [int(v) for v in sm],
                "rounds_equal": bool(np.array_equal(all_rounds, ref_rounds)),
                "values_equal": bool(np.array_equal(all_vals.view(np.uint64), ref.all_values().ravel().view(np.uint64))),
                "n_instances": stats.n_instances,
                "n_converged": stats.n_converged,
                "ref_converged": int(ref.converged().sum()),
                "node_rounds": stats.node_rounds,
                "ref_node_rounds": int(cfg.n_nodes) * int(np.sum(ref_rounds)),
                "hist_total": int(stats.rounds_hist.sum()),
                "max_over_ranks": tmax,
                "torch_imported": "torch" in sys.modules,
            }
        json.dump(verdict, open(out, "w"))
    g.barrier()
    g.close()


if __name__ == "__main__":
    main()
