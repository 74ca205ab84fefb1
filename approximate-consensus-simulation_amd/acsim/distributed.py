"""Multi-GPU orchestration, one process per GPU.

Independent instances (cfg3) shard with NO data-path collective: rank r owns the contiguous
global instance block [offset, offset + count) and runs it on its own GPU; Philox counters carry
the GLOBAL instance id (acs_config.instance_offset), so results are identical at any world size.
The only cross-rank step is the final statistics reduction (one all_reduce of a few scalars and
a rounds histogram).  Every control-plane function takes `group`: an `acsim.rendezvous.Group`
(torch-free sockets: the rank then maps only the HIP runtime and RCCL libacsim.so was built
against; bench.py uses it) or, when `group` is None or a torch ProcessGroup, torch.distributed
(gloo or nccl=RCCL) for callers that already run one.

Single-instance configs (cfg1, cfg2, cfg4) do not shard: at N GPUs they run N independent
replicas (distinct global instance ids), which is what bench.py measures for N > 1.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np

from .config import Config


def shard_range(n_instances: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of instances for `rank`: (offset, count); sizes differ by at most 1."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(int(n_instances), world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


@dataclass
class ShardStats:
    n_instances: int
    n_converged: int
    node_rounds: int
    rounds_max: int
    rounds_hist: np.ndarray      # histogram of per-instance rounds, bins 0..max_rounds
    spread_max: float


def local_stats(cfg: Config, rounds: np.ndarray, converged: np.ndarray, spread: np.ndarray) -> ShardStats:
    hist = np.bincount(rounds.astype(np.int64), minlength=int(cfg.max_rounds) + 1)
    return ShardStats(n_instances=int(rounds.size), n_converged=int(converged.sum()),
                      node_rounds=int(cfg.n_nodes) * int(rounds.astype(np.int64).sum()),
                      rounds_max=int(rounds.max()) if rounds.size else 0,
                      rounds_hist=hist.astype(np.int64),
                      spread_max=float(spread.max()) if spread.size else float("-inf"))


def _is_rdzv(group) -> bool:
    from .rendezvous import Group
    return isinstance(group, Group)


def reduce_stats(s: ShardStats, group=None) -> ShardStats:
    """All-reduce shard statistics (sum counts / max extrema) over `group`."""
    if _is_rdzv(group):
        parts = group.all_gather([s.n_instances, s.n_converged, s.node_rounds, s.rounds_max,
                                  s.rounds_hist.astype(np.int64).tobytes(), s.spread_max])
        hist = np.zeros_like(s.rounds_hist, dtype=np.int64)
        for p in parts:
            hist += np.frombuffer(p[4], dtype=np.int64)
        return ShardStats(n_instances=sum(p[0] for p in parts), n_converged=sum(p[1] for p in parts),
                          node_rounds=sum(p[2] for p in parts), rounds_max=max(p[3] for p in parts),
                          rounds_hist=hist, spread_max=max(p[5] for p in parts))
    import torch
    import torch.distributed as dist
    ints = torch.tensor([s.n_instances, s.n_converged, s.node_rounds], dtype=torch.int64)
    hist = torch.from_numpy(s.rounds_hist.copy())
    mx = torch.tensor([float(s.rounds_max), s.spread_max], dtype=torch.float64)
    dist.all_reduce(ints, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    return ShardStats(n_instances=int(ints[0]), n_converged=int(ints[1]), node_rounds=int(ints[2]),
                      rounds_max=int(mx[0]), rounds_hist=hist.numpy(), spread_max=float(mx[1]))


def max_over_ranks(value: float, group=None) -> float:
    if _is_rdzv(group):
        return group.max(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def make_comm_id(rank: int, group=None, src: int = 0) -> bytes:
    """RCCL unique id created on `src` and broadcast over `group` (a rendezvous Group, or
    torch.distributed gloo / nccl)."""
    from . import _abi
    import ctypes as C
    obj = [None]
    if rank == src:
        lib = _abi.load_library()
        n = lib.acs_comm_id_size()
        buf = C.create_string_buffer(n)
        _abi.check(lib, lib.acs_get_comm_id(buf, n))
        obj = [buf.raw]
    if _is_rdzv(group):
        return group.broadcast(obj[0], src=src)
    import torch.distributed as dist
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]


def partitioned_simulator(cfg: Config, rank: int, world: int, device: int, group=None):
    """This rank's node partition of one RANDOM_REGULAR instance (cfg5): rows of the graph are
    split over `world` GPUs, x^{r+1} is all-gathered over RCCL every round."""
    from .sim import Simulator
    cid = make_comm_id(rank, group)
    return Simulator(cfg, device=device, partitions=world, rank=rank, comm_id=cid)


def run_sharded(cfg: Config, rank: int, world: int, device: int = 0,
                sim_factory: Optional[Callable] = None, group=None,
                return_values: bool = False):
    """Run this rank's instance block of `cfg` and reduce the statistics over all ranks.

    sim_factory(cfg, device) -> simulator (default: acsim.Simulator on `device`); tests pass
    the CPU oracle here to exercise the sharding and reduction logic without a GPU.
    Returns (global ShardStats, local rounds array, local values or None).
    """
    off, cnt = shard_range(cfg.n_instances, world, rank)
    local = cfg.replace(n_instances=max(cnt, 1), instance_offset=int(cfg.instance_offset) + off)
    if sim_factory is None:
        from .sim import Simulator
        sim_factory = lambda c, d: Simulator(c, device=d)  # noqa: E731
    if cnt == 0:   # more ranks than instances: contribute nothing
        empty = ShardStats(0, 0, 0, 0, np.zeros(int(cfg.max_rounds) + 1, np.int64), float("-inf"))
        return reduce_stats(empty, group), np.zeros(0, np.uint32), None
    with sim_factory(local, device) as sim:
        sim.run()
        rounds, conv, spread = sim.rounds(), sim.converged(), sim.spread()
        values = sim.all_values() if return_values else None
    return reduce_stats(local_stats(local, rounds, conv, spread), group), rounds, values
