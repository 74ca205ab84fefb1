"""N > 1 path on CPU: instance sharding + final statistics reduction over gloo with
world sizes 2 and 3; results must equal an unsharded run instance for instance."""
import json
import os
import socket
import subprocess
import sys

import pytest

from acsim.distributed import shard_range

HERE = os.path.dirname(os.path.abspath(__file__))


def test_shard_range_partitions_exactly():
    for B in (1, 2, 7, 100, 100000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(B, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (o1, c1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + c1 == o2
            assert sum(c for _, c in spans) == B
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_unsharded_gloo(tmp_path, oracle_mod, world):
    out = tmp_path / "verdict.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "dist_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    v = json.load(open(out))
    assert v["world"] == world
    assert v["rounds_equal"] and v["values_equal"]
    assert v["n_instances"] == 37
    assert v["n_converged"] == v["ref_converged"]
    assert v["node_rounds"] == v["ref_node_rounds"]
    assert v["rounds_max"] == v["ref_rounds_max"]
    assert v["hist_total"] == 37
    assert v["max_over_ranks"] == world - 1
