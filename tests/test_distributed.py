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


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_group_torch_free(tmp_path, oracle_mod, world):
    """bench.py's control plane (acsim/rendezvous.py): all-gather, barrier, broadcast, max / min /
    sum, and the sharded run's statistics reduction over plain sockets, launched by
    torch.distributed.run like the driver's N > 1 bench; the workers never import torch."""
    out = tmp_path / "verdict.json"
    # the rendezvous listens on its own port (not MASTER_PORT + 1, which nothing reserved)
    env = dict(os.environ, OMP_NUM_THREADS="1", ACSIM_RDZV_PORT=str(free_port()),
               ACSIM_RDZV_TOKEN="test-token")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(HERE, "rdzv_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    v = json.load(open(out))
    assert v["world"] == world
    assert v["gather_ok"] and v["broadcast_ok"]
    assert v["max"] == world - 1 and v["min"] == 0
    assert v["sum"] == [k * world * (world + 1) // 2 for k in range(4)]
    assert v["rounds_equal"] and v["values_equal"]
    assert v["n_instances"] == 37 and v["hist_total"] == 37
    assert v["n_converged"] == v["ref_converged"]
    assert v["node_rounds"] == v["ref_node_rounds"]
    assert v["max_over_ranks"] == world - 1
    assert not v["torch_imported"]


def test_rendezvous_rejects_oversized_message_and_bad_token():
    """Hardening (acsim/rendezvous.py): rank 0 refuses a message above the size cap and a hello
    whose token differs, with a ConnectionError instead of allocating or admitting it."""
    import struct
    import threading
    import time
    from acsim import rendezvous as R

    def serve(port, token, errs):
        try:
            R.Group(0, 2, "127.0.0.1", port, timeout=20.0, token=token).close()
        except ConnectionError as e:
            errs.append(str(e))

    # a client announcing a message above the cap
    port, errs = free_port(), []
    t = threading.Thread(target=serve, args=(port, "good", errs))
    t.start()
    for _ in range(400):
        try:
            c = socket.create_connection(("127.0.0.1", port), timeout=5.0)
            break
        except OSError:
            time.sleep(0.05)
    c.sendall(struct.pack("<Q", R._MAX_MSG + 1))
    t.join(30)
    c.close()
    assert errs and "exceeds" in errs[0]
    # a rank whose token differs
    port, errs = free_port(), []
    t = threading.Thread(target=serve, args=(port, "good", errs))
    t.start()
    g = R.Group(1, 2, "127.0.0.1", port, timeout=20.0, token="bad")
    t.join(30)
    g.close()
    assert errs and "unexpected hello" in errs[0]


def test_rendezvous_single_rank_is_local():
    from acsim.rendezvous import Group
    g = Group(0, 1)
    assert g.all_gather(5) == [5] and g.max(2.0) == 2.0 and g.broadcast(b"x") == b"x"
    g.barrier()
    g.close()


def test_rendezvous_on_a_loopback_address_other_than_127_0_0_1():
    """MASTER_ADDR = 127.0.1.1 (Debian's hostname mapping) or 127.0.0.2: rank 0 listens on the
    address the other ranks connect to (it used to bind 127.0.0.1 for every 127.x
    address, and the other rank was refused until the rendezvous timed out)."""
    import threading
    from acsim import rendezvous as R

    for addr in ("127.0.0.2", "127.0.1.1"):
        port, res = free_port(), {}

        def serve():
            g = R.Group(0, 2, addr, port, timeout=20.0, token="t")
            res["gather"] = g.all_gather(0)
            g.close()

        t = threading.Thread(target=serve)
        t.start()
        g = R.Group(1, 2, addr, port, timeout=20.0, token="t")
        mine = g.all_gather(1)
        g.close()
        t.join(30)
        assert mine == [0, 1] and res["gather"] == [0, 1], addr
