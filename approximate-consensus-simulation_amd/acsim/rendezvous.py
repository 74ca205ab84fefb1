"""Torch-free control plane for one process per GPU on one node.

The data path of a node partition is RCCL inside libacsim.so (acs_create_partitioned); the ranks
only need a few host-side exchanges around it: the RCCL unique id from rank 0, barriers,
max / min / sum of a few scalars and the gather of per-rank results.  Doing those over
torch.distributed would load torch's own HIP runtime and RCCL into every rank before libacsim.so,
and the dynamic loader would then bind libacsim.so to them instead of the ROCm libraries it was
built and tested against (RUNPATH /opt/rocm/lib).  This module does the exchanges over plain TCP
sockets instead, so a rank process maps exactly one HIP runtime and one RCCL: the ones the GPU
test suite runs on.

Topology: a star.  Rank 0 listens, every other rank connects once and stays connected; every
collective is "each rank sends one message to rank 0, rank 0 answers everyone with the list of
all messages" (an all-gather), on which barrier / broadcast / reductions are built.  Messages are
length-prefixed msgpack (bytes, ints, floats, strings, lists, dicts; tuples arrive as lists).

Rendezvous: `Group.from_env()` reads RANK / WORLD_SIZE / MASTER_ADDR as torch.distributed.run sets
them and listens on MASTER_PORT + 1 (torch's launcher keeps its own store on MASTER_PORT), or on
ACSIM_RDZV_PORT when that is set.

Hardening (the listener is unauthenticated): a message may not exceed ACSIM_RDZV_MAX_MSG bytes
(64 MiB by default), so a stray connection cannot make rank 0 allocate arbitrary memory; the
listener binds to the loopback interface when MASTER_ADDR is local (127.0.0.0/8 or localhost);
and when ACSIM_RDZV_TOKEN is set, every rank's hello must carry the same token.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Any, List, Optional

import msgpack
import numpy as np

_HDR = struct.Struct("<Q")
_MAX_MSG = int(os.environ.get("ACSIM_RDZV_MAX_MSG", str(64 << 20)))


def _send(sock: socket.socket, obj: Any) -> None:
    data = msgpack.packb(obj, use_bin_type=True)
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket) -> Any:
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    if n > _MAX_MSG:
        raise ConnectionError(f"rendezvous: message of {n} B exceeds the {_MAX_MSG} B cap "
                              f"(ACSIM_RDZV_MAX_MSG)")
    return msgpack.unpackb(_recv_exact(sock, n), raw=False)


def _bind_addr(addr: str) -> str:
    """The address rank 0 listens on: the one the other ranks connect to.  "localhost" becomes
    127.0.0.1; any other name or literal (127.0.1.1, Debian's hostname mapping, included) is bound
    as given, so a loopback address other than 127.0.0.1 is reachable too."""
    return "127.0.0.1" if addr == "localhost" else addr


class Group:
    """A fixed set of `world` ranks exchanging small messages through rank 0."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29501,
                 timeout: float = 600.0, token: Optional[str] = None):
        if world < 1 or not (0 <= rank < world):
            raise ValueError(f"bad rank {rank} / world {world}")
        self.rank, self.world = rank, world
        self._peers: List[socket.socket] = []   # rank 0: index k = rank k + 1
        self._up: Optional[socket.socket] = None  # ranks > 0: the connection to rank 0
        self._srv: Optional[socket.socket] = None
        if world == 1:
            return
        deadline = time.monotonic() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                srv.bind((_bind_addr(addr), port))
            except OSError as e:
                srv.close()
                raise ConnectionError(
                    f"rendezvous: rank 0 cannot listen on {addr}:{port} ({e}); the port defaults to "
                    f"MASTER_PORT + 1 — set ACSIM_RDZV_PORT to a free port") from e
            srv.listen(world)
            srv.settimeout(max(1.0, deadline - time.monotonic()))
            self._srv = srv
            peers: List[Optional[socket.socket]] = [None] * (world - 1)
            for _ in range(world - 1):
                c, _a = srv.accept()
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(timeout)
                hello = _recv(c)
                r = hello[0] if isinstance(hello, list) and len(hello) == 2 else None
                if (not isinstance(r, int) or not (1 <= r < world) or peers[r - 1] is not None
                        or hello[1] != token):
                    c.close()
                    raise ConnectionError(f"rendezvous: unexpected hello {hello!r}")
                peers[r - 1] = c
            self._peers = peers  # type: ignore[assignment]
        else:
            last = None
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError as e:   # rank 0 not listening yet
                    last = e
                    if time.monotonic() > deadline:
                        raise ConnectionError(f"rendezvous: no rank 0 at {addr}:{port}: {last}") from e
                    time.sleep(0.05)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.settimeout(timeout)
            _send(c, [rank, token])
            self._up = c

    @classmethod
    def from_env(cls, timeout: float = 600.0) -> "Group":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        if "ACSIM_RDZV_PORT" in os.environ:
            port = int(os.environ["ACSIM_RDZV_PORT"])
        else:
            port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        return cls(rank, world, addr, port, timeout, os.environ.get("ACSIM_RDZV_TOKEN"))

    # ---- collectives (every rank calls them in the same order)
    def all_gather(self, obj: Any) -> list:
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [_recv(p) for p in self._peers]
            for p in self._peers:
                _send(p, out)
            return out
        _send(self._up, obj)
        return _recv(self._up)

    def barrier(self) -> None:
        self.all_gather(None)

    def broadcast(self, obj: Any = None, src: int = 0) -> Any:
        return self.all_gather(obj if self.rank == src else None)[src]

    def max(self, v: float) -> float:
        return max(self.all_gather(float(v)))

    def min(self, v: float) -> float:
        return min(self.all_gather(float(v)))

    def sum(self, v):
        """Sum of a number, or elementwise of a numpy array (same shape and dtype on every rank)."""
        if isinstance(v, np.ndarray):
            a = np.ascontiguousarray(v)
            parts = self.all_gather(a.tobytes())
            return sum((np.frombuffer(p, dtype=a.dtype).reshape(a.shape) for p in parts[1:]),
                       np.frombuffer(parts[0], dtype=a.dtype).reshape(a.shape).copy())
        vals = self.all_gather(v)
        total = vals[0]
        for x in vals[1:]:
            total = total + x
        return total

    def close(self) -> None:
        for s in self._peers + ([self._up] if self._up else []) + ([self._srv] if self._srv else []):
            try:
                s.close()
            except OSError:
                pass
        self._peers, self._up, self._srv = [], None, None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
