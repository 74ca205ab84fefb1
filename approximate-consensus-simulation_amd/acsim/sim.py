"""User-facing API: ``simulate(cfg)`` and ``Simulator(cfg).round(k)``.

Thin ctypes layer over libacsim.so (include/acsim.h).  The per-round hot path runs in the
library's HIP kernels; this module only marshals configs and host buffers.  There is no CPU
fallback: ``backend="cpu"`` is rejected (the CPU spec reference is test infrastructure in
oracle/, not part of the product).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _abi
from .config import Config, preset


@dataclass
class RoundInfo:
    round: int
    done: bool
    spread: float
    lo: float
    hi: float
    instances_done: int


@dataclass
class Result:
    rounds: np.ndarray          # uint32 [B]
    converged: np.ndarray       # bool [B]
    spread: np.ndarray          # float64 [B], final spread per instance
    node_rounds: int
    wall_seconds: float
    rounds_max: int
    x_final: Optional[np.ndarray] = None      # [N] for B == 1, [B, N] otherwise (if requested)
    spread_trace: Optional[np.ndarray] = None  # instance 0, if cfg.trace_spread


class Simulator:
    """One device-resident simulation handle (``acs_sim``)."""

    def __init__(self, cfg: Config | str, device: int = 0, backend: str = "hip",
                 partitions: int = 1, rank: int = 0, comm_id: Optional[bytes] = None,
                 csr=None):
        """partitions > 1 node-partitions one RANDOM_REGULAR instance: with
        comm_id (RCCL unique id from acsim.distributed) this handle is `rank`'s partition on
        `device`; without it all partitions are simulated on `device` with private x copies
        (validation mode, see include/acsim.h acs_create_partitioned)."""
        if isinstance(cfg, str):
            cfg = preset(cfg)
        if backend != "hip":
            raise ValueError("acsim implements backend='hip' only; the CPU spec reference is "
                             "test infrastructure (oracle/) and is not a product backend")
        self.cfg = cfg
        self.partitions = int(partitions)
        self._lib = _abi.load_library()
        self._c = cfg.to_c()
        h = C.c_void_p()
        if csr is not None:   # user graph (topology="csr"): csr = (rowptr[N+1], colidx[nnz])
            rp = np.ascontiguousarray(csr[0], dtype=np.uint64)
            ci = np.ascontiguousarray(csr[1], dtype=np.uint32)
            if rp.size != int(cfg.n_nodes) + 1:
                raise ValueError("rowptr must have n_nodes + 1 entries")
            rc = self._lib.acs_create_csr(C.byref(self._c), rp.ctypes.data_as(C.POINTER(C.c_uint64)),
                                          ci.ctypes.data_as(C.POINTER(C.c_uint32)), int(device), C.byref(h))
        elif self.partitions == 1 and comm_id is None:
            devs = (C.c_int * 1)(int(device))
            rc = self._lib.acs_create(C.byref(self._c), _abi.BACKEND_HIP, devs, 1, C.byref(h))
        else:
            idbuf = None if comm_id is None else C.create_string_buffer(bytes(comm_id), len(comm_id))
            rc = self._lib.acs_create_partitioned(C.byref(self._c), int(device), self.partitions,
                                                  int(rank), idbuf, 0 if comm_id is None else len(comm_id),
                                                  C.byref(h))
        _abi.check(self._lib, rc)
        self._h = h

    # -------------------------------------------------------------------------- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.acs_destroy(self._h)
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, code: int) -> None:
        _abi.check(self._lib, code)

    @property
    def N(self) -> int:
        return int(self.cfg.n_nodes)

    @property
    def B(self) -> int:
        return int(self.cfg.n_instances)

    # -------------------------------------------------------------------------- stepping
    def round(self, k: int = 1) -> RoundInfo:
        """Advance every unfinished instance by at most k rounds (stops at convergence)."""
        info = _abi.AcsRoundInfo()
        self._chk(self._lib.acs_round(self._h, int(k), C.byref(info)))
        return RoundInfo(info.round, bool(info.done), info.spread, info.lo, info.hi,
                         info.instances_done)

    def run(self) -> _abi.AcsResult:
        res = _abi.AcsResult()
        self._chk(self._lib.acs_run(self._h, C.byref(res)))
        return res

    def sync(self) -> None:
        self._chk(self._lib.acs_sync(self._h))

    # -------------------------------------------------------------------------- state access
    @property
    def value_dtype(self):
        """numpy dtype of node values: float64, or float32 for dtype="f32" (DESIGN.md §9)."""
        return np.float32 if int(self._c.dtype) == _abi.F32 else np.float64

    def values(self, instance: int = 0) -> np.ndarray:
        out = np.empty(self.N, dtype=self.value_dtype)
        self._chk(self._lib.acs_get_values(self._h, int(instance), out.ctypes.data, out.size))
        return out

    def partition_values(self, partition: int) -> np.ndarray:
        """Virtual partitions: the private x copy of one partition."""
        out = np.empty(self.N, dtype=self.value_dtype)
        self._chk(self._lib.acs_get_partition_values(self._h, int(partition), out.ctypes.data, out.size))
        return out

    def all_values(self) -> np.ndarray:
        """[B, N] values of every instance (one ABI call: acs_get_all_values)."""
        out = np.empty((self.B, self.N), dtype=self.value_dtype)
        self._chk(self._lib.acs_get_all_values(self._h, out.ctypes.data, out.size))
        return out

    def rounds(self) -> np.ndarray:
        out = np.empty(self.B, dtype=np.uint32)
        self._chk(self._lib.acs_get_instance_rounds(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        return out

    def converged(self) -> np.ndarray:
        out = np.empty(self.B, dtype=np.uint8)
        self._chk(self._lib.acs_get_instance_converged(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size))
        return out.astype(bool)

    def spread(self) -> np.ndarray:
        out = np.empty(self.B, dtype=np.float64)
        self._chk(self._lib.acs_get_instance_spread(
            self._h, out.ctypes.data_as(C.POINTER(C.c_double)), out.size))
        return out

    def spread_trace(self, instance: int = 0) -> np.ndarray:
        n = int(self.cfg.max_rounds) + 1
        out = np.empty(n, dtype=np.float64)
        got = C.c_uint64()
        self._chk(self._lib.acs_get_spread_trace(
            self._h, int(instance), out.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(got)))
        return out[: got.value].copy()

    def set_state(self, round: int, x: np.ndarray) -> None:
        xv = np.asarray(x)
        if self.value_dtype == np.float32 and xv.dtype != np.float32 and not np.array_equal(
                xv.astype(np.float32).astype(xv.dtype), xv):
            raise ValueError("fp32 set_state: values must be exactly representable in binary32")
        x = np.ascontiguousarray(xv, dtype=self.value_dtype).reshape(-1)
        self._chk(self._lib.acs_set_state(self._h, int(round), x.ctypes.data, x.size))

    def fault_status(self) -> np.ndarray:
        out = np.empty(self.B * self.N, dtype=np.uint32)
        self._chk(self._lib.acs_get_fault_status(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        return out.reshape(self.B, self.N)

    def neighbors(self) -> np.ndarray:
        d = int(self.cfg.degree)
        out = np.empty(self.N * d, dtype=np.uint32)
        self._chk(self._lib.acs_get_neighbors(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        return out.reshape(self.N, d)

    # -------------------------------------------------------------------------- measurement
    def set_kernel_timing(self, enable, every: int = 1, runs: bool = False) -> None:
        """Bracket round-kernel launches with HIP events: every `every`-th round when enabled, or
        with runs=True one event pair around each run of `every` consecutive rounds (no idle gap
        inside the run; every round counts as one launch)."""
        k = max(1, int(every)) if enable else 0
        self._chk(self._lib.acs_set_kernel_timing(self._h, -k if runs else k))

    def kernel_timing(self):
        """(total_ms, launches, kernel_name) of the round kernel since timing was enabled."""
        ms = C.c_double()
        n = C.c_uint64()
        name = C.create_string_buffer(256)
        self._chk(self._lib.acs_get_kernel_timing(self._h, C.byref(ms), C.byref(n), name, 256))
        return ms.value, n.value, name.value.decode()

    def kernel_name(self) -> str:
        """Name of the round kernel(s) this handle's path launches."""
        return self.kernel_timing()[2]


def simulate(cfg: Config | str, backend: str = "hip", device: int = 0,
             devices: Optional[Sequence[int]] = None, return_values: bool = True,
             csr=None) -> Result:
    """Run one configuration to termination and return its results."""
    if devices is not None:
        devices = list(devices)
        if len(devices) != 1:
            raise ValueError("simulate() drives one device per process; shard instances across "
                             "processes with acsim.distributed (one rank per GPU)")
        device = devices[0]
    with Simulator(cfg, device=device, backend=backend, csr=csr) as sim:
        res = sim.run()
        x = None
        if return_values:
            x = sim.values(0) if sim.B == 1 else sim.all_values()
        trace = sim.spread_trace(0) if sim.cfg.trace_spread else None
        return Result(rounds=sim.rounds(), converged=sim.converged(), spread=sim.spread(),
                      node_rounds=int(res.node_rounds), wall_seconds=float(res.wall_seconds),
                      rounds_max=int(res.rounds_max), x_final=x, spread_trace=trace)
