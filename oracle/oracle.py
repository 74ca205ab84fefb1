"""ctypes wrapper of the CPU spec restatement (oracle/acs_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline.  Upstream parity is UNPINNED (the reference
mount has no code); see acs_oracle.h for what pins this restatement.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG_ROOT = os.path.join(os.path.dirname(_HERE), "approximate-consensus-simulation_amd")
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

from acsim import _abi  # noqa: E402  (struct definitions only: the ABI is shared)
from acsim.config import Config, preset  # noqa: E402

LIB_PATH = os.path.join(_HERE, "build", "libacs_oracle.so")
_lib = None


def build() -> None:
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    P = C.POINTER
    sigs = {
        "acso_philox4x32_10": (None, [P(u32), P(u32), P(u32)]),
        "acso_draw": (u32, [u64, u32, u32, u32, u64]),
        "acso_u53": (C.c_double, [u32, u32]),
        "acso_feistel_perm": (u64, [u64, u64, u32, u64, i32]),
        "acso_drop_threshold": (u32, [C.c_double]),
        "acso_tree_sum": (C.c_double, [P(C.c_double), u64]),
        "acso_validate": (i32, [P(_abi.AcsConfig)]),
        "acso_create": (i32, [P(_abi.AcsConfig), P(vp)]),
        "acso_create_csr": (i32, [P(_abi.AcsConfig), P(u64), P(u32), P(vp)]),
        "acso_round": (i32, [vp, u32, P(_abi.AcsRoundInfo)]),
        "acso_run": (i32, [vp, P(_abi.AcsResult)]),
        "acso_get_values": (i32, [vp, u64, P(C.c_double), u64]),
        "acso_get_instance_rounds": (i32, [vp, P(u32), u64]),
        "acso_get_instance_converged": (i32, [vp, P(C.c_uint8), u64]),
        "acso_get_instance_spread": (i32, [vp, P(C.c_double), u64]),
        "acso_get_spread_trace": (i32, [vp, u64, P(C.c_double), u64, P(u64)]),
        "acso_set_state": (i32, [vp, u32, P(C.c_double), u64]),
        "acso_get_fault_status": (i32, [vp, P(u32), u64]),
        "acso_get_neighbors": (i32, [vp, P(u32), u64]),
        "acso_destroy": (None, [vp]),
        "acso_last_error": (C.c_char_p, []),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _chk(code: int) -> None:
    if code != 0:
        raise _abi.AcsError(code, load().acso_last_error().decode())


# ------------------------------------------------------------------------------ primitives
def philox(ctr, key) -> tuple:
    lib = load()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.acso_philox4x32_10(c, k, o)
    return tuple(o)


def draw(seed, stream, b, r, s) -> int:
    return load().acso_draw(seed, stream, b, r, s)


def feistel(n, graph_seed, k, v, inverse=False) -> int:
    return load().acso_feistel_perm(n, graph_seed, k, v, 1 if inverse else 0)


def drop_threshold(p) -> int:
    return load().acso_drop_threshold(p)


def tree_sum(a) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return load().acso_tree_sum(a.ctypes.data_as(C.POINTER(C.c_double)), a.size)


def validate(cfg: Config) -> int:
    c = cfg.to_c()
    return load().acso_validate(C.byref(c))


# ------------------------------------------------------------------------------ simulation
class OracleSimulator:
    """Same surface as acsim.Simulator, backed by the CPU spec restatement."""

    def __init__(self, cfg: Config | str, threads: int = 1, csr=None):
        if isinstance(cfg, str):
            cfg = preset(cfg)
        if threads and not cfg.omp_threads:
            cfg = cfg.replace(omp_threads=threads)
        self.cfg = cfg
        self._lib = load()
        self._c = cfg.to_c()
        h = C.c_void_p()
        if csr is None:
            _chk(self._lib.acso_create(C.byref(self._c), C.byref(h)))
        else:
            rp = np.ascontiguousarray(csr[0], dtype=np.uint64)
            ci = np.ascontiguousarray(csr[1], dtype=np.uint32)
            _chk(self._lib.acso_create_csr(C.byref(self._c), rp.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           ci.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.acso_destroy(self._h)
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *e):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def N(self):
        return int(self.cfg.n_nodes)

    @property
    def B(self):
        return int(self.cfg.n_instances)

    def round(self, k=1):
        info = _abi.AcsRoundInfo()
        _chk(self._lib.acso_round(self._h, int(k), C.byref(info)))
        return info

    def run(self):
        res = _abi.AcsResult()
        _chk(self._lib.acso_run(self._h, C.byref(res)))
        return res

    @property
    def f32(self):
        return int(self._c.dtype) == _abi.F32

    def values(self, instance=0):
        """Node values in the config dtype (fp32 values are held exactly as doubles in C)."""
        out = np.empty(self.N, dtype=np.float64)
        _chk(self._lib.acso_get_values(self._h, int(instance),
                                       out.ctypes.data_as(C.POINTER(C.c_double)), out.size))
        return out.astype(np.float32) if self.f32 else out

    def all_values(self):
        return np.stack([self.values(b) for b in range(self.B)])

    def rounds(self):
        out = np.empty(self.B, dtype=np.uint32)
        _chk(self._lib.acso_get_instance_rounds(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                out.size))
        return out

    def converged(self):
        out = np.empty(self.B, dtype=np.uint8)
        _chk(self._lib.acso_get_instance_converged(
            self._h, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size))
        return out.astype(bool)

    def spread(self):
        out = np.empty(self.B, dtype=np.float64)
        _chk(self._lib.acso_get_instance_spread(self._h, out.ctypes.data_as(C.POINTER(C.c_double)),
                                                out.size))
        return out

    def spread_trace(self, instance=0):
        n = int(self.cfg.max_rounds) + 1
        out = np.empty(n, dtype=np.float64)
        got = C.c_uint64()
        _chk(self._lib.acso_get_spread_trace(self._h, int(instance),
                                             out.ctypes.data_as(C.POINTER(C.c_double)), n,
                                             C.byref(got)))
        return out[: got.value].copy()

    def set_state(self, round, x):
        x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
        _chk(self._lib.acso_set_state(self._h, int(round), x.ctypes.data_as(C.POINTER(C.c_double)),
                                      x.size))

    def fault_status(self):
        out = np.empty(self.B * self.N, dtype=np.uint32)
        _chk(self._lib.acso_get_fault_status(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                                             out.size))
        return out.reshape(self.B, self.N)

    def neighbors(self):
        d = int(self.cfg.degree)
        out = np.empty(self.N * d, dtype=np.uint32)
        _chk(self._lib.acso_get_neighbors(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32)),
                                          out.size))
        return out.reshape(self.N, d)
