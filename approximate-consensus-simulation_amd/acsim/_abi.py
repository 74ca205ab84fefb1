"""ctypes mirror of include/acsim.h (the C ABI).

Field order and types follow ``acs_config`` exactly; tests/test_abi.py compiles a C probe that
prints ``offsetof`` for every field and checks it against this mirror.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 3

# status codes
OK, EINVAL, ENOMEM, EDEVICE, ECOMM, EUNSUPPORTED = 0, -1, -2, -3, -4, -5
STATUS_NAMES = {OK: "OK", EINVAL: "EINVAL", ENOMEM: "ENOMEM", EDEVICE: "EDEVICE",
                ECOMM: "ECOMM", EUNSUPPORTED: "EUNSUPPORTED"}

# backends
BACKEND_CPU, BACKEND_HIP = 0, 1

# topology / rule / faults / byz / termination / dtype
TOPO_COMPLETE, TOPO_RANDOM_REGULAR, TOPO_CSR = 0, 1, 2
RULE_AVERAGE, RULE_TRIMMED_MEAN, RULE_MIDPOINT, RULE_DLPSW_SELECT, RULE_WMSR = 0, 1, 2, 3, 4
FAULT_NONE, FAULT_CRASH, FAULT_BYZANTINE = 0, 1, 2
BYZ_SPLIT, BYZ_RANDOM, BYZ_CONSTANT = 0, 1, 2
TERM_EPS, TERM_FIXED = 0, 1
F64, F32 = 0, 1
MISSING_SELF, MISSING_OMIT = 0, 1

STREAM_INIT, STREAM_DROP, STREAM_FAULTSET, STREAM_CRASH_ROUND = 0, 1, 2, 3
STREAM_CRASH_PARTIAL, STREAM_BYZ, STREAM_GRAPH = 4, 5, 6

STATUS_HONEST = 0xFFFFFFFF
STATUS_BYZANTINE = 0xFFFFFFFE


class AcsConfig(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("n_nodes", C.c_uint64),
        ("n_instances", C.c_uint64),
        ("topology", C.c_uint32),
        ("degree", C.c_uint32),
        ("rule", C.c_uint32),
        ("trim", C.c_uint32),
        ("fault_model", C.c_uint32),
        ("n_faulty", C.c_uint32),
        ("byz_strategy", C.c_uint32),
        ("byz_delta", C.c_double),
        ("byz_const", C.c_double),
        ("crash_window", C.c_uint32),
        ("loss_p", C.c_double),
        ("mask_group", C.c_uint32),
        ("eps", C.c_double),
        ("max_rounds", C.c_uint32),
        ("termination", C.c_uint32),
        ("dtype", C.c_uint32),
        ("seed", C.c_uint64),
        ("graph_seed", C.c_uint64),
        ("trace_spread", C.c_uint32),
        ("omp_threads", C.c_uint32),
        ("instance_offset", C.c_uint64),
        ("delay_max", C.c_uint32),
        ("missing_policy", C.c_uint32),
    ]


class AcsRoundInfo(C.Structure):
    _fields_ = [
        ("round", C.c_uint32),
        ("done", C.c_uint32),
        ("spread", C.c_double),
        ("lo", C.c_double),
        ("hi", C.c_double),
        ("instances_done", C.c_uint64),
    ]


class AcsResult(C.Structure):
    _fields_ = [
        ("rounds_max", C.c_uint32),
        ("n_converged", C.c_uint32),
        ("node_rounds", C.c_uint64),
        ("wall_seconds", C.c_double),
        ("final_spread_max", C.c_double),
        ("n_instances", C.c_uint64),
    ]


class AcsError(RuntimeError):
    """A non-zero status returned across the C ABI."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG_DIR, "_lib", "libacsim.so")
# experiments only: a variant build of the same sources (Makefile OUTDIR / XFLAGS), e.g. a
# different compile-time receiver-block size; the product loads the in-tree default
if os.environ.get("ACSIM_LIB"):
    LIB_PATH = os.environ["ACSIM_LIB"]

_lib = None


def _declare(lib: C.CDLL) -> None:
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    P = C.POINTER
    sigs = {
        "acs_create": (i32, [P(AcsConfig), i32, P(C.c_int), i32, P(vp)]),
        "acs_create_csr": (i32, [P(AcsConfig), P(u64), P(u32), i32, P(vp)]),
        "acs_comm_id_size": (i32, []),
        "acs_get_comm_id": (i32, [vp, u64]),
        "acs_create_partitioned": (i32, [P(AcsConfig), i32, i32, i32, vp, u64, P(vp)]),
        "acs_get_partition_values": (i32, [vp, i32, vp, u64]),
        "acs_round": (i32, [vp, u32, P(AcsRoundInfo)]),
        "acs_run": (i32, [vp, P(AcsResult)]),
        "acs_get_values": (i32, [vp, u64, vp, u64]),
        "acs_get_all_values": (i32, [vp, vp, u64]),
        "acs_get_instance_rounds": (i32, [vp, P(u32), u64]),
        "acs_get_instance_converged": (i32, [vp, P(C.c_uint8), u64]),
        "acs_get_instance_spread": (i32, [vp, P(C.c_double), u64]),
        "acs_get_spread_trace": (i32, [vp, u64, P(C.c_double), u64, P(u64)]),
        "acs_set_state": (i32, [vp, u32, vp, u64]),
        "acs_get_fault_status": (i32, [vp, P(u32), u64]),
        "acs_get_neighbors": (i32, [vp, P(u32), u64]),
        "acs_set_kernel_timing": (i32, [vp, i32]),
        "acs_get_kernel_timing": (i32, [vp, P(C.c_double), P(u64), C.c_char_p, u64]),
        "acs_sync": (i32, [vp]),
        "acs_device_count": (i32, []),
        "acs_runtime_info": (i32, [C.c_char_p, u64]),
        "acs_destroy": (None, [vp]),
        "acs_last_error": (C.c_char_p, []),
        "acs_abi_version": (i32, []),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def library_path() -> str:
    return LIB_PATH


def load_library() -> C.CDLL:
    """Load the in-tree HIP library.  Fails loudly if it has not been built: there is no
    CPU fallback in the product path (the CPU spec reference lives in oracle/, tests only)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"acsim HIP library not built: {LIB_PATH} is missing. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` (or `make -C "
            "approximate-consensus-simulation_amd/csrc`).")
    lib = C.CDLL(LIB_PATH)
    _declare(lib)
    v = lib.acs_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"libacsim ABI version {v} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def device_count() -> int:
    lib = load_library()
    n = lib.acs_device_count()
    if n < 0:
        check(lib, n)
    return n


def runtime_info() -> dict:
    """The HIP runtime / RCCL versions libacsim.so runs on, and the files this process mapped for
    them (/proc/self/maps): what a multi-rank run compares against the single-GPU run."""
    lib = load_library()
    buf = C.create_string_buffer(128)
    check(lib, lib.acs_runtime_info(buf, 128))
    out = {"versions": buf.value.decode()}
    try:
        with open("/proc/self/maps") as f:
            paths = sorted({ln.split()[-1] for ln in f if ln.rstrip().endswith(".so") or ".so." in ln})
    except OSError:
        paths = []
    for key, stem in (("libamdhip64", "libamdhip64.so"), ("librccl", "librccl.so")):
        out[key] = [p for p in paths if os.path.basename(p).startswith(stem)]
    return out


def check(lib, code: int) -> None:
    if code != OK:
        msg = lib.acs_last_error()
        raise AcsError(code, msg.decode() if msg else "")
