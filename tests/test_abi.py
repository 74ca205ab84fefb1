"""CPU tests of the C-ABI boundary: the library loads, exports every symbol the
header declares, the ctypes mirror matches the C struct layout, and host-side validation
rejects the same configs as the oracle — all without a GPU (no compute calls)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

import acsim
from acsim import _abi
from acsim.config import Config, preset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "acsim.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(acs_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(acsim_lib):
    names = declared_functions()
    assert "acs_create" in names and "acs_round" in names and "acs_run" in names
    missing = [n for n in names if not hasattr(acsim_lib, n)]
    assert not missing, missing
    assert acsim_lib.acs_abi_version() == _abi.ABI_VERSION


def _probe_offsets(struct: str, fields):
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"acsim.h\"\nint main(void){\n"
    src += f'printf("%zu\\n", sizeof({struct}));\n'
    for f in fields:
        src += f'printf("%zu\\n", offsetof({struct}, {f}));\n'
    src += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        exe = os.path.join(d, "p")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


@pytest.mark.parametrize("cstruct,pystruct", [("acs_config", _abi.AcsConfig),
                                              ("acs_round_info", _abi.AcsRoundInfo),
                                              ("acs_result", _abi.AcsResult)])
def test_ctypes_layout_matches_header(cstruct, pystruct):
    fields = [f for f, _ in pystruct._fields_]
    got = _probe_offsets(cstruct, fields)
    assert got[0] == C.sizeof(pystruct)
    assert got[1:] == [getattr(pystruct, f).offset for f in fields]


BAD = [
    dict(n_nodes=0),
    dict(topology=7),
    dict(topology="regular", degree=3),
    dict(topology="regular", degree=0),
    dict(rule="average", trim=1),
    dict(rule="trimmed", trim=8, n_nodes=16),
    dict(rule="dlpsw", trim=0),
    dict(fault_model="none", n_faulty=2),
    dict(fault_model="crash", n_faulty=16, n_nodes=16),
    dict(fault_model="crash", n_faulty=1, crash_window=0),
    dict(loss_p=1.0),
    dict(loss_p=-0.1),
    dict(mask_group=0),
    dict(eps=-1.0),
    dict(termination=5),
    dict(fault_model="byzantine", n_faulty=1, byz_delta=float("inf")),
    dict(topology="complete", n_nodes=200000),
    dict(trace_spread=True, n_instances=1 << 20, max_rounds=1000),
]


@pytest.mark.parametrize("kw", BAD)
def test_invalid_configs_rejected_like_oracle(acsim_lib, oracle_mod, kw):
    cfg = Config(**kw)
    c = cfg.to_c()
    h = C.c_void_p()
    devs = (C.c_int * 1)(0)
    rc = acsim_lib.acs_create(C.byref(c), _abi.BACKEND_HIP, devs, 1, C.byref(h))
    assert rc == _abi.EINVAL, acsim_lib.acs_last_error()
    assert oracle_mod.validate(cfg) == _abi.EINVAL
    assert acsim_lib.acs_last_error()


def test_struct_size_versioning(acsim_lib):
    c = Config().to_c()
    c.struct_size = 8
    h = C.c_void_p()
    devs = (C.c_int * 1)(0)
    assert acsim_lib.acs_create(C.byref(c), _abi.BACKEND_HIP, devs, 1, C.byref(h)) == _abi.EINVAL


def test_cpu_backend_is_not_a_product_path(acsim_lib):
    c = preset("cfg1").to_c()
    h = C.c_void_p()
    devs = (C.c_int * 1)(0)
    assert acsim_lib.acs_create(C.byref(c), _abi.BACKEND_CPU, devs, 1, C.byref(h)) == _abi.EUNSUPPORTED
    with pytest.raises(ValueError):
        acsim.Simulator("cfg1", backend="cpu")


def test_dtype_validation(acsim_lib, oracle_mod):
    """fp32 is a product dtype; its Byzantine parameters must fit binary32 and an
    unknown dtype is rejected — the same verdicts from the library and the oracle."""
    h = C.c_void_p()
    devs = (C.c_int * 1)(0)
    bad = preset("cfg4_byz", n_nodes=4096, dtype="f32", byz_delta=1e31)
    assert oracle_mod.validate(bad) == _abi.EINVAL
    assert acsim_lib.acs_create(C.byref(bad.to_c()), _abi.BACKEND_HIP, devs, 1, C.byref(h)) == _abi.EINVAL
    c = preset("cfg1").to_c()
    c.dtype = 7
    assert acsim_lib.acs_create(C.byref(c), _abi.BACKEND_HIP, devs, 1, C.byref(h)) == _abi.EINVAL
    assert oracle_mod.validate(preset("cfg4", dtype="f32")) == 0


def test_presets_valid(oracle_mod):
    for name, cfg in acsim.PRESETS.items():
        assert oracle_mod.validate(cfg) == 0, name


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(_abi, "_lib", None)
    monkeypatch.setattr(_abi, "LIB_PATH", "/nonexistent/libacsim.so")
    with pytest.raises(ImportError):
        _abi.load_library()


def test_runtime_info_reports_the_rocm_libraries(acsim_lib):
    """acs_runtime_info (no GPU needed): the HIP runtime and RCCL versions, and the files this
    process mapped for them — bench.py records them per rank so an N > 1 run can be checked to
    run on the same libraries as the single-GPU run and the GPU suite."""
    info = _abi.runtime_info()
    m = re.fullmatch(r"hip \d+ rccl \d+ polled-host-flags 0x([0-9a-f]+)", info["versions"])
    assert m, info
    # the host memory the round loop polls (run summary, instance states) is mapped, and requests
    # coherence explicitly (hipHostMallocCoherent 0x40000000, never NonCoherent 0x80000000), so
    # the sequence-number protocol does not rest on the runtime's default
    flags = int(m.group(1), 16)
    assert flags & 0x2, hex(flags)                    # hipHostMallocMapped
    assert flags & 0x40000000, hex(flags)             # hipHostMallocCoherent
    assert not flags & 0x80000000, hex(flags)
    assert len(info["libamdhip64"]) == 1 and info["libamdhip64"][0].startswith("/opt/rocm"), info
    assert len(info["librccl"]) == 1 and info["librccl"][0].startswith("/opt/rocm"), info
