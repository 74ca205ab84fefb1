"""Command line: ``python -m acsim {presets,validate,run,sweep}`` (SURVEY §5 config/flags).

  python -m acsim presets
  python -m acsim validate --preset cfg4 --set n_nodes=4096
  python -m acsim run --preset cfg4_eps --out result.npz [--device 0] [--set key=value ...]
  python -m acsim sweep --preset cfg3 --set n_instances=1000 --grid loss_p=0.1,0.2 --out runs/
  python -m acsim run --preset cfg4 --graph my_graph.npz --set trim=2 ...   (user CSR graph,
      acsim or scipy.sparse .npz layout; topology and n_nodes come from the file)
"""
from __future__ import annotations

import argparse
import ctypes as C
import dataclasses
import json
import sys

from . import _abi
from .config import PRESETS, Config, preset


def _coerce(field: str, text: str):
    ftype = {f.name: f.type for f in dataclasses.fields(Config)}[field]
    if ftype in ("int", int):
        return int(text, 0)
    if ftype in ("float", float):
        return float(text)
    if ftype in ("bool", bool):
        return text.lower() in ("1", "true", "yes", "on")
    return text   # enum names (strings) or ints given as text are both accepted by Config


def _apply(cfg: Config, sets):
    over = {}
    for s in sets or []:
        k, _, v = s.partition("=")
        if k not in {f.name for f in dataclasses.fields(Config)}:
            raise SystemExit(f"unknown config field {k!r}")
        over[k] = _coerce(k, v)
    return cfg.replace(**over)


def _grid(specs):
    grid = {}
    for s in specs or []:
        k, _, v = s.partition("=")
        grid[k] = [_coerce(k, t) for t in v.split(",")]
    return grid


def validate(cfg: Config, csr=None) -> int:
    """Host-side §A.8 validation through the library (no GPU needed: acs_create validates first)."""
    lib = _abi.load_library()
    c = cfg.to_c()
    h = C.c_void_p()
    if csr is not None:
        rp, ci = csr
        rc = lib.acs_create_csr(C.byref(c), rp.ctypes.data_as(C.POINTER(C.c_uint64)),
                                ci.ctypes.data_as(C.POINTER(C.c_uint32)), 0, C.byref(h))
    else:
        rc = lib.acs_create(C.byref(c), _abi.BACKEND_HIP, (C.c_int * 1)(0), 1, C.byref(h))
    if rc == _abi.OK:
        lib.acs_destroy(h)
        return 0
    msg = lib.acs_last_error().decode()
    if rc == _abi.EDEVICE and "no HIP device" in msg:
        return 0   # the config is valid; there is just no GPU here
    print(f"invalid: {_abi.STATUS_NAMES.get(rc, rc)}: {msg}", file=sys.stderr)
    return 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="acsim")
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("presets")
    for name in ("validate", "run", "sweep"):
        p = sub.add_parser(name)
        p.add_argument("--preset", default="cfg1", choices=sorted(PRESETS))
        p.add_argument("--set", action="append", metavar="FIELD=VALUE")
        p.add_argument("--device", type=int, default=0)
        p.add_argument("--graph", metavar="FILE.npz", help="user CSR graph (acsim.graphs.load_csr)")
        if name in ("run", "sweep"):
            p.add_argument("--out")
        if name == "sweep":
            p.add_argument("--grid", action="append", metavar="FIELD=V1,V2,...", required=True)
    a = ap.parse_args(argv)
    if a.cmd == "presets":
        for k, v in PRESETS.items():
            print(k, json.dumps(dataclasses.asdict(v)))
        return 0
    cfg = _apply(preset(a.preset), a.set)
    csr = None
    if a.graph:
        from .graphs import load_csr
        csr = load_csr(a.graph)
        cfg = cfg.replace(topology="csr", n_nodes=int(csr[0].size - 1))
    if a.cmd == "validate":
        rc = validate(cfg, csr)
        if rc == 0:
            print("ok")
        return rc
    if a.cmd == "run":
        from .io import save_result
        from .sim import simulate
        res = simulate(cfg, device=a.device, return_values=bool(a.out), csr=csr)
        from .sweep import summarize
        print(json.dumps(summarize(cfg, res)))
        if a.out:
            save_result(a.out, res, cfg)
        return 0
    from .sweep import sweep
    rows = sweep(cfg, _grid(a.grid), out_dir=a.out, device=a.device, csr=csr)
    for r in rows:
        print(json.dumps(r))
    return 0


if __name__ == "__main__":
    sys.exit(main())
