"""Generate the golden fixtures in tests/golden/ (run: python tests/golden/make_golden.py).

Upstream has no tests or vectors (the reference mount is README.md:1 only), so the fixtures
are produced by the CPU oracle (oracle/acs_oracle.c) and written ONLY where the independent
numpy restatement (tests/spec_np.py) agrees bit for bit.  The Philox vectors are the published
Random123 known-answer tests (external pins), not generated.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "approximate-consensus-simulation_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import oracle as O  # noqa: E402
import spec_np as S  # noqa: E402
from acsim.config import Config, preset  # noqa: E402

# Random123 kat_vectors, philox4x32_10 (ctr, key, expected)
PHILOX_KAT = [
    [[0x00000000, 0x00000000, 0x00000000, 0x00000000], [0x00000000, 0x00000000],
     [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]],
    [[0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff], [0xffffffff, 0xffffffff],
     [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]],
    [[0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]],
]

# Reduced-size presets (SURVEY §4 L0 golden fixtures) plus fault / loss / rule variants.
CASES = {
    "cfg1": preset("cfg1", trace_spread=True),
    "cfg1_avg": preset("cfg1_avg", trace_spread=True),
    "cfg2": preset("cfg2", trace_spread=True, max_rounds=2000),
    "cfg3_b16": preset("cfg3", n_instances=16, trace_spread=True),
    "cfg4_n4096": preset("cfg4_eps", n_nodes=4096, trace_spread=True),
    "cfg4_byz_n4096": preset("cfg4_byz", n_nodes=4096, n_faulty=40, trace_spread=True),
    "cfg5_n8192_fixed": preset("cfg5", n_nodes=8192, max_rounds=20, trace_spread=True),
    "reg8_crash_drop_mid": Config(n_nodes=2000, topology="regular", degree=8, rule="midpoint",
                                  trim=2, fault_model="crash", n_faulty=50, crash_window=5,
                                  loss_p=0.3, eps=1e-6, max_rounds=500, seed=7, trace_spread=True),
    "reg6_generic_trim": Config(n_nodes=999, topology="regular", degree=6, rule="trimmed",
                                trim=1, loss_p=0.05, eps=1e-7, max_rounds=500, seed=5,
                                trace_spread=True),
    "complete100_byzconst_dlpsw": Config(n_nodes=100, topology="complete", rule="dlpsw", trim=10,
                                         fault_model="byzantine", n_faulty=10,
                                         byz_strategy="constant", byz_const=5.0, loss_p=0.1,
                                         eps=1e-6, max_rounds=400, seed=3, trace_spread=True),
    "batched32_byzrand_grouped": Config(n_nodes=32, n_instances=6, topology="complete",
                                        rule="trimmed", trim=3, fault_model="byzantine",
                                        n_faulty=3, byz_strategy="random", byz_delta=0.1,
                                        loss_p=0.25, mask_group=4, eps=1e-8, max_rounds=300,
                                        seed=11, trace_spread=True, instance_offset=5),
}


def hexd(a) -> list:
    return [float(v).hex() for v in np.asarray(a, dtype=np.float64).ravel()]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def cfg_dict(c: Config) -> dict:
    import dataclasses
    return dataclasses.asdict(c)


def main() -> None:
    O.build()
    out = {"philox_kat": PHILOX_KAT}
    # draws: a spread of (stream, b, r, s) for seed 0 and a 64-bit seed
    draws = []
    for seed in (0, 0x0123456789ABCDEF):
        for stream in range(7):
            for (b, r, s) in ((0, 0, 0), (1, 2, 3), (77, 5, 1 << 20), (4294967295, 4294967295, (1 << 34) - 1)):
                v = O.draw(seed, stream, b, r, s)
                assert v == int(S.draw(seed, stream, b, r, s))
                draws.append([seed, stream, b, r, s, v])
    out["draws"] = draws
    # Feistel π_k for N = 1000, graph_seed 0, k = 0..3, first 64 points
    fe = {}
    for k in range(4):
        v = np.arange(64, dtype=np.uint64)
        p = S.feistel(1000, 0, k, v)
        assert all(int(p[i]) == O.feistel(1000, 0, k, i) for i in range(64))
        fe[str(k)] = [int(t) for t in p]
    out["feistel_n1000"] = fe
    out["drop_threshold"] = {str(p): O.drop_threshold(p) for p in (0.0, 0.2, 0.5, 0.999999)}
    sims = {}
    for name, cfg in CASES.items():
        with O.OracleSimulator(cfg) as o:
            o.run()
            ox = o.all_values()
            orr = o.rounds()
            traces = [o.spread_trace(b) for b in range(cfg.n_instances)]
            st = o.fault_status()
            conv = o.converged()
        n = S.NpSim(cfg)
        n.run()
        assert np.array_equal(orr, n.rounds), name
        assert np.array_equal(ox.view(np.uint64), n.x.view(np.uint64)), name
        for b in range(cfg.n_instances):
            assert np.array_equal(traces[b].view(np.uint64), np.array(n.trace[b]).view(np.uint64)), name
        faulty = [np.nonzero(st[b] != 0xFFFFFFFF)[0].tolist() for b in range(cfg.n_instances)]
        sims[name] = {
            "config": cfg_dict(cfg),
            "rounds": [int(v) for v in orr],
            "converged": [bool(v) for v in conv],
            "x_sha256": [sha(ox[b]) for b in range(cfg.n_instances)],
            "x_head": [hexd(ox[b][:16]) for b in range(cfg.n_instances)],
            "trace": [hexd(t) for t in traces[:2]],
            "faulty": faulty[:2],
            "status_of_faulty": [[int(st[b][v]) for v in faulty[b]] for b in range(min(2, cfg.n_instances))],
        }
        print(f"{name}: rounds {orr[:4]} ok")
    out["sims"] = sims
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
