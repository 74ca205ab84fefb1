"""Simulation configuration (Python mirror of ``acs_config``) and the named presets.

Presets follow SURVEY.md §A.10 (sizes from BASELINE.json configs[0..4]; the bracketed
parameters there are frozen by the survey, since the reference mount holds no code).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from dataclasses import dataclass, field

from . import _abi

_ENUMS = {
    "topology": {"complete": _abi.TOPO_COMPLETE, "random_regular": _abi.TOPO_RANDOM_REGULAR,
                 "regular": _abi.TOPO_RANDOM_REGULAR, "csr": _abi.TOPO_CSR},
    "rule": {"average": _abi.RULE_AVERAGE, "trimmed_mean": _abi.RULE_TRIMMED_MEAN,
             "trimmed": _abi.RULE_TRIMMED_MEAN, "midpoint": _abi.RULE_MIDPOINT,
             "dlpsw": _abi.RULE_DLPSW_SELECT, "dlpsw_select": _abi.RULE_DLPSW_SELECT,
             "wmsr": _abi.RULE_WMSR, "w_msr": _abi.RULE_WMSR},
    "fault_model": {"none": _abi.FAULT_NONE, "crash": _abi.FAULT_CRASH,
                    "byzantine": _abi.FAULT_BYZANTINE},
    "byz_strategy": {"split": _abi.BYZ_SPLIT, "random": _abi.BYZ_RANDOM,
                     "constant": _abi.BYZ_CONSTANT},
    "termination": {"eps": _abi.TERM_EPS, "fixed": _abi.TERM_FIXED},
    "missing_policy": {"self": _abi.MISSING_SELF, "omit": _abi.MISSING_OMIT},
    "dtype": {"f64": _abi.F64, "fp64": _abi.F64, "float64": _abi.F64, "f32": _abi.F32,
              "fp32": _abi.F32, "float32": _abi.F32},
}


def _enum(name: str, v) -> int:
    if isinstance(v, str):
        try:
            return _ENUMS[name][v.lower()]
        except KeyError:
            raise ValueError(f"unknown {name} {v!r}; expected one of {sorted(_ENUMS[name])}")
    return int(v)


@dataclass
class Config:
    """One simulation.  Field meanings: include/acsim.h ``acs_config``."""
    n_nodes: int = 16
    n_instances: int = 1
    topology: object = "complete"
    degree: int = 0
    rule: object = "average"
    trim: int = 0
    fault_model: object = "none"
    n_faulty: int = 0
    byz_strategy: object = "split"
    byz_delta: float = 0.0
    byz_const: float = 0.0
    crash_window: int = 1
    loss_p: float = 0.0
    mask_group: int = 1
    eps: float = 1e-6
    max_rounds: int = 1000
    termination: object = "eps"
    dtype: object = "f64"
    seed: int = 0
    graph_seed: int = 0
    trace_spread: bool = False
    omp_threads: int = 0
    instance_offset: int = 0
    delay_max: int = 0          # bounded-delay rounds; 0 = synchronous
    missing_policy: object = "self"   # "self" (§A.6 substitution) or "omit" 

    def replace(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)

    @property
    def m(self) -> int:
        """Entries per receiver: N (complete) or d+1 (random regular), §A.3."""
        return self.n_nodes if _enum("topology", self.topology) == _abi.TOPO_COMPLETE else self.degree + 1

    def to_c(self) -> _abi.AcsConfig:
        c = _abi.AcsConfig()
        c.struct_size = C.sizeof(_abi.AcsConfig)
        c.n_nodes = int(self.n_nodes)
        c.n_instances = int(self.n_instances)
        c.topology = _enum("topology", self.topology)
        c.degree = int(self.degree)
        c.rule = _enum("rule", self.rule)
        c.trim = int(self.trim)
        c.fault_model = _enum("fault_model", self.fault_model)
        c.n_faulty = int(self.n_faulty)
        c.byz_strategy = _enum("byz_strategy", self.byz_strategy)
        c.byz_delta = float(self.byz_delta)
        c.byz_const = float(self.byz_const)
        c.crash_window = int(self.crash_window)
        c.loss_p = float(self.loss_p)
        c.mask_group = int(self.mask_group)
        c.eps = float(self.eps)
        c.max_rounds = int(self.max_rounds)
        c.termination = _enum("termination", self.termination)
        c.dtype = _enum("dtype", self.dtype)
        c.seed = int(self.seed)
        c.graph_seed = int(self.graph_seed)
        c.trace_spread = 1 if self.trace_spread else 0
        c.omp_threads = int(self.omp_threads)
        c.instance_offset = int(self.instance_offset)
        c.delay_max = int(self.delay_max)
        c.missing_policy = _enum("missing_policy", self.missing_policy)
        return c


# ----------------------------------------------------------------------------------- presets
# SURVEY.md §A.10.  "1M" / "64M" are frozen as 2^20 / 2^26.
PRESETS = {
    # BASELINE configs[0]: N=16 complete, crash f=1 [W=1], midpoint/average [t=0], eps=1e-3, seed 0
    "cfg1": Config(n_nodes=16, topology="complete", rule="midpoint", trim=0, fault_model="crash",
                   n_faulty=1, crash_window=1, eps=1e-3, max_rounds=1000, seed=0),
    "cfg1_avg": Config(n_nodes=16, topology="complete", rule="average", trim=0,
                       fault_model="crash", n_faulty=1, crash_window=1, eps=1e-3,
                       max_rounds=1000, seed=0),
    # configs[1]: N=1024 complete, f=341 Byzantine [SPLIT, Δ=0], trimmed t=341, eps=1e-6
    "cfg2": Config(n_nodes=1024, topology="complete", rule="trimmed_mean", trim=341,
                   fault_model="byzantine", n_faulty=341, byz_strategy="split", byz_delta=0.0,
                   eps=1e-6, max_rounds=100000),
    # configs[2]: 1e5 instances x 64 nodes, 20% loss, averaging [G=1, eps=1e-6]
    "cfg3": Config(n_nodes=64, n_instances=100000, topology="complete", rule="average",
                   loss_p=0.2, mask_group=1, eps=1e-6, max_rounds=1000),
    # cfg3 with 16-instance groups sharing drop masks (§A.5 G = 16): the batched W·X MFMA variant
    "cfg3_g16": Config(n_nodes=64, n_instances=100000, topology="complete", rule="average",
                       loss_p=0.2, mask_group=16, eps=1e-6, max_rounds=1000),
    # configs[3]: N=2^20 random 32-regular, trimmed t=5 (headline); timed in FIXED R=100
    "cfg4": Config(n_nodes=1 << 20, topology="random_regular", degree=32, rule="trimmed_mean",
                   trim=5, eps=1e-6, max_rounds=100, termination="fixed"),
    "cfg4_eps": Config(n_nodes=1 << 20, topology="random_regular", degree=32,
                       rule="trimmed_mean", trim=5, eps=1e-6, max_rounds=1000),
    # cfg4 variant: 0.1% Byzantine RANDOM senders
    "cfg4_byz": Config(n_nodes=1 << 20, topology="random_regular", degree=32,
                       rule="trimmed_mean", trim=5, fault_model="byzantine", n_faulty=1048,
                       byz_strategy="random", byz_delta=0.0, eps=1e-6, max_rounds=1000),
    # configs[4]: N=2^26 random 16-regular, [trimmed t=5]; node-partitioned over G GPUs
    "cfg5": Config(n_nodes=1 << 26, topology="random_regular", degree=16, rule="trimmed_mean",
                   trim=5, eps=1e-6, max_rounds=100, termination="fixed"),
}


def preset(name: str, **overrides) -> Config:
    try:
        base = PRESETS[name]
    except KeyError:
        raise ValueError(f"unknown preset {name!r}; have {sorted(PRESETS)}")
    return base.replace(**overrides)
