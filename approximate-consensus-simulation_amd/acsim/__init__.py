"""acsim — MI355X-native approximate-consensus round engine.

Public surface: ``simulate(cfg)``, ``Simulator(cfg).round(k)``, ``Config`` and the ``PRESETS``
(cfg1..cfg5).  The hot path is HIP (libacsim.so, include/acsim.h).
"""
from . import _abi, graphs
from ._abi import AcsError
from .config import Config, PRESETS, preset
from .sim import Result, RoundInfo, Simulator, simulate

__all__ = ["AcsError", "Config", "PRESETS", "preset", "Result", "RoundInfo", "Simulator",
           "simulate", "graphs", "_abi"]
