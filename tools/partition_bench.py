"""cfg5 (N = 2^26, 16-regular, trimmed t = 5) node-partitioned round cost on ONE GPU: the plain
handle, a one-rank RCCL partition and eight virtual partitions (the 8-GPU data flow with device
copies as the exchange), each with the unchunked sequence (ACSIM_XCHUNKS=1: round, all-gather,
fold, all-reduce, verdict) and the chunked exchange.  One JSON line per case:
ms per round over R timed rounds after W warm-up rounds.  usage: python tools/partition_bench.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "approximate-consensus-simulation_amd"))
import acsim  # noqa: E402

W, R = 2, 8


def timed(make, name, chunks):
    os.environ["ACSIM_XCHUNKS"] = str(chunks)
    with make() as s:
        s.round(W)
        s.sync()
        t0 = time.perf_counter()
        s.round(R)
        s.sync()
        dt = time.perf_counter() - t0
        print(json.dumps({"case": name, "xchunks": chunks, "kernel": s.kernel_name(),
                          "ms_per_round": dt / R * 1e3, "node_rounds_per_s": (1 << 26) * R / dt}), flush=True)


def main():
    cfg = acsim.preset("cfg5", max_rounds=W + R)
    lib = acsim._abi.load_library()
    buf = C.create_string_buffer(lib.acs_comm_id_size())
    timed(lambda: acsim.Simulator(cfg), "plain", 1)
    for k in (1, 4):
        acsim._abi.check(lib, lib.acs_get_comm_id(buf, len(buf.raw)))
        timed(lambda: acsim.Simulator(cfg, partitions=1, rank=0, comm_id=buf.raw), "rccl_1rank", k)
    for k in (1, 4):
        timed(lambda: acsim.Simulator(cfg, partitions=8), "virtual_8", k)


if __name__ == "__main__":
    main()
